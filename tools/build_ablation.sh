#!/bin/bash
# Build a variant copy of the working tree's library: build/ab/NAME.so, with PATCHFILE applied to
# its copy of csrc/: a .txt of Python-regex substitutions (each line FILE<TAB>REGEX<TAB>REPLACEMENT,
# each must match), or a .py script run with the copy's csrc path as argv[1].  Ablations compute
# wrong results on purpose (they attribute a kernel's time to one of its parts in tools/ab_libs.py
# runs); candidate variants must match the product's output within tolerance.  Neither ships.
#   tools/build_ablation.sh NAME PATCHFILE
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; PATCH=$2
S=$R/build/ab/src_$NAME
rm -rf "$S"; mkdir -p "$S"
cp -r "$R/extio_sddc_amd/csrc" "$R/include" "$S/"
if [ "${PATCH%.py}" != "$PATCH" ]; then python3 "$PATCH" "$S/csrc"; else
python3 - "$S/csrc" "$PATCH" <<'PY'
import re, sys
root, patch = sys.argv[1], sys.argv[2]
for line in open(patch):
    line = line.rstrip("\n")
    if not line or line.startswith("#"):
        continue
    f, rx, rep = line.split("\t")
    p = f"{root}/{f}"
    s = open(p).read()
    s2, n = re.subn(rx, rep, s)
    assert n > 0, f"{f}: no match for {rx}"
    open(p, "w").write(s2)
PY
fi
bash "$R/tools/build_src_lib.sh" "$NAME"
