#!/bin/bash
# Build libsddc_ddc.so as of a git revision into build/ab/NAME.so, for interleaved A/B timing
# against the working tree with tools/ab_libs.py (the product source carries no A/B switches:
# a variant is a revision, or a scratch copy of the tree).
# usage: tools/build_rev_lib.sh REV NAME        (REV = a git revision, or "tree" for the working tree)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
S=$R/build/ab/src_$NAME
rm -rf "$S"; mkdir -p "$S"
if [ "$REV" = tree ]; then
  cp -r "$R/extio_sddc_amd/csrc" "$R/include" "$S/"
else
  git -C "$R" archive "$REV" extio_sddc_amd/csrc include | tar -x -C "$S"
  mv "$S/extio_sddc_amd/csrc" "$S/csrc"; rmdir "$S/extio_sddc_amd"
fi
C=$S/csrc
O=$S/obj; mkdir -p $O
F="-O3 -std=c++17 -fPIC -fno-slp-vectorize -I$C -I$S/include $EXTRA"
objs=""
for k in $C/*.hip; do
  b=$(basename $k .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $k -o $O/$b.o &
  objs="$objs $O/$b.o"
done
for c in ddc_runtime filterbank fine_tune; do
  /opt/rocm/bin/hipcc $F -ffp-contract=off -c $C/$c.cpp -o $O/$c.o &
  objs="$objs $O/$c.o"
done
for c in fft_avx2 r2iq_cpu; do
  g++ -O3 -std=c++17 -fPIC -mavx2 -mfma -ffp-contract=off -I$C -I$S/include -c $C/cpu/$c.cpp -o $O/cpu_$c.o &
  objs="$objs $O/cpu_$c.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $objs -o $R/build/ab/$NAME.so -ldl
echo built $R/build/ab/$NAME.so
