#!/bin/bash
# Round evidence on one box: GPU tests, smoke, the default bench line, a rocprofv3
# kernel-trace --stats run of the same bench, and FETCH_SIZE / WRITE_SIZE passes (separate
# runs, kernel-trace only) for the headline kernel.  Arg: TAG.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; TAG=${1:-round}; O=$R/gpurun_out/$TAG; mkdir -p $O
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; crashed $rc && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq --pmc $c -d $O/pmc_$c -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_$c.log 2>&1 || exit $?
done
# FETCH/WRITE calibration for the kernel's access widths (4 B/lane loads, 8 B/lane stores)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex calib --pmc $c -d $O/calib_$c -o run -- $R/build/bin/pmc_calib > $O/calib_$c.log 2>&1 || exit $?
done
