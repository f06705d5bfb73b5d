#!/bin/bash
# Round evidence on one box, each GPU step under its own time limit, stopping at the first
# crash-like exit: GPU tests, smoke, the driver's exact bench command, a rocprofv3
# kernel-trace --stats run of that same command, and PMC passes (kernel-trace only, one
# counter group per run) for the headline kernel: VALU issue and HBM bytes.  Arg: TAG.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; TAG=${1:-round}; O=$R/gpurun_out/$TAG; mkdir -p $O
BENCH="bench.py --gpus 1 --steps 20 --warmup 5"
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rfE --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; crashed $rc && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
fi
timeout -k 10 300 python $BENCH > $O/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/$BENCH > $O/trace.log 2>&1 || exit $?
P="python3 $R/bench.py --steps 5 --warmup 2 --warmup-ms 0 --no-cpu-baseline --no-sweep"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq_persistent \
  --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d $O/pmc_valu -o run -- $P > $O/pmc_valu.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq_persistent --pmc $c \
    -d $O/pmc_$c -o run -- $P > $O/pmc_$c.log 2>&1 || exit $?
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex calib --pmc $c \
    -d $O/calib_$c -o run -- $R/build/bin/pmc_calib > $O/calib_$c.log 2>&1 || exit $?
done
echo done > $O/DONE
