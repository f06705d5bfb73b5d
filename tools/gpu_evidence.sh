#!/bin/bash
# Round evidence on one box, each GPU step under its own time limit, stopping at the first
# crash-like exit: GPU tests, smoke, the driver's exact bench command, a rocprofv3
# kernel-trace --stats run of that same command, then tools/gpu_pmc_configs.sh (PMC passes,
# kernel-trace only, one counter group per run, for every config the bench reports).  Arg: TAG.
#   gpurun --timeout 1200 -- 'bash tools/gpu_evidence.sh r05_final'
#   bash tools/save_evidence.sh r05_final r05/final
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
echo "bench done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/$BENCH > $O/trace.log 2>&1 || exit $?
echo "trace done"
[ -n "$SKIP_PMC" ] || bash $R/tools/gpu_pmc_configs.sh $O/pmc || exit $?
echo done > $O/DONE
