#!/bin/bash
# Wave-kernel bring-up on one box: its GPU tests, an interleaved A/B against the persistent
# kernel (variant 2) at d = 0, then the whole GPU suite.  Stops at a crash/timeout.  Arg: TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-wave}
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -m gpu -q -rA --timeout 120 --timeout-method thread > gpurun_out/pytest_wave_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_wave_$TAG.log
crashed $rc && exit $rc
timeout -k 10 300 python tools/ab_kernels.py --d 0 --variants 3 0 --rounds 10 > gpurun_out/ab_wave_$TAG.log 2>&1
rc2=$?; crashed $rc2 && exit $rc2
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_all_$TAG.log 2>&1
rc3=$?; echo "pytest rc=$rc3" >> gpurun_out/pytest_all_$TAG.log
exit $rc3
