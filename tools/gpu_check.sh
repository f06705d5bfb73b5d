#!/bin/bash
# One GPU-box session: gpu parity tests, a bench line, a rocprofv3 kernel-trace summary.
# Stops at the first crash/timeout (rc 124/134/137/139) so nothing else touches a faulted GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-run}
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_$TAG.log
crashed $rc && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-budget 5 > gpurun_out/bench_$TAG.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
