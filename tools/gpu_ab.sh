#!/bin/bash
# GPU tests (stop on crash) then an interleaved A/B of kernel variants.  Args: TAG [ab args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${1:-ab}; shift
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_$TAG.log
crashed $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/ab_kernels.py "$@" > gpurun_out/ab_$TAG.log 2>&1
