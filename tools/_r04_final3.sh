# round 4, final evidence (3) on one box: GPU tests, smoke, the driver's bench command, rocprofv3
# kernel-trace --stats of that command and of its single-stream form, PMC passes per config
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out/r04_final3; mkdir -p $O
BENCH="bench.py --gpus 1 --steps 20 --warmup 5"
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rfE --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; crashed $rc && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python $BENCH > $O/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/$BENCH > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_s1 -o run -- python3 $R/$BENCH --streams 1 --no-c5 --no-sweep --no-cpu-baseline > $O/trace_s1.log 2>&1 || exit $?
cd $R
timeout -k 10 400 bash tools/e2e_benchmark_test.sh $O/e2e > $O/e2e.log 2>&1 || exit $?
bash tools/gpu_pmc_configs.sh $O/pmc_cfg > $O/pmc_cfg.log 2>&1 || exit $?
echo done > $O/DONE
