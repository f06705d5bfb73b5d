# round 4, session p: parity after the pruned forward pass 2 at d = 4; end to end with the drop-in
# taking up to 16 (current), 24 or 28 ring slots per GPU call
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r04_p; mkdir -p $O
bash tools/gpu_step.sh r04_p --testsel "tests/test_gpu_parity.py tests/test_gpu_queue.py tests/test_gpu_sweep.py tests/test_gpu_floor.py" || exit $?
grep -q "rc=0" $O/pytest_sel.log || exit 1
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/grp4.so build/ab/q0.so build/ab/q3.so --d 3 4 5 6 --rounds 6 > $O/ab_q0.log 2>&1 || exit $?
for b in 16 24 28; do
  H=$R/oracle/_ref/radiohandler_harness; [ $b = 16 ] || H=${H}_b$b
  HARNESS=$H timeout -k 10 400 bash tools/e2e_benchmark_test.sh $O/e2e_b$b > $O/e2e_b$b.log 2>&1 || exit $?
done
echo done > $O/DONE
