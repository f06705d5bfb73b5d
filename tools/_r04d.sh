# round 4, session d: tail-wave tests, the d = 3 identity check, A/B at d = 0..4
set -o pipefail
O=gpurun_out/r04_d; mkdir -p $O
bash tools/gpu_step.sh r04_d --testsel "tests/test_gpu_tailwave.py tests/test_gpu_queue.py" || exit $?
timeout -k 10 120 python -u tools/tw_identity.py build/ab/scan.so build/ab/nocontract.so > $O/tw_identity.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/fs1.so build/ab/scan.so build/ab/scan.so:1=0 build/ab/scan.so:1=30 build/ab/scan.so:1=50 --d 0 --rounds 8 > $O/ab_d0.log 2>&1 || exit $?
for d in 4 3 2 1; do
timeout -k 10 400 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/scan.so build/ab/scan.so:3=0 build/ab/scan.so:2=0 build/ab/scan.so:2=50 --d $d --rounds 6 > $O/ab_d$d.log 2>&1 || exit $?
done
echo done > $O/DONE2
