# round 4, session e: queue-path tests, pair tickets and static share at d = 0, d = 1..4 vs round 3
set -o pipefail
O=gpurun_out/r04_e; mkdir -p $O
bash tools/gpu_step.sh r04_e --testsel "tests/test_gpu_parity.py tests/test_gpu_queue.py" || exit $?
timeout -k 10 500 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur.so build/ab/ts1.so build/ab/ts2.so build/ab/ts4.so build/ab/cur.so:1=0 build/ab/ts2.so:1=0 --d 0 --rounds 8 > $O/ab_d0.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur.so build/ab/ts2.so --d 1 2 3 4 --rounds 5 > $O/ab_d14.log 2>&1 || exit $?
bash tools/gpu_step.sh r04_e --bench || exit $?
echo done > $O/DONE2
