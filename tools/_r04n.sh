# round 4, session n: persistent kernel without the queue (slot-weighted split at every d); FS share
set -o pipefail
O=gpurun_out/r04_n; mkdir -p $O
bash tools/gpu_step.sh r04_n --tests || exit $?
timeout -k 10 400 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur6.so build/ab/cur8.so build/ab/cur8.so:1=95 build/ab/cur8.so:1=100 --d 0 --rounds 8 > $O/ab_d0.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur8.so --d 1 2 3 4 5 6 --rounds 5 > $O/ab_d16.log 2>&1 || exit $?
bash tools/gpu_step.sh r04_n --bench || exit $?
echo done > $O/DONE2
