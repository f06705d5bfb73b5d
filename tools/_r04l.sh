# round 4, session l: slot-weighted static split at d = 1, 2; weight tuning at d >= 3; FS per-slot frames
set -o pipefail
O=gpurun_out/r04_l; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur6.so build/ab/wst.so --d 1 2 --rounds 6 > $O/ab_d12.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur6.so build/ab/w2.so --d 3 4 5 6 --rounds 6 > $O/ab_d36.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/fs_stamps.py --kernel fs --libs build/ab/stamps1.so > $O/stamps_fs_slots.log 2>&1 || exit $?
echo done > $O/DONE
