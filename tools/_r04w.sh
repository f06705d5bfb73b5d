# round 4, session w: the d >= 3 inverse tail on wave f mod 4 instead of wave 0 (A/B), and the
# wave -> SIMD mapping from HW_ID in a stamps build
set -o pipefail
O=gpurun_out/r04_w; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur.so build/ab/rot.so --d 3 4 5 6 --rounds 8 > $O/ab_rot.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d 4 --libs build/ab/st1.so > $O/stamps_rot_d4.log 2>&1 || exit $?
echo done > $O/DONE
