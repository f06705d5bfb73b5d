# round 4, session m: slot-weighted static prefix + queue remainder at d = 0..2; weights at d >= 3
set -o pipefail
O=gpurun_out/r04_m; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur6.so build/ab/cur7.so build/ab/cur7.so:1=60 build/ab/cur7.so:2=0 --d 0 --rounds 8 > $O/ab_d0.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur6.so build/ab/cur7.so build/ab/wst.so build/ab/cur7.so:3=60 --d 1 2 --rounds 6 > $O/ab_d12.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur6.so build/ab/w2.so --d 3 4 5 6 --rounds 6 > $O/ab_d36.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/fs_stamps.py --kernel fs --libs build/ab/c7st1.so > $O/stamps_fs.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d 1 --libs build/ab/c7st1.so > $O/stamps_p_d1.log 2>&1 || exit $?
echo done > $O/DONE
