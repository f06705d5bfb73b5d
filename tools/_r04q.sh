# round 4, session q: slot-weight tuning at d = 1..6; per-slot / per-XCD ends of the final tree
set -o pipefail
O=gpurun_out/r04_q; mkdir -p $O
timeout -k 10 400 python -u tools/ab_libs.py --libs build/ab/cur10.so build/ab/wA.so build/ab/wB.so --d 1 2 3 4 5 6 --rounds 6 > $O/ab_w.log 2>&1 || exit $?
for d in 1 4; do
timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d $d --libs build/ab/c10st1.so > $O/stamps_p_d$d.log 2>&1 || exit $?
done
echo done > $O/DONE
