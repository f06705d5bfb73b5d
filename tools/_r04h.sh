# round 4, session h: the ticket read moved to the frame top (persistent kernel), queue at d >= 3
set -o pipefail
O=gpurun_out/r04_h; mkdir -p $O
timeout -k 10 500 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur2.so build/ab/cur3.so build/ab/pqall2.so --d 1 2 3 4 5 6 --rounds 5 > $O/ab.log 2>&1 || exit $?
for d in 1 4; do
timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d $d --libs build/ab/pqst2.so > $O/stamps_pq2_d$d.log 2>&1 || exit $?
done
echo done > $O/DONE
