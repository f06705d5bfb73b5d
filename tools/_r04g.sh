# round 4, session g: the frame queue at d >= 3 (the static split leaves workgroups ending 74..119 us)
set -o pipefail
O=gpurun_out/r04_g; mkdir -p $O
timeout -k 10 400 python -u tools/ab_libs.py --libs build/ab/cur2.so build/ab/pqall.so --d 3 4 5 6 --rounds 6 > $O/ab.log 2>&1 || exit $?
for d in 3 4; do
timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d $d --libs build/ab/pqst1.so > $O/stamps_pq_d$d.log 2>&1 || exit $?
done
echo done > $O/DONE
