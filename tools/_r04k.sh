# round 4, session k: slot-weighted static split at d >= 3
set -o pipefail
O=gpurun_out/r04_k; mkdir -p $O
timeout -k 10 400 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur5.so build/ab/cur5.so:2=0 --d 3 4 5 6 --rounds 6 > $O/ab.log 2>&1 || exit $?
for d in 3 4 6; do
timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d $d --libs build/ab/c5st1.so > $O/stamps_w_d$d.log 2>&1 || exit $?
done
for s in 1 2; do
timeout -k 10 200 python bench.py --d 4 --steps 100 --warmup 50 --streams $s --no-sweep --no-cpu-baseline --no-c5 > $O/bench_d4_s$s.log 2>&1 || exit $?
done
echo done > $O/DONE
