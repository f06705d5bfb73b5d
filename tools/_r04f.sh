# round 4, session f: d = 0..4 vs round 3 after the d = 2 SGPR fix, stream pipelining, stamps
set -o pipefail
O=gpurun_out/r04_f; mkdir -p $O
timeout -k 10 400 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/cur2.so --d 0 1 2 3 4 --rounds 6 > $O/ab.log 2>&1 || exit $?
for s in 1 2 3; do
timeout -k 10 200 python bench.py --steps 100 --warmup 50 --streams $s --no-sweep --no-cpu-baseline --no-c5 > $O/bench_s$s.log 2>&1 || exit $?
done
timeout -k 10 120 python -u tools/fs_stamps.py --kernel fs --libs build/ab/stamps1.so build/ab/stamps2.so build/ab/stamps3.so > $O/stamps_fs.log 2>&1 || exit $?
for d in 3 4; do
timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d $d --libs build/ab/stamps1.so build/ab/stamps2.so build/ab/stamps3.so > $O/stamps_p_d$d.log 2>&1 || exit $?
done
echo done > $O/DONE
