set -o pipefail
O=gpurun_out/ab; mkdir -p $O
for n in 512 1024 2048 4096 8192; do
timeout -k 10 200 python tools/ab_libs.py --libs build/ab/cur.so --d 0 --nblk $n --rounds 8 --reps 10 2>&1 | grep "^d=" >> $O/tail.txt || exit 1
done
cat $O/tail.txt
