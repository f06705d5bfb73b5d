# round 4, session x: forward pass 2 + split fused at d >= 4 (FS-style, DPP mirror): A/B and
# output identity against the current tree over tune bins
set -o pipefail
O=gpurun_out/r04_x; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur.so build/ab/fu.so build/ab/fu4.so --d 4 5 6 --rounds 8 > $O/ab_fuse.log 2>&1 || exit $?
for tb in 0 4 192 1024 2044 2408 2708 3900 4092 4095; do
  timeout -k 10 120 python -u tools/ab_libs.py --libs build/ab/cur.so build/ab/fu4.so --d 4 5 6 --rounds 1 --reps 2 --nblk 64 --tunebin $tb > $O/id_tb$tb.log 2>&1 || exit $?
done
echo done > $O/DONE
