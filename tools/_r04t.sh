# round 4, session t: is the XCD speed pattern stable within a box? stamps twice at d = 0 and d = 1
set -o pipefail
O=gpurun_out/r04_t; mkdir -p $O
for k in 1 2; do
  timeout -k 10 120 python -u tools/fs_stamps.py --kernel fs --libs build/ab/c12st1.so > $O/stamps_fs_$k.log 2>&1 || exit $?
  timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d 1 --libs build/ab/c12st1.so > $O/stamps_p1_$k.log 2>&1 || exit $?
done
echo done > $O/DONE
