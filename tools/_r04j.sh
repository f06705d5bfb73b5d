# round 4, session j: where the d = 4 static split's slow workgroups sit (blockIdx vs CU slot)
set -o pipefail
O=gpurun_out/r04_j; mkdir -p $O
for d in 4 1; do
timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d $d --libs build/ab/stamps1.so > $O/stamps_static_d$d.log 2>&1 || exit $?
done
timeout -k 10 120 python -u tools/fs_stamps.py --kernel p --d 4 --libs build/ab/pqst3.so > $O/stamps_queue_d4.log 2>&1 || exit $?
echo done > $O/DONE
