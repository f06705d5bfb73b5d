# one GPU session (edited per use): each step under its own limit, stop at the first failure
set -o pipefail
O=gpurun_out/r05_f; mkdir -p $O
A="build/ab/cur.so build/ab/pq_l1.so build/ab/no_twl.so build/ab/no_store.so build/ab/in_l2.so"
timeout -k 10 400 python -u tools/ab_libs.py --libs $A --d 0 --rounds 8 > $O/ab_ablation.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur.so build/ab/cur.so:7=0 --d 0 --rounds 6 --input zeros > $O/ab_zeros.log 2>&1 || exit $?
echo done > $O/DONE
