# round 4, session u: d >= 4 inverse tail deferred into the next frame's forward pass 0 (wave 0)
set -o pipefail
O=gpurun_out/r04_u; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur12.so build/ab/dt.so --d 4 5 6 --rounds 8 > $O/ab_dt.log 2>&1 || exit $?
echo done > $O/DONE
