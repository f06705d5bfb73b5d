# round 4, session z: per-XCD frame weights for the d = 0 kernel, calibrated on this box from a
# stamps run (tools/xcd_weights.py), then the same box's A/B against the slot weights alone
set -o pipefail
O=gpurun_out/r04_z; mkdir -p $O
timeout -k 10 120 python -u tools/fs_stamps.py --kernel fs --libs build/ab/xst.so > $O/st_equal.log 2>&1 || exit $?
P=$(python tools/xcd_weights.py < $O/st_equal.log 2>> $O/weights.txt) || exit $?
echo "$P" >> $O/weights.txt
timeout -k 10 120 python -u tools/fs_stamps.py --kernel fs --libs build/ab/xst.so --param ${P%%,*} --param ${P##*,} > $O/st_xcdw.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/xw.so build/ab/xw.so:$P --d 0 --rounds 10 > $O/ab_xcdw.log 2>&1 || exit $?
echo done > $O/DONE
