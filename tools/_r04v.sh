# round 4, session v: the quad first pass at d = 3, 4 with its output select as bit selects
# (the first build read its outputs back through scratch memory)
set -o pipefail
O=gpurun_out/r04_v; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur13.so build/ab/qf.so --d 3 4 --rounds 8 > $O/ab_qf.log 2>&1 || exit $?
echo done > $O/DONE
