#!/bin/bash
# Channel-kernel parity subset + interleaved A/B of two build/ab libraries at C5 (1024 x d=4),
# 128 channels at d = 4 and 6 (v2 kernel) and d = 1 (p kernel).  Args: LIB_A LIB_B OUTNAME
set -o pipefail
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_cs16.py tests/test_gpu_parity.py tests/test_gpu_sweep.py -k "channel or c5 or cs16" > $O/$3_pytest.log 2>&1 || { tail -30 $O/$3_pytest.log; exit 1; }
tail -1 $O/$3_pytest.log
L="build/ab/$1.so build/ab/$2.so build/ab/$1.so build/ab/$2.so"
timeout -k 10 300 python tools/ab_libs.py --libs $L --d 4 --channels 1024 --nblk 256 --rounds 6 > $O/$3_c5.txt 2>&1 || exit 1
timeout -k 10 300 python tools/ab_libs.py --libs $L --d 1 4 6 --channels 128 --nblk 256 --rounds 6 > $O/$3_128.txt 2>&1 || exit 1
grep -hv "^{" $O/$3_c5.txt $O/$3_128.txt
