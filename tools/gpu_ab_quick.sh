#!/bin/bash
# Parity subset + interleaved A/B of two build/ab libraries.  Args: LIB_A LIB_B "d list" OUTNAME [extra ab args]
set -o pipefail
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_nco.py tests/test_gpu_cs16.py > $O/$4_pytest.log 2>&1 || { tail -30 $O/$4_pytest.log; exit 1; }
tail -2 $O/$4_pytest.log
timeout -k 10 300 python tools/ab_libs.py --libs build/ab/$1.so build/ab/$2.so build/ab/$1.so build/ab/$2.so --d $3 --rounds 10 $5 > $O/$4.txt 2>&1 || exit 1
grep -v "^{" $O/$4.txt
