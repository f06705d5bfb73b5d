#!/bin/bash
# Parity subset on the product library, then interleaved A/B of N build/ab libraries.
# Args: OUTNAME "lib names (build/ab/NAME.so)" "d list" [extra ab_libs args]
set -o pipefail
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_sweep.py tests/test_gpu_nco.py tests/test_gpu_cs16.py > $O/$1_pytest.log 2>&1 || { tail -30 $O/$1_pytest.log; exit 1; }
tail -2 $O/$1_pytest.log
LIBS=""; for n in $2; do LIBS="$LIBS build/ab/$n.so"; done
timeout -k 10 400 python tools/ab_libs.py --libs $LIBS --d $3 --rounds 10 $4 > $O/$1.txt 2>&1 || { tail -20 $O/$1.txt; exit 1; }
grep -v "^{" $O/$1.txt
