# one GPU session (edited per use): each step under its own limit, stop at the first failure
set -o pipefail
O=gpurun_out/r05_i; mkdir -p $O
SDDC_PARITY_RECORD=$O/floor.jsonl timeout -k 10 300 python -u -m pytest tests/test_gpu_floor.py -m gpu -q -s --timeout 200 --timeout-method thread > $O/floor.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfE --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/ab_libs.py --libs build/ab/inplace.so build/ab/anchor.so --d 1 2 3 4 5 6 --rounds 8 > $O/ab_anchor.log 2>&1 || exit $?
echo done > $O/DONE
