set -o pipefail
O=gpurun_out/r05_zr; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfE --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for tb in 0 256 3840 1024; do
  timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/head.so build/ab/zr.so --d 0 --tunebin $tb --rounds 12 --reps 10 --input bench > $O/ab_tb$tb.log 2>&1 || exit $?
done
echo done > $O/DONE
