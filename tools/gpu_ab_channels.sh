set -o pipefail
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_cs16.py tests/test_gpu_parity.py tests/test_gpu_sweep.py -k "channel or c5 or cs16" > $O/st_pytest.log 2>&1 || { tail -30 $O/st_pytest.log; exit 1; }
tail -1 $O/st_pytest.log
timeout -k 10 300 python tools/ab_libs.py --libs build/ab/st128.so build/ab/st256.so build/ab/st128.so build/ab/st256.so --d 4 --channels 1024 --nblk 256 --rounds 6 > $O/st_c5.txt 2>&1 || exit 1
grep -v "^{" $O/st_c5.txt
timeout -k 10 300 python tools/ab_libs.py --libs build/ab/st128.so build/ab/st256.so build/ab/st128.so build/ab/st256.so --d 4 --channels 128 --nblk 256 --rounds 8 > $O/st_128.txt 2>&1 || exit 1
grep -v "^{" $O/st_128.txt
