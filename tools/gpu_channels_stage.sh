set -o pipefail
O=gpurun_out/ch; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c5.py tests/test_gpu_cs16.py tests/test_gpu_parity.py tests/test_gpu_sweep.py -k "channel or c5 or cs16" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python tools/ab_libs.py --libs build/ab/nostage.so build/ab/stage.so build/ab/nostage.so build/ab/stage.so --d 5 6 --channels 128 --nblk 256 --rounds 8 > $O/ab_stage_128ch.txt 2>&1 || exit 1
grep -v "^{" $O/ab_stage_128ch.txt
cd /tmp && export TMPDIR=/tmp
for lib in nostage stage; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex channels_v2 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$O/pmc_w_$lib -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_libs.py --libs $GRAFT_REPO_ROOT/build/ab/$lib.so --d 6 --channels 128 --nblk 256 --rounds 2 --reps 3 > $GRAFT_REPO_ROOT/$O/pmc_w_$lib.log 2>&1 || exit 1
done
echo done
