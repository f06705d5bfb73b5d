# one GPU session (edited per use): each step under its own limit, stop at the first failure
set -o pipefail
O=gpurun_out/r05_k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_cs16.py tests/test_gpu_sweep.py -m gpu -q -rfE --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_libs.py --libs build/ab/inplace.so build/ab/chkey.so --d 4 5 6 --nblk 256 --channels 1024 --rounds 8 > $O/ab_c5.log 2>&1 || exit $?
(cd /tmp && export TMPDIR=/tmp && for L in inplace chkey; do timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq_ --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/pmc_$L -o run -- python3 $GRAFT_REPO_ROOT/tools/run_lib.py --lib $GRAFT_REPO_ROOT/build/ab/$L.so --reps 8 --d 4 --channels 1024 --nblk 256 > $O/pmc_$L.log 2>&1 || exit $?; done) || exit $?
echo done > $O/DONE
