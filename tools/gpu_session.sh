# one GPU session (edited per use): each step under its own limit, stop at the first failure
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfE --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_libs.py --libs build/ab/inplace.so build/ab/inpad.so build/ab/cur.so --d 0 --rounds 10 > $O/ab_inpad.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for L in inplace inpad; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq_ --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/pmc_$L -o run -- python3 $R/tools/run_lib.py --lib $R/build/ab/$L.so --reps 8 --d 0 > $O/pmc_$L.log 2>&1 || exit $?
done
echo done > $O/DONE
