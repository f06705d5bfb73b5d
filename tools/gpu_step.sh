#!/bin/bash
# One GPU-box session of steps, each under its own time limit, stopping at the first crash-like
# exit (124/134/137/139): GPU tests (optional), an interleaved A/B of libraries, a bench line.
#   tools/gpu_step.sh TAG [--tests] [--testsel FILES] [--ab "ab_libs args"] [--stamps "fs_stamps args"]
#                         [--pmc "LIBS" "run_lib args"] [--bench] [--prof]
#   (options repeat, in the order given; each --ab writes ab<N>.log, each --pmc pmc<N>/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p $O
nab=0; npmc=0
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
while [ $# -gt 0 ]; do
  case "$1" in
    --tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; crashed $rc && exit $rc ;;
    --testsel)
      timeout -k 10 600 python -u -m pytest $2 -m gpu -q -rfE --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1
      rc=$?; echo "pytest rc=$rc" >> $O/pytest_sel.log; crashed $rc && exit $rc; shift ;;
    --ab)
      nab=$((nab + 1))
      timeout -k 10 600 python -u tools/ab_libs.py $2 > $O/ab$nab.log 2>&1
      rc=$?; echo "ab rc=$rc" >> $O/ab$nab.log; crashed $rc && exit $rc; shift ;;
    --pmc)
      # PMC passes (stalls, LDS conflicts, VALU issue) of build/ab libraries: --pmc "LIBS" "run_lib args"
      npmc=$((npmc + 1))
      timeout -k 10 900 tools/gpu_pmc_libs.sh $TAG/pmc$npmc "$2" $3 > $O/pmc$npmc.log 2>&1
      rc=$?; echo "pmc rc=$rc" >> $O/pmc$npmc.log; crashed $rc && exit $rc; shift 2 ;;
    --stamps)
      timeout -k 10 300 python -u tools/fs_stamps.py $2 >> $O/stamps.log 2>&1
      rc=$?; echo "stamps rc=$rc" >> $O/stamps.log; crashed $rc && exit $rc; shift ;;
    --bench)
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1
      rc=$?; echo "bench rc=$rc" >> $O/bench.log; crashed $rc && exit $rc ;;
    --prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1)
      rc=$?; echo "prof rc=$rc" >> $O/trace.log; crashed $rc && exit $rc ;;
  esac
  shift
done
echo done > $O/DONE
