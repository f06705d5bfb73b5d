#!/bin/bash
# Stall/issue PMC passes (kernel-trace only, one counter group per run) for the single-channel
# kernels of several build/ab libraries.  Args: TAG "lib names" [run_lib args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; TAG=$1; LIBS=$2; shift 2; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in $LIBS; do
  P="python3 $R/tools/run_lib.py --lib $R/build/ab/$n.so --reps 10 $*"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq_ \
    --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    -d $O/${n}_p1 -o run -- $P > $O/${n}_p1.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq_ \
    --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
    -d $O/${n}_p2 -o run -- $P > $O/${n}_p2.log 2>&1 || exit $?
done
echo done > $O/DONE
