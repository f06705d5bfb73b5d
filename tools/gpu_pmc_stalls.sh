#!/bin/bash
# Stall-breakdown PMC passes (kernel-trace only, one counter group per run) for the d=0
# single-channel kernel of the current tree.  Arg: TAG (output under gpurun_out/TAG).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; TAG=${1:-stalls}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/bench.py --steps 5 --warmup 2 --warmup-ms 0 --no-cpu-baseline --no-sweep"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq_persistent \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  -d $O/p1 -o run -- $P > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq_persistent \
  --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
  -d $O/p2 -o run -- $P > $O/p2.log 2>&1 || exit $?
echo done > $O/DONE
