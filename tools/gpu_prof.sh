#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, --kernel-trace only; never with
# sys/runtime traces) + one kernel-trace --stats run, on a short bench.  Args: TAG [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}; shift
BARGS="$@"
[ -z "$BARGS" ] && BARGS="--steps 5 --warmup 2 --no-cpu-baseline"
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $BARGS > $OUT/trace.log 2>&1
rc=$?; crashed $rc && exit $rc
i=0
while read -r grp; do
  i=$((i+1))
  [ -z "$grp" ] && continue
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex 'r2iq' --pmc $grp -d $OUT/pmc$i -o run -- python3 $R/bench.py $BARGS > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc: $grp" >> $OUT/summary.txt
  crashed $rc && exit $rc
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32
SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH
GROUPS
exit 0
