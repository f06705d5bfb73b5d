#!/bin/bash
# Instruction-fetch counters for the persistent (variant 0) and wave (variant 3) kernels at
# d = 0: one rocprofv3 --pmc pass per counter group and variant, kernel-trace only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/icache; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for v in 0 3; do
  while read -r grp; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq --pmc $grp -d $O/v${v}_p$i -o run -- python3 $R/tools/run_variant.py --variant $v --reps 10 > $O/v${v}_p$i.log 2>&1
    rc=$?; echo "v$v p$i rc=$rc: $grp" >> $O/summary.txt
    [ $rc -ne 0 ] && exit $rc
  done <<'GROUPS'
SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_IFETCH_LEVEL
SQC_ICACHE_REQ SQC_ICACHE_MISSES
SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE
GROUPS
done
exit 0
