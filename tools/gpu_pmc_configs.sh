#!/bin/bash
# PMC passes for every BASELINE config the bench reports (the d = 0 headline, the C3 decim
# sweep d = 1..4, C4 and the C5 many-channel launch), each config run by tools/run_lib.py on the
# product library, one counter group per rocprofv3 run (kernel-trace only, never with a trace
# domain), plus the FETCH/WRITE calibration kernel.  tools/pmc_configs.py turns the output into
# profiles/pmc_traffic.json and profiles/pmc_valu.json.  Arg: output dir.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=${1:-$R/gpurun_out/pmc_cfg}; mkdir -p $O; O=$(cd $O && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || exit $?
have() { grep -q "\b$1\b" $O/counters.txt; }
PASSES="fetch:FETCH_SIZE write:WRITE_SIZE
valu:SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAVES,SQ_INSTS_SALU,GRBM_GUI_ACTIVE,GRBM_COUNT
stall:SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAVE_CYCLES"
if have SQ_INSTS_VALU_FMA_F32 && have SQ_INSTS_VALU_ADD_F32 && have SQ_INSTS_VALU_MUL_F32; then
  PASSES="$PASSES
flop:SQ_INSTS_VALU_ADD_F32,SQ_INSTS_VALU_MUL_F32,SQ_INSTS_VALU_FMA_F32,SQ_INSTS_VALU_TRANS_F32,GRBM_GUI_ACTIVE"
fi
CONFIGS="d0|--d 0
d1|--d 1
d2|--d 2
d3|--d 3
d4|--d 4
c4|--d 1 --lsb --rand
c5|--d 4 --channels 1024 --nblk 256"
while IFS='|' read -r cfg args; do
  for p in $PASSES; do
    name=${p%%:*}; ctr=$(echo ${p#*:} | tr ',' ' ')
    timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex r2iq_ --pmc $ctr \
      -d $O/${cfg}_$name -o run -- python3 $R/tools/run_lib.py --reps 8 $args > $O/${cfg}_$name.log 2>&1 || exit $?
  done
  echo "$cfg done"
done <<< "$CONFIGS"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex calib --pmc $c \
    -d $O/calib_$c -o run -- $R/build/bin/pmc_calib > $O/calib_$c.log 2>&1 || exit $?
done
echo done > $O/DONE
