#!/bin/bash
# Copy a tools/gpu_evidence.sh run (gpurun_out/TAG) into profiles/DEST and rebuild the counter
# summaries bench.py reads (profiles/pmc_traffic.json, profiles/pmc_valu.json) from its PMC
# passes with tools/pmc_configs.py.
#   bash tools/save_evidence.sh r05_final r05/final
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/gpurun_out/$1; D=$R/profiles/$2
mkdir -p $D
tail -n 1 $S/bench.log > $D/bench_line.json
grep -o "{\"metric.*" $S/trace.log > $D/bench_line_traced.json
cp "$(find $S/trace -name '*kernel_stats.csv' | head -n 1)" $D/bench_kernel_stats.csv
if [ -f $S/pytest_gpu.log ]; then grep -v "^\s*$" $S/pytest_gpu.log | tail -n 5 > $D/pytest_gpu.txt; fi
if [ -f $S/smoke.log ]; then cp $S/smoke.log $D/smoke.txt; fi
if [ -d $S/pmc ]; then
  for d in $S/pmc/*/; do
    n=$(basename $d); mkdir -p $D/pmc_cfg/$n
    for f in counter_collection kernel_trace; do
      g=$(find $d -name "*_$f.csv" | head -n 1); [ -z "$g" ] || cp "$g" $D/pmc_cfg/$n/run_$f.csv
    done
  done
  (cd $R && python3 tools/pmc_configs.py $D/pmc_cfg profiles/$2/pmc_cfg)
fi
echo "saved $S -> $D"
