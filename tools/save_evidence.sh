#!/bin/bash
# Copy a tools/gpu_evidence.sh run (gpurun_out/TAG) into profiles/DEST and rebuild the counter
# summaries bench.py reads (profiles/pmc_traffic.json, profiles/pmc_valu.json).
#   bash tools/save_evidence.sh r02_c r02/evidence_c
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=$R/gpurun_out/$1; D=$R/profiles/$2
mkdir -p $D
tail -n 1 $S/bench.log > $D/bench_line.json
grep -o "{\"metric.*" $S/trace.log > $D/bench_line_traced.json
cp $S/trace/run_kernel_stats.csv $D/bench_kernel_stats.csv
grep -v "^\s*$" $S/pytest_gpu.log | tail -n 5 > $D/pytest_gpu.txt
cp $S/smoke.log $D/smoke.txt
for c in FETCH_SIZE WRITE_SIZE; do
  cp $S/pmc_$c/run_counter_collection.csv $D/pmc_$c.csv
  cp $S/calib_$c/run_counter_collection.csv $D/calib_$c.csv
done
cp $S/pmc_valu/run_counter_collection.csv $D/pmc_valu.csv
python3 $R/tools/pmc_traffic.py $S profiles/$2 > /dev/null
python3 $R/tools/pmc_valu.py $S/pmc_valu profiles/$2 > /dev/null
echo "saved $S -> $D"
