#!/bin/bash
# The reference's benchmark_test procedure (unittest/benchmark_test.cpp ThroughputBenchmark and
# HighRateThroughputBenchmark) through the reference's unchanged RadioHandler and this repo's
# drop-in fft_mt_r2iq (oracle/_ref/radiohandler_harness --benchmark, built by
# `make -C oracle radiohandler` in the build container).  3 s per srate_idx, on the hip and cpu
# backends; JSON lines into OUT/benchmark_test.jsonl.  Arg: output dir.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=${1:-$R/gpurun_out/e2e}; mkdir -p $O
H=${HARNESS:-$R/oracle/_ref/radiohandler_harness}   # HARNESS: a variant build of the harness
test -x $H || { echo "missing $H (make -C oracle radiohandler)"; exit 2; }
: > $O/benchmark_test.jsonl
for be in hip cpu; do
  SDDC_DDC_BACKEND=$be timeout -k 10 60 $H --benchmark 3 64000000 >> $O/benchmark_test.jsonl || exit $?
done
SDDC_DDC_BACKEND=hip timeout -k 10 60 $H --benchmark 3 128000000 0 5 | sed 's/^{/{"adc_hz": 128000000, /' >> $O/benchmark_test.jsonl || exit $?
cat $O/benchmark_test.jsonl
