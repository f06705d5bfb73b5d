# round 4, session y: bench.py at 1, 2, 3, 4 pipelined streams (d = 0 headline), two interleaved rounds
set -o pipefail
O=gpurun_out/r04_y; mkdir -p $O
for rnd in 1 2; do
  for s in 1 2 3 4; do
    timeout -k 10 120 python -u bench.py --steps 100 --warmup 20 --streams $s --no-c5 --no-cpu-baseline --no-sweep > $O/bench_s${s}_r$rnd.json 2> $O/bench_s${s}_r$rnd.err || exit $?
  done
done
echo done > $O/DONE
