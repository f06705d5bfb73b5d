#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: 2 torchrun ranks share the card over gloo
# (SDDC_BENCH_BACKEND=gloo; RCCL refuses two ranks on one device).  Exercises bench.py's N>1
# paths end to end: time segments of one stream with their halo, channels with each
# broadcast method, barrier + max-over-ranks timing.  Arg: output dir.
set -o pipefail
O=${1:-gpurun_out/rehearsal}; mkdir -p $O
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561"
export SDDC_BENCH_BACKEND=gloo
timeout -k 10 240 $R bench.py --gpus 2 --steps 10 --warmup 3 > $O/single.log 2>&1 || exit $?
timeout -k 10 240 $R bench.py --gpus 2 --mode channels --decim-index 4 --nblk 64 --steps 5 --warmup 2 --bcast bcast > $O/channels_bcast.log 2>&1 || exit $?
timeout -k 10 240 $R bench.py --gpus 2 --mode channels --decim-index 4 --nblk 64 --steps 5 --warmup 2 --bcast sag > $O/channels_sag.log 2>&1
echo "sag rc=$?" >> $O/channels_sag.log
