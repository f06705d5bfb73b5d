"""Work partitioning for N GPUs of one node.

- Time segments (single stream, weak or strong): contiguous block ranges per
  rank; each segment carries the 4096-sample history (halo) of its first block,
  so segments are independent and outputs concatenate in order.
- Channels (C5): contiguous tune-bin ranges per rank; every rank needs the whole
  int16 batch (broadcast from the ingest rank) and computes its own channels.
"""
from __future__ import annotations

HALF_FFT = 4096
BLOCK = 65536


def block_shard(nblk: int, world: int, rank: int) -> tuple[int, int]:
    """Blocks [lo, hi) of an nblk-block stream owned by `rank` (balanced, contiguous)."""
    base, extra = divmod(nblk, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def segment_samples(lo: int, hi: int) -> tuple[int, int]:
    """Sample range [s0, s1) of the [history | blocks] stream a block range needs:
    its own blocks plus the 4096-sample halo in front (Core/fft_mt_r2iq_impl.hpp:32)."""
    return lo * BLOCK, HALF_FFT + hi * BLOCK


def channel_shard(nch: int, world: int, rank: int) -> tuple[int, int]:
    """Channels [lo, hi) computed by `rank`."""
    return block_shard(nch, world, rank)


def broadcast_samples(buf, src: int = 0) -> None:
    """Broadcast an int16 sample batch from `src` to every rank.  NCCL/RCCL and gloo have
    no int16 type, so the (even-length) batch travels as its int32 view — same bytes."""
    import torch
    import torch.distributed as dist
    assert buf.dtype == torch.int16 and buf.numel() % 2 == 0 and buf.is_contiguous()
    dist.broadcast(buf.view(torch.int32), src=src)


def pipelined_batches(bufs, nbatches: int, src: int = 0, fill=None):
    """Yield nbatches input batches, bufs[i % 2] for batch i, every rank receiving the src
    rank's batch by broadcast, with the broadcast of batch i + 1 already in flight while the
    caller processes batch i (overlap the xGMI broadcast with the compute).

    nbatches: None = unbounded (the caller stops with close(), which waits for the broadcast
    already in flight, so every rank leaves with its collectives matched).
    bufs: two equal int16 buffers.  fill(buf, i): on the src rank, writes batch i into buf
    before it is sent (None: the buffers already hold the batch, as in bench.py).
    Ordering on a GPU: an async collective first waits for the work queued on the current
    stream, so the broadcast into bufs[(i + 1) % 2] starts after batch i - 1 (the previous user
    of that buffer) was processed; work.wait() makes the current stream wait for the data.
    """
    import torch
    import torch.distributed as dist
    assert len(bufs) == 2 and all(b.dtype == torch.int16 and b.numel() % 2 == 0 for b in bufs)
    rank = dist.get_rank()

    def send(i):
        b = bufs[i % 2]
        if fill is not None and rank == src:
            fill(b, i)
        return dist.broadcast(b.view(torch.int32), src=src, async_op=True)

    if nbatches is not None and nbatches <= 0:
        return
    work = send(0)
    i = 0
    try:
        while nbatches is None or i < nbatches:
            work.wait()
            work = None
            if nbatches is None or i + 1 < nbatches:
                work = send(i + 1)
            yield bufs[i % 2]
            i += 1
    finally:   # close(): the prefetched broadcast still completes on every rank
        if work is not None:
            work.wait()
