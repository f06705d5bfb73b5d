"""Work partitioning for N GPUs of one node.

- Time segments (single stream, weak or strong): contiguous block ranges per
  rank; each segment carries the 4096-sample history (halo) of its first block,
  so segments are independent and outputs concatenate in order.
- Channels (C5): contiguous tune-bin ranges per rank; every rank needs the whole
  int16 batch (broadcast from the ingest rank) and computes its own channels.

The C5 input broadcast: one 128-channel shard of d = 4 runs at ~111 GS/s per
GPU, i.e. ~222 GB/s of int16 into every GPU, more than one xGMI link (~153 GB/s) carries.  So
the default broadcast is a scatter + all-gather ("sag"): the ingest rank sends 1/N of the
batch to each rank (N - 1 point-to-point transfers leave it on N - 1 different links at once),
then every rank all-gathers the N pieces, a collective that RCCL runs over all the links of
the fully connected node.  The ingest rank's outbound bytes stay ~(N-1)/N of the batch (as
for a plain broadcast) and every rank receives exactly one batch; no single link carries a
whole batch.  "bcast" keeps the one-collective form for comparison.
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


BROADCAST_METHODS = ("sag", "bcast")


def broadcast_samples(buf, src: int = 0, method: str = "sag", async_op: bool = False):
    """Send an int16 sample batch from `src` to every rank, in place.  NCCL/RCCL and gloo have
    no int16 type, so the (even-length) batch travels as its int32 view — same bytes.

    method "sag": scatter the batch in N equal pieces (piece r to rank r, in place), then
    all-gather the pieces (in place); a remainder of fewer than N words is broadcast.
    method "bcast": one broadcast collective.
    async_op: return a work handle whose wait() orders the current stream (GPU) or blocks (CPU)
    after the LAST collective of the method; collectives issued by one rank run in issue order."""
    import torch
    import torch.distributed as dist
    assert buf.dtype == torch.int16 and buf.numel() % 2 == 0 and buf.is_contiguous()
    if method not in BROADCAST_METHODS:
        raise ValueError(f"broadcast method {method!r} not in {BROADCAST_METHODS}")
    w32 = buf.view(torch.int32)
    world, rank = dist.get_world_size(), dist.get_rank()
    if method == "bcast" or world == 1:
        return dist.broadcast(w32, src=src, async_op=async_op)
    piece = w32.numel() // world
    last = None
    if piece:
        pieces = list(w32[: piece * world].view(world, piece).unbind(0))
        # the root receives its own piece into a scratch copy rather than into the slice its
        # scatter_list reads (no aliased send/receive buffers on any backend); every other rank
        # receives in place, which the all-gather below then reads in place
        mine = pieces[rank] if rank != src else torch.empty_like(pieces[rank])
        # RCCL runs one rank's collectives in issue order on its stream; gloo may run queued
        # async collectives concurrently, so there the scatter completes first
        sw = dist.scatter(mine, scatter_list=pieces if rank == src else None, src=src, async_op=async_op)
        if async_op and dist.get_backend() == "gloo":
            sw.wait()
        last = dist.all_gather_into_tensor(w32[: piece * world], mine, async_op=async_op)
    if piece * world < w32.numel():
        if last is not None and async_op and dist.get_backend() == "gloo":
            last.wait()
        last = dist.broadcast(w32[piece * world:], src=src, async_op=async_op)
    return last


def pipelined_batches(bufs, nbatches: int, src: int = 0, fill=None, method: str = "sag"):
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
        return broadcast_samples(b, src=src, method=method, async_op=True)

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
