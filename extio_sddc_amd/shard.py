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
