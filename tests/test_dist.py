"""N>1 data paths on CPU with gloo, world_size 2-4.

- time segments (weak/strong scaling of one stream): each rank processes its own block
  range plus the 4096-sample halo; gathered outputs concatenate to the whole-stream result
  bit-exactly (blocks only depend on their own samples and the history).
- channels (C5): rank 0 owns the int16 batch and broadcasts it (the xGMI/RCCL step on the
  GPU node; gloo here); each rank computes its contiguous channel shard; the gathered
  shards equal every channel computed on one rank.
- pipelined broadcast (bench.py's C5 loop): with batch i + 1's broadcast in flight while batch
  i is used, every rank still sees every batch, in order, with the src rank's content.
- broadcast methods (shard.broadcast_samples): scatter + all-gather ("sag", the default) and
  one broadcast, at world 2, 3 and 4, blocking and async, even and uneven splits: every rank
  ends with the src rank's bytes.
The per-rank compute here is the oracle (no GPU); the partitioning, halo and collective
logic is extio_sddc_amd.shard, the same code bench.py uses on the GPUs.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from extio_sddc_amd.shard import block_shard, broadcast_samples, channel_shard, segment_samples
        from extio_sddc_amd.synth import make_stream
        from oracle import oracle as O
        if mode == "segments":
            nblk, d, tb = 5, 1, 1024
            x = make_stream(nblk, "mix")
            lo, hi = block_shard(nblk, world, rank)
            s0, s1 = segment_samples(lo, hi)
            y = O.r2iq(x[s0:s1], hi - lo, d, tb) if hi > lo else np.zeros(0, np.complex128)
            parts = [None] * world
            dist.all_gather_object(parts, (lo, hi, y))
            if rank == 0:
                full = O.r2iq(x, nblk, d, tb)
                cat = np.concatenate([p[2] for p in sorted(parts, key=lambda p: p[0])])
                q.put(bool(np.array_equal(cat, full)) and sum(p[1] - p[0] for p in parts) == nblk)
        elif mode.startswith("bcast-"):
            # every broadcast method: byte-identical batches on every rank, in order, incl. sizes
            # that do not split evenly over the ranks (the remainder travels by broadcast)
            from extio_sddc_amd.shard import broadcast_samples, pipelined_batches
            method = mode.split("-", 1)[1]
            ok = True
            for n16 in (2 * 65536 + 4096, 2 * 7 * world + 2, 2):
                ref = torch.from_numpy(make_stream(4, "uniform")[:n16].copy())
                b = ref.clone() if rank == 0 else torch.zeros(n16, dtype=torch.int16)
                broadcast_samples(b, src=0, method=method)
                ok &= bool(torch.equal(b, ref))
                b2 = ref.clone() if rank == 0 else torch.full((n16,), 7, dtype=torch.int16)
                broadcast_samples(b2, src=0, method=method, async_op=True).wait()
                ok &= bool(torch.equal(b2, ref))
            stream = make_stream(8, "uniform")
            bufs = [torch.zeros(4096 + 65536, dtype=torch.int16) for _ in range(2)]

            def fill(b, i):
                b.copy_(torch.from_numpy(stream[i * 65536:i * 65536 + b.numel()]))
            seen = [b.numpy().copy() for b in pipelined_batches(bufs, 6, src=0, fill=fill, method=method)]
            ok &= len(seen) == 6 and all(np.array_equal(seen[i], stream[i * 65536:i * 65536 + seen[i].size])
                                         for i in range(6))
            flags = [None] * world
            dist.all_gather_object(flags, ok)
            if rank == 0:
                q.put(all(flags))
        elif mode == "pipelined":
            from extio_sddc_amd.shard import pipelined_batches
            n = 5
            bufs = [torch.zeros(4096 + 2 * 65536, dtype=torch.int16) for _ in range(2)]
            stream = make_stream(2 * n, "uniform")

            def fill(b, i):   # batch i = blocks [2i, 2i + 2) of one stream, with their halo
                b.copy_(torch.from_numpy(stream[i * 2 * 65536:i * 2 * 65536 + b.numel()]))
            seen = [b.numpy().copy() for b in pipelined_batches(bufs, n, src=0, fill=fill)]
            ok = len(seen) == n and all(np.array_equal(seen[i], stream[i * 2 * 65536:i * 2 * 65536 + seen[i].size])
                                        for i in range(n))
            flags = [None] * world
            dist.all_gather_object(flags, ok)
            if rank == 0:
                q.put(all(flags))
        else:
            nblk, d, nch = 2, 4, 6
            tbs = [4 * (97 * c % 1024) for c in range(nch)]
            buf = torch.zeros(4096 + nblk * 65536, dtype=torch.int16)
            if rank == 0:
                buf.copy_(torch.from_numpy(make_stream(nblk, "uniform")))
            broadcast_samples(buf, src=0)
            x = buf.numpy()
            lo, hi = channel_shard(nch, world, rank)
            H = O.filter_bank(1.0)
            mine = [O.r2iq(x, nblk, d, tbs[c], H=H) for c in range(lo, hi)]
            parts = [None] * world
            dist.all_gather_object(parts, (lo, mine))
            if rank == 0:
                got = [y for p in sorted(parts, key=lambda p: p[0]) for y in p[1]]
                ok = len(got) == nch and all(np.array_equal(got[c], O.r2iq(x, nblk, d, tbs[c], H=H))
                                             for c in range(nch))
                q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "segments"), (2, "channels"), (2, "pipelined"), (2, "bcast-sag"),
                                        (4, "bcast-sag"), (3, "bcast-sag"), (2, "bcast-bcast")])
def test_multi_rank_gloo(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def test_shard_partitions():
    from extio_sddc_amd.shard import block_shard, channel_shard, segment_samples
    for n in (1, 7, 2048):
        for w in (1, 2, 3, 8):
            spans = [block_shard(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
    assert channel_shard(1024, 8, 3) == (384, 512)
    assert segment_samples(2, 5) == (2 * 65536, 4096 + 5 * 65536)
