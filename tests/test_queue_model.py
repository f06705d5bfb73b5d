"""CPU model of the single-channel kernels' frame schedule (extio_sddc_amd/csrc/ddc_queue.hpp):
every frame of a launch is processed exactly once, for any interleaving of the workgroups'
device-scope atomics.

The model restates slot_split, FsQueue (take / peek / resolve with its all-shard scan /
set_shard) and FrameSchedule<LA> (a slot-weighted static split of the first ns frames, then the
dynamic queue over the rest; lookahead LA = 1 for the d = 0 fused-split kernel, 2 for the
persistent kernel) line by line, and drives `grid` workgroups as coroutines that yield before
every atomic, so a seeded random scheduler explores the orders in which the shard counters are
incremented.  The GPU tests check the same property on the hardware (tests/test_gpu_queue.py:
NaN-filled outputs at 256 and 2048 blocks, compared with the f64 oracle); this covers the small
and ragged geometries and many orders.
"""
from __future__ import annotations

import random

import pytest

SHARDS = 8
W_FS = 29 | 25 << 8 | 19 << 16 | 15 << 24   # ddc_kernels.h kFsSlotWeights


def slot_split(nframes, G, v, slotw):   # ddc_queue.hpp slot_split
    if slotw == 0 or G & 3:
        return nframes * v // G
    Q = G >> 2
    q, i = v // Q, v - (v // Q) * Q
    sw = tot = 0
    for k in range(4):
        wk = (slotw >> (8 * k)) & 0xFF
        tot += Q * wk
        if k < q:
            sw += Q * wk
        elif k == q:
            sw += i * wk
    return nframes * sw // tot



class Counters:
    """the queue slot: one counter per shard (device-scope atomics)"""

    def __init__(self):
        self.c = [0] * SHARDS

    def add(self, s, v=1):
        old = self.c[s]
        self.c[s] += v
        return old


def workgroup(w, nframes, ns, grid, slotw, LA, ctr, out):
    """one workgroup's frame sequence; yields before each atomic"""
    home = w & (SHARDS - 1)
    nd = nframes - ns
    q = {"shn": 0, "lo": 0, "cnt": 0, "tk": None, "pv": None}

    def shard_lo(s):
        return ns + ((nd * s) >> 3)

    def set_shard(sh):
        q["shn"] = sh
        s = (home + sh) & (SHARDS - 1)
        q["lo"] = shard_lo(s)
        q["cnt"] = shard_lo(s + 1) - q["lo"] if sh < SHARDS else 0

    def take():
        if q["shn"] < SHARDS:
            yield
            q["tk"] = ctr.add((home + q["shn"]) & (SHARDS - 1))
        else:
            q["tk"] = 0   # out of the slot's range: no access

    def peek():
        q["pv"] = q["tk"]

    def resolve():
        dry = q["pv"] >= q["cnt"]
        while dry and q["shn"] < SHARDS:
            yield   # the scan: lanes 0..7 add 0 to one counter each (one device-scope atomic)
            live = 0
            for l in range(SHARDS):
                if ctr.c[l] < shard_lo(l + 1) - shard_lo(l):
                    live |= 1 << l
            rot = ((live >> home) | (live << (SHARDS - home))) & 0xFF
            set_shard((rot & -rot).bit_length() - 1 if rot else SHARDS)
            if not rot:
                break
            yield from take()
            q["pv"] = q["tk"]
            dry = q["pv"] >= q["cnt"]
        return -1 if dry else q["lo"] + q["pv"]

    a, b = slot_split(ns, grid, w, slotw), slot_split(ns, grid, w + 1, slotw)
    set_shard(0)
    known = []
    for i in range(LA):   # init
        if a + i < b:
            known.append(a + i)
        else:
            yield from take()
            peek()
            known.append((yield from resolve()))
    rem, nxt = b - a - LA, a + LA
    if rem <= 0:
        yield from take()
    while known[0] >= 0:
        out.append(known[0])
        if rem <= 0:        # peek() at the frame top
            peek()
        if rem > 0:         # next()
            fn, nxt = nxt, nxt + 1
        else:
            fn = yield from resolve()
        rem -= 1
        if rem <= 0:        # take() behind the frame's last loads
            yield from take()
        known = known[1:] + [fn]


def run(nframes, grid, pct, LA, seed, slotw=W_FS):
    ctr = Counters()
    out = []
    ns = nframes * pct // 100
    gens = [workgroup(w, nframes, ns, grid, slotw, LA, ctr, out) for w in range(grid)]
    rng = random.Random(seed)
    live = list(range(grid))
    while live:
        i = rng.choice(live)
        try:
            next(gens[i])
        except StopIteration:
            live.remove(i)
    return out, ctr


GEOMETRIES = [
    # nframes (11 x blocks), grid (min(1024, nframes))
    (11, 11), (22, 22), (33, 33), (55, 55), (11 * 64, 704), (11 * 93, 1020),
    (11 * 256, 1024), (11 * 300, 1000), (11 * 2048 // 8, 1024),
]


@pytest.mark.parametrize("nframes,grid", GEOMETRIES)
@pytest.mark.parametrize("pct", [0, 40, 85, 100])
@pytest.mark.parametrize("LA", [1, 2])
@pytest.mark.parametrize("slotw", [0, W_FS])
def test_every_frame_exactly_once(nframes, grid, pct, LA, slotw):
    for seed in range(2):
        out, _ = run(nframes, grid, pct, LA, seed, slotw)
        assert sorted(out) == list(range(nframes)), (nframes, grid, pct, LA, seed, slotw)


def test_static_share_takes_few_tickets():
    """at the headline size (2048 blocks = 22528 frames on 1024 workgroups) and 85 % static, the
    workgroups take about a quarter as many tickets as frames (the dynamic 15 % + one dry ticket
    and one scan per workgroup)"""
    nframes, grid = 11 * 2048, 1024
    out, ctr = run(nframes, grid, 85, 1, 5)
    assert sorted(out) == list(range(nframes))
    assert sum(ctr.c) < 0.25 * nframes


def test_last_frame_needs_one_scan():
    """a workgroup that finds every shard dry returns after one scan, not a walk of the shards"""
    nframes, grid = 11 * 256, 1024
    ns = nframes * 85 // 100
    ctr = Counters()
    for s in range(SHARDS):   # every ticket already handed out
        ctr.c[s] = (ns + (((nframes - ns) * (s + 1)) >> 3)) - (ns + (((nframes - ns) * s) >> 3))
    out = []
    g = workgroup(0, nframes, ns, grid, 0, 1, ctr, out)
    steps = sum(1 for _ in g)
    assert out == list(range(slot_split(ns, grid, 1, 0)))   # its static frames only
    assert steps <= 3   # the ticket taken ahead, one scan (and the dry ticket's take)


@pytest.mark.parametrize("nframes,G", [(11 * 2048, 1024), (11 * 256, 1024), (11 * 93, 1020), (11 * 64, 704), (4, 4), (11, 11)])
@pytest.mark.parametrize("slotw", [0, 27 | 24 << 8 | 20 << 16 | 16 << 24, 29 | 25 << 8 | 19 << 16 | 15 << 24])
def test_slot_split_partitions_the_frames(nframes, G, slotw):
    """the slot-weighted static split (d >= 3): contiguous ranges that cover every frame once, in
    the slots' proportions"""
    starts = [slot_split(nframes, G, v, slotw) for v in range(G + 1)]
    assert starts[0] == 0 and starts[-1] == nframes
    assert all(a <= b for a, b in zip(starts, starts[1:]))
    if slotw and G % 4 == 0 and nframes >= 4 * G:
        Q = G // 4
        per = [starts[(q + 1) * Q] - starts[q * Q] for q in range(4)]
        w = [(slotw >> (8 * k)) & 0xFF for k in range(4)]
        for q in range(4):
            assert abs(per[q] / nframes - w[q] / sum(w)) < 1e-3
