"""CPU model of the single-channel kernels' frame schedule (extio_sddc_amd/csrc/ddc_queue.hpp):
every frame of a launch is processed exactly once, for any interleaving of the workgroups'
device-scope atomics.

The model restates fs_shard_lo / fs_shard_nwg / fs_shard_pre, FsQueue (take / peek / resolve with
its all-shard scan / set_shard) and FrameSchedule<LA> (static prefix + dynamic suffix, lookahead LA = 1 for the d = 0
fused-split kernel, 2 for the persistent and tail-wave kernels) line by line, and drives `grid`
workgroups as coroutines that yield before every atomic, so a seeded random scheduler explores
the orders in which the shard counters are incremented.  The GPU tests check the same property
on the hardware (tests/test_gpu_queue.py: NaN-filled outputs at 256 and 2048 blocks, compared
with the f64 oracle); this covers the small and ragged geometries and many orders.
"""
from __future__ import annotations

import random

import pytest

SHARDS = 8


def shard_lo(nframes, s):
    return (nframes * s) >> 3


def shard_nwg(grid, s):
    return (grid - s + SHARDS - 1) // SHARDS


def shard_pre(nframes, grid, s, per):
    cnt = shard_lo(nframes, s + 1) - shard_lo(nframes, s)
    return min(cnt, per * shard_nwg(grid, s))


def kstat_of(nframes, grid, pct, lo=1):   # frame_schedule_kstat
    return max(lo, nframes * pct // (100 * grid))


class Counters:
    """the queue slot: one counter per shard (device-scope atomics)"""

    def __init__(self):
        self.c = [0] * SHARDS

    def add(self, s):
        old = self.c[s]
        self.c[s] += 1
        return old


def shard_pairs(cnt, grid, s, ts):   # fs_shard_pairs
    n = ts * shard_nwg(grid, s)
    return (cnt - n) >> 1 if cnt > n else 0


def workgroup(w, nframes, grid, kstat, LA, ctr, out, ts=4096):
    """one workgroup's frame sequence; yields before each atomic"""
    s_home = w & (SHARDS - 1)
    q = {"shn": 0, "lo": 0, "np": 0, "ntk": 0, "tk": None, "pv": None}

    def dyn(s):
        first = shard_lo(nframes, s) + shard_pre(nframes, grid, s, kstat)
        return first, shard_lo(nframes, s + 1) - first

    def set_shard(sh):
        q["shn"] = sh
        s = (s_home + sh) & (SHARDS - 1)
        q["lo"], cnt = dyn(s)
        if sh >= SHARDS:
            cnt = 0
        q["np"] = shard_pairs(cnt, grid, s, ts)
        q["ntk"] = cnt - q["np"]

    def take():
        if q["shn"] < SHARDS:
            yield
            q["tk"] = ctr.add((s_home + q["shn"]) & (SHARDS - 1))
        else:
            q["tk"] = 0   # out of the slot's range: no access

    def peek():
        q["pv"] = q["tk"]

    def resolve():   # -> (frame, second)
        dry = q["pv"] >= q["ntk"]
        while dry and q["shn"] < SHARDS:
            yield   # the scan: lanes 0..7 add 0 to one counter each (one device-scope atomic)
            live = 0
            for l in range(SHARDS):
                _, cnt = dyn(l)
                if ctr.c[l] < cnt - shard_pairs(cnt, grid, l, ts):
                    live |= 1 << l
            rot = ((live >> s_home) | (live << (SHARDS - s_home))) & 0xFF
            set_shard((rot & -rot).bit_length() - 1 if rot else SHARDS)
            if not rot:
                break
            yield from take()
            q["pv"] = q["tk"]
            dry = q["pv"] >= q["ntk"]
        if dry:
            return -1, -1
        pv, lo, np_ = q["pv"], q["lo"], q["np"]
        return (lo + 2 * pv, lo + 2 * pv + 1) if pv < np_ else (lo + np_ + pv, -1)

    nwg = shard_nwg(grid, s_home)
    slo = shard_lo(nframes, s_home) + w // SHARDS
    pre = shard_pre(nframes, grid, s_home, kstat)
    kw = (pre - w // SHARDS + nwg - 1) // nwg if pre > w // SHARDS else 0
    set_shard(0)
    pend = -1
    known = []
    for i in range(LA):   # first(i)
        if pend >= 0:
            known.append(pend)
            pend = -1
        elif i < kw:
            known.append(slo + i * nwg)
        else:
            yield from take()
            peek()
            f, pend = yield from resolve()
            known.append(f)
    if LA >= kw and pend < 0:
        yield from take()
    j = 0
    while known[0] >= 0:
        out.append(known[0])
        if j + LA >= kw and pend < 0:   # peek()
            peek()
        if pend >= 0:                   # next()
            fn, pend = pend, -1
        elif j + LA < kw:
            fn = slo + (j + LA) * nwg
        else:
            fn, pend = yield from resolve()
        if pend < 0 and j + LA + 1 >= kw:
            yield from take()
        j += 1
        known = known[1:] + [fn]


def run(nframes, grid, pct, LA, seed, ts=4096):
    ctr = Counters()
    out = []
    kstat = kstat_of(nframes, grid, pct, LA)
    gens = [workgroup(w, nframes, grid, kstat, LA, ctr, out, ts) for w in range(grid)]
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
    (11, 11), (22, 22), (33, 33), (55, 55), (11 * 64, 704), (11 * 93, 1023 if 11 * 93 > 1023 else 11 * 93),
    (11 * 256, 1024), (11 * 300, 1000), (11 * 2048 // 8, 1024),
]


@pytest.mark.parametrize("nframes,grid", GEOMETRIES)
@pytest.mark.parametrize("pct", [0, 75, 100])
@pytest.mark.parametrize("LA", [1, 2])
@pytest.mark.parametrize("ts", [0, 1, 2, 4096])
def test_every_frame_exactly_once(nframes, grid, pct, LA, ts):
    for seed in range(2):
        out, _ = run(nframes, grid, pct, LA, seed, ts)
        assert sorted(out) == list(range(nframes)), (nframes, grid, pct, LA, seed, ts)


def test_pair_tickets_halve_the_dequeues():
    """headline size, first frames static: tail singles 2 take ~half the tickets of all-singles"""
    nframes, grid = 11 * 2048, 1024
    _, c1 = run(nframes, grid, 0, 1, 7, ts=4096)
    _, c2 = run(nframes, grid, 0, 1, 7, ts=2)
    assert sum(c2.c) < 0.62 * sum(c1.c), (sum(c1.c), sum(c2.c))


def test_static_share_takes_few_tickets():
    """at the headline size (2048 blocks = 22528 frames on 1024 workgroups) and 75 % static, the
    workgroups take about a third as many tickets as frames (the dynamic quarter + one dry ticket
    per workgroup), against one per frame with no static prefix"""
    nframes, grid = 11 * 2048, 1024
    ctr = Counters()
    out = []
    kstat = kstat_of(nframes, grid, 75)
    gens = [workgroup(w, nframes, grid, kstat, 1, ctr, out) for w in range(grid)]
    rng = random.Random(5)
    live = list(range(grid))
    while live:
        i = rng.choice(live)
        try:
            next(gens[i])
        except StopIteration:
            live.remove(i)
    assert sorted(out) == list(range(nframes))
    assert sum(ctr.c) < 0.35 * nframes


def test_last_frame_needs_one_scan():
    """a workgroup that finds every shard dry returns after one scan, not a walk of the shards"""
    nframes, grid = 11 * 64, 704
    ctr = Counters()
    out = []
    kstat = kstat_of(nframes, grid, 75)
    g = workgroup(0, nframes, grid, kstat, 1, ctr, out)
    for s in range(SHARDS):   # every ticket already handed out
        ctr.c[s] = shard_lo(nframes, s + 1) - shard_lo(nframes, s)
    steps = sum(1 for _ in g)
    assert out == [shard_lo(nframes, 0)]   # its static frame only
    assert steps <= 3   # the ticket taken ahead, one scan, (no more)


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
