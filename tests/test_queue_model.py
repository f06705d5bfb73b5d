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


# ---------------------------------------------------------------------------------------------
# Work stealing (ddc_queue.hpp StealSchedule, the FS kernel's A/B schedule since round 5): per
# workgroup one word (front << 16) | (BIAS + end) over its slot-weighted range; the owner claims
# with add(0x10000) past its private prefix, thieves steal the range's last frame with add(-1).
# The model keeps the kernel's pipelining: the owner's claim for frame j + 2 is issued at frame j
# (take) and read at frame j + 1 (next); a thief's scan is issued at the end of a frame, the steal
# atomic at the next frame's peek and read at its next(); a failed steal rescans (up to 3 probes).
# Every atomic and every scan load is a yield point, so the random scheduler interleaves them.
# ---------------------------------------------------------------------------------------------
BIAS = 0x4000


class StealWords:
    def __init__(self, grid):
        self.w = [0] * grid      # zero slots: "no frames left" (a fresh or dirty ring slot)
        self.a = [0] * grid

    def add(self, v, x):
        old = self.w[v]
        self.w[v] = (old + x) & 0xFFFFFFFF
        return old


def steal_front(x):
    return x >> 16


def steal_end(x):
    return (x & 0xFFFF) - BIAS


def steal_workgroup(w, nframes, grid, slotw, pub, minrem, words, out, rng):
    a = slot_split(nframes, grid, w, slotw)
    b = slot_split(nframes, grid, w + 1, slotw)
    length = b - a
    two = min(length, 2)
    P = length - pub if pub > 0 and length - pub > two else two
    S = (grid >> 6) + 1 if grid >= 128 else 1

    def cands(k):
        res = []
        for lane in range(64):
            if lane >= grid - 1:
                continue
            v = w + 1 + (k & 1) + S * lane
            v = v - grid if v >= grid else v
            v = v - grid if v >= grid else v
            res.append(v)
        return res

    yield   # the swap
    words.w[w] = (P << 16) | (BIAS + length)
    words.a[w] = a
    st = {"mode": "priv", "nx": a + 1, "pe": a + P, "own_left": length - P, "tk": None, "scan": None, "va": 0}
    frames = [a] if length > 0 else []
    if length <= 0:
        st["mode"] = "done"

    def scan(k):
        snap = [(v, words.w[v], words.a[v]) for v in cands(k)]   # sc1 loads (one snapshot per probe)
        st["scan"] = (k, snap)
        st["mode"] = "scan"

    def choose():
        k, snap = st["scan"]
        rems = [(steal_end(x) - steal_front(x), v, av) for v, x, av in snap]
        if not rems:
            st["mode"] = "done"
            return False
        m = max(r for r, _, _ in rems)
        if m < minrem:
            st["mode"] = "done"
            return False
        _, v, av = next(t for t in rems if t[0] == m)
        st["victim"], st["va"], st["mode"] = v, av, "steal"
        return True

    def stolen(old):
        fr, er = steal_front(old), steal_end(old)
        f = st["va"] + er - 1
        return f if er - 1 >= fr and f < nframes else -1

    def take_late():
        if st["mode"] not in ("done",) and st["nx"] >= st["pe"] and st["own_left"] <= 0:
            st["own_left"] = -1
            scan(0)

    if length == 1:
        take_late()
        yield
    while frames:
        f = frames.pop()
        out.append(f)
        # peek (after the frame's forward pass 1): a pending scan becomes a steal
        if st["mode"] == "scan":
            if choose():
                yield
                st["tk"] = words.add(st["victim"], -1)
        # next (inverse pass 0): the frame after this one
        fn = -1
        if st["nx"] < st["pe"]:
            fn = st["nx"]
            st["nx"] += 1
        elif st["mode"] == "own":
            old = st["tk"]
            fr, er = steal_front(old), steal_end(old)
            if fr < er and a + fr < nframes:
                st["own_left"] = er - fr - 1
                fn = a + fr
        elif st["mode"] == "steal":
            fn = stolen(st["tk"])
        if fn < 0 and st["mode"] in ("own", "steal"):
            st["own_left"] = -1
            for k in (1, 2, 3):
                yield
                scan(k)
                if not choose():
                    break
                yield
                fn = stolen(words.add(st["victim"], -1))
                if fn >= 0:
                    break
            if fn < 0:
                st["mode"] = "done"
        if fn < 0:
            break
        frames.append(fn)
        # take (inverse pass 1): the own claim for the frame after fn
        if st["mode"] != "done" and st["nx"] >= st["pe"] and st["own_left"] > 0:
            yield
            st["tk"] = words.add(w, 0x10000)
            st["mode"] = "own"
        # frame end: a thief's scan
        yield
        take_late()


@pytest.mark.parametrize("nframes,grid,slotw,pub,minrem", [
    (11 * 256, 1024, W_FS, 0, 1), (11 * 256, 1024, W_FS, 4, 2), (11 * 64, 128, W_FS, 0, 1),
    (37, 36, 0, 0, 1), (11 * 3, 8, 0, 2, 1), (11 * 40, 64, W_FS, 3, 1), (500, 96, W_FS, 0, 2)])
def test_steal_every_frame_once(nframes, grid, slotw, pub, minrem):
    for seed in range(4):
        rng = random.Random(seed * 7919 + nframes)
        words = StealWords(grid)
        outs = [[] for _ in range(grid)]
        gens = [steal_workgroup(w, nframes, grid, slotw, pub, minrem, words, outs[w], rng) for w in range(grid)]
        live = list(range(grid))
        while live:
            i = rng.randrange(len(live))
            try:
                next(gens[live[i]])
            except StopIteration:
                live.pop(i)
        done = sorted(f for o in outs for f in o)
        assert done == list(range(nframes)), f"seed {seed}: frames missing or doubled"
        stolen = sum(1 for w in range(grid) for f in outs[w]
                     if not slot_split(nframes, grid, w, slotw) <= f < slot_split(nframes, grid, w + 1, slotw))
        if seed == 0:
            print(f"{nframes} frames, {grid} workgroups: {stolen} stolen")
