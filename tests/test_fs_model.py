"""The d = 0 fused-split kernel's algorithm (ddc_fs.hip, r2iq_fs_kernel), modelled step
by step in numpy (tools/fs_model.py), against the f64 oracle: the lane-paired split (mirror
from lane ^ 1, register 15 - k), the inverse on absolute bins and the tune shift as the output
modulation (lane factor g_t + quarter turns).  Also checks the committed lane permutation."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import fs_model as M  # noqa: E402
import fs_perm as P  # noqa: E402
from oracle import oracle as O  # noqa: E402
from extio_sddc_amd.synth import make_stream  # noqa: E402


def test_perm_header_is_a_lane_paired_permutation():
    cols = P.read_header()
    assert P.valid(cols)
    # the il272 layout's I0 stores, F2 loads and F2 twiddle-base loads (W^c at c + [c >= 128]):
    # conflict-free
    assert P.conflicts(cols) == P.BEST[P.LAYOUT] == (0, 0, 0)
    # the unpadded twiddle table (key c mod 32) would not be: pairs c, 256 - c = 0 mod 16 collide
    c = np.asarray(cols)
    assert _conflicts(c, 32) > 0 and _conflicts(c + (c >= 128), 32) == 0


def _slot(R, j):
    return 272 * (R >> 4) + (R >= 128) + 34 * ((R & 15) >> 1) + (R & 1) + 2 * j   # ddc_fs.hip fs_slot


# The in-place LDS layout of the FS kernel (round 6, il272): every exchange's writer stores into
# exactly the slots its threads read in the previous exchange, so only the four read-after-write
# barriers remain.  (thread, register) -> (element, slot) of each store and load, as in ddc_fs.hip.
def _layout(perm):
    t = np.arange(256)[:, None]
    r = np.arange(16)[None, :]
    c = np.asarray(perm)[:, None]
    u = 2 * (t >> 5) + (t & 1)                                        # F1 / I1 pair lane: row u,
    j = (t >> 1) & 15                                                 # column j (fs_pair_lane)
    assert sorted((16 * u + j).ravel().tolist()) == list(range(256))
    fb = _slot(t, r)                                                  # F0 stores, I2 loads
    bb = _slot(16 * r + u, j)                                         # F1 / I1 loads and stores
    cb = _slot(16 * (c >> 4) + r, c & 15)                             # F2 loads, I0 stores
    return [
        # (name, store element, store slot, load element, load slot): element 16 R + j of the
        # exchange's row R, column j, numbered by the writer
        ("F0->F1", 16 * t + r, fb, 16 * (16 * r + u) + j, bb),
        ("F1->F2", 256 * u + 16 * r + j, bb, c + 256 * r, cb),
        ("I0->I1", 16 * c + r, cb, 256 * r + 16 * j + u, bb),
        ("I1->I2", 256 * j + 16 * r + u, bb, t + 256 * r, fb),
    ]


def test_inplace_layout_delivers_every_element():
    for name, se, ss, le, ls in _layout(P.read_header()):
        slot = {}
        for e, s in zip(se.ravel(), ss.ravel()):
            assert e not in slot and s not in slot.values(), name
            slot[int(e)] = int(s)
        assert sorted(slot) == list(range(4096)), name
        assert max(slot.values()) < 4352, name                 # kFsLds
        for e, s in zip(le.ravel(), ls.ravel()):
            assert slot[int(e)] == int(s), f"{name}: element {e}"


def test_inplace_layout_writes_where_it_read():
    lay = _layout(P.read_header())
    for i in range(4):
        _, _, _, _, reads = lay[i]
        _, _, writes, _, _ = lay[(i + 1) % 4]             # the next exchange's stores (I2 -> next F0)
        for t in range(256):
            assert set(writes[t].tolist()) == set(reads[t].tolist()), (lay[i][0], t)


def _conflicts(slots, group):
    """extra LDS cycles of one ds_*_b64 instruction per wave: lane groups of `group` lanes, a slot
    = 2 banks of (a/4) mod 64 (reads, 32-lane groups) or mod 32 (writes, 16-lane groups)"""
    nb = 32 if group == 32 else 16
    tot = 0
    for g0 in range(0, 256, group):
        keys = [int(s) % nb for s in slots[g0:g0 + group]]
        tot += sum(v - 1 for v in __import__("collections").Counter(keys).values())
    return tot


def test_inplace_layout_bank_conflicts():
    # per instruction (one register r), summed over the 4 waves: every store and every load
    # conflict-free (round 5's 17-slot rows left one 2-way conflict per 32 lanes on the F1 and I1
    # loads: 8 extra cycles per instruction and workgroup)
    for name, _, ss, _, ls in _layout(P.read_header()):
        for r in range(16):
            assert _conflicts(ss[:, r], 16) == 0, (name, "st", r)
            assert _conflicts(ls[:, r], 32) == 0, (name, "ld", r)


@pytest.mark.parametrize("split", ["pq", "pr"])
@pytest.mark.parametrize("tb", [0, 4, 284, 1024, 1228, 2048, 3888, 4092])
def test_fs_model_matches_oracle(tb, split):
    """both forms of the split x filter: Z P + conj(Zc) Q (round 5) and P (Z + i r conj(Zc)) with
    the real ratio r = Q / (i P) (round 6, the kernel's: 12 table bytes per bin, 6 VALU)"""
    perm = np.array(P.read_header())
    H = O.filter_bank(1.0)[0]
    x = make_stream(1, "mix")
    y = M.r2iq_fs(x, 1, tb, H, perm, split)
    assert O.max_rel_err(y, O.r2iq(x, 1, 0, tb)) < 1e-12
