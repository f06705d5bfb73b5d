"""The d = 0 fused-split kernel's algorithm (ddc_persistent.hip, r2iq_fs_kernel), modelled step
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
    # the in-place layout's I0 stores, F2 loads and F2 twiddle-base loads (W^c at c + [c >= 128]):
    # conflict-free (keys (c + [c >= 128]) mod 16, 32, 32)
    assert P.conflicts(cols) == P.BEST["inplace"] == (0, 0, 0)
    # the unpadded twiddle table (key c mod 32) would not be: pairs c, 256 - c = 0 mod 16 collide
    c = np.asarray(cols)
    assert _conflicts(c, 32) > 0 and _conflicts(c + (c >= 128), 32) == 0


# The in-place LDS layout of the FS kernel (round 5): every exchange's writer stores into exactly
# the slots it read in the previous exchange, so only the four read-after-write barriers remain.
# (thread, register) -> (element, slot) of each store and load, as in ddc_fs.hip.
def _layout(perm):
    t = np.arange(256)[:, None]
    r = np.arange(16)[None, :]
    c = np.asarray(perm)[:, None]
    hi = (r >= 8).astype(int)                     # the padding map's + [e >= 2048]
    cb = 272 * (c >> 4) + (c & 15) + (c >= 128)
    ib = (t >> 4) + 17 * (t & 15)
    fb = 17 * t + (t >= 128)
    return [
        # (name, store element, store slot, load element, load slot)
        ("F0->F1", 16 * t + r, fb + r, t + 256 * r, t + (t >> 4) + 272 * r + hi),
        ("F1->F2", 256 * (t >> 4) + 16 * r + (t & 15), t + (t >> 4) + 272 * r + hi, c + 256 * r, cb + 17 * r),
        ("I0->I1", 16 * c + r, cb + 17 * r, t + 256 * r, ib + 272 * r + hi),
        ("I1->I2", 256 * (t >> 4) + 16 * r + (t & 15), ib + 272 * r + hi, t + 256 * r, fb + r),
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
    # per instruction (one register r), summed over the 4 waves: every store and the F2 / I2 loads
    # conflict-free; the F1 and I1 loads one 2-way per 32 lanes (the 17-slot rows: t + (t >> 4)
    # wraps once per 32 lanes), as the round-4 layout's F1 loads
    lay = _layout(P.read_header())
    want = {("F0->F1", "st"): 0, ("F0->F1", "ld"): 8, ("F1->F2", "st"): 0, ("F1->F2", "ld"): 0,
            ("I0->I1", "st"): 0, ("I0->I1", "ld"): 8, ("I1->I2", "st"): 0, ("I1->I2", "ld"): 0}
    for name, _, ss, _, ls in lay:
        for r in range(16):
            assert _conflicts(ss[:, r], 16) == want[(name, "st")], (name, "st", r)
            assert _conflicts(ls[:, r], 32) == want[(name, "ld")], (name, "ld", r)


@pytest.mark.parametrize("tb", [0, 4, 284, 1024, 1228, 2048, 3888, 4092])
def test_fs_model_matches_oracle(tb):
    perm = np.array(P.read_header())
    H = O.filter_bank(1.0)[0]
    x = make_stream(1, "mix")
    y = M.r2iq_fs(x, 1, tb, H, perm)
    assert O.max_rel_err(y, O.r2iq(x, 1, 0, tb)) < 1e-12
