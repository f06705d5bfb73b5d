#!/usr/bin/env python3
"""Lane -> column permutation of the d = 0 fused-split kernel (ddc_fs.hip, r2iq_fs_kernel).

Lanes 2p, 2p + 1 hold forward-pass-2 columns c, 256 - c (lanes 0, 1: the self-mirrored 0, 128),
so the split's mirror bins are one DPP quad_perm [1,0,3,2] away.  Which pair goes to which lane
pair sets the LDS bank pattern of three accesses (MI355X_MICROARCH.md, LDS: a ds_read_b64 serves
lane groups of 32 over 64 banks, so slot s = 8-byte index is conflict-free iff s mod 32 is distinct
over the group; ds_write_b64 serves 4 groups of 16 contiguous lanes over 32 banks: s mod 16
distinct):
  * forward pass 2 reads its column's 16 elements, one ds_read_b64 per register (groups of 32);
  * inverse pass 0 stores its 16 outputs in place of those reads (groups of 16);
  * forward pass 2 reads its twiddle bases W^c, W^{4c} (ds_read_b64, groups of 32).
The assignment is solved exactly as a 0/1 program (scipy's HiGHS MILP): pair p goes to one
16-lane half of one 32-lane group, each half takes 8 pairs, and the objective is the extra LDS
cycles per frame (16 reads and 16 stores per frame at the exchange, 2 twiddle-base reads).
Writes extio_sddc_amd/csrc/ddc_fs_perm.h.

  python tools/fs_perm.py [--check]
"""
from __future__ import annotations

import argparse
import os
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "extio_sddc_amd", "csrc", "ddc_fs_perm.h")

LAYOUT = "il272"   # the product's layout (round 6)
# the fewest extra cycles (I0 stores, F2 reads, twiddle-base reads) per instruction and workgroup
BEST = {"inplace": (0, 0, 0), "il272": (0, 0, 0)}
WEIGHTS = (16, 16, 2)   # instructions per frame of each access


def fs_slot(R: int, j: int) -> int:
    """ddc_fs.hip fs_slot (round 6): the LDS slot of row R (0..255), column j (0..15): rows 2i and
    2i + 1 of each 16-row block interleaved in a 32-slot run, runs 34 slots apart, blocks 272
    apart, the upper half one slot further"""
    return 272 * (R >> 4) + (R >= 128) + 34 * ((R & 15) >> 1) + (R & 1) + 2 * j


def pair_lane(t: int):
    """ddc_fs.hip fs_pair_row / fs_pair_col: the (row u, column j) of F1's and I1's thread t"""
    return 2 * (t >> 5) + (t & 1), (t >> 1) & 15


def keys(c: int):
    """(inverse pass-0 store key mod 16, forward pass-2 read key mod 32, twiddle-base read key
    mod 32) of column c; the twiddle bases W^j sit at j + [j >= 128] (ddc_fs.hip kFsTw)"""
    if LAYOUT == "inplace":
        # round 5: F2 reads element c + 256 g at 272 (c >> 4) + (c & 15) + [c >= 128] + 17 g, I0
        # stores at the same slots
        k = c + (c >= 128)
    else:
        # il272 (round 6): F2 column c = 16 h + cl reads rows 16 h + g, column cl, i.e. slot
        # fs_slot(16 h, cl) + 34 (g >> 1) + (g & 1); the odd pad of the upper half keeps the lane
        # pairs c, 256 - c apart, as in round 5
        k = fs_slot(16 * (c >> 4), c & 15)
    kt = c + (c >= 128)
    return k % 16, k % 32, kt % 32


def conflicts(cols):
    """extra cycles per instruction over the workgroup: (I0 stores, F2 reads, twiddle-base reads)"""
    def extra(key, n):
        return sum(sum(v - 1 for v in Counter(keys(c)[key] for c in cols[g:g + n]).values())
                   for g in range(0, 256, n))
    return extra(0, 16), extra(1, 32), extra(2, 32)


def valid(cols) -> bool:
    return (sorted(cols) == list(range(256)) and cols[0] == 0 and cols[1] == 128
            and all((cols[2 * p] + cols[2 * p + 1]) % 256 == 0 for p in range(1, 128)))


def solve(time_limit: float = 600.0):
    """minimum-weight assignment of the 128 lane pairs to (32-lane group, 16-lane half)"""
    import numpy as np
    from scipy.optimize import Bounds, LinearConstraint, milp
    from scipy.sparse import lil_matrix

    pairs = [(0, 128)] + [(c, 256 - c) for c in range(1, 128)]
    NP, NG, NH = 128, 8, 2
    nx = NP * NG * NH
    # slack (extra lanes on one bank) per (group, bank) for the reads, per (half, bank) for the stores
    # (16 banks of 8 bytes for the stores: keys()[0] < 16)
    off_rd, off_tw, off_wr = nx, nx + NG * 32, nx + 2 * NG * 32
    n = off_wr + NG * NH * 32

    def x(p, g, h):
        return (p * NG + g) * NH + h

    rows, lo, hi = [], [], []

    def add(coefs, lb, ub):
        rows.append(coefs)
        lo.append(lb)
        hi.append(ub)

    for p in range(NP):
        add([(x(p, g, h), 1) for g in range(NG) for h in range(NH)], 1, 1)
    for g in range(NG):
        for h in range(NH):
            add([(x(p, g, h), 1) for p in range(NP)], 8, 8)
    add([(x(0, 0, 0), 1)], 1, 1)                      # columns 0, 128 on lanes 0, 1

    def hits(p, key, b):
        return sum(1 for c in pairs[p] if keys(c)[key] == b)
    for g in range(NG):
        for b in range(32):
            for key, off in ((1, off_rd), (2, off_tw)):
                add([(x(p, g, h), hits(p, key, b)) for p in range(NP) for h in range(NH) if hits(p, key, b)]
                    + [(off + 32 * g + b, -1)], -np.inf, 1)
            for h in range(NH):
                add([(x(p, g, h), hits(p, 0, b)) for p in range(NP) if hits(p, 0, b)]
                    + [(off_wr + 32 * (NH * g + h) + b, -1)], -np.inf, 1)
    A = lil_matrix((len(rows), n))
    for i, r in enumerate(rows):
        for j, v in r:
            A[i, j] += v
    cost = np.zeros(n)
    cost[off_rd:off_tw] = WEIGHTS[1]
    cost[off_tw:off_wr] = WEIGHTS[2]
    cost[off_wr:] = WEIGHTS[0]
    ub = np.ones(n)
    ub[nx:] = 16
    res = milp(cost, constraints=LinearConstraint(A.tocsr(), lo, hi), integrality=np.ones(n),
               bounds=Bounds(0, ub), options={"time_limit": time_limit})
    assert res.x is not None, res.message
    sel = res.x.round().astype(int)
    cols = []
    for g in range(NG):
        for h in range(NH):
            ps = [p for p in range(NP) if sel[x(p, g, h)]]
            for p in sorted(ps, key=lambda p: p != 0):
                cols += list(pairs[p])
    return cols, conflicts(cols), res.message


def write_header(cols, cur, path=HDR):
    rows = ",\n".join("    " + ", ".join(f"{c:3d}" for c in cols[i:i + 16]) for i in range(0, 256, 16))
    with open(path, "w") as f:
        f.write(f"""// ddc_fs_perm.h — generated by tools/fs_perm.py: lane -> forward-pass-2 column of the d = 0
// fused-split kernel (lanes 2p, 2p+1: columns c, 256 - c), for the {LAYOUT} exchange layout.  Extra LDS
// cycles per instruction and workgroup: {cur[0]} on the inverse pass-0 stores, {cur[1]} on the forward
// pass-2 reads, {cur[2]} on the forward pass-2 twiddle-base reads (the optimum for this layout).
#pragma once
__constant__ int kFsPerm[256] = {{
{rows}}};
""")


def read_header(name="kFsPerm"):
    """a table of the committed header (kFsPerm: the lane -> column permutation)"""
    txt = open(HDR).read()
    i = txt.index("{", txt.index(name + "["))
    body = txt[i + 1:txt.index("}", i)]
    return [int(x) for x in body.replace("\n", " ").split(",") if x.strip()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true", help="validate the committed header only")
    ap.add_argument("--time-limit", type=float, default=600.0)
    ap.add_argument("--out", default=HDR)
    args = ap.parse_args()
    if args.check:
        cols = read_header()
        assert valid(cols), "not a paired permutation"
        print("extra cycles (stores, reads, twiddle reads):", conflicts(cols))
        return
    cols, cur, msg = solve(args.time_limit)
    assert valid(cols)
    write_header(cols, cur, args.out)
    print(msg)
    print("extra cycles (stores, reads, twiddle reads):", cur)


if __name__ == "__main__":
    main()
