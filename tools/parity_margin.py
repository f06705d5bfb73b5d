#!/usr/bin/env python3
"""Parity margin of several builds of libsddc_ddc.so: the max-rel-err of every single-channel
case of tests/test_gpu_parity.py (CASES) against the f64 oracle, per library, so a numerics
change can be judged by how much of the 1e-5 bar it uses, not only pass/fail.

  python tools/parity_margin.py --libs build/ab/a.so build/ab/b.so
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--nblk", type=int, default=4)
    args = ap.parse_args()

    import torch
    from extio_sddc_amd._lib import SIGNATURES
    from extio_sddc_amd.synth import make_stream
    from oracle import oracle as O
    from test_gpu_parity import CASES

    O.lib()
    H = O.filter_bank(1.0)
    s = torch.cuda.current_stream().cuda_stream
    libs = []
    for p in args.libs:
        L = ctypes.CDLL(os.path.abspath(p))
        for name, (res, a) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, a
        h = ctypes.c_void_p()
        assert L.sddc_ddc_create(1.0, 0, ctypes.byref(h)) == 0, L.sddc_ddc_last_error()
        libs.append((os.path.basename(p), L, h))
    nblk = args.nblk
    out = {}
    for d, tb, lsb, rand, src in CASES:
        x = make_stream(nblk, src)
        r = O.r2iq(x, nblk, d, tb, lsb, rand, H=H)
        d_in = torch.from_numpy(np.ascontiguousarray(x)).to("cuda")
        row = []
        for name, L, h in libs:
            L.sddc_ddc_set_decimation(h, d)
            L.sddc_ddc_set_tunebin(h, tb)
            L.sddc_ddc_set_sideband(h, lsb)
            L.sddc_ddc_set_rand(h, rand)
            d_out = torch.full((nblk * (32768 >> d) * 2,), float("nan"), dtype=torch.float32, device="cuda")
            assert L.sddc_ddc_process_device(h, d_in.data_ptr(), nblk, d_out.data_ptr(), s) == 0
            torch.cuda.synchronize()
            y = d_out.cpu().numpy().view(np.complex64)
            err = O.max_rel_err(y, r)
            out[f"d{d}_tb{tb}_lsb{lsb}_rand{rand}_{src}:{name}"] = err
            row.append(f"{name} {err:.2e}")
        print(f"d={d} tb={tb:4d} lsb={lsb} rand={rand} {src:8s}  " + "  ".join(row), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
