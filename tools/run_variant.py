#!/usr/bin/env python3
"""Run one single-channel kernel variant (sddc_ddc_internal.h) back to back, for profiler
passes:  python tools/run_variant.py --variant 3 [--d 0] [--nblk 2048] [--reps 20]"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--d", type=int, default=0)
    ap.add_argument("--nblk", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from extio_sddc_amd import R2iq, output_samples, _lib
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5DDC)
    d_in = torch.randint(-32768, 32767, (4096 + args.nblk * 65536,), dtype=torch.int16, device=dev, generator=g)
    out = torch.empty(output_samples(args.d, args.nblk) * 2, dtype=torch.float32, device=dev)
    with R2iq(gain=1.0) as r:
        r._L.sddc_ddc_internal_set_variant.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _lib.check(r._L.sddc_ddc_internal_set_variant(r._h, args.variant))
        r.setDecimate(args.d)
        r.setTuneBin(1024)
        for _ in range(args.reps):
            r.process_device(d_in, args.nblk, out)
        torch.cuda.synchronize()
    print("done", args.variant, args.d)


if __name__ == "__main__":
    main()
