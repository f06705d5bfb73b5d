#!/usr/bin/env python3
"""A/B timing of the single-channel kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Prints per (d, variant) median/min ms and GS/s,
and the max relative difference between variants' outputs.

  python tools/ab_kernels.py [--d 0 1 4] [--nblk 2048] [--rounds 10] [--variants 0 1]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    ap.add_argument("--nblk", type=int, default=2048)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--tunebin", type=int, default=1024)
    args = ap.parse_args()

    import torch
    from extio_sddc_amd import R2iq, output_samples
    from extio_sddc_amd import _lib
    L = _lib.load()
    L.sddc_ddc_internal_set_variant.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.sddc_ddc_internal_set_variant.restype = ctypes.c_int

    dev = torch.device("cuda", 0)
    nblk = args.nblk
    g = torch.Generator(device=dev).manual_seed(0x5DDC)
    d_in = torch.randint(-32768, 32767, (4096 + nblk * 65536,), dtype=torch.int16, device=dev, generator=g)
    ddc = R2iq(gain=1.0)
    ddc.setTuneBin(args.tunebin)
    results = {}
    for d in args.d:
        ddc.setDecimate(d)
        outs = {v: torch.empty(output_samples(d, nblk) * 2, dtype=torch.float32, device=dev) for v in args.variants}
        times = {v: [] for v in args.variants}
        for rnd in range(args.rounds + 1):
            for v in args.variants:
                _lib.check(L.sddc_ddc_internal_set_variant(ddc._h, v))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    ddc.process_device(d_in, nblk, outs[v])
                e1.record()
                torch.cuda.synchronize()
                if rnd > 0:
                    times[v].append(e0.elapsed_time(e1) / args.reps)
        ref = outs[args.variants[-1]]
        for v in args.variants:
            ts = sorted(times[v])
            med = ts[len(ts) // 2]
            diff = ((outs[v] - ref).abs().max() / ref.abs().max()).item()
            results[f"d{d}_v{v}"] = {"median_ms": med, "min_ms": ts[0],
                                     "GSps": nblk * 65536 / (med * 1e-3) / 1e9,
                                     "hbm_frac": nblk * 65536 * (2 + 4 / (1 << d)) / (med * 1e-3) / 8e12,
                                     "maxrel_vs_last": diff}
            print(f"d={d} variant={v}: median {med:.3f} ms  min {ts[0]:.3f} ms  "
                  f"{results[f'd{d}_v{v}']['GSps']:.1f} GS/s  roofline {results[f'd{d}_v{v}']['hbm_frac']*100:.1f}%  "
                  f"maxrel vs v{args.variants[-1]} {diff:.2e}", flush=True)
    print(json.dumps(results))


if __name__ == "__main__":
    main()
