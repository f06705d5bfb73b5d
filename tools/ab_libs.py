#!/usr/bin/env python3
"""A/B timing of several builds of libsddc_ddc.so in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Each library gets its own handle; all share
torch's HIP runtime.  Output difference vs the first library is reported too.

  python tools/ab_libs.py --libs build/ab/a.so build/ab/b.so [--d 0 4] [--nblk 2048]
"""
from __future__ import annotations

import argparse
import ctypes
import json

import numpy as np
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--d", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    ap.add_argument("--nblk", type=int, default=2048)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tunebin", type=int, default=1024)
    ap.add_argument("--channels", type=int, default=0, help="time process_channels_device with tune bins 4c")
    ap.add_argument("--rand", action="store_true", help="RAND de-randomisation on (config C4)")
    ap.add_argument("--lsb", action="store_true", help="sideband inversion on (config C4)")
    ap.add_argument("--input", choices=["rand", "bench", "zeros"], default="rand",
                    help="rand: uniform int16; bench: bench.py's tone mix + noise (its make_input)")
    ap.add_argument("--heat-s", type=float, default=2.0)
    args = ap.parse_args()

    import torch
    from extio_sddc_amd._lib import SIGNATURES
    dev = torch.device("cuda", 0)
    libs, handles = [], []
    for spec in args.libs:
        # LIB.so or LIB.so:PARAM=VALUE[,PARAM=VALUE] (sddc_ddc_internal_set_param on its handle)
        p, _, params = spec.partition(":")
        L = ctypes.CDLL(os.path.abspath(p))
        for name, (res, a) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, a
        h = ctypes.c_void_p()
        rc = L.sddc_ddc_create(1.0, 0, ctypes.byref(h))
        assert rc == 0, L.sddc_ddc_last_error()
        L.sddc_ddc_set_tunebin(h, args.tunebin)
        if args.rand:
            assert L.sddc_ddc_set_rand(h, 1) == 0
        if args.lsb:
            assert L.sddc_ddc_set_sideband(h, 1) == 0
        for kv in filter(None, params.split(",")):
            k, v = (int(x) for x in kv.split("="))
            L.sddc_ddc_internal_set_param.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
            assert L.sddc_ddc_internal_set_param(h, k, v) == 0
        libs.append(L)
        handles.append(h)
    nblk = args.nblk
    g = torch.Generator(device=dev).manual_seed(0x5DDC)
    if args.input == "zeros":
        d_in = torch.zeros(4096 + nblk * 65536, dtype=torch.int16, device=dev)
    elif args.input == "bench":
        import bench
        d_in = bench.make_input(torch, nblk, 0x5DDC, dev)
    else:
        d_in = torch.randint(-32768, 32767, (4096 + nblk * 65536,), dtype=torch.int16, device=dev, generator=g)
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    # heat the chip for ~2 s so every variant is timed at the sustained (power-limited) clock
    heat = torch.empty(nblk * 32768 * 2, dtype=torch.float32, device=dev)
    libs[0].sddc_ddc_set_decimation(handles[0], 0)
    t_end = __import__("time").time() + args.heat_s
    while __import__("time").time() < t_end:
        libs[0].sddc_ddc_process_device(handles[0], d_in.data_ptr(), nblk, heat.data_ptr(), s)
        torch.cuda.synchronize()
    del heat
    for d in args.d:
        n_out = nblk * (32768 >> d) * 2
        nch = max(args.channels, 1)
        outs = [torch.empty(n_out * nch, dtype=torch.float32, device=dev) for _ in libs]
        tbs = np.ascontiguousarray(np.arange(nch, dtype=np.int32) * 4)
        times = [[] for _ in libs]
        for L, h in zip(libs, handles):
            L.sddc_ddc_set_decimation(h, d)
        # every variant's output is checked on its own first call into a NaN-filled buffer: a
        # variant that leaves frames unwritten shows NaN (later calls reuse the buffer, so a
        # comparison after the timed rounds alone would not see it)
        unwritten = []
        for i, (L, h) in enumerate(zip(libs, handles)):
            outs[i].fill_(float("nan"))
            if args.channels:
                rc = L.sddc_ddc_process_channels_device(h, d_in.data_ptr(), nblk, tbs.ctypes.data, nch,
                                                        outs[i].data_ptr(), n_out, s)
            else:
                rc = L.sddc_ddc_process_device(h, d_in.data_ptr(), nblk, outs[i].data_ptr(), s)
            assert rc == 0, L.sddc_ddc_last_error()
            torch.cuda.synchronize()
            unwritten.append(int(torch.isnan(outs[i]).sum().item()))
        for rnd in range(args.rounds + 1):
            for i, (L, h) in enumerate(zip(libs, handles)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    if args.channels:
                        rc = L.sddc_ddc_process_channels_device(h, d_in.data_ptr(), nblk, tbs.ctypes.data, nch,
                                                                outs[i].data_ptr(), n_out, s)
                    else:
                        rc = L.sddc_ddc_process_device(h, d_in.data_ptr(), nblk, outs[i].data_ptr(), s)
                    assert rc == 0, L.sddc_ddc_last_error()
                e1.record()
                torch.cuda.synchronize()
                if rnd:
                    times[i].append(e0.elapsed_time(e1) / args.reps)
        for i, p in enumerate(args.libs):
            ts = sorted(times[i])
            med = ts[len(ts) // 2]
            diff = ((outs[i] - outs[0]).abs().max() / outs[0].abs().max()).item()
            gs = nblk * 65536 / (med * 1e-3) / 1e9
            frac = nblk * 65536 * (2 + 4 * nch / (1 << d)) / (med * 1e-3) / 8e12
            res[f"d{d}:{os.path.basename(p)}#{i}"] = {"median_ms": med, "min_ms": ts[0], "GSps": gs, "hbm_frac": frac,
                                                  "maxrel_vs_first": diff, "unwritten_floats": unwritten[i]}
            print(f"d={d} {os.path.basename(p):28s} median {med:.3f} ms min {ts[0]:.3f}  {gs:7.1f} GS/s  "
                  f"roofline {frac*100:5.1f}%  maxrel vs first {diff:.2e}"
                  + (f"  INCOMPLETE: {unwritten[i]} floats unwritten" if unwritten[i] else ""), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
