#!/usr/bin/env python3
"""Experiment (tools only): the d = 0 launch's drain closed by the hardware dispatcher.  The batch
is split into a main part (the persistent FS kernel, static slot-weighted split, full residency)
and a tail of T blocks launched right behind it on a second stream as a non-persistent grid (one
frame per workgroup, SDDC_DDC_PARAM_FS_FRAMES_PER_WG = 1).  The main kernel fills every slot, so
the tail's workgroups start only where main workgroups have finished: the dispatcher hands the
last frames to whichever CU frees first, with no atomics.  Compared, interleaved, with the one
launch of the whole batch; outputs must be bit-identical.

  python tools/tail_split_exp.py [--tails 0 32 64 128] [--nblk 2048]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FS_FRAMES_PER_WG = 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "extio_sddc_amd", "lib", "libsddc_ddc.so"))
    ap.add_argument("--tails", type=int, nargs="+", default=[0, 32, 64, 128])
    ap.add_argument("--fpw", type=int, default=1)
    ap.add_argument("--nblk", type=int, default=2048)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--heat-s", type=float, default=2.0)
    args = ap.parse_args()

    import torch
    import bench
    from extio_sddc_amd._lib import SIGNATURES
    dev = torch.device("cuda", 0)
    L = ctypes.CDLL(os.path.abspath(args.lib))
    for name, (res, a) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, a
    L.sddc_ddc_internal_set_param.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]

    def handle(fpw):
        h = ctypes.c_void_p()
        assert L.sddc_ddc_create(1.0, 0, ctypes.byref(h)) == 0, L.sddc_ddc_last_error()
        L.sddc_ddc_set_tunebin(h, 1024)
        L.sddc_ddc_set_decimation(h, 0)
        if fpw:
            assert L.sddc_ddc_internal_set_param(h, FS_FRAMES_PER_WG, fpw) == 0
        return h
    hm, ht = handle(0), handle(args.fpw)
    nblk = args.nblk
    d_in = bench.make_input(torch, nblk, 0x5DDC, dev)
    n_out = nblk * 32768 * 2
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream(device=dev)
    ref = torch.empty(n_out, dtype=torch.float32, device=dev)
    outs = {T: torch.empty(n_out, dtype=torch.float32, device=dev) for T in args.tails}

    def run(T, out):
        if T == 0:
            assert L.sddc_ddc_process_device(hm, d_in.data_ptr(), nblk, out.data_ptr(), s1.cuda_stream) == 0
            return
        nm = nblk - T
        ev0 = torch.cuda.Event()
        ev0.record(s1)
        s2.wait_event(ev0)
        assert L.sddc_ddc_process_device(hm, d_in.data_ptr(), nm, out.data_ptr(), s1.cuda_stream) == 0
        assert L.sddc_ddc_process_device(ht, d_in.data_ptr() + 2 * 65536 * nm, T,
                                         out.data_ptr() + 4 * 2 * 32768 * nm, s2.cuda_stream) == 0
        ev1 = torch.cuda.Event()
        ev1.record(s2)
        s1.wait_event(ev1)

    import time
    t_end = time.time() + args.heat_s
    while time.time() < t_end:
        run(0, ref)
        torch.cuda.synchronize()
    ref.fill_(float("nan"))
    run(0, ref)
    for T in args.tails:
        outs[T].fill_(float("nan"))
        run(T, outs[T])
    torch.cuda.synchronize()
    for T in args.tails:
        same = bool(torch.equal(outs[T], ref))
        print(f"tail {T:4d} blocks: bit-identical to one launch: {same}, NaN left: {int(torch.isnan(outs[T]).sum())}")
    times = {T: [] for T in args.tails}
    for rnd in range(args.rounds + 1):
        for T in args.tails:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s1)
            for _ in range(args.reps):
                run(T, outs[T])
            e1.record(s1)
            torch.cuda.synchronize()
            if rnd:
                times[T].append(e0.elapsed_time(e1) / args.reps)
    for T in args.tails:
        ts = sorted(times[T])
        med = ts[len(ts) // 2]
        print(f"d=0 tail {T:4d} blocks (fpw {args.fpw})  median {med:.4f} ms min {ts[0]:.4f}  "
              f"{nblk * 65536 / (med * 1e-3) / 1e9:7.1f} GS/s  roofline {nblk * 65536 * 6 / (med * 1e-3) / 8e12 * 100:5.1f}%",
              flush=True)


if __name__ == "__main__":
    main()
