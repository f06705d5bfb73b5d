#!/usr/bin/env python3
"""Per-segment cycle attribution of the single-channel kernels from the SDDC_STAMPS diagnostic
builds (ddc_stamps.hpp: s_memtime right before and after each s_barrier, summed per wave over its
workgroup's frames; build 1 stamps barriers 0..3, build 2 barriers 4..7, build 3 barriers 8..11).

  tools/build_rev_lib.sh tree stamps1   (with EXTRA=-DSDDC_STAMPS=1), likewise stamps2, stamps3
  python tools/fs_stamps.py --kernel fs --libs build/ab/stamps1.so build/ab/stamps2.so
  python tools/fs_stamps.py --kernel p --d 4 --libs build/ab/stamps1.so build/ab/stamps2.so

After >= 2 s of back-to-back launches (MI355X_MICROARCH.md "DVFS give-back" item 6) it runs 20
launches and reads the last one's stamps: per wave index (0..3), the mean over workgroups of
cycles per frame in each work segment and barrier wait; the in-kernel clock is
d(s_memtime) / d(s_memrealtime) x 100 MHz.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEGS = 13   # ddc_stamps.hpp kStampSegs
# barrier i closes the work segment in front of it: what each barrier follows
FS_WORK = ["F0 convert+DFT (frame start)", "F0 row stores", "F1 reads+twiddle+DFT", "F1 row stores",
           "F2 reads+DFT, split, I0 DFT", "I0 row stores (+ queue)", "I1 reads+twiddle+DFT (+ prefetch)",
           "I1 row stores", "-", "-", "-", "-", "I2 reads+twiddle+DFT+emit (frame end)"]
P_WORK = {
    # d = 3 (N = 512): split + radix-2 step to LDS, the two 256-point halves on waves 0 and 1
    3: ["F0 convert+DFT (+ prefetch)", "F0 row stores", "F1 reads+twiddle+DFT", "F1 row stores",
        "F2 reads+twiddle+DFT", "Z stores (+ queue)", "split x filter (Z reads, P/Q loads)", "radix-2 halves to LDS",
        "-", "-", "-", "-", "waves 0-1 inverse halves + emit (frame end)"],
    # d >= 4 (N <= 256): one filtered bin per thread to sb, wave-0 Stockham tail
    4: ["F0 convert+DFT (+ prefetch)", "F0 row stores", "F1 reads+twiddle+DFT", "F1 row stores",
        "F2 reads+twiddle+DFT", "Z stores (+ queue)", "split x filter to sb", "-", "-", "-", "-", "-",
        "wave-0 inverse tail + emit (frame end)"],
    # d = 2 (N = 1024): radix-4 pass 0 from registers, 4 workgroup radix-4 passes (3 barriers inside)
    2: ["F0 convert+DFT (+ prefetch)", "F0 row stores", "F1 reads+twiddle+DFT", "F1 row stores",
        "F2 reads+twiddle+DFT", "Z stores (+ queue)", "split + I0 DFT-4", "I0 stores", "-", "-", "-", "-",
        "wg passes + emit (frame end)"],
    # d = 0, 1 (N = 4096, 2048): radix-N/256, 16, 16 passes
    1: ["F0 convert+DFT (+ prefetch)", "F0 row stores", "F1 reads+twiddle+DFT", "F1 row stores",
        "F2 reads+twiddle+DFT", "Z stores (+ queue)", "split + I0 DFT", "I0 row stores", "I1 reads+twiddle+DFT",
        "I1 row stores", "-", "-", "I2 reads+twiddle+DFT+emit (frame end)"],
}


def run(lib: str, kernel: str, d: int, nblk: int, tb: int, params=()):
    import torch
    from extio_sddc_amd._lib import SIGNATURES
    L = ctypes.CDLL(os.path.abspath(lib))
    for name, (res, a) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, a
    getst = L.sddc_ddc_internal_fs_stamps if kernel == "fs" else L.sddc_ddc_internal_p_stamps
    getst.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    h = ctypes.c_void_p()
    assert L.sddc_ddc_create(1.0, 0, ctypes.byref(h)) == 0
    L.sddc_ddc_set_tunebin(h, tb)
    L.sddc_ddc_set_decimation(h, d)
    for k, v in params:   # sddc_ddc_internal_set_param (e.g. 1=40: the d = 0 static share)
        L.sddc_ddc_internal_set_param.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        assert L.sddc_ddc_internal_set_param(h, k, v) == 0
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5DDC)
    d_in = torch.randint(-32768, 32767, (4096 + nblk * 65536,), dtype=torch.int16, device=dev, generator=g)
    out = torch.empty(nblk * (32768 >> d) * 2, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    t_end = time.time() + 2.0
    while time.time() < t_end:
        for _ in range(10):
            assert L.sddc_ddc_process_device(h, d_in.data_ptr(), nblk, out.data_ptr(), s) == 0
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        assert L.sddc_ddc_process_device(h, d_in.data_ptr(), nblk, out.data_ptr(), s) == 0
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    wpw = ctypes.c_int()
    getst(None, 0, ctypes.byref(wpw))
    ngrid = 256 * 4
    buf = np.zeros(ngrid * 4 * wpw.value, np.uint32)
    rc = getst(buf.ctypes.data, buf.size, None)
    assert rc == 0, rc
    L.sddc_ddc_destroy(h)
    return ms, buf.reshape(ngrid, 4, wpw.value)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--kernel", choices=["fs", "p"], default="fs")
    ap.add_argument("--d", type=int, default=0)
    ap.add_argument("--nblk", type=int, default=2048)
    ap.add_argument("--tunebin", type=int, default=1024)
    ap.add_argument("--param", action="append", default=[], help="PARAM=VALUE (sddc_ddc_internal_set_param)")
    args = ap.parse_args()
    params = [tuple(int(v) for v in kv.split("=")) for kv in args.param]
    work = FS_WORK if args.kernel == "fs" else P_WORK[min(args.d, 4) if args.d >= 2 else 1]
    res = {}
    for lib in args.libs:
        ms, st = run(lib, args.kernel, args.d, args.nblk, args.tunebin, params)
        which = int(st[0, 0, 2 * SEGS + 3])
        fr = st[:, :, 2 * SEGS].astype(np.float64)
        ok = fr > 0
        ticks = st[:, :, 2 * SEGS + 1].astype(np.float64)
        rt = st[:, :, 2 * SEGS + 2].astype(np.float64)
        clk = np.median(ticks[ok] / (rt[ok] * 1e-8)) / 1e9
        print(f"\n{os.path.basename(lib)} kernel {args.kernel} d={args.d} (stamps build {which}): {ms:.4f} ms/launch, "
              f"in-kernel clock {clk:.3f} GHz, {np.median(ticks[ok] / fr[ok]):.0f} cycles per frame per wave (median)")
        rs = st[:, 0, 2 * SEGS + 4].astype(np.int64)
        re = st[:, 0, 2 * SEGS + 5].astype(np.int64)
        t0 = rs.min()
        rs_us, re_us = (rs - t0) * 0.01, (re - t0) * 0.01
        print(f"  workgroup start (us after the first): p50 {np.median(rs_us):.2f} max {rs_us.max():.2f}; "
              f"end: min {re_us.min():.1f} p10 {np.percentile(re_us, 10):.1f} p50 {np.median(re_us):.1f} "
              f"p90 {np.percentile(re_us, 90):.1f} max {re_us.max():.1f}")
        print(f"  frames per workgroup: min {fr[:, 0].min():.0f} p50 {np.median(fr[:, 0]):.0f} max {fr[:, 0].max():.0f}")
        xcd = np.arange(len(re_us)) % 8   # blockIdx % 8: the XCD under round-robin placement
        print("    end p50 by blockIdx % 8 (XCD): " + " ".join(f"{np.median(re_us[xcd == x]):.1f}" for x in range(8))
              + f"; within slot 0, p10..p90 {np.percentile(re_us[:len(re_us) // 4], 10):.1f}.."
              f"{np.percentile(re_us[:len(re_us) // 4], 90):.1f} us")
        hw = st[:, 0, 2 * SEGS + 6].astype(np.int64)
        tg = (hw >> 16) & 0xF   # HW_ID TG_ID (bits 19:16): the workgroup slot on its CU
        for q in range(4):
            sel = (np.arange(len(re_us)) * 4 // len(re_us)) == q
            print(f"    blockIdx quarter {q}: end p50 {np.median(re_us[sel]):.1f} us, frames p50 {np.median(fr[sel, 0]):.0f}"
                  f"; HW slot {q}: {int(np.sum(tg == q))} workgroups, end p50 "
                  f"{np.median(re_us[tg == q]) if np.any(tg == q) else float('nan'):.1f} us")
        for wv in range(4):   # HW_ID SIMD_ID (bits 5:4) of wave wv, over the workgroups
            simd = (st[:, wv, 2 * SEGS + 6].astype(np.int64) >> 4) & 3
            print(f"    wave {wv}: SIMD 0..3 " + " ".join(str(int(np.sum(simd == s))) for s in range(4))
                  + " workgroups; wave - SIMD mod 4: " + " ".join(str(int(np.sum((wv - simd) % 4 == s)))
                                                                 for s in range(4)))
        lo = 4 * (which - 1)
        rows = []
        for i in range(SEGS):
            stamped = (lo <= i < lo + 4) or i == SEGS - 1
            if not stamped or work[i] == "-" and i != SEGS - 1:
                continue
            wk = [np.mean(st[:, w, i][ok[:, w]] / fr[:, w][ok[:, w]]) for w in range(4)]
            wt = [np.mean(st[:, w, SEGS + i][ok[:, w]] / fr[:, w][ok[:, w]]) for w in range(4)] if i < SEGS - 1 else [0] * 4
            name = work[i]
            if i == lo and lo:
                name = f"frame start .. {work[i]} (incl. unstamped barriers 0..{lo - 1})"
            if i == SEGS - 1:
                name = f"after barrier {lo + 3} .. frame end (incl. later unstamped barriers)"
            rows.append((i, name, wk, wt))
            print(f"  seg {i:2d}: {name:66s} work " + " ".join(f"{x:7.0f}" for x in wk)
                  + "   wait " + " ".join(f"{x:6.0f}" for x in wt))
        res[os.path.basename(lib)] = {"ms": ms, "clock_GHz": clk, "build": which, "kernel": args.kernel, "d": args.d,
                                      "wg_end_us": {"min": float(re_us.min()), "p50": float(np.median(re_us)),
                                                    "max": float(re_us.max())},
                                      "xcd_end_p50_us": [float(np.median(re_us[xcd == x])) for x in range(8)],
                                      "rows": [{"seg": i, "what": n, "work_cycles_per_frame_wave0..3": wk,
                                                "barrier_wait_cycles_per_frame_wave0..3": wt}
                                               for i, n, wk, wt in rows]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
