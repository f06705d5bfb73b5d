#!/usr/bin/env python3
"""Per-segment cycle attribution of the d = 0 fused-split kernel from the SDDC_STAMPS diagnostic
builds (ddc_persistent.hip: s_memtime right before and after each s_barrier, summed per wave
over its workgroup's frames; build 1 stamps barriers 0..3, build 2 barriers 4..7).

  python tools/fs_stamps.py --libs build/ab/stamps1.so build/ab/stamps2.so [--nblk 2048]

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

SEGS = 9
# barrier i closes the work segment in front of it: what each barrier follows
WORK = ["F0 convert+DFT (frame start)", "F0 row stores", "F1 reads+twiddle+DFT", "F1 row stores",
        "F2 reads+DFT, split, I0 DFT", "I0 row stores", "I1 reads+twiddle+DFT", "I1 row stores",
        "I2 reads+twiddle+DFT+emit"]


def run(lib: str, nblk: int, tb: int):
    import torch
    from extio_sddc_amd._lib import SIGNATURES
    L = ctypes.CDLL(os.path.abspath(lib))
    for name, (res, a) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, a
    L.sddc_ddc_internal_fs_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    h = ctypes.c_void_p()
    assert L.sddc_ddc_create(1.0, 0, ctypes.byref(h)) == 0
    L.sddc_ddc_set_tunebin(h, tb)
    L.sddc_ddc_set_decimation(h, 0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5DDC)
    d_in = torch.randint(-32768, 32767, (4096 + nblk * 65536,), dtype=torch.int16, device=dev, generator=g)
    out = torch.empty(nblk * 32768 * 2, dtype=torch.float32, device=dev)
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
    L.sddc_ddc_internal_fs_stamps(None, 0, ctypes.byref(wpw))
    ngrid = 256 * 4
    buf = np.zeros(ngrid * 4 * wpw.value, np.uint32)
    rc = L.sddc_ddc_internal_fs_stamps(buf.ctypes.data, buf.size, None)
    assert rc == 0, rc
    L.sddc_ddc_destroy(h)
    return ms, buf.reshape(ngrid, 4, wpw.value)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--nblk", type=int, default=2048)
    ap.add_argument("--tunebin", type=int, default=1024)
    args = ap.parse_args()
    res = {}
    for lib in args.libs:
        ms, st = run(lib, args.nblk, args.tunebin)
        which = int(st[0, 0, 2 * SEGS + 3])
        fr = st[:, :, 2 * SEGS].astype(np.float64)
        ok = fr > 0
        ticks = st[:, :, 2 * SEGS + 1].astype(np.float64)
        rt = st[:, :, 2 * SEGS + 2].astype(np.float64)
        clk = np.median(ticks[ok] / (rt[ok] * 1e-8)) / 1e9
        print(f"\n{os.path.basename(lib)} (stamps build {which}): {ms:.4f} ms/launch, in-kernel clock {clk:.3f} GHz, "
              f"{np.median(ticks[ok] / fr[ok]):.0f} cycles per frame per wave (median)")
        rs = st[:, 0, 2 * SEGS + 4].astype(np.int64)
        re = st[:, 0, 2 * SEGS + 5].astype(np.int64)
        hw = st[:, 0, 2 * SEGS + 6].astype(np.int64)
        tg = (hw >> 16) & 15
        t0 = rs.min()
        rs_us, re_us = (rs - t0) * 0.01, (re - t0) * 0.01
        print(f"  workgroup start (us after the first): p50 {np.median(rs_us):.2f} max {rs_us.max():.2f}; "
              f"end: min {re_us.min():.1f} p10 {np.percentile(re_us, 10):.1f} p50 {np.median(re_us):.1f} "
              f"p90 {np.percentile(re_us, 90):.1f} max {re_us.max():.1f}")
        for s_ in range(4):
            m = tg == s_
            if m.any():
                print(f"    CU slot (HW_ID tg_id) {s_}: {m.sum():4d} workgroups, end p50 {np.median(re_us[m]):.1f} us, "
                      f"min {re_us[m].min():.1f} max {re_us[m].max():.1f}")
        # which SIMD each wave index of a workgroup runs on (HW_ID SIMD_ID, bits 5:4), and, over the
        # workgroups sharing a CU (SE, SH, CU ids), whether wave 0 of every workgroup lands on one SIMD
        hwa = st[:, :, 2 * SEGS + 6].astype(np.int64)
        simd = (hwa >> 4) & 3
        for wv in range(4):
            cnt = np.bincount(simd[:, wv], minlength=4)
            print(f"    wave {wv}: SIMD histogram {cnt.tolist()}")
        cu = (hwa[:, 0] >> 8) & 0x7F   # CU_ID, SH_ID, SE_ID
        same = []
        for c in np.unique(cu):
            m = cu == c
            same.append(len(np.unique(simd[m, 0])))
        print(f"    distinct SIMDs holding wave 0 among the workgroups of one CU id: "
              f"{np.bincount(np.array(same), minlength=5)[1:].tolist()} (count of CU ids with 1, 2, 3, 4)")
        lo = 4 if which >= 2 else 0
        if which == 3:
            for i, what in enumerate(("resolve", "s_next write", "next ticket", "ticket read (frame top)")):
                qwk = [np.mean(st[:, w, i][ok[:, w]] / fr[:, w][ok[:, w]]) for w in range(4)]
                print(f"  queue wave, inside seg 5: {what:36s} work " + " ".join(f"{x:7.0f}" for x in qwk))
        rows = []
        for i in range(SEGS):
            stamped = (lo <= i < lo + 4) or i == SEGS - 1
            if not stamped:
                continue
            wk = [np.mean(st[:, w, i][ok[:, w]] / fr[:, w][ok[:, w]]) for w in range(4)]
            wt = [np.mean(st[:, w, SEGS + i][ok[:, w]] / fr[:, w][ok[:, w]]) for w in range(4)] if i < SEGS - 1 else [0] * 4
            name = WORK[i] if i == lo or i == SEGS - 1 or i > lo else WORK[i]
            if i == lo and lo:
                name = "frame start .. " + WORK[i] + " (incl. unstamped barriers 0..3)"
            if i == SEGS - 1 and lo == 0:
                name = "barrier 3 release .. frame end (incl. unstamped barriers 4..7)"
            rows.append((i, name, wk, wt))
            print(f"  seg {i}: {name:62s} work " + " ".join(f"{x:7.0f}" for x in wk)
                  + "   wait " + " ".join(f"{x:6.0f}" for x in wt))
        res[os.path.basename(lib)] = {"ms": ms, "clock_GHz": clk, "build": which,
                                      "rows": [{"seg": i, "what": n, "work_cycles_per_frame_wave0..3": wk,
                                                "barrier_wait_cycles_per_frame_wave0..3": wt}
                                               for i, n, wk, wt in rows]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
