#!/usr/bin/env python3
"""Run one build of libsddc_ddc.so back to back (single channel), for profiler passes:
  python tools/run_lib.py --lib build/ab/X.so [--d 0] [--nblk 2048] [--reps 20] [--tunebin 1024]
                          [--rand] [--lsb] [--channels N]"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "extio_sddc_amd", "lib", "libsddc_ddc.so"))
    ap.add_argument("--d", type=int, default=0)
    ap.add_argument("--nblk", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tunebin", type=int, default=1024)
    ap.add_argument("--rand", action="store_true")
    ap.add_argument("--lsb", action="store_true")
    ap.add_argument("--channels", type=int, default=0, help="many-channel launch, tune bins 4c")
    args = ap.parse_args()
    import torch
    from extio_sddc_amd._lib import SIGNATURES
    L = ctypes.CDLL(os.path.abspath(args.lib))
    for name, (res, a) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, a
    h = ctypes.c_void_p()
    assert L.sddc_ddc_create(1.0, 0, ctypes.byref(h)) == 0
    assert L.sddc_ddc_set_decimation(h, args.d) == 0 and L.sddc_ddc_set_tunebin(h, args.tunebin) == 0
    assert L.sddc_ddc_set_rand(h, int(args.rand)) == 0 and L.sddc_ddc_set_sideband(h, int(args.lsb)) == 0
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0x5DDC)
    d_in = torch.randint(-32768, 32767, (4096 + args.nblk * 65536,), dtype=torch.int16, device=dev, generator=g)
    nch = max(args.channels, 1)
    n_out = args.nblk * (32768 >> args.d) * 2
    out = torch.empty(n_out * nch, dtype=torch.float32, device=dev)
    tbs = np.ascontiguousarray(np.arange(nch, dtype=np.int32) * 4)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(args.reps):
        if args.channels:
            rc = L.sddc_ddc_process_channels_device(h, d_in.data_ptr(), args.nblk, tbs.ctypes.data, nch,
                                                    out.data_ptr(), n_out, s)
        else:
            rc = L.sddc_ddc_process_device(h, d_in.data_ptr(), args.nblk, out.data_ptr(), s)
        assert rc == 0, L.sddc_ddc_last_error()
    torch.cuda.synchronize()
    L.sddc_ddc_destroy(h)
    print("done", os.path.basename(args.lib), args.d)


if __name__ == "__main__":
    main()
