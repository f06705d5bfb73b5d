#!/usr/bin/env python3
"""Tail-wave vs four-wave persistent kernel on one library build: max |a - b| / max |b| and the
number of differing words per d (GPU).  Used to check whether the d = 3 differences are the
compiler's multiply-add contraction (a build with EXTRA=-ffp-contract=off should be identical).

  python tools/tw_identity.py build/ab/scan.so build/ab/nocontract.so
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from extio_sddc_amd._lib import SIGNATURES
    from extio_sddc_amd.synth import make_stream
    nblk = 4
    x = make_stream(nblk, "mix")
    d_in = torch.from_numpy(np.ascontiguousarray(x)).to("cuda")
    for lib in sys.argv[1:]:
        L = ctypes.CDLL(os.path.abspath(lib))
        for name, (res, a) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, a
        L.sddc_ddc_internal_set_param.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        for d in (3, 4, 5, 6):
            h = ctypes.c_void_p()
            assert L.sddc_ddc_create(1.0, 0, ctypes.byref(h)) == 0
            L.sddc_ddc_set_tunebin(h, 1024)
            L.sddc_ddc_set_decimation(h, d)
            ys = []
            for on in (1, 0):
                assert L.sddc_ddc_internal_set_param(h, 3, on) == 0
                out = torch.full((nblk * (32768 >> d) * 2,), float("nan"), dtype=torch.float32, device="cuda")
                s = torch.cuda.current_stream().cuda_stream
                assert L.sddc_ddc_process_device(h, d_in.data_ptr(), nblk, out.data_ptr(), s) == 0
                torch.cuda.synchronize()
                ys.append(out.cpu().numpy())
            L.sddc_ddc_destroy(h)
            a, b = ys
            print(f"{os.path.basename(lib)} d={d}: max|a-b|/max|b| {np.max(np.abs(a - b)) / np.max(np.abs(b)):.3e}, "
                  f"differing words {int(np.sum(a.view(np.uint32) != b.view(np.uint32)))} of {a.size}")


if __name__ == "__main__":
    main()
