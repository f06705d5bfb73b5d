"""d = 3..6: the tail-wave kernel (a fifth wave runs the previous frame's inverse tail) against the
four-wave persistent kernel and the f64 oracle (pytest -m gpu).

Both kernels compute the same frame (Core/fft_mt_r2iq_impl.hpp:84-138) with the same operations in
the same order; each is held to 1e-5 of the oracle, and at d >= 4 they are bit-identical.  At d = 3
(radix-8 tail passes with twiddles) the compiler contracts the tail's multiply-adds differently in
the two kernels, so there they agree to float32 rounding (max |a - b| <= 1e-6 max |b|) rather than
bit for bit.
The tail wave works one frame behind the others and has its own final pass after the frame loop,
so the cases include one-block batches, batches with fewer frames than workgroups, a 256-block
batch through the frame queue, and the output stage's variants (sideband, rand, CS16, fused NCO).
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

pytestmark = pytest.mark.gpu

TOL = 1e-5
P_TAILWAVE = 3   # sddc_ddc_internal.h SDDC_DDC_PARAM_P_TAILWAVE


def _set_tailwave(r, on: bool):
    from extio_sddc_amd import _lib
    f = r._L.sddc_ddc_internal_set_param
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    f.restype = ctypes.c_int
    _lib.check(f(r._h, P_TAILWAVE, int(on)))


def _run(r, x, nblk, d, cs16=False):
    import torch
    from extio_sddc_amd import output_samples
    d_in = torch.from_numpy(np.ascontiguousarray(x)).to("cuda")
    n = output_samples(d, nblk) * 2
    out = (torch.full((n,), -12345, dtype=torch.int16, device="cuda") if cs16
           else torch.full((n,), float("nan"), dtype=torch.float32, device="cuda"))
    r.process_device(d_in, nblk, out)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    return o if cs16 else o.view(np.complex64)


CASES = [
    # d, tunebin, lsb, rand, source, nblk
    (3, 1024, 0, 0, "mix", 1),
    (3, 3888, 1, 1, "uniform", 3),
    (3, 512, 0, 0, "oob", 256),
    (4, 1024, 0, 0, "mix", 1),
    (4, 0, 1, 0, "oob", 4),
    (4, 4092, 0, 1, "uniform", 256),
    (5, 2048, 0, 1, "mix", 2),
    (5, 2408, 1, 0, "bench", 3),
    (6, 1024, 1, 0, "mix", 5),
    (6, 4, 0, 0, "uniform", 64),
]


@pytest.mark.parametrize("d,tb,lsb,rand,src,nblk", CASES)
def test_tailwave_equals_persistent_and_oracle(oracle, d, tb, lsb, rand, src, nblk):
    import torch
    from extio_sddc_amd import R2iq
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    x = make_stream(nblk, src)
    ys = []
    with R2iq(gain=1.0, device=0) as r:
        r.setDecimate(d)
        r.setTuneBin(tb)
        r.setSideband(bool(lsb))
        r.updateRand(bool(rand))
        for on in (True, False):
            _set_tailwave(r, on)
            ys.append(_run(r, x, nblk, d))
    for y in ys:
        assert np.all(np.isfinite(y)), "samples never written"
    if src != "bench":   # (the bench tone tuned far away is a leakage-only channel: test_gpu_floor.py)
        ref = oracle.r2iq(x, nblk, d, tb, lsb, rand)
        errs = [oracle.max_rel_err(y, ref) for y in ys]
        assert max(errs) <= TOL, errs
    if d >= 4:
        np.testing.assert_array_equal(ys[0].view(np.uint32), ys[1].view(np.uint32))
    else:
        assert np.max(np.abs(ys[0] - ys[1])) <= 1e-6 * np.max(np.abs(ys[1]))


@pytest.mark.parametrize("d", [3, 4, 5, 6])
def test_tailwave_output_stage_variants(d):
    """CS16 and the fused NCO through the tail wave's stores: identical to the persistent kernel."""
    import torch
    from extio_sddc_amd import R2iq
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    nblk = 8
    x = make_stream(nblk, "mix")
    with R2iq(gain=1.0, device=0) as r:
        r.setDecimate(d)
        r.setTuneBin(1228)
        outs = {}
        for on in (True, False):
            _set_tailwave(r, on)
            r.setOutputFormat("CF32")
            r.setFineTune(0.0)
            y = _run(r, x, nblk, d)
            scale = 30000.0 / float(np.max(np.abs(y.view(np.float32))))
            r.setOutputFormat("CS16", scale)
            c = _run(r, x, nblk, d, cs16=True)
            r.setOutputFormat("CF32")
            r.setFineTune(0.0371)
            m = _run(r, x, nblk, d)
            r.setFineTune(0.0)
            outs[on] = (y, c, m)
    for a, b in zip(outs[True], outs[False]):
        if d >= 4:
            np.testing.assert_array_equal(a.view(np.uint32) if a.dtype != np.int16 else a,
                                          b.view(np.uint32) if b.dtype != np.int16 else b)
        elif a.dtype == np.int16:   # CS16: rounding differences move a sample by at most 1 LSB
            assert np.max(np.abs(a.astype(np.int32) - b.astype(np.int32))) <= 1
        else:
            assert np.max(np.abs(a - b)) <= 1e-6 * np.max(np.abs(b))
