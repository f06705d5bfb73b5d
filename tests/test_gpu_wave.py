"""The alternative d = 0 kernels against the oracle and against the default persistent-workgroup
kernel (variant 0), on a real MI355X (pytest -m gpu): the wave kernel (variants/ddc_wave.hip,
internal variant 3) and the two-frames-in-flight persistent kernel (variants/ddc_variants.hip
r2iq_pipe_kernel, variant 4), both in libsddc_ddc_variants.so (marker: variants).

Cases specific to their layouts: every tune-bin class of the wave kernel's per-lane tables
(bins whose mirror is in lane 0 / lane 32, zero-filled bins below 0 and above 4095), sideband /
rand / CS16 / fused NCO output stages, the frame split of the persistent grid (including
workgroups of one frame, where the pipeline is all fill and drain), and kernel-vs-kernel
agreement at the BASELINE size.  Bar: IQ max-rel-err <= 1e-5 (north_star).
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

pytestmark = [pytest.mark.gpu, pytest.mark.variants]

TOL = 1e-5
VARIANTS = [3, 4, 5, 6, 7]


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


@pytest.fixture(scope="module")
def ddc(torch_dev):
    from extio_sddc_amd import R2iq
    r = R2iq(gain=1.0, device=0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def H(oracle):
    return oracle.filter_bank(1.0)


def set_variant(ddc, v):
    from extio_sddc_amd import _lib
    L = ddc._L
    L.sddc_ddc_internal_set_variant.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.sddc_ddc_internal_set_variant.restype = ctypes.c_int
    _lib.check(L.sddc_ddc_internal_set_variant(ddc._h, v))


def run(torch, ddc, d_in, nblk, tb, lsb=0, rand=0, variant=3):
    from extio_sddc_amd import output_samples
    set_variant(ddc, variant)
    try:
        ddc.setDecimate(0)
        ddc.setTuneBin(tb)
        ddc.setSideband(bool(lsb))
        ddc.updateRand(bool(rand))
        out = torch.full((output_samples(0, nblk) * 2,), float("nan"), dtype=torch.float32, device="cuda")
        ddc.process_device(d_in, nblk, out)
        torch.cuda.synchronize()
    finally:
        set_variant(ddc, 0)
    return out


# tune bins: 0 (zero fill below), 4092 (zero fill above), 1024 (C2), multiples of 64 (the
# lane-0 / lane-32 columns), 32 mod 64, odd columns, and an arbitrary legal bin
TBS = [0, 4, 60, 64, 96, 284, 1024, 1228, 2016, 2048, 2080, 3684, 3888, 4032, 4092]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("tb", TBS)
def test_wave_parity_tunebins(torch_dev, ddc, oracle, H, tb, variant):
    nblk = 3
    x = make_stream(nblk, "mix")
    y = run(torch_dev, ddc, torch_dev.from_numpy(x).to("cuda"), nblk, tb, variant=variant).cpu().numpy().view(np.complex64)
    r = oracle.r2iq(x, nblk, 0, tb, H=H)
    assert np.all(np.isfinite(y))
    err = oracle.max_rel_err(y, r)
    assert err <= TOL, f"tb {tb}: max-rel-err {err:.3e}"


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("src,lsb,rand", [("uniform", 0, 1), ("uniform", 1, 1), ("oob", 1, 0), ("bench", 0, 0)])
def test_wave_parity_sources(torch_dev, ddc, oracle, H, src, lsb, rand, variant):
    nblk = 4
    x = make_stream(nblk, src)
    y = run(torch_dev, ddc, torch_dev.from_numpy(x).to("cuda"), nblk, 1024, lsb, rand, variant).cpu().numpy().view(np.complex64)
    r = oracle.r2iq(x, nblk, 0, 1024, lsb, rand, H=H)
    err = oracle.max_rel_err(y, r)
    assert err <= TOL, f"{src} lsb={lsb} rand={rand}: max-rel-err {err:.3e}"


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("nblk", [1, 2, 5, 37, 100])
def test_wave_frame_split(torch_dev, ddc, oracle, H, nblk, variant):
    """Grids smaller than, equal to and larger than the frame count: every frame lands once."""
    x = make_stream(nblk, "mix", seed=nblk)
    y = run(torch_dev, ddc, torch_dev.from_numpy(x).to("cuda"), nblk, 2048, variant=variant).cpu().numpy().view(np.complex64)
    r = oracle.r2iq(x, nblk, 0, 2048, H=H)
    assert oracle.max_rel_err(y, r) <= TOL


@pytest.mark.parametrize("variant", VARIANTS)
def test_wave_vs_persistent_full_size(torch_dev, ddc, variant):
    """BASELINE size (2048 blocks): the alternative kernel and the persistent kernel agree to 1e-5,
    and the alternative kernel over 8 halo'd segments equals one launch bit for bit."""
    torch = torch_dev
    nblk, seg = 2048, 256
    g = torch.Generator(device="cuda").manual_seed(0x5DDC)
    d_in = torch.randint(-32768, 32767, (4096 + nblk * 65536,), dtype=torch.int16, device="cuda", generator=g)
    d_in[:4096] = 0
    yw = run(torch, ddc, d_in, nblk, 1024, variant=variant)
    yp = run(torch, ddc, d_in, nblk, 1024, variant=0)
    assert torch.isfinite(yw).all()
    err = ((yw - yp).abs().max() / yp.abs().max()).item()
    assert err <= TOL, f"wave vs persistent {err:.3e}"
    from extio_sddc_amd import output_samples
    per = output_samples(0, seg) * 2
    parts = torch.empty_like(yw)
    for s in range(nblk // seg):
        parts[s * per:(s + 1) * per] = run(torch, ddc, d_in[s * seg * 65536:], seg, 1024, variant=variant)
    assert torch.equal(yw, parts)


def _run_fmt(torch, ddc, d_in, nblk, tb, variant, cs16_scale=None, fc=0.0):
    from extio_sddc_amd import output_samples
    set_variant(ddc, variant)
    try:
        ddc.setDecimate(0)
        ddc.setTuneBin(tb)
        ddc.setSideband(True)
        ddc.updateRand(False)
        ddc.setFineTune(0.0)
        ddc.setFineTune(fc)            # a new fc restarts the NCO phase at 0
        if cs16_scale is not None:
            ddc.setOutputFormat("CS16", cs16_scale)
            out = torch.zeros(output_samples(0, nblk) * 2, dtype=torch.int16, device="cuda")
        else:
            out = torch.full((output_samples(0, nblk) * 2,), float("nan"), dtype=torch.float32, device="cuda")
        ddc.process_device(d_in, nblk, out)
        torch.cuda.synchronize()
    finally:
        ddc.setOutputFormat("CF32", 1.0)
        ddc.setFineTune(0.0)
        set_variant(ddc, 0)
    return out


@pytest.mark.parametrize("variant", VARIANTS)
def test_wave_output_stages(torch_dev, ddc, variant):
    """CS16 and the fused fine-tune NCO through the wave kernel: CS16 = saturate(rint(x * scale))
    of its own CF32 output (bit-exact); NCO-on output within 1e-5 of the persistent kernel's."""
    torch = torch_dev
    nblk, tb = 6, 1228
    x = torch.from_numpy(make_stream(nblk, "mix")).to("cuda")
    cf = _run_fmt(torch, ddc, x, nblk, tb, variant)
    scale = 3e4 / cf.abs().max().item()
    cs = _run_fmt(torch, ddc, x, nblk, tb, variant, cs16_scale=scale)
    ref = torch.clamp(torch.round(cf * torch.tensor(scale, dtype=torch.float32)), -32768, 32767).to(torch.int16)
    assert torch.equal(cs, ref)
    yw = _run_fmt(torch, ddc, x, nblk, tb, variant, fc=0.0123)
    yp = _run_fmt(torch, ddc, x, nblk, tb, 0, fc=0.0123)
    assert torch.isfinite(yw).all()
    err = ((yw - yp).abs().max() / yp.abs().max()).item()
    assert err <= TOL, f"NCO wave vs persistent {err:.3e}"
