"""CS16 output format on the GPU (pytest -m gpu).

The reference only emits CF32 (SoapySDDC/Streaming.cpp:12-50; libsddc.cpp:79-126), so
the CS16 stage is specified here: int16 (I, Q) = saturate(rint(x * scale)), rint =
round-half-even.  Bar: bit-exact against that numpy restatement applied to the CF32
output of the same path (single, NCO, many-channel v1/v2, host path); <= 1 LSB
against the f64 oracle."""
from __future__ import annotations

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

pytestmark = pytest.mark.gpu


def to_cs16(y: np.ndarray, scale: float) -> np.ndarray:
    f = y.astype(np.complex64).view(np.float32).reshape(-1, 2)
    return np.clip(np.rint(f * np.float32(scale)), -32768, 32767).astype(np.int16)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


def _ddc(d, tb, lsb=False, rand=False):
    from extio_sddc_amd import R2iq
    r = R2iq(gain=1.0)
    r.setDecimate(d)
    r.setTuneBin(tb)
    r.setSideband(lsb)
    r.updateRand(rand)
    return r


def _dev(torch, r, x, nblk, d, cs16):
    from extio_sddc_amd import output_samples
    d_in = torch.from_numpy(np.ascontiguousarray(x)).to("cuda")
    n = output_samples(d, nblk) * 2
    if cs16:
        d_out = torch.full((n,), -12345, dtype=torch.int16, device="cuda")
    else:
        d_out = torch.full((n,), float("nan"), dtype=torch.float32, device="cuda")
    r.process_device(d_in, nblk, d_out)
    torch.cuda.synchronize()
    o = d_out.cpu().numpy()
    return o.reshape(-1, 2) if cs16 else o.view(np.complex64)


@pytest.mark.parametrize("d,tb,lsb,rand", [(0, 1024, False, False), (1, 284, True, True), (3, 1228, True, True),
                                           (4, 2048, False, True), (6, 4, True, False)])
def test_single_cs16_bit_exact(torch_dev, d, tb, lsb, rand):
    nblk = 4
    x = make_stream(nblk, "uniform" if rand else "mix")
    with _ddc(d, tb, lsb, rand) as r:
        y = _dev(torch_dev, r, x, nblk, d, False)
        scale = 30000.0 / float(np.max(np.abs(y.view(np.float32))))
        r.setOutputFormat("CS16", scale)
        c = _dev(torch_dev, r, x, nblk, d, True)
    np.testing.assert_array_equal(c, to_cs16(y, scale))
    assert np.abs(c.astype(np.int32)).max() > 20000          # the range is used


def test_cs16_saturates(torch_dev):
    d, nblk = 0, 2
    x = make_stream(nblk, "mix")
    with _ddc(d, 1024) as r:
        y = _dev(torch_dev, r, x, nblk, d, False)
        scale = 8 * 32767.0 / float(np.max(np.abs(y.view(np.float32))))
        r.setOutputFormat("CS16", scale)
        c = _dev(torch_dev, r, x, nblk, d, True)
    ref = to_cs16(y, scale)
    np.testing.assert_array_equal(c, ref)
    assert (c == 32767).any() and (c == -32768).any()


def test_cs16_vs_oracle_one_lsb(torch_dev, oracle):
    d, tb, nblk = 2, 1228, 4
    x = make_stream(nblk, "mix")
    ref = oracle.r2iq(x, nblk, d, tb, H=oracle.filter_bank(1.0))
    scale = 30000.0 / float(np.max(np.abs(np.concatenate([ref.real, ref.imag]))))
    with _ddc(d, tb) as r:
        r.setOutputFormat("CS16", scale)
        c = _dev(torch_dev, r, x, nblk, d, True)
    exact = np.stack([ref.real, ref.imag], 1) * scale
    assert np.max(np.abs(c - np.rint(exact))) <= 1


def test_cs16_with_fine_tune(torch_dev):
    d, nblk, fc = 1, 4, 0.0123
    x = make_stream(nblk, "mix")
    with _ddc(d, 1024) as r:
        r.setFineTune(fc)
        y = _dev(torch_dev, r, x, nblk, d, False)
    with _ddc(d, 1024) as r:
        r.setFineTune(fc)
        scale = 30000.0 / float(np.max(np.abs(y.view(np.float32))))
        r.setOutputFormat("CS16", scale)
        c = _dev(torch_dev, r, x, nblk, d, True)
    np.testing.assert_array_equal(c, to_cs16(y, scale))


@pytest.mark.parametrize("d", [0, 3, 4])   # channels kernel for d < 4 (2^d channels in flight) and v2 (d >= 4)
def test_channels_cs16_bit_exact(torch_dev, d):
    torch = torch_dev
    from extio_sddc_amd import output_samples
    nblk, tbs = 2, [0, 512, 1024, 2048, 4092]
    x = torch.from_numpy(make_stream(nblk, "mix")).to("cuda")
    per = output_samples(d, nblk) * 2
    with _ddc(d, 1024, lsb=True) as r:
        yf = torch.empty((len(tbs), per), dtype=torch.float32, device="cuda")
        r.process_channels_device(x, nblk, tbs, yf)
        torch.cuda.synchronize()
        y = yf.cpu().numpy()
        scale = 30000.0 / float(np.max(np.abs(y)))
        r.setOutputFormat("CS16", scale)
        yc = torch.empty((len(tbs), per), dtype=torch.int16, device="cuda")
        r.process_channels_device(x, nblk, tbs, yc)
        torch.cuda.synchronize()
        c = yc.cpu().numpy()
    for ch in range(len(tbs)):
        np.testing.assert_array_equal(c[ch].reshape(-1, 2), to_cs16(y[ch].view(np.complex64), scale))


def test_host_path_cs16(torch_dev):
    d, nblk = 0, 70
    x = make_stream(nblk, "mix")
    with _ddc(d, 1024) as r:
        y = r.process(x[4096:])
        scale = 30000.0 / float(np.max(np.abs(y.view(np.float32))))
        r.TurnOn()
        r.setOutputFormat("CS16", scale)
        c = r.process(x[4096:])
    assert c.dtype == np.int16 and c.shape == (y.size, 2)
    np.testing.assert_array_equal(c, to_cs16(y, scale))


def test_bad_format_args(torch_dev):
    from extio_sddc_amd import DDCError
    with _ddc(0, 1024) as r:
        with pytest.raises(DDCError):
            r.setOutputFormat("CS16", 0.0)
        with pytest.raises(KeyError):
            r.setOutputFormat("CU8", 1.0)
