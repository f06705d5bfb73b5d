"""HIP path vs the oracle, on a real MI355X (pytest -m gpu).

Bar: IQ max-rel-err = max|y - r| / max|r| <= 1e-5 over the whole output
stream (BASELINE.json north_star), r = the f64 oracle (oracle/ddc_oracle.c,
the exact answer the reference's float FFTW path approximates to <= 2.6e-6,
SURVEY.md §8(c)).  Every call goes through the C ABI (include/sddc_ddc.h).
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

pytestmark = pytest.mark.gpu

TOL = 1e-5            # north_star: IQ within 1e-5 relative
HERE = os.path.dirname(os.path.abspath(__file__))


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


def run_device(torch, ddc, x, nblk, d, tb, lsb, rand):
    from extio_sddc_amd import output_samples
    ddc.setDecimate(d)
    ddc.setTuneBin(tb)
    ddc.setSideband(bool(lsb))
    ddc.updateRand(bool(rand))
    d_in = torch.from_numpy(np.ascontiguousarray(x)).to("cuda")
    d_out = torch.full((output_samples(d, nblk) * 2,), float("nan"), dtype=torch.float32, device="cuda")
    ddc.process_device(d_in, nblk, d_out)
    torch.cuda.synchronize()
    y = d_out.cpu().numpy().view(np.complex64)
    return y


CASES = [
    # d, tunebin, lsb, rand, source
    (0, 1024, 0, 0, "mix"),      # C2 default tune (Fs/8)
    (0, 0, 0, 0, "mix"),         # zero fill below bin 0
    (0, 4092, 1, 1, "uniform"),  # zero fill above bin 4095, lsb + rand
    (0, 2048, 0, 0, "bench"),
    (1, 1024, 1, 1, "mix"),      # C4 VHF config: decim 4, sideband invert, rand
    (1, 284, 0, 0, "oob"),
    (2, 1228, 0, 1, "uniform"),
    (2, 3684, 1, 0, "mix"),
    (3, 512, 0, 0, "mix"),
    (3, 3888, 0, 1, "bench"),
    (4, 1024, 0, 0, "mix"),
    (4, 0, 1, 0, "oob"),
    (4, 4092, 0, 0, "uniform"),
    (5, 2048, 0, 1, "mix"),
    (6, 1024, 1, 0, "mix"),
    (6, 4, 0, 0, "uniform"),
    # d <= 1 stores Z rotated by the tune bin (ddc_persistent.hip, ZROT): tune bins just
    # below / above a 256-bin block boundary, where lanes split between two rotations
    (0, 1020, 0, 0, "mix"),
    (0, 3844, 0, 1, "bench"),
    (1, 260, 1, 0, "uniform"),
    (1, 2044, 0, 0, "mix"),
    # strong out-of-band tone + weak in-band tone at the BASELINE configs' tune bin (strict bar):
    # C2 (d=0), the C3 decimation sweep (d=1..4) and C4 (d=1, lsb, rand)
    (0, 1024, 0, 0, "oob"),
    (1, 1024, 0, 0, "oob"),
    (2, 1024, 0, 0, "oob"),
    (3, 1024, 0, 0, "oob"),
    (4, 1024, 0, 0, "oob"),
    (1, 1024, 1, 1, "oob"),
]


@pytest.mark.parametrize("d,tb,lsb,rand,src", CASES)
def test_single_channel_parity(torch_dev, ddc, oracle, H, d, tb, lsb, rand, src):
    nblk = 4
    x = make_stream(nblk, src)
    y = run_device(torch_dev, ddc, x, nblk, d, tb, lsb, rand)
    r = oracle.r2iq(x, nblk, d, tb, lsb, rand, H=H)
    assert y.size == r.size == nblk * (32768 >> d)
    assert np.all(np.isfinite(y))
    err = oracle.max_rel_err(y, r)
    assert err <= TOL, f"max-rel-err {err:.3e} (rms {oracle.rms_rel_err(y, r):.3e})"


# Tune bins that are not multiples of 4 (the C ABI takes any bin in [0, 4096); setFreqOffset only
# produces multiples of 4, fft_mt_r2iq.cpp:104): at d = 0 they run the persistent kernel instead of
# the FS kernel, with its forward pass 2 on the il272 columns and Z rotated by the tune bin.
ODD_BINS = [(0, 1, 0, 0, "uniform"), (0, 1023, 1, 1, "mix"), (0, 2046, 0, 0, "uniform"), (0, 4095, 0, 1, "mix"),
            (0, 2049, 1, 0, "uniform"), (1, 3, 0, 0, "mix"), (1, 2047, 1, 1, "uniform"), (2, 1021, 0, 0, "mix"),
            (3, 2050, 0, 1, "uniform"), (6, 4093, 1, 0, "uniform")]


@pytest.mark.parametrize("d,tb,lsb,rand,src", ODD_BINS)
def test_tune_bins_not_multiple_of_4(torch_dev, ddc, oracle, H, d, tb, lsb, rand, src):
    nblk = 3
    x = make_stream(nblk, src)
    y = run_device(torch_dev, ddc, x, nblk, d, tb, lsb, rand)
    r = oracle.r2iq(x, nblk, d, tb, lsb, rand, H=H)
    assert np.all(np.isfinite(y))
    err = oracle.max_rel_err(y, r)
    assert err <= TOL, f"max-rel-err {err:.3e}"


def test_zero_input_gives_zero(torch_dev, ddc):
    y = run_device(torch_dev, ddc, make_stream(2, "zeros"), 2, 0, 1024, 0, 0)
    assert np.all(y == 0)


def test_golden_fixture(torch_dev, ddc):
    with open(os.path.join(HERE, "golden", "iq_golden.json")) as f:
        g = json.load(f)
    for c in g["cases"]:
        x = make_stream(g["nblk"], c["source"])
        y = run_device(torch_dev, ddc, x, g["nblk"], c["d"], c["tunebin"], c["lsb"], c["rand"])
        assert y.size == c["n"]
        head = np.array([complex(*v) for v in c["head"]])
        tail = np.array([complex(*v) for v in c["tail"]])
        scale = c["max_abs"]
        assert np.max(np.abs(y[:64] - head)) / scale <= TOL
        assert np.max(np.abs(y[-64:] - tail)) / scale <= TOL
        assert abs(np.sum(np.abs(y.astype(np.complex128))) - c["sum_abs"]) / c["sum_abs"] <= 1e-5


def test_stateful_host_path_matches_stream(torch_dev, oracle, H):
    """process() across calls keeps the 4096-sample history (impl.hpp:32)."""
    from extio_sddc_amd import R2iq
    nblk = 6
    x = make_stream(nblk, "mix")
    with R2iq(gain=1.0) as r:
        r.setDecimate(1)
        r.setTuneBin(1024)
        r.TurnOn()
        parts = [r.process(x[4096:4096 + 2 * 65536]), r.process(x[4096 + 2 * 65536:4096 + 3 * 65536]),
                 r.process(x[4096 + 3 * 65536:])]
        y = np.concatenate(parts)
        ref = oracle.r2iq(x, nblk, 1, 1024, H=H)
        assert oracle.max_rel_err(y, ref) <= TOL
        # TurnOn() resets the history: the first block restarts from zeros
        r.TurnOn()
        y2 = r.process(x[4096:4096 + 65536])
        np.testing.assert_array_equal(y2, y[: y2.size])


def test_chunked_equals_one_shot_full_size(torch_dev, ddc):
    """Size-independent property at BASELINE size: a 2048-block stream processed in
    one launch equals the same stream processed as 8 halo'd segments (bit-exact)."""
    torch = torch_dev
    nblk, seg = 2048, 256
    g = torch.Generator(device="cuda").manual_seed(0x5DDC)
    d_in = torch.randint(-32768, 32767, (4096 + nblk * 65536,), dtype=torch.int16, device="cuda", generator=g)
    d_in[:4096] = 0
    from extio_sddc_amd import output_samples
    ddc.setDecimate(0)
    ddc.setTuneBin(1024)
    ddc.setSideband(False)
    ddc.updateRand(False)
    full = torch.empty(output_samples(0, nblk) * 2, dtype=torch.float32, device="cuda")
    ddc.process_device(d_in, nblk, full)
    per = output_samples(0, seg) * 2
    parts = torch.empty_like(full)
    for s in range(nblk // seg):
        ddc.process_device(d_in[s * seg * 65536:], seg, parts[s * per:(s + 1) * per])
    torch.cuda.synchronize()
    assert torch.equal(full, parts)
    assert torch.isfinite(full).all()


def test_linearity_full_size(torch_dev, ddc):
    """DDC is linear in its input: y(a) + y(b) == y(a+b) up to float rounding."""
    torch = torch_dev
    nblk = 512
    g = torch.Generator(device="cuda").manual_seed(7)
    a = torch.randint(-16384, 16383, (4096 + nblk * 65536,), dtype=torch.int16, device="cuda", generator=g)
    b = torch.randint(-16384, 16383, (4096 + nblk * 65536,), dtype=torch.int16, device="cuda", generator=g)
    from extio_sddc_amd import output_samples
    ddc.setDecimate(2)
    ddc.setTuneBin(2048)
    ddc.setSideband(False)
    ddc.updateRand(False)
    n = output_samples(2, nblk) * 2
    ya, yb, yab = (torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(3))
    ddc.process_device(a, nblk, ya)
    ddc.process_device(b, nblk, yb)
    ddc.process_device(a + b, nblk, yab)
    torch.cuda.synchronize()
    err = (ya + yb - yab).abs().max() / yab.abs().max()
    assert err.item() <= TOL


@pytest.mark.parametrize("d", [0, 1, 2, 3, 4, 5, 6])
def test_channels_match_single_channel(torch_dev, ddc, oracle, H, d):
    torch = torch_dev
    from extio_sddc_amd import output_samples
    nblk = 3
    x = make_stream(nblk, "mix")
    tbs = [0, 4, 1024, 2048, 3000, 4092, 284, 1228, 512, 3884]
    ddc.setDecimate(d)
    ddc.setSideband(False)
    ddc.updateRand(False)
    d_in = torch.from_numpy(x).to("cuda")
    per = output_samples(d, nblk) * 2
    out = torch.full((len(tbs), per), float("nan"), dtype=torch.float32, device="cuda")
    ddc.process_channels_device(d_in, nblk, tbs, out)
    torch.cuda.synchronize()
    y = out.cpu().numpy()
    for c, tb in enumerate(tbs):
        r = oracle.r2iq(x, nblk, d, tb, H=H)
        yc = y[c].view(np.complex64)
        assert oracle.max_rel_err(yc, r) <= TOL, f"channel {c} tb {tb}"


def test_bad_arguments_raise(torch_dev, ddc):
    from extio_sddc_amd import DDCError
    with pytest.raises(DDCError):
        ddc.setDecimate(7)
    with pytest.raises(DDCError):
        ddc.setTuneBin(4096)
    with pytest.raises(DDCError):
        ddc.process(np.zeros(1000, np.int16))


def test_block_limit_and_empty_calls(torch_dev, ddc):
    """nblk outside 1..SDDC_DDC_MAX_BLOCKS is refused before any device work (32-bit output
    indexing in the kernels); an empty host call is refused too."""
    from extio_sddc_amd import DDCError
    from extio_sddc_amd._lib import check
    torch = torch_dev
    x = torch.zeros(4096 + 65536, dtype=torch.int16, device="cuda")
    y = torch.zeros(2 * 32768, dtype=torch.float32, device="cuda")
    for bad in (0, -1, 32769):
        with pytest.raises(DDCError):
            check(ddc._L.sddc_ddc_process_device(ddc._h, x.data_ptr(), bad, y.data_ptr(), None))
    with pytest.raises(DDCError):
        ddc.process(np.zeros(0, np.int16))


def test_max_blocks_one_launch(torch_dev, ddc):
    """SDDC_DDC_MAX_BLOCKS (32768 blocks = 2^31 samples, 4 GiB in, 8 GiB out) in one launch
    equals the same stream as two halo'd halves, bit-exact; nothing is left unwritten."""
    torch = torch_dev
    from extio_sddc_amd import output_samples
    nblk, half = 32768, 16384
    g = torch.Generator(device="cuda").manual_seed(0x5DDC + 1)
    d_in = torch.randint(-32768, 32767, (4096 + nblk * 65536,), dtype=torch.int16, device="cuda", generator=g)
    ddc.setDecimate(0)
    ddc.setTuneBin(1024)
    ddc.setSideband(False)
    ddc.updateRand(False)
    n = output_samples(0, nblk) * 2
    full = torch.full((n,), float("nan"), dtype=torch.float32, device="cuda")
    ddc.process_device(d_in, nblk, full)
    parts = torch.full((n,), float("nan"), dtype=torch.float32, device="cuda")
    ddc.process_device(d_in, half, parts[: n // 2])
    ddc.process_device(d_in[half * 65536:], half, parts[n // 2:])
    torch.cuda.synchronize()
    assert torch.isfinite(full).all()
    assert torch.equal(full, parts)
    del d_in, full, parts
    torch.cuda.empty_cache()
