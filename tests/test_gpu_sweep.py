"""Seeded random parity sweep on a real MI355X (pytest -m gpu): 48 configurations drawn from
d in 0..6, any legal tune bin (multiple of 4, the setFreqOffset grid, fft_mt_r2iq.cpp:104),
sideband, rand, the synthetic sources and 1..5 blocks, each checked against the f64 oracle.

Bar: IQ max-rel-err <= 1e-5 (north_star) for every channel whose output reaches -40 dB of
full scale; a channel below that is "leakage-only": its strict error is held to the float32
floor (<= 1.2x the oracle's float32 port of the reference algorithm on the same input, the bar of
the 24 draws of test_gpu_floor.py), and, as the documented secondary, its
error measured against the -40 dB level (``leak_aware_err``) to 1e-5.

Full scale S = 1024 * max|x|: the peak IQ an in-band tone of the input's peak amplitude gives at
gain 1 (SURVEY.md §8(a) output contract: |IQ| ~ A * 4096 * (2048/8192) * sum(taps)).  A
leakage-only channel holds only the stopband leakage of a strong out-of-band tone (the "bench"
tone tuned far away), so max|r| is tiny while float32 rounding scales with the strong tone: the
criterion is max|y - r| <= 1e-5 * max(max|r|, 10^(-40/20) * S), i.e. the error stays >= 140 dB
below the strong tone.  Numbers (seeded draws, the oracle's float32 port as a stand-in for any
float32 FFT path, the reference's FFTW included): the three leakage-only draws sit at -48.0,
-56.6 and -58.7 dB with strict errors 1.41e-5, 9.9e-6 and 1.73e-5 and leakage-aware errors
5.6e-6, 1.5e-6 and 2.0e-6; every other draw is at >= -36 dB and held to the strict bar."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

pytestmark = pytest.mark.gpu

TOL = 1e-5
LEAK_DB = -40.0   # below this level (re full scale) a channel is leakage-only
FLOOR_FACTOR = 1.2   # a leakage-only draw's strict error against the float32 port's (test_gpu_floor.py)
SOURCES = ["mix", "uniform", "bench", "oob"]


def _cases(n=48, seed=0x5DDC):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        d = int(rng.integers(0, 7)) if i >= 4 else 0           # a few d = 0 cases for the wave kernel
        out.append((d, 4 * int(rng.integers(0, 1024)), int(rng.integers(0, 2)), int(rng.integers(0, 2)),
                    SOURCES[int(rng.integers(0, len(SOURCES)))], int(rng.integers(1, 6)), int(rng.integers(1, 1 << 30))))
    return out


def _record(row):
    path = os.environ.get("SDDC_PARITY_RECORD")
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(row) + "\n")


def leak_aware_err(y, r, x) -> tuple[float, bool]:
    """(error, leakage_only): max|y - r| / max(max|r|, -40 dB of full scale 1024 * max|x|)."""
    full = 1024.0 * float(np.abs(x.astype(np.float64)).max())
    floor = 10 ** (LEAK_DB / 20) * full
    peak = float(np.max(np.abs(r)))
    return float(np.max(np.abs(y - r))) / max(peak, floor), peak < floor


@pytest.fixture(scope="module")
def ddc():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    from extio_sddc_amd import R2iq
    r = R2iq(gain=1.0, device=0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def H(oracle):
    return oracle.filter_bank(1.0)


@pytest.fixture(scope="module")
def H32(oracle):
    return oracle.filter_bank(1.0, np.float32)


@pytest.mark.parametrize("d,tb,lsb,rand,src,nblk,seed", _cases())
def test_random_config_parity(ddc, oracle, H, H32, d, tb, lsb, rand, src, nblk, seed):
    import torch
    from extio_sddc_amd import output_samples
    x = make_stream(nblk, src, seed=seed)
    r = oracle.r2iq(x, nblk, d, tb, lsb, rand, H=H)
    d_in = torch.from_numpy(x).to("cuda")
    ddc.setDecimate(d)
    ddc.setTuneBin(tb)
    ddc.setSideband(bool(lsb))
    ddc.updateRand(bool(rand))
    out = torch.full((output_samples(d, nblk) * 2,), float("nan"), dtype=torch.float32, device="cuda")
    ddc.process_device(d_in, nblk, out)
    torch.cuda.synchronize()
    y = out.cpu().numpy().view(np.complex64)
    assert np.all(np.isfinite(y))
    err, leak = leak_aware_err(y, r, x)
    if leak:
        # primary: at the float32 floor, i.e. within FLOOR_FACTOR = 1.2x of the oracle's float32
        # port of the reference algorithm on the same input, the bar test_gpu_floor.py holds
        # its 24 leakage draws to (the float32 model of the kernel, tools/fp32_model.py, puts
        # this sweep's three leakage-only draws at 0.89, 0.92 and 0.75x the port); the -40 dB
        # rule stays as the documented secondary
        port = oracle.r2iq(x, nblk, d, tb, lsb, rand, dtype=np.float32, H=H32)
        strict, port_err = oracle.max_rel_err(y, r), oracle.max_rel_err(port, r)
        _record({"test": "sweep leakage-only draw", "d": d, "tunebin": tb, "lsb": lsb, "rand": rand,
                 "source": src, "nblk": nblk, "seed": seed,
                 "peak_db_re_full_scale": 20 * np.log10(float(np.max(np.abs(r))) / (1024.0 * float(
                     np.abs(x.astype(np.float64)).max()))),
                 "strict_max_rel_err": strict, "port_f32_max_rel_err": port_err, "leakage_aware_err": err})
        assert strict <= FLOOR_FACTOR * port_err, \
            f"leakage-only draw {strict:.3e} > {FLOOR_FACTOR} x port {port_err:.3e}"
    assert err <= TOL, f"{'leakage-aware' if leak else 'max-rel'} err {err:.3e}"


def _channel_cases(seed=0x5DDC + 1):
    """Two cases per d (0..6) plus one random d: channel counts across the 32-channel chunks of
    the d < 4 kernel and the 128-channel chunks of the d >= 4 kernel, groups of 2^d channels
    with idle slots, random (repeatable) tune bins, sideband and rand."""
    rng = np.random.default_rng(seed)
    out = []
    for d in list(range(7)) * 2 + [int(rng.integers(0, 7))]:
        nch = int(rng.integers(1, 81)) if d < 4 else int(rng.integers(1, 300))
        out.append((d, nch, int(rng.integers(0, 2)), int(rng.integers(0, 2)),
                    ["mix", "uniform"][int(rng.integers(0, 2))], int(rng.integers(1, 1 << 30))))
    # fewer channels than one group in flight (2^d at d < 4), and exactly one 128-channel chunk + 1
    out += [(3, 1, 0, 0, "mix", 7), (2, 3, 1, 1, "uniform", 8), (4, 129, 0, 1, "mix", 9)]
    return out


@pytest.mark.parametrize("d,nch,lsb,rand,src,seed", _channel_cases())
def test_random_channels(ddc, oracle, H, d, nch, lsb, rand, src, seed):
    """Many-channel kernels (d < 4: r2iq_channels_p_kernel; d >= 4: r2iq_channels_v2_kernel) on
    random tune-bin sets: every channel within 1e-5 of the single-channel kernel on the same
    stream, and three random channels within 1e-5 of the f64 oracle.  Broadband sources only,
    so no channel is leakage-only (see the module docstring)."""
    import torch
    from extio_sddc_amd import output_samples
    rng = np.random.default_rng(seed)
    nblk = 2
    tbs = [4 * int(v) for v in rng.integers(0, 1024, nch)]
    x = make_stream(nblk, src, seed=seed)
    d_in = torch.from_numpy(x).to("cuda")
    ddc.setDecimate(d)
    ddc.setSideband(bool(lsb))
    ddc.updateRand(bool(rand))
    per = output_samples(d, nblk) * 2
    out = torch.full((nch, per), float("nan"), dtype=torch.float32, device="cuda")
    ddc.process_channels_device(d_in, nblk, tbs, out)
    single = torch.empty(per, dtype=torch.float32, device="cuda")
    worst = 0.0
    for c in range(nch):
        ddc.setTuneBin(tbs[c])
        ddc.process_device(d_in, nblk, single)
        torch.cuda.synchronize()
        worst = max(worst, ((out[c] - single).abs().max() / single.abs().max()).item())
    assert torch.isfinite(out).all()
    assert worst <= TOL, f"channels vs single: {worst:.3e}"
    y = out.cpu().numpy()
    for c in rng.choice(nch, size=min(3, nch), replace=False):
        r = oracle.r2iq(x, nblk, d, tbs[c], lsb, rand, H=H)
        err = oracle.max_rel_err(y[c].view(np.complex64), r)
        assert err <= TOL, f"channel {c} tb {tbs[c]}: {err:.3e}"
