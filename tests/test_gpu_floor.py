"""The float32 parity floor, measured (pytest -m gpu).

north_star asks for IQ "within 1e-5 of the FFTW reference".  The reference's own path is float32
(FFTW single precision), and on the adversarial "oob" input (a strong out-of-band tone, a weak
in-band one) every float32 implementation sits close to 1e-5 of the exact answer: the oracle's
float32 port of the reference algorithm (oracle/ddc_oracle.c, _f32), the library's AVX2 CPU
backend and the HIP kernels each land at 5e-6 .. 9e-6 of the f64 oracle at d = 3, 4, and two such
float32 paths can differ from each other by more than 1e-5 ("The float32 floor").
So the bar the tests hold is against the exact (f64) answer, and this test records, per case,
three numbers: HIP vs f64, port vs f64 and HIP vs port; it asserts that the HIP path is within
1e-5 of exact and, where the port itself sits near the floor (>= 2e-6: the d = 3, 4 cases), at
the float32 floor (<= 1.2 x the port's own error).  Far below the floor (d = 0: ~4e-7) the
operation orders differ (the fused split modulates the output instead of shifting bins) and the
bar is a tenth of the tolerance instead.  With SDDC_PARITY_RECORD set, the numbers are appended to
that JSON-lines file.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

pytestmark = pytest.mark.gpu

TOL = 1e-5
FLOOR_FACTOR = 1.2
AT_FLOOR = 2e-6     # the port's own error from which the floor comparison applies

CASES = [
    # d, tunebin, lsb, rand: the BASELINE C3 configs' out-of-band cases at d = 3, 4 (and d = 4 at
    # tune bin 0 with the sideband inverted, the worst one the verdict measured)
    (3, 1024, 0, 0),
    (4, 1024, 0, 0),
    (4, 0, 1, 0),
    (0, 1024, 0, 0),
]


def _record(row):
    path = os.environ.get("SDDC_PARITY_RECORD")
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(row) + "\n")


@pytest.mark.parametrize("d,tb,lsb,rand", CASES)
def test_float32_floor(oracle, d, tb, lsb, rand):
    import torch
    from extio_sddc_amd import DEVICE_CPU, R2iq, output_samples
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    nblk = 4
    x = make_stream(nblk, "oob")
    H64, H32 = oracle.filter_bank(1.0), oracle.filter_bank(1.0, np.float32)
    exact = oracle.r2iq(x, nblk, d, tb, lsb, rand, H=H64)
    port = oracle.r2iq(x, nblk, d, tb, lsb, rand, dtype=np.float32, H=H32)
    with R2iq(gain=1.0, device=0) as r:
        r.setDecimate(d)
        r.setTuneBin(tb)
        r.setSideband(bool(lsb))
        r.updateRand(bool(rand))
        d_in = torch.from_numpy(x).to("cuda")
        out = torch.full((output_samples(d, nblk) * 2,), float("nan"), dtype=torch.float32, device="cuda")
        r.process_device(d_in, nblk, out)
        torch.cuda.synchronize()
        hip = out.cpu().numpy().view(np.complex64)
    with R2iq(gain=1.0, device=DEVICE_CPU) as c:
        c.setDecimate(d)
        c.setTuneBin(tb)
        c.setSideband(bool(lsb))
        c.updateRand(bool(rand))
        cpu = c.process(np.ascontiguousarray(x[4096:4096 + nblk * 65536]))
    e = oracle.max_rel_err
    row = {"d": d, "tunebin": tb, "lsb": lsb, "rand": rand, "source": "oob",
           "hip_vs_f64": e(hip, exact), "port_f32_vs_f64": e(port, exact), "hip_vs_port_f32": e(hip, port),
           "cpu_backend_vs_f64": e(cpu, exact), "cpu_backend_vs_port_f32": e(cpu, port)}
    _record(row)
    print(json.dumps(row))
    assert row["hip_vs_f64"] <= TOL, row
    if row["port_f32_vs_f64"] >= AT_FLOOR:
        assert row["hip_vs_f64"] <= FLOOR_FACTOR * row["port_f32_vs_f64"], row
    else:
        assert row["hip_vs_f64"] <= 0.1 * TOL, row


# Leakage-only channels (test_gpu_sweep.py): a strong tone tuned far outside the channel, whose
# output is only the tone's stopband leakage, 40-70 dB below full scale.  float32 rounding noise
# scales with the strong tone, so relative to such a channel's own peak every float32 path lands
# near or above 1e-5 (the port: 4e-6 .. 6e-5 over the draws below).  Such a draw is held to the
# float32 floor itself: the HIP error against the f64 oracle next to the error of the oracle's
# float32 port of the reference algorithm (radix-4 Stockham with exactly rounded table twiddles,
# the class of FFTW's float path, impl.hpp:88, 98) on the same input, each draw within
# FLOOR_FACTOR (1.2) x the port, as the floor cases above, and the geometric mean over the draws
# at most 1.  The error is the forward FFT's float32 noise (tools/fp32_model.py: an exact forward
# transform leaves < 1.3e-7); its ratio to the port's moves by +-40 % between equivalent
# reorderings, so the HIP path has to be more accurate than the port on average to stay under
# 1.2x on every draw: forward pass 2's twiddles from six exactly rounded anchors
# (fft_device.hpp twiddle_anchor6, round 5) give geomean 0.82, max 1.16 over these 24 draws on
# the GPU (profiles/r05/parity/floor_anchor6.jsonl; the three-term recurrence before it: 0.92,
# max 1.41).  The sweep's three leakage-only draws come first.
SWEEP_LEAK_DRAWS = [(3, 2708, 0, 4, 310165425), (5, 2408, 1, 3, 546231597), (5, 2044, 0, 3, 826057796)]
LEAK_DB = -40.0


def _leak_draws(n_extra=21, seed=0x5DDC + 77):
    from oracle import oracle as O
    rng = np.random.default_rng(seed)
    out = list(SWEEP_LEAK_DRAWS)
    H = O.filter_bank(1.0)
    while len(out) < len(SWEEP_LEAK_DRAWS) + n_extra:
        d, tb, lsb, s = int(rng.integers(3, 7)), 4 * int(rng.integers(0, 1024)), int(rng.integers(0, 2)), int(rng.integers(1, 1 << 30))
        x = make_stream(3, "bench", seed=s)
        r = O.r2iq(x, 3, d, tb, lsb, 0, H=H)
        if 20 * np.log10(np.abs(r).max() / (1024.0 * np.abs(x.astype(np.float64)).max())) < LEAK_DB:
            out.append((d, tb, lsb, 3, s))
    return out


def test_leakage_draws_at_float32_floor(oracle):
    import torch
    from extio_sddc_amd import R2iq, output_samples
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    H64, H32 = oracle.filter_bank(1.0), oracle.filter_bank(1.0, np.float32)
    ratios = []
    with R2iq(gain=1.0, device=0) as r:
        for d, tb, lsb, nblk, seed in _leak_draws():
            x = make_stream(nblk, "bench", seed=seed)
            exact = oracle.r2iq(x, nblk, d, tb, lsb, 0, H=H64)
            port = oracle.r2iq(x, nblk, d, tb, lsb, 0, dtype=np.float32, H=H32)
            r.setDecimate(d)
            r.setTuneBin(tb)
            r.setSideband(bool(lsb))
            r.updateRand(False)
            out = torch.full((output_samples(d, nblk) * 2,), float("nan"), dtype=torch.float32, device="cuda")
            r.process_device(torch.from_numpy(x).to("cuda"), nblk, out)
            torch.cuda.synchronize()
            hip = out.cpu().numpy().view(np.complex64)
            assert np.all(np.isfinite(hip))
            row = {"test": "leakage draw at the float32 floor", "d": d, "tunebin": tb, "lsb": lsb, "nblk": nblk,
                   "seed": seed, "peak_db_re_full_scale": 20 * np.log10(
                       np.abs(exact).max() / (1024.0 * np.abs(x.astype(np.float64)).max())),
                   "hip_vs_f64": oracle.max_rel_err(hip, exact), "port_f32_vs_f64": oracle.max_rel_err(port, exact)}
            row["ratio"] = row["hip_vs_f64"] / row["port_f32_vs_f64"]
            _record(row)
            print(json.dumps(row))
            ratios.append(row["ratio"])
            assert row["ratio"] <= FLOOR_FACTOR, row
    gm = float(np.exp(np.mean(np.log(ratios))))
    _record({"test": "leakage draws: geometric mean HIP / port", "n": len(ratios), "geomean": gm,
             "max": float(np.max(ratios)), "median": float(np.median(ratios))})
    print(f"leakage draws: n={len(ratios)} geomean HIP/port {gm:.3f} max {np.max(ratios):.3f}")
    assert gm <= 1.0, f"geometric mean of HIP / port {gm:.3f} over {len(ratios)} leakage draws"
