"""The oracle (oracle/ddc_oracle.c) pinned before it is trusted (CPU only).

- a5 filter design: bit-exact against the reference's own KaiserWindow (Core/fir.cpp),
  via the committed fixture tests/golden/kaiser_taps.json and, where the reference is
  mounted, live against oracle/_ref/libref_fir.so.
- FFTs: against the DFT definition (numpy float64).
- a2-a7 pipeline: against an independent numpy float64 restatement
  (oracle/ddc_oracle_np.py); f32 port against f64 (the reference's own float path is
  <= 2.6e-6 from exact).
- The reference tests' assertions that touch this path (unittest/core_test.cpp:167 block
  length; signal_integrity_test.cpp properties) re-asserted on the oracle.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def kaiser_fixture():
    with open(os.path.join(HERE, "golden", "kaiser_taps.json")) as f:
        return json.load(f)


def _hex_to_f32(h):
    return np.array([int(v, 16) for v in h], np.uint32).view(np.float32)


def test_kaiser_taps_bit_exact_vs_reference_fixture(oracle, kaiser_fixture):
    for e in kaiser_fixture["per_d"]:
        taps = oracle.filter_taps(e["d"])
        ref = _hex_to_f32(e["taps_f32_hex"])
        assert np.array_equal(taps.view(np.uint32), ref.view(np.uint32)), f"d={e['d']}"
        est = oracle.kaiser(0, 120.0, e["fpass"], e["fstop"])
        assert est == e["estimate"]
    for e in kaiser_fixture["extra"]:
        n, a, fp, fs = e["args"]
        if "taps_f32_hex" in e:
            got = oracle.kaiser(n, a, fp, fs)
            assert np.array_equal(got.view(np.uint32), _hex_to_f32(e["taps_f32_hex"]).view(np.uint32))
        else:
            assert oracle.kaiser(n, a, fp, fs) == e["estimate"]


def test_tap_estimates_match_reference_printout(oracle):
    # NDEBUG-off estimate at fft_mt_r2iq.cpp:51-67
    est = [oracle.kaiser(0, 120.0, 0.85 * (64.0 / 2 ** d) / 128.0, 1.1 * (64.0 / 2 ** d) / 128.0) for d in range(7)]
    assert est == [63, 125, 250, 500, 999, 1998, 3995]


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libref_fir.so")),
                    reason="reference fir.cpp not built (needs /root/reference)")
def test_kaiser_live_vs_reference_build(oracle):
    rng = np.random.default_rng(3)
    for _ in range(20):
        n = int(rng.integers(3, 400))
        a = float(rng.choice([15.0, 30.0, 45.0, 60.0, 90.0, 120.0]))
        fp = float(rng.uniform(0.005, 0.3))
        fs = fp + float(rng.uniform(0.01, 0.2))
        assert np.array_equal(oracle.kaiser(n, a, fp, fs).view(np.uint32),
                              oracle.ref_kaiser(n, a, fp, fs).view(np.uint32))
        assert oracle.kaiser(-n, a, fp, fs) == oracle.ref_kaiser(-n, a, fp, fs)


@pytest.mark.parametrize("n", [64, 128, 256, 512, 1024, 2048, 4096, 8192])
def test_fft_matches_dft_definition(oracle, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    assert np.max(np.abs(oracle.fft(x, -1) - np.fft.fft(x))) < 1e-9 * n
    assert np.max(np.abs(oracle.fft(x, +1) - np.fft.ifft(x) * n)) < 1e-9 * n


def test_forward_r2c_matches_numpy(oracle):
    x = make_stream(1, "uniform", history=False)[:8192]
    for rand in (0, 1):
        X = oracle.forward_r2c(x, rand)
        from oracle.ddc_oracle_np import derand
        ref = np.fft.rfft(derand(x, bool(rand)).astype(np.float64))
        assert np.max(np.abs(X - ref)) / np.max(np.abs(ref)) < 1e-13


def test_filter_bank_matches_numpy_restatement(oracle):
    from oracle import ddc_oracle_np as N
    H = oracle.filter_bank(7.8e-8)
    Hn = N.filter_bank([oracle.filter_taps(d) for d in range(7)], 7.8e-8)
    assert np.max(np.abs(H - Hn)) / np.max(np.abs(H)) < 1e-12


@pytest.mark.parametrize("d,tb,lsb,rand,src", [
    (0, 1024, 0, 0, "mix"), (1, 284, 1, 1, "uniform"), (2, 0, 0, 1, "mix"),
    (3, 4092, 1, 0, "bench"), (4, 3888, 0, 0, "oob"), (6, 2048, 1, 1, "mix"),
])
def test_pipeline_c_vs_numpy_restatement(oracle, d, tb, lsb, rand, src):
    from oracle import ddc_oracle_np as N
    nblk = 2
    x = make_stream(nblk, src)
    H = oracle.filter_bank(1.0)
    a = oracle.r2iq(x, nblk, d, tb, lsb, rand, H=H)
    b = N.r2iq(x, nblk, d, tb, bool(lsb), bool(rand), H[d])
    assert oracle.max_rel_err(b, a) < 1e-12


@pytest.mark.parametrize("d", range(7))
def test_f32_port_within_reference_accuracy(oracle, d):
    x = make_stream(2, "mix")
    a = oracle.r2iq(x, 2, d, 1024)
    b = oracle.r2iq(x, 2, d, 1024, dtype=np.float32)
    assert oracle.max_rel_err(b, a) < 5e-6


def test_golden_iq_fixture_reproduces(oracle):
    with open(os.path.join(HERE, "golden", "iq_golden.json")) as f:
        g = json.load(f)
    H = oracle.filter_bank(1.0)
    for c in g["cases"]:
        x = make_stream(g["nblk"], c["source"])
        y = oracle.r2iq(x, g["nblk"], c["d"], c["tunebin"], c["lsb"], c["rand"], H=H)
        head = np.array([complex(*v) for v in c["head"]])
        assert np.max(np.abs(y[:64] - head)) <= 1e-9 * c["max_abs"]
        assert abs(np.sum(np.abs(y)) - c["sum_abs"]) <= 1e-9 * c["sum_abs"]


# ---- properties the reference's own tests assert on this path --------------------------

@pytest.mark.parametrize("d", range(5))
def test_block_length_is_32768_per_2d_blocks(oracle, d):
    # core_test.cpp:149-174 R2IQTest: every callback carries transferSamples/2 = 32768 samples,
    # i.e. 2^d input blocks -> one 32768-sample output block
    nblk = 1 << d
    y = oracle.r2iq(make_stream(nblk, "bench"), nblk, d, 1024)
    assert y.size == 32768


def test_zero_input_zero_output(oracle):
    # signal_integrity_test.cpp ZeroInput: RMS < 1
    y = oracle.r2iq(make_stream(2, "zeros"), 2, 0, 1024)
    assert np.all(y == 0)


def test_amplitude_scaling_and_linearity(oracle):
    # signal_integrity_test.cpp AmplitudeLinearity: 2x amplitude -> output ratio in (1, 4)
    x = make_stream(2, "bench")
    x2 = (x.astype(np.int32) // 2).astype(np.int16)
    a = oracle.r2iq(x, 2, 0, 1024)
    b = oracle.r2iq(x2, 2, 0, 1024)
    r = np.sqrt(np.mean(np.abs(a[8192:]) ** 2) / np.mean(np.abs(b[8192:]) ** 2))
    assert 1.9 < r < 2.1


def test_inband_tone_lands_at_expected_frequency(oracle):
    # a tone at bin tb + 100 (8192-point grid) appears at +100/4096 cycles/sample after d=0
    n = 4096 + 4 * 65536
    t = np.arange(n)
    f = (1024 + 100) / 8192.0
    x = np.round(8000 * np.cos(2 * np.pi * f * t)).astype(np.int16)
    x[:4096] = 0
    y = oracle.r2iq(x, 4, 0, 1024)[16384:]
    spec = np.abs(np.fft.fft(y))
    k = int(np.argmax(spec))
    assert abs(k / y.size - 100 / 4096.0) < 2.0 / y.size


def test_set_freq_offset_semantics(oracle):
    # fft_mt_r2iq.cpp:101-109
    assert oracle.set_freq_offset(0.25, 0) == (1024, 0.0)
    tb, fc = oracle.set_freq_offset(0.3, 2)
    assert tb == int(np.float32(0.3) * 1024) * 4 and tb % 4 == 0
    assert np.isclose(fc, (tb / 4096 - np.float32(0.3)) * 4, atol=1e-7)
