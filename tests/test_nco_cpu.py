"""Fine-tune NCO oracle (oracle/ddc_oracle.c oracle_nco_*) pinned to the reference's own
mixer: pf_mixer.cpp ALGO H (shift_limited_unroll_C_sse_{init,inp_c}, :750-856), compiled
into oracle/_ref by `make -C oracle ref` here, and the committed reference outputs in
tests/golden/nco_golden.json (the GPU box has no reference tree).  Bar: bit-exact."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))


def _golden():
    with open(os.path.join(HERE, "golden", "nco_golden.json")) as f:
        return json.load(f)


def _hex_to_c64(words):
    return np.array([int(w, 16) for w in words], np.uint32).view(np.float32).view(np.complex64)


def _input(seed, n):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) * np.float32(1000.0)


def test_oracle_nco_matches_golden_chunks():
    for c in _golden()["cases"]:
        x = _input(c["seed"], sum(c["chunks"]))
        nco = O.Nco(c["fc"])
        y, o = [], 0
        for n in c["chunks"]:
            y.append(nco.apply(x[o:o + n]))
            o += n
        y = np.concatenate(y)
        np.testing.assert_array_equal(y.view(np.uint32), _hex_to_c64(c["out_f32_hex"]).view(np.uint32))


def test_oracle_nco_matches_golden_long_run():
    """64 buffers of 32768: the float recurrence's phase drift is reproduced exactly."""
    for c in _golden()["long"]:
        nco = O.Nco(c["fc"])
        ones = np.ones(c["buffer"], np.complex64)
        probes = []
        for b in range(c["buffers"]):
            y = nco.apply(ones)
            probes.append(y[(b * 997) % c["buffer"]])
        np.testing.assert_array_equal(np.array(probes, np.complex64).view(np.uint32),
                                      _hex_to_c64(c["probe_f32_hex"]).view(np.uint32))


@pytest.mark.skipif(not O.ref_mixer_available(), reason="reference mixer not built (no /root/reference)")
@pytest.mark.parametrize("fc", [0.0123, -0.271, 0.4999, 1e-4, 0.25, -0.5])
def test_oracle_nco_matches_reference_mixer(fc):
    rng = np.random.default_rng(7)
    a, b = O.Nco(fc), O.RefMixer(fc)
    for n in [32768, 128, 4096, 32768 * 2, 4]:
        x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) * 3e3
        np.testing.assert_array_equal(a.apply(x).view(np.uint32), b.apply(x).view(np.uint32))


def test_exact_phase_would_not_match():
    """Why the product replicates the float recurrence instead of evaluating phase = n w in
    double: the reference drifts by > 1e-5 relative within one buffer."""
    fc = 0.0123
    y = O.Nco(fc).apply(np.ones(32768, np.complex64))
    inc = np.float64(np.float32(np.float32(2 * np.float32(fc)) * np.float32(np.pi)))
    exact = np.exp(1j * inc * np.arange(32768))
    assert np.max(np.abs(y - exact)) > 1e-4
