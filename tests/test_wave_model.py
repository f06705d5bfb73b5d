"""CPU check of the d = 0 wave kernel's lane/register/LDS bookkeeping (ddc_wave.hip, variant 3):
tools/wave_fft_model.py emulates the kernel's loads, in-register DFTs, per-lane tables, LDS
slots (row stride 33) and v_permlane32_swap in numpy and asserts, stage by stage, against the
direct DFT formulation, plus conflict-free LDS banking under the gfx950 rules.  The GPU
parity of the kernel itself is tests/test_gpu_wave.py."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import wave_fft_model as M  # noqa: E402


@pytest.mark.parametrize("tb", [0, 64, 1024, 2080, 4092])
def test_wave_model_matches_direct_formula(tb):
    rng = np.random.default_rng(tb + 1)
    s = rng.integers(-32768, 32768, 8192).astype(np.int16)
    P = rng.normal(size=4096) + 1j * rng.normal(size=4096)
    Q = rng.normal(size=4096) + 1j * rng.normal(size=4096)
    y, T = M.model_frame(s, tb, P, Q)
    yr, Tr = M.reference(s, tb, P, Q)
    assert np.allclose(T, Tr)
    assert np.max(np.abs(y - yr)) / np.max(np.abs(yr)) < 1e-12


def test_permlane32_swap_semantics():
    a, b = np.arange(64), 100 + np.arange(64)
    a2, b2 = M.permlane32_swap(a, b)
    assert np.array_equal(a2, np.concatenate([a[:32], b[:32]]))
    assert np.array_equal(b2, np.concatenate([a[32:], b[32:]]))
    # the two-swap rotation used by the kernel: swap(p0, p1); swap(p1, p0)
    p0, p1 = M.permlane32_swap(a, b)
    q1, q0 = M.permlane32_swap(p1, p0)
    assert np.array_equal(q1, M.rot32(a)) and np.array_equal(q0, M.rot32(b))
