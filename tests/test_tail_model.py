"""The d >= 2 inverse tails of r2iq_persistent_kernel (ddc_persistent.hip: tail_pass, wg_pass)
restated in numpy (tools/r4_tail_model.py): each radix schedule reproduces the inverse DFT, and
the LDS layouts the kernel hard-codes (tail_swz, wg_swz) are permutations with no bank conflict
on any read or write pattern of the passes.  CPU only."""
from __future__ import annotations

import importlib.util
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("r4m", os.path.join(ROOT, "tools", "r4_tail_model.py"))
M = importlib.util.module_from_spec(spec)
spec.loader.exec_module(M)

# the kernel's layouts (ddc_persistent.hip)
TAIL_SWZ = {512: lambda e: e ^ ((e >> 3) & 31), 256: lambda e: e ^ ((e >> 2) & 31),
            128: lambda e: e ^ ((e >> 2) & 31), 64: lambda e: e ^ ((e >> 1) & 31)}
WG_SWZ = {1024: lambda e: e ^ ((e >> 2) & 31), 2048: lambda e: e ^ ((e >> 2) & 31) ^ ((e >> 5) & 7)}


@pytest.mark.parametrize("N", [512, 256, 128, 64])
def test_wave0_tail(N):
    rng = np.random.default_rng(N)
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    A = TAIL_SWZ[N]
    assert sorted(A(e) for e in range(N)) == list(range(N))
    y = M.stockham_inv(x, N, A)
    ref = np.fft.ifft(x) * N
    assert np.abs(y - ref).max() / np.abs(ref).max() < 1e-12
    assert M.conflicts(A, N) == (1, 0)


@pytest.mark.parametrize("N", [1024, 2048])
def test_workgroup_tail(N):
    rng = np.random.default_rng(N)
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    A = WG_SWZ[N]
    assert sorted(A(e) for e in range(N)) == list(range(N))
    y = M.stockham_wg(x, N, A)
    ref = np.fft.ifft(x) * N
    assert np.abs(y - ref).max() / np.abs(ref).max() < 1e-12
    assert M.conflicts_wg(A, N) == (1, 0)
