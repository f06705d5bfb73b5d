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


@pytest.mark.parametrize("N", [256, 512])
def test_quad_first_pass(N):
    """d = 4 / d = 3: the first Stockham pass run across the quads of all four waves (thread
    t = 4 j + q holds the inputs of butterfly j at r = q (N = 256) or r = 2 q, 2 q + 1 (N = 512),
    broadcasts them by DPP, runs the whole DFT-R and keeps its own outputs) leaves the LDS buffer
    exactly as wave 0's pass 0 does (element R j + r), so wave 0 starts at pass 1"""
    rng = np.random.default_rng(N)
    x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    R = M.SCHED[N][0]
    T = N // R
    ref = np.zeros(N, complex)   # tail_pass<N, 0>: thread j writes (j / 1) R + r
    for j in range(T):
        ref[R * j: R * j + R] = np.fft.ifft(np.array([x[j + T * r] for r in range(R)])) * R
    per = R // 4   # inputs per lane
    got = np.full(N, np.nan + 0j)
    for t in range(4 * T):
        j, q = t >> 2, t & 3
        held = {per * q + h: x[j + T * (per * q + h)] for h in range(per)}   # the split, in butterfly order
        quad = {}
        for lane in range(4):   # quad_bcast of every lane's values
            for h in range(per):
                quad[per * lane + h] = x[j + T * (per * lane + h)]
        assert all(quad[k] == v for k, v in held.items())
        y = np.fft.ifft(np.array([quad[r] for r in range(R)])) * R
        for h in range(per):
            got[per * t + h] = y[per * q + h]   # slot R j + r = per t + h
    assert np.abs(got - ref).max() < 1e-12
