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


def test_d3_two_half_tail():
    """d = 3 (ddc_persistent.hip, tail_emit_half): the 512-point inverse as a radix-2 step in the
    split's registers (E_p[m] = (X[m] + (-1)^p X[m + 256]) e^{2 pi i m p / 512}, m < 256), the d = 4
    Stockham tail (4-4-4-4, layout tail_swz<256>) on each half, and half p's output y'[n'] placed
    at n = 2 n' + p; the kept range of frame k (y[0, 384) for k >= 1, y[128, 384) for k = 0) is
    what the two waves store (u[r] = y'[t + 64 r], r < 3, r >= 1 at k = 0)."""
    rng = np.random.default_rng(512)
    x = rng.standard_normal(512) + 1j * rng.standard_normal(512)
    m = np.arange(256)
    # the kernel's twiddle: TW<+1>(v, W_4096^{8m}) = v * conj(e^{-2 pi i 8 m / 4096})
    w = np.conj(np.exp(-2j * np.pi * 8 * m / 4096))
    halves = [x[:256] + x[256:], (x[:256] - x[256:]) * w]
    y = np.zeros(512, complex)
    for p, e in enumerate(halves):
        yh = M.stockham_inv(e, 256, TAIL_SWZ[256])
        y[2 * np.arange(256) + p] = yh
    ref = np.fft.ifft(x) * 512
    assert np.abs(y - ref).max() / np.abs(ref).max() < 1e-12
    # the stores: lane t of wave p writes u[r] = y'[t + 64 r] at element 2 t + p + 128 r
    for k, rs in ((0, (1, 2)), (1, (0, 1, 2))):
        kept = sorted(2 * (t + 64 * r) + p for p in (0, 1) for t in range(64) for r in rs)
        assert kept == list(range(128 if k == 0 else 0, 384))
