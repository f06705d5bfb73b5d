"""The persistent kernel's (P, r) split x filter (round 6, ddc_persistent.hip build_split_filter_kernel,
ddc_frame_common.hpp split_pr), in tools/fp32_model.py's float32 model: T = P (Zk + i r conj Zc)
with P and r = Q / (i P) rounded to float32, and at bin 2048 (P = 0, r infinite) r = 2^64,
P = Q / (i 2^64).  Against the exact Zk P + conj(Zc) Q (the reference's split x filter,
fft_mt_r2iq_impl.hpp:84-98) at every d >= 1, with bin 2048 inside the band and at its edges."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import fp32_model as F  # noqa: E402
from oracle import oracle as O  # noqa: E402

HALF = 4096


@pytest.fixture(scope="module")
def H():
    return O.filter_bank(1.0)


def _spectrum(seed, frames=2):
    rng = np.random.default_rng(seed)
    z = rng.integers(-32768, 32768, size=(frames, HALF)) + 1j * rng.integers(-32768, 32768, size=(frames, HALF))
    return np.fft.fft(z, axis=1)


@pytest.mark.parametrize("d", [1, 2, 3, 4, 5, 6])
def test_split_pr_matches_exact(H, d):
    """float32 (P, r) split within 2^-21 of the exact one (relative to the frame's max), at tune
    bins with bin 2048 in band (middle, both edges) and out of band"""
    N = HALF >> d
    Z = _spectrum(d)
    for tb in (2048, 2048 - N // 2, 2048 + N // 2 - 4, 1024, 3000, 0, 4092):
        ex = F.split_filter(Z, d, tb, H[d], exact=True)
        pr = F.split_filter(Z, d, tb, H[d], form="pr")
        scale = np.abs(ex).max()
        assert np.abs(pr - ex).max() <= 2.0 ** -21 * scale, (d, tb)


def test_split_pr_bin_2048_entry(H):
    """the bin-2048 entry alone: Q conj(Zc) to float32 precision, though P = 0 and r is infinite"""
    d, tb = 1, 2048
    N = HALF >> d
    Z = _spectrum(7)
    ex = F.split_filter(Z, d, tb, H[d], exact=True)
    pr = F.split_filter(Z, d, tb, H[d], form="pr")
    m = 0                                  # inverse input 0 holds bin tb = 2048
    assert np.all(np.abs(ex[:, m]) > 0)
    rel = np.abs(pr[:, m] - ex[:, m]) / np.abs(ex[:, m])
    assert rel.max() <= 2.0 ** -21
    # the other bins of the band are unaffected by the special case
    assert np.abs(pr[:, 1:N] - ex[:, 1:N]).max() <= 2.0 ** -21 * np.abs(ex).max()
