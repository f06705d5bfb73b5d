"""ORACLE — test infrastructure only.  Independent numpy float64 restatement.

A second, independent restatement of the r2iq hot path written directly from the
reference's equations with numpy's FFT (pocketfft, float64), used only to
cross-check the C oracle (ddc_oracle.c) on small inputs:

  a2 convert_float<rand>      Core/fft_mt_r2iq.h:36-51
  a3 r2c 8192 (fftwf r2c)      Core/fft_mt_r2iq_impl.hpp:88, plan fft_mt_r2iq.cpp:221
  a4 shift_freq + zero fill    Core/fft_mt_r2iq_impl.hpp:76-96, fft_mt_r2iq.h:53-61
  a6 backward c2c mfft         Core/fft_mt_r2iq_impl.hpp:98, plans fft_mt_r2iq.cpp:222-225
  a7 overlap-discard + conj    Core/fft_mt_r2iq_impl.hpp:117-138, fft_mt_r2iq.h:63-81
  a5 filter bank H_d           Core/fft_mt_r2iq.cpp:173-206 (taps from the C oracle's
                               Kaiser, which is pinned bit-exact to Core/fir.cpp)
"""
from __future__ import annotations

import numpy as np

HALF_FFT = 4096
BLOCK = 65536
HOP = 6144
FRAMES = 11


def derand(x: np.ndarray, rand: bool) -> np.ndarray:
    x = x.astype(np.int16)
    if not rand:
        return x
    odd = (x & 1).astype(bool)
    y = x.copy()
    y[odd] = x[odd] ^ np.int16(-2)
    return y


def filter_bank(taps_per_d, gain: float) -> np.ndarray:
    H = np.zeros((len(taps_per_d), HALF_FFT), np.complex128)
    gainadj = np.float32(np.float32(gain) * np.float32(2048.0)) / np.float32(8192.0)
    for d, pht in enumerate(taps_per_d):
        ht = np.zeros(HALF_FFT, np.float64)
        ht[HALF_FFT - 1 - np.arange(len(pht))] = (np.float32(gainadj) * pht.astype(np.float32)).astype(np.float64)
        H[d] = np.fft.fft(ht)
    return H


def r2iq(stream: np.ndarray, nblk: int, d: int, tunebin: int, lsb: bool, rand: bool, Hd: np.ndarray) -> np.ndarray:
    mfft = HALF_FFT >> d
    half = mfft // 2
    x = derand(np.asarray(stream[: HALF_FFT + nblk * BLOCK]), rand).astype(np.float64)
    out = np.zeros(nblk * 8 * mfft, np.complex128)
    count = min(half, HALF_FFT - tunebin)
    start = max(0, half - tunebin)
    H2 = Hd[HALF_FFT - half:]
    for b in range(nblk):
        base = b * BLOCK
        for k in range(FRAMES):
            X = np.fft.rfft(x[base + HOP * k: base + HOP * k + 2 * HALF_FFT])
            t = np.zeros(mfft, np.complex128)
            m = np.arange(count)
            t[m] = X[tunebin + m] * Hd[m]
            m = np.arange(start, half)
            t[half + m] = X[tunebin - half + m] * H2[m]
            y = np.fft.ifft(t) * mfft            # unnormalised backward transform
            if lsb:
                y = np.conj(y)
            o = b * 8 * mfft
            if k == 0:
                out[o: o + half] = y[mfft // 4: 3 * mfft // 4]
            else:
                p = o + half + (3 * mfft // 4) * (k - 1)
                out[p: p + 3 * mfft // 4] = y[: 3 * mfft // 4]
    return out
