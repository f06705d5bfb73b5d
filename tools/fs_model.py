#!/usr/bin/env python3
"""numpy model of the d = 0 fused-split frame (ddc_persistent.hip, FS path): the forward
4096-point FFT as three radix-16 Stockham passes with the last pass's columns c = PERM[lane],
the r2c split x filter fed by the DPP partner lane (lane ^ 1 holds column 256 - c), the
inverse FFT on absolute bin indices, and the tune shift as the output modulation
e^{-2 pi i tb n / 4096}: a per-lane factor g_t on the last pass's twiddles and a quarter turn
per output register (tb mod 16 in {0, 4, 8, 12}).  Checked against the f64
oracle (tests/test_fs_model.py); the kernel follows it step for step.
"""
from __future__ import annotations

import numpy as np

HALF, HOP, BLOCK, FRAMES = 4096, 6144, 65536, 11


def w(n, k, sign=-1):
    return np.exp(sign * 2j * np.pi * np.asarray(k, dtype=np.float64) / n)


def dft16(a, sign):
    """a: [..., 16] -> DFT over the last axis, e^{sign 2 pi i r k / 16}"""
    r = np.arange(16)
    M = np.exp(sign * 2j * np.pi * np.outer(r, r) / 16)
    return a @ M


def frame_fs(x8192, tb, H, perm, split="pr"):
    """one d = 0 frame: 8192 real samples -> 4096 complex outputs (before overlap-discard).
    split "pq": F = Z P + conj(Zc) Q (round 5); "pr" (round 6): Q = i r P with r real, so
    F = P (Z + i r conj(Zc)), except the bin 2048 (column 0, register 8: P = 0), F = Q conj(Z)"""
    z = x8192[0::2] + 1j * x8192[1::2]
    t = np.arange(256)
    # F0: butterfly t, inputs z[t + 256 r], out pos 16 t + k
    A = np.empty(HALF, complex)
    A.reshape(256, 16)[:] = dft16(z.reshape(16, 256).T, -1)
    # F1 (NS = 16): butterfly j, inputs A[j + 256 r] * W256^{(j % 16) r}, out (j/16) 256 + j%16 + 16 k
    r = np.arange(16)
    a = A.reshape(16, 256).T * w(256, np.outer(t % 16, r))
    o = dft16(a, -1)
    B = np.empty(HALF, complex)
    for j in range(256):
        B[(j // 16) * 256 + j % 16 + 16 * r] = o[j]
    # F2 (NS = 256): butterfly of lane l = column c = perm[l]
    c = perm
    a = B.reshape(16, 256).T[c] * w(HALF, np.outer(c, r))
    Zl = dft16(a, -1)                       # Zl[l, k] = Z[c_l + 256 k]
    Z = np.fft.fft(z)
    assert np.allclose(Zl, Z[(c[:, None] + 256 * r[None, :])], atol=1e-6 * np.abs(Z).max())
    # split x filter, bin beta = c + 256 k, mirror from the partner lane l ^ 1, register 15 - k
    beta = (c[:, None] + 256 * r[None, :]) % HALF
    Wb = w(2 * HALF, beta)
    m = (beta - tb) % HALF
    valid = ((beta >= tb) & (beta - tb < HALF // 2)) | ((beta < tb) & (tb - beta <= HALF // 2))
    Hh = H[m] / 2
    P, Q = Hh * (1 - 1j * Wb), Hh * (1 + 1j * Wb)
    P[~valid] = 0
    Q[~valid] = 0
    zc = Zl[np.arange(256) ^ 1][:, ::-1].copy()      # partner lane's register 15 - k
    # self-mirrored columns 0 and 128 (lanes 0 and 1): their own registers
    zc[0] = Zl[0][(16 - r) % 16]
    zc[1] = Zl[1][15 - r]
    assert np.allclose(zc, Z[(-beta) % HALF])
    if split == "pq":
        F = Zl * P + np.conj(zc) * Q
    else:
        # r = Q / (i P) = (1 + i W) / (i (1 - i W)) = cot(pi/4 - pi beta / 8192): real, tune-bin and
        # filter independent; infinite only at beta = 2048 (lane 0, register 8)
        sp = (beta == 2048)
        with np.errstate(divide="ignore", invalid="ignore"):
            rr = np.where(sp, 0.0, ((1 + 1j * Wb) / (1j * (1 - 1j * Wb))).real)
        assert np.allclose(np.where(sp | ~valid, 0, Q - 1j * rr * P), 0, atol=1e-12 * np.abs(Q).max())
        F = P * (Zl + 1j * rr * np.conj(zc))
        F[sp] = Q[sp] * np.conj(Zl[sp])
    # I0 (NS = 1): butterfly c, inputs F[c + 256 s], out pos 16 c + k
    C = np.empty(HALF, complex)
    o = dft16(F, +1)
    for l in range(256):
        C[16 * c[l] + r] = o[l]
    # I1 (NS = 16): out pos (j/16) 256 + j%16 + 16 k
    a = C.reshape(16, 256).T * w(256, np.outer(t % 16, r), +1)
    o = dft16(a, +1)
    D = np.empty(HALF, complex)
    for j in range(256):
        D[(j // 16) * 256 + j % 16 + 16 * r] = o[j]
    # I2 (NS = 256): butterfly t, inputs D[t + 256 r] * g_t W4096^{+t r}, g_t = e^{-2 pi i tb t / 4096};
    # output k then takes W16^{(tb mod 16) k} (a quarter turn per k: tb is a multiple of 4)
    g = w(HALF, tb * t)
    a = D.reshape(16, 256).T * w(HALF, np.outer(t, r), +1) * g[:, None]
    yk = dft16(a, +1) * w(16, (tb % 16) * r)[None, :]
    y = np.empty(HALF, complex)
    y.reshape(16, 256).T[:] = yk
    return y


def r2iq_fs(stream, nblk, tb, H, perm, split="pr"):
    out = np.empty(nblk * 32768, complex)
    for b in range(nblk):
        for k in range(FRAMES):
            s = b * BLOCK + k * HOP
            y = frame_fs(stream[s:s + 2 * HALF].astype(np.float64), tb, H, perm, split)
            if k == 0:
                out[b * 32768: b * 32768 + 2048] = y[1024:3072]
            else:
                o = b * 32768 + 2048 + 3072 * (k - 1)
                out[o:o + 3072] = y[:3072]
    return out
