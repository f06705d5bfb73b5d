"""Design model (not product, not test infrastructure): a numpy emulation of one wave64
running the d = 0 frame transform of ddc_wave.hip with 64 points per lane.

State is an array [64 lanes, n registers] of complex128.  Every step below is written
as the lane/register operation the HIP kernel performs (loads, in-register DFTs,
per-lane twiddle tables, LDS writes/reads at the padded (row stride 33) slot addresses,
v_permlane32_swap, v_cndmask), so the index bookkeeping can be checked on the CPU
against the direct formula:

    z[n]  = s[2n] + i s[2n+1]                     (frame of 8192 int16)
    Z     = FFT_4096(z)                           (forward, unnormalised)
    T[m]  = Z[k] P[m] + conj(Z[-k]) Q[m],  k = (tb + m) mod 4096
    y[n]  = sum_m T[m] e^{+2 pi i m n / 4096}

It also checks that every LDS access is bank-conflict free under the gfx950 rules of
MI355X_MICROARCH.md §LDS (ds_write_b64: 16-lane groups, bank (a/4) mod 32; ds_read_b64:
32-lane groups, bank (a/4) mod 64).

    python tools/wave_fft_model.py
"""
from __future__ import annotations

import numpy as np

L64 = np.arange(64)


def W(N, e):
    return np.exp(-2j * np.pi * np.asarray(e) / N)


def permlane32_swap(a, b):
    """v_permlane32_swap_b32 vdst=a, src=b: lanes 32-63 of a <-> lanes 0-31 of b."""
    a2, b2 = a.copy(), b.copy()
    a2[32:] = b[:32]
    b2[:32] = a[32:]
    return a2, b2


def rot32(x):
    """x rotated by 32 lanes, as two swaps on a register pair (here: on one register)."""
    return np.concatenate([x[32:], x[:32]])


class LDS:
    def __init__(self):
        self.mem = np.full(33 * 64, np.nan + 0j)

    def write(self, slots):                      # one ds_write_b64: slots[lane]
        for g in range(4):                       # 4 x 16 contiguous lanes, bank (a/4) mod 32
            s = slots[16 * g:16 * g + 16]
            banks = (2 * s) % 32
            assert len(set(banks.tolist())) == 16, "ds_write_b64 bank conflict"
        return slots

    def read(self, slots):                       # one ds_read_b64
        for g in range(2):                       # 2 x 32 lanes, bank (a/4) mod 64
            s = slots[32 * g:32 * g + 32]
            assert len(set(((2 * s) % 64).tolist())) == 32, "ds_read_b64 bank conflict"
        return self.mem[slots]


def colF(l):
    """column held by lane l after the forward swap (pairs {c, 64-c}, {0, 32})"""
    lam = l % 32
    if l < 32:
        return lam
    return 32 if lam == 0 else 64 - lam


def cS(l):
    return colF(l)


def cD(l):
    lam = l % 32
    if l < 32:
        return 0 if lam == 0 else 64 - lam
    return 32 if lam == 0 else lam


def model_frame(s, tb, P, Q):
    z = s[0::2].astype(np.float64) + 1j * s[1::2].astype(np.float64)
    lds = LDS()
    lane = L64
    h = (lane >= 32).astype(int)
    lam = lane % 32
    special = (lane % 32) == 0          # lanes 0 and 32 keep their own column

    # ---- load: lane L, register r holds z[L + 64 r]
    R = np.stack([z[lane + 64 * r] for r in range(64)], axis=1)
    # ---- F1: DFT-64 over r, natural order q
    A = np.fft.fft(R, axis=1)
    # ---- twiddle W_4096^{L q} (table twF[q][L])
    B = A * W(4096, np.outer(lane, np.arange(64)))
    # ---- forward exchange, phase 0: registers q < 32
    for q in range(32):
        sl = lds.write(33 * lane + q)
        lds.mem[sl] = B[:, q]
    U = np.zeros((64, 32), complex)
    for i in range(32):
        row = 32 * h + i
        U[:, i] = lds.read(33 * row + lam)
    # phase 1: registers q >= 32; lane l reads column colB(lam) = (lam ? 64-lam : 32)
    for q in range(32, 64):
        sl = lds.write(33 * lane + (q - 32))
        lds.mem[sl] = B[:, q]
    V = np.zeros((64, 32), complex)
    qb = (-lam) & 31                              # colB - 32
    for i in range(32):
        row = 32 * h + i
        V[:, i] = lds.read(33 * row + qb)
    for i in range(32):
        U[:, i], V[:, i] = permlane32_swap(U[:, i], V[:, i])
    # now lane l holds column colF(l): U = rows L < 32, V = rows L >= 32
    for l in range(64):
        c = colF(l)
        assert np.allclose(U[l], B[:32, c]) and np.allclose(V[l], B[32:, c])
    # ---- F2: DIF on the top bit of L, then two DFT-32s
    Sv = U + V
    Dv = (U - V) * W(64, np.arange(32))[None, :]
    Sv = np.fft.fft(Sv, axis=1)              # Z[c + 64 * 2j]
    Dv = np.fft.fft(Dv, axis=1)              # Z[c + 64 * (2j+1)]
    Dr = np.stack([rot32(Dv[:, j]) for j in range(32)], axis=1)
    Dv = np.where(special[:, None], Dv, Dr)
    Zref = np.fft.fft(z)
    for l in range(64):
        assert np.allclose(Sv[l], Zref[cS(l) + 128 * np.arange(32)])
        assert np.allclose(Dv[l], Zref[cD(l) + 64 + 128 * np.arange(32)])
    # ---- split x filter: T = Z P + conj(mirror) Q  (P, Q from the lane-layout table)
    kS = np.array([[cS(l) + 128 * j for j in range(32)] for l in range(64)])
    kD = np.array([[cD(l) + 64 + 128 * j for j in range(32)] for l in range(64)])
    mS, mD = (kS - tb) % 4096, (kD - tb) % 4096
    j = np.arange(32)
    lane0 = (lane == 0)[:, None]
    mirS = np.where(lane0, Sv[:, (32 - j) % 32], Dv[:, 31 - j])
    mirD = np.where(lane0, Dv[:, 31 - j], Sv[:, 31 - j])
    for l in range(64):
        assert np.allclose(mirS[l], Zref[(-kS[l]) % 4096]) and np.allclose(mirD[l], Zref[(-kD[l]) % 4096])
    TS = Sv * P[mS] + np.conj(mirS) * Q[mS]
    TD = Dv * P[mD] + np.conj(mirD) * Q[mD]
    # ---- I1: DIT on the parity of p: backward DFT-32s, odd half x W_64^{-n}
    E = np.fft.ifft(TS, axis=1) * 32
    O = np.fft.ifft(TD, axis=1) * 32 * W(64, -np.arange(32))[None, :]
    Or = np.stack([rot32(O[:, n]) for n in range(32)], axis=1)
    O = np.where(special[:, None], O, Or)
    G = np.concatenate([E + O, E - O], axis=1)          # G[n_lo], n_lo = 0..63
    c = np.array([cS(l) for l in range(64)])
    G = G * W(4096, -np.outer(c - tb, np.arange(64)))    # table twI[n][l]
    mlo = (c - tb) % 64
    # check: G[l][n] = sum over m_hi of T[mlo + 64 m_hi] e^{+2 pi i m_hi n / 64} x W_4096^{-mlo n}
    T = np.zeros(4096, complex)
    T[mS.ravel()] = TS.ravel()
    T[mD.ravel()] = TD.ravel()
    for l in range(64):
        col = T[mlo[l] + 64 * np.arange(64)]
        ref = np.fft.ifft(col) * 64 * W(4096, -mlo[l] * np.arange(64))
        assert np.allclose(G[l], ref)
    # ---- inverse exchange, phase 0 (n < 32) and phase 1 (n >= 32)
    A2 = np.zeros((64, 32), complex)
    B2 = np.zeros((64, 32), complex)
    for ph, dst in ((0, A2), (1, B2)):
        for n in range(32):
            sl = lds.write(33 * mlo + n)
            lds.mem[sl] = G[:, 32 * ph + n]
        for i in range(32):
            m = 32 * h + i
            dst[:, i] = lds.read(33 * m + lam)
    for i in range(32):
        A2[:, i], B2[:, i] = permlane32_swap(A2[:, i], B2[:, i])
    # lane l now holds column n_lo = l: A2 = m_lo < 32, B2 = m_lo >= 32
    # ---- I2: DIF on the top bit of m_lo, backward DFT-32s: even / odd n_hi
    S2 = A2 + B2
    D2 = (A2 - B2) * W(64, -np.arange(32))[None, :]
    Ye = np.fft.ifft(S2, axis=1) * 32           # y[l + 64 * 2j]
    Yo = np.fft.ifft(D2, axis=1) * 32           # y[l + 64 * (2j+1)]
    y = np.zeros(4096, complex)
    for jj in range(32):
        y[lane + 64 * 2 * jj] = Ye[:, jj]
        y[lane + 64 * (2 * jj + 1)] = Yo[:, jj]
    return y, T


def reference(s, tb, P, Q):
    z = s[0::2].astype(np.float64) + 1j * s[1::2].astype(np.float64)
    Z = np.fft.fft(z)
    m = np.arange(4096)
    k = (tb + m) % 4096
    T = Z[k] * P + np.conj(Z[(-k) % 4096]) * Q
    return np.fft.ifft(T) * 4096, T


def main():
    rng = np.random.default_rng(1)
    for tb in (0, 4, 284, 1024, 2048, 3684, 4092):
        s = rng.integers(-32768, 32768, 8192).astype(np.int16)
        P = rng.normal(size=4096) + 1j * rng.normal(size=4096)
        Q = rng.normal(size=4096) + 1j * rng.normal(size=4096)
        y, T = model_frame(s, tb, P, Q)
        yr, Tr = reference(s, tb, P, Q)
        assert np.allclose(T, Tr)
        err = np.max(np.abs(y - yr)) / np.max(np.abs(yr))
        print(f"tb={tb:5d}: max rel err {err:.2e}")
        assert err < 1e-12
    print("wave model OK (index maps + conflict-free LDS)")


if __name__ == "__main__":
    main()
