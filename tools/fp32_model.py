#!/usr/bin/env python3
"""float32 operation-level model of the single-channel kernels' arithmetic (tools only).

Emulates, lane by lane and in the kernels' operation order, the float32 roundings of the
persistent kernel's frame (ddc_persistent.hip): forward pass 0 (int pairs -> float, DFT-16 in
tangent form), pass 1 (table twiddles), pass 2 (recurrence twiddles, twiddle_rec16), the (P, Q)
split x filter, and the inverse: the d >= 3 Stockham tails (tail_pass) or radix-16 passes.
FMAs are emulated as a float64 product-sum rounded once to float32 (exact for the product; the
sum's double rounding is negligible for an error study).  Used to attribute the float32 error
of a case to a stage (exact-vs-emulated per stage) without a GPU.

  python3 tools/fp32_model.py            # the sweep's leakage-only draws + the oob floor cases
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

f32, f64 = np.float32, np.float64
HALF, HOP, BLOCK, FRAMES = 4096, 6144, 65536, 11


def fma(a, b, c):
    return (np.asarray(a, f64) * np.asarray(b, f64) + np.asarray(c, f64)).astype(f32)


def add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def mulj(a, d):   # a * (d i)
    return (a[1], -a[0]) if d < 0 else (-a[1], a[0])


def cmul(a, w):   # the compiler's contraction of (a.x w.x - a.y w.y, a.x w.y + a.y w.x)
    return (fma(a[0], w[0], -(a[1] * w[1])), fma(a[0], w[1], a[1] * w[0]))


def cmulc(a, w):
    return (fma(a[0], w[0], a[1] * w[1]), fma(a[1], w[0], -(a[0] * w[1])))


def TW(a, w, d):
    return cmul(a, w) if d < 0 else cmulc(a, w)


def const(x):
    return f32(x)


kC1, kS1, kR2 = const(np.cos(np.pi / 8)), const(np.sin(np.pi / 8)), const(np.sqrt(0.5))
kT1, kT3 = const(np.tan(np.pi / 8)), const(np.tan(3 * np.pi / 8))


def dft4(a0, a1, a2, a3, d):
    t0, t1 = add(a0, a2), sub(a0, a2)
    t2, t3 = add(a1, a3), mulj(sub(a1, a3), d)
    return add(t0, t2), add(t1, t3), sub(t0, t2), sub(t1, t3)


def rot1(z, tau):
    tau = f32(tau)
    return (fma(-tau, z[1], z[0]), fma(tau, z[0], z[1]))


def axpm(a, c, z):
    c = f32(c)
    return (fma(c, z[0], a[0]), fma(c, z[1], a[1])), (fma(-c, z[0], a[0]), fma(-c, z[1], a[1]))


def ajpm(a, c, z, d):
    dc = f32(d * c)
    return (fma(-dc, z[1], a[0]), fma(dc, z[0], a[1])), (fma(dc, z[1], a[0]), fma(-dc, z[0], a[1]))


def dft16(v, d, plain=False):
    """fft_device.hpp dft16 (tangent form); plain=True: the 4 x 4 form with constant twiddles"""
    b = [dft4(v[n2], v[4 + n2], v[8 + n2], v[12 + n2], d) for n2 in range(4)]
    o = [None] * 16
    o[0], o[4], o[8], o[12] = dft4(b[0][0], b[1][0], b[2][0], b[3][0], d)
    if plain:
        w = lambda m: (f32(np.cos(2 * np.pi * m / 16)), f32(d * np.sin(2 * np.pi * m / 16)))
        for k1 in (1, 2, 3):
            c = [b[0][k1]] + [cmul(b[n2][k1], w(n2 * k1)) for n2 in (1, 2, 3)]
            o[k1], o[k1 + 4], o[k1 + 8], o[k1 + 12] = dft4(*c, d)
        return o
    t0, t1 = axpm(b[0][1], kR2, rot1(b[2][1], d))
    p, q = axpm(rot1(b[1][1], d * kT1), kT1, rot1(b[3][1], d * kT3))
    o[1], o[9] = axpm(t0, kC1, p)
    o[5], o[13] = ajpm(t1, kC1, q, d)
    t0, t1 = ajpm(b[0][2], 1.0, b[2][2], d)
    p, q = axpm(rot1(b[1][2], d), -1.0, rot1(b[3][2], -d))
    o[2], o[10] = axpm(t0, kR2, p)
    o[6], o[14] = ajpm(t1, kR2, q, d)
    t0, t1 = axpm(b[0][3], -kR2, rot1(b[2][3], -d))
    p, q = axpm(rot1(b[1][3], d * kT3), -kT3, rot1(b[3][3], d * kT1))
    o[3], o[11] = axpm(t0, kS1, p)
    o[7], o[15] = ajpm(t1, kS1, q, d)
    return o


def dft8(v, d):
    b0 = dft4(v[0], v[2], v[4], v[6], d)
    b1 = list(dft4(v[1], v[3], v[5], v[7], d))

    def tw(a, c, s):   # tw16: (c a.x - sd a.y, c a.y + sd a.x), contracted
        c, sd = f32(c), f32(d * s)
        return (fma(c, a[0], -(sd * a[1])), fma(c, a[1], sd * a[0]))
    b1[1] = tw(b1[1], kR2, kR2)
    b1[2] = mulj(b1[2], d)
    b1[3] = tw(b1[3], -kR2, kR2)
    o = [None] * 8
    for k1 in range(4):
        o[k1] = add(b0[k1], b1[k1])
        o[k1 + 4] = sub(b0[k1], b1[k1])
    return o


def table(n, k, d=-1):
    a = np.exp(d * 2j * np.pi * np.asarray(k, f64) / n)
    return (a.real.astype(f32), a.imag.astype(f32))


def rec16(a, w1, w4, d, exact=None):
    """twiddle_rec16: a[r] *= W^r from W^1, W^4 (exact: the powers from the table instead)"""
    if exact is not None:
        return [a[0]] + [TW(a[r], exact[r], -1) for r in range(1, 16)]
    if d > 0:
        w1, w4 = (w1[0], -w1[1]), (w4[0], -w4[1])

    def cm_pm(A, w):
        cx, cy = w[0] * A[0], w[0] * A[1]
        return (fma(-w[1], A[1], cx), fma(w[1], A[0], cy)), (fma(w[1], A[1], cx), fma(-w[1], A[0], cy))

    def cheb(c2, x, y):
        return (fma(c2, x[0], -y[0]), fma(c2, x[1], -y[1]))
    c1 = w1[0] + w1[0]
    w8 = cmul(w4, w4)
    w12 = cmul(w8, w4)
    w5, w3 = cm_pm(w4, w1)
    w9, w7 = cm_pm(w8, w1)
    w13, w11 = cm_pm(w12, w1)
    one = (np.ones_like(w1[0]), np.zeros_like(w1[0]))
    w2 = cheb(c1, w1, one)
    w6 = cheb(c1, w5, w4)
    w10 = cheb(c1, w9, w8)
    w14 = cheb(c1, w13, w12)
    w15 = cheb(c1, w14, w13)
    W = [None, w1, w2, w3, w4, w5, w6, w7, w8, w9, w10, w11, w12, w13, w14, w15]
    return [a[0]] + [cmul(a[r], W[r]) for r in range(1, 16)]


def anchor6(a, base):
    """a[r] *= W^r from six exactly rounded anchors W^1, W^2, W^3, W^4, W^8, W^12 of the lane's
    base: W^{4a + b} = W^{4a} W^b, one product per power"""
    A = {k: table(HALF, (base * k) % HALF) for k in (1, 2, 3, 4, 8, 12)}
    W = [None] * 16
    for k in A:
        W[k] = A[k]
    for hi in (4, 8, 12):
        for lo in (1, 2, 3):
            W[hi + lo] = cmul(A[hi], A[lo])
    return [a[0]] + [cmul(a[r], W[r]) for r in range(1, 16)]


def forward(frames, rand=False, twmode="rec", plain=False, r0=0):
    """frames: [F, 8192] int16 -> Z[F, 4096] complex128 (float32 values) of the packed FFT.
    twmode: 'rec' (kernel: pass-2 powers by twiddle_rec16), 'table' (exact rounded powers) or
    'anchor6'.  r0: pass 2's bases rotated by 256 r0 (the pruned kernel at d >= 2): register r
    then holds bin t + 256 (r + r0)."""
    F = frames.shape[0]
    x = frames.astype(np.int32)
    if rand:
        x = np.where(x & 1, -x, x)
    re = x[:, 0::2].astype(f32)
    im = x[:, 1::2].astype(f32)   # z[n] = x[2n] + i x[2n + 1]
    t = np.arange(256)
    # pass 0: thread t, inputs z[t + 256 r]
    a = [(re[:, t + 256 * r], im[:, t + 256 * r]) for r in range(16)]
    o = dft16(a, -1, plain)
    A = [np.empty((F, HALF), f32), np.empty((F, HALF), f32)]
    for k in range(16):
        A[0][:, 16 * t + k], A[1][:, 16 * t + k] = o[k]
    # pass 1 (NS = 16): thread j: A[j + 256 r] * W256^{(j % 16) r}
    a = [(A[0][:, t + 256 * r], A[1][:, t + 256 * r]) for r in range(16)]
    a = [a[0]] + [TW(a[r], table(256, (t % 16) * r), -1) for r in range(1, 16)]
    o = dft16(a, -1, plain)
    B = [np.empty((F, HALF), f32), np.empty((F, HALF), f32)]
    for k in range(16):
        pos = (t // 16) * 256 + t % 16 + 16 * k
        B[0][:, pos], B[1][:, pos] = o[k]
    # pass 2 (NS = 256): thread t: B[t + 256 r] * W4096^{t r}
    a = [(B[0][:, t + 256 * r], B[1][:, t + 256 * r]) for r in range(16)]
    base = t + 256 * r0
    if twmode == "rec":
        a = rec16(a, table(HALF, base % HALF), table(HALF, (4 * base) % HALF), -1)
    elif twmode == "anchor6":
        a = anchor6(a, base)
    else:
        a = rec16(a, None, None, -1, exact=[None] + [table(HALF, (base * r) % HALF) for r in range(1, 16)])
    o = dft16(a, -1, plain)
    Z = np.empty((F, HALF), np.complex128)
    for k in range(16):
        Z[:, t + 256 * ((k + r0) % 16)] = o[k][0].astype(f64) + 1j * o[k][1].astype(f64)
    return Z


def split_filter(Z, d, tb, Hd, exact=False, form="pr"):
    """T[m] (inverse input m < N) = Zk P + conj(Zc) Q, the table in double rounded once.
    form "pr" (round 6, split_pr): P and r = Q / (i P) as float, T = P (Zk + i r conj Zc); bin 2048
    (P = 0) holds r = 2^64, P = Q / (i 2^64).  "pq" (round 5, split_pq): the (P, Q) float4."""
    N = HALF >> d
    m = np.arange(N)
    binv = tb + m - np.where(m >= N // 2, N, 0)
    ok = (binv >= 0) & (binv < HALF)
    bb = np.where(ok, binv, 0)
    Wb = np.exp(-2j * np.pi * bb / (2 * HALF))
    Hh = Hd[np.where(m < N // 2, m, HALF - N + m)] / 2   # the reference's H index (impl.hpp:90-94)
    P = np.where(ok, Hh * (1 - 1j * Wb), 0)
    Q = np.where(ok, Hh * (1 + 1j * Wb), 0)
    zk = Z[:, bb]
    zc = Z[:, (HALF - bb) % HALF]
    if exact:
        return zk * P + np.conj(zc) * Q
    zkx, zky = zk.real.astype(f32), zk.imag.astype(f32)
    zcx, zcy = zc.real.astype(f32), zc.imag.astype(f32)
    if form == "pr":
        sp = ok & (bb == HALF // 2)
        with np.errstate(divide="ignore", invalid="ignore"):
            rr = np.where(ok & ~sp, ((1 + 1j * Wb) / (1j * (1 - 1j * Wb))).real, 0.0)
        rr = np.where(sp, 2.0 ** 64, rr).astype(f32)
        Pm = np.where(sp, Q / (1j * 2.0 ** 64), P)
        px, py = Pm.real.astype(f32), Pm.imag.astype(f32)
        vx, vy = fma(rr, zcy, zkx), fma(rr, zcx, zky)
        return fma(vx, px, -(vy * py)).astype(f64) + 1j * fma(vx, py, vy * px).astype(f64)
    c = [P.real.astype(f32), P.imag.astype(f32), Q.real.astype(f32), Q.imag.astype(f32)]
    # split_pq with contraction: x = ((zk.x c.x - zk.y c.y) + zc.x c.z) + zc.y c.w
    vx = fma(zcy, c[3], fma(zcx, c[2], fma(zkx, c[0], -(zky * c[1]))))
    vy = fma(-zcy, c[2], fma(zcx, c[3], fma(zkx, c[1], zky * c[0])))
    return vx.astype(f64) + 1j * vy.astype(f64)


def inverse_tail(T, N):
    """the d >= 3 Stockham tail (tail_pass): radix schedule 8-8-8, 4-4-4-4, 8-4-4, 4-4-4"""
    sched = {512: [8, 8, 8], 256: [4, 4, 4, 4], 128: [8, 4, 4], 64: [4, 4, 4]}[N]
    F = T.shape[0]
    cur = [T.real.astype(f32), T.imag.astype(f32)]
    ns = 1
    for p, R in enumerate(sched):
        TT = N // R
        j = np.arange(TT)
        a = [(cur[0][:, j + TT * r], cur[1][:, j + TT * r]) for r in range(R)]
        if p > 0:
            kk = j % ns
            a = [a[0]] + [TW(a[r], table(HALF, (kk * r * (HALF // (R * ns))) % HALF), +1) for r in range(1, R)]
        o = dft8(a, +1) if R == 8 else list(dft4(*a, +1))
        nxt = [np.empty((F, N), f32), np.empty((F, N), f32)]
        for r in range(R):
            pos = (j // ns) * R * ns + j % ns + ns * r
            nxt[0][:, pos], nxt[1][:, pos] = o[r]
        cur = nxt
        ns *= R
    return cur[0].astype(f64) + 1j * cur[1].astype(f64)


def r2iq_model(stream, nblk, d, tb, lsb, rand, Hd, twmode="rec", plain=False, exact_fwd=False, exact_inv=False,
               exact_split=False, split_form="pr"):
    """frames -> forward -> split -> inverse -> overlap-discard, as the kernels (d >= 3 tails)"""
    N = HALF >> d
    idx = np.array([BLOCK * b + HOP * k for b in range(nblk) for k in range(FRAMES)])
    frames = np.stack([stream[i:i + 2 * HALF] for i in idx])
    if exact_fwd:
        x = frames.astype(np.int64)
        if rand:
            x = np.where(x & 1, -x, x)
        z = x[:, 0::2] + 1j * x[:, 1::2]
        Z = np.fft.fft(z, axis=1)
    else:
        r0 = (((tb - N // 2) % HALF) >> 8) if N <= 1024 else 0   # the pruned kernel's rotation
        Z = forward(frames, rand, twmode, plain, r0)
    T = split_filter(Z, d, tb, Hd, exact_split, split_form)
    if exact_inv:
        y = np.fft.ifft(T, axis=1) * N
    else:
        y = inverse_tail(T, N)
    out = []
    for i in range(len(idx)):
        k = i % FRAMES
        seg = y[i, N // 4: 3 * N // 4] if k == 0 else y[i, :3 * N // 4]
        out.append(np.conj(seg) if lsb else seg)
    return np.concatenate(out)


def main():
    from oracle import oracle as O
    from extio_sddc_amd.synth import make_stream
    H = O.filter_bank(1.0)
    cases = [(3, 2708, 0, 0, "bench", 4, 310165425), (5, 2408, 1, 0, "bench", 3, 546231597),
             (5, 2044, 0, 0, "bench", 3, 826057796), (3, 1024, 0, 0, "oob", 4, 0x5DDC),
             (4, 1024, 0, 0, "oob", 4, 0x5DDC), (4, 0, 1, 0, "oob", 4, 0x5DDC)]
    for d, tb, lsb, rand, src, nblk, seed in cases:
        x = make_stream(nblk, src, seed=seed)
        ex = O.r2iq(x, nblk, d, tb, lsb, rand, H=H)
        port = O.r2iq(x, nblk, d, tb, lsb, rand, dtype=np.float32, H=O.filter_bank(1.0, np.float32))
        row = {"port": O.max_rel_err(port, ex)}
        for name, kw in [("kernel", {}), ("fwd_table_tw", {"twmode": "table"}), ("anchor6", {"twmode": "anchor6"}),
                         ("fwd_plain16", {"plain": True}),
                         ("fwd_exact", {"exact_fwd": True}), ("inv_exact", {"exact_inv": True}),
                         ("split_exact", {"exact_split": True}), ("split_pq", {"split_form": "pq"}),
                         ("fwd_table_inv_exact", {"twmode": "table", "exact_inv": True})]:
            y = r2iq_model(x, nblk, d, tb, lsb, rand, H[d], **kw)
            row[name] = O.max_rel_err(y, ex)
        print(f"d={d} tb={tb} lsb={lsb} {src}: " + " ".join(f"{k}={v:.2e}" for k, v in row.items()))


if __name__ == "__main__":
    main()
