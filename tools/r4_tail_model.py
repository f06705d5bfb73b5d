#!/usr/bin/env python3
"""numpy model of the d >= 4 inverse tails of r2iq_persistent_kernel (ddc_persistent.hip,
stockham_tail): the N-point inverse DFT (N = 512, 256, 128, 64 at d = 3..6) as mixed-radix
Stockham passes on the lanes of wave 0 (radix schedule 8-8-8, 4-4-4-4, 8-4-4 and 4-4-4).  In the pass
of radix R after a span Ns, thread j < N / R reads elements j + (N / R) r, multiplies them by
e^{+2 pi i k r / (R Ns)} (k = j mod Ns), runs the inverse DFT-R and writes (j / Ns) R Ns + k + Ns r;
the last pass leaves y[j + (N / R) r] in registers.  Checked against numpy's inverse FFT, plus a
search over XOR swizzles e ^ (((e >> a) & m) << b) of the LDS layout, scoring the bank
conflicts of every read and write pattern per 32-lane half of a ds_*_b64 (element slot mod 32).
"""
import numpy as np

SCHED = {512: (8, 8, 8), 256: (4, 4, 4, 4), 128: (8, 4, 4), 64: (4, 4, 4)}


def passes(N):
    ns = 1
    for R in SCHED[N]:
        yield R, ns
        ns *= R


def stockham_inv(x, N, A=lambda e: e):
    buf = np.zeros(1024, complex)
    for e in range(N):
        buf[A(e)] = x[e]
    sched = list(passes(N))
    for p, (R, ns) in enumerate(sched):
        T = N // R
        u = np.zeros((T, R), complex)
        for j in range(T):
            a = np.array([buf[A(j + T * r)] for r in range(R)])
            k = j % ns
            a = a * np.exp(2j * np.pi * k * np.arange(R) / (R * ns))
            u[j] = np.fft.ifft(a) * R
        if p < len(sched) - 1:
            for j in range(T):
                k = j % ns
                for r in range(R):
                    buf[A((j // ns) * R * ns + k + ns * r)] = u[j, r]
    y = np.zeros(N, complex)
    T = N // sched[-1][0]
    for j in range(T):
        for r in range(sched[-1][0]):
            y[j + T * r] = u[j, r]
    return y


def conflicts(A, N):
    tot, worst = 0, 1
    sched = list(passes(N))
    pats = []
    for p, (R, ns) in enumerate(sched):
        T = N // R
        pats.append([[j + T * r for j in range(T)] for r in range(R)])
        if p < len(sched) - 1:
            pats.append([[(j // ns) * R * ns + j % ns + ns * r for j in range(T)] for r in range(R)])
    for pat in pats:
        for lanes in pat:
            for h in range(0, len(lanes), 32):
                sl = [A(e) % 32 for e in lanes[h:h + 32]]
                c = max(np.bincount(sl, minlength=32))
                tot += c - 1
                worst = max(worst, c)
    return worst, tot


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    for N in (512, 256, 128, 64):
        x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
        ref = np.fft.ifft(x) * N
        best = []
        for a in range(1, 9):
            for b in range(0, 6):
                for m in (1, 3, 7, 15, 31):
                    A = lambda e, a=a, b=b, m=m: e ^ (((e >> a) & m) << b)
                    if sorted(A(e) for e in range(N)) != list(range(N)):
                        continue
                    w, t = conflicts(A, N)
                    best.append((w, t, a, b, m))
        best.sort()
        w, t, a, b, m = best[0]
        A = lambda e: e ^ (((e >> a) & m) << b)
        err = np.abs(stockham_inv(x, N, A) - ref).max() / np.abs(ref).max()
        print(f"N={N} schedule {SCHED[N]}: rel err {err:.1e}; plain layout conflicts {conflicts(lambda e: e, N)}, "
              f"best swizzle e ^ (((e >> {a}) & {m}) << {b}): worst {w}-way, {t} extra cycles")
