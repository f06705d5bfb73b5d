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


def stockham_wg(x, N, A=lambda e: e):
    """d = 1, 2 (N = 2048, 1024): radix N/256 from registers (m = t + 256 r) then four radix-4
    passes on all 256 threads (N/1024 butterflies per thread), ping-pong between two regions."""
    R0 = N // 256
    bufs = [np.zeros(N, complex), np.zeros(N, complex)]
    # pass 0: thread t holds m = t + 256 r
    for t in range(256):
        a = np.array([x[t + 256 * r] for r in range(R0)])
        u = np.fft.ifft(a) * R0
        for r in range(R0):
            bufs[0][A(R0 * t + r)] = u[r]
    ns, src = R0, 0
    y = np.zeros(N, complex)
    for p in range(4):
        T = N // 4
        for j in range(T):
            k = j % ns
            a = np.array([bufs[src][A(j + T * r)] for r in range(4)])
            a = a * np.exp(2j * np.pi * k * np.arange(4) / (4 * ns))
            u = np.fft.ifft(a) * 4
            for r in range(4):
                if p < 3:
                    bufs[1 - src][A((j // ns) * 4 * ns + k + ns * r)] = u[r]
                else:
                    y[j + T * r] = u[r]
        ns *= 4
        src = 1 - src
    return y


def conflicts_wg(A, N):
    R0 = N // 256
    T = N // 4
    pats = [[[R0 * t + r for t in range(256)] for r in range(R0)]]
    ns = R0
    for p in range(4):
        pats.append([[j + T * r for j in range(T)] for r in range(4)])
        if p < 3:
            pats.append([[(j // ns) * 4 * ns + j % ns + ns * r for j in range(T)] for r in range(4)])
        ns *= 4
    tot, worst = 0, 1
    for pat in pats:
        for lanes in pat:
            for h in range(0, len(lanes), 32):
                sl = [A(e) % 32 for e in lanes[h:h + 32]]
                c = max(np.bincount(sl, minlength=32))
                tot += c - 1
                worst = max(worst, c)
    return worst, tot


if __name__ == "__main__":
    rng = np.random.default_rng(2)
    for N in (1024, 2048):
        x = rng.standard_normal(N) + 1j * rng.standard_normal(N)
        ref = np.fft.ifft(x) * N
        best = []
        for a in range(1, 10):
            for m in (1, 3, 7, 15, 31):
                A = lambda e, a=a, m=m: e ^ ((e >> a) & m)
                if sorted(A(e) for e in range(N)) != list(range(N)):
                    continue
                w, t = conflicts_wg(A, N)
                best.append((w, t, a, m))
        best.sort()
        w, t, a, m = best[0]
        A = lambda e: e ^ ((e >> a) & m)
        err = np.abs(stockham_wg(x, N, A) - ref).max() / np.abs(ref).max()
        print(f"N={N} workgroup schedule {N // 256}-4-4-4-4: rel err {err:.1e}; plain {conflicts_wg(lambda e: e, N)}, "
              f"best swizzle e ^ ((e >> {a}) & {m}): worst {w}-way, {t} extra")
    # N = 2048: a wider search (two XOR terms)
    N = 2048
    best = []
    for a in range(1, 10):
        for m in (7, 15, 31):
            for a2 in range(a + 1, 11):
                for m2 in (1, 3, 7, 15, 31):
                    A = lambda e, a=a, m=m, a2=a2, m2=m2: e ^ ((e >> a) & m) ^ ((e >> a2) & m2)
                    if sorted(A(e) for e in range(N)) != list(range(N)):
                        continue
                    w, t = conflicts_wg(A, N)
                    best.append((w, t, a, m, a2, m2))
    best.sort()
    print("N=2048 two-term swizzles:", best[:3])
