#!/usr/bin/env python3
"""numpy model of the d = 4 inverse tail of r2iq_persistent_kernel (ddc_persistent.hip, R4T):
the 256-point inverse DFT as four radix-4 Stockham passes on 64 lanes (thread j reads elements
j + 64 r, twiddles e^{+2 pi i k r / (4 Ns)} with k = j mod Ns, writes (j / Ns) 4 Ns + k + Ns r;
the last pass leaves y[j + 64 r] in registers), checked against numpy's inverse FFT, plus a
search over XOR swizzles e ^ (((e >> a) & m) << b) for the LDS layout, scoring the bank
conflicts of every read and write pattern per 32-lane half of a ds_*_b64 (element slot mod 32).
The kernel uses the conflict-free e ^ ((e >> 2) & 31) found here.
"""
import numpy as np, itertools
N=256
def stockham_inv(x, A=lambda e:e):
    buf=np.zeros(512,complex)
    for e in range(N): buf[A(e)]=x[e]
    for p in range(4):
        Ns=4**p
        u=np.zeros((64,4),complex)
        for j in range(64):
            a=np.array([buf[A(j+64*r)] for r in range(4)])
            k=j%Ns
            a=a*np.exp(2j*np.pi*k*np.arange(4)/(4*Ns))
            u[j]=np.array([sum(a[n]*np.exp(2j*np.pi*n*m/4) for n in range(4)) for m in range(4)])
        if p<3:
            for j in range(64):
                k=j%Ns
                for r in range(4): buf[A((j//Ns)*4*Ns+k+Ns*r)]=u[j,r]
    y=np.zeros(N,complex)
    for j in range(64):
        for r in range(4): y[j+64*r]=u[j,r]
    return y
x=np.random.randn(N)+1j*np.random.randn(N)
ref=np.fft.ifft(x)*N
print("plain", np.abs(stockham_inv(x)-ref).max())
def conflicts(A):
    # ds_*_b64: 32-lane groups, bank pair = (2*addr) mod 64 -> element slot addr mod 32
    worst=0
    pats=[]
    for p in range(4):
        Ns=4**p
        pats.append([[j+64*r for j in range(64)] for r in range(4)])           # reads
        if p<3: pats.append([[(j//Ns)*4*Ns+j%Ns+Ns*r for j in range(64)] for r in range(4)])  # writes
    pats.append([[t] for t in range(256)])
    tot=0
    for pat in pats[:-1]:
        for lanes in pat:
            for h in range(2):
                sl=[A(e)%32 for e in lanes[32*h:32*h+32]]
                c=max(np.bincount(sl,minlength=32))
                tot+=c-1; worst=max(worst,c)
    return worst,tot
print("plain conflicts", conflicts(lambda e:e))
best=[]
for a in range(1,8):
  for b in range(0,6):
    for m in [1,3,7,15,31]:
      A=lambda e,a=a,b=b,m=m: e ^ (((e>>a)&m)<<b)
      if len(set(A(e) for e in range(256)))!=256 or max(A(e) for e in range(256))>=256: continue
      w,t=conflicts(A)
      best.append((w,t,a,b,m))
best.sort(); print(best[:8])
w,t,a,b,m=best[0]
A=lambda e: e ^ (((e>>a)&m)<<b)
print("swz err", np.abs(stockham_inv(x,A)-ref).max())
