// fft_device.hpp — register-level DFT cores and the LDS Stockham pass used by the
// fused r2iq kernels (ddc_kernels.hip).  gfx950 / wave64; one workgroup of NT
// threads owns one FFT in LDS.
//
// Conventions: unnormalised DFT, DIR = -1 forward (FFTW_FORWARD, e^{-2 pi i nk/N}),
// DIR = +1 backward (FFTW_BACKWARD) — the sign conventions of the reference's
// fftwf_plan_dft_r2c_1d / fftwf_plan_dft_1d(..., FFTW_BACKWARD) calls
// (Core/fft_mt_r2iq.cpp:221-225).
#pragma once

#include <hip/hip_runtime.h>

namespace sddc {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b)
{
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// a * conj(b)
__device__ __forceinline__ float2 cmulc(float2 a, float2 b)
{
    return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
// a * (DIR * i)
template <int DIR>
__device__ __forceinline__ float2 mulj(float2 a)
{
    return DIR < 0 ? make_float2(a.y, -a.x) : make_float2(-a.y, a.x);
}

// cos/sin(2*pi*m/16), exact-to-float constants
constexpr float kC16_1 = 0.92387953251128675613f;  // cos(pi/8)
constexpr float kS16_1 = 0.38268343236508977173f;  // sin(pi/8)
constexpr float kR2 = 0.70710678118654752440f;     // cos(pi/4)

// a * e^{DIR*2*pi*i*m/16} for a compile-time m (0 <= m < 16)
template <int DIR, int M>
__device__ __forceinline__ float2 tw16(float2 a)
{
    constexpr int m = M & 15;
    if constexpr (m == 0) return a;
    else if constexpr (m == 4) return mulj<DIR>(a);
    else if constexpr (m == 8) return make_float2(-a.x, -a.y);
    else if constexpr (m == 12) return mulj<-DIR>(a);
    else if constexpr (m == 2 || m == 6 || m == 10 || m == 14) {
        // e^{DIR i pi/4 * (m/2)}: (+-r2, +-r2)
        constexpr float c = (m == 2 || m == 14) ? kR2 : -kR2;
        constexpr float s = (m == 2 || m == 6) ? kR2 : -kR2;
        constexpr float sd = DIR * s;
        return make_float2(c * a.x - sd * a.y, c * a.y + sd * a.x);
    } else {
        // odd m: cos/sin of multiples of pi/8
        constexpr float c = (m == 1 || m == 15) ? kC16_1 : (m == 3 || m == 13) ? kS16_1
                          : (m == 5 || m == 11) ? -kS16_1 : -kC16_1;
        constexpr float s = (m == 1 || m == 7) ? kS16_1 : (m == 3 || m == 5) ? kC16_1
                          : (m == 9 || m == 15) ? -kS16_1 : -kC16_1;
        constexpr float sd = DIR * s;
        return make_float2(c * a.x - sd * a.y, c * a.y + sd * a.x);
    }
}

// ---------------------------------------------------------------------------
// In-register DFTs, natural order in -> natural order out (o may alias nothing).
// ---------------------------------------------------------------------------
template <int DIR>
__device__ __forceinline__ void dft2(const float2 *v, float2 *o)
{
    o[0] = cadd(v[0], v[1]);
    o[1] = csub(v[0], v[1]);
}

template <int DIR>
__device__ __forceinline__ void dft4(float2 a0, float2 a1, float2 a2, float2 a3,
                                     float2 &o0, float2 &o1, float2 &o2, float2 &o3)
{
    const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
    const float2 t2 = cadd(a1, a3), t3 = mulj<DIR>(csub(a1, a3));
    o0 = cadd(t0, t2);
    o2 = csub(t0, t2);
    o1 = cadd(t1, t3);
    o3 = csub(t1, t3);
}

template <int DIR>
__device__ __forceinline__ void dft4(const float2 *v, float2 *o)
{
    dft4<DIR>(v[0], v[1], v[2], v[3], o[0], o[1], o[2], o[3]);
}

// 8 = 4 x 2: n = 2 n1 + n2, k = k1 + 4 k2
template <int DIR>
__device__ __forceinline__ void dft8(const float2 *v, float2 *o)
{
    float2 b0[4], b1[4];
    dft4<DIR>(v[0], v[2], v[4], v[6], b0[0], b0[1], b0[2], b0[3]);
    dft4<DIR>(v[1], v[3], v[5], v[7], b1[0], b1[1], b1[2], b1[3]);
    b1[1] = tw16<DIR, 2>(b1[1]);
    b1[2] = tw16<DIR, 4>(b1[2]);
    b1[3] = tw16<DIR, 6>(b1[3]);
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) {
        o[k1] = cadd(b0[k1], b1[k1]);
        o[k1 + 4] = csub(b0[k1], b1[k1]);
    }
}

// z (1 + i tau)
__device__ __forceinline__ float2 rot1(float2 z, float tau)
{
    return make_float2(fmaf(-tau, z.y, z.x), fmaf(tau, z.x, z.y));
}
// p = a + c z, m = a - c z (real c)
__device__ __forceinline__ void axpm(float2 a, float c, float2 z, float2 &p, float2 &m)
{
    p = make_float2(fmaf(c, z.x, a.x), fmaf(c, z.y, a.y));
    m = make_float2(fmaf(-c, z.x, a.x), fmaf(-c, z.y, a.y));
}
// p = a + DIR i c z, m = a - DIR i c z (real c)
template <int DIR>
__device__ __forceinline__ void ajpm(float2 a, float c, float2 z, float2 &p, float2 &m)
{
    const float dc = DIR * c;
    p = make_float2(fmaf(-dc, z.y, a.x), fmaf(dc, z.x, a.y));
    m = make_float2(fmaf(dc, z.y, a.x), fmaf(-dc, z.x, a.y));
}

// 16 = 4 x 4: n = 4 n1 + n2, k = k1 + 4 k2
template <int DIR>
__device__ __forceinline__ void dft16(const float2 *v, float2 *o)
{
    // Second-stage twiddles in tangent form, W^m = cos(m th) (1 + i DIR tan(m th)) with
    // th = 2 pi / 16: each twiddled value enters its radix-4 as a 2-FMA rotation, and the cos
    // scale rides on the FMA that combines it (the pair W^1 / W^3 of columns 1 and 3 shares
    // one scale through the ratio cos 3th / cos th = tan th).  144 VALU instead of 156 for the
    // plain 4 x 4 form with constant twiddle products (its A/B: profiles/r02/ab/dft16_fma.txt;
    // the plain form is in git history), same results to float rounding.
    constexpr float kT1 = 0.41421356237309504880f;   // tan(pi/8) = cos(3pi/8) / cos(pi/8)
    constexpr float kT3 = 2.41421356237309504880f;   // tan(3pi/8)
    float2 b[4][4];  // b[n2][k1]
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++)
        dft4<DIR>(v[n2], v[4 + n2], v[8 + n2], v[12 + n2], b[n2][0], b[n2][1], b[n2][2], b[n2][3]);
    dft4<DIR>(b[0][0], b[1][0], b[2][0], b[3][0], o[0], o[4], o[8], o[12]);
    float2 t0, t1, p, q;
    {   // k1 = 1: W^1 b1, W^2 b2, W^3 b3
        axpm(b[0][1], kR2, rot1(b[2][1], (float)DIR), t0, t1);
        axpm(rot1(b[1][1], DIR * kT1), kT1, rot1(b[3][1], DIR * kT3), p, q);
        axpm(t0, kC16_1, p, o[1], o[9]);
        ajpm<DIR>(t1, kC16_1, q, o[5], o[13]);
    }
    {   // k1 = 2: W^2 b1, W^4 b2 = DIR i b2, W^6 b3
        ajpm<DIR>(b[0][2], 1.f, b[2][2], t0, t1);
        axpm(rot1(b[1][2], (float)DIR), -1.f, rot1(b[3][2], (float)-DIR), p, q);
        axpm(t0, kR2, p, o[2], o[10]);
        ajpm<DIR>(t1, kR2, q, o[6], o[14]);
    }
    {   // k1 = 3: W^3 b1, W^6 b2, W^9 b3 = -W^1 b3
        axpm(b[0][3], -kR2, rot1(b[2][3], (float)-DIR), t0, t1);
        axpm(rot1(b[1][3], DIR * kT3), -kT3, rot1(b[3][3], DIR * kT1), p, q);
        axpm(t0, kS16_1, p, o[3], o[11]);
        ajpm<DIR>(t1, kS16_1, q, o[7], o[15]);
    }
}

// dft16 with inputs known to be zero: ZR > 0: v[16 - ZR .. 15], ZR < 0: v[0 .. -ZR - 1]
// (|ZR| <= 8: in every first-stage radix-4 over n = 4 n1 + n2 at most one input of each
// sum/difference pair (n1, n1 + 2) is zero).  Those radix-4s take their sums and differences from
// the live inputs alone (x + 0 is not folded by the compiler: signed zeros), and the rest is
// dft16's; the outputs equal dft16's on the same values (the zero terms add nothing).
template <int ZR> __host__ __device__ constexpr bool zr_row(int k) { return ZR > 0 ? k >= 16 - ZR : ZR < 0 ? k < -ZR : false; }
template <bool ZA, bool ZB> __device__ __forceinline__ float2 zsum(float2 a, float2 b)
{
    static_assert(!(ZA && ZB), "one zero per pair");
    if constexpr (ZA) return b;
    else if constexpr (ZB) return a;
    else return cadd(a, b);
}
template <bool ZA, bool ZB> __device__ __forceinline__ float2 zdif(float2 a, float2 b)
{
    static_assert(!(ZA && ZB), "one zero per pair");
    if constexpr (ZA) return make_float2(-b.x, -b.y);
    else if constexpr (ZB) return a;
    else return csub(a, b);
}
// the first-stage radix-4 of dft16z for inputs n2, 4 + n2, 8 + n2, 12 + n2
template <int DIR, int ZR, int N2>
__device__ __forceinline__ void dft16z_first(const float2 *v, float2 (&b)[4][4])
{
    constexpr bool z0 = zr_row<ZR>(N2), z1 = zr_row<ZR>(4 + N2), z2 = zr_row<ZR>(8 + N2), z3 = zr_row<ZR>(12 + N2);
    const float2 a0 = v[N2], a1 = v[4 + N2], a2 = v[8 + N2], a3 = v[12 + N2];
    const float2 t0 = zsum<z0, z2>(a0, a2), t1 = zdif<z0, z2>(a0, a2);
    const float2 t2 = zsum<z1, z3>(a1, a3), t3 = mulj<DIR>(zdif<z1, z3>(a1, a3));
    b[N2][0] = cadd(t0, t2);
    b[N2][2] = csub(t0, t2);
    b[N2][1] = cadd(t1, t3);
    b[N2][3] = csub(t1, t3);
}
template <int DIR, int ZR>
__device__ __forceinline__ void dft16z(const float2 *v, float2 *o)
{
    static_assert(ZR >= -8 && ZR <= 8, "zero rows: at most 8 at either end");
    if constexpr (ZR == 0) {
        dft16<DIR>(v, o);
    } else {
        constexpr float kT1 = 0.41421356237309504880f;
        constexpr float kT3 = 2.41421356237309504880f;
        float2 b[4][4];  // b[n2][k1]
        dft16z_first<DIR, ZR, 0>(v, b);
        dft16z_first<DIR, ZR, 1>(v, b);
        dft16z_first<DIR, ZR, 2>(v, b);
        dft16z_first<DIR, ZR, 3>(v, b);
        dft4<DIR>(b[0][0], b[1][0], b[2][0], b[3][0], o[0], o[4], o[8], o[12]);
        float2 t0, t1, p, q;
        {   // k1 = 1 (as dft16)
            axpm(b[0][1], kR2, rot1(b[2][1], (float)DIR), t0, t1);
            axpm(rot1(b[1][1], DIR * kT1), kT1, rot1(b[3][1], DIR * kT3), p, q);
            axpm(t0, kC16_1, p, o[1], o[9]);
            ajpm<DIR>(t1, kC16_1, q, o[5], o[13]);
        }
        {   // k1 = 2
            ajpm<DIR>(b[0][2], 1.f, b[2][2], t0, t1);
            axpm(rot1(b[1][2], (float)DIR), -1.f, rot1(b[3][2], (float)-DIR), p, q);
            axpm(t0, kR2, p, o[2], o[10]);
            ajpm<DIR>(t1, kR2, q, o[6], o[14]);
        }
        {   // k1 = 3
            axpm(b[0][3], -kR2, rot1(b[2][3], (float)-DIR), t0, t1);
            axpm(rot1(b[1][3], DIR * kT3), -kT3, rot1(b[3][3], DIR * kT1), p, q);
            axpm(t0, kS16_1, p, o[3], o[11]);
            ajpm<DIR>(t1, kS16_1, q, o[7], o[15]);
        }
    }
}

// dft16 computing only the outputs o[k1 + 4 k2] of the groups k1 = 0, 1 and, when the
// (wave-uniform) flags ask, k1 = 2, 3: the first stage's k1 = 2, 3 outputs and the whole
// second-stage group are skipped otherwise (same operations as dft16 for what it computes).
// The other outputs are left unwritten.
template <int DIR>
__device__ __forceinline__ void dft16_groups(const float2 *v, float2 *o, bool need2, bool need3)
{
    constexpr float kT1 = 0.41421356237309504880f;
    constexpr float kT3 = 2.41421356237309504880f;
    float2 b[4][4];  // b[n2][k1]
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++) {
        const float2 t0 = cadd(v[n2], v[8 + n2]), t1 = csub(v[n2], v[8 + n2]);
        const float2 t2 = cadd(v[4 + n2], v[12 + n2]), t3 = mulj<DIR>(csub(v[4 + n2], v[12 + n2]));
        b[n2][0] = cadd(t0, t2);
        b[n2][1] = cadd(t1, t3);
        if (need2) b[n2][2] = csub(t0, t2);
        if (need3) b[n2][3] = csub(t1, t3);
    }
    dft4<DIR>(b[0][0], b[1][0], b[2][0], b[3][0], o[0], o[4], o[8], o[12]);
    float2 t0, t1, p, q;
    {   // k1 = 1 (as dft16)
        axpm(b[0][1], kR2, rot1(b[2][1], (float)DIR), t0, t1);
        axpm(rot1(b[1][1], DIR * kT1), kT1, rot1(b[3][1], DIR * kT3), p, q);
        axpm(t0, kC16_1, p, o[1], o[9]);
        ajpm<DIR>(t1, kC16_1, q, o[5], o[13]);
    }
    if (need2) {   // k1 = 2
        ajpm<DIR>(b[0][2], 1.f, b[2][2], t0, t1);
        axpm(rot1(b[1][2], (float)DIR), -1.f, rot1(b[3][2], (float)-DIR), p, q);
        axpm(t0, kR2, p, o[2], o[10]);
        ajpm<DIR>(t1, kR2, q, o[6], o[14]);
    }
    if (need3) {   // k1 = 3
        axpm(b[0][3], -kR2, rot1(b[2][3], (float)-DIR), t0, t1);
        axpm(rot1(b[1][3], DIR * kT3), -kT3, rot1(b[3][3], DIR * kT1), p, q);
        axpm(t0, kS16_1, p, o[3], o[11]);
        ajpm<DIR>(t1, kS16_1, q, o[7], o[15]);
    }
}

// dft16 computing only the outputs the wave-uniform mask `need` asks for (bit r: o[r]), at the
// granularity of dft16's output pairs (k1 + 4h, k1 + 4h + 8), h = 0, 1: the first stage's
// radix-4 halves and the second stage's pair computations whose outputs are all unneeded are
// skipped.  Every computed output takes dft16's operations in dft16's order (bit-identical); the
// others are left unwritten.  Used where the caller keeps a few bins of the transform (the
// persistent kernel's pruned forward pass 2 at d >= 2: 10 of 16 outputs at d = 2, 6 at d = 3,
// 4 at d >= 4).
template <int DIR>
__device__ __forceinline__ void dft16_need(const float2 *v, float2 *o, unsigned need)
{
    constexpr float kT1 = 0.41421356237309504880f;
    constexpr float kT3 = 2.41421356237309504880f;
    // pair (k1, h): outputs k1 + 4 h and k1 + 4 h + 8
    const bool p00 = need & 0x0101u, p01 = need & 0x1010u, p10 = need & 0x0202u, p11 = need & 0x2020u;
    const bool p20 = need & 0x0404u, p21 = need & 0x4040u, p30 = need & 0x0808u, p31 = need & 0x8080u;
    const bool g0 = p00 || p01, g1 = p10 || p11, g2 = p20 || p21, g3 = p30 || p31;
    float2 b[4][4];  // b[n2][k1]
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++) {
        if (g0 || g2) {
            const float2 t0 = cadd(v[n2], v[8 + n2]), t2 = cadd(v[4 + n2], v[12 + n2]);
            if (g0) b[n2][0] = cadd(t0, t2);
            if (g2) b[n2][2] = csub(t0, t2);
        }
        if (g1 || g3) {
            const float2 t1 = csub(v[n2], v[8 + n2]), t3 = mulj<DIR>(csub(v[4 + n2], v[12 + n2]));
            if (g1) b[n2][1] = cadd(t1, t3);
            if (g3) b[n2][3] = csub(t1, t3);
        }
    }
    if (p00) {   // k1 = 0: dft4 over n2
        const float2 t0 = cadd(b[0][0], b[2][0]), t2 = cadd(b[1][0], b[3][0]);
        o[0] = cadd(t0, t2);
        o[8] = csub(t0, t2);
    }
    if (p01) {
        const float2 t1 = csub(b[0][0], b[2][0]), t3 = mulj<DIR>(csub(b[1][0], b[3][0]));
        o[4] = cadd(t1, t3);
        o[12] = csub(t1, t3);
    }
    float2 t0, t1, p, q;
    if (g1) {   // k1 = 1 (as dft16)
        axpm(b[0][1], kR2, rot1(b[2][1], (float)DIR), t0, t1);
        axpm(rot1(b[1][1], DIR * kT1), kT1, rot1(b[3][1], DIR * kT3), p, q);
        if (p10) axpm(t0, kC16_1, p, o[1], o[9]);
        if (p11) ajpm<DIR>(t1, kC16_1, q, o[5], o[13]);
    }
    if (g2) {   // k1 = 2
        ajpm<DIR>(b[0][2], 1.f, b[2][2], t0, t1);
        axpm(rot1(b[1][2], (float)DIR), -1.f, rot1(b[3][2], (float)-DIR), p, q);
        if (p20) axpm(t0, kR2, p, o[2], o[10]);
        if (p21) ajpm<DIR>(t1, kR2, q, o[6], o[14]);
    }
    if (g3) {   // k1 = 3
        axpm(b[0][3], -kR2, rot1(b[2][3], (float)-DIR), t0, t1);
        axpm(rot1(b[1][3], DIR * kT3), -kT3, rot1(b[3][3], DIR * kT1), p, q);
        if (p30) axpm(t0, kS16_1, p, o[3], o[11]);
        if (p31) ajpm<DIR>(t1, kS16_1, q, o[7], o[15]);
    }
}

// a[r] *= W^{r} for r = 1..15 given the forward-direction W^1 and W^4 of this lane
// (conjugated for DIR = +1).
// p = A w, m = A conj(w) for a unit w
__device__ __forceinline__ void cmul_pm(float2 A, float2 w, float2 &p, float2 &m)
{
    const float cx = w.x * A.x, cy = w.x * A.y;
    p = make_float2(fmaf(-w.y, A.y, cx), fmaf(w.y, A.x, cy));
    m = make_float2(fmaf(w.y, A.y, cx), fmaf(-w.y, A.x, cy));
}
// 2 c a - b (real c2 = 2 c): the three-term recurrence W^{m+n} = 2 cos(n th) W^m - W^{m-n}
__device__ __forceinline__ float2 cheb(float c2, float2 a, float2 b)
{
    return make_float2(fmaf(c2, a.x, -b.x), fmaf(c2, a.y, -b.y));
}
template <int DIR>
__device__ __forceinline__ void twiddle_rec16(float2 *a, float2 w1, float2 w4)
{
    if (DIR > 0) {
        w1.y = -w1.y;
        w4.y = -w4.y;
    }
    // W^8, W^12 as products; W^{4k +- 1} as pairs A W, A conj(W) sharing the products cos * A
    // (3 ops each); W^2 and W^{4k + 2}, W^15 by one step of the Chebyshev recurrence
    // W^{m+1} = 2 cos(th) W^m - W^{m-1} (2 FMAs): 38 VALU for the 13 powers instead of 52 for
    // all products (that form is in git history; A/B profiles/r02/ab/twrec_hybrid.txt).
    // float32 model over all 4096 bases: worst power error 4.6e-7 (rms 7.1e-8) against 3.2e-7
    // (6.9e-8) for the all-product form; a pure Chebyshev form (28 VALU, 1.3e-6) leaked past the
    // 1e-5 bar on the out-of-band parity case at d = 4 (profiles/r02/ab/cheb.txt).
    const float c1 = w1.x + w1.x;
    const float2 w8 = cmul(w4, w4), w12 = cmul(w8, w4);
    float2 w3, w5, w7, w9, w11, w13;
    cmul_pm(w4, w1, w5, w3);
    cmul_pm(w8, w1, w9, w7);
    cmul_pm(w12, w1, w13, w11);
    const float2 w2 = cheb(c1, w1, make_float2(1.f, 0.f)), w6 = cheb(c1, w5, w4);
    const float2 w10 = cheb(c1, w9, w8), w14 = cheb(c1, w13, w12), w15 = cheb(c1, w14, w13);
    a[1] = cmul(a[1], w1);
    a[2] = cmul(a[2], w2);
    a[3] = cmul(a[3], w3);
    a[4] = cmul(a[4], w4);
    a[5] = cmul(a[5], w5);
    a[6] = cmul(a[6], w6);
    a[7] = cmul(a[7], w7);
    a[8] = cmul(a[8], w8);
    a[9] = cmul(a[9], w9);
    a[10] = cmul(a[10], w10);
    a[11] = cmul(a[11], w11);
    a[12] = cmul(a[12], w12);
    a[13] = cmul(a[13], w13);
    a[14] = cmul(a[14], w14);
    a[15] = cmul(a[15], w15);
}

// a[r] *= W^r for r = 1..15 (forward, DIR = -1) from six exactly rounded anchors W^1, W^2, W^3,
// W^4, W^8, W^12 of the lane's base: W^{4h + l} = W^{4h} W^l, one product per other power (36
// VALU, as twiddle_rec16's 38).  More accurate than the recurrence: in the float32 model of the
// kernel (tools/fp32_model.py, twmode "anchor6") the leakage-only draws of tests/test_gpu_floor.py
// go from a geometric mean of 0.95 (max 1.68) x the reference-class float32 port's error to 0.81
// (max 1.17), where the exactly rounded table of all 15 powers gives 0.87 (max 1.44).
template <int DIR>
__device__ __forceinline__ void twiddle_anchor6(float2 *a, float2 w1, float2 w2, float2 w3, float2 w4, float2 w8,
                                                float2 w12)
{
    static_assert(DIR < 0, "forward twiddles");
    a[1] = cmul(a[1], w1);
    a[2] = cmul(a[2], w2);
    a[3] = cmul(a[3], w3);
    a[4] = cmul(a[4], w4);
    a[5] = cmul(a[5], cmul(w4, w1));
    a[6] = cmul(a[6], cmul(w4, w2));
    a[7] = cmul(a[7], cmul(w4, w3));
    a[8] = cmul(a[8], w8);
    a[9] = cmul(a[9], cmul(w8, w1));
    a[10] = cmul(a[10], cmul(w8, w2));
    a[11] = cmul(a[11], cmul(w8, w3));
    a[12] = cmul(a[12], w12);
    a[13] = cmul(a[13], cmul(w12, w1));
    a[14] = cmul(a[14], cmul(w12, w2));
    a[15] = cmul(a[15], cmul(w12, w3));
}

// a[r] *= g W^{r} for r = 0..15 (W conjugated for DIR = +1), with g W^0 = u0, g W^1 = u1 and
// g W^4 = u4 given (exactly rounded, from the table) and the lane's forward W^1, W^4 for the
// steps: the same products and Chebyshev steps as twiddle_rec16 on the sequence g W^r (the
// three-term recurrence holds for any geometric sequence), plus the product for r = 0.
template <int DIR>
__device__ __forceinline__ void twiddle_g16(float2 *a, float2 u0, float2 u1, float2 u4, float2 w1, float2 w4)
{
    if (DIR > 0) {
        w1.y = -w1.y;
        w4.y = -w4.y;
    }
    const float c1 = w1.x + w1.x;
    const float2 u8 = cmul(u4, w4), u12 = cmul(u8, w4);
    float2 u3, u5, u7, u9, u11, u13;
    cmul_pm(u4, w1, u5, u3);
    cmul_pm(u8, w1, u9, u7);
    cmul_pm(u12, w1, u13, u11);
    const float2 u2 = cheb(c1, u1, u0), u6 = cheb(c1, u5, u4);
    const float2 u10 = cheb(c1, u9, u8), u14 = cheb(c1, u13, u12), u15 = cheb(c1, u14, u13);
    a[0] = cmul(a[0], u0);
    a[1] = cmul(a[1], u1);
    a[2] = cmul(a[2], u2);
    a[3] = cmul(a[3], u3);
    a[4] = cmul(a[4], u4);
    a[5] = cmul(a[5], u5);
    a[6] = cmul(a[6], u6);
    a[7] = cmul(a[7], u7);
    a[8] = cmul(a[8], u8);
    a[9] = cmul(a[9], u9);
    a[10] = cmul(a[10], u10);
    a[11] = cmul(a[11], u11);
    a[12] = cmul(a[12], u12);
    a[13] = cmul(a[13], u13);
    a[14] = cmul(a[14], u14);
    a[15] = cmul(a[15], u15);
}

template <int R, int DIR>
__device__ __forceinline__ void dft(const float2 *v, float2 *o)
{
    if constexpr (R == 2) dft2<DIR>(v, o);
    else if constexpr (R == 4) dft4<DIR>(v, o);
    else if constexpr (R == 8) dft8<DIR>(v, o);
    else {
        static_assert(R == 16, "radix must be 2, 4, 8 or 16");
        dft16<DIR>(v, o);
    }
}

// ---------------------------------------------------------------------------
// DFT-32 and DFT-64 in registers (the one-wave-per-frame kernel, ddc_wave.hip)
// ---------------------------------------------------------------------------
// cos / sin(2 pi m / 64)
__device__ constexpr float kC64[64] = {
    1.0f, 0.99518472667219693f, 0.98078528040323043f, 0.95694033573220882f, 0.92387953251128674f,
    0.88192126434835505f, 0.83146961230254524f, 0.77301045336273699f, 0.70710678118654757f,
    0.63439328416364549f, 0.55557023301960218f, 0.47139673682599764f, 0.38268343236508978f,
    0.29028467725446233f, 0.19509032201612825f, 0.098017140329560604f, 0.0f, -0.098017140329560604f,
    -0.19509032201612825f, -0.29028467725446233f, -0.38268343236508978f, -0.47139673682599764f,
    -0.55557023301960218f, -0.63439328416364549f, -0.70710678118654757f, -0.77301045336273699f,
    -0.83146961230254524f, -0.88192126434835505f, -0.92387953251128674f, -0.95694033573220882f,
    -0.98078528040323043f, -0.99518472667219693f, -1.0f, -0.99518472667219693f, -0.98078528040323043f,
    -0.95694033573220882f, -0.92387953251128674f, -0.88192126434835505f, -0.83146961230254524f,
    -0.77301045336273699f, -0.70710678118654757f, -0.63439328416364549f, -0.55557023301960218f,
    -0.47139673682599764f, -0.38268343236508978f, -0.29028467725446233f, -0.19509032201612825f,
    -0.098017140329560604f, 0.0f, 0.098017140329560604f, 0.19509032201612825f, 0.29028467725446233f,
    0.38268343236508978f, 0.47139673682599764f, 0.55557023301960218f, 0.63439328416364549f,
    0.70710678118654757f, 0.77301045336273699f, 0.83146961230254524f, 0.88192126434835505f,
    0.92387953251128674f, 0.95694033573220882f, 0.98078528040323043f, 0.99518472667219693f};

// a * e^{DIR 2 pi i m / 64}; m is a constant after unrolling, so the special cases fold
template <int DIR>
__device__ __forceinline__ float2 tw64(float2 a, int m)
{
    m &= 63;
    if (m == 0) return a;
    if (m == 16) return mulj<DIR>(a);
    if (m == 32) return make_float2(-a.x, -a.y);
    if (m == 48) return mulj<-DIR>(a);
    const float c = kC64[m], s = DIR * kC64[(m + 48) & 63];   // sin(x) = cos(x - pi/2)
    return make_float2(c * a.x - s * a.y, c * a.y + s * a.x);
}

// DFT-32, natural order in and out: n = 4 n1 + n2, k = k1 + 8 k2
template <int DIR>
__device__ __forceinline__ void dft32(const float2 *x, float2 *o)
{
    float2 b[4][8];
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++) {
        float2 v[8];
#pragma unroll
        for (int n1 = 0; n1 < 8; n1++) v[n1] = x[4 * n1 + n2];
        dft8<DIR>(v, b[n2]);
    }
#pragma unroll
    for (int n2 = 1; n2 < 4; n2++)
#pragma unroll
        for (int k1 = 1; k1 < 8; k1++) b[n2][k1] = tw64<DIR>(b[n2][k1], 2 * n2 * k1);
#pragma unroll
    for (int k1 = 0; k1 < 8; k1++)
        dft4<DIR>(b[0][k1], b[1][k1], b[2][k1], b[3][k1], o[k1], o[k1 + 8], o[k1 + 16], o[k1 + 24]);
}

// DFT-64, natural order in and out: n = 8 n1 + n2, k = k1 + 8 k2
template <int DIR>
__device__ __forceinline__ void dft64(const float2 *x, float2 *o)
{
    float2 b[8][8];
#pragma unroll
    for (int n2 = 0; n2 < 8; n2++) {
        float2 v[8];
#pragma unroll
        for (int n1 = 0; n1 < 8; n1++) v[n1] = x[8 * n1 + n2];
        dft8<DIR>(v, b[n2]);
    }
#pragma unroll
    for (int n2 = 1; n2 < 8; n2++)
#pragma unroll
        for (int k1 = 1; k1 < 8; k1++) b[n2][k1] = tw64<DIR>(b[n2][k1], n2 * k1);
#pragma unroll
    for (int k1 = 0; k1 < 8; k1++) {
        float2 v[8], w[8];
#pragma unroll
        for (int n2 = 0; n2 < 8; n2++) v[n2] = b[n2][k1];
        dft8<DIR>(v, w);
#pragma unroll
        for (int k2 = 0; k2 < 8; k2++) o[k1 + 8 * k2] = w[k2];
    }
}

// ---------------------------------------------------------------------------
// Packed-FP32 variants (gfx950 v_pk_{add,mul,fma}_f32 on (re, im) register pairs).
// The ±i rotations and the operand swaps of a complex product ride on the VOP3P
// op_sel / op_sel_hi / neg_lo / neg_hi source modifiers, so a butterfly is one
// instruction, a twiddle multiply two, and a radix-16 DFT 80 (vs ~154 scalar).
// ---------------------------------------------------------------------------
namespace pk {
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v V(float2 a) { return f2v{a.x, a.y}; }
__device__ __forceinline__ float2 F(f2v a) { return make_float2(a.x, a.y); }

// t + DIR*i*d  and  t - DIR*i*d  (mulj<DIR>, one instruction each)
template <int DIR>
__device__ __forceinline__ f2v addj(f2v t, f2v d)
{
    f2v r;
    if constexpr (DIR < 0)   // (t.x + d.y, t.y - d.x)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(t), "v"(d));
    else                     // (t.x - d.y, t.y + d.x)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(t), "v"(d));
    return r;
}
template <int DIR>
__device__ __forceinline__ f2v subj(f2v t, f2v d)
{
    return addj<-DIR>(t, d);
}

// a * w and a * conj(w): t = (a.x w.x, a.y w.x); r = t + (a.y, a.x) * (-+w.y, +-w.y)
__device__ __forceinline__ f2v cmul(f2v a, f2v w)
{
    f2v t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]"
        : "=v"(r) : "v"(a), "v"(w), "v"(t));
    return r;
}
__device__ __forceinline__ f2v cmulc(f2v a, f2v w)
{
    f2v t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]"
        : "=v"(r) : "v"(a), "v"(w), "v"(t));
    return r;
}

// e^{DIR*2*pi*i*m/16} as (cos, sin) constants
template <int DIR, int M>
__device__ __forceinline__ f2v w16()
{
    constexpr int m = M & 15;
    constexpr float c = (m == 1 || m == 15) ? kC16_1 : (m == 3 || m == 13) ? kS16_1
                      : (m == 5 || m == 11) ? -kS16_1 : (m == 7 || m == 9) ? -kC16_1
                      : (m == 2 || m == 14) ? kR2 : (m == 6 || m == 10) ? -kR2 : 0.f;
    constexpr float s = (m == 1 || m == 7) ? kS16_1 : (m == 3 || m == 5) ? kC16_1
                      : (m == 9 || m == 15) ? -kS16_1 : (m == 11 || m == 13) ? -kC16_1
                      : (m == 2 || m == 6) ? kR2 : (m == 10 || m == 14) ? -kR2 : 0.f;
    return f2v{c, DIR * s};
}

// natural order in -> natural order out; a2 is multiplied by DIR*i first when J2
template <int DIR, bool J2 = false>
__device__ __forceinline__ void dft4(f2v a0, f2v a1, f2v a2, f2v a3, f2v &o0, f2v &o1, f2v &o2, f2v &o3)
{
    const f2v t0 = J2 ? addj<DIR>(a0, a2) : a0 + a2;
    const f2v t1 = J2 ? subj<DIR>(a0, a2) : a0 - a2;
    const f2v t2 = a1 + a3, d = a1 - a3;
    o0 = t0 + t2;
    o2 = t0 - t2;
    o1 = addj<DIR>(t1, d);
    o3 = subj<DIR>(t1, d);
}

// 16 = 4 x 4 as sddc::dft16, with W_16^4 folded into the second stage
template <int DIR>
__device__ __forceinline__ void dft16(const float2 *v, float2 *o)
{
    f2v b[4][4];
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++)
        dft4<DIR>(V(v[n2]), V(v[4 + n2]), V(v[8 + n2]), V(v[12 + n2]), b[n2][0], b[n2][1], b[n2][2], b[n2][3]);
    b[1][1] = cmul(b[1][1], w16<DIR, 1>());
    b[1][2] = cmul(b[1][2], w16<DIR, 2>());
    b[1][3] = cmul(b[1][3], w16<DIR, 3>());
    b[2][1] = cmul(b[2][1], w16<DIR, 2>());
    b[2][3] = cmul(b[2][3], w16<DIR, 6>());
    b[3][1] = cmul(b[3][1], w16<DIR, 3>());
    b[3][2] = cmul(b[3][2], w16<DIR, 6>());
    b[3][3] = cmul(b[3][3], w16<DIR, 9>());
    f2v r[16];
    dft4<DIR>(b[0][0], b[1][0], b[2][0], b[3][0], r[0], r[4], r[8], r[12]);
    dft4<DIR>(b[0][1], b[1][1], b[2][1], b[3][1], r[1], r[5], r[9], r[13]);
    dft4<DIR, true>(b[0][2], b[1][2], b[2][2], b[3][2], r[2], r[6], r[10], r[14]);   // b[2][2] * W^4
    dft4<DIR>(b[0][3], b[1][3], b[2][3], b[3][3], r[3], r[7], r[11], r[15]);
#pragma unroll
    for (int k = 0; k < 16; k++) o[k] = F(r[k]);
}
}  // namespace pk

// ---------------------------------------------------------------------------
// LDS layout: complex element i lives at float2 slot lds_pad(i) = i + i/16.
// One pad slot per 16 elements keeps the radix-16 "16 consecutive per lane"
// writes of the first pass conflict-free on ds_write_b64 (bank = dword/2 mod 32).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lds_pad(int i) { return i + (i >> 4); }
constexpr int lds_slots(int n) { return n + n / 16; }

// ---------------------------------------------------------------------------
// One Stockham radix-R pass of an N-point transform (DIT, autosort), NT threads.
//   in  position for butterfly j, leg r:  j + r*N/R
//   out position:                          (j/NS)*NS*R + j%NS + r*NS
//   twiddle of leg r:  W_{NS*R}^{(j%NS)*r}, read from tw4096[k] = e^{-2 pi i k/4096}
//                      (conjugated for DIR = +1).  N*... must divide 4096.
// `load(pos)` supplies inputs, `store(pos, value)` consumes outputs.  The caller
// places the barriers: a pass reads everything into registers, then the caller
// syncs, then the pass stores (so one LDS buffer serves in and out).
// ---------------------------------------------------------------------------
template <int N, int R, int NS, int NT>
struct StockhamPass {
    static constexpr int NB = N / R;                 // butterflies
    static constexpr int PER = (NB + NT - 1) / NT;   // butterflies per thread
    static_assert(N % R == 0 && 4096 % (NS * R) == 0, "bad pass geometry");
    float2 v[PER][R];

    template <int DIR, class Load>
    __device__ __forceinline__ void compute(Load load, const float2 *__restrict__ tw4096)
    {
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = (int)threadIdx.x + i * NT;
            if (NB % NT == 0 || j < NB) {
                float2 a[R];
#pragma unroll
                for (int r = 0; r < R; r++) a[r] = load(j + r * NB);
                if constexpr (NS > 1) {
                    const int step = (j % NS) * (4096 / (NS * R));
#pragma unroll
                    for (int r = 1; r < R; r++) {
                        const float2 w = tw4096[step * r];
                        a[r] = DIR < 0 ? cmul(a[r], w) : cmulc(a[r], w);
                    }
                }
                dft<R, DIR>(a, v[i]);
            }
        }
    }

    template <class Store>
    __device__ __forceinline__ void store(Store st) const
    {
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = (int)threadIdx.x + i * NT;
            if (NB % NT == 0 || j < NB) {
                const int base = (j / NS) * NS * R + (j % NS);
#pragma unroll
                for (int r = 0; r < R; r++) st(base + r * NS, v[i][r]);
            }
        }
    }
};

}  // namespace sddc
