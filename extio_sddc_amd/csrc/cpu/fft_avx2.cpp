// fft_avx2.cpp — radix-16/4 Stockham FFTs in AVX2 + FMA for the CPU r2iq backend (fft_avx2.hpp).
//
// One pass of radix R and sub-length L = n / s (m = L / R butterflies per group), decimation in
// frequency:
//   a_k = src[s (p + k m) + q]                        k = 0..R-1, p < m, q < s
//   dst[s (R p + k) + q] = DFT_R(a)_k * W_L^{p k}
// After the passes (radix 16 for n >= 4096, radix 4 below; one radix-2 pass, L = 2, when n is
// 2 * 4^k) dst is in natural order.  Twiddles are e^{-2 pi i p k / L}, evaluated in double and
// rounded once; the backward transform uses their conjugates.  Radix 16 halves the passes of
// n = 4096, whose two 32 KB ping-pong buffers do not fit a 48 KB L1 together: the transform is
// L2-bound, so the pass count sets its time (radix 4: 8.0 us, radix 16: see DESIGN.md §4.7).
#include "fft_avx2.hpp"

#include <immintrin.h>

#include <cmath>
#include <stdexcept>
#include <utility>

namespace sddc {
namespace cpu {
namespace {

// x * w (SIGN < 0) or x * conj(w) (SIGN > 0)
template <int SIGN>
inline void cmul(__m256 &xr, __m256 &xi, __m256 wr, __m256 wi)
{
    const __m256 r = xr, i = xi;
    if (SIGN < 0) {
        xr = _mm256_fmsub_ps(r, wr, _mm256_mul_ps(i, wi));
        xi = _mm256_fmadd_ps(r, wi, _mm256_mul_ps(i, wr));
    } else {
        xr = _mm256_fmadd_ps(r, wr, _mm256_mul_ps(i, wi));
        xi = _mm256_fmsub_ps(i, wr, _mm256_mul_ps(r, wi));
    }
}

// in-register DFT-4 of (a0..a3); SIGN = -1 forward (X1 = t1 - i t3), +1 backward (X1 = t1 + i t3)
template <int SIGN>
inline void dft4(__m256 r[4], __m256 i[4])
{
    const __m256 t0r = _mm256_add_ps(r[0], r[2]), t0i = _mm256_add_ps(i[0], i[2]);
    const __m256 t1r = _mm256_sub_ps(r[0], r[2]), t1i = _mm256_sub_ps(i[0], i[2]);
    const __m256 t2r = _mm256_add_ps(r[1], r[3]), t2i = _mm256_add_ps(i[1], i[3]);
    const __m256 t3r = _mm256_sub_ps(r[1], r[3]), t3i = _mm256_sub_ps(i[1], i[3]);
    r[0] = _mm256_add_ps(t0r, t2r);
    i[0] = _mm256_add_ps(t0i, t2i);
    r[2] = _mm256_sub_ps(t0r, t2r);
    i[2] = _mm256_sub_ps(t0i, t2i);
    if (SIGN < 0) {   // -i t3 = (t3i, -t3r)
        r[1] = _mm256_add_ps(t1r, t3i);
        i[1] = _mm256_sub_ps(t1i, t3r);
        r[3] = _mm256_sub_ps(t1r, t3i);
        i[3] = _mm256_add_ps(t1i, t3r);
    } else {          // +i t3 = (-t3i, t3r)
        r[1] = _mm256_sub_ps(t1r, t3i);
        i[1] = _mm256_add_ps(t1i, t3r);
        r[3] = _mm256_add_ps(t1r, t3i);
        i[3] = _mm256_sub_ps(t1i, t3r);
    }
}

// [x0 | x1 | x2 | x3] (8 lanes each, lane = p) -> 32 floats in (p, k) order
inline void store_transposed(float *dst, __m256 x0, __m256 x1, __m256 x2, __m256 x3)
{
    const __m256 t0 = _mm256_unpacklo_ps(x0, x1), t1 = _mm256_unpackhi_ps(x0, x1);
    const __m256 t2 = _mm256_unpacklo_ps(x2, x3), t3 = _mm256_unpackhi_ps(x2, x3);
    const __m256 u0 = _mm256_shuffle_ps(t0, t2, 0x44), u1 = _mm256_shuffle_ps(t0, t2, 0xEE);
    const __m256 u2 = _mm256_shuffle_ps(t1, t3, 0x44), u3 = _mm256_shuffle_ps(t1, t3, 0xEE);
    _mm256_storeu_ps(dst + 0, _mm256_permute2f128_ps(u0, u1, 0x20));
    _mm256_storeu_ps(dst + 8, _mm256_permute2f128_ps(u2, u3, 0x20));
    _mm256_storeu_ps(dst + 16, _mm256_permute2f128_ps(u0, u1, 0x31));
    _mm256_storeu_ps(dst + 24, _mm256_permute2f128_ps(u2, u3, 0x31));
}

// 8 complex samples of an int16 (re, im) pair stream, with the r2iq de-randomiser
// (rand && (v & 1) ? v ^ 0xFFFE : v, Core/fft_mt_r2iq.h:36-51) when rmask is all ones
inline void load_i16(const int16_t *x, __m256i rmask, __m256 &re, __m256 &im)
{
    const __m256i one = _mm256_set1_epi16(1), fffe = _mm256_set1_epi16((short)0xFFFE);
    __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(x));
    const __m256i odd = _mm256_cmpeq_epi16(_mm256_and_si256(v, one), one);
    v = _mm256_xor_si256(v, _mm256_and_si256(_mm256_and_si256(odd, rmask), fffe));
    re = _mm256_cvtepi32_ps(_mm256_srai_epi32(_mm256_slli_epi32(v, 16), 16));
    im = _mm256_cvtepi32_ps(_mm256_srai_epi32(v, 16));
}

// s = 1: vectors over 8 consecutive p; twiddles [p/8][k-1][re 8 | im 8].  I16: the input is
// int16 (re, im) pairs at xi (the r2iq frame), converted on load.
template <int SIGN, bool I16>
void pass4_s1(int n, const float *tw, const float *sr, const float *si, const int16_t *xi, __m256i rmask,
              float *dr, float *di)
{
    const int m = n / 4;
    for (int p = 0; p < m; p += 8, tw += 48) {
        __m256 r[4], i[4];
        for (int k = 0; k < 4; k++) {
            if (I16) {
                load_i16(xi + 2 * (p + k * m), rmask, r[k], i[k]);
            } else {
                r[k] = _mm256_loadu_ps(sr + p + k * m);
                i[k] = _mm256_loadu_ps(si + p + k * m);
            }
        }
        dft4<SIGN>(r, i);
        for (int k = 1; k < 4; k++)
            cmul<SIGN>(r[k], i[k], _mm256_loadu_ps(tw + 16 * (k - 1)), _mm256_loadu_ps(tw + 16 * (k - 1) + 8));
        store_transposed(dr + 4 * p, r[0], r[1], r[2], r[3]);
        store_transposed(di + 4 * p, i[0], i[1], i[2], i[3]);
    }
}

// s = 4: a vector holds q = 0..3 of p and of p + 1; twiddles [p/2][k-1][re 8 | im 8]
template <int SIGN>
void pass4_s4(int n, const float *tw, const float *sr, const float *si, float *dr, float *di)
{
    const int m = n / 16;
    for (int p = 0; p < m; p += 2, tw += 48) {
        __m256 r[4], i[4];
        for (int k = 0; k < 4; k++) {
            r[k] = _mm256_loadu_ps(sr + 4 * (p + k * m));
            i[k] = _mm256_loadu_ps(si + 4 * (p + k * m));
        }
        dft4<SIGN>(r, i);
        for (int k = 1; k < 4; k++)
            cmul<SIGN>(r[k], i[k], _mm256_loadu_ps(tw + 16 * (k - 1)), _mm256_loadu_ps(tw + 16 * (k - 1) + 8));
        // dst[16 p + 4 k + q] (p) and dst[16 (p + 1) + 4 k + q] (p + 1)
        float *o[2] = {dr + 16 * p, di + 16 * p};
        const __m256 *x[2] = {r, i};
        for (int c = 0; c < 2; c++) {
            const __m256 *v = x[c];
            _mm256_storeu_ps(o[c] + 0, _mm256_permute2f128_ps(v[0], v[1], 0x20));
            _mm256_storeu_ps(o[c] + 8, _mm256_permute2f128_ps(v[2], v[3], 0x20));
            _mm256_storeu_ps(o[c] + 16, _mm256_permute2f128_ps(v[0], v[1], 0x31));
            _mm256_storeu_ps(o[c] + 24, _mm256_permute2f128_ps(v[2], v[3], 0x31));
        }
    }
}

// s >= 16: vectors over q; twiddles [p][k-1][re, im] scalars
template <int SIGN>
void pass4_sN(int n, int s, const float *tw, const float *sr, const float *si, float *dr, float *di)
{
    const int m = n / (4 * s);
    const int step = n / 4;   // s * m
    for (int p = 0; p < m; p++, tw += 6) {
        __m256 wr[3], wi[3];
        for (int k = 0; k < 3; k++) {
            wr[k] = _mm256_broadcast_ss(tw + 2 * k);
            wi[k] = _mm256_broadcast_ss(tw + 2 * k + 1);
        }
        const float *ar = sr + s * p, *ai = si + s * p;
        float *orr = dr + 4 * s * p, *oi = di + 4 * s * p;
        for (int q = 0; q < s; q += 8) {
            __m256 r[4], i[4];
            for (int k = 0; k < 4; k++) {
                r[k] = _mm256_loadu_ps(ar + q + k * step);
                i[k] = _mm256_loadu_ps(ai + q + k * step);
            }
            dft4<SIGN>(r, i);
            if (p != 0)
                for (int k = 1; k < 4; k++) cmul<SIGN>(r[k], i[k], wr[k - 1], wi[k - 1]);
            for (int k = 0; k < 4; k++) {
                _mm256_storeu_ps(orr + q + k * s, r[k]);
                _mm256_storeu_ps(oi + q + k * s, i[k]);
            }
        }
    }
}

// 8 x 8 transpose of (r[0..7]) (row = register, column = lane)
inline void transpose8(__m256 r[8])
{
    const __m256 t0 = _mm256_unpacklo_ps(r[0], r[1]), t1 = _mm256_unpackhi_ps(r[0], r[1]);
    const __m256 t2 = _mm256_unpacklo_ps(r[2], r[3]), t3 = _mm256_unpackhi_ps(r[2], r[3]);
    const __m256 t4 = _mm256_unpacklo_ps(r[4], r[5]), t5 = _mm256_unpackhi_ps(r[4], r[5]);
    const __m256 t6 = _mm256_unpacklo_ps(r[6], r[7]), t7 = _mm256_unpackhi_ps(r[6], r[7]);
    const __m256 u0 = _mm256_shuffle_ps(t0, t2, 0x44), u1 = _mm256_shuffle_ps(t0, t2, 0xEE);
    const __m256 u2 = _mm256_shuffle_ps(t1, t3, 0x44), u3 = _mm256_shuffle_ps(t1, t3, 0xEE);
    const __m256 u4 = _mm256_shuffle_ps(t4, t6, 0x44), u5 = _mm256_shuffle_ps(t4, t6, 0xEE);
    const __m256 u6 = _mm256_shuffle_ps(t5, t7, 0x44), u7 = _mm256_shuffle_ps(t5, t7, 0xEE);
    r[0] = _mm256_permute2f128_ps(u0, u4, 0x20);
    r[1] = _mm256_permute2f128_ps(u1, u5, 0x20);
    r[2] = _mm256_permute2f128_ps(u2, u6, 0x20);
    r[3] = _mm256_permute2f128_ps(u3, u7, 0x20);
    r[4] = _mm256_permute2f128_ps(u0, u4, 0x31);
    r[5] = _mm256_permute2f128_ps(u1, u5, 0x31);
    r[6] = _mm256_permute2f128_ps(u2, u6, 0x31);
    r[7] = _mm256_permute2f128_ps(u3, u7, 0x31);
}

// ---- n = 4096 as 64 x 64 (four-step) --------------------------------------------------------
// x[64 n1 + n2] -> X[k1 + 64 k2] = sum_n2 W_64^{n2 k2} W_4096^{n2 k1} sum_n1 x[64 n1 + n2] W_64^{n1 k1}
//   A: 8 column groups, 8 columns per vector: FFT-64 over n1, times W_4096^{n2 k1}, -> Y[64 k1 + n2]
//   B: 8 row groups, 8 rows per vector (8 x 8 transposes): FFT-64 over n2 -> X[64 k2 + k1]
// Each FFT-64 runs on 64 vectors (4 KB) in L1; the whole transform moves the data through L2
// twice instead of six times.

// In-place radix-4 DIF FFT-64 over v[0..63] (lanes independent).  Frequency k ends at
// position pos64(k) (base-4 digit reversal).  tw: W_64^{p k} (p < 16) then W_16^{p k} (p < 4),
// [p][k - 1] (re, im).
inline int pos64(int k) { return 16 * (k & 3) + 4 * ((k >> 2) & 3) + (k >> 4); }

template <int SIGN>
inline void fft64_vec(__m256 *vr, __m256 *vi, const float *tw)
{
    for (int p = 0; p < 16; p++) {   // L = 64: a_k = v[p + 16 k]
        __m256 r[4] = {vr[p], vr[p + 16], vr[p + 32], vr[p + 48]};
        __m256 i[4] = {vi[p], vi[p + 16], vi[p + 32], vi[p + 48]};
        dft4<SIGN>(r, i);
        for (int k = 0; k < 4; k++) {
            if (p && k) cmul<SIGN>(r[k], i[k], _mm256_broadcast_ss(tw + 6 * p + 2 * (k - 1)), _mm256_broadcast_ss(tw + 6 * p + 2 * (k - 1) + 1));
            vr[p + 16 * k] = r[k];
            vi[p + 16 * k] = i[k];
        }
    }
    const float *t16 = tw + 96;
    for (int b = 0; b < 64; b += 16)   // L = 16: a_k = v[b + p + 4 k]
        for (int p = 0; p < 4; p++) {
            __m256 r[4] = {vr[b + p], vr[b + p + 4], vr[b + p + 8], vr[b + p + 12]};
            __m256 i[4] = {vi[b + p], vi[b + p + 4], vi[b + p + 8], vi[b + p + 12]};
            dft4<SIGN>(r, i);
            for (int k = 0; k < 4; k++) {
                if (p && k) cmul<SIGN>(r[k], i[k], _mm256_broadcast_ss(t16 + 6 * p + 2 * (k - 1)), _mm256_broadcast_ss(t16 + 6 * p + 2 * (k - 1) + 1));
                vr[b + p + 4 * k] = r[k];
                vi[b + p + 4 * k] = i[k];
            }
        }
    for (int b = 0; b < 64; b += 4) dft4<SIGN>(vr + b, vi + b);   // L = 4
}

// twA: W_4096^{(8 g + l) k1} as [g][k1][re 8 | im 8]; tw: fft64_vec's table
template <int SIGN, bool I16>
void fft4096(const float *twA, const float *tw, const float *xr, const float *xi, const int16_t *x16, __m256i rmask,
             float *yr, float *yi, float *Xr, float *Xi)
{
    alignas(32) __m256 vr[64], vi[64];
    for (int g = 0; g < 8; g++, twA += 64 * 16) {   // A: columns 8 g .. 8 g + 7
        for (int n1 = 0; n1 < 64; n1++) {
            if (I16) {
                load_i16(x16 + 2 * (64 * n1 + 8 * g), rmask, vr[n1], vi[n1]);
            } else {
                vr[n1] = _mm256_loadu_ps(xr + 64 * n1 + 8 * g);
                vi[n1] = _mm256_loadu_ps(xi + 64 * n1 + 8 * g);
            }
        }
        fft64_vec<SIGN>(vr, vi, tw);
        for (int k1 = 0; k1 < 64; k1++) {
            __m256 r = vr[pos64(k1)], i = vi[pos64(k1)];
            if (k1) cmul<SIGN>(r, i, _mm256_loadu_ps(twA + 16 * k1), _mm256_loadu_ps(twA + 16 * k1 + 8));
            _mm256_storeu_ps(yr + 64 * k1 + 8 * g, r);
            _mm256_storeu_ps(yi + 64 * k1 + 8 * g, i);
        }
    }
    for (int h = 0; h < 8; h++) {   // B: rows k1 = 8 h .. 8 h + 7
        for (int b = 0; b < 8; b++) {
            for (int l = 0; l < 8; l++) {
                vr[8 * b + l] = _mm256_loadu_ps(yr + 64 * (8 * h + l) + 8 * b);
                vi[8 * b + l] = _mm256_loadu_ps(yi + 64 * (8 * h + l) + 8 * b);
            }
            transpose8(vr + 8 * b);   // vr[8 b + j] = column n2 = 8 b + j, lanes = rows
            transpose8(vi + 8 * b);
        }
        fft64_vec<SIGN>(vr, vi, tw);
        for (int k2 = 0; k2 < 64; k2++) {
            _mm256_storeu_ps(Xr + 64 * k2 + 8 * h, vr[pos64(k2)]);
            _mm256_storeu_ps(Xi + 64 * k2 + 8 * h, vi[pos64(k2)]);
        }
    }
}

// the final radix-2 pass of n = 2 * 4^k (L = 2, m = 1, s = n / 2)
void pass2(int n, const float *sr, const float *si, float *dr, float *di)
{
    const int s = n / 2;
    for (int q = 0; q < s; q += 8) {
        const __m256 ar = _mm256_loadu_ps(sr + q), ai = _mm256_loadu_ps(si + q);
        const __m256 br = _mm256_loadu_ps(sr + q + s), bi = _mm256_loadu_ps(si + q + s);
        _mm256_storeu_ps(dr + q, _mm256_add_ps(ar, br));
        _mm256_storeu_ps(di + q, _mm256_add_ps(ai, bi));
        _mm256_storeu_ps(dr + q + s, _mm256_sub_ps(ar, br));
        _mm256_storeu_ps(di + q + s, _mm256_sub_ps(ai, bi));
    }
}

}  // namespace

FftPlan::FftPlan(int n) : n_(n)
{
    if (n < 32 || n > 8192 || (n & (n - 1)) != 0) throw std::invalid_argument("FftPlan: n must be 2^k in [32, 8192]");
    auto w = [](long num, long den, float *re, float *im) {   // e^{-2 pi i num / den}
        const double a = -2.0 * M_PI * (double)num / (double)den;
        *re = (float)std::cos(a);
        *im = (float)std::sin(a);
    };
    if (n == 4096) {   // four-step: [twA 8192 floats | FFT-64 table 96 + 24 floats]
        tw_.resize(8192 + 120);
        for (int g = 0; g < 8; g++)
            for (int k1 = 0; k1 < 64; k1++)
                for (int l = 0; l < 8; l++) {
                    float *t = tw_.data() + (size_t)(g * 64 + k1) * 16;
                    w((long)(8 * g + l) * k1, 4096, &t[l], &t[8 + l]);
                }
        float *t = tw_.data() + 8192;
        for (int p = 0; p < 16; p++)
            for (int k = 1; k < 4; k++) w((long)p * k, 64, &t[6 * p + 2 * (k - 1)], &t[6 * p + 2 * (k - 1) + 1]);
        for (int p = 0; p < 4; p++)
            for (int k = 1; k < 4; k++) w((long)p * k, 16, &t[96 + 6 * p + 2 * (k - 1)], &t[96 + 6 * p + 2 * (k - 1) + 1]);
        return;
    }
    int s = 1, len = n;
    for (; len >= 4; len /= 4, s *= 4) passes_.push_back({s, 4, 0});
    if (len == 2) passes_.push_back({s, 2, 0});
    for (Pass &ps : passes_) {
        if (ps.radix == 2) continue;
        ps.tw = tw_.size();
        const int L = n / ps.s, m = L / 4;
        if (ps.s == 1) {
            for (int p0 = 0; p0 < m; p0 += 8)
                for (int k = 1; k < 4; k++) {
                    float re[8], im[8];
                    for (int l = 0; l < 8; l++) w((long)(p0 + l) * k, L, &re[l], &im[l]);
                    tw_.insert(tw_.end(), re, re + 8);
                    tw_.insert(tw_.end(), im, im + 8);
                }
        } else if (ps.s == 4) {
            for (int p0 = 0; p0 < m; p0 += 2)
                for (int k = 1; k < 4; k++) {
                    float re[8], im[8];
                    for (int l = 0; l < 8; l++) w((long)(p0 + l / 4) * k, L, &re[l], &im[l]);
                    tw_.insert(tw_.end(), re, re + 8);
                    tw_.insert(tw_.end(), im, im + 8);
                }
        } else {
            for (int p = 0; p < m; p++)
                for (int k = 1; k < 4; k++) {
                    float re, im;
                    w((long)p * k, L, &re, &im);
                    tw_.push_back(re);
                    tw_.push_back(im);
                }
        }
    }
}

template <int SIGN>
int FftPlan::run(float *re, float *im, float *wre, float *wim, const int16_t *x, bool rand) const
{
    const __m256i rmask = rand ? _mm256_set1_epi16(-1) : _mm256_setzero_si256();
    if (n_ == 4096) {   // input (re, im) or x, Y in (wre, wim), result in (re, im)
        if (x)
            fft4096<SIGN, true>(tw_.data(), tw_.data() + 8192, nullptr, nullptr, x, rmask, wre, wim, re, im);
        else
            fft4096<SIGN, false>(tw_.data(), tw_.data() + 8192, re, im, nullptr, rmask, wre, wim, re, im);
        return 0;
    }
    float *sr = re, *si = im, *dr = wre, *di = wim;
    int cur = 0;
    for (const Pass &ps : passes_) {
        const float *tw = tw_.data() + ps.tw;
        if (ps.radix == 2)
            pass2(n_, sr, si, dr, di);
        else if (ps.s == 1 && x)
            pass4_s1<SIGN, true>(n_, tw, nullptr, nullptr, x, rmask, dr, di);
        else if (ps.s == 1)
            pass4_s1<SIGN, false>(n_, tw, sr, si, nullptr, rmask, dr, di);
        else if (ps.s == 4)
            pass4_s4<SIGN>(n_, tw, sr, si, dr, di);
        else
            pass4_sN<SIGN>(n_, ps.s, tw, sr, si, dr, di);
        std::swap(sr, dr);
        std::swap(si, di);
        cur ^= 1;
    }
    return cur;
}

template int FftPlan::run<-1>(float *, float *, float *, float *, const int16_t *, bool) const;
template int FftPlan::run<+1>(float *, float *, float *, float *, const int16_t *, bool) const;

}  // namespace cpu
}  // namespace sddc
