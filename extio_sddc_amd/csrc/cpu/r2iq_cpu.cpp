// r2iq_cpu.cpp — the CPU r2iq backend (r2iq_cpu.h), AVX2 + FMA.
//
// Built with -ffp-contract=off: every fused multiply-add below is an explicit intrinsic, and
// the fine-tune NCO's scalar mix keeps pf_mixer's float operation order (fine_tune.h), so
// its output is bit-identical to the GPU output stage's.
#include "r2iq_cpu.h"

#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>

namespace sddc {
namespace cpu {
namespace {

constexpr int kHalf = 4096;     // halfFft           fft_mt_r2iq.h:18
constexpr int kBlock = 65536;   // transferSamples   config.h:80-81
constexpr int kHop = 6144;      // 3 halfFft / 2     impl.hpp:88
constexpr int kFrames = 11;     // fftPerBuf         fft_mt_r2iq.h:19

template <class T>
struct Aligned {
    T *p = nullptr;
    explicit Aligned(size_t n)
    {
        p = static_cast<T *>(std::aligned_alloc(64, ((n * sizeof(T) + 63) / 64) * 64));
        if (!p) throw std::bad_alloc();
        std::memset(p, 0, n * sizeof(T));
    }
    ~Aligned() { std::free(p); }
    Aligned(const Aligned &) = delete;
    Aligned &operator=(const Aligned &) = delete;
};

// 8 lanes reversed
inline __m256 reverse8(__m256 v) { return _mm256_permutevar8x32_ps(v, _mm256_setr_epi32(7, 6, 5, 4, 3, 2, 1, 0)); }

}  // namespace

bool supported()
{
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
}

struct R2iq::Buf {
    Aligned<int16_t> hist{kHalf}, frame0{2 * kHalf};
    // Z = forward output (+ Z[4096] = Z[0], so the mirror index 4096 - j needs no wrap)
    Aligned<float> ar{kHalf + 8}, ai{kHalf + 8}, br{kHalf + 8}, bi{kHalf + 8};
    Aligned<float> pr{kHalf}, pi{kHalf}, qr{kHalf}, qi{kHalf};
    Aligned<float> stage{(size_t)2 * 8 * kHalf};   // one block of CF32 output (NCO / CS16 path)
};

R2iq::R2iq(const std::complex<double> *H) : b_(new Buf), fwd_(kHalf), H_(H, H + 7 * kHalf)
{
    for (int d = 0; d < 7; d++) inv_.emplace_back(new FftPlan(kHalf >> d));
}

R2iq::~R2iq() = default;

void R2iq::reset() { std::memset(b_->hist.p, 0, kHalf * sizeof(int16_t)); }

void R2iq::set_history(const int16_t *last) { std::memcpy(b_->hist.p, last, kHalf * sizeof(int16_t)); }

// (P, Q) of (d, tb): the split x filter coefficients of every inverse-input bin m, and the
// two valid m ranges of the reference's shift with zero fill (impl.hpp:76-96):
//   [0, count)            j = tb + m,          count = min(mfft/2, 4096 - tb)
//   [mfft/2 + start, mfft) j = tb - mfft + m,  start = max(0, mfft/2 - tb)
void R2iq::build_pq(int d, int tb)
{
    if (d == pq_d_ && tb == pq_tb_) return;
    const int mfft = kHalf >> d, half = mfft / 2;
    const int count = std::min(half, kHalf - tb), start = std::max(0, half - tb);
    lo_ = count;
    hi_ = half + start;
    const std::complex<double> *Hd = H_.data() + (size_t)d * kHalf;
    for (int m = 0; m < mfft; m++) {
        const bool ok = m < count || m >= half + start;
        std::complex<double> P = 0, Q = 0;
        if (ok) {
            const int j = m < half ? tb + m : tb - mfft + m;
            const std::complex<double> h = 0.5 * Hd[m < half ? m : kHalf - mfft + m];   // filter2, impl.hpp:7
            const double a = -2.0 * M_PI * j / (2.0 * kHalf);
            const std::complex<double> iw(-std::sin(a), std::cos(a));                  // i W_8192^j
            P = h * (1.0 - iw);
            Q = h * (1.0 + iw);
        }
        b_->pr.p[m] = (float)P.real();
        b_->pi.p[m] = (float)P.imag();
        b_->qr.p[m] = (float)Q.real();
        b_->qi.p[m] = (float)Q.imag();
    }
    pq_d_ = d;
    pq_tb_ = tb;
}

// One 8192-sample frame x -> y = IFFT_mfft(T) (mfft = 4096 >> d); *yr, *yi point at y
// (in the work buffers, valid until the next frame).
void R2iq::frame(const int16_t *x, int d, bool rand, const float **yr, const float **yi)
{
    Buf &B = *b_;
    // ---- Z = FFT4096 of x[2n] + i x[2n+1] (the r2c 8192 before its split, impl.hpp:88), the
    // int16 -> float conversion (+ rand, fft_mt_r2iq.h:36-51) done by the first pass ----
    float *zr = B.ar.p, *zi = B.ai.p;
    if (fwd_.forward_i16(x, rand, B.ar.p, B.ai.p, B.br.p, B.bi.p)) {
        zr = B.br.p;
        zi = B.bi.p;
    }
    zr[kHalf] = zr[0];
    zi[kHalf] = zi[0];
    // ---- T[m] = Z_j P[m] + conj(Z_-j) Q[m] on the two valid ranges, 0 elsewhere ----
    const int mfft = kHalf >> d;
    float *tr = zr == B.ar.p ? B.br.p : B.ar.p, *ti = zr == B.ar.p ? B.bi.p : B.ai.p;
    const int tb = pq_tb_;
    auto run = [&](int m0, int m1, int joff) {   // j = m + joff
        int m = m0;
        for (; m + 8 <= m1; m += 8) {
            const int j = m + joff;
            const __m256 ajr = _mm256_loadu_ps(zr + j), aji = _mm256_loadu_ps(zi + j);
            const __m256 bmr = reverse8(_mm256_loadu_ps(zr + kHalf - j - 7));
            const __m256 bmi = reverse8(_mm256_loadu_ps(zi + kHalf - j - 7));
            const __m256 Pr = _mm256_loadu_ps(B.pr.p + m), Pi = _mm256_loadu_ps(B.pi.p + m);
            const __m256 Qr = _mm256_loadu_ps(B.qr.p + m), Qi = _mm256_loadu_ps(B.qi.p + m);
            // Re = ajr Pr - aji Pi + bmr Qr + bmi Qi;  Im = ajr Pi + aji Pr + bmr Qi - bmi Qr
            __m256 re = _mm256_mul_ps(ajr, Pr);
            re = _mm256_fnmadd_ps(aji, Pi, re);
            re = _mm256_fmadd_ps(bmr, Qr, re);
            re = _mm256_fmadd_ps(bmi, Qi, re);
            __m256 im = _mm256_mul_ps(ajr, Pi);
            im = _mm256_fmadd_ps(aji, Pr, im);
            im = _mm256_fmadd_ps(bmr, Qi, im);
            im = _mm256_fnmadd_ps(bmi, Qr, im);
            _mm256_storeu_ps(tr + m, re);
            _mm256_storeu_ps(ti + m, im);
        }
        for (; m < m1; m++) {
            const int j = m + joff;
            const float a_r = zr[j], a_i = zi[j], b_r = zr[kHalf - j], b_i = zi[kHalf - j];
            const float *P_r = B.pr.p, *P_i = B.pi.p, *Q_r = B.qr.p, *Q_i = B.qi.p;
            tr[m] = a_r * P_r[m] - a_i * P_i[m] + b_r * Q_r[m] + b_i * Q_i[m];
            ti[m] = a_r * P_i[m] + a_i * P_r[m] + b_r * Q_i[m] - b_i * Q_r[m];
        }
    };
    run(0, lo_, tb);
    std::memset(tr + lo_, 0, (size_t)(hi_ - lo_) * sizeof(float));
    std::memset(ti + lo_, 0, (size_t)(hi_ - lo_) * sizeof(float));
    run(hi_, mfft, tb - mfft);
    // ---- y = IFFT_mfft(T) (impl.hpp:98) ----
    float *wr = tr == B.ar.p ? B.br.p : B.ar.p, *wi = tr == B.ar.p ? B.bi.p : B.ai.p;
    const bool w = inv_[d]->backward(tr, ti, wr, wi) != 0;
    *yr = w ? wr : tr;
    *yi = w ? wi : ti;
}

void R2iq::process(const int16_t *const *blocks, int nblk, void *out, const Params &p)
{
    Buf &B = *b_;
    const int d = p.d, mfft = kHalf >> d, half = mfft / 2, keep = 3 * mfft / 4;
    build_pq(d, p.tunebin);
    const bool post = p.cs16 || p.nco_trig;
    const size_t per_blk = (size_t)8 * mfft;   // complex outputs per block
    const __m256 sgn = _mm256_castsi256_ps(_mm256_set1_epi32(p.lsb ? (int)0x80000000 : 0));
    for (int b = 0; b < nblk; b++) {
        const int16_t *blk = blocks[b];
        float *o = post ? B.stage.p : static_cast<float *>(out) + 2 * per_blk * b;
        for (int k = 0; k < kFrames; k++) {
            const int16_t *x;
            if (k == 0) {   // [history | block[0, 4096)]
                std::memcpy(B.frame0.p, B.hist.p, kHalf * sizeof(int16_t));
                std::memcpy(B.frame0.p + kHalf, blk, kHalf * sizeof(int16_t));
                x = B.frame0.p;
            } else {
                x = blk + kHop * k - kHalf;
            }
            const float *yr, *yi;
            frame(x, d, p.rand, &yr, &yi);
            // ---- overlap-discard + sideband (impl.hpp:117-138, fft_mt_r2iq.h:63-81) ----
            const int i0 = k == 0 ? mfft / 4 : 0, n = k == 0 ? half : keep;
            float *dst = o + 2 * (k == 0 ? 0 : half + (size_t)keep * (k - 1));
            for (int i = 0; i < n; i += 8) {
                const __m256 re = _mm256_loadu_ps(yr + i0 + i);
                const __m256 im = _mm256_xor_ps(_mm256_loadu_ps(yi + i0 + i), sgn);
                const __m256 lo = _mm256_unpacklo_ps(re, im), hi = _mm256_unpackhi_ps(re, im);
                _mm256_storeu_ps(dst + 2 * i, _mm256_permute2f128_ps(lo, hi, 0x20));
                _mm256_storeu_ps(dst + 2 * i + 8, _mm256_permute2f128_ps(lo, hi, 0x31));
            }
        }
        std::memcpy(B.hist.p, blk + kBlock - kHalf, kHalf * sizeof(int16_t));
        if (!post) continue;
        // ---- fused fine-tune NCO (pf_mixer.cpp:808-833 order) and CS16 ----
        float *s = B.stage.p;
        if (p.nco_trig) {
            for (size_t i = 0; i < per_blk; i++) {
                const size_t ot = per_blk * b + i;   // sample index in this call's output
                const float *sb = p.nco_starts + 2 * ((ot >> 7) * 4 + (ot & 3));
                const int q = (int)((ot >> 2) & 31);
                float px = sb[0], py = sb[1];
                if (q) {
                    const float *tq = p.nco_trig + 2 * (q - 1);
                    px = tq[0] * sb[0] - tq[1] * sb[1];
                    py = tq[1] * sb[0] + tq[0] * sb[1];
                }
                const float vx = s[2 * i], vy = s[2 * i + 1];
                s[2 * i] = vx * px - vy * py;
                s[2 * i + 1] = vy * px + vx * py;
            }
        }
        if (p.cs16) {
            int16_t *c = static_cast<int16_t *>(out) + 2 * per_blk * b;
            for (size_t i = 0; i < 2 * per_blk; i++) {
                float v = std::nearbyint(s[i] * p.scale);   // round half even (default mode)
                v = std::min(std::max(v, -32768.f), 32767.f);
                c[i] = (int16_t)v;
            }
        } else {
            std::memcpy(static_cast<float *>(out) + 2 * per_blk * b, s, 2 * per_blk * sizeof(float));
        }
    }
}

}  // namespace cpu
}  // namespace sddc
