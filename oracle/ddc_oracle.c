/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product (extio_sddc_amd/).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / the timed
 * CPU baseline.
 *
 * CPU restatement of the ExtIO_sddc real-to-IQ hot path (SURVEY.md §8(a) rows
 * a2-a7, a5, a9).  Every function cites the reference file:line it restates
 * (paths relative to the reference tree, Core/...).
 *
 * Parity pinning:
 *   - a5 (Kaiser filter design) is pinned BIT-EXACT against the reference's own
 *     Core/fir.cpp compiled from /root/reference into oracle/_ref/ (tests/
 *     test_oracle.py, and the committed fixture tests/golden/kaiser_taps.json).
 *   - a2-a4, a6, a7 (convert, r2c, shift*filter, inverse c2c, overlap-discard)
 *     are restated from the reference sources; the reference's own build of
 *     this path is unbuildable here (it needs <fftw3.h>, which this image lacks)
 *     and its tests hold no IQ golden vectors, so IQ-level parity against the
 *     reference binary is UNPINNED.  The FFTs are pinned to the DFT definition
 *     (numpy float64 cross-check) and the pipeline to the reference tests'
 *     assertions (core_test.cpp:167 block length; signal_integrity_test.cpp
 *     properties), re-asserted in tests/test_oracle.py.
 *
 * Two instantiations of the same restatement:
 *   *_f64 : double arithmetic end to end (the parity checker: the exact
 *           answer the reference's float FFTW path approximates);
 *   *_f32 : float arithmetic like the reference (the CPU baseline "port").
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_HALF_FFT 4096          /* halfFft = FFTN_R_ADC/2      fft_mt_r2iq.h:18, config.h:49 */
#define OR_FFTN     8192          /* FFTN_R_ADC                  config.h:49 */
#define OR_HOP      6144          /* 3*halfFft/2                 fft_mt_r2iq_impl.hpp:88 */
#define OR_BLOCK    65536         /* transferSamples             config.h:80-81 */
#define OR_FRAMES   11            /* fftPerBuf                   fft_mt_r2iq.h:19 */
#define OR_NDEC     7             /* NDECIDX                     r2iq.h:5 */
#define OR_NTAPS    (OR_HALF_FFT / 4 + 1)   /* 1025              fft_mt_r2iq.cpp:181,191 */

#define OR_PI_F   3.141592653f    /* K_PI                        fir.cpp:4 */
#define OR_2PI_F  (2 * OR_PI_F)   /* K_2PI                       fir.cpp:5 */

/* ------------------------------------------------------------------------- */
/* a5: filter design.  Restates fir.cpp with identical float operation order   */
/* so results are bit-identical (build with -ffp-contract=off).               */
/* ------------------------------------------------------------------------- */

/* Modified Bessel I0 by its power series; fir.cpp:7-25. */
static float or_bessel_i0(float x)
{
    const float half = x / 2.0f;
    float acc = 1.0f, term = 1.0f, k = 1.0f;
    for (;;) {
        float q = half / k;
        q *= q;
        term *= q;
        acc += term;
        k += 1.0;                         /* double add, as fir.cpp:21 */
        if (!(term >= 1e-9f * acc)) break;
    }
    return acc;
}

/* Kaiser-windowed sinc low-pass; fir.cpp:48-105.  Returns the tap count. */
int oracle_kaiser(int ntaps, float astop, float fpass, float fstop, float *coef)
{
    const float fcut = (fstop + fpass) / 2.0f;
    float beta;
    if (astop < 20.96f)
        beta = 0.0f;
    else if (astop >= 50.0f)
        beta = .1102f * (astop - 8.71f);
    else
        beta = .5842f * powf((astop - 20.96f), 0.4f) + .07886f * (astop - 20.96f);

    int n_est = (int)((astop - 8.0) / (2.285 * OR_2PI_F * (fstop - fpass)) + 1);
    if (ntaps < 0 && n_est > -ntaps) n_est = -ntaps;
    if (n_est < 3) n_est = 3;
    if (ntaps <= 0 && !coef) return n_est;
    const int n_taps = ntaps > 0 ? ntaps : n_est;

    const float centre = .5f * (float)(n_taps - 1);
    const float i0_beta = or_bessel_i0(beta);
    for (int n = 0; n < n_taps; n++) {
        const float t = (float)n - centre;
        float sinc;
        if ((float)n == centre)
            sinc = 2.0f * fcut;
        else
            sinc = (float)sinf(OR_2PI_F * t * fcut) / (OR_PI_F * t);
        const float u = ((float)n - ((float)n_taps - 1.0f) / 2.0f) / (((float)n_taps - 1.0f) / 2.0f);
        coef[n] = 1.0f * sinc * or_bessel_i0(beta * sqrtf(1 - (u * u))) / i0_beta;
    }
    return n_taps;
}

/* The taps used for decimation index d; fft_mt_r2iq.cpp:181-191. */
void oracle_filter_taps(int d, float *pht)
{
    const float bw = 64.0f / (float)(1 << d);           /* mratio[d] = 2^d, fft_mt_r2iq.cpp:32-36 */
    oracle_kaiser(OR_NTAPS, 120.0f, 0.85f * bw / 128.0f, 1.1f * bw / 128.0f, pht);
}

/* ------------------------------------------------------------------------- */
/* FFT: unnormalised complex DFT, Stockham radix-4 (+ one radix-2 pass).      */
/* sign = -1 forward (FFTW_FORWARD), +1 backward (FFTW_BACKWARD).              */
/* ------------------------------------------------------------------------- */
/* Twiddle tables e^{-2 pi i k/n}, k < n, computed in double; one per size,  */
/* built on first use (call oracle_init() before using from several threads). */
#define OR_MAXLOG 14
static double *or_tab64[OR_MAXLOG + 1];
static float  *or_tab32[OR_MAXLOG + 1];

static int or_log2(int n) { int l = 0; while ((1 << l) < n) l++; return l; }

static const double *or_table_f64(int n)
{
    int l = or_log2(n);
    if (!or_tab64[l]) {
        double *t = (double *)malloc(sizeof(double) * 2 * (size_t)n);
        for (int k = 0; k < n; k++) {
            double th = -2.0 * M_PI * (double)k / (double)n;
            t[2 * k] = cos(th); t[2 * k + 1] = sin(th);
        }
        or_tab64[l] = t;
    }
    return or_tab64[l];
}

static const float *or_table_f32(int n)
{
    int l = or_log2(n);
    if (!or_tab32[l]) {
        const double *d = or_table_f64(n);
        float *t = (float *)malloc(sizeof(float) * 2 * (size_t)n);
        for (int k = 0; k < 2 * n; k++) t[k] = (float)d[k];
        or_tab32[l] = t;
    }
    return or_tab32[l];
}

void oracle_init(void)
{
    for (int l = 1; l <= 13; l++) { or_table_f64(1 << l); or_table_f32(1 << l); }
}

#define OR_DEFINE_FFT(T, SUF)                                                     \
static void or_fft_##SUF(T *x, T *y, int n, int sign)                            \
{                                                                                \
    /* x,y: interleaved complex, n points; result in x. */                       \
    const T *tab = or_table_##SUF(n);                                            \
    const T ws = (T)(-sign);       /* imag sign: table holds e^{-i...} */        \
    T *src = x, *dst = y;                                                        \
    int s = 1, n0 = n;                                                           \
    for (; n0 >= 4; n0 /= 4, s *= 4) {                                           \
        const int m = n0 / 4;                                                    \
        for (int p = 0; p < m; p++) {                                            \
            const T w1r = tab[2 * (p * s)],     w1i = ws * tab[2 * (p * s) + 1];     \
            const T w2r = tab[2 * (2 * p * s)], w2i = ws * tab[2 * (2 * p * s) + 1]; \
            const T w3r = tab[2 * (3 * p * s)], w3i = ws * tab[2 * (3 * p * s) + 1]; \
            const T *a = src + 2 * (s * p);                                      \
            const T *b = src + 2 * (s * (p + m));                                \
            const T *c = src + 2 * (s * (p + 2 * m));                            \
            const T *d = src + 2 * (s * (p + 3 * m));                            \
            T *o = dst + 2 * (s * 4 * p);                                        \
            for (int q = 0; q < s; q++) {                                        \
                T apcr = a[2*q] + c[2*q], apci = a[2*q+1] + c[2*q+1];            \
                T amcr = a[2*q] - c[2*q], amci = a[2*q+1] - c[2*q+1];            \
                T bpdr = b[2*q] + d[2*q], bpdi = b[2*q+1] + d[2*q+1];            \
                T bmdr = b[2*q] - d[2*q], bmdi = b[2*q+1] - d[2*q+1];            \
                /* j = sign*i applied to (b-d) */                                \
                T jr = -(T)sign * bmdi, ji = (T)sign * bmdr;                     \
                T r1r = amcr + jr, r1i = amci + ji;                              \
                T r2r = apcr - bpdr, r2i = apci - bpdi;                          \
                T r3r = amcr - jr, r3i = amci - ji;                              \
                o[2*q] = apcr + bpdr; o[2*q+1] = apci + bpdi;                    \
                o[2*(q+s)] = r1r * w1r - r1i * w1i; o[2*(q+s)+1] = r1r * w1i + r1i * w1r;         \
                o[2*(q+2*s)] = r2r * w2r - r2i * w2i; o[2*(q+2*s)+1] = r2r * w2i + r2i * w2r;     \
                o[2*(q+3*s)] = r3r * w3r - r3i * w3i; o[2*(q+3*s)+1] = r3r * w3i + r3i * w3r;     \
            }                                                                    \
        }                                                                        \
        T *t = src; src = dst; dst = t;                                          \
    }                                                                            \
    if (n0 == 2) {                                                               \
        for (int q = 0; q < s; q++) {                                            \
            const T *a = src + 2 * q, *b = src + 2 * (q + s);                    \
            T *o0 = dst + 2 * q, *o1 = dst + 2 * (q + s);                        \
            T ar = a[0], ai = a[1], br = b[0], bi = b[1];                        \
            o0[0] = ar + br; o0[1] = ai + bi; o1[0] = ar - br; o1[1] = ai - bi;  \
        }                                                                        \
        T *t = src; src = dst; dst = t;                                          \
    }                                                                            \
    if (src != x) memcpy(x, src, sizeof(T) * 2 * (size_t)n);                     \
}

OR_DEFINE_FFT(double, f64)
OR_DEFINE_FFT(float, f32)

void oracle_fft_c64(double *x, int n, int sign)
{
    double *w = (double *)malloc(sizeof(double) * 2 * (size_t)n);
    or_fft_f64(x, w, n, sign);
    free(w);
}

/* H_d = FFT_4096^fwd(ht),  ht[4095-t] = gain*2048/8192*pht[t];                */
/* fft_mt_r2iq.cpp:173-206.  Output H[d][4096] interleaved (re,im), double.    */
void oracle_filter_bank_f64(float gain, double *H)
{
    float pht[OR_NTAPS];
    double *work = (double *)malloc(sizeof(double) * 2 * OR_HALF_FFT);
    const float gainadj = gain * 2048.0f / (float)OR_FFTN;          /* fft_mt_r2iq.cpp:193 */
    for (int d = 0; d < OR_NDEC; d++) {
        double *h = H + (size_t)d * 2 * OR_HALF_FFT;
        oracle_filter_taps(d, pht);
        memset(h, 0, sizeof(double) * 2 * OR_HALF_FFT);
        for (int t = 0; t < OR_NTAPS; t++)
            h[2 * (OR_HALF_FFT - 1 - t)] = (double)(gainadj * pht[t]); /* float product, as :202 */
        or_fft_f64(h, work, OR_HALF_FFT, -1);
    }
    free(work);
}

/* ------------------------------------------------------------------------- */
/* a2: convert_float<rand>  fft_mt_r2iq.h:36-51                                */
/* ------------------------------------------------------------------------- */
static inline int or_derand(int16_t v, int rand)
{
    return (rand && (v & 1)) ? (int16_t)(v ^ (-2)) : v;
}

/* a9: setFreqOffset  fft_mt_r2iq.cpp:101-109.  Returns the residual fc. */
float oracle_set_freq_offset(float offset, int d, int *tunebin)
{
    const int tb = (int)(offset * OR_HALF_FFT / 4) * 4;
    const float delta = ((float)tb / OR_HALF_FFT) - offset;
    *tunebin = tb;
    return delta * (float)(1 << d);
}

/* ------------------------------------------------------------------------- */
/* a2-a7 for nblk consecutive blocks.                                          */
/*   in  : 4096 history samples followed by nblk*65536 samples (int16)        */
/*   out : nblk * 8*mfft complex samples, interleaved (I,Q)                   */
/* Block b's time buffer is in[65536b, 65536b+69632): the history is the tail */
/* of block b-1 (impl.hpp:32 peekReadPtr(-1)+transferSamples-halfFft).        */
/* ------------------------------------------------------------------------- */
#define OR_DEFINE_R2IQ(T, SUF)                                                    \
int oracle_r2iq_##SUF(const T *Hd, int d, int tunebin, int lsb, int rand,        \
                      const int16_t *in, int nblk, T *out)                       \
{                                                                                \
    if (d < 0 || d >= OR_NDEC || tunebin < 0 || tunebin >= OR_HALF_FFT) return -1; \
    const int mfft = OR_HALF_FFT >> d;                   /* fft_mt_r2iq.cpp:44-48 */ \
    const int half = mfft / 2;                                                   \
    T *z    = (T *)malloc(sizeof(T) * 2 * OR_HALF_FFT);                          \
    T *X    = (T *)malloc(sizeof(T) * 2 * (OR_HALF_FFT + 1));                    \
    T *tmp  = (T *)malloc(sizeof(T) * 2 * OR_HALF_FFT);                          \
    T *work = (T *)malloc(sizeof(T) * 2 * OR_HALF_FFT);                          \
    const T *tw = or_table_##SUF(OR_FFTN);  /* e^{-2 pi i k / 8192} */          \
    /* impl.hpp:76-80 */                                                         \
    const int count = half < OR_HALF_FFT - tunebin ? half : OR_HALF_FFT - tunebin; \
    const int start = half - tunebin > 0 ? half - tunebin : 0;                   \
    const T *H2 = Hd + 2 * (OR_HALF_FFT - half);         /* impl.hpp:7 filter2 */ \
    for (int b = 0; b < nblk; b++) {                                             \
        const int16_t *tb = in + (size_t)b * OR_BLOCK;                           \
        T *pout = out + (size_t)b * 2 * 8 * mfft;         /* impl.hpp:118-122 */  \
        for (int k = 0; k < OR_FRAMES; k++) {                                    \
            const int16_t *fr = tb + OR_HOP * k;                                 \
            /* a3: r2c 8192 (impl.hpp:88) via the packed 4096-point transform */ \
            for (int n = 0; n < OR_HALF_FFT; n++) {                              \
                z[2 * n] = (T)or_derand(fr[2 * n], rand);                        \
                z[2 * n + 1] = (T)or_derand(fr[2 * n + 1], rand);                \
            }                                                                    \
            or_fft_##SUF(z, work, OR_HALF_FFT, -1);                              \
            for (int j = 0; j <= OR_HALF_FFT; j++) {                             \
                const int a = j & (OR_HALF_FFT - 1), c = (OR_HALF_FFT - j) & (OR_HALF_FFT - 1); \
                T zr = z[2 * a], zi = z[2 * a + 1], cr = z[2 * c], ci = -z[2 * c + 1]; \
                T er = (T)0.5 * (zr + cr), ei = (T)0.5 * (zi + ci);              \
                T dr = (T)0.5 * (zr - cr), di = (T)0.5 * (zi - ci);              \
                /* O = (Z - conj Z')/(2i) = (di, -dr) */                         \
                T or_ = di, oi = -dr;                                            \
                T wr, wi;                                                        \
                if (j < OR_HALF_FFT) { wr = tw[2 * j]; wi = tw[2 * j + 1]; }     \
                else { wr = (T)-1; wi = (T)0; }                                  \
                X[2 * j] = er + (or_ * wr - oi * wi);                            \
                X[2 * j + 1] = ei + (or_ * wi + oi * wr);                        \
            }                                                                    \
            /* a4: shift_freq + zero fill (impl.hpp:90-96; fft_mt_r2iq.h:53-61) */ \
            for (int m = 0; m < mfft; m++) { tmp[2 * m] = 0; tmp[2 * m + 1] = 0; } \
            for (int m = 0; m < count; m++) {                                    \
                const T *s = X + 2 * (tunebin + m), *h = Hd + 2 * m;             \
                tmp[2 * m] = s[0] * h[0] - s[1] * h[1];                          \
                tmp[2 * m + 1] = s[1] * h[0] + s[0] * h[1];                      \
            }                                                                    \
            for (int m = start; m < half; m++) {                                 \
                const T *s = X + 2 * (tunebin - half + m), *h = H2 + 2 * m;      \
                tmp[2 * (half + m)] = s[0] * h[0] - s[1] * h[1];                 \
                tmp[2 * (half + m) + 1] = s[1] * h[0] + s[0] * h[1];             \
            }                                                                    \
            /* a6: inverse c2c (impl.hpp:98) */                                  \
            or_fft_##SUF(tmp, work, mfft, +1);                                   \
            /* a7: overlap-discard + sideband copy (impl.hpp:124-138) */         \
            const T sg = lsb ? (T)-1 : (T)1;                                     \
            if (k == 0) {                                                        \
                for (int i = 0; i < half; i++) {                                 \
                    pout[2 * i] = tmp[2 * (mfft / 4 + i)];                       \
                    pout[2 * i + 1] = sg * tmp[2 * (mfft / 4 + i) + 1];          \
                }                                                                \
            } else {                                                             \
                T *po = pout + 2 * (half + (3 * mfft / 4) * (k - 1));            \
                for (int i = 0; i < 3 * mfft / 4; i++) {                         \
                    po[2 * i] = tmp[2 * i];                                      \
                    po[2 * i + 1] = sg * tmp[2 * i + 1];                         \
                }                                                                \
            }                                                                    \
        }                                                                        \
    }                                                                            \
    free(z); free(X); free(tmp); free(work);                           \
    return 0;                                                                    \
}

OR_DEFINE_R2IQ(double, f64)
OR_DEFINE_R2IQ(float, f32)

/* Float copy of the filter bank for the f32 port (H computed in double, then  */
/* rounded once — the reference computes it with a float FFTW c2c).           */
void oracle_filter_bank_f32(float gain, float *H)
{
    double *h = (double *)malloc(sizeof(double) * 2 * OR_HALF_FFT * OR_NDEC);
    oracle_filter_bank_f64(gain, h);
    for (int i = 0; i < 2 * OR_HALF_FFT * OR_NDEC; i++) H[i] = (float)h[i];
    free(h);
}

/* a3 alone, for stage tests: 8192 int16 -> 4097 bins (double). */
void oracle_forward_r2c_f64(const int16_t *frame, int rand, double *X)
{
    double *x = (double *)malloc(sizeof(double) * 2 * OR_FFTN);
    double *w = (double *)malloc(sizeof(double) * 2 * OR_FFTN);
    for (int n = 0; n < OR_FFTN; n++) { x[2 * n] = or_derand(frame[n], rand); x[2 * n + 1] = 0; }
    or_fft_f64(x, w, OR_FFTN, -1);
    memcpy(X, x, sizeof(double) * 2 * (OR_HALF_FFT + 1));
    free(x); free(w);
}

/* ------------------------------------------------------------------------------------------
 * Fine-tune NCO: restatement of ALGO H, the x86/SSE build of
 * shift_limited_unroll_C_sse_init / _inp_c (Core/pffft/pf_mixer.cpp:750-856), applied by
 * RadioHandlerClass::OnDataPacket to every 32768-sample output buffer when fc != 0
 * (Core/RadioHandler.cpp:33-37), with init(fc, 0) on every fc change (:291-296).
 * Four lanes (SIMD_SZ, pf_mixer.h:134) carry the phasors of samples 4j+lane; blocks of
 * 128 samples (UNROLL_SIZE, pf_mixer.h:133) multiply the lane starts by a table of
 * 4(j+1)-step phasors, and the starts are renormalised after every block.  Plain float
 * arithmetic in the SSE operation order (mul, mul, sub/add; sqrt; div), no fused ops.
 * ------------------------------------------------------------------------------------------ */
#define OR_NCO_LANES 4
#define OR_NCO_BLOCK 128
#define OR_NCO_PI ((float)3.14159265358979323846)          /* pf_mixer.cpp:40 */

typedef struct {
    float trig_c[OR_NCO_BLOCK / OR_NCO_LANES + 1];   /* dinterl_trig cos of entry i/4 */
    float trig_s[OR_NCO_BLOCK / OR_NCO_LANES + 1];   /* dinterl_trig sin */
    float start_c[OR_NCO_LANES], start_s[OR_NCO_LANES];   /* phase_state_i/q */
} oracle_nco_t;

/* pf_mixer.cpp:750-789 */
void oracle_nco_init(float relative_freq, float phase_start_rad, oracle_nco_t *d)
{
    const float inc = 2 * relative_freq * OR_NCO_PI;
    float ph = 0.0f;
    for (int e = 0; e <= OR_NCO_BLOCK / OR_NCO_LANES; e++) {
        for (int k = 0; k < OR_NCO_LANES; k++) {
            ph += inc;
            while (ph > OR_NCO_PI) ph -= 2 * OR_NCO_PI;
            while (ph < -OR_NCO_PI) ph += 2 * OR_NCO_PI;
        }
        d->trig_c[e] = cosf(ph);
        d->trig_s[e] = sinf(ph);
    }
    ph = phase_start_rad;
    for (int k = 0; k < OR_NCO_LANES; k++) {
        d->start_c[k] = cosf(ph);
        d->start_s[k] = sinf(ph);
        ph += inc;
        while (ph > OR_NCO_PI) ph -= 2 * OR_NCO_PI;
        while (ph < -OR_NCO_PI) ph += 2 * OR_NCO_PI;
    }
}

/* pf_mixer.cpp:791-856; iq = interleaved (I,Q) float, n_cplx a multiple of 4 */
void oracle_nco_apply(float *iq, int n_cplx, oracle_nco_t *d)
{
    float sc[OR_NCO_LANES], ss[OR_NCO_LANES], vc[OR_NCO_LANES], vs[OR_NCO_LANES];
    for (int k = 0; k < OR_NCO_LANES; k++) {
        sc[k] = vc[k] = d->start_c[k];
        ss[k] = vs[k] = d->start_s[k];
    }
    while (n_cplx) {
        const int nb = n_cplx >= OR_NCO_BLOCK ? OR_NCO_BLOCK : n_cplx;
        for (int j = 0; j < nb / OR_NCO_LANES; j++) {
            for (int k = 0; k < OR_NCO_LANES; k++) {
                float *p = iq + 2 * (OR_NCO_LANES * j + k);
                const float re = p[0], im = p[1];
                const float a = re * vc[k], b = im * vs[k];
                const float c = im * vc[k], e = re * vs[k];
                p[0] = a - b;
                p[1] = c + e;
            }
            for (int k = 0; k < OR_NCO_LANES; k++) {
                const float tr = d->trig_c[j], ti = d->trig_s[j];
                const float a = tr * sc[k], b = ti * ss[k];
                const float c = ti * sc[k], e = tr * ss[k];
                vc[k] = a - b;
                vs[k] = c + e;
            }
        }
        iq += 2 * nb;
        n_cplx -= nb;
        for (int k = 0; k < OR_NCO_LANES; k++) {
            const float m2 = vc[k] * vc[k] + vs[k] * vs[k];
            const float m = sqrtf(m2);
            sc[k] = vc[k] = vc[k] / m;
            ss[k] = vs[k] = vs[k] / m;
        }
    }
    for (int k = 0; k < OR_NCO_LANES; k++) {
        d->start_c[k] = sc[k];
        d->start_s[k] = ss[k];
    }
}

int oracle_nco_state_size(void) { return (int)sizeof(oracle_nco_t); }
