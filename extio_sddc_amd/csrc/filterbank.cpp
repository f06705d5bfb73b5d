// filterbank.cpp — init-time filter design for the DDC (host side).
//
// Restates the reference's Kaiser-windowed sinc low-pass (Core/fir.cpp:7-105)
// and the per-decimation filter bank (Core/fft_mt_r2iq.cpp:163-208).  The Kaiser
// arithmetic keeps fir.cpp's float operation order so the taps are bit-identical
// (tests/test_capi_cpu.py pins them, through the C ABI, to the reference's own fir.cpp built in
// oracle/_ref and the committed fixture tests/golden/kaiser_taps.json).  Compile
// with -ffp-contract=off.  H_d = FFT4096 of the taps is evaluated in double here
// (the reference does it with a float FFTW plan) and rounded once to float.
#include <cmath>
#include <complex>
#include <cstring>
#include <vector>

#include "filterbank.h"

namespace sddc {

namespace {

constexpr float kPi = 3.141592653f;      // K_PI, fir.cpp:4
constexpr float kTwoPi = 2 * kPi;        // K_2PI, fir.cpp:5

// zeroth-order modified Bessel function, power series (fir.cpp:7-25)
float bessel_i0(float x)
{
    const float h = x / 2.0f;
    float sum = 1.0f;
    float term = 1.0f;
    float k = 1.0f;
    do {
        float r = h / k;
        r *= r;
        term *= r;
        sum += term;
        k += 1.0;
    } while (term >= 1e-9f * sum);
    return sum;
}

void fft_inplace(std::vector<std::complex<double>> &a, int sign)
{
    const size_t n = a.size();
    for (size_t i = 1, j = 0; i < n; i++) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        for (size_t i = 0; i < n; i += len) {
            for (size_t k = 0; k < len / 2; k++) {
                const double th = sign * 2.0 * M_PI * (double)k / (double)len;
                const std::complex<double> w(std::cos(th), std::sin(th));
                const std::complex<double> u = a[i + k], v = a[i + k + len / 2] * w;
                a[i + k] = u + v;
                a[i + k + len / 2] = u - v;
            }
        }
    }
}

}  // namespace

int kaiser_window(int num_taps, float astop, float fpass, float fstop, float *coef)
{
    const float fcut = (fstop + fpass) / 2.0f;
    float beta = 0.0f;
    if (astop >= 50.0f)
        beta = .1102f * (astop - 8.71f);
    else if (astop >= 20.96f)
        beta = .5842f * powf((astop - 20.96f), 0.4f) + .07886f * (astop - 20.96f);

    int taps = (int)((astop - 8.0) / (2.285 * kTwoPi * (fstop - fpass)) + 1);
    if (num_taps < 0 && taps > -num_taps) taps = -num_taps;
    if (taps < 3) taps = 3;
    if (num_taps <= 0 && coef == nullptr) return taps;
    if (num_taps > 0) taps = num_taps;

    const float mid = .5f * (float)(taps - 1);
    const float norm = bessel_i0(beta);
    for (int n = 0; n < taps; n++) {
        const float off = (float)n - mid;
        const float ideal = ((float)n == mid) ? 2.0f * fcut
                                              : (float)sinf(kTwoPi * off * fcut) / (kPi * off);
        const float u = ((float)n - ((float)taps - 1.0f) / 2.0f) / (((float)taps - 1.0f) / 2.0f);
        coef[n] = 1.0f * ideal * bessel_i0(beta * sqrtf(1 - (u * u))) / norm;
    }
    return taps;
}

void filter_taps(int d, float *taps)
{
    // Bw = 64 / mratio[d]; fpass = 0.85 Bw/128, fstop = 1.1 Bw/128 (fft_mt_r2iq.cpp:182-191)
    const float bw = 64.0f / (float)(1 << d);
    kaiser_window(kNumTaps, 120.0f, 0.85f * bw / 128.0f, 1.1f * bw / 128.0f, taps);
}

void filter_response(float gain, int d, std::complex<double> *H)
{
    float taps[kNumTaps];
    filter_taps(d, taps);
    const float g = gain * 2048.0f / (float)kFftN;   // gainadj, fft_mt_r2iq.cpp:193
    std::vector<std::complex<double>> h(kHalfFft, 0.0);
    for (int t = 0; t < kNumTaps; t++) h[kHalfFft - 1 - t] = (double)(g * taps[t]);
    fft_inplace(h, -1);
    for (int i = 0; i < kHalfFft; i++) H[i] = h[i];
}

}  // namespace sddc
