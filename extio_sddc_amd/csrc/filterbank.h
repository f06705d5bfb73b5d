// filterbank.h — host-side filter design (see filterbank.cpp).
#pragma once

#include <complex>

namespace sddc {

constexpr int kHalfFft = 4096;          // halfFft          fft_mt_r2iq.h:18
constexpr int kFftN = 8192;             // FFTN_R_ADC       config.h:49
constexpr int kNumTaps = kHalfFft / 4 + 1;  // 1025         fft_mt_r2iq.cpp:181
constexpr int kNumDec = 7;              // NDECIDX          r2iq.h:5

int kaiser_window(int num_taps, float astop, float fpass, float fstop, float *coef);
void filter_taps(int d, float *taps);
void filter_response(float gain, int d, std::complex<double> *H /* [4096] */);

}  // namespace sddc
