// fft_avx2.hpp — complex FFTs for the CPU r2iq backend (AVX2 + FMA, split re/im arrays).
//
// The reference runs its r2iq on FFTW plans (Core/fft_mt_r2iq.cpp:221-225: an r2c of 8192
// and backward c2c plans of 4096 >> d).  This is the CPU backend's own transform: unnormalised
// DFT, forward e^{-2 pi i jk/n} (FFTW_FORWARD) and backward e^{+2 pi i jk/n} (FFTW_BACKWARD),
// radix-4 Stockham passes (self-sorting, out of place between two buffer pairs) plus one
// radix-2 pass for sizes 2 * 4^k.  Data are split: re[n] and im[n], so every vector holds 8
// real or 8 imaginary parts and a complex multiply is 2 mul + 2 fma.
//
// Pass with stride s (s = 1, 4, 16, ..., m = n / (4 s) butterflies per group):
//   a_k = src[s (p + k m) + q],  k = 0..3,  p < m, q < s
//   dst[4 s p + q + k s] = DFT4(a)_k * W_{4 m}^{p k}      (W_{4m} = W_n^{s})
// s >= 8 vectorises over q (contiguous loads and stores, one twiddle set per p); s = 4 over
// (p, q) pairs: two p per vector, 128-bit stores; s = 1 over 8 consecutive p, with an 8x4
// transpose before the stores.
#pragma once

#include <cstddef>
#include <vector>

namespace sddc {
namespace cpu {

class FftPlan {
public:
    explicit FftPlan(int n);   // n = 2^k, 32 <= n <= 8192
    int size() const { return n_; }

    // In: (re, im).  Work buffers (wre, wim) of n floats.  The result is left in one of the
    // two pairs; the returned index says which: 0 = (re, im), 1 = (wre, wim).
    int forward(float *re, float *im, float *wre, float *wim) const { return run<-1>(re, im, wre, wim); }
    int backward(float *re, float *im, float *wre, float *wim) const { return run<+1>(re, im, wre, wim); }

private:
    struct Pass {
        int s;            // stride (sub-transform size so far); radix 2 when r2
        bool r2;
        size_t tw;        // offset of this pass's twiddles in tw_
    };
    template <int SIGN>
    int run(float *re, float *im, float *wre, float *wim) const;

    int n_;
    std::vector<Pass> passes_;
    std::vector<float> tw_;   // forward twiddles; the backward transform conjugates them
};

}  // namespace cpu
}  // namespace sddc
