// fft_avx2.hpp — complex FFTs for the CPU r2iq backend (AVX2 + FMA, split re/im arrays).
//
// The reference runs its r2iq on FFTW plans (Core/fft_mt_r2iq.cpp:221-225: an r2c of 8192
// and backward c2c plans of 4096 >> d).  This is the CPU backend's own transform: unnormalised
// DFT, forward e^{-2 pi i jk/n} (FFTW_FORWARD) and backward e^{+2 pi i jk/n} (FFTW_BACKWARD),
// Stockham passes (self-sorting, out of place between two buffer pairs): radix 16 for
// n >= 4096, radix 4 below, plus one radix-2 pass for sizes 2 * 4^k.  Data are split: re[n]
// and im[n], so every vector holds 8 real or 8 imaginary parts and a complex multiply is
// 2 mul + 2 fma.
//
// Radix-R pass with stride s (m = n / (R s) butterflies per group):
//   a_k = src[s (p + k m) + q],  k = 0..R-1,  p < m, q < s
//   dst[R s p + q + k s] = DFT_R(a)_k * W_{R m}^{p k}      (W_{R m} = W_n^{s})
// s >= 8 vectorises over q (contiguous loads and stores, one twiddle set per p); s = 4 over
// (p, q) pairs: two p per vector, 128-bit stores; s = 1 over 8 consecutive p, with 8 x 4
// (radix 4) or 8 x 8 (radix 16) transposes before the stores.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace sddc {
namespace cpu {

class FftPlan {
public:
    explicit FftPlan(int n);   // n = 2^k, 32 <= n <= 8192
    int size() const { return n_; }

    // In: (re, im).  Work buffers (wre, wim) of n floats.  The result is left in one of the
    // two pairs; the returned index says which: 0 = (re, im), 1 = (wre, wim).
    int forward(float *re, float *im, float *wre, float *wim) const { return run<-1>(re, im, wre, wim, nullptr, false); }
    int backward(float *re, float *im, float *wre, float *wim) const { return run<+1>(re, im, wre, wim, nullptr, false); }
    // Forward transform of x[2j] + i x[2j+1] (n int16 pairs, the r2iq frame), converted with the
    // de-randomiser (rand) inside the first pass.  Needs n >= 4096.  (re, im) are work buffers too.
    int forward_i16(const int16_t *x, bool rand, float *re, float *im, float *wre, float *wim) const
    {
        return run<-1>(re, im, wre, wim, x, rand);
    }

private:
    struct Pass {
        int s;            // stride (sub-transform size so far)
        int radix;        // 16, 4 or 2
        size_t tw;        // offset of this pass's twiddles in tw_
    };
    template <int SIGN>
    int run(float *re, float *im, float *wre, float *wim, const int16_t *x, bool rand) const;

    int n_;
    std::vector<Pass> passes_;
    std::vector<float> tw_;   // forward twiddles; the backward transform conjugates them
};

}  // namespace cpu
}  // namespace sddc
