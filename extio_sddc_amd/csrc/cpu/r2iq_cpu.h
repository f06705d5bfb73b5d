// r2iq_cpu.h — the CPU r2iq backend: the reference's overlap-save worker
// (Core/fft_mt_r2iq_impl.hpp:15-152, AVX2 variant Core/fft_mt_r2iq_avx2.cpp:11-328) restated
// for x86-64 AVX2 + FMA on this library's own FFTs (fft_avx2.hpp), without FFTW.
//
// It is the host half of the C ABI's CPU handles (sddc_ddc_create with device
// SDDC_DDC_DEVICE_CPU): an explicit backend choice, never a silent fallback of a GPU handle.
// No HIP header is included here, so the drop-in class, the C ABI front and this file can be
// built and run under ASan/UBSan/TSan in a container without a GPU.
//
// Per input block (65536 int16) and frame k = 0..10 (8192 samples at 6144 k of
// [history 4096 | block], impl.hpp:84-88):
//   convert (+ rand: v odd ? -v : v)       fft_mt_r2iq.h:36-51
//   Z = FFT4096(x[2n] + i x[2n+1])          r2c 8192 (impl.hpp:88) as a packed complex FFT
//   T[m] = Z_j P[m] + conj(Z_-j) Q[m]       split x shift x filter with zero fill
//          (j = tb + m, or tb - mfft + m for m >= mfft/2; P = H/2 (1 - i W^j), Q = H/2 (1 + i W^j))
//   y = IFFT_mfft(T)                         impl.hpp:98 (unnormalised, FFTW_BACKWARD)
//   keep y[mfft/4, 3mfft/4) (k = 0) or y[0, 3mfft/4) (k >= 1), conj if lsb   impl.hpp:117-138
#pragma once

#include <complex>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

#include "fft_avx2.hpp"

namespace sddc {
namespace cpu {

struct Params {
    int d = 0;              // decimation index 0..6, mfft = 4096 >> d
    int tunebin = 1024;     // multiple of 4 in [0, 4096)
    bool lsb = false;       // sideband flip (conj)
    bool rand = false;      // ADC de-randomiser
    bool cs16 = false;      // output int16 (I, Q) = saturate(rint(x * scale)) instead of float
    float scale = 1.f;
    // fused fine-tune NCO (fine_tune.h): T[32] and per-128-sample lane starts [blocks][4] of
    // this call's output, as (cos, sin) float pairs; null = off
    const float *nco_trig = nullptr;
    const float *nco_starts = nullptr;
};

bool supported();   // this CPU has AVX2 and FMA

class R2iq {
public:
    // H[d][4096]: the filter bank (filterbank.h filter_response), double precision
    explicit R2iq(const std::complex<double> *H);
    ~R2iq();
    R2iq(const R2iq &) = delete;
    R2iq &operator=(const R2iq &) = delete;

    void reset();                                   // zero history (TurnOn)
    void set_history(const int16_t *last4096);      // history = these 4096 samples
    // nblk blocks, block i at blocks[i]; writes nblk * (32768 >> d) complex samples to out
    // (CF32: float (I, Q); CS16: int16 (I, Q)) and keeps the last 4096 input samples
    void process(const int16_t *const *blocks, int nblk, void *out, const Params &p);

private:
    struct Buf;
    void build_pq(int d, int tb);
    void frame(const int16_t *x, int d, bool rand, const float **yr, const float **yi);

    std::unique_ptr<Buf> b_;
    FftPlan fwd_;
    std::vector<std::unique_ptr<FftPlan>> inv_;     // per d
    std::vector<std::complex<double>> H_;           // [7][4096]
    int pq_d_ = -1, pq_tb_ = -1;
    int lo_ = 0, hi_ = 0;                           // valid m ranges of the (P, Q) table
};

}  // namespace cpu
}  // namespace sddc
