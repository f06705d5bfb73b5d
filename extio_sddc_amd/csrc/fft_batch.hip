// fft_batch.hip — batched complex and real-to-complex FFTs for gfx950 (include/sddc_fft.h).
//
// One 256-thread workgroup owns 4096 / n transforms (n / 16 threads each).  Passes are
// LDS Stockham steps of radix 16, 16 and n / 256 (radix n / 16 for n <= 256): the first
// reads global memory, the last writes it, in between the data stays in padded LDS.
// r2c(n) is the n/2-point complex FFT of x[2m] + i x[2m+1] followed by the split
//   X[k] = 1/2 [(Z_k + conj Z_{n/2-k}) - i W_n^k (Z_k - conj Z_{n/2-k})],  k = 0..n/2,
// the same packing the DDC path uses (ddc_persistent.hip).  Twiddles come from one
// 8192-entry table evaluated in double on the device and rounded once.
#include <hip/hip_runtime.h>

#include <mutex>

#include "fft_device.hpp"
#include "sddc_fft.h"

namespace sddc {
namespace {

constexpr int NT = 256;
constexpr int kTw = 8192;

__device__ float2 g_tw[kTw];   // e^{-2 pi i k / 8192}

__global__ void init_twiddles(float2 *tw)
{
    const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k < kTw) {
        double s, c;
        sincospi(-2.0 * k / kTw, &s, &c);
        tw[k] = make_float2((float)c, (float)s);
    }
}

// W_m^e for m | 8192 (forward sign), conjugated for DIR = +1
template <int DIR>
__device__ __forceinline__ float2 twiddle(int e, int m)
{
    float2 w = g_tw[(e * (kTw / m)) & (kTw - 1)];
    if (DIR > 0) w.y = -w.y;
    return w;
}

// One Stockham radix-R pass over n points (NS = product of the previous radices),
// TPT threads per transform, local thread lt.  in position j + r n/R, out position
// (j/NS) NS R + j%NS + r NS, twiddle W_{NS R}^{(j%NS) r}.
template <int n, int R, int NS, int TPT, int DIR, class Load, class Store>
__device__ __forceinline__ void pass(int lt, Load load, Store store)
{
    constexpr int NB = n / R;
    constexpr int PER = NB / TPT;
    static_assert(NB % TPT == 0, "pass geometry");
    float2 v[PER][R];
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = lt + i * TPT;
        float2 a[R];
#pragma unroll
        for (int r = 0; r < R; r++) a[r] = load(j + r * NB);
        if constexpr (NS > 1) {
#pragma unroll
            for (int r = 1; r < R; r++) a[r] = cmul(a[r], twiddle<DIR>((j % NS) * r, NS * R));
        }
        dft<R, DIR>(a, v[i]);
    }
    __syncthreads();   // every read of this pass is done before any write
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = lt + i * TPT;
        const int base = (j / NS) * NS * R + (j % NS);
#pragma unroll
        for (int r = 0; r < R; r++) store(base + r * NS, v[i][r]);
    }
}

// n-point transform of this thread's slot: load(pos) from wherever, result in LDS
// (natural order, padded) unless STORE_OUT, in which case the last pass calls out(pos, v).
template <int n, int DIR, class Load, class Out>
__device__ __forceinline__ void fft_n(int lt, float2 *sl, Load load, Out out)
{
    constexpr int TPT = n / 16;
    auto lds_ld = [&](int p) { return sl[lds_pad(p)]; };
    auto lds_st = [&](int p, float2 v) { sl[lds_pad(p)] = v; };
    if constexpr (n <= 256) {
        // n = 16 * R1: radix 16 then radix n/16
        pass<n, 16, 1, TPT, DIR>(lt, load, lds_st);
        __syncthreads();
        pass<n, n / 16, 16, TPT, DIR>(lt, lds_ld, out);
    } else {
        pass<n, 16, 1, TPT, DIR>(lt, load, lds_st);
        __syncthreads();
        pass<n, 16, 16, TPT, DIR>(lt, lds_ld, lds_st);
        __syncthreads();
        pass<n, n / 256, 256, TPT, DIR>(lt, lds_ld, out);
    }
}

template <int n, int DIR>
__global__ __launch_bounds__(NT) void fft_c2c_kernel(const float2 *in, float2 *out, int batch)
{
    constexpr int TPT = n / 16, TPW = NT / TPT;
    __shared__ float2 lds[TPW * lds_slots(n)];
    const int sub = (int)threadIdx.x / TPT, lt = (int)threadIdx.x % TPT;
    const long b = (long)blockIdx.x * TPW + sub;
    const bool ok = b < batch;
    const float2 *src = in + b * n;
    float2 *dst = out + b * n;
    float2 *sl = lds + sub * lds_slots(n);
    fft_n<n, DIR>(
        lt, sl, [&](int p) { return ok ? src[p] : make_float2(0.f, 0.f); },
        [&](int p, float2 v) {
            if (ok) dst[p] = v;
        });
}

template <int n>
__global__ __launch_bounds__(NT) void fft_r2c_kernel(const float2 *in, float2 *out, int batch)
{
    constexpr int m = n / 2;                 // complex FFT size
    constexpr int TPT = m / 16, TPW = NT / TPT;
    __shared__ float2 lds[TPW * lds_slots(m)];
    const int sub = (int)threadIdx.x / TPT, lt = (int)threadIdx.x % TPT;
    const long b = (long)blockIdx.x * TPW + sub;
    const bool ok = b < batch;
    const float2 *src = in + b * m;          // x[2i], x[2i+1] pairs
    float2 *dst = out + b * (m + 1);
    float2 *sl = lds + sub * lds_slots(m);
    fft_n<m, -1>(
        lt, sl, [&](int p) { return ok ? src[p] : make_float2(0.f, 0.f); },
        [&](int p, float2 v) { sl[lds_pad(p)] = v; });
    __syncthreads();
    if (!ok) return;
    for (int k = lt; k <= m; k += TPT) {
        const float2 zk = sl[lds_pad(k & (m - 1))];
        const float2 zc = sl[lds_pad((m - k) & (m - 1))];
        const float2 A = make_float2(zk.x + zc.x, zk.y - zc.y);         // Z_k + conj Z_{m-k}
        const float2 Bi = make_float2(zk.y + zc.y, zc.x - zk.x);        // (Z_k - conj Z_{m-k}) / i
        const float2 w = twiddle<-1>(k, n);
        const float2 t = cadd(A, cmul(Bi, w));
        dst[k] = make_float2(0.5f * t.x, 0.5f * t.y);
    }
}

template <int n, int DIR>
hipError_t c2c_n(const void *in, void *out, int batch, hipStream_t s)
{
    constexpr int TPW = NT / (n / 16);
    const unsigned grid = (unsigned)((batch + TPW - 1) / TPW);
    hipLaunchKernelGGL((fft_c2c_kernel<n, DIR>), dim3(grid), dim3(NT), 0, s, static_cast<const float2 *>(in),
                       static_cast<float2 *>(out), batch);
    return hipGetLastError();
}

template <int n>
hipError_t r2c_n(const float *in, void *out, int batch, hipStream_t s)
{
    constexpr int TPW = NT / (n / 32);
    const unsigned grid = (unsigned)((batch + TPW - 1) / TPW);
    hipLaunchKernelGGL((fft_r2c_kernel<n>), dim3(grid), dim3(NT), 0, s, reinterpret_cast<const float2 *>(in),
                       static_cast<float2 *>(out), batch);
    return hipGetLastError();
}

template <int DIR>
hipError_t c2c_dir(const void *in, void *out, int n, int batch, hipStream_t s)
{
    switch (n) {
    case 64: return c2c_n<64, DIR>(in, out, batch, s);
    case 128: return c2c_n<128, DIR>(in, out, batch, s);
    case 256: return c2c_n<256, DIR>(in, out, batch, s);
    case 512: return c2c_n<512, DIR>(in, out, batch, s);
    case 1024: return c2c_n<1024, DIR>(in, out, batch, s);
    case 2048: return c2c_n<2048, DIR>(in, out, batch, s);
    case 4096: return c2c_n<4096, DIR>(in, out, batch, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

// per-device twiddle table, filled once per device by a small kernel
hipError_t fft_prepare(hipStream_t s)
{
    static std::mutex mu;
    static bool ready[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(mu);
    if (ready[dev]) return hipSuccess;
    void *p = nullptr;
    if ((e = hipGetSymbolAddress(&p, HIP_SYMBOL(g_tw))) != hipSuccess) return e;
    hipLaunchKernelGGL(init_twiddles, dim3(kTw / 256), dim3(256), 0, s, static_cast<float2 *>(p));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    ready[dev] = true;
    return hipSuccess;
}

hipError_t fft_c2c(const void *in, void *out, int n, int batch, int dir, hipStream_t s)
{
    return dir < 0 ? c2c_dir<-1>(in, out, n, batch, s) : c2c_dir<+1>(in, out, n, batch, s);
}

hipError_t fft_r2c(const float *in, void *out, int n, int batch, hipStream_t s)
{
    switch (n) {
    case 128: return r2c_n<128>(in, out, batch, s);
    case 256: return r2c_n<256>(in, out, batch, s);
    case 512: return r2c_n<512>(in, out, batch, s);
    case 1024: return r2c_n<1024>(in, out, batch, s);
    case 2048: return r2c_n<2048>(in, out, batch, s);
    case 4096: return r2c_n<4096>(in, out, batch, s);
    case 8192: return r2c_n<8192>(in, out, batch, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace sddc
