// ddc_kernels.hip — the fused r2iq frame kernels for gfx950 (MI355X).
//
// One workgroup (256 threads = 4 wave64) owns one overlap-save FRAME: 8192 real
// input samples at hop 6144 (Core/fft_mt_r2iq_impl.hpp:84-88).  Everything
// between the int16 read and the float2 IQ write stays in LDS/registers:
//
//   a2 convert_float<rand>          fft_mt_r2iq.h:36-51        -> pass-0 loader
//   a3 r2c 8192 = 4096-pt complex   impl.hpp:88                -> 3 x radix-16 LDS Stockham
//      FFT of z[n] = x[2n] + i x[2n+1] plus the split post-twiddle
//   a4 shift_freq x H_d + zero fill impl.hpp:76-96, .h:53-61   -> fused into the inverse pass-0 loader
//   a6 backward c2c mfft            impl.hpp:98                -> LDS Stockham (radix 2..16)
//   a7 overlap-discard (+conj)      impl.hpp:117-138, .h:63-81 -> last-pass storer, coalesced float2
//
// HBM traffic per frame: 8192 int16 in (25 % re-read from L2 by the neighbouring
// frame) and 6144/2^(d+1) or 4096/2^(d+1) float2 out.  Tables (twiddles, H_d) are
// small and L2-resident.
#include <hip/hip_runtime.h>

#include "fft_device.hpp"
#include "ddc_device_io.hpp"
#include "variants_api.h"

namespace sddc {

constexpr int kNT = 256;          // threads per workgroup
constexpr int kHalf = 4096;       // halfFft
constexpr int kHop = 6144;        // 3*halfFft/2
constexpr int kBlock = 65536;     // transferSamples
constexpr int kFrames = 11;       // fftPerBuf

__device__ __forceinline__ float derand(int v, int rand)
{
    // fft_mt_r2iq.h:41-44: odd samples are XORed with 0xFFFE (int16 -2) when rand is on
    return (float)(v ^ (-2 & -(v & rand & 1)));
}

// ---------------------------------------------------------------------------
// Forward half: frame samples -> Z (4096-pt FFT of the even/odd packing) in LDS,
// natural order at lds_pad(k).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void forward_4096(const int *__restrict__ frame32, int rand,
                                             float2 *lds, const float2 *__restrict__ tw)
{
    {
        StockhamPass<kHalf, 16, 1, kNT> p;
        p.compute<-1>([&](int n) {
            const int w = frame32[n];
            return make_float2(derand((int)(short)(w & 0xffff), rand), derand(w >> 16, rand));
        }, tw);
        p.store([&](int pos, float2 v) { lds[lds_pad(pos)] = v; });
    }
    __syncthreads();
    {
        StockhamPass<kHalf, 16, 16, kNT> p;
        p.compute<-1>([&](int n) { return lds[lds_pad(n)]; }, tw);
        __syncthreads();
        p.store([&](int pos, float2 v) { lds[lds_pad(pos)] = v; });
    }
    __syncthreads();
    {
        StockhamPass<kHalf, 16, 256, kNT> p;
        p.compute<-1>([&](int n) { return lds[lds_pad(n)]; }, tw);
        __syncthreads();
        p.store([&](int pos, float2 v) { lds[lds_pad(pos)] = v; });
    }
    __syncthreads();
}

// X[bin] * H from Z in LDS: the r2c split (E + W^bin O) times the (pre-halved) filter.
// Returns 0 for bins the reference zero-fills (impl.hpp:91-92, 95-96).
template <int N>
__device__ __forceinline__ float2 shifted_bin(const float2 *lds, int m, int tunebin,
                                              const float2 *__restrict__ post,
                                              const float2 *__restrict__ hsel)
{
    const int bin = tunebin + m - (m >= N / 2 ? N : 0);
    if (bin < 0 || bin >= kHalf) return make_float2(0.f, 0.f);
    const float2 zk = lds[lds_pad(bin)];
    const float2 zc = lds[lds_pad((kHalf - bin) & (kHalf - 1))];
    // A = Zk + conj(Zc), B = Zk - conj(Zc);  X = (A + W^bin * B / i) / 2
    const float2 A = make_float2(zk.x + zc.x, zk.y - zc.y);
    const float2 B = make_float2(zk.x - zc.x, zk.y + zc.y);
    const float2 Bi = make_float2(B.y, -B.x);
    const float2 X2 = cadd(A, cmul(Bi, post[bin]));
    return cmul(X2, hsel[m]);   // hsel already carries the factor 1/2
}

// ---------------------------------------------------------------------------
// Inverse half: mfft-point backward FFT of the shifted/filtered bins; the last
// pass hands (n, y[n]) to `emit`.
// ---------------------------------------------------------------------------
template <int N, class Emit>
__device__ __forceinline__ void inverse_from_Z(float2 *lds, int tunebin,
                                               const float2 *__restrict__ post,
                                               const float2 *__restrict__ hsel,
                                               const float2 *__restrict__ tw, Emit emit)
{
    auto ldsload = [&](int n) { return lds[lds_pad(n)]; };
    auto ldsstore = [&](int pos, float2 v) { lds[lds_pad(pos)] = v; };
    auto binload = [&](int m) { return shifted_bin<N>(lds, m, tunebin, post, hsel); };
    if constexpr (N >= 512) {
        // radix plan [N/256, 16, 16]: the first pass has exactly 256 butterflies
        constexpr int R0 = N / 256;
        {
            StockhamPass<N, R0, 1, kNT> p;
            p.template compute<+1>(binload, tw);
            __syncthreads();
            p.store(ldsstore);
        }
        __syncthreads();
        {
            StockhamPass<N, 16, R0, kNT> p;
            p.template compute<+1>(ldsload, tw);
            __syncthreads();
            p.store(ldsstore);
        }
        __syncthreads();
        {
            StockhamPass<N, 16, R0 * 16, kNT> p;
            p.template compute<+1>(ldsload, tw);
            p.store(emit);
        }
    } else {
        // N <= 256: materialise the N filtered bins, then [N/16, 16]
        float2 t = make_float2(0.f, 0.f);
        const int m = (int)threadIdx.x;
        if (m < N) t = binload(m);
        __syncthreads();
        if (m < N) lds[lds_pad(m)] = t;
        __syncthreads();
        constexpr int R0 = N / 16;
        {
            StockhamPass<N, R0, 1, kNT> p;
            p.template compute<+1>(ldsload, tw);
            __syncthreads();
            p.store(ldsstore);
        }
        __syncthreads();
        {
            StockhamPass<N, 16, R0, kNT> p;
            p.template compute<+1>(ldsload, tw);
            p.store(emit);
        }
    }
}

// Overlap-discard placement of frame k's inverse output inside its block's
// output span (impl.hpp:117-138): k = 0 keeps y[N/4, 3N/4) at 0; k >= 1 keeps
// y[0, 3N/4) at N/2 + (3N/4)(k-1).
template <int N>
__device__ __forceinline__ void emit_sample(float2 *__restrict__ out_blk, int k, int n, float2 v, float conj_sign)
{
    v.y *= conj_sign;
    if (k == 0) {
        if (n >= N / 4 && n < 3 * N / 4) out_blk[n - N / 4] = v;
    } else if (n < 3 * N / 4) {
        out_blk[N / 2 + (3 * N / 4) * (k - 1) + n] = v;
    }
}

// the same into a CF32 or CS16 stream (many-channel v1 path)
template <int N>
__device__ __forceinline__ void emit_sample_fmt(char *__restrict__ ob, int cs16, float scale, int k, int n,
                                                float2 v, float conj_sign)
{
    v.y *= conj_sign;
    int idx = -1;
    if (k == 0) {
        if (n >= N / 4 && n < 3 * N / 4) idx = n - N / 4;
    } else if (n < 3 * N / 4) {
        idx = N / 2 + (3 * N / 4) * (k - 1) + n;
    }
    if (idx < 0) return;
    if (cs16)
        reinterpret_cast<unsigned *>(ob)[idx] = cs16_pack(v, scale);
    else
        reinterpret_cast<float2 *>(ob)[idx] = v;
}

// ---------------------------------------------------------------------------
// Single-channel fused frame kernel.  grid = nblk * 11 workgroups.
//   in32 : int16 pairs of [history 4096 | nblk * 65536]
//   out  : nblk * 8*N float2
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(kNT) void r2iq_frame_kernel(const int *__restrict__ in32,
                                                         float2 *__restrict__ out,
                                                         const float2 *__restrict__ tw4096,
                                                         const float2 *__restrict__ post8192,
                                                         const float2 *__restrict__ hsel,
                                                         int tunebin, int lsb, int rand)
{
    constexpr int N = kHalf >> D;
    __shared__ float2 lds[lds_slots(kHalf)];

    const int f = (int)blockIdx.x;
    const int blk = f / kFrames;
    const int k = f - blk * kFrames;
    const int *frame32 = in32 + ((size_t)blk * kBlock + (size_t)k * kHop) / 2;

    forward_4096(frame32, rand, lds, tw4096);

    float2 *out_blk = out + (size_t)blk * 8 * N;
    const float cs = lsb ? -1.f : 1.f;
    inverse_from_Z<N>(lds, tunebin, post8192, hsel, tw4096,
                      [&](int n, float2 v) { emit_sample<N>(out_blk, k, n, v, cs); });
}

// ---------------------------------------------------------------------------
// Many-channel kernel: one workgroup per (frame, channel group).  The forward
// transform is computed once per workgroup and shared by `cpg` channels
// (SURVEY.md §8(e)): per channel the shift x H, the inverse and the write.
//   out: channel c's stream at complex element c*stride, CF32 or (cs16) int16 pairs
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(kNT) void r2iq_channels_kernel(const int *__restrict__ in32,
                                                            void *__restrict__ out, size_t stride,
                                                            const float2 *__restrict__ tw4096,
                                                            const float2 *__restrict__ post8192,
                                                            const float2 *__restrict__ hsel,
                                                            const int *__restrict__ tunebins,
                                                            int nch, int cpg, int lsb, int rand,
                                                            int cs16, float cs16_scale)
{
    constexpr int N = kHalf >> D;
    __shared__ float2 zbuf[lds_slots(kHalf)];
    __shared__ float2 work[lds_slots(N)];

    const int f = (int)blockIdx.x;
    const int blk = f / kFrames;
    const int k = f - blk * kFrames;
    const int *frame32 = in32 + ((size_t)blk * kBlock + (size_t)k * kHop) / 2;
    forward_4096(frame32, rand, zbuf, tw4096);

    const float cs = lsb ? -1.f : 1.f;
    const int c0 = (int)blockIdx.y * cpg;
    for (int c = c0; c < c0 + cpg && c < nch; c++) {
        const int tb = tunebins[c];
        char *ob = static_cast<char *>(out) + ((size_t)c * stride + (size_t)blk * 8 * N) * (cs16 ? 4 : 8);
        // first inverse pass reads Z from zbuf; the rest run in `work`
        auto ldsload = [&](int n) { return work[lds_pad(n)]; };
        auto ldsstore = [&](int pos, float2 v) { work[lds_pad(pos)] = v; };
        auto emit = [&](int n, float2 v) { emit_sample_fmt<N>(ob, cs16, cs16_scale, k, n, v, cs); };
        auto binload = [&](int m) { return shifted_bin<N>(zbuf, m, tb, post8192, hsel); };
        if constexpr (N >= 512) {
            constexpr int R0 = N / 256;
            {
                StockhamPass<N, R0, 1, kNT> p;
                p.template compute<+1>(binload, tw4096);
                p.store(ldsstore);
            }
            __syncthreads();
            {
                StockhamPass<N, 16, R0, kNT> p;
                p.template compute<+1>(ldsload, tw4096);
                __syncthreads();
                p.store(ldsstore);
            }
            __syncthreads();
            {
                StockhamPass<N, 16, R0 * 16, kNT> p;
                p.template compute<+1>(ldsload, tw4096);
                p.store(emit);
            }
        } else {
            const int m = (int)threadIdx.x;
            if (m < N) work[lds_pad(m)] = binload(m);
            __syncthreads();
            constexpr int R0 = N / 16;
            {
                StockhamPass<N, R0, 1, kNT> p;
                p.template compute<+1>(ldsload, tw4096);
                __syncthreads();
                p.store(ldsstore);
            }
            __syncthreads();
            {
                StockhamPass<N, 16, R0, kNT> p;
                p.template compute<+1>(ldsload, tw4096);
                p.store(emit);
            }
        }
        __syncthreads();   // `work` is reused by the next channel
    }
}

// ---------------------------------------------------------------------------
// Host-side launchers (C++ linkage, called from ddc_runtime.cpp)
// ---------------------------------------------------------------------------
template <int D>
static hipError_t launch_frames_d(const KernelTables &t, const int16_t *d_in, int nblk, float *d_out,
                                  int tunebin, int lsb, int rand, hipStream_t s)
{
    dim3 grid((unsigned)(nblk * kFrames)), block(kNT);
    hipLaunchKernelGGL(r2iq_frame_kernel<D>, grid, block, 0, s,
                       reinterpret_cast<const int *>(d_in), reinterpret_cast<float2 *>(d_out),
                       t.tw4096, t.post8192, t.hsel[D], tunebin, lsb, rand);
    return hipGetLastError();
}

hipError_t launch_frames(const KernelTables &t, int d, const int16_t *d_in, int nblk, float *d_out,
                         int tunebin, int lsb, int rand, hipStream_t s)
{
    switch (d) {
    case 0: return launch_frames_d<0>(t, d_in, nblk, d_out, tunebin, lsb, rand, s);
    case 1: return launch_frames_d<1>(t, d_in, nblk, d_out, tunebin, lsb, rand, s);
    case 2: return launch_frames_d<2>(t, d_in, nblk, d_out, tunebin, lsb, rand, s);
    case 3: return launch_frames_d<3>(t, d_in, nblk, d_out, tunebin, lsb, rand, s);
    case 4: return launch_frames_d<4>(t, d_in, nblk, d_out, tunebin, lsb, rand, s);
    case 5: return launch_frames_d<5>(t, d_in, nblk, d_out, tunebin, lsb, rand, s);
    case 6: return launch_frames_d<6>(t, d_in, nblk, d_out, tunebin, lsb, rand, s);
    default: return hipErrorInvalidValue;
    }
}

template <int D>
static hipError_t launch_channels_d(const KernelTables &t, const int16_t *d_in, int nblk,
                                    const int *d_tunebins, int nch, void *d_out, size_t stride,
                                    int lsb, int rand, int cs16, float cs16_scale, hipStream_t s)
{
    const int cpg = channels_per_group(D, nch);
    dim3 grid((unsigned)(nblk * kFrames), (unsigned)((nch + cpg - 1) / cpg)), block(kNT);
    hipLaunchKernelGGL(r2iq_channels_kernel<D>, grid, block, 0, s, reinterpret_cast<const int *>(d_in), d_out,
                       stride / 2, t.tw4096, t.post8192, t.hsel[D], d_tunebins, nch, cpg, lsb, rand, cs16,
                       cs16_scale);
    return hipGetLastError();
}

int channels_per_group(int d, int nch)
{
    // amortise the forward transform over up to 16 channels per workgroup at
    // small mfft; keep the grid large enough to fill 256 CUs
    const int cap = d >= 3 ? 16 : d >= 1 ? 8 : 4;
    return nch < cap ? nch : cap;
}

hipError_t launch_channels(const KernelTables &t, int d, const int16_t *d_in, int nblk,
                           const int *d_tunebins, int nch, void *d_out, size_t stride,
                           int lsb, int rand, int cs16, float cs16_scale, hipStream_t s)
{
#define SDDC_CH(D) launch_channels_d<D>(t, d_in, nblk, d_tunebins, nch, d_out, stride, lsb, rand, cs16, cs16_scale, s)
    switch (d) {
    case 0: return SDDC_CH(0);
    case 1: return SDDC_CH(1);
    case 2: return SDDC_CH(2);
    case 3: return SDDC_CH(3);
    case 4: return SDDC_CH(4);
    case 5: return SDDC_CH(5);
    case 6: return SDDC_CH(6);
    default: return hipErrorInvalidValue;
    }
#undef SDDC_CH
}

}  // namespace sddc
