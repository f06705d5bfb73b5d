// ddc_frame_common.hpp — device helpers shared by the single-channel frame kernels: the
// default persistent kernel (ddc_persistent.hip) and the d = 0 A/B variants built into
// libsddc_ddc_variants.so (variants/ddc_variants.hip).
//
// Frame k of input block b is the 8192 samples at 65536 b + 6144 k of the batch's
// [history 4096 | blocks] buffer (Core/fft_mt_r2iq_impl.hpp:84-88); one 256-thread
// workgroup transforms it in LDS, 16 points per thread.
#pragma once

#include <hip/hip_runtime.h>

#include "ddc_device_io.hpp"
#include "ddc_kernels.h"
#include "fft_device.hpp"

namespace sddc {
namespace {

constexpr int NT = 256;       // threads per frame
constexpr int HALF = 4096;    // halfFft            fft_mt_r2iq.h:18
constexpr int HOP = 6144;     // 3 halfFft / 2      impl.hpp:88
constexpr int BLOCK = 65536;  // transferSamples    config.h:80-81
constexpr int FRAMES = 11;    // fftPerBuf          fft_mt_r2iq.h:19

// LDS XOR swizzle: the 16-consecutive-per-lane writes of the first pass and the
// 64-consecutive reads are bank-conflict free, and swz(e + 256 r) = swz(e) + 256 r.
__device__ __forceinline__ int swz(int e) { return e ^ ((e >> 4) & 15); }

// convert_float<rand>, Core/fft_mt_r2iq.h:36-51.  With RAND the odd int16 samples are XORed
// with 0xFFFE, which for an odd 16-bit value is exactly its negation (v ^ 0xFFFE = ~v ^ 1 = -v),
// so the de-randomised float is (v odd ? -v : v): a sign-bit XOR with the sample's LSB.
template <bool RAND>
__device__ __forceinline__ float derand(int v)
{
    const float f = (float)v;
    if constexpr (!RAND) return f;
    return __int_as_float(__float_as_int(f) ^ (v << 31));
}

// a * W (DIR < 0) or a * conj(W) (DIR > 0)
template <int DIR>
__device__ __forceinline__ float2 TW(float2 a, float2 w) { return DIR < 0 ? cmul(a, w) : cmulc(a, w); }

// X[bin] * Hh[m] from Z (Hh = H/2): the r2c split E + W^bin O, times the filter, with the
// reference's zero fill for out-of-band bins (impl.hpp:91-92, 95-96):
//   X Hh = Hh [(Zk + conj Zc) - i W^bin (Zk - conj Zc)] = Zk P + conj(Zc) Q,
//   P = Hh (1 - i W^bin),  Q = Hh (1 + i W^bin)     (Zc = Z[(4096 - bin) mod 4096])
// from the per-(d, tunebin) table c = (P, Q) of build_split_filter_kernel, zero out of band.
__device__ __forceinline__ float2 split_pq(float2 zk, float2 zc, float4 c)
{
    float2 v;
    v.x = zk.x * c.x - zk.y * c.y + zc.x * c.z + zc.y * c.w;
    v.y = zk.x * c.y + zk.y * c.x + zc.x * c.w - zc.y * c.z;
    return v;
}

// Frame k of a block: output base of the kept samples, relative to the block's output
template <int N>
__device__ __forceinline__ int emit_base(int k)
{
    return k == 0 ? -N / 4 : N / 2 + (3 * N / 4) * (k - 1);
}

// The kept outputs n = t + NB r of frame k (r in [4, 12) for k = 0, [0, 12) otherwise).
// fbase: the frame's first kept output slot relative to the batch (also the NCO index).
template <int NB, bool NCO, bool CS16>
__device__ __forceinline__ void emit_frame(void *__restrict__ out, int fbase, int k, int t, const float2 (&u)[16],
                                           const OutArgs &oa, const NcoArgs &nco)
{
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(static_cast<char *>(out) + (size_t)fbase * out_bytes<CS16>());
    const int r0 = k == 0 ? 4 : 0;   // wave-uniform
#pragma unroll
    for (int r = 0; r < 12; r++) {
        if (r < r0) continue;
        float2 v = flip(u[r], oa.lsbmask);
        if constexpr (NCO) v = nco_mix(v, nco, fbase + t + NB * r);
        store_iq<CS16>(v, ro, (unsigned)t, (unsigned)(NB * r), oa);
    }
}

// this thread's 16 int16 pairs of frame k of block blk: pair t + 256 r
__device__ __forceinline__ void load_frame(const int *__restrict__ in32, int blk, int k, int (&x)[16])
{
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(in32 + ((size_t)blk * BLOCK + (size_t)k * HOP) / 2);
    const unsigned vo = 4u * threadIdx.x;
#pragma unroll
    for (int r = 0; r < 16; r++) x[r] = buf_load4<SDDC_LD_AUX>(rs, vo, 4u * NT * r);
}

}  // namespace
}  // namespace sddc
