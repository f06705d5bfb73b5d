// ddc_frame_common.hpp — device helpers shared by the single-channel frame kernels: the
// persistent kernel (ddc_persistent.hip, d >= 1) and the d = 0 fused-split kernel (ddc_fs.hip).
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
// Q = i r P with r = Q / (i P) = cot(pi/4 - pi bin / 8192) real (independent of H and the tune
// bin), so X Hh = P (Zk + i r conj Zc) = P (Zk.x + r Zc.y, Zk.y + r Zc.x): 6 VALU and a float2
// of P per bin (build_split_filter_kernel; r held in registers where the kernel has them).
__device__ __forceinline__ float2 split_pr(float2 zk, float2 zc, float2 p, float r)
{
    const float vx = fmaf(r, zc.y, zk.x), vy = fmaf(r, zc.x, zk.y);
    return make_float2(fmaf(vx, p.x, -vy * p.y), fmaf(vx, p.y, vy * p.x));
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

// One LDS read per value.  The compiler pairs reads of r and r + 1 into ds_read2st64_b64 /
// ds_read2_b64, which the LDS serves at 8 cycles per pair against 2 + 2 for two ds_read_b64
// (MI355X_MICROARCH.md, LDS table); an empty asm with a memory clobber after each read keeps
// them apart at no VALU cost.  Exchange reads: +2 % at d = 0, 1, 4, bit-identical
// (profiles/r02/ab/xrd.txt); the same for the pass-1 twiddle-table reads was neutral
// (profiles/r02/ab/twrd.txt).
#define XRD(dst, expr) do { dst = (expr); asm volatile("" ::: "memory"); } while (0)

// Order LDS accesses within one wave: the wave's LDS operations execute in order, so a pass
// whose readers and writers are all lanes of one wave needs program order only (the fences keep
// the compiler from moving LDS accesses across), not a workgroup barrier.
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Swizzled row stores.  Element 16 q + (r ^ x) of a frame buffer (x = t & 15, q >= 0) sits at
// byte (128 q + 8 x) ^ 8 r: the lane's base A = 128 q + 8 x is formed once per frame, and each
// of the 16 stores costs one v_xor_b32 with an immediate (an extra row offset 128 r rides on the
// ds_write immediate), instead of the xor, mask, shift and or the compiler emits for the index.
// d >= 1: d = 1 +0.6 %, d = 4 +2.8 %, bit-identical (profiles/r02/ab/xst.txt).  At d = 0 all
// four row stores together were 0.4 % slower; split up, the forward pass-0 rows lose 1.2-1.7 %
// and the inverse pass-0 rows gain 0-1.3 % (xst_d0_parts.txt, xst_inv0_confirm.txt), so d = 0
// takes the latter only.
__device__ __forceinline__ void st_row(float2 *buf, unsigned A, int r, int rstride, float2 v)
{
    *(reinterpret_cast<float2 *>(reinterpret_cast<char *>(buf) + (A ^ (8u * (unsigned)r))) + rstride * r) = v;
}

// Swizzled element Lane + R with no carry between the two (disjoint bits): the swizzle is linear
// over XOR, swz(Lane ^ R) = swz(Lane) ^ swz(R), so with lane8 = 8 swz(Lane) formed once per pass
// the byte address is lane8 ^ 8 swz(R), one v_xor_b32 with an immediate per access instead of
// the add, shift, xor-and-mask and scale the index form costs per access.  Used by the inverse
// passes at d >= 1 (their N/16-strided reads and R0-row stores): static VALU -115..-124 at
// d = 1..3, -90 at d = 4; d = 1 +3-5 %, d = 2, 3 +4-5 %, d = 4 +3 %, d = 5, 6 +2 %, bit-identical
// (profiles/r02/ab/lx_xor_linear_addresses.txt).
__device__ __forceinline__ float2 &lds_x(float2 *buf, unsigned lane8, int R)
{
    return *reinterpret_cast<float2 *>(reinterpret_cast<char *>(buf) + (lane8 ^ (8u * (unsigned)swz(R))));
}
#define LX(buf, lane, R) lds_x(buf, 8u * (unsigned)swz(lane), R)

// Pass-1 table twiddles at d <= 1: issued in two groups (8 + 7) right behind the data reads, so
// the products wait on two LDS round trips instead of one per ds_read2 pair (the compiler's own
// schedule); the kernel is held to 128 VGPRs for it.  d = 0 +1-2.7 %, d = 1 +1 %; one group of
// 15 spills and loses at every d, and at d >= 2 either form loses 1-5 % (profiles/r02/ab/early.txt).

// a[r] *= tbl[(r - 1) S + j] (conjugated for DIR > 0), r = 1..15.  EARLY: the table reads are
// issued in two groups (8 + 7) right behind the caller's exchange reads, each group before its
// products (empty asm with a memory clobber), so the products wait on two LDS round trips; the
// compiler's own schedule issues one ds_read2 pair at a time and waits lgkmcnt(0) after each.
// Each read is its own ds_read_b64 (XRD): merged into ds_read2_b64 pairs (8 LDS cycles each
// against 2 per ds_read_b64 on gfx950, MI355X_MICROARCH.md LDS table) the FS kernel ran
// 1.3 % slower on average (+2.8 / -0.3 / +1.7 / +1.0 %, d = 1 neutral;
// profiles/r06/ab/table_twiddle_single_b64_reads.txt).
template <int DIR, bool EARLY>
__device__ __forceinline__ void table_twiddle(float2 *a, const float2 *tbl, int S, int j)
{
    if constexpr (EARLY) {
        float2 tw[15];
#pragma unroll
        for (int r = 1; r <= 8; r++) XRD(tw[r - 1], tbl[(r - 1) * S + j]);
#pragma unroll
        for (int r = 1; r <= 8; r++) a[r] = TW<DIR>(a[r], tw[r - 1]);
#pragma unroll
        for (int r = 9; r < 16; r++) XRD(tw[r - 1], tbl[(r - 1) * S + j]);
#pragma unroll
        for (int r = 9; r < 16; r++) a[r] = TW<DIR>(a[r], tw[r - 1]);
    } else {
        // unpaired too (no ds_read2_b64): d = 2 +1.6 / +2.0 %, d = 3 +0.8 / +1.1 %, d = 4..6 -0.3 to
        // +0.7 % (profiles/r06/ab/persistent_pass1_twiddles_unpaired_d2_6.txt)
#pragma unroll
        for (int r = 1; r < 16; r++) {
            float2 w;
            XRD(w, tbl[(r - 1) * S + j]);
            a[r] = TW<DIR>(a[r], w);
        }
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
