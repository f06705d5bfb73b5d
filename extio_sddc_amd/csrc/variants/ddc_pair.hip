// ddc_pair.hip — d = 0 single-channel kernel with lane pairs (internal variant 6,
// libsddc_ddc_variants.so): the default kernel's 3 + 3 radix-16 passes and 5 LDS exchanges per
// frame, on 512 threads instead of 256.  Each radix-16 butterfly runs on two adjacent lanes,
// 8 points each, with its radix-2 stage across the pair by DPP (lane ^ 1) and a DFT-8 in
// registers, so a frame needs <= 64 VGPRs per lane and a CU keeps 8 waves per SIMD resident
// (4 frames) at the same 5 exchanges.  It tests the one combination the layouts of DESIGN.md
// §4.1 left open: more resident waves without more exchanges (variant 5 paid 7 for them).
//
// Butterfly forms (W16 = e^{DIR 2 pi i / 16}; lane h = 0, 1 of the pair):
//   DIF: lane h holds inputs 8h + i; c = a_i +- a_{i+8} across the pair, the odd half times
//        W16^i, then a DFT-8: lane h ends with outputs 2k + h;
//   DIT: lane h holds inputs 2i + h; a DFT-8 first, the odd half times W16^k, then the
//        radix-2 across the pair: lane h ends with outputs 8h + k.
// LDS: each exchange stores element e at e ^ ((e >> 4) & 15) with bit 4 further XORed by a
// parity of e chosen per exchange so that the two lanes of a pair (whose elements differ by
// 256 or 2048) never share a bank in one instruction, while every address is a per-lane base
// plus an immediate (see the per-pass notes).
#include <hip/hip_runtime.h>

#include "ddc_frame_common.hpp"
#include "variants_api.h"

namespace sddc {
namespace {

constexpr int NTP = 512;

// the pair partner's value (lane ^ 1; DPP quad_perm [1, 0, 3, 2])
__device__ __forceinline__ float pair_xchg(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

// hi lanes: c[I] *= W16^{I + 8} (= -W16^I), lo lanes keep c[I]; I = 0..7
template <int DIR, int I = 0>
__device__ __forceinline__ void hi_twiddle(float2 *c, bool hi)
{
    if constexpr (I < 8) {
        const float2 t = tw16<DIR, I + 8>(c[I]);
        c[I].x = hi ? t.x : c[I].x;
        c[I].y = hi ? t.y : c[I].y;
        hi_twiddle<DIR, I + 1>(c, hi);
    }
}

// DIF radix-16 on a lane pair: a = inputs 8h + i (twiddled), o = outputs 2k + h.  sg = hi ? -1 : 1.
template <int DIR>
__device__ __forceinline__ void pair16_dif(const float2 (&a)[8], float sg, bool hi, float2 (&o)[8])
{
    float2 c[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        // lo: a_i + a_{i+8}; hi: a_{i+8} - a_i = -(a_i - a_{i+8})
        c[i].x = fmaf(sg, pair_xchg(a[i].x), a[i].x);
        c[i].y = fmaf(sg, pair_xchg(a[i].y), a[i].y);
    }
    hi_twiddle<DIR>(c, hi);   // hi: (a_i - a_{i+8}) W16^i
    dft8<DIR>(c, o);
}

// DIT radix-16 on a lane pair: a = inputs 2i + h, o = outputs 8h + k.  sg = hi ? -1 : 1.
template <int DIR>
__device__ __forceinline__ void pair16_dit(const float2 (&a)[8], float sg, bool hi, float2 (&o)[8])
{
    float2 e[8];
    dft8<DIR>(a, e);          // lo: E_k (even inputs), hi: O_k (odd inputs)
    hi_twiddle<DIR>(e, hi);   // hi: -W16^k O_k
#pragma unroll
    for (int k = 0; k < 8; k++) {
        // lo: E + W O; hi: -W O + E
        o[k].x = fmaf(-sg, pair_xchg(e[k].x), e[k].x);
        o[k].y = fmaf(-sg, pair_xchg(e[k].y), e[k].y);
    }
}

// NS = 256 pass twiddles of inputs 8h + i: W_4096^{b (8h + i)} = g W^{b i}, g = W_4096^{8 b h}
// (conjugated for DIR > 0).  The bases are re-read (L1) per pass rather than held: the pair
// kernel has 64 VGPRs.
template <int DIR>
__device__ __forceinline__ void pair_rec_twiddle(float2 (&a)[8], const float2 *__restrict__ rec_f,
                                                 const float2 *__restrict__ post8192, int b, int h)
{
    const float2 w1 = rec_f[b], w4 = rec_f[NT + b];
    const float2 g = post8192[16 * b * h];   // 1 on the lo lane
    const float2 gw1 = cmul(g, w1), gw4 = cmul(g, w4);
    const float2 gw2 = cmul(gw1, w1), gw3 = cmul(gw2, w1);
    const float2 gw5 = cmul(gw4, w1), gw6 = cmul(gw5, w1), gw7 = cmul(gw6, w1);
    a[0] = TW<DIR>(a[0], g);
    a[1] = TW<DIR>(a[1], gw1);
    a[2] = TW<DIR>(a[2], gw2);
    a[3] = TW<DIR>(a[3], gw3);
    a[4] = TW<DIR>(a[4], gw4);
    a[5] = TW<DIR>(a[5], gw5);
    a[6] = TW<DIR>(a[6], gw6);
    a[7] = TW<DIR>(a[7], gw7);
}

template <bool RAND, bool NCO, bool CS16>
__global__ __launch_bounds__(NTP, 8) void r2iq_pair_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes, const float2 *__restrict__ tw_p1,
    const float2 *__restrict__ rec_f, const float2 *__restrict__ post8192, const float4 *__restrict__ pq,
    int tunebin, OutArgs oa, NcoArgs nco)
{
    constexpr int N = HALF;
    __shared__ __attribute__((aligned(16))) float2 lds[HALF];
    // pass-1 twiddles W_256^{(b%16) s} at [s][b%16], row 0 = 1 (both lanes run the same code)
    __shared__ __attribute__((aligned(16))) float2 twl[16 * 16];

    const int tid = (int)threadIdx.x;
    const int G = (int)gridDim.x, w = (int)blockIdx.x;
    const int f0 = (int)(((long long)nframes * w) / G);
    const int f1 = (int)(((long long)nframes * (w + 1)) / G);
    if (f0 >= f1) return;

    for (int i = tid; i < 16 * 16; i += NTP) twl[i] = i < 16 ? make_float2(1.f, 0.f) : tw_p1[i - 16];
    const int b_ = tid >> 1, h_ = tid & 1;

    int blk = f0 / FRAMES, k = f0 - blk * FRAMES;
    // this lane's 8 int16 pairs of a frame: pair b + 256 (8h + i)
    int x[8];
    auto load = [&](int lb, int lk) {
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(in32 + ((size_t)lb * BLOCK + (size_t)lk * HOP) / 2);
        const unsigned vo = 4u * (unsigned)(b_ + 2048 * h_);
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = buf_load4<SDDC_LD_AUX>(rs, vo, 4u * 256u * i);
    };
    load(blk, k);

    for (int f = f0; f < f1; f++) {
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z;
        const int b = t >> 1, h = t & 1;
        const bool hi = h != 0;
        const float sg = hi ? -1.f : 1.f;
        const float4 *pqz = pq + z;
        const int b15 = b & 15, b7 = (b >> 7) & 1;
        // exchange reads of inputs b + 256 (8h + i): bit 11 of the element is h
        const int rbase = (swz(b) ^ (h << 4)) + 2048 * h;
        const int oblk = blk * 8 * N;
        const int kc = k;
        float2 v[8];
        // ---- forward pass 0 (DIF, NS 1): convert + pair butterfly ----
        {
            float2 a[8];
#pragma unroll
            for (int i = 0; i < 8; i++)
                a[i] = make_float2(derand<RAND>((int)(short)(x[i] & 0xffff)), derand<RAND>(x[i] >> 16));
            pair16_dif<-1>(a, sg, hi, v);
        }
        __syncthreads();
        {
            // E1: element 16b + 2k' + h, bit-4 parity = bit 11 (= b7)
            const int base = (16 * b) ^ (b7 << 4), xr = b15 ^ h;
#pragma unroll
            for (int q = 0; q < 8; q++) lds[base + ((2 * q) ^ xr)] = v[q];
        }
        __syncthreads();
        // ---- forward pass 1 (DIF, NS 16): table twiddles ----
        {
            float2 a[8];
#pragma unroll
            for (int i = 0; i < 8; i++) a[i] = lds[rbase + 256 * i];
            const int tb = 128 * h + b15;
#pragma unroll
            for (int i = 0; i < 8; i++) a[i] = TW<-1>(a[i], twl[tb + 16 * i]);
            pair16_dif<-1>(a, sg, hi, v);
        }
        __syncthreads();
        // E2: element 256 (b >> 4) + b15 + 16 (2k' + h), bit-4 parity = bit 11 (= b7)
        const int base2 = 256 * (b >> 4) + 16 * (h ^ b7), x2 = b15 ^ h;
#pragma unroll
        for (int q = 0; q < 8; q++) lds[base2 + 32 * q + ((2 * q) ^ x2)] = v[q];
        __syncthreads();
        // ---- forward pass 2 (DIF, NS 256): recurrence twiddles -> Z ----
        {
            float2 a[8];
#pragma unroll
            for (int i = 0; i < 8; i++) a[i] = lds[rbase + 256 * i];
            pair_rec_twiddle<-1>(a, rec_f, post8192, b, h);
            pair16_dif<-1>(a, sg, hi, v);
        }
        __syncthreads();
        {
            // Z: element b + 256 (2k' + h), bit-4 parity = bit 8 (= h)
            const int zb = (swz(b) ^ (h << 4)) + 256 * h;
#pragma unroll
            for (int q = 0; q < 8; q++) lds[zb + 512 * q] = v[q];
        }
        __syncthreads();
        // ---- inverse pass 0 (DIT, NS 1): split x filter for m = b + 256 (2i + h) ----
        float2 u[8];
        {
            const int jb = (tunebin + b) & (HALF - 1);        // bin of m = b
            const int jm = (HALF - jb) & (HALF - 1);          // its mirror
            // bit 8 of bin jb + 256 (2i + h) is bit 0 of (jb >> 8) + h, for every i
            const unsigned kb = (unsigned)((swz(jb) ^ ((((jb >> 8) + h) & 1) << 4)) + 256 * h);
            const unsigned cb = (unsigned)((swz(jm) ^ ((((jm >> 8) + h) & 1) << 4)) - 256 * h);
            const __amdgpu_buffer_rsrc_t rpq = buf_rsrc(pqz);
            const unsigned pv = 16u * (unsigned)(b + 256 * h);
            float2 a[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                // four (P, Q) loads in flight at a time (VGPR budget of 8 waves/SIMD)
                if (i == 4) asm volatile("" ::: "memory");
                const float2 zk = lds[(kb + 512u * i) & (HALF - 1)];
                const float2 zc = lds[(cb - 512u * i) & (HALF - 1)];
                a[i] = split_pq(zk, zc, buf_load16(rpq, pv, 16u * 512u * i));
            }
            pair16_dit<+1>(a, sg, hi, u);
        }
        // prefetch the next frame here, past this frame's widest register point
        if (++k == FRAMES) {
            k = 0;
            ++blk;
        }
        if (f + 1 < f1) load(blk, k);
        __syncthreads();
        {
            // E4: element 16b + 8h + k, bit-4 parity = bit 3 ^ bit 11 (= h ^ b7)
            const int base = (16 * b) ^ ((h ^ b7) << 4), xr = b15 ^ (8 * h);
#pragma unroll
            for (int q = 0; q < 8; q++) lds[base + (q ^ xr)] = u[q];
        }
        __syncthreads();
        // ---- inverse pass 1 (DIF, NS 16) ----
        {
            // E4 reads: element b + 256 (8h + i), parity = b3 ^ h
            const int rb4 = (swz(b) ^ ((((b >> 3) ^ h) & 1) << 4)) + 2048 * h;
            float2 a[8];
#pragma unroll
            for (int i = 0; i < 8; i++) a[i] = lds[rb4 + 256 * i];
            const int tb = 128 * h + b15;
#pragma unroll
            for (int i = 0; i < 8; i++) a[i] = TW<+1>(a[i], twl[tb + 16 * i]);
            pair16_dif<+1>(a, sg, hi, u);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 8; q++) lds[base2 + 32 * q + ((2 * q) ^ x2)] = u[q];   // E5 = E2's layout
        __syncthreads();
        // ---- inverse pass 2 (DIF, NS 256): overlap-discard write of y[b + 256 (2k' + h)] ----
        {
            float2 a[8];
#pragma unroll
            for (int i = 0; i < 8; i++) a[i] = lds[rbase + 256 * i];
            pair_rec_twiddle<+1>(a, rec_f, post8192, b, h);
            pair16_dif<+1>(a, sg, hi, u);
        }
        {
            const int fbase = oblk + emit_base<N>(kc);
            const __amdgpu_buffer_rsrc_t ro = buf_rsrc(static_cast<char *>(out) + (size_t)fbase * out_bytes<CS16>());
            const int q0 = kc == 0 ? 2 : 0;   // kept r = 2k' + h in [4, 12) or [0, 12)
            const unsigned vo = (unsigned)(b + 256 * h);
#pragma unroll
            for (int q = 0; q < 6; q++) {
                if (q < q0) continue;
                float2 y = flip(u[q], oa.lsbmask);
                if constexpr (NCO) y = nco_mix(y, nco, fbase + (int)vo + 512 * q);
                store_iq<CS16>(y, ro, vo, 512u * q, oa);
            }
        }
    }
}


template <bool RAND, bool NCO, bool CS16>
hipError_t launch_pair(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                       int tunebin, OutArgs oa, NcoArgs nco, int device, hipStream_t s)
{
    auto kern = r2iq_pair_kernel<RAND, NCO, CS16>;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(kern), NTP, device, &occ, &cus);
    if (e != hipSuccess) return e;
    const int nframes = nblk * FRAMES;
    int grid = cus * occ;
    if (grid > nframes) grid = nframes;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NTP), 0, s, reinterpret_cast<const int *>(d_in), d_out,
                       nframes, t.tw_p1, t.rec_f, t.post8192, pq, tunebin, oa, nco);
    return hipGetLastError();
}

template <bool RAND, bool NCO>
hipError_t launch_pair_f(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                         int tunebin, OutArgs oa, NcoArgs nco, int device, hipStream_t s, bool cs16)
{
    return cs16 ? launch_pair<RAND, NCO, true>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s)
                : launch_pair<RAND, NCO, false>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s);
}

}  // namespace

hipError_t launch_frames_pair(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                              int tunebin, int lsb, int rand, int cs16, float cs16_scale, const float2 *nco_starts,
                              const float2 *nco_trig, int device, hipStream_t s)
{
    const OutArgs oa{lsb ? 0x80000000u : 0u, cs16_scale};
    const NcoArgs nco{nco_starts, nco_trig};
    const bool f = cs16 != 0;
    if (rand)
        return nco_starts ? launch_pair_f<true, true>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s, f)
                          : launch_pair_f<true, false>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s, f);
    return nco_starts ? launch_pair_f<false, true>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s, f)
                      : launch_pair_f<false, false>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s, f);
}

}  // namespace sddc
