// ddc_variants.hip — the measured-slower d = 0 layouts of the single-channel kernel, kept for
// A/B timing outside the product library (libsddc_ddc_variants.so, selected through
// sddc_ddc_internal_set_variant; DESIGN.md §4.1 has their measurements):
//   variant 4  r2iq_pipe_kernel  two frames in flight per workgroup (3 exchanges per frame, 2 waves/SIMD)
//   variant 5  r2iq_r8_kernel    radix 8 x 512 threads per frame (7 exchanges, 8 waves/SIMD)
// Same frame algorithm, tables and output stage as the default r2iq_persistent_kernel
// (ddc_persistent.hip, helpers in ddc_frame_common.hpp).
#include <hip/hip_runtime.h>

#include "ddc_frame_common.hpp"
#include "variants_api.h"

namespace sddc {
namespace {

// d = 0, two frames in flight per workgroup (internal variant 4).  Iteration f runs the forward
// FFT of frame f and the inverse of frame f - 1 pass by pass, so one LDS exchange (write,
// barrier, read) serves both: 3 exchanges and 6 barriers per frame instead of 5 and 10, and
// every wave carries two independent dependency chains between barriers.  Forward passes
// live in buffer P (Z stays there for the next iteration's split), inverse passes in Q:
// 64 KB + 3.8 KB per workgroup, 2 workgroups (2 waves/SIMD) per CU.  The pipeline fill and
// drain compute one garbage half each (uninitialised Z; stale input), never stored.
#ifndef SDDC_PIPE_WAVES
#define SDDC_PIPE_WAVES 2
#endif
template <bool RAND, bool NCO, bool CS16>
__global__ __launch_bounds__(NT, SDDC_PIPE_WAVES) void r2iq_pipe_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes, const float2 *__restrict__ tw_p1,
    const float2 *__restrict__ tw_q1, const float2 *__restrict__ rec_f, const float4 *__restrict__ pq,
    int tunebin, OutArgs oa, NcoArgs nco)
{
    constexpr int N = HALF;
    __shared__ __attribute__((aligned(16))) float2 P[HALF];
    __shared__ __attribute__((aligned(16))) float2 Q[HALF];
    __shared__ __attribute__((aligned(16))) float2 twl[2 * 15 * 16];

    const int tid = (int)threadIdx.x;
    const int G = (int)gridDim.x, w = (int)blockIdx.x;
    const int f0 = (int)(((long long)nframes * w) / G);
    const int f1 = (int)(((long long)nframes * (w + 1)) / G);
    if (f0 >= f1) return;

    const float2 fw1_ = rec_f[tid], fw4_ = rec_f[NT + tid];
    for (int i = tid; i < 2 * 15 * 16; i += NT) twl[i] = i < 15 * 16 ? tw_p1[i] : tw_q1[i - 15 * 16];

    int blk = f0 / FRAMES, k = f0 - blk * FRAMES;   // forward frame
    int gblk = blk, gk = k;                          // inverse frame (one behind)
    int x[16];
    load_frame(in32, blk, k, x);

    for (int f = f0; f <= f1; f++) {
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z;
        const float4 *pqz = pq + z;
        float2 fw1 = fw1_, fw4 = fw4_;
        asm volatile("" : "+v"(fw1), "+v"(fw4));
        const int sT = swz(t);
        const int x15 = t & 15;
        const int b1 = (t >> 4) * 256;
        float2 v[16], u[16];
        // ---- phase 0: forward pass 0 of f (input registers) | split x filter + inverse pass 0 of f-1 ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++)
                a[r] = make_float2(derand<RAND>((int)(short)(x[r] & 0xffff)), derand<RAND>(x[r] >> 16));
            if (++k == FRAMES) {
                k = 0;
                ++blk;
            }
            if (f + 1 < f1) load_frame(in32, blk, k, x);
            dft16<-1>(a, v);
        }
        {
            const int b0 = tunebin + t;
            const unsigned sb0b = 8u * (unsigned)swz(b0), sc0b = 8u * (unsigned)swz(HALF - b0);
            const unsigned tb16 = 16u * (unsigned)t;
            const char *pb = reinterpret_cast<const char *>(P);
            const __amdgpu_buffer_rsrc_t rpq = buf_rsrc(pqz);
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int sh = NT * r - (NT * r >= N / 2 ? N : 0);
                const float2 zk = *reinterpret_cast<const float2 *>(pb + ((sb0b + 8u * (unsigned)sh) & (8u * HALF - 8u)));
                const float2 zc = *reinterpret_cast<const float2 *>(pb + ((sc0b - 8u * (unsigned)sh) & (8u * HALF - 8u)));
                a[r] = split_pq(zk, zc, buf_load16(rpq, tb16, 16u * NT * r));
            }
            dft16<+1>(a, u);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; r++) {
            P[16 * t + (r ^ x15)] = v[r];
            Q[16 * t + (r ^ x15)] = u[r];
        }
        __syncthreads();
        // ---- phase 1: pass 1 of both (table twiddles W_256^{(t%16) r}) ----
        {
            float2 a[16], c[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                a[r] = P[sT + NT * r];
                c[r] = Q[sT + NT * r];
            }
#pragma unroll
            for (int r = 1; r < 16; r++) {
                a[r] = TW<-1>(a[r], twl[(r - 1) * 16 + x15]);
                c[r] = TW<+1>(c[r], twl[15 * 16 + (r - 1) * 16 + x15]);
            }
            dft16<-1>(a, v);
            dft16<+1>(c, u);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; r++) {
            P[b1 + 16 * r + (x15 ^ r)] = v[r];
            Q[b1 + 16 * r + (x15 ^ r)] = u[r];
        }
        __syncthreads();
        // ---- phase 2: forward pass 2 of f -> Z | inverse pass 2 of f-1 -> overlap-discard store ----
        {
            float2 a[16], c[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                a[r] = P[sT + NT * r];
                c[r] = Q[sT + NT * r];
            }
            twiddle_rec16<-1>(a, fw1, fw4);
            twiddle_rec16<+1>(c, fw1, fw4);
            dft16<-1>(a, v);
            dft16<+1>(c, u);
        }
        if (f > f0) {
            emit_frame<N / 16, NCO, CS16>(out, gblk * 8 * N + emit_base<N>(gk), gk, t, u, oa, nco);
            if (++gk == FRAMES) {
                gk = 0;
                ++gblk;
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; r++) P[sT + NT * r] = v[r];   // Z, natural order
        __syncthreads();
    }
}

// d = 0, radix 8, 512 threads (8 waves) per frame (internal variant 5).  The same frame in
// the same 32 KB of LDS, split over twice the waves: 8 points per thread, 4096 = 8^4, so
// 7 LDS exchanges per frame instead of 5, at <= 64 VGPRs so that 4 workgroups (8 waves per
// SIMD) are resident instead of 4 waves.  A wave issues VALU at most every ~4-5 cycles and the
// SIMD needs >= 2 ready waves to reach its rate (profiles/r01/microbench_valu.txt); this
// variant tests whether more resident waves beat fewer exchanges.
// Stockham pass p (NS = 8^p): thread j reads j + 512 r, applies W_{8 NS}^{(j mod NS) r},
// writes (j / NS) 8 NS + (j mod NS) + NS r.  LDS swizzle sw8 below: conflict-free (32 lanes
// of ds_*_b64) for the pass-0 and pass-1 writes, and sw8(e + 512 r) = sw8(e) + 512 r.
constexpr int NT8 = 512;
#ifndef SDDC_R8_WAVES
#define SDDC_R8_WAVES 8
#endif
__device__ __forceinline__ int sw8(int e) { return e ^ ((e >> 5) & 7) ^ ((e >> 3) & 24); }

// a[r] *= W^{r} for r = 1..7 given the forward-direction W^1 and W^4 of this lane
template <int DIR>
__device__ __forceinline__ void twiddle_rec8(float2 *a, float2 w1, float2 w4)
{
    if (DIR > 0) {
        w1.y = -w1.y;
        w4.y = -w4.y;
    }
    const float2 w2 = cmul(w1, w1), w3 = cmul(w2, w1);
    a[1] = cmul(a[1], w1);
    a[2] = cmul(a[2], w2);
    a[3] = cmul(a[3], w3);
    a[4] = cmul(a[4], w4);
    a[5] = cmul(a[5], cmul(w4, w1));
    a[6] = cmul(a[6], cmul(w4, w2));
    a[7] = cmul(a[7], cmul(w4, w3));
}

__device__ __forceinline__ void load_frame8(const int *__restrict__ in32, int blk, int k, int (&x)[8])
{
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(in32 + ((size_t)blk * BLOCK + (size_t)k * HOP) / 2);
    const unsigned vo = 4u * threadIdx.x;
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = buf_load4<SDDC_LD_AUX>(rs, vo, 4u * NT8 * r);
}

// kept outputs n = t + 512 r of frame k: r in [2, 6) for k = 0, [0, 6) otherwise
template <bool NCO, bool CS16>
__device__ __forceinline__ void emit_frame8(void *__restrict__ out, int fbase, int k, int t, const float2 (&u)[8],
                                            const OutArgs &oa, const NcoArgs &nco)
{
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(static_cast<char *>(out) + (size_t)fbase * out_bytes<CS16>());
    const int r0 = k == 0 ? 2 : 0;   // wave-uniform
#pragma unroll
    for (int r = 0; r < 6; r++) {
        if (r < r0) continue;
        float2 v = flip(u[r], oa.lsbmask);
        if constexpr (NCO) v = nco_mix(v, nco, fbase + t + NT8 * r);
        store_iq<CS16>(v, ro, (unsigned)t, (unsigned)(NT8 * r), oa);
    }
}

template <bool RAND, bool NCO, bool CS16>
__global__ __launch_bounds__(NT8, SDDC_R8_WAVES) void r2iq_r8_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes, const float2 *__restrict__ post8192,
    const float4 *__restrict__ pq, int tunebin, OutArgs oa, NcoArgs nco)
{
    constexpr int N = HALF;
    __shared__ __attribute__((aligned(16))) float2 lds[HALF];
    // pass-1 twiddles W_64^{(j%8) r} at [r-1][j%8], pass-2 twiddles W_512^{(j%64) r} at 56 + [r-1][j%64]
    __shared__ __attribute__((aligned(16))) float2 twl[7 * 8 + 7 * 64];

    const int tid = (int)threadIdx.x;
    const int G = (int)gridDim.x, w = (int)blockIdx.x;
    const int f0 = (int)(((long long)nframes * w) / G);
    const int f1 = (int)(((long long)nframes * (w + 1)) / G);
    if (f0 >= f1) return;

    const float2 fw1_ = post8192[2 * tid], fw4_ = post8192[8 * tid];   // W_4096^t, W_4096^{4t}
    for (int i = tid; i < 7 * 8 + 7 * 64; i += NT8) {
        const int m = i < 56 ? 128 * (i & 7) * (i / 8 + 1) : 16 * ((i - 56) & 63) * ((i - 56) / 64 + 1);
        twl[i] = post8192[m];
    }

    int blk = f0 / FRAMES, k = f0 - blk * FRAMES;
    int x[8];
    load_frame8(in32, blk, k, x);

    for (int f = f0; f < f1; f++) {
        int z = 0;
        asm volatile("" : "+s"(z));
        int t = tid + z;
        const float4 *pqz = pq + z;
        float2 fw1 = fw1_, fw4 = fw4_;
        asm volatile("" : "+v"(fw1), "+v"(fw4));
        int sT = sw8(t);
        const int oblk = blk * 8 * N;
        const int kc = k;
        float2 v[8];
        // ---- forward pass 0 (NS 1): convert + DFT8 ----
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++)
                a[r] = make_float2(derand<RAND>((int)(short)(x[r] & 0xffff)), derand<RAND>(x[r] >> 16));
            if (++k == FRAMES) {
                k = 0;
                ++blk;
            }
            if (f + 1 < f1) load_frame8(in32, blk, k, x);
            dft8<-1>(a, v);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(8 * t + r)] = v[r];
        __syncthreads();
        // ---- forward passes 1 (NS 8) and 2 (NS 64): table twiddles ----
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
#pragma unroll
            for (int r = 1; r < 8; r++) a[r] = TW<-1>(a[r], twl[(r - 1) * 8 + (t & 7)]);
            dft8<-1>(a, v);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(64 * (t >> 3) + (t & 7) + 8 * r)] = v[r];
        __syncthreads();
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
#pragma unroll
            for (int r = 1; r < 8; r++) a[r] = TW<-1>(a[r], twl[56 + (r - 1) * 64 + (t & 63)]);
            dft8<-1>(a, v);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(512 * (t >> 6) + (t & 63) + 64 * r)] = v[r];
        __syncthreads();
        // ---- forward pass 3 (NS 512): recurrence twiddles W_4096^{t r} -> Z, natural order ----
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
            twiddle_rec8<-1>(a, fw1, fw4);
            dft8<-1>(a, v);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sT + NT8 * r] = v[r];
        __syncthreads();
        // ---- inverse pass 0: split x filter for bins tb + t + 512 r (- 4096 for r >= 4) ----
        // (a fresh opaque thread index: the inverse recomputes its LDS addresses instead of
        // keeping the forward passes' 24 live across them)
        asm volatile("" : "+s"(z));
        t = tid + z;
        sT = sw8(t);
        float2 u[8];
        {
            const int b0 = tunebin + t;
            const unsigned sb0 = (unsigned)sw8(b0 & (HALF - 1)), sc0 = (unsigned)sw8((HALF - b0) & (HALF - 1));
            const __amdgpu_buffer_rsrc_t rpq = buf_rsrc(pqz);
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const float2 zk = lds[(sb0 + NT8 * r) & (HALF - 1)];
                const float2 zc = lds[(sc0 - NT8 * r) & (HALF - 1)];
                a[r] = split_pq(zk, zc, buf_load16(rpq, 16u * (unsigned)t, 16u * NT8 * r));
            }
            dft8<+1>(a, u);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(8 * t + r)] = u[r];
        __syncthreads();
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
#pragma unroll
            for (int r = 1; r < 8; r++) a[r] = TW<+1>(a[r], twl[(r - 1) * 8 + (t & 7)]);
            dft8<+1>(a, u);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(64 * (t >> 3) + (t & 7) + 8 * r)] = u[r];
        __syncthreads();
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
#pragma unroll
            for (int r = 1; r < 8; r++) a[r] = TW<+1>(a[r], twl[56 + (r - 1) * 64 + (t & 63)]);
            dft8<+1>(a, u);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(512 * (t >> 6) + (t & 63) + 64 * r)] = u[r];
        __syncthreads();
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
            twiddle_rec8<+1>(a, fw1, fw4);
            dft8<+1>(a, u);
        }
        emit_frame8<NCO, CS16>(out, oblk + emit_base<N>(kc), kc, t, u, oa, nco);
    }
}


struct Launch {
    const int16_t *d_in;
    int nblk;
    void *d_out;
    const float4 *pq;
    int tunebin;
    int device;
    hipStream_t s;
    OutArgs oa;
    NcoArgs nco;
};


template <bool RAND, bool NCO, bool CS16>
hipError_t launch_pipe(const KernelTables &t, const Launch &L)
{
    auto kern = r2iq_pipe_kernel<RAND, NCO, CS16>;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(kern), NT, L.device, &occ, &cus);
    if (e != hipSuccess) return e;
    const int nframes = L.nblk * FRAMES;
    int grid = cus * occ;
    if (grid > nframes) grid = nframes;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, L.s, reinterpret_cast<const int *>(L.d_in), L.d_out,
                       nframes, t.tw_p1, t.tw_q1[0], t.rec_f, L.pq, L.tunebin, L.oa, L.nco);
    return hipGetLastError();
}

template <bool RAND, bool NCO>
hipError_t launch_pipe_f(const KernelTables &t, const Launch &L, bool cs16)
{
    return cs16 ? launch_pipe<RAND, NCO, true>(t, L) : launch_pipe<RAND, NCO, false>(t, L);
}


template <bool RAND, bool NCO, bool CS16>
hipError_t launch_r8(const KernelTables &t, const Launch &L)
{
    auto kern = r2iq_r8_kernel<RAND, NCO, CS16>;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(kern), NT8, L.device, &occ, &cus);
    if (e != hipSuccess) return e;
    const int nframes = L.nblk * FRAMES;
    int grid = cus * occ;
    if (grid > nframes) grid = nframes;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT8), 0, L.s, reinterpret_cast<const int *>(L.d_in), L.d_out,
                       nframes, t.post8192, L.pq, L.tunebin, L.oa, L.nco);
    return hipGetLastError();
}

template <bool RAND, bool NCO>
hipError_t launch_r8_f(const KernelTables &t, const Launch &L, bool cs16)
{
    return cs16 ? launch_r8<RAND, NCO, true>(t, L) : launch_r8<RAND, NCO, false>(t, L);
}

}  // namespace

hipError_t launch_frames_r8(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                            int tunebin, int lsb, int rand, int cs16, float cs16_scale, const float2 *nco_starts,
                            const float2 *nco_trig, int device, hipStream_t s)
{
    const Launch L{d_in, nblk, d_out, pq, tunebin, device, s, OutArgs{lsb ? 0x80000000u : 0u, cs16_scale},
                   NcoArgs{nco_starts, nco_trig}};
    const bool f = cs16 != 0, nco = nco_starts != nullptr;
    if (rand) return nco ? launch_r8_f<true, true>(t, L, f) : launch_r8_f<true, false>(t, L, f);
    return nco ? launch_r8_f<false, true>(t, L, f) : launch_r8_f<false, false>(t, L, f);
}

hipError_t launch_frames_pipelined(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out,
                                   const float4 *pq, int tunebin, int lsb, int rand, int cs16, float cs16_scale,
                                   const float2 *nco_starts, const float2 *nco_trig, int device, hipStream_t s)
{
    const Launch L{d_in, nblk, d_out, pq, tunebin, device, s, OutArgs{lsb ? 0x80000000u : 0u, cs16_scale},
                   NcoArgs{nco_starts, nco_trig}};
    const bool f = cs16 != 0, nco = nco_starts != nullptr;
    if (rand) return nco ? launch_pipe_f<true, true>(t, L, f) : launch_pipe_f<true, false>(t, L, f);
    return nco ? launch_pipe_f<false, true>(t, L, f) : launch_pipe_f<false, false>(t, L, f);
}

}  // namespace sddc

extern "C" const sddc_variants_api *sddc_variants_get(void)
{
    static const sddc_variants_api api = {
        SDDC_VARIANTS_API_VERSION, sddc::launch_frames,    sddc::launch_channels,    sddc::launch_frames_pipelined,
        sddc::launch_frames_r8,    sddc::launch_build_wave_tables, sddc::launch_frames_wave,
        sddc::launch_frames_pair,  sddc::launch_frames_inplace,
    };
    return &api;
}
