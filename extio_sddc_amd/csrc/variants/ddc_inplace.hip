// ddc_inplace.hip — d = 0 single-channel kernel with in-place LDS passes (internal variant 7,
// libsddc_ddc_variants.so).  The default kernel's butterflies, twiddles and frame loop, but
// the radix-16 passes whose inputs and outputs can share storage write their outputs back to
// the 16 slots they read, so they need no barrier before the writes: 7 barriers per frame
// instead of 10.
//
// Storage of the Stockham exchange elements (thread t = 16 g + i, register r):
//   forward pass 0 -> 1 and inverse 1 -> 2:  element 16 u + k at (u & 15) + 16 k + 256 (u >> 4)
//     (pass 0 thread u writes register k there; the inverse pass 2 of thread u reads the same
//     16 slots, so the next frame's pass-0 writes follow the last reads of the same thread)
//   forward pass 1 (in place):               reads and writes (t >> 4) + 16 i + 256 r
//   forward pass 2 reads:                    r + 16 i + 256 g
//   Z (forward pass 2 out, split in):        natural order, as the default (barrier-separated)
//   inverse pass 0 -> 1 (pass 1 in place):   natural order 16 t + k / t + 256 r
// with the LDS swizzle phi(p) = p ^ ((p >> 4) & 15) ^ (bit 8 of p) << 4, under which every one
// of these patterns is bank-conflict free (32-lane reads, 16-lane writes) and costs at most
// one XOR or one base select per access.
#include <hip/hip_runtime.h>

#include "ddc_frame_common.hpp"
#include "variants_api.h"

namespace sddc {
namespace {

// one ds_read_b64 per value (no read2st64 pairing), as the default kernel's exchange reads
#define XRD(dst, expr) do { dst = (expr); asm volatile("" ::: "memory"); } while (0)

template <bool RAND, bool NCO, bool CS16>
__global__ __launch_bounds__(NT, 4) void r2iq_inplace_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes, const float2 *__restrict__ tw_p1,
    const float2 *__restrict__ rec_f, const float4 *__restrict__ pq, int tunebin, OutArgs oa, NcoArgs nco)
{
    constexpr int N = HALF;
    __shared__ __attribute__((aligned(16))) float2 lds[HALF];
    __shared__ __attribute__((aligned(16))) float2 twl[15 * 16];

    const int tid = (int)threadIdx.x;
    const int G = (int)gridDim.x, w = (int)blockIdx.x;
    const int f0 = (int)(((long long)nframes * w) / G);
    const int f1 = (int)(((long long)nframes * (w + 1)) / G);
    if (f0 >= f1) return;

    const float2 fw1_ = rec_f[tid], fw4_ = rec_f[NT + tid];
    for (int i = tid; i < 15 * 16; i += NT) twl[i] = tw_p1[i];
    __syncthreads();

    int blk = f0 / FRAMES, k = f0 - blk * FRAMES;
    int x[16];
    load_frame(in32, blk, k, x);

    for (int f = f0; f < f1; f++) {
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z;
        const float4 *pqz = pq + z;
        float2 fw1 = fw1_, fw4 = fw4_;
        asm volatile("" : "+v"(fw1), "+v"(fw4));
        const int i = t & 15, g = t >> 4, gb = g & 1;
        const int oblk = blk * 8 * N;
        const int kc = k;
        // slots of the pass 0 -> 1 / inverse 1 -> 2 layout: 256 g + ((17 r) ^ xa)
        const int abase = 256 * g, xa = i ^ (gb << 4);
        float2 v[16];
        // ---- forward pass 0: convert + DFT16, written to the slots this thread read last frame ----
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
#pragma unroll
        for (int r = 0; r < 16; r++) lds[abase + ((17 * r) ^ xa)] = v[r];
        __syncthreads();
        // ---- forward pass 1 (NS 16), in place at (t >> 4) + 16 i + 256 r ----
        {
            const int b0 = 16 * i + (g ^ i), b1 = b0 ^ 16;
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], lds[((r & 1) ? b1 : b0) + 256 * r]);
#pragma unroll
            for (int r = 1; r < 16; r++) a[r] = TW<-1>(a[r], twl[(r - 1) * 16 + i]);
            dft16<-1>(a, v);
#pragma unroll
            for (int r = 0; r < 16; r++) lds[((r & 1) ? b1 : b0) + 256 * r] = v[r];
        }
        __syncthreads();
        // ---- forward pass 2 (NS 256): reads r + 16 i + 256 g, writes Z in natural order ----
        {
            const int cb = 256 * g + 16 * (i ^ gb);
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], lds[cb + (r ^ i)]);
            twiddle_rec16<-1>(a, fw1, fw4);
            dft16<-1>(a, v);
        }
        __syncthreads();
        {
            const int sT = swz(t);
#pragma unroll
            for (int r = 0; r < 16; r++) lds[sT + NT * r] = v[r];
        }
        __syncthreads();
        // ---- inverse pass 0: split x filter for bins tb + t + 256 r, DFT16 ----
        float2 u[16];
        {
            const int b0 = tunebin + t;
            const int sb0 = swz(b0), sc0 = swz(HALF - b0);
            const char *lb = reinterpret_cast<const char *>(lds);
            const unsigned sb0b = 8u * (unsigned)sb0, sc0b = 8u * (unsigned)sc0, tb16 = 16u * (unsigned)t;
            const __amdgpu_buffer_rsrc_t rpq = buf_rsrc(pqz);
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int sh = NT * r - (NT * r >= N / 2 ? N : 0);
                const float2 zk = *reinterpret_cast<const float2 *>(lb + ((sb0b + 8u * (unsigned)sh) & (8u * HALF - 8u)));
                const float2 zc = *reinterpret_cast<const float2 *>(lb + ((sc0b - 8u * (unsigned)sh) & (8u * HALF - 8u)));
                a[r] = split_pq(zk, zc, buf_load16(rpq, tb16, 16u * NT * r));
            }
            dft16<+1>(a, u);
        }
        __syncthreads();
        {
            const int cb = 256 * g + 16 * (i ^ gb);   // element 16 t + r, natural order
#pragma unroll
            for (int r = 0; r < 16; r++) lds[cb + (r ^ i)] = u[r];
        }
        __syncthreads();
        // ---- inverse pass 1 (NS 16), in place at t + 256 r ----
        {
            const int e0 = 16 * g + (i ^ g), e1 = e0 ^ 16;
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], lds[((r & 1) ? e1 : e0) + 256 * r]);
#pragma unroll
            for (int r = 1; r < 16; r++) a[r] = TW<+1>(a[r], twl[(r - 1) * 16 + i]);
            dft16<+1>(a, u);
#pragma unroll
            for (int r = 0; r < 16; r++) lds[((r & 1) ? e1 : e0) + 256 * r] = u[r];
        }
        __syncthreads();
        // ---- inverse pass 2 (NS 256): reads the pass 0 -> 1 slots, overlap-discard store ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], lds[abase + ((17 * r) ^ xa)]);
            twiddle_rec16<+1>(a, fw1, fw4);
            dft16<+1>(a, u);
            emit_frame<N / 16, NCO, CS16>(out, oblk + emit_base<N>(kc), kc, t, u, oa, nco);
        }
    }
}


template <bool RAND, bool NCO, bool CS16>
hipError_t launch_inplace(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                          int tunebin, OutArgs oa, NcoArgs nco, int device, hipStream_t s)
{
    auto kern = r2iq_inplace_kernel<RAND, NCO, CS16>;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(kern), NT, device, &occ, &cus);
    if (e != hipSuccess) return e;
    const int nframes = nblk * FRAMES;
    int grid = cus * occ;
    if (grid > nframes) grid = nframes;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, s, reinterpret_cast<const int *>(d_in), d_out, nframes,
                       t.tw_p1, t.rec_f, pq, tunebin, oa, nco);
    return hipGetLastError();
}

template <bool RAND, bool NCO>
hipError_t launch_inplace_f(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                            int tunebin, OutArgs oa, NcoArgs nco, int device, hipStream_t s, bool cs16)
{
    return cs16 ? launch_inplace<RAND, NCO, true>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s)
                : launch_inplace<RAND, NCO, false>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s);
}

}  // namespace

hipError_t launch_frames_inplace(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                                 int tunebin, int lsb, int rand, int cs16, float cs16_scale, const float2 *nco_starts,
                                 const float2 *nco_trig, int device, hipStream_t s)
{
    const OutArgs oa{lsb ? 0x80000000u : 0u, cs16_scale};
    const NcoArgs nco{nco_starts, nco_trig};
    const bool f = cs16 != 0;
    if (rand)
        return nco_starts ? launch_inplace_f<true, true>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s, f)
                          : launch_inplace_f<true, false>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s, f);
    return nco_starts ? launch_inplace_f<false, true>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s, f)
                      : launch_inplace_f<false, false>(t, d_in, nblk, d_out, pq, tunebin, oa, nco, device, s, f);
}

}  // namespace sddc
