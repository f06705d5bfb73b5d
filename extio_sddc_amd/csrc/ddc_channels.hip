// ddc_channels.hip — many-channel DDC for gfx950 (up to 1024
// tune offsets of one stream).  r2iq_channels_v2_kernel covers d >= 4 (mfft N <= 256),
// r2iq_channels_p_kernel (below) d = 0..3.
//
// v2: work item = (frame, chunk of <= 128 channels).  Per item the workgroup computes the
// frame's forward transform ONCE (as ddc_persistent.hip: 3 x radix-16 Stockham in 32 KB
// of swizzled LDS, int16 -> float with optional RAND), then walks the chunk G = 256/TPC
// channels at a time, TPC = N/16 threads per channel:
//   split   the r2c split X2[bin] = (Z_k + conj Z_-k) - i W_8192^bin (Z_k - conj Z_-k) once per
//           item, for the bins the chunk's channels read (fft_mt_r2iq_impl.hpp:88 gives X)
//   pass A  filter multiply X2[tb + m] * H[m]/2 for the channel's N bins around its tune bin
//           (Core/fft_mt_r2iq_impl.hpp:76-96), DFT-16 in registers, -> per-channel LDS slice
//   pass B  radix-(N/16) Stockham step with W_256 twiddles from LDS, overlap-discard
//           write of the kept outputs to the channel's stream (impl.hpp:117-138)
// Channel c's output stream starts at complex element c * stride of out (CF32 or CS16).  Persistent grid:
// CUs x resident workgroups, contiguous item ranges.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "ddc_kernels.h"
#include "fft_device.hpp"
#include "ddc_device_io.hpp"

namespace sddc {
namespace {

constexpr int NT = 256;
constexpr int HALF = 4096;
constexpr int HOP = 6144;
constexpr int BLOCK = 65536;
constexpr int FRAMES = 11;
constexpr int CHUNK = 128;    // channels per work item
constexpr int ZC_MAX = 1536;  // compact window of split bins per chunk

__device__ __forceinline__ int swz(int e) { return e ^ ((e >> 4) & 15); }
// Swizzled element Lane + R with no carry between the two (disjoint bits): swz is linear over
// XOR, swz(Lane ^ R) = swz(Lane) ^ swz(R), so the byte address is 8 swz(Lane) ^ 8 swz(R), one
// v_xor_b32 with an immediate per access (8 swz(Lane) is formed once) instead of the add, shift,
// xor-and-mask and scale of the index form (as ddc_persistent.hip's inverse passes).  Here
// neutral (C5 +-0.1 %, 128 channels +0.3 %), bit-identical (profiles/r02/ab/chlx_*.txt).
__device__ __forceinline__ float2 &lds_x(float2 *buf, unsigned lane8, int R)
{
    return *reinterpret_cast<float2 *>(reinterpret_cast<char *>(buf) + (lane8 ^ (8u * (unsigned)swz(R))));
}
#define LX(buf, lane, R) lds_x(buf, 8u * (unsigned)swz(lane), R)

#ifndef SDDC_CH_NT
#define SDDC_CH_NT 1          // non-temporal IQ stores
#endif
// N <= STAGE_MAX_N (d = 5, 6): stage the IQ through the channel slices, 16-B stores.  At d = 4
// (128-B pieces already) staging measured 2 % slower for C5 (profiles/r02/channels/ab_stage_d4_*).
constexpr int STAGE_MAX_N = 128;
#ifndef SDDC_CH_WAVESYNC
#define SDDC_CH_WAVESYNC 1   // the per-channel exchange is wave-local: order it within the wave only
#endif

// A channel's TPC threads are consecutive lanes of one wave and only they touch its slice of
// `work`, so the pass A -> pass B exchange (and the WAR before the next group) needs program
// order within the wave, not a workgroup barrier.  LDS operations of a wave execute in order.
__device__ __forceinline__ void channel_sync()
{
    if constexpr (SDDC_CH_WAVESYNC) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

template <bool RAND>
__device__ __forceinline__ float derand(int v)
{
    const float f = (float)v;
    if constexpr (!RAND) return f;
    return __int_as_float(__float_as_int(f) ^ (v << 31));   // odd int16 ^ 0xFFFE == -v
}

// 2 X[k] = (Z_k + conj Z_-k) - i W_8192^k (Z_k - conj Z_-k), Z = FFT4096(x_even + i x_odd)
__device__ __forceinline__ float2 split2(float2 zk, float2 zc, float2 wk)
{
    const float2 A = make_float2(zk.x + zc.x, zk.y - zc.y);
    const float2 Bi = make_float2(zk.y + zc.y, zc.x - zk.x);   // (Zk - conj Zc)/i
    return cadd(A, cmul(Bi, wk));
}

// The r2c split is evaluated once per item and shared by the chunk's channels: a channel bin
// then costs one LDS read and one complex multiply (it was two reads and ~20 VALU per channel).
// COMPACT: the split spectrum of the chunk's bins [lo, lo + w) (host-checked to fit ZC_MAX)
// goes into a window xw with N/2 zeros either side, so every channel bin, in band or not, reads
// xw[bin - lo + N/2] without a range test; the per-channel slices reuse the transform buffer
// (3 workgroups per CU).  Otherwise the split is done in place over all 4096 bins.
template <int D, bool RAND, bool CS16, bool COMPACT, bool STAGE_OK>
__global__ __launch_bounds__(NT, 2) void r2iq_channels_v2_kernel(
    const int *__restrict__ in32, void *__restrict__ out, size_t stride, int nframes,
    const int *__restrict__ tunebins, int nch, const float2 *__restrict__ tw_p1,
    const float2 *__restrict__ rec_f, const float2 *__restrict__ post8192, const float2 *__restrict__ hsel,
    OutArgs oa, const int2 *__restrict__ windows, float2 *__restrict__ scratch)
{
    constexpr int N = HALF >> D;
    static_assert(N <= 256 && N >= 64, "channels v2 covers d = 4..6");
    constexpr int TPC = N / 16;          // threads per channel
    constexpr int G = NT / TPC;          // channels in flight
    constexpr int RB = N / 16;           // pass-B radix
    constexpr int BPT = 16 / TPC;        // pass-B butterflies per thread
    // d = 5, 6: stage the stores through LDS (needs 16-B aligned channel rows: STAGE_OK)
    constexpr bool STAGE = STAGE_OK && N <= STAGE_MAX_N;

    static_assert(G * N == HALF, "per-channel slices fill exactly one transform buffer");
    __shared__ __attribute__((aligned(16))) float2 zbuf[COMPACT ? HALF + ZC_MAX + N : 2 * HALF];
    float2 *const zl = zbuf;                              // forward transform, then (!COMPACT) X2
    float2 *const work = COMPACT ? zbuf : zbuf + HALF;    // channel slices (reuse zl when COMPACT)
    float2 *const xw = zbuf + HALF;                       // COMPACT: [N/2 zeros | X2 window | N/2 zeros]
    __shared__ __attribute__((aligned(16))) float2 twl[15 * 16];

    const int tid = (int)threadIdx.x;
    const int nchunks = (nch + CHUNK - 1) / CHUNK;
    const long long items = (long long)nframes * nchunks;
    const int i0 = (int)(items * blockIdx.x / gridDim.x), i1 = (int)(items * (blockIdx.x + 1) / gridDim.x);
    if (i0 >= i1) return;
    // COMPACT with several chunks per frame: the frame's full X2 goes to this workgroup's
    // scratch row once, and the frame's later chunks (the next items of the contiguous range)
    // fill their windows from it instead of redoing the forward transform
    const bool reuse = COMPACT && scratch != nullptr && nchunks > 1;   // uniform
    float2 *const scr = reuse ? scratch + (size_t)blockIdx.x * HALF : nullptr;
    int zf = -1;
    for (int i = tid; i < 15 * 16; i += NT) twl[i] = tw_p1[i];
    const float2 fw1_ = rec_f[tid], fw4_ = rec_f[NT + tid];
    const int l_ = tid % TPC, g_ = tid / TPC;
    float2 hr[16];   // this thread's filter taps H[m]/2, m = l + TPC r, for every channel and frame
#pragma unroll
    for (int r = 0; r < 16; r++) hr[r] = hsel[l_ + TPC * r];

    for (int it = i0; it < i1; it++) {
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z, l = l_ + z, g = g_ + z;
        float2 fw1 = fw1_, fw4 = fw4_;
        asm volatile("" : "+v"(fw1), "+v"(fw4));
        const int f = it / nchunks, chunk = it - f * nchunks;
        const int blk = f / FRAMES, k = f - blk * FRAMES;
        const int sT = swz(t), x15 = t & 15;
        const bool fresh = !reuse || f != zf;
        if (fresh) {
        zf = f;
        // ---------------- forward: Z = FFT4096(x_even + i x_odd) in zl ----------------
        float2 v[16];
        {
            const int *p = in32 + ((size_t)blk * BLOCK + (size_t)k * HOP) / 2 + t;
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int w = p[NT * r];
                a[r] = make_float2(derand<RAND>((int)(short)(w & 0xffff)), derand<RAND>(w >> 16));
            }
            dft16<-1>(a, v);
        }
        __syncthreads();   // previous item's readers of zl / twl done
#pragma unroll
        for (int r = 0; r < 16; r++) zl[16 * t + (r ^ x15)] = v[r];
        __syncthreads();
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) a[r] = zl[sT + NT * r];
#pragma unroll
            for (int r = 1; r < 16; r++) a[r] = cmul(a[r], twl[(r - 1) * 16 + x15]);
            dft16<-1>(a, v);
        }
        __syncthreads();
        {
            const int b1 = (t >> 4) * 256;
#pragma unroll
            for (int r = 0; r < 16; r++) zl[b1 + 16 * r + (x15 ^ r)] = v[r];
        }
        __syncthreads();
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) a[r] = zl[sT + NT * r];
            twiddle_rec16<-1>(a, fw1, fw4);
            dft16<-1>(a, v);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; r++) zl[sT + NT * r] = v[r];
        __syncthreads();
        if (!COMPACT || reuse) {
            // in place over all bins: thread-owned pairs (k, 4096 - k)
            for (int k0 = t; k0 <= HALF / 2; k0 += NT) {
                const int k1 = (HALF - k0) & (HALF - 1);
                const float2 z0 = zl[swz(k0)], z1 = zl[swz(k1)];
                const float2 x0 = split2(z0, z1, post8192[k0]), x1 = split2(z1, z0, post8192[k1]);
                zl[swz(k0)] = x0;
                if (k1 != k0) zl[swz(k1)] = x1;
                if (reuse) {
                    scr[k0] = x0;
                    if (k1 != k0) scr[k1] = x1;
                }
            }
            __syncthreads();
        }
        } else {
            __syncthreads();   // the previous item's readers of xw are done
        }
        int lo = 0;
        if constexpr (COMPACT) {
            // X2 of bins [lo, lo + w1) of this chunk's channels at xw[N/2 + bin - lo]
            const int2 wv = windows[chunk];
            lo = wv.x;
            const int w1 = wv.y;
            for (int i = t; i < w1 + N; i += NT) {
                const int bin = lo + i - N / 2;
                float2 x2 = make_float2(0.f, 0.f);
                if (i >= N / 2 && i < N / 2 + w1) {
                    if (!reuse) x2 = split2(zl[swz(bin)], zl[swz((HALF - bin) & (HALF - 1))], post8192[bin]);
                    else if (fresh) x2 = zl[swz(bin)];
                    else x2 = scr[bin];   // written by this workgroup before an earlier __syncthreads
                }
                xw[i] = x2;
            }
            __syncthreads();   // zl is overwritten by the channel slices from here on
        }

        // ---------------- channels, G at a time ----------------
        const int cbeg = chunk * CHUNK;
        const int cend = min(cbeg + CHUNK, nch);
        float2 *wg = work + g * N;
        // per-slice XOR key of the pass A stores and pass B loads: channels that share a 16-lane
        // store group or a 32-lane load group (TPC lanes each) land on disjoint banks.  Without
        // it every pass-B load at d = 4 was a 2-way conflict (the two channels of a 32-lane group
        // on the same 16 slots), as were d = 5, 6 stores and loads (tools/channel_banks.py)
        const unsigned kg = 8u * (unsigned)(TPC * (g & (16 / TPC - 1)) + 16 * ((g / (16 / TPC)) & 1));
        for (int cg = cbeg; cg < cend; cg += G) {
            const int c = cg + g;
            const bool cok = c < cend;
            const int tb = cok ? tunebins[c] : lo;   // idle lanes read in-range, never store
            // pass A: bins tb + m (- N), m = l + TPC r; X2 x filter; DFT-16
            {
                float2 a[16];
                const float2 *xb = xw + (tb - lo + N / 2 + l);   // COMPACT: xb[TPC r - N wrap]
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int m = l + TPC * r;
                    const bool wrap = TPC * r >= N / 2;
                    if constexpr (COMPACT) {
                        a[r] = cmul(xb[TPC * r - (wrap ? N : 0)], hr[r]);   // zero out of band
                    } else {
                        const int bin = tb + m - (wrap ? N : 0);
                        const bool ok = (unsigned)bin < (unsigned)HALF;
                        const float2 val = cmul(zl[swz(bin & (HALF - 1))], hr[r]);
                        a[r] = ok ? val : make_float2(0.f, 0.f);
                    }
                }
                float2 u[16];
                dft16<+1>(a, u);
#pragma unroll
                for (int r = 0; r < 16; r++) lds_x(wg, (8u * (unsigned)swz(16 * l)) ^ kg, r) = u[r];
            }
            channel_sync();
            // pass B: radix-RB Stockham step (NS = 16), twiddles W_N^{j q} = W_256^{(256/N) j q}
            if constexpr (STAGE) {
                // N < 256: a channel's TPC lanes hold only TPC * 8 B (32 B at d = 6) of each output
                // row, so direct stores write 32-byte pieces.  Instead the outputs go back into the
                // channel's LDS slice in stream order, and the wave stores its channels' kept runs
                // 16 B per lane, consecutive lanes on consecutive bytes: whole lines.
                float2 y[BPT][RB];
#pragma unroll
                for (int b = 0; b < BPT; b++) {
                    const int j = l + TPC * b;
                    float2 a[RB];
#pragma unroll
                    for (int q = 0; q < RB; q++) a[q] = lds_x(wg, (8u * (unsigned)swz(j)) ^ kg, 16 * q);
#pragma unroll
                    for (int q = 1; q < RB; q++) a[q] = cmulc(a[q], twl[((256 / N) * q - 1) * 16 + j]);
                    dft<RB, +1>(a, y[b]);
                }
                channel_sync();   // every lane of the wave has read its slice
                const int sw = (g * TPC) & 12;   // keeps pairs (2p, 2p + 1) adjacent; conflict-free writes
#pragma unroll
                for (int b = 0; b < BPT; b++)
#pragma unroll
                    for (int q = 0; q < RB; q++) wg[(l + TPC * b + 16 * q) ^ sw] = flip(y[b][q], oa.lsbmask);
                channel_sync();
                constexpr int CW = 64 / TPC;                          // channels per wave
                const int lane = t & 63, cw0 = cg + (g & ~(CW - 1)); // the wave's first channel
                const float2 *slices = work + (g & ~(CW - 1)) * N;
                const int n0 = k == 0 ? N / 4 : 0;                    // first kept output of the frame
                const int o0 = k == 0 ? 0 : N / 2 + (3 * N / 4) * (k - 1);
                auto run = [&](auto kept) {
                    constexpr int K = decltype(kept)::value;          // kept outputs per channel
                    constexpr int PER = CS16 ? 4 : 2;                 // complex per 16-B piece
                    constexpr int NP = K / PER;
#pragma unroll
                    for (int e0 = 0; e0 < CW * NP; e0 += 64) {
                        const int e = e0 + lane;
                        const int cl = e / NP, pc = e - cl * NP;
                        const int c = cw0 + cl;
                        if (e >= CW * NP || c >= cend) continue;
                        const int swc = (((g & ~(CW - 1)) + cl) * TPC) & 12;
                        const float2 *src = slices + cl * N;
                        const int n = n0 + PER * pc;
                        const float4 p0 = *reinterpret_cast<const float4 *>(src + (n ^ swc));
                        char *ob = static_cast<char *>(out) +
                                   ((size_t)c * stride + (size_t)blk * 8 * N + o0 + (n - n0)) * out_bytes<CS16>();
                        if constexpr (CS16) {
                            const float4 p1 = *reinterpret_cast<const float4 *>(src + ((n + 2) ^ swc));
                            u32x4 v;
                            v.x = cs16_pack(make_float2(p0.x, p0.y), oa.scale);
                            v.y = cs16_pack(make_float2(p0.z, p0.w), oa.scale);
                            v.z = cs16_pack(make_float2(p1.x, p1.y), oa.scale);
                            v.w = cs16_pack(make_float2(p1.z, p1.w), oa.scale);
                            __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(ob));
                        } else {
                            typedef float f4x __attribute__((ext_vector_type(4)));
                            const f4x v = {p0.x, p0.y, p0.z, p0.w};
                            __builtin_nontemporal_store(v, reinterpret_cast<f4x *>(ob));
                        }
                    }
                };
                if (k == 0)
                    run(std::integral_constant<int, N / 2>{});
                else
                    run(std::integral_constant<int, 3 * N / 4>{});
            } else if (cok) {
                char *ob = static_cast<char *>(out) + ((size_t)c * stride + (size_t)blk * 8 * N) * out_bytes<CS16>();
                auto put = [&](int idx, float2 o) {   // streaming (nt) stores, as the single-channel kernel's
                    if constexpr (CS16) {
                        unsigned *p = reinterpret_cast<unsigned *>(ob) + idx;
                        if constexpr (SDDC_CH_NT) __builtin_nontemporal_store(cs16_pack(o, oa.scale), p);
                        else *p = cs16_pack(o, oa.scale);
                    } else {
                        typedef float f2x __attribute__((ext_vector_type(2)));
                        f2x *p = reinterpret_cast<f2x *>(ob) + idx;
                        const f2x v = {o.x, o.y};
                        if constexpr (SDDC_CH_NT) __builtin_nontemporal_store(v, p);
                        else *p = v;
                    }
                };
#pragma unroll
                for (int b = 0; b < BPT; b++) {
                    const int j = l + TPC * b;          // butterfly 0..15
                    float2 a[RB], y[RB];
#pragma unroll
                    for (int q = 0; q < RB; q++) a[q] = lds_x(wg, (8u * (unsigned)swz(j)) ^ kg, 16 * q);
#pragma unroll
                    for (int q = 1; q < RB; q++) a[q] = cmulc(a[q], twl[((256 / N) * q - 1) * 16 + j]);
                    dft<RB, +1>(a, y);
                    // outputs n = j + 16 q; keep y[N/4, 3N/4) for k = 0, y[0, 3N/4) otherwise
#pragma unroll
                    for (int q = 0; q < RB; q++) {
                        const int n = j + 16 * q;
                        if (16 * q >= 3 * N / 4) continue;
                        const float2 o = flip(y[q], oa.lsbmask);
                        if (k == 0) {
                            if (16 * q >= N / 4) put(n - N / 4, o);
                        } else {
                            put(N / 2 + (3 * N / 4) * (k - 1) + n, o);
                        }
                    }
                }
            }
            channel_sync();   // wg is rewritten by the next channel group (same lanes)
        }
    }
}

// ---------------------------------------------------------------------------------------
// Many channels at d = 0..3 (N = 4096 >> d >= 512): persistent, work item = (frame, chunk of
// <= CHUNK_P channels).  Per frame the forward transform (as ddc_persistent.hip) and the
// shared r2c split X2 in place over all bins (buffer zl, kept for the frame's next chunks in
// the workgroup's contiguous item range); per item the channels CG = 2^d at a
// time, so every inverse pass keeps all 256 threads busy with 16 points each:
//   pass 0  radix N/256 per channel (each thread: CG channels x N/256 bins; the filter taps of
//           its bins live in registers), into the channels' N-element slices of `wi`
//   pass 1  radix 16, NS = N/256: thread t -> channel t / (N/16), butterfly t % (N/16)
//   pass 2  radix 16, NS = N/16, register-recurrence twiddles, overlap-discard store
// d = 0: 32 KB transform + 32 KB of channel slices + twiddles, 2 workgroups per CU.
// d >= 1 (L2X2): the split spectrum goes to the workgroup's scratch row in L2 instead and the
// forward transform runs in the slice buffer: 36 KB of LDS, 3 workgroups per CU (VGPR-bound).
#ifndef SDDC_CHUNK_P
#define SDDC_CHUNK_P 32       // channels per work item
#endif
constexpr int CHUNK_P = SDDC_CHUNK_P;

#ifndef SDDC_CHP_WAVES
#define SDDC_CHP_WAVES 3      // __launch_bounds__ min waves per SIMD of the L2X2 form
#endif
#ifndef SDDC_CHP_HREG
#define SDDC_CHP_HREG 1       // filter taps of the pass-0 bins in registers (else loaded per channel)
#endif
template <int D, bool RAND, bool CS16, bool L2X2>
__global__ __launch_bounds__(NT, L2X2 ? SDDC_CHP_WAVES : 2) void r2iq_channels_p_kernel(
    const int *__restrict__ in32, void *__restrict__ out, size_t stride, int nframes,
    const int *__restrict__ tunebins, int nch, const float2 *__restrict__ tw_p1, const float2 *__restrict__ tw_q1,
    const float2 *__restrict__ rec_f, const float2 *__restrict__ rec_i, const float2 *__restrict__ post8192,
    const float2 *__restrict__ hsel, OutArgs oa, float2 *__restrict__ scratch)
{
    constexpr int N = HALF >> D;
    static_assert(N >= 512, "d = 0..3");
    constexpr int R0 = N / 256;          // inverse pass-0 radix
    constexpr int NB = N / 16;           // radix-16 butterflies per channel in passes 1, 2
    constexpr int CG = NT / NB;          // channels in flight (2^d)
    // L2X2: the split spectrum goes to this workgroup's scratch row (L2-resident) instead of
    // a second 32 KB of LDS, and the forward transform runs in the channel-slice buffer
    __shared__ __attribute__((aligned(16))) float2 zbuf[L2X2 ? 1 : HALF];
    __shared__ __attribute__((aligned(16))) float2 wi[CG * N];
    float2 *const zl = L2X2 ? wi : zbuf;
    float2 *const scr = L2X2 ? scratch + (size_t)blockIdx.x * HALF : nullptr;
    __shared__ __attribute__((aligned(16))) float2 twl[15 * 16 + 15 * R0];

    const int tid = (int)threadIdx.x;
    const int nchunks = (nch + CHUNK_P - 1) / CHUNK_P;
    const long long items = (long long)nframes * nchunks;
    const int i0 = (int)(items * blockIdx.x / gridDim.x), i1 = (int)(items * (blockIdx.x + 1) / gridDim.x);
    if (i0 >= i1) return;
    for (int i = tid; i < 15 * 16 + 15 * R0; i += NT) twl[i] = i < 15 * 16 ? tw_p1[i] : tw_q1[i - 15 * 16];
    const float2 fw1_ = rec_f[tid], fw4_ = rec_f[NT + tid];
    const int jb_ = tid % NB, cb_ = tid / NB;    // passes 1, 2: butterfly, channel in group
    const float2 iw1_ = rec_i[jb_], iw4_ = rec_i[NT + jb_];
    float2 hr[R0];   // H[m]/2 for this thread's pass-0 bins m = t + 256 r
    if constexpr (SDDC_CHP_HREG || !L2X2) {
#pragma unroll
        for (int r = 0; r < R0; r++) hr[r] = hsel[tid + NT * r];
    }

    int zf = -1;   // frame whose split spectrum X2 is in zl (consecutive chunks of a frame reuse it)
    for (int it = i0; it < i1; it++) {
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z, jb = jb_ + z, cb = cb_ + z;
        float2 fw1 = fw1_, fw4 = fw4_, iw1 = iw1_, iw4 = iw4_;
        asm volatile("" : "+v"(fw1), "+v"(fw4), "+v"(iw1), "+v"(iw4));
        const int f = it / nchunks, chunk = it - f * nchunks;
        const int blk = f / FRAMES, k = f - blk * FRAMES;
        const int sT = swz(t), x15 = t & 15;
        if (f != zf) {   // workgroup-uniform
        zf = f;
        // ---------------- forward: Z = FFT4096(x_even + i x_odd) in zl ----------------
        float2 v[16];
        {
            const __amdgpu_buffer_rsrc_t rs = buf_rsrc(in32 + ((size_t)blk * BLOCK + (size_t)k * HOP) / 2);
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int w = buf_load4<SDDC_LD_AUX>(rs, 4u * (unsigned)t, 4u * NT * r);
                a[r] = make_float2(derand<RAND>((int)(short)(w & 0xffff)), derand<RAND>(w >> 16));
            }
            dft16<-1>(a, v);
        }
        __syncthreads();   // the previous item's readers of zl / wi are done
#pragma unroll
        for (int r = 0; r < 16; r++) zl[16 * t + (r ^ x15)] = v[r];
        __syncthreads();
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) a[r] = zl[sT + NT * r];
#pragma unroll
            for (int r = 1; r < 16; r++) a[r] = cmul(a[r], twl[(r - 1) * 16 + x15]);
            dft16<-1>(a, v);
        }
        __syncthreads();
        {
            const int b1 = (t >> 4) * 256;
#pragma unroll
            for (int r = 0; r < 16; r++) zl[b1 + 16 * r + (x15 ^ r)] = v[r];
        }
        __syncthreads();
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) a[r] = zl[sT + NT * r];
            twiddle_rec16<-1>(a, fw1, fw4);
            dft16<-1>(a, v);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; r++) zl[sT + NT * r] = v[r];
        __syncthreads();
        // ---------------- shared split, in place: thread-owned pairs (k, 4096 - k) ----------------
        for (int k0 = t; k0 <= HALF / 2; k0 += NT) {
            const int k1 = (HALF - k0) & (HALF - 1);
            const float2 z0 = zl[swz(k0)], z1 = zl[swz(k1)];
            const float2 x0 = split2(z0, z1, post8192[k0]), x1 = split2(z1, z0, post8192[k1]);
            if constexpr (L2X2) {
                scr[k0] = x0;
                if (k1 != k0) scr[k1] = x1;
            } else {
                zl[swz(k0)] = x0;
                if (k1 != k0) zl[swz(k1)] = x1;
            }
        }
        __syncthreads();   // (L2X2: the scratch row is visible to the workgroup; wi is free)
        }

        // ---------------- channels, CG at a time ----------------
        const int cbeg = chunk * CHUNK_P, cend = min(cbeg + CHUNK_P, nch);
        for (int c0 = cbeg; c0 < cend; c0 += CG) {
            // pass 0: bins tb + m (- N), m = t + 256 r; X2 x H/2; DFT-R0 -> slice
#pragma unroll
            for (int g = 0; g < CG; g++) {
                const int c = min(c0 + g, cend - 1);   // idle slots redo the last channel, never stored
                const int tb = tunebins[c];
                float2 a[R0], u[R0];
                if constexpr (L2X2) {
                    const __amdgpu_buffer_rsrc_t rx = buf_rsrc(scr);
                    float2 xv[R0], hv[R0];
#pragma unroll
                    for (int r = 0; r < R0; r++) {
                        const int bin = tb + t + NT * r - (NT * r >= N / 2 ? N : 0);
                        xv[r] = buf_load8(rx, 8u * (unsigned)(bin & (HALF - 1)), 0u);
                        hv[r] = SDDC_CHP_HREG ? hr[r] : hsel[t + NT * r];
                    }
#pragma unroll
                    for (int r = 0; r < R0; r++) {
                        const int bin = tb + t + NT * r - (NT * r >= N / 2 ? N : 0);
                        a[r] = (unsigned)bin < (unsigned)HALF ? cmul(xv[r], hv[r]) : make_float2(0.f, 0.f);
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < R0; r++) {
                        const int m = t + NT * r;
                        const int bin = tb + m - (NT * r >= N / 2 ? N : 0);
                        const float2 val = cmul(zl[swz(bin & (HALF - 1))], hr[r]);
                        a[r] = (unsigned)bin < (unsigned)HALF ? val : make_float2(0.f, 0.f);
                    }
                }
                if constexpr (R0 == 16) dft16<+1>(a, u);
                else dft<R0, +1>(a, u);
                float2 *sl = wi + g * N;
                if constexpr (R0 == 16) {
#pragma unroll
                    for (int r = 0; r < 16; r++) sl[16 * t + (r ^ x15)] = u[r];
                } else {
#pragma unroll
                    for (int r = 0; r < R0; r++) LX(sl, R0 * t, r) = u[r];
                }
            }
            __syncthreads();
            // pass 1: radix 16, NS = R0, table twiddles W_{16 R0}^{(j % R0) r}
            float2 *sl = wi + cb * N;
            float2 u[16];
            {
                float2 a[16];
#pragma unroll
                for (int r = 0; r < 16; r++) a[r] = LX(sl, jb, NB * r);
#pragma unroll
                for (int r = 1; r < 16; r++) a[r] = cmulc(a[r], twl[15 * 16 + (r - 1) * R0 + (jb % R0)]);
                dft16<+1>(a, u);
            }
            __syncthreads();
            {
                const int base = (jb / R0) * (16 * R0) + (jb % R0);
#pragma unroll
                for (int r = 0; r < 16; r++) LX(sl, base, R0 * r) = u[r];
            }
            __syncthreads();
            // pass 2: radix 16, NS = N/16, recurrence twiddles W_N^{j r}; overlap-discard store
            {
                float2 a[16];
#pragma unroll
                for (int r = 0; r < 16; r++) a[r] = LX(sl, jb, NB * r);
                twiddle_rec16<+1>(a, iw1, iw4);
                dft16<+1>(a, u);
            }
            const int c = c0 + cb;
            if (c < cend) {
                const int fbase = blk * 8 * N + (k == 0 ? -N / 4 : N / 2 + (3 * N / 4) * (k - 1));
                const __amdgpu_buffer_rsrc_t ro =
                    buf_rsrc(static_cast<char *>(out) + ((size_t)c * stride + (size_t)fbase) * out_bytes<CS16>());
                const int r0 = k == 0 ? 4 : 0;
#pragma unroll
                for (int r = 0; r < 12; r++) {
                    if (r < r0) continue;
                    store_iq<CS16>(flip(u[r], oa.lsbmask), ro, (unsigned)jb, (unsigned)(NB * r), oa);
                }
            }
            __syncthreads();   // the slices are rewritten by the next group
        }
    }
}

struct ChLaunch {
    const int16_t *d_in;
    int nblk;
    const int *d_tunebins;
    int nch;
    void *d_out;
    size_t stride;
    OutArgs oa;
    const int2 *windows;   // per-chunk compact windows, or nullptr
    float2 *scratch;       // v2 COMPACT: per-workgroup X2 rows (scratch_rows x 4096), or nullptr
    int scratch_rows;
    int device;
    hipStream_t s;
};

template <int D, bool RAND, bool CS16, bool COMPACT, bool STAGE_OK>
hipError_t launch_v(const KernelTables &t, const ChLaunch &L)
{
    auto kern = r2iq_channels_v2_kernel<D, RAND, CS16, COMPACT, STAGE_OK>;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(kern), NT, L.device, &occ, &cus);
    if (e != hipSuccess) return e;
    const int nframes = L.nblk * FRAMES;
    const long long items = (long long)nframes * ((L.nch + CHUNK - 1) / CHUNK);
    const int grid = (int)(items < (long long)cus * occ ? items : (long long)cus * occ);
    float2 *scratch = grid <= L.scratch_rows ? L.scratch : nullptr;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, L.s, reinterpret_cast<const int *>(L.d_in), L.d_out,
                       L.stride / 2, nframes, L.d_tunebins, L.nch, t.tw_p1, t.rec_f, t.post8192, t.hsel[D], L.oa,
                       L.windows, scratch);
    return hipGetLastError();
}

template <int D, bool RAND, bool CS16, bool COMPACT>
hipError_t launch_s(const KernelTables &t, const ChLaunch &L)
{
    // the staged 16-B stores of d = 5, 6 need every channel row 16-B aligned
    const size_t row = L.stride * (CS16 ? 2 : 4);   // bytes (stride counts components)
    const bool al = (HALF >> D) <= STAGE_MAX_N && ((uintptr_t)L.d_out & 15) == 0 && (L.nch == 1 || (row & 15) == 0);
    return al ? launch_v<D, RAND, CS16, COMPACT, true>(t, L) : launch_v<D, RAND, CS16, COMPACT, false>(t, L);
}

template <int D, bool RAND, bool CS16>
hipError_t launch_c(const KernelTables &t, const ChLaunch &L)
{
    return L.windows ? launch_s<D, RAND, CS16, true>(t, L) : launch_s<D, RAND, CS16, false>(t, L);
}

template <int D>
hipError_t launch_d(const KernelTables &t, const ChLaunch &L, int rand, int cs16)
{
    if (rand) return cs16 ? launch_c<D, true, true>(t, L) : launch_c<D, true, false>(t, L);
    return cs16 ? launch_c<D, false, true>(t, L) : launch_c<D, false, false>(t, L);
}

template <int D, bool RAND, bool CS16, bool L2X2>
hipError_t launch_p2(const KernelTables &t, const ChLaunch &L)
{
    auto kern = r2iq_channels_p_kernel<D, RAND, CS16, L2X2>;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(kern), NT, L.device, &occ, &cus);
    if (e != hipSuccess) return e;
    const int nframes = L.nblk * FRAMES;
    const long long items = (long long)nframes * ((L.nch + CHUNK_P - 1) / CHUNK_P);
    const int grid = (int)(items < (long long)cus * occ ? items : (long long)cus * occ);
    if constexpr (L2X2) {
        if (grid > L.scratch_rows) {   // one scratch row per workgroup: more workgroups than rows -> LDS form
            ChLaunch L0 = L;
            L0.scratch = nullptr;
            return launch_p2<D, RAND, CS16, false>(t, L0);
        }
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, L.s, reinterpret_cast<const int *>(L.d_in), L.d_out,
                       L.stride / 2, nframes, L.d_tunebins, L.nch, t.tw_p1, t.tw_q1[D], t.rec_f, t.rec_i[D],
                       t.post8192, t.hsel[D], L.oa, L.scratch);
    return hipGetLastError();
}

#ifndef SDDC_CHP_L2
#define SDDC_CHP_L2 1         // d >= 1: the L2X2 form when the handle's scratch rows cover the grid
#endif                        // (+8-16 % at d = 1..3; at d = 0 it needs > 168 VGPRs and is no faster,
                              // profiles/r01/channels/ab_channels_lowd_l2.txt)
template <int D, bool RAND, bool CS16>
hipError_t launch_p(const KernelTables &t, const ChLaunch &L)
{
    // the grid is at most CUs x 4 resident workgroups; the scratch holds L.scratch_rows rows
    if constexpr (SDDC_CHP_L2 && D >= 1) {
        if (L.scratch) {
            int occ = 0, cus = 0;
            hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(r2iq_channels_p_kernel<D, RAND, CS16, true>),
                                           NT, L.device, &occ, &cus);
            if (e != hipSuccess) return e;
            if (cus * 4 <= L.scratch_rows) return launch_p2<D, RAND, CS16, true>(t, L);
        }
    }
    ChLaunch L0 = L;
    L0.scratch = nullptr;
    return launch_p2<D, RAND, CS16, false>(t, L0);
}

template <int D>
hipError_t launch_pd(const KernelTables &t, const ChLaunch &L, int rand, int cs16)
{
    if (rand) return cs16 ? launch_p<D, true, true>(t, L) : launch_p<D, true, false>(t, L);
    return cs16 ? launch_p<D, false, true>(t, L) : launch_p<D, false, false>(t, L);
}

}  // namespace

hipError_t launch_channels_p(const KernelTables &t, int d, const int16_t *d_in, int nblk, const int *d_tunebins,
                             int nch, void *d_out, size_t stride, int lsb, int rand, int cs16, float cs16_scale,
                             float2 *d_scratch, int scratch_rows, int device, hipStream_t s)
{
    const ChLaunch L{d_in, nblk, d_tunebins, nch, d_out, stride, OutArgs{lsb ? 0x80000000u : 0u, cs16_scale},
                     nullptr, d_scratch, scratch_rows, device, s};
    switch (d) {
    case 0: return launch_pd<0>(t, L, rand, cs16);
    case 1: return launch_pd<1>(t, L, rand, cs16);
    case 2: return launch_pd<2>(t, L, rand, cs16);
    case 3: return launch_pd<3>(t, L, rand, cs16);
    default: return hipErrorInvalidValue;
    }
}

bool channel_windows(int d, const int *tunebins, int nch, int2 *windows)
{
    const int N = HALF >> d;
    for (int c0 = 0, k = 0; c0 < nch; c0 += CHUNK, k++) {
        int mn = HALF, mx = -1;
        for (int c = c0; c < c0 + CHUNK && c < nch; c++) {
            mn = std::min(mn, tunebins[c]);
            mx = std::max(mx, tunebins[c]);
        }
        const int lo = std::max(0, mn - N / 2), hi = std::min(HALF, mx + N / 2);
        if (hi - lo > ZC_MAX) return false;
        windows[k] = make_int2(lo, hi - lo);
    }
    return true;
}

hipError_t launch_channels_v2(const KernelTables &t, int d, const int16_t *d_in, int nblk, const int *d_tunebins,
                              int nch, void *d_out, size_t stride, int lsb, int rand, int cs16, float cs16_scale,
                              const int2 *d_windows, float2 *d_scratch, int scratch_rows, int device,
                              hipStream_t s)
{
    const ChLaunch L{d_in, nblk, d_tunebins, nch, d_out, stride, OutArgs{lsb ? 0x80000000u : 0u, cs16_scale},
                     d_windows, d_scratch, scratch_rows, device, s};
    switch (d) {
    case 4: return launch_d<4>(t, L, rand, cs16);
    case 5: return launch_d<5>(t, L, rand, cs16);
    case 6: return launch_d<6>(t, L, rand, cs16);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace sddc
