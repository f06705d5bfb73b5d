// ddc_persistent.hip — v2 single-channel r2iq kernel for gfx950: persistent workgroups.
//
// Same per-frame algorithm as ddc_kernels.hip (see its header for the mapping of
// the reference's fft_mt_r2iq_impl.hpp:76-138 onto the passes), restructured for
// throughput on MI355X:
//   * persistent grid (CUs x resident workgroups); each workgroup walks a
//     contiguous range of frames, so consecutive frames (which share 2048 input
//     samples) stay on one CU / XCD L2;
//   * the next frame's 16 int16 pairs per thread are loaded into registers while
//     the current frame is transformed (hides the HBM latency the v1 kernel paid
//     at every workgroup start);
//   * LDS is addressed through an XOR swizzle e ^ ((e >> 4) & 15) instead of
//     padding: 32 KB per frame, and both the 16-consecutive-per-lane writes of
//     the first pass and the 64-consecutive reads are bank-conflict free;
//   * twiddles: small [r][s] tables for the NS <= 16 passes (L1 resident), and a
//     register recurrence from per-thread W^j, W^{4j} for the NS = 256 passes
//     (no 30 KB L2 table stream per frame); the r2c split twiddle W_8192^bin is a
//     per-thread base times a compile-time W_32 constant.
#include <hip/hip_runtime.h>

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
#ifndef SDDC_DB
#define SDDC_DB 0
#endif
// Double-buffered LDS (two 32 KB frames, one barrier per pass) vs one buffer (two
// barriers per pass, twice the workgroups per CU).  Build-time switch for A/B timing.
constexpr bool kDB = SDDC_DB != 0;
#ifndef SDDC_WAVES
#define SDDC_WAVES 2          // __launch_bounds__ min waves per SIMD
#endif
#ifndef SDDC_TWTAB
#define SDDC_TWTAB 0          // NS=N/16 passes: 1 = coalesced [r][t] twiddle table, 0 = register recurrence
#endif
#ifndef SDDC_FAKE
#define SDDC_FAKE 0           // timing-only builds: 1 = no filter/PQ loads, 2 = no pass-1 twiddle reads,
                              // 4 = no loop barriers, 8 = no output stores, 16 = no input loads,
                              // 32 = no LDS exchange reads (N >= 512), 64 = no LDS exchange writes (N >= 512)
#endif
#ifndef SDDC_PQ
#define SDDC_PQ 1             // split x filter from the per-(d, tunebin) coefficient table (P, Q)
#endif
#ifndef SDDC_PK
#define SDDC_PK 0             // 1: radix-16 DFTs and twiddle products in packed FP32 (measured slower)
#endif
#ifndef SDDC_PREFETCH
#define SDDC_PREFETCH 1       // load the next frame's input during the current one
#endif

// W_32^q = e^{-2 pi i q/32}
__device__ constexpr float kW32re[32] = {
    1.0f, 9.807852804e-01f, 9.238795325e-01f, 8.314696123e-01f, 7.071067812e-01f, 5.555702330e-01f,
    3.826834324e-01f, 1.950903220e-01f, 0.0f, -1.950903220e-01f, -3.826834324e-01f, -5.555702330e-01f,
    -7.071067812e-01f, -8.314696123e-01f, -9.238795325e-01f, -9.807852804e-01f, -1.0f, -9.807852804e-01f,
    -9.238795325e-01f, -8.314696123e-01f, -7.071067812e-01f, -5.555702330e-01f, -3.826834324e-01f,
    -1.950903220e-01f, 0.0f, 1.950903220e-01f, 3.826834324e-01f, 5.555702330e-01f, 7.071067812e-01f,
    8.314696123e-01f, 9.238795325e-01f, 9.807852804e-01f};
__device__ constexpr float kW32im[32] = {
    0.0f, -1.950903220e-01f, -3.826834324e-01f, -5.555702330e-01f, -7.071067812e-01f, -8.314696123e-01f,
    -9.238795325e-01f, -9.807852804e-01f, -1.0f, -9.807852804e-01f, -9.238795325e-01f, -8.314696123e-01f,
    -7.071067812e-01f, -5.555702330e-01f, -3.826834324e-01f, -1.950903220e-01f, 0.0f, 1.950903220e-01f,
    3.826834324e-01f, 5.555702330e-01f, 7.071067812e-01f, 8.314696123e-01f, 9.238795325e-01f,
    9.807852804e-01f, 1.0f, 9.807852804e-01f, 9.238795325e-01f, 8.314696123e-01f, 7.071067812e-01f,
    5.555702330e-01f, 3.826834324e-01f, 1.950903220e-01f};

#define LOOP_SYNC() do { if constexpr (!(SDDC_FAKE & 4)) __syncthreads(); } while (0)
#define LDS_RD(expr, fake) ((SDDC_FAKE & 32) ? (fake) : (expr))
#define LDS_WR if constexpr (!(SDDC_FAKE & 64))

__device__ __forceinline__ int swz(int e) { return e ^ ((e >> 4) & 15); }

template <int DIR>
__device__ __forceinline__ float2 tmul(float2 a, float2 w) { return DIR < 0 ? cmul(a, w) : cmulc(a, w); }

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

// a[r] *= W^{r} for r = 1..15 given the forward-direction W^1 and W^4 of this lane
// (conjugated for DIR = +1).  Every power is at most three products away.
template <int DIR>
__device__ __forceinline__ void twiddle_rec16(float2 *a, float2 w1, float2 w4)
{
    if (DIR > 0) {
        w1.y = -w1.y;
        w4.y = -w4.y;
    }
    const float2 w2 = cmul(w1, w1), w3 = cmul(w2, w1);
    const float2 w8 = cmul(w4, w4), w12 = cmul(w8, w4);
    a[1] = cmul(a[1], w1);
    a[2] = cmul(a[2], w2);
    a[3] = cmul(a[3], w3);
    a[4] = cmul(a[4], w4);
    a[5] = cmul(a[5], cmul(w4, w1));
    a[6] = cmul(a[6], cmul(w4, w2));
    a[7] = cmul(a[7], cmul(w4, w3));
    a[8] = cmul(a[8], w8);
    a[9] = cmul(a[9], cmul(w8, w1));
    a[10] = cmul(a[10], cmul(w8, w2));
    a[11] = cmul(a[11], cmul(w8, w3));
    a[12] = cmul(a[12], w12);
    a[13] = cmul(a[13], cmul(w12, w1));
    a[14] = cmul(a[14], cmul(w12, w2));
    a[15] = cmul(a[15], cmul(w12, w3));
}

// DFT-16 and twiddle products, packed (SDDC_PK) or scalar
template <int DIR>
__device__ __forceinline__ void DFT16(const float2 *a, float2 *v)
{
    if constexpr (SDDC_PK) pk::dft16<DIR>(a, v);
    else dft16<DIR>(a, v);
}
// a * W (DIR < 0) or a * conj(W) (DIR > 0)
template <int DIR>
__device__ __forceinline__ float2 TW(float2 a, float2 w)
{
    if constexpr (SDDC_PK) return pk::F(DIR < 0 ? pk::cmul(pk::V(a), pk::V(w)) : pk::cmulc(pk::V(a), pk::V(w)));
    else return DIR < 0 ? cmul(a, w) : cmulc(a, w);
}
// twiddle_rec16 with packed products
template <int DIR>
__device__ __forceinline__ void TWREC16(float2 *a, float2 w1_, float2 w4_)
{
    if constexpr (!SDDC_PK) {
        twiddle_rec16<DIR>(a, w1_, w4_);
        return;
    }
    using namespace pk;
    f2v w1 = V(w1_), w4 = V(w4_);
    if (DIR > 0) {
        w1.y = -w1.y;
        w4.y = -w4.y;
    }
    const f2v w2 = cmul(w1, w1), w3 = cmul(w2, w1), w8 = cmul(w4, w4), w12 = cmul(w8, w4);
    a[1] = F(cmul(V(a[1]), w1));
    a[2] = F(cmul(V(a[2]), w2));
    a[3] = F(cmul(V(a[3]), w3));
    a[4] = F(cmul(V(a[4]), w4));
    a[5] = F(cmul(V(a[5]), cmul(w4, w1)));
    a[6] = F(cmul(V(a[6]), cmul(w4, w2)));
    a[7] = F(cmul(V(a[7]), cmul(w4, w3)));
    a[8] = F(cmul(V(a[8]), w8));
    a[9] = F(cmul(V(a[9]), cmul(w8, w1)));
    a[10] = F(cmul(V(a[10]), cmul(w8, w2)));
    a[11] = F(cmul(V(a[11]), cmul(w8, w3)));
    a[12] = F(cmul(V(a[12]), w12));
    a[13] = F(cmul(V(a[13]), cmul(w12, w1)));
    a[14] = F(cmul(V(a[14]), cmul(w12, w2)));
    a[15] = F(cmul(V(a[15]), cmul(w12, w3)));
}

// X[bin] * Hh[m] from Z in LDS (Hh = H/2): the r2c split E + W^bin O, times the filter.
// Zero for bins the reference zero-fills (impl.hpp:91-92, 95-96).
//   X Hh = Hh [(Zk + conj Zc) - i W^bin (Zk - conj Zc)] = Zk P + conj(Zc) Q,
//   P = Hh (1 - i W^bin),  Q = Hh (1 + i W^bin)     (Zc = Z[(4096 - bin) mod 4096])
// split_pq evaluates the right-hand form from the table built by build_split_filter_kernel,
// whose entries are zero for out-of-band bins; split_bin is the direct form (SDDC_PQ=0).
__device__ __forceinline__ float2 split_pq(float2 zk, float2 zc, float4 c)
{
    float2 v;
    v.x = zk.x * c.x - zk.y * c.y + zc.x * c.z + zc.y * c.w;
    v.y = zk.x * c.y + zk.y * c.x + zc.x * c.w - zc.y * c.z;
    return v;
}

__device__ __forceinline__ float2 split_bin(const float2 *lds, int bin, float2 wbin, float2 hh)
{
    if (bin < 0 || bin >= HALF) return make_float2(0.f, 0.f);
    const float2 zk = lds[swz(bin)];
    const float2 zc = lds[swz((HALF - bin) & (HALF - 1))];
    const float2 A = make_float2(zk.x + zc.x, zk.y - zc.y);
    const float2 Bi = make_float2(zk.y + zc.y, zc.x - zk.x);   // (Zk - conj Zc) / i
    return cmul(cadd(A, cmul(Bi, wbin)), hh);
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
        if constexpr (SDDC_FAKE & 8) {   // keep v live, store practically never
            if (v.x == 1.2345e30f) store_iq<CS16>(v, ro, (unsigned)t, (unsigned)(NB * r), oa);
        } else {
            store_iq<CS16>(v, ro, (unsigned)t, (unsigned)(NB * r), oa);
        }
    }
}

__device__ __forceinline__ void load_frame(const int *__restrict__ in32, int blk, int k, int (&x)[16])
{
    if constexpr (SDDC_FAKE & 16) {   // synthetic frame, no memory traffic
#pragma unroll
        for (int r = 0; r < 16; r++) x[r] = (int)(threadIdx.x * 2654435761u + r * 40503u + blk * 7u + k);
        return;
    }
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(in32 + ((size_t)blk * BLOCK + (size_t)k * HOP) / 2);
    const unsigned vo = 4u * threadIdx.x;
#pragma unroll
    for (int r = 0; r < 16; r++) x[r] = buf_load4<SDDC_LD_AUX>(rs, vo, 4u * NT * r);
}

template <int D, bool RAND, bool NCO, bool CS16>
__global__ __launch_bounds__(NT, SDDC_WAVES) void r2iq_persistent_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes,
    const float2 *__restrict__ tw_p1, const float2 *__restrict__ tw_q1,
    const float2 *__restrict__ rec_f, const float2 *__restrict__ rec_i,
    const float2 *__restrict__ twt_f, const float2 *__restrict__ twt_i,
    const float2 *__restrict__ post8192, const float2 *__restrict__ hsel,
    const float4 *__restrict__ pq, int tunebin, OutArgs oa, NcoArgs nco)
{
    constexpr int N = HALF >> D;
    __shared__ __attribute__((aligned(16))) float2 lds[kDB ? 2 * HALF : HALF];
    // pass-1 twiddle tables, copied once per workgroup: [15][16] forward, [15][S] inverse
    constexpr int SQ = N >= 512 ? N / 256 : N / 16;
    __shared__ __attribute__((aligned(16))) float2 twl[15 * 16 + 15 * SQ];
    float2 *w0 = lds, *w1 = kDB ? lds + HALF : lds;   // this frame's pass buffers

    const int tid = (int)threadIdx.x;
    const int G = (int)gridDim.x, w = (int)blockIdx.x;
    const int f0 = (int)(((long long)nframes * w) / G);
    const int f1 = (int)(((long long)nframes * (w + 1)) / G);
    if (f0 >= f1) return;

    // per-thread constants, live for the whole frame loop
    const float2 fw1_ = rec_f[tid], fw4_ = rec_f[NT + tid];
    float2 iw1_ = fw1_, iw4_ = fw4_;
    if constexpr (N >= 512 && N < HALF) {
        if (tid < N / 16) {
            iw1_ = rec_i[tid];
            iw4_ = rec_i[NT + tid];
        }
    }
    const float2 pb_ = post8192[(tunebin + tid) & 8191];   // W_8192^{tb + tid}
    for (int i = tid; i < 15 * 16 + 15 * SQ; i += NT)
        twl[i] = i < 15 * 16 ? tw_p1[i] : tw_q1[i - 15 * 16];   // visible after the first frame's pass-0 barrier

    int blk = f0 / FRAMES, k = f0 - blk * FRAMES;
    int x[16];
    if (SDDC_PREFETCH) load_frame(in32, blk, k, x);

    for (int f = f0; f < f1; f++) {
        // Opaque per-iteration copies of the thread index and table pointers: without
        // them the compiler hoists every loop-invariant LDS address and table load out
        // of the frame loop and spills them.
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z;
        const float2 *hs = hsel + z, *pst = post8192 + z;
        const float4 *pqz = pq + z;
        const float2 *ttf = twt_f + z, *tti = twt_i + z;
        float2 fw1 = fw1_, fw4 = fw4_, iw1 = iw1_, iw4 = iw4_, pb = pb_;
        asm volatile("" : "+v"(fw1), "+v"(fw4), "+v"(iw1), "+v"(iw4), "+v"(pb));
        const int sT = swz(t);            // swz(t + 256 r) = sT + 256 r
        const int x15 = t & 15;
        const int oblk = blk * 8 * N;   // first output slot of the block (batch-relative)
        const int kc = k;
        // ---- forward pass 0 (R16, NS1): convert + DFT16 from registers ----
        float2 v[16];
        {
            if (!SDDC_PREFETCH) load_frame(in32, blk, k, x);
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++)
                a[r] = make_float2(derand<RAND>((int)(short)(x[r] & 0xffff)), derand<RAND>(x[r] >> 16));
            if (++k == FRAMES) {
                k = 0;
                ++blk;
            }
            if (SDDC_PREFETCH && f + 1 < f1) load_frame(in32, blk, k, x);   // prefetch the next frame
            DFT16<-1>(a, v);
        }
        if constexpr (!kDB) LOOP_SYNC();   // the previous frame's last LDS reads are done
#pragma unroll
        for (int r = 0; r < 16; r++) LDS_WR w0[16 * t + (r ^ x15)] = v[r];          // swz(16t + r)
        LOOP_SYNC();
        // ---- forward pass 1 (R16, NS16): table twiddles W_256^{(t%16) r} ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) a[r] = LDS_RD(w0[sT + NT * r], v[r]);
#pragma unroll
            for (int r = 1; r < 16; r++)
                a[r] = TW<-1>(a[r], (SDDC_FAKE & 2) ? make_float2(0.7f, 0.01f * (r + x15)) : twl[(r - 1) * 16 + x15]);
            DFT16<-1>(a, v);
        }
        if constexpr (!kDB) LOOP_SYNC();
        {
            const int b1 = (t >> 4) * 256;                                     // swz(b1 + x15 + 16 r)
#pragma unroll
            for (int r = 0; r < 16; r++) LDS_WR w1[b1 + 16 * r + (x15 ^ r)] = v[r];
        }
        LOOP_SYNC();
        // ---- forward pass 2 (R16, NS256): recurrence twiddles W_4096^{t r} ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) a[r] = LDS_RD(w1[sT + NT * r], v[r]);
            if constexpr (SDDC_TWTAB) {
#pragma unroll
                for (int r = 1; r < 16; r++) a[r] = TW<-1>(a[r], ttf[(r - 1) * NT + t]);
            } else {
                TWREC16<-1>(a, fw1, fw4);
            }
            DFT16<-1>(a, v);
        }
        if constexpr (!kDB) LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 16; r++) LDS_WR w0[sT + NT * r] = v[r];   // Z, natural order
        LOOP_SYNC();

        if constexpr (N >= 512) {
            constexpr int R0 = N / 256;
            // ---- inverse pass 0 (R0, NS1): r2c split x filter, bins tb-N/2 .. tb+N/2 ----
            float2 u[16];
            {
                const int b0 = tunebin + t;                  // bin of r = 0
                const int sb0 = swz(b0);                     // swz(b0 + 256 r - N w) = sb0 + 256 r - N w
                const int sc0 = swz(HALF - b0);              // mirror bin, same separability
                const char *w0b = reinterpret_cast<const char *>(w0);
                const unsigned sb0b = 8u * (unsigned)sb0, sc0b = 8u * (unsigned)sc0, tb16 = 16u * (unsigned)t;
                const __amdgpu_buffer_rsrc_t rpq = buf_rsrc(pqz);
                float2 a[R0];
#pragma unroll
                for (int r = 0; r < R0; r++) {
                    const bool wrap = (NT * r >= N / 2);
                    const int sh = NT * r - (wrap ? N : 0);
                    const int bin = b0 + sh;
                    const int q = (r - (wrap ? N / NT : 0)) & 31;       // W_8192^{256 r - N wrap}
                    // branch-free: read a valid (wrapped) address; out-of-band bins have P = Q = 0
                    if constexpr (SDDC_PQ) {
                        // byte offsets: the wrap is one AND, the scale folds away
                        const float2 zk = LDS_RD(*reinterpret_cast<const float2 *>(
                            w0b + ((sb0b + 8u * (unsigned)sh) & (8u * HALF - 8u))), v[r]);
                        const float2 zc = LDS_RD(*reinterpret_cast<const float2 *>(
                            w0b + ((sc0b - 8u * (unsigned)sh) & (8u * HALF - 8u))), v[(r + 1) & 15]);
                        float4 c;
                        if constexpr (SDDC_FAKE & 1)
                            c = make_float4(0.5f, 0.25f * r, 0.1f, 0.2f);
                        else
                            c = buf_load16(rpq, tb16, 16u * NT * r);
                        a[r] = split_pq(zk, zc, c);
                        continue;
                    }
                    const float2 zk = w0[(sb0 + sh) & (HALF - 1)];
                    const float2 zc = w0[(sc0 - sh) & (HALF - 1)];
                    {
                        const bool ok = (unsigned)bin < (unsigned)HALF;
                        const float2 A = make_float2(zk.x + zc.x, zk.y - zc.y);
                        const float2 Bi = make_float2(zk.y + zc.y, zc.x - zk.x);   // (Zk - conj Zc)/i
                        const float2 wb = cmul(pb, make_float2(kW32re[q], kW32im[q]));
                        const float2 hv = (SDDC_FAKE & 1) ? make_float2(0.5f, 0.25f * r) : hs[t + NT * r];
                        const float2 val = cmul(cadd(A, cmul(Bi, wb)), hv);
                        a[r] = ok ? val : make_float2(0.f, 0.f);
                    }
                }
                if constexpr (R0 == 16) DFT16<+1>(a, u);
                else dft<R0, +1>(a, u);
            }
            if constexpr (!kDB) LOOP_SYNC();
            if constexpr (R0 == 16) {
#pragma unroll
                for (int r = 0; r < 16; r++) LDS_WR w1[16 * t + (r ^ x15)] = u[r];
            } else {
#pragma unroll
                for (int r = 0; r < R0; r++) w1[swz(R0 * t + r)] = u[r];
            }
            LOOP_SYNC();
            // ---- inverse pass 1 (R16, NS = R0): table twiddles W_{16 R0}^{(j%R0) r} ----
            constexpr int NB = N / 16;
            const bool act = (NB == NT) || t < NB;
            if (act) {
                float2 a[16];
                if constexpr (NB == NT) {
#pragma unroll
                    for (int r = 0; r < 16; r++) a[r] = LDS_RD(w1[sT + NT * r], u[r]);
                } else {
#pragma unroll
                    for (int r = 0; r < 16; r++) a[r] = w1[swz(t + NB * r)];
                }
#pragma unroll
                for (int r = 1; r < 16; r++)
                    a[r] = TW<+1>(a[r], (SDDC_FAKE & 2) ? make_float2(0.7f, 0.01f * (r + t % R0)) : twl[15 * 16 + (r - 1) * R0 + (t % R0)]);
                DFT16<+1>(a, u);
            }
            if constexpr (!kDB) LOOP_SYNC();
            if (act) {
                if constexpr (R0 == 16) {
                    const int b1 = (t >> 4) * 256;
#pragma unroll
                    for (int r = 0; r < 16; r++) LDS_WR w0[b1 + 16 * r + (x15 ^ r)] = u[r];
                } else {
                    const int base = (t / R0) * (16 * R0) + (t % R0);
#pragma unroll
                    for (int r = 0; r < 16; r++) w0[swz(base + R0 * r)] = u[r];
                }
            }
            LOOP_SYNC();
            // ---- inverse pass 2 (R16, NS = N/16): recurrence twiddles, overlap-discard write ----
            if (act) {
                float2 a[16];
                if constexpr (NB == NT) {
#pragma unroll
                    for (int r = 0; r < 16; r++) a[r] = LDS_RD(w0[sT + NT * r], u[r]);
                } else {
#pragma unroll
                    for (int r = 0; r < 16; r++) a[r] = w0[swz(t + NB * r)];
                }
                if constexpr (SDDC_TWTAB) {
#pragma unroll
                    for (int r = 1; r < 16; r++) a[r] = TW<+1>(a[r], (N == HALF ? ttf : tti)[(r - 1) * NB + t]);
                } else {
                    TWREC16<+1>(a, iw1, iw4);
                }
                DFT16<+1>(a, u);
                emit_frame<NB, NCO, CS16>(out, oblk + emit_base<N>(kc), kc, t, u, oa, nco);
            }
        } else {
            // ---- N <= 256: materialise the N filtered bins, then [N/16, 16] ----
            constexpr int R0 = N / 16;
            float2 tv = make_float2(0.f, 0.f);
            if (t < N) {
                const int m = t;
                const int bin = tunebin + m - (m >= N / 2 ? N : 0);
                if constexpr (SDDC_PQ)
                    tv = split_pq(w0[swz(bin & (HALF - 1))], w0[swz((HALF - bin) & (HALF - 1))], pqz[m]);
                else
                    tv = split_bin(w0, bin, pst[bin & 8191], hs[m]);
            }
            if constexpr (!kDB) LOOP_SYNC();
            if (t < N) w1[swz(t)] = tv;
            LOOP_SYNC();
            float2 u[16];
            if (t < 16) {
                float2 a[R0];
#pragma unroll
                for (int r = 0; r < R0; r++) a[r] = w1[swz(t + 16 * r)];
                dft<R0, +1>(a, u);
            }
            if constexpr (!kDB) LOOP_SYNC();
            if (t < 16) {
#pragma unroll
                for (int r = 0; r < R0; r++) w0[swz(R0 * t + r)] = u[r];
            }
            LOOP_SYNC();
            constexpr int NB = N / 16;   // = R0
            if (t < NB) {
                float2 a[16];
#pragma unroll
                for (int r = 0; r < 16; r++) a[r] = w0[swz(t + NB * r)];
#pragma unroll
                for (int r = 1; r < 16; r++) a[r] = TW<+1>(a[r], twl[15 * 16 + (r - 1) * NB + t]);
                DFT16<+1>(a, u);
                emit_frame<NB, NCO, CS16>(out, oblk + emit_base<N>(kc), kc, t, u, oa, nco);
            }
        }
        if constexpr (kDB) {   // the next frame writes the buffer this frame's last pass did not read
            float2 *tmp = w0;
            w0 = w1;
            w1 = tmp;
        }
    }
}

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
            DFT16<-1>(a, v);
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
            DFT16<+1>(a, u);
        }
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 16; r++) {
            P[16 * t + (r ^ x15)] = v[r];
            Q[16 * t + (r ^ x15)] = u[r];
        }
        LOOP_SYNC();
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
            DFT16<-1>(a, v);
            DFT16<+1>(c, u);
        }
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 16; r++) {
            P[b1 + 16 * r + (x15 ^ r)] = v[r];
            Q[b1 + 16 * r + (x15 ^ r)] = u[r];
        }
        LOOP_SYNC();
        // ---- phase 2: forward pass 2 of f -> Z | inverse pass 2 of f-1 -> overlap-discard store ----
        {
            float2 a[16], c[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                a[r] = P[sT + NT * r];
                c[r] = Q[sT + NT * r];
            }
            TWREC16<-1>(a, fw1, fw4);
            TWREC16<+1>(c, fw1, fw4);
            DFT16<-1>(a, v);
            DFT16<+1>(c, u);
        }
        if (f > f0) {
            emit_frame<N / 16, NCO, CS16>(out, gblk * 8 * N + emit_base<N>(gk), gk, t, u, oa, nco);
            if (++gk == FRAMES) {
                gk = 0;
                ++gblk;
            }
        }
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 16; r++) P[sT + NT * r] = v[r];   // Z, natural order
        LOOP_SYNC();
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
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(8 * t + r)] = v[r];
        LOOP_SYNC();
        // ---- forward passes 1 (NS 8) and 2 (NS 64): table twiddles ----
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
#pragma unroll
            for (int r = 1; r < 8; r++) a[r] = TW<-1>(a[r], twl[(r - 1) * 8 + (t & 7)]);
            dft8<-1>(a, v);
        }
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(64 * (t >> 3) + (t & 7) + 8 * r)] = v[r];
        LOOP_SYNC();
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
#pragma unroll
            for (int r = 1; r < 8; r++) a[r] = TW<-1>(a[r], twl[56 + (r - 1) * 64 + (t & 63)]);
            dft8<-1>(a, v);
        }
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(512 * (t >> 6) + (t & 63) + 64 * r)] = v[r];
        LOOP_SYNC();
        // ---- forward pass 3 (NS 512): recurrence twiddles W_4096^{t r} -> Z, natural order ----
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
            twiddle_rec8<-1>(a, fw1, fw4);
            dft8<-1>(a, v);
        }
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sT + NT8 * r] = v[r];
        LOOP_SYNC();
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
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(8 * t + r)] = u[r];
        LOOP_SYNC();
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
#pragma unroll
            for (int r = 1; r < 8; r++) a[r] = TW<+1>(a[r], twl[(r - 1) * 8 + (t & 7)]);
            dft8<+1>(a, u);
        }
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(64 * (t >> 3) + (t & 7) + 8 * r)] = u[r];
        LOOP_SYNC();
        {
            float2 a[8];
#pragma unroll
            for (int r = 0; r < 8; r++) a[r] = lds[sT + NT8 * r];
#pragma unroll
            for (int r = 1; r < 8; r++) a[r] = TW<+1>(a[r], twl[56 + (r - 1) * 64 + (t & 63)]);
            dft8<+1>(a, u);
        }
        LOOP_SYNC();
#pragma unroll
        for (int r = 0; r < 8; r++) lds[sw8(512 * (t >> 6) + (t & 63) + 64 * r)] = u[r];
        LOOP_SYNC();
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

// Split x filter coefficients for one (d, tunebin): pq[m] = (P, Q) of inverse input m, with
// bin = tb + m - (m >= N/2 ? N : 0) (fft_mt_r2iq_impl.hpp:84-98); zero outside [0, 4096).
// Evaluated in double from the float tables and rounded once.
__global__ void build_split_filter_kernel(const float2 *__restrict__ hsel, const float2 *__restrict__ post8192,
                                          int N, int tunebin, float4 *__restrict__ pq)
{
    const int m = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (m >= N) return;
    const int bin = tunebin + m - (m >= N / 2 ? N : 0);
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bin >= 0 && bin < HALF) {
        const double hr = hsel[m].x, hi = hsel[m].y;
        const double wr = post8192[bin].x, wi = post8192[bin].y;
        // 1 - i W = (1 + wi, -wr), 1 + i W = (1 - wi, wr)
        const double pr = 1.0 + wi, pi = -wr, qr = 1.0 - wi, qi = wr;
        c.x = (float)(hr * pr - hi * pi);
        c.y = (float)(hr * pi + hi * pr);
        c.z = (float)(hr * qr - hi * qi);
        c.w = (float)(hr * qi + hi * qr);
    }
    pq[m] = c;
}

int g_occupancy[7][8] = {};
int g_cus = 0;

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

template <int D, bool RAND, bool NCO, bool CS16>
hipError_t launch_v(const KernelTables &t, const Launch &L)
{
    auto kern = r2iq_persistent_kernel<D, RAND, NCO, CS16>;
    int &occ = g_occupancy[D][(RAND ? 4 : 0) + (NCO ? 2 : 0) + (CS16 ? 1 : 0)];
    if (occ == 0) {
        int nb = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, NT, 0);
        if (e != hipSuccess) return e;
        int cus = 0;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, L.device);
        if (e != hipSuccess) return e;
        g_cus = cus;
        occ = nb > 0 ? nb : 1;
    }
    const int nframes = L.nblk * FRAMES;
    int grid = g_cus * occ;
    if (grid > nframes) grid = nframes;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, L.s, reinterpret_cast<const int *>(L.d_in),
                       L.d_out, nframes, t.tw_p1, t.tw_q1[D], t.rec_f, t.rec_i[D], t.twt_f, t.twt_i[D],
                       t.post8192, t.hsel[D], L.pq, L.tunebin, L.oa, L.nco);
    return hipGetLastError();
}

template <int D, bool RAND, bool NCO>
hipError_t launch_f(const KernelTables &t, const Launch &L, bool cs16)
{
    return cs16 ? launch_v<D, RAND, NCO, true>(t, L) : launch_v<D, RAND, NCO, false>(t, L);
}

template <int D>
hipError_t launch_d(const KernelTables &t, const Launch &L, int rand, bool cs16)
{
    const bool nco = L.nco.starts != nullptr;
    if (rand) return nco ? launch_f<D, true, true>(t, L, cs16) : launch_f<D, true, false>(t, L, cs16);
    return nco ? launch_f<D, false, true>(t, L, cs16) : launch_f<D, false, false>(t, L, cs16);
}

int g_pipe_occ[8] = {};

template <bool RAND, bool NCO, bool CS16>
hipError_t launch_pipe(const KernelTables &t, const Launch &L)
{
    auto kern = r2iq_pipe_kernel<RAND, NCO, CS16>;
    int &occ = g_pipe_occ[(RAND ? 4 : 0) + (NCO ? 2 : 0) + (CS16 ? 1 : 0)];
    if (occ == 0) {
        int nb = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, NT, 0);
        if (e != hipSuccess) return e;
        e = hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, L.device);
        if (e != hipSuccess) return e;
        occ = nb > 0 ? nb : 1;
    }
    const int nframes = L.nblk * FRAMES;
    int grid = g_cus * occ;
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

int g_r8_occ[8] = {};

template <bool RAND, bool NCO, bool CS16>
hipError_t launch_r8(const KernelTables &t, const Launch &L)
{
    auto kern = r2iq_r8_kernel<RAND, NCO, CS16>;
    int &occ = g_r8_occ[(RAND ? 4 : 0) + (NCO ? 2 : 0) + (CS16 ? 1 : 0)];
    if (occ == 0) {
        int nb = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, NT8, 0);
        if (e != hipSuccess) return e;
        e = hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, L.device);
        if (e != hipSuccess) return e;
        occ = nb > 0 ? nb : 1;
    }
    const int nframes = L.nblk * FRAMES;
    int grid = g_cus * occ;
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

hipError_t launch_build_split_filter(const KernelTables &t, int d, int tunebin, float4 *pq, hipStream_t s)
{
    if (d < 0 || d > 6) return hipErrorInvalidValue;
    const int N = HALF >> d;
    hipLaunchKernelGGL(build_split_filter_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, t.hsel[d],
                       t.post8192, N, tunebin, pq);
    return hipGetLastError();
}

hipError_t launch_frames_persistent(const KernelTables &t, int d, const int16_t *d_in, int nblk, void *d_out,
                                    const float4 *pq, int tunebin, int lsb, int rand, int cs16, float cs16_scale,
                                    const float2 *nco_starts, const float2 *nco_trig, int device, hipStream_t s)
{
    const Launch L{d_in, nblk, d_out, pq, tunebin, device, s, OutArgs{lsb ? 0x80000000u : 0u, cs16_scale},
                   NcoArgs{nco_starts, nco_trig}};
    const bool f = cs16 != 0;
    switch (d) {
    case 0: return launch_d<0>(t, L, rand, f);
    case 1: return launch_d<1>(t, L, rand, f);
    case 2: return launch_d<2>(t, L, rand, f);
    case 3: return launch_d<3>(t, L, rand, f);
    case 4: return launch_d<4>(t, L, rand, f);
    case 5: return launch_d<5>(t, L, rand, f);
    case 6: return launch_d<6>(t, L, rand, f);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace sddc
