// ddc_wave.hip — d = 0 single-channel r2iq kernel for gfx950: one wave64 per frame,
// 64 points per lane in registers, 4096 = 64 x 64.
//
// The per-frame algorithm is the reference's (Core/fft_mt_r2iq_impl.hpp:76-138:
// convert_float, r2c 8192, shift x filter, c2c 4096 backward, overlap-discard copy), laid
// out so that a frame never leaves its wave:
//
//   load      lane L, register r  <-  z[L + 64 r]  (z[n] = s[2n] + i s[2n+1], one dword)
//   F1        DFT-64 over r in registers; x W_4096^{L q}           (table twF[q][L])
//   exchange  LDS transpose, two 16 KB phases; v_permlane32_swap gives lane l the full
//             column colF(l) of the 64 x 64 matrix (columns paired {c, 64-c}, {0, 32})
//   F2        DIF on the top row bit, two DFT-32s: Z[c + 64 p] for even p (S) / odd p (D);
//             D rotated by 32 lanes so a lane holds column c even-p and column 64-c odd-p,
//             i.e. every bin's mirror -k is in the same lane (lanes 0, 32: own column)
//   split     T = Z_k P + conj(Z_-k) Q in registers, (P, Q) per (register, lane) for the
//             current tune bin (pqW, built by build_wave_tables_kernel)
//   I1        DIT on the parity of p: two backward DFT-32s, odd half x W_64^{-n}, D rotated
//             back, butterflies: lane l holds G[n], n = 0..63, of one m_lo; x twI[n][l]
//   exchange  LDS transpose (two phases) + v_permlane32_swap: lane l holds column n_lo = l
//   I2        DIF on the top bit of m_lo, two backward DFT-32s: y[l + 64 n_hi]; only the
//             kept n_hi are stored (the rest of the last radix stage is dead code)
//
// tools/wave_fft_model.py emulates exactly these lane/register/LDS operations in numpy and
// checks them against the direct formula and the gfx950 LDS bank rules (conflict-free).
//
// One 64-thread workgroup per wave; no s_barrier anywhere (a wave's LDS operations are
// ordered).  16.5 KB LDS per wave; persistent grid, each wave walks a contiguous frame range
// (consecutive frames share 2048 samples, which then come from the same CU's L2).
#include <hip/hip_runtime.h>

#include "variants_api.h"
#include "fft_device.hpp"
#include "ddc_device_io.hpp"

namespace sddc {
namespace {

constexpr int HALF = 4096;
constexpr int HOP = 6144;
constexpr int BLOCK = 65536;
constexpr int FRAMES = 11;
constexpr int LDS_STRIDE = 33;   // padded row: writes and reads are base + immediate, conflict-free

#ifndef SDDC_WV_FAKE
#define SDDC_WV_FAKE 0           // timing-only builds: 1 = no table loads, 2 = no LDS exchange reads,
                                 // 4 = no IQ stores, 8 = no input (DMA + LDS reads),
                                 // 16 = no v_permlane32_swap (swaps and rotations are identities),
                                 // 32 = no lane-0/32 selects
#endif

#ifndef SDDC_WV_WAVES
#define SDDC_WV_WAVES 2          // __launch_bounds__ min waves per SIMD (<= 256 VGPRs)
#endif

// (a, b) <- v_permlane32_swap(a, b): lanes 32-63 of a <-> lanes 0-31 of b, both components
__device__ __forceinline__ void swap32(float2 &a, float2 &b)
{
    if constexpr (SDDC_WV_FAKE & 16) return;
    const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
    const auto y = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
    a = make_float2(__uint_as_float(x[0]), __uint_as_float(y[0]));
    b = make_float2(__uint_as_float(x[1]), __uint_as_float(y[1]));
}

// Rotate the 32 registers d[] by 32 lanes (two swaps per register pair), except in the
// lanes where keep is set.
__device__ __forceinline__ void rotate32_except(float2 *d, bool keep)
{
#pragma unroll
    for (int a = 0; a < 32; a += 2) {
        float2 p0 = d[a], p1 = d[a + 1];
        swap32(p0, p1);   // p0 = [d0 lo | d1 lo], p1 = [d0 hi | d1 hi]
        swap32(p1, p0);   // p1 = [d0 hi | d0 lo] = rot d0, p0 = [d1 hi | d1 lo] = rot d1
        if constexpr (SDDC_WV_FAKE & 32) {
            d[a] = p1;
            d[a + 1] = p0;
        } else {
            d[a] = keep ? d[a] : p1;
            d[a + 1] = keep ? d[a + 1] : p0;
        }
    }
}

// Scheduling-region fence: keeps the table loads in their groups (the machine scheduler
// otherwise hoists all 64 (P, Q) float4 loads, 256 VGPRs, in front of the split).
#define SDDC_SB() __builtin_amdgcn_sched_barrier(0)
// LDS hand-off between the lanes of one wave: a wave's LDS operations execute in order, so
// no s_barrier / s_waitcnt is needed; the wavefront-scope fences keep the compiler from
// moving the other lanes' reads across the writes (they compile to nothing).
#define WAVE_SYNC()                                                \
    do {                                                           \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");     \
        __builtin_amdgcn_wave_barrier();                           \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");     \
    } while (0)

#ifndef SDDC_WV_LDSX
#define SDDC_WV_LDSX 1           // 0: every half-wave exchange by v_permlane32_swap; 1: the two
                                 // rotations through LDS (the half-swaps through LDS as well needed
                                 // exec-masked halves, which hipcc if-converted and spilled: 6x
                                 // slower; removed, in git history)
#endif

// The two 32-lane rotations through the (then idle) LDS exchange buffer instead of
// v_permlane32_swap: a swap issues at ~7.5 cycles per SIMD and does not overlap across waves
// (profiles/r01/wave/microbench_permlane.txt), while these 32 + 32 LDS operations per set use
// the otherwise lightly loaded LDS pipe.  Row stride LDS_STRIDE keeps them conflict-free.
//   rotate_lds(d, keep) == rotate32_except(d, keep): every lane reads lane^32's d[], the keep
//   lanes (0 and 32) read their own, so no selects
__device__ __forceinline__ void rotate_lds(float2 *d, bool keep, float2 *xl, int lane)
{
    const int w = LDS_STRIDE * lane, r = LDS_STRIDE * (keep ? lane : (lane ^ 32));
#pragma unroll
    for (int i = 0; i < 32; i++) xl[w + i] = d[i];
    WAVE_SYNC();
#pragma unroll
    for (int i = 0; i < 32; i++) d[i] = xl[r + i];
    WAVE_SYNC();
}

template <bool RAND>
__device__ __forceinline__ float derand_w(int v)
{
    const float f = (float)v;
    if constexpr (!RAND) return f;
    return __int_as_float(__float_as_int(f) ^ (v << 31));   // convert_float<rand>, fft_mt_r2iq.h:36-51
}

// Next frame's 8192 int16 (4096 dwords) into the LDS exchange buffer by LDS-DMA, natural
// order (dword n at xl + 4 n): 16 global_load_lds_dwordx4, lane-linear destinations.
__device__ __forceinline__ void load_frame_lds(const int *__restrict__ in32, int blk, int k, float2 *xl)
{
    const int *src = in32 + ((size_t)blk * BLOCK + (size_t)k * HOP) / 2 + 4 * threadIdx.x;
    int *dst = reinterpret_cast<int *>(xl);
#pragma unroll
    for (int r = 0; r < 16; r++)
        __builtin_amdgcn_global_load_lds(src + 256 * r, (__attribute__((address_space(3))) void *)(dst + 256 * r),
                                         16, 0, 0);
}

// Table twiddles R[q] *= tab[q][lane], q = 1..63, in 8 groups of 8 with the loads kept two
// groups ahead (ring w[3][8]).  tw_pre issues groups 0 and 1; the caller places it well
// before tw_apply (in front of the DFT that produces R), so the L2 latency of the first
// groups is covered by that DFT and later groups by the two groups in between.
__device__ __forceinline__ void tw_load(float2 (&w)[8], __amdgpu_buffer_rsrc_t r, unsigned l8, int g)
{
#pragma unroll
    for (int i = (g == 0); i < 8; i++)
        w[i] = (SDDC_WV_FAKE & 1) ? make_float2(__uint_as_float(0x3f000000u | l8), 0.25f) : buf_load8(r, l8, 512u * (8 * g + i));
}
__device__ __forceinline__ void tw_pre(float2 (&w)[3][8], __amdgpu_buffer_rsrc_t r, unsigned l8)
{
    tw_load(w[0], r, l8, 0);
    tw_load(w[1], r, l8, 1);
}
__device__ __forceinline__ void tw_apply(float2 *R, float2 (&w)[3][8], __amdgpu_buffer_rsrc_t r, unsigned l8)
{
#pragma unroll
    for (int g = 0; g < 8; g++) {
        if (g + 2 < 8) tw_load(w[(g + 2) % 3], r, l8, g + 2);
#pragma unroll
        for (int i = (g == 0); i < 8; i++) R[8 * g + i] = cmul(R[8 * g + i], w[g % 3][i]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// (P, Q) of split quad j: S registers j, 31-j and D registers j, 31-j
__device__ __forceinline__ void pq_load(float4 (&c)[4], __amdgpu_buffer_rsrc_t r, unsigned l16, int j)
{
    if constexpr (SDDC_WV_FAKE & 1) {
        const float f = __uint_as_float(0x3f000000u | l16);
        c[0] = c[1] = c[2] = c[3] = make_float4(f, 0.25f, 0.5f, f);
        return;
    }
    c[0] = buf_load16(r, l16, 1024u * j);
    c[1] = buf_load16(r, l16, 1024u * (31 - j));
    c[2] = buf_load16(r, l16, 1024u * (32 + j));
    c[3] = buf_load16(r, l16, 1024u * (63 - j));
}

__device__ __forceinline__ float2 split_w(float2 zk, float2 zc, float4 c)
{
    float2 v;
    v.x = zk.x * c.x - zk.y * c.y + zc.x * c.z + zc.y * c.w;
    v.y = zk.x * c.y + zk.y * c.x + zc.x * c.w - zc.y * c.z;
    return v;
}

template <bool RAND, bool NCO, bool CS16>
__global__ __launch_bounds__(64, SDDC_WV_WAVES) void r2iq_wave_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes, const float2 *__restrict__ twF,
    const float4 *__restrict__ pqW, const float2 *__restrict__ twI, int tunebin, OutArgs oa, NcoArgs nco)
{
    __shared__ __attribute__((aligned(16))) float2 xl[LDS_STRIDE * 64];

    const int G = (int)gridDim.x, wg = (int)blockIdx.x;
    const int f0 = (int)(((long long)nframes * wg) / G);
    const int f1 = (int)(((long long)nframes * (wg + 1)) / G);
    if (f0 >= f1) return;

    const int lane = (int)threadIdx.x;
    const int h = lane >> 5, lam = lane & 31;
    const bool keep = lam == 0;        // lanes 0 and 32 hold columns 0 and 32 whole
    const bool lane0 = lane == 0;
    const int col = lane < 32 ? lam : (lam == 0 ? 32 : 64 - lam);
    const int mlo = (col - tunebin) & 63;
    // LDS element offsets (per-lane part; the register part is an immediate)
    const int wF = LDS_STRIDE * lane;                   // forward writes: row L = lane
    const int rA = LDS_STRIDE * 32 * h + lam;           // reads of column lam, rows 32h + i
    const int rB = LDS_STRIDE * 32 * h + ((-lam) & 31); // forward phase 1: column colB - 32
    const int wI = LDS_STRIDE * mlo;                    // inverse writes: row m_lo

    int blk = f0 / FRAMES, k = f0 - blk * FRAMES;
    load_frame_lds(in32, blk, k, xl);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the loop's vmcnt(32) assumes >= 32 younger stores

    for (int f = f0; f < f1; f++) {
        // opaque per-iteration zero: keeps the table loads inside the loop (no LICM into spills)
        int z = 0;
        asm volatile("" : "+s"(z));
        const __amdgpu_buffer_rsrc_t rtf = buf_rsrc(twF + z), rti = buf_rsrc(twI + z), rpq = buf_rsrc(pqW + z);
        const unsigned l8 = 8u * (unsigned)lane, l16 = 16u * (unsigned)lane;
        const int kc = k, blk_c = blk, k_c = k, oblk = blk * 8 * HALF;

        float2 R[64];
        float2 tw[3][8];
        {
            float2 a[64];
            // this frame, staged by LDS-DMA.  hipcc inserts no wait between an LDS-DMA and the
            // ds_reads of its data, so wait here: the DMA is older than the 32 or 48 IQ stores
            // issued after it, so vmcnt(32) retires it without draining those stores
            asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
            const int *xi = reinterpret_cast<const int *>(xl) + lane;
#pragma unroll
            for (int r = 0; r < 64; r++) {
                const int v = (SDDC_WV_FAKE & 8) ? (int)(lane * 2654435761u + r * 40503u + f) : xi[64 * r];
                a[r] = make_float2(derand_w<RAND>((int)(short)(v & 0xffff)), derand_w<RAND>(v >> 16));
            }
            if (++k == FRAMES) {
                k = 0;
                ++blk;
            }
            __builtin_amdgcn_wave_barrier();
            tw_pre(tw, rtf, l8);
            SDDC_SB();
            dft64<-1>(a, R);   // F1
        }
        tw_apply(R, tw, rtf, l8);

        // ---- forward exchange: phase 0 (q < 32) -> U, phase 1 (q >= 32) -> V ----
#pragma unroll
        for (int q = 0; q < 32; q++) xl[wF + q] = R[q];
        WAVE_SYNC();
#pragma unroll
        for (int i = 0; i < 32; i++) R[i] = (SDDC_WV_FAKE & 2) ? R[i] : xl[rA + LDS_STRIDE * i];
        WAVE_SYNC();
#pragma unroll
        for (int q = 0; q < 32; q++) xl[wF + q] = R[32 + q];
        WAVE_SYNC();
#pragma unroll
        for (int i = 0; i < 32; i++) R[32 + i] = (SDDC_WV_FAKE & 2) ? R[32 + i] : xl[rB + LDS_STRIDE * i];
        WAVE_SYNC();

        // ---- F2: full column per lane, DIF on the row's top bit ----
        float2 S[32], D[32];
        float4 cq[3][4];   // (P, Q) of three quads: loads run two quads ahead
        {
            float2 s[32], d[32];
#pragma unroll
            for (int i = 0; i < 32; i++) {
                swap32(R[i], R[32 + i]);
                s[i] = cadd(R[i], R[32 + i]);
                d[i] = tw64<-1>(csub(R[i], R[32 + i]), i);
            }
            pq_load(cq[0], rpq, l16, 0);
            pq_load(cq[1], rpq, l16, 1);
            SDDC_SB();
            dft32<-1>(s, S);   // Z[c + 64 * 2j]
            dft32<-1>(d, D);   // Z[c + 64 * (2j + 1)]
        }
        if constexpr (SDDC_WV_LDSX) rotate_lds(D, keep, xl, lane);
        else rotate32_except(D, keep);

        // ---- split x filter (T = Z_k P + conj(Z_-k) Q), mirrors in the same lane ----
        // Generic lanes pair S[j] with D[31-j]; lane 0 (column 0) pairs S[j] with S[32-j] and
        // D[j] with D[31-j].  Quads {S[j], S[31-j], D[j], D[31-j]} in order j = 0..15 are closed
        // under both except lane 0's S[32-j], which belongs to quad j-1: it is read one quad
        // after its own, so the transform stays in place (S, D die as T is produced).
        float2 TS[32], TD[32];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int jb = 31 - j;
            if (j + 2 < 16) pq_load(cq[(j + 2) % 3], rpq, l16, j + 2);
            const float4 *c = cq[j % 3];
            const bool l0 = (SDDC_WV_FAKE & 32) ? false : lane0;
            const float2 ms0 = l0 ? S[(32 - j) & 31] : D[jb];
            const float2 ms1 = l0 ? S[(32 - jb) & 31] : D[j];
            const float2 md0 = l0 ? D[jb] : S[jb];
            const float2 md1 = l0 ? D[j] : S[j];
            TS[j] = split_w(S[j], ms0, c[0]);
            TS[jb] = split_w(S[jb], ms1, c[1]);
            TD[j] = split_w(D[j], md0, c[2]);
            TD[jb] = split_w(D[jb], md1, c[3]);
            SDDC_SB();
        }
        // ---- I1: DIT on the parity of p ----
        {
            float2 E[32], O[32];
            tw_pre(tw, rti, l8);
            SDDC_SB();
            dft32<+1>(TS, E);
            dft32<+1>(TD, O);
#pragma unroll
            for (int n = 1; n < 32; n++) O[n] = tw64<+1>(O[n], n);
            if constexpr (SDDC_WV_LDSX) rotate_lds(O, keep, xl, lane);
            else rotate32_except(O, keep);
#pragma unroll
            for (int n = 0; n < 32; n++) {
                R[n] = cadd(E[n], O[n]);
                R[n + 32] = csub(E[n], O[n]);
            }
        }
        tw_apply(R, tw, rti, l8);

        // ---- inverse exchange: phase 0 (n < 32) -> A, phase 1 (n >= 32) -> B ----
#pragma unroll
        for (int n = 0; n < 32; n++) xl[wI + n] = R[n];
        WAVE_SYNC();
#pragma unroll
        for (int i = 0; i < 32; i++) R[i] = (SDDC_WV_FAKE & 2) ? R[i] : xl[rA + LDS_STRIDE * i];
        WAVE_SYNC();
#pragma unroll
        for (int n = 0; n < 32; n++) xl[wI + n] = R[32 + n];
        WAVE_SYNC();
#pragma unroll
        for (int i = 0; i < 32; i++) R[32 + i] = (SDDC_WV_FAKE & 2) ? R[32 + i] : xl[rA + LDS_STRIDE * i];
        WAVE_SYNC();

        // ---- I2: lane l holds column n_lo = l; DIF on the top bit of m_lo ----
        float2 Ye[32], Yo[32];
        {
            float2 s[32], d[32];
#pragma unroll
            for (int i = 0; i < 32; i++) {
                swap32(R[i], R[32 + i]);
                s[i] = cadd(R[i], R[32 + i]);
                d[i] = tw64<+1>(csub(R[i], R[32 + i]), i);
            }
            // the exchange buffer is free again: stage the next frame (the swaps above consumed
            // every read of it); the last frame of the range stages itself again, unused
            __builtin_amdgcn_wave_barrier();
            if constexpr (!(SDDC_WV_FAKE & 8)) load_frame_lds(in32, f + 1 < f1 ? blk : blk_c, f + 1 < f1 ? k : k_c, xl);
            dft32<+1>(s, Ye);   // y[l + 64 * 2j]
            dft32<+1>(d, Yo);   // y[l + 64 * (2j + 1)]
        }

        // ---- overlap-discard: frame 0 keeps n in [1024, 3072), others [0, 3072) ----
        const int fbase = oblk + (kc == 0 ? -HALF / 4 : HALF / 2 + (3 * HALF / 4) * (kc - 1));
        const __amdgpu_buffer_rsrc_t ro = buf_rsrc(static_cast<char *>(out) + (long long)fbase * out_bytes<CS16>());
        const int j0 = kc == 0 ? 8 : 0;   // wave-uniform
#pragma unroll
        for (int j = 0; j < 24; j++) {
            if (j < j0) continue;
#pragma unroll
            for (int par = 0; par < 2; par++) {
                const int nhi = 2 * j + par;
                float2 v = flip(par ? Yo[j] : Ye[j], oa.lsbmask);
                if constexpr (NCO) v = nco_mix(v, nco, fbase + lane + 64 * nhi);
                if (!(SDDC_WV_FAKE & 4) || v.x == 1.2345e30f) store_iq<CS16>(v, ro, (unsigned)lane, (unsigned)(64 * nhi), oa);
            }
        }
    }
}

// Per-(tunebin) tables of the wave kernel (d = 0), evaluated in double and rounded once:
//   pqW[r][l]  (P, Q) of lane l's register r (r < 32: S set bin cS + 128 r; r >= 32: D set bin
//              cD + 64 + 128 (r - 32)), at inverse input m = (bin - tb) mod 4096, as
//              build_split_filter_kernel (zero outside the reference's band)
//   twI[n][l]  e^{+2 pi i n (cS(l) - tb) / 4096}
__global__ void build_wave_tables_kernel(const float2 *__restrict__ hsel, const float2 *__restrict__ post8192,
                                         int tunebin, float4 *__restrict__ pqW, float2 *__restrict__ twI)
{
    const int idx = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (idx >= 64 * 64) return;
    const int r = idx >> 6, l = idx & 63, lam = l & 31;
    const int cS = l < 32 ? lam : (lam == 0 ? 32 : 64 - lam);
    const int cD = l < 32 ? (lam == 0 ? 0 : 64 - lam) : (lam == 0 ? 32 : lam);
    const int kbin = r < 32 ? cS + 128 * r : cD + 64 + 128 * (r - 32);
    const int m = (kbin - tunebin) & (HALF - 1);
    const int bin = tunebin + m - (m >= HALF / 2 ? HALF : 0);
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bin >= 0 && bin < HALF) {
        const double hr = hsel[m].x, hi = hsel[m].y;
        const double wr = post8192[bin].x, wi = post8192[bin].y;
        const double pr = 1.0 + wi, pi = -wr, qr = 1.0 - wi, qi = wr;
        c.x = (float)(hr * pr - hi * pi);
        c.y = (float)(hr * pi + hi * pr);
        c.z = (float)(hr * qr - hi * qi);
        c.w = (float)(hr * qi + hi * qr);
    }
    pqW[idx] = c;
    const int e = (r * (cS - tunebin)) & (HALF - 1);   // twI row n = r
    const double a = 2.0 * 3.14159265358979323846 * (double)e / HALF;
    twI[idx] = make_float2((float)cos(a), (float)sin(a));
}

template <bool RAND, bool NCO, bool CS16>
hipError_t launch_w(const float2 *twF, const float4 *pqW, const float2 *twI, const int16_t *d_in, int nblk,
                    void *d_out, int tunebin, OutArgs oa, NcoArgs nco, int device, hipStream_t s, LaunchCache *lc)
{
    auto kern = r2iq_wave_kernel<RAND, NCO, CS16>;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(lc, reinterpret_cast<const void *>(kern), 64, device, &occ, &cus);
    if (e != hipSuccess) return e;
#ifdef SDDC_WV_OCC
    occ = occ < SDDC_WV_OCC ? occ : SDDC_WV_OCC;   // A/B builds: resident waves per CU
#endif
    const int nframes = nblk * FRAMES;
    int grid = cus * occ;
    if (grid > nframes) grid = nframes;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64), 0, s, reinterpret_cast<const int *>(d_in), d_out,
                       nframes, twF, pqW, twI, tunebin, oa, nco);
    return hipGetLastError();
}

template <bool RAND, bool NCO>
hipError_t launch_wc(const float2 *twF, const float4 *pqW, const float2 *twI, const int16_t *d_in, int nblk,
                     void *d_out, int tunebin, OutArgs oa, NcoArgs nco, bool cs16, int device, hipStream_t s,
                     LaunchCache *lc)
{
    return cs16 ? launch_w<RAND, NCO, true>(twF, pqW, twI, d_in, nblk, d_out, tunebin, oa, nco, device, s, lc)
                : launch_w<RAND, NCO, false>(twF, pqW, twI, d_in, nblk, d_out, tunebin, oa, nco, device, s, lc);
}

}  // namespace

hipError_t launch_build_wave_tables(const KernelTables &t, int tunebin, float4 *pqW, float2 *twI, hipStream_t s)
{
    hipLaunchKernelGGL(build_wave_tables_kernel, dim3(16), dim3(256), 0, s, t.hsel[0], t.post8192, tunebin, pqW,
                       twI);
    return hipGetLastError();
}

hipError_t launch_frames_wave(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out,
                              const float4 *pqW, const float2 *twI, int tunebin, int lsb, int rand, int cs16,
                              float cs16_scale, const float2 *nco_starts, const float2 *nco_trig, int device,
                              hipStream_t s)
{
    const OutArgs oa{lsb ? 0x80000000u : 0u, cs16_scale};
    const NcoArgs nco{nco_starts, nco_trig};
    const bool c = cs16 != 0, n = nco_starts != nullptr;
    if (rand)
        return n ? launch_wc<true, true>(t.twf64, pqW, twI, d_in, nblk, d_out, tunebin, oa, nco, c, device, s, t.lc)
                 : launch_wc<true, false>(t.twf64, pqW, twI, d_in, nblk, d_out, tunebin, oa, nco, c, device, s, t.lc);
    return n ? launch_wc<false, true>(t.twf64, pqW, twI, d_in, nblk, d_out, tunebin, oa, nco, c, device, s, t.lc)
             : launch_wc<false, false>(t.twf64, pqW, twI, d_in, nblk, d_out, tunebin, oa, nco, c, device, s, t.lc);
}

}  // namespace sddc
