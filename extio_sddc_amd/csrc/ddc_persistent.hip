// ddc_persistent.hip — the single-channel r2iq kernel for gfx950 (the product's default):
// persistent workgroups.
//
// The per-frame algorithm maps the reference's worker (Core/fft_mt_r2iq_impl.hpp:76-138):
//   convert (+ rand) -> r2c 8192 as a 4096-point packed complex FFT (3 radix-16 LDS passes)
//   -> split x shift x filter from the (P, Q) table of (d, tunebin), zero fill out of band
//   -> inverse mfft-point FFT (radix N/256 or N/16, then 16, 16) -> overlap-discard store
// and is laid out for throughput on MI355X:
//   * persistent grid (CUs x resident workgroups); each workgroup walks a contiguous range of
//     frames, so consecutive frames (which share 2048 input samples) stay on one CU / XCD L2;
//   * the next frame's 16 int16 pairs per thread are loaded into registers while the current
//     frame is transformed;
//   * LDS is addressed through an XOR swizzle e ^ ((e >> 4) & 15) instead of padding: 32 KB
//     per frame, and both the 16-consecutive-per-lane writes of the first pass and the
//     64-consecutive reads are bank-conflict free;
//   * twiddles: small [r][s] tables copied to LDS once per workgroup for the NS <= 16 passes,
//     a register recurrence from per-thread W^j, W^{4j} for the NS = 256 passes; the r2c split
//     twiddle and the filter are one (P, Q) float4 per inverse input (build_split_filter_kernel).
// The measured-slower layouts and the first-generation kernels are in variants/ (built into
// libsddc_ddc_variants.so); the timing-only builds of the A/B study are in git history.
#include <hip/hip_runtime.h>

#include "ddc_frame_common.hpp"
#include "ddc_queue.hpp"

namespace sddc {
namespace {

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
template <int DIR, bool EARLY>
__device__ __forceinline__ void table_twiddle(float2 *a, const float2 *tbl, int S, int j)
{
    if constexpr (EARLY) {
        float2 tw[15];
#pragma unroll
        for (int r = 1; r <= 8; r++) tw[r - 1] = tbl[(r - 1) * S + j];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 1; r <= 8; r++) a[r] = TW<DIR>(a[r], tw[r - 1]);
#pragma unroll
        for (int r = 9; r < 16; r++) tw[r - 1] = tbl[(r - 1) * S + j];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 9; r < 16; r++) a[r] = TW<DIR>(a[r], tw[r - 1]);
    } else {
#pragma unroll
        for (int r = 1; r < 16; r++) a[r] = TW<DIR>(a[r], tbl[(r - 1) * S + j]);
    }
}

// d = 3..6 (N = 512, 256, 128, 64): the N-point inverse as mixed-radix Stockham passes on the
// lanes of wave 0, radix schedule 8-8-8, 4-4-4-4, 8-4-4, 4-4-4.  The pass of radix R after a span Ns runs on
// threads j < N / R: reads elements j + (N / R) r, twiddles W_{R Ns}^{-k r} (k = j mod Ns),
// inverse DFT-R, writes (j / Ns) R Ns + k + Ns r; the last pass leaves y[j + (N / 4) r] in
// registers.  LDS element e sits at e ^ ((e >> s) & 31) (s = 3, 2, 2, 1): conflict-
// free for every read and write pattern (tools/r4_tail_model.py, which also checks the passes
// against numpy).  The [N/16, 16] form it replaces kept 16 lanes busy (d = 4) or fewer; its two
// passes cost 8-11 % of the launch at d = 4..6 (timing-only build, profiles/r03/ab).
template <int N> constexpr int tail_radix(int p) { return N == 512 || (N == 128 && p == 0) ? 8 : 4; }
template <int N> constexpr int tail_passes() { return N == 256 ? 4 : 3; }
template <int N> constexpr int tail_ns(int p)
{
    int ns = 1;
    for (int q = 0; q < p; q++) ns *= tail_radix<N>(q);
    return ns;
}
template <int N> constexpr int tail_twoff(int p)   // first twiddle of pass p in the tail's table
{
    int o = 0;
    for (int q = 1; q < p; q++) o += (tail_radix<N>(q) - 1) * tail_ns<N>(q);
    return o;
}
template <int N> constexpr int tail_twn() { return tail_twoff<N>(tail_passes<N>()); }
template <int N> __device__ __forceinline__ int tail_swz(int e) { return e ^ ((e >> (N == 64 ? 1 : N == 512 ? 3 : 2)) & 31); }

// the forward twiddle W_{R Ns}^{k r} of entry e of the tail's table
template <int N> __device__ __forceinline__ float2 tail_twiddle(const float2 *__restrict__ tw4096, int e)
{
    int p = 1;
    while (p + 1 < tail_passes<N>() && e >= tail_twoff<N>(p + 1)) p++;
    const int ns = tail_ns<N>(p), R = tail_radix<N>(p);
    const int o = e - tail_twoff<N>(p), r = o / ns + 1, kk = o % ns;
    return tw4096[(kk * r * (HALF / (R * ns))) & (HALF - 1)];
}

// the kept outputs of the last pass, u[r] = y[t + (N / R) r]: y[0, 3N/4) (k >= 1), y[N/4, 3N/4) (k = 0)
template <int N, bool NCO, bool CS16>
__device__ __forceinline__ void tail_emit(void *__restrict__ out, int fbase, int k, int t, const float2 (&u)[8],
                                          const OutArgs &oa, const NcoArgs &nco)
{
    constexpr int R = tail_radix<N>(tail_passes<N>() - 1), T = N / R;
    if (t < T) {
        const __amdgpu_buffer_rsrc_t ro = buf_rsrc(static_cast<char *>(out) + (size_t)fbase * out_bytes<CS16>());
#pragma unroll
        for (int r = 0; r < 3 * R / 4; r++) {
            if (r < R / 4 && k == 0) continue;
            float2 v = flip(u[r], oa.lsbmask);
            if constexpr (NCO) v = nco_mix(v, nco, fbase + t + T * r);
            store_iq<CS16>(v, ro, (unsigned)t, (unsigned)(T * r), oa);
        }
    }
}

// d = 2 (N = 1024; N = 2048 with SDDC_P_WGT=2): the inverse as a radix-N/256 pass from the split's registers
// (m = t + 256 r) and four radix-4 Stockham passes on all 256 threads (N / 1024 butterflies per
// thread), ping-pong between two regions of the frame buffer with one barrier per pass, instead
// of radix-16 passes on 2 waves (d = 1) or wave 0 (d = 2) while the other waves wait.  The
// twiddles of the pass after a span Ns are W_{4 Ns}^{k r} = w^r with w = W_{4 Ns}^k from an LDS
// table of (N - N/256) / 3 entries.  Element e at wg_swz(e) in either region: conflict-free
// (tools/r4_tail_model.py, stockham_wg).
template <int N> __device__ __forceinline__ int wg_swz(int e)
{
    if constexpr (N == 2048) return e ^ ((e >> 2) & 31) ^ ((e >> 5) & 7);
    else return e ^ ((e >> 2) & 31);
}
template <int N> constexpr int wg_twoff(int ns) { return (ns - N / 256) / 3; }
template <int N> constexpr int wg_twn() { return (N - N / 256) / 3; }
template <int N, int NS, bool LAST>
__device__ __forceinline__ void wg_pass(const float2 *src, float2 *dst, const float2 *twq, int t,
                                        float2 (&u)[N / 1024][4])
{
    constexpr int B = N / 1024, T = N / 4;
#pragma unroll
    for (int b = 0; b < B; b++) {
        const int j = t + 256 * b;
        float2 a[4];
#pragma unroll
        for (int r = 0; r < 4; r++) a[r] = src[wg_swz<N>(j + T * r)];
        const int kk = j & (NS - 1);
        const float2 w1 = twq[wg_twoff<N>(NS) + kk];
        const float2 w2 = cmul(w1, w1), w3 = cmul(w2, w1);
        a[1] = TW<+1>(a[1], w1);
        a[2] = TW<+1>(a[2], w2);
        a[3] = TW<+1>(a[3], w3);
        dft4<+1>(a, u[b]);
    }
    if constexpr (!LAST) {
#pragma unroll
        for (int b = 0; b < B; b++) {
            const int j = t + 256 * b, kk = j & (NS - 1);
#pragma unroll
            for (int r = 0; r < 4; r++) dst[wg_swz<N>((j / NS) * 4 * NS + kk + NS * r)] = u[b][r];
        }
        __syncthreads();
    }
}

template <int N, int P>
__device__ __forceinline__ void tail_pass(float2 *sb, const float2 *twq, int t, float2 (&u)[8])
{
    constexpr int R = tail_radix<N>(P), NS = tail_ns<N>(P), T = N / R;
    const int kk = t & (NS - 1);
    if (t < T) {
        float2 a[R];
#pragma unroll
        for (int r = 0; r < R; r++) a[r] = sb[tail_swz<N>(t + T * r)];
        if constexpr (P > 0) {
#pragma unroll
            for (int r = 1; r < R; r++) a[r] = TW<+1>(a[r], twq[tail_twoff<N>(P) + (r - 1) * NS + kk]);
        }
        if constexpr (R == 8) dft8<+1>(a, u);
        else dft4<+1>(a, u);
    }
    if constexpr (P + 1 < tail_passes<N>()) {
        wave_lds_sync();   // this wave's reads of the pass are done
        if (t < T) {
#pragma unroll
            for (int r = 0; r < R; r++) sb[tail_swz<N>((t / NS) * R * NS + kk + NS * r)] = u[r];
        }
        wave_lds_sync();
    }
}

template <int D, bool RAND, bool NCO, bool CS16>
__global__ __launch_bounds__(NT, D <= 1 ? 4 : 2) void r2iq_persistent_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes,
    const float2 *__restrict__ tw_p1, const float2 *__restrict__ tw_q1,
    const float2 *__restrict__ rec_f, const float2 *__restrict__ rec_i, const float2 *__restrict__ tw4096,
    const float4 *__restrict__ pq, int tunebin, OutArgs oa, NcoArgs nco, unsigned *__restrict__ wq)
{
    constexpr int N = HALF >> D;
    // d >= 2 (N <= 1024): the inverse reads only the band [s0, s0 + N) of Z and its mirror
    // [m0, m0 + N) (s0 = tb - N/2, m0 = 1 - s0 - N, mod 4096).  Forward pass 2 then writes
    // only the NB of its 16 outputs per thread that can fall in either window: its twiddle
    // bases are rotated by 256 r0 (r0 = s0 / 256), so output register r holds bin
    // t + 256 (r + r0) and the band sits in registers 0 .. NB - 1, the mirror in
    // MREL .. MREL + NB - 1 (mod 16; a uniform test per register).  4 of 16 Z writes per
    // thread at d >= 4, 6 at d = 3, 10 at d = 2: +5-7 % at d = 3..6, +2-3 % at d = 2
    // (profiles/r02/ab/prune_d3_6.txt, prune_d2.txt).
    constexpr bool PRUNE = N <= 1024;
    constexpr bool TW_EARLY = D <= 1;   // (held to 128 VGPRs by the launch bounds)
    // st_row stores: the forward pass-0 rows at d >= 1 only (at d = 0 1.2-1.7 % slower), the
    // other rows at every d (inverse pass-0 rows at d = 0: +0.9-1.3 % on one box, xst_d0_parts.txt,
    // neutral on another, xst_inv0_confirm.txt; bit-identical, 15 VALU fewer)
    constexpr bool XST = D >= 1, XF0 = XST, XI0 = true;
    constexpr int NB = N >= 512 ? N / 256 + 1 : 2;
    const int s0 = (tunebin - N / 2) & (HALF - 1), r0 = PRUNE ? s0 >> 8 : 0;
    // Z (forward pass 2 -> split) is stored without the XOR swizzle, bin j at j: the split's
    // reads are runs of consecutive bins, ascending (Z_k) and descending (the mirror), which an
    // XOR swizzle turns into one 2-way bank conflict per 32-lane group wherever a run crosses a
    // 16-bin block (32 conflict cycles per wave-frame at d = 0), while the pass-2 writes (16
    // consecutive bins per instruction) need no swizzle.
    // d <= 1: Z is stored rotated by the tune bin, bin j at (j - tb) mod 4096, so the
    // inverse's reads of bins tb + m are t + 256 r with no wrap (the mirror reads keep theirs).
    // Forward pass 2 gets it for free: per-lane twiddle bases rotated by 256 zr make output
    // register r hold bin t + 256 (r + zr), i.e. tb + ((t - tb) mod 256) + 256 r.  d = 0 +1.5-2 %,
    // d = 1 +1 % (profiles/r02/ab/zrot.txt).
    constexpr bool ZROT = !PRUNE;
    const int zd = tunebin & 255;
    const int mrel = ((((1 - s0 - N) & (HALF - 1)) >> 8) - r0) & 15;
    // d >= 5: the pruned pass 2 keeps registers {0, 1, mrel, mrel + 1}, i.e. the DFT-16 output
    // groups k1 = r & 3 in {0, 1, mrel & 3, (mrel + 1) & 3}; groups 2, 3 are computed only when
    // the mirror needs them (dft16_groups, uniform flags): d = 5, 6 +1-2.8 % (tb 192 / 1024),
    // bit-identical, d = 4 unchanged (profiles/r02/ab/grp5_d5_6*.txt).  At
    // d = 4 the branches raise the kernel to 142 VGPRs (3 waves/SIMD, 9-13 % slower; held to 128
    // it spills), so d = 4 keeps dft16 (profiles/r02/ab/grp_partial_dft16*.txt).
    constexpr bool GRP = PRUNE && NB == 2 && D >= 5;
    const bool need2 = ((mrel & 3) - 1u) <= 1u, need3 = (mrel & 3) >= 2;
    __shared__ __attribute__((aligned(16))) float2 lds[HALF];
    // pass-1 twiddle tables, copied once per workgroup: [15][16] forward, [15][S] inverse
    constexpr int SQ = N >= 512 ? N / 256 : N / 16;
    // d >= 4: the inverse runs as Stockham passes on wave 0 (tail_pass); their twiddles take the
    // inverse table's place
#ifndef SDDC_P_R4TAIL
#define SDDC_P_R4TAIL 1
#endif
    constexpr bool R4T = SDDC_P_R4TAIL && (N <= 256 || N == 512);
#ifndef SDDC_P_WGT
#define SDDC_P_WGT 1
#endif
    // d = 2 only: at d = 1 (N = 2048, two butterflies per thread per pass) the same form measured
    // 7-8 % slower than the two-wave radix-16 tail (profiles/r03/ab/d12_wg.txt)
    constexpr bool WGT = SDDC_P_WGT && (N == 1024 || (SDDC_P_WGT > 1 && N == 2048));
    constexpr int TWQ = R4T ? tail_twn<N>() : WGT ? wg_twn<N>() : 15 * SQ;
    __shared__ __attribute__((aligned(16))) float2 twl[15 * 16 + TWQ];
    float2 *const w0 = lds, *const w1 = lds;   // the pass buffers (one 32 KB frame buffer)
    // d >= 2: the inverse's last passes run on one wave (N/16 <= 64 butterflies), so they are
    // ordered within that wave (wave_lds_sync) and the other waves go on to the next frame's
    // pass 0.  N <= 256: the filtered bins go to their own buffer sb (N <= 256 float2, 2 KB),
    // so the split needs no barrier between its Z reads and its writes.  7 barriers per frame
    // instead of 10 at d >= 4, 8 at d = 2, 3: d = 4 +1 %, d = 5, 6 +0.5 %, d = 2, 3 neutral,
    // bit-identical (profiles/r02/ab/winv.txt); LDS at d = 4 38.7 KB, still 4 workgroups per CU.
    constexpr bool WINV = N <= 1024;
    constexpr bool SEPB = N <= 256;
    __shared__ __attribute__((aligned(16))) float2 sb[SEPB ? N : 1];

    const int tid = (int)threadIdx.x;
    const int G = (int)gridDim.x, w = (int)blockIdx.x;
    // d <= 2: frames come from the dynamic frame queue (ddc_queue.hpp), worked by wave 3: the frame
    // after the next one is resolved in the middle of each frame (the next one's input is
    // prefetched at the frame's start), from a ticket taken a frame earlier.  d = 1 +4 %, d = 2
    // +1 %, but d = 3 -2 % and d = 4 -4 % (their inverse runs on one wave, and the queue's scalar
    // state spills), so d >= 3 (and SDDC_P_QUEUE=0, timing only) keep the static contiguous split
    // (profiles/r03/ab/pq_dynamic_queue_d1_4.txt).
#ifndef SDDC_P_QUEUE
#define SDDC_P_QUEUE 1
#endif
#ifndef SDDC_P_QUEUE_DMAX   // re-measured after the d >= 3 tail rewrite: still 2-14 % slower at d = 3..6
#define SDDC_P_QUEUE_DMAX 2   // (profiles/r03/ab/p_queue_d3_6_after_tails.txt)
#endif
    constexpr bool PQ = SDDC_P_QUEUE && D <= SDDC_P_QUEUE_DMAX;
    __shared__ int s_first, s_next;
    constexpr int QLANE = 64 * 3;
    const bool qw = __builtin_amdgcn_readfirstlane(tid >> 6) == 3;
    const int f1s = (int)(((long long)nframes * (w + 1)) / G);   // the static split's range end
    FsQueue q;
#ifndef SDDC_P_SFIRST
#define SDDC_P_SFIRST 1
#endif
    // the first two frames static (fs_static_frame): no atomic round trip before the first frame
    constexpr int PSTAT = SDDC_P_SFIRST ? 2 : 0;
    if constexpr (PQ) q.init(wq, nframes, w & (FS_SHARDS - 1), PSTAT ? G : 0, PSTAT ? PSTAT : 1);
    if (qw) {
        int g0, g1;
        if constexpr (PQ) {
            g0 = PSTAT ? fs_static_frame(nframes, G, w, 0, PSTAT) : -1;
            g1 = PSTAT ? fs_static_frame(nframes, G, w, 1, PSTAT) : -1;
            if (g0 < 0) {   // no static frames (small batches): both from the queue
                q.take();
                q.peek();
                g0 = q.resolve();
            }
            if (g1 < 0) {
                q.take();
                q.peek();
                g1 = g0 >= 0 ? q.resolve() : -1;
            }
            q.take();
        } else {
            const int f0 = (int)(((long long)nframes * w) / G);
            g0 = f0 < f1s ? f0 : -1;
            g1 = f0 + 1 < f1s ? f0 + 1 : -1;
        }
        if (tid == QLANE) {
            s_first = g0;
            s_next = g1;
        }
    }

    // per-thread constants, live for the whole frame loop
    const int zr = ZROT ? (tunebin >> 8) + (tid < zd ? 1 : 0) : r0;
    const float2 fw1_ = tw4096[(tid + 256 * zr) & (HALF - 1)];   // rotated bases (PRUNE: r0, ZROT: zr)
    const float2 fw4_ = tw4096[(4 * tid + 1024 * zr) & (HALF - 1)];
    float2 iw1_ = ZROT ? rec_f[tid] : fw1_, iw4_ = ZROT ? rec_f[NT + tid] : fw4_;
    if constexpr (N >= 512 && N < HALF) {
        if (tid < N / 16) {
            iw1_ = rec_i[tid];
            iw4_ = rec_i[NT + tid];
        }
    }
    for (int i = tid; i < 15 * 16 + TWQ; i += NT) {
        if ((!R4T && !WGT) || i < 15 * 16) {
            twl[i] = i < 15 * 16 ? tw_p1[i] : tw_q1[i - 15 * 16];   // visible after the first frame's pass-0 barrier
        } else if constexpr (R4T) {
            twl[i] = tail_twiddle<N>(tw4096, i - 15 * 16);
        } else if constexpr (WGT) {
            const int e = i - 15 * 16;   // W_{4 Ns}^k, Ns = N/256 x 1, 4, 16, 64
            constexpr int r0 = N / 256;
            const int ns = e < wg_twoff<N>(4 * r0) ? r0 : e < wg_twoff<N>(16 * r0) ? 4 * r0
                         : e < wg_twoff<N>(64 * r0) ? 16 * r0 : 64 * r0;
            twl[i] = tw4096[((e - wg_twoff<N>(ns)) * (HALF / (4 * ns))) & (HALF - 1)];
        }
    }

    __syncthreads();   // s_first, s_next
    int f = s_first;
    int blk = f / FRAMES, k = f - blk * FRAMES;
    int x[16];
    if (f >= 0) load_frame(in32, blk, k, x);

    while (f >= 0) {
        const int fn = s_next;   // the next frame (written in the previous frame's middle)
        // Opaque per-iteration copies of the thread index and table pointers: without
        // them the compiler hoists every loop-invariant LDS address and table load out
        // of the frame loop and spills them.
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z;
        const float4 *pqz = pq + z;
        float2 fw1 = fw1_, fw4 = fw4_, iw1 = iw1_, iw4 = iw4_;
        asm volatile("" : "+v"(fw1), "+v"(fw4), "+v"(iw1), "+v"(iw4));
        const int sT = swz(t);            // swz(t + 256 r) = sT + 256 r
        const int x15 = t & 15;
        // row-store bases (st_row): 16 t + (r ^ x15) and 256 (t >> 4) + 16 r + (r ^ x15)
        const unsigned xa0 = 128u * (unsigned)t + 8u * (unsigned)x15;
        const unsigned xa1 = 2048u * (unsigned)(t >> 4) + 8u * (unsigned)x15;
        const int oblk = blk * 8 * N;   // first output slot of the block (batch-relative)
        const int kc = k;
        // ---- forward pass 0 (R16, NS1): convert + DFT16 from registers ----
        float2 v[16];
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++)
                if constexpr (RAND) {
                    // convert_float<rand> on the int16 pair itself: an odd sample is XORed with
                    // 0xFFFE (fft_mt_r2iq.h:36-51), i.e. word ^ (word & 0x10001) * 0xFFFE; the
                    // conversion then stays integer-exact, as without RAND (the compiler's int16
                    // first-stage butterflies apply): -17 VALU, the d = 0 RAND kernels' 2 spills
                    // gone; with RAND + LSB d = 0 0 to +0.9 %, d = 1 neutral, d = 4 +1.1 %,
                    // bit-identical (profiles/r02/ab/irand_rand_lsb.txt)
                    const int w = x[r] ^ (int)(((unsigned)x[r] & 0x10001u) * 0xFFFEu);
                    a[r] = make_float2((float)(int)(short)(w & 0xffff), (float)(w >> 16));
                } else {
                    a[r] = make_float2((float)(int)(short)(x[r] & 0xffff), (float)(x[r] >> 16));
                }
            if (fn >= 0) {   // prefetch the next frame
                blk = fn / FRAMES;
                k = fn - blk * FRAMES;
                load_frame(in32, blk, k, x);
            }
            dft16<-1>(a, v);
        }
        __syncthreads();   // the previous frame's last LDS reads are done
#pragma unroll
        for (int r = 0; r < 16; r++)   // swz(16t + r)
            if constexpr (XF0) st_row(w0, xa0, r, 0, v[r]);
            else w0[16 * t + (r ^ x15)] = v[r];
        __syncthreads();
        // ---- forward pass 1 (R16, NS16): table twiddles W_256^{(t%16) r} ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], w0[sT + NT * r]);
            table_twiddle<-1, TW_EARLY>(a, twl, 16, x15);
            dft16<-1>(a, v);
        }
        __syncthreads();
        {
            const int b1 = (t >> 4) * 256;                                     // swz(b1 + x15 + 16 r)
#pragma unroll
            for (int r = 0; r < 16; r++)
                if constexpr (XST) st_row(w1, xa1, r, 16, v[r]);
                else w1[b1 + 16 * r + (x15 ^ r)] = v[r];
        }
        __syncthreads();
        // ---- forward pass 2 (R16, NS256): recurrence twiddles W_4096^{t r} ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], w1[sT + NT * r]);
            twiddle_rec16<-1>(a, fw1, fw4);
            if constexpr (GRP) dft16_groups<-1>(a, v, need2, need3);
            else dft16<-1>(a, v);
        }
        __syncthreads();
        if constexpr (PRUNE) {
#pragma unroll
            for (int r = 0; r < 16; r++)   // Z, natural order: the band's and the mirror's registers
                if (r < NB || ((r - mrel) & 15) < NB) w0[t + NT * ((r + r0) & 15)] = v[r];
        } else {
            const int sZ = (t - zd) & 255;
#pragma unroll
            for (int r = 0; r < 16; r++) w0[sZ + NT * r] = v[r];   // Z, rotated by tb
        }
        if (qw) {   // the frame after the next one (read by every wave at the next frame's start)
            if constexpr (PQ) {
                q.peek();
                const int g = q.resolve();
                if (tid == QLANE) s_next = g;
                q.take();
            } else if (tid == QLANE) {
                s_next = fn >= 0 && fn + 1 < f1s ? fn + 1 : -1;
            }
        }
        __syncthreads();

        if constexpr (N >= 512) {
            constexpr int R0 = N / 256;
            // ---- inverse pass 0 (R0, NS1): r2c split x filter, bins tb-N/2 .. tb+N/2 ----
            float2 u[16];
            {
                const int b0 = tunebin + t;                  // bin of r = 0
                const int sb0 = b0;
                // mirror bin, same separability (rotated storage: HALF - b0 - tb)
                const int sc0 = ZROT ? (HALF - b0 - tunebin) & (HALF - 1) : HALF - b0;   // (PRUNE: d = 2, 3)
                const char *w0b = reinterpret_cast<const char *>(w0);
                const unsigned sb0b = 8u * (unsigned)sb0, sc0b = 8u * (unsigned)sc0, tb16 = 16u * (unsigned)t;
                const __amdgpu_buffer_rsrc_t rpq = buf_rsrc(pqz);
                float2 a[R0];
#pragma unroll
                for (int r = 0; r < R0; r++) {
                    const bool wrap = (NT * r >= N / 2);
                    const int sh = NT * r - (wrap ? N : 0);
                    // branch-free: read a valid (wrapped) address, out-of-band bins have P = Q = 0;
                    // byte offsets: the wrap is one AND, the scale folds away
                    float2 zk;
                    // unpaired (XRD) at d = 1: +1 %; at d = 0 the clobbers cost 5 % (profiles/r02/ab/zrot.txt)
                    if constexpr (ZROT && D > 0) XRD(zk, w0[t + (sh & (HALF - 1))]);
                    else if constexpr (ZROT) zk = w0[t + (sh & (HALF - 1))];
                    else zk = *reinterpret_cast<const float2 *>(w0b + ((sb0b + 8u * (unsigned)sh) & (8u * HALF - 8u)));
                    const float2 zc = *reinterpret_cast<const float2 *>(w0b + ((sc0b - 8u * (unsigned)sh) & (8u * HALF - 8u)));
                    a[r] = split_pq(zk, zc, buf_load16(rpq, tb16, 16u * NT * r));
                }
                if constexpr (WGT) {
                    constexpr int B = N / 1024, T = N / 4;
                    {
                        float2 u0[R0];
                        if constexpr (R0 == 8) dft8<+1>(a, u0);   // pass 0 (Ns = 1)
                        else dft4<+1>(a, u0);
                        __syncthreads();   // every wave's Z reads are done
#pragma unroll
                        for (int r = 0; r < R0; r++) w1[wg_swz<N>(R0 * t + r)] = u0[r];
                    }
                    __syncthreads();
                    float2 *const ra = w1, *const rb = w1 + N;
                    const float2 *twq = twl + 15 * 16;
                    float2 u4[B][4];
                    wg_pass<N, R0, false>(ra, rb, twq, t, u4);
                    wg_pass<N, 4 * R0, false>(rb, ra, twq, t, u4);
                    wg_pass<N, 16 * R0, false>(ra, rb, twq, t, u4);
                    wg_pass<N, 64 * R0, true>(rb, ra, twq, t, u4);
                    // u4[b][r] = y[t + 256 b + (N/4) r]; kept: y[0, 3N/4) (k >= 1), y[N/4, 3N/4) (k = 0)
                    const int fbase = oblk + emit_base<N>(kc);
                    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(static_cast<char *>(out) + (size_t)fbase * out_bytes<CS16>());
#pragma unroll
                    for (int r = 0; r < 3; r++) {
                        if (r == 0 && kc == 0) continue;
#pragma unroll
                        for (int b = 0; b < B; b++) {
                            const int n = t + 256 * b + T * r;
                            float2 vv = flip(u4[b][r], oa.lsbmask);
                            if constexpr (NCO) vv = nco_mix(vv, nco, fbase + n);
                            store_iq<CS16>(vv, ro, (unsigned)t, (unsigned)(256 * b + T * r), oa);
                        }
                    }
                    f = fn;
                    continue;
                }
                if constexpr (N == 512 && R4T) {
                    // d = 3: the 512 filtered bins (inverse input m = t + 256 r) go to LDS, and wave 0
                    // runs the inverse as three radix-8 Stockham passes (tail_pass) instead of the
                    // radix-2 pass on every thread and two radix-16 passes on 32 lanes
                    __syncthreads();   // every wave's Z reads are done
#pragma unroll
                    for (int r = 0; r < R0; r++) w1[tail_swz<N>(t + NT * r)] = a[r];
                    __syncthreads();
                    if (t < 64) {
                        float2 v8[8];
                        const float2 *twq = twl + 15 * 16;
                        tail_pass<N, 0>(w1, twq, t, v8);
                        tail_pass<N, 1>(w1, twq, t, v8);
                        tail_pass<N, 2>(w1, twq, t, v8);
                        tail_emit<N, NCO, CS16>(out, oblk + emit_base<N>(kc), kc, t, v8, oa, nco);
                    }
                    f = fn;
                    continue;
                }
                if constexpr (R0 == 16) dft16<+1>(a, u);
                else dft<R0, +1>(a, u);
            }
            __syncthreads();
            if constexpr (R0 == 16) {
#pragma unroll
                for (int r = 0; r < 16; r++)
                    if constexpr (XI0) st_row(w1, xa0, r, 0, u[r]);
                    else w1[16 * t + (r ^ x15)] = u[r];
            } else {
#pragma unroll
                for (int r = 0; r < R0; r++) LX(w1, R0 * t, r) = u[r];
            }
            __syncthreads();
            // ---- inverse pass 1 (R16, NS = R0): table twiddles W_{16 R0}^{(j%R0) r} ----
            constexpr int NB = N / 16;
            const bool act = (NB == NT) || t < NB;
            if (act) {
                float2 a[16];
                if constexpr (NB == NT) {
#pragma unroll
                    for (int r = 0; r < 16; r++) XRD(a[r], w1[sT + NT * r]);
                } else {
#pragma unroll
                    for (int r = 0; r < 16; r++) a[r] = LX(w1, t, NB * r);
                }
#ifdef SDDC_FAKE_TAIL2   // timing only: no arithmetic in inverse passes 1, 2 (wrong results)
#pragma unroll
                for (int r = 0; r < 16; r++) u[r] = a[r];
#else
                table_twiddle<+1, TW_EARLY>(a, twl + 15 * 16, R0, t % R0);
                dft16<+1>(a, u);
#endif
            }
            if constexpr (WINV) wave_lds_sync();
            else __syncthreads();
            if (act) {
                if constexpr (R0 == 16) {
                    const int b1 = (t >> 4) * 256;
#pragma unroll
                    for (int r = 0; r < 16; r++)
                        if constexpr (XST) st_row(w0, xa1, r, 16, u[r]);
                        else w0[b1 + 16 * r + (x15 ^ r)] = u[r];
                } else {
                    const int base = (t / R0) * (16 * R0) + (t % R0);
#pragma unroll
                    for (int r = 0; r < 16; r++) LX(w0, base, R0 * r) = u[r];
                }
            }
            if constexpr (WINV) wave_lds_sync();
            else __syncthreads();
            // ---- inverse pass 2 (R16, NS = N/16): recurrence twiddles, overlap-discard write ----
            if (act) {
                float2 a[16];
                if constexpr (NB == NT) {
#pragma unroll
                    for (int r = 0; r < 16; r++) XRD(a[r], w0[sT + NT * r]);
                } else {
#pragma unroll
                    for (int r = 0; r < 16; r++) a[r] = LX(w0, t, NB * r);
                }
#ifdef SDDC_FAKE_TAIL2
#pragma unroll
                for (int r = 0; r < 16; r++) u[r] = a[r];
#else
                twiddle_rec16<+1>(a, iw1, iw4);
                dft16<+1>(a, u);
#endif
                emit_frame<NB, NCO, CS16>(out, oblk + emit_base<N>(kc), kc, t, u, oa, nco);
            }
        } else {
            // ---- N <= 256: materialise the N filtered bins, then [N/16, 16] ----
            constexpr int R0 = N / 16;
            float2 tv = make_float2(0.f, 0.f);
            if (t < N) {
                const int m = t;
                const int bin = tunebin + m - (m >= N / 2 ? N : 0);
                tv = split_pq(w0[bin & (HALF - 1)], w0[(HALF - bin) & (HALF - 1)], pqz[m]);
            }
            if constexpr (R4T) {
                if (t < N) sb[tail_swz<N>(t)] = tv;
                __syncthreads();
                if (t < 64) {
                    float2 u[8];
                    const float2 *twq = twl + 15 * 16;
                    tail_pass<N, 0>(sb, twq, t, u);
                    tail_pass<N, 1>(sb, twq, t, u);
                    tail_pass<N, 2>(sb, twq, t, u);
                    if constexpr (tail_passes<N>() == 4) tail_pass<N, 3>(sb, twq, t, u);
                    tail_emit<N, NCO, CS16>(out, oblk + emit_base<N>(kc), kc, t, u, oa, nco);
                }
                f = fn;
                continue;
            }
            // SEPB: the bins go to sb, and wave 0 alone runs the two passes below on sb
            float2 *const v0 = SEPB ? sb : w1, *const v1 = SEPB ? sb : w0;
            if constexpr (!SEPB) __syncthreads();
            if (t < N) v0[swz(t)] = tv;
            __syncthreads();
            float2 u[16];
            if (t < 16) {
                float2 a[R0];
#pragma unroll
                for (int r = 0; r < R0; r++) a[r] = LX(v0, t, 16 * r);
#ifdef SDDC_FAKE_TAIL   // timing only: no inverse arithmetic at N <= 256 (wrong results)
#pragma unroll
                for (int r = 0; r < R0; r++) u[r] = a[r];
#else
                dft<R0, +1>(a, u);
#endif
            }
            if constexpr (SEPB) wave_lds_sync();
            else __syncthreads();
            if (t < 16) {
#pragma unroll
                for (int r = 0; r < R0; r++) LX(v1, R0 * t, r) = u[r];
            }
            if constexpr (SEPB) wave_lds_sync();
            else __syncthreads();
            constexpr int NB = N / 16;   // = R0
            if (t < NB) {
                float2 a[16];
#pragma unroll
                for (int r = 0; r < 16; r++) a[r] = LX(v1, t, NB * r);
#ifdef SDDC_FAKE_TAIL
#pragma unroll
                for (int r = 0; r < 16; r++) u[r] = a[r];
#else
#pragma unroll
                for (int r = 1; r < 16; r++) a[r] = TW<+1>(a[r], twl[15 * 16 + (r - 1) * NB + t]);
                dft16<+1>(a, u);
#endif
                emit_frame<NB, NCO, CS16>(out, oblk + emit_base<N>(kc), kc, t, u, oa, nco);
            }
        }
        f = fn;
    }
    if constexpr (PQ)
        if (tid == QLANE) fs_queue_done(wq, (unsigned)G);
}

// ---------------------------------------------------------------------------------------------
// d = 0, fused split (FS): the forward pass 2, the r2c split x filter and the inverse pass 0 of
// a frame run in registers, with no LDS exchange between them.
//
// Forward pass 2's butterfly on lane l is column c = kFsPerm[l]: it produces Z[c + 256 k],
// k = 0..15.  The split of bin b needs Z[-b]; for b = c + 256 k that is Z[(256 - c) + 256 (15 - k)],
// and lane l ^ 1 holds column 256 - c (the permutation pairs the lanes), so the mirror is the
// partner lane's register 15 - k: a DPP quad_perm [1,0,3,2] operand of the split's FMAs
// (v_fmac_f32_dpp, no extra instruction).  The self-mirrored columns 0 and 128 (lanes 0, 1 of
// wave 0) read their own registers instead (a wave-uniform branch, selects in wave 0 only).
//
// The inverse then runs on absolute bin indices: inverse pass 0's butterfly c takes the split
// values of bins c + 256 s, i.e. the lane's own registers.  The tune shift, which the reference
// applies as an input offset (T[m] = X[tb + m] H[m], impl.hpp:84-96), becomes the output
// modulation y[n] = e^{-2 pi i tb n / 4096} y'[n] (y' the inverse FFT over bins):
//   n = t + 256 k:  e^{-2 pi i tb t / 4096} (lane factor g_t, folded into the last pass's
//   twiddles) x W_16^{(tb mod 16) k} (a quarter turn per output register: tb is a multiple of 4).
// The (P, Q) table is indexed by bin (zero out of band) and laid out in lane order.
// Removed per frame: the Z exchange (16 writes, 32 mirror/band reads per thread, 2 barriers) and
// the band/mirror address arithmetic; 8 barriers per frame instead of 10.
// tools/fs_model.py models it step by step against the oracle.
// ---------------------------------------------------------------------------------------------

// lane -> column of forward pass 2: lanes 2p, 2p+1 hold columns c, 256 - c (lanes 0, 1: 0, 128);
// chosen (tools/fs_perm.py) so that pass 2's reads (swz(c) mod 32 per 32 lanes) and inverse
// pass 0's row stores (c mod 16 per 16 lanes) are bank-conflict free up to the one 2-way
// conflict per 16 lanes that the pairing forces (c = -c mod 16 for c = 0, 8 mod 16).
#include "ddc_fs_perm.h"

__device__ __forceinline__ float dpp_partner(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}

// f += conj(zp) q for the bin pair (k, 15 - k), zp = the partner lane's registers: the DPP
// operand feeds the FMA directly.  s_nop 1: a DPP read of a VGPR needs two wait states after
// the VALU write of it (the compiler cannot see into the asm).
__device__ __forceinline__ void split_dpp2(float2 &fa, float2 &fb, float2 za, float2 zb, float4 qa, float4 qb)
{
    asm("s_nop 1\n\t"
        "v_fmac_f32_dpp %0, %4, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %5, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %4, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, -%5, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %2, %6, %10 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %2, %7, %11 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %3, %6, %11 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %3, -%7, %10 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
        : "+v"(fa.x), "+v"(fa.y), "+v"(fb.x), "+v"(fb.y)
        : "v"(za.x), "v"(za.y), "v"(zb.x), "v"(zb.y), "v"(qa.z), "v"(qa.w), "v"(qb.z), "v"(qb.w));
}

// Zk P (own registers)
__device__ __forceinline__ float2 zk_p(float2 zk, float4 c)
{
    return make_float2(fmaf(zk.x, c.x, -zk.y * c.y), fmaf(zk.x, c.y, zk.y * c.x));
}
__device__ __forceinline__ float2 zc_q(float2 f, float2 zc, float4 c)
{
    f.x = fmaf(zc.x, c.z, f.x);
    f.x = fmaf(zc.y, c.w, f.x);
    f.y = fmaf(zc.x, c.w, f.y);
    f.y = fmaf(-zc.y, c.z, f.y);
    return f;
}

// v (-i)^s; s is a constant after unrolling (output register r times W_16^{4 QT r} = (-i)^{QT r})
__device__ __forceinline__ float2 quarter(float2 v, int s)
{
    s &= 3;
    if (s == 0) return v;
    if (s == 1) return make_float2(v.y, -v.x);
    if (s == 2) return make_float2(-v.x, -v.y);
    return make_float2(-v.y, v.x);
}

template <int QT, bool NCO, bool CS16>
__device__ __forceinline__ void emit_frame_q(void *__restrict__ out, int fbase, int k, int t, const float2 (&u)[16],
                                             const OutArgs &oa, const NcoArgs &nco)
{
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(static_cast<char *>(out) + (size_t)fbase * out_bytes<CS16>());
    const int r0 = k == 0 ? 4 : 0;   // wave-uniform
#pragma unroll
    for (int r = 0; r < 12; r++) {
        if (r < r0) continue;
        float2 v = flip(quarter(u[r], QT * r), oa.lsbmask);
        if constexpr (NCO) v = nco_mix(v, nco, fbase + t + NT * r);
        store_iq<CS16>(v, ro, (unsigned)t, (unsigned)(NT * r), oa);
    }
}


// Diagnostic build (-DSDDC_STAMPS, tools/fs_stamps.py; never the product): per wave, the cycles
// (s_memtime) of each work segment between two barriers and of each barrier wait, summed over
// the workgroup's frames in SGPRs, and written once at the end by lane 0 (vector stores) to a
// stamp buffer of their own: [workgroup][wave][kFsStampWords].  A stamp sits right before and
// right after each s_barrier, where the barrier's own lgkmcnt(0) drain already is.
#ifndef SDDC_FS_PQ
#define SDDC_FS_PQ 1   // (P, Q) bin pairs the FS kernel's split loads run ahead of their use
#endif
constexpr int kFsSegs = 9;                         // work segments: 8 barriers + the frame tail
// work[9], wait[9] (wait[8] unused), frames, ticks, realtime ticks, build, realtime start, end, HW_ID
constexpr int kFsStampWords = 2 * kFsSegs + 7;
#ifdef SDDC_STAMPS
// SDDC_STAMPS = 1 stamps barriers 0..3, = 2 barriers 4..7 (all eight in one build spill: the
// accumulators live in SGPRs); the time of an unstamped barrier falls into the next work segment.
// = 3: as 2, and the queue wave's dequeue in work[0..3]: resolve, the s_next write, the next ticket,
// and the ticket's read at the frame top.
__device__ unsigned g_fs_stamps[2048 * 4 * kFsStampWords];
constexpr int kStLo = SDDC_STAMPS >= 2 ? 4 : 0;
#define FS_STAMP_INIT()                                                                              \
    unsigned st_work[kFsSegs] = {}, st_wait[kFsSegs] = {}, st_frames = 0;                          \
    unsigned long long st_t = __builtin_amdgcn_s_memtime(), st_a = st_t;                          \
    const unsigned long long st_t0 = st_t, st_r0 = __builtin_amdgcn_s_memrealtime()
#define FS_SYNC(i)                                                                                   \
    do {                                                                                             \
        if constexpr ((i) >= kStLo && (i) < kStLo + 4) {                                             \
            st_a = __builtin_amdgcn_s_memtime();                                                     \
            st_work[i] += (unsigned)(st_a - st_t);                                                   \
            __syncthreads();                                                                         \
            st_t = __builtin_amdgcn_s_memtime();                                                     \
            st_wait[i] += (unsigned)(st_t - st_a);                                                   \
        } else {                                                                                     \
            __syncthreads();                                                                         \
        }                                                                                            \
    } while (0)
#define FS_STAMP_FRAME_END()                                                                         \
    do {                                                                                             \
        st_a = __builtin_amdgcn_s_memtime();                                                         \
        st_work[kFsSegs - 1] += (unsigned)(st_a - st_t);                                             \
        st_t = st_a;                                                                                 \
        st_frames++;                                                                                 \
    } while (0)
#define FS_QSTAMP(i, x)                                                                              \
    do {                                                                                             \
        if constexpr (SDDC_STAMPS == 3) {                                                            \
            const unsigned long long q0 = __builtin_amdgcn_s_memtime();                              \
            x;                                                                                       \
            st_work[i] += (unsigned)(__builtin_amdgcn_s_memtime() - q0);                             \
        } else {                                                                                     \
            x;                                                                                       \
        }                                                                                            \
    } while (0)
#define FS_STAMP_WRITE(wg, tid, nfr)                                                                 \
    do {                                                                                             \
        const unsigned long long st_r1 = __builtin_amdgcn_s_memrealtime();                          \
        if (((tid) & 63) == 0) {                                                                     \
            unsigned *o = g_fs_stamps + ((size_t)(wg) * 4 + ((tid) >> 6)) * kFsStampWords;           \
            for (int i = 0; i < kFsSegs; i++) {                                                      \
                o[i] = st_work[i];                                                                   \
                o[kFsSegs + i] = st_wait[i];                                                         \
            }                                                                                        \
            o[2 * kFsSegs] = (unsigned)(nfr);                                                        \
            o[2 * kFsSegs + 1] = (unsigned)(st_t - st_t0);                                           \
            o[2 * kFsSegs + 2] = (unsigned)(st_r1 - st_r0);                                          \
            o[2 * kFsSegs + 3] = (unsigned)SDDC_STAMPS;                                              \
            o[2 * kFsSegs + 4] = (unsigned)st_r0;                                                    \
            o[2 * kFsSegs + 5] = (unsigned)st_r1;                                                    \
            o[2 * kFsSegs + 6] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));             \
        }                                                                                            \
    } while (0)
#else
#define FS_STAMP_INIT() (void)0
#define FS_SYNC(i) __syncthreads()
#define FS_STAMP_FRAME_END() (void)0
#define FS_QSTAMP(i, x) x
#define FS_STAMP_WRITE(wg, tid, nfr) (void)0
#endif

template <bool RAND, bool NCO, bool CS16>
__global__ __launch_bounds__(NT, 4) void r2iq_fs_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes,
    const float2 *__restrict__ tw_p1, const float2 *__restrict__ tw_q1,
    const float2 *__restrict__ rec_f, const float2 *__restrict__ tw4096,
    const float4 *__restrict__ pqf, const float2 *__restrict__ fsl, int tunebin, OutArgs oa, NcoArgs nco,
    unsigned *__restrict__ wq)
{
    __shared__ __attribute__((aligned(16))) float2 lds[HALF];
    // pass-1 twiddles W_256^{s r} [15][16] (the inverse pass conjugates them: at d = 0 its table is
    // the same); the NS = 256 passes' bases W^j, W^{4j} (j < 256: forward pass 2 reads them at the
    // lane's column, inverse pass 2 at its thread index) and the lane factors g_t.  40832 B per
    // workgroup: 4 workgroups per CU fill the 160 KB exactly.  In LDS, not registers or L2: the
    // L2 loads' waits (vmcnt, in issue order) also waited for the input prefetch and the stores.
    __shared__ __attribute__((aligned(16))) float2 twl[15 * 16];
    __shared__ __attribute__((aligned(16))) float2 wtab[2 * NT];
    __shared__ __attribute__((aligned(16))) float2 gtab[NT];

    __shared__ int s_next;   // the workgroup's next frame (the queue wave's dequeue), -1 when none is left

    const int tid = (int)threadIdx.x;
    const int w = (int)blockIdx.x;
    // the dynamic frame queue (ddc_queue.hpp), worked by wave SDDC_FS_QWAVE: a ticket is
    // resolved a frame after it was taken (the frame after the current one is known at its
    // inverse pass 0, for the prefetch; the one after that is in flight)
#ifndef SDDC_FS_QWAVE
#define SDDC_FS_QWAVE 3   // not wave 0, which also carries the self-mirrored columns' split
#endif
    constexpr int QLANE = 64 * SDDC_FS_QWAVE;
    const bool qw = __builtin_amdgcn_readfirstlane(tid >> 6) == SDDC_FS_QWAVE;
    FsQueue q;
    // home shard: blockIdx % 8, the XCD under round-robin placement.  The first frame is static
    // (fs_static_first): its input loads go out at once, ahead of the table copies, with no device-
    // scope atomic round trip in front of them (+0.4-1.7 %, profiles/r03/ab/fs_static_first*.txt)
#ifndef SDDC_FS_QTOP
#define SDDC_FS_QTOP 0
#endif
#ifndef SDDC_FS_SPER
#define SDDC_FS_SPER 1   // static frames per workgroup; 2 (frame 0 resolves no ticket) measured 1.7 % slower
                         // (profiles/r03/ab/fs_two_static_frames.txt)
#endif
    q.init(wq, nframes, w & (FS_SHARDS - 1), (int)gridDim.x, SDDC_FS_SPER);
#ifdef SDDC_FS_QSTATIC
    const int f_stat = -1;
    const int f_stat1 = -1;
#else
    const int f_stat = fs_static_frame(nframes, (int)gridDim.x, w, 0, SDDC_FS_SPER);   // wave-uniform; -1: none
    int f_stat1 = SDDC_FS_SPER > 1 && f_stat >= 0 ? fs_static_frame(nframes, (int)gridDim.x, w, 1, SDDC_FS_SPER) : -1;
#endif
    int x[16];
    if (f_stat >= 0) load_frame(in32, f_stat / FRAMES, f_stat % FRAMES, x);
#ifndef SDDC_FS_QALL
#define SDDC_FS_QALL 0
#endif
    if constexpr (SDDC_FS_QALL) {
        // every wave runs the dequeue's scalar bookkeeping inside inverse pass 0's DFT (no branch,
        // so it interleaves with the VALU); only the queue wave's atomics are in range
        q.mine = qw;
        if (!qw) q.take();   // a zero ticket (out of range)
    }
    if (qw) {
#ifdef SDDC_FS_QSTATIC
        const int f_first = w < nframes ? w : -1;
#else
        int f_first = f_stat;
        if (f_stat < 0) {   // only when a shard has fewer frames than workgroups (small batches)
            q.take();
            q.peek();
            f_first = q.resolve();
        }
        q.take();
#endif
        if (tid == QLANE) s_next = f_first;
    }

    // per-lane constants: the column, and (reloaded every frame from L2, to keep them out of
    // the registers of the other passes) the twiddle bases of the two NS = 256 passes
    const int col_ = kFsPerm[tid];
    for (int i = tid; i < 15 * 16; i += NT) twl[i] = tw_p1[i];
    wtab[tid] = rec_f[tid];
    wtab[NT + tid] = rec_f[NT + tid];
    gtab[tid] = fsl[tid];
    const int qt = (tunebin >> 2) & 3;               // (tb mod 16) / 4: the output quarter turns
#ifdef SDDC_FS_FAKE_W0   // timing only: wave 0 takes the DPP path too (lanes 0, 1 wrong)
    const bool w0 = false;
#else
    const bool w0 = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;   // the wave holding columns 0, 128
#endif

    __syncthreads();
    int f = s_next;
    int blk = f / FRAMES, k = f - blk * FRAMES;
    if (f >= 0 && f_stat < 0) load_frame(in32, blk, k, x);
    FS_STAMP_INIT();

    while (f >= 0) {
        if ((qw || SDDC_FS_QALL) && f_stat1 < 0) FS_QSTAMP(3, q.peek());   // (frame 0 with a static second frame: no ticket read)
#if SDDC_FS_QTOP && !defined(SDDC_FS_QSTATIC)
        // the dequeue at the frame top (the ticket was taken a frame ago): the next frame into
        // s_next (read after barrier 5) and a ticket for the frame after it
        if (qw && f_stat1 < 0) {
            const int f_n = q.resolve();
            if (tid == QLANE) s_next = f_n;
            q.take();
        }
#endif
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z;
        const int c = col_ + z;
        const int sT = swz(t);
        const int x15 = t & 15;
        const int oblk = blk * 8 * HALF;
        const int kc = k;
        // ---- forward pass 0 (R16, NS1): convert + DFT16 from registers ----
        float2 v[16];
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++)
                if constexpr (RAND) {
                    const int wd = x[r] ^ (int)(((unsigned)x[r] & 0x10001u) * 0xFFFEu);   // as r2iq_persistent_kernel
                    a[r] = make_float2((float)(int)(short)(wd & 0xffff), (float)(wd >> 16));
                } else {
                    a[r] = make_float2((float)(int)(short)(x[r] & 0xffff), (float)(x[r] >> 16));
                }
            dft16<-1>(a, v);
        }
        FS_SYNC(0);   // the previous frame's last LDS reads are done
#pragma unroll
        for (int r = 0; r < 16; r++) lds[16 * t + (r ^ x15)] = v[r];
        FS_SYNC(1);
        // ---- forward pass 1 (R16, NS16): table twiddles W_256^{(t%16) r} ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], lds[sT + NT * r]);
            table_twiddle<-1, true>(a, twl, 16, x15);
            dft16<-1>(a, v);
        }
        FS_SYNC(2);
        {
            const int b1 = (t >> 4) * 256;
#pragma unroll
            for (int r = 0; r < 16; r++) lds[b1 + 16 * r + (x15 ^ r)] = v[r];
        }
        FS_SYNC(3);
        // ---- forward pass 2 (R16, NS256) on column c: Z[c + 256 k] in v[k] ----
        // The split's (P, Q) loads (bin pairs p, 15 - p) run a pair ahead of their use, the first
        // issued before pass 2 so that its reads and arithmetic cover the L2 latency (an empty asm
        // with a memory clobber pins each group; the compiler's own schedule waits for every pair
        // right after issuing it).  Two pairs ahead of pass 2 spill at 128 VGPRs.
        const __amdgpu_buffer_rsrc_t rpq = buf_rsrc(pqf + z);
        const unsigned t16 = 16u * (unsigned)t;
        float4 qa[8], qb[8];
#pragma unroll
        for (int p = 0; p < SDDC_FS_PQ; p++) {
            qa[p] = buf_load16(rpq, t16, 16u * NT * p);
            qb[p] = buf_load16(rpq, t16, 16u * NT * (15 - p));
        }
        asm volatile("" ::: "memory");
        {
            float2 a[16];
            const int sC = swz(c);
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], lds[sC + NT * r]);
            const float2 fw1 = wtab[c], fw4 = wtab[NT + c];   // W^c, W^{4c}
            twiddle_rec16<-1>(a, fw1, fw4);
            dft16<-1>(a, v);
        }
        // ---- split x filter (bins c + 256 k, mirror from the partner lane) -> inverse pass 0 ----
        float2 u[16];
        {
            float2 a[16];
            if (!w0) {
#pragma unroll
                for (int p = 0; p < 8; p++) {
                    if (p + SDDC_FS_PQ < 8) {
                        qa[p + SDDC_FS_PQ] = buf_load16(rpq, t16, 16u * NT * (p + SDDC_FS_PQ));
                        qb[p + SDDC_FS_PQ] = buf_load16(rpq, t16, 16u * NT * (15 - SDDC_FS_PQ - p));
                        asm volatile("" ::: "memory");
                    }
                    float2 fa = zk_p(v[p], qa[p]), fb = zk_p(v[15 - p], qb[p]);
                    split_dpp2(fa, fb, v[15 - p], v[p], qa[p], qb[p]);
                    a[p] = fa;
                    a[15 - p] = fb;
                }
            } else {
                // wave 0: lanes 0 (column 0: mirror of register k is its own (16 - k) mod 16) and
                // 1 (column 128: its own 15 - k) are self-mirrored
                const int lane = t & 63;
#pragma unroll
                for (int p = 0; p < 8; p++) {
                    if (p + SDDC_FS_PQ < 8) {
                        qa[p + SDDC_FS_PQ] = buf_load16(rpq, t16, 16u * NT * (p + SDDC_FS_PQ));
                        qb[p + SDDC_FS_PQ] = buf_load16(rpq, t16, 16u * NT * (15 - SDDC_FS_PQ - p));
                        asm volatile("" ::: "memory");
                    }
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const int kk = h ? 15 - p : p;
                        const float4 q = h ? qb[p] : qa[p];
                        const float2 vm = v[15 - kk], v0m = v[(16 - kk) & 15];
                        float2 zc = make_float2(dpp_partner(vm.x), dpp_partner(vm.y));
                        zc = lane == 1 ? vm : zc;
                        zc = lane == 0 ? v0m : zc;
                        a[kk] = zc_q(zk_p(v[kk], q), zc, q);
                    }
                }
            }
#if SDDC_FS_QALL && !defined(SDDC_FS_QSTATIC)
            if (f_stat1 >= 0) {
                if (tid == QLANE) s_next = f_stat1;
            } else {
                const int f_n = q.resolve();
                if (tid == QLANE) s_next = f_n;
                q.take();
            }
#endif
            dft16<+1>(a, u);
        }
        FS_SYNC(4);   // every wave's pass-2 reads are done
        {
            // row 16 c + (r ^ (swz(c) & 15)): the key XORs in c >> 4 so that the lane pairs c, -c
            // (equal c mod 16 for c = 0, 8 mod 16) never share a bank (tools/fs_perm.py)
            const unsigned xc0 = 128u * (unsigned)c + 8u * (unsigned)(swz(c) & 15);
#pragma unroll
            for (int r = 0; r < 16; r++) st_row(lds, xc0, r, 0, u[r]);
        }
        // the next frame from the ticket read at this frame's top, then a ticket for the one after
        // it (ddc_queue.hpp)
        if (qw) {
#ifdef SDDC_FS_QSTATIC   // timing only: a static stride instead of the queue
            FS_QSTAMP(1, {
                if (tid == QLANE) s_next = f + (int)gridDim.x < nframes ? f + (int)gridDim.x : -1;
            });
#else
            int f_n;
            if (SDDC_FS_QTOP || SDDC_FS_QALL) {
                // done at the frame top
            } else if (f_stat1 >= 0) {   // frame 0: the static second frame; the ticket taken at start waits a frame
                f_n = f_stat1;
                if (tid == QLANE) s_next = f_n;
            } else {
                FS_QSTAMP(0, f_n = q.resolve());
                FS_QSTAMP(1, if (tid == QLANE) s_next = f_n);
                FS_QSTAMP(2, q.take());
            }
#endif
        }
#ifndef SDDC_FS_QSTATIC
        f_stat1 = -1;
#endif
        FS_SYNC(5);
        // the next frame's input: issued here rather than in pass 0, so its 16 registers are
        // free through forward pass 2 and the split, and the loads' waits never hold pass 2
// the next frame's number (s_next) is read behind inverse pass 1's data reads, so its LDS round
// trip runs under theirs: +0.4-0.8 % in three interleaved rounds, bit-identical
// (profiles/r03/ab/fs_late_next_frame_read.txt)
#ifndef SDDC_FS_LATE_NEXT
#define SDDC_FS_LATE_NEXT 1
#endif
#if !SDDC_FS_LATE_NEXT
        const int fn = s_next;
        if (fn >= 0) {
            blk = fn / FRAMES;
            k = fn - blk * FRAMES;
            load_frame(in32, blk, k, x);
        }
#else
        int fn;
#endif
        // ---- inverse pass 1 (R16, NS16): table twiddles W_256^{-(t%16) r} ----
        // inverse pass 2's bases: W^t, W^{4t} and the lane's modulation factor g_t
        {
            float2 a[16];
            // element j + 256 r was stored by inverse pass-0 column (j >> 4) + 16 r under the key
            // swz(column) & 15 = (j >> 4) ^ r: byte (8 sT ^ 8 r) + 2048 r, one v_xor per read
            const unsigned sT8 = 8u * (unsigned)sT;
#pragma unroll
            for (int r = 0; r < 16; r++)
                XRD(a[r], *reinterpret_cast<const float2 *>(reinterpret_cast<const char *>(lds) + ((sT8 ^ (8u * r)) + 2048u * r)));
#if SDDC_FS_LATE_NEXT   // the next frame read behind the pass's data reads (its LDS round trip under theirs)
            fn = s_next;
            if (fn >= 0) {
                blk = fn / FRAMES;
                k = fn - blk * FRAMES;
                load_frame(in32, blk, k, x);
            }
#endif
            table_twiddle<+1, true>(a, twl, 16, x15);
            dft16<+1>(a, u);
        }
        FS_SYNC(6);
        {
            // the same addresses as the forward pass-1 stores: recomputed from an opaque copy of
            // t, or the compiler keeps those 16 addresses live through pass 2 and spills them
            int t1 = t;
            asm volatile("" : "+v"(t1));
            const int b1 = (t1 >> 4) * 256, y15 = t1 & 15;
#pragma unroll
            for (int r = 0; r < 16; r++) lds[b1 + 16 * r + (y15 ^ r)] = u[r];
        }
        FS_SYNC(7);
        // ---- inverse pass 2 (R16, NS256): twiddles g_t W^{-t r}, quarter turns, overlap-discard ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], lds[sT + NT * r]);
            const float2 rw1 = wtab[t], rw4 = wtab[NT + t], g0 = gtab[t];   // W^t, W^{4t}, g_t
            twiddle_g16<+1>(a, g0, cmulc(g0, rw1), cmulc(g0, rw4), rw1, rw4);   // g W^{-t}, g W^{-4t}
            dft16<+1>(a, u);
            const int fb = oblk + emit_base<HALF>(kc);
            switch (qt) {
            case 0: emit_frame_q<0, NCO, CS16>(out, fb, kc, t, u, oa, nco); break;
            case 1: emit_frame_q<1, NCO, CS16>(out, fb, kc, t, u, oa, nco); break;
            case 2: emit_frame_q<2, NCO, CS16>(out, fb, kc, t, u, oa, nco); break;
            default: emit_frame_q<3, NCO, CS16>(out, fb, kc, t, u, oa, nco); break;
            }
        }
        FS_STAMP_FRAME_END();
        f = fn;
    }
    FS_STAMP_WRITE(w, tid, st_frames);
#ifndef SDDC_FS_QSTATIC
    if (tid == QLANE) fs_queue_done(wq, (unsigned)gridDim.x);
#endif
}

// FS tables of one tunebin: pqf[l + 256 k] = (P, Q) of bin b = kFsPerm[l] + 256 k (inverse input
// m = (b - tb) mod 4096, zero unless b is in the reference's band: tb <= b < tb + 2048, b < 4096,
// or tb - 2048 <= b < tb); fsl = [g_t | g_t W^{-t} | g_t W^{-4t}], g_t = e^{-2 pi i tb t / 4096},
// looked up exactly in the 4096-point table.
__global__ void build_fs_tables_kernel(const float2 *__restrict__ hsel0, const float2 *__restrict__ post8192,
                                       const float2 *__restrict__ tw4096, int tunebin, float4 *__restrict__ pqf,
                                       float2 *__restrict__ fsl)
{
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= HALF) return;
    const int l = i & (NT - 1), kk = i >> 8;
    const int b = kFsPerm[l] + NT * kk;
    const bool band = (b >= tunebin && b - tunebin < HALF / 2) || (b < tunebin && tunebin - b <= HALF / 2);
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
    if (band) {
        const int m = (b - tunebin) & (HALF - 1);
        const double hr = hsel0[m].x, hi = hsel0[m].y;
        const double wr = post8192[b].x, wi = post8192[b].y;
        const double pr = 1.0 + wi, pi = -wr, qr = 1.0 - wi, qi = wr;   // 1 - i W, 1 + i W
        c.x = (float)(hr * pr - hi * pi);
        c.y = (float)(hr * pi + hi * pr);
        c.z = (float)(hr * qr - hi * qi);
        c.w = (float)(hr * qi + hi * qr);
    }
    pqf[i] = c;
    if (i < NT) {
        fsl[i] = tw4096[(tunebin * i) & (HALF - 1)];
        fsl[NT + i] = tw4096[((tunebin - 1) * i) & (HALF - 1)];
        fsl[2 * NT + i] = tw4096[((tunebin - 4) * i) & (HALF - 1)];
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
    unsigned *wq;   // a zeroed dynamic-frame-queue slot (kFsQueueWords)
};

template <int D, bool RAND, bool NCO, bool CS16>
hipError_t launch_v(const KernelTables &t, const Launch &L)
{
    auto kern = r2iq_persistent_kernel<D, RAND, NCO, CS16>;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(kern), NT, L.device, &occ, &cus);
    if (e != hipSuccess) return e;
    const int nframes = L.nblk * FRAMES;
    int grid = cus * occ;
    if (grid > nframes) grid = nframes;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, L.s, reinterpret_cast<const int *>(L.d_in),
                       L.d_out, nframes, t.tw_p1, t.tw_q1[D], t.rec_f, t.rec_i[D], t.tw4096, L.pq, L.tunebin, L.oa,
                       L.nco, L.wq);
    return hipGetLastError();
}

template <bool RAND, bool NCO, bool CS16>
hipError_t launch_fs_v(const KernelTables &t, const Launch &L, const float4 *pqf, const float2 *fsl, unsigned *wq)
{
    auto kern = r2iq_fs_kernel<RAND, NCO, CS16>;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(kern), NT, L.device, &occ, &cus);
    if (e != hipSuccess) return e;
    const int nframes = L.nblk * FRAMES;
    int grid = cus * occ;
    if (grid > nframes) grid = nframes;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, L.s, reinterpret_cast<const int *>(L.d_in),
                       L.d_out, nframes, t.tw_p1, t.tw_q1[0], t.rec_f, t.tw4096, pqf, fsl, L.tunebin, L.oa, L.nco,
                       wq);
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

}  // namespace

hipError_t launch_build_split_filter(const KernelTables &t, int d, int tunebin, float4 *pq, hipStream_t s)
{
    if (d < 0 || d > 6) return hipErrorInvalidValue;
    const int N = HALF >> d;
    hipLaunchKernelGGL(build_split_filter_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, t.hsel[d],
                       t.post8192, N, tunebin, pq);
    return hipGetLastError();
}

bool fs_path(int d, int tunebin)
{
#if SDDC_D0_FS
    return d == 0 && (tunebin & 3) == 0;
#else
    (void)d;
    (void)tunebin;
    return false;
#endif
}

hipError_t launch_build_fs_tables(const KernelTables &t, int tunebin, float4 *pqf, float2 *fsl, hipStream_t s)
{
    if (tunebin < 0 || tunebin >= HALF || (tunebin & 3)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(build_fs_tables_kernel, dim3(HALF / 256), dim3(256), 0, s, t.hsel[0], t.post8192, t.tw4096,
                       tunebin, pqf, fsl);
    return hipGetLastError();
}

hipError_t launch_frames_fs(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pqf,
                            const float2 *fsl, int tunebin, int lsb, int rand, int cs16, float cs16_scale,
                            const float2 *nco_starts, const float2 *nco_trig, unsigned *wq, int device, hipStream_t s)
{
    if (tunebin & 3) return hipErrorInvalidValue;
    const Launch L{d_in, nblk, d_out, nullptr, tunebin, device, s, OutArgs{lsb ? 0x80000000u : 0u, cs16_scale},
                   NcoArgs{nco_starts, nco_trig}, wq};
    const bool nco = nco_starts != nullptr;
    if (rand) {
        if (nco) return cs16 ? launch_fs_v<true, true, true>(t, L, pqf, fsl, wq) : launch_fs_v<true, true, false>(t, L, pqf, fsl, wq);
        return cs16 ? launch_fs_v<true, false, true>(t, L, pqf, fsl, wq) : launch_fs_v<true, false, false>(t, L, pqf, fsl, wq);
    }
    if (nco) return cs16 ? launch_fs_v<false, true, true>(t, L, pqf, fsl, wq) : launch_fs_v<false, true, false>(t, L, pqf, fsl, wq);
    return cs16 ? launch_fs_v<false, false, true>(t, L, pqf, fsl, wq) : launch_fs_v<false, false, false>(t, L, pqf, fsl, wq);
}

hipError_t launch_frames_persistent(const KernelTables &t, int d, const int16_t *d_in, int nblk, void *d_out,
                                    const float4 *pq, int tunebin, int lsb, int rand, int cs16, float cs16_scale,
                                    const float2 *nco_starts, const float2 *nco_trig, unsigned *wq, int device,
                                    hipStream_t s)
{
    const Launch L{d_in, nblk, d_out, pq, tunebin, device, s, OutArgs{lsb ? 0x80000000u : 0u, cs16_scale},
                   NcoArgs{nco_starts, nco_trig}, wq};
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

// Diagnostic (SDDC_STAMPS builds only): copy the d = 0 fused-split kernel's stamp buffer of the
// last launch ([workgroup][wave][words], tools/fs_stamps.py) to host memory; -1 in product builds.
extern "C" int sddc_ddc_internal_fs_stamps(unsigned *host, int nwords, int *words_per_wave)
{
    if (words_per_wave) *words_per_wave = sddc::kFsStampWords;
#ifdef SDDC_STAMPS
    const size_t n = sizeof(sddc::g_fs_stamps) / sizeof(unsigned);
    if (!host || nwords < 0 || (size_t)nwords > n) return -2;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(sddc::g_fs_stamps), (size_t)nwords * sizeof(unsigned), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
#else
    (void)host;
    (void)nwords;
    return -1;
#endif
}
