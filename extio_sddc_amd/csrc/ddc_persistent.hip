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
//     twiddle and the filter are P (a float2 per inverse input) and the real r = Q / (i P), held in
//     registers at d >= 1 (split_pr, build_split_filter_kernel).
// The measured-slower layouts, the first-generation kernels and the timing-only builds of the
// A/B study are in git history (DESIGN.md §8 keeps their numbers).
#include <hip/hip_runtime.h>

#include "ddc_frame_common.hpp"
#include "ddc_queue.hpp"
#include "ddc_stamps.hpp"

namespace sddc {
namespace {

#ifdef SDDC_STAMPS
__device__ unsigned g_p_stamps[2048 * 4 * kStampWords];
#endif

// d = 3..6 (N = 512, 256, 128, 64): the N-point inverse as mixed-radix Stockham passes on the
// lanes of wave 0, radix schedule 8-8-8, 4-4-4-4, 8-4-4, 4-4-4.  The pass of radix R after a span Ns runs on
// threads j < N / R: reads elements j + (N / R) r, twiddles W_{R Ns}^{-k r} (k = j mod Ns),
// inverse DFT-R, writes (j / Ns) R Ns + k + Ns r; the last pass leaves y[j + (N / 4) r] in
// registers.  LDS element e sits at e ^ ((e >> s) & 31) (s = 3, 2, 2, 1): conflict-
// free for every read and write pattern (tools/r4_tail_model.py, which also checks the passes
// against numpy).  The [N/16, 16] form it replaces kept 16 lanes busy (d = 4) or fewer; its two
// passes cost 8-11 % of the launch at d = 4..6 (timing-only build, profiles/r03/ab).
// The split tables' layout (build_split_filter_kernel): for N >= 512 thread t's inverse inputs
// m = t + 256 r sit so that each load is 16 bytes per lane and coalesced over the lanes: P of
// (t, r) at float2 2 (256 (r >> 1) + t) + (r & 1) (pairs r, r + 1), r of (t, r) at float
// 2 N + G (256 (r / G) + t) + r % G, G = min(R0, 4) (quads); N <= 256: at m.
__host__ __device__ constexpr int pq_p_index(int N, int m)
{
    return N >= 512 ? 2 * (256 * ((m >> 8) >> 1) + (m & 255)) + ((m >> 8) & 1) : m;
}
__host__ __device__ constexpr int pq_r_index(int N, int m)
{
    return N >= 512 ? (N / 256 < 4 ? N / 256 : 4) * (256 * ((m >> 8) / (N / 256 < 4 ? N / 256 : 4)) + (m & 255))
                          + (m >> 8) % (N / 256 < 4 ? N / 256 : 4)
                    : m;
}

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

// d = 3 (N = 512): the inverse as two independent 256-point halves on waves 0 and 1.  With
// m = m' + 256 s and n = 2 n' + p, y[2 n' + p] = IDFT_256(E_p)[n'], E_p[m'] = (X[m'] + (-1)^p
// X[m' + 256]) e^{2 pi i m' p / 512}: one radix-2 step in the registers of the thread holding
// X[m'], X[m' + 256] (the split's), then the d = 4 tail on each half.  Kept: y[0, 384) (k >= 1),
// y[128, 384) (k = 0), i.e. u[r] = y[2 (t + 64 r) + p] for r < 3 (r >= 1 at k = 0).  The two waves'
// stores interleave (8 bytes every 16), so they go write-back rather than nt: L2 merges the halves
// into whole lines (nt: WRITE_SIZE +35 %; write-back: equal to the one-tail kernel's, at the same
// speed; exchanging the halves through LDS to store whole runs needed a workgroup barrier and
// was slower than both, profiles/r05/ab/persistent_d3_halves*.txt).
template <bool NCO, bool CS16>
__device__ __forceinline__ void tail_emit_half(void *__restrict__ out, int fbase, int k, int t, int p,
                                               const float2 (&u)[8], const OutArgs &oa, const NcoArgs &nco)
{
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(static_cast<char *>(out) + (size_t)fbase * out_bytes<CS16>());
#pragma unroll
    for (int r = 0; r < 3; r++) {
        if (r == 0 && k == 0) continue;
        float2 v = flip(u[r], oa.lsbmask);
        if constexpr (NCO) v = nco_mix(v, nco, fbase + 2 * (t + 64 * r) + p);
        store_iq<CS16, 0>(v, ro, (unsigned)(2 * t + p), (unsigned)(128 * r), oa);
    }
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

// d = 2 (N = 1024): the inverse as a radix-N/256 pass from the split's registers
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

// element e of a tail buffer, with e = lane ^ R for bits of lane and R that do not overlap: the
// swizzle is linear over XOR (tail_swz(a ^ b) = tail_swz(a) ^ tail_swz(b)), so the byte offset is
// (8 tail_swz(lane)) ^ (8 tail_swz(R)), one v_xor_b32 with an immediate per access (as lds_x)
template <int N>
__device__ __forceinline__ float2 &tail_x(float2 *buf, unsigned lane8, int R)
{
    return *reinterpret_cast<float2 *>(reinterpret_cast<char *>(buf) + (lane8 ^ (8u * (unsigned)tail_swz<N>(R))));
}

template <int N, int P>
__device__ __forceinline__ void tail_pass(float2 *sb, const float2 *twq, int t, float2 (&u)[8])
{
    constexpr int R = tail_radix<N>(P), NS = tail_ns<N>(P), T = N / R;
    const int kk = t & (NS - 1);
    if (t < T) {
        float2 a[R];
        // reads t + T r: t < T, so the two terms share no bit.  Data and twiddle reads each one
        // ds_read_b64 (XRD; the compiler's ds_read2(st64)_b64 pairs take 8 LDS cycles against
        // 2 per ds_read_b64): d = 4 +1.2 to +2.0 %, d = 3 -0.2 to +2.1 %, d = 5 +1.3 %, d = 6
        // -0.3 %, bit-identical (profiles/r06/ab/persistent_tail_single_b64_reads.txt)
        const unsigned rd8 = 8u * (unsigned)tail_swz<N>(t);
#pragma unroll
        for (int r = 0; r < R; r++) XRD(a[r], tail_x<N>(sb, rd8, T * r));
        if constexpr (P > 0) {
            float2 w[R];
#pragma unroll
            for (int r = 1; r < R; r++) XRD(w[r], twq[tail_twoff<N>(P) + (r - 1) * NS + kk]);
#pragma unroll
            for (int r = 1; r < R; r++) a[r] = TW<+1>(a[r], w[r]);
        }
        if constexpr (R == 8) dft8<+1>(a, u);
        else dft4<+1>(a, u);
    }
    if constexpr (P + 1 < tail_passes<N>()) {
        wave_lds_sync();   // this wave's reads of the pass are done
        if (t < T) {
            // writes (t / NS) R NS + kk + NS r: kk < NS, NS r < R NS, so again disjoint bits
            const unsigned wr8 = 8u * (unsigned)tail_swz<N>((t / NS) * R * NS + kk);
#pragma unroll
            for (int r = 0; r < R; r++) tail_x<N>(sb, wr8, NS * r) = u[r];
        }
        wave_lds_sync();
    }
}

template <int D, bool RAND, bool NCO, bool CS16>
__global__ __launch_bounds__(NT, 4) void r2iq_persistent_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes,
    const float2 *__restrict__ tw_p1, const float2 *__restrict__ tw_q1,
    const float2 *__restrict__ rec_f, const float2 *__restrict__ rec_i, const float2 *__restrict__ tw4096,
    const float4 *__restrict__ pq, int tunebin, OutArgs oa, NcoArgs nco, unsigned slotw)
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
    // The pruned pass 2 computes only the DFT-16 outputs it stores: registers 0 .. NB - 1 and
    // mrel .. mrel + NB - 1 (mod 16), dft16_need with a wave-uniform mask (output pairs r, r + 8
    // skipped when both are unneeded, first-stage halves with them): 10 of 16 outputs at d = 2,
    // 6 at d = 3, 4 at d >= 4.  Rounds 2-5 pruned only whole k1 groups and only at d >= 4
    // (dft16_groups: d = 5, 6 +1-2.8 %, d = 4 +4 %, profiles/r02/ab/grp5_d5_6*.txt,
    // profiles/r04/ab/pruned_f2_d4.txt); round 6 (profiles/r06/ab/persistent_f2_need_*.txt).  At
    // d = 5, 6 dft16_need takes the kernel past 128 VGPRs (137 / 129: 3 waves per SIMD), so they
    // keep the k1-group form.
    constexpr bool NEED = PRUNE && D <= 4, GRP = PRUNE && D >= 5;
    const unsigned nbm = (1u << NB) - 1u;
    const unsigned need = __builtin_amdgcn_readfirstlane((nbm | (nbm << mrel) | (nbm >> (16 - mrel))) & 0xffffu);
    const bool need2 = ((mrel & 3) - 1u) <= 1u, need3 = (mrel & 3) >= 2;
    __shared__ __attribute__((aligned(16))) float2 lds[HALF];
    // pass-1 twiddle tables, copied once per workgroup: [15][16] forward, [15][S] inverse
    constexpr int SQ = N >= 512 ? N / 256 : N / 16;
    // d = 3 and d >= 4: the inverse runs as Stockham passes on wave 0 (tail_pass); their twiddles
    // take the inverse table's place
    constexpr bool R4T = N <= 256 || N == 512;
    constexpr int TN = N == 512 ? 256 : N;   // the tail's size (d = 3: two 256-point halves)
    // d = 2 only: the inverse as radix-4 passes on all 256 threads (wg_pass).  At d = 1 (N = 2048,
    // two butterflies per thread per pass) the same form measured 7-8 % slower than the two-wave
    // radix-16 tail (profiles/r03/ab/d12_wg.txt)
    constexpr bool WGT = N == 1024;
    constexpr int TWQ = R4T ? tail_twn<TN>() : WGT ? wg_twn<N>() : 15 * SQ;
    __shared__ __attribute__((aligned(16))) float2 twl[15 * 16 + TWQ];
    float2 *const w0 = lds, *const w1 = lds;   // the pass buffers (one 32 KB frame buffer)
    // d >= 2: the inverse's last passes run on one wave, so they are ordered within that wave
    // (wave_lds_sync) and the other waves go on to the next frame's pass 0.  N <= 256: the
    // filtered bins go to their own buffer sb (N <= 256 float2, 2 KB), so the split needs no
    // barrier between its Z reads and its writes (profiles/r02/ab/winv.txt); LDS at d = 4
    // 38.7 KB, still 4 workgroups per CU.
    constexpr bool WINV = N <= 1024;
    constexpr bool SEPB = N <= 256;
    // N <= 256 (d >= 4): the bins of TB frames, whose tails run side by side on TB waves (below):
    // TB = 2 at d = 4 (LDS 40.8 KB), 4 at d = 5, 6 (39.7 / 37.2 KB), still 4 workgroups per CU
    constexpr int TB = N == 256 ? 2 : 4;
    __shared__ __attribute__((aligned(16))) float2 sb[SEPB ? TB * N : 1];

    const int tid = (int)threadIdx.x;
    const int G = (int)gridDim.x, w = (int)blockIdx.x;
    // Frames: a static split, each workgroup one contiguous range, sized by its CU slot's measured
    // speed (ddc_queue.hpp slot_split; equal shares off full residency).  Wave 3 writes the next
    // frame number for the next frame's start.  Round 3 fed d = 1, 2 from the dynamic frame
    // queue (two static frames, then one ticket per frame) and split d >= 3 equally; the weighted
    // split beats both: d = 1 +3 %, d = 2 +6-8 % against the queue, d = 3..6 +10-14 % against the
    // equal split (profiles/r04/ab/slot_weighted_*.txt).  The queue cost this kernel ~1-2k cycles
    // of a 10-16k-cycle frame even with its ticket read and taken where no load waits for it
    // (profiles/r04/stamps/stamps_p_d*_queue_*.txt).
    __shared__ int s_first, s_next;
    constexpr int QLANE = 64 * 3;
    const bool qw = __builtin_amdgcn_readfirstlane(tid >> 6) == 3;
    const int f1s = slot_split(nframes, G, w + 1, slotw);   // the range's end
    if (qw) {
        const int f0 = slot_split(nframes, G, w, slotw);
        if (tid == QLANE) {
            s_first = f0 < f1s ? f0 : -1;
            s_next = f0 + 1 < f1s ? f0 + 1 : -1;
        }
    }

    // per-thread constants, live for the whole frame loop
    const int zr = ZROT ? (tunebin >> 8) + (tid < zd ? 1 : 0) : r0;
    const float2 fw1_ = tw4096[(tid + 256 * zr) & (HALF - 1)];   // rotated bases (PRUNE: r0, ZROT: zr)
    const float2 fw4_ = tw4096[(4 * tid + 1024 * zr) & (HALF - 1)];
    // forward pass 2's other anchors W^{2b}, W^{3b}, W^{8b}, W^{12b} (twiddle_anchor6)
    const int fb_ = tid + 256 * zr;
    const float2 fw2_ = tw4096[(2 * fb_) & (HALF - 1)], fw3_ = tw4096[(3 * fb_) & (HALF - 1)];
    const float2 fw8_ = tw4096[(8 * fb_) & (HALF - 1)], fw12_ = tw4096[(12 * fb_) & (HALF - 1)];
    float2 iw1_ = ZROT ? rec_f[tid] : fw1_, iw4_ = ZROT ? rec_f[NT + tid] : fw4_;
    // d = 3: the halves' twiddle e^{2 pi i t / 512} (applied as the conjugate of W_4096^{8t})
    const float2 hw_ = N == 512 ? tw4096[(8 * tid) & (HALF - 1)] : make_float2(1.f, 0.f);
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
            twl[i] = tail_twiddle<TN>(tw4096, i - 15 * 16);
        } else if constexpr (WGT) {
            const int e = i - 15 * 16;   // W_{4 Ns}^k, Ns = N/256 x 1, 4, 16, 64
            constexpr int r0 = N / 256;
            const int ns = e < wg_twoff<N>(4 * r0) ? r0 : e < wg_twoff<N>(16 * r0) ? 4 * r0
                         : e < wg_twoff<N>(64 * r0) ? 16 * r0 : 64 * r0;
            twl[i] = tw4096[((e - wg_twoff<N>(ns)) * (HALF / (4 * ns))) & (HALF - 1)];
        }
    }

    // d >= 2: the split's r of the thread's inverse inputs m = t + 256 r, held in registers for the
    // launch (table reads per frame: the float2 P, 8 bytes per bin, instead of the (P, Q) float4's
    // 16); d = 1 (126 VGPRs before; its 8 r spilled 12 VGPRs) and d = 0 (16 bins per thread)
    // read r every frame, 12 bytes per bin
    constexpr int RR = N >= 512 ? N / 256 : 1;
    constexpr bool RREG = D >= 2;
    float rreg[RR];
    if constexpr (RREG) {
        const float *rt = reinterpret_cast<const float *>(pq) + 2 * N;
#pragma unroll
        for (int r = 0; r < RR; r++) rreg[r] = (N >= 512 || tid < N) ? rt[pq_r_index(N, tid + NT * r)] : 0.f;
    }

    __syncthreads();   // s_first, s_next
    int f = s_first;
    int fi = 0;                 // frames done by this workgroup (N <= 256: the slot in the batch of TB)
    int pfb0 = 0, pfb1 = 0, pfb2 = 0, pkc0 = 0, pkc1 = 0, pkc2 = 0;   // the batch's earlier frames (output base, k)
    int blk = f / FRAMES, k = f - blk * FRAMES;
    int x[16];
    if (f >= 0) load_frame(in32, blk, k, x);
    ST_INIT();

    while (f >= 0) {
        const int fn = s_next;   // the next frame (written in the previous frame's middle)
        // Opaque per-iteration copies of the thread index and table pointers: without
        // them the compiler hoists every loop-invariant LDS address and table load out
        // of the frame loop and spills them.
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z;
        const float2 *pqz = reinterpret_cast<const float2 *>(pq) + z;   // P (split_pr)
        float2 fw1 = fw1_, fw4 = fw4_, iw1 = iw1_, iw4 = iw4_;
        asm volatile("" : "+v"(fw1), "+v"(fw4), "+v"(iw1), "+v"(iw4));
        float2 fw2 = fw2_, fw3 = fw3_, fw8 = fw8_, fw12 = fw12_;
        asm volatile("" : "+v"(fw2), "+v"(fw3), "+v"(fw8), "+v"(fw12));
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
        ST_SYNC(0);   // the previous frame's last LDS reads are done
#pragma unroll
        for (int r = 0; r < 16; r++)   // swz(16t + r)
            if constexpr (XF0) st_row(w0, xa0, r, 0, v[r]);
            else w0[16 * t + (r ^ x15)] = v[r];
        ST_SYNC(1);
        // ---- forward pass 1 (R16, NS16): table twiddles W_256^{(t%16) r} ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], w0[sT + NT * r]);
            table_twiddle<-1, TW_EARLY>(a, twl, 16, x15);
            dft16<-1>(a, v);
        }
        ST_SYNC(2);
        {
            const int b1 = (t >> 4) * 256;                                     // swz(b1 + x15 + 16 r)
#pragma unroll
            for (int r = 0; r < 16; r++)
                if constexpr (XST) st_row(w1, xa1, r, 16, v[r]);
                else w1[b1 + 16 * r + (x15 ^ r)] = v[r];
        }
        ST_SYNC(3);
        // ---- forward pass 2 (R16, NS256): recurrence twiddles W_4096^{t r} ----
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], w1[sT + NT * r]);
            twiddle_anchor6<-1>(a, fw1, fw2, fw3, fw4, fw8, fw12);
            if constexpr (NEED) dft16_need<-1>(a, v, need);
            else if constexpr (GRP) dft16_groups<-1>(a, v, need2, need3);
            else dft16<-1>(a, v);
        }
        ST_SYNC(4);
        if constexpr (PRUNE) {
#pragma unroll
            for (int r = 0; r < 16; r++)   // Z, natural order: the band's and the mirror's registers
                if (r < NB || ((r - mrel) & 15) < NB) w0[t + NT * ((r + r0) & 15)] = v[r];
        } else {
            const int sZ = (t - zd) & 255;
#pragma unroll
            // Z, rotated by tb: one ds_write_b64 per register (not the compiler's ds_write2st64_b64
            // pairs): d = 1 +1.6 / +2.1 %, C4 +1.0 / +1.2 %, bit-identical
            // (profiles/r06/ab/persistent_d1_single_z_stores.txt)
            for (int r = 0; r < 16; r++) {
                w0[sZ + NT * r] = v[r];
                asm volatile("" ::: "memory");
            }
        }
        if (tid == QLANE)   // the frame after the next one (read by every wave at the next frame's start)
            s_next = fn >= 0 && fn + 1 < f1s ? fn + 1 : -1;
        ST_SYNC(5);

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
                const unsigned sb0b = 8u * (unsigned)sb0, sc0b = 8u * (unsigned)sc0, t8 = 8u * (unsigned)t;
                const __amdgpu_buffer_rsrc_t rpq = buf_rsrc(pqz);
                const __amdgpu_buffer_rsrc_t rrt = buf_rsrc(reinterpret_cast<const float *>(pqz) + 2 * N);
                float2 a[R0];
                constexpr int G = R0 < 4 ? R0 : 4;
                float2 pp[2];
                float rq[4];
#pragma unroll
                for (int r = 0; r < R0; r++) {
                    if ((r & 1) == 0) {   // P of r, r + 1: one 16-byte load
                        const float4 q = buf_load16(rpq, 2u * t8, 4096u * (unsigned)(r >> 1));
                        pp[0] = make_float2(q.x, q.y);
                        pp[1] = make_float2(q.z, q.w);
                    }
                    if constexpr (!RREG) {
                        if (r % G == 0) {   // r of r .. r + 3: one 16-byte load
                            const float4 q = buf_load16(rrt, 2u * t8, 4096u * (unsigned)(r / G));
                            rq[0] = q.x, rq[1] = q.y, rq[2] = q.z, rq[3] = q.w;
                        }
                    }
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
                    a[r] = split_pr(zk, zc, pp[r & 1], RREG ? rreg[r] : rq[r % G]);
                }
                if constexpr (WGT) {
                    constexpr int B = N / 1024, T = N / 4;
                    {
                        float2 u0[R0];
                        if constexpr (R0 == 8) dft8<+1>(a, u0);   // pass 0 (Ns = 1)
                        else dft4<+1>(a, u0);
                        ST_SYNC(6);   // every wave's Z reads are done
#pragma unroll
                        for (int r = 0; r < R0; r++) w1[wg_swz<N>(R0 * t + r)] = u0[r];
                    }
                    ST_SYNC(7);
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
                    ST_FRAME_END();
                    f = fn;
                    continue;
                }
                if constexpr (N == 512) {
                    // d = 3: the 512 filtered bins (inverse input m = t + 256 r) as two 256-point
                    // halves (tail_emit_half): the radix-2 step here, then waves 0 and 1 each run
                    // the d = 4 tail (four radix-4 Stockham passes) on one half.  One 512-point
                    // tail on wave 0 (three radix-8 passes) held waves 1..3 at the next frame's
                    // first barrier for twice as long.
                    float2 hw = hw_;
                    asm volatile("" : "+v"(hw));
                    const float2 e0 = make_float2(a[0].x + a[1].x, a[0].y + a[1].y);
                    const float2 e1 = TW<+1>(make_float2(a[0].x - a[1].x, a[0].y - a[1].y), hw);
                    ST_SYNC(6);   // every wave's Z reads are done
                    w1[tail_swz<TN>(t)] = e0;
                    w1[TN + tail_swz<TN>(t)] = e1;
                    ST_SYNC(7);
                    const int p = __builtin_amdgcn_readfirstlane(tid >> 6);
                    if (p < 2) {
                        const int lt = t & 63;
                        float2 *const hb = w1 + TN * p;
                        float2 v8[8];
                        const float2 *twq = twl + 15 * 16;
                        tail_pass<TN, 0>(hb, twq, lt, v8);
                        tail_pass<TN, 1>(hb, twq, lt, v8);
                        tail_pass<TN, 2>(hb, twq, lt, v8);
                        tail_pass<TN, 3>(hb, twq, lt, v8);
                        tail_emit_half<NCO, CS16>(out, oblk + emit_base<N>(kc), kc, lt, p, v8, oa, nco);
                    }
                    ST_FRAME_END();
                    f = fn;
                    continue;
                }
                if constexpr (R0 == 16) dft16<+1>(a, u);
                else dft<R0, +1>(a, u);
            }
            ST_SYNC(6);
            if constexpr (R0 == 16) {
#pragma unroll
                for (int r = 0; r < 16; r++)
                    if constexpr (XI0) st_row(w1, xa0, r, 0, u[r]);
                    else w1[16 * t + (r ^ x15)] = u[r];
            } else {
#pragma unroll
                for (int r = 0; r < R0; r++) LX(w1, R0 * t, r) = u[r];
            }
            ST_SYNC(7);
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
                table_twiddle<+1, TW_EARLY>(a, twl + 15 * 16, R0, t % R0);
                dft16<+1>(a, u);
            }
            if constexpr (WINV) wave_lds_sync();
            else ST_SYNC(8);
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
            else ST_SYNC(9);
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
                twiddle_rec16<+1>(a, iw1, iw4);
                dft16<+1>(a, u);
                emit_frame<NB, NCO, CS16>(out, oblk + emit_base<N>(kc), kc, t, u, oa, nco);
            }
        } else {
            // ---- N <= 256: the N filtered bins (split x filter), one per thread ----
            float2 tv = make_float2(0.f, 0.f);
            if (t < N) {
                const int m = t;
                const int bin = tunebin + m - (m >= N / 2 ? N : 0);
                tv = split_pr(w0[bin & (HALF - 1)], w0[(HALF - bin) & (HALF - 1)], pqz[m], rreg[0]);
            }
            // The N filtered bins to sb, and the inverse as Stockham passes on one wave (the tail).
            // Frames go in batches of TB: frame j of a batch leaves its bins in sb[jN .. (j+1)N)
            // and its tail for later; after the batch's last frame, wave j runs frame j's tail,
            // the TB tails side by side.  One frame's tail ran on wave 0 while waves 1..3 waited
            // at the next frame's first barrier (≈20 % of their frame at d = 4,
            // profiles/r05/stamps/stamps_p_d4.txt); batched, that wait comes once per TB frames.
            // A range's last frames (fewer than TB) run theirs at its last frame.
            const int slot = fi & (TB - 1);
            if (t < N) sb[N * slot + tail_swz<N>(t)] = tv;
            ST_SYNC(6);
            const int fbase = oblk + emit_base<N>(kc);
            const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
            if ((slot == TB - 1 || fn < 0) && wv <= slot) {
                float2 u[8];
                const float2 *twq = twl + 15 * 16;
                float2 *const sbw = sb + N * wv;
                const int lt = t & 63;
                tail_pass<N, 0>(sbw, twq, lt, u);
                tail_pass<N, 1>(sbw, twq, lt, u);
                tail_pass<N, 2>(sbw, twq, lt, u);
                if constexpr (tail_passes<N>() == 4) tail_pass<N, 3>(sbw, twq, lt, u);
                const int ob = wv == slot ? fbase : wv == 0 ? pfb0 : wv == 1 ? pfb1 : pfb2;
                const int ok = wv == slot ? kc : wv == 0 ? pkc0 : wv == 1 ? pkc1 : pkc2;
                tail_emit<N, NCO, CS16>(out, ob, ok, lt, u, oa, nco);
            }
            if (slot == 0) pfb0 = fbase, pkc0 = kc;
            else if (slot == 1) pfb1 = fbase, pkc1 = kc;
            else if (slot == 2) pfb2 = fbase, pkc2 = kc;
            fi++;
        }
        ST_FRAME_END();
        f = fn;
    }
    ST_WRITE(g_p_stamps, w, tid);
}

// ---------------------------------------------------------------------------------------------
// Split x filter coefficients for one (d, tunebin), inverse input m (bin = tb + m - (m >= N/2 ? N : 0),
// fft_mt_r2iq_impl.hpp:84-98; zero outside [0, 4096)): P as float2 (bytes 0 .. 8 N) and
// r = Q / (i P) as float from float index 2 N (split_pr), at pq_p_index / pq_r_index.  r is infinite at bin 2048 (P = 0,
// X Hh = Q conj Zc): there r = 2^64 and P = Q / (i 2^64), exact power-of-two scalings, so that
// P (Zk + i r conj Zc) = Q conj Zc - i 2^-64 Q Zk, the second term far below float32's resolution
// of the first (|Zc| < 2^28: no overflow).  Evaluated in double from the float tables and rounded once.
__global__ void build_split_filter_kernel(const float2 *__restrict__ hsel, const float2 *__restrict__ post8192,
                                          int N, int tunebin, float4 *__restrict__ pq)
{
    const int m = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (m >= N) return;
    const int bin = tunebin + m - (m >= N / 2 ? N : 0);
    float2 p = make_float2(0.f, 0.f);
    float r = 0.f;
    if (bin >= 0 && bin < HALF) {
        const double hr = hsel[m].x, hi = hsel[m].y;
        const double wr = post8192[bin].x, wi = post8192[bin].y;
        // 1 - i W = (1 + wi, -wr), 1 + i W = (1 - wi, wr)
        const double pr = 1.0 + wi, pi = -wr, qr = 1.0 - wi, qi = wr;
        if (bin == HALF / 2) {
            constexpr double s = 0x1p-64;
            const double q0 = hr * qr - hi * qi, q1 = hr * qi + hi * qr;
            p = make_float2((float)(q1 * s), (float)(-q0 * s));   // -i Q 2^-64
            r = 0x1p64f;
        } else {
            p = make_float2((float)(hr * pr - hi * pi), (float)(hr * pi + hi * pr));
            r = (float)((-qr * pi + qi * pr) / (pi * pi + pr * pr));   // Re[(qr + i qi) / (-pi + i pr)]
        }
    }
    reinterpret_cast<float2 *>(pq)[pq_p_index(N, m)] = p;
    reinterpret_cast<float *>(pq)[2 * N + pq_r_index(N, m)] = r;
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
    unsigned slotw; // the static split's slot weights (ddc_queue.hpp slot_split), 0: equal
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
                       L.nco, occ == 4 && grid == cus * occ ? L.slotw : 0u);
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

hipError_t launch_frames_persistent(const KernelTables &t, int d, const int16_t *d_in, int nblk, void *d_out,
                                    const float4 *pq, int tunebin, int lsb, int rand, int cs16, float cs16_scale,
                                    const float2 *nco_starts, const float2 *nco_trig, int slot_weights, int device,
                                    hipStream_t s)
{
    const Launch L{d_in, nblk, d_out, pq, tunebin, device, s, OutArgs{lsb ? 0x80000000u : 0u, cs16_scale},
                   NcoArgs{nco_starts, nco_trig}, slot_weights && d >= 0 && d <= 6 ? kSlotWeights[d] : 0u};
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

// Diagnostic (SDDC_STAMPS builds only): copy the persistent kernel's stamp buffer of the last
// launch ([workgroup][wave][words], tools/fs_stamps.py --kernel p) to host memory; -1 in product
// builds.
extern "C" int sddc_ddc_internal_p_stamps(unsigned *host, int nwords, int *words_per_wave)
{
    if (words_per_wave) *words_per_wave = sddc::kStampWords;
#ifdef SDDC_STAMPS
    const size_t n = sizeof(sddc::g_p_stamps) / sizeof(unsigned);
    if (!host || nwords < 0 || (size_t)nwords > n) return -2;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(sddc::g_p_stamps), (size_t)nwords * sizeof(unsigned), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
#else
    (void)host;
    (void)nwords;
    return -1;
#endif
}
