// ddc_fs.hip — the d = 0 single-channel kernel for gfx950 (the BASELINE C2 path, decim = 2):
// the fused-split (FS) frame kernel.
//
// Per frame it runs the reference's worker (Core/fft_mt_r2iq_impl.hpp:76-138): convert (+ rand),
// r2c 8192 as a 4096-point packed complex FFT, split x shift x filter with the zero fill, the
// inverse 4096-point FFT and the overlap-discard store, as six radix-16 passes on 256 threads
// (16 points each) with four LDS exchanges:
//   F0 convert + DFT-16 from registers      -> LDS
//   F1 table twiddles + DFT-16               -> LDS
//   F2 recurrence twiddles + DFT-16, then the split x filter and I0's DFT-16 in registers
//                                            -> LDS
//   I1 table twiddles + DFT-16               -> LDS
//   I2 twiddles g_t W^{-t r} + DFT-16, quarter turns, overlap-discard IQ stores.
// Every exchange writes in place of its own reads (the pair-interleaved row layout fs_slot,
// below), so a frame has four barriers, every LDS access is one base plus a per-register
// immediate, and no access has a bank conflict.
//
// The fused split.  F2's butterfly on lane l is column c = kFsPerm[l]: it produces Z[c + 256 k],
// k = 0..15.  The split of bin b needs Z[-b]; for b = c + 256 k that is Z[(256 - c) + 256 (15 - k)],
// and lane l ^ 1 holds column 256 - c (the permutation pairs the lanes), so the mirror is the
// partner lane's register 15 - k: a DPP quad_perm [1,0,3,2] operand of the split's FMAs
// (v_fmac_f32_dpp, no extra instruction).  The self-mirrored columns 0 and 128 (lanes 0, 1 of
// wave 0) read their own registers instead (a wave-uniform branch, selects in wave 0 only).
// The inverse then runs on absolute bin indices: I0's butterfly c takes the split values of
// bins c + 256 s, i.e. the lane's own registers.  The tune shift, which the reference applies as
// an input offset (T[m] = X[tb + m] H[m], impl.hpp:84-96), becomes the output modulation
// y[n] = e^{-2 pi i tb n / 4096} y'[n] (y' the inverse FFT over bins):
//   n = t + 256 k:  e^{-2 pi i tb t / 4096} (lane factor g_t, folded into I2's twiddles)
//   x W_16^{(tb mod 16) k} (a quarter turn per output register: tb is a multiple of 4).
// The (P, Q) table is indexed by bin (zero out of band: the reference's zero fill) in lane order.
// tools/fs_model.py models the frame step by step against the f64 oracle.
//
// Layout for MI355X: one 256-thread workgroup (4 wave64) per frame in flight, 4 workgroups per
// CU (40 852 B of LDS each fill the 160 KB), persistent grid (CUs x 4) fed by the slot-weighted
// static frame split of ddc_queue.hpp (queue, work stealing: options), the next frame's input prefetched into
// registers under inverse pass 1, all global memory through raw buffer instructions (scalar base
// + lane offset), nt IQ stores.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "ddc_frame_common.hpp"
#include "ddc_queue.hpp"
#include "ddc_stamps.hpp"
#include "ddc_fs_perm.h"

namespace sddc {
namespace {

#ifdef SDDC_STAMPS
__device__ unsigned g_fs_stamps[2048 * 4 * kStampWords];
#endif

__device__ __forceinline__ float dpp_partner(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}

// The split x filter of bin b from P (the per-tune-bin table) and r = Q / (i P) (real, tune-bin
// independent, held in registers; build_fs_tables_kernel):
//   F = Z_b P + conj(Z_-b) Q = P (Z_b + i r conj(Z_-b)),   Z_b + i r conj(Z_-b) = (Z.x + r Zm.y, Z.y + r Zm.x)
// with Z_-b the partner lane's register 15 - k: the DPP operand of two FMAs (v_fmac_f32_dpp), then
// the product with P.  s_nop 1: a DPP read of a VGPR needs two wait states after the VALU write
// of it (the compiler cannot see into the asm).
// Both bins of the pair (k, 15 - k): vb (a copy of zb, the register 15 - k) takes its partner term
// first, while za (register k, updated in place) is still unmodified in every lane; za's own
// partner term then reads the untouched zb.
__device__ __forceinline__ void split_v2(float2 &za, float2 &vb, float2 zb, float ra, float rb)
{
    asm("s_nop 1\n\t"
        "v_fmac_f32_dpp %2, %1, %7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %3, %0, %7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %5, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %4, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
        : "+v"(za.x), "+v"(za.y), "+&v"(vb.x), "+&v"(vb.y)
        : "v"(zb.x), "v"(zb.y), "v"(ra), "v"(rb));
}

// one bin: z += i r conj(z of the partner lane), in place (the partner's register is not written)
__device__ __forceinline__ void split_v1(float2 &z, float2 zp, float r)
{
    asm("s_nop 1\n\t"
        "v_fmac_f32_dpp %0, %3, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %2, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
        : "+v"(z.x), "+v"(z.y)
        : "v"(zp.x), "v"(zp.y), "v"(r));
}

// F = P V
__device__ __forceinline__ float2 p_mul(float2 v, float2 q)
{
    return make_float2(fmaf(v.x, q.x, -v.y * q.y), fmaf(v.x, q.y, v.y * q.x));
}

// v (-i)^s, then the sideband flip (imag sign) when LSB: s and LSB are constants after unrolling,
// so the whole output stage is at most one sign XOR per component
template <bool LSB>
__device__ __forceinline__ float2 quarter_flip(float2 v, int s)
{
    s &= 3;
    float2 o = s == 0 ? v : s == 1 ? make_float2(v.y, -v.x) : s == 2 ? make_float2(-v.x, -v.y) : make_float2(-v.y, v.x);
    if constexpr (LSB) o.y = -o.y;
    return o;
}

template <int QT, bool LSB, bool NCO, bool CS16>
__device__ __forceinline__ void emit_frame_q(void *__restrict__ out, int fbase, int k, int t, const float2 (&u)[16],
                                             const OutArgs &oa, const NcoArgs &nco)
{
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(static_cast<char *>(out) + (size_t)fbase * out_bytes<CS16>());
    const int r0 = k == 0 ? 4 : 0;   // wave-uniform
#pragma unroll
    for (int r = 0; r < 12; r++) {
        if (r < r0) continue;
        float2 v = quarter_flip<LSB>(u[r], QT * r);
        if constexpr (NCO) v = nco_mix(v, nco, fbase + t + NT * r);
        store_iq<CS16>(v, ro, (unsigned)t, (unsigned)(NT * r), oa);
    }
}

// The queue wave (not wave 0, which also carries the self-mirrored columns' split)
constexpr int kQWave = 3;
// P table loads in flight ahead of the split's use, in bin pairs (p, 15 - p).  Two pairs
// (113 VGPRs with the 12-byte (P, r) table) measured 1 % slower (profiles/r06/ab/fs_pq_ahead2_*.txt);
// holding forward pass 2's eight product twiddle powers in registers across frames (26 VALU per
// wave-frame fewer, 128 VGPRs, spills in the NCO / CS16 instances) measured neutral (same files).
constexpr int kFsPqAhead = 1;
// fs_slot(t, 0): the F0 / I2 row of thread t
__device__ __forceinline__ int fs_row_slot(int t) { return 272 * (t >> 4) + (t >= 128) + 34 * ((t & 15) >> 1) + (t & 1); }
// fs_pair_lane: F1's and I1's thread t takes row u = 2 (t >> 5) + (t & 1) of each 16-row block,
// column j = (t >> 1) & 15: its base slot fs_slot(u, j) = 34 (t >> 5) + (t & 31) = t + 2 (t >> 5)
// (the block's 272 r + [r >= 8] is the immediate)
__device__ __forceinline__ int fs_pair_row(int t) { return 2 * (t >> 5) + (t & 1); }
__device__ __forceinline__ int fs_pair_col(int t) { return (t >> 1) & 15; }
__device__ __forceinline__ int fs_pair_slot(int t) { return t + 2 * (t >> 5); }
// The exchanges' LDS layout (round 6): row R (0..255), column j (0..15) at
//   fs_slot(R, j) = 272 (R >> 4) + [R >= 128] + 34 ((R & 15) >> 1) + (R & 1) + 2 j:
// rows 2i and 2i + 1 of a 16-row block interleave (even and odd slots) in a 32-slot run, the runs
// 34 slots apart.  The access patterns (gfx950 banking, MI355X_MICROARCH.md LDS table: a
// ds_read_b64 serves 32-lane groups, conflict-free iff the slots differ mod 32; ds_write_b64
// 16-lane groups, mod 16), each one base plus a per-register immediate:
//   F0 stores / I2 reads: thread t's row t, base fs_slot(t, 0) + 2 r: slot = (t & 15) + 2 r
//     mod 16 and 16 ((t >> 4) & 1) + (t & 15) + 2 r mod 32 (272 = 16 mod 32);
//   F1, I1 (reads and in-place stores): thread t takes the row pair q = t >> 5, row
//     u = 2 q + (t & 1), column j = (t >> 1) & 15 (fs_pair_lane): slots 34 q + (t & 31) + 272 r
//     + [r >= 8], 32 consecutive per 32-lane group;
//   F2 reads / I0 stores: column c = 16 h + cl reads rows 16 h + r, column cl: base
//     272 h + [h >= 8] + 2 cl, immediate 34 (r >> 1) + (r & 1), conflict-free for kFsPerm
//     (tools/fs_perm.py; the odd upper-half pad keeps the lane pairs c, 256 - c apart).
// Round 5's 17-slot rows left one 2-way conflict per 32 lanes on every F1 and I1 read (11 % of the
// LDS cycles), which no lane assignment removes on contiguous rows.  A skewed layout with the F0
// rows permuted across lanes (fs_slot 264-slot blocks, rows rotated in each 32-lane run) was
// conflict-free too but 4 % slower: its input loads and IQ stores were no longer in lane order
// (DESIGN.md §4.1, round 6).  tests/test_fs_model.py checks every exchange's delivery, the in-place
// property and the bank keys.
constexpr int kFsLds = 4352;
// twiddle bases W^j (j < 256) at j + [j >= 128], W^{4j} kFsTw later: F2 reads them at its column
// c = kFsPerm[t], whose key c + [c >= 128] the permutation keeps distinct mod 32 over 32 lanes
// (tools/fs_perm.py), I2 at t; both ds_read_b64 and conflict-free.  (Unpadded, the lane pairs
// c, 256 - c with c = 0 mod 16 hit one bank.)
constexpr int kFsTw = NT + 1;

// the frame schedules (ddc_queue.hpp): the slot-weighted static split alone (the default), the
// static prefix + dynamic queue (round 3/4), work stealing over the static split (round 5)
enum { kSchedStatic = 0, kSchedQueue = 1, kSchedSteal = 2 };
template <int SCHED> struct SchedOf { using T = StealSchedule; };
template <> struct SchedOf<kSchedStatic> { using T = StaticSchedule; };
template <> struct SchedOf<kSchedQueue> { using T = FrameSchedule<1>; };

// ZR: whole rows of the inverse input known zero for this tune bin (the reference's zero fill,
// impl.hpp:91-96; fs_zero_rows): ZR > 0 = rows 16 - ZR .. 15, ZR < 0 = rows 0 .. -ZR - 1, 2 to 8
// rows (tb = 1024, the benchmark's: rows 12..15).  Their (P, Q) loads and split FMAs
// are skipped and I0's first radix-4s take only the live rows (dft16z).
template <int ZR>
__device__ __forceinline__ constexpr bool zrow(int k) { return zr_row<ZR>(k); }

template <int SCHED, int ZR, bool RAND, bool LSB, bool NCO, bool CS16>
__global__ __launch_bounds__(NT, 4) void r2iq_fs_kernel(
    const int *__restrict__ in32, void *__restrict__ out, int nframes, const float2 *__restrict__ tw_p1,
    const float2 *__restrict__ rec_f, const float4 *__restrict__ pqf, const float2 *__restrict__ fsl, int tunebin,
    OutArgs oa, NcoArgs nco, unsigned *__restrict__ wq, int ns, unsigned slotw, int xmap, int minrem, int pub)
{
    __shared__ __attribute__((aligned(16))) float2 lds[kFsLds];
    // F1 twiddles W_256^{s r} [15][16] (I1 conjugates them: at d = 0 its table is the same) and
    // the NS = 256 passes' bases W^j, W^{4j} (j < 256: F2 reads them at the lane's column, I2 at
    // its thread index).  In LDS, not registers or L2: the L2 loads' waits (vmcnt, in issue
    // order) would also wait for the input prefetch and the stores.
    __shared__ __attribute__((aligned(16))) float2 twl[15 * 16];
    __shared__ __attribute__((aligned(16))) float2 wtab[2 * kFsTw];
    __shared__ int s_next;   // the workgroup's next frame (the queue wave's schedule), -1 when none is left
    static_assert(sizeof(float2) * (kFsLds + 15 * 16 + 2 * kFsTw) + sizeof(int) <= 163840 / 4,
                  "four workgroups per CU");

    const int tid = (int)threadIdx.x;
    // xmap (non-persistent grids): blockIdx b runs on XCD b % 8 under round-robin placement, and
    // takes frame range (b % 8) G / 8 + b / 8, so that each XCD walks a contiguous stretch
    const int w = xmap ? (int)(blockIdx.x & 7u) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    constexpr int QLANE = 64 * kQWave;
    const bool qw = __builtin_amdgcn_readfirstlane(tid >> 6) == kQWave;
    typename SchedOf<SCHED>::T fsch;
    int x[16];
    {
        // every wave knows the first frame (it is static unless the batch is small): its input
        // loads go out at once, ahead of the table copies
        const int G = (int)gridDim.x, a0 = slot_split(ns, G, w, slotw);
        const int f0s = a0 < slot_split(ns, G, w + 1, slotw) ? a0 : -1;
        if (f0s >= 0) load_frame(in32, f0s / FRAMES, f0s % FRAMES, x);
        if (qw) {
            int f0[1];
            if constexpr (SCHED == kSchedSteal) fsch.init(wq, nframes, ns, w, G, slotw, f0, minrem, pub);
            else fsch.init(wq, nframes, ns, w, G, slotw, f0);
            if (tid == QLANE) s_next = f0[0];
        }
        for (int i = tid; i < 15 * 16; i += NT) twl[i] = tw_p1[i];
        wtab[tid + (tid >= 128)] = rec_f[tid];
        wtab[kFsTw + tid + (tid >= 128)] = rec_f[NT + tid];
        __syncthreads();
        const int f = s_next;
        if (f >= 0 && f0s < 0) load_frame(in32, f / FRAMES, f % FRAMES, x);
    }
    int f = s_next;
    int blk = f / FRAMES, k = f - blk * FRAMES;
    const int col_ = kFsPerm[tid];
    const int qt = (tunebin >> 2) & 3;   // (tb mod 16) / 4: the output quarter turns
    const bool w0 = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;   // the wave holding columns 0, 128
    // The frame loop runs in two phases.  Phase A: frames of the workgroup's own range whose next
    // frame and the one after it are private too (StaticSchedule: all of them), the next frame
    // f + 1, known to every wave, no schedule state.  Phase B: the rest, with the schedule object
    // on the queue wave and the next frame through s_next (the queue: every frame; work stealing:
    // the range's public end and what it steals).  Phase A is a copy of the frame body without
    // the schedule's registers, so the owner's frames cost what the static schedule's do.
    // Frame-invariant lane values held in registers for the whole launch (read once here instead
    // of from L2 every frame): the split's r of the lane's live bins (16 - |ZR| VGPRs; the P table
    // drops to 8 bytes per bin) and, for the static schedule, I2's lane factors g_t, g_t W^{-t},
    // g_t W^{-4t} (6 VGPRs; the queue and stealing schedules, at 124-128 VGPRs, keep the loads).
    // Per frame 12 KB of table reads fewer at tb = 1024: +2.5-3 % (profiles/r06/ab/
    // fs_cached_r_and_lane_factors_*.txt).  118 VGPRs at ZR = 4 (128 with the P pairs below).
    float cr[16];
    {
        const __amdgpu_buffer_rsrc_t rr = buf_rsrc(reinterpret_cast<const float *>(pqf) + 2 * HALF);
#pragma unroll
        for (int k = 0; k < 16; k++)
            if (!zrow<ZR>(k)) cr[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, 4u * tid, 4u * NT * k, 0));
    }
    // The plain static instances with zero rows (108-120 VGPRs before) also hold P of their first
    // pairs p, 15 - p in registers: the |ZR| single-bin pairs (one row zero) and, at |ZR| = 4..7,
    // one two-bin pair (at |ZR| = 7, 8 every live row; 122-126 VGPRs).  At tb 1024 (|ZR| = 4)
    // 6 of 12 P loads per lane and frame stay: +1.4 %; |ZR| = 5..8: +1.2-2.7 %, bit-identical
    // (profiles/r06/ab/fs_cached_p_*.txt)
    constexpr int AZR = ZR > 0 ? ZR : -ZR;
    constexpr int CPP = SCHED == kSchedStatic && !NCO && !CS16 && AZR >= 3 ? (AZR >= 4 && AZR <= 7 ? AZR + 1 : AZR) : 0;
    float2 cp[16];
    if constexpr (CPP > 0) {
        const __amdgpu_buffer_rsrc_t rq = buf_rsrc(pqf);
#pragma unroll
        for (int k = 0; k < 16; k++)
            if (!zrow<ZR>(k) && (k < CPP || 15 - k < CPP))
                cp[k] = buf_load8(rq, 16u * tid, 4096u * (k < 8 ? k : 15 - k) + (k < 8 ? 0u : 8u));
    }
    constexpr bool GREG = SCHED == kSchedStatic;
    float2 cg0, cg1, cg4;
    if constexpr (GREG) {
        const __amdgpu_buffer_rsrc_t rfs = buf_rsrc(fsl);
        const unsigned t8 = 8u * (unsigned)tid;
        cg0 = buf_load8(rfs, t8, 0);
        cg1 = buf_load8(rfs, t8, 8u * NT);
        cg4 = buf_load8(rfs, t8, 16u * NT);
    }
    int pA = -1, fend = -1;
    {
        const int G = (int)gridDim.x, a = slot_split(ns, G, w, slotw), b = slot_split(ns, G, w + 1, slotw);
        if constexpr (SCHED == kSchedStatic) {
            pA = b + 2;
            fend = b;
        } else if constexpr (SCHED == kSchedSteal) {
            const int len = b - a, two = len < 2 ? len : 2;
            pA = minrem <= 0 ? b + 2 : a + (pub > 0 && len - pub > two ? len - pub : two);
            fend = minrem <= 0 ? b : pA;
        }
    }
    ST_INIT();

    auto frame = [&](auto phase) __attribute__((always_inline)) {
        constexpr bool PB = decltype(phase)::value;
        if constexpr (PB && SCHED != kSchedSteal)
            if (qw) fsch.peek();
        // opaque per-frame copies of the thread index and column: without them the compiler
        // hoists every loop-invariant LDS address out of the frame loop and spills them
        int z = 0;
        asm volatile("" : "+s"(z));
        const int t = tid + z;
        const int c = col_ + z;
        const int oblk = blk * 8 * HALF;
        const int kc = k;
        // ---- F0 (R16, NS1): convert + DFT16 from registers ----
        float2 v[16];
        {
            float2 a[16];
#pragma unroll
            for (int r = 0; r < 16; r++)
                if constexpr (RAND) {
                    // convert_float<rand> (fft_mt_r2iq.h:36-51) on the int16 pair: an odd sample is
                    // XORed with 0xFFFE, i.e. word ^ (word & 0x10001) * 0xFFFE, integer-exact
                    const int wd = x[r] ^ (int)(((unsigned)x[r] & 0x10001u) * 0xFFFEu);
                    a[r] = make_float2((float)(int)(short)(wd & 0xffff), (float)(wd >> 16));
                } else {
                    a[r] = make_float2((float)(int)(short)(x[r] & 0xffff), (float)(x[r] >> 16));
                }
            dft16<-1>(a, v);
        }
        // no barrier: this thread's row is exactly what it read in the previous frame's inverse
        // pass 2 (every exchange writes in place of its own reads)
        {
            float2 *const row = lds + fs_row_slot(t);
#pragma unroll
            for (int r = 0; r < 16; r++) row[2 * r] = v[r];
        }
        ST_SYNC(1);
        // ---- F1 (R16, NS16): table twiddles W_256^{j r} ----
        // rows 16 r + u, column j of the thread's pair lane (u, j) (fs_pair_lane)
        {
            float2 a[16];
            const float2 *const col = lds + fs_pair_slot(t);
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], col[272 * r + (r >= 8)]);
            table_twiddle<-1, true>(a, twl, 16, fs_pair_col(t));
            dft16<-1>(a, v);
        }
        {
            // in place of the reads (no barrier)
            float2 *const col = lds + fs_pair_slot(t);
#pragma unroll
            for (int r = 0; r < 16; r++) col[272 * r + (r >= 8)] = v[r];
        }
        ST_SYNC(3);
        if constexpr (PB && SCHED == kSchedSteal)
            if (qw) fsch.peek();
        // ---- F2 (R16, NS256) on column c: Z[c + 256 k] in v[k] ----
        // The split's P loads (bin pairs p, 15 - p; 8 bytes per bin) run a pair ahead of their
        // use, the first issued before F2 so that its reads and arithmetic cover the L2 latency
        // (an empty asm with a memory clobber pins each group; the compiler's own schedule waits
        // for every pair right after issuing it).  Issuing the first pair after the register-held
        // ones before F2 instead measured -2.4 to +0.9 % (fs_first_uncached_p_before_f2_NEUTRAL.txt).
        const __amdgpu_buffer_rsrc_t rpq = buf_rsrc(pqf + z);
        const unsigned t16 = 16u * (unsigned)t;
        float2 qa[8], qb[8];
        // pair p's P (rows p and 15 - p side by side, build_fs_tables_kernel): one 16-byte load,
        // or 8 bytes when a row is zero; the first CPP pairs from registers
        // (8-byte halves where a 16-byte load would spill: ZR = +-2, the stealing schedule)
        constexpr bool P16 = ZR != 2 && ZR != -2 && SCHED != kSchedSteal;
        auto pload = [&](int p) __attribute__((always_inline)) {
            const bool za = zrow<ZR>(p), zb = zrow<ZR>(15 - p);
            if (p < CPP) {
                if (!za) qa[p] = cp[p];
                if (!zb) qb[p] = cp[15 - p];
            } else if (!za && !zb && !P16) {
                qa[p] = buf_load8(rpq, t16, 4096u * p);
                qb[p] = buf_load8(rpq, t16, 4096u * p + 8u);
            } else if (!za && !zb) {
                const float4 q = buf_load16(rpq, t16, 4096u * p);
                qa[p] = make_float2(q.x, q.y);
                qb[p] = make_float2(q.z, q.w);
            } else if (!za) {
                qa[p] = buf_load8(rpq, t16, 4096u * p);
            } else if (!zb) {
                qb[p] = buf_load8(rpq, t16, 4096u * p + 8u);
            }
        };
#pragma unroll
        for (int p = 0; p < kFsPqAhead; p++) {
            pload(p);
        }
        asm volatile("" ::: "memory");
        {
            float2 a[16];
            // F1 output c >> 4 of its pair lanes (r, c & 15): rows 16 (c >> 4) + r, column c & 15
            // at 272 (c >> 4) + [c >= 128] + 2 (c & 15) + 34 (r >> 1) + (r & 1): base + immediate,
            // conflict-free with kFsPerm (tools/fs_perm.py)
            const float2 *const cb = lds + 272 * (c >> 4) + (c >= 128) + 2 * (c & 15);
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], cb[34 * (r >> 1) + (r & 1)]);
            const int cw = c + (c >= 128);
            const float2 fw1 = wtab[cw], fw4 = wtab[kFsTw + cw];   // W^c, W^{4c}
            twiddle_rec16<-1>(a, fw1, fw4);
            dft16<-1>(a, v);
        }
        // ---- split x filter (bins c + 256 k, mirror from the partner lane) -> I0 DFT ----
        float2 u[16];
        {
            float2 a[16];
            auto split_w0 = [&]() __attribute__((always_inline)) {
                // wave 0: lanes 0 (column 0: mirror of register k is its own (16 - k) mod 16) and
                // 1 (column 128: its own 15 - k) are self-mirrored.  Bin 2048 (lane 0, register 8)
                // has P = 0 (r infinite): its table entry holds Q, and F = Q conj(Z) there.
                const int lane = t & 63;
#pragma unroll
                for (int p = 0; p < 8; p++) {
                    if (p + kFsPqAhead < 8) {
                        const int pn = p + kFsPqAhead;
                        pload(pn);
                        asm volatile("" ::: "memory");
                    }
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const int kk = h ? 15 - p : p;
                        if (zrow<ZR>(kk)) continue;
                        const float2 q = h ? qb[p] : qa[p];
                        const float2 vm = v[15 - kk], v0m = v[(16 - kk) & 15];
                        float2 zc = make_float2(dpp_partner(vm.x), dpp_partner(vm.y));
                        zc = lane == 1 ? vm : zc;
                        zc = lane == 0 ? v0m : zc;
                        float2 vv = make_float2(fmaf(cr[kk], zc.y, v[kk].x), fmaf(cr[kk], zc.x, v[kk].y));
                        if (kk == 8) vv = lane == 0 ? make_float2(v[8].x, -v[8].y) : vv;
                        a[kk] = p_mul(vv, q);
                    }
                }
            };
            auto split_generic = [&]() __attribute__((always_inline)) {
#pragma unroll
                for (int p = 0; p < 8; p++) {
                    if (p + kFsPqAhead < 8) {
                        const int pn = p + kFsPqAhead;
                        pload(pn);
                        asm volatile("" ::: "memory");
                    }
                    if (zrow<ZR>(15 - p)) {   // row 15 - p zero: row p's bin alone (v[15 - p] unwritten)
                        split_v1(v[p], v[15 - p], cr[p]);
                        a[p] = p_mul(v[p], qa[p]);
                    } else if (zrow<ZR>(p)) {
                        split_v1(v[15 - p], v[p], cr[15 - p]);
                        a[15 - p] = p_mul(v[15 - p], qb[p]);
                    } else {
                        float2 vb = v[15 - p];
                        split_v2(v[p], vb, v[15 - p], cr[p], cr[15 - p]);
                        a[p] = p_mul(v[p], qa[p]);
                        a[15 - p] = p_mul(vb, qb[p]);
                    }
                }
            };
            // wave 0's path first, then the generic one, as two ifs on conditions the compiler
            // cannot relate (an opaque wave index): as an if / else the compiler laid the generic
            // path out first, so the Z registers it updates in place stayed live for wave 0's path
            // and every update went through a copy (16 v_mov per wave-frame).  Without zero rows
            // the two-if form spills 2-4 VGPRs, so ZR = 0 keeps the if / else.
            if constexpr (ZR != 0) {
                int wv = __builtin_amdgcn_readfirstlane(t >> 6);
                asm volatile("" : "+s"(wv));
                if (w0) split_w0();
                if (wv != 0) split_generic();
            } else {
                if (w0) split_w0();
                else split_generic();
            }
            dft16z<+1, ZR>(a, u);
        }
        {
            // in place of this thread's F2 reads (no barrier): output r at row 16 (c >> 4) + r
            int c1 = c;
            asm volatile("" : "+v"(c1));
            float2 *const cb = lds + 272 * (c1 >> 4) + (c1 >= 128) + 2 * (c1 & 15);
#pragma unroll
            for (int r = 0; r < 16; r++) cb[34 * (r >> 1) + (r & 1)] = u[r];
        }
        // the next frame (phase B: the schedule's, from the ticket read at this frame's top;
        // ddc_queue.hpp)
        if constexpr (PB) {
            if (qw) {
                const int f_n = fsch.next();
                if (tid == QLANE) s_next = f_n;
            }
        }
        ST_SYNC(5);
        // I2's lane factors g_t, g_t W^{-t}, g_t W^{-4t} (exactly rounded, from the per-tunebin
        // table): issued ahead of the input prefetch, so that their wait does not include it
        const __amdgpu_buffer_rsrc_t rfs = buf_rsrc(fsl);
        const unsigned t8 = 8u * (unsigned)t;
        float2 g0, g1, g4;
        if constexpr (GREG) {
            g0 = cg0;
            g1 = cg1;
            g4 = cg4;
        } else {
            g0 = buf_load8(rfs, t8, 0);
            g1 = buf_load8(rfs, t8, 8u * NT);
            g4 = buf_load8(rfs, t8, 16u * NT);
        }
        int fn;
        // ---- I1 (R16, NS16): table twiddles W_256^{-s r} ----
        {
            float2 a[16];
            // I0 output s of columns 16 r + cl, for the pair lane (s, cl) = (u, j) of this
            // thread (fs_pair_lane): rows 16 r + s, column cl, the slots F1 used
            const float2 *const ib = lds + fs_pair_slot(t);
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], ib[272 * r + (r >= 8)]);
            // the next frame's number is read behind the data reads (its LDS round trip under
            // theirs), and its input loads are issued here rather than in F0, so their 16
            // registers are free through F2 and the split
            if constexpr (PB) fn = s_next;
            else fn = f + 1 < fend ? f + 1 : -1;
            if (fn >= 0) {
                blk = fn / FRAMES;
                k = fn - blk * FRAMES;
                load_frame(in32, blk, k, x);
            }
            // the ticket for the frame after the next one, when that one is dynamic: behind this
            // frame's last loads (vmcnt counts in issue order: taken at inverse pass 0, the wait
            // for I2's lane factors included the atomic); read at the next frame's top
            if constexpr (PB)
                if (qw) fsch.take();
            table_twiddle<+1, true>(a, twl, 16, fs_pair_row(t));
            dft16<+1>(a, u);
        }
        {
            // in place of this thread's I1 reads (no barrier), recomputed from an opaque copy of
            // t (else kept live through the pass): output g at row 16 g + s, column cl
            int t1 = t;
            asm volatile("" : "+v"(t1));
            float2 *const ib = lds + fs_pair_slot(t1);
#pragma unroll
            for (int r = 0; r < 16; r++) ib[272 * r + (r >= 8)] = u[r];
        }
        ST_SYNC(7);
        // ---- I2 (R16, NS256): twiddles g_t W^{-t r}, quarter turns, overlap-discard ----
        {
            float2 a[16];
            // row t (I1 outputs t >> 4 of its pair lanes (t & 15, r)): the next frame's F0 row of
            // this thread
            const float2 *const rb = lds + fs_row_slot(t);
#pragma unroll
            for (int r = 0; r < 16; r++) XRD(a[r], rb[2 * r]);
            const int tw = t + (t >= 128);
            const float2 rw1 = wtab[tw], rw4 = wtab[kFsTw + tw];   // W^t, W^{4t}
            twiddle_g16<+1>(a, g0, g1, g4, rw1, rw4);
            dft16<+1>(a, u);
            const int fb = oblk + emit_base<HALF>(kc);
            switch (qt) {
            case 0: emit_frame_q<0, LSB, NCO, CS16>(out, fb, kc, t, u, oa, nco); break;
            case 1: emit_frame_q<1, LSB, NCO, CS16>(out, fb, kc, t, u, oa, nco); break;
            case 2: emit_frame_q<2, LSB, NCO, CS16>(out, fb, kc, t, u, oa, nco); break;
            default: emit_frame_q<3, LSB, NCO, CS16>(out, fb, kc, t, u, oa, nco); break;
            }
        }
        if constexpr (SCHED == kSchedSteal) {
            if constexpr (PB)
                if (qw) fsch.take_late();
        }
        ST_FRAME_END();
        f = fn;
    };
    if constexpr (SCHED != kSchedQueue)
        while (f >= 0 && f + 2 < pA) frame(std::false_type{});
    if constexpr (SCHED != kSchedStatic) {
        if constexpr (SCHED == kSchedSteal)
            if (qw) fsch.enter(f);
        while (f >= 0) frame(std::true_type{});
    }
    ST_WRITE(g_fs_stamps, w, tid);
    if constexpr (SCHED == kSchedQueue)
        if (tid == QLANE) fs_queue_done(wq, (unsigned)gridDim.x);
}

// FS tables of one tunebin, for lane l and row k (bin b = kFsPerm[l] + 256 k): P as float2 at
// float2 index 2 (256 p + l) + [k >= 8], p = min(k, 15 - k), i.e. the pair's rows k, 15 - k side by
// side for one 16-byte load (bytes 0 .. 32 K), and r as float at byte 32 K + 4 (l + 256 k) (inverse input
// m = (b - tb) mod 4096; P and Q = i r P zero unless b is in the reference's band:
// tb <= b < tb + 2048, b < 4096, or tb - 2048 <= b < tb).  With P = H (1 - i W), Q = H (1 + i W)
// (H = H_0[m] / 2, W = e^{-2 pi i b / 8192}), r = Q / (i P) = (1 + i W) / (i (1 - i W))
// = cot(pi/4 - pi b / 8192) is real and does not depend on H or the tune bin; it is infinite only
// at b = 2048 (column 0, register 8), whose entry holds (Q, 0) instead (the kernel's wave-0 path).
// Versus the (P, Q) float4 of round 5: 6 or 7 VALU per bin instead of 8, and 8 bytes per bin read
// from L2 every frame instead of 16 (r is read once per launch).  tools/fs_model.py (split "pr")
// models it.
// fsl = [g_t | g_t W^{-t} | g_t W^{-4t}], g_t = e^{-2 pi i tb t / 4096}, looked up exactly in the
// 4096-point table.
__global__ void build_fs_tables_kernel(const float2 *__restrict__ hsel0, const float2 *__restrict__ post8192,
                                       const float2 *__restrict__ tw4096, int tunebin, float4 *__restrict__ pqf,
                                       float2 *__restrict__ fsl)
{
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= HALF) return;
    const int l = i & (NT - 1), kk = i >> 8;
    const int b = kFsPerm[l] + NT * kk;
    const bool band = (b >= tunebin && b - tunebin < HALF / 2) || (b < tunebin && tunebin - b <= HALF / 2);
    float3 c = make_float3(0.f, 0.f, 0.f);
    if (band) {
        const int m = (b - tunebin) & (HALF - 1);
        const double hr = hsel0[m].x, hi = hsel0[m].y;
        const double wr = post8192[b].x, wi = post8192[b].y;
        const double pr = 1.0 + wi, pi = -wr, qr = 1.0 - wi, qi = wr;   // 1 - i W, 1 + i W
        if (b == HALF / 2) {   // P = 0: (Q, 0)
            c.x = (float)(hr * qr - hi * qi);
            c.y = (float)(hr * qi + hi * qr);
        } else {
            c.x = (float)(hr * pr - hi * pi);
            c.y = (float)(hr * pi + hi * pr);
            // r = Re[(1 + i W) / (i (1 - i W))] = Re[(qr + i qi) / (-pi + i pr)]
            c.z = (float)((-qr * pi + qi * pr) / (pi * pi + pr * pr));
        }
    }
    // P of rows kk and 15 - kk side by side: float2 index 2 (256 p + l) + [kk >= 8], p = min(kk, 15 - kk)
    reinterpret_cast<float2 *>(pqf)[2 * (NT * (kk < 8 ? kk : 15 - kk) + l) + (kk >= 8)] = make_float2(c.x, c.y);
    reinterpret_cast<float *>(pqf)[2 * HALF + i] = c.z;
    if (i < NT) {
        fsl[i] = tw4096[(tunebin * i) & (HALF - 1)];
        fsl[NT + i] = tw4096[((tunebin - 1) * i) & (HALF - 1)];
        fsl[2 * NT + i] = tw4096[((tunebin - 4) * i) & (HALF - 1)];
    }
}

template <int SCHED, int ZR, bool RAND, bool LSB, bool NCO, bool CS16>
hipError_t launch_fs_s(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pqf,
                       const float2 *fsl, int tunebin, const OutArgs &oa, const NcoArgs &nco, unsigned *wq,
                       const FsSched &fs, int device, hipStream_t s)
{
    auto kern = r2iq_fs_kernel<SCHED, ZR, RAND, LSB, NCO, CS16>;
    const int static_pct = SCHED == kSchedQueue ? fs.static_pct : 100, fpw = fs.fpw;
    int occ = 0, cus = 0;
    hipError_t e = launch_geometry(t.lc, reinterpret_cast<const void *>(kern), NT, device, &occ, &cus);
    if (e != hipSuccess) return e;
    const int nframes = nblk * FRAMES;
    int grid = cus * occ;
    if (grid > nframes) grid = nframes;
    int ns = frame_schedule_static(nframes, static_pct);
    unsigned slotw = occ == 4 && grid == cus * occ ? (fs.slotw ? fs.slotw : kFsSlotWeights) : 0u;
    int xmap = 0;
    if (fpw > 0) {   // non-persistent: fpw frames per workgroup, the hardware dispatcher balances
        grid = (nframes + fpw - 1) / fpw;
        ns = nframes;
        slotw = 0u;
        xmap = (grid & 7) == 0 && grid * fpw == nframes;
    }
    int minrem = fs.minrem;
    // a steal slot counts at most kStealMaxRange frames of a range, for at most kFsStealMax
    // workgroups (the largest range of the weighted split is below 2 nframes / G + 1); a launch
    // past either runs the static split alone (minrem 0)
    if (SCHED == kSchedSteal && (grid > kFsStealMax || 2LL * nframes / grid + 1 > kStealMaxRange)) minrem = 0;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), 0, s, reinterpret_cast<const int *>(d_in), d_out, nframes,
                       t.tw_p1, t.rec_f, pqf, fsl, tunebin, oa, nco, wq, ns, slotw, xmap, minrem, fs.pub);
    return hipGetLastError();
}

// zero rows of the inverse input for tune bin tb (ZR of r2iq_fs_kernel): the band is
// [tb - 2048, tb + 2048) clipped to [0, 4096) (the reference's zero fill, impl.hpp:91-96), so rows
// k >= ceil((tb + 2048) / 256) are zero (tb < 2048, ZR > 0) or rows k < floor((tb - 2048) / 256)
// (tb > 2048, ZR < 0), at most 8 (dft16z; 8 only at tb = 0: tb <= 4092 leaves at most 7 at the
// bottom); a single zero row runs unskipped (with it the compiler's schedule of the (P, Q) prefetch
// spills 5-6 VGPRs)
int fs_zero_rows(int tunebin)
{
    const int top = 16 - (tunebin + 2048 + 255) / 256, bot = tunebin > 2048 ? (tunebin - 2048) / 256 : 0;
    const int z = top > 0 ? top : bot > 0 ? -bot : 0;
    return z > 8 ? 8 : z < -8 ? -8 : z == 1 || z == -1 ? 0 : z;
}

template <int ZR, bool RAND, bool LSB, bool NCO, bool CS16>
hipError_t launch_fs_z(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pqf,
                       const float2 *fsl, int tunebin, const OutArgs &oa, const NcoArgs &nco, unsigned *wq,
                       const FsSched &fs, int device, hipStream_t s)
{
    if (fs.sched == kSchedStatic)
        return launch_fs_s<kSchedStatic, ZR, RAND, LSB, NCO, CS16>(t, d_in, nblk, d_out, pqf, fsl, tunebin, oa, nco, wq, fs, device, s);
    if constexpr (!RAND && !LSB && !NCO && !CS16 && ZR % 4 == 0) {
        if (fs.sched == kSchedSteal)
            return launch_fs_s<kSchedSteal, ZR, false, false, false, false>(t, d_in, nblk, d_out, pqf, fsl, tunebin, oa, nco, wq, fs, device, s);
        if (fs.sched == kSchedQueue)
            return launch_fs_s<kSchedQueue, ZR, false, false, false, false>(t, d_in, nblk, d_out, pqf, fsl, tunebin, oa, nco, wq, fs, device, s);
    }
    return hipErrorNotSupported;
}

// the schedule: every output configuration runs the static schedule (the default); work stealing
// and the queue (A/B, tests) are built for the plain configuration only.  fs.zr != 0 (default):
// skip the tune bin's zero rows (fs_zero_rows), 0: compute them (A/B, tests)
template <bool RAND, bool LSB, bool NCO, bool CS16>
hipError_t launch_fs_v(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pqf,
                       const float2 *fsl, int tunebin, const OutArgs &oa, const NcoArgs &nco, unsigned *wq,
                       const FsSched &fs, int device, hipStream_t s)
{
    // every zero-row count for the CF32 outputs without NCO; the fused-NCO and CS16 outputs (and
    // the A/B schedules) take 0 or 4 (fewer instances: the file compiles in parallel with nothing,
    // and each count is a whole kernel per output configuration)
    constexpr bool FINE = !NCO && !CS16;
    int zr = fs.zr ? fs_zero_rows(tunebin) : 0;
    if (!FINE || fs.sched != kSchedStatic) zr = zr >= 4 ? 4 : zr <= -4 ? -4 : 0;
#define SDDC_FS_ZR(z) \
    if (zr == (z)) return launch_fs_z<(z), RAND, LSB, NCO, CS16>(t, d_in, nblk, d_out, pqf, fsl, tunebin, oa, nco, wq, fs, device, s);
    SDDC_FS_ZR(4) SDDC_FS_ZR(-4)
    if constexpr (FINE) {
        SDDC_FS_ZR(8) SDDC_FS_ZR(7) SDDC_FS_ZR(6) SDDC_FS_ZR(5) SDDC_FS_ZR(3) SDDC_FS_ZR(2)
        SDDC_FS_ZR(-2) SDDC_FS_ZR(-3) SDDC_FS_ZR(-5) SDDC_FS_ZR(-6) SDDC_FS_ZR(-7)
    }
#undef SDDC_FS_ZR
    return launch_fs_z<0, RAND, LSB, NCO, CS16>(t, d_in, nblk, d_out, pqf, fsl, tunebin, oa, nco, wq, fs, device, s);
}

template <bool RAND, bool LSB>
hipError_t launch_fs_rl(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pqf,
                        const float2 *fsl, int tunebin, bool cs16, const OutArgs &oa, const NcoArgs &nco,
                        unsigned *wq, const FsSched &fs, int device, hipStream_t s)
{
    if (nco.starts)
        return cs16 ? launch_fs_v<RAND, LSB, true, true>(t, d_in, nblk, d_out, pqf, fsl, tunebin, oa, nco, wq, fs, device, s)
                    : launch_fs_v<RAND, LSB, true, false>(t, d_in, nblk, d_out, pqf, fsl, tunebin, oa, nco, wq, fs, device, s);
    return cs16 ? launch_fs_v<RAND, LSB, false, true>(t, d_in, nblk, d_out, pqf, fsl, tunebin, oa, nco, wq, fs, device, s)
                : launch_fs_v<RAND, LSB, false, false>(t, d_in, nblk, d_out, pqf, fsl, tunebin, oa, nco, wq, fs, device, s);
}

}  // namespace

bool fs_path(int d, int tunebin) { return d == 0 && (tunebin & 3) == 0; }

hipError_t launch_build_fs_tables(const KernelTables &t, int tunebin, float4 *pqf, float2 *fsl, hipStream_t s)
{
    if (tunebin < 0 || tunebin >= HALF || (tunebin & 3)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(build_fs_tables_kernel, dim3(HALF / 256), dim3(256), 0, s, t.hsel[0], t.post8192, t.tw4096,
                       tunebin, pqf, fsl);
    return hipGetLastError();
}

hipError_t launch_frames_fs(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pqf,
                            const float2 *fsl, int tunebin, int lsb, int rand, int cs16, float cs16_scale,
                            const float2 *nco_starts, const float2 *nco_trig, unsigned *wq, const FsSched &fs,
                            int device, hipStream_t s)
{
    if (tunebin & 3) return hipErrorInvalidValue;
    if (fs.static_pct < 0 || fs.static_pct > 100 || fs.sched < 0 || fs.sched > 2) return hipErrorInvalidValue;
    const OutArgs oa{0u, cs16_scale};   // the sideband flip is a template parameter here
    const NcoArgs nco{nco_starts, nco_trig};
    const bool c = cs16 != 0;
    if (rand)
        return lsb ? launch_fs_rl<true, true>(t, d_in, nblk, d_out, pqf, fsl, tunebin, c, oa, nco, wq, fs, device, s)
                   : launch_fs_rl<true, false>(t, d_in, nblk, d_out, pqf, fsl, tunebin, c, oa, nco, wq, fs, device, s);
    return lsb ? launch_fs_rl<false, true>(t, d_in, nblk, d_out, pqf, fsl, tunebin, c, oa, nco, wq, fs, device, s)
               : launch_fs_rl<false, false>(t, d_in, nblk, d_out, pqf, fsl, tunebin, c, oa, nco, wq, fs, device, s);
}

}  // namespace sddc

// Diagnostic (SDDC_STAMPS builds only): copy the d = 0 fused-split kernel's stamp buffer of the
// last launch ([workgroup][wave][words], tools/fs_stamps.py) to host memory; -1 in product builds.
extern "C" int sddc_ddc_internal_fs_stamps(unsigned *host, int nwords, int *words_per_wave)
{
    if (words_per_wave) *words_per_wave = sddc::kStampWords;
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
