// ddc_queue.hpp — frame distribution for the single-channel frame kernels (ddc_fs.hip,
// ddc_persistent.hip): a static prefix per workgroup, then a dynamic queue.
#pragma once

#include <hip/hip_runtime.h>

namespace sddc {
namespace {

// Dynamic frame distribution.  With a static split (each workgroup a fixed contiguous range)
// the four workgroups of a CU finish far apart: the SIMDs arbitrate by age, so the first-
// dispatched workgroup of a CU runs ~1.6x faster than the last, and the CU spends the last
// ~40 % of the launch with 3, 2, then 1 workgroup resident (s_memtime / s_memrealtime stamps
// by HW_ID slot, profiles/r03/stamps).  The frames past each workgroup's static prefix are handed
// out one at a time instead: 8 shards of consecutive frames (one counter each, on its own 64-B
// line; a workgroup starts on shard blockIdx % 8 and moves on when it runs dry), so consecutive
// frames, which share 2048 input samples, mostly stay in one XCD's L2.  The queue wave reads a
// ticket at the top of the frame after the one it was taken in, resolves it where the kernel
// needs the next frame (for its input prefetch) and takes the next ticket right after.  A
// device-scope atomic's value is waited for with vmcnt, in issue order with every other vector-
// memory operation of the wave; waiting for it in the frame it was taken cost ~1800 cycles per
// frame (profiles/r03/stamps/stamps_q.txt .. stamps_q18.txt trace the variants; A/B in
// profiles/r03/ab).
// wq: this launch's slot of the handle's queue ring, zero at entry; the last workgroup to leave
// clears it for the slot's next launch (the counters are touched only by device-scope atomics).
constexpr int FS_SHARDS = 8;
static_assert(kFsQueueWords == 16 * (FS_SHARDS + 1), "queue slot: one 64-B line per shard counter + the done count");
// first frame of shard s (32-bit: nframes * 8 < 2^31 for any batch the C ABI accepts)
__device__ __forceinline__ int fs_shard_lo(int nframes, int s) { return (nframes * s) >> 3; }

// The queue is worked by one wave (wave-uniform, so the bookkeeping is scalar); only the atomic
// increment is its lane 0's.  Every wave instruction costs ~20 cycles of wall time at 4 waves per
// SIMD, and the other waves wait for this one at the next barrier, so the per-frame path is a
// handful of instructions: the ticket taken a frame earlier is read from lane 0
// (v_readfirstlane), compared with the current shard's size, and the next one is taken.  The
// whole wave issues the ticket's atomic as a buffer atomic whose lanes other than 0 fall outside
// the buffer's range (dropped, no memory access): issued from a lane-0 branch instead, the
// ticket register became a merge of two values and the merge copy waited for the atomic's
// return right there, a device-scope round trip (~1200 cycles of the queue wave per frame at
// inverse pass 0, profiles/r03/stamps/stamps_q8.txt).
constexpr unsigned FS_OOB = 0x80000000u;   // a buffer offset past the queue slot's range
// The first frame of every workgroup can also be static: the first pre_s = min(size, workgroups
// homed there) frames of shard s go to its home workgroups in blockIdx order (frame lo_s + blockIdx
// / 8), and the shard's tickets count from there.  The first frame's input then loads at once,
// with no device-scope atomic round trip in front of it (grid = 0: every frame from the queue).
// per: static frames per workgroup (the persistent kernel's d = 1, 2 queue takes two, its first
// and its second frame, so neither waits for an atomic).
__device__ __forceinline__ int fs_shard_nwg(int grid, int s) { return (grid - s + FS_SHARDS - 1) / FS_SHARDS; }
__device__ __forceinline__ int fs_shard_pre(int nframes, int grid, int s, int per)
{
    const int cnt = fs_shard_lo(nframes, s + 1) - fs_shard_lo(nframes, s);
    const int n = per * fs_shard_nwg(grid, s);
    return cnt < n ? cnt : n;
}
// static frame i (< per) of workgroup w: frame lo_s + i nwg_s + blockIdx / 8 of its home shard s
__device__ __forceinline__ int fs_static_frame(int nframes, int grid, int w, int i, int per)
{
    const int s = w & (FS_SHARDS - 1), e = i * fs_shard_nwg(grid, s) + w / FS_SHARDS;
    return e < fs_shard_pre(nframes, grid, s, per) ? fs_shard_lo(nframes, s) + e : -1;
}
__device__ __forceinline__ int fs_static_first(int nframes, int grid, int w) { return fs_static_frame(nframes, grid, w, 0, 1); }
// Pair tickets (kTailSingles >= 0): the first tickets of a shard stand for two consecutive frames
// each, the last ones (kTailSingles per workgroup homed there) for one.  A workgroup then dequeues about
// once per two frames (each dequeue is ~1000 cycles of the queue wave that the other waves wait
// for at the next barrier, profiles/r03/stamps), and the queue still ends in single frames, so
// the launch's tail keeps the granularity of one frame.  Shard s's dynamic frames (past its static
// prefix) are lo_s + [0, 2 np_s) in pairs (ticket t: lo_s + 2t, lo_s + 2t + 1) and lo_s + 2 np_s ..
// one per ticket (ticket t >= np_s: lo_s + np_s + t); its tickets number cnt_s - np_s.
// TS < 0: every ticket one frame.  kTailSingles: the d = 0 kernel's (FrameSchedule).
constexpr int kTailSingles = -1;
template <int TS>
__device__ __forceinline__ int fs_shard_pairs(int cnt, int grid, int s)
{
    if constexpr (TS < 0) return 0;
    const int n = TS * fs_shard_nwg(grid, s);
    return cnt > n ? (cnt - n) >> 1 : 0;
}
template <int TS>
struct FsQueue {
    __amdgpu_buffer_rsrc_t rq;   // the queue slot as a buffer (kFsQueueWords words)
    int nframes, sh0, grid, per;
    int shn;        // shard of the pending ticket (8: every shard dry)
    int lo;         // first dynamic frame of that shard
    int np, ntk;    // its pair tickets and all its tickets (ntk = 0 once every shard is dry)
    int tk;         // lane 0: the pending ticket
    int pv;         // its value, read by peek()

    __device__ __forceinline__ void init(unsigned *wq, int nframes_, int home, int grid_, int per_)
    {
        rq = __builtin_amdgcn_make_buffer_rsrc(wq, (short)0, 4 * kFsQueueWords, 0x00020000);
        nframes = nframes_;
        sh0 = home;
        grid = grid_;
        per = per_;
        set_shard(0);
    }
    // the dynamic frames of shard s (past its static prefix)
    __device__ __forceinline__ int dyn(int s, int &first) const
    {
        const int pre = fs_shard_pre(nframes, grid, s, per);
        first = fs_shard_lo(nframes, s) + pre;
        return fs_shard_lo(nframes, s + 1) - first;
    }
    __device__ __forceinline__ void set_shard(int sh)
    {
        shn = sh;
        const int s = (sh0 + sh) & (FS_SHARDS - 1);
        const int cnt = sh < FS_SHARDS ? dyn(s, lo) : 0;
        np = fs_shard_pairs<TS>(cnt, grid, s);
        ntk = cnt - np;
    }
    // takes a ticket of the current shard (lane 0; no wait).  Called by the whole wave; the
    // offset is recomputed here (a few scalar instructions and one select) rather than kept in
    // registers across the frame.
    __device__ __forceinline__ void take()
    {
        const unsigned off = shn < FS_SHARDS ? 64u * (unsigned)((sh0 + shn) & (FS_SHARDS - 1)) : FS_OOB;
        const unsigned voff = (threadIdx.x & 63) == 0 ? off : FS_OOB;
        tk = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rq, voff, 0, 0);
    }
    // reads the pending ticket (waits for its atomic): at the top of a frame, where the wait is
    // free (the atomic is older than the frame's input loads, which are needed there anyway) and
    // nothing reads the result soon (v_readfirstlane's SGPR feeding a scalar compare right away
    // stalled the queue wave ~500 cycles per frame at inverse pass 0, stamps_q15.txt)
    __device__ __forceinline__ void peek() { pv = __builtin_amdgcn_readfirstlane(tk); }
    // the frame of the peeked ticket (second: the pair's second frame, or -1), -1 when every shard
    // is dry.  A ticket past its shard's end (this happens only as the queue runs out) scans all
    // eight counters at once (lanes 0..7 add 0 to one counter each and compare it with that
    // shard's ticket count: one device-scope round trip, vector temporaries only; the same test
    // as a scalar loop over the shards spilled 6 more SGPRs at d = 2) and moves to the first
    // shard in walk order from home that still has frames, where it takes (and waits for) a new
    // ticket; with none left it returns at once.  Walking the shards one atomic at a time instead cost every
    // workgroup's last frame 7 serial round trips (~1.2 us each while the chip streams,
    // MI355X_MICROARCH.md dequeue row) on the launch's critical tail.  The counters only grow
    // (until the last workgroup has left), so a shard seen dry stays dry, and a ticket below its
    // shard's size is a frame no other ticket maps to: every frame is taken exactly once
    // (tests/test_queue_model.py restates this and drives it with random interleavings).
    __device__ __forceinline__ int resolve()
    {
        int second;
        return resolve(second);
    }
    __device__ __forceinline__ int resolve(int &second)
    {
        bool dry = pv >= ntk;
        while (__builtin_expect(dry && shn < FS_SHARDS, 0)) {
            const int l = (int)(threadIdx.x & 63);
            const unsigned voff = l < FS_SHARDS ? 64u * (unsigned)l : FS_OOB;
            const int seen = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(0, rq, voff, 0, 0);
            int first;
            const int cnt = dyn(l & (FS_SHARDS - 1), first);
            const unsigned live = (unsigned)__builtin_amdgcn_ballot_w64(
                                      l < FS_SHARDS && seen < cnt - fs_shard_pairs<TS>(cnt, grid, l)) & 0xffu;
            const unsigned rot = ((live >> sh0) | (live << (FS_SHARDS - sh0))) & 0xffu;   // bit k: shard home + k
            set_shard(rot ? __builtin_ctz(rot) : FS_SHARDS);
            if (!rot) break;
            take();
            pv = __builtin_amdgcn_readfirstlane(tk);
            dry = pv >= ntk;
        }
        if constexpr (TS < 0) {
            second = -1;
            return dry ? -1 : lo + pv;
        }
        second = !dry && pv < np ? lo + 2 * pv + 1 : -1;
        return dry ? -1 : pv < np ? lo + 2 * pv : lo + np + pv;
    }
};
// Static prefix + dynamic suffix: each workgroup first takes kstat static frames of its home
// shard (fs_static_frame, interleaved: static frame i is lo_s + i nwg_s + blockIdx / 8), with no
// atomic, and only then draws from the shard's queue (tickets count from past the static frames).
// The queue absorbs the imbalance (the SIMDs arbitrate by age, so the four workgroups of a CU run
// at different speeds) and the tail; the static prefix saves its per-frame cost (one device-scope
// atomic round trip, ~1000 cycles of the queue wave per frame, which the other waves wait for at
// the next barrier) for most frames.  kstat is chosen on the host (a fraction of the frames per
// workgroup small enough that the slowest workgroup of a CU still finishes its static frames
// before the queue runs dry).
// Worked by the queue wave only (all bookkeeping wave-uniform, scalar).  Per frame j of the
// workgroup's sequence: at the frame top, top() reads a pending ticket (taken a frame earlier);
// at inverse pass 0, next() returns frame j + 1 (static, or the pending ticket resolved) and takes
// the ticket for frame j + 2 when that one is dynamic.
// LA: lookahead, the number of frames known ahead of the current one (1: the FS kernel, which
// learns frame j + 1 at frame j's inverse pass 0; 2: the persistent kernel, which prefetches
// frame j + 1 at frame j's top and learns frame j + 2 in frame j's middle).
template <int LA, int TS = kTailSingles>
struct FrameSchedule {
    FsQueue<TS> q;
    int rem;        // static frames left past the LA known ones (<= 0: the rest is dynamic)
    int nxt, nwg;   // the next of them, and the stride between them (static frame i: slo + i nwg)
    int pend = -1;  // the second frame of the last pair ticket, not yet handed out
    static constexpr bool PAIRS = TS >= 0;

    // sets up the schedule; f[0..LA) receive the first LA frames (-1: none).  kstat: static frames
    // per workgroup
    __device__ __forceinline__ void init(unsigned *wq, int nframes, int w, int grid, int kstat, int (&f)[LA])
    {
        const int s = w & (FS_SHARDS - 1);
        nwg = fs_shard_nwg(grid, s);
        const int slo = fs_shard_lo(nframes, s) + w / FS_SHARDS;
        const int pre = fs_shard_pre(nframes, grid, s, kstat);
        const int kw = pre > w / FS_SHARDS ? (pre - w / FS_SHARDS + nwg - 1) / nwg : 0;
        q.init(wq, nframes, s, grid, kstat);
        for (int i = 0; i < LA; i++) {   // frame i: static, or from the queue at once (small batches)
            if (PAIRS && pend >= 0) {
                f[i] = pend;
                pend = -1;
            } else if (i < kw) {
                f[i] = slo + i * nwg;
            } else {
                q.take();
                q.peek();
                f[i] = q.resolve(pend);
            }
        }
        rem = kw - LA;
        nxt = slo + LA * nwg;
        if (rem <= 0 && (!PAIRS || pend < 0)) q.take();   // frame LA is dynamic and not known: its ticket now
    }
    // reads the pending ticket, if any (taken a frame earlier): call at a point where its wait
    // is free, before next()
    __device__ __forceinline__ void peek()
    {
        if (rem <= 0 && (!PAIRS || pend < 0)) q.peek();
    }
    // the frame LA after the current one, and the ticket for the one after that when it is
    // dynamic and not the second of a pair
    __device__ __forceinline__ int next()
    {
        int fn;
        if (PAIRS && pend >= 0) {
            fn = pend;
            pend = -1;
        } else if (rem > 0) {
            fn = nxt;
            nxt += nwg;
        } else {
            fn = q.resolve(pend);
        }
        rem--;
        if (rem <= 0 && (!PAIRS || pend < 0)) q.take();
        return fn;
    }
};

// Slot-weighted static split.  A full-residency launch (grid = 4 x CUs) places blockIdx quarter q
// on CU slot q (HW_ID TG_ID, all 1024 workgroups, stamps in profiles/r04/stamps), and a CU's
// SIMDs arbitrate by age, so slot q runs at a fixed fraction of slot 0's speed (d = 4: 1, 0.89,
// 0.74, 0.59 frames per us while all four are resident).  An equal contiguous split left slot 0
// done at 75 us and slot 3 at 113 us of a 124 us launch; weighted shares end them together.
// slotw: four 8-bit weights (slot 0 in the low byte), 0: equal shares.  First frame of workgroup
// v (v = G: nframes).
__device__ __forceinline__ int slot_split(int nframes, int G, int v, unsigned slotw)
{
    if (slotw == 0u || (G & 3)) return (int)(((long long)nframes * v) / G);
    const int Q = G >> 2, q = v / Q, i = v - q * Q;
    long long sw = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int wk = (int)((slotw >> (8 * k)) & 0xffu);
        tot += (long long)Q * wk;
        if (k < q) sw += (long long)Q * wk;
        else if (k == q) sw += (long long)i * wk;
    }
    return (int)(((long long)nframes * sw) / tot);
}

// static frames per workgroup for a static share of pct percent, at least lo (the schedule's
// lookahead: the frames a workgroup needs before its first ticket could have returned)
inline int frame_schedule_kstat(int nframes, int grid, int pct, int lo)
{
    const int k = (int)((long long)nframes * pct / (100LL * grid));
    return k < lo ? lo : k;
}

__device__ __forceinline__ void fs_queue_done(unsigned *wq, unsigned grid)
{
    if (atomicAdd(wq + 16 * FS_SHARDS, 1u) == grid - 1) {
        for (int s = 0; s <= FS_SHARDS; s++) atomicExch(wq + 16 * s, 0u);
    }
}

}  // namespace
}  // namespace sddc
