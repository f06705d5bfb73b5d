// ddc_queue.hpp — frame distribution for the single-channel frame kernels (ddc_fs.hip,
// ddc_persistent.hip): a slot-weighted static split of the first frames, then a dynamic queue.
#pragma once

#include <hip/hip_runtime.h>

namespace sddc {
namespace {

// Why not a plain static split.  A full-residency launch (grid = 4 x CUs) places blockIdx quarter
// q on CU slot q (HW_ID TG_ID, all 1024 workgroups; profiles/r04/stamps/*by_slot*), and a CU's
// SIMDs arbitrate by age, so slot q runs at a fixed fraction of slot 0's speed (d = 4: 1, 0.89,
// 0.74, 0.59 frames per us while all four are resident).  An equal contiguous split left slot 0
// done at 75 us and slot 3 at 113 us of a 124 us launch (stamps_p_d4_static_by_slot.txt).
//
// The schedule: frames [0, ns) are split statically, workgroup w taking the contiguous range
// [slot_split(ns, G, w), slot_split(ns, G, w + 1)), with shares weighted by its slot's measured
// speed (slotw; equal shares when slotw = 0 or the launch is not at full residency).  Frames
// [ns, nframes) are handed out one at a time by a dynamic queue, which absorbs what the weights do
// not predict and ends the launch frame-granular (the FS kernel, d = 0).  The persistent kernel
// (d >= 1) uses the weighted split alone: there the queue's per-frame cost was larger than the
// imbalance it removed (ddc_persistent.hip).
//
// The queue: 8 shards of consecutive frames (one counter each, on its own 64-B line); a workgroup
// starts on shard blockIdx % 8 (its XCD under round-robin placement: neighbouring frames, which
// share 2048 input samples, stay in one L2) and moves on when it runs dry.  The queue wave reads a
// ticket at the top of the frame after the one it was taken in (before that frame's prefetch:
// vmcnt counts in issue order, so the read then waits only for loads that have landed), resolves
// it where the kernel learns its next frame, and takes the next ticket once the frame's last
// loads have been consumed (profiles/r03/stamps, profiles/r04/stamps).
// wq: this launch's slot of the handle's queue ring, zero at entry; the last workgroup to leave
// clears it for the slot's next launch (the counters are touched only by device-scope atomics).
constexpr int FS_SHARDS = 8;
static_assert(kFsQueueWords == 16 * (FS_SHARDS + 1), "queue slot: one 64-B line per shard counter + the done count");
constexpr unsigned FS_OOB = 0x80000000u;   // a buffer offset past the queue slot's range

// first frame of workgroup v (v = G: ns) of the slot-weighted static split of ns frames.
// slotw: four 8-bit weights (slot 0 in the low byte), 0: equal shares.
__device__ __forceinline__ int slot_split(int ns, int G, int v, unsigned slotw)
{
    if (slotw == 0u || (G & 3)) return (int)(((long long)ns * v) / G);
    const int Q = G >> 2, q = v / Q, i = v - q * Q;
    long long sw = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int wk = (int)((slotw >> (8 * k)) & 0xffu);
        tot += (long long)Q * wk;
        if (k < q) sw += (long long)Q * wk;
        else if (k == q) sw += (long long)i * wk;
    }
    return (int)(((long long)ns * sw) / tot);
}

// The queue is worked by one wave (wave-uniform, so the bookkeeping is scalar); only the atomic
// increment is its lane 0's.  The whole wave issues the ticket's atomic as a buffer atomic whose
// lanes other than 0 fall outside the buffer's range (dropped, no memory access): issued from a
// lane-0 branch instead, the ticket register became a merge of two values and the merge copy
// waited for the atomic's return right there (profiles/r03/stamps/stamps_q8.txt).
struct FsQueue {
    __amdgpu_buffer_rsrc_t rq;   // the queue slot as a buffer (kFsQueueWords words)
    int base, nd;   // the dynamic frames [base, base + nd)
    int sh0;        // home shard
    int shn;        // shard of the pending ticket, relative to home (8: every shard dry)
    int lo, cnt;    // first frame and size of that shard (cnt = 0 once every shard is dry)
    int tk;         // lane 0: the pending ticket
    int pv;         // its value, read by peek()

    // first frame of dynamic shard s (32-bit: nd * 8 < 2^31 for any batch the C ABI accepts)
    __device__ __forceinline__ int shard_lo(int s) const { return base + ((nd * s) >> 3); }
    __device__ __forceinline__ void init(unsigned *wq, int base_, int nd_, int home)
    {
        rq = __builtin_amdgcn_make_buffer_rsrc(wq, (short)0, 4 * kFsQueueWords, 0x00020000);
        base = base_;
        nd = nd_;
        sh0 = home;
        set_shard(0);
    }
    __device__ __forceinline__ void set_shard(int sh)
    {
        shn = sh;
        const int s = (sh0 + sh) & (FS_SHARDS - 1);
        lo = shard_lo(s);
        cnt = sh < FS_SHARDS ? shard_lo(s + 1) - lo : 0;
    }
    // takes a ticket of the current shard (lane 0; no wait).  Called by the whole wave.
    __device__ __forceinline__ void take()
    {
        const unsigned off = shn < FS_SHARDS ? 64u * (unsigned)((sh0 + shn) & (FS_SHARDS - 1)) : FS_OOB;
        const unsigned voff = (threadIdx.x & 63) == 0 ? off : FS_OOB;
        tk = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, rq, voff, 0, 0);
    }
    // reads the pending ticket (waits for its atomic): at a point where the wait is free
    __device__ __forceinline__ void peek() { pv = __builtin_amdgcn_readfirstlane(tk); }
    // the frame of the peeked ticket, -1 when every shard is dry.  A ticket past its shard's end
    // (this happens only as the queue runs out) scans all eight counters at once (lanes 0..7 add
    // 0 to one counter each and compare it with that shard's size: one device-scope round trip,
    // vector temporaries only; the same test as a scalar loop over the shards spilled 6 more SGPRs
    // at d = 2) and moves to the first shard in walk order from home that still has frames, where
    // it takes (and waits for) a new ticket; with none left it returns at once.  Walking the
    // shards one atomic at a time instead cost every workgroup's last frame 7 serial round trips
    // (~1.2 us each while the chip streams, MI355X_MICROARCH.md dequeue row) on the launch's
    // critical tail.  The counters only grow (until the last workgroup has left), so a shard seen
    // dry stays dry, and a ticket below its shard's size is a frame no other ticket maps to: every
    // frame is taken exactly once (tests/test_queue_model.py restates this and drives it with
    // random interleavings).
    __device__ __forceinline__ int resolve()
    {
        bool dry = pv >= cnt;
        while (__builtin_expect(dry && shn < FS_SHARDS, 0)) {
            const int l = (int)(threadIdx.x & 63);
            const unsigned voff = l < FS_SHARDS ? 64u * (unsigned)l : FS_OOB;
            const int seen = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(0, rq, voff, 0, 0);
            const int ls = l & (FS_SHARDS - 1);
            const unsigned live = (unsigned)__builtin_amdgcn_ballot_w64(
                                      l < FS_SHARDS && seen < shard_lo(ls + 1) - shard_lo(ls)) & 0xffu;
            const unsigned rot = ((live >> sh0) | (live << (FS_SHARDS - sh0))) & 0xffu;   // bit k: shard home + k
            set_shard(rot ? __builtin_ctz(rot) : FS_SHARDS);
            if (!rot) break;
            take();
            pv = __builtin_amdgcn_readfirstlane(tk);
            dry = pv >= cnt;
        }
        return dry ? -1 : lo + pv;
    }
};

// A workgroup's frame sequence: its static range, then the queue.  Worked by the queue wave only
// (all bookkeeping wave-uniform, scalar).  LA: lookahead, the number of frames known ahead of the
// current one (1: the FS kernel, which learns frame j + 1 at frame j's inverse pass 0; 2: the
// persistent kernel's form, which prefetches frame j + 1 at frame j's top and learns frame j + 2
// in frame j's middle; measured and retired there, kept in tests/test_queue_model.py).
template <int LA>
struct FrameSchedule {
    FsQueue q;
    int rem;   // static frames left past the LA known ones (<= 0: the rest is dynamic)
    int nxt;   // the next of them

    // sets up the schedule; f[0..LA) receive the first LA frames (-1: none).  ns: the statically
    // split frames, slotw: the split's slot weights (slot_split)
    __device__ __forceinline__ void init(unsigned *wq, int nframes, int ns, int w, int G, unsigned slotw,
                                         int (&f)[LA])
    {
        const int a = slot_split(ns, G, w, slotw), b = slot_split(ns, G, w + 1, slotw);
        q.init(wq, ns, nframes - ns, w & (FS_SHARDS - 1));
        for (int i = 0; i < LA; i++) {   // frame i: static, or from the queue at once
            if (a + i < b) {
                f[i] = a + i;
            } else {
                q.take();
                q.peek();
                f[i] = q.resolve();
            }
        }
        rem = b - a - LA;
        nxt = a + LA;
        if (rem <= 0) q.take();   // frame LA is dynamic: its ticket now
    }
    // reads the pending ticket, if any (taken a frame earlier): call at a point where its wait
    // is free, before next()
    __device__ __forceinline__ void peek()
    {
        if (rem <= 0) q.peek();
    }
    // the frame LA after the current one
    __device__ __forceinline__ int next()
    {
        const int fn = rem > 0 ? nxt++ : q.resolve();
        rem--;
        return fn;
    }
    // the ticket for the frame after that one, when it is dynamic: call once the frame's last
    // loads have been issued and consumed (after next())
    __device__ __forceinline__ void take()
    {
        if (rem <= 0) q.take();
    }
};

// frames statically split for a static share of pct percent
inline int frame_schedule_static(int nframes, int pct) { return (int)((long long)nframes * pct / 100); }

__device__ __forceinline__ void fs_queue_done(unsigned *wq, unsigned grid)
{
    if (atomicAdd(wq + 16 * FS_SHARDS, 1u) == grid - 1) {
        for (int s = 0; s <= FS_SHARDS; s++) atomicExch(wq + 16 * s, 0u);
    }
}

}  // namespace
}  // namespace sddc
