// ddc_queue.hpp — frame distribution for the single-channel frame kernels (ddc_fs.hip,
// ddc_persistent.hip): a slot-weighted static split of the first frames, then a dynamic queue.
#pragma once

#include <hip/hip_runtime.h>

#include "ddc_device_io.hpp"

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
static_assert(kFsQueueLineWords == 16 * (FS_SHARDS + 1), "queue slot: one 64-B line per shard counter + the done count");
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
        rq = __builtin_amdgcn_make_buffer_rsrc(wq, (short)0, 4 * kFsQueueLineWords, 0x00020000);
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

// The static schedule: the slot-weighted split alone (no atomics).  Same interface as
// FrameSchedule<1> and StealSchedule (init / peek / next / take), worked by the queue wave.
struct StaticSchedule {
    int nxt, end;
    __device__ __forceinline__ void init(unsigned *, int, int ns, int w, int G, unsigned slotw, int (&f)[1])
    {
        const int a = slot_split(ns, G, w, slotw), b = slot_split(ns, G, w + 1, slotw);
        f[0] = a < b ? a : -1;
        nxt = a + 1;
        end = b;
    }
    __device__ __forceinline__ void peek() {}
    __device__ __forceinline__ int next() { return nxt < end ? nxt++ : -1; }
    __device__ __forceinline__ void take() {}
};

// Work stealing (the FS kernel's default schedule, round 5).  Each workgroup owns the range
// [a, b) of the slot-weighted split and claims its frames in order; a workgroup whose range is
// exhausted steals single frames from the END of other ranges.  Per workgroup one 8-byte slot in
// the launch's queue slot: the word (front << 16) | (kStealBias + end), front / end relative to a,
// and a itself.
//   owner claim:  old = atomic_add(word, 0x10000)  -> frame a + old.front   if old.front < old.end
//   steal:        old = atomic_add(word, -1)       -> frame a + old.end - 1 if old.end - 1 >= old.front
// Both are agent-scope atomics on one word, so every frame of a range is claimed exactly once
// (an owner claim of x needs end > x, a steal of x leaves end = x; a steal of x needs front <= x,
// an owner claim of x leaves front = x + 1; tests/test_queue_model.py drives this with random
// interleavings).  A failed steal only lowers end further, which no claim can pass again; the bias
// keeps end from borrowing into front (at most kStealBias failed steals per word).
// Pipelining (the queue wave, like FrameSchedule): the claim that decides frame j + 2 is issued at
// frame j's inverse pass 1 (take) and read at frame j + 1's I0 (next).  A thief issues its
// candidate scan at frame j's end instead (take_late: one 8-byte sc1 load per lane, 64 slots
// spread over XCDs and CU slots), picks the candidate with the most unclaimed frames after frame
// j + 1's forward pass 1 (peek) and issues the steal there; a scan that finds nothing worth
// stealing ends the workgroup.  (Issued at inverse pass 1 and read at the frame top, the scan's
// two lane values spilled.)  Only a
// failed steal (the victim drained meanwhile) waits in next(): up to three synchronous rescans.
// The slots need no reset between launches: each owner swaps its slot in (one 8-byte atomic) at
// the start, the swap claiming its first two frames, and a stale slot (the previous launch's, or
// zero) reads as no frames left.
constexpr unsigned kStealBias = 0x4000u;
constexpr int kStealMaxRange = 0x3fff;   // frames per range a word can count (the host checks)
static_assert(kFsQueueWords >= kFsQueueLineWords + 2 * kFsStealMax, "queue slot: queue lines + steal slots");
constexpr unsigned STEAL_OOB = 0x80000000u;

__device__ __forceinline__ int steal_front(unsigned x) { return (int)(x >> 16); }
__device__ __forceinline__ int steal_end(unsigned x) { return (int)(x & 0xffffu) - (int)kStealBias; }

struct StealSchedule {
    enum { kOwn, kScan, kSteal, kDone, kPriv, kStatic };
    __amdgpu_buffer_rsrc_t rs;   // the launch's steal slots, [G] x {word, a}
    int a;          // own range start (absolute frame)
    int nx, pe;     // the next private frame and the private prefix's end (absolute)
    int own_left;   // public own frames not yet claimed, as the last claim saw them; -1: stealing
    int mode;       // what is pending
    int tk;         // lane 0: the pending atomic's result; every lane: its candidate's word
    int ta;         // every lane: its candidate's range start (scan)
    int va;         // the pending steal's victim range start
    int lim;        // frames of the launch (no claim returns a frame past it)
    int minrem;     // steal only from ranges with at least this many unclaimed frames
    int self;       // this workgroup's range (and steal slot) index: blockIdx.x, or the XCD-mapped
                    // index of a non-persistent grid (ddc_fs.hip xmap); every slot access uses it

    // this lane's scan candidate of probe k (byte offset of its slot): 64 slots spread over the
    // range indices (persistent grids: XCDs = index % 8, CU slots = index / (G / 4)); stride S odd
    // and > G / 64 for G >= 128, so the 64 are distinct and not self; lanes past G - 1 candidates
    // are out of the buffer (dropped)
    __device__ __forceinline__ unsigned cand_off(int k) const
    {
        const int G = (int)gridDim.x, w = self;
        const int l = (int)(threadIdx.x & 63);
        if (l >= G - 1) return STEAL_OOB;
        const int S = G >= 128 ? (G >> 6) + 1 : 1;
        int v = w + 1 + (k & 1) + S * l;   // < 3 G
        v = v >= G ? v - G : v;
        v = v >= G ? v - G : v;
        return 8u * (unsigned)v;
    }
    __device__ __forceinline__ void claim_own()
    {
        const unsigned voff = (threadIdx.x & 63) == 0 ? 8u * (unsigned)self : STEAL_OOB;
        tk = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(0x10000, rs, voff, 0, 0);
        mode = kOwn;
    }
    __device__ __forceinline__ void scan(int k)
    {
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, cand_off(k), 0, 16);   // sc1: the atomics' values
        tk = (int)v.x;
        ta = (int)v.y;
        mode = kScan;
    }
    // from the scan in tk / ta: the candidate with the most unclaimed frames; issues the steal
    // (mode kSteal) or, with none at minrem or more, ends (kDone)
    __device__ __forceinline__ void choose(int k)
    {
        const unsigned off = cand_off(k);
        const int rem = off != STEAL_OOB ? steal_end((unsigned)tk) - steal_front((unsigned)tk) : -0x7fff;
        int m = rem;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
        m = __builtin_amdgcn_readfirstlane(m);
        if (m < minrem) {
            mode = kDone;
            return;
        }
        const int lane = __builtin_ctzll(__builtin_amdgcn_ballot_w64(rem == m));
        const unsigned voff = __builtin_amdgcn_readlane((int)off, lane);
        va = __builtin_amdgcn_readlane(ta, lane);
        tk = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(-1, rs, (threadIdx.x & 63) == 0 ? voff : STEAL_OOB, 0, 0);
        mode = kSteal;
    }
    // the frame the steal in tk claimed, or -1
    __device__ __forceinline__ int stolen() const
    {
        const unsigned old = (unsigned)__builtin_amdgcn_readfirstlane(tk);
        const int fr = steal_front(old), er = steal_end(old), f = va + er - 1;
        return er - 1 >= fr && f < lim ? f : -1;
    }

    // pub: frames at the end of each range that thieves may take (0: all but the first two);
    // the owner takes the rest (its private prefix) without atomics.  minrem <= 0: the static
    // split alone (no atomics at all).
    __device__ __forceinline__ void init(unsigned *wq, int nframes, int ns, int w, int G, unsigned slotw, int (&f)[1],
                                         int minrem_, int pub)
    {
        unsigned *slots = wq + kFsQueueLineWords;
        rs = __builtin_amdgcn_make_buffer_rsrc(slots, (short)0, 8 * G, 0x00020000);
        lim = nframes;
        minrem = minrem_;
        self = w;
        a = slot_split(ns, G, w, slotw);
        const int len = slot_split(ns, G, w + 1, slotw) - a;
        f[0] = len > 0 ? a : -1;
        nx = a + 1;
        if (minrem <= 0) {
            pe = a + len;
            mode = kStatic;
            return;
        }
        // the private prefix: at least the first two frames, so that the first atomic claim is
        // issued a frame after the swap (same lane, same word: in order anyway)
        const int two = len < 2 ? len : 2;
        const int P = pub > 0 && len - pub > two ? len - pub : two;
        pe = a + P;
        own_left = len - P;
        mode = kPriv;
        if ((threadIdx.x & 63) == 0) {
            const unsigned long long v = ((unsigned long long)(unsigned)a << 32) |
                                         (((unsigned)P << 16) | (kStealBias + (unsigned)len));
            (void)atomicExch(reinterpret_cast<unsigned long long *>(slots) + w, v);
        }
        if (len <= 0) mode = kDone;   // nothing of its own (a tiny batch)
    }
    // phase B of the frame loop (ddc_fs.hip) starts at frame f, the private frames before it done
    // without this object: the state of the end of frame f - 1, and its scan (a one- or two-frame
    // range steals from its first frame on)
    __device__ __forceinline__ void enter(int f)
    {
        if (f < 0) return;
        nx = f + 1;
        take_late();
    }
    __device__ __forceinline__ void peek()
    {
        if (mode == kScan) choose(0);
    }
    __device__ __forceinline__ int next()
    {
        if (nx < pe) return nx++;
        if (mode == kDone || mode == kStatic) return -1;
        if (mode == kOwn) {
            const unsigned old = (unsigned)__builtin_amdgcn_readfirstlane(tk);
            const int fr = steal_front(old), er = steal_end(old);
            if (fr < er && a + fr < lim) {
                own_left = er - fr - 1;
                return a + fr;
            }
        } else if (mode == kSteal) {
            const int f = stolen();
            if (f >= 0) return f;
        }
        // the own claim or the steal failed: steal with waits, up to three probes
        own_left = -1;
        for (int k = 1; k <= 3; k++) {
            scan(k);
            choose(k);
            if (mode == kDone) return -1;
            const int f = stolen();
            if (f >= 0) return f;
        }
        mode = kDone;
        return -1;
    }
    // at inverse pass 1: the own claim for the frame after the next one, past the private prefix
    __device__ __forceinline__ void take()
    {
        if (mode != kDone && mode != kStatic && nx >= pe && own_left > 0) claim_own();
    }
    // at the frame's end (the IQ stores issued): a thief's scan, read at the next frame's peek
    __device__ __forceinline__ void take_late()
    {
        if (mode != kDone && mode != kStatic && nx >= pe && own_left <= 0) scan(0), own_left = -1;
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
