// ddc_stamps.hpp — diagnostic s_memtime segment stamps for the single-channel frame kernels
// (tools/fs_stamps.py).  Only a build with -DSDDC_STAMPS=1|2|3 contains them (never the
// product, whose macros below expand to a plain __syncthreads()).
//
// Per wave, the cycles (s_memtime) of each work segment between two barriers and of each
// barrier wait are summed over the workgroup's frames in SGPRs and written once at the end by
// lane 0 (vector stores) to a stamp buffer of their own: [workgroup][wave][kStampWords].  A
// stamp sits right before and right after an s_barrier, where the barrier's own lgkmcnt(0) drain
// already is.  SDDC_STAMPS = 1 stamps barriers 0..3, = 2 barriers 4..7, = 3 barriers 8..11 (all
// of them in one build spill: the accumulators live in SGPRs); the time of an unstamped barrier
// falls into the next work segment.  SYNC indices above a kernel's barrier count are unused.
#pragma once

#include <hip/hip_runtime.h>

namespace sddc {

constexpr int kStampSegs = 13;   // work segments: up to 12 barriers + the frame tail
// work[13], wait[13] (wait[12] unused), frames, ticks, realtime ticks, build, realtime start, end, HW_ID
constexpr int kStampWords = 2 * kStampSegs + 7;

#ifdef SDDC_STAMPS
constexpr int kStLo = 4 * (SDDC_STAMPS - 1);
#define ST_INIT()                                                                                    \
    unsigned st_work[kStampSegs] = {}, st_wait[kStampSegs] = {}, st_frames = 0;                    \
    unsigned long long st_t = __builtin_amdgcn_s_memtime(), st_a = st_t;                          \
    const unsigned long long st_t0 = st_t, st_r0 = __builtin_amdgcn_s_memrealtime()
#define ST_SYNC(i)                                                                                   \
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
#define ST_FRAME_END()                                                                               \
    do {                                                                                             \
        st_a = __builtin_amdgcn_s_memtime();                                                         \
        st_work[kStampSegs - 1] += (unsigned)(st_a - st_t);                                          \
        st_t = st_a;                                                                                 \
        st_frames++;                                                                                 \
    } while (0)
#define ST_WRITE(buf, wg, tid)                                                                       \
    do {                                                                                             \
        const unsigned long long st_r1 = __builtin_amdgcn_s_memrealtime();                          \
        if (((tid) & 63) == 0 && (tid) < 256) {   /* waves 0..3 (a fifth wave is not recorded) */   \
            unsigned *o = (buf) + ((size_t)(wg) * 4 + ((tid) >> 6)) * kStampWords;                   \
            for (int i = 0; i < kStampSegs; i++) {                                                   \
                o[i] = st_work[i];                                                                   \
                o[kStampSegs + i] = st_wait[i];                                                      \
            }                                                                                        \
            o[2 * kStampSegs] = st_frames;                                                           \
            o[2 * kStampSegs + 1] = (unsigned)(st_t - st_t0);                                        \
            o[2 * kStampSegs + 2] = (unsigned)(st_r1 - st_r0);                                       \
            o[2 * kStampSegs + 3] = (unsigned)SDDC_STAMPS;                                           \
            o[2 * kStampSegs + 4] = (unsigned)st_r0;                                                 \
            o[2 * kStampSegs + 5] = (unsigned)st_r1;                                                 \
            o[2 * kStampSegs + 6] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));          \
        }                                                                                            \
    } while (0)
#else
#define ST_INIT() (void)0
#define ST_SYNC(i) __syncthreads()
#define ST_FRAME_END() (void)0
#define ST_WRITE(buf, wg, tid) (void)0
#endif

}  // namespace sddc
