// fine_tune.h — the fine-tune NCO that follows the DDC.
//
// The reference mixes every 32768-sample output buffer with pf_mixer's ALGO H
// (shift_limited_unroll_C_sse_{init,inp_c}, Core/pffft/pf_mixer.cpp:750-856) when the
// residual offset fc != 0 (Core/RadioHandler.cpp:33-37, re-initialised with phase 0 on
// every fc change, :291-296).  Its phasor for output sample 128 b + 4 q + l is
//     P = S_b[l]                 (q = 0)
//     P = T[q - 1] * S_b[l]      (q = 1..31, float mul/mul/sub, mul/mul/add)
// with T the 4(j+1)-step table and S_b the four lane starts of block b, renormalised
// after every block.  S_b depends only on (fc, phase0, b), not on the data, so the host
// runs that sequential float chain (this class) and the GPU applies P in the DDC kernel's
// output stage.  All arithmetic is plain float in the reference's order: this file is
// compiled with -ffp-contract=off.
#pragma once

#include <hip/hip_vector_types.h>

namespace sddc {

class FineTune {
public:
    static constexpr int kLanes = 4;      // PF_SHIFT_LIMITED_SIMD_SZ, pf_mixer.h:134
    static constexpr int kBlock = 128;    // PF_SHIFT_LIMITED_UNROLL_SIZE, pf_mixer.h:133
    static constexpr int kTable = kBlock / kLanes;   // 32 table entries used per block

    // shift_limited_unroll_C_sse_init(relative_freq, phase_start), pf_mixer.cpp:750-789
    void init(float relative_freq, float phase_start);
    // Lane starts of the next nblocks blocks of 128 samples, [nblocks][4] (cos, sin); the
    // state advances past them exactly as _inp_c does over full blocks (pf_mixer.cpp:800-851).
    void starts(long nblocks, float2 *out);
    const float2 *table() const { return trig_; }   // T[0..31]: (cos, sin) of 4 (j+1) steps

private:
    float2 trig_[kTable + 1] = {};
    float2 start_[kLanes] = {};
};

}  // namespace sddc
