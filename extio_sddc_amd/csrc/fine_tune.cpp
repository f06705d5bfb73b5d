// fine_tune.cpp — host side of the fused fine-tune NCO; see fine_tune.h.
#include "fine_tune.h"

#include <cmath>

namespace sddc {
namespace {
constexpr float kPi = (float)3.14159265358979323846;   // pf_mixer.cpp:40 (float PI)

inline void wrap(float &ph)
{
    while (ph > kPi) ph -= 2 * kPi;
    while (ph < -kPi) ph += 2 * kPi;
}
}  // namespace

void FineTune::init(float relative_freq, float phase_start)
{
    const float inc = 2 * relative_freq * kPi;
    // table entry j: the phase after 4 (j + 1) increments, accumulated in float with the
    // reference's wrap after every step (pf_mixer.cpp:759-773)
    float ph = 0.0f;
    for (int j = 0; j <= kTable; j++) {
        for (int l = 0; l < kLanes; l++) {
            ph += inc;
            wrap(ph);
        }
        trig_[j] = make_float2(cosf(ph), sinf(ph));
    }
    // lane l starts at phase_start + l increments (pf_mixer.cpp:778-786)
    ph = phase_start;
    for (int l = 0; l < kLanes; l++) {
        start_[l] = make_float2(cosf(ph), sinf(ph));
        ph += inc;
        wrap(ph);
    }
}

void FineTune::starts(long nblocks, float2 *out)
{
    const float tr = trig_[kTable - 1].x, ti = trig_[kTable - 1].y;   // 128-step phasor
    float c[kLanes], s[kLanes];
    for (int l = 0; l < kLanes; l++) {
        c[l] = start_[l].x;
        s[l] = start_[l].y;
    }
    for (long b = 0; b < nblocks; b++) {
        for (int l = 0; l < kLanes; l++) {
            out[b * kLanes + l] = make_float2(c[l], s[l]);
            // vals = T[31] * starts, then starts = vals / |vals| (pf_mixer.cpp:831-850)
            const float vc = tr * c[l] - ti * s[l];
            const float vs = ti * c[l] + tr * s[l];
            const float m = sqrtf(vc * vc + vs * vs);
            c[l] = vc / m;
            s[l] = vs / m;
        }
    }
    for (int l = 0; l < kLanes; l++) start_[l] = make_float2(c[l], s[l]);
}

}  // namespace sddc
