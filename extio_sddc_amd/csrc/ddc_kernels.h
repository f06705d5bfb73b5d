// ddc_kernels.h — internal (C++) interface between the runtime and the HIP kernels of the
// product library.  (The measured-slower A/B kernels of rounds 1-5 are in git history; DESIGN.md
// §8 keeps their numbers.)
#pragma once

#include <hip/hip_runtime_api.h>
#include <hip/hip_vector_types.h>
#include <stddef.h>
#include <stdint.h>

namespace sddc {

// Launch geometry, per handle: the device's CU count and, per kernel (function pointer), the
// resident workgroups per CU, queried on first use and kept in the handle (all launches run
// under the handle's lock), so no launch path writes namespace-scope state.
struct LaunchCache {
    static constexpr int kSlots = 256;
    int cus = 0;
    int n = 0;
    const void *fn[kSlots] = {};
    int occ[kSlots] = {};
};

// occ = resident workgroups per CU of kernel fn (`threads` per workgroup, static LDS), cus = the
// device's CUs; cached in *lc when lc is non-null.
inline hipError_t launch_geometry(LaunchCache *lc, const void *fn, int threads, int device, int *occ, int *cus)
{
    if (lc) {
        for (int i = 0; i < lc->n; i++)
            if (lc->fn[i] == fn) {
                *occ = lc->occ[i];
                *cus = lc->cus;
                return hipSuccess;
            }
    }
    int nb = 0, c = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, threads, 0);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) return e;
    *occ = nb > 0 ? nb : 1;
    *cus = c;
    if (lc && lc->n < LaunchCache::kSlots) {
        lc->cus = c;
        lc->fn[lc->n] = fn;
        lc->occ[lc->n] = *occ;
        lc->n++;
    }
    return hipSuccess;
}

// Device-resident constant tables, built once per handle (the reference's
// fft_mt_r2iq::Init builds filterHw and the FFTW plans, fft_mt_r2iq.cpp:147-227).
// All twiddles are evaluated in double on the host and rounded once to float.
struct KernelTables {
    const float2 *tw4096 = nullptr;    // e^{-2 pi i k/4096}, k < 4096 (v1 FFT twiddles)
    const float2 *post8192 = nullptr;  // e^{-2 pi i k/8192}, k < 8192 (r2c split twiddles)
    const float2 *hsel[7] = {};        // per d: mfft filter taps in inverse-input order, x 1/2
    // persistent kernel (v2) twiddle sets
    const float2 *tw_p1 = nullptr;     // [15][16]: W_256^{s r}     forward pass 1 (NS = 16)
    const float2 *tw_q1[7] = {};       // [15][S]:  W_{16S}^{s r}   inverse pass 1, S = NS of that pass
    const float2 *rec_f = nullptr;     // [2][256]: W_4096^{j}, W_4096^{4j}  forward pass 2 recurrence
    const float2 *rec_i[7] = {};       // [2][256]: W_N^{j}, W_N^{4j}        inverse pass 2 (N >= 512)
    LaunchCache *lc = nullptr;         // the handle's launch geometry (written under the handle's lock)
};

// v2 (default): persistent workgroups, input prefetch, swizzled LDS.  pq: the split x filter
// coefficients of (d, tunebin) built by launch_build_split_filter: N = HALF >> d float2 P, then N
// float r (12 N bytes of the HALF float4 allocation).
// nco_starts/nco_trig: fused fine-tune NCO tables (fine_tune.h), or nullptr for none.
// cs16: write saturate(rint(x * cs16_scale)) int16 (I, Q) pairs instead of complex float.
hipError_t launch_frames_persistent(const KernelTables &t, int d, const int16_t *d_in, int nblk,
                                    void *d_out, const float4 *pq, int tunebin, int lsb, int rand,
                                    int cs16, float cs16_scale, const float2 *nco_starts,
                                    const float2 *nco_trig, int slot_weights, int device, hipStream_t s);
// slot_weights: split the frames over the workgroups by their CU slot's measured speed
// (kSlotWeights[d]: slot 0 in the low byte; ddc_queue.hpp slot_split), 0: equal contiguous
// ranges.  The frames per slot of a balanced (queue-fed) run gave the weights: d = 1 29 / 25 /
// 19 / 15, d = 4 27 / 24 / 20 / 16, tuned at d >= 3 to 29 / 25 / 20 / 15 (+3-6 %,
// profiles/r04/ab/slot_weights_d3_6.txt; the four slots then end within 1 us of each other,
// stamps_p_d4_final_by_slot.txt) and at d <= 2 to 31 / 26 / 18 / 13 (d = 1 +4 %, d = 2 +2 %,
// slot_weights_tuning_d1_6.txt).
constexpr unsigned slot_weights4(unsigned a, unsigned b, unsigned c, unsigned e) { return a | (b << 8) | (c << 16) | (e << 24); }
constexpr unsigned kSlotWeights[7] = {slot_weights4(31, 26, 18, 13), slot_weights4(31, 26, 18, 13), slot_weights4(31, 26, 18, 13),
                                      slot_weights4(29, 25, 20, 15), slot_weights4(29, 25, 20, 15),
                                      slot_weights4(29, 25, 20, 15), slot_weights4(29, 25, 20, 15)};
constexpr int kSlotWeighting = 1;
hipError_t launch_build_split_filter(const KernelTables &t, int d, int tunebin, float4 *pq, hipStream_t s);

// d = 0 fused-split kernel (ddc_fs.hip, FS): used when fs_path(d, tunebin) (d = 0, tunebin a
// multiple of 4: every tune bin setFreqOffset produces, fft_mt_r2iq.cpp:104).  Its per-tunebin
// tables: pqf (4096 float4, the split x filter by bin in lane order) and fsl (3 x 256 float2, the
// output modulation's lane factors), built by launch_build_fs_tables.
bool fs_path(int d, int tunebin);
hipError_t launch_build_fs_tables(const KernelTables &t, int tunebin, float4 *pqf, float2 *fsl, hipStream_t s);
// wq: a zeroed slot of kFsQueueWords unsigned words (the dynamic frame queue); the launch leaves it
// zeroed again.  Launches that may run at the same time need different slots.
// static_pct: the share (percent) of each workgroup's frames taken statically before it draws
// from the queue (ddc_queue.hpp FrameSchedule); kFsStaticPct by default.
constexpr int kFsQueueLineWords = 16 * 9;                  // the dynamic queue's counters
constexpr int kFsStealMax = 2048;                         // steal slots (2 words): workgroups per launch
constexpr int kFsQueueWords = kFsQueueLineWords + 2 * kFsStealMax;
constexpr int kFsStaticPct = 100;   // (85 / 95 / 100 %: 0.240 / 0.238 / 0.235 ms, profiles/r04/ab/fs_static_share_d0.txt)
constexpr unsigned kFsSlotWeights = slot_weights4(31, 26, 18, 13);   // (between the boxes' optima, fs_slot_weights_d0.txt)
// The FS kernel's frame schedule (ddc_queue.hpp): sched 0 the slot-weighted static split alone
// (default; every output configuration), 2 work stealing, 1 the static prefix of static_pct
// percent + the dynamic queue (1 and 2: the plain configuration only, A/B and tests).  fpw > 0: a
// non-persistent grid of fpw frames per workgroup (A/B).  minrem: a thief steals only from ranges
// with at least minrem unclaimed frames (0: none, the static split inside the stealing kernel).
struct FsSched {
    int sched = 0;
    int static_pct = kFsStaticPct;
    int fpw = 0;
    int minrem = 1;
    int pub = 0;   // frames at the end of each range open to thieves (0: all but the first two)
    int zr = 1;    // skip the tune bin's whole zero rows of the inverse input (0: never; A/B)
    unsigned slotw = 0u;   // the static split's slot weights (slot_weights4 packing); 0: kFsSlotWeights
};
hipError_t launch_frames_fs(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pqf,
                            const float2 *fsl, int tunebin, int lsb, int rand, int cs16, float cs16_scale,
                            const float2 *nco_starts, const float2 *nco_trig, unsigned *wq, const FsSched &fs,
                            int device, hipStream_t s);

// many-channel v2 (d = 4..6): persistent, forward once per (frame, 128-channel chunk)
// stride: scalar components (float or int16) per channel row; cs16 as above.  d_windows:
// per-128-channel-chunk forward-bin windows from channel_windows (device copy), or nullptr.
// d_scratch: scratch_rows x 4096 float2, one row per workgroup, where a frame's split spectrum
// is kept for its later chunks (used when the grid fits; nullptr = recompute per chunk).
hipError_t launch_channels_v2(const KernelTables &t, int d, const int16_t *d_in, int nblk, const int *d_tunebins,
                              int nch, void *d_out, size_t stride, int lsb, int rand, int cs16, float cs16_scale,
                              const int2 *d_windows, float2 *d_scratch, int scratch_rows, int device,
                              hipStream_t s);
// many-channel, d = 0..3: persistent, forward + split once per frame, 2^d channels' inverses
// in flight.  d_scratch (scratch_rows x 4096 float2, >= CUs x 4 rows) holds each workgroup's
// split spectrum in L2 instead of LDS; nullptr keeps it in LDS.
hipError_t launch_channels_p(const KernelTables &t, int d, const int16_t *d_in, int nblk, const int *d_tunebins,
                             int nch, void *d_out, size_t stride, int lsb, int rand, int cs16, float cs16_scale,
                             float2 *d_scratch, int scratch_rows, int device, hipStream_t s);
// host: the compact windows of every chunk; false if a chunk's window does not fit
bool channel_windows(int d, const int *tunebins, int nch, int2 *windows);

// batched FFTs (fft_batch.hip, include/sddc_fft.h); fft_prepare fills the device's twiddle
// table once (synchronises s the first time)
hipError_t fft_prepare(hipStream_t s);
hipError_t fft_c2c(const void *in, void *out, int n, int batch, int dir, hipStream_t s);
hipError_t fft_r2c(const float *in, void *out, int n, int batch, hipStream_t s);

}  // namespace sddc
