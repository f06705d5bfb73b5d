// variants_api.h — the A/B kernel variants library (libsddc_ddc_variants.so): the layouts of
// the single-channel kernel and the first-generation kernels that were measured slower than
// the product's defaults and stay buildable and parity-tested for
// A/B timing.  The product library loads this one only when a handle selects a variant
// (sddc_ddc_internal_set_variant), through the function table below.
#pragma once

#include "ddc_kernels.h"

namespace sddc {

// v1 (internal variant 1): one workgroup per frame, global twiddle tables (ddc_v1.hip)
hipError_t launch_frames(const KernelTables &t, int d, const int16_t *d_in, int nblk, float *d_out,
                         int tunebin, int lsb, int rand, hipStream_t s);
hipError_t launch_channels(const KernelTables &t, int d, const int16_t *d_in, int nblk,
                           const int *d_tunebins, int nch, void *d_out, size_t stride,
                           int lsb, int rand, int cs16, float cs16_scale, hipStream_t s);
int channels_per_group(int d, int nch);

// d = 0, two frames in flight per workgroup (variant 4) and radix 8 x 512 threads (variant 5);
// the arguments and tables of launch_frames_persistent (ddc_variants.hip)
hipError_t launch_frames_pipelined(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out,
                                   const float4 *pq, int tunebin, int lsb, int rand, int cs16, float cs16_scale,
                                   const float2 *nco_starts, const float2 *nco_trig, int device, hipStream_t s);
hipError_t launch_frames_r8(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                            int tunebin, int lsb, int rand, int cs16, float cs16_scale, const float2 *nco_starts,
                            const float2 *nco_trig, int device, hipStream_t s);

// d = 0, lane pairs: 512 threads per frame, 8 points per lane (variant 6, ddc_pair.hip); the
// arguments and tables of launch_frames_persistent
hipError_t launch_frames_pair(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                              int tunebin, int lsb, int rand, int cs16, float cs16_scale, const float2 *nco_starts,
                              const float2 *nco_trig, int device, hipStream_t s);

// d = 0, in-place LDS passes, 7 barriers per frame (variant 7, ddc_inplace.hip)
hipError_t launch_frames_inplace(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out, const float4 *pq,
                                 int tunebin, int lsb, int rand, int cs16, float cs16_scale, const float2 *nco_starts,
                                 const float2 *nco_trig, int device, hipStream_t s);

// d = 0, one wave64 per frame, 64 points per lane (variant 3, ddc_wave.hip).  pqW (4096
// float4) and twI (4096 float2) are its per-tunebin tables, built by launch_build_wave_tables.
hipError_t launch_build_wave_tables(const KernelTables &t, int tunebin, float4 *pqW, float2 *twI, hipStream_t s);
hipError_t launch_frames_wave(const KernelTables &t, const int16_t *d_in, int nblk, void *d_out,
                              const float4 *pqW, const float2 *twI, int tunebin, int lsb, int rand, int cs16,
                              float cs16_scale, const float2 *nco_starts, const float2 *nco_trig, int device,
                              hipStream_t s);

}  // namespace sddc

#define SDDC_VARIANTS_API_VERSION 3

extern "C" {
struct sddc_variants_api {
    int version;   // SDDC_VARIANTS_API_VERSION
    decltype(&sddc::launch_frames) frames_v1;
    decltype(&sddc::launch_channels) channels_v1;
    decltype(&sddc::launch_frames_pipelined) frames_pipelined;
    decltype(&sddc::launch_frames_r8) frames_r8;
    decltype(&sddc::launch_build_wave_tables) build_wave_tables;
    decltype(&sddc::launch_frames_wave) frames_wave;
    decltype(&sddc::launch_frames_pair) frames_pair;
    decltype(&sddc::launch_frames_inplace) frames_inplace;
};
// the table (exported by libsddc_ddc_variants.so, looked up with dlsym)
const sddc_variants_api *sddc_variants_get(void);
}
