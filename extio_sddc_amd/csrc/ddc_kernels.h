// ddc_kernels.h — internal (C++) interface between the runtime and the HIP kernels.
#pragma once

#include <hip/hip_runtime_api.h>
#include <hip/hip_vector_types.h>
#include <stddef.h>
#include <stdint.h>

namespace sddc {

// Device-resident constant tables, built once per handle (fft_mt_r2iq::Init).
struct KernelTables {
    const float2 *tw4096 = nullptr;    // e^{-2 pi i k/4096}, k < 4096 (FFT twiddles)
    const float2 *post8192 = nullptr;  // e^{-2 pi i k/8192}, k < 4096 (r2c split twiddles)
    const float2 *hsel[7] = {};        // per d: mfft filter taps in inverse-input order, x 1/2
};

hipError_t launch_frames(const KernelTables &t, int d, const int16_t *d_in, int nblk, float *d_out,
                         int tunebin, int lsb, int rand, hipStream_t s);

int channels_per_group(int d, int nch);

hipError_t launch_channels(const KernelTables &t, int d, const int16_t *d_in, int nblk,
                           const int *d_tunebins, int nch, float *d_out, size_t stride_floats,
                           int lsb, int rand, hipStream_t s);

}  // namespace sddc
