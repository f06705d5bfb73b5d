/*
 * sddc_fft.h — batched FFTs on gfx950 at the DDC path's sizes:
 * the compute behind the HIP FFTBackend (extio_sddc_amd/csrc/fft_backend/), which
 * replaces Core/fft_backend_{fftw,mkl,accelerate}.cpp behind the FFTBackend API
 * (Core/fft_backend.h:22-50) so Core/fft_benchmark.cpp times the GPU.
 *
 * Conventions are FFTW's (fft_backend_fftw.cpp): unnormalised, forward e^{-2 pi i nk/n},
 * backward e^{+2 pi i nk/n}; r2c writes n/2+1 bins.  Complex data are interleaved
 * float (re, im).  Pointers are device pointers or host memory mapped into the GPU
 * (hipHostMalloc); transforms are contiguous, `batch` of them back to back.
 */
#ifndef SDDC_FFT_H
#define SDDC_FFT_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDDC_FFT_FORWARD (-1)
#define SDDC_FFT_BACKWARD (+1)

/* 1 if a transform of this kind and size is supported: c2c n = 64..4096,
 * r2c n = 128..8192, powers of two (the sizes fft_mt_r2iq plans, fft_mt_r2iq.cpp:221-225,
 * and fft_benchmark.cpp:12's table). kind: 0 = c2c, 1 = r2c. */
int sddc_fft_supported(int kind, int n);

/* batch x n-point complex FFTs, in -> out (may alias: in place is allowed).
 * Enqueued on hip_stream (NULL = default); returns after launch.  0 = OK, else an
 * SDDC_ERR_* code (sddc_ddc.h) with sddc_ddc_last_error() set. */
int sddc_fft_c2c(const void *in, void *out, int n, int batch, int direction, void *hip_stream);

/* batch x n-point real-to-complex FFTs: in = batch*n floats, out = batch*(n/2+1)
 * complex.  Not in place. */
int sddc_fft_r2c(const float *in, void *out, int n, int batch, void *hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* SDDC_FFT_H */
