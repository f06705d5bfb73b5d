/*
 * sddc_compat/fft_backend.h — standalone stand-in for ExtIO_sddc's FFT backend interface
 * (Core/fft_backend.h:1-59), used ONLY when this repository is built without the
 * ExtIO_sddc tree (tests, the GPU box).  In the integration build the reference's own
 * header is found first and this file is never seen.
 *
 * Restates the same interface: the abstract class FFTBackend with the same virtual
 * functions in the same declaration order (so the Itanium vtable layout matches), the
 * FFTPlanHandle / FFTDirection / fft_complex types and the getFFTBackend() factory.
 */
#ifndef SDDC_COMPAT_FFT_BACKEND_H
#define SDDC_COMPAT_FFT_BACKEND_H
#pragma once

#include <complex>
#include <cstddef>

using fft_complex = std::complex<float>;   /* interleaved (re, im), fftwf_complex compatible */
typedef void *FFTPlanHandle;

enum class FFTDirection { Forward, Backward };

class FFTBackend {
public:
    virtual ~FFTBackend() = default;
    virtual const char *name() const = 0;
    virtual FFTPlanHandle plan_r2c(int n, float *in, fft_complex *out) = 0;
    virtual FFTPlanHandle plan_c2c(int n, fft_complex *in, fft_complex *out, FFTDirection dir) = 0;
    virtual void execute_r2c(FFTPlanHandle plan, float *in, fft_complex *out) = 0;
    virtual void execute_c2c(FFTPlanHandle plan, fft_complex *in, fft_complex *out) = 0;
    virtual void destroy_plan(FFTPlanHandle plan) = 0;
    virtual void import_wisdom(const char *filename) { (void)filename; }
    virtual void export_wisdom(const char *filename) { (void)filename; }
    virtual void *alloc(size_t bytes) = 0;
    virtual void free(void *ptr) = 0;
};

FFTBackend *getFFTBackend();

#define FFT_BACKEND_NAME "HIP"

#endif /* SDDC_COMPAT_FFT_BACKEND_H */
