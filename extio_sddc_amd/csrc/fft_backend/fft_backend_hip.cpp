// fft_backend_hip.cpp — the FFTBackend API (Core/fft_backend.h:22-50) on gfx950, replacing
// Core/fft_backend_{fftw,mkl,accelerate}.cpp.  Compiled against
// the reference's own fft_backend.h in the integration build, or include/sddc_compat/.
//
// Semantics follow fft_backend_fftw.cpp: plans carry size and direction only, execute_*
// may be given other arrays of the same size, transforms are unnormalised and the
// results are in `out` when execute_* returns (it synchronises its stream).  Buffers
// from alloc() are pinned host memory mapped into the GPU, so kernels read and write
// them in place over PCIe; any other host pointer is staged through device memory.
#include "fft_backend.h"

#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <mutex>

#include "sddc_ddc.h"
#include "sddc_fft.h"

namespace {

struct HipPlan {
    int kind;   // 0 = c2c, 1 = r2c
    int n;
    int dir;    // SDDC_FFT_FORWARD / SDDC_FFT_BACKWARD
};

class HipFFTBackend final : public FFTBackend {
public:
    ~HipFFTBackend() override
    {
        if (stage_) (void)hipFree(stage_);
        if (stream_) (void)hipStreamDestroy(stream_);
    }

    const char *name() const override { return "HIP (gfx950)"; }

    FFTPlanHandle plan_r2c(int n, float *, fft_complex *) override
    {
        if (!sddc_fft_supported(1, n)) return report("plan_r2c: unsupported size", n);
        return new HipPlan{1, n, SDDC_FFT_FORWARD};
    }

    FFTPlanHandle plan_c2c(int n, fft_complex *, fft_complex *, FFTDirection dir) override
    {
        if (!sddc_fft_supported(0, n)) return report("plan_c2c: unsupported size", n);
        return new HipPlan{0, n, dir == FFTDirection::Forward ? SDDC_FFT_FORWARD : SDDC_FFT_BACKWARD};
    }

    void execute_r2c(FFTPlanHandle plan, float *in, fft_complex *out) override
    {
        const HipPlan *p = static_cast<const HipPlan *>(plan);
        if (!p || p->kind != 1) return;
        run(p, in, (size_t)p->n * sizeof(float), out, (size_t)(p->n / 2 + 1) * sizeof(fft_complex));
    }

    void execute_c2c(FFTPlanHandle plan, fft_complex *in, fft_complex *out) override
    {
        const HipPlan *p = static_cast<const HipPlan *>(plan);
        if (!p || p->kind != 0) return;
        const size_t bytes = (size_t)p->n * sizeof(fft_complex);
        run(p, in, bytes, out, bytes);
    }

    void destroy_plan(FFTPlanHandle plan) override { delete static_cast<HipPlan *>(plan); }

    void *alloc(size_t bytes) override
    {
        void *p = nullptr;
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
        return p;
    }

    void free(void *ptr) override
    {
        if (ptr) (void)hipHostFree(ptr);
    }

private:
    static void *report(const char *what, int n)
    {
        std::fprintf(stderr, "HipFFTBackend %s (%d)\n", what, n);
        return nullptr;
    }

    // true if the GPU can access ptr directly (device memory or pinned/registered host)
    static bool gpu_visible(const void *ptr)
    {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, ptr) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeHost || a.type == hipMemoryTypeManaged;
    }

    void run(const HipPlan *p, const void *in, size_t in_bytes, void *out, size_t out_bytes)
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (!stream_ && hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) return;
        const void *src = in;
        void *dst = out;
        const bool stage_in = !gpu_visible(in), stage_out = !gpu_visible(out);
        if (stage_in || stage_out) {
            const size_t need = in_bytes + out_bytes;
            if (need > stage_bytes_) {
                if (stage_) (void)hipFree(stage_);
                stage_ = nullptr;
                stage_bytes_ = 0;
                if (hipMalloc(&stage_, need) != hipSuccess) return;
                stage_bytes_ = need;
            }
            char *s = static_cast<char *>(stage_);
            if (stage_in) {
                if (hipMemcpyAsync(s, in, in_bytes, hipMemcpyHostToDevice, stream_) != hipSuccess) return;
                src = s;
            }
            if (stage_out) dst = s + in_bytes;
        }
        const int rc = p->kind == 1
                           ? sddc_fft_r2c(static_cast<const float *>(src), dst, p->n, 1, stream_)
                           : sddc_fft_c2c(src, dst, p->n, 1, p->dir, stream_);
        if (rc != SDDC_OK) {
            std::fprintf(stderr, "HipFFTBackend: %s\n", sddc_ddc_last_error());
            return;
        }
        if (stage_out) (void)hipMemcpyAsync(out, dst, out_bytes, hipMemcpyDeviceToHost, stream_);
        (void)hipStreamSynchronize(stream_);
    }

    std::mutex mu_;
    hipStream_t stream_ = nullptr;
    void *stage_ = nullptr;
    size_t stage_bytes_ = 0;
};

}  // namespace

FFTBackend *getFFTBackend()
{
    static HipFFTBackend backend;
    return &backend;
}
