// fft_backend_harness.cpp — drives the HIP FFTBackend (extio_sddc_amd/csrc/fft_backend/)
// through the FFTBackend API only, plus the batched C ABI underneath (include/sddc_fft.h).
//
//   fft_backend_harness dump FILE   for each size of the path (r2c 128..8192, c2c 64..4096
//                                   both directions): deterministic input, one execute via
//                                   alloc()ed (GPU-mapped) buffers and one via malloc()ed
//                                   (staged) buffers; writes [kind n dir | in | out | out2]
//                                   records for tests/test_gpu_fft.py to check vs numpy.
//   fft_backend_harness bench       per-call latency through the API (warm-up 10, 1000
//                                   executes, the shape of Core/fft_benchmark.cpp's table)
//                                   and batched device-resident throughput per size.
#include "fft_backend.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sddc_fft.h"

static uint64_t g_state = 0x5DDC5DDCull;
static float urand()
{
    g_state = g_state * 6364136223846793005ull + 1442695040888963407ull;
    return (float)((g_state >> 40) & 0xFFFFFF) / 16777216.0f - 0.5f;
}

static void put(FILE *f, const void *p, size_t bytes)
{
    if (fwrite(p, 1, bytes, f) != bytes) {
        perror("fwrite");
        exit(1);
    }
}

static int dump(const char *path)
{
    FFTBackend *be = getFFTBackend();
    FILE *f = fopen(path, "wb");
    if (!f) return perror(path), 1;
    for (int kind = 0; kind < 2; kind++) {
        for (int n = kind ? 128 : 64; n <= (kind ? 8192 : 4096); n *= 2) {
            for (int dir = -1; dir <= (kind ? -1 : 1); dir += 2) {
                const size_t nin = kind ? (size_t)n : 2 * (size_t)n;             // floats
                const size_t nout = kind ? 2 * (size_t)(n / 2 + 1) : 2 * (size_t)n;
                float *in = static_cast<float *>(be->alloc(nin * sizeof(float)));
                float *out = static_cast<float *>(be->alloc(nout * sizeof(float)));
                std::vector<float> in2(nin), out2(nout, NAN);
                for (size_t i = 0; i < nin; i++) in2[i] = in[i] = urand();
                FFTPlanHandle p;
                if (kind) {
                    p = be->plan_r2c(n, in, reinterpret_cast<fft_complex *>(out));
                    be->execute_r2c(p, in, reinterpret_cast<fft_complex *>(out));
                    be->execute_r2c(p, in2.data(), reinterpret_cast<fft_complex *>(out2.data()));
                } else {
                    p = be->plan_c2c(n, reinterpret_cast<fft_complex *>(in), reinterpret_cast<fft_complex *>(out),
                                     dir < 0 ? FFTDirection::Forward : FFTDirection::Backward);
                    be->execute_c2c(p, reinterpret_cast<fft_complex *>(in), reinterpret_cast<fft_complex *>(out));
                    be->execute_c2c(p, reinterpret_cast<fft_complex *>(in2.data()),
                                    reinterpret_cast<fft_complex *>(out2.data()));
                }
                if (!p) return fprintf(stderr, "plan failed kind %d n %d\n", kind, n), 1;
                be->destroy_plan(p);
                const int32_t hdr[3] = {kind, n, dir};
                put(f, hdr, sizeof hdr);
                put(f, in, nin * sizeof(float));
                put(f, out, nout * sizeof(float));
                put(f, out2.data(), nout * sizeof(float));
                be->free(in);
                be->free(out);
            }
        }
    }
    fclose(f);
    printf("dump ok: %s\n", path);
    return 0;
}

static double per_call_us(FFTBackend *be, FFTPlanHandle p, int kind, void *in, void *out)
{
    auto run = [&] {
        if (kind) be->execute_r2c(p, static_cast<float *>(in), static_cast<fft_complex *>(out));
        else be->execute_c2c(p, static_cast<fft_complex *>(in), static_cast<fft_complex *>(out));
    };
    for (int i = 0; i < 10; i++) run();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) run();
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 1000;
}

static int bench()
{
    FFTBackend *be = getFFTBackend();
    printf("backend: %s\n", be->name());
    printf("per call through the FFTBackend API (mapped host buffers, execute = launch + sync):\n");
    printf("  size |  r2c (us) | c2c fwd (us) | c2c bwd (us)\n");
    const int sizes[] = {4096, 2048, 1024, 512, 256, 128};   // Core/fft_benchmark.cpp:12
    for (int n : sizes) {
        void *ri = be->alloc(n * sizeof(float)), *ro = be->alloc((n / 2 + 1) * sizeof(fft_complex));
        void *ci = be->alloc(n * sizeof(fft_complex)), *co = be->alloc(n * sizeof(fft_complex));
        memset(ri, 0, n * sizeof(float));
        memset(ci, 0, n * sizeof(fft_complex));
        FFTPlanHandle pr = be->plan_r2c(n, static_cast<float *>(ri), static_cast<fft_complex *>(ro));
        FFTPlanHandle pf = be->plan_c2c(n, static_cast<fft_complex *>(ci), static_cast<fft_complex *>(co), FFTDirection::Forward);
        FFTPlanHandle pb = be->plan_c2c(n, static_cast<fft_complex *>(co), static_cast<fft_complex *>(ci), FFTDirection::Backward);
        printf("  %4d | %9.2f | %12.2f | %12.2f\n", n, per_call_us(be, pr, 1, ri, ro), per_call_us(be, pf, 0, ci, co),
               per_call_us(be, pb, 0, co, ci));
        be->destroy_plan(pr);
        be->destroy_plan(pf);
        be->destroy_plan(pb);
        be->free(ri);
        be->free(ro);
        be->free(ci);
        be->free(co);
    }
    printf("batched, device-resident (2^24 complex points per launch, hipEvent timing, median of 20):\n");
    printf("  kind  size |  batch  |  us/launch | Gpoints/s | GFLOP/s (5 n log2 n) | HBM GB/s (r+w)\n");
    const size_t pts = size_t(1) << 24;
    void *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, pts * 8 * 2) != hipSuccess || hipMalloc(&b, pts * 8 * 2) != hipSuccess) return 1;
    (void)hipMemset(a, 0, pts * 16);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int kind = 0; kind < 2; kind++) {
        for (int n = kind ? 128 : 64; n <= (kind ? 8192 : 4096); n *= 2) {
            const int batch = (int)((kind ? 2 * pts : pts) / n);
            std::vector<float> t;
            for (int rep = 0; rep < 23; rep++) {
                (void)hipEventRecord(e0, s);
                const int rc = kind ? sddc_fft_r2c(static_cast<float *>(a), b, n, batch, s)
                                    : sddc_fft_c2c(a, b, n, batch, SDDC_FFT_FORWARD, s);
                (void)hipEventRecord(e1, s);
                (void)hipEventSynchronize(e1);
                if (rc) return fprintf(stderr, "fft rc %d\n", rc), 1;
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (rep >= 3) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            const double us = t[t.size() / 2] * 1e3;
            const double cpts = kind ? (double)batch * n / 2 : (double)batch * n;   // complex points transformed
            const double flops = (kind ? 2.5 : 5.0) * (double)batch * n * std::log2((double)n);
            const double bytes = kind ? (double)batch * (n * 4.0 + (n / 2 + 1) * 8.0) : (double)batch * n * 16.0;
            printf("  %s %5d | %7d | %10.1f | %9.1f | %20.0f | %8.0f\n", kind ? "r2c" : "c2c", n, batch, us,
                   cpts / us * 1e-3, flops / us * 1e-3, bytes / us * 1e-3);
        }
    }
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc >= 3 && !strcmp(argv[1], "dump")) return dump(argv[2]);
    if (argc >= 2 && !strcmp(argv[1], "bench")) return bench();
    fprintf(stderr, "usage: %s dump FILE | bench\n", argv[0]);
    return 2;
}
