// microbench_dft.hip — issue rate of the compiled in-register DFT cores (fft_device.hpp) on
// gfx950, no memory traffic in the loop: cycles per VALU instruction per SIMD at 1 and 2
// waves per SIMD, next to the VALU count of one call (from the ISA, passed on the command
// line).  One-off measurement tool; results go to profiles/.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -Iextio_sddc_amd/csrc tools/microbench_dft.hip -o build/microbench_dft
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "fft_device.hpp"

using namespace sddc;
#define ITERS 256

template <int KIND>
__global__ __launch_bounds__(64, 2) void k(float2 *io)
{
    float2 R[64], T[64];
    const int base = (blockIdx.x * 64 + threadIdx.x) * 64;
#pragma unroll
    for (int i = 0; i < 64; i++) R[i] = io[base + i];
    for (int it = 0; it < ITERS; it++) {
        if constexpr (KIND == 0) {        // one DFT-64 forward + one backward
            dft64<-1>(R, T);
            dft64<+1>(T, R);
        } else {                          // four DFT-32s forward + backward
            dft32<-1>(R, T);
            dft32<-1>(R + 32, T + 32);
            dft32<+1>(T, R);
            dft32<+1>(T + 32, R + 32);
        }
    }
#pragma unroll
    for (int i = 0; i < 64; i++) io[base + i] = R[i];
}

template <int KIND>
void run(const char *name, int valu_per_iter)
{
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float2 *io;
    (void)hipMalloc(&io, (size_t)cus * 8 * 64 * 64 * sizeof(float2));
    (void)hipMemset(io, 0, (size_t)cus * 8 * 64 * 64 * sizeof(float2));
    for (int wps = 1; wps <= 2; wps++) {
        const int blocks = cus * 4 * wps;   // 64-thread blocks: 4 per CU = 1 wave per SIMD
        hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(64), 0, 0, io);
        (void)hipDeviceSynchronize();
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        for (int rep = 0; rep < 10; rep++) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(64), 0, 0, io);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        const double per_simd = (double)wps * ITERS * valu_per_iter;
        printf("%-10s waves/SIMD=%d  %.3f ms  %.2f cycles/VALU/SIMD @2.1GHz (%d VALU per iteration)\n", name, wps, ms,
               ms * 1e-3 * 2.1e9 / per_simd, valu_per_iter);
    }
    (void)hipFree(io);
}

int main(int argc, char **argv)
{
    const int v64 = argc > 1 ? atoi(argv[1]) : 2160, v32 = argc > 2 ? atoi(argv[2]) : 1744;
    run<0>("dft64 x2", v64);
    run<1>("dft32 x4", v32);
    return 0;
}
