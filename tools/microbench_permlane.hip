// microbench_permlane.hip — issue cost of v_permlane32_swap_b32 on gfx950: independent swaps,
// swaps whose inputs were just written by a VALU op (the 2-wait-state hazard), and dependent
// swap pairs (the two-swap rotation), at 1 and 2 waves per SIMD.  One-off measurement tool.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_permlane.hip -o build/microbench_permlane
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048

template <int KIND>
__global__ __launch_bounds__(64, 2) void k(unsigned *out)
{
    unsigned r[16];
    for (int i = 0; i < 16; i++) r[i] = threadIdx.x * 16 + i;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            if (KIND == 0) {          // independent swaps (no VALU write right before)
                auto x = __builtin_amdgcn_permlane32_swap(r[i], r[i + 1], false, false);
                r[i] = x[0];
                r[i + 1] = x[1];
            } else if (KIND == 1) {   // VALU op, then a swap of its result (hazard)
                r[i] += 1u;
                auto x = __builtin_amdgcn_permlane32_swap(r[i], r[i + 1], false, false);
                r[i] = x[0];
                r[i + 1] = x[1];
            } else if (KIND == 2) {   // two dependent swaps (rotation of two registers)
                auto x = __builtin_amdgcn_permlane32_swap(r[i], r[i + 1], false, false);
                auto y = __builtin_amdgcn_permlane32_swap(x[1], x[0], false, false);
                r[i] = y[0];
                r[i + 1] = y[1];
            } else {                  // reference: two plain VALU ops
                r[i] = r[i] * 3u + 1u;
                r[i + 1] ^= r[i];
            }
        }
    }
    unsigned s = 0;
    for (int i = 0; i < 16; i++) s += r[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int KIND>
void run(const char *name, int insts_per_pair)
{
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *out;
    (void)hipMalloc(&out, cus * 8 * 64 * sizeof(unsigned));
    for (int wps = 1; wps <= 2; wps++) {
        const int blocks = cus * 4 * wps;
        hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(64), 0, 0, out);
        (void)hipDeviceSynchronize();
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        for (int rep = 0; rep < 10; rep++) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(64), 0, 0, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        const double per_simd = (double)wps * ITERS * 8 * insts_per_pair;
        printf("%-26s waves/SIMD=%d  %.3f ms  %.2f cycles per instruction per SIMD @2.1GHz\n", name, wps, ms,
               ms * 1e-3 * 2.1e9 / per_simd);
    }
    (void)hipFree(out);
}

int main()
{
    run<3>("2 plain VALU (reference)", 2);
    run<0>("independent swap", 1);
    run<1>("VALU + swap of its result", 2);
    run<2>("2 dependent swaps", 2);
    return 0;
}
