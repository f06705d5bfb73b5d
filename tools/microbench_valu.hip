// microbench_valu.hip — VALU throughput on gfx950 by opcode and encoding size (4-byte VOP2,
// 8-byte VOP2+literal / VOP3, packed VOP3P)
// at 1..8 waves per SIMD (one-off measurement tool; results go to profiles/).
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu.hip -o build/microbench_valu
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096

template <int KIND>
__global__ void k(float *out, float a0)
{
    float r[16];
    for (int i = 0; i < 16; i++) r[i] = a0 + threadIdx.x + i;
    const float m = 1.0001f, c = 0.0001f;
    for (int it = 0; it < ITERS; it++) {
        if (KIND == 0) {
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(m), "v"(c));
        } else if (KIND == 1) {
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double *)&r[i]) : "v"(*(double *)&r[0]), "v"(*(double *)&r[2]));
            }
        } else if (KIND == 2) {
#pragma unroll
            for (int i = 0; i < 16; i += 2)
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(double *)&r[i]) : "v"(*(double *)&r[4]));
        } else if (KIND == 3) {
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r[i]) : "v"(m));
        } else if (KIND == 4) {
#pragma unroll
            for (int i = 0; i < 16; i += 2)
                asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(*(double *)&r[i]) : "v"(*(double *)&r[4]));
        } else if (KIND == 5) {   // VOP2 with a 32-bit literal: 8-byte encoding, 2 operands
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("v_add_f32 %0, 0x3f800347, %0" : "+v"(r[i]));
        } else if (KIND == 6) {   // VOP2 fmac: 4-byte encoding, 3 operands (dst read)
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(r[i]) : "v"(m), "v"(c));
        } else if (KIND == 7) {   // fmac with a literal: 8-byte encoding, 3 operands
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("v_fmac_f32 %0, 0x3f800347, %1" : "+v"(r[i]) : "v"(c));
        } else if (KIND == 8) {   // VOP2 mul: 4-byte encoding, 2 operands
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[i]) : "v"(m));
        } else {                  // FFT-like mix: add, sub, fmac-literal, mul-literal
#pragma unroll
            for (int i = 0; i < 16; i += 4) {
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(r[i]) : "v"(m));
                asm volatile("v_sub_f32 %0, %0, %1" : "+v"(r[i + 1]) : "v"(m));
                asm volatile("v_fmac_f32 %0, 0x3f800347, %1" : "+v"(r[i + 2]) : "v"(c));
                asm volatile("v_mul_f32 %0, 0x3f800347, %0" : "+v"(r[i + 3]));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 16; i++) s += r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
void run(const char *name, int flops_per_inst_lane)
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    hipMalloc(&out, 256 * 1024 * 64 * sizeof(float));
    for (int wps = 1; wps <= 8; wps *= 2) {
        // one block of 256 threads = 4 waves = 1 per SIMD; wps blocks per CU
        const int blocks = cus * wps;
        hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, out, 1.f);
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        for (int rep = 0; rep < 5; rep++) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, out, 1.f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        const double insts = (double)blocks * 4 /*waves*/ * ITERS * (KIND == 1 || KIND == 2 || KIND == 4 ? 8 : 16);
        const double per_simd = insts / (cus * 4);
        const double ghz = 2.1;
        printf("%-14s waves/SIMD=%d  %.3f ms  %.2f cycles/inst/SIMD @%.1fGHz  %.1f TFLOP/s\n", name, wps, ms,
               ms * 1e-3 * ghz * 1e9 / per_simd, ghz, insts * 64 * flops_per_inst_lane / (ms * 1e-3) / 1e12);
    }
    hipFree(out);
}

int main()
{
    run<0>("v_fma_f32", 2);
    run<3>("v_add_f32", 1);
    run<1>("v_pk_fma_f32", 4);
    run<2>("v_pk_add_f32", 2);
    run<4>("v_pk_mul_f32", 2);
    run<5>("v_add lit (8B)", 1);
    run<6>("v_fmac (4B)", 2);
    run<7>("v_fmac lit(8B)", 2);
    run<8>("v_mul (4B)", 1);
    run<9>("fft mix", 1);
    return 0;
}
