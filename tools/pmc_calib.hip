// pmc_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the DDC kernel's access
// widths (MI355X_MICROARCH.md "HBM": only 16 B/lane streaming reads are calibrated).
// One streaming pass that reads `in_bytes` with 4 B/lane buffer loads (the frame loads) and
// writes 2x as many bytes with 8 B/lane buffer stores (the IQ stores) — the d = 0 byte ratio —
// from a persistent grid like r2iq_persistent_kernel's.  Prints the known byte counts.
//   build/bin/pmc_calib [MiB of input, default 256]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void calib_stream_kernel(const int *in, float2 *out, long n_words)
{
    const long per = (n_words + gridDim.x - 1) / gridDim.x;
    const long b0 = per * blockIdx.x;
    const long b1 = b0 + per < n_words ? b0 + per : n_words;
    for (long base = b0; base < b1; base += 256 * 16) {
        __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), (short)0,
                                                                      (int)((b1 - base) * 4), 0x00020000);
        __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(out + base), (short)0,
                                                                      (int)((b1 - base) * 8), 0x00020000);
        int v[16];
#pragma unroll
        for (int r = 0; r < 16; r++)
            v[r] = (int)__builtin_amdgcn_raw_buffer_load_b32(ri, 4u * threadIdx.x, 4u * 256 * r, 0);
#pragma unroll
        for (int r = 0; r < 16; r++) {
            u32x2 u;
            u.x = (unsigned)v[r];
            u.y = (unsigned)(v[r] ^ 0x5a5a);
            __builtin_amdgcn_raw_buffer_store_b64(u, ro, 8u * threadIdx.x, 8u * 256 * r, 0);
        }
    }
}

int main(int argc, char **argv)
{
    const long mib = argc > 1 ? std::atol(argv[1]) : 256;
    const long n_words = mib * 1024 * 1024 / 4;
    int *in = nullptr;
    float2 *out = nullptr;
    if (hipMalloc(&in, n_words * 4) != hipSuccess || hipMalloc(&out, n_words * 8) != hipSuccess) return 1;
    (void)hipMemset(in, 1, n_words * 4);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(calib_stream_kernel, dim3(cus * 4), dim3(256), 0, 0, in, out, n_words);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("{\"read_bytes\": %ld, \"write_bytes\": %ld, \"launches\": 3, \"grid\": %d}\n", n_words * 4,
                n_words * 8, cus * 4);
    return 0;
}
