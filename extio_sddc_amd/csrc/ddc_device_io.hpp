// ddc_device_io.hpp — global-memory I/O shared by the persistent kernels: raw buffer
// loads/stores, the fused fine-tune NCO and the output format stage (CF32 / CS16).
#pragma once

#include <hip/hip_runtime.h>

namespace sddc {

// Raw buffer access: a wave-uniform base (SGPRs), a per-thread byte offset and a uniform
// byte offset (SGPR or immediate), so per-access address arithmetic is scalar.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base)
{
    // raw (stride 0) buffer, byte range checked against 2^31 - 1; dword3 for gfx950
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 buf_load16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff)
{
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ float2 buf_load8(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff)
{
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    return make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
}
template <int AUX = 0>
__device__ __forceinline__ int buf_load4(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff)
{
    return (int)__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX);
}
// Cache policy of the IQ stores: nt (streaming; the output is never re-read by the kernel).
// Measured +2.6 / +4.4 / +1.8 % at d = 0 / 1 / 4 over the default policy; sc0 is neutral
// (profiles/r01/ab/ab_cache_policy.txt).
#ifndef SDDC_ST_AUX
#define SDDC_ST_AUX 2
#endif
// Cache policy of the ADC frame loads: default.  nt loses 2-3 %: consecutive frames overlap
// by 2048 samples, and that quarter is re-read from L2.
#ifndef SDDC_LD_AUX
#define SDDC_LD_AUX 0
#endif
template <int AUX = SDDC_ST_AUX>
__device__ __forceinline__ void buf_store8(float2 v, __amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff)
{
    u32x2 u;
    u.x = __float_as_uint(v.x);
    u.y = __float_as_uint(v.y);
    __builtin_amdgcn_raw_buffer_store_b64(u, r, voff, soff, AUX);
}
template <int AUX = SDDC_ST_AUX>
__device__ __forceinline__ void buf_store4(unsigned v, __amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff)
{
    __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, soff, AUX);
}

// Fine-tune NCO on output sample o of the batch (fine_tune.h): phasor T[q-1] * S_b[l] for
// o = 128 b + 4 q + l, then the mix, in pf_mixer.cpp:808-833's float operation order.
struct NcoArgs {
    const float2 *starts;   // [blocks][4] lane starts of this batch (host chain)
    const float2 *trig;     // [32] T
};

__device__ __forceinline__ float2 nco_mix(float2 v, const NcoArgs &nco, int o)
{
#pragma clang fp contract(off)
    const float2 sb = nco.starts[(o >> 7) * 4 + (o & 3)];
    const int q = (o >> 2) & 31;
    const float2 tq = nco.trig[(q + 31) & 31];   // T[q-1]; unused for q = 0
    const float2 pq = make_float2(tq.x * sb.x - tq.y * sb.y, tq.y * sb.x + tq.x * sb.y);
    const float2 p = q ? pq : sb;
    return make_float2(v.x * p.x - v.y * p.y, v.y * p.x + v.x * p.y);
}

// Output stage.  lsbmask: 0x80000000 flips the imaginary sign (copy<flip=true>,
// fft_mt_r2iq.h:63-71), else 0.  CS16: (I, Q) int16 = saturate(rint(x * scale)).
struct OutArgs {
    unsigned lsbmask;
    float scale;
};

__device__ __forceinline__ float2 flip(float2 v, unsigned lsbmask)
{
    v.y = __uint_as_float(__float_as_uint(v.y) ^ lsbmask);
    return v;
}

__device__ __forceinline__ unsigned cs16_pack(float2 v, float scale)
{
    int i = __float2int_rn(v.x * scale), q = __float2int_rn(v.y * scale);
    i = min(max(i, -32768), 32767);
    q = min(max(q, -32768), 32767);
    return ((unsigned)i & 0xffffu) | ((unsigned)q << 16);
}

template <bool CS16>
constexpr unsigned out_bytes() { return CS16 ? 4u : 8u; }

// store complex v at element (voff_el + soff_el) of the buffer r; AUX: the cache policy (default
// nt; 0 = write-back, for stores whose lines other waves complete, so that L2 merges them)
template <bool CS16, int AUX = SDDC_ST_AUX>
__device__ __forceinline__ void store_iq(float2 v, __amdgpu_buffer_rsrc_t r, unsigned voff_el, unsigned soff_el,
                                         const OutArgs &oa)
{
    if constexpr (CS16)
        buf_store4<AUX>(cs16_pack(v, oa.scale), r, 4u * voff_el, 4u * soff_el);
    else
        buf_store8<AUX>(v, r, 8u * voff_el, 8u * soff_el);
}

}  // namespace sddc
