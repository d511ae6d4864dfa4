// chronos_hip.h — shared device helpers for the gfx950 (CDNA4, MI355X) kernel library.
//
// Conventions used by every kernel in csrc/kernels:
//   * bf16 tensors travel as raw 16-bit words (uint16_t) and are moved 16 B per lane (8 elements) wherever the
//     layout allows (cdna_hip_programming.md Guideline 13: hipcc never vectorises scalar bf16 loads).
//   * f32 -> bf16 uses the compiler cast (v_cvt_pk_bf16_f32 on gfx950, RNE, NaN-preserving), never bit tricks.
//   * wave = 64 lanes; block sizes are multiples of 64; cross-lane reductions use __shfl_xor over 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace chronos {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_sum(v);
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = (threadIdx.x < (unsigned)nw) ? red[threadIdx.x] : 0.f;
    if (w == 0) t = wave_sum(t);
    if (threadIdx.x == 0) red[0] = t;
    __syncthreads();
    float r = red[0];
    __syncthreads();
    return r;
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"): consecutive logical
// tiles land on the same XCD (shared L2).  Speed only; correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

}  // namespace chronos
