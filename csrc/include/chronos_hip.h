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

// Write-through (sc1) stores and L1-bypassing sc1 loads of a 16-byte fp32 vector, for hand-offs between workgroups
// that need no release / acquire fence (MI355X_MICROARCH.md hand-off table, first row: every store of the handed-off
// bytes sc1, one lane per storing workgroup signals with an agent-scope atomic after all its waves' vmcnt(0) and a
// barrier, every load of them sc1 after the signal was seen).  Vector memory instructions only.
__device__ __forceinline__ void st_wt(float* p, const f32x4& v) {
    typedef float f32x2v __attribute__((ext_vector_type(2)));
    uint64_t* q = reinterpret_cast<uint64_t*>(p);
    __hip_atomic_store(q, __builtin_bit_cast(uint64_t, f32x2v{v[0], v[1]}), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, __builtin_bit_cast(uint64_t, f32x2v{v[2], v[3]}), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ f32x4 ld_wt(const float* p) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        v[i] = __uint_as_float(__hip_atomic_load(q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    return v;
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

// ---- fp8 e4m3 (OCP "fn" encoding on gfx950 — not MI300's fnuz) KV-cache helpers ---------------------------------
constexpr float kFp8Max = 448.f;
__device__ __forceinline__ uint32_t f32x4_to_fp8x4(float a, float b, float c, float d) {
    a = fminf(fmaxf(a, -kFp8Max), kFp8Max);  // e4m3fn has no infinity: saturate instead of producing NaN
    b = fminf(fmaxf(b, -kFp8Max), kFp8Max);
    c = fminf(fmaxf(c, -kFp8Max), kFp8Max);
    d = fminf(fmaxf(d, -kFp8Max), kFp8Max);
    int r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
    return (uint32_t)r;
}
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16x4 fp8x4_to_bf16x4(uint32_t v, float scale) {
    const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)v, false);
    const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)v, true);
    return bf16x4{(__bf16)(lo[0] * scale), (__bf16)(lo[1] * scale), (__bf16)(hi[0] * scale), (__bf16)(hi[1] * scale)};
}
// Unscaled e4m3 -> bf16 (exact: every e4m3 value is a bf16 value), two per v_cvt_scalef32_pk_bf16_fp8 (gfx950; scale
// 1.0).  For kernels that fold the cache scale into a later multiply instead of scaling every element.
__device__ __forceinline__ bf16x8 fp8x8_to_bf16x8_raw(uint32_t v0, uint32_t v1) {
    typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
    const bf16x2_v a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v0, 1.f, false);
    const bf16x2_v b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v0, 1.f, true);
    const bf16x2_v c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v1, 1.f, false);
    const bf16x2_v d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v1, 1.f, true);
    return bf16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}
__device__ __forceinline__ bf16x8 fp8x8_to_bf16x8(uint32_t v0, uint32_t v1, float scale) {
    const bf16x4 a = fp8x4_to_bf16x4(v0, scale), b = fp8x4_to_bf16x4(v1, scale);
    return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"): consecutive logical
// tiles land on the same XCD (shared L2).  Speed only; correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

}  // namespace chronos

namespace chronos {
// ---- decode early-exit gate ------------------------------------------------------------------------------------
// A captured decode burst runs k steps back to back.  For a small decode bucket (n <= kGateMax rows, the single- /
// few-stream regime) every kernel of a step first reads the n slot states the previous step's sampler wrote and
// returns at once when none is live (state > 0; DONE == 0, empty slot == -1), so the steps of a burst that follow
// the last verdict's end cost a launch each instead of a full forward.  Set from Python around decode capture
// (torch.ops.chronos.set_decode_gate); launchers read the host globals below and pass them as kernel arguments.
constexpr int kGateMax = 8;
extern const int32_t* g_gate_state;
extern int g_gate_n;
// launcher helper: the (state pointer, n) kernel-argument pair of the current gate, or (nullptr, 0)
#define CHRONOS_GATE (g_gate_n > 0 && g_gate_n <= kGateMax ? g_gate_state : nullptr), \
                     (g_gate_n > 0 && g_gate_n <= kGateMax ? g_gate_n : 0)
__device__ __forceinline__ bool gate_closed(const int32_t* st, int n) {
    if (n <= 0) return false;
    bool live = false;
    for (int i = 0; i < n; ++i) live |= st[i] > 0;
    return !live;
}

// Workgroups of `kernel` (block threads, no dynamic LDS) resident on the whole device at once: the occupancy
// calculator's per-CU count times the CU count, cached per kernel (bindings.cpp).  Persistent grids are sized by it: a
// grid larger than what fits serialises its surplus workgroups behind the first ones.
int resident_workgroups_of(const void* kernel, int threads);
template <typename K>
inline int resident_workgroups(K kernel, int threads) {
    return resident_workgroups_of(reinterpret_cast<const void*>(kernel), threads);
}

// Host-side tuning knobs (defined in bindings.cpp): value set through torch.ops.chronos.set_knob(name, v), else the
// environment variable CHRONOS_<NAME>, else `dflt`.  Used for in-process A/B of kernel variants
// (cdna_hip_programming.md §5.4 rule 24: interleave variants in ONE process).
int knob(const char* name, int dflt);
}  // namespace chronos
