// elementwise.hip — memory-bound kernels of the Llama-3 block:
//   embedding gather (vocab-parallel aware), RMSNorm with fused residual add, RoPE fused with the paged KV-cache
//   write, SiLU(gate)*up.
//
// All bf16 traffic is 16 B per lane (8 elements).  Each kernel reads/writes its tensors exactly once; the residual
// add, the norm and the KV-cache write are fused into the producer of the next GEMM's input so no intermediate round
// trips through HBM.
#include "chronos_hip.h"

namespace chronos {

// ------------------------------------------------------------------------------------------------------------------
// K1 embedding gather.  out[t, :] = table[ids[t] - vstart, :] if vstart <= ids[t] < vstart + vrows else 0 (the
// zero rows of a vocab-parallel shard are summed away by the TP all-reduce).
// ------------------------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) embedding_kernel(const int32_t* __restrict__ ids, const uint16_t* __restrict__ table,
                                                        uint16_t* __restrict__ out, int d, int64_t vstart, int64_t vrows,
                                                        const int32_t* __restrict__ gst, int gn) {
    if (gate_closed(gst, gn)) return;
    const int t = blockIdx.x;
    const int64_t id = (int64_t)ids[t] - vstart;
    const bool ok = id >= 0 && id < vrows;
    const u16x8* src = reinterpret_cast<const u16x8*>(table + (ok ? id : 0) * (int64_t)d);
    u16x8* dst = reinterpret_cast<u16x8*>(out + (int64_t)t * d);
    for (int i = threadIdx.x; i < d / 8; i += blockDim.x) {
        u16x8 v = ok ? src[i] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        dst[i] = v;
    }
}

// ------------------------------------------------------------------------------------------------------------------
// K2 RMSNorm (+ fused residual add).  One 256-thread block per row; the row is held in registers between the
// reduction and the scaling pass (d <= 256*8*MAXV).
//   plain:     y = x * rsqrt(mean(x^2) + eps) * w
//   residual:  r = bf16(x + r) (written back), y = rmsnorm(r) * w       (HF Llama: residual kept in bf16)
// ------------------------------------------------------------------------------------------------------------------
template <int MAXV, bool RESID>
__global__ void __launch_bounds__(256) rmsnorm_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ resid,
                                                      const uint16_t* __restrict__ w, uint16_t* __restrict__ y, int d,
                                                      float eps, const int32_t* __restrict__ gst, int gn) {
    __shared__ float red[16];
    if (gate_closed(gst, gn)) return;
    const int64_t row = blockIdx.x;
    const u16x8* xv = reinterpret_cast<const u16x8*>(x + row * d);
    u16x8* rv = reinterpret_cast<u16x8*>(resid + row * d);
    const u16x8* wv = reinterpret_cast<const u16x8*>(w);
    u16x8* yv = reinterpret_cast<u16x8*>(y + row * d);
    const int nv = d / 8;
    // every load of the row (x, resid and the norm weight) issued before the first use: indices past the row are
    // clamped (in-bounds re-reads) and masked, so hipcc does not branch around each load and wait per element
    u16x8 a[MAXV], b[MAXV], g[MAXV];
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int i = min((int)threadIdx.x + k * 256, nv - 1);
        a[k] = xv[i];
        if constexpr (RESID) b[k] = rv[i];
        g[k] = wv[i];
    }
    float vals[MAXV][8];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int i = threadIdx.x + k * 256;
        if constexpr (RESID) {
            u16x8 sv;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                sv[j] = f2bf(bf2f(a[k][j]) + bf2f(b[k][j]));
                vals[k][j] = bf2f(sv[j]);
            }
            if (i < nv) rv[i] = sv;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) vals[k][j] = bf2f(a[k][j]);
        }
        if (i < nv) {
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += vals[k][j] * vals[k][j];
        }
    }
    const float tot = block_sum(ss, red);
    const float inv = rsqrtf(tot / (float)d + eps);
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < nv) {
            u16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(f2bf(vals[k][j] * inv)) * bf2f(g[k][j]));
            yv[i] = o;
        }
    }
}

// ------------------------------------------------------------------------------------------------------------------
// K4 RoPE + paged KV-cache write (+ K13: optional fp8-e4m3 cache with a per-layer scale).  Input: the QKV GEMM output qkv[T, (Hq + 2*Hkv) * 128].
//   q  -> q_out[T, Hq, 128]                rotated (HF rotate-half convention)
//   k  -> k_cache[blk, h, t % BS, :]        rotated       (row-major per token: B operand of S^T = K Q^T)
//   v  -> v_cache[blk, h, :, t % BS]        transposed    (A operand of O^T = V^T P^T, see attention.hip)
// The cache slot is derived on device from block_table[tok_seq[t], pos / BS] so a captured decode graph needs no
// host-side slot mapping.  cos_sin[pos, 0:64] = cos, [64:128] = sin (f32, precomputed on the host incl. Llama-3.1
// frequency scaling).
// Thread map per token (blockIdx.x = token, blockIdx.y * 256 + threadIdx.x = g):
//   g <  8*(Hq+Hkv):  8 threads per q/k head, each owning dims {8i..8i+7} and {64+8i..64+8i+7} (16-B loads/stores);
//   g >= 8*(Hq+Hkv):  one wave per v head, lane l owning dims l and 64+l.  The transposed V row is 128 values each
//                     BS*2 bytes apart: with a whole wave on consecutive dims, one store instruction covers 64 dims
//                     in 16 cache lines (4 lanes per line, merged), instead of 64 lines with 8 threads per head.
// ------------------------------------------------------------------------------------------------------------------
template <bool FP8>
__global__ void __launch_bounds__(256) rope_kv_write_kernel(
    const uint16_t* __restrict__ qkv, const int32_t* __restrict__ pos, const int32_t* __restrict__ tok_seq,
    const int32_t* __restrict__ block_table, int bt_stride, const float* __restrict__ cos_sin,
    uint16_t* __restrict__ q_out, void* __restrict__ k_cache, void* __restrict__ v_cache, int hq, int hkv,
    int block_size, int write_q, float k_inv_scale, float v_inv_scale, const int32_t* __restrict__ gst, int gn) {
    constexpr int D = 128;
    if (gate_closed(gst, gn)) return;
    const int t = blockIdx.x;
    const int g = blockIdx.y * 256 + threadIdx.x;
    const int nh = hq + 2 * hkv;
    const int nrope = 8 * (hq + hkv);
    if (g >= nrope + 64 * hkv) return;
    const int p = pos[t];
    const int seq = tok_seq[t];
    const int64_t blk = block_table[(int64_t)seq * bt_stride + p / block_size];
    const int off = p % block_size;
    if (g < nrope) {
        const int unit = g >> 3, i = g & 7;
        if (unit < hq && !write_q) return;
        const uint16_t* src = qkv + ((int64_t)t * nh + unit) * D;
        const u16x8 a = *reinterpret_cast<const u16x8*>(src + 8 * i);
        const u16x8 b = *reinterpret_cast<const u16x8*>(src + 64 + 8 * i);
        const float* cs = cos_sin + (int64_t)p * D;
        const float4 c0 = *reinterpret_cast<const float4*>(cs + 8 * i);
        const float4 c1 = *reinterpret_cast<const float4*>(cs + 8 * i + 4);
        const float4 s0 = *reinterpret_cast<const float4*>(cs + 64 + 8 * i);
        const float4 s1 = *reinterpret_cast<const float4*>(cs + 64 + 8 * i + 4);
        const float c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        float fa[8], fb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float x1 = bf2f(a[j]), x2 = bf2f(b[j]);
            fa[j] = x1 * c[j] - x2 * s[j];
            fb[j] = x2 * c[j] + x1 * s[j];
        }
        if (unit < hq || !FP8) {
            u16x8 ra, rb;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                ra[j] = f2bf(fa[j]);
                rb[j] = f2bf(fb[j]);
            }
            uint16_t* dst = unit < hq ? q_out + ((int64_t)t * hq + unit) * D
                                      : reinterpret_cast<uint16_t*>(k_cache) +
                                            (((blk * hkv + (unit - hq)) * block_size) + off) * D;
            *reinterpret_cast<u16x8*>(dst + 8 * i) = ra;
            *reinterpret_cast<u16x8*>(dst + 64 + 8 * i) = rb;
        } else {  // fp8 K row: 128 bytes per token
            uint8_t* dst = reinterpret_cast<uint8_t*>(k_cache) + (((blk * hkv + (unit - hq)) * block_size) + off) * D;
            uint2 qa, qb;
            qa.x = f32x4_to_fp8x4(fa[0] * k_inv_scale, fa[1] * k_inv_scale, fa[2] * k_inv_scale, fa[3] * k_inv_scale);
            qa.y = f32x4_to_fp8x4(fa[4] * k_inv_scale, fa[5] * k_inv_scale, fa[6] * k_inv_scale, fa[7] * k_inv_scale);
            qb.x = f32x4_to_fp8x4(fb[0] * k_inv_scale, fb[1] * k_inv_scale, fb[2] * k_inv_scale, fb[3] * k_inv_scale);
            qb.y = f32x4_to_fp8x4(fb[4] * k_inv_scale, fb[5] * k_inv_scale, fb[6] * k_inv_scale, fb[7] * k_inv_scale);
            *reinterpret_cast<uint2*>(dst + 8 * i) = qa;
            *reinterpret_cast<uint2*>(dst + 64 + 8 * i) = qb;
        }
    } else {
        const int h = (g - nrope) >> 6, l = (g - nrope) & 63;
        const uint16_t* src = qkv + ((int64_t)t * nh + hq + hkv + h) * D;
        const uint16_t a = src[l], b = src[64 + l];
        const int64_t base = ((blk * hkv + h) * D) * (int64_t)block_size + off;
        if constexpr (FP8) {
            uint8_t* dst = reinterpret_cast<uint8_t*>(v_cache) + base;
            const uint32_t q = f32x4_to_fp8x4(bf2f(a) * v_inv_scale, bf2f(b) * v_inv_scale, 0.f, 0.f);
            dst[(int64_t)l * block_size] = (uint8_t)q;
            dst[(int64_t)(64 + l) * block_size] = (uint8_t)(q >> 8);
        } else {
            uint16_t* dst = reinterpret_cast<uint16_t*>(v_cache) + base;
            dst[(int64_t)l * block_size] = a;
            dst[(int64_t)(64 + l) * block_size] = b;
        }
    }
}

// ------------------------------------------------------------------------------------------------------------------
// K9 SwiGLU: out[t, f] = silu(gu[t, f]) * gu[t, F + f]
// ------------------------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) silu_mul_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out,
                                                       int64_t rows, int f) {
    // one thread = 2 consecutive 8-element chunks of a row (f % 16 == 0), all four loads issued before any math: the
    // M = 1024 decode shape (1024 x 14336) ran 26 us as a capped grid-stride loop with one chunk per iteration, i.e.
    // ~3.4 TB/s on 88 MB
    const int np = f / 16;  // chunk pairs per row
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * np) return;
    const int64_t r = idx / np;
    const int c = 2 * (int)(idx - r * np);
    const u16x8* g = reinterpret_cast<const u16x8*>(gu + r * 2 * f);
    const u16x8* u = reinterpret_cast<const u16x8*>(gu + r * 2 * f + f);
    const u16x8 g0 = g[c], g1 = g[c + 1], u0 = u[c], u1 = u[c + 1];
    u16x8 o0, o1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x0 = bf2f(g0[j]), x1 = bf2f(g1[j]);
        o0[j] = f2bf(bf2f(f2bf(x0 / (1.f + __expf(-x0)))) * bf2f(u0[j]));
        o1[j] = f2bf(bf2f(f2bf(x1 / (1.f + __expf(-x1)))) * bf2f(u1[j]));
    }
    u16x8* ov = reinterpret_cast<u16x8*>(out + r * f);
    ov[c] = o0;
    ov[c + 1] = o1;
}

// f % 16 != 0: one chunk per thread
__global__ void __launch_bounds__(256) silu_mul1_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out,
                                                        int64_t rows, int f) {
    const int nv = f / 8;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * nv) return;
    const int64_t r = idx / nv;
    const int c = (int)(idx - r * nv);
    const u16x8 g = reinterpret_cast<const u16x8*>(gu + r * 2 * f)[c];
    const u16x8 u = reinterpret_cast<const u16x8*>(gu + r * 2 * f + f)[c];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = bf2f(g[j]);
        o[j] = f2bf(bf2f(f2bf(x / (1.f + __expf(-x)))) * bf2f(u[j]));
    }
    reinterpret_cast<u16x8*>(out + r * f)[c] = o;
}

// ------------------------------------------------------------------------------------------------------------------
// Host launchers (called from bindings.cpp)
// ------------------------------------------------------------------------------------------------------------------
void launch_embedding(const int32_t* ids, const uint16_t* table, uint16_t* out, int t, int d, int64_t vstart,
                      int64_t vrows, hipStream_t st) {
    if (t == 0) return;
    hipLaunchKernelGGL(embedding_kernel, dim3(t), dim3(256), 0, st, ids, table, out, d, vstart, vrows, CHRONOS_GATE);
}

void launch_rmsnorm(const uint16_t* x, uint16_t* resid, const uint16_t* w, uint16_t* y, int rows, int d, float eps,
                    hipStream_t st) {
    if (rows == 0) return;
    const int nv = d / 8;
    const dim3 g(rows), b(256);
#define RMS_CASE(V)                                                                                         \
    if (nv <= 256 * V) {                                                                                    \
        if (resid)                                                                                          \
            hipLaunchKernelGGL((rmsnorm_kernel<V, true>), g, b, 0, st, x, resid, w, y, d, eps, CHRONOS_GATE);  \
        else                                                                                                \
            hipLaunchKernelGGL((rmsnorm_kernel<V, false>), g, b, 0, st, x, resid, w, y, d, eps, CHRONOS_GATE); \
        return;                                                                                             \
    }
    RMS_CASE(1) RMS_CASE(2) RMS_CASE(4) RMS_CASE(8)
#undef RMS_CASE
}

void launch_rope_kv_write(const uint16_t* qkv, const int32_t* pos, const int32_t* tok_seq, const int32_t* block_table,
                          int bt_stride, const float* cos_sin, uint16_t* q_out, void* k_cache, void* v_cache, int t,
                          int hq, int hkv, int block_size, int write_q, bool fp8, float k_scale, float v_scale,
                          hipStream_t st) {
    if (t == 0) return;
    const dim3 g(t, (8 * (hq + hkv) + 64 * hkv + 255) / 256), b(256);
    if (fp8)
        hipLaunchKernelGGL(rope_kv_write_kernel<true>, g, b, 0, st, qkv, pos, tok_seq, block_table, bt_stride, cos_sin,
                           q_out, k_cache, v_cache, hq, hkv, block_size, write_q, 1.f / k_scale, 1.f / v_scale,
                           CHRONOS_GATE);
    else
        hipLaunchKernelGGL(rope_kv_write_kernel<false>, g, b, 0, st, qkv, pos, tok_seq, block_table, bt_stride,
                           cos_sin, q_out, k_cache, v_cache, hq, hkv, block_size, write_q, 1.f, 1.f, CHRONOS_GATE);
}

void launch_silu_mul(const uint16_t* gu, uint16_t* out, int64_t rows, int f, hipStream_t st) {
    if (rows == 0) return;
    const bool pairs = f % 16 == 0;
    const int64_t total = rows * (pairs ? f / 16 : f / 8);
    const int64_t blocks = (total + 255) / 256;
    if (pairs)
        hipLaunchKernelGGL(silu_mul_kernel, dim3((unsigned)blocks), dim3(256), 0, st, gu, out, rows, f);
    else
        hipLaunchKernelGGL(silu_mul1_kernel, dim3((unsigned)blocks), dim3(256), 0, st, gu, out, rows, f);
}

}  // namespace chronos
