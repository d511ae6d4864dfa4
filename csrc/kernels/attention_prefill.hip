// attention_prefill.hip — flash-style causal prefill attention over the paged KV cache.
//
// The decode kernel (attention.hip) gives every wave the same query rows and splits the keys; for prefill that
// re-reads the whole K/V prefix once per 32 query rows, which is hopeless at 128k tokens.  Here a workgroup owns
// 128 query rows (= 128/G tokens x the G query heads of one kv head) — 32 per wave — and the 4 waves share every
// 32-token K/V tile through LDS:
//   * staging: each thread issues its 2+2 16-byte global loads for tile s+1 at the top of step s and writes them to
//     the other LDS buffer at the end (async-STAGE split, cdna_hip_programming.md T14): one barrier per tile;
//   * K image [32 tok][128 dim] with the 16-byte unit XOR-swizzled by (row & 15) so the 16 rows an MFMA A-operand read
//     touches land on distinct banks (T2); V^T image [128 dim][32 tok] with an 80-byte row pitch (64 B + 16 B pad)
//     which makes the two ds_read_b64 of the P·V operand conflict-free;
//   * math identical to the decode kernel: S^T = K·Q^T so P stays in registers, O^T += V^T·P^T with the shared
//     k-permutation, online softmax in the exp2 domain, -inf masking for the causal edge and the chunk end.
// Tiles are visited heaviest-first (the last query tiles of a sequence see the most keys).
#include "chronos_hip.h"

namespace chronos {

constexpr int kPD = 128;        // head dim
constexpr int kKImg = 32 * 256; // K tile image bytes
constexpr int kVPitch = 80;     // V^T row pitch (bytes)
constexpr int kVImg = 128 * kVPitch;
constexpr int kStage = kKImg + kVImg;

template <bool FP8>
__global__ void __launch_bounds__(256, 2) attn_prefill_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ kcv, const void* __restrict__ vcv,
    const int32_t* __restrict__ block_table, int bt_stride, const int32_t* __restrict__ q_start,
    const int32_t* __restrict__ ctx_len, const int32_t* __restrict__ tiles, int ntiles, uint16_t* __restrict__ out,
    int hq, int hkv, int block_size, float scale_log2, float k_scale, float v_scale) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint16_t* kc = reinterpret_cast<const uint16_t*>(kcv);
    const uint16_t* vc = reinterpret_cast<const uint16_t*>(vcv);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, h4 = lane >> 4;
    const int G = hq / hkv;
    const int h = blockIdx.y;
    const int tile = ntiles - 1 - (int)blockIdx.x;  // heaviest first
    const int seq = tiles[2 * tile], rel0 = tiles[2 * tile + 1];
    const int qbase = q_start[seq], qlen = q_start[seq + 1] - qbase;
    const int ctx = ctx_len[seq], ctx0 = ctx - qlen;
    const int32_t* bt = block_table + (int64_t)seq * bt_stride;

    // ---- this wave's 32 rows: Q fragments (B operand of S^T = K Q^T) ----
    int rpos[2];
    bf16x8 qf[2][4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        const int R = w * 32 + mt * 16 + r;
        const int tr = rel0 + R / G, hd = h * G + R % G;
        const bool valid = tr < qlen;
        rpos[mt] = valid ? ctx0 + tr : -1;
        const uint16_t* qp = q + ((int64_t)(qbase + (valid ? tr : 0)) * hq + hd) * kPD + 8 * h4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            bf16x8 v = *reinterpret_cast<const bf16x8*>(qp + 32 * c);
            if (!valid) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
            qf[mt][c] = v;
        }
    }
    int last_tr = rel0 + 128 / G - 1;
    if (last_tr > qlen - 1) last_tr = qlen - 1;
    const int kv_end = ctx0 + last_tr + 1;
    const int nsteps = (kv_end + 31) >> 5;
    // first position any row of this wave can have (rows are token-major): keys below it need no causal mask
    const int wave_min_pos = ctx0 + rel0 + (w * 32) / G;

    // ---- staging assignment ----
    const int krow = threadIdx.x >> 3, kunit = (threadIdx.x & 7) * 2;     // K: 32 rows x 16 units of 16 B
    const int vrow = threadIdx.x >> 1, vhalf = threadIdx.x & 1;           // V^T: 128 rows x 2 halves of 32 B
    u16x8 ks[2], vs[2];
    auto gload = [&](int s) {
        const int tok = s * 32 + krow;
        if (tok < kv_end) {
            const int64_t blk = bt[tok / block_size];
            const int64_t e = (((blk * hkv + h) * block_size) + tok % block_size) * kPD + kunit * 8;
            if constexpr (FP8) {  // 16 fp8 -> 16 bf16 during staging: the LDS image and the math stay bf16
                const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(kcv) + e);
                ks[0] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.x, v.y, k_scale));
                ks[1] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.z, v.w, k_scale));
            } else {
                const u16x8* p = reinterpret_cast<const u16x8*>(kc + e);
                ks[0] = p[0];
                ks[1] = p[1];
            }
        } else {
            ks[0] = ks[1] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
        const int vt = s * 32 + vhalf * 16;
        if (vt < kv_end) {
            const int64_t blk = bt[vt / block_size];
            const int64_t e = ((blk * hkv + h) * kPD + vrow) * (int64_t)block_size + vt % block_size;
            if constexpr (FP8) {
                const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(vcv) + e);
                vs[0] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.x, v.y, v_scale));
                vs[1] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.z, v.w, v_scale));
            } else {
                const u16x8* p = reinterpret_cast<const u16x8*>(vc + e);
                vs[0] = p[0];
                vs[1] = p[1];
            }
        } else {
            vs[0] = vs[1] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    };
    auto swrite = [&](int buf) {
        unsigned char* base = lds + buf * kStage;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int u = (kunit + j) ^ (krow & 15);
            *reinterpret_cast<u16x8*>(base + krow * 256 + u * 16) = ks[j];
            *reinterpret_cast<u16x8*>(base + kKImg + vrow * kVPitch + vhalf * 32 + j * 16) = vs[j];
        }
    };

    float m[2] = {-1e30f, -1e30f}, lsum[2] = {0.f, 0.f};
    f32x4 o[2][8];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[mt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (nsteps > 0) {
        gload(0);
        swrite(0);
    }
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        if (s + 1 < nsteps) gload(s + 1);  // in flight under this step's MFMAs
        const unsigned char* base = lds + (s & 1) * kStage;
        const int t0 = s * 32;
        // K fragments, shared by both m-tiles
        bf16x8 kf[2][4];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int row = g * 16 + r;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int u = (4 * c + h4) ^ (row & 15);
                kf[g][c] = *reinterpret_cast<const bf16x8*>(base + row * 256 + u * 16);
            }
        }
        bf16x8 vf[8];
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            const unsigned char* vr = base + kKImg + (dt * 16 + r) * kVPitch;
            const bf16x4 a = *reinterpret_cast<const bf16x4*>(vr + 8 * h4);
            const bf16x4 b = *reinterpret_cast<const bf16x4*>(vr + 32 + 8 * h4);
            vf[dt] = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
        }
        const bool edge = (t0 + 32 > kv_end) || (t0 + 31 > wave_min_pos);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            f32x4 sc[2];
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[g][c], qf[mt][c], acc, 0, 0, 0);
                sc[g] = acc;
            }
            float mx = -INFINITY;
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float v = sc[g][i] * scale_log2;
                    if (edge) {
                        const int tok = t0 + 16 * g + 4 * h4 + i;
                        if (tok >= kv_end || tok > rpos[mt]) v = -INFINITY;
                    } else if (rpos[mt] < 0) {
                        v = -INFINITY;
                    }
                    sc[g][i] = v;
                    mx = fmaxf(mx, v);
                }
            mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
            const float mnew = fmaxf(m[mt], mx);
            const float alpha = exp2f(m[mt] - mnew);
            m[mt] = mnew;
            float ps = 0.f;
            bf16x8 pf;
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float p = exp2f(sc[g][i] - mnew);
                    ps += p;
                    pf[4 * g + i] = (__bf16)p;
                }
            lsum[mt] = lsum[mt] * alpha + ps;
#pragma unroll
            for (int dt = 0; dt < 8; ++dt) {
                o[mt][dt] *= alpha;
                o[mt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[dt], pf, o[mt][dt], 0, 0, 0);
            }
        }
        if (s + 1 < nsteps) swrite((s + 1) & 1);
        __syncthreads();
    }

    // ---- epilogue: normalise and store this wave's rows ----
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        float lt = lsum[mt];
        lt += __shfl_xor(lt, 16, 64);
        lt += __shfl_xor(lt, 32, 64);
        const int R = w * 32 + mt * 16 + r;
        const int tr = rel0 + R / G, hd = h * G + R % G;
        if (tr >= qlen) continue;
        const float inv = lt > 0.f ? 1.f / lt : 0.f;
        uint16_t* op = out + ((int64_t)(qbase + tr) * hq + hd) * kPD + 4 * h4;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            u16x4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = f2bf(o[mt][dt][i] * inv);
            *reinterpret_cast<u16x4*>(op + dt * 16) = v;
        }
    }
}

void launch_attn_prefill(const uint16_t* q, const void* kc, const void* vc, const int32_t* block_table,
                         int bt_stride, const int32_t* q_start, const int32_t* ctx_len, const int32_t* tiles,
                         int ntiles, uint16_t* out, int hq, int hkv, int block_size, float scale, bool fp8,
                         float k_scale, float v_scale, hipStream_t st) {
    if (ntiles == 0) return;
    static bool attr = [] {
        return hipFuncSetAttribute((const void*)attn_prefill_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   2 * kStage) == hipSuccess &&
               hipFuncSetAttribute((const void*)attn_prefill_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   2 * kStage) == hipSuccess;
    }();
    (void)attr;
    const float sl = scale * 1.4426950408889634f;
    if (fp8)
        hipLaunchKernelGGL(attn_prefill_kernel<true>, dim3(ntiles, hkv), dim3(256), 2 * kStage, st, q, kc, vc,
                           block_table, bt_stride, q_start, ctx_len, tiles, ntiles, out, hq, hkv, block_size, sl,
                           k_scale, v_scale);
    else
        hipLaunchKernelGGL(attn_prefill_kernel<false>, dim3(ntiles, hkv), dim3(256), 2 * kStage, st, q, kc, vc,
                           block_table, bt_stride, q_start, ctx_len, tiles, ntiles, out, hq, hkv, block_size, sl,
                           1.f, 1.f);
}

}  // namespace chronos
