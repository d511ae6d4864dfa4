// attention.hip — paged GQA attention for prefill (chunked, causal, varlen) and decode.
//
// One kernel serves both phases.  Work item = (q tile, kv head, kv split):
//   * a q tile is NQT x 16 "rows"; row R = (token rel0 + R / G, q head h*G + R % G), G = Hq / Hkv.  All rows of a tile
//     share one kv head, so every K/V byte a workgroup loads feeds G query heads (GQA reuse in registers).
//   * the 4 waves of a workgroup split the tile's kv range in interleaved 32-token steps; each keeps its own online
//     softmax state and the four are merged through LDS at the end.  Long contexts additionally split the kv range
//     over workgroups (grid.z) and a combine kernel merges the partial (O, lse) pairs (flash-decoding).
//
// MFMA mapping (v_mfma_f32_16x16x32_bf16, cdna_hip_programming.md §3 operand maps):
//   S^T[16 tok][16 rows] = K[16 tok][128] · Q^T  — "swapped" QK^T, 4 MFMAs per 16 tokens (K chunk of 32 dims each).
//       A = K rows straight from the cache (k_cache[blk][h][tok][128], 16 B per lane), B = Q^T fragments in VGPRs.
//       Result: lane l holds S^T[tok 4(l>>4)+i][row l&15] — the query row is the lane, so the row max/sum needs only
//       two xor-shuffles (16, 32) and P never leaves registers.
//   O^T[16 dims][16 rows] += V^T[16 dims][32 tok] · P^T[32 tok][16 rows] — 8 MFMAs per 32 tokens.
//       The k (token) order inside the MFMA is permuted identically on both operands: k = 8h + j <-> token
//       4h + j (j < 4) or 16 + 4h + (j - 4) (j >= 4), which is exactly where the S^T accumulator left P.  V is cached
//       transposed (v_cache[blk][h][dim][tok]) so the A fragment is two 8-byte row reads.
//
// Masking: keys > the row's position (causal) or >= the split end get score -inf; rows with no key yield 0.  V lanes
// of keys past the split end are zeroed so stale cache bytes can never reach the accumulator (p = 0 * NaN guard).
#include "chronos_hip.h"

namespace chronos {

constexpr int kD = 128;
constexpr int kOStride = 132;  // LDS row stride (floats) of the merge buffer: breaks the 512-B row bank aliasing

// One (tile, kv head)'s merge of the nsplit partial outputs (shared by the combine kernel and the in-launch combine).
template <int NQT>
__device__ __forceinline__ void combine_tile(const float* __restrict__ part_o, const float* __restrict__ part_lse,
                                             uint16_t* __restrict__ out, int tile, int h, int rel0, int qbase,
                                             int qlen, int hq, int hkv, int nsplit, int ntiles) {
    constexpr int ROWS = NQT * 16;
    const int G = hq / hkv;
    if (NQT == 1 && rel0 == 0 && qlen * G <= 16) {
        // decode (one query row per sequence, or qlen <= 16 / G tokens of one sequence): only qlen x G of the 16
        // rows are live, so the (row, 8-column group) items take P adjacent lanes each, the lanes split the splits
        // between them and merge through shuffles — P times fewer dependent global-load rounds than one lane walking
        // all nsplit partials (128k decode: 32 splits x 8 kv heads, 17.5 -> a few us per layer)
        const int items = qlen * G * 16;
        const int P = items <= 16 ? 16 : items <= 32 ? 8 : items <= 64 ? 4 : items <= 128 ? 2 : 1;
        const int item = threadIdx.x / P, sub = threadIdx.x % P;
        const bool live = item < items;
        const int row = live ? item >> 4 : 0, c8 = item & 15;
        const int64_t base = ((int64_t)tile * hkv + h) * ROWS + row;
        const int64_t sstride = (int64_t)ntiles * hkv * ROWS;
        float M = -INFINITY;
        if (live)
            for (int s = sub; s < nsplit; s += P) M = fmaxf(M, part_lse[base + s * sstride]);
        for (int o = 1; o < P; o <<= 1) M = fmaxf(M, __shfl_xor(M, o));
        float L = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (live && M > -INFINITY) {
#pragma unroll 4
            for (int s = sub; s < nsplit; s += P) {
                const int64_t prow = base + s * sstride;
                const float l = part_lse[prow];
                const f32x4 a = *reinterpret_cast<const f32x4*>(part_o + prow * kD + c8 * 8);
                const f32x4 b = *reinterpret_cast<const f32x4*>(part_o + prow * kD + c8 * 8 + 4);
                const bool on = l > -INFINITY;  // an empty split's partial row may be stale: never multiply it
                const float f = on ? exp2f(l - M) : 0.f;
                L += f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[j] += on ? a[j] * f : 0.f;
                    acc[4 + j] += on ? b[j] * f : 0.f;
                }
            }
        }
        for (int o = 1; o < P; o <<= 1) {
            L += __shfl_xor(L, o);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += __shfl_xor(acc[j], o);
        }
        if (live && sub == 0) {
            const float inv = L > 0.f ? 1.f / L : 0.f;
            u16x8 ov;
#pragma unroll
            for (int j = 0; j < 8; ++j) ov[j] = f2bf(acc[j] * inv);
            *reinterpret_cast<u16x8*>(out + ((int64_t)(qbase + row / G) * hq + h * G + row % G) * kD + c8 * 8) = ov;
        }
        return;
    }
    for (int idx = threadIdx.x; idx < ROWS * 16; idx += 256) {
        const int row = idx >> 4, c8 = idx & 15;
        const int tr = rel0 + row / G, hd = h * G + row % G;
        if (tr >= qlen) continue;
        float M = -INFINITY;
        for (int s = 0; s < nsplit; ++s)
            M = fmaxf(M, part_lse[(((int64_t)s * ntiles + tile) * hkv + h) * ROWS + row]);
        float L = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (M > -INFINITY) {
            for (int s = 0; s < nsplit; ++s) {
                const int64_t prow = (((int64_t)s * ntiles + tile) * hkv + h) * ROWS + row;
                const float f = exp2f(part_lse[prow] - M);
                if (f == 0.f) continue;
                L += f;
                const float* po = part_o + prow * kD + c8 * 8;
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] += po[j] * f;
            }
        }
        const float inv = L > 0.f ? 1.f / L : 0.f;
        u16x8 ov;
#pragma unroll
        for (int j = 0; j < 8; ++j) ov[j] = f2bf(acc[j] * inv);
        *reinterpret_cast<u16x8*>(out + ((int64_t)(qbase + tr) * hq + hd) * kD + c8 * 8) = ov;
    }
}

template <int NQT, bool FP8, bool PF = false>
__global__ void __launch_bounds__(256, PF ? 2 : 1) paged_attn_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ kcv, const void* __restrict__ vcv,
    const int32_t* __restrict__ block_table, int bt_stride, const int32_t* __restrict__ q_start,
    const int32_t* __restrict__ ctx_len, const int32_t* __restrict__ tiles, uint16_t* __restrict__ out,
    float* __restrict__ part_o, float* __restrict__ part_lse, int hq, int hkv, int block_size, float scale_log2,
    float k_scale, float v_scale, const int32_t* __restrict__ gst, int gn, int* __restrict__ cnt) {
    constexpr int ROWS = NQT * 16;
    if (gate_closed(gst, gn)) return;
    const uint16_t* kc = reinterpret_cast<const uint16_t*>(kcv);
    const uint16_t* vc = reinterpret_cast<const uint16_t*>(vcv);
    const uint8_t* kc8 = reinterpret_cast<const uint8_t*>(kcv);
    const uint8_t* vc8 = reinterpret_cast<const uint8_t*>(vcv);
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sm = smem;                 // [4][ROWS]
    float* sl = sm + 4 * ROWS;        // [4][ROWS]
    float* so = sl + 4 * ROWS;        // [4][ROWS][kOStride]

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, h4 = lane >> 4;
    const int G = hq / hkv;
    const int h = blockIdx.y;
    const int tile = blockIdx.x;
    const int nsplit = gridDim.z;

    int seq, rel0, qbase, qlen;
    if (tiles) {
        seq = tiles[2 * tile];
        rel0 = tiles[2 * tile + 1];
        qbase = q_start[seq];
        qlen = q_start[seq + 1] - qbase;
    } else {  // decode: tile i = sequence i, one query token each
        seq = tile;
        rel0 = 0;
        qbase = tile;
        qlen = 1;
    }
    const int ctx = ctx_len[seq];
    const int ctx0 = ctx - qlen;  // position of the first query token of this sequence's chunk

    int rpos[NQT];
    bf16x8 qf[NQT][4];
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) {
        const int R = qt * 16 + r;
        const int tr = rel0 + R / G, hd = h * G + R % G;
        const bool valid = tr < qlen;
        rpos[qt] = valid ? ctx0 + tr : -1;
        const uint16_t* qp = q + ((int64_t)(qbase + (valid ? tr : 0)) * hq + hd) * kD + 8 * h4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            bf16x8 v = *reinterpret_cast<const bf16x8*>(qp + 32 * c);
            if (!valid) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
            qf[qt][c] = v;
        }
    }
    int last_tr = rel0 + ROWS / G - 1;
    if (last_tr > qlen - 1) last_tr = qlen - 1;
    const int kv_end = ctx0 + last_tr + 1;
    int chunk = (kv_end + nsplit - 1) / nsplit;
    chunk = (chunk + 31) & ~31;
    const int ks = blockIdx.z * chunk;
    const int ke = min(kv_end, ks + chunk);

    float m[NQT], lsum[NQT];
    f32x4 o[NQT][8];
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) {
        m[qt] = -1e30f;
        lsum[qt] = 0.f;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[qt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int32_t* bt = block_table + (int64_t)seq * bt_stride;

    auto load = [&](int t0, bf16x8 (&kf)[2][4], bf16x4 (&vf)[2][8]) {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int tg = t0 + 16 * g;
            if (tg < ke) {
                const int64_t blk = bt[tg / block_size];
                const int off = tg % block_size;
                const int64_t koff = (((blk * hkv + h) * block_size) + off + r) * kD + 8 * h4;
                const int64_t voff = ((blk * hkv + h) * kD) * (int64_t)block_size + off + 4 * h4;
                if constexpr (FP8) {  // 1-byte e4m3 cache, dequantised to the bf16 MFMA operands in registers
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const uint2 v = *reinterpret_cast<const uint2*>(kc8 + koff + 32 * c);
                        kf[g][c] = fp8x8_to_bf16x8(v.x, v.y, k_scale);
                    }
#pragma unroll
                    for (int dt = 0; dt < 8; ++dt)
                        vf[g][dt] = fp8x4_to_bf16x4(
                            *reinterpret_cast<const uint32_t*>(vc8 + voff + (int64_t)(dt * 16 + r) * block_size), v_scale);
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c) kf[g][c] = *reinterpret_cast<const bf16x8*>(kc + koff + 32 * c);
#pragma unroll
                    for (int dt = 0; dt < 8; ++dt)
                        vf[g][dt] = *reinterpret_cast<const bf16x4*>(vc + voff + (int64_t)(dt * 16 + r) * block_size);
                }
            } else {
#pragma unroll
                for (int c = 0; c < 4; ++c) kf[g][c] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                for (int dt = 0; dt < 8; ++dt) vf[g][dt] = bf16x4{0, 0, 0, 0};
            }
        }
    };
    auto compute = [&](int t0, bf16x8 (&kf)[2][4], bf16x4 (&vf)[2][8]) {
        if (t0 + 32 > ke) {  // partial step: zero V of keys past the end (uniform branch)
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (t0 + 16 * g + 4 * h4 + i >= ke)
#pragma unroll
                        for (int dt = 0; dt < 8; ++dt) vf[g][dt][i] = (__bf16)0.f;
        }
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt) {
            f32x4 s[2];
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[g][c], qf[qt][c], acc, 0, 0, 0);
                s[g] = acc;
            }
            float mx = -INFINITY;
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int tok = t0 + 16 * g + 4 * h4 + i;
                    float v = s[g][i] * scale_log2;
                    if (tok >= ke || tok > rpos[qt]) v = -INFINITY;
                    s[g][i] = v;
                    mx = fmaxf(mx, v);
                }
            mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
            const float mnew = fmaxf(m[qt], mx);
            const float alpha = exp2f(m[qt] - mnew);
            m[qt] = mnew;
            float ps = 0.f;
            bf16x8 pf;
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float p = exp2f(s[g][i] - mnew);
                    ps += p;
                    pf[4 * g + i] = (__bf16)p;
                }
            lsum[qt] = lsum[qt] * alpha + ps;
#pragma unroll
            for (int dt = 0; dt < 8; ++dt) {
                o[qt][dt] *= alpha;
                const bf16x8 va = __builtin_shufflevector(vf[0][dt], vf[1][dt], 0, 1, 2, 3, 4, 5, 6, 7);
                o[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pf, o[qt][dt], 0, 0, 0);
            }
        }
    };
    if constexpr (PF) {  // decode over long contexts: the wave's next 32-token step (t0 + 128) in flight under this one
        bf16x8 kA[2][4], kB[2][4];
        bf16x4 vA[2][8], vB[2][8];
        int t0 = ks + w * 32;
        if (t0 < ke) load(t0, kA, vA);
        for (; t0 < ke; t0 += 256) {
            if (t0 + 128 < ke) load(t0 + 128, kB, vB);
            compute(t0, kA, vA);
            if (t0 + 128 >= ke) break;
            if (t0 + 256 < ke) load(t0 + 256, kA, vA);
            compute(t0 + 128, kB, vB);
        }
    } else {
        for (int t0 = ks + w * 32; t0 < ke; t0 += 128) {
            bf16x8 kf[2][4];
            bf16x4 vf[2][8];
            load(t0, kf, vf);
            compute(t0, kf, vf);
        }
    }

    // ---- merge the four waves' (m, l, O) through LDS -----------------------------------------------------------
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) {
        float lt = lsum[qt];
        lt += __shfl_xor(lt, 16, 64);
        lt += __shfl_xor(lt, 32, 64);
        const int row = qt * 16 + r;
        if (h4 == 0) {
            sm[w * ROWS + row] = m[qt];
            sl[w * ROWS + row] = lt;
        }
        float* orow = so + (w * ROWS + row) * kOStride;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) *reinterpret_cast<f32x4*>(orow + dt * 16 + 4 * h4) = o[qt][dt];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < ROWS * 16; idx += 256) {
        const int row = idx >> 4, c8 = idx & 15;
        const int tr = rel0 + row / G, hd = h * G + row % G;
        if (tr >= qlen) continue;
        float M = -1e30f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, sm[ww * ROWS + row]);
        float L = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) {
            const float f = exp2f(sm[ww * ROWS + row] - M);
            L += sl[ww * ROWS + row] * f;
            const float* orow = so + (ww * ROWS + row) * kOStride + c8 * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += orow[j] * f;
        }
        const float inv = L > 0.f ? 1.f / L : 0.f;
        if (nsplit == 1) {
            u16x8 ov;
#pragma unroll
            for (int j = 0; j < 8; ++j) ov[j] = f2bf(acc[j] * inv);
            *reinterpret_cast<u16x8*>(out + ((int64_t)(qbase + tr) * hq + hd) * kD + c8 * 8) = ov;
        } else {
            const int64_t prow = (((int64_t)blockIdx.z * gridDim.x + tile) * hkv + h) * ROWS + row;
            float* po = part_o + prow * kD + c8 * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) po[j] = acc[j] * inv;
            if (c8 == 0) part_lse[prow] = L > 0.f ? M + __log2f(L) : -INFINITY;
        }
    }
    if (nsplit == 1 || cnt == nullptr) return;
    // ---- in-launch flash-decoding combine: the last split of this (tile, head) to finish merges all of them ------
    // cdna_hip_programming.md §5 "In-launch split-K reduction": every wave drains its partial stores, one agent-scope
    // release, a relaxed agent-scope ticket; the last arriver resets the ticket, acquires, and reads every split's
    // partials.  Correct for any placement of the splits over XCDs; saves the separate combine launch.
    int* flag = reinterpret_cast<int*>(sm);  // the merge above is done with sm/sl/so after this barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int* c = cnt + (int64_t)tile * hkv + h;
        const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == nsplit - 1;
        if (last) {
            __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    combine_tile<NQT>(part_o, part_lse, out, tile, h, rel0, qbase, qlen, hq, hkv, nsplit, gridDim.x);
}

// ------------------------------------------------------------------------------------------------------------------
// Long-context decode with a kv split (flash-decoding; the 128k config): the split-over-waves
// kernel above loads K straight into the MFMA layout (16 rows x 64 B per instruction) and V^T as 8-byte pieces, so
// at 128k it issues 24 small loads per 32-token step and wave and runs at the address unit's rate, not HBM's: 125 us
// per layer with bf16 KV and the same with fp8 (half the bytes, the same instructions).  Here every wave streams its
// steps through a private LDS ring with lane-linear 1 KiB LDS-DMA pieces (bf16: 8 K + 8 V^T pieces per step, fp8:
// 4 + 4 — the instruction count follows the bytes), NB steps in flight, and reads the MFMA fragments back with
// conflict-free ds_reads (K chunks XOR-swizzled by row on the source address); fp8 converts with
// v_cvt_scalef32_pk_bf16_fp8 (the cache scales folded into the score scale and the output).  The same token <->
// operand map, softmax and four-wave merge / split combine as paged_attn_kernel<1>, so results agree to rounding.
// ------------------------------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* sd_lds_ptr_t;
typedef __attribute__((address_space(1))) void* sd_gbl_ptr_t;

template <bool FP8>
constexpr int sd_step_bytes() { return FP8 ? 8192 : 16384; }  // K + V^T of one 32-token step (two 16-token pages)
template <bool FP8, int NB>
constexpr int sd_smem() {
    constexpr int ring = 4 * NB * sd_step_bytes<FP8>();
    constexpr int merge = (8 * 16 + 4 * 16 * kOStride) * 4;
    return ring > merge ? ring : merge;
}

// One 1 KiB LDS-DMA piece as inline asm (lane l's 16 bytes from its own source address to LDS dst + 16 l).  hipcc
// cannot see it write LDS, so it does not drain the whole ring (vmcnt(0)) before every ds_read of the step being
// computed; its completion is counted by the kernel's own sd_vmcnt waits (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void sd_dma(const void* gsrc, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds) : "memory");
}

template <int N>
__device__ __forceinline__ void sd_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

template <bool FP8, int NB>
__global__ void __launch_bounds__(256, 1) split_decode_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ kcv, const void* __restrict__ vcv,
    const int32_t* __restrict__ block_table, int bt_stride, const int32_t* __restrict__ ctx_len,
    uint16_t* __restrict__ out, float* __restrict__ part_o, float* __restrict__ part_lse, int hq, int hkv,
    float scale_log2, float k_scale, float v_scale, const int32_t* __restrict__ gst, int gn, int* __restrict__ cnt,
    const int32_t* __restrict__ q_start = nullptr, int mq = 1) {
    // mq > 1: sequence seq has q_start[seq + 1] - q_start[seq] <= 16 / G query tokens (a jump-forward chunk over a
    // long context), its last one at the context's end: MFMA column r = token r / G, q head r % G, and column r's
    // keys stop at ctx - (tokens after it) — one pass over the K/V for all of them instead of one per token
    constexpr int block_size = 16, ROWS = 16;
    constexpr int SB = sd_step_bytes<FP8>();            // bytes of one step in the ring
    constexpr int KB = SB / 2;                          // K part (2 pages); V^T part after it
    constexpr int PK = KB / 1024, PV = KB / 1024;       // LDS-DMA pieces per step: K, V^T
    constexpr int NP = PK + PV;
    if (gate_closed(gst, gn)) return;
    extern __shared__ __attribute__((aligned(1024))) unsigned char sd_smem_raw[];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 15, h4 = lane >> 4;
    const int G = hq / hkv, h = blockIdx.y, seq = blockIdx.x, nsplit = gridDim.z;
    const int ctx = ctx_len[seq];
    const int qb = mq > 1 ? q_start[seq] : seq, ql = mq > 1 ? q_start[seq + 1] - qb : 1;
    const int tq = r / G, gq = r - tq * G;  // column r: token tq of the sequence, q head gq of the group
    const int kcap = tq < ql ? ctx - (ql - 1 - tq) : ctx;
    unsigned char* ring = sd_smem_raw + w * NB * SB;  // this wave's ring of NB steps

    bf16x8 qf[4];
    {
        const bool valid = tq < ql;
        const uint16_t* qp = q + ((int64_t)(qb + (valid ? tq : 0)) * hq + h * G + (valid ? gq : 0)) * kD + 8 * h4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            bf16x8 v = *reinterpret_cast<const bf16x8*>(qp + 32 * c);
            if (!valid) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
            qf[c] = v;
        }
    }
    sd_vmcnt<0>();  // q landed: the ring's waits below count only this wave's DMA pieces
    int chunk = (ctx + nsplit - 1) / nsplit;
    chunk = (chunk + 31) & ~31;
    const int ks = blockIdx.z * chunk;
    const int ke = min(ctx, ks + chunk);
    const int kl = min(ke, kcap);  // this lane's column: keys past it are masked
    const int32_t* bt = block_table + (int64_t)seq * bt_stride;
    const float sl2 = FP8 ? scale_log2 * k_scale : scale_log2;  // fp8: K's cache scale folded into the score scale

    // stage step t0 (wave-uniform) into ring slot j: pages A = t0 / 16, B = A + 1 (past the range: A again, masked)
    auto stage = [&](int t0, int j) {
        const uint32_t dl = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(ring + j * SB));
        const int64_t pa = bt[t0 / block_size];
        const int64_t pb = t0 + block_size < ke ? bt[t0 / block_size + 1] : pa;
        if constexpr (!FP8) {
            // K page: 16 rows x 256 B; piece i of page g = rows 4 i .. +3, lane -> row 4 i + (l >> 4), slot l & 15,
            // holding the row's chunk slot ^ row (the fragment reads then hit 16 distinct slots)
#pragma unroll
            for (int i = 0; i < PK; ++i) {
                const int g = i >> 2, row = 4 * (i & 3) + (lane >> 4);
                const int64_t pg = g ? pb : pa;
                const uint16_t* src = reinterpret_cast<const uint16_t*>(kcv) +
                                      ((pg * hkv + h) * block_size + row) * kD + 8 * ((lane & 15) ^ row);
                sd_dma(src, dl + i * 1024);
            }
            // V^T page: 128 dims x 32 B contiguous in the cache; piece i of page g = dims 32 (i & 3) .. +31
#pragma unroll
            for (int i = 0; i < PV; ++i) {
                const int g = i >> 2;
                const int64_t pg = g ? pb : pa;
                const uint16_t* src = reinterpret_cast<const uint16_t*>(vcv) + (pg * hkv + h) * kD * block_size +
                                      (i & 3) * 512 + 8 * lane;
                sd_dma(src, dl + KB + i * 1024);
            }
        } else {
            // fp8 K page: 16 rows x 128 B = 2 pieces (rows 8 i .. +7, lane -> row 8 i + (l >> 3), slot l & 7 holding
            // chunk slot ^ (row & 7)); V^T page: 128 dims x 16 B = 2 pieces of 64 dims
#pragma unroll
            for (int i = 0; i < PK; ++i) {
                const int g = i >> 1, row = 8 * (i & 1) + (lane >> 3);
                const int64_t pg = g ? pb : pa;
                const uint8_t* src = reinterpret_cast<const uint8_t*>(kcv) + ((pg * hkv + h) * block_size + row) * kD +
                                     16 * ((lane & 7) ^ (row & 7));
                sd_dma(src, dl + i * 1024);
            }
#pragma unroll
            for (int i = 0; i < PV; ++i) {
                const int g = i >> 1;
                const int64_t pg = g ? pb : pa;
                const uint8_t* src = reinterpret_cast<const uint8_t*>(vcv) + (pg * hkv + h) * kD * block_size +
                                     (i & 1) * 1024 + 16 * lane;
                sd_dma(src, dl + KB + i * 1024);
            }
        }
    };

    float m = -1e30f, lsum = 0.f;
    f32x4 o[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int t0, int j) {
        const unsigned char* src = ring + j * SB;
        bf16x8 kf[2][4];
        bf16x4 vf[2][8];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int row = r;  // page g's token row r
            if constexpr (!FP8) {
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    kf[g][c] = *reinterpret_cast<const bf16x8*>(src + g * 4096 + row * 256 + (((4 * c + h4) ^ row) << 4));
#pragma unroll
                for (int dt = 0; dt < 8; ++dt)
                    vf[g][dt] = *reinterpret_cast<const bf16x4*>(src + KB + g * 4096 + (dt * 16 + r) * 32 + 8 * h4);
            } else {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    // dims 32 c + 8 h4 .. +8 = 16-B chunk 2 c + (h4 >> 1), half h4 & 1
                    const uint2 v = *reinterpret_cast<const uint2*>(
                        src + g * 2048 + row * 128 + (((2 * c + (h4 >> 1)) ^ (row & 7)) << 4) + 8 * (h4 & 1));
                    kf[g][c] = fp8x8_to_bf16x8_raw(v.x, v.y);
                }
#pragma unroll
                for (int dt = 0; dt < 8; ++dt) {
                    const uint32_t v = *reinterpret_cast<const uint32_t*>(src + KB + g * 2048 + (dt * 16 + r) * 16 +
                                                                          4 * h4);
                    const bf16x8 e = fp8x8_to_bf16x8_raw(v, 0u);
                    vf[g][dt] = bf16x4{e[0], e[1], e[2], e[3]};
                }
            }
        }
        if (t0 + 32 > ke) {  // partial step: zero V of keys past the end (uniform branch)
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (t0 + 16 * g + 4 * h4 + i >= ke)
#pragma unroll
                        for (int dt = 0; dt < 8; ++dt) vf[g][dt][i] = (__bf16)0.f;
        }
        f32x4 sc[2];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[g][c], qf[c], acc, 0, 0, 0);
            sc[g] = acc;
        }
        float mx = -INFINITY;
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v = sc[g][i] * sl2;
                if (t0 + 16 * g + 4 * h4 + i >= kl) v = -INFINITY;
                sc[g][i] = v;
                mx = fmaxf(mx, v);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m, mx);
        const float alpha = exp2f(m - mnew);
        m = mnew;
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
        lsum = lsum * alpha + ps;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            o[dt] *= alpha;
            const bf16x8 va = __builtin_shufflevector(vf[0][dt], vf[1][dt], 0, 1, 2, 3, 4, 5, 6, 7);
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pf, o[dt], 0, 0, 0);
        }
    };

    // the wave's steps: t0 = ks + 32 w + 128 i; NB of them in flight (ring slot i % NB)
    const int t_first = ks + 32 * w;
    const int nsteps = t_first < ke ? (ke - t_first + 127) / 128 : 0;
#pragma unroll
    for (int i = 0; i < NB - 1; ++i)
        if (i < nsteps) stage(t_first + 128 * i, i);
    for (int i = 0; i < nsteps; ++i) {
        const int ahead = i + NB - 1;
        const bool more = ahead < nsteps;  // wave-uniform
        if (more) stage(t_first + 128 * ahead, ahead % NB);
        // step i landed: the pieces issued after it (up to NB - 1 steps) may stay in flight
        const int newer = min(nsteps - 1 - i, NB - 1);
        if (newer >= 2) sd_vmcnt<2 * NP>();
        else if (newer == 1) sd_vmcnt<NP>();
        else sd_vmcnt<0>();
        compute(t_first + 128 * i, i % NB);
    }
    sd_vmcnt<0>();
    __syncthreads();  // the ring is reused as the merge buffer below

    float* sm = reinterpret_cast<float*>(sd_smem_raw);
    float* sl = sm + 4 * ROWS;
    float* so = sl + 4 * ROWS;
    const float oscale = FP8 ? v_scale : 1.f;  // fp8: V's cache scale applied once to the merged output
    {
        float lt = lsum;
        lt += __shfl_xor(lt, 16, 64);
        lt += __shfl_xor(lt, 32, 64);
        if (h4 == 0) {
            sm[w * ROWS + r] = m;
            sl[w * ROWS + r] = lt;
        }
        float* orow = so + (w * ROWS + r) * kOStride;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) *reinterpret_cast<f32x4*>(orow + dt * 16 + 4 * h4) = o[dt];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < ROWS * 16; idx += 256) {
        const int row = idx >> 4, c8 = idx & 15;
        if (row >= ql * G) continue;
        const int64_t orow_out = (int64_t)(qb + row / G) * hq + h * G + row % G;
        float M = -1e30f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, sm[ww * ROWS + row]);
        float L = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) {
            const float f = exp2f(sm[ww * ROWS + row] - M);
            L += sl[ww * ROWS + row] * f;
            const float* orow = so + (ww * ROWS + row) * kOStride + c8 * 8;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) acc[jj] += orow[jj] * f;
        }
        const float inv = L > 0.f ? oscale / L : 0.f;
        if (nsplit == 1) {
            u16x8 ov;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) ov[jj] = f2bf(acc[jj] * inv);
            *reinterpret_cast<u16x8*>(out + orow_out * kD + c8 * 8) = ov;
        } else {
            const int64_t prow = (((int64_t)blockIdx.z * gridDim.x + seq) * hkv + h) * ROWS + row;
            float* po = part_o + prow * kD + c8 * 8;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) po[jj] = acc[jj] * inv;
            if (c8 == 0) part_lse[prow] = L > 0.f ? M + __log2f(L) : -INFINITY;
        }
    }
    if (nsplit == 1 || cnt == nullptr) return;
    int* flag = reinterpret_cast<int*>(sm);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int* c = cnt + (int64_t)seq * hkv + h;
        const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == nsplit - 1;
        if (last) {
            __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    combine_tile<1>(part_o, part_lse, out, seq, h, 0, qb, ql, hq, hkv, nsplit, gridDim.x);
}

template <int NQT>
__global__ void __launch_bounds__(256) paged_attn_combine_kernel(
    const float* __restrict__ part_o, const float* __restrict__ part_lse, const int32_t* __restrict__ q_start,
    const int32_t* __restrict__ tiles, uint16_t* __restrict__ out, int hq, int hkv, int nsplit, int ntiles,
    const int32_t* __restrict__ gst, int gn, int mq = 1) {
    if (gate_closed(gst, gn)) return;
    const int tile = blockIdx.x, h = blockIdx.y;
    int rel0, qbase, qlen;
    if (tiles) {
        const int seq = tiles[2 * tile];
        rel0 = tiles[2 * tile + 1];
        qbase = q_start[seq];
        qlen = q_start[seq + 1] - qbase;
    } else if (mq > 1) {  // split_decode_kernel's multi-token sequences
        rel0 = 0;
        qbase = q_start[tile];
        qlen = q_start[tile + 1] - qbase;
    } else {
        rel0 = 0;
        qbase = tile;
        qlen = 1;
    }
    combine_tile<NQT>(part_o, part_lse, out, tile, h, rel0, qbase, qlen, hq, hkv, nsplit, ntiles);
}

// ------------------------------------------------------------------------------------------------------------------
// Decode attention for short/medium contexts (no kv split): ONE WAVE per (sequence, kv head) walks the whole context
// in 32-token steps with the next step's K/V already in flight (two register sets), so there is no LDS merge, no
// workgroup barrier and no partial output.  The sequence's block-table entries are fetched 64 at a time into one
// VGPR (lane i = entry i of the window) and read with a shuffle, instead of a dependent global load per 16 tokens.
// With ~100-200-token verdict contexts the split-over-waves kernel above spent most of its time in those fixed
// costs (one 32-token step per wave, then merge); this form is bound by the K/V bytes.  The same MFMAs as
// paged_attn_kernel<1> with the keys of a step permuted inside the MFMA (see load()), so results agree to rounding.
// ------------------------------------------------------------------------------------------------------------------
constexpr float kRescaleThrD = 8.f;  // decode LEAN defer-max threshold (log2 units)

// OCC: minimum workgroups per CU the register allocation must allow (3 = 3 waves per SIMD, <= 168 VGPRs: this
// kernel is bound by K/V load latency, so more waves in flight is more bytes in flight; 1 = unconstrained)
//
// RP (bf16 KV only): RoPE + paged-KV write fused in (the wave's decode step without rope_kv_write).  q is then the
// raw [B, hq + 2 hkv, 128] QKV projection; the wave applies RoPE to its query rows in registers (every lane holds
// both halves of its rotate-half pairs: dims 8 h4 + 32 c with c and c + 2) and writes the new token's (position
// pos[seq], the last of the context) roped K and V into the cache before walking the context.
typedef __attribute__((address_space(3))) void* pd_lds_ptr_t;
typedef __attribute__((address_space(1))) void* pd_gbl_ptr_t;
// dynamic LDS of the bf16 one-register-set variants: one 8 KiB K tile per wave + one 256-B row per wave parking the
// fused-RoPE variant's new K row until its step
constexpr int kPdKlds = 4 * 8192 + 4 * 256;

// KLDS (bf16, one register set): a step's 32 K rows reach the wave through LDS-DMA (eight lane-linear 1 KiB pieces =
// 4 whole 256-B rows each, into the wave's private 8 KiB, XOR-swizzled on the source address) and are read back in
// the MFMA layout with conflict-free ds_read_b128.  Loaded straight into the MFMA layout each instruction touches 16
// rows x 64 B, which the L2 -> CU path serves at ~18 B/clk per CU against ~60 for lane-linear LDS-DMA pieces
// (csrc/microbench/l2_feed.hip, profiles/r3s2_decode_attn.md).
template <bool FP8, bool PF, bool LEAN, int OCC, bool RP = false, bool KL = true>
__global__ void __launch_bounds__(256, OCC) paged_decode_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ kcv, const void* __restrict__ vcv,
    const int32_t* __restrict__ block_table, int bt_stride, const int32_t* __restrict__ ctx_len,
    uint16_t* __restrict__ out, int nitems, int hq, int hkv, float scale_log2, float k_scale, float v_scale,
    const int32_t* __restrict__ gst, int gn, const int32_t* __restrict__ pos = nullptr,
    const float* __restrict__ cos_sin = nullptr, const int32_t* __restrict__ casc = nullptr,
    const uint16_t* __restrict__ opre = nullptr, const float* __restrict__ lpre = nullptr) {
    static_assert(!(RP && FP8), "fused RoPE / KV write: bf16 KV only");
    constexpr bool KLDS = KL && !FP8 && !PF;  // KL = false: K straight to VGPRs (A/B knob decode_klds)
    extern __shared__ __attribute__((aligned(1024))) unsigned char pd_smem[];
    constexpr int block_size = 16;
    if (gate_closed(gst, gn)) return;  // the engine's page size; compile-time so every K/V address is base + immediate
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane tells hipcc so, so ctx / pos / the table window are scalar loads
    // and the step loop is a scalar loop instead of an exec-masked one (168 -> 161 VGPRs, no scratch)
    const int item = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (item >= nitems) return;  // whole wave; the kernel has no workgroup-level synchronisation
    const uint16_t* kc = reinterpret_cast<const uint16_t*>(kcv);
    const uint16_t* vc = reinterpret_cast<const uint16_t*>(vcv);
    const uint8_t* kc8 = reinterpret_cast<const uint8_t*>(kcv);
    const uint8_t* vc8 = reinterpret_cast<const uint8_t*>(vcv);
    const int seq = item / hkv, h = item - seq * hkv;
    const int r = lane & 15, h4 = lane >> 4, G = hq / hkv;
    unsigned char* kl = pd_smem + (threadIdx.x >> 6) * 8192;  // KLDS: this wave's K tile (32 rows x 256 B)
    // KLDS swizzle: row t's 16-B chunk q sits in slot q ^ kswz(t); the fragment rows of one ds_read (8 (r >> 2) + 4 g
    // + (r & 3), r = 0..15) map to kswz = r, 16 distinct slots of a 256-B bank row
    auto kswz = [](int t) { return (t & 3) | ((t >> 3) << 2); };
    const int ctx = ctx_len[seq];
    const int32_t* bt = block_table + (int64_t)seq * bt_stride;
    const int nblk = (ctx + block_size - 1) / block_size;
    int win = 0;
    // the first 64 block-table entries without waiting for ctx (entries past the context are never shuffled out):
    // the table load, ctx and pos all issue together instead of as a ctx -> table dependent pair
    int btv = lane < bt_stride ? bt[lane] : 0;

    // cascade (shared prefix): a sequence whose first P blocks are the cascade prefix (casc[1..P]) and that has
    // tokens past it starts its walk at token 16 P; casc_prefix_kernel already attended its rows over the prefix and
    // left (normalised O, log2-sum-exp) for the merge after the loop.  The producer makes the same test.
    int t_start = 0;
    bool cmem = false;
    if (casc != nullptr) {
        const int P = casc[0];
        if (P > 0 && ctx > 16 * P) {
            const int cb = lane < P ? casc[1 + lane] : 0;
            cmem = __all(lane >= P || btv == cb);
        }
        if (cmem) t_start = 16 * P;
    }
    const int tb = t_start & 31;  // the 32-token steps start at t_start: offset of the step grid

    const int nh = hq + 2 * hkv;  // RP: heads per token row of the QKV projection
    const int pnew = RP ? pos[seq] : 0;
    const float* cs = RP ? cos_sin + (int64_t)pnew * kD : nullptr;
    // rotate-half RoPE of one lane's 32 dims (chunks c = 0..3 at 8 h4 + 32 c; pairs (0, 2) and (1, 3)), rounded to
    // bf16 exactly as rope_kv_write_kernel does
    auto rope4 = [&](bf16x8 (&x)[4]) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int d0 = 32 * c + 8 * h4;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float co = cs[d0 + j], si = cs[64 + d0 + j];
                const float x1 = (float)x[c][j], x2 = (float)x[c + 2][j];
                x[c][j] = (__bf16)(x1 * co - x2 * si);
                x[c + 2][j] = (__bf16)(x2 * co + x1 * si);
            }
        }
    };

    bf16x8 qf[4];
    {
        const bool valid = r < G;
        const uint16_t* qp = RP ? q + ((int64_t)seq * nh + h * G + (valid ? r : 0)) * kD + 8 * h4
                                : q + ((int64_t)seq * hq + h * G + (valid ? r : 0)) * kD + 8 * h4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            bf16x8 v = *reinterpret_cast<const bf16x8*>(qp + 32 * c);
            if (!valid) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
            qf[c] = v;
        }
        if constexpr (RP) rope4(qf);
    }
    // RP + KLDS: the new token's roped K is parked in the wave's spare LDS row (not in VGPRs) and copied into the K tile
    // of its step after that step's DMA lands (the DMA may still fetch the pre-write bytes from the cache)
    const int u = (pnew - tb) & 31;  // the new token's slot in its 32-token step (token <-> lane map: load() below)
    const bool kwriter = RP && r == 4 * (u >> 3) + (u & 3);
    unsigned char* kpark = pd_smem + 4 * 8192 + (threadIdx.x >> 6) * 256;
    if constexpr (RP) {
        // The new token's K (roped) and V go to the cache before the loop.  Each element is written by the very lane
        // that later loads it (K: lane (r = slot, h4); V^T: lane (r, h4 = slot / 4)), so same-thread ordering makes
        // the loop read the fresh values; no other wave touches this sequence's private last block.
        const int tn = pnew & (block_size - 1);
        const int64_t blkn = pnew / block_size < 64 ? __shfl(btv, pnew / block_size, 64) : bt[pnew / block_size];
        const uint16_t* row = q + (int64_t)seq * nh * kD;
        if (kwriter) {
            const uint16_t* kr = row + (int64_t)(hq + h) * kD + 8 * h4;
            bf16x8 kn[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) kn[c] = *reinterpret_cast<const bf16x8*>(kr + 32 * c);
            rope4(kn);
            uint16_t* kdst = const_cast<uint16_t*>(kc) + (((blkn * hkv + h) * block_size) + tn) * kD + 8 * h4;
#pragma unroll
            for (int c = 0; c < 4; ++c) *reinterpret_cast<bf16x8*>(kdst + 32 * c) = kn[c];
            if constexpr (KLDS) {
#pragma unroll
                for (int c = 0; c < 4; ++c) *reinterpret_cast<bf16x8*>(kpark + (((4 * c + h4) ^ kswz(u)) << 4)) = kn[c];
            }
        }
        if (h4 == (u >> 3)) {
            const uint16_t* vr = row + (int64_t)(hq + hkv + h) * kD + r;
            uint16_t* vdst = const_cast<uint16_t*>(vc) + ((blkn * hkv + h) * kD) * (int64_t)block_size + tn;
#pragma unroll
            for (int dt = 0; dt < 8; ++dt) vdst[(int64_t)(dt * 16 + r) * block_size] = vr[16 * dt];
        }
    }

    // One 32-token step = pages A (tokens 0-15) and B (16-31).  Token <-> lane map, chosen so that every lane's 8 P
    // values are 8 CONSECUTIVE tokens: MFMA g's row R holds token 8 (R >> 2) + 4 g + (R & 3), so lane (r, h4)'s
    // accumulator i of S^T[g] is token 8 h4 + 4 g + i and its PV operand element j is token 8 h4 + j — one 16-B V^T
    // load per (lane, 16 dims) instead of two 8-B ones (8 V loads per step instead of 16; the texture addresser was
    // 70-75 % busy on the wave's decode shape, profiles/r3s2_decode_attn_pmc.txt).
    auto load = [&](int t0, bf16x8 (&kf)[2][4], bf16x8 (&vf)[8]) {
        if (t0 < ctx) {
            const int bi = t0 / block_size;  // page A (B = bi + 1): both must sit in the 64-entry window
            if (bi + 1 >= win + 64) {  // wave-uniform: the window of 64 block-table entries from page A on
                win = bi;
                btv = win + lane < nblk ? bt[win + lane] : 0;
            }
            const int64_t blkA = __shfl(btv, bi - win, 64);
            // past the context the B lanes re-read page A (valid memory); those tokens are masked in step()
            const int64_t blkB = t0 + block_size < ctx ? (int64_t)__shfl(btv, bi + 1 - win, 64) : blkA;
            if constexpr (KLDS) {
                // piece i = step rows 4 i .. 4 i + 3, lane l -> row 4 i + (l >> 4), slot l & 15 <- chunk slot ^ kswz
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int t = 4 * i + (lane >> 4);
                    const int64_t pg = t < 16 ? blkA : blkB;
                    const uint16_t* src = kc + (((pg * hkv + h) * block_size) + (t & 15)) * kD + 8 * ((lane & 15) ^ kswz(t));
                    __builtin_amdgcn_global_load_lds((pd_gbl_ptr_t)src, (pd_lds_ptr_t)(kl + i * 1024), 16, 0, 0);
                }
            }
            const int64_t kblk = r < 8 ? blkA : blkB;
#pragma unroll
            for (int g = 0; KLDS ? false : g < 2; ++g) {
                const int off = (8 * (r >> 2) + 4 * g + (r & 3)) & (block_size - 1);
                const int64_t koff = (((kblk * hkv + h) * block_size) + off) * kD + 8 * h4;
                if constexpr (FP8) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const uint2 v = *reinterpret_cast<const uint2*>(kc8 + koff + 32 * c);
                        kf[g][c] = fp8x8_to_bf16x8(v.x, v.y, k_scale);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c) kf[g][c] = *reinterpret_cast<const bf16x8*>(kc + koff + 32 * c);
                }
            }
            const int64_t vblk = h4 < 2 ? blkA : blkB;
            const int64_t voff = ((vblk * hkv + h) * kD) * (int64_t)block_size + 8 * (h4 & 1);
            if constexpr (FP8) {
#pragma unroll
                for (int dt = 0; dt < 8; ++dt) {
                    const uint2 v = *reinterpret_cast<const uint2*>(vc8 + voff + (int64_t)(dt * 16 + r) * block_size);
                    vf[dt] = fp8x8_to_bf16x8(v.x, v.y, v_scale);
                }
            } else {
#pragma unroll
                for (int dt = 0; dt < 8; ++dt)
                    vf[dt] = *reinterpret_cast<const bf16x8*>(vc + voff + (int64_t)(dt * 16 + r) * block_size);
            }
        } else {
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int c = 0; c < 4; ++c) kf[g][c] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int dt = 0; dt < 8; ++dt) vf[dt] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    };

    float m = -1e30f, lsum = 0.f;
    f32x4 o[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto step = [&](int t0, bf16x8 (&kf)[2][4], bf16x8 (&vf)[8]) {
        if constexpr (KLDS) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's K pieces are in LDS (and V in VGPRs)
            if (RP && t0 == pnew - u && kwriter) {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int o = ((4 * c + h4) ^ kswz(u)) << 4;
                    *reinterpret_cast<bf16x8*>(kl + u * 256 + o) = *reinterpret_cast<const bf16x8*>(kpark + o);
                }
            }
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    kf[g][c] = *reinterpret_cast<const bf16x8*>(kl + (8 * (r >> 2) + 4 * g + (r & 3)) * 256 +
                                                                (((4 * c + h4) ^ r) << 4));
        }
        if (t0 + 32 > ctx) {  // partial step: zero V of keys past the end (uniform branch)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (t0 + 8 * h4 + j >= ctx)
#pragma unroll
                    for (int dt = 0; dt < 8; ++dt) vf[dt][j] = (__bf16)0.f;
        }
        f32x4 s[2];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[g][c], qf[c], acc, 0, 0, 0);
            s[g] = acc;
        }
        float mx = -INFINITY;
        float alpha = 1.f;
        float ps = 0.f;
        bf16x8 pf;
        if constexpr (LEAN) {
            // VALU-lean form (as the flash prefill's LEAN): raw scores, masking only in the partial last step, the
            // scale applied to the max and fused into the exponent's fma, raw v_exp_f32, and the defer-max rescale
            // (O and l rescaled only when the max grows past kRescaleThrD in log2 units: p <= 2^8 otherwise).
            if (t0 + 32 > ctx) {
                const int lim = ctx - (t0 + 8 * h4);
#pragma unroll
                for (int g = 0; g < 2; ++g)
#pragma unroll
                    for (int i = 0; i < 4; ++i) s[g][i] = (4 * g + i) >= lim ? -INFINITY : s[g][i];
            }
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) mx = fmaxf(mx, s[g][i]);
            mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * scale_log2;
            if (__any(mx > m + kRescaleThrD)) {
                const float mnew = fmaxf(m, mx);
                alpha = __builtin_amdgcn_exp2f(m - mnew);
                m = mnew;
#pragma unroll
                for (int dt = 0; dt < 8; ++dt) o[dt] *= alpha;
            }
            const float nm = -m;
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float p = __builtin_amdgcn_exp2f(fmaf(s[g][i], scale_log2, nm));
                    ps += p;
                    pf[4 * g + i] = (__bf16)p;
                }
            lsum = lsum * alpha + ps;
#pragma unroll
            for (int dt = 0; dt < 8; ++dt) o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[dt], pf, o[dt], 0, 0, 0);
            return;
        }
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v = s[g][i] * scale_log2;
                if (t0 + 8 * h4 + 4 * g + i >= ctx) v = -INFINITY;
                s[g][i] = v;
                mx = fmaxf(mx, v);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m, mx);
        alpha = exp2f(m - mnew);
        m = mnew;
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float p = exp2f(s[g][i] - mnew);
                ps += p;
                pf[4 * g + i] = (__bf16)p;
            }
        lsum = lsum * alpha + ps;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            o[dt] *= alpha;
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[dt], pf, o[dt], 0, 0, 0);
        }
    };

    if constexpr (PF) {  // next step's K/V in flight while this one computes (two register sets, 1 wave/SIMD)
        bf16x8 kA[2][4], kB[2][4];
        bf16x8 vA[8], vB[8];
        load(t_start, kA, vA);
        for (int t0 = t_start; t0 < ctx; t0 += 64) {
            if (t0 + 32 < ctx) load(t0 + 32, kB, vB);
            step(t0, kA, vA);
            if (t0 + 32 >= ctx) break;
            if (t0 + 64 < ctx) load(t0 + 64, kA, vA);
            step(t0 + 32, kB, vB);
        }
    } else {  // one register set: latency hidden by occupancy instead (3 waves/SIMD)
        bf16x8 kA[2][4];
        bf16x8 vA[8];
        for (int t0 = t_start; t0 < ctx; t0 += 32) {
            load(t0, kA, vA);
            step(t0, kA, vA);
        }
    }

    float lt = lsum;
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    if (r < G && cmem) {
        // merge with the prefix part: out = (o 2^(m - M) + Op l_p 2^(m_p - M)) / (l 2^(m - M) + l_p 2^(m_p - M)),
        // M = max(m, lse_p), with the producer's Op = its O / l_p and lse_p = m_p + log2 l_p (scaled log2 units)
        const int64_t row = (int64_t)seq * hq + h * G + r;
        const float lp = lpre[row];
        const float M = fmaxf(m, lp);
        const float a = exp2f(m - M), b = exp2f(lp - M);
        const float inv = 1.f / (lt * a + b);
        const uint16_t* pp = opre + row * kD + 4 * h4;
        uint16_t* op = out + row * kD + 4 * h4;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            const u16x4 pv = *reinterpret_cast<const u16x4*>(pp + 16 * dt);
            u16x4 ov;
#pragma unroll
            for (int i = 0; i < 4; ++i) ov[i] = f2bf((o[dt][i] * a + bf2f(pv[i]) * b) * inv);
            *reinterpret_cast<u16x4*>(op + 16 * dt) = ov;
        }
    } else if (r < G) {
        const float inv = lt > 0.f ? 1.f / lt : 0.f;
        uint16_t* op = out + ((int64_t)seq * hq + h * G + r) * kD + 4 * h4;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            u16x4 ov;
#pragma unroll
            for (int i = 0; i < 4; ++i) ov[i] = f2bf(o[dt][i] * inv);
            *reinterpret_cast<u16x4*>(op + 16 * dt) = ov;
        }
    }
}

// ------------------------------------------------------------------------------------------------------------------
// Cascade decode attention, producer.  The wave's chains all start with the same prompt template,
// so the leading KV blocks of every decode row are the SAME physical blocks (prefix cache).  The one-wave-per-(seq,
// kv head) decode kernel re-reads them once per row; here each wave attends 16 query rows of ONE kv head — the G q
// heads of 16 / G sequences — over the shared prefix tokens [0, 16 P) with the same MFMA mapping (S^T = K · Q^T, P
// kept in registers, O^T += V^T · P^T), so the prefix K/V bytes are read once per 16 / G rows instead of once per row
// and every MFMA row is a live query row (the decode kernel uses G of its 16).  Per member row it leaves the normalised
// O (bf16) and lse = m + log2 l (scaled log2 units); paged_decode_kernel then walks only tokens >= 16 P and merges.
// Membership (same test in both kernels): the sequence's first P block-table entries equal casc[1..P] and its context
// is longer than the prefix.  casc[0] = P (0: off).  RP: q is the raw QKV projection, RoPE'd here per row.
// ------------------------------------------------------------------------------------------------------------------
template <bool RP>
__global__ void __launch_bounds__(256) casc_prefix_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ casc, const int32_t* __restrict__ block_table, int bt_stride,
    const int32_t* __restrict__ ctx_len, uint16_t* __restrict__ opre, float* __restrict__ lpre, int n, int hq,
    int hkv, float scale_log2, const int32_t* __restrict__ gst, int gn, const int32_t* __restrict__ pos,
    const float* __restrict__ cos_sin) {
    constexpr int block_size = 16;
    if (gate_closed(gst, gn)) return;
    const int P = casc[0];
    if (P <= 0) return;
    const int L = block_size * P;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int h = blockIdx.y, G = hq / hkv, SPW = 16 / G;
    const int r = lane & 15, h4 = lane >> 4;
    const int seq = (blockIdx.x * 4 + wv) * SPW + r / G;  // this lane's query row: (seq, head)
    const int head = h * G + r % G;
    bool mem = seq < n;
    if (mem) {
        mem = ctx_len[seq] > L;
        const int32_t* bt = block_table + (int64_t)seq * bt_stride;
        for (int j = 0; j < P; ++j) mem = mem && bt[j] == casc[1 + j];
    }
    if (!__any(mem)) return;  // whole wave: no member row

    bf16x8 qf[4];
    {
        const int nh = RP ? hq + 2 * hkv : hq;
        const uint16_t* qp = q + ((int64_t)(mem ? seq : 0) * nh + head) * kD + 8 * h4;
#pragma unroll
        for (int c = 0; c < 4; ++c) qf[c] = *reinterpret_cast<const bf16x8*>(qp + 32 * c);
        if constexpr (RP) {
            const float* cs = cos_sin + (int64_t)(mem ? pos[seq] : 0) * kD;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int d0 = 32 * c + 8 * h4;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float co = cs[d0 + j], si = cs[64 + d0 + j];
                    const float x1 = (float)qf[c][j], x2 = (float)qf[c + 2][j];
                    qf[c][j] = (__bf16)(x1 * co - x2 * si);
                    qf[c + 2][j] = (__bf16)(x2 * co + x1 * si);
                }
            }
        }
        if (!mem) {
#pragma unroll
            for (int c = 0; c < 4; ++c) qf[c] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }

    float m = -1e30f, lsum = 0.f;
    f32x4 o[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int t0 = 0; t0 < L; t0 += 32) {
        // pages A (tokens t0 .. +15) and B (+16 .. +31); past the prefix B re-reads A (masked below)
        const int64_t blkA = casc[1 + t0 / block_size];
        const int64_t blkB = t0 + block_size < L ? casc[2 + t0 / block_size] : blkA;
        bf16x8 kf[2][4], vf[8];
        const int64_t kblk = r < 8 ? blkA : blkB;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int off = (8 * (r >> 2) + 4 * g + (r & 3)) & (block_size - 1);
            const int64_t koff = (((kblk * hkv + h) * block_size) + off) * kD + 8 * h4;
#pragma unroll
            for (int c = 0; c < 4; ++c) kf[g][c] = *reinterpret_cast<const bf16x8*>(kc + koff + 32 * c);
        }
        const int64_t vblk = h4 < 2 ? blkA : blkB;
        const int64_t voff = ((vblk * hkv + h) * kD) * (int64_t)block_size + 8 * (h4 & 1);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
            vf[dt] = *reinterpret_cast<const bf16x8*>(vc + voff + (int64_t)(dt * 16 + r) * block_size);
        f32x4 sc[2];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[g][c], qf[c], acc, 0, 0, 0);
            sc[g] = acc;
        }
        // lane (r, h4): S^T token 8 h4 + 4 g + i of row r; PV operand element j = token 8 h4 + j (decode kernel map)
        if (t0 + 32 > L) {
            const int lim = L - (t0 + 8 * h4);
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) sc[g][i] = (4 * g + i) >= lim ? -INFINITY : sc[g][i];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j >= lim)
#pragma unroll
                    for (int dt = 0; dt < 8; ++dt) vf[dt][j] = (__bf16)0.f;
        }
        float mx = -INFINITY;
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) mx = fmaxf(mx, sc[g][i]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * scale_log2;
        const float mnew = fmaxf(m, mx);
        const float alpha = exp2f(m - mnew);
        m = mnew;
        float ps = 0.f;
        bf16x8 pf;
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float p = exp2f(fmaf(sc[g][i], scale_log2, -m));
                ps += p;
                pf[4 * g + i] = (__bf16)p;
            }
        lsum = lsum * alpha + ps;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            o[dt] *= alpha;
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[dt], pf, o[dt], 0, 0, 0);
        }
    }
    float lt = lsum;
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    if (mem) {
        const int64_t row = (int64_t)seq * hq + head;
        const float inv = 1.f / lt;  // lt >= 1: the row's max key contributes 2^0
        uint16_t* op = opre + row * kD + 4 * h4;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            u16x4 ov;
#pragma unroll
            for (int i = 0; i < 4; ++i) ov[i] = f2bf(o[dt][i] * inv);
            *reinterpret_cast<u16x4*>(op + 16 * dt) = ov;
        }
        if (h4 == 0) lpre[row] = m + __log2f(lt);
    }
}

// Fused decode step (RP): RoPE + paged-KV write + one-wave-per-(seq, kv head) attention.  Returns false (nothing
// launched) off the shapes the one-wave kernel serves; the caller then runs rope_kv_write + launch_paged_attn.
bool launch_decode_attn_rope(const uint16_t* qkv, const int32_t* pos, const float* cos_sin, void* kc, void* vc,
                             const int32_t* block_table, int bt_stride, const int32_t* ctx_len, uint16_t* out, int n,
                             int hq, int hkv, int block_size, float scale, hipStream_t st, const int32_t* casc,
                             uint16_t* opre, float* lpre) {
    const int nitems = n * hkv;
    if (n == 0 || hq / hkv > 16 || block_size != 16 || nitems < knob("decode_min_items", 1024) ||
        knob("decode_attn_legacy", 0) ||
        knob("decode_pf", 0) || !knob("decode_lean", 1) || !knob("decode_rope_fused", 1))
        return false;
    const float scale_log2 = scale * 1.4426950408889634f;
    if (casc != nullptr) {  // the shared-prefix part first; the decode kernel merges it
        const int G = hq / hkv;
        const dim3 grid((n + 4 * (16 / G) - 1) / (4 * (16 / G)), hkv);
        hipLaunchKernelGGL(casc_prefix_kernel<true>, grid, dim3(256), 0, st, qkv, (const uint16_t*)kc,
                           (const uint16_t*)vc, casc, block_table, bt_stride, ctx_len, opre, lpre, n, hq, hkv,
                           scale_log2, CHRONOS_GATE, pos, cos_sin);
    }
    if (!knob("decode_klds", 1))
        hipLaunchKernelGGL((paged_decode_kernel<false, false, true, 3, true, false>), dim3((nitems + 3) / 4),
                           dim3(256), 0, st, qkv, kc, vc, block_table, bt_stride, ctx_len, out, nitems, hq, hkv,
                           scale_log2, 1.f, 1.f, CHRONOS_GATE, pos, cos_sin, casc, opre, lpre);
    else if (knob("decode_occ3", 1))
        hipLaunchKernelGGL((paged_decode_kernel<false, false, true, 3, true>), dim3((nitems + 3) / 4), dim3(256), kPdKlds,
                           st, qkv, kc, vc, block_table, bt_stride, ctx_len, out, nitems, hq, hkv, scale_log2, 1.f,
                           1.f, CHRONOS_GATE, pos, cos_sin, casc, opre, lpre);
    else
        hipLaunchKernelGGL((paged_decode_kernel<false, false, true, 1, true>), dim3((nitems + 3) / 4), dim3(256), kPdKlds,
                           st, qkv, kc, vc, block_table, bt_stride, ctx_len, out, nitems, hq, hkv, scale_log2, 1.f,
                           1.f, CHRONOS_GATE, pos, cos_sin, casc, opre, lpre);
    return true;
}

// Split-completion tickets for the in-launch combine: one zeroed int per (tile, kv head), per device, allocated once by
// attn_init() before any graph capture (hipMalloc is not capturable); every launch leaves them at zero again.
constexpr int64_t kTicketCap = 1 << 20;
static int* g_tickets[64] = {nullptr};

void attn_init() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || g_tickets[dev]) return;
    int* p = nullptr;
    if (hipMalloc(&p, kTicketCap * sizeof(int)) != hipSuccess) return;
    if (hipMemset(p, 0, kTicketCap * sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(p);
        return;
    }
    g_tickets[dev] = p;
}

static int* tickets_for(int64_t n) {
    int dev = 0;
    if (n > kTicketCap || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    return knob("attn_inkernel_combine", 1) ? g_tickets[dev] : nullptr;
}

size_t paged_attn_smem(int nqt) { return (size_t)(8 * nqt * 16 + 4 * nqt * 16 * kOStride) * sizeof(float); }

void launch_paged_attn(const uint16_t* q, const void* kc, const void* vc, const int32_t* block_table, int bt_stride,
                       const int32_t* q_start, const int32_t* ctx_len, const int32_t* tiles, int ntiles, int nqt,
                       int nsplit, uint16_t* out, float* part_o, float* part_lse, int hq, int hkv, int block_size,
                       float scale, bool fp8, float k_scale, float v_scale, hipStream_t st, int max_q) {
    if (ntiles == 0) return;
    const float scale_log2 = scale * 1.4426950408889634f;
    // decode without a kv split and enough (seq, kv head) items to fill the chip one wave each; fewer items keep the
    // split-over-waves form (profiles/r1_attn_decode.json: B=64 x 1k ctx is 1.5x faster there, B >= 256 at 128-512
    // ctx 1.0-1.3x slower).  Threshold 2048 -> 1024 items in r5: the T = 128 bucket at 200-token contexts runs
    // 21.7 vs 26.7 us per layer on the one-wave kernel, 6.14 -> 5.98 ms per forward; T = 64 (512 items) is neutral
    // (profiles/r5/decode_min_items_ab.jsonl)
    const int nitems = ntiles * hkv;
    if (tiles == nullptr && nqt == 1 && nsplit == 1 && max_q == 1 && hq / hkv <= 16 && block_size == 16 &&
        nitems >= knob("decode_min_items", 1024)) {
        if (knob("decode_attn_legacy", 0)) goto legacy;  // A/B against the split-over-waves kernel
        const int pf = knob("decode_pf", 0);
        const bool lean = knob("decode_lean", 1) != 0;
        const bool occ3 = knob("decode_occ3", 1) != 0;
#define PD_LAUNCH(F, P, L, O)                                                                                   \
    hipLaunchKernelGGL((paged_decode_kernel<F, P, L, O>), dim3((nitems + 3) / 4), dim3(256), (!F && !P) ? kPdKlds : 0, \
                       st, q, kc, vc,                                                                               \
                       block_table, bt_stride, ctx_len, out, nitems, hq, hkv, scale_log2, k_scale, v_scale, CHRONOS_GATE)
#define PD_OCC(F, L)                                                                                            \
    if (!F && !knob("decode_klds", 1) && occ3)                                                                  \
        hipLaunchKernelGGL((paged_decode_kernel<F, false, L, 3, false, false>), dim3((nitems + 3) / 4), dim3(256), \
                           0, st, q, kc, vc, block_table, bt_stride, ctx_len, out, nitems, hq, hkv, scale_log2,   \
                           k_scale, v_scale, CHRONOS_GATE);                                                       \
    else if (occ3) PD_LAUNCH(F, false, L, 3);                                                                   \
    else PD_LAUNCH(F, false, L, 1);
        if (fp8) {
            if (pf) PD_LAUNCH(true, true, false, 1);
            else if (lean) { PD_OCC(true, true) }
            else { PD_OCC(true, false) }
        } else {
            if (pf) PD_LAUNCH(false, true, false, 1);
            else if (lean) { PD_OCC(false, true) }
            else { PD_OCC(false, false) }
        }
#undef PD_OCC
#undef PD_LAUNCH
        return;
    }
legacy:
    const dim3 grid(ntiles, hkv, nsplit), block(256);
    if (tiles == nullptr && nqt == 1 && hq / hkv <= 16 && block_size == 16 &&
        (max_q > 1 || (nsplit > 1 && knob("split_lds", 1)))) {
        // long-context decode: the LDS-staged split kernel (lane-linear LDS-DMA, NB steps in flight per wave)
        int* cnt = nsplit <= knob("sd_inkernel_max_split", 4) ? tickets_for((int64_t)ntiles * hkv) : nullptr;
        int nb = knob("split_lds_nb", 0);  // ring depth (steps in flight per wave); <= 0: the default
        if (nb <= 0) nb = 2;  // (r5 sweep after the parallel combine: fp8 nb2 52.5 us vs nb3 54.7 at 128k)
#define SD_LAUNCH(F, NB)                                                                                          \
    {                                                                                                           \
        constexpr int shm = sd_smem<F, NB>();                                                                    \
        auto kern = split_decode_kernel<F, NB>;                                                                  \
        static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,     \
                                               shm) == hipSuccess;                                              \
        (void)attr;                                                                                             \
        hipLaunchKernelGGL(kern, grid, block, shm, st, q, kc, vc, block_table, bt_stride, ctx_len, out, part_o,   \
                           part_lse, hq, hkv, scale_log2, k_scale, v_scale, CHRONOS_GATE, cnt, q_start, max_q); \
    }
        if (fp8) {
            if (nb >= 4) SD_LAUNCH(true, 4) else if (nb == 3) SD_LAUNCH(true, 3) else SD_LAUNCH(true, 2)
        } else {
            if (nb >= 2) SD_LAUNCH(false, 2) else SD_LAUNCH(false, 1)
        }
#undef SD_LAUNCH
        if (nsplit > 1 && cnt == nullptr)
            hipLaunchKernelGGL(paged_attn_combine_kernel<1>, dim3(ntiles, hkv), block, 0, st, part_o, part_lse,
                               q_start, tiles, out, hq, hkv, nsplit, ntiles, CHRONOS_GATE, max_q);
        return;
    }
    // in-launch combine (last split merges) only for a few splits: with many splits the per-workgroup agent-scope
    // release + ticket costs more than the separate combine launch it saves (128k single-sequence decode, 64 splits:
    // 147 vs 132 us per layer; profiles/r2_attn_split_combine.jsonl)
    int* cnt = nsplit > 1 && nsplit <= knob("inkernel_combine_max_split", 4) ? tickets_for((int64_t)ntiles * hkv)
                                                                              : nullptr;
    const size_t sh = paged_attn_smem(nqt);
#define PA_LAUNCH(N, F, ...)                                                                                    \
    hipLaunchKernelGGL((paged_attn_kernel<N, F, ##__VA_ARGS__>), grid, block, sh, st, q, kc, vc, block_table,       \
                       bt_stride, q_start, ctx_len, tiles, out, part_o, part_lse, hq, hkv, block_size, scale_log2,   \
                       k_scale, v_scale, CHRONOS_GATE, cnt)
    if (nqt == 1) {
        // decode with a kv split (long contexts): register-prefetch the wave's next 32-token step
        const bool pf1 = tiles == nullptr && nsplit > 1 && knob("split_pf", 1) != 0;
        if (pf1) {
            if (fp8) PA_LAUNCH(1, true, true); else PA_LAUNCH(1, false, true);
        } else if (fp8) PA_LAUNCH(1, true); else PA_LAUNCH(1, false);
    } else {
        static bool attr = [] {  // > 64 KiB dynamic LDS needs the opt-in (gfx950 has 160 KiB per CU)
            const int b = (int)paged_attn_smem(2);
            return hipFuncSetAttribute((const void*)paged_attn_kernel<2, false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, b) == hipSuccess &&
                   hipFuncSetAttribute((const void*)paged_attn_kernel<2, true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, b) == hipSuccess;
        }();
        (void)attr;
        if (fp8) PA_LAUNCH(2, true); else PA_LAUNCH(2, false);
    }
#undef PA_LAUNCH
    if (nsplit > 1 && cnt == nullptr) {
        if (nqt == 1)
            hipLaunchKernelGGL(paged_attn_combine_kernel<1>, dim3(ntiles, hkv), block, 0, st, part_o, part_lse,
                               q_start, tiles, out, hq, hkv, nsplit, ntiles, CHRONOS_GATE);
        else
            hipLaunchKernelGGL(paged_attn_combine_kernel<2>, dim3(ntiles, hkv), block, 0, st, part_o, part_lse,
                               q_start, tiles, out, hq, hkv, nsplit, ntiles, CHRONOS_GATE);
    }
}

}  // namespace chronos
