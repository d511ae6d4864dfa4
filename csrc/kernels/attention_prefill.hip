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

// SUB = 32-token K/V sub-tiles staged per barrier (1: the original 32-token step; 2: 64 tokens per stage, so every
// barrier / prefetch round trip carries twice the MFMA work — the kernel is bound by the K/V load latency with one
// stage of lookahead, profiles/r1s4_prefill_attn.jsonl).
template <bool FP8, int SUB>
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
    const int nsub = (kv_end + 31) >> 5;          // 32-token sub-tiles
    const int nsteps = (nsub + SUB - 1) / SUB;    // stages (one barrier each)
    // first position any row of this wave can have (rows are token-major): keys below it need no causal mask
    const int wave_min_pos = ctx0 + rel0 + (w * 32) / G;

    // ---- staging assignment ----
    const int krow = threadIdx.x >> 3, kunit = (threadIdx.x & 7) * 2;     // K: 32 rows x 16 units of 16 B
    const int vrow = threadIdx.x >> 1, vhalf = threadIdx.x & 1;           // V^T: 128 rows x 2 halves of 32 B
    u16x8 ks[SUB][2], vs[SUB][2];
    auto gload = [&](int s) {
#pragma unroll
        for (int j = 0; j < SUB; ++j) {
            const int tok = (s * SUB + j) * 32 + krow;
            if (tok < kv_end) {
                const int64_t blk = bt[tok / block_size];
                const int64_t e = (((blk * hkv + h) * block_size) + tok % block_size) * kPD + kunit * 8;
                if constexpr (FP8) {  // 16 fp8 -> 16 bf16 during staging: the LDS image and the math stay bf16
                    const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(kcv) + e);
                    ks[j][0] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.x, v.y, k_scale));
                    ks[j][1] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.z, v.w, k_scale));
                } else {
                    const u16x8* p = reinterpret_cast<const u16x8*>(kc + e);
                    ks[j][0] = p[0];
                    ks[j][1] = p[1];
                }
            } else {
                ks[j][0] = ks[j][1] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            }
            const int vt = (s * SUB + j) * 32 + vhalf * 16;
            if (vt < kv_end) {
                const int64_t blk = bt[vt / block_size];
                const int64_t e = ((blk * hkv + h) * kPD + vrow) * (int64_t)block_size + vt % block_size;
                if constexpr (FP8) {
                    const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(vcv) + e);
                    vs[j][0] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.x, v.y, v_scale));
                    vs[j][1] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.z, v.w, v_scale));
                } else {
                    const u16x8* p = reinterpret_cast<const u16x8*>(vc + e);
                    vs[j][0] = p[0];
                    vs[j][1] = p[1];
                }
            } else {
                vs[j][0] = vs[j][1] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            }
        }
    };
    auto swrite = [&](int buf) {
#pragma unroll
        for (int j = 0; j < SUB; ++j) {
            unsigned char* base = lds + (buf * SUB + j) * kStage;
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const int u = (kunit + jj) ^ (krow & 15);
                *reinterpret_cast<u16x8*>(base + krow * 256 + u * 16) = ks[j][jj];
                *reinterpret_cast<u16x8*>(base + kKImg + vrow * kVPitch + vhalf * 32 + jj * 16) = vs[j][jj];
            }
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
        if (s + 1 < nsteps) gload(s + 1);  // in flight under this stage's MFMAs
#pragma unroll
        for (int j = 0; j < SUB; ++j) {
            const int sub = s * SUB + j;
            if (sub < nsub) {  // uniform
            const unsigned char* base = lds + ((s & 1) * SUB + j) * kStage;
            const int t0 = sub * 32;
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

// ------------------------------------------------------------------------------------------------------------------
// v2: 32x32x16 MFMAs with the score tile reused in registers as the P·V operand (cdna_hip_programming.md §3 "An
// accumulator tile as the next MFMA's operand").  Per wave 32 query rows, 64 keys per stage:
//   S^T[key, row] = K[key, :] . Q[row, :]   — mfma_32x32x16(A = K rows from LDS, B = Q^T in registers), 2 key blocks;
//     a lane owns ONE query row (col = lane & 31) and 32 of the stage's 64 keys (rows (r&3)+8(r>>2)+4h of each block),
//     so the row max is 31 in-lane fmax + one exchange with the partner lane (lane ^ 32) — no 16-lane shuffles;
//   O^T[dim, row] += V^T[dim, key] . P^T[key, row] — the exp'd scores converted pairwise to bf16 ARE the B operand
//     (registers 8s..8s+7 = k-step s); the V^T fragment is read in the same permuted key order (two 8-byte reads).
// LDS per stage: K [64 keys][256 B] with the 16-B unit XOR-swizzled by (key & 15) (conflict-free ds_read_b128 of the
// A fragments); V^T [128 dims][64 keys] with a 144-B row pitch (9 x 16 B: the 16 lanes of a ds_read_b128 group land
// on distinct bank quads) and the keys of every 16-key group stored in the P operand's k order
// [0-3, 8-11, 4-7, 12-15], so each V^T fragment is ONE 16-byte read.  Register-staged K/V for stage s+1 are in
// flight under stage s, one barrier per stage.
// LEAN (default): PMC counters showed the kernel VALU-issue-bound, not MFMA- or LDS-bound (SQ_INSTS_VALU ~19.5 per
// MFMA, profiles/r2_prefill_pmc_v2.txt).  LEAN cuts the per-stage VALU work: the raw v_exp_f32
// (__builtin_amdgcn_exp2f, no denormal range fix-up), the score scale fused into the exponent's fma and applied to
// the max instead of to all 32 scores, masking only in edge stages as one compare + select against a per-lane limit
// (invalid tail rows included), the staging-register masks only in the stage that reaches past kv_end, and staging
// addresses as one 64-bit block base + a per-thread constant (the general path spent ~100 VALU ops per stage on
// 64-bit index arithmetic).  650 -> 876 -> 966 TFLOP/s on 16k-token chunks over a 112k prefix, 588 -> 892
// causal-only (profiles/r2_prefill_attn_lean.jsonl, r2_prefill_attn_lean_staging.jsonl).  Measured and not kept:
// the stage loop unrolled by LDS buffer (immediate LDS offsets) + block ids fetched a stage ahead: 939-953, within
// run-to-run noise of the plain loop; "optimistic" P against the running max before the rescale decision (so the
// first key block's exponentials could issue under the second block's QK^T): 924-934 vs 934-943, not kept
// (profiles/r2_prefill_attn_optimistic_not_kept.jsonl).
// ------------------------------------------------------------------------------------------------------------------
constexpr int kK2Img = 64 * 256;        // K image bytes per stage
constexpr int kV2Pitch = 144;           // V^T row pitch (bytes)
constexpr int kV2Img = 128 * kV2Pitch;  // V^T image bytes per stage
constexpr int kStage2 = kK2Img + kV2Img;
constexpr float kRescaleThr = 8.f;     // defer-max threshold (log2 units)

// WPG (bf16 LEAN, default; knob prefill_wpg=0 for the per-lane form): wave w stages page w of the stage for K and V
// (2 dims of V per lane), so the block id is wave-uniform — a scalar load per stage instead of three per-lane loads
// (attn_prefill8_kernel's WPG, +6.8 % there).  bf16, bit-identical: +0.4-1.6 % on 16k chunks (MFMA-heavier than fp8),
// +8.6 % on the 1024-stream wave's 93-token prompts (profiles/r5/prefill_bf16_wpg_ab.jsonl).
template <bool FP8, bool LEAN, bool WPG = false>
__global__ void __launch_bounds__(256, 2) attn_prefill2_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ kcv, const void* __restrict__ vcv,
    const int32_t* __restrict__ block_table, int bt_stride, const int32_t* __restrict__ q_start,
    const int32_t* __restrict__ ctx_len, const int32_t* __restrict__ tiles, int ntiles, uint16_t* __restrict__ out,
    int hq, int hkv, int block_size, float scale_log2_in, float k_scale, float v_scale) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    typedef float f32x16_t __attribute__((ext_vector_type(16)));
    // LEAN fp8 KV: K/V images hold the unscaled e4m3 values (exact in bf16); k_scale moves into the score scale and
    // v_scale into the output normalisation, so staging is one conversion per two elements and no multiply.
    constexpr bool kFold = FP8 && LEAN;
    const float scale_log2 = kFold ? scale_log2_in * k_scale : scale_log2_in;
    const uint16_t* kc = reinterpret_cast<const uint16_t*>(kcv);
    const uint16_t* vc = reinterpret_cast<const uint16_t*>(vcv);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int col = lane & 31, hf = lane >> 5;
    const int G = hq / hkv;
    const int h = blockIdx.y;
    const int tile = ntiles - 1 - (int)blockIdx.x;  // heaviest first
    const int seq = tiles[2 * tile], rel0 = tiles[2 * tile + 1];
    const int qbase = q_start[seq], qlen = q_start[seq + 1] - qbase;
    const int ctx = ctx_len[seq], ctx0 = ctx - qlen;
    const int32_t* bt = block_table + (int64_t)seq * bt_stride;

    // ---- this lane's query row: Q^T fragments (B operand: k = dims 16c + 8hf + j, col = row) ----
    const int R = w * 32 + col;
    const int tr = rel0 + R / G, hd = h * G + R % G;
    const bool rvalid = tr < qlen;
    const int rpos = rvalid ? ctx0 + tr : -1;
    bf16x8 qf[8];
    {
        const uint16_t* qp = q + ((int64_t)(qbase + (rvalid ? tr : 0)) * hq + hd) * kPD + 8 * hf;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            bf16x8 v = *reinterpret_cast<const bf16x8*>(qp + 16 * c);
            if (!rvalid) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
            qf[c] = v;
        }
    }
    int last_tr = rel0 + 128 / G - 1;
    if (last_tr > qlen - 1) last_tr = qlen - 1;
    const int kv_end = ctx0 + last_tr + 1;
    const int nsteps = (kv_end + 63) >> 6;
    const int wave_min_pos = ctx0 + rel0 + (w * 32) / G;  // keys below it need no causal mask for this wave

    // ---- staging: K 64 keys x 4 x 16 B per thread-quarter; V^T 128 dims x 2 halves of 32 keys ----
    const int kkey = threadIdx.x >> 2, kq = threadIdx.x & 3;
    const int vdim = threadIdx.x >> 1, vh = threadIdx.x & 1;
    u16x8 ks[4], vs[4];
    // Out-of-range keys load from the sequence's first page (always mapped) and are zeroed by a mask: no branch
    // around the loads, so the compiler keeps the staging registers (a branch made it merge them through scratch
    // and wait for the loads right away) and the tile stays in flight under the MFMAs.  Zeroed V keeps stale cache
    // bytes (possibly NaN) out of O even though their P is 0.
    // LEAN staging addresses (block_size 16, checked by the launcher): a stage's 64 keys are pages s*4 .. s*4+3, so
    // a thread's page index and in-page offsets are constants plus s*4; the page index is clamped to the last page
    // (keys past kv_end are zeroed at write time, swrite) and each load address is one 64-bit block base + a
    // per-thread constant — a handful of VALU ops per stage instead of the general path's 64-bit index arithmetic.
    const int64_t blk_el = (int64_t)hkv * 16 * kPD;                // elements (bytes for fp8) per cache block
    const int nblk_m1 = (kv_end + 15) / 16 - 1;
    const int koffc = (h * 16 + (kkey & 15)) * kPD + kq * 32;      // K: this thread's 64 B of its key
    const int voffc = (h * kPD + vdim) * 16;                       // V^T: this thread's dim row of a page
    const int kpg = kkey >> 4, vpg = vh * 2;
    static_assert(!WPG || (LEAN && !FP8), "page-per-wave staging: bf16 LEAN");
    const int wv = __builtin_amdgcn_readfirstlane(w);
    auto gload_lean = [&](int s) {
        if constexpr (WPG) {
            const int64_t blk = bt[min(s * 4 + wv, nblk_m1)];  // wave-uniform
            const u16x8* kp = reinterpret_cast<const u16x8*>(kc + blk * blk_el + koffc);
#pragma unroll
            for (int j = 0; j < 4; ++j) ks[j] = kp[j];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const u16x8* vp = reinterpret_cast<const u16x8*>(vc + blk * blk_el + (h * kPD + 2 * lane + j) * 16);
                vs[2 * j] = vp[0];
                vs[2 * j + 1] = vp[1];
            }
            return;
        }
        const int64_t kblk = bt[min(s * 4 + kpg, nblk_m1)];
        if constexpr (FP8) {
            const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(kcv) + kblk * blk_el + koffc);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint4 v = p[j];
                ks[2 * j] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8_raw(v.x, v.y));
                ks[2 * j + 1] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8_raw(v.z, v.w));
            }
        } else {
            const u16x8* p = reinterpret_cast<const u16x8*>(kc + kblk * blk_el + koffc);
#pragma unroll
            for (int j = 0; j < 4; ++j) ks[j] = p[j];
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int64_t vblk = bt[min(s * 4 + vpg + b, nblk_m1)];
            if constexpr (FP8) {
                const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(vcv) + vblk * blk_el + voffc);
                vs[2 * b] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8_raw(v.x, v.y));
                vs[2 * b + 1] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8_raw(v.z, v.w));
            } else {
                const u16x8* p = reinterpret_cast<const u16x8*>(vc + vblk * blk_el + voffc);
                vs[2 * b] = p[0];
                vs[2 * b + 1] = p[1];
            }
        }
    };
    auto gload = [&](int s) {
        if constexpr (LEAN) {
            gload_lean(s);
            return;
        }
        const int tok = s * 64 + kkey;
        const bool kval = tok < kv_end;
        const int tk = kval ? tok : 0;
        const uint16_t km = kval ? 0xFFFF : 0;
        {
            const int64_t blk = bt[tk / block_size];
            const int64_t e = (((blk * hkv + h) * block_size) + tk % block_size) * kPD + kq * 32;
            if constexpr (FP8) {
                const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(kcv) + e);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint4 v = p[j];
                    ks[2 * j] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.x, v.y, k_scale));
                    ks[2 * j + 1] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.z, v.w, k_scale));
                }
            } else {
                const u16x8* p = reinterpret_cast<const u16x8*>(kc + e);
#pragma unroll
                for (int j = 0; j < 4; ++j) ks[j] = p[j];
            }
            if constexpr (!LEAN) {
#pragma unroll
                for (int j = 0; j < 4; ++j) ks[j] &= km;
            }
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) {  // two 16-token pages of this thread's 32-key half
            const int vt = s * 64 + vh * 32 + b * 16;
            const bool vval = vt < kv_end;
            const int tv = vval ? vt : 0;
            const uint16_t vm = vval ? 0xFFFF : 0;
            const int64_t blk = bt[tv / block_size];
            const int64_t e = ((blk * hkv + h) * kPD + vdim) * (int64_t)block_size + tv % block_size;
            if constexpr (FP8) {
                const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(vcv) + e);
                vs[2 * b] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.x, v.y, v_scale));
                vs[2 * b + 1] = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8(v.z, v.w, v_scale));
            } else {
                const u16x8* p = reinterpret_cast<const u16x8*>(vc + e);
                vs[2 * b] = p[0];
                vs[2 * b + 1] = p[1];
            }
            if constexpr (!LEAN) {
                vs[2 * b] &= vm;
                vs[2 * b + 1] &= vm;
            }
        }
    };
    auto swrite = [&](int buf, int s) {
        if constexpr (LEAN) {
            // LEAN: the staged keys are masked only in the stage that reaches past kv_end (wave-uniform branch, at
            // write time when the data is in registers anyway); every other stage writes the loads untouched.
            if (s * 64 + 64 > kv_end) {
                const uint16_t km = s * 64 + kkey < kv_end ? 0xFFFF : 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) ks[j] &= km;
                if constexpr (WPG) {
                    const uint16_t vm = s * 64 + wv * 16 < kv_end ? 0xFFFF : 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) vs[j] &= vm;
                } else {
#pragma unroll
                    for (int b = 0; b < 2; ++b) {
                        const uint16_t vm = s * 64 + vh * 32 + b * 16 < kv_end ? 0xFFFF : 0;
                        vs[2 * b] &= vm;
                        vs[2 * b + 1] &= vm;
                    }
                }
            }
        }
        unsigned char* base = lds + buf * kStage2;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int u = (kq * 4 + j) ^ (kkey & 15);
            *reinterpret_cast<u16x8*>(base + kkey * 256 + u * 16) = ks[j];
        }
        if constexpr (WPG) {  // dims 2 lane + j, keys of page wv = 16-key group wv (byte offset 32 wv of the row)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                unsigned char* vp = base + kK2Img + (2 * lane + j) * kV2Pitch + wv * 32;
                const u16x8 lo = vs[2 * j], hi = vs[2 * j + 1];
                *reinterpret_cast<u16x4*>(vp) = u16x4{lo[0], lo[1], lo[2], lo[3]};
                *reinterpret_cast<u16x4*>(vp + 16) = u16x4{lo[4], lo[5], lo[6], lo[7]};
                *reinterpret_cast<u16x4*>(vp + 8) = u16x4{hi[0], hi[1], hi[2], hi[3]};
                *reinterpret_cast<u16x4*>(vp + 24) = u16x4{hi[4], hi[5], hi[6], hi[7]};
            }
            return;
        }
        unsigned char* vr = base + kK2Img + vdim * kV2Pitch + vh * 64;
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // vs[j] = keys 8j..8j+7 of this thread's 32: quads go to k-order slots
            const u16x8 v = vs[j];
            const int g16 = (j >> 1) * 32, odd = j & 1;  // byte offset of the 16-key group; upper half of it?
            *reinterpret_cast<u16x4*>(vr + g16 + 8 * odd) = u16x4{v[0], v[1], v[2], v[3]};       // keys 8o+0..3
            *reinterpret_cast<u16x4*>(vr + g16 + 16 + 8 * odd) = u16x4{v[4], v[5], v[6], v[7]};  // keys 8o+4..7
        }
    };

    float m = -1e30f, lsum = 0.f;
    f32x16_t o[4];
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[db][i] = 0.f;

    if (nsteps > 0) {
        gload(0);
        swrite(0, 0);
    }
    const bool wave_invalid = __any(rpos < 0);  // tail tile: some rows of this wave are past the chunk end
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        if (s + 1 < nsteps) gload(s + 1);  // in flight under this stage's MFMAs
        const unsigned char* base = lds + (s & 1) * kStage2;
        const int t0 = s * 64;
        // ---- S^T for the stage's two 32-key blocks ----
        f32x16_t sc[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16_t acc;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = 0.f;
            const int row = kb * 32 + col;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int u = (2 * c + hf) ^ (row & 15);
                const bf16x8 kf = *reinterpret_cast<const bf16x8*>(base + row * 256 + u * 16);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[c], acc, 0, 0, 0);
            }
            sc[kb] = acc;
        }
        // ---- online softmax over this lane's 32 keys + the partner lane's 32 ----
        const bool edge = (t0 + 64 > kv_end) || (t0 + 63 > wave_min_pos) || (LEAN && wave_invalid);
        float mx = -INFINITY;
        if constexpr (LEAN) {
            // raw scores (scale > 0 keeps the order): the scale is applied once to the max and fused into the
            // exponent's fma below.  Masking only in edge stages, as one compare against a per-lane limit
            // (min(kv_end, rpos + 1); an invalid row has rpos = -1 and masks everything) and a select.
            if (edge) {
                const int lim = min(kv_end, rpos + 1) - (t0 + 4 * hf);
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        sc[kb][i] = (kb * 32 + (i & 3) + 8 * (i >> 2)) >= lim ? -INFINITY : sc[kb][i];
            }
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int i = 0; i < 16; ++i) mx = fmaxf(mx, sc[kb][i]);
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * scale_log2;
        } else {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    float v = sc[kb][i] * scale_log2;
                    if (edge) {
                        const int tok = t0 + kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
                        if (tok >= kv_end || tok > rpos) v = -INFINITY;
                    } else if (rpos < 0) {
                        v = -INFINITY;
                    }
                    sc[kb][i] = v;
                    mx = fmaxf(mx, v);
                }
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        }
        // defer-max (cdna_hip_programming.md T13): O and l are rescaled only when some row's max grew more than
        // kRescaleThr (log2 units) past the max its running sums use — a wave-uniform branch, rare once the causal
        // prefix has been seen; otherwise p = 2^(s - stale max) <= 2^kRescaleThr, exact in f32, fine as bf16.  The
        // decision is taken before this tile's P is formed, so every P.V and l term of the tile sees one factor.
        float ps = 0.f;
        bf16x8 pf[2][2];
        auto form_p = [&]() {
            ps = 0.f;
            const float nm = -m;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    // LEAN: the raw v_exp_f32 (no denormal range fix-up: p < 2^-126 flushing to 0 is harmless)
                    const float p = LEAN ? __builtin_amdgcn_exp2f(fmaf(sc[kb][i], scale_log2, nm))
                                         : exp2f(sc[kb][i] - m);
                    ps += p;
                    pf[kb][i >> 3][i & 7] = (__bf16)p;
                }
        };
        auto rescale = [&]() {
            const float mnew = fmaxf(m, mx);
            const float alpha = LEAN ? __builtin_amdgcn_exp2f(m - mnew) : exp2f(m - mnew);
            m = mnew;
            lsum *= alpha;
#pragma unroll
            for (int db = 0; db < 4; ++db) o[db] *= alpha;
        };
        if (__any(mx > m + kRescaleThr)) rescale();
        form_p();
        lsum += ps;
        // ---- O^T += V^T . P^T (k-step (kb, s2): keys kb*32 + 16 s2 + 8 (j>>2) + 4 hf + (j&3)) ----
#pragma unroll
        for (int db = 0; db < 4; ++db) {
            const unsigned char* vr = base + kK2Img + (db * 32 + col) * kV2Pitch;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const bf16x8 vf = *reinterpret_cast<const bf16x8*>(vr + 2 * (kb * 32 + 16 * s2 + 8 * hf));
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kb][s2], o[db], 0, 0, 0);
                }
        }
        if (s + 1 < nsteps) swrite((s + 1) & 1, s + 1);
        __syncthreads();
    }

    // ---- epilogue: lane holds O^T[dims 32 db + 8 g + 4 hf + (0..3)][its row] ----
    const float lt = lsum + __shfl_xor(lsum, 32, 64);
    if (!rvalid) return;
    const float inv = (lt > 0.f ? 1.f / lt : 0.f) * (kFold ? v_scale : 1.f);
    uint16_t* op = out + ((int64_t)(qbase + tr) * hq + hd) * kPD + 4 * hf;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            u16x4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = f2bf(o[db][4 * g + i] * inv);
            *reinterpret_cast<u16x4*>(op + 32 * db + 8 * g) = v;
        }
}

// ------------------------------------------------------------------------------------------------------------------
// v8: fp8 KV cache on the block-scaled fp8 MFMA (BASELINE.json config "128k-token kill-chain context window, paged KV +
// CDNA4 fp8 MFMA").  Same tiling as v2 LEAN (4 waves x 32 query rows, 64 keys per stage, S^T = K Q^T with the score
// tile reused in registers as the P operand), but both products run on v_mfma_scale_f32_32x32x64_f8f6f4 with unit MX
// scales: 4x the K of the bf16 32x32x16 in 2x its cycles, so a stage is 8 MFMAs (4 QK^T + 4 PV) instead of 32.
// PMC on v2 LEAN fp8 (profiles/r5/prefill_pmc_v2_fp8.txt): 8.1 VALU per MFMA, issue-bound — the 32 per-stage fp8 -> bf16
// conversions of K and V and 24 of the 32 MFMA issue slots are what this variant removes; K / V stay e4m3 from HBM to
// the MFMA.
//   * Q: each row is quantised once in the prologue to e4m3 with its own scale (amax / 448 over the 128 dims, the lane
//     pair lane / lane ^ 32 holds one row); that scale, k_scale and softmax_scale * log2(e) form one per-lane score
//     multiplier, applied to the row max and fused into the exponent's fma as in v2 LEAN.
//   * P: the exp'd scores (<= 2^kRescaleThr = 256 < 448 under the deferred max) are packed to e4m3 (v_cvt_pk_fp8_f32,
//     16 per stage, as many as v2's bf16 packs); row sums stay f32.  v_scale folds into the output normalisation.
//   * fragments: lane l of the f8f6f4 MFMA holds 32 k-bytes of row / column l & 31 for lane half l >> 5, the same
//     (half, byte) -> k map for A and B, so any k permutation shared by both operands is exact.  QK^T: byte j of half
//     hf = head dim 64c + 32hf + j (MFMA c = 0, 1).  PV: byte j of half hf = key (j >> 4) * 32 + 8 ((j >> 2) & 3) +
//     4 hf + (j & 3) — exactly the keys the lane's S^T accumulators hold (registers 16 kb + i of S^T block kb) — so
//     the V^T image stores each dim row's 64 keys in that order and every operand is two conflict-free ds_read_b128.
//   * LDS per stage: K [64 keys][128 B] with the 16-B chunk c of key k at slot c ^ ((k >> 1) & 7) (the 16 lanes of a
//     ds_read_b128 group cover both row parities x 8 slots); V^T [128 dims][64 key bytes] at an 80-B pitch.  18 KiB per
//     stage, two stages, register-staged (T14 split) with one barrier per stage.
// Accuracy: Q and P take one more e4m3 rounding each, the rounding the cache already applies to K and V
// (tests/test_prefill_fp8_mfma_gpu.py checks against the fp32 reference on the dequantised cache).
// ------------------------------------------------------------------------------------------------------------------
constexpr int kK8Img = 64 * 128;
// key <-> K image row within a 16-key page: bits 2 and 3 swapped (an involution)
__device__ __forceinline__ int kperm(int k) { return (k & ~12) | ((k >> 1) & 4) | ((k << 1) & 8); }
constexpr int kV8Pitch = 80;
constexpr int kV8Img = 128 * kV8Pitch;
template <bool PV8>
constexpr int stage8_bytes() { return kK8Img + (PV8 ? kV8Img : kV2Img); }

// PV8 = false: only Q K^T on the fp8 MFMA; V is converted to bf16 at staging and P.V runs on the bf16 32x32x16 MFMA
// exactly as in v2 LEAN (the P operand keeps bf16 precision) — the accuracy / speed middle point (knob value 2).
// FOLD (knob values 1, 2; 3 = PV8 without it, for A/B): with 8 MFMAs a stage the kernel is VALU-issue-bound, so the
// per-score VALU goes into the MFMAs —
//   * k_scale * softmax_scale * log2(e) multiplies Q before quantisation and the row's quantisation scale is a power
//     of two fed to the MFMA's own E8M0 scale operand (per lane = per query row), so S^T comes out in log2 units;
//   * the QK^T accumulators start from -m (a 16-register copy of the running max, C != D), so p = v_exp_f32(S^T)
//     directly: no per-score fma.  m starts at the first stage's row max (set, not rescaled, at s = 0);
//   * (PV8) row sums come from one more fp8 MFMA against an all-ones A operand (e4m3 1.0 = 0x38): the sum of the
//     e4m3 P the P.V product used, instead of 32 v_add_f32 per stage.
// Measured and not kept: two stages of register lookahead (loads for s + 2 issued at the top of s into a second
// register set): 1640 vs 1632 TFLOP/s, within noise — the kernel is not load-latency-bound at one stage
// (profiles/r5/prefill_fp8_mfma_depth_ab.jsonl).
// MSUM (PV8 only): the row sums from the all-ones fp8 MFMA (part of FOLD, separable for A/B).
// PIPE: see the loop below (three LDS stages, next stage's Q K^T under this stage's softmax).
// WPG (PV8): wave w stages page w of the stage for both K (its 16 keys) and V (all 128 dims, 2 per lane), so the
// block id is wave-uniform — one scalar load per stage instead of three per-lane loads + 64-bit address VALU — and
// the V^T image takes 8-byte halves (ds_write2) with no register shuffles.
template <bool PV8, bool FOLD, bool MSUM, bool PIPE = false, bool WPG = false>
__global__ void __launch_bounds__(256, 2) attn_prefill8_kernel(
    const uint16_t* __restrict__ q, const uint8_t* __restrict__ kc, const uint8_t* __restrict__ vc,
    const int32_t* __restrict__ block_table, int bt_stride, const int32_t* __restrict__ q_start,
    const int32_t* __restrict__ ctx_len, const int32_t* __restrict__ tiles, int ntiles, uint16_t* __restrict__ out,
    int hq, int hkv, float scale_log2, float k_scale, float v_scale, int blk_lg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    typedef float f32x16_t __attribute__((ext_vector_type(16)));
    typedef int i32x8_t __attribute__((ext_vector_type(8)));
    typedef int i32x4_t __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int col = lane & 31, hf = lane >> 5;
    const int G = hq / hkv;
    const int h = blockIdx.y;
    const int tile = ntiles - 1 - (int)blockIdx.x;  // heaviest first
    const int seq = tiles[2 * tile], rel0 = tiles[2 * tile + 1];
    const int qbase = q_start[seq], qlen = q_start[seq + 1] - qbase;
    const int ctx = ctx_len[seq], ctx0 = ctx - qlen;
    const int32_t* bt = block_table + (int64_t)seq * bt_stride;

    // ---- this lane's query row, quantised: dims 64c + 32hf + j in byte j of qf[c] ----
    const int R = w * 32 + col;
    const int tr = rel0 + R / G, hd = h * G + R % G;
    const bool rvalid = tr < qlen;
    const int rpos = rvalid ? ctx0 + tr : -1;
    i32x8_t qf[2];
    float cl;      // score multiplier: q scale * k_scale * softmax scale * log2(e) (not FOLD)
    int qe = 127;  // FOLD: E8M0 scale of this row's e4m3 Q
    {
        const uint16_t* qp = q + ((int64_t)(qbase + (rvalid ? tr : 0)) * hq + hd) * kPD + 32 * hf;
        u16x8 raw[8];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) raw[4 * c + j] = *reinterpret_cast<const u16x8*>(qp + 64 * c + 8 * j);
        float amax = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(bf2f(raw[i][e])));
        amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
        if (!rvalid) amax = 0.f;
        float inv;
        if constexpr (FOLD) {
            const float sl = k_scale * scale_log2;
            int e = 0;
            if (amax > 0.f) {
                (void)frexpf(amax * sl / kFp8Max, &e);  // 2^e >= amax * sl / 448
                e = min(max(e, -126), 126);
            }
            inv = amax > 0.f ? ldexpf(sl, -e) : 0.f;
            qe = e + 127;
            cl = 1.f;
        } else {
            inv = amax > 0.f ? kFp8Max / amax : 0.f;  // invalid / all-zero row: every byte 0
            cl = (amax > 0.f ? amax / kFp8Max : 1.f) * k_scale * scale_log2;
        }
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int d = 0; d < 8; ++d) {
                const u16x8& v = raw[4 * c + (d >> 1)];
                const int o = 4 * (d & 1);
                qf[c][d] = (int)f32x4_to_fp8x4(bf2f(v[o]) * inv, bf2f(v[o + 1]) * inv, bf2f(v[o + 2]) * inv,
                                               bf2f(v[o + 3]) * inv);
            }
    }
    int last_tr = rel0 + 128 / G - 1;
    if (last_tr > qlen - 1) last_tr = qlen - 1;
    const int kv_end = ctx0 + last_tr + 1;
    const int nsteps = (kv_end + 63) >> 6;
    const int wave_min_pos = ctx0 + rel0 + (w * 32) / G;

    // ---- staging (block_size 16, checked by the launcher): K 32 B of one key per thread, V^T 2 pages x 16 B of one
    // dim row per thread; addresses = one 64-bit block base + a per-thread constant (v2 LEAN) ----
    const int kkey = threadIdx.x >> 2, kq = threadIdx.x & 3;
    const int vdim = threadIdx.x >> 1, vh = threadIdx.x & 1;
    const int64_t blk_el = (int64_t)hkv * 16 * kPD;  // bytes per cache block
    const int nblk_m1 = (kv_end + 15) / 16 - 1;
    const int koffc = (h * 16 + (kkey & 15)) * kPD + kq * 32;
    const int voffc = (h * kPD + vdim) * 16;
    const int kpg = kkey >> 4, vpg = vh * 2;
    constexpr int kStage8 = stage8_bytes<PV8>();
    uint4 ks[2], vs[2];
    // block byte offset: a 64-bit shift when the block size is a power of two (hkv = 8: 16 KiB) instead of the
    // int64 multiply (6 quarter-rate v_mul_lo_u32 + sign extensions per stage in the ISA)
    // (the launcher routes only power-of-two hkv here; blk_lg = log2 of the block's bytes)
    auto blk_off = [&](int blk) -> int64_t { return (int64_t)((uint64_t)(uint32_t)blk << blk_lg); };
    const int wv = __builtin_amdgcn_readfirstlane(w);
    static_assert(!WPG || PV8, "page-per-wave staging: fp8 V image");
    auto gload = [&](int s) {
        if constexpr (WPG) {
            const int64_t boff = blk_off(bt[min(s * 4 + wv, nblk_m1)]);  // wave-uniform
            const uint4* kp = reinterpret_cast<const uint4*>(kc + boff + koffc);
            ks[0] = kp[0];
            ks[1] = kp[1];
            const uint4* vp = reinterpret_cast<const uint4*>(vc + boff + (h * kPD + 2 * lane) * 16);
            vs[0] = vp[0];
            vs[1] = vp[1];
            return;
        }
        const int kblk = bt[min(s * 4 + kpg, nblk_m1)];
        const uint4* kp = reinterpret_cast<const uint4*>(kc + blk_off(kblk) + koffc);
        ks[0] = kp[0];
        ks[1] = kp[1];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int vblk = bt[min(s * 4 + vpg + b, nblk_m1)];
            vs[b] = *reinterpret_cast<const uint4*>(vc + blk_off(vblk) + voffc);
        }
    };
    auto swrite = [&](int buf, int s) {
        if (s * 64 + 64 > kv_end) {  // the stage reaching past kv_end: zero keys / pages past it (wave-uniform)
            if (s * 64 + kkey >= kv_end) ks[0] = ks[1] = uint4{0u, 0u, 0u, 0u};
            if constexpr (WPG) {
                if (s * 64 + wv * 16 >= kv_end) vs[0] = vs[1] = uint4{0u, 0u, 0u, 0u};
            } else {
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    if (s * 64 + vh * 32 + b * 16 >= kv_end) vs[b] = uint4{0u, 0u, 0u, 0u};
            }
        }
        unsigned char* base = lds + buf * kStage8;
        const int krow = WPG ? kperm(kkey) : kkey;
        const int sw = (krow >> 1) & 7;
        *reinterpret_cast<uint4*>(base + krow * 128 + (((2 * kq) ^ sw) << 4)) = ks[0];
        *reinterpret_cast<uint4*>(base + krow * 128 + (((2 * kq + 1) ^ sw) << 4)) = ks[1];
        if constexpr (WPG) {
            // K rows are stored with key bits 2 and 3 swapped (kperm), so S^T lane half hf holds keys with bit 3 = hf:
            // page wv = keys 32 kb + 16 b + t (kb = wv >> 1, b = wv & 1) -> half t >> 3, bytes 16 kb + 8 b + (t & 7),
            // i.e. words {x, y} -> half 0 and {z, w} -> half 1, 8 contiguous bytes each (no register shuffles)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                unsigned char* vr = base + kK8Img + (2 * lane + j) * kV8Pitch + (wv >> 1) * 16 + (wv & 1) * 8;
                *reinterpret_cast<uint2*>(vr) = uint2{vs[j].x, vs[j].y};
                *reinterpret_cast<uint2*>(vr + 32) = uint2{vs[j].z, vs[j].w};
            }
        } else if constexpr (PV8) {
            // page b word wd = keys vh*32 + 16b + 4wd + 0..3 -> half wd & 1, dword 2b + (wd >> 1) of 16-B block vh
            unsigned char* vr = base + kK8Img + vdim * kV8Pitch + vh * 16;
            *reinterpret_cast<uint4*>(vr) = uint4{vs[0].x, vs[0].z, vs[1].x, vs[1].z};
            *reinterpret_cast<uint4*>(vr + 32) = uint4{vs[0].y, vs[0].w, vs[1].y, vs[1].w};
        } else {  // v2's bf16 V^T image: keys of every 16-key group in the P operand's k order
            unsigned char* vr = base + kK8Img + vdim * kV2Pitch + vh * 64;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const u16x8 lo = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8_raw(vs[b].x, vs[b].y));
                const u16x8 hi = __builtin_bit_cast(u16x8, fp8x8_to_bf16x8_raw(vs[b].z, vs[b].w));
                *reinterpret_cast<u16x4*>(vr + 32 * b) = u16x4{lo[0], lo[1], lo[2], lo[3]};
                *reinterpret_cast<u16x4*>(vr + 32 * b + 16) = u16x4{lo[4], lo[5], lo[6], lo[7]};
                *reinterpret_cast<u16x4*>(vr + 32 * b + 8) = u16x4{hi[0], hi[1], hi[2], hi[3]};
                *reinterpret_cast<u16x4*>(vr + 32 * b + 24) = u16x4{hi[4], hi[5], hi[6], hi[7]};
            }
        }
    };

    float m = FOLD ? 0.f : -1e30f, lsum = 0.f;
    f32x16_t o[4], negm, lacc;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[db][i] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) negm[i] = lacc[i] = 0.f;
    constexpr bool kMfmaSum = PV8 && MSUM;
    i32x8_t pf8 = {0, 0, 0, 0, 0, 0, 0, 0};  // e4m3 P; persists so each pack's first half merges into a live register
    const i32x8_t ones = {0x38383838, 0x38383838, 0x38383838, 0x38383838,
                          0x38383838, 0x38383838, 0x38383838, 0x38383838};

    const bool wave_invalid = __any(rpos < 0);
    // PIPE: this lane's quantised Q row in LDS after the three stages (row = w * 32 + col, 128 B, chunk c at slot
    // c ^ ((col >> 1) & 7))
    unsigned char* qimg = lds + 3 * kStage8 + (w * 32 + col) * 128;
    const int qsw = (col >> 1) & 7;
    if constexpr (PIPE) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int u = 4 * c + 2 * hf;
            *reinterpret_cast<i32x4_t*>(qimg + ((u ^ qsw) << 4)) = i32x4_t{qf[c][0], qf[c][1], qf[c][2], qf[c][3]};
            *reinterpret_cast<i32x4_t*>(qimg + (((u + 1) ^ qsw) << 4)) =
                i32x4_t{qf[c][4], qf[c][5], qf[c][6], qf[c][7]};
        }
    }
    // S^T of one stage from its LDS buffer
    auto qk = [&](const unsigned char* base, f32x16_t (&sc)[2]) {
        // ---- S^T for the stage's two 32-key blocks: 2 fp8 MFMAs each ----
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16_t acc;
            if constexpr (FOLD) {
                acc = negm;
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[i] = 0.f;
            }
            const int row = kb * 32 + col;
            const int sw = (row >> 1) & 7;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int u = 4 * c + 2 * hf;
                const i32x4_t lo = *reinterpret_cast<const i32x4_t*>(base + row * 128 + ((u ^ sw) << 4));
                const i32x4_t hi = *reinterpret_cast<const i32x4_t*>(base + row * 128 + (((u + 1) ^ sw) << 4));
                const i32x8_t kf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                i32x8_t qv = qf[c];
                if constexpr (PIPE) {  // Q from its LDS image (same swizzle as K): 16 VGPRs fewer across the loop
                    const i32x4_t ql = *reinterpret_cast<const i32x4_t*>(qimg + ((u ^ qsw) << 4));
                    const i32x4_t qh = *reinterpret_cast<const i32x4_t*>(qimg + (((u + 1) ^ qsw) << 4));
                    qv = __builtin_shufflevector(ql, qh, 0, 1, 2, 3, 4, 5, 6, 7);
                }
                acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kf, qv, acc, 0, 0, 0, 127, 0, qe);
            }
            sc[kb] = acc;
        }
    };
    // mask, online softmax and P.V of stage s (S^T in sc, V in the LDS buffer at base)
    auto smpv = [&](int s, const unsigned char* base, f32x16_t (&sc)[2]) {
        const int t0 = s * 64;
        // ---- online softmax (v2 LEAN with the per-lane multiplier cl) ----
        const bool edge = (t0 + 64 > kv_end) || (t0 + 63 > wave_min_pos) || wave_invalid;
        if (edge) {
            // S^T register i of block kb, lane half hf = K image row kb*32 + (i&3) + 8(i>>2) + 4hf; WPG stores key
            // kperm(row) there (bits 2 and 3 swapped)
            const int lim = min(kv_end, rpos + 1) - (t0 + (WPG ? 8 : 4) * hf);
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int ko = WPG ? kb * 32 + (i & 3) + 4 * ((i >> 2) & 1) + 16 * (i >> 3)
                                       : kb * 32 + (i & 3) + 8 * (i >> 2);
                    sc[kb][i] = ko >= lim ? -INFINITY : sc[kb][i];
                }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) mx = fmaxf(mx, sc[kb][i]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * cl;
        if constexpr (FOLD) {
            // mx is relative to m (the accumulators started at -m)
            if (s == 0 || __any(mx > kRescaleThr)) {
                float d = s == 0 ? mx : fmaxf(mx, 0.f);
                if (!(d > -INFINITY)) d = 0.f;  // every key masked (invalid row): keep m
                if (s > 0) {
                    const float alpha = __builtin_amdgcn_exp2f(-d);
                    lsum *= alpha;
                    lacc *= alpha;
#pragma unroll
                    for (int db = 0; db < 4; ++db) o[db] *= alpha;
                }
                m += d;
#pragma unroll
                for (int kb = 0; kb < 2; ++kb) sc[kb] -= d;
#pragma unroll
                for (int i = 0; i < 16; ++i) negm[i] = -m;
            }
        } else if (__any(mx > m + kRescaleThr)) {
            const float mnew = fmaxf(m, mx);
            const float alpha = __builtin_amdgcn_exp2f(m - mnew);
            m = mnew;
            lsum *= alpha;
#pragma unroll
            for (int db = 0; db < 4; ++db) o[db] *= alpha;
        }
        float ps = 0.f;
        const float nm = -m;
        auto expo = [&](float x) {
            return FOLD ? __builtin_amdgcn_exp2f(x) : __builtin_amdgcn_exp2f(fmaf(x, cl, nm));
        };
        if constexpr (PV8) {
            i32x8_t& pf = pf8;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int i = 0; i < 16; i += 4) {
                    float p[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        p[e] = expo(sc[kb][i + e]);
                        if constexpr (!kMfmaSum) ps += p[e];
                    }
                    const int r = __builtin_amdgcn_cvt_pk_fp8_f32(p[0], p[1], pf[kb * 4 + (i >> 2)], false);
                    pf[kb * 4 + (i >> 2)] = __builtin_amdgcn_cvt_pk_fp8_f32(p[2], p[3], r, true);
                }
            // ---- O^T += V^T . P^T: one fp8 MFMA per 32-dim block ----
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                const unsigned char* vr = base + kK8Img + (db * 32 + col) * kV8Pitch + hf * 32;
                const i32x4_t lo = *reinterpret_cast<const i32x4_t*>(vr);
                const i32x4_t hi = *reinterpret_cast<const i32x4_t*>(vr + 16);
                const i32x8_t vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                o[db] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf, pf, o[db], 0, 0, 0, 127, 0, 127);
                if constexpr (PIPE) __builtin_amdgcn_sched_barrier(0);  // one V fragment live at a time
            }
            if constexpr (kMfmaSum) lacc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ones, pf, lacc, 0, 0, 0, 127,
                                                                                           0, 127);
        } else {
            bf16x8 pf[2][2];
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float p = expo(sc[kb][i]);
                    ps += p;
                    pf[kb][i >> 3][i & 7] = (__bf16)p;
                }
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                const unsigned char* vr = base + kK8Img + (db * 32 + col) * kV2Pitch;
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(vr + 2 * (kb * 32 + 16 * s2 + 8 * hf));
                        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kb][s2], o[db], 0, 0, 0);
                    }
            }
        }
        lsum += ps;
    };
    if constexpr (!PIPE) {
        if (nsteps > 0) {
            gload(0);
            swrite(0, 0);
        }
        __syncthreads();
        for (int s = 0; s < nsteps; ++s) {
            if (s + 1 < nsteps) gload(s + 1);  // in flight under this stage's MFMAs
            const unsigned char* base = lds + (s & 1) * kStage8;
            f32x16_t sc[2];
            qk(base, sc);
            smpv(s, base, sc);
            if (s + 1 < nsteps) swrite((s + 1) & 1, s + 1);
            __syncthreads();
        }
    } else {
        // PIPE: three LDS buffers; stage s + 1's Q K^T MFMAs are issued before stage s's softmax, so the matrix pipe
        // runs them under the exp / pack VALU (cdna_hip_programming.md T15).  Unrolled by two so the two S^T register
        // sets swap roles without copies.
        if (nsteps > 0) {
            gload(0);
            swrite(0, 0);
        }
        if (nsteps > 1) {
            gload(1);
            swrite(1, 1);
        }
        __syncthreads();
        f32x16_t sa[2], sb[2];
        if (nsteps > 0) qk(lds, sa);
        int b0 = 0, b1 = 1, b2 = 2;  // LDS buffers of stages s, s + 1, s + 2
        auto step = [&](int s, f32x16_t (&cur)[2], f32x16_t (&nxt)[2]) {
            if (s + 2 < nsteps) gload(s + 2);
            if (s + 1 < nsteps) qk(lds + b1 * kStage8, nxt);
            smpv(s, lds + b0 * kStage8, cur);
            if (s + 2 < nsteps) swrite(b2, s + 2);
            __syncthreads();
            const int t = b0;
            b0 = b1;
            b1 = b2;
            b2 = t;
        };
        for (int s = 0; s < nsteps; s += 2) {
            step(s, sa, sb);
            if (s + 1 < nsteps) step(s + 1, sb, sa);
        }
    }

    // ---- epilogue: lane holds O^T[dims 32 db + 8 g + 4 hf + (0..3)][its row] ----
    const float lt = kMfmaSum ? lacc[0] : lsum + __shfl_xor(lsum, 32, 64);
    if (!rvalid) return;
    const float inv = (lt > 0.f ? 1.f / lt : 0.f) * v_scale;
    uint16_t* op = out + ((int64_t)(qbase + tr) * hq + hd) * kPD + 4 * hf;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            u16x4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = f2bf(o[db][4 * g + i] * inv);
            *reinterpret_cast<u16x4*>(op + 32 * db + 8 * g) = v;
        }
}

void launch_attn_prefill(const uint16_t* q, const void* kc, const void* vc, const int32_t* block_table,
                         int bt_stride, const int32_t* q_start, const int32_t* ctx_len, const int32_t* tiles,
                         int ntiles, uint16_t* out, int hq, int hkv, int block_size, float scale, bool fp8,
                         float k_scale, float v_scale, hipStream_t st) {
    if (ntiles == 0) return;
    // 2 (default): v2 LEAN; 5: v2 as before LEAN (kept for in-process A/B); 0 / 1: the 32-key-step kernel
    const int variant = knob("prefill_variant", 2);
    const int f8 = fp8 && variant == 2 && block_size == 16 && (hkv & (hkv - 1)) == 0 ? knob("prefill_fp8_mfma", 1) : 0;
    const int blk_lg = __builtin_ctz((unsigned)(hkv * 16 * kPD));
    // 1: Q K^T and P V on the fp8 MFMA; 2: Q K^T only (FOLD); 3: 1 with FOLD; 4: 2 without.  FOLD measured neutral to
    // negative with P V on the fp8 MFMA (1605 vs 1638 TFLOP/s on the 112k-prefix chunk, its 9th MFMA and the -m copies
    // cost what the removed VALU saved) and +3.8 % for Q K^T only (profiles/r5/prefill_fp8_mfma_fold_ab.jsonl)
    // 5: 1 with the MFMA row sums only; 6: 1 with PIPE; 7: 1 with per-lane block ids (before WPG)
    // 8: 1 with the MFMA row sums (MSUM) on top of the page-per-wave staging
    if (f8 >= 1 && f8 <= 8) {
        static bool attr8 = [] {
            bool ok = true;
            for (const void* f : {(const void*)attn_prefill8_kernel<true, true, true>,
                                  (const void*)attn_prefill8_kernel<true, false, false>,
                                  (const void*)attn_prefill8_kernel<true, false, false, false, true>,
                                  (const void*)attn_prefill8_kernel<true, false, true, false, true>,
                                  (const void*)attn_prefill8_kernel<true, false, true>})
                ok &= hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * stage8_bytes<true>()) ==
                      hipSuccess;
            ok &= hipFuncSetAttribute((const void*)attn_prefill8_kernel<true, false, false, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      3 * stage8_bytes<true>() + 16384) == hipSuccess;
            for (const void* f : {(const void*)attn_prefill8_kernel<false, true, false>,
                                  (const void*)attn_prefill8_kernel<false, false, false>})
                ok &= hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * stage8_bytes<false>()) ==
                      hipSuccess;
            return ok;
        }();
        (void)attr8;
        const float sl2 = scale * 1.4426950408889634f;
        const uint8_t* k8 = static_cast<const uint8_t*>(kc);
        const uint8_t* v8 = static_cast<const uint8_t*>(vc);
#define AP8_LAUNCH(PV, FO, MS)                                                                              \
    hipLaunchKernelGGL((attn_prefill8_kernel<PV, FO, MS>), dim3(ntiles, hkv), dim3(256), 2 * stage8_bytes<PV>(), \
                       st, q, k8, v8, block_table, bt_stride, q_start, ctx_len, tiles, ntiles, out, hq, hkv, sl2,  \
                       k_scale, v_scale, blk_lg)
        if (f8 == 1)
            hipLaunchKernelGGL((attn_prefill8_kernel<true, false, false, false, true>), dim3(ntiles, hkv), dim3(256),
                               2 * stage8_bytes<true>(), st, q, k8, v8, block_table, bt_stride, q_start, ctx_len, tiles,
                               ntiles, out, hq, hkv, sl2, k_scale, v_scale, blk_lg);
        else if (f8 == 7) AP8_LAUNCH(true, false, false);
        else if (f8 == 8)
            hipLaunchKernelGGL((attn_prefill8_kernel<true, false, true, false, true>), dim3(ntiles, hkv), dim3(256),
                               2 * stage8_bytes<true>(), st, q, k8, v8, block_table, bt_stride, q_start, ctx_len, tiles,
                               ntiles, out, hq, hkv, sl2, k_scale, v_scale, blk_lg);
        else if (f8 == 2) AP8_LAUNCH(false, true, false);
        else if (f8 == 3) AP8_LAUNCH(true, true, true);
        else if (f8 == 5) AP8_LAUNCH(true, false, true);
        else if (f8 == 6)
            hipLaunchKernelGGL((attn_prefill8_kernel<true, false, false, true>), dim3(ntiles, hkv), dim3(256),
                               3 * stage8_bytes<true>() + 16384, st, q, k8, v8, block_table, bt_stride, q_start,
                               ctx_len, tiles, ntiles, out, hq, hkv, sl2, k_scale, v_scale, blk_lg);
        else AP8_LAUNCH(false, false, false);
#undef AP8_LAUNCH
        return;
    }
    if (variant == 2 || variant == 5) {
        static bool attr2 = [] {
            bool ok = true;
            for (const void* f : {(const void*)attn_prefill2_kernel<false, false>,
                                  (const void*)attn_prefill2_kernel<true, false>,
                                  (const void*)attn_prefill2_kernel<false, true>,
                                  (const void*)attn_prefill2_kernel<false, true, true>,
                                  (const void*)attn_prefill2_kernel<true, true>})
                ok &= hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kStage2) == hipSuccess;
            return ok;
        }();
        (void)attr2;
        const float sl2 = scale * 1.4426950408889634f;
#define AP2_LAUNCH(F, L, KS, VS, ...)                                                                              \
    hipLaunchKernelGGL((attn_prefill2_kernel<F, L, ##__VA_ARGS__>), dim3(ntiles, hkv), dim3(256), 2 * kStage2, st, q, \
                       kc, vc, block_table, bt_stride, q_start, ctx_len, tiles, ntiles, out, hq, hkv, block_size, sl2, KS, \
                       VS)
        if (variant == 2 && block_size == 16) {
            if (fp8) AP2_LAUNCH(true, true, k_scale, v_scale);
            else if (knob("prefill_wpg", 1)) AP2_LAUNCH(false, true, 1.f, 1.f, true);
            else AP2_LAUNCH(false, true, 1.f, 1.f);
        } else {
            if (fp8) AP2_LAUNCH(true, false, k_scale, v_scale); else AP2_LAUNCH(false, false, 1.f, 1.f);
        }
#undef AP2_LAUNCH
        return;
    }
    const int sub = variant == 1 ? 2 : 1;
    static bool attr = [] {
        bool ok = true;
        ok &= hipFuncSetAttribute((const void*)attn_prefill_kernel<false, 1>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kStage) == hipSuccess;
        ok &= hipFuncSetAttribute((const void*)attn_prefill_kernel<true, 1>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kStage) == hipSuccess;
        ok &= hipFuncSetAttribute((const void*)attn_prefill_kernel<false, 2>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kStage) == hipSuccess;
        ok &= hipFuncSetAttribute((const void*)attn_prefill_kernel<true, 2>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kStage) == hipSuccess;
        return ok;
    }();
    (void)attr;
    const float sl = scale * 1.4426950408889634f;
    const size_t lds = (size_t)2 * sub * kStage;
#define AP_LAUNCH(F, S, KS, VS)                                                                                    \
    hipLaunchKernelGGL((attn_prefill_kernel<F, S>), dim3(ntiles, hkv), dim3(256), lds, st, q, kc, vc, block_table, \
                       bt_stride, q_start, ctx_len, tiles, ntiles, out, hq, hkv, block_size, sl, KS, VS)
    if (fp8) {
        if (sub == 2) AP_LAUNCH(true, 2, k_scale, v_scale); else AP_LAUNCH(true, 1, k_scale, v_scale);
    } else {
        if (sub == 2) AP_LAUNCH(false, 2, 1.f, 1.f); else AP_LAUNCH(false, 1, 1.f, 1.f);
    }
#undef AP_LAUNCH
}

}  // namespace chronos
