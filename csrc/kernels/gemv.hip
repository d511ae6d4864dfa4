// gemv.hip — decode-regime projection GEMM (M <= 8 rows) streaming the weights once at HBM rate
// (SURVEY.md §2.3 K3/K7/K8/K10/K11 decode column; §7.3 hard part 1: "decode at the HBM roofline").
//
//   y[M, N] = x[M, K] · W[N, K]^T      (W row-major [out, in], the HF layout; bf16 in, f32 accumulate, bf16 out)
//
// At M <= 8 the op is a pure weight stream (16 GB per Llama-3-8B decode step), so the kernel is shaped around the
// load path, not the arithmetic:
//   * every wave-wide load is one CONTIGUOUS 1 KiB piece of one weight row (64 lanes x 16 B = 8 full 128-B lines) —
//     an MFMA operand layout would touch 32 partial lines per instruction;
//   * weights go straight to VGPRs (cdna_hip_programming.md §5 "GEMV / M <= 16: load straight to VGPRs, deep
//     unroll"), in a register ring DEPTH chunks deep so HBM latency hides behind the arithmetic; x is re-read from L2;
//   * arithmetic is v_dot2_f32_bf16 (2 MACs per lane-op, no bf16->f32 unpacking): M/2 VALU ops per weight element;
//   * the R x M partial sums of a wave are butterfly-reduced across the wave and the 4 waves of the workgroup,
//     which split K, meet in LDS.
// One 256-thread workgroup owns R output rows.  Fused SwiGLU epilogue for the gate/up projection (w = [gate; up]):
// the workgroup streams R gate rows and the matching R up rows and writes silu(g) * u directly.
#include "chronos_hip.h"
#include "chronos_gemv.h"

namespace chronos {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) {
    return __builtin_nontemporal_load(p);
}

// Pairs are extracted with shufflevector: hipcc (ROCm 7.2) mis-lowers a bit_cast of a runtime-unrolled u32 vector
// element into the dot2 operand (all four v_dot2c read the same register) — keep this form.
__device__ __forceinline__ float dot8(const u16x8& w, const u16x8& x, float acc) {
    const bf16x8 wb = __builtin_bit_cast(bf16x8, w), xb = __builtin_bit_cast(bf16x8, x);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 0, 1), __builtin_shufflevector(xb, xb, 0, 1),
                                          acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 2, 3), __builtin_shufflevector(xb, xb, 2, 3),
                                          acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 4, 5), __builtin_shufflevector(xb, xb, 4, 5),
                                          acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 6, 7), __builtin_shufflevector(xb, xb, 6, 7),
                                          acc, false);
    return acc;
}

// W8A16: a 16-B piece of 16 e4m3 weights becomes 8 bf16 pairs with v_cvt_scalef32_pk_bf16_fp8 (exact: e4m3 fits
// bf16) — once per piece, shared by the M activation rows — and meets x (two 16-B pieces) in the same
// v_dot2_f32_bf16 as dot8
__device__ __forceinline__ void q2bf(const u16x8& w, bf16x2_t (&wb)[8]) {
    const i32x4 wi = __builtin_bit_cast(i32x4, w);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        wb[2 * j] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(wi[j], 1.f, false);
        wb[2 * j + 1] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(wi[j], 1.f, true);
    }
}

__device__ __forceinline__ float dot16(const bf16x2_t (&wb)[8], const u16x8& x0, const u16x8& x1, float acc) {
    const bf16x8 a = __builtin_bit_cast(bf16x8, x0), b = __builtin_bit_cast(bf16x8, x1);
    acc = __builtin_amdgcn_fdot2_f32_bf16(wb[0], __builtin_shufflevector(a, a, 0, 1), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(wb[1], __builtin_shufflevector(a, a, 2, 3), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(wb[2], __builtin_shufflevector(a, a, 4, 5), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(wb[3], __builtin_shufflevector(a, a, 6, 7), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(wb[4], __builtin_shufflevector(b, b, 0, 1), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(wb[5], __builtin_shufflevector(b, b, 2, 3), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(wb[6], __builtin_shufflevector(b, b, 4, 5), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(wb[7], __builtin_shufflevector(b, b, 6, 7), acc, false);
    return acc;
}

// Fused decode-step variants (M <= 2 rows: one sensor stream or two), chronos_gemv.h:
//   * kResid epilogue (O / down projection, TP=1): instead of y, write the new residual s = bf16(bf16(y) + r) and the
//     workgroup's per-row sum of s^2 — the producer half of the next RMSNorm;
//   * NORMP (QKV / gate_up / LM head): x is the raw residual stream s.  The norm weight is folded into the projection
//     weights at load time (W' = W diag(w), models/llama.py), so rmsnorm(s) w @ W^T = inv * (s @ W'^T) with
//     inv = rsqrt(sum of the producer's partials / K + eps): the prologue reduces the partials per wave (no barrier,
//     fixed order) and the epilogue scales the row sums by inv — no norm launch, no per-element work, no extra
//     bytes over the plain GEMV;
//   * ROPE epilogue (QKV): with P = R/2 rotate-half pairs per workgroup, workgroup b owns dims {Pj..Pj+P-1} and
//     {64+Pj..64+Pj+P-1} of head b/(64/P) (j = b%(64/P)) — the
//     rotate-half pairs — so it applies RoPE and writes q to q_out and k, v straight into the paged cache (bf16 or
//     fp8-e4m3), exactly as rope_kv_write_kernel does from the bf16 qkv output.
// Together they take a TP=1 decode layer from 9 launches (norm, qkv, rope, attn, combine, o, norm, gate_up, down) to 6.
enum : int { kPlain = 0, kSwiglu = 1, kRope = 2, kRope8 = 3, kResid = 4 };

// gemv_kernel: row group g = R output rows.  One group per workgroup (grid = ngroups), or — knob gemv_persist — a
// smaller grid whose workgroups loop over groups g, g + grid, ...  In the loop the NEXT group's first weight ring is
// issued as soon as the current group's last dot products have consumed the ring, so its loads are in flight during
// the current group's cross-wave reduction, barrier and epilogue (the weight stream does not stop between groups).
//
// WQ (W8A16, the fp8-weight decode step): W is e4m3 bytes with a per-row scale (nrm.wscale).  A lane's 16-B weight
// piece is then 16 elements, a chunk 1024 elements, and x comes as two 16-B pieces per chunk; every fused epilogue is
// the same, the row sums scaled by their row's weight scale first.  Half the weight bytes of the bf16 kernel, no
// activation quantisation launch (the W8A8 qgemv path needs one per projection).
template <int M, int R, int MODE, bool NORMP, bool WQ = false>
__global__ void __launch_bounds__(256) gemv_kernel(const uint16_t* __restrict__ x, int mrows, int K,
                                                   const uint16_t* __restrict__ W, uint16_t* __restrict__ y,
                                                   int nout, int half, GemvNorm nrm, GemvRope rp,
                                                   const int32_t* __restrict__ gst, int gn, int ngroups) {
    constexpr bool SWIGLU = MODE == kSwiglu;
    constexpr bool ROPE = MODE == kRope || MODE == kRope8;
    static_assert(!ROPE || R == 8 || R == 4 || R == 2, "rope epilogue: R/2 rotate-half pairs per workgroup");
    constexpr int RP = R / 2;            // rope: rotate-half pairs per workgroup
    constexpr int RWG = ROPE ? 64 / RP : 1;  // rope: workgroups per head
    constexpr int NPQ = M == 1 ? 8 : 4;  // NORMP: float4 partials per lane (<= 2048 / 1024 per row)
    constexpr int NR = SWIGLU ? 2 * R : R;  // weight rows streamed per group
    constexpr int V = NR * M;               // partial sums per lane
    // register ring depth (VGPR budget): M = 2 with 8 rows at depth 3 took all 256 VGPRs (one wave per SIMD)
    constexpr int XV = WQ ? 2 : 1;         // 16-B x pieces per lane per chunk
    constexpr int DEPTH = (NR + XV * M) * 4 < 40 ? 3 : 2;
    // gn < 0: check the decode gate BEFORE the first weight loads (a closed gate then streams no weights; an open one
    // pays the state read's latency up front).  gn > 0: after them (below).
    if (gn < 0 && gate_closed(gst, -gn)) return;
    int g = blockIdx.x;
    if (g >= ngroups) return;
    __shared__ float red[4][V];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nchunk = WQ ? K >> 10 : K >> 9;  // 1 KiB weight chunks per row (512 bf16 / 1024 e4m3 elements)
    // weight row of the group's r-th streamed row
    auto rowidx = [&](int bid, int r) {
        if constexpr (ROPE) return (bid / RWG) * 128 + (r < RP ? 0 : 64) + RP * (bid % RWG) + (r % RP);
        else return (SWIGLU && r >= R) ? half + bid * R + (r - R) : bid * R + r;
    };
    // row bases are wave-uniform (SGPR pairs); the per-lane part is one 32-bit offset (lane + 64 * chunk) * 16 B
    const u16x8* wrow[NR];
    auto set_rows = [&](int bid) {
#pragma unroll
        for (int r = 0; r < NR; ++r)
            wrow[r] = reinterpret_cast<const u16x8*>(reinterpret_cast<const uint8_t*>(W) +
                                                     (int64_t)rowidx(bid, r) * K * (WQ ? 1 : 2));
    };
    const u16x8* xr = reinterpret_cast<const u16x8*>(x);
    const int xstride = K >> 3;
    u16x8 wr[DEPTH][NR], xv[DEPTH][M][XV];
    auto load = [&](int c, int d) {
        const int off = c * 64 + lane;
#pragma unroll
        for (int r = 0; r < NR; ++r) wr[d][r] = ld_nt(wrow[r] + off);
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int v = 0; v < XV; ++v)
                xv[d][m][v] = m < mrows ? xr[m * xstride + (WQ ? c * 128 + 2 * lane + v : off)]
                                        : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    };
    // wave w takes chunks w, w+4, w+8, ... of every row
    auto prologue = [&]() {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d)
            if (w + 4 * d < nchunk) load(w + 4 * d, d);
    };
    // NORMP: the producer's partials (<= 1024 per row; the same for every group) are fetched FIRST, as up to 4
    // float4 per lane all in flight, so the reduction below waits only for them (vmcnt is in order) and never for
    // the weight ring issued after them
    float4 pv[M][NPQ];
    if constexpr (NORMP) {
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int q = 0; q < NPQ; ++q) {
                const int i = (q * 64 + lane) * 4;
                pv[m][q] = (m < mrows && i < nrm.nparts)
                               ? *reinterpret_cast<const float4*>(nrm.part + m * nrm.nparts + i)
                               : float4{0.f, 0.f, 0.f, 0.f};
            }
    }
    set_rows(g);
    prologue();
    // late gate: checked with the first loads already in flight (a closed gate then wastes their bandwidth)
    if (gn > 0 && gate_closed(gst, gn)) return;
    float inv[M];
#pragma unroll
    for (int m = 0; m < M; ++m) inv[m] = 1.f;
    if constexpr (NORMP) {
        // every wave reduces the partials itself in the same fixed order: no barrier, identical inv in all waves
#pragma unroll
        for (int m = 0; m < M; ++m) {
            float ss = 0.f;
#pragma unroll
            for (int q = 0; q < NPQ; ++q) ss += (pv[m][q].x + pv[m][q].y) + (pv[m][q].z + pv[m][q].w);
            inv[m] = rsqrtf(wave_sum(ss) / (float)K + nrm.eps);
        }
    }
    // row sums (NORMP: times the row's inv — the folded RMSNorm; 1 otherwise)
    auto invm = [&](int m) {  // select chain: a runtime index into inv[] would put it in scratch
        float v = inv[0];
#pragma unroll
        for (int j = 1; j < M; ++j) v = m == j ? inv[j] : v;
        return v;
    };
    auto tot = [&](int i) { return (red[0][i] + red[1][i] + red[2][i] + red[3][i]) * invm(i % M); };
    while (true) {
        float acc[V];
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] = 0.f;
        for (int c0 = w; c0 < nchunk; c0 += 4 * DEPTH) {
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
                const int c = c0 + 4 * d;
                if (c < nchunk) {
#pragma unroll
                    for (int r = 0; r < NR; ++r) {
                        if constexpr (WQ) {
                            bf16x2_t wb[8];
                            q2bf(wr[d][r], wb);
#pragma unroll
                            for (int m = 0; m < M; ++m)
                                acc[r * M + m] = dot16(wb, xv[d][m][0], xv[d][m][1], acc[r * M + m]);
                        } else {
#pragma unroll
                            for (int m = 0; m < M; ++m) acc[r * M + m] = dot8(wr[d][r], xv[d][m][0], acc[r * M + m]);
                        }
                    }
                    if (c + 4 * DEPTH < nchunk) load(c + 4 * DEPTH, d);
                }
            }
        }
        const int bid = g, n0 = g * R;
        // the row sum of output i (= r * M + m) with its row's fp8 weight scale
        auto totw = [&](int i) {
            float v = tot(i);
            if constexpr (WQ) v *= nrm.wscale[rowidx(bid, i / M)];
            return v;
        };
        g += gridDim.x;
        const bool more = g < ngroups;
        if (more) {  // the ring is consumed: start the next group's weight stream before this group's epilogue
            set_rows(g);
            prologue();
        }
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const float s = wave_sum(acc[i]);
            if (lane == 0) red[w][i] = s;
        }
        __syncthreads();
        if constexpr (ROPE) {
            // thread t < RP*M: pair (r, r+RP) of row m; the unfused path rounds the GEMM output to bf16 before RoPE
            const int t = threadIdx.x;
            const int pr = t / M, m = t % M;
            if (t < RP * M && m < mrows) {
                const int unit = bid / RWG, d = RP * (bid % RWG) + pr;  // head (q | k | v), dim in [0, 64)
                const float x1 = bf2f(f2bf(totw(pr * M + m))), x2 = bf2f(f2bf(totw((pr + RP) * M + m)));
                const int p = rp.pos[m];
                const int64_t blk = rp.bt[(int64_t)rp.tok_seq[m] * rp.bt_stride + p / rp.bs];
                const int off = p % rp.bs;
                if (unit < rp.hq + rp.hkv) {
                    const float c = rp.cos_sin[(int64_t)p * 128 + d], sn = rp.cos_sin[(int64_t)p * 128 + 64 + d];
                    const float fa = x1 * c - x2 * sn, fb = x2 * c + x1 * sn;
                    if (unit < rp.hq) {
                        uint16_t* dst = rp.q_out + ((int64_t)m * rp.hq + unit) * 128;
                        dst[d] = f2bf(fa);
                        dst[64 + d] = f2bf(fb);
                    } else if constexpr (MODE == kRope8) {
                        uint8_t* dst =
                            reinterpret_cast<uint8_t*>(rp.kc) + ((blk * rp.hkv + (unit - rp.hq)) * rp.bs + off) * 128;
                        const uint32_t q = f32x4_to_fp8x4(fa * rp.k_inv, fb * rp.k_inv, 0.f, 0.f);
                        dst[d] = (uint8_t)q;
                        dst[64 + d] = (uint8_t)(q >> 8);
                    } else {
                        uint16_t* dst =
                            reinterpret_cast<uint16_t*>(rp.kc) + ((blk * rp.hkv + (unit - rp.hq)) * rp.bs + off) * 128;
                        dst[d] = f2bf(fa);
                        dst[64 + d] = f2bf(fb);
                    }
                } else {  // v: transposed [blk, h, dim, slot]
                    const int64_t base = ((blk * rp.hkv + (unit - rp.hq - rp.hkv)) * 128) * (int64_t)rp.bs + off;
                    if constexpr (MODE == kRope8) {
                        uint8_t* dst = reinterpret_cast<uint8_t*>(rp.vc) + base;
                        const uint32_t q = f32x4_to_fp8x4(x1 * rp.v_inv, x2 * rp.v_inv, 0.f, 0.f);
                        dst[(int64_t)d * rp.bs] = (uint8_t)q;
                        dst[(int64_t)(64 + d) * rp.bs] = (uint8_t)(q >> 8);
                    } else {
                        uint16_t* dst = reinterpret_cast<uint16_t*>(rp.vc) + base;
                        dst[(int64_t)d * rp.bs] = f2bf(x1);
                        dst[(int64_t)(64 + d) * rp.bs] = f2bf(x2);
                    }
                }
            }
        } else if constexpr (MODE == kResid) {
            // s = bf16(bf16(y) + r) -> rout; per-row sum of s^2 over this group's R outputs -> part_out (fixed order)
            __shared__ float sq[R * M];
            const int t = threadIdx.x;
            if (t < R * M) {
                const int r = t / M, m = t % M;
                float v = 0.f;
                if (m < mrows) {
                    const int64_t i = (int64_t)m * nout + n0 + r;
                    const uint16_t sb = f2bf(bf2f(f2bf(totw(t))) + bf2f(nrm.rin[i]));
                    nrm.rout[i] = sb;
                    v = bf2f(sb) * bf2f(sb);
                }
                sq[t] = v;
            }
            __syncthreads();
            if (t < M && t < mrows) {
                float ss = 0.f;
#pragma unroll
                for (int r = 0; r < R; ++r) ss += sq[r * M + t];
                nrm.part_out[t * ngroups + bid] = ss;
            }
        } else {
            for (int t = threadIdx.x; t < R * M; t += 256) {
                const int r = t / M, m = t % M;
                if (m >= mrows) continue;
                const float gv = totw(r * M + m);
                if constexpr (SWIGLU) {
                    const float u = totw((R + r) * M + m);
                    const float gb = bf2f(f2bf(gv)), ub = bf2f(f2bf(u));  // the unfused path rounds the GEMM outputs
                    const float sg = bf2f(f2bf(gb / (1.f + __expf(-gb))));
                    y[(int64_t)m * nout + n0 + r] = f2bf(sg * ub);
                } else {
                    y[(int64_t)m * nout + n0 + r] = f2bf(gv);
                }
            }
        }
        if (!more) break;
        __syncthreads();  // red / sq are rewritten by the next group
    }
}

// R rows per workgroup: as many as the in-wave reduce-scatter (<= 64 sums per lane) allows, so x (re-read from L2 per
// chunk) stays a small fraction of the weight bytes.
template <int M>
constexpr int rows_plain() { return M <= 2 ? 8 : 4; }
template <int M>
constexpr int rows_swiglu() { return M <= 2 ? 4 : 2; }

// kResid rows per workgroup at M = 1: 4 (or 2 / 8 by knob) while the consumer's partial reduction (<= 2048 per row at
// M = 1) still covers N / R, else 8.  The partials buffer is sized by gemv_resid_parts with the same choice.
// fp8 weights (WQ): twice the rows per group — a group then streams the same bytes as the bf16 kernel's (at K = 4096
// a wave holds a single 1 KiB chunk per row, so the per-group reduction / epilogue is amortised over 2x the rows)
static int resid_rows(int N, bool wq = false) {
    const int r = wq ? knob("gemv_q_r_resid", 8) : knob("gemv_r_resid", 4);
    if (r == 2 && N / 2 <= 2048 && N % 2 == 0) return 2;
    return (r == 4 && N / 4 <= 2048 && N % 4 == 0) ? 4 : 8;
}

// Rows per workgroup at M = 1 (one sensor stream), knobs gemv_r_plain / gemv_r_swiglu / gemv_r_resid / gemv_r_rope for
// in-process A/B; values that are not instantiated fall back to the default.  Isolated kernels on cold weights run
// 5-13 % faster with fewer rows per workgroup (profiles/r2_gemv_rows.json: LM head 155.6 -> 141 us at R = 2, gate_up
// 40.7 -> 35.9 us at R = 2), but inside the captured single-stream decode step only the two small-N projections gain:
// QKV+RoPE and the residual producers at R = 4 (768 -> 1536 and 512 -> 1024 workgroups: one round of 2-3 workgroups
// per CU is latency-bound) give 3.16-3.18 ms/token against 3.24 for R = 8; gate_up stays at 4 (R = 8: 3.72, R = 2:
// 3.25) and the plain GEMV at 8 (scripts/single_stream.py --knob-ab, profiles/r2_single_stream_gemv_rows_ab2.json).
static int rows_knob(const char* name, int dflt) {
    const int v = knob(name, dflt);
    return (v == 1 || v == 2 || v == 4 || v == 8 || v == 16) ? v : dflt;
}

template <int M, bool WQ = false>
static void launch_m(const uint16_t* x, int mrows, int K, const uint16_t* W, int N, uint16_t* y, int mode,
                     const GemvNorm* nrm, const GemvRope* rp, hipStream_t st, const float* wscale = nullptr) {
    // WQ: twice the plain rows (O / down / QKV groups then stream the bf16 kernel's bytes); SwiGLU keeps its rows
    // (gate_up at M = 1: 27.4 us with 4 + 4 rows, 35.9 with 8 + 8; profiles/r5/w8a16_*)
    constexpr int R1 = rows_plain<M>() * (WQ ? 2 : 1), R2 = rows_swiglu<M>();
    constexpr int RP = rows_plain<M>();  // kResid / M = 2 rope rows (the partials layout: gemv_resid_parts)
    const GemvNorm nz{};
    const GemvRope rz{};
    GemvNorm na = nrm ? *nrm : nz;
    na.wscale = wscale;
    const GemvRope ra = rp ? *rp : rz;
    const bool np = nrm && nrm->part;  // consumer of a kResid producer
    const int32_t* gst = g_gate_n > 0 && g_gate_n <= kGateMax ? g_gate_state : nullptr;
    // early gate by default: a gated single-stream step (after the verdict closed or the row parked for a jump)
    // costs 0.28 ms instead of 2.25 (the late check let every workgroup issue its first ring of weight loads, which
    // at K = 4096 is the whole row), and the live step is no slower (3.60 vs 3.72 ms/token; profiles/r2_studies.md)
    const int gn = gst ? (knob("gemv_early_gate", 1) ? -g_gate_n : g_gate_n) : 0;
    // Persistent grid: the workgroups that fit on the device at once (occupancy x CUs), each looping over row groups
    // with the next group's weight ring prefetched.  A grid of 512 for every kernel (two per CU, what the 2-wave
    // gate_up fits) measured 2.88 ms/token in the single-stream decode step against 3.06 with one workgroup per group
    // (256: 3.55, 384: 3.10, 640: 3.17, 1024: 2.95 — counts beyond what fits serialise; profiles/
    // r2_single_stream_gemv_persist_ab.json).  Knob gemv_persist: 0 = one workgroup per group, N > 0 = at most N.
    const int persist = knob("gemv_persist", -1);
#define GV(MODE_, NP_, RR, GRID, NOUT, HALF)                                                                     \
    do {                                                                                                         \
        const int fit_ = resident_workgroups(gemv_kernel<M, RR, MODE_, NP_, WQ>, 256);                          \
        const int cap_ = persist == 0 ? (GRID) : persist > 0 && persist < fit_ ? persist : fit_;                 \
        hipLaunchKernelGGL((gemv_kernel<M, RR, MODE_, NP_, WQ>), dim3(cap_ < (GRID) ? cap_ : (GRID)), dim3(256), \
                           0,                                                                                    \
                           st, x, mrows, K, W, y, NOUT, HALF, na, ra, gst, gn, (GRID));                          \
    } while (0)
    if (mode == kSwiglu) {
        const int F = N / 2;
        if constexpr (M == 1) {
            const int r = rows_knob(WQ ? "gemv_q_r_swiglu" : "gemv_r_swiglu", R2);
            if (r == 1) {
                if (np) GV(kSwiglu, true, 1, F, F, F); else GV(kSwiglu, false, 1, F, F, F);
                return;
            }
            if (r == 2 && F % 2 == 0) {
                if (np) GV(kSwiglu, true, 2, F / 2, F, F); else GV(kSwiglu, false, 2, F / 2, F, F);
                return;
            }
            if (r == 8 && F % 8 == 0) {
                if (np) GV(kSwiglu, true, 8, F / 8, F, F); else GV(kSwiglu, false, 8, F / 8, F, F);
                return;
            }
        }
        if (np) GV(kSwiglu, true, R2, F / R2, F, F);
        else GV(kSwiglu, false, R2, F / R2, F, F);
    } else if (mode == kPlain) {
        if constexpr (M == 1) {
            const int r = rows_knob(WQ ? "gemv_q_r_plain" : "gemv_r_plain", R1);
            if (r == 2 && N % 2 == 0) {
                if (np) GV(kPlain, true, 2, N / 2, N, 0); else GV(kPlain, false, 2, N / 2, N, 0);
                return;
            }
            if (r == 4 && N % 4 == 0) {
                if (np) GV(kPlain, true, 4, N / 4, N, 0); else GV(kPlain, false, 4, N / 4, N, 0);
                return;
            }
            if (r == 16 && N % 16 == 0) {
                if (np) GV(kPlain, true, 16, N / 16, N, 0); else GV(kPlain, false, 16, N / 16, N, 0);
                return;
            }
        }
        if (np) GV(kPlain, true, R1, N / R1, N, 0);
        else GV(kPlain, false, R1, N / R1, N, 0);
    } else if constexpr (M <= 2) {
        if (mode == kResid) {
            const int r = M == 1 ? resid_rows(N, WQ) : RP;
            if constexpr (M == 1) {
                if (r == 4) {
                    GV(kResid, false, 4, N / 4, N, 0);
                    return;
                }
                if (r == 2) {
                    GV(kResid, false, 2, N / 2, N, 0);
                    return;
                }
            }
            GV(kResid, false, RP, N / RP, N, 0);
        } else {
            const int r = M == 1 ? rows_knob(WQ ? "gemv_q_r_rope" : "gemv_r_rope", WQ ? 8 : 4) : 8;
            if (mode == kRope) {
                if (r == 4) {
                    if (np) GV(kRope, true, 4, N / 4, N, 0); else GV(kRope, false, 4, N / 4, N, 0);
                } else if (r == 2) {
                    if (np) GV(kRope, true, 2, N / 2, N, 0); else GV(kRope, false, 2, N / 2, N, 0);
                } else {
                    if (np) GV(kRope, true, 8, N / 8, N, 0); else GV(kRope, false, 8, N / 8, N, 0);
                }
            } else {
                if (r == 4) {
                    if (np) GV(kRope8, true, 4, N / 4, N, 0); else GV(kRope8, false, 4, N / 4, N, 0);
                } else if (r == 2) {
                    if (np) GV(kRope8, true, 2, N / 2, N, 0); else GV(kRope8, false, 2, N / 2, N, 0);
                } else {
                    if (np) GV(kRope8, true, 8, N / 8, N, 0); else GV(kRope8, false, 8, N / 8, N, 0);
                }
            }
        }
    }
#undef GV
}

void launch_gemv(const uint16_t* x, int M, int K, const uint16_t* W, int N, uint16_t* y, bool swiglu,
                 hipStream_t st) {
    if (M <= 0) return;
    const int mode = swiglu ? kSwiglu : kPlain;
    if (M == 1) launch_m<1>(x, M, K, W, N, y, mode, nullptr, nullptr, st);
    else if (M == 2) launch_m<2>(x, M, K, W, N, y, mode, nullptr, nullptr, st);
    else if (M <= 4) launch_m<4>(x, M, K, W, N, y, mode, nullptr, nullptr, st);
    else launch_m<8>(x, M, K, W, N, y, mode, nullptr, nullptr, st);
}

void launch_gemv_ex(const uint16_t* x, int M, int K, const uint16_t* W, int N, uint16_t* y, bool swiglu,
                    const GemvNorm* nrm, const GemvRope* rope, bool fp8, hipStream_t st, const float* wscale) {
    if (M <= 0) return;
    const int mode = rope ? (fp8 ? kRope8 : kRope) : swiglu ? kSwiglu : kPlain;
    if (wscale) {
        if (M == 1) launch_m<1, true>(x, M, K, W, N, y, mode, nrm, rope, st, wscale);
        else launch_m<2, true>(x, M, K, W, N, y, mode, nrm, rope, st, wscale);
        return;
    }
    if (M == 1) launch_m<1>(x, M, K, W, N, y, mode, nrm, rope, st);
    else launch_m<2>(x, M, K, W, N, y, mode, nrm, rope, st);
}

int gemv_resid_parts(int M, int N, bool wq) {
    return N / (M == 1 ? resid_rows(N, wq) : M <= 2 ? rows_plain<2>() : rows_plain<4>());
}

void launch_gemv_q(const uint16_t* x, int M, int K, const uint8_t* W, const float* wscale, int N, uint16_t* y,
                   bool swiglu, hipStream_t st) {
    if (M <= 0) return;
    const uint16_t* w = reinterpret_cast<const uint16_t*>(W);
    const int mode = swiglu ? kSwiglu : kPlain;
    if (M == 1) launch_m<1, true>(x, M, K, w, N, y, mode, nullptr, nullptr, st, wscale);
    else if (M == 2) launch_m<2, true>(x, M, K, w, N, y, mode, nullptr, nullptr, st, wscale);
    else launch_m<4, true>(x, M, K, w, N, y, mode, nullptr, nullptr, st, wscale);
}

int launch_gemv_resid(const uint16_t* x, int M, int K, const uint16_t* W, int N, const uint16_t* rin, uint16_t* rout,
                      float* part_out, hipStream_t st, const float* wscale) {
    if (M <= 0) return 0;
    GemvNorm nrm{};
    nrm.rin = rin;
    nrm.rout = rout;
    nrm.part_out = part_out;
    if (wscale) {
        if (M == 1) launch_m<1, true>(x, M, K, W, N, nullptr, kResid, &nrm, nullptr, st, wscale);
        else launch_m<2, true>(x, M, K, W, N, nullptr, kResid, &nrm, nullptr, st, wscale);
    } else if (M == 1) launch_m<1>(x, M, K, W, N, nullptr, kResid, &nrm, nullptr, st);
    else launch_m<2>(x, M, K, W, N, nullptr, kResid, &nrm, nullptr, st);
    return gemv_resid_parts(M, N, wscale != nullptr);
}

}  // namespace chronos
