// fp8.hip — W8A8 fp8-e4m3 (OCP e4m3fn) projection path on the CDNA4 block-scaled MFMA (SURVEY.md §2.3 K3/K7/K8/K10
// "fp8 path via mfma_scale_f32_*_f8f6f4", §7.2 step 9; BASELINE.json config "CDNA4 fp8 MFMA").
//
//   y[M, N] = (Xq[M, K] · Wq[N, K]^T) · sx[m] · sw[n]          bf16 out, fp32 accumulate
//
// Xq / Wq are e4m3fn bytes, sx a per-token and sw a per-output-channel fp32 scale (weights quantised once at load,
// activations quantised dynamically by the producer kernels below, which have the whole row in registers).
//
// Why fp8 pays on MI355X: the non-scaled fp8 MFMA runs at the bf16 rate; the block-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 runs 4x the K of v_mfma_f32_16x16x32_bf16 in 2x its cycles, i.e. 2x the bf16
// FLOP rate (MI355X_MICROARCH.md §Matrix cores).  The hardware MX scales are fed the unit exponent (127 = 2^0) and the
// real per-token / per-channel scales are applied once in the epilogue.  Every staged byte carries twice the K of the
// bf16 kernel (csrc/kernels/gemm.hip): a 128 x 128 tile at BK = 128 bytes moves the same 32 KiB per K-step for twice
// the MFMA work, which is what the per-CU load path (the bf16 kernel's wall at ~0.9 PF) needed.
//
// Kernels:
//   quant_rows_kernel<MAXV, MODE>  one block per row: [residual add +] [RMSNorm +] amax -> e4m3 bytes + row scale
//   qgemm_kernel<STAGES, SWIGLU>   128x128x128 tile, 4 waves (2x2, 64x64 each = 4x4 scaled MFMAs per K-step), LDS-DMA
//                                  ring with counted vmcnt + raw barrier, XCD-aware tile order, fused SwiGLU epilogue
//   qgemv_kernel<M, R, SWIGLU>     M <= 8 decode rows: 1 KiB contiguous weight pieces straight to VGPRs; fp8 -> bf16
//                                  is exact (3 mantissa bits fit in 7), so v_dot2_f32_bf16 gives the MFMA path's math
#include "chronos_hip.h"

namespace chronos {
namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint8_t u8x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kScaleOne = 127;  // e8m0 exponent of 1.0 for the MX scale operands

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ float block_max(float v, float* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_max(v);
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = (threadIdx.x < (unsigned)nw) ? red[threadIdx.x] : 0.f;
    if (w == 0) t = wave_max(t);
    if (threadIdx.x == 0) red[0] = t;
    __syncthreads();
    const float r = red[0];
    __syncthreads();
    return r;
}

// ------------------------------------------------------------------------------------------------------------------
// Row quantisation producers.  MODE 0: q = quant(x); 1: q = quant(rmsnorm(x) * w); 2: r = bf16(x + r) written back,
// q = quant(rmsnorm(r) * w); 3: x is a [gate | up] row of 2d values, q = quant(silu(gate) * up).  The normalised value is rounded to bf16 first (the bf16 path's rounding), then scaled
// by 448 / amax(row) and converted with saturation; s[row] = amax / 448 (1 for an all-zero row).
// ------------------------------------------------------------------------------------------------------------------
template <int MAXV, int MODE>
__global__ void __launch_bounds__(256) quant_rows_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ resid,
                                                         const uint16_t* __restrict__ w, uint8_t* __restrict__ q,
                                                         float* __restrict__ qs, int d, float eps) {
    __shared__ float red[16];
    const int64_t row = blockIdx.x;
    const u16x8* xv = reinterpret_cast<const u16x8*>(x + row * (MODE == 3 ? 2 * d : d));
    const int nv = d / 8;
    float vals[MAXV][8];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < nv) {
            const u16x8 a = xv[i];
            if constexpr (MODE == 3) {  // SwiGLU of a [gate | up] row, rounded as silu_mul_kernel does
                const u16x8 u = xv[nv + i];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float g = bf2f(a[j]);
                    vals[k][j] = bf2f(f2bf(bf2f(f2bf(g / (1.f + __expf(-g)))) * bf2f(u[j])));
                }
            } else if constexpr (MODE == 2) {
                u16x8* rv = reinterpret_cast<u16x8*>(resid + row * d);
                const u16x8 b = rv[i];
                u16x8 s;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    s[j] = f2bf(bf2f(a[j]) + bf2f(b[j]));
                    vals[k][j] = bf2f(s[j]);
                }
                rv[i] = s;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) vals[k][j] = bf2f(a[j]);
            }
            if constexpr (MODE == 1 || MODE == 2) {
#pragma unroll
                for (int j = 0; j < 8; ++j) ss += vals[k][j] * vals[k][j];
            }
        }
    }
    float amax = 0.f;
    if constexpr (MODE == 1 || MODE == 2) {
        const float inv = rsqrtf(block_sum(ss, red) / (float)d + eps);
        const u16x8* wv = reinterpret_cast<const u16x8*>(w);
#pragma unroll
        for (int k = 0; k < MAXV; ++k) {
            const int i = threadIdx.x + k * 256;
            if (i < nv) {
                const u16x8 g = wv[i];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    vals[k][j] = bf2f(f2bf(bf2f(f2bf(vals[k][j] * inv)) * bf2f(g[j])));
                    amax = fmaxf(amax, fabsf(vals[k][j]));
                }
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < MAXV; ++k)
            if (threadIdx.x + k * 256 < nv)
#pragma unroll
                for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(vals[k][j]));
    }
    amax = block_max(amax, red);
    const float s = amax > 0.f ? amax / kFp8Max : 1.f;
    const float r = amax > 0.f ? kFp8Max / amax : 1.f;
    uint2* qv = reinterpret_cast<uint2*>(q + row * d);
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < nv) {
            const float* v = vals[k];
            qv[i] = uint2{f32x4_to_fp8x4(v[0] * r, v[1] * r, v[2] * r, v[3] * r),
                          f32x4_to_fp8x4(v[4] * r, v[5] * r, v[6] * r, v[7] * r)};
        }
    }
    if (threadIdx.x == 0) qs[row] = s;
}

// ------------------------------------------------------------------------------------------------------------------
// MFMA GEMM.  Swapped product D = W · X^T per 16x16 tile (W rows are the MFMA rows), so a lane's 4 accumulators are 4
// consecutive output columns of one token row (8-byte bf16 stores) and the SwiGLU pair (gate f, up F+f) sits in one
// lane.  The LDS images are [128 rows][128 B] with the 16-B chunk c of row r at slot c ^ (r & 7): the XOR is applied to
// the per-lane GLOBAL source of the lane-linear LDS-DMA (cdna_hip_programming.md §5.4 rule 21) and undone on read.
// Fragment of v_mfma_scale_f32_16x16x128_f8f6f4: lane l holds 32 k-bytes of row l & 15 — chunks 2(l>>4), 2(l>>4)+1 —
// for BOTH operands, so the instruction's k order is the same permutation on A and B and the dot product is exact.
// ------------------------------------------------------------------------------------------------------------------
constexpr int QBK = 128;           // K bytes per stage (one scaled-MFMA K step)
constexpr int kQRowBytes = QBK;    // one LDS image row

__device__ __forceinline__ i32x4 lds16(const unsigned char* img, int row, int chunk) {
    return *reinterpret_cast<const i32x4*>(img + row * kQRowBytes + ((chunk ^ (row & 7)) << 4));
}

// Tile geometry: WN x WM waves, each owning SN x SM 16x16 output sub-tiles -> TN = 16 WN SN W rows (output columns)
// by TM = 16 WM SM token rows.  <2,2,4,4> = 128x128 (4 waves, 3-stage ring fits 96 KiB of LDS); <4,2,4,8> = 256x256
// (8 waves, 2 stages = 128 KiB): 4x the MFMA work per staged byte of the 128x128 tile at 2x the bytes — the per-CU
// load path is latency-bound at a fixed number of bytes in flight, so FLOPs per byte are what buys throughput.
template <int WN, int WM, int SN, int SM, int STAGES, bool SWIGLU>
__global__ void __launch_bounds__(64 * WN * WM) qgemm_kernel(const uint8_t* __restrict__ x, const float* __restrict__ xs,
                                                            const uint8_t* __restrict__ w, const float* __restrict__ ws,
                                                            uint16_t* __restrict__ y, int M, int N, int K, int F) {
    constexpr int NW = WN * WM, TN = 16 * WN * SN, TM = 16 * WM * SM;
    constexpr int LW = TN / (8 * NW), LX = TM / (8 * NW);  // LDS-DMA instructions per wave per stage
    constexpr int WIMG = TN * kQRowBytes, XIMG = TM * kQRowBytes, STAGE = WIMG + XIMG;
    static_assert(LW >= 1 && LX >= 1 && TN % (8 * NW) == 0 && TM % (8 * NW) == 0, "tile / wave split");
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];  // STAGES x {W image, X image}
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int mt = (M + TM - 1) / TM;
    const int nt = SWIGLU ? F / (TN / 2) : N / TN;
    const int tile = xcd_remap(blockIdx.x, mt * nt);
    const int tn = tile / mt, tm = tile - tn * mt;  // token-row tiles fastest: neighbours share the W tile
    const int m0 = tm * TM;

    // per-lane LDS-DMA sources: instruction g (= wave * L + i) fills image rows [8g, 8g + 8); lane l -> row
    // 8g + (l >> 3), LDS slot l & 7 <- global chunk (l & 7) ^ (row & 7)
    const uint8_t* wsrc[LW];
    const uint8_t* xsrc[LX];
#pragma unroll
    for (int i = 0; i < LW; ++i) {
        const int r = 8 * (wave * LW + i) + (lane >> 3);
        const int c = (lane & 7) ^ (r & 7);
        int wrow;
        if constexpr (SWIGLU) wrow = r < TN / 2 ? tn * (TN / 2) + r : F + tn * (TN / 2) + (r - TN / 2);
        else wrow = tn * TN + r;
        wsrc[i] = w + (int64_t)wrow * K + c * 16;
    }
#pragma unroll
    for (int i = 0; i < LX; ++i) {
        const int r = 8 * (wave * LX + i) + (lane >> 3);
        const int c = (lane & 7) ^ (r & 7);
        xsrc[i] = x + (int64_t)min(m0 + r, M - 1) * K + c * 16;
    }
    auto issue = [&](int kt) {
        unsigned char* st = smem + (kt % STAGES) * STAGE;
        const int koff = kt * QBK;
#pragma unroll
        for (int i = 0; i < LW; ++i)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(wsrc[i] + koff), (lds_ptr_t)(st + (wave * LW + i) * 1024), 16,
                                             0, 0);
#pragma unroll
        for (int i = 0; i < LX; ++i)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(xsrc[i] + koff),
                                             (lds_ptr_t)(st + WIMG + (wave * LX + i) * 1024), 16, 0, 0);
    };

    const int wn = wave / WM, wm = wave - (wave / WM) * WM;
    int wrow0[SN];
#pragma unroll
    for (int s = 0; s < SN; ++s) {
        if constexpr (SWIGLU) wrow0[s] = s < SN / 2 ? 8 * SN * wn + 16 * s : TN / 2 + 8 * SN * wn + 16 * (s - SN / 2);
        else wrow0[s] = 16 * SN * wn + 16 * s;
    }
    f32x4 acc[SN][SM];
#pragma unroll
    for (int s = 0; s < SN; ++s)
#pragma unroll
        for (int t = 0; t < SM; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int KT = K / QBK;
#pragma unroll
    for (int p = 0; p < STAGES - 1; ++p)
        if (p < KT) issue(p);

    const int c0 = 2 * (lane >> 4), fr = lane & 15;
    for (int kt = 0; kt < KT; ++kt) {
        // retire stage kt (this wave's LW + LX DMAs of it); the younger stages stay in flight across the barrier
        if constexpr (STAGES > 2) {
            if (kt + STAGES - 2 < KT) wait_vmcnt<(LW + LX) * (STAGES - 2)>();
            else wait_vmcnt<0>();
        } else {
            wait_vmcnt<0>();
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + STAGES - 1 < KT) issue(kt + STAGES - 1);  // into the stage every wave finished reading at kt-1
        const unsigned char* wimg = smem + (kt % STAGES) * STAGE;
        const unsigned char* ximg = wimg + WIMG;
        i32x8 a[SN];
#pragma unroll
        for (int s = 0; s < SN; ++s) {
            const int r = wrow0[s] + fr;
            a[s] = __builtin_shufflevector(lds16(wimg, r, c0), lds16(wimg, r, c0 + 1), 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int t = 0; t < SM; ++t) {
            const int r = 16 * SM * wm + 16 * t + fr;
            const i32x8 b = __builtin_shufflevector(lds16(ximg, r, c0), lds16(ximg, r, c0 + 1), 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
            for (int s = 0; s < SN; ++s)
                acc[s][t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[s], b, acc[s][t], 0, 0, 0, kScaleOne, 0,
                                                                              kScaleOne);
        }
    }

    // epilogue: lane holds D[n = 4 (lane >> 4) + i][m = lane & 15] of each 16x16 tile = y[m][n .. n+3]
#pragma unroll
    for (int t = 0; t < SM; ++t) {
        const int m = m0 + 16 * SM * wm + 16 * t + fr;
        if (m >= M) continue;
        const float sxm = xs[m];
        if constexpr (SWIGLU) {
#pragma unroll
            for (int s = 0; s < SN / 2; ++s) {
                const int f = tn * (TN / 2) + 8 * SN * wn + 16 * s + 4 * (lane >> 4);
                const f32x4 sg = *reinterpret_cast<const f32x4*>(ws + f);
                const f32x4 su = *reinterpret_cast<const f32x4*>(ws + F + f);
                u16x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float g = bf2f(f2bf(acc[s][t][i] * sxm * sg[i]));
                    const float u = bf2f(f2bf(acc[s + SN / 2][t][i] * sxm * su[i]));
                    o[i] = f2bf(bf2f(f2bf(g / (1.f + __expf(-g)))) * u);
                }
                *reinterpret_cast<u16x4*>(y + (int64_t)m * F + f) = o;
            }
        } else {
#pragma unroll
            for (int s = 0; s < SN; ++s) {
                const int n = tn * TN + wrow0[s] + 4 * (lane >> 4);
                const f32x4 sw = *reinterpret_cast<const f32x4*>(ws + n);
                u16x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[s][t][i] * sxm * sw[i]);
                *reinterpret_cast<u16x4*>(y + (int64_t)m * N + n) = o;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------------------------
// Decode GEMV (M <= 8).  Every wave-wide load is one contiguous 1 KiB piece (1024 e4m3 weights) of one weight row;
// the matching 16 activation bytes of each token row come from L2.  Both are widened to bf16 exactly
// (v_cvt_scalef32_pk_bf16_fp8, scale 1) and multiplied with v_dot2_f32_bf16.  4 waves split K and meet in LDS.
// ------------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ float qdot16(const u8x16& wq, const bf16x2_t (&xb)[8], float acc) {
    const i32x4 wi = __builtin_bit_cast(i32x4, wq);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bf16x2_t lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(wi[j], 1.f, false);
        const bf16x2_t hi = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(wi[j], 1.f, true);
        acc = __builtin_amdgcn_fdot2_f32_bf16(lo, xb[2 * j], acc, false);
        acc = __builtin_amdgcn_fdot2_f32_bf16(hi, xb[2 * j + 1], acc, false);
    }
    return acc;
}

// Like gemv.hip's gemv_kernel: a grid of at most `gemv_persist` workgroups loops over the row groups (R rows each),
// issuing the next group's weight ring as soon as the current group's dot products have consumed it.
template <int M, int R, bool SWIGLU>
__global__ void __launch_bounds__(256) qgemv_kernel(const uint8_t* __restrict__ x, const float* __restrict__ xs,
                                                    int mrows, int K, const uint8_t* __restrict__ W,
                                                    const float* __restrict__ ws, uint16_t* __restrict__ y, int nout,
                                                    int half, const int32_t* __restrict__ gst, int gn, int ngroups) {
    if (gate_closed(gst, gn)) return;  // decode early-exit gate, read before any weight load (chronos_hip.h)
    int g = blockIdx.x;
    if (g >= ngroups) return;
    constexpr int NR = SWIGLU ? 2 * R : R;
    constexpr int V = NR * M;
    constexpr int DEPTH = (NR + M) * 4 <= 40 ? 3 : 2;
    __shared__ float red[4][V];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nchunk = K >> 10;  // 1024-byte chunks per row
    const u8x16* wrow[NR];
    auto set_rows = [&](int bid) {
        const int n0 = bid * R;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int row = (SWIGLU && r >= R) ? half + n0 + (r - R) : n0 + r;
            wrow[r] = reinterpret_cast<const u8x16*>(W + (int64_t)row * K);
        }
    };
    const u8x16* xr = reinterpret_cast<const u8x16*>(x);
    const int xstride = K >> 4;
    u8x16 wr[DEPTH][NR], xv[DEPTH][M];
    auto load = [&](int c, u8x16 (&wd)[NR], u8x16 (&xd)[M]) {
        const int off = c * 64 + lane;
#pragma unroll
        for (int r = 0; r < NR; ++r) wd[r] = __builtin_nontemporal_load(wrow[r] + off);
#pragma unroll
        for (int m = 0; m < M; ++m) xd[m] = m < mrows ? xr[m * xstride + off] : u8x16{};
    };
    auto prologue = [&]() {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d)
            if (w + 4 * d < nchunk) load(w + 4 * d, wr[d], xv[d]);
    };
    set_rows(g);
    prologue();
    while (true) {
        float acc[V];
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] = 0.f;
        for (int cb = w; cb < nchunk; cb += 4 * DEPTH) {
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
                const int c = cb + 4 * d;
                if (c < nchunk) {
#pragma unroll
                    for (int m = 0; m < M; ++m) {
                        bf16x2_t xb[8];
                        const i32x4 xi = __builtin_bit_cast(i32x4, xv[d][m]);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            xb[2 * j] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(xi[j], 1.f, false);
                            xb[2 * j + 1] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(xi[j], 1.f, true);
                        }
#pragma unroll
                        for (int r = 0; r < NR; ++r) acc[r * M + m] = qdot16(wr[d][r], xb, acc[r * M + m]);
                    }
                    if (c + 4 * DEPTH < nchunk) load(c + 4 * DEPTH, wr[d], xv[d]);
                }
            }
        }
        const int n0 = g * R;
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
        for (int t = threadIdx.x; t < R * M; t += 256) {
            const int r = t / M, m = t % M;
            if (m >= mrows) continue;
            const float sxm = xs[m];
            const float gv = (red[0][r * M + m] + red[1][r * M + m] + red[2][r * M + m] + red[3][r * M + m]) * sxm *
                             ws[n0 + r];
            if constexpr (SWIGLU) {
                const int ru = (R + r) * M + m;
                const float u = (red[0][ru] + red[1][ru] + red[2][ru] + red[3][ru]) * sxm * ws[half + n0 + r];
                const float gb = bf2f(f2bf(gv)), ub = bf2f(f2bf(u));
                y[(int64_t)m * nout + n0 + r] = f2bf(bf2f(f2bf(gb / (1.f + __expf(-gb)))) * ub);
            } else {
                y[(int64_t)m * nout + n0 + r] = f2bf(gv);
            }
        }
        if (!more) break;
        __syncthreads();  // red is rewritten by the next group
    }
}

template <int WN, int WM, int SN, int SM, int STAGES, bool SWIGLU>
void qgemm_geo(const uint8_t* x, const float* xs, const uint8_t* w, const float* ws, uint16_t* y, int M, int N, int K,
               int F, hipStream_t st) {
    constexpr int TN = 16 * WN * SN, TM = 16 * WM * SM;
    const int mt = (M + TM - 1) / TM;
    const int nt = SWIGLU ? F / (TN / 2) : N / TN;
    const int lds = STAGES * (TN + TM) * kQRowBytes;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(qgemm_kernel<WN, WM, SN, SM, STAGES, SWIGLU>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    hipLaunchKernelGGL((qgemm_kernel<WN, WM, SN, SM, STAGES, SWIGLU>), dim3(mt * nt), dim3(64 * WN * WM), lds, st, x, xs,
                       w, ws, y, M, N, K, F);
}

template <int M>
void qgemv_m(const uint8_t* x, const float* xs, int mrows, int K, const uint8_t* W, const float* ws, int N, uint16_t* y,
             bool swiglu, hipStream_t st) {
    constexpr int R1 = M <= 2 ? 8 : 4;
    constexpr int R2 = M <= 2 ? 4 : 2;
    const int persist = knob("gemv_persist", -1);  // as gemv.hip: resident workgroups; 0 = one per row group
    auto grid = [&](int groups, int fit) {
        const int cap = persist == 0 ? groups : persist > 0 && persist < fit ? persist : fit;
        return cap < groups ? cap : groups;
    };
    if (swiglu) {
        const int F = N / 2;
        hipLaunchKernelGGL((qgemv_kernel<M, R2, true>), dim3(grid(F / R2, resident_workgroups(qgemv_kernel<M, R2, true>, 256))),
                           dim3(256), 0, st, x, xs, mrows, K, W, ws, y, F, F, CHRONOS_GATE, F / R2);
    } else {
        hipLaunchKernelGGL((qgemv_kernel<M, R1, false>),
                           dim3(grid(N / R1, resident_workgroups(qgemv_kernel<M, R1, false>, 256))), dim3(256), 0, st,
                           x, xs, mrows, K, W, ws, y, N, 0, CHRONOS_GATE, N / R1);
    }
}

}  // namespace

void launch_quant_rows(const uint16_t* x, uint16_t* resid, const uint16_t* w, uint8_t* q, float* qs, int rows, int d,
                       float eps, int mode, hipStream_t st) {
    if (rows == 0) return;
    const int nv = d / 8;
    const dim3 g(rows), b(256);
#define QR_CASE(V)                                                                                               \
    if (nv <= 256 * V) {                                                                                         \
        if (mode == 0) hipLaunchKernelGGL((quant_rows_kernel<V, 0>), g, b, 0, st, x, resid, w, q, qs, d, eps);   \
        else if (mode == 1) hipLaunchKernelGGL((quant_rows_kernel<V, 1>), g, b, 0, st, x, resid, w, q, qs, d, eps); \
        else if (mode == 2) hipLaunchKernelGGL((quant_rows_kernel<V, 2>), g, b, 0, st, x, resid, w, q, qs, d, eps); \
        else hipLaunchKernelGGL((quant_rows_kernel<V, 3>), g, b, 0, st, x, resid, w, q, qs, d, eps);             \
        return;                                                                                                  \
    }
    QR_CASE(1) QR_CASE(2) QR_CASE(4) QR_CASE(8)
#undef QR_CASE
}

// y = (xq · wq^T) * xs * ws; swiglu: wq = [gate; up] (N = 2F rows) and y = silu(gate) * up, [M, F]
void launch_qlinear(const uint8_t* x, const float* xs, const uint8_t* w, const float* ws, uint16_t* y, int M, int N,
                    int K, bool swiglu, hipStream_t st) {
    if (M == 0) return;
    const int gemv_max = knob("qgemv_max_m", 4);
    if (M <= gemv_max && M <= 8 && K % 1024 == 0) {  // GEMV streams whole 1 KiB row pieces
        if (M == 1) qgemv_m<1>(x, xs, M, K, w, ws, N, y, swiglu, st);
        else if (M == 2) qgemv_m<2>(x, xs, M, K, w, ws, N, y, swiglu, st);
        else if (M <= 4) qgemv_m<4>(x, xs, M, K, w, ws, N, y, swiglu, st);
        else qgemv_m<8>(x, xs, M, K, w, ws, N, y, swiglu, st);
        return;
    }
    const int F = N / 2;
    // 256x256 tiles where they fill the chip (and the shape divides), else 128x128
    int geo = knob("qgemm_tile", 0);
    const bool fits256 = (swiglu ? F % 128 : N % 256) == 0;
    if (geo == 0) {
        const int64_t t256 = (int64_t)((M + 255) / 256) * (swiglu ? F / 128 : N / 256);
        geo = (t256 >= 256 && fits256) ? 256 : 128;
    }
    if (!fits256) geo = 128;  // a forced knob never launches a geometry the shape does not divide
    if (geo == 256) {
        if (swiglu) qgemm_geo<4, 2, 4, 8, 2, true>(x, xs, w, ws, y, M, N, K, F, st);
        else qgemm_geo<4, 2, 4, 8, 2, false>(x, xs, w, ws, y, M, N, K, F, st);
    } else {
        if (swiglu) qgemm_geo<2, 2, 4, 4, 3, true>(x, xs, w, ws, y, M, N, K, F, st);
        else qgemm_geo<2, 2, 4, 4, 3, false>(x, xs, w, ws, y, M, N, K, F, st);
    }
}

}  // namespace chronos
