// gemm_skinny.hip — skinny-M projection GEMM (M = 3..128 rows): jump-forward forwards, the tail decode buckets and
// 70B TP=8 per-GPU decode (SURVEY.md §2.3 K3/K7/K8/K10/K11, §7.3 hard part 1; VERDICT r2 "skinny-M GEMM").
//
//   y[M, N] = x[M, K] · W[N, K]^T   (bf16 in, fp32 accumulate) with the batched family's epilogues (chronos_gemm.h):
//   plain, SwiGLU (w = [gate; up]), residual add + RMSNorm partial sums (kResid producer), folded-norm row scale
//   (NORMP consumer of a kResid producer's partials).
//
// At these M the op is a weight stream (the whole W once per call) with at most 64 columns of arithmetic per weight
// element, so the design is the decode GEMV's (gemv.hip) with the dot products moved onto the matrix cores:
//   * a workgroup owns 16*RT output rows (RT MFMA A tiles) and a K range; its NW waves split that range in 64-k
//     units (wave w takes units w, w+NW, ...), so the main loop has no barrier and no LDS at all.  NW up to 16 waves
//     gives the latency hiding of 4 waves per SIMD without splitting K across workgroups: a cross-workgroup split
//     costs an agent-scope release per workgroup (an L2 write-back) plus the slab round trip — 15-25 us on the 8B
//     decode shapes, more than the whole weight stream (profiles/r3_gemm_table.md);
//   * W goes straight from HBM into VGPRs in the v_mfma_f32_16x16x32_bf16 A layout (lane l: row l&15, k 8(l>>4)..+8
//     of each 32-k block).  A unit is two such loads per A tile, i.e. one full 128-B line of each of 16 rows;
//     x (L2-resident: <= 128 x K bf16) comes the same way as the B operand (column = x row l&15), rows >= M clamped;
//   * a register ring D units deep keeps D * RT KiB of weights in flight per wave (in-order vmcnt: the compiler's
//     counted waits retire the oldest unit only);
//   * MT x tiles of 16 rows (M <= 16 MT), RT W tiles: x bytes / W bytes = MT / RT per wave, kept <= 2 so the TCP
//     carries the weight stream plus the x re-reads;
//   * the NW waves' accumulators meet in LDS (fixed order), optional split-K across workgroups through write-through
//     fp32 slabs and an agent-scope ticket whose last arriver sums the slabs in slice order (no fences; bitwise
//     reproducible, graph == eager);
//   * epilogue per (row m, 4 consecutive outputs): 8-byte stores, CPR consecutive lanes cover a row's 16 RT outputs.
#include <algorithm>

#include "chronos_gemm.h"
#include "chronos_hip.h"

namespace chronos {
namespace {

enum : int { kPlain = kPPPlain, kSwiglu = kPPSwiglu, kResid = kPPResid };
constexpr int XL_MIN_MT = 2;  // x staged through LDS from MT = 2 (x bytes >= the weight bytes per wave)

template <int RT, int MT, int D, int NW, int MODE, bool NORMP>
__global__ void __launch_bounds__(64 * NW) skinny_kernel(PPArgs a) {
    static_assert(MODE != kSwiglu || RT % 2 == 0, "swiglu: RT/2 gate tiles + RT/2 up tiles");
    constexpr int NT = 64 * NW;                        // threads
    constexpr int UNITS = RT * MT * 64;                // f32x4 accumulators per wave
    constexpr int CPR = MODE == kSwiglu ? 2 * RT : 4 * RT;  // output units (4 columns each) per row
    constexpr int NOUT = 16 * MT * CPR;                // output units per workgroup (a multiple of 64)
    constexpr int VP = NOUT >= NT ? NOUT / NT : 1;     // output units per thread
    constexpr int PAIR = MODE == kSwiglu ? 2 : 1;       // swiglu: a gate unit and its up unit
    constexpr int NP = NOUT + NOUT / 16;               // one padded half (pad: 1 slot per 16, see red_at)
    constexpr int SZ = PAIR * NP;                      // f32x4 slots per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    f32x4* red = reinterpret_cast<f32x4*>(smem);       // [NW waves][SZ]
    float* inv = reinterpret_cast<float*>(smem + NW * SZ * 16);  // [16 MT]
    int* flag = reinterpret_cast<int*>(inv + 16 * MT);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int M = a.M, K = a.K, S = a.splitk;
    const int G = MODE == kSwiglu ? a.F / (8 * RT) : a.N / (16 * RT);
    const int task = xcd_remap(blockIdx.x, G * S);
    const int g = task / S, s = task - g * S;
    const int KS = K / S;
    const int NU = KS / (64 * NW);  // 64-k units per wave
    const int kbase = s * KS + wave * 64 + 8 * (lane >> 4);

    const bf16x8* wp[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        int row;
        if constexpr (MODE == kSwiglu)
            row = rt < RT / 2 ? g * 8 * RT + 16 * rt : a.F + g * 8 * RT + 16 * (rt - RT / 2);
        else
            row = g * 16 * RT + 16 * rt;
        wp[rt] = reinterpret_cast<const bf16x8*>(a.w + (int64_t)(row + (lane & 15)) * K + kbase);
    }
    // XL (MT >= XL_MIN_MT, x bytes = MT / RT x the weight bytes): x is loaded in whole 128-B lines (lane l: row 8 i + l / 8,
    // 16-B chunk l % 8 of the unit's 64 k) and turned into the MFMA B layout through the wave's private LDS tile
    // (swizzled ds_write_b128, ds_read_b128).  Loads shaped like the MFMA operand (16 rows x 64 B per instruction)
    // reach only ~18 B/clk per CU from L2 against ~50 for whole lines (csrc/microbench/l2_feed.hip): at M = 128 the x
    // re-reads, not the weight stream, set the kernel time.
    constexpr bool XL = MT >= XL_MIN_MT;
    const bf16x8* xp[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        if constexpr (XL)  // pieces of 8 rows: xp[i] for i < 2 MT covers rows 8 i .. 8 i + 7
            xp[mt] = nullptr;
        else
            xp[mt] = reinterpret_cast<const bf16x8*>(a.x + (int64_t)min(16 * mt + (lane & 15), M - 1) * K + kbase);
    }
    const bf16x8* xl[XL ? 2 * MT : 1];
    if constexpr (XL) {
#pragma unroll
        for (int i = 0; i < 2 * MT; ++i)
            xl[i] = reinterpret_cast<const bf16x8*>(a.x + (int64_t)min(8 * i + (lane >> 3), M - 1) * K + s * KS +
                                                    wave * 64 + 8 * (lane & 7));
    }
    unsigned char* xs = smem + wave * (MT * 2048);  // XL: this wave's x tile, 16 MT rows x 128 B

    // unit u of this wave covers k = kbase + 64 NW u + {0, 32} (+ 8 (lane >> 4) already in the pointers)
    bf16x8 wr[D][RT][2], xr[D][MT][2];
    auto load = [&](int u, int d) {
        const int off = u * 8 * NW;  // 64 NW bf16 = 8 NW bf16x8
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            wr[d][rt][0] = __builtin_nontemporal_load(wp[rt] + off);
            wr[d][rt][1] = __builtin_nontemporal_load(wp[rt] + off + 4);
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            if constexpr (XL) {  // the same registers, in the line layout: piece 2 mt + h
                xr[d][mt][0] = xl[2 * mt][off];
                xr[d][mt][1] = xl[2 * mt + 1][off];
            } else {
                xr[d][mt][0] = xp[mt][off];
                xr[d][mt][1] = xp[mt][off + 4];
            }
        }
    };
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (d < NU) load(d, d);

    f32x4 acc[RT][MT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[rt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int u0 = 0; u0 < NU; u0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int u = u0 + d;
            if (u < NU) {
                if constexpr (XL) {
                    // line layout -> LDS (row t = 8 i + lane / 8, chunk lane % 8 in slot chunk ^ (t & 7)) -> MFMA layout
                    // (row 16 mt + lane % 16, chunk 4 h + lane / 16); LDS ops of a wave run in order, so the previous
                    // unit's reads are served before these writes
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int t = 8 * (2 * mt + h) + (lane >> 3);
                            *reinterpret_cast<bf16x8*>(xs + t * 128 + (((lane & 7) ^ (t & 7)) << 4)) = xr[d][mt][h];
                        }
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int t = 16 * mt + (lane & 15);
                            xr[d][mt][h] = *reinterpret_cast<const bf16x8*>(
                                xs + t * 128 + (((4 * h + (lane >> 4)) ^ (t & 7)) << 4));
                        }
                }
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
                            acc[rt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[d][rt][h], xr[d][mt][h],
                                                                                  acc[rt][mt], 0, 0, 0);
                if (u + D < NU) load(u + D, d);
            }
        }
    }

    // XL: the reduction slots, inv and the flag alias the other waves' x tiles — wait until every wave's loop is done
    if constexpr (XL) __syncthreads();
    // NORMP: inv[m] of the x rows from the producer's partials — fetched only now, so these loads never sit in front
    // of the weight ring in the in-order vmcnt queue
    if constexpr (NORMP) {
        // every load of the wave's rows issued before any is reduced: one memory latency, not one per row
        constexpr int RPW = (16 * MT + NW - 1) / NW;
        float pv[RPW];
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int m = min(wave + NW * j, M - 1);
            pv[j] = lane < a.nparts_in ? a.part_in[(int64_t)m * a.nparts_in + lane] : 0.f;
        }
        if (a.nparts_in > 64) {
#pragma unroll
            for (int j = 0; j < RPW; ++j) {
                const int m = min(wave + NW * j, M - 1);
                for (int i = lane + 64; i < a.nparts_in; i += 64) pv[j] += a.part_in[(int64_t)m * a.nparts_in + i];
            }
        }
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int r = wave + NW * j;
            const float ss = wave_sum(pv[j]);
            if (lane == 0 && r < 16 * MT) inv[r] = rsqrtf(ss / (float)K + a.eps);
        }
    }
    // Output unit v = r * CPR + c: row r, outputs 4c..4c+3 of the workgroup's (gate) rows.  A lane's accumulator
    // acc[rt][mt] is unit (16 mt + (lane & 15), 4 (rt mod RT/2) + (lane >> 4)) of half rt / (RT/2) (swiglu; else rt).
    // Slots are padded by one per 16 (v + v/16): the lane-consecutive writes (unit stride CPR) and the
    // thread-consecutive reads (unit stride 1) both hit distinct banks.
    auto red_at = [&](int w, int p, int v) { return w * SZ + p * NP + v + (v >> 4); };
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            constexpr int HALF = MODE == kSwiglu ? RT / 2 : RT;
            const int p = rt / HALF, c = 4 * (rt % HALF) + (lane >> 4);
            red[red_at(wave, p, (16 * mt + (lane & 15)) * CPR + c)] = acc[rt][mt];
        }
    __syncthreads();

    f32x4 val[VP][PAIR];
    const bool active = tid < NOUT;  // wave-uniform (NOUT % 64 == 0)
    if (active) {
#pragma unroll
        for (int j = 0; j < VP; ++j)
#pragma unroll
            for (int p = 0; p < PAIR; ++p) {
                const int v = tid + NT * j;
                f32x4 acc4 = red[red_at(0, p, v)];
#pragma unroll
                for (int w = 1; w < NW; ++w) acc4 += red[red_at(w, p, v)];
                val[j][p] = acc4;
            }
    }

    if (S > 1) {  // split-K: slab per task in output-unit order, ticket per row group, last arriver sums in order
        // fence-free hand-off (chronos_hip.h st_wt / ld_wt): write-through slab stores, one lane's ticket after every
        // wave drained its stores, sc1 slab loads by the last arriver — an agent release + acquire pair per workgroup
        // (an L2 write-back + an L1 invalidate) cost 15-25 us on the decode shapes, more than the split saved
        constexpr int SLAB = NOUT * PAIR;  // f32x4 per task
        float* slab = a.ws + (int64_t)task * SLAB * 4;
        if (active) {
#pragma unroll
            for (int j = 0; j < VP; ++j)
#pragma unroll
                for (int p = 0; p < PAIR; ++p) st_wt(slab + ((tid + NT * j) * PAIR + p) * 4, val[j][p]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const int old = __hip_atomic_fetch_add(a.cnt + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == S - 1;
            if (last) __hip_atomic_store(a.cnt + g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = last;
        }
        __syncthreads();
        if (!*flag) return;
        if (active) {
            const float* base = a.ws + (int64_t)g * S * SLAB * 4;
            for (int o = 0; o < S; ++o) {
#pragma unroll
                for (int j = 0; j < VP; ++j)
#pragma unroll
                    for (int p = 0; p < PAIR; ++p) {
                        const f32x4 v = ld_wt(base + ((int64_t)o * SLAB + (tid + NT * j) * PAIR + p) * 4);
                        val[j][p] = o == 0 ? v : val[j][p] + v;
                    }
            }
        }
    }
    if (!active) return;

#pragma unroll
    for (int j = 0; j < VP; ++j) {
        const int v = tid + NT * j;
        const int r = v / CPR, c = v % CPR;
        const bool live = r < M;
        float sc = 1.f;
        if constexpr (NORMP) sc = inv[r];
        if constexpr (MODE == kSwiglu) {
            if (live) {
                u16x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float gv = bf2f(f2bf(val[j][0][i] * sc));
                    const float sg = bf2f(f2bf(gv / (1.f + __expf(-gv))));
                    o[i] = f2bf(sg * bf2f(f2bf(val[j][1][i] * sc)));
                }
                *reinterpret_cast<u16x4*>(a.y + (int64_t)r * a.F + g * 8 * RT + 4 * c) = o;
            }
        } else if constexpr (MODE == kResid) {
            const int64_t at = (int64_t)r * a.N + g * 16 * RT + 4 * c;
            float ss = 0.f;
            if (live) {
                const u16x4 rv = *reinterpret_cast<const u16x4*>(a.resid + at);
                u16x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float sv = bf2f(f2bf(bf2f(f2bf(val[j][0][i])) + bf2f(rv[i])));
                    o[i] = f2bf(sv);
                    ss += sv * sv;
                }
                *reinterpret_cast<u16x4*>(a.y + at) = o;
            }
            // the CPR consecutive lanes of a row hold its 16 RT outputs: butterfly in a fixed order
#pragma unroll
            for (int off = 1; off < CPR; off <<= 1) ss += __shfl_xor(ss, off, 64);
            if (c == 0 && live) a.part_out[(int64_t)r * (a.N / (16 * RT)) + g] = ss;
        } else {
            if (live) {
                u16x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = f2bf(val[j][0][i] * sc);
                *reinterpret_cast<u16x4*>(a.y + (int64_t)r * a.N + g * 16 * RT + 4 * c) = o;
            }
        }
    }
}

template <int RT, int MT, int D, int NW, int MODE, bool NORMP>
void launch_cfg(const PPArgs& a, hipStream_t st) {
    constexpr int UNITS = RT * MT * 64;
    // the reduction slots (+ inv, flag) alias the XL x tiles, which are dead once the main loop ends
    const int lds = std::max(NW * (UNITS + UNITS / 16) * 16 + 16 * MT * 4 + 16, MT >= XL_MIN_MT ? NW * MT * 2048 : 0);
    auto kern = skinny_kernel<RT, MT, D, NW, MODE, NORMP>;
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    const int G = MODE == kSwiglu ? a.F / (8 * RT) : a.N / (16 * RT);
    hipLaunchKernelGGL(kern, dim3(G * a.splitk), dim3(64 * NW), lds, st, a);
}

// configs {RT (W tiles of 16 rows per workgroup), MT (x tiles: M <= 16 MT), D (ring depth in 64-k units), NW (waves
// splitting K inside the workgroup; K % (64 NW splitk) == 0)}
#define SK_CONFIGS(X)  \
    X(0, 1, 1, 4, 16)  \
    X(1, 2, 1, 4, 8)   \
    X(2, 4, 1, 4, 4)   \
    X(3, 2, 2, 4, 8)   \
    X(4, 4, 2, 3, 4)   \
    X(5, 2, 4, 3, 4)   \
    X(6, 4, 4, 2, 4)   \
    X(7, 2, 8, 2, 4)   \
    X(8, 1, 2, 4, 16)  \
    X(9, 1, 4, 2, 16)  \
    X(10, 2, 4, 2, 8)  \
    X(11, 1, 1, 4, 8)

template <int MODE, bool NORMP>
bool launch_mode(int cfg, const PPArgs& a, hipStream_t st) {
    switch (cfg) {
#define SK_CASE(ID, RT_, MT_, D_, NW_)                                     \
    case ID:                                                               \
        if constexpr (MODE == kSwiglu && RT_ % 2) return false;            \
        else {                                                             \
            launch_cfg<RT_, MT_, D_, NW_, MODE, NORMP>(a, st);             \
            return true;                                                   \
        }
        SK_CONFIGS(SK_CASE)
#undef SK_CASE
        default: return false;
    }
}

}  // namespace

int gemm_skinny_rt(int cfg) {
    switch (cfg) {
#define SK_RT(ID, RT_, MT_, D_, NW_) case ID: return RT_;
        SK_CONFIGS(SK_RT)
#undef SK_RT
        default: return 0;
    }
}
int gemm_skinny_nw(int cfg) {
    switch (cfg) {
#define SK_NW(ID, RT_, MT_, D_, NW_) case ID: return NW_;
        SK_CONFIGS(SK_NW)
#undef SK_NW
        default: return 0;
    }
}
int gemm_skinny_mt(int cfg) {
    switch (cfg) {
#define SK_MT(ID, RT_, MT_, D_, NW_) case ID: return MT_;
        SK_CONFIGS(SK_MT)
#undef SK_MT
        default: return 0;
    }
}

bool launch_gemm_skinny(int cfg, int mode, bool normp, const PPArgs& a, hipStream_t st) {
    if (a.M == 0) return true;
    if (mode == kResid) return normp ? false : launch_mode<kResid, false>(cfg, a, st);
    if (mode == kSwiglu) return normp ? launch_mode<kSwiglu, true>(cfg, a, st) : launch_mode<kSwiglu, false>(cfg, a, st);
    return normp ? launch_mode<kPlain, true>(cfg, a, st) : launch_mode<kPlain, false>(cfg, a, st);
}

}  // namespace chronos
