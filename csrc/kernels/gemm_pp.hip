// gemm_pp.hip — the batched projection GEMM family (SURVEY.md §2.3 K3 / K7 / K8+K9 / K10 / K11 at M >= 3):
// y[M, N] = x[M, K] · W[N, K]^T, bf16 in, fp32 accumulate, with the epilogues of the Llama decoder fused in.
//
// Structure: "ping-pong" — one 512-thread workgroup (8 waves = 2 per SIMD) per output tile, the two wave GROUPS
// (waves 0-3, waves 4-7; waves w and w+4 share a SIMD) run the same program offset by one barrier, so on every SIMD
// one wave issues a pure MFMA block while its partner reads the next fragments from LDS and issues the next LDS-DMA
// loads.  Every interval between two workgroup barriers is {group A: 32 MFMAs | group B: LDS reads + DMA issue}:
//
//   * tile BM (x rows) x BN (W rows); an LDS stage holds BK = 64 (two 32-deep intervals, 128-B rows) or, HALF, BK = 32
//     (one interval, 64-B rows — twice the ring depth in the same LDS, so more bytes in flight per CU);
//     group g owns x rows [g*BM/2, (g+1)*BM/2), wave j of a group owns BN/4 W rows (SwiGLU: BN/8 gate rows and the
//     matching BN/8 up rows, so gate and up of one output sit in the same lane);
//   * v_mfma_f32_16x16x32_bf16, swapped product D = W · x^T: a lane's accumulator holds 4 CONSECUTIVE output columns
//     of one output row, so row-wise epilogues (residual, RMSNorm partial sums, norm scale, SwiGLU pairs) need no
//     cross-lane shuffles beyond the 4 lanes that share a row;
//   * operands reach LDS only by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction, no staging VGPRs) into
//     a STAGES-deep ring; the chunk XOR swizzle (128-B rows: chunk ^ row&7; 64-B rows: chunk ^ G[(row>>2)&3] with
//     G = {0,3,2,1}) is applied on the per-lane global SOURCE address and undone on the ds_read_b128 fragment read;
//     both are bank-conflict-free for the 16x16x32 operand maps (cdna_hip_programming.md §5.4 rule 21, T2);
//   * the DMA of stage j+STAGES-1 is issued at the start of each group's load interval of stage j, into the buffer both
//     groups finished reading one interval earlier; each wave retires its own DMAs with a COUNTED s_waitcnt vmcnt as
//     late as the barrier before the stage's first reader allows (group 0 after its MFMA block, group 1 after its
//     reads), and only raw s_barrier is used (never __syncthreads, which would drain the ring);
//   * split-K (decode shapes whose tile grid under-fills 256 CUs): each K slice writes an fp32 slab in register
//     order — write-through (sc1) stores and no fences for slabs up to 64 KiB (chronos_hip.h st_wt / ld_wt), plain
//     stores + an agent release / acquire pair for bigger ones — takes an agent-scope ticket (
//     cdna_hip_programming.md §5 "In-launch split-K reduction"), and the last arriver of a tile sums the slabs and
//     runs the epilogue;
//   * XCD-aware task order: a tile's split-K slices and the x-row tiles of one W panel are consecutive task ids,
//     which the bijective remap keeps on one XCD (shared L2); correctness never depends on placement.
//
// Epilogues (MODE): kPlain y = acc; kSwiglu y[:, f] = silu(acc_gate) * acc_up (w = [gate; up], [2F, K]); kResid
// s = bf16(bf16(acc) + resid) and the per-row sums of s^2 over each wave's BN/4 columns (the next RMSNorm's partials,
// the same contract as gemv.hip's kResid producer).  NORMP (QKV / gate_up / LM head consumers of a kResid producer):
// x is the raw residual stream and the folded RMSNorm is one per-row scale inv = rsqrt(sum(partials)/K + eps).
#include "chronos_hip.h"
#include "chronos_gemm.h"

namespace chronos {
namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

enum : int { kPlain = kPPPlain, kSwiglu = kPPSwiglu, kResid = kPPResid };

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

// workgroup barrier that nothing is scheduled across (MFMAs are register-only, so "memory" alone would not pin them)
__device__ __forceinline__ void pp_bar() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// 64-B-row chunk swizzle: conflict-free 16x16x32 fragment reads (rows of a 16-row tile x 4 chunks per ds_read_b128
// lane group land on 16 distinct 16-B slots)
__device__ __forceinline__ int swz64(int row) { return (4 - ((row >> 2) & 3)) & 3; }

// SPLIT (HALF only): separate rings — group 0 DMAs only W into a DW-deep ring, group 1 only x into a DX-deep one.
// s_waitcnt vmcnt retires a wave's loads in issue order, so with one shared ring the far-ahead prefetch of the cold
// weight stream would have to complete as early as the near-ahead x tile; with one operand per wave group each
// group's counted wait covers only its own operand and the W ring can run DW-1 chunks ahead.
template <int BM, int BN, int STAGES, bool HALF, int MODE, bool NORMP, bool PRIO, int DW = STAGES, int DX = STAGES,
          bool SPLIT = false>
__global__ void __launch_bounds__(512, 2) gemm_pp_kernel(PPArgs a) {
    constexpr int RB = HALF ? 64 : 128;                        // LDS row bytes (k per stage * 2)
    constexpr int RPI = 1024 / RB;                             // image rows per LDS-DMA instruction
    constexpr int WIMG = BN * RB, XIMG = BM * RB, STAGE = WIMG + XIMG;
    // LDS-DMA instructions per wave per stage: all 8 waves share both operands, or (SPLIT) 4 waves per operand
    constexpr int WI = SPLIT ? BN / RPI / 4 : BN / RPI / 8, XI = SPLIT ? BM / RPI / 4 : BM / RPI / 8;
    constexpr int NPER = WI + XI;
    constexpr int NT = BN / 64;                                // 16-row W tiles per wave
    constexpr int MT = BM / 32;                                // 16-row x tiles per wave
    constexpr int EXTRA = SPLIT ? DW * WIMG + DX * XIMG : STAGES * STAGE;  // flag + inv[BM] after the ring(s)
    static_assert(!SPLIT || (HALF && DW >= 2 && DX >= 2), "split rings: 32-deep stages, >= 2 buffers each");
    static_assert(WI >= 1 && XI >= 1, "tile too small for 8 loader waves");
    static_assert(MODE != kSwiglu || (BN / 8) % 16 == 0, "swiglu: BN/8 gate rows per wave, multiple of 16");
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = __builtin_amdgcn_readfirstlane(wave >> 2), wj = wave & 3;
    const int M = a.M, K = a.K;
    const int mt = (M + BM - 1) / BM;
    const int ntl = MODE == kSwiglu ? a.F / (BN / 2) : (a.N + BN - 1) / BN;
    const int S = a.splitk;
    const int task = xcd_remap(blockIdx.x, mt * ntl * S);
    const int ks = task % S, tile = task / S;
    // tile order: with gm > 0 the M-tiles come in groups of gm, every W panel of a group before the next group, so
    // the 32 tiles an XCD runs at once form a gm x (32 / gm) block that shares x rows AND W rows in its L2 (at large
    // M the default order puts 32 different x tiles and one W panel there: every x byte then comes from beyond L2)
    int tm, tn;
    if (a.gm > 0 && mt > a.gm) {
        const int per = a.gm * ntl, grp = tile / per, r = tile - grp * per;
        const int gsz = min(a.gm, mt - grp * a.gm);
        tm = grp * a.gm + r % gsz;
        tn = r / gsz;
    } else {
        tm = tile % mt;
        tn = tile / mt;
    }
    const int m0 = tm * BM;
    const int NS = HALF ? 2 * a.kts : a.kts;  // stages of this task's K range
    const int64_t kbeg = (int64_t)ks * a.kts * 64;

    // ---- LDS-DMA sources: image row r of the tile; lane l fills row r0 + l / (RB/16), physical chunk l % (RB/16),
    // from the logical chunk that the read-side swizzle maps there
    auto src_chunk = [&](int r) {
        if constexpr (HALF) return (lane & 3) ^ swz64(r);
        else return (lane & 7) ^ (r & 7);
    };
    const uint16_t* wsrc[WI];
    const uint16_t* xsrc[XI];
    const int wslot = SPLIT ? wj : wave;  // this wave's share of the DMA instructions of a stage
#pragma unroll
    for (int i = 0; i < WI; ++i) {
        const int r = (wslot * WI + i) * RPI + lane / (RB / 16);
        int wrow;
        const int tnw = (a.ablate & 16) ? 0 : tn;  // diagnostics: every W tile aliased onto tile 0 (L2-resident)
        if constexpr (MODE == kSwiglu)
            wrow = r < BN / 2 ? tnw * (BN / 2) + r : a.F + tnw * (BN / 2) + (r - BN / 2);
        else
            wrow = min(tnw * BN + r, a.N - 1);  // a partial last W tile re-reads row N-1 (never stored)
        wsrc[i] = a.w + (int64_t)wrow * K + kbeg + src_chunk(r) * 8;
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {
        const int r = (wslot * XI + i) * RPI + lane / (RB / 16);
        const int xr = (a.ablate & 32) ? r % M : min(m0 + r, M - 1);  // diagnostics: x tiles aliased onto tile 0
        xsrc[i] = a.x + (int64_t)xr * K + kbeg + src_chunk(r) * 8;
    }
    const bool wnt = a.ablate & 8;
    // LDS images of stage (or, SPLIT, chunk) j
    auto wbuf = [&](int j) -> unsigned char* {
        if constexpr (SPLIT) return smem + (j % DW) * WIMG;
        else return smem + (j % STAGES) * STAGE;
    };
    auto xbuf = [&](int j) -> unsigned char* {
        if constexpr (SPLIT) return smem + DW * WIMG + (j % DX) * XIMG;
        else return smem + (j % STAGES) * STAGE + WIMG;
    };
    auto issue_w = [&](int j) {
        unsigned char* st = wbuf(j);
        const int koff = j * (RB / 2);
        if (wnt) {  // non-temporal policy on the streamed weights (knob pp_wnt)
#pragma unroll
            for (int i = 0; i < WI; ++i)
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(wsrc[i] + koff),
                                                 (lds_ptr_t)(st + (wslot * WI + i) * 1024), 16, 0, 2);
        } else {
#pragma unroll
            for (int i = 0; i < WI; ++i)
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(wsrc[i] + koff),
                                                 (lds_ptr_t)(st + (wslot * WI + i) * 1024), 16, 0, 0);
        }
    };
    auto issue_x = [&](int j) {
        unsigned char* st = xbuf(j);
        const int koff = j * (RB / 2);
#pragma unroll
        for (int i = 0; i < XI; ++i)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(xsrc[i] + koff), (lds_ptr_t)(st + (wslot * XI + i) * 1024),
                                             16, 0, 0);
    };
    auto issue = [&](int j) {
        issue_w(j);
        issue_x(j);
    };

    // ---- fragment addressing: W rows (MFMA A) and x rows (MFMA B); the swizzle term is lane-constant
    int wrow0[NT];
#pragma unroll
    for (int s = 0; s < NT; ++s) {
        if constexpr (MODE == kSwiglu)
            wrow0[s] = s < NT / 2 ? wj * (BN / 8) + 16 * s : BN / 2 + wj * (BN / 8) + 16 * (s - NT / 2);
        else
            wrow0[s] = wj * (BN / 4) + 16 * s;
    }
    const int xrow0 = g * (BM / 2);
    int loff0, loff1;
    if constexpr (HALF) {
        loff0 = loff1 = (lane & 15) * 64 + (((lane >> 4) ^ swz64(lane & 15)) << 4);
    } else {
        loff0 = (lane & 15) * 128 + (((lane >> 4) ^ (lane & 7)) << 4);
        loff1 = (lane & 15) * 128 + (((4 + (lane >> 4)) ^ (lane & 7)) << 4);
    }

    f32x4 acc[NT][MT];
#pragma unroll
    for (int s = 0; s < NT; ++s)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // NORMP: the producer's partials of this wave's x rows, ALL loads issued before the DMA prologue (they are the
    // oldest entries of the in-order vmcnt queue, so the reduction below waits for them alone, and one HBM latency
    // covers every row — a row-by-row load -> wave_sum loop cost BM/8 serial latencies, 50 us per gate_up tile)
    constexpr int RPW = BM / 8;  // x rows per wave
    float pv[NORMP ? RPW : 1];
    if constexpr (NORMP) {
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int m = min(m0 + wave + 8 * j, M - 1);
            pv[j] = lane < a.nparts_in ? a.part_in[(int64_t)m * a.nparts_in + lane] : 0.f;
        }
    }

    // ---- prologue: stages 0 .. STAGES-2 in flight (SPLIT: W chunks 0 .. DW-2 by group 0, x 0 .. DX-2 by group 1)
    if constexpr (SPLIT) {
        if (g == 0) {
#pragma unroll
            for (int p = 0; p < DW - 1; ++p)
                if (p < NS) issue_w(p);
        } else {
#pragma unroll
            for (int p = 0; p < DX - 1; ++p)
                if (p < NS) issue_x(p);
        }
    } else {
#pragma unroll
        for (int p = 0; p < STAGES - 1; ++p)
            if (p < NS) issue(p);
    }

    if constexpr (NORMP) {
        // inv[r] of the tile's x rows, while the first stages are in flight (producers with > 64 partials per row
        // add the rest here, rare: only the M = 1 GEMV producer has more)
        float* inv = reinterpret_cast<float*>(smem + EXTRA + 16);
        if (a.nparts_in > 64) {
#pragma unroll
            for (int j = 0; j < RPW; ++j) {
                const int m = min(m0 + wave + 8 * j, M - 1);
                for (int i = lane + 64; i < a.nparts_in; i += 64) pv[j] += a.part_in[(int64_t)m * a.nparts_in + i];
            }
        }
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const float ss = wave_sum(pv[j]);
            if (lane == 0) inv[wave + 8 * j] = rsqrtf(ss / (float)K + a.eps);
        }
    }
    if constexpr (SPLIT) {
        if (g == 0) {
            if (NS > DW - 2) wait_vmcnt<WI * (DW - 2)>();
            else wait_vmcnt<0>();
        } else {
            if (NS > DX - 2) wait_vmcnt<XI * (DX - 2)>();
            else wait_vmcnt<0>();
        }
    } else {
        if (NS > STAGES - 2) wait_vmcnt<NPER * (STAGES - 2)>();
        else wait_vmcnt<0>();
    }
    pp_bar();
    if (g == 1) pp_bar();  // the stagger: group 1 runs one interval behind group 0

    bf16x8 fa[NT], fb[MT];
#pragma unroll
    for (int s = 0; s < NT; ++s) fa[s] = bf16x8{};
#pragma unroll
    for (int t = 0; t < MT; ++t) fb[t] = bf16x8{};
    const int abl = a.ablate;
    auto load_frags = [&](int j, int loff) {
        if (abl & 2) return;
        const unsigned char* wb = wbuf(j);
        const unsigned char* xb = xbuf(j);
#pragma unroll
        for (int s = 0; s < NT; ++s) fa[s] = *reinterpret_cast<const bf16x8*>(wb + wrow0[s] * RB + loff);
#pragma unroll
        for (int t = 0; t < MT; ++t) fb[t] = *reinterpret_cast<const bf16x8*>(xb + (xrow0 + 16 * t) * RB + loff);
    };
    auto mfma_block = [&]() {
        if (abl & 4) return;
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < NT; ++s)
#pragma unroll
            for (int t = 0; t < MT; ++t)
                acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s], fb[t], acc[s][t], 0, 0, 0);
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    };
    // this wave's DMAs of stage j+1 have landed (the younger stages stay in flight across the barrier)
    auto retire_next = [&](int nx) {
        if (nx < NS) wait_vmcnt<NPER * (STAGES - 2)>();
        else wait_vmcnt<0>();
    };

    if constexpr (SPLIT) {
        // group 0: W chunk j+DW-1 in, W chunk j+1 retired after its MFMA block; group 1: x chunk j+DX-1 in, x chunk
        // j+1 retired after its reads — both before the barrier that ends interval 2j+1
        for (int j = 0; j < NS; ++j) {
            if (g == 0) {
                if (j + DW - 1 < NS && !(abl & 1)) issue_w(j + DW - 1);
            } else {
                if (j + DX - 1 < NS && !(abl & 1)) issue_x(j + DX - 1);
            }
            load_frags(j, loff0);
            if (g == 1) {
                if (j + DX - 1 < NS) wait_vmcnt<XI * (DX - 2)>();
                else wait_vmcnt<0>();
            }
            pp_bar();
            mfma_block();
            if (g == 0) {
                if (j + DW - 1 < NS) wait_vmcnt<WI * (DW - 2)>();
                else wait_vmcnt<0>();
            }
            pp_bar();
        }
    } else if constexpr (HALF) {
        // one stage per L/C interval pair; stage j+1 must land before the barrier that ends interval 2j+1
        for (int j = 0; j < NS; ++j) {
            const int nx = j + STAGES - 1;
            if (nx < NS && !(abl & 1)) issue(nx);
            load_frags(j, loff0);
            if (g == 1) retire_next(nx);
            pp_bar();
            mfma_block();
            if (g == 0) retire_next(nx);
            pp_bar();
        }
    } else {
        for (int t = 0; t < NS; ++t) {
            const int nx = t + STAGES - 1;
            if (nx < NS && !(abl & 1)) issue(nx);
            load_frags(t, loff0);  // L0
            pp_bar();
            mfma_block();  // C0
            pp_bar();
            load_frags(t, loff1);  // L1
            if (g == 1) retire_next(nx);
            pp_bar();
            mfma_block();  // C1
            if (g == 0) retire_next(nx);
            pp_bar();
        }
    }
    if (g == 0) pp_bar();

    // ---- split-K: slab, ticket, last arriver sums.  Slabs up to 64 KiB per task (128 x 128 tiles) go write-through
    // with no fences (2-5 us per split); bigger ones through plain stores + one release / acquire pair, which
    // measured cheaper for 256 KiB slabs (down at M = 1024: 132 against 189 us; profiles/r3_gemm_table_*)
    constexpr bool WT = BM * BN <= 128 * 128;
    if (S > 1) {
        float* slab = a.ws + (int64_t)task * (BM * BN);
#pragma unroll
        for (int s = 0; s < NT; ++s)
#pragma unroll
            for (int t = 0; t < MT; ++t)
            {
                float* p = slab + (((wave * NT + s) * MT + t) * 64 + lane) * 4;
                if constexpr (WT) st_wt(p, acc[s][t]);  // write-through: no fences
                else *reinterpret_cast<f32x4*>(p) = acc[s][t];
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* flag = reinterpret_cast<int*>(smem + EXTRA);
        if (tid == 0) {
            if constexpr (!WT) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const int old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == S - 1;
            if (last) {
                if constexpr (!WT) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            *flag = last;
        }
        __syncthreads();
        if (!*flag) return;
        // every slab in slice order, this block's own included: the sum must not depend on which slice arrived last
        // (bitwise-reproducible outputs, so a captured graph replays exactly what the eager step computed)
        for (int o = 0; o < S; ++o) {
            const float* sl = a.ws + (int64_t)(tile * S + o) * (BM * BN);
#pragma unroll
            for (int s = 0; s < NT; ++s)
#pragma unroll
                for (int t = 0; t < MT; ++t) {
                    const float* p = sl + (((wave * NT + s) * MT + t) * 64 + lane) * 4;
                    const f32x4 v = WT ? ld_wt(p) : *reinterpret_cast<const f32x4*>(p);
                    acc[s][t] = o == 0 ? v : acc[s][t] + v;
                }
        }
    }

    // ---- epilogue: lane holds D[n = wrow0[s] + 4*(lane>>4) + i][m = xrow0 + 16*t + (lane&15)]
    const float* inv = reinterpret_cast<const float*>(smem + EXTRA + 16);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        const int r = xrow0 + 16 * t + (lane & 15);
        const int m = m0 + r;
        float sc = 1.f;
        if constexpr (NORMP) sc = inv[r];
        if constexpr (MODE == kSwiglu) {
            if (m < M) {
#pragma unroll
                for (int s = 0; s < NT / 2; ++s) {
                    u16x4 o;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float gv = bf2f(f2bf(acc[s][t][i] * sc));
                        const float sg = bf2f(f2bf(gv / (1.f + __expf(-gv))));
                        o[i] = f2bf(sg * bf2f(f2bf(acc[s + NT / 2][t][i] * sc)));
                    }
                    const int f = tn * (BN / 2) + wrow0[s] + 4 * (lane >> 4);
                    *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.F + f) = o;
                }
            }
        } else if constexpr (MODE == kResid) {
            float ss = 0.f;
            if (m < M) {
#pragma unroll
                for (int s = 0; s < NT; ++s) {
                    const int n = tn * BN + wrow0[s] + 4 * (lane >> 4);
                    const u16x4 rv = *reinterpret_cast<const u16x4*>(a.resid + (int64_t)m * a.N + n);
                    u16x4 o;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float v = bf2f(f2bf(bf2f(f2bf(acc[s][t][i])) + bf2f(rv[i])));
                        o[i] = f2bf(v);
                        ss += v * v;
                    }
                    *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.N + n) = o;
                }
            }
            // the 4 lanes of a row (lane ^ 16, ^ 32) hold disjoint columns of the wave's BN/4
            ss += __shfl_xor(ss, 16, 64);
            ss += __shfl_xor(ss, 32, 64);
            if (lane < 16 && m < M) a.part_out[(int64_t)m * (a.N / (BN / 4)) + tn * 4 + wj] = ss;
        } else {
            if (m < M) {
#pragma unroll
                for (int s = 0; s < NT; ++s) {
                    u16x4 o;
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[s][t][i] * sc);
                    const int n = tn * BN + wrow0[s] + 4 * (lane >> 4);
                    if (n < a.N) *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.N + n) = o;  // N % 4 == 0
                }
            }
        }
    }
}

template <int BM, int BN, int STAGES, bool HALF, int MODE, bool NORMP, bool PRIO, int DW, int DX, bool SPLIT>
void launch_cfg(const PPArgs& a, hipStream_t st) {
    constexpr int RB = HALF ? 64 : 128;
    const int lds = (SPLIT ? DW * BN * RB + DX * BM * RB : STAGES * (BM + BN) * RB) + 16 + BM * 4;
    auto kern = gemm_pp_kernel<BM, BN, STAGES, HALF, MODE, NORMP, PRIO, DW, DX, SPLIT>;
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    const int mt = (a.M + BM - 1) / BM;
    const int ntl = MODE == kSwiglu ? a.F / (BN / 2) : (a.N + BN - 1) / BN;
    hipLaunchKernelGGL(kern, dim3(mt * ntl * a.splitk), dim3(512), lds, st, a);
}

// tile configs: {BM, BN, STAGES, HALF, DW, DX, SPLIT}
#define PP_CONFIGS(X)                            \
    X(0, 256, 256, 2, false, 2, 2, false)        \
    X(1, 128, 256, 3, false, 3, 3, false)        \
    X(2, 256, 128, 3, false, 3, 3, false)        \
    X(3, 128, 128, 4, false, 4, 4, false)        \
    X(4, 256, 256, 4, true, 4, 4, false)         \
    X(5, 128, 256, 6, true, 6, 6, false)         \
    X(6, 256, 128, 6, true, 6, 6, false)         \
    X(7, 128, 128, 8, true, 8, 8, false)         \
    X(8, 256, 256, 6, true, 6, 3, true)          \
    X(9, 128, 256, 6, true, 6, 4, true)          \
    X(10, 256, 128, 8, true, 8, 4, true)         \
    X(11, 128, 128, 10, true, 10, 6, true)

template <int MODE, bool NORMP, bool PRIO>
bool launch_mode(int cfg, const PPArgs& a, hipStream_t st) {
    switch (cfg) {
#define PP_CASE(ID, BM_, BN_, ST_, H_, DW_, DX_, SP_) \
    case ID: launch_cfg<BM_, BN_, ST_, H_, MODE, NORMP, PRIO, DW_, DX_, SP_>(a, st); return true;
        PP_CONFIGS(PP_CASE)
#undef PP_CASE
        default: return false;
    }
}

}  // namespace

int gemm_pp_bm(int cfg) {
    switch (cfg) {
#define PP_BM(ID, BM_, BN_, ST_, H_, DW_, DX_, SP_) case ID: return BM_;
        PP_CONFIGS(PP_BM)
#undef PP_BM
        default: return 0;
    }
}
int gemm_pp_bn(int cfg) {
    switch (cfg) {
#define PP_BN(ID, BM_, BN_, ST_, H_, DW_, DX_, SP_) case ID: return BN_;
        PP_CONFIGS(PP_BN)
#undef PP_BN
        default: return 0;
    }
}

bool launch_gemm_pp(int cfg, int mode, bool normp, bool prio, const PPArgs& a, hipStream_t st) {
    if (a.M == 0) return true;
    if (mode == kResid) {
        if (normp || prio) return false;
        return launch_mode<kResid, false, false>(cfg, a, st);
    }
    if (prio) return mode == kPlain && !normp ? launch_mode<kPlain, false, true>(cfg, a, st) : false;
    if (mode == kSwiglu) return normp ? launch_mode<kSwiglu, true, false>(cfg, a, st) : launch_mode<kSwiglu, false, false>(cfg, a, st);
    return normp ? launch_mode<kPlain, true, false>(cfg, a, st) : launch_mode<kPlain, false, false>(cfg, a, st);
}

}  // namespace chronos
