// gemm_w4.hip — experiment for the large-M projection GEMM: one wave per SIMD, a 256 x 256 output
// tile per workgroup, 128 x 128 per wave (64 accumulators of 16x16x32 MFMA = 256 registers, held in AGPRs), 64-deep
// slabs in two LDS buffers filled by LDS-DMA through buffer descriptors.  Per wave and slab: 128 MFMAs, 32 ds_read_b128,
// 16 LDS-DMA pieces — the instruction mix of hipBLASLt's MT256x256x64_MI16x16x1 kernel (profiles/r4_studies.md), i.e.
// 2/3 of the fragment reads per MFMA of the 8-wave slab kernel in gemm_lg.hip.
//
// Built as a small shared library (extern "C" launcher) and timed from Python against torch.matmul (hipBLASLt) and the
// production gemm_lg configs in one process (scripts/r5/bench_w4.py).  Plain epilogue only (y = x W^T, bf16).
#include "chronos_hip.h"

#include <type_traits>

using namespace chronos;

namespace {
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void w4_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void w4_bar() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void w4_dma(const __amdgpu_buffer_rsrc_t& r, unsigned char* dst, uint32_t voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 16, voff, soff, 0, 0);
}

// the DMA piece as inline asm: hipcc cannot see it write LDS, so it never waits for earlier ds_reads before it (the
// ring buffers written and read in one k-step are disjoint by construction); M0 written in the same statement
__device__ __forceinline__ void w4_dma_asm(const __amdgpu_buffer_rsrc_t& r, uint32_t lds, uint32_t voff, int soff) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds" ::"v"(voff), "s"(r),
                 "s"(lds), "s"(soff)
                 : "memory");
}


// Tile order.  gm < 256: groups of gm M-tiles sweeping all N tiles (gemm_lg's order).  gm = g | SM << 8 | SN << 16:
// the tile grid is cut into SM x SN super-blocks (one XCD's share of consecutive logical tiles after xcd_remap), each
// walked in groups of g M-tiles x SN N-tiles — so an XCD's L2 sees a near-square block of x and W tiles (fewer
// MALL / HBM bytes than a strip of all N tiles), and the ~32 tiles it runs together share g x tiles and SN W tiles.
// Tiles past the last whole super-block row / column fall back to the plain group order.
__device__ __forceinline__ void w4_tile_map(int tile, int mt, int ntl, int gm, int& tm, int& tn) {
    const int g = gm & 0xff, SM = (gm >> 8) & 0xff, SN = gm >> 16;
    if (SM > 0 && SN > 0 && mt % SM == 0 && ntl % SN == 0 && SM % g == 0) {
        const int per = SM * SN, sup = tile / per, sub = tile - sup * per;
        const int sbm = mt / SM;  // super-blocks along M
        const int sm0 = (sup % sbm) * SM, sn0 = (sup / sbm) * SN;
        const int gper = g * SN, gi = sub / gper, r = sub - gi * gper;
        tm = sm0 + gi * g + r % g;
        tn = sn0 + r / g;
        return;
    }
    if (g > 0 && mt > g) {
        const int per = g * ntl, grp = tile / per, r = tile - grp * per;
        const int gsz = min(g, mt - grp * g);
        tm = grp * g + r % gsz;
        tn = r / gsz;
    } else {
        tm = tile % mt;
        tn = tile / mt;
    }
}

// VAR bit 1: DMA as inline asm (hipcc adds no lgkmcnt wait in front of it); bit 2: MFMA in inline asm with the
// accumulator pinned to AGPRs ("+a"); bit 4: issue order written out and pinned by sched_barrier(0) (else
// sched_group_barrier interleave, which cannot see asm MFMAs); bit 8: (pinned) DMA pieces at the head of k-step B
template <int VAR>
__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                         uint16_t* __restrict__ y, int M, int N, int K, int gm) {
    constexpr int WN = 256, XM = 256, RB = 128;  // tile rows of W / x, LDS row bytes (64-deep slab)
    constexpr int STAGE = (WN + XM) * RB;        // 64 KiB per slab
    constexpr int NT = 8, MT = 8;                // 16-row W / x blocks per wave
    constexpr int NPER = 16;                     // LDS-DMA pieces per wave per slab
    constexpr bool ASMDMA = VAR & 1, ASMMMA = VAR & 2, PIN = VAR & 4;
    constexpr int DS = VAR & 8 ? 1 : 4;          // (PIN) MFMAs per DMA piece in k-step B: 1 = at the head, 4 = spread
    constexpr int NR = NT + MT, RS = 3;          // (PIN) fragment reads per k-step, one per RS MFMAs
    // timing-only ablations (wrong results): 16 no DMA in the loop, 32 no vmcnt wait / barrier, 64 no fragment reads
    constexpr bool NODMA = VAR & 16, NOBAR = VAR & 32, NORD = VAR & 64;
    // bit 128: split each slab's DMA between k-step B (pieces [0, SPLIT_NB)) and the next k-step A (the rest)
    constexpr bool SPLIT = VAR & 128;
    constexpr int SPLIT_NB = (VAR >> 8) ? (VAR >> 8) : 10;
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wi = wave >> 1, wj = wave & 1;
    const int mt = (M + XM - 1) / XM, ntl = (N + WN - 1) / WN;
    const int tile = xcd_remap(blockIdx.x, mt * ntl);
    int tm, tn;
    w4_tile_map(tile, mt, ntl, gm, tm, tn);
    const int m0 = tm * XM, n0 = tn * WN;
    const int NS = K / 64;

    // waves 0-1 stage W rows, waves 2-3 x rows: one descriptor per wave (wave-uniform base: no waterfall loop)
    const bool isw = wave < 2;
    const uint16_t* src = isw ? w : x;
    const int rows = isw ? N : M;
    const uint64_t sb = (uint64_t)src;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)sb), hi = __builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane((int)((int64_t)rows * K * 2));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((uint64_t)hi << 32) | lo), (short)0, nbytes, 0x00020000);
    uint32_t voff[NPER];
    const int r0 = (wave & 1) * 128;  // this wave's first row within the operand's 256-row tile
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
        const int r = r0 + i * 8 + (lane >> 3);
        const int pc = lane & 7;
        const int lc = pc ^ (r & 7);
        const int grow = (isw ? n0 : m0) + r;
        voff[i] = (uint32_t)((int64_t)grow * K * 2 + lc * 16);
    }
    const int dbase = (isw ? 0 : WN * RB) + r0 * RB;  // LDS byte offset of this wave's first piece within a slab
    const int NS1 = NS - 1;
    auto issue = [&](int j) {
        unsigned char* st = smem + (j & 1) * STAGE + dbase;
        const int kb = min(j, NS1) * RB;
#pragma unroll
        for (int i = 0; i < NPER; ++i) w4_dma(rs, st + i * 1024, voff[i], kb);
    };

    int loff[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) loff[kk] = (lane & 15) * 128 + (((4 * kk + (lane >> 4)) ^ (lane & 7)) << 4);
    const int abase = wi * 128 * RB, bbase = WN * RB + wj * 128 * RB;

    f32x4 acc[NT][MT];
#pragma unroll
    for (int s = 0; s < NT; ++s)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    bf16x8 fa0[NT], fb0[MT], fa1[NT], fb1[MT];
    auto rd = [&](int j, int kk, bf16x8 (&fa)[NT], bf16x8 (&fb)[MT]) {
        const unsigned char* b = smem + (j & 1) * STAGE;
#pragma unroll
        for (int s = 0; s < NT; ++s) fa[s] = *reinterpret_cast<const bf16x8*>(b + abase + 16 * s * RB + loff[kk]);
#pragma unroll
        for (int t = 0; t < MT; ++t) fb[t] = *reinterpret_cast<const bf16x8*>(b + bbase + 16 * t * RB + loff[kk]);
    };
    auto mm = [&](bf16x8 (&fa)[NT], bf16x8 (&fb)[MT]) {
#pragma unroll
        for (int s = 0; s < NT; ++s)
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                if constexpr (ASMMMA)
                    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[s][t]) : "v"(fa[s]), "v"(fb[t]));
                else
                    acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s], fb[t], acc[s][t], 0, 0, 0);
            }
    };

    issue(0);
    if constexpr (SPLIT) {
        unsigned char* st = smem + STAGE + dbase;
#pragma unroll
        for (int i = 0; i < SPLIT_NB; ++i) w4_dma(rs, st + i * 1024, voff[i], min(1, NS1) * RB);
        w4_vmcnt<SPLIT_NB>();
    } else {
        issue(1);
        w4_vmcnt<NPER>();
    }
    w4_bar();
    rd(0, 0, fa0, fb0);
    constexpr int MF = NT * MT;  // 64 MFMAs per k-step
    if constexpr (!PIN) {
        for (int j = 0; j < NS; ++j) {
            // k-step A: MFMAs on set 0 || fragments of (j, k-step B) into set 1
            rd(j, 1, fa1, fb1);
            mm(fa0, fb0);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, MF - 48, 0);
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            w4_vmcnt<0>();  // slab j+1 landed (this wave's pieces); the barrier makes every wave's visible
            w4_bar();
            // k-step B: DMA of slab j+2 into buffer j & 1 || MFMAs on set 1 || fragments of (j+1, k-step A)
            issue(j + 2);
            rd(j + 1, 0, fa0, fb0);
            mm(fa1, fb1);
#pragma unroll
            for (int i = 0; i < NPER; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, MF - 48, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
        // issue order written out: MFMA i, then (k-step B) DMA piece i / DS when i % DS == 0, then fragment read r after
        // MFMA r * RS + RS - 1 (the last MFMAs of a k-step read nothing, so the next k-step's first fragments have
        // landed); sched_barrier(0) after each group pins it.  hipcc counts the fragment reads itself (lgkmcnt before
        // the first MFMA that consumes one); the asm DMA is counted by the explicit vmcnt before the slab barrier.
        // DMA plan per k-step: pieces [P0, P0 + NP) of slab jd, piece q at MFMA POS + q * STEP
        auto kstep = [&](auto P0_, auto NP_, auto POS_, auto STEP_, bf16x8 (&fa)[NT], bf16x8 (&fb)[MT], int jr, int kkr,
                         bf16x8 (&na)[NT], bf16x8 (&nb)[MT], int jd) {
            constexpr int P0 = decltype(P0_)::value, NP = decltype(NP_)::value;
            constexpr int POS = decltype(POS_)::value, STEP = decltype(STEP_)::value;
            const unsigned char* b = smem + (jr & 1) * STAGE;
            const uint32_t dst = (uint32_t)(uintptr_t)(smem + (jd & 1) * STAGE + dbase);
            const int kb = min(jd, NS1) * RB;
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                const int s = i / MT, t = i % MT;
                if constexpr (!NODMA && NP > 0) {
                    if (i >= POS && (i - POS) % STEP == 0 && (i - POS) / STEP < NP) {
                        const int q = P0 + (i - POS) / STEP;
                        if constexpr (ASMDMA)
                            w4_dma_asm(rs, __builtin_amdgcn_readfirstlane(dst + q * 1024), voff[q], kb);
                        else
                            w4_dma(rs, smem + (jd & 1) * STAGE + dbase + q * 1024, voff[q], kb);
                    }
                }
                if constexpr (ASMMMA)
                    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[s][t]) : "v"(fa[s]), "v"(fb[t]));
                else
                    acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s], fb[t], acc[s][t], 0, 0, 0);
                if (!NORD && i % RS == RS - 1 && i / RS < NR) {
                    // read order: fa[0], fb[0..7], fa[1..7] (the next k-step's first MFMAs need fa[0] and fb[*])
                    const int r = i / RS;
                    if (r == 0) na[0] = *reinterpret_cast<const bf16x8*>(b + abase + loff[kkr]);
                    else if (r <= MT) nb[r - 1] = *reinterpret_cast<const bf16x8*>(b + bbase + 16 * (r - 1) * RB + loff[kkr]);
                    else na[r - MT] = *reinterpret_cast<const bf16x8*>(b + abase + 16 * (r - MT) * RB + loff[kkr]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        using I = std::integral_constant<int, 0>;
        // SPLIT: slab j+2's pieces [0, NB) in k-step B of slab j (one per SB MFMAs), [NB, 16) in k-step A of slab
        // j+1 (one per SA MFMAs from its first MFMA): the address work of a slab's DMA spread over two k-steps
        constexpr int NB = SPLIT ? SPLIT_NB : NPER, SB = SPLIT ? MF / NB : DS, SA = 5;
        for (int j = 0; j < NS; ++j) {
            if constexpr (SPLIT)
                kstep(std::integral_constant<int, NB>{}, std::integral_constant<int, NPER - NB>{}, I{},
                      std::integral_constant<int, SA>{}, fa0, fb0, j, 1, fa1, fb1, j + 1);
            else
                kstep(I{}, I{}, I{}, std::integral_constant<int, 1>{}, fa0, fb0, j, 1, fa1, fb1, 0);
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) as a builtin: hipcc's own wait bookkeeping sees it
            if constexpr (!NOBAR) {
                w4_vmcnt<0>();
                w4_bar();
            }
            if constexpr (NORD) {
#pragma unroll
                for (int q = 0; q < NT; ++q) asm volatile("" : "+v"(fa1[q]), "+v"(fa0[q]));
#pragma unroll
                for (int q = 0; q < MT; ++q) asm volatile("" : "+v"(fb1[q]), "+v"(fb0[q]));
            }
            kstep(I{}, std::integral_constant<int, NB>{}, I{}, std::integral_constant<int, SB>{}, fa1, fb1, j + 1, 0,
                  fa0, fb0, j + 2);
        }
    }
    w4_vmcnt<0>();
    if constexpr (ASMMMA) {
        // the last MFMAs' results: 8-pass XDL -> any other reader needs the pipeline drained (s_nops), and every
        // accumulator is re-defined after the nops so no accvgpr read is scheduled above them
        asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
        for (int s = 0; s < NT; ++s)
#pragma unroll
            for (int t = 0; t < MT; ++t) asm volatile("" : "+a"(acc[s][t]));
    }

    // epilogue: lane holds D[n = wi*128 + 16 s + 4 (lane >> 4) + i][m = wj*128 + 16 t + (lane & 15)]
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        const int m = m0 + wj * 128 + 16 * t + (lane & 15);
        if (m >= M) continue;
#pragma unroll
        for (int s = 0; s < NT; ++s) {
            const int n = n0 + wi * 128 + 16 * s + 4 * (lane >> 4);
            u16x4 o;
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[s][t][i]);
            if (n < N) *reinterpret_cast<u16x4*>(y + (int64_t)m * N + n) = o;
        }
    }
}

template <int VAR>
int w4_launch(const void* x, const void* w, void* y, int M, int N, int K, int gm, hipStream_t st) {
    const int lds = 2 * (256 + 256) * 128;
    auto kern = gemm_w4_kernel<VAR>;
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(256), lds, st, (const uint16_t*)x, (const uint16_t*)w, (uint16_t*)y, M, N,
                       K, gm);
    return (int)hipGetLastError();
}

// ---- w4b: the pinned one-wave-per-SIMD schedule with per-operand LDS rings.  LDS = 160 KiB split into 32 KiB
// operand slabs: T3 = 0 two W + two x slabs (the w4 kernel above), 1 three W + two x, 2 two W + three x.  The operand
// with three slabs is fetched two slabs ahead (its DMA of slab j+3 issued in k-step B of slab j, waited for at the
// barrier of slab j+2), the other one slab ahead as before.  Waves 0-1 stage W rows, waves 2-3 x rows, so the
// three-slab operand's waves keep 16 more pieces in flight across each barrier (their vmcnt(16) instead of 0).
template <int T3, int DSP>
__global__ void __launch_bounds__(256, 1) gemm_w4b_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                          uint16_t* __restrict__ y, int M, int N, int K, int gm) {
    constexpr int WN = 256, XM = 256, RB = 128, SL = 256 * RB;  // 32 KiB operand slab
    constexpr int NBW = T3 == 1 ? 3 : 2, NBX = T3 == 2 ? 3 : 2;
    constexpr int XOFF = NBW * SL;  // x slabs after the W slabs
    constexpr int NT = 8, MT = 8, NPER = 16, MF = NT * MT, NR = NT + MT, RS = 3;
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wi = wave >> 1, wj = wave & 1;
    const int mt = (M + XM - 1) / XM, ntl = (N + WN - 1) / WN;
    const int tile = xcd_remap(blockIdx.x, mt * ntl);
    int tm, tn;
    w4_tile_map(tile, mt, ntl, gm, tm, tn);
    const int m0 = tm * XM, n0 = tn * WN;
    const int NS = K / 64, NS1 = NS - 1;

    const bool isw = wave < 2;
    const uint16_t* src = isw ? w : x;
    const int rows = isw ? N : M;
    const uint64_t sb = (uint64_t)src;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)sb), hi = __builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane((int)((int64_t)rows * K * 2));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((uint64_t)hi << 32) | lo), (short)0, nbytes, 0x00020000);
    uint32_t voff[NPER];
    const int r0 = (wave & 1) * 128;
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
        const int r = r0 + i * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ (r & 7);
        voff[i] = (uint32_t)((int64_t)((isw ? n0 : m0) + r) * K * 2 + lc * 16);
    }
    // this wave's operand: its slab count (3 = two slabs ahead) and LDS region
    const bool deep = (T3 == 1 && isw) || (T3 == 2 && !isw);
    const int nbuf = deep ? 3 : 2;
    const int region = (isw ? 0 : XOFF) + r0 * RB;
    auto wslab = [&](int j) { return j % NBW; };
    auto xslab = [&](int j) { return j % NBX; };
    auto dst_of = [&](int j) -> uint32_t {
        return (uint32_t)(uintptr_t)(smem + region + (j % nbuf) * SL);
    };
    auto issue_all = [&](int j) {
        const uint32_t d = dst_of(j);
        const int kb = min(j, NS1) * RB;
#pragma unroll
        for (int i = 0; i < NPER; ++i) w4_dma_asm(rs, __builtin_amdgcn_readfirstlane(d + i * 1024), voff[i], kb);
    };

    int loff[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) loff[kk] = (lane & 15) * 128 + (((4 * kk + (lane >> 4)) ^ (lane & 7)) << 4);
    const int abase = wi * 128 * RB, bbase = XOFF + wj * 128 * RB;

    f32x4 acc[NT][MT];
#pragma unroll
    for (int s = 0; s < NT; ++s)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa0[NT], fb0[MT], fa1[NT], fb1[MT];
    auto rd = [&](int j, int kk, bf16x8 (&fa)[NT], bf16x8 (&fb)[MT]) {
        const unsigned char* wb = smem + abase + wslab(j) * SL;
        const unsigned char* xb = smem + bbase + xslab(j) * SL;
#pragma unroll
        for (int s = 0; s < NT; ++s) fa[s] = *reinterpret_cast<const bf16x8*>(wb + 16 * s * RB + loff[kk]);
#pragma unroll
        for (int t = 0; t < MT; ++t) fb[t] = *reinterpret_cast<const bf16x8*>(xb + 16 * t * RB + loff[kk]);
    };

    // prologue: slabs 0 .. nbuf-2 in flight, slab 0 landed
    issue_all(0);
    issue_all(1);
    if (deep) {
        issue_all(2);
        w4_vmcnt<2 * NPER>();
    } else {
        w4_vmcnt<NPER>();
    }
    w4_bar();
    rd(0, 0, fa0, fb0);

    auto kstep = [&](auto DMA_ON, bf16x8 (&fa)[NT], bf16x8 (&fb)[MT], int jr, int kkr, bf16x8 (&na)[NT],
                     bf16x8 (&nb)[MT], int jd) {
        constexpr bool dma_on = decltype(DMA_ON)::value;
        const unsigned char* wb = smem + abase + wslab(jr) * SL;
        const unsigned char* xb = smem + bbase + xslab(jr) * SL;
        const uint32_t d = dst_of(jd);
        const int kb = min(jd, NS1) * RB;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int s = i / MT, t = i % MT;
            if constexpr (dma_on) {
                if (i % DSP == 0 && i / DSP < NPER)
                    w4_dma_asm(rs, __builtin_amdgcn_readfirstlane(d + (i / DSP) * 1024), voff[i / DSP], kb);
            }
            acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s], fb[t], acc[s][t], 0, 0, 0);
            if (i % RS == RS - 1 && i / RS < NR) {
                const int r = i / RS;
                if (r == 0) na[0] = *reinterpret_cast<const bf16x8*>(wb + loff[kkr]);
                else if (r <= MT) nb[r - 1] = *reinterpret_cast<const bf16x8*>(xb + 16 * (r - 1) * RB + loff[kkr]);
                else na[r - MT] = *reinterpret_cast<const bf16x8*>(wb + 16 * (r - MT) * RB + loff[kkr]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    for (int j = 0; j < NS; ++j) {
        kstep(std::integral_constant<bool, false>{}, fa0, fb0, j, 1, fa1, fb1, 0);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        // slab j+1 landed for this wave's operand (the deep operand keeps slab j+2 in flight)
        if (deep) w4_vmcnt<NPER>();
        else w4_vmcnt<0>();
        w4_bar();
        kstep(std::integral_constant<bool, true>{}, fa1, fb1, j + 1, 0, fa0, fb0, j + nbuf);
    }
    w4_vmcnt<0>();
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        const int m = m0 + wj * 128 + 16 * t + (lane & 15);
        if (m >= M) continue;
#pragma unroll
        for (int s = 0; s < NT; ++s) {
            const int n = n0 + wi * 128 + 16 * s + 4 * (lane >> 4);
            u16x4 o;
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[s][t][i]);
            if (n < N) *reinterpret_cast<u16x4*>(y + (int64_t)m * N + n) = o;
        }
    }
}

template <int T3, int DSP>
int w4b_launch(const void* x, const void* w, void* y, int M, int N, int K, int gm, hipStream_t st) {
    const int lds = 160 * 1024;
    auto kern = gemm_w4b_kernel<T3, DSP>;
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(256), lds, st, (const uint16_t*)x, (const uint16_t*)w, (uint16_t*)y, M, N,
                       K, gm);
    return (int)hipGetLastError();
}
}  // namespace

extern "C" int gemm_w4(const void* x, const void* w, void* y, int M, int N, int K, int var, int gm, void* stream) {
    if (K % 64 || N % 4 || M < 1) return -1;
    if ((int64_t)(N + 256) * K * 2 >= (1LL << 31) || (int64_t)(M + 256) * K * 2 >= (1LL << 31)) return -2;
    hipStream_t st = (hipStream_t)stream;
    switch (var) {
        case 0: return w4_launch<0>(x, w, y, M, N, K, gm, st);
        case 6: return w4_launch<6>(x, w, y, M, N, K, gm, st);   // asm MFMA, pinned, builtin DMA spread
        case 7: return w4_launch<7>(x, w, y, M, N, K, gm, st);   // asm MFMA, pinned, asm DMA spread
        case 14: return w4_launch<14>(x, w, y, M, N, K, gm, st); // asm MFMA, pinned, builtin DMA at the head
        case 15: return w4_launch<15>(x, w, y, M, N, K, gm, st); // asm MFMA, pinned, asm DMA at the head
        case 4: return w4_launch<4>(x, w, y, M, N, K, gm, st);   // builtin MFMA, pinned, builtin DMA spread
        case 5: return w4_launch<5>(x, w, y, M, N, K, gm, st);   // builtin MFMA, pinned, asm DMA spread
        case 12: return w4_launch<12>(x, w, y, M, N, K, gm, st); // builtin MFMA, pinned, builtin DMA at the head
        case 13: return w4_launch<13>(x, w, y, M, N, K, gm, st); // builtin MFMA, pinned, asm DMA at the head
        case 133: return w4_launch<133>(x, w, y, M, N, K, gm, st); // 5 + split DMA, 10 in k-step B, 6 in k-step A
        case 128 + 5 + (8 << 8): return w4_launch<128 + 5 + (8 << 8)>(x, w, y, M, N, K, gm, st);  // split 8 / 8
        case 128 + 5 + (12 << 8): return w4_launch<128 + 5 + (12 << 8)>(x, w, y, M, N, K, gm, st);  // split 12 / 4
        case 128 + 5 + (6 << 8): return w4_launch<128 + 5 + (6 << 8)>(x, w, y, M, N, K, gm, st);  // split 6 / 10
        case 21: return w4_launch<21>(x, w, y, M, N, K, gm, st); // ablation: 5 without loop DMA
        case 37: return w4_launch<37>(x, w, y, M, N, K, gm, st); // ablation: 5 without vmcnt / barrier
        case 69: return w4_launch<69>(x, w, y, M, N, K, gm, st); // ablation: 5 without fragment reads
        case 85: return w4_launch<85>(x, w, y, M, N, K, gm, st); // ablation: MFMA + barrier only
        case 117: return w4_launch<117>(x, w, y, M, N, K, gm, st); // ablation: MFMA only
        case 1000: return w4b_launch<0, 4>(x, w, y, M, N, K, gm, st);  // w4b 2+2 slabs, DMA one per 4 MFMAs
        case 1001: return w4b_launch<1, 4>(x, w, y, M, N, K, gm, st);  // w4b 3 W + 2 x slabs
        case 1002: return w4b_launch<2, 4>(x, w, y, M, N, K, gm, st);  // w4b 2 W + 3 x slabs
        case 1011: return w4b_launch<1, 1>(x, w, y, M, N, K, gm, st);  // 3 W slabs, DMA at the head
        case 1012: return w4b_launch<2, 1>(x, w, y, M, N, K, gm, st);  // 3 x slabs, DMA at the head
        default: return -3;
    }
}
