// gemm_lg.hip — the software-pipelined projection GEMM family (SURVEY.md §2.3 K3 / K7 / K8+K9 / K10 / K11):
// y[M, N] = x[M, K] · W[N, K]^T, bf16 (or W8A8 e4m3fn) in, fp32 accumulate, the Llama decoder's epilogues fused in
// (same PPArgs and epilogue contract as gemm_pp.hip).  One kernel template, three tile regimes routed per shape by
// ops/gemm_plan.json: 256-row tiles for M >= 512 (the 1024-row decode step), 64-W-row tiles with 64-256-row x panels
// for M = 48-512, 32-row x tiles for M <= 48; and fp8 configs of the ring schedule for W8A8.
//
//   * workgroup = 2 x NWX waves (NWX = 2: one wave per SIMD, 4: two); wave (wi, wj) owns W rows [wi*WN/2, +WN/2) and
//     x rows [wj*XM/NWX, +XM/NWX) of the WN x XM output tile (the production 256 x 256 tile: 8 waves, 128 x 64 each);
//   * swapped product D = W · x^T: a lane's accumulator holds 4 CONSECUTIVE output columns of one output row, so the
//     row epilogues (residual, RMSNorm partials, folded-norm scale, SwiGLU pairs, fp8 scales) need no cross-lane
//     traffic beyond the 4 lanes of a row;
//   * operands reach LDS only through LDS-DMA (buffer_load_dwordx4 ... lds through one buffer descriptor per operand:
//     32-bit per-lane offsets, rows past the end read as zeros by the range check); the 16-B chunk swizzle is applied on
//     the per-lane SOURCE address and undone on the ds_read_b128 fragment read (cdna_hip_programming.md §5.4 rule 21,
//     T2), conflict-free for the 16x16x32 maps;
//   * ring schedule (ST >= 3), stage t with its fragments already in registers (set t & 1):
//         part 1: DMA issue of stage t+ST-1 (into the buffer every wave finished reading before the previous
//                 barrier)  ||  the first half of the stage's MFMAs
//         s_waitcnt vmcnt(n): this wave's DMA of stage t+1 has landed, stages t+2 .. t+ST-1 stay in flight
//         s_barrier          : every wave's DMA of stage t+1 has landed -> visible to every wave
//         part 2: ds_read of stage t+1's fragments into the other register set  ||  the second half of the MFMAs
//     slab schedule (ST == 2, 64-deep slabs in two buffers): fragments pipelined per 32-deep k-step, one barrier per
//     slab (below).  The only sync point is a raw s_barrier (never __syncthreads, whose vmcnt(0) would drain the ring);
//     the interleave inside each part is fixed with __builtin_amdgcn_sched_group_barrier (T19);
//   * split-K (shapes whose tile grid under-fills 256 CUs): fp32 slabs, an agent release / acquire ticket, the last
//     arriver sums the slabs in slice order and runs the epilogue (cdna_hip_programming.md §5 "In-launch split-K");
//   * XCD-aware task order (xcd_remap + M-tile grouping as in gemm_pp.hip): the tiles an XCD runs together share x
//     rows and W rows in its L2.  Correctness never depends on placement.
//
// What bounds the large-M configs against hipBLASLt (ablations, PMC, microbenchmarks): profiles/r4_studies.md.
#include "chronos_hip.h"
#include "chronos_gemm.h"

#include <type_traits>
#include <utility>

namespace chronos {
namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

enum : int { kPlain = kPPPlain, kSwiglu = kPPSwiglu, kResid = kPPResid };

template <int N>
__device__ __forceinline__ void lg_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

// raw workgroup barrier nothing is scheduled across
__device__ __forceinline__ void lg_bar() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// compile-time interleave of one MFMA block (T19: sched_group_barrier masks MFMA 0x008, VMEM 0x010, DS read 0x100):
// the NV DMA pieces one per MFMA at the head, then the NR ds_reads spread over the remaining MFMAs.  Every DMA goes
// before every ds_read of the block: an LDS-DMA issued after a ds_read makes hipcc wait for that read (lgkmcnt) first,
// since it cannot tell the two touch different buffers
// The last quarter of the block issues no read, so the next block's first MFMAs find their fragments landed.
template <int I, int MF, int NV, int NR>
__device__ __forceinline__ void lg_sched() {
    if constexpr (I < MF) {
        constexpr int R0 = NV < MF ? NV : MF;                   // first MFMA after the DMA head
        constexpr int R1 = MF - MF / 4 > R0 ? MF - MF / 4 : MF;  // reads spread over MFMAs [R0, R1)
        constexpr int r = (I < R0 || I >= R1) ? 0 : ((I - R0 + 1) * NR / (R1 - R0) - (I - R0) * NR / (R1 - R0));
        if constexpr (I < NV) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if constexpr (r > 0) __builtin_amdgcn_sched_group_barrier(0x100, r, 0);
        lg_sched<I + 1, MF, NV, NR>();
    }
}

// One 1 KiB LDS-DMA piece through a buffer descriptor (base / size wave-uniform: kernel arguments): lane l's 16 bytes
// from byte voff + soff of the buffer to LDS dst + 16 l; bytes past `bytes` read as zeros.  (A descriptor held in
// a kernel-body variable made hipcc's host pass drop the kernel stubs; built here it is hoisted all the same.)
__device__ __forceinline__ void lg_dma16(const void* base, int bytes, unsigned char* dst, uint32_t voff, int soff) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes,
                                                                       0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 16, voff, soff, 0, 0);
}

// The same piece as inline asm (VAR 2): M0 = the LDS destination, written in the same statement that reads it
// (cdna_hip_programming.md §5.7).  No VGPR destination; completion is counted by the kernel's own vmcnt waits.
typedef int lg_i32x4 __attribute__((ext_vector_type(4)));
template <bool NOP = true>
__device__ __forceinline__ void lg_dma16_asm(const void* base, int bytes, uint32_t lds, uint32_t voff, int soff) {
    const uint64_t b = (uint64_t)base;
    const lg_i32x4 r = {(int)(uint32_t)b, (int)(uint32_t)(b >> 32), bytes, 0x00020000};
    if constexpr (NOP)
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                     ::"v"(voff), "s"(r), "s"(lds), "s"(soff) : "memory");
    else  // (hipBLASLt's gfx950 code issues the LDS-DMA right after its M0 write)
        asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                     ::"v"(voff), "s"(r), "s"(lds), "s"(soff) : "memory");
}

// HB: image row of W fragment block s relative to block 0 (SwiGLU: gate blocks 0 .. 3, then the up blocks at WN / 2)
constexpr int hb_wrow(int s, bool swiglu, int WN) { return swiglu ? (s < 4 ? 16 * s : WN / 2 + 16 * (s - 4)) : 16 * s; }
// ... of 32-row block S (F8HB)
constexpr int hb_wrow32(int S, bool swiglu, int WN) { return swiglu ? (S < 2 ? 32 * S : WN / 2 + 32 * (S - 2)) : 32 * S; }
// HB bit 7 (HBV & 128): k-step 0 of a slab in growing-square order — MFMA (s, t) as soon as fa[s] and fb[t] can
// have landed — with the set-0 reads alternating fa[0], fb[0], fb[1], fa[1], fb[2], fa[2], ...: the slab head's first
// k MFMAs need ~2 sqrt(k) of the 16 reads issued at the end of the previous slab instead of k + 1, so fewer of them
// wait on the tail of that read burst
constexpr int hb_isqrt(int v) {
    int n = 0;
    while ((n + 1) * (n + 1) <= v) ++n;
    return n;
}
constexpr int hb_sq_s(int ii) { return ii - hb_isqrt(ii) * hb_isqrt(ii) < hb_isqrt(ii) ? ii - hb_isqrt(ii) * hb_isqrt(ii) : hb_isqrt(ii); }
constexpr int hb_sq_t(int ii) {
    return ii - hb_isqrt(ii) * hb_isqrt(ii) < hb_isqrt(ii) ? hb_isqrt(ii) : ii - hb_isqrt(ii) * hb_isqrt(ii) - hb_isqrt(ii);
}
// set-0 read r of the alternating order: W (fa) or x (fb) block index; r = 0 -> fa[0], 1 -> fb[0], 2 n -> fb[n],
// 2 n + 1 -> fa[n]
constexpr bool hb_sq_isw(int r) { return r == 0 || (r >= 2 && (r & 1)); }
constexpr int hb_sq_blk(int r) { return r < 2 ? 0 : r / 2; }
// F8HB slab schedule (32 MFMA slots): x pieces spread over [B1, B2), W pieces over [B2, B3)
constexpr int hb8_piece(int i, int B1, int B2, int B3, int NPW, int NPX) {
    for (int p = 0; p < NPX; ++p)
        if (B1 + p * (B2 - B1) / NPX == i) return NPW + p;
    for (int p = 0; p < NPW; ++p)
        if (B2 + p * (B3 - B2) / NPW == i) return p;
    return -1;
}

// HB slab schedule: the DMA piece issued before MFMA i of the 128 (-1: none).  Pieces 0 .. NPW-1 are W, the rest x.
constexpr int hb_piece(int i, int B1, int B2, int B3, int DX, int DW, int NPW, int NPX) {
    return (i >= B1 && i < B2 && (i - B1) % DX == 0 && (i - B1) / DX < NPX) ? NPW + (i - B1) / DX
           : (i >= B2 && i < B3 && (i - B2) % DW == 0 && (i - B2) / DW < NPW) ? (i - B2) / DW
                                                                              : -1;
}
// hipBLASLt's distribution: x pieces 0-4 after B1 and 5-7 after B2 (every 2 MFMAs), W pieces 0-4 spread over
// B2+8 .. B3 and 5-7 after B3
constexpr int hb_piece_lib(int i, int B1, int B2, int B3, int NPW, int NPX) {
    return (i >= B1 && i < B1 + 10 && (i - B1) % 2 == 0) ? NPW + (i - B1) / 2
           : (i >= B2 && i < B2 + 6 && (i - B2) % 2 == 0) ? NPW + 5 + (i - B2) / 2
           : (i >= B2 + 8 && i < B2 + 58 && (i - B2 - 8) % 10 == 0) ? (i - B2 - 8) / 10
           : (i >= B3 + 4 && i < B3 + 16 && (i - B3 - 4) % 4 == 0) ? 5 + (i - B3 - 4) / 4
                                                                    : -1;
}

// W8A8 fp8 (F8): a fragment of v_mfma_scale_f32_16x16x128_f8f6f4 is 32 k-bytes per lane (two 16-B chunks)
typedef int lg_i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 lg_mma(const bf16x8& a, const bf16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// block-scaled form fed the unit MX exponent (127 = 2^0): the per-token / per-channel scales go in the epilogue
__device__ __forceinline__ f32x4 lg_mma(const lg_i32x8& a, const lg_i32x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// f(std::integral_constant<int, I>{}) for every I of the sequence, in order (a compile-time unrolled loop)
template <typename F, int... Is>
__device__ __forceinline__ void lg_static_for(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}

// 64-B-row chunk swizzle (the 16x16x32 fragment reads of a 16-row block land on 16 distinct 16-B slots)
__device__ __forceinline__ int lg_swz64(int row) { return (4 - ((row >> 2) & 3)) & 3; }

// ABL (timing diagnostics only, plain mode): 1 no DMA in the loop, 2 no fragment reads in the loop, 4 no MFMA,
// 8 every tile's DMA sources aliased onto tile (0, 0) (operands L2-resident), 16 (slab) no vmcnt wait before the
// barrier, 32 (slab) no barrier either — 16/32 read LDS the DMA may not have filled: timing only, wrong results
// STG (slab schedule, 8 waves): the slab's DMA is split between the wave groups — waves 0-3 issue theirs in k-step B,
// waves 4-7 (their SIMD partners) in the next k-step A — so one wave of each SIMD issues DMA while the other runs MFMAs
// VAR (slab schedule): 0 the compiler places the DMA by sched_group_barrier (every DMA before the block's first
// ds_read), 1 STG, 2 MAN: each k-step written out in issue order, DMA pieces as inline-asm buffer_load ... lds spread
// evenly through k-step B among the MFMAs and ds_reads (hipcc cannot see an asm DMA write LDS, so it adds no
// lgkmcnt wait in front of it; the ring buffers it writes are disjoint from the ones being read by construction)
// F8 (ring schedule only): W8A8 e4m3fn operands (PPArgs x / w hold the bytes), one 128-deep MFMA k-step per 128-B
// stage row, y = (x W^T) * xsc[m] * wsc[n] in the epilogue (plain / SwiGLU)
template <int WN, int XM, int RB, int ST, int MODE, bool NORMP, int NWX, int ABL = 0, int VAR = 0, bool F8 = false>
__global__ void __launch_bounds__(128 * NWX, 1) gemm_lg_kernel(PPArgs a) {
    constexpr bool STG = VAR == 1, MAN = VAR == 2;
    // VAR 3 (M32): the slab schedule on v_mfma_f32_32x32x16_bf16 — 32 x 32 blocks, half the MFMA issues per k-step
    // for the same fragment reads (the 16x16x32 fragments of a wave are regrouped as 32-row blocks x two 16-deep k
    // halves); the accumulators are copied into the 16x16 register order before split-K / the epilogue, which then
    // maps (block, register) -> (n, m) with the 32x32 output layout
    constexpr bool M32 = VAR == 3;
    // VAR 4 (HB): one wave per SIMD (NWX = 2), 128 x 128 outputs per wave, and the slab loop of three barriers per
    // 64-deep slab (profiles/r6_gemm_isa_diff.md): the wave reads ALL of slab j's fragments into registers early (k-step
    // 0 at the end of slab j-1, k-step 1 in the first quarter of slab j), so the slab's LDS buffer is released per
    // operand after a quarter (x) / half (W) of the slab and slab j+2's LDS-DMA gets ~1.5 slabs to land (vmcnt counted,
    // never 0); every wave stages a share of both operands, so each release barrier is followed by DMA on all waves
    // HB variants (timing study, VAR 5-11 = 4 + bits; every one computes the same result): bit 0 LDS-DMA pieces
    // without the s_nop after the M0 write; bit 1 hipBLASLt's DMA distribution (x: 5 pieces after B1 + 3 after B2,
    // W: 5 after B2 + 3 after B3, vmcnt(13)); bit 2 lgkmcnt(0) before the slab's last MFMA instead of hipcc's counted
    // waits at the next slab's head; bit 3 precomputed addressing (below); bit 4 LDS-staged epilogue; bit 5 the next
    // slab's reads from MFMA 94 (below)
    constexpr bool HB = VAR >= 4 && VAR < 260;
    constexpr int HBV = HB ? VAR - 4 : 0;
    constexpr int ES = F8 ? 1 : 2;  // operand bytes per element
    // F8 + HB (VAR with bits 8 and 16: precomputed addressing, staged epilogue): the HB slab loop on
    // v_mfma_scale_f32_32x32x64_f8f6f4 (F8HB below)
    static_assert(!F8 || (RB == 128 && MODE != kResid && !NORMP && ABL == 0 &&
                          (ST >= 3 ? VAR == 0 : (HB && (HBV & 24) == 24 && !(HBV & 2) && !(HBV & 32)))),
                  "fp8: ring schedule or the HB slab loop, 128-B rows, plain / SwiGLU epilogue");
    constexpr bool F8HB = F8 && HB;
    // bit 6 (HBV & 64, bf16): the F8HB loop on v_mfma_f32_32x32x16_bf16 — a slot is two 16-deep MFMAs (the lo / hi
    // 16 B of a 32-B fragment), so a slab is 32 slots of 64 MFMA cycles as in F8HB, with half the MFMA issues of
    // the 16x16x32 loop
    constexpr bool B32HB = HB && !F8 && (HBV & 64);
    constexpr bool XHB = F8HB || B32HB;  // the 32-slot slab loop
    static_assert(!B32HB || ((HBV & 24) == 24 && !(HBV & 2) && !(HBV & 32)), "32x32 HB: precomputed + staged");
    constexpr bool L32 = M32 || XHB;  // 32x32 accumulator blocks
    using FT = std::conditional_t<F8, lg_i32x8, bf16x8>;  // MFMA operand fragment
    constexpr int NW = 2 * NWX;                       // waves: 2 along W x NWX along x (NWX = 4: two per SIMD)
    constexpr int RPI = 1024 / RB;                    // image rows per LDS-DMA instruction
    constexpr int KS = F8 ? 1 : RB / 64;              // MFMA k-steps per stage (bf16 32 deep, F8 128 deep)
    constexpr int WIMG = WN * RB, XIMG = XM * RB, STAGE = WIMG + XIMG;
    constexpr int NINS = (WN + XM) / RPI;             // DMA instructions per stage (whole workgroup)
    constexpr int NPER = NINS / NW;                   // ... per wave
    constexpr int NT = WN / 32, MT = XM / (16 * NWX); // 16-row W / x blocks per wave
    constexpr int NA = NT * KS, NB = MT * KS;         // fragments per stage per wave
    constexpr int H1 = NT / 2;                        // W blocks of part 1
    constexpr int MF1 = H1 * MT * KS, MF2 = (NT - H1) * MT * KS;  // MFMAs of part 1 / part 2
    constexpr int EXTRA = ST * STAGE;                 // flag + inv[XM] after the ring
    static_assert(NINS % NW == 0 && NPER >= 1 && MT >= 1, "tile too small for the loader waves");
    // ST == 2: the slab schedule (two 64-deep LDS buffers, fragments pipelined per 32-deep k-step, one barrier per
    // slab); ST >= 3: the ring schedule (DMA of stage t+ST-1 into the buffer of stage t-1)
    constexpr bool SLAB = ST == 2;
    static_assert(!STG || (SLAB && NWX == 4), "staggered DMA: slab schedule, two waves per SIMD");
    static_assert(!MAN || SLAB, "issue-ordered k-steps: slab schedule");
    static_assert(!M32 || (SLAB && !F8 && ABL == 0 && NT % 2 == 0 && MT % 2 == 0), "32x32 MFMA: slab schedule, bf16");
    static_assert(!HB || (SLAB && ABL == 0 && NWX == 2 && NT == 8 && MT == 8), "HB: 256 x 256 slab, 4 waves");
    static_assert(ST >= 3 || (SLAB && RB == 128), "slab schedule: 64-deep (128-B row) slabs");
    static_assert(MODE != kSwiglu || (WN / 4) % 16 == 0, "swiglu: WN/4 gate rows per wave, multiple of 16");
    static_assert(RB == 64 || RB == 128, "stage depth 32 or 64");
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wi = wave / NWX, wj = wave % NWX;
    const int M = a.M, K = a.K;
    const int mt = (M + XM - 1) / XM;
    const int ntl = MODE == kSwiglu ? a.F / (WN / 2) : (a.N + WN - 1) / WN;
    const int S = a.splitk;
    const int task = xcd_remap(blockIdx.x, mt * ntl * S);
    const int ks = task % S, tile = task / S;
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
    const int m0 = tm * XM;
    const int tns = (ABL & 8) ? 0 : tn, m0s = (ABL & 8) ? 0 : m0;  // DMA source tile (diagnostics may alias)
    // stages of this task's K range: kts = 64-deep units (bf16) / 128-deep units (F8, one per stage)
    const int NS = F8 ? a.kts : a.kts * (64 / (RB / 2));
    const int64_t kbeg = (int64_t)ks * a.kts * (F8 ? 128 : 64);

    // ---- LDS-DMA sources: instruction q of the stage (q = wave * NPER + i) fills image rows q*RPI .. +RPI of the
    // concatenated [W rows; x rows] image; lane l fills row q*RPI + l / (RB/16), physical chunk l % (RB/16), from the
    // logical chunk the read-side swizzle maps there.  buffer_load ... lds through one descriptor per operand: a 32-bit
    // per-lane byte offset (half the VGPRs of flat 64-bit addresses), the stage's k offset in the scalar soffset, and
    // rows past the end of W / x (partial last tiles) read as zeros by the descriptor's range check (never stored)
    const int wbytes = (int)((MODE == kSwiglu ? 2 * a.F : a.N) * (int64_t)K * ES), xbytes = (int)((int64_t)M * K * ES);
    uint32_t voff[NPER];
    int dsto[NPER];
    bool isw[NPER];
    // HB: wave w stages W image pieces [w NPW, +NPW) (pieces 0 .. NPW-1 of its list) and x pieces [w NPX, +NPX)
    constexpr int NPW = WN / RPI / NW, NPX = XM / RPI / NW;
#pragma unroll
    for (int i = 0; i < NPER; ++i) {
        const int q = HB ? (i < NPW ? wave * NPW + i : WN / RPI + wave * NPX + (i - NPW)) : wave * NPER + i;
        const int r = q * RPI + lane / (RB / 16);
        const int pc = lane % (RB / 16);
        dsto[i] = q * 1024;
        isw[i] = q * RPI < WN;  // wave-uniform
        if (r < WN) {
            int wrow;
            if constexpr (MODE == kSwiglu)
                wrow = r < WN / 2 ? tns * (WN / 2) + r : a.F + tns * (WN / 2) + (r - WN / 2);
            else
                wrow = tns * WN + r;
            const int lc = RB == 64 ? pc ^ lg_swz64(r) : pc ^ (r & 7);
            voff[i] = (uint32_t)(((int64_t)wrow * K + kbeg) * ES + lc * 16);
        } else {
            const int xr = r - WN;
            const int lc = RB == 64 ? pc ^ lg_swz64(xr) : pc ^ (xr & 7);
            voff[i] = (uint32_t)(((int64_t)(m0s + xr) * K + kbeg) * ES + lc * 16);
        }
    }
    // DMA of stage j into ring buffer j % ST.  Issued unconditionally so it shares a basic block with the MFMAs it is
    // interleaved with (and every stage leaves the same vmcnt count): a stage past the end re-reads the last stage's
    // source into a buffer no later stage reads
    const int NS1 = NS - 1;
    auto issue = [&](int j) {
        unsigned char* st = smem + (j % ST) * STAGE;
        const int kb = min(j, NS1) * RB;  // byte offset of stage j in the row
#pragma unroll
        for (int i = 0; i < NPER; ++i)
            lg_dma16(isw[i] ? (const void*)a.w : (const void*)a.x, isw[i] ? wbytes : xbytes, st + dsto[i], voff[i], kb);
    };

    // ---- fragment addressing: W rows (MFMA A) and x rows (MFMA B); the swizzle term is lane-constant
    int wrow0[NT];
#pragma unroll
    for (int s = 0; s < NT; ++s) {
        if constexpr (MODE == kSwiglu)
            wrow0[s] = s < NT / 2 ? wi * (WN / 4) + 16 * s : WN / 2 + wi * (WN / 4) + 16 * (s - NT / 2);
        else
            wrow0[s] = wi * (WN / 2) + 16 * s;
    }
    const int xrow0 = wj * (XM / NWX);
    // M32: first W row of each 32-row block (SwiGLU: gate blocks, then the matching up blocks)
    int wrow32[L32 ? NT / 2 : 1];
    if constexpr (L32) {
#pragma unroll
        for (int S = 0; S < NT / 2; ++S) {
            if constexpr (MODE == kSwiglu)
                wrow32[S] = S < NT / 4 ? wi * (WN / 4) + 32 * S : WN / 2 + wi * (WN / 4) + 32 * (S - NT / 4);
            else
                wrow32[S] = wi * (WN / 2) + 32 * S;
        }
    }
    // F8: the two chunks 2 (lane >> 4) and 2 (lane >> 4) + 1 of the lane's 128-B row, swizzled like the bf16 reads
    int loff[F8 ? 2 : KS];
#pragma unroll
    for (int kk = 0; kk < (F8 ? 2 : KS); ++kk) {
        if constexpr (F8)
            loff[kk] = (lane & 15) * 128 + (((2 * (lane >> 4) + kk) ^ (lane & 7)) << 4);
        else if constexpr (RB == 64)
            loff[kk] = (lane & 15) * 64 + (((lane >> 4) ^ lg_swz64(lane & 15)) << 4);
        else
            loff[kk] = (lane & 15) * 128 + (((4 * kk + (lane >> 4)) ^ (lane & 7)) << 4);
    }

    f32x4 acc[NT][MT];
#pragma unroll
    for (int s = 0; s < NT; ++s)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // NORMP: the producer's partials of the tile's x rows, all loads issued before the DMA prologue.  Lane l < RPW
    // of wave w owns local row w RPW + l and sums that row's partials itself (16-B loads of up to 64 partials, the
    // rest in a tail loop): no cross-lane reduction (the per-row wave_sum of 6 shuffles cost the 4-wave 256-row tiles
    // 64 dependent reductions per wave before the first MFMA)
    constexpr int RPW = XM / NW;  // x rows per wave for the inv computation
    static_assert(RPW <= 64, "one x row per lane");
    f32x4 pv4[NORMP ? 16 : 1];
    const int prow = wave * RPW + lane;  // (lanes >= RPW: a clamped duplicate row, never written)
    const bool pv_vec = NORMP && (a.nparts_in & 3) == 0;
    if constexpr (NORMP) {
        const float* pp = a.part_in + (int64_t)min(m0 + min(prow, XM - 1), M - 1) * a.nparts_in;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            pv4[i] = pv_vec && 4 * i < a.nparts_in ? *reinterpret_cast<const f32x4*>(pp + 4 * i) : f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // F8HB: the tile's scales, loaded before the prologue and parked in LDS after the ring ([WN] wsc of the image's W
    // rows — SwiGLU: gate rows, then up rows — then [XM] xsc), so the epilogue reads them from LDS instead of issuing
    // dependent global loads between its LDS stores (measured: ~10 us per tile of serialised L2 round trips)
    constexpr int NSCL = F8HB ? (WN + XM + 128 * NWX - 1) / (128 * NWX) : 1;
    float scv[NSCL];
    float* scl = reinterpret_cast<float*>(smem + EXTRA + 16 + XM * 4);
    if constexpr (F8HB) {
#pragma unroll
        for (int q = 0; q < NSCL; ++q) {
            const int i = tid + q * 128 * NWX;
            int wr;
            if constexpr (MODE == kSwiglu)
                wr = i < WN / 2 ? tn * (WN / 2) + i : a.F + tn * (WN / 2) + (i - WN / 2);
            else
                wr = min(tn * WN + i, a.N - 1);
            scv[q] = i < WN ? a.wsc[wr] : a.xsc[min(m0 + min(i - WN, XM - 1), M - 1)];
        }
    }

    // ---- prologue: stages 0 .. ST-2 in flight (slab schedule: slabs 0 and 1)
    const int grp = wave >> 2;  // wave group (STG): waves w and w+4 share a SIMD
#pragma unroll
    for (int p = 0; p < (SLAB ? 2 : ST - 1); ++p)
        if (!(STG && p == 1 && grp == 1)) issue(p);  // (STG: group 1 issues its part of slab 1 in slab 0's k-step A)
    if constexpr (F8HB) {
#pragma unroll
        for (int q = 0; q < NSCL; ++q)
            if (tid + q * 128 * NWX < WN + XM) scl[tid + q * 128 * NWX] = scv[q];
    }

    if constexpr (NORMP) {
        float* inv = reinterpret_cast<float*>(smem + EXTRA + 16);
        const float* pp = a.part_in + (int64_t)min(m0 + min(prow, XM - 1), M - 1) * a.nparts_in;
        f32x4 t4 = (pv4[0] + pv4[1]) + (pv4[2] + pv4[3]);
#pragma unroll
        for (int i = 4; i < 16; i += 4) t4 += (pv4[i] + pv4[i + 1]) + (pv4[i + 2] + pv4[i + 3]);
        float ss = (t4[0] + t4[1]) + (t4[2] + t4[3]);
        for (int i = pv_vec ? 64 : 0; i < a.nparts_in; ++i) ss += pp[i];
        if (lane < RPW) inv[prow] = rsqrtf(ss / (float)K + a.eps);
    }

    if constexpr (SLAB) {
        // ---- slab schedule.  Slab j (64-deep) lives in buffer j % 2; its k-step 0 fragments go to set 0, k-step 1
        // to set 1.  Slab j:
        //   k-step A: MFMAs on set 0  ||  ds_read of slab j k-step 1 into set 1
        //   lgkmcnt(0) (every read of buffer j % 2 done), vmcnt(0) (this wave's DMA of slab j+1 landed), s_barrier
        //   k-step B: DMA of slab j+2 into buffer j % 2  ||  MFMAs on set 1  ||  ds_read of slab j+1 k-step 0 (set 0)
        // The DMA of a slab has one whole slab of MFMAs (k-step B + the next k-step A) to land; every DMA piece reads
        // whole 128-B lines.
        bf16x8 fa0[NT], fb0[MT], fa1[NT], fb1[MT];
        auto rd = [&](int j, int kk, bf16x8 (&fa)[NT], bf16x8 (&fb)[MT]) {
            const unsigned char* wb = smem + (j & 1) * STAGE;
            const unsigned char* xb = wb + WIMG;
            if constexpr (M32) {
                // lane (r = lane & 31, h = lane >> 5): row r of the 32-row block, the 16-B chunk 2 k16 + h of the
                // k-step's four (the same XOR swizzle by row & 7 as the 16x16 reads)
                const int r = lane & 31;
#pragma unroll
                for (int k16 = 0; k16 < 2; ++k16) {
                    const int co = (((4 * kk + 2 * k16 + (lane >> 5)) ^ (r & 7)) << 4);
#pragma unroll
                    for (int S = 0; S < NT / 2; ++S)
                        fa[2 * S + k16] = *reinterpret_cast<const bf16x8*>(wb + (wrow32[S] + r) * RB + co);
#pragma unroll
                    for (int U = 0; U < MT / 2; ++U)
                        fb[2 * U + k16] = *reinterpret_cast<const bf16x8*>(xb + (xrow0 + 32 * U + r) * RB + co);
                }
                return;
            }
#pragma unroll
            for (int s = 0; s < NT; ++s) fa[s] = *reinterpret_cast<const bf16x8*>(wb + wrow0[s] * RB + loff[kk]);
#pragma unroll
            for (int t = 0; t < MT; ++t)
                fb[t] = *reinterpret_cast<const bf16x8*>(xb + (xrow0 + 16 * t) * RB + loff[kk]);
        };
        f32x16 acc32[L32 ? NT / 2 : 1][L32 ? MT / 2 : 1];
        if constexpr (L32) {
#pragma unroll
            for (int S = 0; S < NT / 2; ++S)
#pragma unroll
                for (int U = 0; U < MT / 2; ++U)
#pragma unroll
                    for (int i = 0; i < 16; ++i) acc32[S][U][i] = 0.f;
        }
        // F8HB fragments (v_mfma_scale_f32_32x32x64_f8f6f4): block S (32 W rows) / U (32 x rows) of the slab's 64-deep
        // k-step kk; lane (r = lane & 31, hf = lane >> 5) holds k-bytes 64 kk + 32 hf .. +31 of row r, i.e. logical
        // chunks 4 kk + 2 hf and + 1 of the 128-B image row, each one ds_read_b128 at its XOR-swizzled slot (chunk ^
        // (r & 7), as the DMA wrote it).  Both operands use the same (half, byte) -> k map.  One base VGPR per
        // (buffer parity, operand, k-step, half); block offsets are immediates.
        // (B32HB: a 32-deep k-step is two 16-deep MFMAs; lane half hf holds k 8 hf .. +7 of each, i.e. chunks
        // 4 kk + hf (lo) and 4 kk + 2 + hf (hi))
        lg_i32x8 ga0[XHB ? NT / 2 : 1], gb0[XHB ? MT / 2 : 1], ga1[XHB ? NT / 2 : 1], gb1[XHB ? MT / 2 : 1];
        const unsigned char* f8b[XHB ? 2 : 1][2][2][2];
        if constexpr (XHB) {
            const int r = lane & 31, hf = lane >> 5;
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int co = ((F8 ? 4 * kk + 2 * hf + h : 4 * kk + 2 * h + hf) ^ (r & 7)) << 4;
                        f8b[p][0][kk][h] = smem + p * STAGE + (wrow32[0] + r) * RB + co;
                        f8b[p][1][kk][h] = smem + p * STAGE + WIMG + (xrow0 + r) * RB + co;
                    }
        }
        // one F8HB fragment: parity p, operand op (0 W, 1 x), k-step kk, block row offset off (bytes)
        auto f8rd = [&](int p, int op, int kk, int off) -> lg_i32x8 {
            const lg_i32x4 lo = *reinterpret_cast<const lg_i32x4*>(f8b[XHB ? p : 0][op][kk][0] + off);
            const lg_i32x4 hi = *reinterpret_cast<const lg_i32x4*>(f8b[XHB ? p : 0][op][kk][1] + off);
            return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        };
        auto mm = [&](bf16x8 (&fa)[NT], bf16x8 (&fb)[MT]) {
            if constexpr (M32) {
#pragma unroll
                for (int k16 = 0; k16 < 2; ++k16)
#pragma unroll
                    for (int S = 0; S < NT / 2; ++S)
#pragma unroll
                        for (int U = 0; U < MT / 2; ++U)
                            acc32[S][U] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2 * S + k16], fb[2 * U + k16],
                                                                                   acc32[S][U], 0, 0, 0);
            } else if constexpr (!(ABL & 4)) {
#pragma unroll
                for (int s = 0; s < NT; ++s)
#pragma unroll
                    for (int u = 0; u < MT; ++u)
                        acc[s][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s], fb[u], acc[s][u], 0, 0, 0);
            } else {
#pragma unroll
                for (int i = 0; i < NT; ++i) asm volatile("" ::"v"(fa[i]));
#pragma unroll
                for (int i = 0; i < MT; ++i) asm volatile("" ::"v"(fb[i]));
            }
        };
        constexpr int MF = M32 ? NT * MT / 2 : NT * MT, NR = NT + MT;
        if constexpr (STG) {
            if (grp == 0) lg_vmcnt<NPER>();  // slab 0 landed (group 0's part of slab 1 in flight)
            else lg_vmcnt<0>();
        } else {
            lg_vmcnt<NPER>();  // slab 0 landed (slab 1 in flight)
        }
        lg_bar();
        if constexpr (XHB) {
            ga0[0] = f8rd(0, 0, 0, 0);  // (the loop's set-0 read order: ga[0], gb[*], ga[1..])
#pragma unroll
            for (int u = 0; u < MT / 2; ++u) gb0[u] = f8rd(0, 1, 0, 32 * RB * u);
#pragma unroll
            for (int s = 1; s < NT / 2; ++s) ga0[s] = f8rd(0, 0, 0, hb_wrow32(s, MODE == kSwiglu, WN) * RB);
        } else if constexpr (HB && (HBV & 128)) {  // (the loop's alternating set-0 read order, see hb_sq_isw)
#pragma unroll
            for (int r = 0; r < NT + MT; ++r) {
                const int b = hb_sq_blk(r);
                if (hb_sq_isw(r)) fa0[b] = *reinterpret_cast<const bf16x8*>(smem + wrow0[b] * RB + loff[0]);
                else fb0[b] = *reinterpret_cast<const bf16x8*>(smem + WIMG + (xrow0 + 16 * b) * RB + loff[0]);
            }
        } else if constexpr (HB) {
            // the order of the loop's set-0 reads (fa[0], fb[*], fa[1..]): the same pending-read state enters the loop
            // from the prologue and from the back edge, so hipcc's waits at the first MFMAs stay counted
            fa0[0] = *reinterpret_cast<const bf16x8*>(smem + wrow0[0] * RB + loff[0]);
#pragma unroll
            for (int t = 0; t < MT; ++t)
                fb0[t] = *reinterpret_cast<const bf16x8*>(smem + WIMG + (xrow0 + 16 * t) * RB + loff[0]);
#pragma unroll
            for (int s = 1; s < NT; ++s) fa0[s] = *reinterpret_cast<const bf16x8*>(smem + wrow0[s] * RB + loff[0]);
        } else {
            rd(0, 0, fa0, fb0);
        }
        // STG: one straight-line loop per wave group (the DMA sits in a different k-step), so each keeps its
        // compile-time interleave
        // MAN: k-step in issue order.  MFMA i of the block is (W block i / MT, x block i % MT); DMA piece d goes before
        // MFMA d * DS, fragment read r after MFMA r * RS + RS - 1 (the last quarter of the block reads nothing)
        auto kstep_man = [&](auto DMA_ON, bf16x8 (&fa)[NT], bf16x8 (&fb)[MT], int jr, int kkr, bf16x8 (&na)[NT],
                             bf16x8 (&nb)[MT], int jd) {
            constexpr bool dma_on = decltype(DMA_ON)::value;
            constexpr int DS = MF / NPER > 0 ? MF / NPER : 1;
            constexpr int RS = (MF - MF / 4) / NR > 0 ? (MF - MF / 4) / NR : 1;
            const unsigned char* wb = smem + (jr & 1) * STAGE;
            const unsigned char* xb = wb + WIMG;
            unsigned char* db = smem + (jd & 1) * STAGE;
            const int kb = min(jd, NS1) * RB;
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                if constexpr (dma_on) {
                    if (i % DS == 0 && i / DS < NPER) {
                        const int d = i / DS;
                        lg_dma16_asm(isw[d] ? (const void*)a.w : (const void*)a.x, isw[d] ? wbytes : xbytes,
                                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(db + dsto[d])),
                                     voff[d], kb);
                    }
                }
                if constexpr (!(ABL & 4))
                    acc[i / MT][i % MT] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i / MT], fb[i % MT], acc[i / MT][i % MT], 0, 0, 0);
                else
                    asm volatile("" ::"v"(fa[i / MT]), "v"(fb[i % MT]));
                if (!(ABL & 2) && i % RS == RS - 1 && i / RS < NR) {
                    const int r = i / RS;
                    if (r < NT) na[r] = *reinterpret_cast<const bf16x8*>(wb + wrow0[r] * RB + loff[kkr]);
                    else nb[r - NT] = *reinterpret_cast<const bf16x8*>(xb + (xrow0 + 16 * (r - NT)) * RB + loff[kkr]);
                }
                // pin the order at every DMA slot (hipcc would otherwise sink the asm pieces to the block's end)
                if (i % DS == DS - 1) __builtin_amdgcn_sched_barrier(0);
            }
        };
        if constexpr (HB) {
            // slab j, MFMA i of 128 (k-step i / 64; W block s = (i % 64) / 8, x block t = i % 8), issue order pinned:
            //   i = 1, 3, .. 15 : ds_read of slab j k-step 1 x fragments (set 1)
            //   B1 (before 22)  : lgkmcnt(0) + barrier — every wave holds slab j's x fragments: x buffer released
            //   22 .. 51        : the wave's NPX x pieces of slab j+2 (one per 3 MFMAs) + slab j k-step 1 W reads
            //   B2 (before 52)  : lgkmcnt(0) + barrier — W buffer released
            //   52 .. 111       : the wave's NPW W pieces of slab j+2 (one per 7 MFMAs)
            //   B3 (before 112) : vmcnt(NPER) (this wave's slab j+1 pieces landed; slab j+2's stay in flight) + barrier
            //   112 .. 127      : ds_read of slab j+1 k-step 0 (set 0): fa[0], fb[0..7], fa[1..7]
            // hipcc inserts the counted lgkmcnt waits of the set-0 reads at the next slab's first MFMAs.
            // bit 5 (HBV & 32): hipBLASLt's B3 placement — the next slab's fragment reads start at MFMA 94 and are
            // spread one per two MFMAs (instead of one per MFMA from 112), the W pieces one per 5 MFMAs before it
            constexpr int MFK = NT * MT, B1 = 22, B2 = 52, B3 = (HBV & 32) ? 94 : 2 * MFK - (NT + MT);
            constexpr int RSP = (HBV & 32) ? 2 : 1;  // MFMAs per set-0 read after B3
            constexpr int DX = 3, DW = (HBV & 32) ? 5 : 7;
            static_assert(NPW == 8 && NPX == 8, "HB: 8 W + 8 x pieces per wave and slab");
            const int pstride = RPI * K * ES;  // source bytes between a wave's consecutive pieces of one operand
            static_assert(B1 >= 2 * MT + 2 && B1 + DX * NPX <= B2 && B1 + 1 + 3 * NT <= B2 && B2 + DW * NPW <= B3 &&
                              B3 + RSP * (NT + MT) <= 2 * MFK,
                          "HB schedule");
            // the accumulators live in AGPRs across the whole loop: pinned at both ends, so the epilogue's VGPR use
            // (resid / SwiGLU / norm-scale forms) cannot make the register allocator shuffle them inside the loop
            auto pin_acc = [&]() {
                if constexpr (XHB) {
#pragma unroll
                    for (int S = 0; S < NT / 2; ++S)
#pragma unroll
                        for (int U = 0; U < MT / 2; ++U) asm volatile("" : "+a"(acc32[S][U]));
                } else {
#pragma unroll
                    for (int s = 0; s < NT; ++s)
#pragma unroll
                        for (int t = 0; t < MT; ++t) asm volatile("" : "+a"(acc[s][t]));
                }
            };
            pin_acc();
            if constexpr (XHB) {
                // W8A8 on the HB loop: a 128-B slab row is 128 e4m3 k = two 64-deep k-steps of 16
                // v_mfma_scale_f32_32x32x64_f8f6f4 (4 W x 4 x blocks of 32, each MFMA 4x the issue time of a bf16
                // 16x16x32), so a slab is 32 MFMA slots with the same per-slab bytes, fragment reads (2 ds_read_b128
                // per fragment, 32 per slab) and DMA pieces as the bf16 loop's 128, and the same three barriers:
                //   slots 0-3    : set-1 (k-step 1) x fragments of slab j
                //   B1 (5)       : lgkmcnt(0) + barrier — x buffer released; x pieces of slab j+2 over [B1, B2)
                //   6, 8, 10, 12 : set-1 W fragments
                //   B2 (14)      : W buffer released; W pieces of slab j+2 over [B2, B3)
                //   B3 (28)      : vmcnt(NPER) + barrier — slab j+1 landed
                //   28-31        : set-0 fragments of slab j+1, two per slot (ga[0], gb[*], ga[1..])
                constexpr int MK = (NT / 2) * (MT / 2), F1 = 5, F2 = 14, F3 = 28;
                static_assert(MK == 16 && F1 >= MT / 2 + 1 && F1 + 1 + 2 * (NT / 2 - 1) < F2 - 1 && F3 + 4 == 2 * MK,
                              "F8HB schedule");
                uint32_t m0w[2], m0x[2];
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    m0w[p] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(smem + p * STAGE + dsto[0]));
                    m0x[p] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(smem + p * STAGE + dsto[NPW]));
                }
                const uint32_t vw = voff[0], vx = voff[NPW];
                auto half = [&](auto PC, int j) {
                    constexpr int P = decltype(PC)::value;  // slab j in buffer P, slab j+1 in 1 - P
                    const int kb = min(j + 2, NS1) * RB;
                    const void* bw = (const unsigned char*)a.w + kb;
                    const void* bx = (const unsigned char*)a.x + kb;
                    const int nw = wbytes - kb, nx = xbytes - kb;
                    auto slot = [&](auto IC) {
                        constexpr int i = decltype(IC)::value;
                        if constexpr (i == F1 || i == F2) {
                            __builtin_amdgcn_s_waitcnt(0xC07F);
                            lg_bar();
                        }
                        if constexpr (i == F3) {
                            lg_vmcnt<NPER>();
                            lg_bar();
                        }
                        constexpr int piece = hb8_piece(i, F1, F2, F3, NPW, NPX);
                        if constexpr (piece >= 0) {
                            constexpr bool isW = piece < NPW;
                            constexpr int q = isW ? piece : piece - NPW;
                            const uint64_t b = (uint64_t)(isW ? bw : bx);
                            const lg_i32x4 r = {(int)(uint32_t)b, (int)(uint32_t)(b >> 32), isW ? nw : nx, 0x00020000};
                            if constexpr (q == 0)
                                asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                                             ::"v"(isW ? vw : vx), "s"(r), "s"(isW ? m0w[P] : m0x[P]) : "memory");
                            else
                                asm volatile("s_add_u32 m0, m0, 0x400\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                                             ::"v"(isW ? vw : vx), "s"(r), "s"(q * pstride) : "memory");
                        }
                        constexpr int ii = i % MK, S = ii / (MT / 2), U = ii % (MT / 2);
                        const lg_i32x8& fa = i < MK ? ga0[S] : ga1[S];
                        const lg_i32x8& fb = i < MK ? gb0[U] : gb1[U];
                        if constexpr (F8)
                            acc32[S][U] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa, fb, acc32[S][U], 0, 0, 0,
                                                                                        127, 0, 127);
                        else {  // B32HB: the two 16-deep halves
                            typedef __bf16 lg_bf16x8 __attribute__((ext_vector_type(8)));
                            acc32[S][U] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                __builtin_bit_cast(lg_bf16x8, __builtin_shufflevector(fa, fa, 0, 1, 2, 3)),
                                __builtin_bit_cast(lg_bf16x8, __builtin_shufflevector(fb, fb, 0, 1, 2, 3)), acc32[S][U], 0, 0,
                                0);
                            acc32[S][U] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                __builtin_bit_cast(lg_bf16x8, __builtin_shufflevector(fa, fa, 4, 5, 6, 7)),
                                __builtin_bit_cast(lg_bf16x8, __builtin_shufflevector(fb, fb, 4, 5, 6, 7)), acc32[S][U], 0, 0,
                                0);
                        }
                        if constexpr (i < MT / 2) gb1[i] = f8rd(P, 1, 1, 32 * RB * i);
                        if constexpr (i > F1 && (i - F1 - 1) % 2 == 0 && (i - F1 - 1) / 2 < NT / 2) {
                            constexpr int s = (i - F1 - 1) / 2;
                            ga1[s] = f8rd(P, 0, 1, hb_wrow32(s, MODE == kSwiglu, WN) * RB);
                        }
                        if constexpr (i >= F3) {
                            lg_static_for(
                                [&](auto RC) {
                                    constexpr int r = 2 * (i - F3) + decltype(RC)::value;  // ga[0], gb[0..3], ga[1..3]
                                    if constexpr (r == 0) ga0[0] = f8rd(1 - P, 0, 0, 0);
                                    else if constexpr (r <= MT / 2) gb0[r - 1] = f8rd(1 - P, 1, 0, 32 * RB * (r - 1));
                                    else
                                        ga0[r - MT / 2] =
                                            f8rd(1 - P, 0, 0, hb_wrow32(r - MT / 2, MODE == kSwiglu, WN) * RB);
                                },
                                std::make_integer_sequence<int, 2>{});
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    };
                    lg_static_for(slot, std::make_integer_sequence<int, 2 * MK>{});
                };
                for (int j = 0; j < NS; j += 2) {
                    half(std::integral_constant<int, 0>{}, j);
                    if (j + 1 < NS) half(std::integral_constant<int, 1>{}, j + 1);
                }
            } else if constexpr (HBV & 8) {
                // precomputed addressing: the slab loop unrolled by two, so each half's LDS buffer is a compile-time
                // parity; fragment reads from 8 per-lane base VGPRs (parity x operand x k-step) + immediate offsets;
                // the LDS-DMA destination kept in M0 (one s_mov per operand and slab, then s_add 1 KiB per piece, as
                // hipBLASLt's gfx950 code does: nothing else in the loop uses M0) and the source's k offset folded
                // into the descriptor base once per slab, so a piece's scalar offset is a loop-invariant row stride
                const unsigned char* rbw[2][2];
                const unsigned char* rbx[2][2];
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int kk = 0; kk < 2; ++kk) {
                        rbw[p][kk] = smem + p * STAGE + wrow0[0] * RB + loff[kk];
                        rbx[p][kk] = smem + p * STAGE + WIMG + xrow0 * RB + loff[kk];
                    }
                uint32_t m0w[2], m0x[2];
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    m0w[p] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(smem + p * STAGE + dsto[0]));
                    m0x[p] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uintptr_t)(smem + p * STAGE + dsto[NPW]));
                }
                const uint32_t vw = voff[0], vx = voff[NPW];
                auto half = [&](auto PC, int j) {
                    constexpr int P = decltype(PC)::value;  // slab j lives in buffer P, slab j+1 in 1 - P
                    const int kb = min(j + 2, NS1) * RB;
                    const void* bw = (const unsigned char*)a.w + kb;
                    const void* bx = (const unsigned char*)a.x + kb;
                    const int nw = wbytes - kb, nx = xbytes - kb;
                    auto slot = [&](auto IC) {
                        constexpr int i = decltype(IC)::value;
                        if constexpr (i == B1 || i == B2) {
                            __builtin_amdgcn_s_waitcnt(0xC07F);
                            lg_bar();
                        }
                        if constexpr (i == B3) {
                            lg_vmcnt<(HBV & 2) ? 13 : NPER>();
                            lg_bar();
                        }
                        if constexpr ((HBV & 4) && i == 2 * MFK - 1) __builtin_amdgcn_s_waitcnt(0xC07F);
                        constexpr int piece = (HBV & 2) ? hb_piece_lib(i, B1, B2, B3, NPW, NPX)
                                                        : hb_piece(i, B1, B2, B3, DX, DW, NPW, NPX);
                        if constexpr (piece >= 0) {
                            constexpr bool isW = piece < NPW;
                            constexpr int q = isW ? piece : piece - NPW;
                            const uint64_t b = (uint64_t)(isW ? bw : bx);
                            const lg_i32x4 r = {(int)(uint32_t)b, (int)(uint32_t)(b >> 32), isW ? nw : nx, 0x00020000};
                            if constexpr (q == 0)
                                asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                                             ::"v"(isW ? vw : vx), "s"(r), "s"(isW ? m0w[P] : m0x[P]) : "memory");
                            else
                                asm volatile("s_add_u32 m0, m0, 0x400\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                                             ::"v"(isW ? vw : vx), "s"(r), "s"(q * pstride) : "memory");
                        }
                        constexpr int ii = i % MFK;
                        constexpr bool SQ = (HBV & 128) && i < MFK;  // (k-step 0 only: k-step 1's reads land early)
                        constexpr int s = SQ ? hb_sq_s(ii) : ii / MT, t = SQ ? hb_sq_t(ii) : ii % MT;
                        if constexpr (i < MFK)
                            acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[s], fb0[t], acc[s][t], 0, 0, 0);
                        else
                            acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[s], fb1[t], acc[s][t], 0, 0, 0);
                        if constexpr (i < B1 && (i & 1) && i / 2 < MT)
                            fb1[i / 2] = *reinterpret_cast<const bf16x8*>(rbx[P][1] + 16 * RB * (i / 2));
                        if constexpr (i > B1 && i < B2 && (i - B1 - 1) % 3 == 0 && (i - B1 - 1) / 3 < NT) {
                            constexpr int r = (i - B1 - 1) / 3;
                            fa1[r] = *reinterpret_cast<const bf16x8*>(rbw[P][1] + hb_wrow(r, MODE == kSwiglu, WN) * RB);
                        }
                        if constexpr ((HBV & 128) && i >= B3 && (i - B3) % RSP == 0 && (i - B3) / RSP < NT + MT) {
                            constexpr int r = (i - B3) / RSP, b = hb_sq_blk(r);  // fa0, fb0, fb1, fa1, fb2, fa2, ...
                            if constexpr (hb_sq_isw(r))
                                fa0[b] = *reinterpret_cast<const bf16x8*>(rbw[1 - P][0] + hb_wrow(b, MODE == kSwiglu, WN) * RB);
                            else
                                fb0[b] = *reinterpret_cast<const bf16x8*>(rbx[1 - P][0] + 16 * RB * b);
                        } else if constexpr (i >= B3 && (i - B3) % RSP == 0 && (i - B3) / RSP < NT + MT) {
                            constexpr int r = (i - B3) / RSP;  // fa[0], fb[0..MT-1], fa[1..NT-1]
                            if constexpr (r == 0) fa0[0] = *reinterpret_cast<const bf16x8*>(rbw[1 - P][0]);
                            else if constexpr (r <= MT)
                                fb0[r - 1] = *reinterpret_cast<const bf16x8*>(rbx[1 - P][0] + 16 * RB * (r - 1));
                            else
                                fa0[r - MT] = *reinterpret_cast<const bf16x8*>(
                                    rbw[1 - P][0] + hb_wrow(r - MT, MODE == kSwiglu, WN) * RB);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    };
                    lg_static_for(slot, std::make_integer_sequence<int, 2 * MFK>{});
                };
                for (int j = 0; j < NS; j += 2) {
                    half(std::integral_constant<int, 0>{}, j);
                    if (j + 1 < NS) half(std::integral_constant<int, 1>{}, j + 1);
                }
            } else
            for (int j = 0; j < NS; ++j) {
                const unsigned char* cwb = smem + (j & 1) * STAGE;        // slab j (W image, x image at + WIMG)
                const unsigned char* nwb = smem + ((j + 1) & 1) * STAGE;  // slab j+1
                const uint32_t dbase = (uint32_t)(uintptr_t)(smem + (j & 1) * STAGE);  // slab j+2 lands here
                const int kb = min(j + 2, NS1) * RB;
                // one MFMA slot of the slab, everything decided at compile time
                auto slot = [&](auto IC) {
                    constexpr int i = decltype(IC)::value;
                    if constexpr (i == B1 || i == B2) {
                        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), visible to hipcc's wait bookkeeping
                        lg_bar();
                    }
                    if constexpr (i == B3) {
                        lg_vmcnt<(HBV & 2) ? 13 : NPER>();  // (the pieces this wave issued since the last B3)
                        lg_bar();
                    }
                    if constexpr ((HBV & 4) && i == 2 * MFK - 1) __builtin_amdgcn_s_waitcnt(0xC07F);
                    constexpr int piece = (HBV & 2) ? hb_piece_lib(i, B1, B2, B3, NPW, NPX)
                                                    : hb_piece(i, B1, B2, B3, DX, DW, NPW, NPX);
                    // a wave's pieces of one operand are consecutive 8-row groups of the source (the chunk swizzle
                    // depends on lane / 8 only): one VGPR offset per operand, the piece's rows in the scalar offset
                    if constexpr (piece >= 0)
                        lg_dma16_asm<!(HBV & 1)>(piece < NPW ? (const void*)a.w : (const void*)a.x, piece < NPW ? wbytes : xbytes,
                                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(dbase + dsto[piece])),
                                     piece < NPW ? voff[0] : voff[NPW],
                                     kb + (piece < NPW ? piece : piece - NPW) * pstride);
                    constexpr int ii = i % MFK, s = ii / MT, t = ii % MT;
                    if constexpr (i < MFK)
                        acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[s], fb0[t], acc[s][t], 0, 0, 0);
                    else
                        acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[s], fb1[t], acc[s][t], 0, 0, 0);
                    if constexpr (i < B1 && (i & 1) && i / 2 < MT)
                        fb1[i / 2] = *reinterpret_cast<const bf16x8*>(cwb + WIMG + (xrow0 + 16 * (i / 2)) * RB + loff[1]);
                    if constexpr (i > B1 && i < B2 && (i - B1 - 1) % 3 == 0 && (i - B1 - 1) / 3 < NT) {
                        constexpr int r = (i - B1 - 1) / 3;
                        fa1[r] = *reinterpret_cast<const bf16x8*>(cwb + wrow0[r] * RB + loff[1]);
                    }
                    if constexpr (i >= B3) {
                        constexpr int r = i - B3;  // fa[0], fb[0..MT-1], fa[1..NT-1]
                        if constexpr (r == 0) fa0[0] = *reinterpret_cast<const bf16x8*>(nwb + wrow0[0] * RB + loff[0]);
                        else if constexpr (r <= MT)
                            fb0[r - 1] =
                                *reinterpret_cast<const bf16x8*>(nwb + WIMG + (xrow0 + 16 * (r - 1)) * RB + loff[0]);
                        else fa0[r - MT] = *reinterpret_cast<const bf16x8*>(nwb + wrow0[r - MT] * RB + loff[0]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                };
                lg_static_for(slot, std::make_integer_sequence<int, 2 * MFK>{});
            }
            pin_acc();
        }
        if constexpr (MAN) {
            for (int j = 0; j < NS; ++j) {
                kstep_man(std::integral_constant<bool, false>{}, fa0, fb0, j, 1, fa1, fb1, 0);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                lg_vmcnt<0>();
                lg_bar();
                kstep_man(std::integral_constant<bool, true>{}, fa1, fb1, j + 1, 0, fa0, fb0, j + 2);
            }
        }
        auto loop_stg = [&](auto G) {
            constexpr int g = decltype(G)::value;
            for (int j = 0; j < NS; ++j) {
                // k-step A (group 1: its part of slab j+1's DMA, into buffer (j+1) % 2, free since barrier j-1)
                if constexpr (g == 1) issue(j + 1);
                rd(j, 1, fa1, fb1);
                mm(fa0, fb0);
                lg_sched<0, MF, g == 1 ? NPER : 0, NR>();
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                lg_vmcnt<0>();
                lg_bar();
                // k-step B (group 0: its part of slab j+2)
                if constexpr (g == 0) issue(j + 2);
                rd(j + 1, 0, fa0, fb0);
                mm(fa1, fb1);
                lg_sched<0, MF, g == 0 ? NPER : 0, NR>();
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        if constexpr (MAN || HB) {
        } else if constexpr (STG) {
            if (grp == 0) loop_stg(std::integral_constant<int, 0>{});
            else loop_stg(std::integral_constant<int, 1>{});
        } else
        for (int j = 0; j < NS; ++j) {
            // k-step A
            if constexpr (!(ABL & 2)) rd(j, 1, fa1, fb1);
            else {
#pragma unroll
                for (int i = 0; i < NT; ++i) fa1[i] = fa0[i];
#pragma unroll
                for (int i = 0; i < MT; ++i) fb1[i] = fb0[i];
            }
            mm(fa0, fb0);
            lg_sched<0, MF, 0, NR>();
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr (!(ABL & 16)) lg_vmcnt<0>();  // (ABL 16/32: timing only, races by design)
            if constexpr (!(ABL & 32)) lg_bar();
            // k-step B
            if constexpr (!(ABL & 1)) issue(j + 2);
            if constexpr (!(ABL & 2)) rd(j + 1, 0, fa0, fb0);
            else {
#pragma unroll
                for (int i = 0; i < NT; ++i) fa0[i] = fa1[i];
#pragma unroll
                for (int i = 0; i < MT; ++i) fb0[i] = fb1[i];
            }
            mm(fa1, fb1);
            lg_sched<0, MF, (ABL & 1) ? 0 : NPER, NR>();
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (L32) {
            // 32x32 accumulator register 4 g + i -> acc[2 S + (g >> 1)][2 U + (g & 1)][i]
#pragma unroll
            for (int S = 0; S < NT / 2; ++S)
#pragma unroll
                for (int U = 0; U < MT / 2; ++U)
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        acc[2 * S + (g >> 1)][2 * U + (g & 1)] =
                            f32x4{acc32[S][U][4 * g], acc32[S][U][4 * g + 1], acc32[S][U][4 * g + 2],
                                  acc32[S][U][4 * g + 3]};
        }
    } else {
    // stage 0 landed for every wave (stages 1 .. ST-2 stay in flight)
    lg_vmcnt<(ST - 2) * NPER>();
    lg_bar();

    FT fa0[NA], fb0[NB], fa1[NA], fb1[NB];
    // one fragment of the 16-row block starting at LDS row pointer p (F8: two ds_read_b128)
    auto frag = [&](const unsigned char* p, int kk) -> FT {
        if constexpr (F8) {
            typedef int i32x4_t __attribute__((ext_vector_type(4)));
            const i32x4_t lo = *reinterpret_cast<const i32x4_t*>(p + loff[0]);
            const i32x4_t hi = *reinterpret_cast<const i32x4_t*>(p + loff[1]);
            return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        } else {
            return *reinterpret_cast<const bf16x8*>(p + loff[kk]);
        }
    };
    auto read_frags = [&](int j, FT (&fa)[NA], FT (&fb)[NB]) {
        const unsigned char* wb = smem + (j % ST) * STAGE;
        const unsigned char* xb = wb + WIMG;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
            for (int s = 0; s < NT; ++s) fa[kk * NT + s] = frag(wb + wrow0[s] * RB, kk);
#pragma unroll
            for (int t = 0; t < MT; ++t) fb[kk * MT + t] = frag(xb + (xrow0 + 16 * t) * RB, kk);
        }
    };
    read_frags(0, fa0, fb0);

    // one K stage; the fragments of stage t are in (fa, fb), stage t+1's are read into (na, nb)
    auto stage = [&](int t, FT (&fa)[NA], FT (&fb)[NB], FT (&na)[NA], FT (&nb)[NB]) {
        // part 1: DMA of stage t+ST-1 || MFMAs over W blocks [0, H1)
        if constexpr (!(ABL & 1)) issue(t + ST - 1);
        if constexpr (!(ABL & 4)) {
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
#pragma unroll
                for (int s = 0; s < H1; ++s)
#pragma unroll
                    for (int u = 0; u < MT; ++u) acc[s][u] = lg_mma(fa[kk * NT + s], fb[kk * MT + u], acc[s][u]);
        } else {
#pragma unroll
            for (int i = 0; i < NA; ++i) asm volatile("" ::"v"(fa[i]));
#pragma unroll
            for (int i = 0; i < NB; ++i) asm volatile("" ::"v"(fb[i]));
        }
#pragma unroll
        for (int i = 0; i < NPER; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                               // one DMA (VMEM read)
            __builtin_amdgcn_sched_group_barrier(0x008, MF1 / NPER > 0 ? MF1 / NPER : 1, 0);  // then its MFMA group
        }
        __builtin_amdgcn_sched_barrier(0);
        // this wave's DMA of stage t+1 landed; stages t+2 .. t+ST-1 stay in flight across the barrier
        if constexpr (ABL & 1) lg_vmcnt<0>();
        else lg_vmcnt<(ST - 2) * NPER>();
        lg_bar();
        // part 2: fragments of stage t+1 (past the end: stale LDS bytes nobody uses) || MFMAs over W blocks [H1, NT)
        if constexpr (!(ABL & 2)) read_frags(t + 1, na, nb);
        else {
#pragma unroll
            for (int i = 0; i < NA; ++i) na[i] = fa[i];
#pragma unroll
            for (int i = 0; i < NB; ++i) nb[i] = fb[i];
        }
        if constexpr (!(ABL & 4)) {
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
#pragma unroll
                for (int s = H1; s < NT; ++s)
#pragma unroll
                    for (int u = 0; u < MT; ++u) acc[s][u] = lg_mma(fa[kk * NT + s], fb[kk * MT + u], acc[s][u]);
        }
        {
            constexpr int NR = (NA + NB) * (F8 ? 2 : 1);  // ds_read_b128 per stage
            constexpr int G = MF2 / NR > 0 ? MF2 / NR : 1;
#pragma unroll
            for (int i = 0; i < NR; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one ds_read
                __builtin_amdgcn_sched_group_barrier(0x008, G, 0);  // then G MFMAs
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };

    for (int t = 0; t < NS; t += 2) {
        stage(t, fa0, fb0, fa1, fb1);
        if (t + 1 < NS) stage(t + 1, fa1, fb1, fa0, fb0);
    }
    }  // ring schedule
    lg_vmcnt<0>();  // the past-the-end DMAs must land before the workgroup's LDS is released

    if constexpr (HB && (HBV & 16)) {
        if (S > 1) {
            // ---- split-K for the staged HB configs (M <= 2048 shapes whose 256 x 256 tile grid under-fills the chip):
            // every slice stores its fp32 tile in register order (plain stores + agent release), the last arriver of
            // the ticket sums all slices' slabs in slice order (deterministic) into its accumulators, one W block at a
            // time (a compiler barrier per block keeps hipcc from hoisting all 64 slab loads at once), then runs the
            // staged epilogue below like an unsplit tile
            float* slab = a.ws + (int64_t)task * (WN * XM);
#pragma unroll
            for (int s = 0; s < NT; ++s)
#pragma unroll
                for (int u = 0; u < MT; ++u)
                    *reinterpret_cast<f32x4*>(slab + (((wave * NT + s) * MT + u) * 64 + lane) * 4) = acc[s][u];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            int* flag = reinterpret_cast<int*>(smem + EXTRA);
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int last = old == S - 1;
                if (last) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                *flag = last;
            }
            __syncthreads();
            if (!*flag) return;
            // per W block: the MT slab pieces of one slice are loaded together (one round trip per slice and block,
            // not per piece); the arriving slice's own piece comes from its registers (the same fp32 bits it stored),
            // so the sum is still slice 0 + 1 + ... in order whoever arrives last
#pragma unroll
            for (int s = 0; s < NT; ++s) {
                f32x4 t[MT], v[MT];
                for (int o = 0; o < S; ++o) {
                    if (o == ks) {
#pragma unroll
                        for (int u = 0; u < MT; ++u) v[u] = acc[s][u];
                    } else {
                        const float* sl = a.ws + (int64_t)(tile * S + o) * (WN * XM);
#pragma unroll
                        for (int u = 0; u < MT; ++u)
                            v[u] = *reinterpret_cast<const f32x4*>(sl + (((wave * NT + s) * MT + u) * 64 + lane) * 4);
                    }
#pragma unroll
                    for (int u = 0; u < MT; ++u) t[u] = o == 0 ? v[u] : t[u] + v[u];
                }
#pragma unroll
                for (int u = 0; u < MT; ++u) acc[s][u] = t[u];
                asm volatile("" ::: "memory");
            }
        }
        // ---- staged epilogue (HB bit 4): the wave's bf16 results go through its own 32 KiB of the (now free) LDS
        // ring, so every global store is a 16-B-per-lane piece of whole 128-B lines (32 dwordx4 stores per lane instead
        // of 64 dwordx2 ones covering 32-B segments); the residual form reads its residual the same way.  Register
        // phase: lane (row r = 16 u + lane % 16, columns 16 s + 4 (lane / 16) .. +3) writes 8 B into row r of the
        // image at 16-B chunk c ^ (r % chunks-per-row) (conflict-free ds_write_b64); store phase: 16 (8 SwiGLU) lanes
        // per row, one chunk each.
        constexpr int NCH0 = (MODE == kSwiglu ? WN / 4 : WN / 2) * 2 / 16, RPI0 = 64 / NCH0, NK = XM / 2 / RPI0;
        // kResid: the residual tile's loads go out first (16 B per lane, whole lines), so their latency hides behind
        // the staging; the store phase only waits for them
        u16x8 rvp[MODE == kResid ? NK : 1];
        if constexpr (MODE == kResid) {
            const int c = lane % NCH0;
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int m = min(m0 + xrow0 + RPI0 * k + lane / NCH0, M - 1);
                rvp[k] = *reinterpret_cast<const u16x8*>(a.resid + (int64_t)m * a.N + tn * WN + wi * (WN / 2) + c * 8);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        lg_bar();  // every wave's DMA landed and fragment reads done: the ring is free
        unsigned char* stg = smem + wave * 32768;
        const float* inv = reinterpret_cast<const float*>(smem + EXTRA + 16);
        constexpr int OC = MODE == kSwiglu ? WN / 4 : WN / 2;  // output columns per wave (64 / 128)
        constexpr int RBY = OC * 2, NCH = RBY / 16;             // image row bytes, 16-B chunks per row
        // 16x16 blocks: acc[s][u] covers row 16 u + lane % 16, columns 16 s + 4 (lane / 16) .. +3; L32 (F8HB):
        // acc[s][u] is 32x32 block (s / 2, u / 2), register group g = 2 (s & 1) + (u & 1): row 32 (u / 2) + lane % 32,
        // columns 32 (s / 2) + 8 g + 4 (lane / 32) .. +3 (within the wave's OC)
        static_assert(!F8 || L32, "fp8 HB: 32x32 blocks");
        auto row_of = [&](int u) { return L32 ? 32 * (u >> 1) + (lane & 31) : 16 * u + (lane & 15); };
        auto col_of = [&](int s, int u) {
            return L32 ? 32 * (s >> 1) + 8 * (2 * (s & 1) + (u & 1)) + 4 * (lane >> 5) : 16 * s + 4 * (lane >> 4);
        };
        // F8: every scale the register phase needs, loaded up front with clamped indices (no branches, one wait):
        // per-token xsc of the lane's rows, per-channel wsc of its column groups (SwiGLU: gate and up)
        constexpr int NSC = MODE == kSwiglu ? NT / 2 : NT;
        f32x4 c8a[F8 ? NSC : 1][2], c8b[F8 && MODE == kSwiglu ? NSC : 1][2];
        float xs8[F8 ? MT : 1];
        if constexpr (F8) {
#pragma unroll
            for (int s = 0; s < NSC; ++s)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    c8a[s][h] = *reinterpret_cast<const f32x4*>(scl + wi * OC + col_of(s, h));
                    if constexpr (MODE == kSwiglu)
                        c8b[s][h] = *reinterpret_cast<const f32x4*>(scl + WN / 2 + wi * OC + col_of(s, h));
                }
#pragma unroll
            for (int u = 0; u < MT; ++u) xs8[u] = scl[WN + xrow0 + row_of(u)];
        }
#pragma unroll
        for (int u = 0; u < MT; ++u) {
            const int r = row_of(u);
            float sc = 1.f;
            if constexpr (NORMP) sc = inv[xrow0 + r];
            if constexpr (F8) sc = xs8[u];  // per-token scale (rows past M: never stored)
#pragma unroll
            for (int s = 0; s < (MODE == kSwiglu ? NT / 2 : NT); ++s) {
                const int cl = col_of(s, u);  // first output column of the lane's 4
                u16x4 o;
                if constexpr (MODE == kSwiglu) {
                    f32x4 cg = {1.f, 1.f, 1.f, 1.f}, cu = {1.f, 1.f, 1.f, 1.f};
                    if constexpr (F8) {  // per-channel scales of the gate / up rows
                        cg = c8a[s][u & 1];
                        cu = c8b[s][u & 1];
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float gv = bf2f(f2bf(acc[s][u][i] * sc * cg[i]));
                        const float sg = bf2f(f2bf(gv / (1.f + __expf(-gv))));
                        o[i] = f2bf(sg * bf2f(f2bf(acc[s + NT / 2][u][i] * sc * cu[i])));
                    }
                } else {
                    f32x4 cw = {1.f, 1.f, 1.f, 1.f};
                    if constexpr (F8) cw = c8a[s][u & 1];
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[s][u][i] * sc * cw[i]);
                }
                *reinterpret_cast<u16x4*>(stg + r * RBY + (((cl >> 3) ^ (r % NCH)) << 4) + ((cl >> 2) & 1) * 8) = o;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // (own region: the wave reads back only what it wrote)
        constexpr int RPI_ = 64 / NCH;         // image rows per store instruction
        static_assert(RPI_ == RPI0 && NCH == NCH0, "staging geometry");
        const int c = lane % NCH;
        float ssr[MODE == kResid ? NK : 1];  // kResid: this lane's partial of row RPI_ k + lane / NCH
        // plain / SwiGLU: the image rows are read in batches of SB before their stores (pinned in registers), so
        // the LDS reads overlap instead of each guarded store waiting for its own read
        constexpr int SB = MODE == kResid ? 1 : 8;
        static_assert(NK % SB == 0, "store batches");
#pragma unroll
        for (int k0 = 0; k0 < NK; k0 += SB) {
            u16x8 vb[SB];
#pragma unroll
            for (int kk = 0; kk < SB; ++kk) {
                const int r = RPI_ * (k0 + kk) + lane / NCH;
                vb[kk] = *reinterpret_cast<const u16x8*>(stg + r * RBY + ((c ^ (r % NCH)) << 4));
            }
            if constexpr (SB > 1) {
#pragma unroll
                for (int kk = 0; kk < SB; ++kk) asm volatile("" : "+v"(vb[kk]));
            }
#pragma unroll
            for (int kk = 0; kk < SB; ++kk) {
                const int k = k0 + kk;
                const int r = RPI_ * k + lane / NCH;
                const int m = m0 + xrow0 + r;
                const u16x8 v = vb[kk];
                if constexpr (MODE == kSwiglu) {
                    if (m < M) *reinterpret_cast<u16x8*>(a.y + (int64_t)m * a.F + tn * (WN / 2) + wi * OC + c * 8) = v;
                } else if constexpr (MODE == kResid) {
                    const int n = tn * WN + wi * OC + c * 8;
                    float ss = 0.f;
                    const u16x8 rv = rvp[k];
                    u16x8 o;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const float y = bf2f(f2bf(bf2f(v[i]) + bf2f(rv[i])));
                        o[i] = f2bf(y);
                        ss += y * y;
                    }
                    if (m < M) *reinterpret_cast<u16x8*>(a.y + (int64_t)m * a.N + n) = o;
                    ssr[k] = ss;  // (the row's 16 lanes: summed below)
                } else {
                    const int n = tn * WN + wi * OC + c * 8;
                    if (m < M) {
                        if (n + 8 <= a.N) *reinterpret_cast<u16x8*>(a.y + (int64_t)m * a.N + n) = v;
                        else if (n < a.N) *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.N + n) = u16x4{v[0], v[1], v[2], v[3]};
                    }
                }
            }
        }
        if constexpr (MODE == kResid) {
            // the RMSNorm partial of each of the wave's 128 rows over its WN / 2 columns: the lanes' partials go to
            // the wave's image region (read out by now), [row][16], and lane l sums rows l and l + 64
            float* ssl = reinterpret_cast<float*>(stg);
#pragma unroll
            for (int k = 0; k < NK; ++k) ssl[(RPI_ * k + lane / NCH) * 16 + c] = ssr[k];
            __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int r = lane + 64 * h;
                const f32x4* q = reinterpret_cast<const f32x4*>(ssl + r * 16);
                const f32x4 t = (q[0] + q[1]) + (q[2] + q[3]);
                const float ss = (t[0] + t[1]) + (t[2] + t[3]);
                const int m = m0 + xrow0 + r;
                if (m < M) a.part_out[(int64_t)m * (a.N / (WN / 2)) + tn * 2 + wi] = ss;
            }
        }
        return;
    }

    // ---- split-K: fp32 slab in register order, ticket, the last arriver sums every slab in slice order
    if (!HB && S > 1) {  // (HB: no split-K; its fp32 slab code doubles the kernel's register pressure)
        // slab hand-off: plain stores + agent release / acquire fences (each a write-back / invalidate of the XCD's
        // L2), or write-through stores + agent-scope loads with no fence (gemm_skinny.hip's form).  Write-through
        // wins on the 8-16 KB slabs of the 32/64-row tiles (O M = 128 cfg39 split-K 2: 17.5 vs 20.1 us) and loses
        // from 32 KB up (256 KB: 15-20 % slower; profiles/r4_gemm_lg_handoff_small_ab.jsonl,
        // r4_gemm_lg_streamk_handoff_ab.jsonl).  a.handoff: knob lg_handoff (-1 auto, 0 fences, 1 write-through)
        const bool wt = a.handoff < 0 ? WN * XM * 4 <= 16384 : a.handoff != 0;
        float* slab = a.ws + (int64_t)task * (WN * XM);
#pragma unroll
        for (int s = 0; s < NT; ++s)
#pragma unroll
            for (int u = 0; u < MT; ++u) {
                float* p = slab + (((wave * NT + s) * MT + u) * 64 + lane) * 4;
                if (wt) st_wt(p, acc[s][u]);
                else *reinterpret_cast<f32x4*>(p) = acc[s][u];
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* flag = reinterpret_cast<int*>(smem + EXTRA);
        if (tid == 0) {
            if (!wt) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == S - 1;
            if (last) {
                if (!wt) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            *flag = last;
        }
        __syncthreads();
        if (!*flag) return;
        for (int o = 0; o < S; ++o) {
            const float* sl = a.ws + (int64_t)(tile * S + o) * (WN * XM);
#pragma unroll
            for (int s = 0; s < NT; ++s)
#pragma unroll
                for (int u = 0; u < MT; ++u) {
                    const float* p = sl + (((wave * NT + s) * MT + u) * 64 + lane) * 4;
                    const f32x4 v = wt ? ld_wt(p) : *reinterpret_cast<const f32x4*>(p);
                    acc[s][u] = o == 0 ? v : acc[s][u] + v;
                }
        }
    }

    // ---- epilogue: lane holds D[n = wrow0[s] + 4*(lane>>4) + i][m = xrow0 + 16*u + (lane&15)]
    const float* inv = reinterpret_cast<const float*>(smem + EXTRA + 16);
    if constexpr (M32) {
        // 32x32 layout: acc[s][2 U + gu] holds D[n = wrow32[s >> 1] + 8 g + 4 (lane >> 5) + i][m = xrow0 + 32 U +
        // (lane & 31)], g = 2 (s & 1) + gu — both gu share the lane's row m, and lanes l, l ^ 32 the row's columns
#pragma unroll
        for (int U = 0; U < MT / 2; ++U) {
            const int r = xrow0 + 32 * U + (lane & 31);
            const int m = m0 + r;
            float sc = 1.f;
            if constexpr (NORMP) sc = inv[r];
            float ss = 0.f;
#pragma unroll
            for (int gu = 0; gu < 2; ++gu) {
                const int u = 2 * U + gu;
                if constexpr (MODE == kSwiglu) {
                    if (m < M) {
#pragma unroll
                        for (int s = 0; s < NT / 2; ++s) {
                            const int g = 2 * (s & 1) + gu;
                            const int f = tn * (WN / 2) + wrow32[s >> 1] + 8 * g + 4 * (lane >> 5);
                            u16x4 o;
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const float gv = bf2f(f2bf(acc[s][u][i] * sc));
                                const float sg = bf2f(f2bf(gv / (1.f + __expf(-gv))));
                                o[i] = f2bf(sg * bf2f(f2bf(acc[s + NT / 2][u][i] * sc)));
                            }
                            *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.F + f) = o;
                        }
                    }
                } else if constexpr (MODE == kResid) {
                    if (m < M) {
#pragma unroll
                        for (int s = 0; s < NT; ++s) {
                            const int g = 2 * (s & 1) + gu;
                            const int n = tn * WN + wrow32[s >> 1] + 8 * g + 4 * (lane >> 5);
                            const u16x4 rv = *reinterpret_cast<const u16x4*>(a.resid + (int64_t)m * a.N + n);
                            u16x4 o;
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const float v = bf2f(f2bf(bf2f(f2bf(acc[s][u][i])) + bf2f(rv[i])));
                                o[i] = f2bf(v);
                                ss += v * v;
                            }
                            *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.N + n) = o;
                        }
                    }
                } else {
                    if (m < M) {
#pragma unroll
                        for (int s = 0; s < NT; ++s) {
                            const int g = 2 * (s & 1) + gu;
                            const int n = tn * WN + wrow32[s >> 1] + 8 * g + 4 * (lane >> 5);
                            u16x4 o;
#pragma unroll
                            for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[s][u][i] * sc);
                            if (n < a.N) *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.N + n) = o;
                        }
                    }
                }
            }
            if constexpr (MODE == kResid) {
                ss += __shfl_xor(ss, 32, 64);
                if (lane < 32 && m < M) a.part_out[(int64_t)m * (a.N / (WN / 2)) + tn * 2 + wi] = ss;
            }
        }
        return;
    }
#pragma unroll
    for (int u = 0; u < MT; ++u) {
        const int r = xrow0 + 16 * u + (lane & 15);
        const int m = m0 + r;
        float sc = 1.f;
        if constexpr (NORMP) sc = inv[r];
        if constexpr (F8) sc = m < M ? a.xsc[m] : 0.f;  // per-token scale; the per-channel one below
        if constexpr (MODE == kSwiglu) {
            if (m < M) {
#pragma unroll
                for (int s = 0; s < NT / 2; ++s) {
                    const int f = tn * (WN / 2) + wrow0[s] + 4 * (lane >> 4);
                    f32x4 cg = {1.f, 1.f, 1.f, 1.f}, cu = {1.f, 1.f, 1.f, 1.f};
                    if constexpr (F8) {
                        cg = *reinterpret_cast<const f32x4*>(a.wsc + f);
                        cu = *reinterpret_cast<const f32x4*>(a.wsc + a.F + f);
                    }
                    u16x4 o;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float gv = bf2f(f2bf(acc[s][u][i] * sc * cg[i]));
                        const float sg = bf2f(f2bf(gv / (1.f + __expf(-gv))));
                        o[i] = f2bf(sg * bf2f(f2bf(acc[s + NT / 2][u][i] * sc * cu[i])));
                    }
                    *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.F + f) = o;
                }
            }
        } else if constexpr (MODE == kResid) {
            float ss = 0.f;
            if (m < M) {
#pragma unroll
                for (int s = 0; s < NT; ++s) {
                    const int n = tn * WN + wrow0[s] + 4 * (lane >> 4);
                    const u16x4 rv = *reinterpret_cast<const u16x4*>(a.resid + (int64_t)m * a.N + n);
                    u16x4 o;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float v = bf2f(f2bf(bf2f(f2bf(acc[s][u][i])) + bf2f(rv[i])));
                        o[i] = f2bf(v);
                        ss += v * v;
                    }
                    *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.N + n) = o;
                }
            }
            // the 4 lanes of a row (lane ^ 16, ^ 32) hold disjoint columns of the wave's WN/2
            ss += __shfl_xor(ss, 16, 64);
            ss += __shfl_xor(ss, 32, 64);
            if (lane < 16 && m < M) a.part_out[(int64_t)m * (a.N / (WN / 2)) + tn * 2 + wi] = ss;
        } else {
            if (m < M) {
#pragma unroll
                for (int s = 0; s < NT; ++s) {
                    const int n = tn * WN + wrow0[s] + 4 * (lane >> 4);
                    f32x4 cw = {1.f, 1.f, 1.f, 1.f};
                    if constexpr (F8)
                        if (n < a.N) cw = *reinterpret_cast<const f32x4*>(a.wsc + n);
                    u16x4 o;
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[s][u][i] * sc * cw[i]);
                    if (n < a.N) *reinterpret_cast<u16x4*>(a.y + (int64_t)m * a.N + n) = o;  // N % 4 == 0
                }
            }
        }
    }
}

template <int WN, int XM, int RB, int ST, int MODE, bool NORMP, int NWX, int ABL = 0, int VAR = 0, bool F8 = false>
void lg_launch(const PPArgs& a, hipStream_t st) {
    const int lds = ST * (WN + XM) * RB + 16 + XM * 4 + (F8 && ST == 2 ? (WN + XM) * 4 : 0);
    auto kern = gemm_lg_kernel<WN, XM, RB, ST, MODE, NORMP, NWX, ABL, VAR, F8>;
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    const int mt = (a.M + XM - 1) / XM;
    const int ntl = MODE == kSwiglu ? a.F / (WN / 2) : (a.N + WN - 1) / WN;
    hipLaunchKernelGGL(kern, dim3(mt * ntl * a.splitk), dim3(128 * NWX), lds, st, a);
}

// tile configs (ids continue gemm_pp's): {WN = W rows, XM = x rows, RB = LDS row bytes (BK = RB/2), ST = ring depth,
// NWX = waves along x (2: one wave per SIMD; 4: two)}.  72-75 (ids after the ablation range): 32 x rows for
// M <= 32 (jump-forward forwards, drained buckets).  32-39: mid-M (64-256 rows) weight streaming — 64 W rows per
// workgroup so the tile grid x split-K covers the chip with few slices, the whole x panel shared by the W-row waves
// through LDS (x bytes <= 2-4x the weight bytes per workgroup, L2-resident), a 4-6 stage ring for the HBM latency
#define LG_CONFIGS(X)              \
    X(12, 256, 256, 64, 4, 2)      \
    X(13, 256, 128, 64, 6, 2)      \
    X(14, 128, 256, 64, 6, 2)      \
    X(15, 128, 128, 128, 4, 2)     \
    X(16, 256, 256, 64, 4, 4)      \
    X(17, 256, 128, 64, 6, 4)      \
    X(18, 128, 256, 64, 6, 4)      \
    X(19, 128, 128, 128, 4, 4)     \
    X(20, 256, 256, 128, 2, 4)     \
    X(21, 256, 256, 128, 2, 2)     \
    X(22, 256, 128, 128, 2, 4)     \
    X(23, 128, 128, 128, 2, 2)     \
    X(24, 256, 256, 128, 2, 4, 1)  \
    X(25, 256, 128, 128, 2, 4, 1)  \
    X(26, 256, 256, 128, 2, 4, 2)  \
    X(27, 256, 128, 128, 2, 4, 2)  \
    X(28, 128, 128, 128, 2, 2, 2)  \
    X(29, 256, 128, 128, 3, 4)     \
    X(30, 128, 256, 128, 3, 4)     \
    X(31, 128, 128, 128, 3, 2)     \
    X(32, 64, 128, 128, 4, 2)      \
    X(33, 64, 64, 128, 4, 2)       \
    X(34, 64, 128, 128, 6, 2)      \
    X(35, 64, 256, 128, 3, 4)      \
    X(36, 64, 64, 128, 8, 2)       \
    X(37, 64, 128, 128, 5, 2)      \
    X(38, 128, 64, 128, 6, 2)      \
    X(39, 64, 64, 128, 6, 2)       \
    X(72, 64, 32, 128, 8, 2)       \
    X(73, 128, 32, 128, 6, 2)      \
    X(74, 64, 32, 128, 4, 2)       \
    X(75, 128, 32, 128, 4, 2)      \
    X(76, 192, 128, 128, 3, 4)     \
    X(77, 192, 128, 128, 3, 2)     \
    X(78, 128, 32, 128, 7, 2)      \
    X(79, 64, 32, 128, 12, 2)      \
    X(80, 256, 256, 128, 2, 4, 3)  \
    X(81, 256, 256, 128, 2, 2, 4)  \
    X(82, 256, 256, 128, 2, 2, 5)  \
    X(83, 256, 256, 128, 2, 2, 6)  \
    X(84, 256, 256, 128, 2, 2, 8)  \
    X(85, 256, 256, 128, 2, 2, 7)  \
    X(86, 256, 256, 128, 2, 2, 13) \
    X(87, 256, 256, 128, 2, 2, 15) \
    X(88, 256, 256, 128, 2, 2, 29) \
    X(89, 256, 256, 128, 2, 2, 31) \
    X(90, 256, 256, 128, 2, 2, 60) \
    X(91, 256, 256, 128, 2, 2, 93) \
    X(92, 256, 256, 128, 2, 2, 157) \
    X(93, 256, 256, 128, 2, 2, 159) \
    X(94, 256, 256, 128, 2, 2, 189)

template <int MODE, bool NORMP>
bool lg_mode(int cfg, const PPArgs& a, hipStream_t st) {
    switch (cfg) {
#define LG_CASE(ID, WN_, XM_, RB_, ST_, NWX_, ...) \
    case ID: lg_launch<WN_, XM_, RB_, ST_, MODE, NORMP, NWX_, 0, ##__VA_ARGS__>(a, st); return true;
        LG_CONFIGS(LG_CASE)
#undef LG_CASE
        default: break;
    }
    // timing-only ablations of configs 12 / 16 (plain mode): 40 + 8 * (cfg == 16) + ABL.  Several return wrong results
    // by design, so they exist only in a diagnostics build (CHRONOS_GEMM_ABLATIONS=1 at build time, native.py)
#ifdef CHRONOS_GEMM_ABLATIONS
    if constexpr (MODE == kPlain && !NORMP) {
        switch (cfg) {
            case 41: lg_launch<256, 256, 64, 4, MODE, NORMP, 2, 1>(a, st); return true;
            case 42: lg_launch<256, 256, 64, 4, MODE, NORMP, 2, 2>(a, st); return true;
            case 43: lg_launch<256, 256, 64, 4, MODE, NORMP, 2, 3>(a, st); return true;
            case 44: lg_launch<256, 256, 64, 4, MODE, NORMP, 2, 4>(a, st); return true;
            case 49: lg_launch<256, 256, 64, 4, MODE, NORMP, 4, 1>(a, st); return true;
            case 50: lg_launch<256, 256, 64, 4, MODE, NORMP, 4, 2>(a, st); return true;
            case 51: lg_launch<256, 256, 64, 4, MODE, NORMP, 4, 3>(a, st); return true;
            case 52: lg_launch<256, 256, 64, 4, MODE, NORMP, 4, 4>(a, st); return true;
            case 53: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 1>(a, st); return true;
            case 54: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 3>(a, st); return true;
            case 55: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 4>(a, st); return true;
            case 56: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 6>(a, st); return true;
            case 57: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 8>(a, st); return true;
            case 58: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 14>(a, st); return true;
            case 59: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 12>(a, st); return true;
            case 60: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 2>(a, st); return true;
            case 61: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 4, 1>(a, st); return true;
            case 62: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 4, 2>(a, st); return true;
            case 63: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 2, 2>(a, st); return true;
            case 64: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 16>(a, st); return true;
            case 65: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 48>(a, st); return true;
            case 66: lg_launch<256, 256, 128, 2, MODE, NORMP, 4, 48 | 2>(a, st); return true;
            default: break;
        }
    }
#endif
    return false;
}

}  // namespace

bool gemm_lg_ablations_built() {
#ifdef CHRONOS_GEMM_ABLATIONS
    return true;
#else
    return false;
#endif
}

int gemm_lg_xm(int cfg) {
    if (gemm_lg_ablations_built() && cfg >= 40 && cfg < 72) return 256;  // ablation ids
    switch (cfg) {
#define LG_XM(ID, WN_, XM_, RB_, ST_, NWX_, ...) case ID: return XM_;
        LG_CONFIGS(LG_XM)
#undef LG_XM
        default: return 0;
    }
}
bool gemm_lg_splitk_ok(int cfg) { return cfg < 81 || cfg > 94 || cfg >= 88; }

int gemm_lg_wn(int cfg) {
    if (gemm_lg_ablations_built() && cfg >= 40 && cfg < 72) return 256;
    switch (cfg) {
#define LG_WN(ID, WN_, XM_, RB_, ST_, NWX_, ...) case ID: return WN_;
        LG_CONFIGS(LG_WN)
#undef LG_WN
        default: return 0;
    }
}

// W8A8 fp8 configs {id, WN, XM, RB, ST, NWX}: ring schedule, one 128-deep v_mfma_scale_f32_16x16x128_f8f6f4 k-step
// per 128-B stage row (every staged byte carries twice the bf16 kernel's K)
// 4 (F8HB): the HB slab loop (4 waves, 128 x 128 outputs per wave, three barriers per slab) on
// v_mfma_scale_f32_32x32x64_f8f6f4, precomputed addressing + LDS-staged epilogue (VAR 29 = bf16 cfg 88's bits)
#define LG_F8_CONFIGS(X)       \
    X(0, 256, 128, 128, 3, 4)  \
    X(1, 128, 256, 128, 3, 4)  \
    X(2, 128, 128, 128, 4, 2)  \
    X(3, 128, 128, 128, 3, 4)  \
    X(4, 256, 256, 128, 2, 2, 29)

namespace {
constexpr int lg_f8_var(int v = 0) { return v; }  // (the config's VAR, 0 when the row gives none)
template <int MODE>
bool lg_f8_mode(int cfg, const PPArgs& a, hipStream_t st) {
    switch (cfg) {
#define LG_F8_CASE(ID, WN_, XM_, RB_, ST_, NWX_, ...) \
    case ID: lg_launch<WN_, XM_, RB_, ST_, MODE, false, NWX_, 0, lg_f8_var(__VA_ARGS__), true>(a, st); return true;
        LG_F8_CONFIGS(LG_F8_CASE)
#undef LG_F8_CASE
        default: return false;
    }
}
}  // namespace

int gemm_lg_f8_xm(int cfg) {
    switch (cfg) {
#define LG_F8_XM(ID, WN_, XM_, RB_, ST_, NWX_, ...) case ID: return XM_;
        LG_F8_CONFIGS(LG_F8_XM)
#undef LG_F8_XM
        default: return 0;
    }
}
int gemm_lg_f8_wn(int cfg) {
    switch (cfg) {
#define LG_F8_WN(ID, WN_, XM_, RB_, ST_, NWX_, ...) case ID: return WN_;
        LG_F8_CONFIGS(LG_F8_WN)
#undef LG_F8_WN
        default: return 0;
    }
}

bool launch_gemm_lg_f8(int cfg, bool swiglu, const PPArgs& a, hipStream_t st) {
    if (a.M == 0) return true;
    return swiglu ? lg_f8_mode<kSwiglu>(cfg, a, st) : lg_f8_mode<kPlain>(cfg, a, st);
}

bool launch_gemm_lg(int cfg, int mode, bool normp, const PPArgs& a, hipStream_t st) {
    if (a.M == 0) return true;
    if (mode == kResid) return normp ? false : lg_mode<kResid, false>(cfg, a, st);
    if (mode == kSwiglu) return normp ? lg_mode<kSwiglu, true>(cfg, a, st) : lg_mode<kSwiglu, false>(cfg, a, st);
    return normp ? lg_mode<kPlain, true>(cfg, a, st) : lg_mode<kPlain, false>(cfg, a, st);
}

}  // namespace chronos
