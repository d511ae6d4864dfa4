// chronos_gemm.h — host/device interface of the batched projection GEMM family (csrc/kernels/gemm_pp.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace chronos {

struct PPArgs {
    const uint16_t* x;
    const uint16_t* w;
    uint16_t* y;            // output (kResid: the new residual stream s)
    const uint16_t* resid;  // kResid input residual
    float* part_out;        // kResid: [M, N / (BN/4)] partial sums of s^2
    const float* part_in;   // NORMP: [M, nparts_in] producer partials
    float* ws;              // split-K fp32 slabs, [tiles * splitk, BM * BN]
    int32_t* cnt;           // split-K tickets, one per tile (zero between calls: the last arriver resets its own)
    int M, N, K, F, nparts_in, splitk, kts;
    float eps;
    int gm;      // tile order: M-tiles per group (0 = every M-tile of a W panel consecutive); knob pp_gm
    int handoff;       // gemm_lg split-K slab hand-off (knob lg_handoff): -1 auto, 0 fences, 1 write-through
    const float* xsc;  // gemm_lg F8 (W8A8 e4m3fn bytes in x / w): per-token scales [M]
    const float* wsc;  // ... and per-output-channel scales [N]
    int ablate;  // timing-only diagnostics (knob pp_ablate): 1 skip loop DMA, 2 skip LDS reads, 4 skip MFMA, 8 nt weights, 16/32 alias every W/x tile onto tile 0
};

// epilogue modes
enum : int { kPPPlain = 0, kPPSwiglu = 1, kPPResid = 2 };
constexpr int kPPConfigs = 12;
int gemm_pp_bm(int cfg);  // x rows per tile
int gemm_pp_bn(int cfg);  // W rows per tile
bool launch_gemm_pp(int cfg, int mode, bool normp, bool prio, const PPArgs& a, hipStream_t st);

// large-M family (csrc/kernels/gemm_lg.hip): config ids kPPConfigs .. kPPConfigs + kLGConfigs - 1 of the same PPArgs
// interface; tile = WN W rows x XM x rows, 4 or 8 waves (2 x NWX), kResid partials are [M, N / (WN / 2)]
constexpr int kLGConfigs = 28;
// gemm_lg 72-75 (32-row x tiles, after the 40-71 timing-ablation ids), 76-77 (192 W x 128 x rows: 256 tiles at
// N = 6144, M = 1024 — one round on 256 CUs) and 78-79 (32-row x tiles with 7 / 12-stage rings: mid-M weight streams
// are bound by the W bytes in flight per CU, so nearly all of the 160 KiB LDS holds W stages) and 80 (cfg 20's slab
// schedule on 32x32x16 MFMAs) and 81-90 (4 waves, 128 x 128 per wave, the three-barrier slab loop: VAR 4-60 in gemm_lg.hip)
constexpr int kLGTinyFirst = 72, kLGTinyConfigs = 23;
int gemm_lg_xm(int cfg);  // x rows per tile
int gemm_lg_wn(int cfg);  // W rows per tile
bool gemm_lg_splitk_ok(int cfg);  // false for the HB configs (VAR 4): no split-K path
bool gemm_lg_ablations_built();  // the timing-only ablation ids 40-71 exist (CHRONOS_GEMM_ABLATIONS build)
bool launch_gemm_lg(int cfg, int mode, bool normp, const PPArgs& a, hipStream_t st);
// W8A8 fp8 configs of the same kernel (ring schedule, 128-deep stages; a.kts counts 128-deep units), own id space
constexpr int kLGF8Configs = 5;
int gemm_lg_f8_xm(int cfg);
int gemm_lg_f8_wn(int cfg);
bool launch_gemm_lg_f8(int cfg, bool swiglu, const PPArgs& a, hipStream_t st);

// skinny-M family (csrc/kernels/gemm_skinny.hip, M <= 16 * MT): same PPArgs / epilogues; the workgroup owns 16 * RT
// W rows (swiglu: 8 * RT gate + 8 * RT up), ws holds [groups * splitk, 64 * RT * MT] f32x4 slabs, cnt one ticket per
// group, kResid partials are [M, N / (16 * RT)]; K % (64 * NW * splitk) == 0
constexpr int kSkinnyConfigs = 12;
int gemm_skinny_rt(int cfg);
int gemm_skinny_mt(int cfg);
int gemm_skinny_nw(int cfg);  // waves per workgroup
bool launch_gemm_skinny(int cfg, int mode, bool normp, const PPArgs& a, hipStream_t st);

}  // namespace chronos
