// gemm.hip — projection GEMM for the decode / mid-size regime: y[M, N] = x[M, K] · W[N, K]^T (bf16 in, fp32
// accumulate, bf16 out), with an optional fused SwiGLU epilogue for the gate_up projection (K3/K7/K8/K10/K11,
// SURVEY.md §2.3).
//
// Why a hand-written kernel: at decode batch sizes (M = 64..1024 rows) the library's tile choices leave most of the
// 256 CUs idle on the N = 4096 / 6144 projections (64-96 tiles of 256x256, profiles/r1_*): hipBLASLt reaches
// 0.84-1.0 PFLOP/s there.  This kernel is built for one 128x128 tile per CU-slot:
//
//   * tile 128 (W rows = output cols) x 128 (x rows), BK = 64; 4 waves as 2 x 2, each wave 64 x 64 =
//     4 x 4 v_mfma_f32_16x16x32_bf16 tiles (64 accumulator VGPRs);
//   * swapped product D = W · x^T: the W tile is the MFMA A operand and x the B operand, so a lane's 4 accumulator
//     registers are 4 CONSECUTIVE output columns of one row -> 8-byte stores, and the SwiGLU pair (gate col f, up col
//     F+f) of a row sits in the same lane;
//   * operands reach LDS by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave-instruction, no VGPR staging) into a
//     STAGES-deep ring of [128 rows][64 k] images; the XOR-8 chunk swizzle is applied on the per-lane GLOBAL source
//     address (LDS stays lane-linear, cdna_hip_programming.md §5.4 rule 21) and undone on the ds_read_b128 fragment
//     read, which makes the 16x16x32 fragment reads bank-conflict-free (all 16 lanes of each ds_read_b128 lane group
//     land on distinct 16-B slots);
//   * one raw s_barrier per K-step, preceded by a COUNTED s_waitcnt vmcnt that retires only the oldest stage (the
//     next STAGES-2 stay in flight across the barrier) — __syncthreads() would emit vmcnt(0) and drain the ring
//     (cdna_hip_programming.md §5 "Pipelining across barriers");
//   * XCD-aware tile order: the 8 XCDs each get a contiguous run of tiles, ordered N-major, so the x rows a W tile
//     meets are re-read from that XCD's L2 and each W tile is fetched by one XCD.
// M is arbitrary (rows >= M are clamped on load and never stored); N % 128 == 0 (SwiGLU: F % 64 == 0); K % 64 == 0.
#include "chronos_hip.h"

namespace chronos {
namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int BM = 128;  // x rows per tile
constexpr int BN = 128;  // W rows per tile
constexpr int BK = 64;
constexpr int kTileBytes = 128 * BK * 2;  // one operand image: 16 KiB

// s_waitcnt with only vmcnt restricted (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ bf16x8 lds_frag(const unsigned char* img, int row, int chunk) {
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + ((chunk ^ (row & 7)) << 4));
}

template <int STAGES, bool SWIGLU>
__global__ void __launch_bounds__(256) gemm_bf16_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                        uint16_t* __restrict__ y, int M, int N, int K, int F,
                                                        const int32_t* __restrict__ gst, int gn) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];  // STAGES x {W image, x image}
    if (gate_closed(gst, gn)) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int mt = (M + BM - 1) / BM;
    const int nt = (SWIGLU ? F / 64 : N / BN);
    const int tile = xcd_remap(blockIdx.x, mt * nt);
    const int tn = tile / mt, tm = tile - tn * mt;
    const int m0 = tm * BM;

    // ---- per-lane LDS-DMA sources.  Wave `wave` fills rows [32*wave, 32*wave+32) of each image with 4
    // instructions of 8 rows x 128 B; lane l covers row r = 32*wave + 8*i + (l>>3), 16-B chunk (l&7), fetched from
    // global chunk (l&7) ^ (r&7).
    const uint16_t* wsrc[4];
    const uint16_t* xsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = 32 * wave + 8 * i + (lane >> 3);
        const int c = (lane & 7) ^ (r & 7);
        int wrow;
        if constexpr (SWIGLU) wrow = r < 64 ? tn * 64 + r : F + tn * 64 + (r - 64);  // gate rows | matching up rows
        else wrow = tn * BN + r;
        wsrc[i] = w + (int64_t)wrow * K + c * 8;
        const int xr = min(m0 + r, M - 1);
        xsrc[i] = x + (int64_t)xr * K + c * 8;
    }
    auto issue = [&](int kt) {
        unsigned char* st = smem + (kt % STAGES) * 2 * kTileBytes;
        const int koff = kt * BK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(wsrc[i] + koff), (lds_ptr_t)(st + (4 * wave + i) * 1024), 16,
                                             0, 0);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(xsrc[i] + koff),
                                             (lds_ptr_t)(st + kTileBytes + (4 * wave + i) * 1024), 16, 0, 0);
        }
    };

    // ---- wave tile: W rows (MFMA rows) and x rows (MFMA cols)
    const int wn = wave >> 1, wm = wave & 1;
    int wrow0[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        if constexpr (SWIGLU) wrow0[s] = (s < 2 ? 32 * wn + 16 * s : 64 + 32 * wn + 16 * (s - 2));
        else wrow0[s] = 64 * wn + 16 * s;
    }
    f32x4 acc[4][4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[s][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int KT = K / BK;
#pragma unroll
    for (int p = 0; p < STAGES - 1; ++p)
        if (p < KT) issue(p);

    for (int kt = 0; kt < KT; ++kt) {
        // retire stage kt (this wave's 8 DMAs of it); leave the younger stages in flight across the barrier
        if (kt + STAGES - 2 < KT) wait_vmcnt<8 * (STAGES - 2)>();
        else wait_vmcnt<0>();
        asm volatile("" ::: "memory");  // keep the fragment reads below the barrier (it is IntrNoMem to LLVM)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + STAGES - 1 < KT) issue(kt + STAGES - 1);  // into the stage every wave finished reading at kt-1
        const unsigned char* wimg = smem + (kt % STAGES) * 2 * kTileBytes;
        const unsigned char* ximg = wimg + kTileBytes;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int chunk = h * 4 + (lane >> 4);
            bf16x8 a[4], b[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) a[s] = lds_frag(wimg, wrow0[s] + (lane & 15), chunk);
#pragma unroll
            for (int t = 0; t < 4; ++t) b[t] = lds_frag(ximg, 64 * wm + 16 * t + (lane & 15), chunk);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], b[t], acc[s][t],
                                                                                                0, 0, 0);
        }
    }

    // ---- epilogue: lane holds D[n = 4*(lane>>4) + i][m = lane&15] of each 16x16 tile = y[m][n..n+3]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int m = m0 + 64 * wm + 16 * t + (lane & 15);
        if (m >= M) continue;
        if constexpr (SWIGLU) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                u16x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float g = bf2f(f2bf(acc[s][t][i]));
                    const float sg = bf2f(f2bf(g / (1.f + __expf(-g))));
                    o[i] = f2bf(sg * bf2f(f2bf(acc[s + 2][t][i])));
                }
                const int f = tn * 64 + 32 * wn + 16 * s + 4 * (lane >> 4);
                *reinterpret_cast<u16x4*>(y + (int64_t)m * F + f) = o;
            }
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                u16x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[s][t][i]);
                const int n = tn * BN + wrow0[s] + 4 * (lane >> 4);
                *reinterpret_cast<u16x4*>(y + (int64_t)m * N + n) = o;
            }
        }
    }
}

template <int STAGES, bool SWIGLU>
void launch_stages(const uint16_t* x, const uint16_t* w, uint16_t* y, int M, int N, int K, int F, hipStream_t st) {
    const int mt = (M + BM - 1) / BM;
    const int nt = SWIGLU ? F / 64 : N / BN;
    const int lds = STAGES * 2 * kTileBytes;
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_bf16_kernel<STAGES, SWIGLU>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    hipLaunchKernelGGL((gemm_bf16_kernel<STAGES, SWIGLU>), dim3(mt * nt), dim3(256), lds, st, x, w, y, M, N, K, F,
                       CHRONOS_GATE);
}

}  // namespace

// swiglu: w is [2F, K] (gate rows then up rows), y is [M, F] = silu(x W_g^T) * (x W_u^T)
void launch_gemm(const uint16_t* x, const uint16_t* w, uint16_t* y, int M, int N, int K, bool swiglu, int stages,
                 hipStream_t st) {
    if (M == 0) return;
    const int F = N / 2;
    if (stages == 3) {
        if (swiglu) launch_stages<3, true>(x, w, y, M, N, K, F, st);
        else launch_stages<3, false>(x, w, y, M, N, K, F, st);
    } else if (stages == 2) {
        if (swiglu) launch_stages<2, true>(x, w, y, M, N, K, F, st);
        else launch_stages<2, false>(x, w, y, M, N, K, F, st);
    } else {
        if (swiglu) launch_stages<4, true>(x, w, y, M, N, K, F, st);
        else launch_stages<4, false>(x, w, y, M, N, K, F, st);
    }
}

}  // namespace chronos
