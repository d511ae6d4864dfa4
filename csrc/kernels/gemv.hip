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

namespace chronos {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

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

template <int M, int R, bool SWIGLU>
__global__ void __launch_bounds__(256) gemv_kernel(const uint16_t* __restrict__ x, int mrows, int K,
                                                   const uint16_t* __restrict__ W, uint16_t* __restrict__ y,
                                                   int nout, int half) {
    constexpr int NR = SWIGLU ? 2 * R : R;  // weight rows streamed by this workgroup
    constexpr int V = NR * M;               // partial sums per lane
    constexpr int DEPTH = (NR + M) * 4 <= 40 ? 3 : 2;  // register ring depth (VGPR budget)
    __shared__ float red[4][V];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n0 = blockIdx.x * R;
    const int nchunk = K >> 9;  // 512-element (1 KiB) chunks per row
    // row bases are wave-uniform (SGPR pairs); the per-lane part is one 32-bit offset (lane + 64 * chunk) * 16 B
    const u16x8* wrow[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int row = (SWIGLU && r >= R) ? half + n0 + (r - R) : n0 + r;
        wrow[r] = reinterpret_cast<const u16x8*>(W + (int64_t)row * K);
    }
    const u16x8* xr = reinterpret_cast<const u16x8*>(x);
    const int xstride = K >> 3;

    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    u16x8 wr[DEPTH][NR], xv[DEPTH][M];
    auto load = [&](int c, u16x8 (&wd)[NR], u16x8 (&xd)[M]) {
        const int off = c * 64 + lane;
#pragma unroll
        for (int r = 0; r < NR; ++r) wd[r] = ld_nt(wrow[r] + off);
#pragma unroll
        for (int m = 0; m < M; ++m) xd[m] = m < mrows ? xr[m * xstride + off] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    };
    // wave w takes chunks w, w+4, w+8, ...
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
        if (w + 4 * d < nchunk) load(w + 4 * d, wr[d], xv[d]);
    for (int c0 = w; c0 < nchunk; c0 += 4 * DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int c = c0 + 4 * d;
            if (c < nchunk) {
#pragma unroll
                for (int r = 0; r < NR; ++r)
#pragma unroll
                    for (int m = 0; m < M; ++m) acc[r * M + m] = dot8(wr[d][r], xv[d][m], acc[r * M + m]);
                if (c + 4 * DEPTH < nchunk) load(c + 4 * DEPTH, wr[d], xv[d]);
            }
        }
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
        const float g = red[0][r * M + m] + red[1][r * M + m] + red[2][r * M + m] + red[3][r * M + m];
        if constexpr (SWIGLU) {
            const int ru = (R + r) * M + m;
            const float u = red[0][ru] + red[1][ru] + red[2][ru] + red[3][ru];
            const float gb = bf2f(f2bf(g)), ub = bf2f(f2bf(u));  // the unfused path rounds the GEMM outputs
            const float sg = bf2f(f2bf(gb / (1.f + __expf(-gb))));
            y[(int64_t)m * nout + n0 + r] = f2bf(sg * ub);
        } else {
            y[(int64_t)m * nout + n0 + r] = f2bf(g);
        }
    }
}

template <int M>
static void launch_m(const uint16_t* x, int mrows, int K, const uint16_t* W, int N, uint16_t* y, bool swiglu,
                     hipStream_t st) {
    // R rows per workgroup: as many as the in-wave reduce-scatter (<= 64 sums per lane) allows, so x (re-read from L2
    // per chunk) stays a small fraction of the weight bytes.
    constexpr int R1 = M <= 2 ? 8 : 4;
    constexpr int R2 = M <= 2 ? 4 : 2;
    if (swiglu) {
        const int F = N / 2;
        hipLaunchKernelGGL((gemv_kernel<M, R2, true>), dim3(F / R2), dim3(256), 0, st, x, mrows, K, W, y, F, F);
    } else {
        hipLaunchKernelGGL((gemv_kernel<M, R1, false>), dim3(N / R1), dim3(256), 0, st, x, mrows, K, W, y, N, 0);
    }
}

void launch_gemv(const uint16_t* x, int M, int K, const uint16_t* W, int N, uint16_t* y, bool swiglu,
                 hipStream_t st) {
    if (M <= 0) return;
    if (M == 1) launch_m<1>(x, M, K, W, N, y, swiglu, st);
    else if (M == 2) launch_m<2>(x, M, K, W, N, y, swiglu, st);
    else if (M <= 4) launch_m<4>(x, M, K, W, N, y, swiglu, st);
    else launch_m<8>(x, M, K, W, N, y, swiglu, st);
}

}  // namespace chronos
