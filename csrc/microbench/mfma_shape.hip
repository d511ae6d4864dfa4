// mfma_shape.hip — sustained bf16 MFMA rate of v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 (VERDICT r4
// suggested moving gemm_lg to the 32x32 form: half the MFMA issues for the same work).  Every wave keeps 8 (16x16) or
// 2 (32x32) independent accumulator chains busy on operands loaded from a random buffer (the chip's clock under load
// depends on the data: cdna_hip_programming.md "DVFS give-back"), 8 waves per CU on every CU, and the same FLOPs per
// wave for both shapes; reports TFLOP/s.  Also a zero-filled run of each.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_shape mfma_shape.hip && ./mfma_shape
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// 16x16x32: 16*16*32*2 = 16384 FLOP per MFMA; 32x32x16: 32768 FLOP per MFMA
template <bool BIG>
__global__ void __launch_bounds__(512) mfma_loop(const bf16x8* __restrict__ src, float* out, int iters) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    bf16x8 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = src[(tid * 8 + i) & 0xFFFF];
        b[i] = src[(tid * 8 + 4 + i) & 0xFFFF];
    }
    float s = 0.f;
    if constexpr (!BIG) {
        f32x4 c[8] = {};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j & 3], b[(j >> 1) & 3], c[j], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += c[j][0] + c[j][3];
    } else {
        f32x16 c[4] = {};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[j], b[3 - j], c[j], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) s += c[j][0] + c[j][15];
    }
    if (s == 1.2345f) out[tid] = s;  // keeps the chains live
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int n = 1 << 16;
    std::vector<unsigned short> h(n * 8);
    unsigned x = 12345u;
    for (auto& v : h) {  // random bf16 in about +-[0.5, 2): full mantissa, both signs
        x = x * 1664525u + 1013904223u;
        v = (unsigned short)(0x3f00 | (x >> 25) | ((x >> 9) & 0x8000)) ^ (unsigned short)((x >> 16) & 0x7f);
    }
    bf16x8 *rnd, *zero;
    float* out;
    hipMalloc(&rnd, n * 16);
    hipMalloc(&zero, n * 16);
    hipMalloc(&out, cus * 512 * 4 * 4);
    hipMemcpy(rnd, h.data(), n * 16, hipMemcpyHostToDevice);
    hipMemset(zero, 0, n * 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = cus * 2;  // 2 x 512 threads = 16 waves per CU (4 per SIMD)
    const int it16 = 20000, it32 = 20000;  // 8 x 16384 vs 4 x 32768 FLOP per iteration: equal work
    for (int rep = 0; rep < 2; ++rep) {
        for (int big = 0; big < 2; ++big) {
            for (int z = 0; z < 2; ++z) {
                const bf16x8* src = z ? zero : rnd;
                auto k = big ? mfma_loop<true> : mfma_loop<false>;
                const int iters = big ? it32 : it16;
                hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, src, out, 100);
                hipEventRecord(e0);
                hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, src, out, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                const double flop = (double)blocks * 8 /*waves*/ * iters * (big ? 4.0 * 32768 : 8.0 * 16384);
                printf("{\"mfma\": \"%s\", \"data\": \"%s\", \"ms\": %.3f, \"TFLOPs\": %.1f}\n",
                       big ? "32x32x16_bf16" : "16x16x32_bf16", z ? "zero" : "random", ms, flop / ms / 1e9);
            }
        }
    }
    return 0;
}
