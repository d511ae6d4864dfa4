// mfma_dma.hip — what an LDS-DMA piece costs a stream of MFMAs (the gemm_lg.hip ablations: DMA + MFMA ran 33 % over
// MFMA alone with the operands L2-resident, so the cost is in issue, not in memory).
//
// Every wave runs ITERS iterations of {NMF v_mfma_f32_16x16x32_bf16 on 8 independent accumulators, NDMA 1 KiB loads
// interleaved (sched_group_barrier)}; loads keep one iteration in flight (counted vmcnt), the source is a 2 MiB
// L2-resident buffer, no barriers.  KIND: 0 buffer_load_dwordx4 ... lds, 1 global_load_lds_dwordx4, 2
// global_load_dwordx4 to VGPRs.  Reports cycles per iteration per wave (s_memtime) and the per-SIMD MFMA-pipe
// utilisation (waves per SIMD x NMF x 16 cycles / cycles per iteration).
//
//   hipcc --offload-arch=gfx950 -O3 -o mfma_dma mfma_dma.hip && ./mfma_dma
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

template <int N>
__device__ __forceinline__ void vmcnt() {
    __builtin_amdgcn_s_waitcnt((N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

// MFMA i is preceded by its share of the NV loads and followed by its share of the NR ds_reads; HEAD: every load
// before the first MFMA, the reads spread over the MFMAs after the first NV
template <int I, int MF, int NV, int NR, bool HEAD>
__device__ __forceinline__ void sched() {
    if constexpr (I < MF) {
        constexpr int v = HEAD ? (I == 0 ? NV : 0) : (I + 1) * NV / MF - I * NV / MF;
        constexpr int R0 = HEAD ? (NV < MF ? NV : 0) : 0;
        constexpr int r = I < R0 ? 0 : (I - R0 + 1) * NR / (MF - R0) - (I - R0) * NR / (MF - R0);
        if constexpr (v > 0) __builtin_amdgcn_sched_group_barrier(0x010, v, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if constexpr (r > 0) __builtin_amdgcn_sched_group_barrier(0x100, r, 0);
        sched<I + 1, MF, NV, NR, HEAD>();
    }
}

__device__ __forceinline__ void dma_buf(const void* base, unsigned char* dst, uint32_t voff) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 1 << 21,
                                                                       0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 16, voff, 0, 0, 0);
}

template <int NMF, int NDMA, int KIND, int NRD = 0, bool HEAD = false>
__global__ void __launch_bounds__(512, 1) kern(const uint16_t* src, float* out, long long* cyc, int iters) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    bf16x8 a = *reinterpret_cast<const bf16x8*>(src + lane * 8);
    bf16x8 b = *reinterpret_cast<const bf16x8*>(src + 512 + lane * 8);
    bf16x8 rf[NRD > 0 ? NRD : 1];
    const unsigned char* rsrc = smem + 65536 - 16384 + (lane & 15) * 128 + (((lane >> 4) ^ (lane & 7)) << 4);
    f32x4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint32_t voff = ((blockIdx.x * 8 + wave) * 4096 + lane * 16) & ((1 << 21) - 1);
    unsigned char* dst = smem + wave * 8192;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 reg[NDMA > 0 && KIND == 2 ? NDMA : 1];
    vmcnt<0>();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int d = 0; d < NDMA; ++d) {
            const uint32_t off = (voff + (uint32_t)(it * NDMA + d) * 1024u) & ((1u << 21) - 1u);
            if constexpr (KIND == 0) dma_buf(src, dst + (d & 7) * 1024, off);
            else if constexpr (KIND == 1)
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)((const unsigned char*)src + off),
                                                 (lds_ptr_t)(dst + (d & 7) * 1024), 16, 0, 0);
            else reg[d] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>((const unsigned char*)src + off));
        }
#pragma unroll
        for (int i = 0; i < NMF; ++i) acc[i & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i & 7], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < NRD; ++r) rf[r] = *reinterpret_cast<const bf16x8*>(rsrc + (r & 7) * 2048);
        sched<0, NMF, NDMA, NRD, HEAD>();
        if constexpr (NRD > 0) {
#pragma unroll
            for (int r = 0; r < NRD; ++r) asm volatile("" ::"v"(rf[r]));
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (KIND == 2 && NDMA > 0) {
#pragma unroll
            for (int d = 0; d < NDMA; ++d) asm volatile("" ::"v"(reg[d]));
        } else {
            vmcnt<NDMA>();  // one iteration's pieces stay in flight
        }
    }
    vmcnt<0>();
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int NMF, int NDMA, int KIND, int NRD = 0, bool HEAD = false>
void run(const char* name, int waves, const uint16_t* src, float* out, long long* cyc) {
    const int iters = 2000, grid = 256;
    auto k = kern<NMF, NDMA, KIND, NRD, HEAD>;
    hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * waves), 65536, 0, src, out, cyc, iters);
    hipDeviceSynchronize();
    std::vector<long long> h(grid * 8);
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double sum = 0;
    int n = 0;
    // the slowest wave of each workgroup (two waves on a SIMD share it: the younger one finishes last)
    for (int b = 0; b < grid; ++b) {
        long long mx = 0;
        for (int w = 0; w < waves; ++w) mx = h[b * 8 + w] > mx ? h[b * 8 + w] : mx;
        sum += mx, ++n;
    }
    const double per = sum / n / iters;
    const double util = (waves / 4.0) * NMF * 16 / per;
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"mfma\": %d, \"dma\": %d, \"kind\": %d, \"reads\": %d, "
           "\"dma_head\": %d, \"cyc_per_iter\": %.1f, \"mfma_pipe_util\": %.3f}\n", name, waves / 4, NMF, NDMA, KIND,
           NRD, (int)HEAD, per, util);
}

int main() {
    uint16_t* src;
    float* out;
    long long* cyc;
    hipMalloc(&src, 1 << 21);
    hipMemset(src, 0x3c, 1 << 21);
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&cyc, 256 * 8 * 8);
    for (int waves : {4, 8}) {
        run<32, 0, 0>("mfma only", waves, src, out, cyc);
        run<32, 8, 0>("buffer lds x8", waves, src, out, cyc);
        run<32, 0, 0, 12>("reads x12", waves, src, out, cyc);
        run<32, 8, 0, 12>("buffer lds x8 + reads x12 interleaved", waves, src, out, cyc);
        run<32, 8, 0, 12, true>("buffer lds x8 head + reads x12", waves, src, out, cyc);
        run<32, 4, 0, 12>("buffer lds x4 + reads x12", waves, src, out, cyc);
        run<64, 16, 0, 16>("128x128/wave: 64 mfma, 16 dma, 16 reads", waves, src, out, cyc);
        run<64, 16, 0, 16, true>("128x128/wave: 64 mfma, 16 dma head, 16 reads", waves, src, out, cyc);
        run<32, 8, 2, 12>("global vgpr x8 + reads x12", waves, src, out, cyc);
    }
    hipFree(src);
    hipFree(out);
    hipFree(cyc);
    return 0;
}
