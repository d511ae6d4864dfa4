// dma_seg.hip — LDS-DMA delivery rate per CU as a function of the row-segment length of one instruction (round-5
// study for the GEMM operand stream).  Every instruction moves 1 KiB lane-linear (16 B per lane) into LDS; the
// 64 lanes cover R = 1024 / SEG rows x SEG contiguous bytes, rows 8 KiB apart (the K-major weight / activation
// layout at K = 4096).  SEG = 128 is the gemm_lg slab row (8 rows x 128 B), SEG = 1024 the lane-linear piece of
// l2_feed.hip mode 0 (~60 B/clk/CU).  Two sources:
//   L2: one 512-thread workgroup per CU streams a private 64 KiB panel (16 rows x 4 KiB) over and over
//   HBM: each workgroup walks its own 16-row x 8 KiB slabs of a buffer far larger than the 256 MiB Infinity Cache
//   hipcc --offload-arch=gfx950 -O3 -o dma_seg dma_seg.hip && ./dma_seg
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kRowBytes = 8192;

template <int SEG>
__device__ __forceinline__ const unsigned char* piece_addr(const unsigned char* base, int rows, int piece, int lane) {
    constexpr int R = 1024 / SEG, LPR = SEG / 16;  // rows per instruction, lanes per row segment
    const int groups = rows / R;                    // row groups in the panel / slab
    const int rg = piece % groups, col = piece / groups;
    const int row = rg * R + lane / LPR;
    return base + (size_t)row * kRowBytes + (size_t)col * SEG + (lane % LPR) * 16;
}

template <int SEG>
__global__ void __launch_bounds__(512) feed_l2(const unsigned char* __restrict__ src, unsigned* out, int iters) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // 16 rows x the first 4 KiB of each (64 KiB, L2-resident after the first pass)
    const unsigned char* panel = src + (size_t)blockIdx.x * 16 * kRowBytes;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int piece = wave * 8 + i;  // 64 x 1 KiB
            const unsigned char* p = piece_addr<SEG>(panel, 16, piece, lane);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)p, (lds_ptr_t)(smem + (wave * 8 + i) * 1024), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (reinterpret_cast<unsigned*>(smem)[tid] == 0x12345678u) out[blockIdx.x] = 1;
}

template <int SEG>
__global__ void __launch_bounds__(512) feed_hbm(const unsigned char* __restrict__ src, unsigned* out, int slabs) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int sb = 0; sb < slabs; ++sb) {
        const unsigned char* slab = src + ((size_t)blockIdx.x * slabs + sb) * 16 * kRowBytes;  // 128 KiB
#pragma unroll 4
        for (int i = 0; i < 16; ++i) {
            const int piece = wave * 16 + i;  // 128 x 1 KiB
            const unsigned char* p = piece_addr<SEG>(slab, 16, piece, lane);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)p, (lds_ptr_t)(smem + (wave * 8 + (i & 7)) * 1024), 16, 0,
                                             0);
            if ((i & 7) == 7) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (reinterpret_cast<unsigned*>(smem)[tid] == 0x12345678u) out[blockIdx.x] = 1;
}

template <int SEG>
static void run(int cus, const unsigned char* src, const unsigned char* big, size_t hb, int slabs, unsigned* out) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(feed_l2<SEG>), hipFuncAttributeMaxDynamicSharedMemorySize,
                        65536);
    hipFuncSetAttribute(reinterpret_cast<const void*>(feed_hbm<SEG>), hipFuncAttributeMaxDynamicSharedMemorySize,
                        65536);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 4000;
    float best_l2 = 1e30f, best_hbm = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        float ms;
        hipLaunchKernelGGL(feed_l2<SEG>, dim3(cus), dim3(512), 65536, 0, src, out, 10);
        hipEventRecord(a);
        hipLaunchKernelGGL(feed_l2<SEG>, dim3(cus), dim3(512), 65536, 0, src, out, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        best_l2 = ms < best_l2 ? ms : best_l2;
        hipEventRecord(a);
        hipLaunchKernelGGL(feed_hbm<SEG>, dim3(cus), dim3(512), 65536, 0, big, out, slabs);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        best_hbm = ms < best_hbm ? ms : best_hbm;
    }
    const double l2b = (double)cus * 65536.0 * iters;
    printf("{\"seg_bytes\": %d, \"rows_per_instr\": %d, \"l2_TBps\": %.2f, \"l2_B_per_clk_cu_2.4GHz\": %.1f, "
           "\"hbm_TBps\": %.2f}\n",
           SEG, 1024 / SEG, l2b / best_l2 / 1e9, l2b / cus / (best_l2 * 1e-3) / 2.4e9, hb / best_hbm / 1e9);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    unsigned char *src, *big;
    unsigned* out;
    const size_t bytes = (size_t)cus * 16 * kRowBytes;
    const int slabs = 24;
    const size_t hb = (size_t)cus * slabs * 16 * kRowBytes;  // 768 MiB at 256 CUs
    hipMalloc(&src, bytes);
    hipMalloc(&big, hb);
    hipMalloc(&out, cus * 4);
    hipMemset(src, 1, bytes);
    hipMemset(big, 1, hb);
    run<64>(cus, src, big, hb, slabs, out);
    run<128>(cus, src, big, hb, slabs, out);
    run<256>(cus, src, big, hb, slabs, out);
    run<512>(cus, src, big, hb, slabs, out);
    run<1024>(cus, src, big, hb, slabs, out);
    hipDeviceSynchronize();
    return 0;
}
