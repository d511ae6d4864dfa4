// l2_feed.hip — per-CU operand delivery rate from L2 for the three ways a GEMM tile can be fed (round-3 study):
//   0: LDS-DMA (global_load_lds_dwordx4, 1 KiB lane-linear pieces into an LDS ring, counted vmcnt)
//   1: global_load_dwordx4 to VGPRs in the 16x16x32 MFMA operand layout (16 rows x 64 B per instruction)
//   2: global_load_dwordx4 to VGPRs, full 128-B lines (8 rows x 128 B per instruction)
// One 512-thread workgroup per CU streams a private 64 KiB panel (rows of 8 KiB, the K-major weight layout) over and
// over: every byte after the first pass is an L2 hit, so the rate is the CU's L2 -> CU path, not HBM.
//   hipcc --offload-arch=gfx950 -O3 -o l2_feed l2_feed.hip && ./l2_feed
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kRowBytes = 8192, kRows = 8;  // panel: 8 rows x 8 KiB = 64 KiB per workgroup

template <int MODE>
__global__ void __launch_bounds__(512) feed(const unsigned char* __restrict__ src, unsigned* out, int iters) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned char* panel0 = src + (size_t)blockIdx.x * kRows * kRowBytes;
    u32x4 acc = {0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
        // alternate between the panel and the one 4 KiB further (loop-variant addresses: nothing can be hoisted)
        const unsigned char* panel = panel0 + ((it & 1) << 12);
        // each wave covers 8 KiB of the panel per pass (8 waves = 64 KiB), 8 instructions of 1 KiB
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int piece = wave * 8 + i;  // 64 pieces of 1 KiB
            if constexpr (MODE == 0) {
                // lane-linear 1 KiB: 8 lanes per 128-B line segment of one row
                const unsigned char* p = panel + (size_t)(piece & 7) * kRowBytes + (piece >> 3) * 1024 + lane * 16;
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)p, (lds_ptr_t)(smem + (wave * 8 + i) * 1024), 16, 0, 0);
            } else if constexpr (MODE == 1) {
                // fragment layout: lane -> row (lane & 15) of a 16-row tile (rows spread over the 8 panel rows x 2
                // halves), 16 B at column 16 * (lane >> 4) of a 64-B k slice
                const int row = lane & 15;
                const unsigned char* p = panel + (size_t)(row & 7) * kRowBytes + (row >> 3) * 4096 + piece * 64 +
                                         16 * (lane >> 4);
                acc ^= *reinterpret_cast<const u32x4*>(p);
            } else {
                const int row = lane >> 3;
                const unsigned char* p = panel + (size_t)row * kRowBytes + piece * 128 + 16 * (lane & 7);
                acc ^= *reinterpret_cast<const u32x4*>(p);
            }
        }
        if constexpr (MODE == 0) {
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // one pass of 8 pieces stays in flight
        }
    }
    if constexpr (MODE == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        acc.x = reinterpret_cast<unsigned*>(smem)[tid];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[blockIdx.x] = 1;  // keeps the loads live
}

// HBM streaming (every byte read once, buffer >> the 256 MiB Infinity Cache): the same two VGPR layouts.  Each
// workgroup walks 16-row x 8 KiB slabs of its own region; a pass = one 1 KiB instruction per wave per 1 KiB of slab.
template <int MODE>
__global__ void __launch_bounds__(512) stream(const unsigned char* __restrict__ src, unsigned* out, int slabs) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    u32x4 acc = {0, 0, 0, 0};
    for (int sb = 0; sb < slabs; ++sb) {
        const unsigned char* slab = src + ((size_t)blockIdx.x * slabs + sb) * 16 * kRowBytes;  // 128 KiB
#pragma unroll 4
        for (int i = 0; i < 16; ++i) {
            const int piece = wave * 16 + i;  // 128 pieces of 1 KiB
            const unsigned char* p;
            if constexpr (MODE == 1) {  // 16 rows x 64 B (k slice piece)
                p = slab + (size_t)(lane & 15) * kRowBytes + piece * 64 + 16 * (lane >> 4);
            } else {  // 8 rows x 128 B
                p = slab + (size_t)(8 * (piece & 1) + (lane >> 3)) * kRowBytes + (piece >> 1) * 128 + 16 * (lane & 7);
            }
            acc ^= *reinterpret_cast<const u32x4*>(p);
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[blockIdx.x] = 1;
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const size_t bytes = (size_t)cus * kRows * kRowBytes + 8192;
    unsigned char* src;
    unsigned* out;
    hipMalloc(&src, bytes);
    hipMalloc(&out, cus * 4);
    hipMemset(src, 1, bytes);
    const int iters = 4000;
    hipFuncSetAttribute(reinterpret_cast<const void*>(feed<0>), hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[3] = {"LDS-DMA 1 KiB lane-linear", "VGPR fragment (16 rows x 64 B)", "VGPR full lines (8 x 128 B)"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 3; ++mode) {
            auto k = mode == 0 ? feed<0> : mode == 1 ? feed<1> : feed<2>;
            hipLaunchKernelGGL(k, dim3(cus), dim3(512), mode == 0 ? 65536 : 0, 0, src, out, 10);
            hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3(cus), dim3(512), mode == 0 ? 65536 : 0, 0, src, out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double tot = (double)cus * 65536.0 * iters;
            printf("%-34s %8.2f TB/s chip, %6.1f GB/s per CU (%.1f B/clk at 2.1 GHz)\n", names[mode],
                   tot / ms / 1e9, tot / cus / ms / 1e6, tot / cus / (ms * 1e-3) / 2.1e9);
        }
    }
    // HBM: 256 workgroups x 24 slabs x 128 KiB = 768 MiB per launch
    const int slabs = 24;
    const size_t hb = (size_t)cus * slabs * 16 * kRowBytes;
    unsigned char* big;
    hipMalloc(&big, hb);
    hipMemset(big, 1, hb);
    const char* hn[2] = {"HBM VGPR fragment (16 rows x 64 B)", "HBM VGPR full lines (8 x 128 B)"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 1; mode <= 2; ++mode) {
            auto k = mode == 1 ? stream<1> : stream<2>;
            hipLaunchKernelGGL(k, dim3(cus), dim3(512), 0, 0, big, out, slabs);
            hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3(cus), dim3(512), 0, 0, big, out, slabs);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("%-34s %8.2f TB/s chip\n", hn[mode - 1], hb / ms / 1e9);
        }
    }
    return 0;
}
