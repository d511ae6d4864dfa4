// allreduce.hip — one-shot all-reduce over IPC-mapped peer buffers for tensor-parallel decode (SURVEY.md §2.3 K14,
// §5.8).  Decode-time TP all-reduces are latency-bound (70B TP8: 160 per step of 16 KiB x tokens); a ring
// collective pays 2(W-1) dependent hops, this pays one: every rank publishes its shard in its own buffer, raises a
// flag in each peer's flag array, waits for all peers' flags, then reads the W shards straight over xGMI (all 7
// links in parallel) and sums them in fp32.
//
// Protocol (per call, per block b; W ranks run the same sequence of calls):
//   epoch e   = a device-side counter read at kernel start (advanced by the LAST block of the call to finish, so
//               every block of a call sees the same e, replays of a captured hipGraph keep counting, and all ranks
//               agree without host involvement);
//   data      = my buffer, half (e & 1) — parity double buffering: a peer that raised flag >= e-1 in call e-1 had
//               finished call e-2 (stream order), i.e. finished reading the half I overwrite now, so one barrier per
//               call suffices;
//   publish   : block b copies its chunk of the input into data[e&1], all threads drain their stores, one thread
//               fences (release, system scope: writes back this GPU's L2) and stores e into flags[peer][me][b] of
//               every peer (uncached fine-grained memory, system-scope atomic store);
//   wait      : one thread polls my flags[me][p][b] >= e for all p (acquire, system scope), with a bounded spin — a
//               lost peer makes the call fail loudly (error word + early exit) instead of hanging the GPU;
//   reduce    : after an acquire fence (invalidates stale peer lines in L2), every thread reads its 16-B slices of the W
//               peer buffers, sums in fp32, writes bf16 output.
// Memory ordering follows MI355X_MICROARCH.md's cross-agent hand-off table: release by the storing side before the
// flag, acquire by the polling side before the data loads.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "chronos_hip.h"

namespace chronos {

constexpr int kArMaxWorld = 8;
constexpr int kArMaxBlocks = 64;
constexpr int kArThreads = 256;

struct ArPeers {
    uint16_t* data[kArMaxWorld];   // each rank's data buffer (2 halves of half_elems bf16), mapped into this process
    uint32_t* flags[kArMaxWorld];  // each rank's flag array [kArMaxWorld src][kArMaxBlocks], mapped
};

// local (non-shared) control words: [0] epoch, [1] finished-block counter, [2] error
__global__ void __launch_bounds__(kArThreads) allreduce_kernel(ArPeers peers, const uint16_t* __restrict__ in,
                                                               uint16_t* __restrict__ out, int64_t n,
                                                               int64_t half_elems, int rank, int world,
                                                               uint32_t* __restrict__ ctl, int64_t spin_limit) {
    __shared__ uint32_t s_epoch;
    __shared__ int s_ok;
    const int b = blockIdx.x, nb = gridDim.x;
    if (threadIdx.x == 0) s_epoch = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __syncthreads();
    const uint32_t e = s_epoch;
    // this block's chunk (whole 8-element vectors; n % 8 == 0 is checked on the host)
    const int64_t nv = n / 8;
    const int64_t per = (nv + nb - 1) / nb;
    const int64_t v0 = (int64_t)b * per, v1 = v0 + per < nv ? v0 + per : nv;
    uint16_t* mine = peers.data[rank] + (int64_t)(e & 1) * half_elems;

    // ---- publish
    for (int64_t v = v0 + threadIdx.x; v < v1; v += kArThreads)
        reinterpret_cast<u16x8*>(mine)[v] = reinterpret_cast<const u16x8*>(in)[v];
    __builtin_amdgcn_s_waitcnt(0);  // every thread's stores issued and retired before the block barrier
    __syncthreads();
    if (threadIdx.x == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope: make the data visible to other agents
        for (int p = 0; p < world; ++p)
            __hip_atomic_store(&peers.flags[p][rank * kArMaxBlocks + b], e, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        // ---- wait for every peer's chunk b
        int ok = 1;
        for (int p = 0; p < world && ok; ++p) {
            const uint32_t* f = &peers.flags[rank][p * kArMaxBlocks + b];
            int64_t spins = 0;
            while ((int32_t)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
                if (++spins > spin_limit) {
                    ok = 0;
                    __hip_atomic_store(&ctl[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        s_ok = ok;
    }
    __syncthreads();
    if (s_ok) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);  // drop any stale lines of peer buffers before reading them
        // ---- reduce
        for (int64_t v = v0 + threadIdx.x; v < v1; v += kArThreads) {
            float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int p = 0; p < world; ++p) {
                const u16x8 x = reinterpret_cast<const u16x8*>(peers.data[p] + (int64_t)(e & 1) * half_elems)[v];
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] += bf2f(x[j]);
            }
            u16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
            reinterpret_cast<u16x8*>(out)[v] = o;
        }
    }
    // ---- the last block of this call advances the epoch (all blocks read it above)
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t done = __hip_atomic_fetch_add(&ctl[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (done == (uint32_t)nb - 1) {
            __hip_atomic_store(&ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl[0], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ------------------------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------------------------
namespace {
void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("allreduce: ") + what + ": " + hipGetErrorString(e));
}
}  // namespace

struct IpcAllReduce {
    int rank, world;
    int64_t half_elems;
    uint16_t* data = nullptr;   // local data buffer (2 halves)
    uint32_t* flags = nullptr;  // local flag array (fine-grained, uncached)
    uint32_t* ctl = nullptr;    // local control words
    ArPeers peers{};
    std::vector<void*> opened;

    IpcAllReduce(int r, int w, int64_t max_bytes) : rank(r), world(w) {
        if (w < 1 || w > kArMaxWorld || r < 0 || r >= w) throw std::runtime_error("allreduce: bad rank/world");
        half_elems = ((max_bytes / 2) + 63) / 64 * 64;
        hip_ok(hipMalloc(&data, (size_t)half_elems * 2 * sizeof(uint16_t)), "hipMalloc data");
        hip_ok(hipExtMallocWithFlags((void**)&flags, kArMaxWorld * kArMaxBlocks * sizeof(uint32_t),
                                     hipDeviceMallocUncached),
               "hipExtMallocWithFlags flags");
        hip_ok(hipMemset(flags, 0, kArMaxWorld * kArMaxBlocks * sizeof(uint32_t)), "memset flags");
        hip_ok(hipMalloc((void**)&ctl, 4 * sizeof(uint32_t)), "hipMalloc ctl");
        hip_ok(hipMemset(ctl, 0, 4 * sizeof(uint32_t)), "memset ctl");
        hip_ok(hipDeviceSynchronize(), "sync");
    }

    // 2 x 64-byte IPC handles (data, flags)
    std::vector<uint8_t> handles() const {
        hipIpcMemHandle_t hd, hf;
        hip_ok(hipIpcGetMemHandle(&hd, data), "hipIpcGetMemHandle data");
        hip_ok(hipIpcGetMemHandle(&hf, flags), "hipIpcGetMemHandle flags");
        std::vector<uint8_t> out(2 * sizeof(hipIpcMemHandle_t));
        memcpy(out.data(), &hd, sizeof(hd));
        memcpy(out.data() + sizeof(hd), &hf, sizeof(hf));
        return out;
    }

    void open(const std::vector<std::vector<uint8_t>>& all) {
        if ((int)all.size() != world) throw std::runtime_error("allreduce: need one handle pair per rank");
        for (int p = 0; p < world; ++p) {
            if (p == rank) {
                peers.data[p] = data;
                peers.flags[p] = flags;
                continue;
            }
            hipIpcMemHandle_t hd, hf;
            memcpy(&hd, all[p].data(), sizeof(hd));
            memcpy(&hf, all[p].data() + sizeof(hd), sizeof(hf));
            void *pd = nullptr, *pf = nullptr;
            hip_ok(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle data");
            hip_ok(hipIpcOpenMemHandle(&pf, hf, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle flags");
            opened.push_back(pd);
            opened.push_back(pf);
            peers.data[p] = reinterpret_cast<uint16_t*>(pd);
            peers.flags[p] = reinterpret_cast<uint32_t*>(pf);
        }
    }

    void run(const uint16_t* in, uint16_t* out, int64_t n, int64_t spin_limit, hipStream_t st) {
        if (n == 0) return;
        if (n % 8 || n > half_elems) throw std::runtime_error("allreduce: n must be a multiple of 8 and fit the buffer");
        int64_t nb = (n / 8 + kArThreads * 2 - 1) / (kArThreads * 2);  // >= 2 vectors per thread
        if (nb > kArMaxBlocks) nb = kArMaxBlocks;
        if (nb < 1) nb = 1;
        hipLaunchKernelGGL(allreduce_kernel, dim3((unsigned)nb), dim3(kArThreads), 0, st, peers, in, out, n,
                           half_elems, rank, world, ctl, spin_limit);
    }

    uint32_t error() const {
        uint32_t v = 0;
        hip_ok(hipMemcpy(&v, ctl + 2, sizeof(v), hipMemcpyDeviceToHost), "read error word");
        return v;
    }

    ~IpcAllReduce() {
        for (void* p : opened) (void)hipIpcCloseMemHandle(p);
        if (data) (void)hipFree(data);
        if (flags) (void)hipFree(flags);
        if (ctl) (void)hipFree(ctl);
    }
};

// flat C-style API for bindings.cpp
void* ar_create(int rank, int world, int64_t max_bytes) { return new IpcAllReduce(rank, world, max_bytes); }
std::vector<uint8_t> ar_handles(void* h) { return static_cast<IpcAllReduce*>(h)->handles(); }
void ar_open(void* h, const std::vector<std::vector<uint8_t>>& all) { static_cast<IpcAllReduce*>(h)->open(all); }
void ar_run(void* h, const uint16_t* in, uint16_t* out, int64_t n, int64_t spin_limit, hipStream_t st) {
    static_cast<IpcAllReduce*>(h)->run(in, out, n, spin_limit, st);
}
uint32_t ar_error(void* h) { return static_cast<IpcAllReduce*>(h)->error(); }
int64_t ar_capacity(void* h) { return static_cast<IpcAllReduce*>(h)->half_elems; }
void ar_destroy(void* h) { delete static_cast<IpcAllReduce*>(h); }

}  // namespace chronos
