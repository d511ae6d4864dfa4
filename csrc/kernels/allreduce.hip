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
//
// Two-shot variant (mid-sized messages, e.g. 70B TP8 decode at B >= 64: 1-8 MiB).  One-shot reads W full copies
// per rank, so above ~1 MiB it is bound by the W-fold xGMI reads.  Two-shot splits the message into W slices, rank r
// owning slice r: (A) publish all slices as above; (B) reduce-scatter: rank r reads slice r from every peer, sums,
// writes it to its output and back over slice r of its own exchange buffer, then raises a second flag;
// (C) all-gather: after every peer's second flag, rank r reads slice p from peer p's buffer.  Each rank reads
// 2(W-1)/W of the message over xGMI instead of (W-1), in two dependent hops instead of one.
// Flag values: phase A of call e stores 2e-1, phase B stores 2e, so one flag array serves both kernels and the
// values stay monotonic whichever kernel each call uses (waits are "flag - target >= 0").
// Overwriting slice r in place is safe: in phase B peers only read their own slice p != r of my buffer, and slice r
// of my buffer is read by peers only after my phase-B flag.  A peer still gathering from call e-2 (same parity half)
// cannot exist: my call e started after my call e-1 saw that peer's phase-B flag of call e-1, which the peer raised
// after its call e-2 kernel had finished (stream order).
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

// One thread: wait until every peer's flag for block b has reached target (bounded spin; a lost peer sets the error
// word and returns 0 instead of hanging the GPU).
__device__ int ar_wait_peers(const ArPeers& peers, int rank, int world, int b, uint32_t target, uint32_t* ctl,
                             int64_t spin_limit) {
    for (int p = 0; p < world; ++p) {
        const uint32_t* f = &peers.flags[rank][p * kArMaxBlocks + b];
        int64_t spins = 0;
        while ((int32_t)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
            if (++spins > spin_limit) {
                __hip_atomic_store(&ctl[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return 0;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return 1;
}

// One thread: release this block's stores to other agents, then raise flag value v in every peer's array.
__device__ void ar_signal_peers(const ArPeers& peers, int rank, int world, int b, uint32_t v) {
    __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope: write back this GPU's L2 before the flag
    for (int p = 0; p < world; ++p)
        __hip_atomic_store(&peers.flags[p][rank * kArMaxBlocks + b], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The last block of a call to finish advances the epoch (every block read it at its start).
__device__ void ar_finish_call(uint32_t* ctl, uint32_t e, int nb) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t done = __hip_atomic_fetch_add(&ctl[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (done == (uint32_t)nb - 1) {
            __hip_atomic_store(&ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl[0], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

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
        ar_signal_peers(peers, rank, world, b, 2 * e - 1);
        s_ok = ar_wait_peers(peers, rank, world, b, 2 * e - 1, ctl, spin_limit);  // every peer's chunk b
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
    ar_finish_call(ctl, e, nb);
}

// Two-shot: n % (8 * world) == 0 (checked on the host).  Slice r = vectors [r * sv, (r + 1) * sv); block b owns
// sub-chunk b of every slice.
__global__ void __launch_bounds__(kArThreads) allreduce2_kernel(ArPeers peers, const uint16_t* __restrict__ in,
                                                                uint16_t* __restrict__ out, int64_t n,
                                                                int64_t half_elems, int rank, int world,
                                                                uint32_t* __restrict__ ctl, int64_t spin_limit) {
    __shared__ uint32_t s_epoch;
    __shared__ int s_ok;
    const int b = blockIdx.x, nb = gridDim.x;
    if (threadIdx.x == 0) s_epoch = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __syncthreads();
    const uint32_t e = s_epoch;
    const int64_t sv = n / 8 / world;  // vectors per slice
    const int64_t per = (sv + nb - 1) / nb;
    const int64_t c0 = (int64_t)b * per, c1 = c0 + per < sv ? c0 + per : sv;
    const int64_t half = (int64_t)(e & 1) * half_elems;
    u16x8* mine = reinterpret_cast<u16x8*>(peers.data[rank] + half);
    const u16x8* src = reinterpret_cast<const u16x8*>(in);
    u16x8* dst = reinterpret_cast<u16x8*>(out);

    // ---- (A) publish sub-chunk b of every slice
    for (int s = 0; s < world; ++s)
        for (int64_t v = s * sv + c0 + threadIdx.x; v < s * sv + c1; v += kArThreads) mine[v] = src[v];
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        ar_signal_peers(peers, rank, world, b, 2 * e - 1);
        s_ok = ar_wait_peers(peers, rank, world, b, 2 * e - 1, ctl, spin_limit);
    }
    __syncthreads();
    if (s_ok) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        // ---- (B) reduce my slice's sub-chunk over the W buffers (my own is peers.data[rank]); write it to out and
        // back over my buffer for the peers' gather
        for (int64_t v = rank * sv + c0 + threadIdx.x; v < rank * sv + c1; v += kArThreads) {
            float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int p = 0; p < world; ++p) {
                const u16x8 x = reinterpret_cast<const u16x8*>(peers.data[p] + half)[v];
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] += bf2f(x[j]);
            }
            u16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
            mine[v] = o;
            dst[v] = o;
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0 && s_ok) {
        ar_signal_peers(peers, rank, world, b, 2 * e);
        s_ok = ar_wait_peers(peers, rank, world, b, 2 * e, ctl, spin_limit);
    }
    __syncthreads();
    if (s_ok) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        // ---- (C) gather every other slice's reduced sub-chunk from its owner
        for (int p = 0; p < world; ++p) {
            if (p == rank) continue;
            const u16x8* theirs = reinterpret_cast<const u16x8*>(peers.data[p] + half);
            for (int64_t v = p * sv + c0 + threadIdx.x; v < p * sv + c1; v += kArThreads) dst[v] = theirs[v];
        }
    }
    ar_finish_call(ctl, e, nb);
}

// One-shot all-reduce fused with the residual add and RMSNorm that follow every row-parallel projection in a TP
// layer: resid <- bf16(bf16(sum of the W partials) + resid), y <- rmsnorm(resid) * w.  Same
// exchange protocol and flag values as allreduce_kernel (the two interleave freely), but each block owns whole rows,
// so the norm's sum of squares is a block reduction and the normalised rows leave in the same launch: one launch and
// one [T, d] round trip fewer per projection.  Rounding is the unfused path's exactly (all-reduce output in bf16,
// then rmsnorm_kernel<RESID=true>'s arithmetic).
template <int MAXV>
__global__ void __launch_bounds__(kArThreads) allreduce_norm_kernel(
    ArPeers peers, const uint16_t* __restrict__ in, uint16_t* __restrict__ resid, const uint16_t* __restrict__ w,
    uint16_t* __restrict__ y, int64_t rows, int d, float eps, int64_t half_elems, int rank, int world,
    uint32_t* __restrict__ ctl, int64_t spin_limit) {
    __shared__ uint32_t s_epoch;
    __shared__ int s_ok;
    __shared__ float red[16];
    const int b = blockIdx.x, nb = gridDim.x;
    if (threadIdx.x == 0) s_epoch = __hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    __syncthreads();
    const uint32_t e = s_epoch;
    const int nv = d / 8;
    const int64_t rpb = (rows + nb - 1) / nb;
    const int64_t r0 = (int64_t)b * rpb, r1 = r0 + rpb < rows ? r0 + rpb : rows;
    const int64_t half = (int64_t)(e & 1) * half_elems;
    u16x8* mine = reinterpret_cast<u16x8*>(peers.data[rank] + half);

    // ---- publish this block's rows
    for (int64_t v = r0 * nv + threadIdx.x; v < r1 * nv; v += kArThreads)
        mine[v] = reinterpret_cast<const u16x8*>(in)[v];
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        ar_signal_peers(peers, rank, world, b, 2 * e - 1);
        s_ok = ar_wait_peers(peers, rank, world, b, 2 * e - 1, ctl, spin_limit);
    }
    __syncthreads();
    if (s_ok) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        const u16x8* wv = reinterpret_cast<const u16x8*>(w);
        for (int64_t r = r0; r < r1; ++r) {
            u16x8* rv = reinterpret_cast<u16x8*>(resid + r * d);
            u16x8* yv = reinterpret_cast<u16x8*>(y + r * d);
            float vals[MAXV][8];
            float ss = 0.f;
#pragma unroll
            for (int k = 0; k < MAXV; ++k) {
                const int i = threadIdx.x + k * kArThreads;
                if (i < nv) {
                    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                    for (int p = 0; p < world; ++p) {
                        const u16x8 x = reinterpret_cast<const u16x8*>(peers.data[p] + half)[r * nv + i];
#pragma unroll
                        for (int j = 0; j < 8; ++j) acc[j] += bf2f(x[j]);
                    }
                    const u16x8 old = rv[i];
                    u16x8 nr;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        nr[j] = f2bf(bf2f(f2bf(acc[j])) + bf2f(old[j]));
                        vals[k][j] = bf2f(nr[j]);
                        ss += vals[k][j] * vals[k][j];
                    }
                    rv[i] = nr;
                }
            }
            const float inv = rsqrtf(block_sum(ss, red) / (float)d + eps);
#pragma unroll
            for (int k = 0; k < MAXV; ++k) {
                const int i = threadIdx.x + k * kArThreads;
                if (i < nv) {
                    const u16x8 g = wv[i];
                    u16x8 o;
#pragma unroll
                    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(f2bf(vals[k][j] * inv)) * bf2f(g[j]));
                    yv[i] = o;
                }
            }
        }
    }
    ar_finish_call(ctl, e, nb);
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
            // recorded as soon as mapped, so a failure on a later peer still unmaps these on destroy
            hip_ok(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle data");
            opened.push_back(pd);
            hip_ok(hipIpcOpenMemHandle(&pf, hf, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle flags");
            opened.push_back(pf);
            peers.data[p] = reinterpret_cast<uint16_t*>(pd);
            peers.flags[p] = reinterpret_cast<uint32_t*>(pf);
        }
    }

    // algo: 1 = one-shot, 2 = two-shot (needs n % (8 * world) == 0)
    void run(const uint16_t* in, uint16_t* out, int64_t n, int64_t spin_limit, int algo, hipStream_t st) {
        if (n == 0) return;
        if (n % 8 || n > half_elems) throw std::runtime_error("allreduce: n must be a multiple of 8 and fit the buffer");
        if (algo == 2 && n % (8 * world)) throw std::runtime_error("allreduce: two-shot needs n % (8 * world) == 0");
        // >= 2 vectors per thread: of the whole message (one-shot), of one slice (two-shot)
        const int64_t vec = algo == 2 ? n / 8 / world : n / 8;
        int64_t nb = (vec + kArThreads * 2 - 1) / (kArThreads * 2);
        if (nb > kArMaxBlocks) nb = kArMaxBlocks;
        if (nb < 1) nb = 1;
        if (algo == 2)
            hipLaunchKernelGGL(allreduce2_kernel, dim3((unsigned)nb), dim3(kArThreads), 0, st, peers, in, out, n,
                               half_elems, rank, world, ctl, spin_limit);
        else
            hipLaunchKernelGGL(allreduce_kernel, dim3((unsigned)nb), dim3(kArThreads), 0, st, peers, in, out, n,
                               half_elems, rank, world, ctl, spin_limit);
    }

    // rows x d bf16 partials -> resid (in place) and y; d % 8 == 0, d <= 8 * kArThreads * 8
    void run_norm(const uint16_t* in, uint16_t* resid, const uint16_t* w, uint16_t* y, int64_t rows, int d, float eps,
                  int64_t spin_limit, hipStream_t st) {
        if (rows == 0) return;
        if (d % 8 || rows * d > half_elems) throw std::runtime_error("allreduce_norm: d % 8 and rows * d <= capacity");
        const int vpt = (d / 8 + kArThreads - 1) / kArThreads;
        int64_t nb = rows < kArMaxBlocks ? rows : kArMaxBlocks;
        const dim3 g((unsigned)nb), blk(kArThreads);
#define ARN_CASE(V)                                                                                              \
    if (vpt <= V) {                                                                                              \
        hipLaunchKernelGGL((allreduce_norm_kernel<V>), g, blk, 0, st, peers, in, resid, w, y, rows, d, eps,       \
                           half_elems, rank, world, ctl, spin_limit);                                            \
        return;                                                                                                  \
    }
        ARN_CASE(1) ARN_CASE(2) ARN_CASE(4) ARN_CASE(8)
#undef ARN_CASE
        throw std::runtime_error("allreduce_norm: d too large");
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
void ar_run(void* h, const uint16_t* in, uint16_t* out, int64_t n, int64_t spin_limit, int algo, hipStream_t st) {
    static_cast<IpcAllReduce*>(h)->run(in, out, n, spin_limit, algo, st);
}
void ar_run_norm(void* h, const uint16_t* in, uint16_t* resid, const uint16_t* w, uint16_t* y, int64_t rows, int d,
                 float eps, int64_t spin_limit, hipStream_t st) {
    static_cast<IpcAllReduce*>(h)->run_norm(in, resid, w, y, rows, d, eps, spin_limit, st);
}
uint32_t ar_error(void* h) { return static_cast<IpcAllReduce*>(h)->error(); }
int64_t ar_capacity(void* h) { return static_cast<IpcAllReduce*>(h)->half_elems; }
void ar_destroy(void* h) { delete static_cast<IpcAllReduce*>(h); }

}  // namespace chronos
