// decode_fused.hip — single-stream decode (M = 1, TP = 1): the attention of the new token AND the O projection with
// its residual epilogue in ONE persistent launch (SURVEY.md §2.3 K6 + K7; VERDICT r2 "cut single-stream launch
// boundaries").
//
// In the separate form, every layer runs the decode attention (8 workgroups: one per kv head, ~6 us, HBM nearly
// idle) and then the O GEMV, whose weight stream (33.6 MB for Llama-3-8B) only starts after a kernel boundary.  Here
// the launch is the O GEMV's persistent grid; its first hkv workgroups compute the attention first, publish the
// [hq * 128] output through a release + counter, and join the GEMV.  Every other workgroup issues its first weight
// ring (D x R rows of 1 KiB per wave) BEFORE it waits on that counter, so most of the O weights are in flight while
// the attention runs (the weights do not depend on it; MI355X_MICROARCH.md price list, prefetch-credit), then stages
// the attention output in LDS and streams the rest.
//
// Arithmetic is the separate kernels' exactly: the attention is paged_attn_kernel<1>'s single-split path (same
// 32-token steps, online softmax, four-wave LDS merge), the GEMV is gemv_kernel<1, R, kResid>'s (v_dot2 chunks, the
// same wave split of K, wave_sum, cross-wave sum in wave order, s = bf16(bf16(y) + r), per-group sum of s^2) — so the
// fused step is bit-identical to attention-then-gemv_resid (tests/test_decode_fused_gpu.py).
//
// Hand-off without fences (MI355X_MICROARCH.md hand-off table, third row): the attention workgroup writes its output
// with write-through sc1 dword stores (every 128-B line by one store instruction of one wave) -> every storing wave
// s_waitcnt vmcnt(0) -> __syncthreads -> lane 0 relaxed agent atomic add.  Consumer: lane 0 polls the counter with
// sc1 loads + s_sleep (bounded: on timeout it sets the error word and proceeds, never hangs) -> __syncthreads ->
// sc1 dword loads of the output.  (The fenced form — release + acquire — cost more than the boundary it removed.)  The attention
// workgroups have the lowest indices, are dispatched first and wait on nothing, so the grid cannot deadlock even if
// it were not fully resident.  The last workgroup to finish resets both counters for the next launch (graph replay).
#include "chronos_hip.h"

namespace chronos {

namespace {

constexpr int kHd = 128;
constexpr int kOS = 132;  // LDS row stride (floats) of the attention merge buffer

struct AttnOArgs {
    // attention (one query token, bf16 paged cache)
    const uint16_t* q;      // [hq, 128]
    const uint16_t* kc;     // [blk, hkv, bs, 128]
    const uint16_t* vc;     // [blk, hkv, 128, bs]
    const int32_t* bt;      // block table row of the sequence
    const int32_t* ctx_len; // [1]
    int hq, hkv, block_size;
    float scale_log2;
    // O projection + residual epilogue
    const uint16_t* w;      // [N, K] (K = hq * 128)
    const uint16_t* rin;    // [N]
    uint16_t* rout;         // [N]
    float* part_out;        // [N / R]
    int N, K;
    uint16_t* attn_out;     // [K] scratch: the attention output handed to the GEMV
    int* sync;              // [2]: attention arrivals, finished workgroups (zero between launches)
    int* err;               // set when a wait timed out
    int spin_limit;
    int pre;                // weight ring entries (of DEPTH) issued before the wait (knob attn_o_pre)
    int sleep;              // s_sleep(1) repetitions between polls (knob attn_o_sleep)
    const int32_t* gst;     // decode gate (see chronos_hip.h)
    int gn;
};

// paged_attn_kernel<1, false, false> with one split, sequence 0, query row 0, as a device function of workgroup h
__device__ void attn_head(const AttnOArgs& a, int h, float* smem, uint16_t* ob) {
    constexpr int ROWS = 16;
    float* sm = smem;           // [4][ROWS]
    float* sl = sm + 4 * ROWS;  // [4][ROWS]
    float* so = sl + 4 * ROWS;  // [4][ROWS][kOS]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, h4 = lane >> 4;
    const int G = a.hq / a.hkv;
    const int ctx = a.ctx_len[0];
    const int ctx0 = ctx - 1;
    const int tr = r / G, hd = h * G + r % G;
    const bool valid = tr < 1;
    const int rpos = valid ? ctx0 : -1;
    bf16x8 qf[4];
    const uint16_t* qp = a.q + (int64_t)hd * kHd + 8 * h4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        bf16x8 v = *reinterpret_cast<const bf16x8*>(qp + 32 * c);
        if (!valid) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        qf[c] = v;
    }
    const int ke = ctx0 + 1;
    float m = -1e30f, lsum = 0.f;
    f32x4 o[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int bs = a.block_size;
    for (int t0 = w * 32; t0 < ke; t0 += 128) {
        bf16x8 kf[2][4];
        bf16x4 vf[2][8];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int tg = t0 + 16 * g;
            if (tg < ke) {
                const int64_t blk = a.bt[tg / bs];
                const int off = tg % bs;
                const int64_t koff = (((blk * a.hkv + h) * bs) + off + r) * kHd + 8 * h4;
                const int64_t voff = ((blk * a.hkv + h) * kHd) * (int64_t)bs + off + 4 * h4;
#pragma unroll
                for (int c = 0; c < 4; ++c) kf[g][c] = *reinterpret_cast<const bf16x8*>(a.kc + koff + 32 * c);
#pragma unroll
                for (int dt = 0; dt < 8; ++dt)
                    vf[g][dt] = *reinterpret_cast<const bf16x4*>(a.vc + voff + (int64_t)(dt * 16 + r) * bs);
            } else {
#pragma unroll
                for (int c = 0; c < 4; ++c) kf[g][c] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                for (int dt = 0; dt < 8; ++dt) vf[g][dt] = bf16x4{0, 0, 0, 0};
            }
        }
        if (t0 + 32 > ke) {
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (t0 + 16 * g + 4 * h4 + i >= ke)
#pragma unroll
                        for (int dt = 0; dt < 8; ++dt) vf[g][dt][i] = (__bf16)0.f;
        }
        f32x4 s[2];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[g][c], qf[c], acc, 0, 0, 0);
            s[g] = acc;
        }
        float mx = -INFINITY;
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int tok = t0 + 16 * g + 4 * h4 + i;
                float v = s[g][i] * a.scale_log2;
                if (tok >= ke || tok > rpos) v = -INFINITY;
                s[g][i] = v;
                mx = fmaxf(mx, v);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m, mx);
        const float alpha = exp2f(m - mnew);
        m = mnew;
        float ps = 0.f;
        bf16x8 pf;
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float p = exp2f(s[g][i] - mnew);
                ps += p;
                pf[4 * g + i] = (__bf16)p;
            }
        lsum = lsum * alpha + ps;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            o[dt] *= alpha;
            const bf16x8 va = __builtin_shufflevector(vf[0][dt], vf[1][dt], 0, 1, 2, 3, 4, 5, 6, 7);
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pf, o[dt], 0, 0, 0);
        }
    }
    float lt = lsum;
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    if (h4 == 0) {
        sm[w * ROWS + r] = m;
        sl[w * ROWS + r] = lt;
    }
    float* orow = so + (w * ROWS + r) * kOS;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) *reinterpret_cast<f32x4*>(orow + dt * 16 + 4 * h4) = o[dt];
    __syncthreads();
    for (int idx = threadIdx.x; idx < ROWS * 16; idx += 256) {
        const int row = idx >> 4, c8 = idx & 15;
        if (row / G >= 1) continue;
        const int hdd = h * G + row % G;
        float M = -1e30f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, sm[ww * ROWS + row]);
        float L = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) {
            const float f = exp2f(sm[ww * ROWS + row] - M);
            L += sl[ww * ROWS + row] * f;
            const float* orr = so + (ww * ROWS + row) * kOS + c8 * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += orr[j] * f;
        }
        const float inv = L > 0.f ? 1.f / L : 0.f;
        u16x8 ov;
#pragma unroll
        for (int j = 0; j < 8; ++j) ov[j] = f2bf(acc[j] * inv);
        *reinterpret_cast<u16x8*>(ob + (row % G) * kHd + c8 * 8) = ov;  // staged: published as whole lines below
    }
    // publish the head group's G x 128 outputs as write-through (sc1) dword stores, one per thread, so every 128-B
    // line leaves in ONE store instruction of one wave (MI355X_MICROARCH.md hand-off table, third row): the consumer
    // then needs no acquire fence, and this workgroup no release fence (each costs 1.7-6.5 us: more than the kernel
    // boundary this launch removes)
    __syncthreads();
    const uint32_t* obw = reinterpret_cast<const uint32_t*>(ob);
    uint32_t* dst = reinterpret_cast<uint32_t*>(a.attn_out + (int64_t)h * G * kHd);
    for (int i = threadIdx.x; i < G * kHd / 2; i += 256)
        __hip_atomic_store(dst + i, obw[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float dot8f(const u16x8& w, const u16x8& x, float acc) {
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

// R output rows per task; DEPTH 1-KiB chunks per row in the register ring (gemv_kernel<1, R, kResid>'s choice:
// DEPTH = 3 for R = 4)
template <int R, int DEPTH, int KMAX>
__global__ void __launch_bounds__(256) attn_o_kernel(AttnOArgs a) {
    constexpr int ROWS = 16;
    __shared__ __attribute__((aligned(16))) float smem[8 * ROWS + 4 * ROWS * kOS];  // attention merge
    __shared__ __attribute__((aligned(16))) uint16_t xs[KMAX];                       // the attention output
    __shared__ float red[4][R];
    __shared__ float sq[R];
    __shared__ int s_ok;
    if (a.gn < 0 && gate_closed(a.gst, -a.gn)) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int K = a.K, nchunk = K >> 9;
    const int ntasks = a.N / R;

    // ---- phase 1: the attention workgroups
    if ((int)blockIdx.x < a.hkv) {
        attn_head(a, blockIdx.x, smem, reinterpret_cast<uint16_t*>(xs));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave's sc1 stores have landed
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(a.sync, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();  // xs (the staging buffer) is reused for the GEMV input below
    }

    // ---- phase 2: the O GEMV (persistent over row groups), first weight ring issued before the wait
    int g = blockIdx.x;
    const u16x8* wrow[R];
    auto set_rows = [&](int grp) {
#pragma unroll
        for (int r = 0; r < R; ++r) wrow[r] = reinterpret_cast<const u16x8*>(a.w + (int64_t)(grp * R + r) * K);
    };
    u16x8 wr[DEPTH][R];
    auto load = [&](int c, int d) {
        const int off = c * 64 + lane;
#pragma unroll
        for (int r = 0; r < R; ++r) wr[d][r] = __builtin_nontemporal_load(wrow[r] + off);
    };
    auto prologue = [&]() {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d)
            if (w + 4 * d < nchunk) load(w + 4 * d, d);
    };
    // the first ring: a.pre entries before the wait (they stream while the attention runs; more of them compete with
    // the attention's own K/V reads for HBM), the rest after it
    if (g < ntasks) {
        set_rows(g);
#pragma unroll
        for (int d = 0; d < DEPTH; ++d)
            if (d < a.pre && w + 4 * d < nchunk) load(w + 4 * d, d);
    }
    // wait for the attention output, then stage it in LDS (every workgroup, also those without a task: they still
    // count as finished below)
    if (threadIdx.x == 0) {
        int ok = 1, n = 0;
        while (__hip_atomic_load(a.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.hkv) {
            for (int z = 0; z < a.sleep; ++z) __builtin_amdgcn_s_sleep(1);
            if (++n > a.spin_limit) {
                ok = 0;
                break;
            }
        }
        if (!ok) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_ok = ok;
    }
    __syncthreads();  // the poll matched: every load of the handed-off bytes below is an sc1 load
    if (g < ntasks) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d)
            if (d >= a.pre && w + 4 * d < nchunk) load(w + 4 * d, d);
    }
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.attn_out);
        uint32_t* xw = reinterpret_cast<uint32_t*>(xs);
        for (int i = threadIdx.x; i < K / 2; i += 256)
            xw[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const u16x8* xl = reinterpret_cast<const u16x8*>(xs);
    while (g < ntasks) {
        float acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = 0.f;
        for (int c0 = w; c0 < nchunk; c0 += 4 * DEPTH) {
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
                const int c = c0 + 4 * d;
                if (c < nchunk) {
                    const u16x8 xv = xl[c * 64 + lane];
#pragma unroll
                    for (int r = 0; r < R; ++r) acc[r] = dot8f(wr[d][r], xv, acc[r]);
                    if (c + 4 * DEPTH < nchunk) load(c + 4 * DEPTH, d);
                }
            }
        }
        const int bid = g, n0 = g * R;
        g += gridDim.x;
        const bool more = g < ntasks;
        if (more) {  // the ring is consumed: the next group's weights stream during this group's epilogue
            set_rows(g);
            prologue();
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float s = wave_sum(acc[r]);
            if (lane == 0) red[w][r] = s;
        }
        __syncthreads();
        const int t = threadIdx.x;
        if (t < R) {
            const float tot = red[0][t] + red[1][t] + red[2][t] + red[3][t];
            const uint16_t sb = f2bf(bf2f(f2bf(tot)) + bf2f(a.rin[n0 + t]));
            a.rout[n0 + t] = sb;
            sq[t] = bf2f(sb) * bf2f(sb);
        }
        __syncthreads();
        if (t == 0) {
            float ss = 0.f;
#pragma unroll
            for (int r = 0; r < R; ++r) ss += sq[r];
            a.part_out[bid] = ss;
        }
        if (!more) break;
        __syncthreads();  // red / sq are rewritten by the next group
    }
    // ---- the last workgroup out resets the counters for the next launch
    __syncthreads();
    if (threadIdx.x == 0) {
        const int done = __hip_atomic_fetch_add(a.sync + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done == (int)gridDim.x - 1) {
            __hip_atomic_store(a.sync, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.sync + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace

// Returns false (nothing launched) off the supported shapes; the caller then runs the two separate kernels.
bool launch_attn_o(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const int32_t* bt,
                   const int32_t* ctx_len, int hq, int hkv, int block_size, float scale_log2, const uint16_t* w,
                   const uint16_t* rin, uint16_t* rout, float* part_out, int N, int K, uint16_t* attn_out, int* sync,
                   int* err, int grid_cap, hipStream_t st) {
    constexpr int R = 4, DEPTH = 3, KMAX = 8192;
    if (K != hq * kHd || K % 512 || K > KMAX || N % R || hq % hkv || hkv > 64) return false;
    if (!knob("attn_o", 1)) return false;  // in-process A/B: 0 = the separate kernels
    AttnOArgs a{};
    a.q = q;
    a.kc = kc;
    a.vc = vc;
    a.bt = bt;
    a.ctx_len = ctx_len;
    a.hq = hq;
    a.hkv = hkv;
    a.block_size = block_size;
    a.scale_log2 = scale_log2;
    a.w = w;
    a.rin = rin;
    a.rout = rout;
    a.part_out = part_out;
    a.N = N;
    a.K = K;
    a.attn_out = attn_out;
    a.sync = sync;
    a.err = err;
    a.spin_limit = knob("attn_o_spin", 1 << 22);
    a.pre = knob("attn_o_pre", DEPTH);
    a.sleep = knob("attn_o_sleep", 1);
    const int32_t* gst = g_gate_n > 0 && g_gate_n <= kGateMax ? g_gate_state : nullptr;
    a.gst = gst;
    a.gn = gst ? -g_gate_n : 0;
    const int ntasks = N / R;
    const int fit = resident_workgroups(attn_o_kernel<R, DEPTH, KMAX>, 256);
    int grid = fit < ntasks ? fit : ntasks;
    if (grid_cap <= 0) grid_cap = knob("attn_o_grid", 0);
    if (grid_cap > 0 && grid_cap < grid) grid = grid_cap;
    if (grid < hkv) grid = hkv;
    hipLaunchKernelGGL((attn_o_kernel<R, DEPTH, KMAX>), dim3(grid), dim3(256), 0, st, a);
    return true;
}

int attn_o_parts(int N) { return N / 4; }

}  // namespace chronos
