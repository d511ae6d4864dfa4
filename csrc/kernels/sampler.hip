// sampler.hip — grammar-constrained token selection fused with the decode-state advance.
//
// The Brain answers `format: "json"` / a JSON schema (reference chronos_sensor.py:118) by constraining every decode
// step with a token-level DFA compiled on the host (csrc/constrain/).  The DFA lives on the device:
//   next[S][V] int16   next state after emitting token v in state s, -1 = token illegal there
//   dist[S]    int16   fewest tokens that lead from s to DONE (EOS included); DONE has dist 0
// Per row b the kernel picks argmax_v score(v) over legal v with dist[next[s][v]] <= remaining[b] - 1 ("budget
// forcing": the verdict always closes within max_tokens), where score = logit (greedy) or logit / T + Gumbel noise
// (exact sampling from softmax(logit / T) via the Gumbel-max trick, counter-based RNG, so replays are reproducible),
// optionally restricted to the top-k / top-p nucleus (Ollama options) by an exact radix select on the logit keys.
//
// It then advances the per-slot decode state in place — ids, positions, context length, DFA state, budget, output
// ring — so a captured decode graph can be replayed for many steps with no host round trip.  Rows whose state is
// DONE (or < 0: -1 = empty slot, <= -2 = parked) are left untouched.
//
// Jump-forward (optional `jump[S]`): when the sampled token leads into a state whose continuation the grammar forces
// for several tokens (`, "verdict": "`), the row is parked as state -2 - s instead of s — only if its remaining
// budget can take the run: jump[s] is the budget a jump from s needs (run length + the grammar's shortest finish
// after it, 0 = no run), so a row that could not be jumped keeps decoding instead of parking at every state of the
// run and being refused each time.  A parked row is not
// live for the sampler or the decode gate; the host harvests it, appends the forced tokens in one small prefill-mode
// forward (brain/engine/engine.py Engine._jump) and resumes decoding after them.
#include "chronos_hip.h"

namespace chronos {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <typename LT>
__device__ __forceinline__ float logit_at(const LT* p, int64_t i);
template <>
__device__ __forceinline__ float logit_at<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <>
__device__ __forceinline__ float logit_at<float>(const float* p, int64_t i) { return p[i]; }

// Monotone 16-bit key of a logit (its bf16 rounding): larger key <=> larger value.  Ranks for top-k / top-p.
__device__ __forceinline__ uint32_t ord_key(float x) {
    const uint32_t b = f2bf(x);
    return (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u);
}

template <typename LT, bool VEC>
__global__ void __launch_bounds__(1024) constrained_sample_kernel(
    const LT* __restrict__ logits, int64_t lstride, const int32_t* __restrict__ row_of_slot, int vocab,
    const int16_t* __restrict__ next, const int16_t* __restrict__ dist, const int16_t* __restrict__ jump,
    int done_state, int32_t* __restrict__ state,
    int32_t* __restrict__ remaining, const float* __restrict__ temperature, const int32_t* __restrict__ seed,
    const int32_t* __restrict__ topk, const float* __restrict__ topp,
    int32_t* __restrict__ ids, int32_t* __restrict__ pos, int32_t* __restrict__ ctx, int32_t* __restrict__ nout,
    int32_t* __restrict__ out_tokens, int max_out) {
    __shared__ float bv[16];
    __shared__ int bi[16];
    __shared__ int hc[256];
    __shared__ float hm[256];
    __shared__ uint32_t sh_thr, sh_bk, sh_bp;
    __shared__ int sh_above_k;
    __shared__ float sh_above_p, sh_target_p;
    const int slot = blockIdx.x;
    const int s = state[slot];
    if (s < 0 || s == done_state) return;
    const int row = row_of_slot ? row_of_slot[slot] : slot;
    if (row < 0) return;  // slot not sampled in this launch (e.g. a prefill step that covers other slots)
    const LT* lg = logits + (int64_t)row * lstride;
    const int16_t* nx = next + (int64_t)s * vocab;
    const int budget = remaining[slot] - 1;
    const float temp = temperature ? temperature[slot] : 0.f;
    const float invt = temp > 0.f ? 1.f / temp : 0.f;
    const uint32_t key = mix32((uint32_t)(seed ? seed[slot] : 0) * 0x9E3779B9U ^ (uint32_t)nout[slot] * 0x85EBCA6BU ^
                               (uint32_t)slot);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    auto legal = [&](int v) {
        const int ns = nx[v];
        return ns >= 0 && dist[ns] <= budget;
    };

    // ---- optional top-k / top-p (llama.cpp order: on the raw logits, before temperature) -------------------------
    // Exact two-level radix select on the 16-bit keys: a 256-bin histogram of the high byte (counts and softmax mass),
    // then one of the low byte inside the bin that crosses k (resp. p * Z).  Tokens with key >= threshold survive.
    const int tk = topk ? topk[slot] : 0;
    const float tp = topp ? topp[slot] : 1.f;
    uint32_t thr = 0;
    if (temp > 0.f && (tk > 0 || tp < 1.f)) {
        float mx = -INFINITY;
        for (int v = threadIdx.x; v < vocab; v += blockDim.x)
            if (legal(v)) mx = fmaxf(mx, logit_at<LT>(lg, v));
        mx = wave_max(mx);
        if (lane == 0) bv[w] = mx;
        for (int i = threadIdx.x; i < 256; i += blockDim.x) {
            hc[i] = 0;
            hm[i] = 0.f;
        }
        __syncthreads();
        mx = bv[0];
        for (int k = 1; k < nw; ++k) mx = fmaxf(mx, bv[k]);
        for (int v = threadIdx.x; v < vocab; v += blockDim.x)
            if (legal(v)) {
                const float x = logit_at<LT>(lg, v);
                const uint32_t kk = ord_key(x) >> 8;
                atomicAdd(&hc[kk], 1);
                atomicAdd(&hm[kk], __expf(x - mx));
            }
        __syncthreads();
        if (threadIdx.x == 0) {
            float z = 0.f;
            for (int i = 0; i < 256; ++i) z += hm[i];
            int cnt = 0;
            float mass = 0.f;
            uint32_t bk = 0xFFFFFFFFu, bp = 0xFFFFFFFFu;
            for (int i = 255; i >= 0; --i) {
                if (tk > 0 && bk == 0xFFFFFFFFu && cnt + hc[i] >= tk) {
                    bk = i;
                    sh_above_k = cnt;
                }
                if (tp < 1.f && bp == 0xFFFFFFFFu && mass + hm[i] >= tp * z) {
                    bp = i;
                    sh_above_p = mass;
                }
                cnt += hc[i];
                mass += hm[i];
            }
            sh_bk = bk;
            sh_bp = bp;
            sh_target_p = tp * z;
        }
        __syncthreads();
        const uint32_t bk = sh_bk, bp = sh_bp;
        for (int i = threadIdx.x; i < 256; i += blockDim.x) {
            hc[i] = 0;
            hm[i] = 0.f;
        }
        __syncthreads();
        if (bk != 0xFFFFFFFFu || bp != 0xFFFFFFFFu) {
            for (int v = threadIdx.x; v < vocab; v += blockDim.x)
                if (legal(v)) {
                    const float x = logit_at<LT>(lg, v);
                    const uint32_t kk = ord_key(x);
                    if ((kk >> 8) == bk) atomicAdd(&hc[kk & 255], 1);
                    if ((kk >> 8) == bp) atomicAdd(&hm[kk & 255], __expf(x - mx));
                }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            if (bk != 0xFFFFFFFFu) {
                int cnt = sh_above_k;
                for (int i = 255; i >= 0; --i) {
                    cnt += hc[i];
                    if (cnt >= tk) {
                        t = (bk << 8) | (uint32_t)i;
                        break;
                    }
                }
            }
            if (bp != 0xFFFFFFFFu) {
                float mass = sh_above_p;
                for (int i = 255; i >= 0; --i) {
                    mass += hm[i];
                    if (mass >= sh_target_p) {
                        const uint32_t tpk = (bp << 8) | (uint32_t)i;
                        t = t > tpk ? t : tpk;
                        break;
                    }
                }
            }
            sh_thr = t;
        }
        __syncthreads();
        thr = sh_thr;
    }

    // ---- greedy / Gumbel-max over the legal (and, if filtered, surviving) tokens ---------------------------------
    float best = -INFINITY;
    int besti = 0x7fffffff;
    if (VEC && temp == 0.f && thr == 0 && (vocab & 7) == 0) {
        // Greedy fast path: 8 consecutive tokens per thread per iteration (16-byte loads of the DFA row and of the
        // logits), and the dependent dist[] gather only for a token that would beat this thread's best so far
        // (lazy legality; a thread walks ascending token ids, so ">" keeps the smallest id among equal maxima, and
        // the reduction below breaks cross-thread ties by id; the first legal token is always taken, as in the
        // general loop, so an all -inf row still advances).
        for (int v0 = threadIdx.x * 8; v0 < vocab; v0 += blockDim.x * 8) {
            const int4 nv = *reinterpret_cast<const int4*>(nx + v0);
            float x[8];
            if constexpr (sizeof(LT) == 2) {
                const u16x8 lv = *reinterpret_cast<const u16x8*>(reinterpret_cast<const uint16_t*>(lg) + v0);
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = bf2f(lv[j]);
            } else {
                const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(lg) + v0);
                const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(lg) + v0 + 4);
                x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
            }
            const int nw32[4] = {nv.x, nv.y, nv.z, nv.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int ns = (int)(int16_t)(nw32[j >> 1] >> (16 * (j & 1)));
                if (ns >= 0 && (x[j] > best || besti == 0x7fffffff) && dist[ns] <= budget) {
                    best = x[j];
                    besti = v0 + j;
                }
            }
        }
    } else
    for (int v = threadIdx.x; v < vocab; v += blockDim.x) {
        if (!legal(v)) continue;
        float sc = logit_at<LT>(lg, v);
        if (thr && ord_key(sc) < thr) continue;
        if (temp > 0.f) {
            const uint32_t hsh = mix32(key ^ (uint32_t)v * 0xC2B2AE35U);
            const float u = ((hsh >> 8) + 0.5f) * (1.f / 16777216.f);
            sc = sc * invt - __logf(-__logf(u));
        }
        if (sc > best || (sc == best && v < besti)) {
            best = sc;
            besti = v;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(besti, o, 64);
        if (ov > best || (ov == best && oi < besti)) {
            best = ov;
            besti = oi;
        }
    }
    __syncthreads();  // bv/bi may still be read by the top-k pass above
    if (lane == 0) {
        bv[w] = best;
        bi[w] = besti;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < nw; ++k)
            if (bv[k] > best || (bv[k] == best && bi[k] < besti)) {
                best = bv[k];
                besti = bi[k];
            }
        if (besti == 0x7fffffff) {  // no legal token at all (cannot happen with a well-formed DFA): stop the row
            state[slot] = done_state;
            return;
        }
        const int ns = nx[besti];
        const int n = nout[slot];
        if (n < max_out) out_tokens[(int64_t)slot * max_out + n] = besti;
        nout[slot] = n + 1;
        remaining[slot] = budget;
        state[slot] = (jump && ns != done_state && jump[ns] > 0 && budget >= jump[ns]) ? -2 - ns : ns;
        if (ns != done_state) {
            ids[slot] = besti;
            pos[slot] += 1;
            ctx[slot] += 1;
        }
    }
}

void launch_constrained_sample(const void* logits, bool logits_f32, int64_t lstride, const int32_t* row_of_slot,
                               int nslots, int vocab, const int16_t* next, const int16_t* dist, const int16_t* jump,
                               int done_state,
                               int32_t* state, int32_t* remaining, const float* temperature, const int32_t* seed,
                               const int32_t* topk, const float* topp, int32_t* ids, int32_t* pos, int32_t* ctx,
                               int32_t* nout, int32_t* out_tokens, int max_out, hipStream_t st) {
    if (nslots == 0) return;
    // the greedy fast path loads 16 B of each logits row and DFA row per lane: only for 16-B-aligned rows (a sliced or
    // padded logits view with another row stride takes the scalar loop)
    const size_t esz = logits_f32 ? 4 : 2;
    const bool aligned = ((uintptr_t)logits % 16 == 0) && ((size_t)lstride * esz) % 16 == 0 &&
                         ((uintptr_t)next % 16 == 0) && (vocab & 7) == 0;
    const bool vec = knob("sampler_vec", 1) != 0 && aligned;
#define CS_LAUNCH(LT, V)                                                                                        \
    hipLaunchKernelGGL((constrained_sample_kernel<LT, V>), dim3(nslots), dim3(1024), 0, st, (const LT*)logits, \
                       lstride, row_of_slot, vocab, next, dist, jump, done_state, state, remaining, temperature, seed,  \
                       topk, topp, ids, pos, ctx, nout, out_tokens, max_out)
    if (logits_f32) {
        if (vec) CS_LAUNCH(float, true); else CS_LAUNCH(float, false);
    } else {
        if (vec) CS_LAUNCH(uint16_t, true); else CS_LAUNCH(uint16_t, false);
    }
#undef CS_LAUNCH
}

}  // namespace chronos
