// sampler.hip — grammar-constrained token selection fused with the decode-state advance.
//
// The Brain answers `format: "json"` / a JSON schema (reference chronos_sensor.py:118) by constraining every decode
// step with a token-level DFA compiled on the host (csrc/constrain/).  The DFA lives on the device:
//   next[S][V] int16   next state after emitting token v in state s, -1 = token illegal there
//   dist[S]    int16   fewest tokens that lead from s to DONE (EOS included); DONE has dist 0
// Per row b the kernel picks argmax_v score(v) over legal v with dist[next[s][v]] <= remaining[b] - 1 ("budget
// forcing": the verdict always closes within max_tokens), where score = logit (greedy) or logit / T + Gumbel noise
// (exact sampling from softmax(logit / T) via the Gumbel-max trick, counter-based RNG, so replays are reproducible).
//
// It then advances the per-slot decode state in place — ids, positions, context length, DFA state, budget, output
// ring — so a captured decode graph can be replayed for many steps with no host round trip.  Rows whose state is
// DONE (or < 0 = empty slot) are left untouched.
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

template <typename LT>
__global__ void __launch_bounds__(1024) constrained_sample_kernel(
    const LT* __restrict__ logits, int64_t lstride, const int32_t* __restrict__ row_of_slot, int vocab,
    const int16_t* __restrict__ next, const int16_t* __restrict__ dist, int done_state, int32_t* __restrict__ state,
    int32_t* __restrict__ remaining, const float* __restrict__ temperature, const int32_t* __restrict__ seed,
    int32_t* __restrict__ ids, int32_t* __restrict__ pos, int32_t* __restrict__ ctx, int32_t* __restrict__ nout,
    int32_t* __restrict__ out_tokens, int max_out) {
    __shared__ float bv[16];
    __shared__ int bi[16];
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

    float best = -INFINITY;
    int besti = 0x7fffffff;
    for (int v = threadIdx.x; v < vocab; v += blockDim.x) {
        const int ns = nx[v];
        if (ns < 0 || dist[ns] > budget) continue;
        float sc = logit_at<LT>(lg, v);
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
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
        bv[w] = best;
        bi[w] = besti;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nw = blockDim.x >> 6;
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
        state[slot] = ns;
        if (ns != done_state) {
            ids[slot] = besti;
            pos[slot] += 1;
            ctx[slot] += 1;
        }
    }
}

void launch_constrained_sample(const void* logits, bool logits_f32, int64_t lstride, const int32_t* row_of_slot,
                               int nslots, int vocab, const int16_t* next, const int16_t* dist, int done_state,
                               int32_t* state, int32_t* remaining, const float* temperature, const int32_t* seed,
                               int32_t* ids, int32_t* pos, int32_t* ctx, int32_t* nout, int32_t* out_tokens,
                               int max_out, hipStream_t st) {
    if (nslots == 0) return;
    if (logits_f32)
        hipLaunchKernelGGL(constrained_sample_kernel<float>, dim3(nslots), dim3(1024), 0, st,
                           (const float*)logits, lstride, row_of_slot, vocab, next, dist, done_state, state, remaining,
                           temperature, seed, ids, pos, ctx, nout, out_tokens, max_out);
    else
        hipLaunchKernelGGL(constrained_sample_kernel<uint16_t>, dim3(nslots), dim3(1024), 0, st,
                           (const uint16_t*)logits, lstride, row_of_slot, vocab, next, dist, done_state, state,
                           remaining, temperature, seed, ids, pos, ctx, nout, out_tokens, max_out);
}

}  // namespace chronos
