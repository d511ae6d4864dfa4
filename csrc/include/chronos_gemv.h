// chronos_gemv.h — host/device interface of the fused decode GEMV variants (csrc/kernels/gemv.hip), shared with the
// torch bindings.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace chronos {

// Producer side (kResid epilogue, the O / down projection of a TP=1 decode step): s = bf16(bf16(y) + rin) is
// written to rout (the new residual stream) and each workgroup's sum of s^2 per row to part_out[m * gridDim.x + wg].
// Consumer side (NORMP, the next QKV / gate_up / LM-head GEMV, whose weights have the norm weight folded in): reads s
// as its x and the producer's partials, inv = rsqrt(sum(part) / K + eps) per wave (fixed order: deterministic), and
// scales its row sums by inv — the RMSNorm costs no launch and no extra pass over x.
struct GemvNorm {
    const float* part;     // consumer: producer partials [M, nparts]
    int nparts;
    float eps;
    const uint16_t* rin;   // producer: residual in [M, N]
    uint16_t* rout;        // producer: residual out [M, N]
    float* part_out;       // producer: partials [M, gridDim.x]
    const float* wscale;   // fp8-e4m3 weights (W8A16): per-output-row scale [N]; nullptr = bf16 weights
};

struct GemvRope {
    const int32_t* pos;      // [M] positions
    const int32_t* tok_seq;  // [M] token -> block-table row
    const int32_t* bt;       // [B, bt_stride] block table
    int bt_stride;
    const float* cos_sin;    // [P, 128] f32: cos | sin
    uint16_t* q_out;         // [M, hq, 128] bf16
    void* kc;                // [NB, hkv, BS, 128] bf16 or fp8 bytes
    void* vc;                // [NB, hkv, 128, BS]
    int hq, hkv, bs;
    float k_inv, v_inv;      // fp8 cache: 1 / scale
};

// consumer: x = s (the residual stream a kResid producer wrote), nrm->part/nparts/w/eps set; rope != nullptr: QKV with
// the RoPE + paged-KV epilogue (y unused).  nrm == nullptr: plain input.
// wscale != nullptr: W is fp8-e4m3 bytes [N, K] with per-row scales (W8A16: bf16 activations, K % 1024 == 0, M <= 2)
void launch_gemv_ex(const uint16_t* x, int M, int K, const uint16_t* W, int N, uint16_t* y, bool swiglu,
                    const GemvNorm* nrm, const GemvRope* rope, bool fp8, hipStream_t st, const float* wscale = nullptr);
// producer: rout = bf16(bf16(x @ W^T) + rin), part_out[m, wg] = per-workgroup sum of rout^2; returns nparts
int launch_gemv_resid(const uint16_t* x, int M, int K, const uint16_t* W, int N, const uint16_t* rin, uint16_t* rout,
                      float* part_out, hipStream_t st, const float* wscale = nullptr);
int gemv_resid_parts(int M, int N, bool wq = false);
// W8A16 plain / SwiGLU GEMV for M <= 4 rows (jump-forward forwards of the fp8-weight model): W e4m3 bytes [N, K]
void launch_gemv_q(const uint16_t* x, int M, int K, const uint8_t* W, const float* wscale, int N, uint16_t* y,
                   bool swiglu, hipStream_t st);

}  // namespace chronos
