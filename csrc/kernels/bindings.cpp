// bindings.cpp — registers the gfx950 HIP kernels as torch operators (torch.ops.chronos.*).
//
// Every op checks dtype/shape/contiguity on the host BEFORE launching (a bad launch geometry on a hand-written kernel
// can fault the whole GPU box), launches on the current HIP stream (so ops are hipGraph-capturable), and never
// allocates inside a captured region except through torch's caching allocator.
#include <ATen/ATen.h>
// ROCm torch presents HIP devices as DeviceType::CUDA ("masquerading"): guards/streams must use these forms.
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <tuple>
#include <string>
#include <unordered_map>
#include <vector>
#include <cstring>

#include "chronos_gemv.h"
#include "chronos_gemm.h"

namespace chronos {
void launch_embedding(const int32_t*, const uint16_t*, uint16_t*, int, int, int64_t, int64_t, hipStream_t);
void launch_rmsnorm(const uint16_t*, uint16_t*, const uint16_t*, uint16_t*, int, int, float, hipStream_t);
void launch_rope_kv_write(const uint16_t*, const int32_t*, const int32_t*, const int32_t*, int, const float*,
                          uint16_t*, void*, void*, int, int, int, int, int, bool, float, float, hipStream_t);
void launch_silu_mul(const uint16_t*, uint16_t*, int64_t, int, hipStream_t);
size_t paged_attn_smem(int nqt);
bool launch_decode_attn_rope(const uint16_t*, const int32_t*, const float*, void*, void*, const int32_t*, int,
                             const int32_t*, uint16_t*, int, int, int, int, float, hipStream_t, const int32_t*,
                             uint16_t*, float*);
void launch_paged_attn(const uint16_t*, const void*, const void*, const int32_t*, int, const int32_t*,
                       const int32_t*, const int32_t*, int, int, int, uint16_t*, float*, float*, int, int, int, float,
                       bool, float, float, hipStream_t, int);
void launch_constrained_sample(const void*, bool, int64_t, const int32_t*, int, int, const int16_t*, const int16_t*,
                               const int16_t*, int, int32_t*, int32_t*, const float*, const int32_t*, const int32_t*, const float*,
                               int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, int, hipStream_t);
void launch_gemv(const uint16_t*, int, int, const uint16_t*, int, uint16_t*, bool, hipStream_t);
void attn_init();
void launch_gemm(const uint16_t*, const uint16_t*, uint16_t*, int, int, int, bool, int, hipStream_t);
void* ar_create(int, int, int64_t);
std::vector<uint8_t> ar_handles(void*);
void ar_open(void*, const std::vector<std::vector<uint8_t>>&);
void ar_run(void*, const uint16_t*, uint16_t*, int64_t, int64_t, int, hipStream_t);
void ar_run_norm(void*, const uint16_t*, uint16_t*, const uint16_t*, uint16_t*, int64_t, int, float, int64_t,
                 hipStream_t);
uint32_t ar_error(void*);
int64_t ar_capacity(void*);
void ar_destroy(void*);
void launch_attn_prefill(const uint16_t*, const void*, const void*, const int32_t*, int, const int32_t*,
                         const int32_t*, const int32_t*, int, uint16_t*, int, int, int, float, bool, float, float,
                         hipStream_t);
void launch_quant_rows(const uint16_t*, uint16_t*, const uint16_t*, uint8_t*, float*, int, int, float, int,
                       hipStream_t);
void launch_qlinear(const uint8_t*, const float*, const uint8_t*, const float*, uint16_t*, int, int, int, bool,
                    hipStream_t);
}  // namespace chronos

namespace chronos {
// decode early-exit gate (chronos_hip.h): read by the launchers, baked into captured graphs as kernel arguments
const int32_t* g_gate_state = nullptr;
int g_gate_n = 0;

namespace {
std::mutex g_knob_mu;
std::unordered_map<std::string, int> g_knobs;
}  // namespace

int resident_workgroups_of(const void* kernel, int threads) {
    static std::mutex mu;
    static std::unordered_map<const void*, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(kernel);
    if (it != cache.end()) return it->second;
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0);
    const int v = per_cu > 0 && cus > 0 ? per_cu * cus : 256;
    cache[kernel] = v;
    return v;
}

int knob(const char* name, int dflt) {
    std::lock_guard<std::mutex> lk(g_knob_mu);
    auto it = g_knobs.find(name);
    if (it != g_knobs.end()) return it->second;
    std::string env = "CHRONOS_";
    for (const char* c = name; *c; ++c) env += (char)toupper(*c);
    const char* e = getenv(env.c_str());
    const int v = e ? atoi(e) : dflt;
    g_knobs[name] = v;
    return v;
}
}  // namespace chronos

namespace {

using at::Tensor;

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
inline const uint16_t* bf(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
inline uint16_t* bfm(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
inline const int32_t* i32(const Tensor& t) { return t.data_ptr<int32_t>(); }
inline int32_t* i32m(const Tensor& t) { return t.data_ptr<int32_t>(); }

#define CHK(c, msg) TORCH_CHECK((c), "chronos: ", msg)
inline void chk_gpu(const Tensor& t, const char* n) {
    CHK(t.is_cuda(), std::string(n) + " must be a GPU tensor");
    CHK(t.is_contiguous(), std::string(n) + " must be contiguous");
}
inline void chk_bf16(const Tensor& t, const char* n) {
    chk_gpu(t, n);
    CHK(t.scalar_type() == at::kBFloat16, std::string(n) + " must be bfloat16");
}
inline void chk_i32(const Tensor& t, const char* n) {
    chk_gpu(t, n);
    CHK(t.scalar_type() == at::kInt, std::string(n) + " must be int32");
}

// Decode GEMV weights: bf16 [N, K], or (ws given) fp8-e4m3 bytes [N, K] with per-row f32 scales [N] (W8A16: the
// fp8-weight model's decode step keeps bf16 activations; csrc/kernels/gemv.hip WQ).  Returns the scale pointer.
inline const float* chk_gemv_w(const Tensor& w, const c10::optional<Tensor>& ws, int64_t K, int64_t M) {
    chk_gpu(w, "w");
    if (!ws.has_value()) {
        CHK(w.scalar_type() == at::kBFloat16, "w must be bfloat16 (or uint8 e4m3 with ws)");
        return nullptr;
    }
    chk_gpu(*ws, "ws");
    CHK(w.scalar_type() == at::kByte, "w must be uint8 (e4m3 bytes) when ws is given");
    CHK(ws->scalar_type() == at::kFloat && ws->numel() == w.size(0), "ws must be [N] f32");
    CHK(K % 1024 == 0 && M <= 4, "fp8-weight GEMV: K % 1024 == 0, M <= 4 (the fused epilogues: M <= 2)");
    return ws->data_ptr<float>();
}

// KV caches are bf16 or fp8-e4m3 stored as uint8 (OCP e4m3fn bytes; dequantised with a per-layer scale)
inline bool chk_kv(const Tensor& k, const Tensor& v) {
    chk_gpu(k, "k_cache");
    chk_gpu(v, "v_cache");
    CHK(k.scalar_type() == v.scalar_type(), "k/v cache dtypes differ");
    CHK(k.scalar_type() == at::kBFloat16 || k.scalar_type() == at::kByte, "kv cache must be bf16 or uint8 (fp8 e4m3)");
    return k.scalar_type() == at::kByte;
}

Tensor embedding(const Tensor& ids, const Tensor& table, int64_t vstart) {
    chk_i32(ids, "ids");
    chk_bf16(table, "table");
    CHK(table.dim() == 2 && table.size(1) % 8 == 0, "table must be [V, d] with d % 8 == 0");
    c10::hip::HIPGuardMasqueradingAsCUDA g(ids.device());
    auto out = at::empty({ids.numel(), table.size(1)}, table.options());
    chronos::launch_embedding(i32(ids), bf(table), bfm(out), (int)ids.numel(), (int)table.size(1), vstart,
                              table.size(0), cur_stream());
    return out;
}

Tensor rmsnorm(const Tensor& x, const Tensor& w, double eps) {
    chk_bf16(x, "x");
    chk_bf16(w, "w");
    const int64_t d = x.size(-1);
    CHK(w.numel() == d && d % 8 == 0 && d <= 16384, "rmsnorm: d must match w, be % 8 and <= 16384");
    c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
    auto y = at::empty_like(x);
    chronos::launch_rmsnorm(bf(x), nullptr, bf(w), bfm(y), (int)(x.numel() / d), (int)d, (float)eps, cur_stream());
    return y;
}

// resid <- bf16(x + resid); returns rmsnorm(resid) * w
Tensor add_rmsnorm(const Tensor& x, const Tensor& resid, const Tensor& w, double eps) {
    chk_bf16(x, "x");
    chk_bf16(resid, "resid");
    chk_bf16(w, "w");
    const int64_t d = x.size(-1);
    CHK(resid.sizes() == x.sizes(), "add_rmsnorm: shape mismatch");
    CHK(w.numel() == d && d % 8 == 0 && d <= 16384, "add_rmsnorm: d must match w, be % 8 and <= 16384");
    c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
    auto y = at::empty_like(x);
    chronos::launch_rmsnorm(bf(x), bfm(resid), bf(w), bfm(y), (int)(x.numel() / d), (int)d, (float)eps, cur_stream());
    return y;
}

void rope_kv_write(const Tensor& qkv, const Tensor& pos, const Tensor& tok_seq, const Tensor& block_table,
                   const Tensor& cos_sin, const Tensor& q_out, const Tensor& k_cache, const Tensor& v_cache, int64_t hq,
                   int64_t hkv, bool write_q, double k_scale, double v_scale) {
    chk_bf16(qkv, "qkv");
    chk_i32(pos, "pos");
    chk_i32(tok_seq, "tok_seq");
    chk_i32(block_table, "block_table");
    chk_gpu(cos_sin, "cos_sin");
    CHK(cos_sin.scalar_type() == at::kFloat && cos_sin.dim() == 2 && cos_sin.size(1) == 128, "cos_sin [P,128] f32");
    chk_bf16(q_out, "q_out");
    const bool fp8 = chk_kv(k_cache, v_cache);
    const int64_t t = qkv.size(0);
    CHK(qkv.dim() == 2 && qkv.size(1) == (hq + 2 * hkv) * 128, "qkv must be [T, (hq+2hkv)*128]");
    CHK(pos.numel() == t && tok_seq.numel() == t, "pos/tok_seq must have T entries");
    CHK(!write_q || q_out.numel() >= t * hq * 128, "q_out too small");
    CHK(k_cache.dim() == 4 && k_cache.size(1) == hkv && k_cache.size(3) == 128, "k_cache [NB, hkv, BS, 128]");
    CHK(v_cache.dim() == 4 && v_cache.size(1) == hkv && v_cache.size(2) == 128 && v_cache.size(3) == k_cache.size(2),
        "v_cache [NB, hkv, 128, BS]");
    CHK(block_table.dim() == 2, "block_table [B, max_blocks]");
    c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
    chronos::launch_rope_kv_write(bf(qkv), i32(pos), i32(tok_seq), i32(block_table), (int)block_table.size(1),
                                  cos_sin.data_ptr<float>(), bfm(q_out), k_cache.data_ptr(), v_cache.data_ptr(), (int)t,
                                  (int)hq, (int)hkv, (int)k_cache.size(2), write_q ? 1 : 0, fp8, (float)k_scale,
                                  (float)v_scale, cur_stream());
}

// Decode step attention with RoPE + paged-KV write fused in (attention.hip paged_decode_kernel<..., RP = true>).
// Returns the [n, hq, 128] attention output, or an empty tensor when the fused kernel does not serve this shape (the
// caller then runs rope_kv_write + paged_attention).  Decode rows only: row i is sequence i, its one token at pos[i]
// is the last of its context (ctx_len[i] == pos[i] + 1).
// casc (optional, int32 [1 + P_max] on the device: P, then the shared prefix's block ids) with casc_o (bf16 [>= n, hq,
// 128]) and casc_l (f32 [>= n, hq]) scratch: cascade attention over the shared prefix (attention.hip
// casc_prefix_kernel) merged into the decode kernel.  casc[0] = 0 turns it off without re-capturing a graph.
Tensor decode_attention_rope(const Tensor& qkv, const Tensor& pos, const Tensor& cos_sin, const Tensor& k_cache,
                             const Tensor& v_cache, const Tensor& block_table, const Tensor& ctx_len, int64_t n,
                             int64_t hq, double scale, const c10::optional<Tensor>& casc,
                             const c10::optional<Tensor>& casc_o, const c10::optional<Tensor>& casc_l) {
    chk_bf16(qkv, "qkv");
    chk_i32(pos, "pos");
    chk_i32(block_table, "block_table");
    chk_i32(ctx_len, "ctx_len");
    chk_gpu(cos_sin, "cos_sin");
    CHK(cos_sin.scalar_type() == at::kFloat && cos_sin.dim() == 2 && cos_sin.size(1) == 128, "cos_sin [P,128] f32");
    const bool fp8 = chk_kv(k_cache, v_cache);
    const int64_t hkv = k_cache.size(1), bs = k_cache.size(2);
    CHK(qkv.dim() == 2 && qkv.size(0) >= n && qkv.size(1) == (hq + 2 * hkv) * 128, "qkv must be [>=n, (hq+2hkv)*128]");
    CHK(pos.numel() >= n && ctx_len.numel() >= n && block_table.dim() == 2 && block_table.size(0) >= n,
        "pos / ctx_len / block_table need n rows");
    CHK(hq % hkv == 0 && 16 % (hq / hkv) == 0, "GQA group Hq/Hkv must divide 16");
    CHK(k_cache.dim() == 4 && k_cache.size(3) == 128 && v_cache.size(2) == 128 && v_cache.size(3) == bs,
        "k_cache [NB, hkv, BS, 128], v_cache [NB, hkv, 128, BS]");
    c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
    if (fp8) return at::empty({0}, qkv.options());
    const int32_t* cp = nullptr;
    uint16_t* co = nullptr;
    float* cl = nullptr;
    if (casc.has_value()) {
        chk_i32(*casc, "casc");
        CHK(casc_o.has_value() && casc_l.has_value(), "casc needs casc_o and casc_l");
        chk_bf16(*casc_o, "casc_o");
        chk_gpu(*casc_l, "casc_l");
        CHK(casc->numel() >= 2 && casc->numel() <= 65, "casc: [1 + P_max], P_max <= 64");
        CHK(casc_o->numel() >= n * hq * 128 && casc_l->scalar_type() == at::kFloat && casc_l->numel() >= n * hq,
            "casc_o [>= n, hq, 128] bf16, casc_l [>= n, hq] f32");
        cp = i32(*casc);
        co = bfm(*casc_o);
        cl = casc_l->data_ptr<float>();
    }
    auto out = at::empty({n, hq, 128}, qkv.options());
    if (!chronos::launch_decode_attn_rope(bf(qkv), i32(pos), cos_sin.data_ptr<float>(), k_cache.data_ptr(),
                                          v_cache.data_ptr(), i32(block_table), (int)block_table.size(1), i32(ctx_len),
                                          bfm(out), (int)n, (int)hq, (int)hkv, (int)bs, (float)scale, cur_stream(),
                                          cp, co, cl))
        return at::empty({0}, qkv.options());
    return out;
}

Tensor silu_mul(const Tensor& gu) {
    chk_bf16(gu, "gate_up");
    const int64_t f2 = gu.size(-1);
    CHK(f2 % 16 == 0, "gate_up last dim must be 2F with F % 8 == 0");
    c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
    auto sizes = gu.sizes().vec();
    sizes.back() = f2 / 2;
    auto out = at::empty(sizes, gu.options());
    chronos::launch_silu_mul(bf(gu), bfm(out), gu.numel() / f2, (int)(f2 / 2), cur_stream());
    return out;
}

Tensor paged_attention(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_table,
                       const Tensor& q_start, const Tensor& ctx_len, const c10::optional<Tensor>& tiles,
                       int64_t ntiles, int64_t nqt, int64_t nsplit, double scale, double k_scale, double v_scale,
                       int64_t max_q) {
    chk_bf16(q, "q");
    const bool fp8 = chk_kv(k_cache, v_cache);
    chk_i32(block_table, "block_table");
    chk_i32(q_start, "q_start");
    chk_i32(ctx_len, "ctx_len");
    CHK(q.dim() == 3 && q.size(2) == 128, "q must be [T, Hq, 128]");
    const int64_t hq = q.size(1), hkv = k_cache.size(1), bs = k_cache.size(2);
    CHK(hq % hkv == 0 && 16 % (hq / hkv) == 0, "GQA group Hq/Hkv must divide 16");
    CHK(bs % 16 == 0, "block size must be a multiple of 16");
    CHK(v_cache.size(2) == 128 && v_cache.size(3) == bs, "v_cache [NB, hkv, 128, BS]");
    CHK(nqt == 1 || nqt == 2 || nqt == 8, "nqt must be 1, 2 (split-K paged kernel) or 8 (flash prefill)");
    CHK(nsplit >= 1 && nsplit <= 256, "nsplit in [1, 256]");
    const int32_t* tp = nullptr;
    if (tiles.has_value()) {
        chk_i32(*tiles, "tiles");
        CHK(tiles->numel() >= 2 * ntiles, "tiles must be [ntiles, 2]");
        tp = i32(*tiles);
    } else if (max_q > 1) {
        CHK(nqt == 1 && max_q * (hq / hkv) <= 16 && bs == 16, "multi-token decode: nqt 1, max_q x GQA group <= 16");
        CHK(q_start.numel() >= ntiles + 1 && ctx_len.numel() >= ntiles, "multi-token decode: q_start [B + 1], ctx [B]");
    } else {
        CHK(ctx_len.numel() >= ntiles && q.size(0) >= ntiles, "decode mode: one query token per tile");
    }
    c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
    auto out = at::empty_like(q);
    Tensor po, pl;
    if (nsplit > 1 && nqt != 8) {
        const int64_t rows = nsplit * ntiles * hkv * nqt * 16;
        po = at::empty({rows, 128}, q.options().dtype(at::kFloat));
        pl = at::empty({rows}, q.options().dtype(at::kFloat));
    }
    if (nqt == 8) {  // flash prefill kernel: 128 query rows per workgroup, K/V tiles shared through LDS
        CHK(tp != nullptr, "nqt=8 (flash prefill) needs a tile list");
        chronos::launch_attn_prefill(bf(q), k_cache.data_ptr(), v_cache.data_ptr(), i32(block_table),
                                     (int)block_table.size(1), i32(q_start), i32(ctx_len), tp, (int)ntiles, bfm(out),
                                     (int)hq, (int)hkv, (int)bs, (float)scale, fp8, (float)k_scale, (float)v_scale,
                                     cur_stream());
        return out;
    }
    chronos::launch_paged_attn(bf(q), k_cache.data_ptr(), v_cache.data_ptr(), i32(block_table),
                               (int)block_table.size(1), i32(q_start), i32(ctx_len), tp, (int)ntiles, (int)nqt,
                               (int)nsplit, bfm(out), nsplit > 1 ? po.data_ptr<float>() : nullptr,
                               nsplit > 1 ? pl.data_ptr<float>() : nullptr, (int)hq, (int)hkv, (int)bs, (float)scale,
                               fp8, (float)k_scale, (float)v_scale, cur_stream(), (int)max_q);
    return out;
}

void constrained_sample(const Tensor& logits, const c10::optional<Tensor>& row_of_slot, const Tensor& next,
                        const Tensor& dist, int64_t done_state, const Tensor& state, const Tensor& remaining,
                        const c10::optional<Tensor>& temperature, const c10::optional<Tensor>& seed, const Tensor& ids,
                        const Tensor& pos, const Tensor& ctx, const Tensor& nout, const Tensor& out_tokens,
                        const c10::optional<Tensor>& topk, const c10::optional<Tensor>& topp,
                        const c10::optional<Tensor>& jump) {
    CHK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits [rows, V] row-contiguous");
    CHK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat, "logits bf16 or f32");
    chk_gpu(next, "next");
    CHK(next.scalar_type() == at::kShort && next.dim() == 2, "next must be int16 [S, V]");
    CHK(dist.scalar_type() == at::kShort && dist.numel() == next.size(0), "dist must be int16 [S]");
    const int64_t vocab = next.size(1);
    CHK(logits.size(1) >= vocab, "logits narrower than the DFA vocabulary");
    chk_i32(state, "state");
    const int64_t n = state.numel();
    for (const Tensor* t : {&remaining, &ids, &pos, &ctx, &nout}) {
        chk_i32(*t, "slot tensor");
        CHK(t->numel() >= n, "slot tensors must have one entry per slot");
    }
    chk_i32(out_tokens, "out_tokens");
    CHK(out_tokens.dim() == 2 && out_tokens.size(0) >= n, "out_tokens [slots, max_out]");
    const int32_t* rp = nullptr;
    if (row_of_slot.has_value()) {
        chk_i32(*row_of_slot, "row_of_slot");
        rp = i32(*row_of_slot);
    } else {
        CHK(logits.size(0) >= n, "one logits row per slot");
    }
    const float* tp = nullptr;
    if (temperature.has_value()) {
        chk_gpu(*temperature, "temperature");
        CHK(temperature->scalar_type() == at::kFloat, "temperature f32");
        tp = temperature->data_ptr<float>();
    }
    const int32_t* sp = nullptr;
    if (seed.has_value()) {
        chk_i32(*seed, "seed");
        sp = i32(*seed);
    }
    const int32_t* kp = nullptr;
    if (topk.has_value()) {
        chk_i32(*topk, "topk");
        CHK(topk->numel() >= n, "topk: one entry per slot");
        kp = i32(*topk);
    }
    const float* pp = nullptr;
    if (topp.has_value()) {
        chk_gpu(*topp, "topp");
        CHK(topp->scalar_type() == at::kFloat && topp->numel() >= n, "topp: f32, one entry per slot");
        pp = topp->data_ptr<float>();
    }
    const int16_t* jp = nullptr;
    if (jump.has_value()) {
        chk_gpu(*jump, "jump");
        CHK(jump->scalar_type() == at::kShort && jump->numel() == next.size(0), "jump must be int16 [S]");
        jp = jump->data_ptr<int16_t>();
    }
    c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
    chronos::launch_constrained_sample(logits.data_ptr(), logits.scalar_type() == at::kFloat, logits.stride(0), rp,
                                       (int)n, (int)vocab, next.data_ptr<int16_t>(), dist.data_ptr<int16_t>(), jp,
                                       (int)done_state, i32m(state), i32m(remaining), tp, sp, kp, pp, i32m(ids),
                                       i32m(pos), i32m(ctx), i32m(nout), i32m(out_tokens), (int)out_tokens.size(1),
                                       cur_stream());
}

// y = x @ w.T for M <= 8 rows (decode); swiglu: w = [gate; up] -> y = silu(x@gate.T) * (x@up.T)
Tensor gemv(const Tensor& x, const Tensor& w, bool swiglu, const c10::optional<Tensor>& ws) {
    chk_bf16(x, "x");
    const int64_t K = x.size(-1), M = x.numel() / K, N = w.size(0);
    const float* wsc = chk_gemv_w(w, ws, K, M);
    CHK(w.dim() == 2 && w.size(1) == K, "gemv: w must be [N, K]");
    CHK(M >= 1 && M <= 8, "gemv: 1 <= M <= 8");
    CHK(K % 512 == 0, "gemv: K % 512 == 0");
    CHK(N % 16 == 0, "gemv: N % 16 == 0");
    c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
    auto y = at::empty({M, swiglu ? N / 2 : N}, x.options());
    if (wsc)
        chronos::launch_gemv_q(bf(x), (int)M, (int)K, reinterpret_cast<const uint8_t*>(w.data_ptr()), wsc, (int)N,
                               bfm(y), swiglu, cur_stream());
    else
        chronos::launch_gemv(bf(x), (int)M, (int)K, bf(w), (int)N, bfm(y), swiglu, cur_stream());
    return y;
}

// Decode gate: state = the engine's slot-state vector (int32, >= n rows); n in [1, 8] arms it for the launches that
// follow, n = 0 disarms.  Only decode steps of a small bucket arm it (a prefill or a large bucket never does).
void set_decode_gate(const c10::optional<Tensor>& state, int64_t n) {
    if (!state.has_value() || n <= 0) {
        chronos::g_gate_state = nullptr;
        chronos::g_gate_n = 0;
        return;
    }
    chk_i32(*state, "gate state");
    CHK(n <= 8 && state->numel() >= n, "decode gate: 1 <= n <= 8 and n <= numel(state)");
    chronos::g_gate_state = i32(*state);
    chronos::g_gate_n = (int)n;
}

// Decode producer (O / down projection at TP=1, M <= 2): resid_out = bf16(bf16(x @ w.T) + resid_in); returns the
// per-workgroup sums of resid_out^2 [M, P] f32 that the consuming GEMV's norm prologue reduces (chronos_gemv.h).
Tensor gemv_resid(const Tensor& x, const Tensor& w, const Tensor& resid_in, const Tensor& resid_out,
                  const c10::optional<Tensor>& ws) {
    chk_bf16(x, "x");
    chk_bf16(resid_in, "resid_in");
    chk_bf16(resid_out, "resid_out");
    const int64_t K = x.size(-1), M = x.numel() / K, N = w.size(0);
    const float* wsc = chk_gemv_w(w, ws, K, M);
    CHK(w.dim() == 2 && w.size(1) == K, "gemv_resid: w must be [N, K]");
    CHK(M >= 1 && M <= 2 && K % 512 == 0 && N % 16 == 0, "gemv_resid: M <= 2, K % 512, N % 16");
    CHK(resid_in.numel() == M * N && resid_out.numel() == M * N, "gemv_resid: residuals must be [M, N]");
    CHK(resid_in.data_ptr() != resid_out.data_ptr(), "gemv_resid: out of place only");
    c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
    CHK(wsc == nullptr || M <= 2, "gemv_resid: M <= 2");
    auto part = at::empty({M, chronos::gemv_resid_parts((int)M, (int)N, wsc != nullptr)}, x.options().dtype(at::kFloat));
    chronos::launch_gemv_resid(bf(x), (int)M, (int)K, bf(w), (int)N, bf(resid_in), bfm(resid_out),
                               part.data_ptr<float>(), cur_stream(), wsc);
    return part;
}

inline chronos::GemvNorm normp_args(const Tensor& s, const Tensor& part, double eps, int64_t M) {
    chk_gpu(part, "part");
    CHK(part.scalar_type() == at::kFloat && part.dim() == 2 && part.size(0) == M, "part must be [M, P] f32");
    CHK(part.size(1) % 4 == 0 && part.size(1) <= (M == 1 ? 2048 : 1024),
        "part: P % 4 == 0, P <= 2048 (one row) / 1024 (two rows)");
    (void)s;
    chronos::GemvNorm n{};
    n.part = part.data_ptr<float>();
    n.nparts = (int)part.size(1);
    n.eps = (float)eps;
    return n;
}

// Decode consumer: y = rmsnorm(s) @ w.T for a projection w whose norm weight is folded in (models/llama.py
// fold_norm), the norm's sum of squares taken from a gemv_resid producer's partials (swiglu: gate/up pair ->
// silu(g) * u).  s: [M, K], M <= 2.
Tensor gemv_normp(const Tensor& s, const Tensor& part, double eps, const Tensor& w, bool swiglu,
                  const c10::optional<Tensor>& ws) {
    chk_bf16(s, "s");
    const int64_t K = s.size(-1), M = s.numel() / K, N = w.size(0);
    const float* wsc = chk_gemv_w(w, ws, K, M);
    CHK(w.dim() == 2 && w.size(1) == K, "gemv_normp: w must be [N, K]");
    CHK(M >= 1 && M <= 2 && K % 512 == 0 && N % 16 == 0, "gemv_normp: M <= 2, K % 512, N % 16");
    const chronos::GemvNorm n = normp_args(s, part, eps, M);
    c10::hip::HIPGuardMasqueradingAsCUDA g(s.device());
    auto y = at::empty({M, swiglu ? N / 2 : N}, s.options());
    chronos::launch_gemv_ex(bf(s), (int)M, (int)K, bf(w), (int)N, bfm(y), swiglu, &n, nullptr, false, cur_stream(),
                            wsc);
    return y;
}

// Decode QKV projection with the RoPE + paged-KV epilogue (rope_kv_write's semantics): q -> q_out, k/v -> the caches.
// part given: x is the residual stream s and the (folded) input RMSNorm is fused as in gemv_normp; else x is the
// normalised input.  M <= 2 tokens, token m belongs to block-table row tok_seq[m].
void qkv_rope(const Tensor& x, const c10::optional<Tensor>& part, double eps,
              const Tensor& w, const Tensor& pos, const Tensor& tok_seq, const Tensor& block_table,
              const Tensor& cos_sin, const Tensor& q_out, const Tensor& k_cache, const Tensor& v_cache, int64_t hq,
              int64_t hkv, double k_scale, double v_scale, const c10::optional<Tensor>& ws) {
    chk_bf16(x, "x");
    chk_i32(pos, "pos");
    chk_i32(tok_seq, "tok_seq");
    chk_i32(block_table, "block_table");
    chk_gpu(cos_sin, "cos_sin");
    CHK(cos_sin.scalar_type() == at::kFloat && cos_sin.dim() == 2 && cos_sin.size(1) == 128, "cos_sin [P,128] f32");
    chk_bf16(q_out, "q_out");
    const bool fp8 = chk_kv(k_cache, v_cache);
    const int64_t K = x.size(-1), M = x.numel() / K, N = w.size(0);
    const float* wsc = chk_gemv_w(w, ws, K, M);
    CHK(M >= 1 && M <= 2 && K % 512 == 0, "qkv_rope: M <= 2, K % 512 == 0");
    CHK(w.dim() == 2 && w.size(1) == K && N == (hq + 2 * hkv) * 128, "w must be [(hq+2hkv)*128, K]");
    CHK(pos.numel() >= M && tok_seq.numel() >= M && q_out.numel() >= M * hq * 128, "pos/tok_seq/q_out too small");
    CHK(k_cache.dim() == 4 && k_cache.size(1) == hkv && k_cache.size(3) == 128, "k_cache [NB, hkv, BS, 128]");
    CHK(v_cache.dim() == 4 && v_cache.size(1) == hkv && v_cache.size(2) == 128 && v_cache.size(3) == k_cache.size(2),
        "v_cache [NB, hkv, 128, BS]");
    CHK(block_table.dim() == 2, "block_table [B, max_blocks]");
    chronos::GemvNorm n{};
    if (part.has_value()) n = normp_args(x, *part, eps, M);
    c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
    chronos::GemvRope rp{i32(pos), i32(tok_seq), i32(block_table), (int)block_table.size(1), cos_sin.data_ptr<float>(),
                         bfm(q_out), k_cache.data_ptr(), v_cache.data_ptr(), (int)hq, (int)hkv, (int)k_cache.size(2),
                         (float)(1.0 / k_scale), (float)(1.0 / v_scale)};
    chronos::launch_gemv_ex(bf(x), (int)M, (int)K, bf(w), (int)N, nullptr, false, part.has_value() ? &n : nullptr,
                            &rp, fp8, cur_stream(), wsc);
}

// y = x @ w.T on MFMA (gemm.hip); swiglu as gemv.  stages = depth of the LDS-DMA ring (2..4)
Tensor gemm(const Tensor& x, const Tensor& w, bool swiglu, int64_t stages) {
    chk_bf16(x, "x");
    chk_bf16(w, "w");
    const int64_t K = x.size(-1), M = x.numel() / K, N = w.size(0);
    CHK(w.dim() == 2 && w.size(1) == K, "gemm: w must be [N, K]");
    CHK(K % 64 == 0, "gemm: K % 64 == 0");
    CHK(N % 128 == 0, "gemm: N % 128 == 0");
    CHK(M < (1LL << 31) / 128 && N * K < (1LL << 40), "gemm: size");
    CHK(stages >= 2 && stages <= 4, "gemm: stages in [2, 4]");
    c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
    auto y = at::empty({M, swiglu ? N / 2 : N}, x.options());
    chronos::launch_gemm(bf(x), bf(w), bfm(y), (int)M, (int)N, (int)K, swiglu, (int)stages, cur_stream());
    return y;
}


// Split-K tickets: one zeroed int buffer per (device, stream), at least n long; every call leaves it zeroed (each
// group's last arriver resets its own counter), so calls on one stream — and graph replays — share it.
static int32_t* split_tickets(const Tensor& x, int64_t n) {
    static std::mutex mu;
    static std::unordered_map<int64_t, Tensor> cnts;
    std::lock_guard<std::mutex> lk(mu);
    const int64_t key = ((int64_t)x.get_device() << 48) ^ (int64_t)(intptr_t)cur_stream();
    auto it = cnts.find(key);
    if (it == cnts.end() || it->second.numel() < n)
        it = cnts.insert_or_assign(key, at::zeros({std::max<int64_t>(n, 1 << 16)}, x.options().dtype(at::kInt))).first;
    return it->second.data_ptr<int32_t>();
}

// Batched projection GEMM family (gemm_pp.hip): y = x @ w.T with a fused epilogue, M >= 3.
//   mode 0 plain (y [M, N]); 1 swiglu (w = [gate; up] [2F, K], y [M, F] = silu(x Wg^T) * (x Wu^T)); 2 resid (y = the
//   new residual stream bf16(bf16(x @ w.T) + resid), second output = per-row partial sums of y^2 [M, N / (BN/4)]).
//   part_in given (modes 0/1): x is the raw residual stream s and the folded input RMSNorm is applied as the per-row
//   scale rsqrt(sum(part_in[m]) / K + eps).  cfg = tile config (gemm_pp_bm / gemm_pp_bn), splitk divides K / 64.
std::tuple<Tensor, Tensor> gemm_pp(const Tensor& x, const Tensor& w, int64_t mode, int64_t cfg, int64_t splitk,
                                   const c10::optional<Tensor>& resid, const c10::optional<Tensor>& part_in,
                                   double eps, bool prio) {
    chk_bf16(x, "x");
    chk_bf16(w, "w");
    const int64_t K = x.size(-1), M = x.numel() / K, N = w.size(0);
    CHK(w.dim() == 2 && w.size(1) == K, "gemm_pp: w must be [N, K]");
    const bool lg = cfg >= chronos::kPPConfigs;  // gemm_lg.hip configs continue the id space
    // 40-71: gemm_lg's timing-only ablations (wrong results by design), rejected unless built in
    CHK((cfg >= 0 && cfg < chronos::kPPConfigs + chronos::kLGConfigs) ||
            (chronos::gemm_lg_ablations_built() && cfg >= 40 && cfg < 72) ||
            (cfg >= chronos::kLGTinyFirst && cfg < chronos::kLGTinyFirst + chronos::kLGTinyConfigs), "gemm_pp: cfg");
    CHK(mode >= 0 && mode <= 2, "gemm_pp: mode");
    const int BM = lg ? chronos::gemm_lg_xm((int)cfg) : chronos::gemm_pp_bm((int)cfg);
    const int BN = lg ? chronos::gemm_lg_wn((int)cfg) : chronos::gemm_pp_bn((int)cfg);
    const int PCOLS = lg ? BN / 2 : BN / 4;  // output columns per RMSNorm partial (kResid)
    // gemm_lg addresses both operands through buffer descriptors: 32-bit byte offsets, with one tile of slack
    CHK(!lg || ((N + BN) * K * 2 < (1LL << 31) && (M + BM) * K * 2 < (1LL << 31)), "gemm_lg: operand > 2 GiB");
    CHK(M >= 1 && M < (1LL << 31) / BM && K % 64 == 0 && K <= (1 << 20) && N * K < (1LL << 40), "gemm_pp: size");
    CHK(splitk >= 1 && (K / 64) % splitk == 0, "gemm_pp: splitk must divide K / 64");
    CHK(!lg || splitk == 1 || chronos::gemm_lg_splitk_ok((int)cfg), "gemm_lg: this config has no split-K");
    CHK(mode == 0 ? N % 4 == 0 : N % BN == 0, "gemm_pp: N % 4 (plain) / N % BN (swiglu, resid)");
    CHK(mode != 1 || (lg ? (BN / 4) % 16 == 0 : (BN / 8) % 16 == 0), "gemm_pp: swiglu needs BN >= 128 (gemm_lg: 64)");
    CHK(mode != 2 || !part_in.has_value(), "gemm_pp: resid mode has no norm prologue");
    c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
    chronos::PPArgs a{};
    a.x = bf(x);
    a.w = bf(w);
    a.M = (int)M;
    a.N = (int)N;
    a.K = (int)K;
    a.F = (int)(N / 2);
    a.splitk = (int)splitk;
    a.kts = (int)(K / 64 / splitk);
    a.eps = (float)eps;
    // timing-only diagnostics (wrong results by design): honoured only in a CHRONOS_GEMM_ABLATIONS build
    a.ablate = chronos::gemm_lg_ablations_built() ? chronos::knob("pp_ablate", 0) : 0;
    a.gm = chronos::knob("pp_gm", 8);  // +7-9 % at M = 16384 (profiles/r3_gemm_tile_order_m16384.jsonl)
    a.handoff = chronos::knob("lg_handoff", -1);
    Tensor y = at::empty({M, mode == 1 ? N / 2 : N}, x.options());
    a.y = bfm(y);
    Tensor part_out;
    if (mode == 2) {
        CHK(resid.has_value(), "gemm_pp: resid mode needs resid");
        chk_bf16(*resid, "resid");
        CHK(resid->numel() == M * N, "gemm_pp: resid must be [M, N]");
        a.resid = bf(*resid);
        part_out = at::empty({M, N / PCOLS}, x.options().dtype(at::kFloat));
        a.part_out = part_out.data_ptr<float>();
    }
    if (part_in.has_value()) {
        chk_gpu(*part_in, "part_in");
        CHK(part_in->scalar_type() == at::kFloat && part_in->dim() == 2 && part_in->size(0) == M, "part_in [M, P] f32");
        a.part_in = part_in->data_ptr<float>();
        a.nparts_in = (int)part_in->size(1);
    }
    const int64_t tiles = ((M + BM - 1) / BM) * (mode == 1 ? (N / 2) / (BN / 2) : (N + BN - 1) / BN);
    Tensor ws;
    if (splitk > 1) {
        ws = at::empty({tiles * splitk * BM * BN}, x.options().dtype(at::kFloat));
        a.ws = ws.data_ptr<float>();
        a.cnt = split_tickets(x, tiles);
    }
    if (lg) {
        CHK(!prio && chronos::launch_gemm_lg((int)cfg, (int)mode, part_in.has_value(), a, cur_stream()), "gemm_lg: launch");
    } else {
        CHK(chronos::launch_gemm_pp((int)cfg, (int)mode, part_in.has_value(), prio, a, cur_stream()), "gemm_pp: launch");
    }
    return {y, part_out};
}

// Skinny-M GEMM (gemm_skinny.hip), M <= 16 * MT of the config: same epilogues and tensors as gemm_pp; the kResid
// partials are [M, N / (16 * RT)].
std::tuple<Tensor, Tensor> gemm_skinny(const Tensor& x, const Tensor& w, int64_t mode, int64_t cfg, int64_t splitk,
                                       const c10::optional<Tensor>& resid, const c10::optional<Tensor>& part_in,
                                       double eps) {
    chk_bf16(x, "x");
    chk_bf16(w, "w");
    const int64_t K = x.size(-1), M = x.numel() / K, N = w.size(0);
    CHK(w.dim() == 2 && w.size(1) == K, "gemm_skinny: w must be [N, K]");
    CHK(cfg >= 0 && cfg < chronos::kSkinnyConfigs, "gemm_skinny: cfg");
    CHK(mode >= 0 && mode <= 2, "gemm_skinny: mode");
    const int RT = chronos::gemm_skinny_rt((int)cfg), MT = chronos::gemm_skinny_mt((int)cfg);
    const int NW = chronos::gemm_skinny_nw((int)cfg);
    CHK(M >= 1 && M <= 16 * MT, "gemm_skinny: M must be in [1, 16 * MT] of the config");
    CHK(splitk >= 1 && K % (64 * NW * splitk) == 0 && K <= (1 << 20) && N * K < (1LL << 40),
        "gemm_skinny: K % (64 * NW * splitk) == 0");
    CHK(mode == 1 ? RT % 2 == 0 && (N / 2) % (8 * RT) == 0 && N % 2 == 0 : N % (16 * RT) == 0,
        "gemm_skinny: N % (16 RT) (swiglu: F % (8 RT), RT even)");
    CHK(mode != 2 || !part_in.has_value(), "gemm_skinny: resid mode has no norm prologue");
    c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
    chronos::PPArgs a{};
    a.x = bf(x);
    a.w = bf(w);
    a.M = (int)M;
    a.N = (int)N;
    a.K = (int)K;
    a.F = (int)(N / 2);
    a.splitk = (int)splitk;
    a.eps = (float)eps;
    Tensor y = at::empty({M, mode == 1 ? N / 2 : N}, x.options());
    a.y = bfm(y);
    Tensor part_out;
    if (mode == 2) {
        CHK(resid.has_value(), "gemm_skinny: resid mode needs resid");
        chk_bf16(*resid, "resid");
        CHK(resid->numel() == M * N, "gemm_skinny: resid must be [M, N]");
        a.resid = bf(*resid);
        part_out = at::empty({M, N / (16 * RT)}, x.options().dtype(at::kFloat));
        a.part_out = part_out.data_ptr<float>();
    }
    if (part_in.has_value()) {
        chk_gpu(*part_in, "part_in");
        CHK(part_in->scalar_type() == at::kFloat && part_in->dim() == 2 && part_in->size(0) == M, "part_in [M, P] f32");
        a.part_in = part_in->data_ptr<float>();
        a.nparts_in = (int)part_in->size(1);
    }
    const int64_t groups = mode == 1 ? (N / 2) / (8 * RT) : N / (16 * RT);
    Tensor ws;
    if (splitk > 1) {
        ws = at::empty({groups * splitk * 64 * RT * MT * 4}, x.options().dtype(at::kFloat));
        a.ws = ws.data_ptr<float>();
        a.cnt = split_tickets(x, groups);
    }
    CHK(chronos::launch_gemm_skinny((int)cfg, (int)mode, part_in.has_value(), a, cur_stream()), "gemm_skinny: launch");
    return {y, part_out};
}

// ---- W8A8 fp8-e4m3 path (fp8.hip).  Quantised tensors travel as uint8 (OCP e4m3fn bytes) + fp32 scales.
// mode 0: quant(x); 1: quant(rmsnorm(x) * w); 2: resid <- bf16(x + resid), quant(rmsnorm(resid) * w);
// 3: x = [gate | up] rows of 2F, quant(silu(gate) * up)
std::tuple<Tensor, Tensor> quant_rows(const Tensor& x, const c10::optional<Tensor>& resid,
                                      const c10::optional<Tensor>& w, double eps, int64_t mode) {
    chk_bf16(x, "x");
    CHK(mode >= 0 && mode <= 3, "quant_rows: mode in {0, 1, 2, 3}");
    const int64_t d = mode == 3 ? x.size(-1) / 2 : x.size(-1), rows = x.numel() / x.size(-1);
    CHK(d % 8 == 0 && d <= 16384, "quant_rows: d must be % 8 and <= 16384");
    CHK(mode != 3 || x.size(-1) == 2 * d, "quant_rows: mode 3 needs [rows, 2F]");
    const bool norm = mode == 1 || mode == 2;
    if (norm) {
        CHK(w.has_value(), "quant_rows: rmsnorm modes need w");
        chk_bf16(*w, "w");
        CHK(w->numel() == d, "quant_rows: w must have d entries");
    }
    if (mode == 2) {
        CHK(resid.has_value(), "quant_rows: mode 2 needs resid");
        chk_bf16(*resid, "resid");
        CHK(resid->sizes() == x.sizes(), "quant_rows: resid shape mismatch");
    }
    c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
    auto q = at::empty({rows, d}, x.options().dtype(at::kByte));
    auto s = at::empty({rows}, x.options().dtype(at::kFloat));
    chronos::launch_quant_rows(bf(x), mode == 2 ? bfm(*resid) : nullptr, norm ? bf(*w) : nullptr,
                               q.data_ptr<uint8_t>(), s.data_ptr<float>(), (int)rows, (int)d, (float)eps, (int)mode,
                               cur_stream());
    return {q, s};
}

// y = (xq @ wq.T) * xs[:, None] * ws[None, :] (bf16); swiglu: wq = [gate; up] -> silu(gate) * up
Tensor qlinear(const Tensor& xq, const Tensor& xs, const Tensor& wq, const Tensor& ws, bool swiglu) {
    chk_gpu(xq, "xq");
    chk_gpu(wq, "wq");
    chk_gpu(xs, "xs");
    chk_gpu(ws, "ws");
    CHK(xq.scalar_type() == at::kByte && wq.scalar_type() == at::kByte, "qlinear: xq / wq must be uint8 (e4m3fn)");
    CHK(xs.scalar_type() == at::kFloat && ws.scalar_type() == at::kFloat, "qlinear: scales must be f32");
    const int64_t K = xq.size(-1), M = xq.numel() / K, N = wq.size(0);
    CHK(wq.dim() == 2 && wq.size(1) == K, "qlinear: wq must be [N, K]");
    CHK(xs.numel() == M && ws.numel() == N, "qlinear: one scale per token row / weight row");
    CHK(K % 128 == 0, "qlinear: K % 128 == 0");
    CHK(N % 128 == 0 && (!swiglu || (N / 2) % 64 == 0), "qlinear: N % 128 == 0 (SwiGLU: F % 64 == 0)");
    CHK(M < (1LL << 31) / 128 && N * K < (1LL << 40), "qlinear: size");
    c10::hip::HIPGuardMasqueradingAsCUDA g(xq.device());
    auto y = at::empty({M, swiglu ? N / 2 : N}, xq.options().dtype(at::kBFloat16));
    chronos::launch_qlinear(xq.data_ptr<uint8_t>(), xs.data_ptr<float>(), wq.data_ptr<uint8_t>(), ws.data_ptr<float>(),
                            bfm(y), (int)M, (int)N, (int)K, swiglu, cur_stream());
    return y;
}

// W8A8 on gemm_lg.hip's ring schedule (fp8 configs, gemm_lg_f8_*): the same result as qlinear for M >= 256 shapes.
// splitk divides K / 128.
Tensor qgemm_lg(const Tensor& xq, const Tensor& xs, const Tensor& wq, const Tensor& ws, bool swiglu, int64_t cfg,
                int64_t splitk) {
    chk_gpu(xq, "xq");
    chk_gpu(wq, "wq");
    chk_gpu(xs, "xs");
    chk_gpu(ws, "ws");
    CHK(xq.scalar_type() == at::kByte && wq.scalar_type() == at::kByte, "qgemm_lg: xq / wq must be uint8 (e4m3fn)");
    CHK(xs.scalar_type() == at::kFloat && ws.scalar_type() == at::kFloat, "qgemm_lg: scales must be f32");
    CHK(cfg >= 0 && cfg < chronos::kLGF8Configs, "qgemm_lg: cfg");
    const int64_t K = xq.size(-1), M = xq.numel() / K, N = wq.size(0);
    const int BM = chronos::gemm_lg_f8_xm((int)cfg), BN = chronos::gemm_lg_f8_wn((int)cfg);
    CHK(wq.dim() == 2 && wq.size(1) == K, "qgemm_lg: wq must be [N, K]");
    CHK(xs.numel() == M && ws.numel() == N, "qgemm_lg: one scale per token row / weight row");
    CHK(K % 128 == 0 && K <= (1 << 20) && splitk >= 1 && (K / 128) % splitk == 0, "qgemm_lg: splitk must divide K / 128");
    CHK(swiglu ? N % BN == 0 : N % 4 == 0, "qgemm_lg: N % 4 (plain) / N % BN (swiglu)");
    CHK(M >= 1 && (N + BN) * K < (1LL << 31) && (M + BM) * K < (1LL << 31), "qgemm_lg: operand > 2 GiB");
    c10::hip::HIPGuardMasqueradingAsCUDA g(xq.device());
    chronos::PPArgs a{};
    a.x = reinterpret_cast<const uint16_t*>(xq.data_ptr<uint8_t>());
    a.w = reinterpret_cast<const uint16_t*>(wq.data_ptr<uint8_t>());
    a.xsc = xs.data_ptr<float>();
    a.wsc = ws.data_ptr<float>();
    a.M = (int)M;
    a.N = (int)N;
    a.K = (int)K;
    a.F = (int)(N / 2);
    a.splitk = (int)splitk;
    a.kts = (int)(K / 128 / splitk);
    a.gm = chronos::knob("pp_gm", 8);
    a.handoff = chronos::knob("lg_handoff", -1);
    Tensor y = at::empty({M, swiglu ? N / 2 : N}, xq.options().dtype(at::kBFloat16));
    a.y = bfm(y);
    const int64_t tiles = ((M + BM - 1) / BM) * (swiglu ? (N / 2) / (BN / 2) : (N + BN - 1) / BN);
    Tensor wsl;
    if (splitk > 1) {
        wsl = at::empty({tiles * splitk * BM * BN}, xs.options());
        a.ws = wsl.data_ptr<float>();
        a.cnt = split_tickets(xq, tiles);
    }
    CHK(chronos::launch_gemm_lg_f8((int)cfg, swiglu, a, cur_stream()), "qgemm_lg: launch");
    return y;
}

// value < 0: forget the setting (the next read takes CHRONOS_<NAME> or the built-in default again)
void set_knob(const std::string& name, int64_t value) {
    std::lock_guard<std::mutex> lk(chronos::g_knob_mu);
    if (value < 0) chronos::g_knobs.erase(name);
    else chronos::g_knobs[name] = (int)value;
}

// ---- K14 IPC one-shot all-reduce (allreduce.hip); the handle is the C++ object's address as an int
int64_t ar_create(int64_t rank, int64_t world, int64_t max_bytes) {
    return reinterpret_cast<int64_t>(chronos::ar_create((int)rank, (int)world, max_bytes));
}
Tensor ar_handles(int64_t h) {
    auto v = chronos::ar_handles(reinterpret_cast<void*>(h));
    auto t = at::empty({(int64_t)v.size()}, at::TensorOptions().dtype(at::kByte));
    memcpy(t.data_ptr(), v.data(), v.size());
    return t;
}
void ar_open(int64_t h, const Tensor& all) {
    CHK(!all.is_cuda() && all.scalar_type() == at::kByte && all.dim() == 2, "ar_open: uint8 [world, bytes] CPU");
    auto c = all.contiguous();
    std::vector<std::vector<uint8_t>> v;
    for (int64_t i = 0; i < c.size(0); ++i) {
        const uint8_t* p = c.data_ptr<uint8_t>() + i * c.size(1);
        v.emplace_back(p, p + c.size(1));
    }
    chronos::ar_open(reinterpret_cast<void*>(h), v);
}
void ar_all_reduce(int64_t h, const Tensor& inp, const Tensor& out, int64_t spin_limit, int64_t algo) {
    chk_bf16(inp, "inp");
    chk_bf16(out, "out");
    CHK(inp.numel() == out.numel(), "ar_all_reduce: size mismatch");
    CHK(inp.numel() % 8 == 0 && inp.numel() <= chronos::ar_capacity(reinterpret_cast<void*>(h)),
        "ar_all_reduce: numel must be % 8 and fit the IPC buffer");
    c10::hip::HIPGuardMasqueradingAsCUDA g(inp.device());
    CHK(algo == 1 || algo == 2, "ar_all_reduce: algo must be 1 (one-shot) or 2 (two-shot)");
    chronos::ar_run(reinterpret_cast<void*>(h), bf(inp), bfm(out), inp.numel(), spin_limit, (int)algo, cur_stream());
}
// fused one-shot all-reduce + residual add + RMSNorm: resid <- bf16(sum(inp) + resid), y <- rmsnorm(resid) * w
void ar_all_reduce_norm(int64_t h, const Tensor& inp, const Tensor& resid, const Tensor& w, const Tensor& y, double eps,
                        int64_t spin_limit) {
    chk_bf16(inp, "inp");
    chk_bf16(resid, "resid");
    chk_bf16(w, "w");
    chk_bf16(y, "y");
    CHK(inp.dim() == 2 && resid.sizes() == inp.sizes() && y.sizes() == inp.sizes(), "ar_all_reduce_norm: [T, d] rows");
    CHK(w.numel() == inp.size(1) && inp.size(1) % 8 == 0 && inp.size(1) <= 8 * 256 * 8, "ar_all_reduce_norm: d");
    CHK(inp.numel() <= chronos::ar_capacity(reinterpret_cast<void*>(h)), "ar_all_reduce_norm: exceeds the IPC buffer");
    c10::hip::HIPGuardMasqueradingAsCUDA g(inp.device());
    chronos::ar_run_norm(reinterpret_cast<void*>(h), bf(inp), bfm(resid), bf(w), bfm(y), inp.size(0),
                         (int)inp.size(1), (float)eps, spin_limit, cur_stream());
}
int64_t ar_error(int64_t h) { return chronos::ar_error(reinterpret_cast<void*>(h)); }
int64_t ar_capacity(int64_t h) { return chronos::ar_capacity(reinterpret_cast<void*>(h)); }
void ar_destroy(int64_t h) { chronos::ar_destroy(reinterpret_cast<void*>(h)); }

}  // namespace

TORCH_LIBRARY(chronos, m) {
    m.def("embedding(Tensor ids, Tensor table, int vstart) -> Tensor");
    m.def("rmsnorm(Tensor x, Tensor w, float eps) -> Tensor");
    m.def("add_rmsnorm(Tensor x, Tensor(a!) resid, Tensor w, float eps) -> Tensor");
    m.def("rope_kv_write(Tensor qkv, Tensor pos, Tensor tok_seq, Tensor block_table, Tensor cos_sin, "
          "Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, int hq, int hkv, bool write_q, "
          "float k_scale=1.0, float v_scale=1.0) -> ()");
    m.def("silu_mul(Tensor gate_up) -> Tensor");
    m.def("gemv(Tensor x, Tensor w, bool swiglu, Tensor? ws=None) -> Tensor");
    m.def("gemm(Tensor x, Tensor w, bool swiglu, int stages=3) -> Tensor");
    m.def("gemm_pp(Tensor x, Tensor w, int mode, int cfg, int splitk, Tensor? resid, Tensor? part_in, float eps, bool prio) -> (Tensor, Tensor)");
    m.def("gemm_skinny(Tensor x, Tensor w, int mode, int cfg, int splitk, Tensor? resid, Tensor? part_in, float eps) "
          "-> (Tensor, Tensor)");
    m.def("gemv_resid(Tensor x, Tensor w, Tensor resid_in, Tensor(a!) resid_out, Tensor? ws=None) -> Tensor");
    m.def("gemv_normp(Tensor s, Tensor part, float eps, Tensor w, bool swiglu, Tensor? ws=None) -> Tensor");
    m.def("qkv_rope(Tensor x, Tensor? part, float eps, Tensor w, Tensor pos, Tensor tok_seq, "
          "Tensor block_table, Tensor cos_sin, Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, int hq, "
          "int hkv, float k_scale=1.0, float v_scale=1.0, Tensor? ws=None) -> ()");
    m.def("set_decode_gate(Tensor? state, int n) -> ()", &set_decode_gate);
    m.def("attn_init() -> ()", [] { chronos::attn_init(); });
    m.def("quant_rows(Tensor x, Tensor(a!)? resid, Tensor? w, float eps, int mode) -> (Tensor, Tensor)");
    m.def("qlinear(Tensor xq, Tensor xs, Tensor wq, Tensor ws, bool swiglu) -> Tensor");
    m.def("qgemm_lg(Tensor xq, Tensor xs, Tensor wq, Tensor ws, bool swiglu, int cfg, int splitk) -> Tensor");
    m.def("set_knob(str name, int value) -> ()", &set_knob);
    m.def("ar_create(int rank, int world, int max_bytes) -> int", &ar_create);
    m.def("ar_handles(int h) -> Tensor", &ar_handles);
    m.def("ar_open(int h, Tensor all) -> ()", &ar_open);
    m.def("ar_all_reduce(int h, Tensor inp, Tensor(a!) out, int spin_limit, int algo=1) -> ()");
    m.def("ar_all_reduce_norm(int h, Tensor inp, Tensor(a!) resid, Tensor w, Tensor(b!) y, float eps, int spin_limit) -> ()");
    m.def("ar_error(int h) -> int", &ar_error);
    m.def("ar_capacity(int h) -> int", &ar_capacity);
    m.def("ar_destroy(int h) -> ()", &ar_destroy);
    m.def("decode_attention_rope(Tensor qkv, Tensor pos, Tensor cos_sin, Tensor(a!) k_cache, Tensor(b!) v_cache, "
          "Tensor block_table, Tensor ctx_len, int n, int hq, float scale, Tensor? casc=None, Tensor(c!)? casc_o=None, "
          "Tensor(d!)? casc_l=None) -> Tensor");
    m.def("paged_attention(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_table, Tensor q_start, "
          "Tensor ctx_len, Tensor? tiles, int ntiles, int nqt, int nsplit, float scale, float k_scale=1.0, "
          "float v_scale=1.0, int max_q=1) -> Tensor");
    m.def("constrained_sample(Tensor logits, Tensor? row_of_slot, Tensor next, Tensor dist, int done_state, "
          "Tensor(a!) state, Tensor(b!) remaining, Tensor? temperature, Tensor? seed, Tensor(c!) ids, Tensor(d!) pos, "
          "Tensor(e!) ctx, Tensor(f!) nout, Tensor(g!) out_tokens, Tensor? topk=None, Tensor? topp=None, "
          "Tensor? jump=None) -> ()");
}

TORCH_LIBRARY_IMPL(chronos, CUDA, m) {
    m.impl("embedding", &embedding);
    m.impl("rmsnorm", &rmsnorm);
    m.impl("add_rmsnorm", &add_rmsnorm);
    m.impl("rope_kv_write", &rope_kv_write);
    m.impl("silu_mul", &silu_mul);
    m.impl("gemv", &gemv);
    m.impl("gemm", &gemm);
    m.impl("gemm_pp", &gemm_pp);
    m.impl("gemm_skinny", &gemm_skinny);
    m.impl("gemv_resid", &gemv_resid);
    m.impl("gemv_normp", &gemv_normp);
    m.impl("qkv_rope", &qkv_rope);
    m.impl("quant_rows", &quant_rows);
    m.impl("qlinear", &qlinear);
    m.impl("qgemm_lg", &qgemm_lg);
    m.impl("paged_attention", &paged_attention);
    m.impl("decode_attention_rope", &decode_attention_rope);
    m.impl("constrained_sample", &constrained_sample);
    m.impl("ar_all_reduce", &ar_all_reduce);
    m.impl("ar_all_reduce_norm", &ar_all_reduce_norm);
}
