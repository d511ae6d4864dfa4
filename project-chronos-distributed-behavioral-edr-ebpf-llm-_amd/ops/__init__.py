"""Op dispatch: hand-written gfx950 HIP kernels on the GPU, fp32 PyTorch references on the CPU.

There is no silent fallback on a GPU: a CUDA/HIP tensor always goes to ``torch.ops.chronos.*``; if the in-tree
extension (``_C*.so``, built by :mod:`chronos.native`) cannot be built or loaded the op raises.  CPU tensors (tests,
the gloo-backed distributed tests, the CPU plumbing config) take :mod:`.reference`.

Kernel sources: csrc/kernels/{elementwise,attention,sampler}.hip.
"""
from __future__ import annotations

import math
import os

import torch

from . import reference as ref
from .gemm import (LazyNorm, ResidOut, gate_up_silu, gemv_ok, gemv_q_ok, gemv_resid, is_q, linear,  # noqa: F401
                   resid_ok)

_loaded = False

# Debug-mode device-index validation: GPU AddressSanitizer is not available on the MI355X pool, and an
# out-of-bounds paged-KV access can fault the whole GPU, so with CHRONOS_CHECK_INPUTS=1 every index a hand-written
# kernel will dereference (block-table entries, positions, slots, grammar states, tiles) is range-checked on the host
# BEFORE the launch and a bad one raises IndexError instead.  Costs a device->host copy per op: a debug mode (skipped
# inside graph capture, where a copy would break the capture; the eager steps exercise the same indices).
_CHECK = os.environ.get("CHRONOS_CHECK_INPUTS", "0") not in ("", "0")


def set_input_checks(on: bool) -> None:
    global _CHECK
    _CHECK = bool(on)


def _checking(t: torch.Tensor) -> bool:
    return _CHECK and t.is_cuda and not torch.cuda.is_current_stream_capturing()


def _need(cond: bool, what: str) -> None:
    if not cond:
        raise IndexError(f"chronos input check: {what}")


def _check_paged(block_table, k_cache, tok_rows, kv_len, what: str) -> None:
    """Every cache block a kernel can touch exists: rows tok_rows of block_table over the first kv_len tokens."""
    bt = block_table.cpu()
    nb, bs = k_cache.shape[0], k_cache.shape[2]
    rows = tok_rows.cpu().long()
    lens = kv_len.cpu().long()
    _need(bool(((rows >= 0) & (rows < bt.shape[0])).all()), f"{what}: block-table row out of range")
    _need(bool(((lens >= 0) & ((lens + bs - 1) // bs <= bt.shape[1])).all()), f"{what}: length exceeds block table")
    for r, n in zip(rows.tolist(), lens.tolist()):
        used = bt[r, :(n + bs - 1) // bs]
        _need(bool(((used >= 0) & (used < nb)).all()), f"{what}: block id out of range in row {r}")


def load() -> None:
    """Load (building in-tree if stale) the HIP kernel library; raises on failure."""
    global _loaded
    if not _loaded:
        from ..native import kernels_lib

        kernels_lib()
        _loaded = True
        if torch.cuda.is_available():
            torch.ops.chronos.attn_init()  # current device; Engine repeats it after selecting its own


def _k():
    load()
    return torch.ops.chronos


def device_init() -> None:
    """Per-device kernel state for the current HIP device (the attention kernel's split-completion tickets); call
    after set_device and before any graph capture.  Idempotent."""
    _k().attn_init()


def embedding(ids: torch.Tensor, table: torch.Tensor, vstart: int = 0) -> torch.Tensor:
    if ids.is_cuda:
        return _k().embedding(ids, table, vstart)
    return ref.embedding(ids, table, vstart)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    if x.is_cuda:
        return _k().rmsnorm(x, w, eps)
    return ref.rmsnorm(x, w, eps)


def add_rmsnorm(x: torch.Tensor, resid: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """resid <- bf16(x + resid) in place; returns rmsnorm(resid) * w."""
    if x.is_cuda:
        return _k().add_rmsnorm(x, resid, w, eps)
    return ref.add_rmsnorm(x, resid, w, eps)


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    if gu.is_cuda:
        return _k().silu_mul(gu)
    return ref.silu_mul(gu)


def quant_rows(x: torch.Tensor, resid: torch.Tensor | None = None, w: torch.Tensor | None = None, eps: float = 1e-5,
               mode: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
    """Dynamic per-row e4m3 quantisation, optionally fused with (residual add +) RMSNorm (csrc/kernels/fp8.hip):
    mode 0 = quant(x), 1 = quant(rmsnorm(x) * w), 2 = resid <- bf16(x + resid) then quant(rmsnorm(resid) * w),
    3 = quant(silu(gate) * up) of [gate | up] rows."""
    if x.is_cuda:
        return _k().quant_rows(x, resid, w, eps, mode)
    return ref.quant_rows(x, resid, w, eps, mode)


# W8A8 GEMM routing, by measured shape: the "qplans" rows of ops/gemm_plan.json (scripts/tune_gemm_pp.py --fp8: the
# hand-written fp8 GEMV / block-scaled MFMA GEMM against hipBLASLt's fp8 GEMM with row-wise scales, torch._scaled_mm,
# per (N, K, SwiGLU) and M; the library only where it measured > 3 % faster).  Unmeasured shapes: the round-1 rule
# (profiles/r1_fp8_gemm.json) — own GEMV at M <= 4, own SwiGLU GEMM at M <= 128.  CHRONOS_QGEMM=own|lib|auto.
_QGEMM = os.environ.get("CHRONOS_QGEMM", "auto")
_F8 = torch.float8_e4m3fn


def _qown(m: int, n: int, k: int, swiglu: bool) -> bool:
    if _QGEMM != "auto":
        return _QGEMM == "own"
    from .gemm import qplan_own

    own = qplan_own(m, n, k, swiglu)  # the measured A/B of ops/gemm_plan.json "qplans"
    if own is not None:
        return own
    return (m <= 4 and k % 1024 == 0) or (swiglu and m <= 128)


def _qlib(xq, xs, wq, ws) -> torch.Tensor:
    return torch._scaled_mm(xq.view(_F8), wq.view(_F8).t(), scale_a=xs.view(-1, 1), scale_b=ws.view(1, -1),
                            out_dtype=torch.bfloat16)


def qlinear(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor, swiglu: bool = False) -> torch.Tensor:
    """W8A8 fp8 projection: y = (xq @ wq.T) * xs * ws in bf16 (swiglu: wq = [gate; up] -> silu(gate) * up)."""
    if xq.is_cuda:
        m, k = xq.numel() // xq.shape[-1], xq.shape[-1]
        if _qown(m, wq.shape[0], k, swiglu):
            from .gemm import QLG_BASE, qplan_route

            r = qplan_route(m, wq.shape[0], k, swiglu) if _QGEMM == "auto" else None
            if r is not None and r[0] >= QLG_BASE:  # gemm_lg.hip fp8 config (the large-M ring schedule)
                return _k().qgemm_lg(xq, xs, wq, ws, swiglu, r[0] - QLG_BASE, r[1])
            return _k().qlinear(xq, xs, wq, ws, swiglu)
        y = _qlib(xq, xs, wq, ws)
        return silu_mul(y) if swiglu else y
    return ref.qlinear(xq, xs, wq, ws, swiglu)


def qgate_up_quant(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor):
    """The MLP's fp8 middle: (e4m3 bytes, row scale) of silu(x Wg^T) * (x Wu^T), ready for the down projection.
    Fused SwiGLU GEMM epilogue + row quant at small M; library GEMM + one fused SwiGLU-and-quantise pass otherwise."""
    if xq.is_cuda:
        m, k = xq.numel() // xq.shape[-1], xq.shape[-1]
        if not _qown(m, wq.shape[0], k, True):
            return quant_rows(_qlib(xq, xs, wq, ws), mode=3)
    return quant_rows(qlinear(xq, xs, wq, ws, True))


def rope_kv_write(qkv, pos, tok_seq, block_table, cos_sin, q_out, k_cache, v_cache, hq: int, hkv: int,
                  write_q: bool = True, k_scale: float = 1.0, v_scale: float = 1.0) -> None:
    """RoPE q/k + write k/v into the paged cache (bf16, or fp8-e4m3 bytes when the cache is uint8)."""
    if _checking(qkv):
        p = pos.cpu().long()
        _need(bool(((p >= 0) & (p < cos_sin.shape[0])).all()), "rope_kv_write: position outside the rope table")
        _check_paged(block_table, k_cache, tok_seq, p + 1, "rope_kv_write")
    if qkv.is_cuda:
        _k().rope_kv_write(qkv, pos, tok_seq, block_table, cos_sin, q_out, k_cache, v_cache, hq, hkv, write_q,
                           k_scale, v_scale)
    else:
        ref.rope_kv_write(qkv, pos, tok_seq, block_table, cos_sin, q_out, k_cache, v_cache, hq, hkv, write_q,
                          k_scale, v_scale)


def qkv_rope(x, w_qkv, pos, tok_seq, block_table, cos_sin, q_out, k_cache, v_cache, hq: int, hkv: int,
             k_scale: float = 1.0, v_scale: float = 1.0) -> bool:
    """Decode QKV projection + RoPE + paged-KV write in one GEMV launch (csrc/kernels/gemv.hip ROPE epilogue), with the
    input RMSNorm folded in when x is a LazyNorm.  Returns False (nothing done) off the decode GEMV shapes; the caller
    then runs the unfused ops."""
    lazy = isinstance(x, LazyNorm)
    if lazy and not x.fusable():
        return False
    t = x.s if lazy else x
    m, n, k = t.numel() // t.shape[-1], w_qkv.shape[0], t.shape[-1]
    fp8w = is_q(w_qkv)  # fp8 weights: the W8A16 GEMV (e4m3 bytes + per-row scales)
    if not (t.is_cuda and m <= 2 and (gemv_q_ok(m, n, k) if fp8w else gemv_ok(m, n, k))):
        return False
    _k().qkv_rope(t.reshape(m, k), x.part if lazy else None, x.eps if lazy else 0.0, w_qkv.q if fp8w else w_qkv,
                  pos, tok_seq, block_table, cos_sin, q_out, k_cache, v_cache, hq, hkv, k_scale, v_scale,
                  w_qkv.s if fp8w else None)
    return True


def set_decode_gate(state: torch.Tensor | None, n: int = 0) -> None:
    """Arm (1 <= n <= 8) / disarm (n = 0) the decode early-exit gate for the launches that follow: every kernel of a
    decode step returns at once when none of ``state[:n]`` is live (chronos_hip.h).  No-op without the GPU library."""
    if state is not None and state.is_cuda:
        _k().set_decode_gate(state, n)
    elif _loaded:
        torch.ops.chronos.set_decode_gate(None, 0)


def paged_attention(q, k_cache, v_cache, block_table, q_start, ctx_len, tiles=None, ntiles: int = 0, nqt: int = 1,
                    nsplit: int = 1, scale: float | None = None, k_scale: float = 1.0,
                    v_scale: float = 1.0, max_q: int = 1) -> torch.Tensor:
    """Paged attention: prefill tiles (``tiles``), decode rows (tiles None: token i is sequence i), or — tiles None,
    ``max_q`` > 1 — sequences of up to max_q query tokens (q_start ranges, the last token at the end of its context)
    in one pass over each sequence's K/V (split-K decode kernel; max_q x GQA group <= 16)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if _checking(q):
        nseq = ctx_len.shape[0] if tiles is None else q_start.shape[0] - 1
        if tiles is None and max_q > 1:
            qs = q_start.cpu().long()[:ntiles + 1]
            _need(bool(((qs[1:] - qs[:-1]) <= max_q).all()) and int(qs[-1]) <= q.shape[0],
                  "paged_attention: multi-token decode q_start")
        elif tiles is None:
            _need(ntiles <= ctx_len.shape[0] and ntiles <= q.shape[0], "paged_attention: decode rows")
        else:
            tl = tiles.cpu().long()
            _need(bool(((tl[:, 0] >= 0) & (tl[:, 0] < nseq)).all()), "paged_attention: tile sequence out of range")
            qs = q_start.cpu().long()
            _need(bool((qs[1:] >= qs[:-1]).all()) and int(qs[-1]) <= q.shape[0], "paged_attention: q_start")
        _check_paged(block_table, k_cache, torch.arange(nseq), ctx_len[:nseq], "paged_attention")
    if q.is_cuda:
        return _k().paged_attention(q, k_cache, v_cache, block_table, q_start, ctx_len, tiles, ntiles, nqt, nsplit,
                                    scale, k_scale, v_scale, max_q)
    return ref.paged_attention(q, k_cache, v_cache, block_table, q_start, ctx_len, tiles, ntiles, nqt, nsplit, scale,
                               k_scale, v_scale, max_q)


def decode_attention_rope(qkv, pos, cos_sin, k_cache, v_cache, block_table, ctx_len, n: int, hq: int,
                          scale: float, casc=None):
    """Decode step (row i = sequence i, one token at pos[i], ctx_len[i] == pos[i] + 1): RoPE + paged-KV write + paged
    attention in one launch (csrc/kernels/attention.hip paged_decode_kernel RP).  Returns the [n, hq, 128] output, or
    None when the fused kernel does not serve the shape (fp8 KV, < 1024 (row, kv head) items, ...): the caller then
    runs rope_kv_write + paged_attention, which compute the same thing.

    ``casc``: optional (casc [1 + P_max] int32, o scratch [S, hq, 128] bf16, lse scratch [S, hq] f32) — cascade
    attention over a shared prompt prefix (casc[0] = P blocks, then their ids): rows whose block table starts with
    those blocks attend the prefix in one MFMA pass per 16 / G rows and merge it into the walk over their own tokens
    (csrc/kernels/attention.hip casc_prefix_kernel).  Mathematically the same attention; casc[0] = 0 disables it."""
    if not qkv.is_cuda:
        return None
    if _checking(qkv):
        p, c = pos[:n].cpu().long(), ctx_len[:n].cpu().long()
        _need(bool((c == p + 1).all()), "decode_attention_rope: ctx_len must be pos + 1 (decode rows)")
        _need(bool(((p >= 0) & (p < cos_sin.shape[0])).all()), "decode_attention_rope: position outside the rope table")
        _check_paged(block_table, k_cache, torch.arange(n), c, "decode_attention_rope")
        if casc is not None:
            cv = casc[0].cpu().long()
            P = int(cv[0])
            _need(0 <= P < cv.numel(), "decode_attention_rope: cascade prefix length")
            _need(bool(((cv[1:1 + P] >= 0) & (cv[1:1 + P] < k_cache.shape[0])).all()), "cascade block id out of range")
    if casc is not None:
        out = _k().decode_attention_rope(qkv, pos, cos_sin, k_cache, v_cache, block_table, ctx_len, n, hq, scale,
                                         casc[0], casc[1], casc[2])
    else:
        out = _k().decode_attention_rope(qkv, pos, cos_sin, k_cache, v_cache, block_table, ctx_len, n, hq, scale)
    return out if out.numel() else None


def constrained_sample(logits, row_of_slot, next_tab, dist, done_state: int, state, remaining, temperature, seed,
                       ids, pos, ctx, nout, out_tokens, topk=None, topp=None, jump=None) -> None:
    """``jump``: optional int8 [S] flags — a row whose sampled token leads into a flagged state is parked as state
    ``-2 - s`` (csrc/kernels/sampler.hip, Engine._jump)."""
    if _checking(logits):
        st = state.cpu().long()
        S = next_tab.shape[0]
        _need(bool(((st >= -1 - S) & (st < S)).all()), "constrained_sample: grammar state out of range")
        _need(next_tab.shape[1] <= logits.shape[-1], "constrained_sample: grammar table wider than the logits")
        if row_of_slot is not None:
            rs = row_of_slot.cpu().long()
            _need(bool(((rs >= -1) & (rs < logits.shape[0])).all()), "constrained_sample: logits row out of range")
        else:
            _need(state.shape[0] <= logits.shape[0], "constrained_sample: more slots than logits rows")
    if logits.is_cuda:
        _k().constrained_sample(logits, row_of_slot, next_tab, dist, done_state, state, remaining, temperature, seed,
                                ids, pos, ctx, nout, out_tokens, topk, topp, jump)
    else:
        ref.constrained_sample(logits, row_of_slot, next_tab, dist, done_state, state, remaining, temperature, seed,
                               ids, pos, ctx, nout, out_tokens, topk, topp, jump)


def attention_tiles(q_lens: list[int], hq: int, hkv: int, nqt: int) -> list[tuple[int, int]]:
    """Host tile list for prefill: (seq, first query token of the tile relative to the seq)."""
    tpw = nqt * 16 // (hq // hkv)
    out = []
    for b, n in enumerate(q_lens):
        for r in range(0, n, tpw):
            out.append((b, r))
    return out


# target split-K decode workgroups per CU: 1 measured best at every long-context shape (profiles/r2_attn_nsplit_sweep.json:
# 1 x 128k 150 -> 125 us per layer (64 -> 32 splits), 4 x 32k 113 -> 110, 16 x 8k 117 -> 113); 2 over-splits
_SPLIT_WGS = int(os.environ.get("CHRONOS_DECODE_SPLIT_WGS", "1"))
_SPLIT_MAX = int(os.environ.get("CHRONOS_DECODE_SPLIT_MAX", "64"))


def pick_nsplit(n_workgroups: int, max_ctx: int, cus: int = 256) -> int:
    """Flash-decoding split: enough workgroups to cover the chip, >= 256 keys per split."""
    if n_workgroups >= _SPLIT_WGS * cus:
        return 1
    want = (_SPLIT_WGS * cus + n_workgroups - 1) // n_workgroups
    cap = max(1, max_ctx // 256)
    return int(max(1, min(want, cap, _SPLIT_MAX)))
