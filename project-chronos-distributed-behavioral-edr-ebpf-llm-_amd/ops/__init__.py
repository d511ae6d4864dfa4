"""Op dispatch: hand-written gfx950 HIP kernels on the GPU, fp32 PyTorch references on the CPU.

There is no silent fallback on a GPU: a CUDA/HIP tensor always goes to ``torch.ops.chronos.*``; if the in-tree
extension (``_C*.so``, built by :mod:`chronos.native`) cannot be built or loaded the op raises.  CPU tensors (tests,
the gloo-backed distributed tests, the CPU plumbing config) take :mod:`.reference`.

Kernel sources: csrc/kernels/{elementwise,attention,sampler}.hip.
"""
from __future__ import annotations

import math

import torch

from . import reference as ref
from .gemm import gate_up_silu, linear  # noqa: F401  (re-export)

_loaded = False


def load() -> None:
    """Load (building in-tree if stale) the HIP kernel library; raises on failure."""
    global _loaded
    if not _loaded:
        from ..native import kernels_lib

        kernels_lib()
        _loaded = True


def _k():
    load()
    return torch.ops.chronos


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


def rope_kv_write(qkv, pos, tok_seq, block_table, cos_sin, q_out, k_cache, v_cache, hq: int, hkv: int,
                  write_q: bool = True, k_scale: float = 1.0, v_scale: float = 1.0) -> None:
    """RoPE q/k + write k/v into the paged cache (bf16, or fp8-e4m3 bytes when the cache is uint8)."""
    if qkv.is_cuda:
        _k().rope_kv_write(qkv, pos, tok_seq, block_table, cos_sin, q_out, k_cache, v_cache, hq, hkv, write_q,
                           k_scale, v_scale)
    else:
        ref.rope_kv_write(qkv, pos, tok_seq, block_table, cos_sin, q_out, k_cache, v_cache, hq, hkv, write_q,
                          k_scale, v_scale)


def paged_attention(q, k_cache, v_cache, block_table, q_start, ctx_len, tiles=None, ntiles: int = 0, nqt: int = 1,
                    nsplit: int = 1, scale: float | None = None, k_scale: float = 1.0,
                    v_scale: float = 1.0) -> torch.Tensor:
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda:
        return _k().paged_attention(q, k_cache, v_cache, block_table, q_start, ctx_len, tiles, ntiles, nqt, nsplit,
                                    scale, k_scale, v_scale)
    return ref.paged_attention(q, k_cache, v_cache, block_table, q_start, ctx_len, tiles, ntiles, nqt, nsplit, scale,
                               k_scale, v_scale)


def constrained_sample(logits, row_of_slot, next_tab, dist, done_state: int, state, remaining, temperature, seed,
                       ids, pos, ctx, nout, out_tokens, topk=None, topp=None) -> None:
    if logits.is_cuda:
        _k().constrained_sample(logits, row_of_slot, next_tab, dist, done_state, state, remaining, temperature, seed,
                                ids, pos, ctx, nout, out_tokens, topk, topp)
    else:
        ref.constrained_sample(logits, row_of_slot, next_tab, dist, done_state, state, remaining, temperature, seed,
                               ids, pos, ctx, nout, out_tokens, topk, topp)


def attention_tiles(q_lens: list[int], hq: int, hkv: int, nqt: int) -> list[tuple[int, int]]:
    """Host tile list for prefill: (seq, first query token of the tile relative to the seq)."""
    tpw = nqt * 16 // (hq // hkv)
    out = []
    for b, n in enumerate(q_lens):
        for r in range(0, n, tpw):
            out.append((b, r))
    return out


def pick_nsplit(n_workgroups: int, max_ctx: int, cus: int = 256) -> int:
    """Flash-decoding split: enough workgroups to cover the chip, >= 256 keys per split."""
    if n_workgroups >= 2 * cus:
        return 1
    want = (2 * cus + n_workgroups - 1) // n_workgroups
    cap = max(1, max_ctx // 256)
    return int(max(1, min(want, cap, 64)))
