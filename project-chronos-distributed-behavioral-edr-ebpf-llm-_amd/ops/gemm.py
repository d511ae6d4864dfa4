"""Projection GEMMs.

``linear(x, w)`` computes ``x @ w.T`` for weights stored [out, in] (HF layout).  Plain projection GEMMs go to the
vendor library (hipBLASLt via torch.matmul) — the task's rule for "plain library GEMMs"; the fused / skinny shapes
that a library does not serve well get hand-written MFMA kernels registered in ``_custom`` (see csrc/kernels/gemm*.hip)
and are selected per shape by :func:`linear`.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

# (M, N, K) -> bool predicate + kernel; filled by the HIP GEMM module once it is loaded
_custom: list[tuple[Callable[[int, int, int], bool], Callable[[torch.Tensor, torch.Tensor], torch.Tensor]]] = []


def register(pred: Callable[[int, int, int], bool], fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor]) -> None:
    _custom.append((pred, fn))


def gemv_ok(m: int, n: int, k: int, swiglu: bool = False) -> bool:
    """Shapes routed to the hand-written decode GEMV (csrc/kernels/gemv.hip): K % 512, N % 16 and the M range where it
    beats hipBLASLt on cold weights (profiles/r1_kernels.json): M == 1 always, M == 2 below LM-head widths."""
    if k % 512 or n % 16:
        return False
    return m == 1 or (m == 2 and n <= 32768)


def _gemv(x: torch.Tensor, w: torch.Tensor, swiglu: bool = False) -> torch.Tensor:
    from . import _k

    k = x.shape[-1]
    y = _k().gemv(x.reshape(-1, k), w, swiglu)
    return y.view(*x.shape[:-1], y.shape[-1])


def gate_up_silu(x: torch.Tensor, w_gu: torch.Tensor) -> torch.Tensor:
    """silu(x @ gate.T) * (x @ up.T) with w_gu = [gate; up].  Decode: one fused GEMV launch; else GEMM + silu_mul."""
    from . import silu_mul

    if x.is_cuda and gemv_ok(x.numel() // x.shape[-1], w_gu.shape[0], x.shape[-1], swiglu=True):
        return _gemv(x, w_gu, True)
    return silu_mul(linear(x, w_gu))


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if x.is_cuda:
        m, k = x.numel() // x.shape[-1], x.shape[-1]
        n = w.shape[0]
        if gemv_ok(m, n, k):
            return _gemv(x, w)
        for pred, fn in _custom:
            if pred(m, n, k):
                return fn(x, w)
    if out is not None:
        return torch.matmul(x, w.t(), out=out)
    return torch.matmul(x, w.t())
