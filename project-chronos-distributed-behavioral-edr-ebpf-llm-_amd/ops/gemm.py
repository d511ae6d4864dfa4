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


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if x.is_cuda and _custom:
        m, k = x.numel() // x.shape[-1], x.shape[-1]
        n = w.shape[0]
        for pred, fn in _custom:
            if pred(m, n, k):
                return fn(x, w)
    if out is not None:
        return torch.matmul(x, w.t(), out=out)
    return torch.matmul(x, w.t())
