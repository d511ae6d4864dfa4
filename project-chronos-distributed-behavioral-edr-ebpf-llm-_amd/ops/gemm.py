"""Projection GEMMs.

``linear(x, w)`` computes ``x @ w.T`` for weights stored [out, in] (HF layout); ``gate_up_silu`` is the fused K8+K9.
Routing is by measured shape (profiles/r1_gemm_vs_hipblaslt.json, cold weights, one MI355X):

* M <= 2 (single-stream decode): the hand-written GEMV (csrc/kernels/gemv.hip), 1 KiB row-contiguous weight
  streaming — beats hipBLASLt on every decode shape;
* gate_up at 3 <= M <= 128: the MFMA GEMM with the fused SwiGLU epilogue (csrc/kernels/gemm.hip) — 1.05-1.24x over
  hipBLASLt + the separate silu_mul pass, which it removes;
* everything else: hipBLASLt via torch.matmul (the "plain library GEMM" rule).  Measured alternatives that did not
  pay at the wave's M = 1024 decode bucket: a TunableOp sweep over every library solution (~1 % of the wave,
  profiles/r1s4_tunableop_gemm_study.jsonl) and two half-batches on two HIP streams so the under-filled N = 4096 /
  6144 projections run side by side (-2 % decode GPU time, but a slower wave: 580 vs 608 chains/s).  The hand-written 128x128-tile MFMA
  GEMM loses there: one tile per CU is bound by the per-CU load path (~0.7 us per 64-deep K-step), the same wall
  hipBLASLt's 128x128 tiles hit, and it has no answer to the small-grid shapes (N = 4096 at M <= 128).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Optional

import torch

# Largest M routed to the GEMV (gemv_ok).  Env CHRONOS_GEMV_MAX_M; scripts/single_stream.py A/Bs it (py_gemv_max_m).
GEMV_MAX_M = int(os.environ.get("CHRONOS_GEMV_MAX_M", "2"))

# (M, N, K) -> bool predicate + kernel; extension point for further shape-specialised kernels
_custom: list[tuple[Callable[[int, int, int], bool], Callable[[torch.Tensor, torch.Tensor], torch.Tensor]]] = []


def register(pred: Callable[[int, int, int], bool], fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor]) -> None:
    _custom.append((pred, fn))


@dataclass
class ResidOut:
    """Output of a decode producer GEMV with the residual epilogue (``gemv_resid``): the new residual stream
    ``s = bf16(bf16(x @ w.T) + resid)`` and the per-workgroup partial sums of s^2 the next RMSNorm needs."""
    s: torch.Tensor
    part: torch.Tensor


@dataclass
class LazyNorm:
    """``rmsnorm(s) * w`` of a residual stream a ResidOut producer just wrote, not computed yet.

    Only built for models whose norm weights are folded into the consuming projections (``w`` is then ones).  A decode
    GEMV consumer (``linear`` / ``gate_up_silu`` / the fused QKV projection) applies it as one per-row scale of its
    outputs (csrc/kernels/gemv.hip NORMP: inv from the producer's partials), so the norm costs no launch; any other
    consumer calls ``materialize`` (the standalone RMSNorm kernel: equal up to rounding)."""
    s: torch.Tensor
    part: torch.Tensor
    w: torch.Tensor
    eps: float
    _y: Optional[torch.Tensor] = None

    @property
    def shape(self):
        return self.s.shape

    def rows(self) -> int:
        return self.s.numel() // self.s.shape[-1]

    def fusable(self) -> bool:
        return self.s.is_cuda and self._y is None

    def materialize(self) -> torch.Tensor:
        if self._y is None:
            from . import rmsnorm

            self._y = rmsnorm(self.s, self.w, self.eps)
        return self._y

    @staticmethod
    def force(x):
        """A tensor for anything that is not a GEMV consumer."""
        return x.materialize() if isinstance(x, LazyNorm) else x


def gemv_resid(x: torch.Tensor, w: torch.Tensor, resid: torch.Tensor) -> ResidOut:
    """Decode producer: the new residual stream and the RMSNorm partials in one GEMV launch (M <= 2)."""
    from . import _k

    s = torch.empty(resid.shape, dtype=resid.dtype, device=resid.device)
    part = _k().gemv_resid(x.reshape(-1, x.shape[-1]), w, resid, s)
    return ResidOut(s, part)


def resid_ok(m: int, n: int, k: int) -> bool:
    """Shapes of the residual-epilogue producer (gemv.hip kResid): the M <= 2 GEMV shapes."""
    return m <= 2 and gemv_ok(m, n, k)


def gemv_ok(m: int, n: int, k: int, swiglu: bool = False) -> bool:
    """Shapes routed to the hand-written decode GEMV (csrc/kernels/gemv.hip): K % 512, N % 16 and the M range where it
    beats hipBLASLt on cold weights (profiles/r1_kernels.json): M == 1 always, M == 2 below LM-head widths."""
    if k % 512 or n % 16:
        return False
    return m == 1 or (m <= GEMV_MAX_M and n <= 32768)


def mfma_swiglu_ok(m: int, n: int, k: int) -> bool:
    """Fused gate_up + SwiGLU on the MFMA GEMM: the measured winning range (3 <= M <= 128)."""
    return 3 <= m <= 128 and k % 64 == 0 and n % 128 == 0


def _gemv(x: torch.Tensor, w: torch.Tensor, swiglu: bool = False) -> torch.Tensor:
    from . import _k

    k = x.shape[-1]
    y = _k().gemv(x.reshape(-1, k), w, swiglu)
    return y.view(*x.shape[:-1], y.shape[-1])


def mfma_gemm(x: torch.Tensor, w: torch.Tensor, swiglu: bool = False, stages: int = 3) -> torch.Tensor:
    from . import _k

    k = x.shape[-1]
    y = _k().gemm(x.reshape(-1, k), w, swiglu, stages)
    return y.view(*x.shape[:-1], y.shape[-1])


def gate_up_silu(x: torch.Tensor, w_gu: torch.Tensor) -> torch.Tensor:
    """silu(x @ gate.T) * (x @ up.T) with w_gu = [gate; up]: one fused launch for decode batches, else GEMM + silu_mul."""
    from . import _k, silu_mul

    if isinstance(x, LazyNorm):
        m, n, k = x.rows(), w_gu.shape[0], x.shape[-1]
        if x.fusable() and gemv_ok(m, n, k, swiglu=True):
            return _k().gemv_normp(x.s, x.part, x.eps, w_gu, True)
        x = x.materialize()
    if x.is_cuda:
        m, n, k = x.numel() // x.shape[-1], w_gu.shape[0], x.shape[-1]
        if gemv_ok(m, n, k, swiglu=True):
            return _gemv(x, w_gu, True)
        if mfma_swiglu_ok(m, n, k):
            return mfma_gemm(x, w_gu, True)
    return silu_mul(linear(x, w_gu))


def linear(x, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if isinstance(x, LazyNorm):
        if x.fusable() and out is None and gemv_ok(x.rows(), w.shape[0], x.shape[-1]):
            from . import _k

            return _k().gemv_normp(x.s, x.part, x.eps, w, False)
        x = x.materialize()
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
