"""Projection GEMMs.

``linear(x, w)`` computes ``x @ w.T`` for weights stored [out, in] (HF layout); ``gate_up_silu`` is the fused K8+K9.
Routing is by measured shape:

* M <= 2 (single-stream decode): the hand-written GEMV (csrc/kernels/gemv.hip), 1 KiB row-contiguous weight
  streaming — beats hipBLASLt on every decode shape;
* M >= 3: the hand-written MFMA GEMM families with their fused epilogues — the decoder's residual add + RMSNorm
  partial sums on O / down (``gemv_resid`` -> ResidOut), the folded RMSNorm as a per-row scale on QKV / gate_up / LM
  head (a LazyNorm input), SwiGLU on gate_up: the skinny-M weight-streaming kernel (csrc/kernels/gemm_skinny.hip,
  M <= 128: jump-forward forwards, tail decode buckets) and the ping-pong tile GEMM (csrc/kernels/gemm_pp.hip) above,
  with the kernel, tile config and split-K of the measured plan (``gemm_plan.json``: per (N, K, epilogue) the best
  by M range, from ``scripts/tune_gemm_pp.py`` on one MI355X, random operands, cold weights; plan cfg >= 100 is
  skinny config cfg - 100);
* hipBLASLt (torch.matmul) only where the plan records that the library wins by more than 3 % (the "plain library
  GEMM" rule), or for shapes the kernel does not take (K % 64, N % 4).  CHRONOS_PP=lib|own|auto forces a side.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Optional

import torch

# Largest M routed to the GEMV (gemv_ok).  Env CHRONOS_GEMV_MAX_M; scripts/single_stream.py A/Bs it (py_gemv_max_m).
# M = 2 goes to the skinny MFMA GEMM: the two-row GEMV streams at 1-3.5 TB/s against 4-5.5 at M = 1 and the skinny
# kernel's 3.4-4.9 at M = 3 (profiles/r3_gemm_table.md).
GEMV_MAX_M = int(os.environ.get("CHRONOS_GEMV_MAX_M", "1"))

# ---- the batched GEMM family (gemm_pp.hip) ----------------------------------------------------------------------
PP_MODE = os.environ.get("CHRONOS_PP", "auto")  # auto | own | lib
PP_PLAIN, PP_SWIGLU, PP_RESID = 0, 1, 2
# x rows (BM) / W rows (BN) per tile.  0-11: gemm_pp.hip (ping-pong); 12-35: gemm_lg.hip (software-pipelined: 12-19 and
# 29-31 the ring schedule, 20-28 the 64-deep slab schedule, 32-39 mid-M weight streaming with 64 W rows, 72-75 the
# same for M <= 32 with 32-row x tiles; 76-77 192 W rows x 128 x rows; 78-79 32-row x tiles with 7 / 12-stage rings;
# 80 = 20 on 32x32x16 MFMAs; 81-89 the 4-wave HB slab loop, 256 x 256 tiles, no split-K: 86 / 87 precomputed addressing
# (87: hipBLASLt's DMA distribution), 88 / 89 the same + the LDS-staged epilogue, 90 = 88 with the next slab's
# fragment reads from MFMA 94)
_PP_BM = {0: 256, 1: 128, 2: 256, 3: 128, 4: 256, 5: 128, 6: 256, 7: 128, 8: 256, 9: 128, 10: 256, 11: 128,
          12: 256, 13: 128, 14: 256, 15: 128, 16: 256, 17: 128, 18: 256, 19: 128, 20: 256, 21: 256, 22: 128, 23: 128,
          24: 256, 25: 128, 26: 256, 27: 128, 28: 128, 29: 128, 30: 256, 31: 128, 32: 128, 33: 64, 34: 128, 35: 256,
          36: 64, 37: 128, 38: 64, 39: 64, 72: 32, 73: 32, 74: 32, 75: 32, 76: 128, 77: 128, 78: 32, 79: 32, 80: 256,
          **{c: 256 for c in range(81, 95)}}
_PP_BN = {0: 256, 1: 256, 2: 128, 3: 128, 4: 256, 5: 256, 6: 128, 7: 128, 8: 256, 9: 256, 10: 128, 11: 128,
          12: 256, 13: 256, 14: 128, 15: 128, 16: 256, 17: 256, 18: 128, 19: 128, 20: 256, 21: 256, 22: 256, 23: 128,
          24: 256, 25: 256, 26: 256, 27: 256, 28: 128, 29: 256, 30: 128, 31: 128, 32: 64, 33: 64, 34: 64, 35: 64, 36: 64, 37: 64, 38: 128, 39: 64, 72: 64, 73: 128, 74: 64, 75: 128, 76: 192, 77: 192, 78: 128, 79: 64, 80: 256,
          **{c: 256 for c in range(81, 95)}}
HB_FIRST, HB_LAST = 81, 94  # gemm_lg.hip HB configs (91: the 32x32x16 MFMA form; 92 / 93: 88 / 89 + square order;
# 94: 92 + the set-0 reads from MFMA 94)
HB_SPLITK = (88, 89, 90, 91, 92, 93, 94)  # ... with the staged epilogue: the only ones with a split-K path
LG_FIRST = 12  # first gemm_lg.hip config: kResid partials every BN/2 columns (gemm_pp: BN/4)
# relative per-CU MAC rate of each tile config at full occupancy (gate_up M = 1024 / 16384 sweeps, profiles/r3_gemm_pp_*,
# profiles/r4_gemm_lg_*)
_PP_RATE = {0: 1.0, 1: 0.84, 2: 0.84, 3: 0.66, 4: 1.0, 5: 0.71, 6: 0.73, 7: 0.6, 8: 1.0, 9: 0.84, 10: 0.84, 11: 0.66,
            12: 0.95, 13: 0.7, 14: 0.7, 15: 0.75, 16: 0.98, 17: 0.7, 18: 0.7, 19: 0.75, 20: 1.05, 21: 0.7, 22: 0.7,
            23: 0.75, 24: 1.1, 25: 0.8, 26: 1.1, 27: 0.8, 28: 0.75, 29: 0.8, 30: 0.8, 31: 0.75, 32: 0.5,
            33: 0.4, 34: 0.5, 35: 0.55, 36: 0.4, 37: 0.5, 38: 0.5, 39: 0.4, 72: 0.3,
            73: 0.3, 74: 0.3, 75: 0.3, 76: 0.75, 77: 0.7, 78: 0.3, 79: 0.3, 80: 1.05,
            **{c: 1.15 for c in range(81, 95)}}
# skinny-M configs (gemm_skinny.hip SK_CONFIGS): plan id SK_BASE + c -> (RT: W tiles of 16 rows, MT: M <= 16 MT,
# NW: waves splitting K inside the workgroup)
SK_BASE = 100
_SK = {0: (1, 1, 16), 1: (2, 1, 8), 2: (4, 1, 4), 3: (2, 2, 8), 4: (4, 2, 4), 5: (2, 4, 4), 6: (4, 4, 4),
       7: (2, 8, 4), 8: (1, 2, 16), 9: (1, 4, 16), 10: (2, 4, 8), 11: (1, 1, 8)}
SKINNY_MAX_M = 128
_plan_cache: dict = {}
_plan_table: Optional[dict] = None
_qplan_table: Optional[dict] = None


def _plan_file() -> dict:
    global _plan_table, _qplan_table
    if _plan_table is None:
        import json

        override = os.environ.get("CHRONOS_GEMM_PLAN")
        path = override or os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_plan.json")
        try:
            with open(path) as fh:
                raw = json.load(fh)
        except FileNotFoundError:
            if override:  # an explicit A/B override that does not exist must not silently measure the library
                raise FileNotFoundError(f"CHRONOS_GEMM_PLAN={override!r}: no such plan file") from None
            raw = {}
        key = lambda k: tuple(int(v) for v in k.split(","))  # noqa: E731
        _plan_table = {key(k): rows for k, rows in raw.get("plans", {}).items()}
        _qplan_table = {key(k): rows for k, rows in raw.get("qplans", {}).items()}
    return _plan_table


QLG_BASE = 10  # qplan code >= QLG_BASE: gemm_lg.hip's fp8 config (code - QLG_BASE), row [M, code, split-K]
QLG_GEO = {0: (128, 256), 1: (256, 128), 2: (128, 128), 3: (128, 128),  # fp8 config -> (x rows, W rows) per tile
           4: (256, 256)}  # 4: the HB slab loop on the 32x32x64 fp8 MFMA (gemm_lg.hip F8HB)


def qplan_route(m: int, n: int, k: int, swiglu: bool) -> Optional[tuple[int, int]]:
    """W8A8 fp8 projection route from ops/gemm_plan.json "qplans" (``scripts/tune_gemm_pp.py --fp8``), rows
    [measured M, code(, split-K)] per (N, K, swiglu) read like the bf16 plan's: code 0 = the library's fp8 GEMM, 1 =
    fp8.hip (qgemv / block-scaled MFMA qgemm), QLG_BASE + c = gemm_lg.hip fp8 config c.  None = not measured."""
    _plan_file()
    rows = (_qplan_table or {}).get((n, k, int(swiglu)))
    if not rows:
        return None
    pick = next((r for r in rows if m <= r[0]), rows[-1])
    return int(pick[1]), int(pick[2]) if len(pick) > 2 else 1


def qplan_own(m: int, n: int, k: int, swiglu: bool) -> Optional[bool]:
    """True = a hand-written fp8 kernel (fp8.hip or gemm_lg.hip), False = the library, None = not measured."""
    r = qplan_route(m, n, k, swiglu)
    return None if r is None else r[0] != 0


def _sk_valid(c: int, m: int, n: int, k: int, mode: int, sk: int) -> bool:
    rt, mt, nw = _SK[c]
    if m > 16 * mt or k % (64 * nw * sk):
        return False
    return (rt % 2 == 0 and n % 2 == 0 and (n // 2) % (8 * rt) == 0) if mode == PP_SWIGLU else n % (16 * rt) == 0


def _sk_model(m: int, n: int, k: int, mode: int, cus: int = 256) -> Optional[tuple[int, int]]:
    """Cost-model pick of a skinny config: the narrowest x tile covering M, W tiles >= x tiles (x re-read bytes <=
    weight bytes), split-K until the grid covers the CUs twice."""
    best = None
    for c, (rt, mt, nw) in _SK.items():
        if m > 16 * mt or (mt > 1 and m <= 8 * mt):
            continue
        groups = (n // 2) // (8 * rt) if mode == PP_SWIGLU else n // (16 * rt)
        for sk in (1, 2, 4, 7, 8, 14, 16):
            if not _sk_valid(c, m, n, k, mode, sk):
                continue
            # a cross-workgroup split costs more than it hides (profiles/r3_gemm_table.md): only when the grid
            # would otherwise leave CUs idle; then the widest workgroups
            t = (sk > 1 and groups >= cus, rt < mt, -min(groups * sk, cus), sk, -nw, -rt)
            if best is None or t < best[0]:
                best = (t, (SK_BASE + c, sk))
    return best[1] if best else None


def _pp_valid(cfg: int, n: int, k: int, mode: int, sk: int, m: int = 0) -> bool:
    if cfg >= SK_BASE:
        return cfg - SK_BASE in _SK and _sk_valid(cfg - SK_BASE, m, n, k, mode, sk)
    bn = _PP_BN[cfg]
    if k % 64 or (k // 64) % sk or (HB_FIRST <= cfg <= HB_LAST and sk != 1 and cfg not in HB_SPLITK):
        return False
    return n % 4 == 0 if mode == PP_PLAIN else n % bn == 0


def _pp_model(m: int, n: int, k: int, mode: int, cus: int = 256) -> tuple[int, int]:
    """Cost-model pick for a shape the measured plan does not list: whole rounds of tiles over the CUs at each
    config's per-CU rate, plus the split-K slab traffic."""
    best, arg = None, (0, 1)
    for cfg in (0, 1, 2, 3):
        bm, bn = _PP_BM[cfg], _PP_BN[cfg]
        tiles = -(-m // bm) * -(-n // bn)
        for sk in (1, 2, 4):
            if not _pp_valid(cfg, n, k, mode, sk) or (sk > 1 and tiles * sk > 2 * cus):
                continue
            rounds = -(-tiles * sk // cus)
            t = rounds * bm * bn * (k // sk) / _PP_RATE[cfg] / 256.0 ** 2 + (sk > 1) * tiles * sk * bm * bn * 4 / 5e5
            if best is None or t < best:
                best, arg = t, (cfg, sk)
    return arg


def pp_plan(m: int, n: int, k: int, mode: int = PP_PLAIN) -> Optional[tuple[int, int]]:
    """(config, split-K) of the hand-written batched GEMM for this shape — config >= SK_BASE is the skinny kernel —
    or None for the library."""
    if m <= GEMV_MAX_M or PP_MODE == "lib":
        return None
    key = (m, n, k, mode)
    hit = _plan_cache.get(key, False)
    if hit is not False:
        return hit
    out = None
    if k % 64 == 0 and (n % 4 == 0 if mode == PP_PLAIN else n % 128 == 0):
        rows = _plan_file().get((n, k, mode))
        if PP_MODE == "own":
            out = (_sk_model(m, n, k, mode) if m <= SKINNY_MAX_M else None) or _pp_model(m, n, k, mode)
        elif rows:
            # rows [measured M, cfg, split-K] sorted by M: a measured M decides (previous M, M]; the last row also
            # everything above it.  cfg < 0 = the library measured faster.
            pick = next((r for r in rows if m <= r[0]), rows[-1])
            out = None if pick[1] < 0 else (pick[1], pick[2])
        # auto, shape never measured: the library (a hand-written config is routed only on a recorded A/B)
        if out is not None and not _pp_valid(out[0], n, k, mode, out[1], m):
            out = None
    _plan_cache[key] = out
    return out


def pp_gemm(x: torch.Tensor, w: torch.Tensor, mode: int, plan: tuple[int, int], resid=None, part=None,
            eps: float = 1e-5):
    """One launch of gemm_pp.hip (or gemm_skinny.hip for a skinny plan): returns (y, partials) — partials only for
    the residual epilogue."""
    from . import _k

    k = x.shape[-1]
    if plan[0] >= SK_BASE:
        return _k().gemm_skinny(x.reshape(-1, k), w, mode, plan[0] - SK_BASE, plan[1], resid, part, eps)
    y, pt = _k().gemm_pp(x.reshape(-1, k), w, mode, plan[0], plan[1], resid, part, eps, False)
    return y, pt

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


def is_q(w) -> bool:
    """An fp8 projection weight (models/llama.py QTensor: e4m3 bytes ``q`` [N, K] + per-row scales ``s``)."""
    return not isinstance(w, torch.Tensor) and hasattr(w, "q") and hasattr(w, "s")


def gemv_q_ok(m: int, n: int, k: int) -> bool:
    """Shapes of the W8A16 decode GEMV (gemv.hip WQ: fp8 weights, bf16 activations): up to 4 rows (the fused
    norm / RoPE / residual epilogues: 2), whole 1 KiB weight chunks."""
    return m <= 4 and k % 1024 == 0 and n % 16 == 0


def _q_fallback(x, w, swiglu: bool = False) -> torch.Tensor:
    """fp8 weight off the W8A16 GEMV shapes: quantise the activations and run the W8A8 op."""
    from . import qlinear, quant_rows

    xq, xs = quant_rows(LazyNorm.force(x).reshape(-1, w.shape[1]))
    y = qlinear(xq, xs, w.q, w.s, swiglu)
    return y.view(*x.shape[:-1], y.shape[-1])


def gemv_resid(x: torch.Tensor, w: torch.Tensor, resid: torch.Tensor) -> ResidOut:
    """Producer (O / down projection, TP=1): the new residual stream s = bf16(bf16(x @ w.T) + resid) and the RMSNorm
    partial sums of s^2, in one launch — the GEMV at M <= 2, the batched GEMM's kResid epilogue above.  ``w`` may be
    an fp8 QTensor at the W8A16 GEMV shapes (resid_ok(..., fp8=True))."""
    from . import _k

    m, k = x.numel() // x.shape[-1], x.shape[-1]
    if is_q(w):
        s = torch.empty(resid.shape, dtype=resid.dtype, device=resid.device)
        part = _k().gemv_resid(x.reshape(-1, k), w.q, resid, s, w.s)
        return ResidOut(s, part)
    if m > GEMV_MAX_M:
        s, part = pp_gemm(x, w, PP_RESID, pp_plan(m, w.shape[0], k, PP_RESID), resid.reshape(m, -1))
        return ResidOut(s.view(resid.shape), part)
    s = torch.empty(resid.shape, dtype=resid.dtype, device=resid.device)
    part = _k().gemv_resid(x.reshape(-1, x.shape[-1]), w, resid, s)
    return ResidOut(s, part)


def resid_ok(m: int, n: int, k: int, fp8: bool = False) -> bool:
    """Shapes of the residual-epilogue producer: the M <= 2 GEMV shapes (gemv.hip kResid) and the batched GEMM's
    (gemm_pp.hip kResid) where the plan takes it; fp8 weights: the W8A16 GEMV shapes only."""
    if fp8:
        return m <= min(GEMV_MAX_M, 2) and gemv_q_ok(m, n, k)
    if m <= GEMV_MAX_M:
        return m <= 2 and gemv_ok(m, n, k)  # (the GEMV's residual epilogue: M <= 2)
    return pp_plan(m, n, k, PP_RESID) is not None


def gemv_ok(m: int, n: int, k: int, swiglu: bool = False) -> bool:
    """Shapes routed to the hand-written decode GEMV (csrc/kernels/gemv.hip): K % 512, N % 16, M <= GEMV_MAX_M (1 by
    default; M = 2 only below LM-head widths when raised)."""
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
    """silu(x @ gate.T) * (x @ up.T) with w_gu = [gate; up]: one fused launch (GEMV at M <= 2, the batched GEMM's
    SwiGLU epilogue above, with the folded input norm when x is a LazyNorm), else GEMM + silu_mul."""
    from . import _k, silu_mul

    if is_q(w_gu):  # fp8 weights: the W8A16 GEMV (folded norm fused when x is a LazyNorm), else W8A8
        m, n, k = (x.rows() if isinstance(x, LazyNorm) else x.numel() // x.shape[-1]), w_gu.shape[0], x.shape[-1]
        if isinstance(x, LazyNorm) and x.fusable() and m <= 2 and gemv_q_ok(m, n, k):
            return _k().gemv_normp(x.s, x.part, x.eps, w_gu.q, True, w_gu.s)
        x = LazyNorm.force(x)
        if x.is_cuda and gemv_q_ok(m, n, k):
            y = _k().gemv(x.reshape(-1, k), w_gu.q, True, w_gu.s)
            return y.view(*x.shape[:-1], y.shape[-1])
        return _q_fallback(x, w_gu, True)
    if isinstance(x, LazyNorm):
        m, n, k = x.rows(), w_gu.shape[0], x.shape[-1]
        if x.fusable() and gemv_ok(m, n, k, swiglu=True):
            return _k().gemv_normp(x.s, x.part, x.eps, w_gu, True)
        plan = pp_plan(m, n, k, PP_SWIGLU) if x.fusable() else None
        if plan is not None:
            y, _ = pp_gemm(x.s, w_gu, PP_SWIGLU, plan, None, x.part, x.eps)
            return y.view(*x.shape[:-1], n // 2)
        x = x.materialize()
    if x.is_cuda:
        m, n, k = x.numel() // x.shape[-1], w_gu.shape[0], x.shape[-1]
        if gemv_ok(m, n, k, swiglu=True):
            return _gemv(x, w_gu, True)
        plan = pp_plan(m, n, k, PP_SWIGLU)
        if plan is not None:
            y, _ = pp_gemm(x, w_gu, PP_SWIGLU, plan)
            return y.view(*x.shape[:-1], n // 2)
        if mfma_swiglu_ok(m, n, k):
            return mfma_gemm(x, w_gu, True)
    return silu_mul(linear(x, w_gu))


def linear(x, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if is_q(w):  # fp8 weights: the W8A16 GEMV (folded norm fused when x is a LazyNorm), else W8A8
        from . import _k

        m, n, k = (x.rows() if isinstance(x, LazyNorm) else x.numel() // x.shape[-1]), w.shape[0], x.shape[-1]
        if isinstance(x, LazyNorm) and x.fusable() and m <= 2 and gemv_q_ok(m, n, k):
            return _k().gemv_normp(x.s, x.part, x.eps, w.q, False, w.s)
        x = LazyNorm.force(x)
        if x.is_cuda and gemv_q_ok(m, n, k):
            y = _k().gemv(x.reshape(-1, k), w.q, False, w.s)
            return y.view(*x.shape[:-1], n)
        return _q_fallback(x, w)
    if isinstance(x, LazyNorm):
        m, n, k = x.rows(), w.shape[0], x.shape[-1]
        if x.fusable() and out is None and gemv_ok(m, n, k):
            from . import _k

            return _k().gemv_normp(x.s, x.part, x.eps, w, False)
        plan = pp_plan(m, n, k, PP_PLAIN) if x.fusable() and out is None else None
        if plan is not None:
            y, _ = pp_gemm(x.s, w, PP_PLAIN, plan, None, x.part, x.eps)
            return y.view(*x.shape[:-1], n)
        x = x.materialize()
    if x.is_cuda:
        m, k = x.numel() // x.shape[-1], x.shape[-1]
        n = w.shape[0]
        if gemv_ok(m, n, k):
            return _gemv(x, w)
        for pred, fn in _custom:
            if pred(m, n, k):
                return fn(x, w)
        plan = pp_plan(m, n, k, PP_PLAIN) if out is None else None
        if plan is not None:
            y, _ = pp_gemm(x, w, PP_PLAIN, plan)
            return y.view(*x.shape[:-1], n)
    if out is not None:
        return torch.matmul(x, w.t(), out=out)
    return torch.matmul(x, w.t())
