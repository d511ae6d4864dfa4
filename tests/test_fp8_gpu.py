"""W8A8 fp8-e4m3 path (csrc/kernels/fp8.hip) vs its fp32 PyTorch references.

* quant_rows: the fused (residual +) RMSNorm + per-row quantisation must produce the reference bytes (a rare one-code
  difference at a rounding tie is tolerated) and the reference scales;
* qlinear: given the SAME quantised operands the block-scaled MFMA GEMM / fp8 GEMV must equal an fp32 matmul of the
  dequantised operands up to accumulation order and the bf16 output rounding — at decode and prefill row counts,
  with partial M tiles, the fused SwiGLU epilogue, and a one-hot probe that pins the operand/output layouts;
* the fp8 model tracks the bf16 model (same random weights) and the engine still emits schema-valid verdicts.
"""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from chronos import ops

    ops.load()


def _deq(q, s):
    return q.view(torch.float8_e4m3fn).float() * s.float()[:, None]


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("rows,d", [(1, 4096), (37, 4096), (3, 14336), (5, 1024)])
def test_quant_rows(mode, rows, d):
    from chronos import ops
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(rows * d + mode)
    x = (torch.randn(rows, 2 * d if mode == 3 else d, device=DEV, generator=g) * 3 + 0.25).to(torch.bfloat16)
    x[0, 7] = 40.0  # one outlier sets the row scale
    w = (torch.rand(d, device=DEV, generator=g) + 0.5).to(torch.bfloat16)
    r1 = torch.randn(rows, d, device=DEV, generator=g).to(torch.bfloat16)
    r2 = r1.clone()
    q, s = ops.quant_rows(x, r1 if mode == 2 else None, w if mode else None, 1e-5, mode)
    qr, sr = ref.quant_rows(x, r2 if mode == 2 else None, w if mode else None, 1e-5, mode)
    if mode == 2:
        assert torch.equal(r1, r2)
    torch.testing.assert_close(s, sr, rtol=1e-6, atol=0)
    same = (q == qr).float().mean().item()
    assert same > 0.99, f"only {same:.4f} of the bytes match"  # hardware vs torch rounding of subnormals / ties
    # any mismatch is a one-code rounding difference
    diff = (_deq(q, s) - _deq(qr, sr)).abs()
    step = _deq(qr, sr).abs() / 8 + s[:, None] * 2 ** -9
    assert bool((diff <= step).all())


def _qpair(m, n, k, g, swiglu=False):
    from chronos.ops import reference as ref

    x = (torch.randn(m, k, device=DEV, generator=g) + 0.1).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV, generator=g) * 0.02 + 0.001 * torch.arange(k, device=DEV) / k)
    w = w.to(torch.bfloat16)
    xq, xs = ref.quant_rows(x)
    wq, ws = ref.quantize_weight(w)
    return xq.contiguous(), xs.contiguous(), wq, ws


@pytest.mark.parametrize("m", [1, 2, 3, 4, 5, 8, 64, 130, 1024])
@pytest.mark.parametrize("n,k,swiglu", [(6144, 4096, False), (4096, 14336, False), (28672, 4096, True),
                                        (384, 1024, False), (256, 2048, True)])
def test_qlinear(m, n, k, swiglu):
    """The hand-written kernels (torch.ops.chronos.qlinear: fp8 GEMV at M <= 4, block-scaled MFMA GEMM above) and the
    routed op (ops.qlinear: those kernels or hipBLASLt fp8 by shape) against the fp32 reference."""
    from chronos import ops
    from chronos.ops import reference as ref

    if m >= 1024 and n * k > 6144 * 4096:
        pytest.skip("large shapes covered at M <= 130")
    g = torch.Generator(device=DEV).manual_seed(m * 7 + n + k)
    xq, xs, wq, ws = _qpair(m, n, k, g, swiglu)
    yr = ref.qlinear(xq, xs, wq, ws, swiglu)
    tol = dict(rtol=2e-2, atol=2e-2 * float(yr.float().abs().mean()) + 1e-6)
    torch.testing.assert_close(ops.qlinear(xq, xs, wq, ws, swiglu).float(), yr.float(), **tol)
    if swiglu:
        aq, asc = ops.qgate_up_quant(xq, xs, wq, ws)
        torch.testing.assert_close(_deq(aq, asc), yr.float(), rtol=0.07, atol=tol["atol"] * 4)
    y = torch.ops.chronos.qlinear(xq, xs, wq, ws, swiglu)
    assert y.shape == yr.shape == (m, n // 2 if swiglu else n)
    torch.testing.assert_close(y.float(), yr.float(), **tol)
    if m <= 4:  # fp8 GEMV: one workgroup per row group, and an uneven 37-workgroup loop, give the same bits
        for persist in (0, 37):
            torch.ops.chronos.set_knob("gemv_persist", persist)
            try:
                assert torch.equal(torch.ops.chronos.qlinear(xq, xs, wq, ws, swiglu), y)
            finally:
                torch.ops.chronos.set_knob("gemv_persist", -1)


@pytest.mark.parametrize("tile", [128, 256])
@pytest.mark.parametrize("m,n,k,swiglu", [(130, 6144, 4096, False), (300, 2048, 14336, False), (512, 1024, 4096, True),
                                          (1024, 28672, 4096, True)])
def test_qlinear_tile_geometries(tile, m, n, k, swiglu):
    """Both MFMA tile geometries (forced through the kernel knob) at partial and full M tiles."""
    from chronos import ops
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(m + n + tile)
    xq, xs, wq, ws = _qpair(m, n, k, g, swiglu)
    torch.ops.chronos.set_knob("qgemm_tile", tile)
    try:
        y = torch.ops.chronos.qlinear(xq, xs, wq, ws, swiglu)
    finally:
        torch.ops.chronos.set_knob("qgemm_tile", 0)
    yr = ref.qlinear(xq, xs, wq, ws, swiglu)
    torch.testing.assert_close(y.float(), yr.float(), rtol=2e-2, atol=2e-2 * float(yr.float().abs().mean()) + 1e-6)


@pytest.mark.parametrize("m", [1, 4, 200, 700])
def test_qlinear_onehot_layout(m):
    """x row i = one-hot at column c_i (exact in e4m3): y[i, :] must be W[:, c_i] * scales — pins which token row, which
    output column and which k every lane's bytes belong to (a transposed or k-permuted operand fails)."""
    from chronos import ops
    from chronos.ops import reference as ref

    k, n = 2048, 512
    g = torch.Generator(device=DEV).manual_seed(m)
    cols = torch.randint(0, k, (m,), device=DEV, generator=g)
    xq = torch.zeros(m, k, dtype=torch.float8_e4m3fn, device=DEV)
    xq[torch.arange(m, device=DEV), cols] = 1.0
    xq = xq.view(torch.uint8)
    xs = torch.rand(m, device=DEV, generator=g) + 0.5
    w = torch.randn(n, k, device=DEV, generator=g).to(torch.bfloat16)
    wq, ws = ref.quantize_weight(w)
    y = torch.ops.chronos.qlinear(xq, xs, wq, ws, False)
    want = (_deq(wq, ws)[:, cols].t() * xs[:, None]).to(torch.bfloat16)
    torch.testing.assert_close(y.float(), want.float(), rtol=1e-2, atol=1e-6)


def test_fp8_model_tracks_bf16_and_engine_valid():
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.models.llama import build_model, make_prefill_batch, KVCache
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    mb = build_model("small", DEV, seed=3)
    mq = build_model("small", DEV, seed=3, weight_dtype="fp8")
    prompts = [list(range(100, 160)), list(range(7, 90))]
    outs = []
    for m in (mb, mq):
        kv = KVCache(m.cfg, m.tp, 64, 16, DEV)
        bts = [list(range(0, 8)), list(range(8, 16))]
        sb = make_prefill_batch(prompts, [0, 0], bts, m.cfg, m.tp, DEV, max_blocks=16, nqt=8)
        outs.append(m.forward(sb, kv).float())
    cos = torch.nn.functional.cosine_similarity(outs[0], outs[1], dim=-1)
    assert float(cos.min()) > 0.98, cos
    eng = Engine(EngineConfig(model="small", device=DEV, max_slots=8, max_model_len=512, weight_dtype="fp8"))
    reqs = [eng.submit(build_prompt(["[EXEC] bash -> curl", f"[OPEN] curl -> /tmp/x{i}"]), fmt=VERDICT_SCHEMA,
                       num_predict=48) for i in range(5)]
    eng.run_until_idle()
    for r in reqs:
        assert {"risk_score", "verdict", "reason"} <= set(json.loads(r.text))


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("m,n,k,swiglu,splitk", [(300, 2048, 2048, False, 1), (257, 1024, 4096, True, 1),
                                                 (130, 2052, 1024, False, 2), (77, 512, 2048, True, 4)])
def test_qgemm_lg(cfg, m, n, k, swiglu, splitk):
    """gemm_lg.hip's fp8 configs (ring schedule, one v_mfma_scale_f32_16x16x128_f8f6f4 k-step per 128-B stage) against
    the fp32 reference: partial M and N tiles (N % 4 only, plain), SwiGLU, split-K (tickets left at zero: 3 calls)."""
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(cfg * 31 + m + n + k)
    xq, xs, wq, ws = _qpair(m, n, k, g, swiglu)
    yr = ref.qlinear(xq, xs, wq, ws, swiglu)
    tol = dict(rtol=2e-2, atol=2e-2 * float(yr.float().abs().mean()) + 1e-6)
    for _ in range(3):
        y = torch.ops.chronos.qgemm_lg(xq, xs, wq, ws, swiglu, cfg, splitk)
        assert y.shape == yr.shape
        torch.testing.assert_close(y.float(), yr.float(), **tol)


@pytest.mark.parametrize("m,n,k,swiglu", [(300, 512, 128, False), (520, 1024, 1152, True), (600, 776, 1152, False),
                                          (1, 256, 384, False)])
def test_qgemm_lg_hb_slab_counts(m, n, k, swiglu):
    """fp8 config 4 (the HB slab loop on v_mfma_scale_f32_32x32x64_f8f6f4, unrolled by two slabs): one slab, an odd
    number of slabs, a partial W tile in the staged epilogue, one row."""
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(m + n + k)
    xq, xs, wq, ws = _qpair(m, n, k, g, swiglu)
    yr = ref.qlinear(xq, xs, wq, ws, swiglu)
    y = torch.ops.chronos.qgemm_lg(xq, xs, wq, ws, swiglu, 4, 1)
    torch.testing.assert_close(y.float(), yr.float(), rtol=2e-2, atol=2e-2 * float(yr.float().abs().mean()) + 1e-6)


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
def test_qgemm_lg_onehot_layout(cfg):
    """One-hot x rows (exact in e4m3): pins the fp8 fragment layout (row, column, k of every lane's 32 bytes)."""
    from chronos.ops import reference as ref

    m, k, n = 300, 2048, 512
    g = torch.Generator(device=DEV).manual_seed(cfg)
    cols = torch.randint(0, k, (m,), device=DEV, generator=g)
    xq = torch.zeros(m, k, dtype=torch.float8_e4m3fn, device=DEV)
    xq[torch.arange(m, device=DEV), cols] = 1.0
    xq = xq.view(torch.uint8)
    xs = torch.rand(m, device=DEV, generator=g) + 0.5
    w = torch.randn(n, k, device=DEV, generator=g).to(torch.bfloat16)
    wq, ws = ref.quantize_weight(w)
    y = torch.ops.chronos.qgemm_lg(xq, xs, wq, ws, False, cfg, 1)
    want = (_deq(wq, ws)[:, cols].t() * xs[:, None]).to(torch.bfloat16)
    torch.testing.assert_close(y.float(), want.float(), rtol=1e-2, atol=1e-6)
