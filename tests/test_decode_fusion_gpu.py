"""Fused decode-step kernels (csrc/kernels/gemv.hip NORM / ROPE variants) and the decode early-exit gate.

Each fused op is checked against the unfused kernel chain it replaces (standalone RMSNorm -> GEMV, GEMV -> RoPE +
paged-KV write): same bits where the arithmetic order is the same, fp32-reference tolerance otherwise.  The gate test
arms it on an all-finished state vector and checks that every gated kernel leaves its outputs untouched.
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
    import chronos.native as n

    assert "_C" in n._loaded, "HIP kernel library must be the one running"


@pytest.fixture(autouse=True)
def _two_row_gemv(monkeypatch):
    """These tests pin the GEMV kernels at M = 1 and 2; the engine routes M = 2 to the skinny GEMM by default
    (ops/gemm.py GEMV_MAX_M), so the two-row GEMV variants are exercised here explicitly."""
    from chronos.ops import gemm

    monkeypatch.setattr(gemm, "GEMV_MAX_M", 2)


@pytest.fixture(params=[0, 37], ids=["grid", "persist37"])
def persist(request):
    """gemv.hip knob gemv_persist: 0 = one workgroup per row group; 37 = a 37-workgroup grid looping over the groups
    with the next group's weight ring prefetched (uneven: some workgroups get one group more)."""
    torch.ops.chronos.set_knob("gemv_persist", request.param)
    yield request.param
    torch.ops.chronos.set_knob("gemv_persist", -1)


def _rand(g, *shape, scale=1.0):
    return (torch.randn(*shape, device=DEV, generator=g) * scale).to(torch.bfloat16)


def _close(a, b, atol, rtol):
    d = (a.float() - b.float()).abs()
    assert bool((d <= atol + rtol * b.float().abs()).all()), f"max err {float(d.max()):.4g}"


@pytest.mark.parametrize("m", [1, 2])
@pytest.mark.parametrize("n_out", [4096, 8192])
def test_gemv_resid_producer(m, n_out, persist):
    """resid_out = bf16(bf16(x W^T) + resid) bit-exact vs GEMV + add; partials sum to sum(resid_out^2)."""
    from chronos import ops
    from chronos.ops import gemm

    g = torch.Generator(device=DEV).manual_seed(m + n_out)
    x = _rand(g, m, 4096)
    w = _rand(g, n_out, 4096, scale=0.02)
    r = _rand(g, m, n_out)
    out = ops.gemv_resid(x, w, r)
    exp = (gemm._gemv(x, w).float() + r.float()).to(torch.bfloat16)
    assert torch.equal(out.s, exp)
    # rows per workgroup: 4 at M = 1 (gemv.hip resid_rows default, while N / 4 <= 2048), 8 at M = 2
    assert out.part.shape == (m, n_out // (4 if m == 1 and n_out // 4 <= 2048 else 8))
    ss = exp.float().pow(2).sum(-1)
    _close(out.part.sum(-1), ss, 1e-3, 1e-5)


@pytest.mark.parametrize("m", [1, 2])
@pytest.mark.parametrize("swiglu,n", [(False, 6144), (True, 2 * 1792)])
def test_gemv_normp_consumer(m, swiglu, n, persist):
    """The folded norm (norm weight inside W, inv from the producer's partials) equals the standalone RMSNorm -> GEMV
    on the unfolded weights, to bf16 rounding; and it is deterministic."""
    from chronos import ops
    from chronos.models.llama import fold_norm
    from chronos.ops import gemm

    g = torch.Generator(device=DEV).manual_seed(m * 3 + n)
    x = _rand(g, m, 4096)
    wo = _rand(g, 4096, 4096, scale=0.02)
    r = _rand(g, m, 4096, scale=2.0)
    nw = (torch.rand(4096, device=DEV, generator=g) + 0.5).to(torch.bfloat16)
    w = _rand(g, n, 4096, scale=0.02)
    wf = fold_norm(w, nw)
    ones = torch.ones_like(nw)
    prod = ops.gemv_resid(x, wo, r)
    ln = ops.LazyNorm(prod.s, prod.part, ones, 1e-5)
    y = ops.gate_up_silu(ln, wf) if swiglu else ops.linear(ln, wf)
    y_ref = gemm._gemv(ops.rmsnorm(prod.s, nw, 1e-5), w, swiglu)
    _close(y, y_ref, 2.5e-2, 2.5e-2)  # |err| ~ 2^-9 * std(y) per rounding (W diag(w) and s * inv), absolute
    ln2 = ops.LazyNorm(prod.s, prod.part, ones, 1e-5)
    y2 = ops.gate_up_silu(ln2, wf) if swiglu else ops.linear(ln2, wf)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("m,hq,hkv", [(1, 32, 8), (2, 32, 8), (1, 8, 1)])
@pytest.mark.parametrize("folded", [False, True])
def test_qkv_rope_equals_unfused(fp8, m, hq, hkv, folded, persist):
    """QKV GEMV + RoPE/paged-KV epilogue == GEMV then rope_kv_write (bit-exact on a plain input; with the folded norm
    — norm weight inside W, inv from partials — against the standalone-norm chain, to bf16 rounding)."""
    from chronos import ops
    from chronos.models.llama import get_config, rope_table
    from chronos.ops import gemm

    g = torch.Generator(device=DEV).manual_seed(hq + m + fp8 + 10 * folded)
    k, bs, nb = 4096, 16, 40
    s = _rand(g, m, k, scale=2.0)
    w = _rand(g, (hq + 2 * hkv) * 128, k, scale=0.02)
    nw = (torch.rand(k, device=DEV, generator=g) + 0.5).to(torch.bfloat16)
    cs = rope_table(get_config("llama3.1-8b"), 2048, DEV)
    bt = torch.randperm(nb, device=DEV, generator=g).to(torch.int32).view(2, nb // 2)
    pos = torch.tensor([333, 17][:m], dtype=torch.int32, device=DEV)
    tok_seq = torch.arange(m, dtype=torch.int32, device=DEV)
    if fp8:
        kc = torch.randint(0, 100, (nb, hkv, bs, 128), dtype=torch.uint8, device=DEV)
        vc = torch.randint(0, 100, (nb, hkv, 128, bs), dtype=torch.uint8, device=DEV)
        ks, vs = 0.5, 0.25
    else:
        kc = _rand(g, nb, hkv, bs, 128)
        vc = _rand(g, nb, hkv, 128, bs)
        ks = vs = 1.0
    kc2, vc2 = kc.clone(), vc.clone()
    q1 = torch.zeros(m, hq, 128, device=DEV, dtype=torch.bfloat16)
    q2 = torch.zeros_like(q1)
    x = ops.rmsnorm(s, nw, 1e-5)
    ops.rope_kv_write(gemm._gemv(x, w), pos, tok_seq, bt, cs, q2, kc2, vc2, hq, hkv, True, ks, vs)
    if folded:
        from chronos.models.llama import fold_norm

        part = s.float().pow(2).view(m, -1, 8).sum(-1).contiguous()  # a producer's partials for s
        src, wq = ops.LazyNorm(s, part, torch.ones_like(nw), 1e-5), fold_norm(w, nw)
    else:
        src, wq = x, w
    assert ops.qkv_rope(src, wq, pos, tok_seq, bt, cs, q1, kc, vc, hq, hkv, ks, vs)
    torch.cuda.synchronize()
    if folded:
        _close(q1, q2, 2e-2, 2e-2)
        if fp8:  # dequantised e4m3: one rounding step (2^-3 relative) or a near-zero sign flip apart
            f8 = lambda t: t.view(torch.float8_e4m3fn).float()  # noqa: E731
            _close(f8(kc), f8(kc2), 4e-2 / ks, 0.13)
            _close(f8(vc), f8(vc2), 4e-2 / vs, 0.13)
        else:
            _close(kc, kc2, 2e-2, 2e-2)
            _close(vc, vc2, 2e-2, 2e-2)
    else:
        assert torch.equal(q1, q2)
        assert torch.equal(kc, kc2)
        assert torch.equal(vc, vc2)


def test_decode_gate_skips_finished_steps(persist):
    """Armed on a state vector with no live row, in-place kernels (residual norm, fused QKV + KV write) leave their
    outputs untouched; one live row and they run again."""
    from chronos import ops
    from chronos.models.llama import get_config, rope_table

    g = torch.Generator(device=DEV).manual_seed(3)
    hq, hkv, k = 8, 1, 4096
    x = _rand(g, 1, k)
    r = _rand(g, 1, k)
    nw = (torch.rand(k, device=DEV, generator=g) + 0.5).to(torch.bfloat16)
    w = _rand(g, (hq + 2 * hkv) * 128, k, scale=0.02)
    cs = rope_table(get_config("llama3-8b"), 64, DEV)
    bt = torch.arange(4, dtype=torch.int32, device=DEV).view(1, 4)
    pos = torch.tensor([5], dtype=torch.int32, device=DEV)
    ts = torch.zeros(1, dtype=torch.int32, device=DEV)
    kc, vc = _rand(g, 4, hkv, 16, 128), _rand(g, 4, hkv, 128, 16)
    q = torch.zeros(1, hq, 128, device=DEV, dtype=torch.bfloat16)
    r0, kc0, vc0 = r.clone(), kc.clone(), vc.clone()
    state = torch.tensor([0, -1, 0, 0], dtype=torch.int32, device=DEV)  # DONE / empty: nothing live

    def run():
        ops.add_rmsnorm(x, r, nw, 1e-5)
        assert ops.qkv_rope(x, w, pos, ts, bt, cs, q, kc, vc, hq, hkv)

    try:
        ops.set_decode_gate(state, 4)
        run()
        torch.cuda.synchronize()
        assert torch.equal(r, r0) and torch.equal(kc, kc0) and torch.equal(vc, vc0)
        assert not bool(q.abs().sum())
        state[2] = 5  # one live row: the same launches compute again
        run()
        torch.cuda.synchronize()
    finally:
        ops.set_decode_gate(None, 0)
    assert not torch.equal(r, r0) and not torch.equal(kc, kc0) and not torch.equal(vc, vc0)
    assert bool(q.abs().sum())


def test_engine_fused_decode_matches_unfused(monkeypatch):
    """Greedy verdicts with the fused decode path + gate vs the separate kernels (one stream and two, graphs on): the
    folded norm sums squares in another order, so the first tokens must agree and the verdicts must parse; the fused
    engine is deterministic run to run."""
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.models import llama
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    chains = [["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"],
              ["[EXEC] bash -> chmod", "[OPEN] chmod -> /tmp/x", "[EXEC] bash -> cat"]]
    outs = []
    for fuse in (True, False, True):
        monkeypatch.setattr(llama, "_FUSE_NORM", fuse)
        res = []
        for n in (1, 2):
            eng = Engine(EngineConfig(model="small", device=DEV, max_slots=n, max_model_len=256, decode_burst=8,
                                      decode_gate=fuse))
            reqs = [eng.submit(build_prompt(c), fmt=VERDICT_SCHEMA, num_predict=40) for c in chains[:n]]
            eng.run_until_idle()
            for r in reqs:
                json.loads(r.text)
            res.append([r.out_ids for r in reqs])
        outs.append(res)
    assert outs[0] == outs[2]
    for a, b in zip(outs[0], outs[1]):
        for x, y in zip(a, b):
            assert x[:8] == y[:8]


def test_rope_kv_write_kv_only_layout():
    """Context-parallel gathered K/V rows ([T, 2*hkv*128], hq = 0, no q) are written like the K/V part of a full QKV
    row (parallel/context_parallel.py)."""
    from chronos import ops
    from chronos.models.llama import get_config, rope_table

    g = torch.Generator(device=DEV).manual_seed(11)
    hq, hkv, T, nb, bs = 32, 8, 77, 16, 16
    qkv = _rand(g, T, (hq + 2 * hkv) * 128)
    cs = rope_table(get_config("llama3.1-8b"), 1024, DEV)
    bt = torch.randperm(nb, device=DEV, generator=g).to(torch.int32).view(1, nb)
    pos = torch.randperm(nb * bs, device=DEV, generator=g)[:T].to(torch.int32)
    ts = torch.zeros(T, dtype=torch.int32, device=DEV)
    k1, v1 = _rand(g, nb, hkv, bs, 128), _rand(g, nb, hkv, 128, bs)
    k2, v2 = k1.clone(), v1.clone()
    q = torch.empty(T, hq, 128, device=DEV, dtype=torch.bfloat16)
    ops.rope_kv_write(qkv, pos, ts, bt, cs, q, k1, v1, hq, hkv, False)
    kv_only = qkv[:, hq * 128:].contiguous()
    ops.rope_kv_write(kv_only, pos, ts, bt, cs, q[:1], k2, v2, 0, hkv, False)
    torch.cuda.synchronize()
    assert torch.equal(k1, k2) and torch.equal(v1, v2)


@pytest.mark.parametrize("nsplit", [2, 5])
def test_inlaunch_combine_matches_combine_kernel_and_replays(nsplit):
    """Split-K decode attention with the last-arriver combine inside the launch == the separate combine kernel (same
    merge code, so bit-exact), and the split tickets return to zero: a captured graph replays correctly."""
    from chronos import ops

    g = torch.Generator(device=DEV).manual_seed(nsplit)
    hq, hkv, bs, B = 32, 8, 16, 6
    ctx = [700, 33, 1, 480, 1024, 260]
    nb = sum((c + bs - 1) // bs for c in ctx) + 2
    k, v = _rand(g, nb, hkv, bs, 128), _rand(g, nb, hkv, 128, bs)
    perm = torch.randperm(nb, generator=torch.Generator().manual_seed(1)).tolist()
    bt = torch.zeros(B, 64, dtype=torch.int32)
    o = 0
    for b, c in enumerate(ctx):
        n = (c + bs - 1) // bs
        bt[b, :n] = torch.tensor(perm[o:o + n])
        o += n
    bt = bt.to(DEV)
    q = _rand(g, B, hq, 128, scale=2.0)
    qs = torch.arange(B + 1, dtype=torch.int32, device=DEV)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    run = lambda: ops.paged_attention(q, k, v, bt, qs, cl, None, B, 1, nsplit)  # noqa: E731
    torch.ops.chronos.set_knob("attn_inkernel_combine", 0)
    try:
        ref = run()
    finally:
        torch.ops.chronos.set_knob("attn_inkernel_combine", 1)
    out = run()
    assert torch.equal(out, ref)
    static = torch.empty_like(ref)
    graph = torch.cuda.CUDAGraph()
    run()
    torch.cuda.synchronize()
    with torch.cuda.graph(graph):
        static.copy_(run())
    for _ in range(3):
        static.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(static, ref)


def test_input_checks_catch_bad_indices_before_launch():
    """CHRONOS_CHECK_INPUTS debug mode: a block id past the cache, a position past the rope table or a stray grammar
    state raise IndexError on the host instead of reaching a kernel; good inputs pass; an engine runs with it on."""
    from chronos import ops
    from chronos.models.llama import get_config, rope_table

    g = torch.Generator(device=DEV).manual_seed(5)
    hq, hkv, nb, bs, T = 8, 2, 6, 16, 3
    cs = rope_table(get_config("llama3-8b"), 64, DEV)
    qkv = _rand(g, T, (hq + 2 * hkv) * 128)
    k, v = _rand(g, nb, hkv, bs, 128), _rand(g, nb, hkv, 128, bs)
    q = torch.empty(T, hq, 128, device=DEV, dtype=torch.bfloat16)
    ts = torch.zeros(T, dtype=torch.int32, device=DEV)
    pos = torch.tensor([0, 17, 40], dtype=torch.int32, device=DEV)
    ops.set_input_checks(True)
    try:
        good = torch.tensor([[1, 2, 3, 0]], dtype=torch.int32, device=DEV)
        ops.rope_kv_write(qkv, pos, ts, good, cs, q, k, v, hq, hkv)
        bad = torch.tensor([[1, 2, 99, 0]], dtype=torch.int32, device=DEV)  # block 99 of a 6-block cache
        with pytest.raises(IndexError):
            ops.rope_kv_write(qkv, pos, ts, bad, cs, q, k, v, hq, hkv)
        with pytest.raises(IndexError):  # position 500 is past the 64-row rope table
            ops.rope_kv_write(qkv, torch.tensor([0, 1, 500], dtype=torch.int32, device=DEV), ts, good, cs, q, k, v,
                              hq, hkv)
        qs = torch.arange(2, dtype=torch.int32, device=DEV)
        with pytest.raises(IndexError):
            ops.paged_attention(q[:1], k, v, bad, qs, torch.tensor([41], dtype=torch.int32, device=DEV), None, 1)
        from chronos.brain.engine.engine import Engine, EngineConfig
        from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

        eng = Engine(EngineConfig(model="small", device=DEV, max_slots=2, max_model_len=256, use_graphs=False))
        r = eng.submit(build_prompt(["[EXEC] bash -> curl", "[OPEN] curl -> /tmp/x"]), fmt=VERDICT_SCHEMA,
                       num_predict=16)
        eng.run_until_idle()
        assert r.done_reason in ("stop", "length") and r.out_ids
    finally:
        ops.set_input_checks(False)


@pytest.mark.parametrize("kv", ["bf16", "fp8"])
@pytest.mark.parametrize("spike", ["big", "small"])
@pytest.mark.parametrize("variant", [0, 2, 5])
def test_flash_prefill_forced_rescale(variant, spike, kv):
    """The flash prefill kernels' rescale paths, forced: late keys whose scores jump past the running max, against
    one query row, over a 1200-token chunk on a 900-token prefix; full-tensor fp32 reference.

    spike="big": the stage max beats the running one by far more than v2's deferred-max threshold (8 in log2 units),
    so the rescale branch runs.  spike="small": it rises by ~3-4 log2 units, below the threshold, so v2 keeps the
    stale max and accumulates p up to 2^8 (cdna_hip_programming.md §5.4 rule 26).  kv="fp8" runs the same branches
    in attn_prefill2_kernel<true> on dequantised e4m3 scores; the fp8-MFMA kernel that is the default
    for an fp8 cache has its own copy of this test (tests/test_prefill_fp8_mfma_gpu.py)."""
    from chronos import ops
    from chronos.ops import reference as ref

    torch.ops.chronos.set_knob("prefill_variant", variant)
    torch.ops.chronos.set_knob("prefill_fp8_mfma", 0)
    try:
        g = torch.Generator(device=DEV).manual_seed(123 + variant)
        hq, hkv, bs = 32, 8, 16
        q_lens, prefix = [1200], [900]
        ctx = [p + n for p, n in zip(prefix, q_lens)]
        nb = (ctx[0] + bs - 1) // bs + 1
        k = (torch.randn(nb, hkv, bs, 128, device=DEV, generator=g) * 0.3).to(torch.bfloat16)
        v = torch.randn(nb, hkv, 128, bs, device=DEV, generator=g).to(torch.bfloat16)
        bt = torch.arange(1, nb, dtype=torch.int32, device=DEV).view(1, -1)
        q = torch.randn(q_lens[0], hq, 128, device=DEV, generator=g).to(torch.bfloat16)
        # keys 1500..1563 (stage 23) of kv head 3 aligned with q rows: score jump ~+14 (big) / ~+3.5 (small) log2
        amp = 0.9 if spike == "big" else 0.25
        for t in range(1500, 1564):
            k[1 + t // bs, 3, t % bs] = (q[t - 900, 12].float() * amp).to(torch.bfloat16)
        ks = vs = 1.0
        if kv == "fp8":
            ks, vs = 0.25, 0.5
            k, v = ref.to_fp8_bytes(k, 1 / ks), ref.to_fp8_bytes(v, 1 / vs)
        qs = torch.tensor([0, q_lens[0]], dtype=torch.int32, device=DEV)
        cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
        tiles = ops.attention_tiles(q_lens, hq, hkv, 8)
        tt = torch.tensor(tiles, dtype=torch.int32, device=DEV).view(-1, 2)
        out = ops.paged_attention(q, k, v, bt, qs, cl, tt, len(tiles), 8, 1, None, ks, vs)
        exp = ref.paged_attention(q, k, v, bt, qs, cl, tt, len(tiles), 8, 1, None, ks, vs)
        d = (out.float() - exp.float()).abs()
        assert bool((d <= 2e-2 + 2e-2 * exp.float().abs()).all()), float(d.max())
    finally:
        torch.ops.chronos.set_knob("prefill_variant", 2)
        torch.ops.chronos.set_knob("prefill_fp8_mfma", 1)
