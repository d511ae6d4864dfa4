"""Numerics of every gfx950 HIP kernel vs its fp32 PyTorch reference (chronos.ops.reference).

Run on a real MI355X: ``python -m pytest tests -m gpu``.  Inputs are asymmetric random data at odd shapes (GQA
groups 4 and 8, page boundaries, varlen chunks with a cached prefix, partial last pages, split-K decode).
"""
import math

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


def _close(a, b, atol, rtol=0.0):
    d = (a.float() - b.float()).abs()
    lim = atol + rtol * b.float().abs()
    assert bool((d <= lim).all()), f"max err {float(d.max()):.4g}"


@pytest.mark.parametrize("rows,d", [(1, 4096), (37, 4096), (5, 8192), (3, 256), (2, 1024)])
def test_rmsnorm(rows, d):
    from chronos import ops
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(rows * d)
    x = torch.randn(rows, d, device=DEV, generator=g).to(torch.bfloat16) * 3 + 0.5
    w = torch.rand(d, device=DEV, generator=g).to(torch.bfloat16) + 0.5
    _close(ops.rmsnorm(x, w, 1e-5), ref.rmsnorm(x, w, 1e-5), 1e-2, 1e-2)
    r1 = torch.randn(rows, d, device=DEV, generator=g).to(torch.bfloat16)
    r2 = r1.clone()
    y1 = ops.add_rmsnorm(x, r1, w, 1e-5)
    y2 = ref.add_rmsnorm(x, r2, w, 1e-5)
    assert torch.equal(r1, r2)
    _close(y1, y2, 1e-2, 1e-2)


def test_silu_mul_and_embedding():
    from chronos import ops
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(1)
    gu = (torch.randn(19, 2 * 1408, device=DEV, generator=g) * 4).to(torch.bfloat16)
    _close(ops.silu_mul(gu), ref.silu_mul(gu), 2e-2, 1e-2)
    table = torch.randn(1000, 512, device=DEV, generator=g).to(torch.bfloat16)
    ids = torch.tensor([0, 999, 5, 500, 1200, -3 + 2000], dtype=torch.int32, device=DEV)
    assert torch.equal(ops.embedding(ids, table, 0), ref.embedding(ids, table, 0))
    assert torch.equal(ops.embedding(ids, table, 500), ref.embedding(ids, table, 500))


def _cache(nb, hkv, bs, g):
    k = (torch.randn(nb, hkv, bs, 128, device=DEV, generator=g)).to(torch.bfloat16)
    v = (torch.randn(nb, hkv, 128, bs, device=DEV, generator=g)).to(torch.bfloat16)
    return k, v


@pytest.mark.parametrize("hq,hkv,bs", [(32, 8, 16), (8, 1, 32), (4, 2, 16)])
def test_rope_kv_write(hq, hkv, bs):
    from chronos import ops
    from chronos.models.llama import get_config, rope_table
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(hq)
    T = 45
    cs = rope_table(get_config("llama3.1-8b"), 4096, DEV)
    qkv = torch.randn(T, (hq + 2 * hkv) * 128, device=DEV, generator=g).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=DEV, generator=g).to(torch.int32)
    # distinct slots: token t -> block perm[t], offset t % bs
    nb = 64
    bt = torch.randperm(nb, device=DEV, generator=g).to(torch.int32).view(1, nb)
    pos = (torch.arange(T, device=DEV) * 7 % (nb * bs)).to(torch.int32)
    tok_seq = torch.zeros(T, dtype=torch.int32, device=DEV)
    k1, v1 = _cache(nb, hkv, bs, g)
    k2, v2 = k1.clone(), v1.clone()
    q1 = torch.empty(T, hq, 128, device=DEV, dtype=torch.bfloat16)
    q2 = torch.empty_like(q1)
    ops.rope_kv_write(qkv, pos, tok_seq, bt, cs, q1, k1, v1, hq, hkv, True)
    ref.rope_kv_write(qkv, pos, tok_seq, bt, cs, q2, k2, v2, hq, hkv, True)
    _close(q1, q2, 2e-2, 1e-2)
    _close(k1, k2, 2e-2, 1e-2)
    assert torch.equal(v1, v2)


def _attn_case(q_lens, ctx_lens, hq, hkv, bs, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    B = len(q_lens)
    nbs = [(c + bs - 1) // bs for c in ctx_lens]
    nb = sum(nbs) + 3
    k, v = _cache(nb, hkv, bs, g)
    perm = torch.randperm(nb, device=DEV, generator=g).tolist()
    mb = max(nbs)
    bt = torch.zeros(B, mb, dtype=torch.int32)
    o = 0
    for b, n in enumerate(nbs):
        bt[b, :n] = torch.tensor(perm[o:o + n])
        o += n
    T = sum(q_lens)
    q = (torch.randn(T, hq, 128, device=DEV, generator=g) * 2).to(torch.bfloat16)
    qs = [0]
    for n in q_lens:
        qs.append(qs[-1] + n)
    return q, k, v, bt.to(DEV), torch.tensor(qs, dtype=torch.int32, device=DEV), \
        torch.tensor(ctx_lens, dtype=torch.int32, device=DEV)


@pytest.mark.parametrize("nqt", [1, 2, 8])
@pytest.mark.parametrize("hq,hkv,bs", [(32, 8, 16), (16, 2, 16), (8, 1, 32), (4, 4, 16)])
@pytest.mark.parametrize("nsplit", [1, 3])
def test_paged_attention_prefill(nqt, hq, hkv, bs, nsplit):
    from chronos import ops
    from chronos.ops import reference as ref

    q_lens = [1, 17, 64, 5, 100]
    ctx_lens = [1, 17, 200, 37, 100]  # seq 2 and 3 have a cached prefix (chunked prefill)
    q, k, v, bt, qs, ctx = _attn_case(q_lens, ctx_lens, hq, hkv, bs, seed=hq + nqt)
    tiles = ops.attention_tiles(q_lens, hq, hkv, nqt)
    tt = torch.tensor(tiles, dtype=torch.int32, device=DEV).view(-1, 2)
    out = ops.paged_attention(q, k, v, bt, qs, ctx, tt, len(tiles), nqt, nsplit)
    exp = ref.paged_attention(q, k, v, bt, qs, ctx, tt, len(tiles), nqt, nsplit)
    _close(out, exp, 2e-2, 2e-2)


def test_flash_prefill_long_prefix():
    """Chunked prefill of 300 tokens on a 1700-token cached prefix + a fresh 513-token prompt (flash kernel)."""
    from chronos import ops
    from chronos.ops import reference as ref

    q_lens, ctx_lens = [300, 513], [2000, 513]
    q, k, v, bt, qs, ctx = _attn_case(q_lens, ctx_lens, 32, 8, 16, seed=77)
    tiles = ops.attention_tiles(q_lens, 32, 8, 8)
    tt = torch.tensor(tiles, dtype=torch.int32, device=DEV).view(-1, 2)
    out = ops.paged_attention(q, k, v, bt, qs, ctx, tt, len(tiles), 8, 1)
    exp = ref.paged_attention(q, k, v, bt, qs, ctx, tt, len(tiles), 8, 1)
    _close(out, exp, 2e-2, 2e-2)


@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (8, 1)])
@pytest.mark.parametrize("nsplit", [1, 4, 16])
def test_paged_attention_decode(hq, hkv, nsplit):
    from chronos import ops
    from chronos.ops import reference as ref

    ctx_lens = [1, 15, 16, 33, 511, 1000, 2049]
    q, k, v, bt, qs, ctx = _attn_case([1] * len(ctx_lens), ctx_lens, hq, hkv, 16, seed=hq * nsplit)
    out = ops.paged_attention(q, k, v, bt, qs, ctx, None, len(ctx_lens), 1, nsplit)
    exp = ref.paged_attention(q, k, v, bt, qs, ctx, None, len(ctx_lens), 1, nsplit)
    _close(out, exp, 2e-2, 2e-2)


@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8)])
def test_paged_attention_decode_one_wave_kernel(hq, hkv):
    """>= 1024 (seq, kv head) items select the one-wave-per-item decode kernel: ragged contexts from 1 token to past
    the 64-entry block-table window (1100 tokens = 69 blocks), prefetch on and off, against the fp32 reference."""
    from chronos import ops
    from chronos.ops import reference as ref

    g = torch.Generator().manual_seed(hq)
    ctx_lens = torch.randint(1, 260, (260,), generator=g).tolist()
    ctx_lens[:6] = [1, 16, 17, 1024, 1025, 1100]
    q, k, v, bt, qs, ctx = _attn_case([1] * len(ctx_lens), ctx_lens, hq, hkv, 16, seed=hq + 1)
    exp = ref.paged_attention(q, k, v, bt, qs, ctx, None, len(ctx_lens), 1, 1)
    C = torch.ops.chronos
    try:
        for pf in (0, 1):
            C.set_knob("decode_pf", pf)
            out = ops.paged_attention(q, k, v, bt, qs, ctx, None, len(ctx_lens), 1, 1)
            _close(out, exp, 2e-2, 2e-2)
    finally:
        C.set_knob("decode_pf", 0)


@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8)])
def test_decode_attention_rope_fused_matches_unfused(hq, hkv):
    """Batched decode step with RoPE + paged-KV write fused into the one-wave decode attention vs rope_kv_write +
    paged_attention (and the fp32 reference): ragged contexts incl. a new token at every block offset and past the
    64-entry block-table window; the caches must hold the same new K / V afterwards."""
    _decode_rope_case(hq, hkv)


def _decode_rope_case(hq, hkv):
    from chronos import ops
    from chronos.models.llama import get_config, rope_table
    from chronos.ops import reference as ref

    g = torch.Generator().manual_seed(hq + 5)
    ctx_lens = torch.randint(1, 300, (270,), generator=g).tolist()
    ctx_lens[:20] = [1, 2, 15, 16, 17, 31, 32, 33, 1024, 1025, 1100, 47, 48, 49, 63, 64, 65, 4, 8, 12]
    B = len(ctx_lens)
    _, k1, v1, bt, qs, ctx = _attn_case([1] * B, ctx_lens, hq, hkv, 16, seed=hq + 9)
    gd = torch.Generator(device=DEV).manual_seed(hq)
    qkv = (torch.randn(B, (hq + 2 * hkv) * 128, device=DEV, generator=gd) * 2).to(torch.bfloat16)
    pos = (ctx - 1).to(torch.int32)
    cs = rope_table(get_config("llama3.1-8b"), 2048, DEV)
    tok = torch.arange(B, dtype=torch.int32, device=DEV)
    k2, v2 = k1.clone(), v1.clone()
    qb = torch.empty(B, hq, 128, device=DEV, dtype=torch.bfloat16)
    ops.rope_kv_write(qkv, pos, tok, bt, cs, qb, k2, v2, hq, hkv, True)
    exp = ops.paged_attention(qb, k2, v2, bt, qs, ctx, None, B, 1, 1)
    want = ref.paged_attention(qb, k2, v2, bt, qs, ctx, None, B, 1, 1)
    out = ops.decode_attention_rope(qkv, pos, cs, k1, v1, bt, ctx, B, hq, 1.0 / math.sqrt(128))
    assert out is not None, "the fused kernel must serve >= 1024 (row, kv head) items"
    torch.cuda.synchronize()
    _close(k1, k2, 1e-2, 1e-2)  # RoPE rounding may differ by an fma contraction
    assert torch.equal(v1, v2)
    _close(out, exp, 2e-2, 2e-2)
    _close(out, want, 2e-2, 2e-2)
    # below the one-wave threshold the op declines and the caller runs the unfused pair
    assert ops.decode_attention_rope(qkv, pos, cs, k1, v1, bt, ctx, 8, hq, 1.0 / math.sqrt(128)) is None


def test_paged_attention_spike_rescale():
    """Force the online-softmax rescale: one key dominates late in a long context."""
    from chronos import ops
    from chronos.ops import reference as ref

    q, k, v, bt, qs, ctx = _attn_case([1, 1], [700, 300], 32, 8, 16, seed=9)
    # spike key 650 of seq 0 (block index 650 // 16 of its table) against q head 0's direction
    blk = int(bt[0, 650 // 16])
    k[blk, 0, 650 % 16] = (q[0, 0].float() * 4).to(torch.bfloat16)
    out = ops.paged_attention(q, k, v, bt, qs, ctx, None, 2, 1, 1)
    exp = ref.paged_attention(q, k, v, bt, qs, ctx, None, 2, 1, 1)
    _close(out, exp, 2e-2, 2e-2)


def test_constrained_sample_matches_reference():
    from chronos import ops
    from chronos.brain.constrain import DONE, GrammarBank
    from chronos.brain.tokenizer import ChronosBPE
    from chronos.ops import reference as ref
    from chronos.sensor.prompt import VERDICT_SCHEMA

    tok = ChronosBPE()
    bank = GrammarBank(tok.token_bytes_list(), tok.stop_ids, 128256, 1024, DEV)
    gs = bank.get(VERDICT_SCHEMA)
    gj = bank.get("json")
    S = 6
    g = torch.Generator(device=DEV).manual_seed(3)
    i32 = dict(dtype=torch.int32, device=DEV)
    state = torch.tensor([gs.start, gj.start, -1, gs.start, gj.start, gs.start], **i32)
    rem = torch.tensor([40, 30, 5, 16, 3, 40], **i32)
    temp = torch.tensor([0, 0, 0, 0.7, 0, 1.3], dtype=torch.float32, device=DEV)
    seed = torch.arange(S, **i32)
    bufs1 = [torch.zeros(S, **i32) for _ in range(4)] + [torch.zeros(S, 64, **i32)]
    bufs2 = [b.clone() for b in bufs1]
    st1, st2 = state.clone(), state.clone()
    r1, r2 = rem.clone(), rem.clone()
    for step in range(45):
        logits = (torch.randn(S, 128256, device=DEV, generator=g) * 3).to(torch.bfloat16)
        ops.constrained_sample(logits, None, bank.next, bank.dist, DONE, st1, r1, temp, seed, *bufs1)
        # reference on greedy rows only (the Gumbel RNG streams differ by design)
        greedy = (temp == 0)
        st2g = torch.where(greedy, st2, torch.full_like(st2, -1))
        ref.constrained_sample(logits, None, bank.next, bank.dist, DONE, st2g, r2, temp, seed, *bufs2)
        st2 = torch.where(greedy, st2g, st1)
        r2 = torch.where(greedy, r2, r1)
        assert torch.equal(st1[greedy], st2[greedy]), step
    nout = bufs1[3]
    out = bufs1[4]
    assert torch.equal(out[temp == 0], bufs2[4][temp == 0])
    # every non-empty row finished within its budget with a grammar-valid string
    import json

    for s in [0, 1, 3, 4, 5]:
        assert int(st1[s]) == DONE, s
        ids = out[s, : int(nout[s])].tolist()
        assert ids[-1] in tok.stop_ids
        text = tok.decode(ids[:-1])
        json.loads(text)
        assert int(nout[s]) <= int(rem[s])


def test_model_gpu_matches_cpu_reference():
    from chronos.models.llama import KVCache, build_model, make_prefill_batch

    torch.manual_seed(0)
    mg = build_model("tiny", DEV, seed=5)
    mc = build_model("tiny", "cpu", seed=5)
    # same weights (generated on different devices) -> copy GPU weights to CPU model
    for lg, lc in zip(mg.w.layers, mc.w.layers):
        for n in ("attn_norm", "wqkv", "wo", "mlp_norm", "w_gu", "w_down"):
            getattr(lc, n).copy_(getattr(lg, n).cpu())
    mc.w.embed.copy_(mg.w.embed.cpu())
    mc.w.lm_head.copy_(mg.w.lm_head.cpu())
    prompts = [[128000 + 0] + list(range(10, 40)), list(range(100, 113))]
    bts = [[1, 2, 3], [4]]
    kvg = KVCache(mg.cfg, mg.tp, 8, 16, DEV)
    kvc = KVCache(mc.cfg, mc.tp, 8, 16, "cpu")
    sbg = make_prefill_batch(prompts, [0, 0], bts, mg.cfg, mg.tp, DEV, max_blocks=3)
    sbc = make_prefill_batch(prompts, [0, 0], bts, mc.cfg, mc.tp, "cpu", max_blocks=3)
    lg = mg.forward(sbg, kvg).float().cpu()
    lc = mc.forward(sbc, kvc).float()
    assert (lg - lc).abs().max() < 0.05 * lc.abs().max() + 0.05
    assert (lg.argmax(-1) == lc.argmax(-1)).float().mean() >= 0.5


def test_engine_graph_equals_eager():
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    chains = [["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"],
              ["[EXEC] bash -> chmod", "[OPEN] chmod -> /tmp/x", "[EXEC] bash -> cat"],
              ["[OPEN] sshd -> /var/log/auth.log", "[EXEC] sshd -> bash"]]
    outs = []
    for graphs in (True, False):
        eng = Engine(EngineConfig(model="small", device=DEV, max_slots=4, max_model_len=256, use_graphs=graphs,
                                  decode_burst=4))
        reqs = [eng.submit(build_prompt(c), fmt=VERDICT_SCHEMA, num_predict=48) for c in chains]
        eng.run_until_idle()
        outs.append([r.out_ids for r in reqs])
        import json

        for r in reqs:
            v = json.loads(r.text)
            assert {"risk_score", "verdict", "reason"} <= set(v)
    assert outs[0] == outs[1]


@pytest.mark.parametrize("m", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("n,k", [(6144, 4096), (4096, 14336), (1024, 512), (48, 2560)])
def test_gemv_matches_matmul(m, n, k):
    from chronos.ops import gemm

    g = torch.Generator(device=DEV).manual_seed(m * n + k)
    x = torch.randn(m, k, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    y = gemm._gemv(x, w)
    ref = (x.float() @ w.float().t())
    _close(y, ref, 2e-2, 2e-2)


@pytest.mark.parametrize("m", [1, 2, 4, 7, 8])
def test_gemv_fused_swiglu(m):
    from chronos import ops
    from chronos.ops import gemm
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(m)
    x = torch.randn(m, 4096, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(2 * 1792, 4096, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    y = gemm._gemv(x, w, True)
    exp = ref.silu_mul((x.float() @ w.float().t()).to(torch.bfloat16))
    _close(y, exp, 2e-2, 3e-2)
    assert ops.gate_up_silu(x, w).shape == (m, 1792)


@pytest.mark.parametrize("m,n,k,stages", [(3, 256, 128, 3), (100, 384, 640, 2), (129, 1024, 4096, 3),
                                          (300, 512, 1024, 4), (1024, 4096, 256, 3)])
@pytest.mark.parametrize("swiglu", [False, True])
def test_mfma_gemm_matches_fp32(m, n, k, stages, swiglu):
    """csrc/kernels/gemm.hip vs an fp32 reference: ragged M (clamped loads, masked stores), multi-stage LDS-DMA ring
    incl. K shorter than the ring, asymmetric data (catches a transposed fragment map), fused SwiGLU epilogue."""
    from chronos.ops import gemm
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(m + n + k)
    x = (torch.randn(m, k, device=DEV, generator=g) + torch.arange(k, device=DEV) / k).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV, generator=g) * 0.05 + torch.linspace(-0.02, 0.03, n, device=DEV)[:, None])
    w = w.to(torch.bfloat16)
    y = gemm.mfma_gemm(x, w, swiglu, stages)
    full = x.float() @ w.float().t()
    exp = ref.silu_mul(full.to(torch.bfloat16)) if swiglu else full
    _close(y, exp, 2e-2, 3e-2)


# ---------------------------------------------------------------------------------------------------------------
# fp8-e4m3 (OCP) KV cache
# ---------------------------------------------------------------------------------------------------------------

def test_fp8_conversion_is_ocp_e4m3fn():
    """The cache bytes written by the kernel must decode with torch.float8_e4m3fn (OCP), not the MI300 fnuz format."""
    from chronos import ops
    from chronos.models.llama import get_config, rope_table
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(5)
    hq, hkv, bs, T = 32, 8, 16, 20
    cs = rope_table(get_config("llama3-8b"), 512, DEV)
    qkv = (torch.randn(T, (hq + 2 * hkv) * 128, device=DEV, generator=g) * 3).to(torch.bfloat16)
    pos = torch.arange(T, device=DEV, dtype=torch.int32)
    bt = torch.arange(4, device=DEV, dtype=torch.int32).view(1, 4)
    ts = torch.zeros(T, dtype=torch.int32, device=DEV)
    k1 = torch.zeros(4, hkv, bs, 128, dtype=torch.uint8, device=DEV)
    v1 = torch.zeros(4, hkv, 128, bs, dtype=torch.uint8, device=DEV)
    k2, v2 = k1.clone(), v1.clone()
    q1 = torch.empty(T, hq, 128, device=DEV, dtype=torch.bfloat16)
    q2 = torch.empty_like(q1)
    ops.rope_kv_write(qkv, pos, ts, bt, cs, q1, k1, v1, hq, hkv, True, 0.5, 2.0)
    ref.rope_kv_write(qkv, pos, ts, bt, cs, q2, k2, v2, hq, hkv, True, 0.5, 2.0)
    assert torch.equal(v1, v2)
    kd1, kd2 = ref.from_fp8_bytes(k1, 0.5), ref.from_fp8_bytes(k2, 0.5)
    # rounding of the rotated value may differ in the last fp8 ulp (f32 vs reference op order)
    assert (kd1 - kd2).abs().max() <= 0.0625 * kd2.abs().max()
    assert (k1 != k2).float().mean() < 0.01


@pytest.mark.parametrize("nqt", [1, 8])
def test_fp8_paged_attention(nqt):
    from chronos import ops
    from chronos.ops import reference as ref

    q_lens, ctx_lens = ([1] * 5, [1, 17, 200, 513, 1000]) if nqt == 1 else ([33, 100], [90, 300])
    q, k, v, bt, qs, ctx = _attn_case(q_lens, ctx_lens, 32, 8, 16, seed=13)
    k8 = ref.to_fp8_bytes(k, 1 / 0.25)
    v8 = ref.to_fp8_bytes(v, 1 / 0.5)
    if nqt == 1:
        tt, nt = None, len(q_lens)
    else:
        tiles = ops.attention_tiles(q_lens, 32, 8, nqt)
        tt, nt = torch.tensor(tiles, dtype=torch.int32, device=DEV).view(-1, 2), len(tiles)
    exp = ref.paged_attention(q, k8, v8, bt, qs, ctx, tt, nt, nqt, 1, None, 0.25, 0.5)
    if nqt == 1:
        out = ops.paged_attention(q, k8, v8, bt, qs, ctx, tt, nt, nqt, 2, None, 0.25, 0.5)
        _close(out, exp, 2e-2, 2e-2)
        return
    # prefill tiles: the default fp8 cache kernel runs Q K^T and P V on the fp8 MFMA (Q, P in e4m3: relative-error
    # bound, tests/test_prefill_fp8_mfma_gpu.py); the bf16-MFMA kernel (knob 0) keeps the tight elementwise bound
    out = ops.paged_attention(q, k8, v8, bt, qs, ctx, tt, nt, nqt, 1, None, 0.25, 0.5)
    assert float((out.float() - exp.float()).norm() / exp.float().norm()) < 0.05
    torch.ops.chronos.set_knob("prefill_fp8_mfma", 0)
    try:
        out = ops.paged_attention(q, k8, v8, bt, qs, ctx, tt, nt, nqt, 1, None, 0.25, 0.5)
    finally:
        torch.ops.chronos.set_knob("prefill_fp8_mfma", 1)
    _close(out, exp, 2e-2, 2e-2)


def test_fp8_decode_one_wave_kernel():
    """fp8 KV through the one-wave-per-(seq, kv head) decode kernel (>= 2048 items, no kv split)."""
    from chronos import ops
    from chronos.ops import reference as ref

    g = torch.Generator().manual_seed(3)
    ctx_lens = torch.randint(1, 300, (256,), generator=g).tolist()
    ctx_lens[:3] = [1, 33, 1100]
    q, k, v, bt, qs, ctx = _attn_case([1] * len(ctx_lens), ctx_lens, 32, 8, 16, seed=21)
    k8, v8 = ref.to_fp8_bytes(k, 1 / 0.25), ref.to_fp8_bytes(v, 1 / 0.5)
    out = ops.paged_attention(q, k8, v8, bt, qs, ctx, None, len(ctx_lens), 1, 1, None, 0.25, 0.5)
    exp = ref.paged_attention(q, k8, v8, bt, qs, ctx, None, len(ctx_lens), 1, 1, None, 0.25, 0.5)
    _close(out, exp, 2e-2, 2e-2)


def test_engine_fp8_kv_end_to_end():
    import json

    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    eng = Engine(EngineConfig(model="small", device=DEV, max_slots=4, max_model_len=256, kv_dtype="fp8",
                              decode_burst=4))
    assert eng.kv.buf.dtype == torch.uint8
    r = eng.submit(build_prompt(["[EXEC] bash -> curl", "[OPEN] curl -> /tmp/x"]), fmt=VERDICT_SCHEMA, num_predict=40)
    eng.run_until_idle()
    assert {"risk_score", "verdict", "reason"} <= set(json.loads(r.text))


@pytest.mark.parametrize("tk,tp", [(5, 1.0), (0, 0.5), (40, 0.9), (1, 1.0)])
def test_topk_topp_sampling_stays_in_nucleus(tk, tp):
    """Sampled tokens must lie in the exact top-k / top-p set of the reference (keys of the bf16 logits)."""
    from chronos import ops
    from chronos.brain.constrain import DONE, GrammarBank
    from chronos.brain.tokenizer import ChronosBPE
    from chronos.ops import reference as ref

    tok = ChronosBPE()
    bank = GrammarBank(tok.token_bytes_list(), tok.stop_ids, 128256, 64, DEV)
    g0 = bank.get(None)
    S = 64
    gen = torch.Generator(device=DEV).manual_seed(tk * 7 + int(tp * 10))
    logits = (torch.randn(S, 128256, device=DEV, generator=gen) * 2).to(torch.bfloat16)
    logits[:, 1000:1010] += 8.0  # a peaked head so top-p cuts somewhere interesting
    i32 = dict(dtype=torch.int32, device=DEV)
    state = torch.full((S,), g0.start, **i32)
    rem = torch.full((S,), 50, **i32)
    temp = torch.full((S,), 1.0, dtype=torch.float32, device=DEV)
    seed = torch.arange(S, **i32)
    ids, pos, ctx, nout = (torch.zeros(S, **i32) for _ in range(4))
    out = torch.zeros(S, 4, **i32)
    topk = torch.full((S,), tk, **i32)
    topp = torch.full((S,), tp, dtype=torch.float32, device=DEV)
    ops.constrained_sample(logits, None, bank.next, bank.dist, DONE, state, rem, temp, seed, ids, pos, ctx, nout,
                           out, topk, topp)
    legal = (bank.next[g0.start].long() >= 0).cpu()
    legal &= bank.dist.cpu()[bank.next[g0.start].long().clamp(min=0).cpu()] <= 49
    for s in range(S):
        lg = logits[s].float().cpu()
        thr = ref.topkp_threshold(lg, legal, tk, tp)
        t = int(out[s, 0])
        assert bool(legal[t]) and int(ref.ord_key(lg[t:t + 1])[0]) >= thr, (s, t)
    if tk == 1:  # top-1 sampling is greedy (up to ties of the bf16 maximum, all of which are kept)
        lgl = torch.where(legal, logits.float().cpu(), -1e30)
        picked = lgl.gather(1, out[:, :1].long().cpu()).squeeze(1)
        assert torch.equal(picked, lgl.max(-1).values)


@pytest.mark.parametrize("spike", ["big", "small"])
def test_decode_one_wave_forced_rescale(spike):
    """The one-wave decode kernel's defer-max branch (LEAN), forced (cdna_hip_programming.md §5.4 rule 26): in 2048+
    items, a late key of several sequences is aligned with the query so the score jumps far past the running max
    (big: the rescale runs) or by less than the 8 (log2) threshold (small: the stale max is kept, p up to 2^8).
    Every variant (LEAN on / off, occupancy hint on / off) against the full fp32 reference."""
    from chronos import ops
    from chronos.ops import reference as ref

    g = torch.Generator().manual_seed(5)
    ctx_lens = torch.randint(100, 400, (260,), generator=g).tolist()
    q, k, v, bt, qs, ctx = _attn_case([1] * len(ctx_lens), ctx_lens, 32, 8, 16, seed=31)
    amp = 4.0 if spike == "big" else 0.1  # score ~ amp * |q|^2 / sqrt(128) * log2(e) ~ amp * 65 (log2)
    for b in range(0, 260, 7):
        t = ctx_lens[b] - 3  # in the last 32-key step of the sequence
        blk = int(bt[b, t // 16])
        for h in range(8):
            k[blk, h, t % 16] = (q[b, 4 * h].float() * amp).to(torch.bfloat16)
    exp = ref.paged_attention(q, k, v, bt, qs, ctx, None, len(ctx_lens), 1, 1)
    C = torch.ops.chronos
    try:
        for lean in (1, 0):
            for occ in (1, 0):
                C.set_knob("decode_lean", lean)
                C.set_knob("decode_occ3", occ)
                out = ops.paged_attention(q, k, v, bt, qs, ctx, None, len(ctx_lens), 1, 1)
                _close(out, exp, 2e-2, 2e-2)
    finally:
        C.set_knob("decode_lean", 1)
        C.set_knob("decode_occ3", 1)
