"""Whole-model numerics at Llama-3-8B layer shapes: a 2-layer model with d = 4096, 32 query /
8 KV heads, FFN 14336, random init, GPU forward (every hand-written kernel and fusion on its real routing) against the
CPU reference forward (chronos.ops.reference, fp32 compute) on the same weights and the same paged KV cache:

* prefill: three prompts, one continuing from a cached prefix (flash prefill kernel, batched GEMM with the residual
  and folded-norm epilogues, prefill LazyNorm into the LM head);
* decode at buckets 1 and 2 (GEMV ResidOut / LazyNorm / QKV+RoPE+KV-write), 128 (batched GEMM + rope_kv_write +
  paged decode attention) and 1024 (batched GEMM + RoPE-fused one-wave decode attention), eager, and the 128 bucket
  again replayed from a captured hipGraph.

Tolerances: max |logit difference| <= 2 % of max |logit| and argmax agreement >= 95 %.  The vocabulary is cut to
32768 rows so the CPU reference stays fast; the LM head is scaled up (std 0.2) so that random-weight logits have
resolvable maxima (near-ties between bf16 roundings would make argmax agreement a coin flip at any precision).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def models():
    from chronos import ops
    from chronos.models.llama import LlamaConfig, build_model

    ops.load()
    cfg = LlamaConfig(name="l3-8b-2l", vocab_size=32768, num_layers=2, max_position=4096)
    mg = build_model(cfg, DEV, seed=3)
    g = torch.Generator(device=DEV).manual_seed(9)
    mg.w.lm_head.copy_((torch.randn(mg.w.lm_head.shape, device=DEV, generator=g) * 0.2).to(torch.bfloat16))
    mc = build_model(cfg, "cpu", seed=3)
    for lg, lc in zip(mg.w.layers, mc.w.layers):
        for n in ("attn_norm", "wqkv", "wo", "mlp_norm", "w_gu", "w_down"):
            getattr(lc, n).copy_(getattr(lg, n).cpu())
    mc.w.embed.copy_(mg.w.embed.cpu())
    mc.w.lm_head.copy_(mg.w.lm_head.cpu())
    mc.w.norm.copy_(mg.w.norm.cpu())
    assert mg.w.norms_folded
    return mg, mc


def _kv(mg, mc, nblocks, seed):
    from chronos.models.llama import KVCache

    kvg = KVCache(mg.cfg, mg.tp, nblocks, 16, DEV)
    kvc = KVCache(mc.cfg, mc.tp, nblocks, 16, "cpu")
    g = torch.Generator(device=DEV).manual_seed(seed)
    kvg.buf.copy_((torch.randn(kvg.buf.shape, device=DEV, generator=g) * 0.5).to(torch.bfloat16))
    kvc.buf.copy_(kvg.buf.cpu())
    return kvg, kvc


def _compare(lg, lc, what):
    lg, lc = lg.float().cpu(), lc.float()
    err = (lg - lc).abs().max().item()
    scale = lc.abs().max().item()
    agree = (lg.argmax(-1) == lc.argmax(-1)).float().mean().item()
    assert err <= 0.02 * scale, f"{what}: max |dlogit| {err:.4g} > 2% of {scale:.4g}"
    assert agree >= 0.95, f"{what}: argmax agreement {agree:.3f}"


def test_prefill_8b_shapes(models):
    from chronos.models.llama import make_prefill_batch

    mg, mc = models
    kvg, kvc = _kv(mg, mc, 64, 1)
    g = torch.Generator().manual_seed(2)
    lens, starts = [37, 190, 77], [0, 0, 48]  # the third continues after a 48-token cached prefix
    prompts = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in lens]
    bts, nxt = [], 1
    for n, s0 in zip(lens, starts):
        nb = (n + s0 + 15) // 16
        bts.append(list(range(nxt, nxt + nb)))
        nxt += nb
    sbg = make_prefill_batch(prompts, starts, bts, mg.cfg, mg.tp, DEV, max_blocks=16)
    sbc = make_prefill_batch(prompts, starts, bts, mc.cfg, mc.tp, "cpu", max_blocks=16)
    _compare(mg.forward(sbg, kvg), mc.forward(sbc, kvc), "prefill")


def _decode_batch(n, cfg, tp, dev, ctx, bt):
    from chronos.models.llama import StepBatch, to_device
    from chronos import ops

    g = torch.Generator().manual_seed(n)
    i32 = lambda x: torch.tensor(x, dtype=torch.int32)  # noqa: E731
    ids = torch.randint(0, 32000, (n,), generator=g).to(torch.int32)
    ar = torch.arange(n + 1, dtype=torch.int32)
    nsplit = ops.pick_nsplit(n * cfg.num_kv_heads, 512)
    sb = StepBatch(ids, i32([c - 1 for c in ctx]), ar[:n].clone(), bt, ar.clone(), i32(ctx),
                   torch.arange(n, dtype=torch.int64), None, n, 1, nsplit)
    return to_device(sb, dev)


@pytest.mark.parametrize("n", [1, 2, 128, 1024])
def test_decode_8b_shapes(models, n):
    mg, mc = models
    g = torch.Generator().manual_seed(100 + n)
    ctx = torch.randint(20, 200, (n,), generator=g).tolist()
    mb = 13  # 208 tokens per sequence
    bt = torch.arange(1, 1 + n * mb, dtype=torch.int32).view(n, mb)
    kvg, kvc = _kv(mg, mc, 1 + n * mb, 7 + n)
    lg = mg.forward(_decode_batch(n, mg.cfg, mg.tp, DEV, ctx, bt), kvg)
    lc = mc.forward(_decode_batch(n, mc.cfg, mc.tp, "cpu", ctx, bt), kvc)
    _compare(lg, lc, f"decode n={n}")
    # the new token's K/V landed in the same place on both sides
    li = 0
    k_g, k_c = kvg.k[li].float().cpu(), kvc.k[li].float()
    assert (k_g - k_c).abs().max().item() <= 0.05 * k_c.abs().max().item()


def test_decode_graph_replay_8b_shapes(models):
    mg, mc = models
    n = 128
    g = torch.Generator().manual_seed(5)
    ctx = torch.randint(20, 200, (n,), generator=g).tolist()
    mb = 13
    bt = torch.arange(1, 1 + n * mb, dtype=torch.int32).view(n, mb)
    kvg, kvc = _kv(mg, mc, 1 + n * mb, 55)
    sb = _decode_batch(n, mg.cfg, mg.tp, DEV, ctx, bt)
    base = kvg.buf.clone()
    eager = mg.forward(sb, kvg).clone()
    kvg.buf.copy_(base)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = mg.forward(sb, kvg)
    kvg.buf.copy_(base)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager), "graph replay differs from eager"
    lc = mc.forward(_decode_batch(n, mc.cfg, mc.tp, "cpu", ctx, bt), kvc)
    _compare(out, lc, "decode graph n=128")
