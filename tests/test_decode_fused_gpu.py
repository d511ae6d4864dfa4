"""Single-stream decode: attention + O projection + residual epilogue in one persistent launch
(csrc/kernels/decode_fused.hip) against the two separate kernels it replaces (paged_attention, then gemv_resid).

The fused launch uses the same arithmetic in the same order, so it must be bit-identical, across contexts that end
inside / on a 32-token step and a cache block, over repeated launches (the kernel resets its own hand-off counters),
inside a captured graph, and with a small persistent grid (every workgroup loops over many row groups)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from chronos import ops

    ops.load()
    import chronos.native as n

    assert "_C" in n._loaded


def _case(ctx, hq=32, hkv=8, d=4096, bs=16, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed + ctx)
    nb = (ctx + bs - 1) // bs + 3
    kc = (torch.randn(nb, hkv, bs, 128, device=DEV, generator=g)).to(torch.bfloat16)
    vc = (torch.randn(nb, hkv, 128, bs, device=DEV, generator=g)).to(torch.bfloat16)
    bt = torch.randperm(nb, device=DEV, generator=g).to(torch.int32).view(1, nb)
    q = torch.randn(1, hq, 128, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(d, hq * 128, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    r = torch.randn(1, d, device=DEV, generator=g).to(torch.bfloat16)
    ctx_len = torch.tensor([ctx], dtype=torch.int32, device=DEV)
    return q, kc, vc, bt, ctx_len, w, r


def _unfused(q, kc, vc, bt, ctx_len, w, r, scale):
    from chronos import ops

    q_start = torch.tensor([0, 1], dtype=torch.int32, device=DEV)
    attn = ops.paged_attention(q, kc, vc, bt, q_start, ctx_len, None, 1, 1, 1, scale)
    return ops.gemv_resid(attn.view(1, -1), w, r)


@pytest.mark.parametrize("ctx", [1, 31, 32, 33, 150, 511])
@pytest.mark.parametrize("grid_cap", [0, 37])
def test_attn_o_bit_identical(ctx, grid_cap):
    from chronos import ops

    q, kc, vc, bt, ctx_len, w, r = _case(ctx)
    scale = 128 ** -0.5
    ref = _unfused(q, kc, vc, bt, ctx_len, w, r, scale)
    for _ in range(3):  # the hand-off counters must be back at zero after every launch
        out = ops.attn_o(q, kc, vc, bt, ctx_len, w, r, scale, grid_cap)
        assert out is not None
        torch.cuda.synchronize()
        assert torch.equal(out.s, ref.s)
        assert torch.equal(out.part, ref.part)


def test_attn_o_graph_replay_and_gqa_shapes():
    from chronos import ops

    for hq, hkv, d in ((32, 8, 4096), (8, 1, 2048), (64, 8, 8192)):
        q, kc, vc, bt, ctx_len, w, r = _case(77, hq, hkv, d, seed=hq)
        scale = 128 ** -0.5
        ref = _unfused(q, kc, vc, bt, ctx_len, w, r, scale)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ops.attn_o(q, kc, vc, bt, ctx_len, w, r, scale)  # warm (scratch allocation outside the capture)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = ops.attn_o(q, kc, vc, bt, ctx_len, w, r, scale)
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(out.s, ref.s) and torch.equal(out.part, ref.part)


def test_attn_o_declines_unsupported():
    from chronos import ops

    q, kc, vc, bt, ctx_len, w, r = _case(40)
    assert ops.attn_o(torch.cat([q, q]), kc, vc, bt, ctx_len, w, torch.cat([r, r]), 0.1) is None  # two rows
    k8 = torch.zeros(kc.shape, dtype=torch.uint8, device=DEV)
    v8 = torch.zeros(vc.shape, dtype=torch.uint8, device=DEV)
    assert ops.attn_o(q, k8, v8, bt, ctx_len, w, r, 0.1) is None  # fp8 KV


def test_single_stream_engine_same_tokens_fused_or_not(monkeypatch):
    """A verdict decoded through the fused launch equals the separate kernels' verdict token for token."""
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.models import llama
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    outs = {}
    for fused in (False, True):
        monkeypatch.setattr(llama, "_FUSE_ATTN_O", fused)  # explicit: the model default is off
        eng = Engine(EngineConfig(model="small", device="cuda", max_slots=2, max_model_len=384, decode_burst=4,
                                  seed=0, jump_forward=False))
        req = eng.submit(build_prompt(["[OPEN] attack_chain.sh -> /tmp/malware.bin",
                                       "[EXEC] attack_chain.sh -> curl"]), fmt=VERDICT_SCHEMA, num_predict=40)
        eng.run_until_idle()
        outs[fused] = list(req.out_ids)
    assert outs[True] == outs[False]
