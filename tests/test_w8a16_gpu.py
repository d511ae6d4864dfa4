"""W8A16 decode GEMV (csrc/kernels/gemv.hip WQ: fp8-e4m3 weights with per-row scales, bf16 activations) against fp32
references of the same ops: plain and SwiGLU, the residual producer (kResid), the folded-norm consumer (NORMP) and
the QKV + RoPE + paged-KV epilogue (bf16 and fp8 caches), at the 8B decode shapes; and the fp8-weight model's decode
step on the W8A16 path against the W8A8 path and the bf16 model."""
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


def _wx(m, n, k, seed):
    from chronos.ops import reference as ref

    g = torch.Generator(device=DEV).manual_seed(seed)
    x = (torch.randn(m, k, device=DEV, generator=g) + 0.1).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    wq, ws = ref.quantize_weight(w)
    return x, wq.contiguous(), ws.contiguous(), g


def _close(y, want):
    err = (y.float() - want.float()).abs().max().item()
    assert err <= 1e-2 * want.float().abs().max().item() + 1e-3, (err, want.float().abs().max().item())


@pytest.mark.parametrize("m", [1, 2, 3, 4])
@pytest.mark.parametrize("n,k,swiglu", [(6144, 4096, False), (4096, 14336, False), (28672, 4096, True),
                                        (4096, 4096, False), (512, 1024, True)])
def test_gemv_w8a16(m, n, k, swiglu):
    x, wq, ws, _ = _wx(m, n, k, m * n + k)
    y = torch.ops.chronos.gemv(x, wq, swiglu, ws)
    full = x.float() @ _deq(wq, ws).t()
    if swiglu:
        gt, up = full[:, :n // 2].bfloat16().float(), full[:, n // 2:].bfloat16().float()
        want = (gt / (1 + torch.exp(-gt))).bfloat16().float() * up
    else:
        want = full
    assert y.shape == want.shape
    _close(y, want)


@pytest.mark.parametrize("m", [1, 2])
@pytest.mark.parametrize("n,k", [(4096, 4096), (4096, 14336)])
def test_gemv_resid_w8a16(m, n, k):
    x, wq, ws, g = _wx(m, n, k, 7 * n + k + m)
    r = torch.randn(m, n, device=DEV, generator=g).to(torch.bfloat16)
    s = torch.empty_like(r)
    part = torch.ops.chronos.gemv_resid(x, wq, r, s, ws)
    want = ((x.float() @ _deq(wq, ws).t()).bfloat16().float() + r.float())
    _close(s, want)
    torch.testing.assert_close(part.sum(1), (s.float() ** 2).sum(1), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("m", [1, 2])
@pytest.mark.parametrize("n,swiglu", [(6144, False), (28672, True)])
def test_gemv_normp_w8a16(m, n, swiglu):
    k = 4096
    x, wq, ws, g = _wx(m, n, k, 11 * n + m)
    # producer: a bf16 residual GEMV writes s and its partial sums of squares
    wo = (torch.randn(k, k, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    r = torch.randn(m, k, device=DEV, generator=g).to(torch.bfloat16)
    s = torch.empty_like(r)
    part = torch.ops.chronos.gemv_resid(x, wo, r, s)
    y = torch.ops.chronos.gemv_normp(s, part, 1e-5, wq, swiglu, ws)
    sf = s.float()
    xn = sf * torch.rsqrt((sf * sf).mean(-1, keepdim=True) + 1e-5)
    full = xn @ _deq(wq, ws).t()
    if swiglu:
        gt, up = full[:, :n // 2].bfloat16().float(), full[:, n // 2:].bfloat16().float()
        want = (gt / (1 + torch.exp(-gt))).bfloat16().float() * up
    else:
        want = full
    _close(y, want)


@pytest.mark.parametrize("m", [1, 2])
@pytest.mark.parametrize("kv_fp8", [False, True])
def test_qkv_rope_w8a16_matches_unfused(m, kv_fp8):
    from chronos import ops
    from chronos.models.llama import LlamaConfig, QTensor, rope_table

    hq, hkv, k = 32, 8, 4096
    n = (hq + 2 * hkv) * 128
    x, wq, ws, g = _wx(m, n, k, 3 + m + 10 * kv_fp8)
    nb, bs = 64, 16
    dt = torch.uint8 if kv_fp8 else torch.bfloat16
    kc = torch.zeros(nb, hkv, bs, 128, device=DEV, dtype=dt)
    vc = torch.zeros(nb, hkv, 128, bs, device=DEV, dtype=dt)
    bt = torch.arange(1, 1 + 4 * m, device=DEV, dtype=torch.int32).view(m, 4)
    pos = torch.tensor([37, 50][:m], device=DEV, dtype=torch.int32)
    tok_seq = torch.arange(m, device=DEV, dtype=torch.int32)
    cs = rope_table(LlamaConfig(name="t"), 4096, DEV)
    ksc, vsc = (0.5, 0.25) if kv_fp8 else (1.0, 1.0)
    outs = []
    for fused in (True, False):
        k2, v2 = kc.clone(), vc.clone()
        q = torch.zeros(m, hq, 128, device=DEV, dtype=torch.bfloat16)
        if fused:
            assert ops.qkv_rope(x, QTensor(wq, ws), pos, tok_seq, bt, cs, q, k2, v2, hq, hkv, ksc, vsc)
        else:
            qkv = torch.ops.chronos.gemv(x, wq, False, ws)
            ops.rope_kv_write(qkv, pos, tok_seq, bt, cs, q, k2, v2, hq, hkv, True, ksc, vsc)
        outs.append((q, k2, v2))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    # and the projection itself against fp32 (the q rows before RoPE are checked through the unfused path)
    _close(torch.ops.chronos.gemv(x, wq, False, ws), x.float() @ _deq(wq, ws).t())


def test_fp8_model_decode_w8a16_vs_w8a8_and_bf16():
    from chronos.models import llama
    from chronos.models.llama import KVCache, StepBatch, build_model, make_prefill_batch

    mb = build_model("small", DEV, seed=5)
    mq = build_model("small", DEV, seed=5, weight_dtype="fp8")
    prompt = list(range(100, 161))
    res = {}
    for name, m, w16 in (("bf16", mb, True), ("w8a16", mq, True), ("w8a8", mq, False)):
        llama._W8A16_DECODE = w16
        kv = KVCache(m.cfg, m.tp, 16, 16, DEV)
        bt = list(range(1, 6))
        sb = make_prefill_batch([prompt], [0], [bt], m.cfg, m.tp, DEV, max_blocks=8, nqt=8)
        m.forward(sb, kv)
        it = lambda v: torch.tensor(v, dtype=torch.int32, device=DEV)  # noqa: E731
        bt_t = torch.zeros(1, 8, dtype=torch.int32, device=DEV)
        bt_t[0, :5] = it(bt)
        dec = StepBatch(it([777]), it([61]), it([0]), bt_t, it([0, 1]), it([62]),
                        torch.zeros(1, dtype=torch.int64, device=DEV), None, 1)
        res[name] = m.forward(dec, kv).float()
        # a jump-forward-sized prefill chunk (T = 3 tokens after the cached prompt): the unfused W8A16 GEMVs
        jf = make_prefill_batch([[5, 6, 7]], [62], [bt], m.cfg, m.tp, DEV, max_blocks=8, nqt=2)
        res[name + "_jf"] = m.forward(jf, kv).float()
    llama._W8A16_DECODE = True
    cos = lambda a, b: torch.nn.functional.cosine_similarity(a, b, dim=-1).min().item()  # noqa: E731
    assert cos(res["w8a16"], res["w8a8"]) > 0.995
    assert cos(res["w8a16"], res["bf16"]) > 0.98
    assert cos(res["w8a16_jf"], res["w8a8_jf"]) > 0.995
    assert cos(res["w8a16_jf"], res["bf16_jf"]) > 0.98
