"""Cascade (shared-prefix) decode attention (csrc/kernels/attention.hip casc_prefix_kernel + the merge in
paged_decode_kernel) against the fp32 reference attention.

Rows that hold the cascade prefix (their first P block-table entries are the prefix blocks, context longer than the
prefix) attend it in the MFMA pass and merge it into their own walk; every other row must be untouched.  Mixed in one
batch: members, rows sharing only the first prefix block, rows with no shared block, rows whose context ends exactly
one token past the prefix, odd and even P, ragged batch sizes; plus the engine path (refcounts changing as verdicts
finish mid-wave) against an engine with the cascade off.
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


def _setup(n, P, hq=32, hkv=8, bs=16, seed=0, nblk_max=24):
    from chronos.models.llama import LlamaConfig, rope_table

    g = torch.Generator(device=DEV).manual_seed(seed)
    nb = max(4096, 24 * n)
    kc = (torch.randn(nb, hkv, bs, 128, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    vc = (torch.randn(nb, hkv, 128, bs, device=DEV, generator=g)).to(torch.bfloat16)
    prefix = list(range(1, P + 1))
    nxt = P + 1
    bt = torch.zeros(n, nblk_max, dtype=torch.int32)
    ctx = []
    kinds = []
    gh = torch.Generator().manual_seed(seed)
    for i in range(n):
        kind = i % 5  # 0-2 members, 3 first block only, 4 private
        if i % 17 == 9:
            kind = 5  # context ends right after the prefix: one token past it -> member with a 1-token suffix
        L = 16 * P
        if kind in (0, 1, 2):
            c = L + 1 + int(torch.randint(0, 200, (1,), generator=gh))
        elif kind == 5:
            c = L + 1
        elif kind == 3:  # past the shared first block (a decode row never writes into a shared block)
            c = 17 + int(torch.randint(0, 240, (1,), generator=gh))
        else:
            c = 1 + int(torch.randint(0, 260, (1,), generator=gh))
        nb_i = (c + bs - 1) // bs
        if kind in (0, 1, 2, 5):
            blocks = prefix[:min(P, nb_i)] + list(range(nxt, nxt + max(0, nb_i - P)))
            nxt += max(0, nb_i - P)
        elif kind == 3:
            blocks = prefix[:1] + list(range(nxt, nxt + nb_i - 1))
            nxt += nb_i - 1
        else:
            blocks = list(range(nxt, nxt + nb_i))
            nxt += nb_i
        assert nxt < nb
        bt[i, :len(blocks)] = torch.tensor(blocks, dtype=torch.int32)
        ctx.append(c)
        kinds.append(kind)
    cfg = LlamaConfig(name="t", hidden_size=hq * 128, num_heads=hq, num_kv_heads=hkv)
    cos_sin = rope_table(cfg, 4096, DEV)
    qkv = (torch.randn(n, (hq + 2 * hkv) * 128, device=DEV, generator=g)).to(torch.bfloat16)
    ctx_t = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    pos = ctx_t - 1
    return kc, vc, bt.to(DEV), ctx_t, pos, cos_sin, qkv, prefix, kinds


def _reference(qkv, pos, cos_sin, kc, vc, bt, ctx, hq, hkv, scale):
    from chronos.ops import reference as ref

    n = qkv.shape[0]
    k2, v2 = kc.clone(), vc.clone()
    q = torch.empty(n, hq, 128, dtype=torch.bfloat16, device=DEV)
    ref.rope_kv_write(qkv, pos, torch.arange(n, device=DEV, dtype=torch.int32), bt, cos_sin, q, k2, v2, hq, hkv)
    out = ref.paged_attention(q, k2, v2, bt, None, ctx, None, n, 1, 1, scale)
    return out, k2, v2


@pytest.mark.parametrize("P", [3, 2, 5])
@pytest.mark.parametrize("n", [260, 301])
def test_cascade_matches_reference(P, n):
    from chronos import ops

    hq, hkv = 32, 8
    kc, vc, bt, ctx, pos, cos_sin, qkv, prefix, kinds = _setup(n, P, hq, hkv, seed=P * 100 + n)
    scale = 1.0 / 128 ** 0.5
    want, k_ref, v_ref = _reference(qkv, pos, cos_sin, kc, vc, bt, ctx, hq, hkv, scale)
    casc = torch.tensor([P] + prefix + [0] * (8 - P), dtype=torch.int32, device=DEV)
    co = torch.full((n, hq, 128), float("nan"), dtype=torch.bfloat16, device=DEV)
    cl = torch.full((n, hq), float("nan"), dtype=torch.float32, device=DEV)
    outs = {}
    for name, c in (("plain", None), ("casc", (casc, co, cl))):
        k2, v2 = kc.clone(), vc.clone()
        o = ops.decode_attention_rope(qkv, pos, cos_sin, k2, v2, bt, ctx, n, hq, scale, c)
        assert o is not None
        torch.cuda.synchronize()
        outs[name] = o.float()
        # the fused K/V write is unchanged by the cascade
        assert torch.equal(k2, k_ref) or (k2.float() - k_ref.float()).abs().max() < 1e-2
    err_plain = (outs["plain"] - want.float()).abs().max().item()
    err_casc = (outs["casc"] - want.float()).abs().max().item()
    scale_o = want.float().abs().max().item()
    assert err_casc <= max(2e-2 * scale_o, 1.5 * err_plain), (err_casc, err_plain, scale_o)
    members = [i for i, k in enumerate(kinds) if k in (0, 1, 2, 5)]
    others = [i for i, k in enumerate(kinds) if k not in (0, 1, 2, 5)]
    # the producer wrote exactly the member rows (the rest of the scratch is untouched NaN)
    assert not torch.isnan(cl[members]).any() and torch.isnan(cl[others]).all()
    # non-members are computed exactly as without the cascade
    assert torch.equal(outs["casc"][others], outs["plain"][others])


def test_cascade_off_is_bit_identical():
    from chronos import ops

    n, hq, hkv, P = 280, 32, 8, 3
    kc, vc, bt, ctx, pos, cos_sin, qkv, prefix, _ = _setup(n, P, hq, hkv, seed=7)
    casc = torch.zeros(9, dtype=torch.int32, device=DEV)  # P = 0
    co = torch.empty(n, hq, 128, dtype=torch.bfloat16, device=DEV)
    cl = torch.empty(n, hq, dtype=torch.float32, device=DEV)
    a = ops.decode_attention_rope(qkv, pos, cos_sin, kc.clone(), vc.clone(), bt, ctx, n, hq, 0.088, None)
    b = ops.decode_attention_rope(qkv, pos, cos_sin, kc.clone(), vc.clone(), bt, ctx, n, hq, 0.088, (casc, co, cl))
    assert torch.equal(a, b)


def test_engine_cascade_wave_matches_cascade_off():
    """A wave of chains sharing the template prefix: with the cascade on (refcounts change as verdicts finish and
    rows compact) every verdict is valid JSON and the greedy tokens agree with the cascade off except where the
    bf16 rounding of the merged attention flips a near-tie; the cascade must have been active."""
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    # tiny70: the 70B head geometry (8 KV heads, GQA 8) in a small model, so 320 decode rows are >= 2048 (row, kv
    # head) items: the fused one-wave decode kernel (and with it the cascade) serves the batch
    chains = synthetic_chains(300, seed=13, native=False)
    res = {}
    for on in (False, True):
        eng = Engine(EngineConfig(model="tiny70", device=DEV, max_slots=320, max_model_len=512, cascade=on,
                                  cascade_min_rows=16, decode_burst=4))
        reqs = [eng.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=32 + (i % 5) * 4)
                for i, c in enumerate(chains)]
        eng.run_until_idle()
        torch.cuda.synchronize()
        for r in reqs:
            assert r.done_reason in ("stop", "length"), r.error
            json.loads(r.text)
        res[on] = ([r.out_ids for r in reqs], dict(eng.stats), eng.stats.get("cascade_max_blocks", 0))
    assert res[True][1].get("cascade_updates", 0) >= 1 and res[True][2] >= 2  # a prefix of >= 2 blocks was used
    same = sum(a == b for a, b in zip(res[False][0], res[True][0]))
    assert same >= 0.8 * len(chains), same
