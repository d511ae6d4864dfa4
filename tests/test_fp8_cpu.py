"""W8A8 fp8 plumbing on the CPU reference path (the GPU kernels are checked in test_fp8_gpu.py): weight quantisation
round trip, the fp8 model tracking the bf16 model built from the same random weights, and the engine serving
schema-valid verdicts with fp8 projections."""
import json

import torch


def test_quantize_weight_roundtrip():
    from chronos.ops import reference as ref

    g = torch.Generator().manual_seed(0)
    w = (torch.randn(64, 512, generator=g) * torch.linspace(0.01, 1.0, 64)[:, None]).to(torch.bfloat16)
    q, s = ref.quantize_weight(w)
    assert q.dtype == torch.uint8 and s.shape == (64,)
    deq = q.view(torch.float8_e4m3fn).float() * s[:, None]
    rel = (deq - w.float()).abs() / w.float().abs().amax(-1, keepdim=True)
    assert float(rel.max()) <= 2 ** -4  # e4m3: half a step of 3 mantissa bits, relative to the row max
    # the row max is represented exactly (448 * s)
    assert torch.allclose(deq.abs().amax(-1), w.float().abs().amax(-1), rtol=1e-6)


def test_quant_rows_modes():
    from chronos.ops import reference as ref

    g = torch.Generator().manual_seed(1)
    x = torch.randn(5, 256, generator=g).to(torch.bfloat16)
    w = (torch.rand(256, generator=g) + 0.5).to(torch.bfloat16)
    r = torch.randn(5, 256, generator=g).to(torch.bfloat16)
    r0 = r.clone()
    q, s = ref.quant_rows(x, r, w, 1e-5, 2)
    assert torch.equal(r, (x.float() + r0.float()).to(torch.bfloat16))
    y = ref.rmsnorm(r, w, 1e-5).float()
    deq = q.view(torch.float8_e4m3fn).float() * s[:, None]
    assert float(((deq - y).abs() / y.abs().amax(-1, keepdim=True)).max()) <= 2 ** -4


def test_fp8_model_and_engine_cpu():
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.models.llama import KVCache, QTensor, build_model, make_prefill_batch
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    mb = build_model("tiny", "cpu", seed=3)
    mq = build_model("tiny", "cpu", seed=3, weight_dtype="fp8")
    assert isinstance(mq.w.layers[0].w_gu, QTensor) and mq.w.fp8 and not mb.w.fp8
    outs = []
    for m in (mb, mq):
        kv = KVCache(m.cfg, m.tp, 64, 16, "cpu")
        sb = make_prefill_batch([list(range(100, 160)), list(range(7, 90))], [0, 0],
                                [list(range(8)), list(range(8, 16))], m.cfg, m.tp, "cpu", max_blocks=16, nqt=8)
        outs.append(m.forward(sb, kv).float())
    cos = torch.nn.functional.cosine_similarity(outs[0], outs[1], dim=-1)
    assert float(cos.min()) > 0.98
    eng = Engine(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False,
                              weight_dtype="fp8"))
    reqs = [eng.submit(build_prompt(["[EXEC] bash -> curl", f"[OPEN] curl -> /tmp/{i}"]), fmt=VERDICT_SCHEMA,
                       num_predict=40) for i in range(3)]
    eng.run_until_idle()
    for r in reqs:
        assert {"risk_score", "verdict", "reason"} <= set(json.loads(r.text))
