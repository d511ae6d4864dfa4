"""Model-level cost of the default fp8-MFMA flash prefill.

``prefill_fp8_mfma=1`` (the default with an fp8 KV cache) quantises Q and P to e4m3 on top of the e4m3 cache.  The
kernel tests (tests/test_prefill_fp8_mfma_gpu.py) bound its per-call attention error; here the whole 32-layer
Llama-3.1-8B (random init, real geometry) prefills one 32k-token prompt in the engine's 16k-token chunks three ways:

* bf16 KV cache (the truth),
* fp8 KV + the bf16-MFMA prefill kernel (``prefill_fp8_mfma=0``: the e4m3 cache alone),
* fp8 KV + the fp8-MFMA prefill kernel (``prefill_fp8_mfma=1``, the default),

and compares the last-token logits (relative L2, max abs) and a 12-token greedy continuation.  The fp8-MFMA drift must
stay within 1.5x the cache-only drift.  Numbers are written to gpurun_out/prefill_fp8_model_drift.json.
"""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
T, CHUNK, BS, NGEN = 32768, 16384, 16, 12


def _prefill_and_generate(model, kv, ids, nqt):
    from chronos.models.llama import make_prefill_batch
    from chronos.parallel.tp import TPContext

    tp = TPContext.single()
    nb = kv.num_blocks
    blocks = list(range(1, nb))
    logits = None
    for s in range(0, len(ids), CHUNK):
        sb = make_prefill_batch([ids[s:s + CHUNK]], [s], [blocks], model.cfg, tp, DEV, max_blocks=nb, nqt=nqt)
        logits = model.forward(sb, kv, torch.float32)
    first = logits[0].clone()
    out, seq = [], list(ids)
    tok = int(first.argmax())
    for _ in range(NGEN):  # greedy continuation, one token per forward through the same paged cache
        out.append(tok)
        sb = make_prefill_batch([[tok]], [len(seq)], [blocks], model.cfg, tp, DEV, max_blocks=nb, nqt=nqt)
        seq.append(tok)
        tok = int(model.forward(sb, kv, torch.float32)[0].argmax())
    return first, out


def test_fp8_mfma_prefill_logit_drift_at_32k():
    from chronos import ops
    from chronos.models.llama import KVCache, build_model
    from chronos.parallel.tp import TPContext

    ops.load()
    model = build_model("llama3.1-8b", DEV, seed=0, max_position=T + 64)
    g = torch.Generator().manual_seed(7)
    ids = torch.randint(1000, 120000, (T,), generator=g).tolist()
    nb = (T + NGEN) // BS + 3
    res = {}
    try:
        for name, dt, knob in (("bf16", "bf16", 1), ("fp8_cache", "fp8", 0), ("fp8_mfma", "fp8", 1)):
            torch.ops.chronos.set_knob("prefill_fp8_mfma", knob)
            kv = KVCache(model.cfg, TPContext.single(), nb, BS, DEV, dt, 1.0, 1.0)
            res[name] = _prefill_and_generate(model, kv, ids, 8)
            del kv
            torch.cuda.empty_cache()
    finally:
        torch.ops.chronos.set_knob("prefill_fp8_mfma", 1)
    ref = res["bf16"][0]

    def drift(x):
        d = x - ref
        return float(d.norm() / ref.norm()), float(d.abs().max())

    c_l2, c_max = drift(res["fp8_cache"][0])
    m_l2, m_max = drift(res["fp8_mfma"][0])
    top = lambda x: set(x.topk(10).indices.tolist())  # noqa: E731
    rep = {"tokens": T, "chunk": CHUNK, "fp8_cache_rel_l2": c_l2, "fp8_cache_max_abs": c_max,
           "fp8_mfma_rel_l2": m_l2, "fp8_mfma_max_abs": m_max, "ratio_rel_l2": m_l2 / max(c_l2, 1e-12),
           "top10_overlap_cache": len(top(res["fp8_cache"][0]) & top(ref)),
           "top10_overlap_mfma": len(top(res["fp8_mfma"][0]) & top(ref)),
           "greedy_bf16": res["bf16"][1], "greedy_fp8_cache": res["fp8_cache"][1], "greedy_fp8_mfma": res["fp8_mfma"][1]}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/prefill_fp8_model_drift.json", "w") as fh:
        json.dump(rep, fh, indent=1)
    print(json.dumps(rep))
    assert torch.isfinite(res["fp8_mfma"][0]).all()
    assert m_l2 <= 1.5 * c_l2 + 1e-3, rep
    assert m_max <= 1.5 * c_max + 1e-2, rep
