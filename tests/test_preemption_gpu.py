"""Recompute preemption on the MI355X: one 64k-token chain plus 256 short chains on a KV budget
that cannot hold them together.  Every request completes with a schema-valid verdict; the short chains' growth
preempts the newest sequences, which re-prefill (prompt + generated ids) through the prefix cache and resume their
grammar.  Token identity with an unconstrained run is pinned on the CPU (tests/test_preemption.py): on the GPU the
projection kernels are picked per batch size, so outputs are batch-dependent by design."""
import json

import pytest

pytestmark = pytest.mark.gpu


def test_long_chain_plus_short_chains_under_kv_pressure():
    import torch

    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    long_tokens = 64 * 1024
    bs = 16
    budget = long_tokens // bs + 16 + 900  # the long chain + ~100 short chains' prompts: far below the demand
    eng = Engine(EngineConfig(model="small", device="cuda", max_slots=320, max_model_len=long_tokens + 256,
                              kv_blocks=budget, block_size=bs, max_prefill_tokens=16384, kv_lookahead=32,
                              kv_watermark=0.0, decode_burst=8))
    g = torch.Generator().manual_seed(0)
    body = torch.randint(1000, 100000, (long_tokens - 200,), generator=g).tolist()
    head = eng.tok.chat_ids(build_prompt(["[EXEC] bash -> curl"]))
    long_req = eng.submit(head[:-8] + body + head[-8:], fmt=VERDICT_SCHEMA, num_predict=48)
    chains = synthetic_chains(256, seed=17, native=False)
    short = [eng.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=48 + (i % 3) * 8)
             for i, c in enumerate(chains)]
    eng.run_until_idle()
    torch.cuda.synchronize()
    assert long_req.done_reason in ("stop", "length"), long_req.error
    json.loads(long_req.text)
    for r in short:
        assert r.done_reason in ("stop", "length"), (r.done_reason, r.error)
        assert {"risk_score", "verdict", "reason"} <= set(json.loads(r.text))
        assert len(r.out_ids) <= 64
    assert eng.stats["preemptions"] > 0, dict(eng.stats)
    assert any(r.preemptions for r in short)
    # every block is back in the pool (idle cached prefix blocks count as free)
    assert eng.blocks.free == budget - 1
