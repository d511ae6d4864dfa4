"""Mixed prefill + decode steps on the MI355X (Engine._mixed_step; CPU semantics: tests/test_mixed_batching.py).

The hybrid forward — prefill rows through the flash prefill kernel and the batched GEMMs, decode rows through the paged
decode attention in the same launch sequence — must serve arrivals while graph-captured decode bursts run between
them, finish every request with a valid verdict, leave the KV pool whole, and decode what plain scheduling decodes
(greedy; different kernels per row kind make bf16 rounding differ, so the comparison is on shared prefixes)."""
import json

import pytest

pytestmark = pytest.mark.gpu


def _chains(n, seed=4):
    from chronos.sensor.prompt import build_prompt
    from chronos.sensor.replay import synthetic_chains

    return [build_prompt(c.history) for c in synthetic_chains(n, seed=seed, native=False)]


@pytest.mark.parametrize("model", ["tiny", "small"])
def test_mixed_steps_on_gpu(model):
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA

    prompts = _chains(24)
    outs = {}
    for mixed in (False, True):
        eng = Engine(EngineConfig(model=model, device="cuda", max_slots=16, max_model_len=384, use_graphs=True,
                                  decode_burst=4, max_prefill_tokens=512, jump_forward=False, seed=0,
                                  mixed_batching=mixed, mixed_prefill_tokens=128, mixed_ratio=2))
        reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=40) for p in prompts[:6]]
        for _ in range(3):
            eng.step()
        nxt = 6
        while eng.has_work() or nxt < len(prompts):
            if nxt < len(prompts):  # two arrivals per step while anything decodes
                reqs += [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=40) for p in prompts[nxt:nxt + 2]]
                nxt += 2
            eng.step()
        assert (eng.stats["mixed_steps"] > 0) == mixed, dict(eng.stats)
        for r in reqs:
            assert r.error is None, r.error
            if r.done_reason == "stop":
                assert set(json.loads(r.text)) == {"risk_score", "verdict", "reason"}
        assert eng.blocks.free == eng.blocks.num_blocks - 1 and not eng.running
        outs[mixed] = [list(r.out_ids) for r in reqs]
    agree = 0.0
    for a, b in zip(outs[False], outs[True]):
        n = min(len(a), len(b))
        k = next((i for i in range(n) if a[i] != b[i]), n)
        agree += k / max(1, n)
    assert agree / len(outs[False]) > 0.6, agree / len(outs[False])
