"""Lazy KV reservation + recompute preemption (brain/engine/engine.py ``kv_alloc="lazy"``; SURVEY.md §7.2 step 6,
§4.2 "greedy determinism under continuous batching and preemption"; VERDICT r4 missing 2 / next 7).

With a KV budget far below the in-flight demand (every request's prompt + num_predict), every request must still
complete, and a greedy request must produce exactly the tokens of an unconstrained run: the preempted request's
re-prefill (prompt + generated ids) computes the pending token's logits the way the interrupted decode step would
have, and its grammar resumes from the saved automaton state.
"""
import json

import pytest

from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
from chronos.sensor.replay import synthetic_chains
from test_jump_forward import _teacher_forced_ok


def _engine(**kw):
    from chronos.brain.engine.engine import Engine, EngineConfig

    base = dict(model="tiny", device="cpu", max_slots=8, max_model_len=384, use_graphs=False, decode_burst=4,
                jump_forward=False, kv_lookahead=16)
    base.update(kw)
    return Engine(EngineConfig(**base))


def _run(eng, chains, budgets, stream=False):
    streamed = {}
    reqs = []
    for i, (c, n) in enumerate(zip(chains, budgets)):
        meta = {"on_tokens": lambda ids, i=i: streamed.setdefault(i, []).extend(ids)} if stream else None
        reqs.append(eng.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=n, meta=meta))
    eng.run_until_idle()
    return reqs, streamed


@pytest.mark.parametrize("mixed,jf,ah", [(False, False, False), (True, False, False), (False, True, False),
                                         (False, True, True), (True, True, True)])
def test_preemption_under_kv_pressure_matches_unconstrained(mixed, jf, ah):
    """Greedy tokens under KV pressure equal the full-reservation run's, also with jump-forward (preemption from
    inside _jump, rows whose run ends the verdict re-queued or finished) and with async harvest (a preemption while
    a harvest snapshot is pending: the preempt_seq guard)."""
    chains = synthetic_chains(10, seed=21, native=False)
    budgets = [24 + 4 * (i % 5) for i in range(10)]
    ref_eng = _engine(kv_alloc="full", mixed_batching=mixed, jump_forward=jf, async_harvest=ah)
    ref, _ = _run(ref_eng, chains, budgets)
    assert ref_eng.stats["preemptions"] == 0
    demand = sum(ref_eng.blocks.blocks_for(len(r.prompt_ids) + r.num_predict) for r in ref)
    nb = 1 + demand // 4  # a quarter of the in-flight demand
    eng = _engine(kv_alloc="lazy", kv_blocks=nb, mixed_batching=mixed, kv_watermark=0.0, jump_forward=jf,
                  async_harvest=ah)
    got, _ = _run(eng, chains, budgets)
    if jf:
        assert eng.stats["jumps"] > 0, dict(eng.stats)
    assert eng.stats["preemptions"] > 0, dict(eng.stats)
    for a, b in zip(got, ref):
        assert a.done_reason in ("stop", "length"), (a.done_reason, a.error)
        assert len(a.prompt_ids) == len(b.prompt_ids)  # the prompt is restored after re-prefills
        assert a.num_predict == b.num_predict  # ... and the request's budget
        json.loads(a.text)
        if mixed and jf:
            # Mixed steps + jump-forward: lazy admission packs other prompts into the mixed forwards than the full
            # engine does, and the tiny random model has exact logit ties (two tokens within 1e-6) that the batch
            # composition's rounding breaks either way.  Both runs are checked as greedy-legal token by token against
            # a from-scratch forward (tests/test_jump_forward.py) instead of against each other.
            _teacher_forced_ok(eng, a, tol=1e-4)
            _teacher_forced_ok(ref_eng, b, tol=1e-4)
        else:
            assert a.done_reason == b.done_reason
            assert a.out_ids == b.out_ids
            assert a.text == b.text
    assert eng.blocks.free == nb - 1 or eng.blocks.prefix_cache  # nothing leaked (cached blocks are evictable)
    assert sum(1 for r in got if r.preemptions) >= 1


def test_preemption_streams_every_token_once():
    chains = synthetic_chains(8, seed=5, native=False)
    budgets = [30] * 8
    ref, _ = _run(_engine(kv_alloc="full"), chains, budgets)
    probe = _engine(kv_alloc="full")
    demand = sum(probe.blocks.blocks_for(len(r.prompt_ids) + r.num_predict) for r in ref)
    eng = _engine(kv_alloc="lazy", kv_blocks=1 + demand // 3, kv_watermark=0.0)
    got, streamed = _run(eng, chains, budgets, stream=True)
    assert eng.stats["preemptions"] > 0
    for i, (a, b) in enumerate(zip(got, ref)):
        assert a.out_ids == b.out_ids
        s = streamed.get(i, [])
        assert s == a.out_ids or s[:-1] == a.out_ids  # (the stream may carry the stop token)


def test_lazy_without_pressure_never_preempts_and_matches_full():
    chains = synthetic_chains(6, seed=3, native=False)
    budgets = [40] * 6
    a, _ = _run(_engine(kv_alloc="full"), chains, budgets)
    eng = _engine(kv_alloc="lazy")
    b, _ = _run(eng, chains, budgets)
    assert eng.stats["preemptions"] == 0 and eng.stats["kv_grow_blocks"] > 0
    assert [r.out_ids for r in a] == [r.out_ids for r in b]


def test_request_larger_than_cache_is_an_error_not_a_stall():
    eng = _engine(kv_alloc="lazy", kv_blocks=4)
    r = eng.submit(build_prompt(["[EXEC] bash -> curl"] * 8), fmt=VERDICT_SCHEMA, num_predict=30)
    eng.run_until_idle(max_steps=50)
    assert r.done_reason == "error" and "KV blocks" in (r.error or "")
    assert not eng.has_work()


def test_auto_reservation_picks_by_pool_size():
    """kv_alloc="auto": full reservation when the pool holds every slot at max_model_len (no pressure possible),
    lazy growth + preemption when it does not."""
    assert _engine(kv_alloc="auto").kv_alloc == "full"
    assert _engine(kv_alloc="auto", kv_blocks=40).kv_alloc == "lazy"


def test_small_bucket_bursts_match_full_bursts():
    """EngineConfig.small_burst (1-step bursts for buckets of <= 2 rows, the single-stream regime) changes only when
    the host harvests, never the tokens: greedy verdicts equal the 4-step-burst engine's, chain after chain."""
    chains = synthetic_chains(4, seed=8, native=False)
    outs = []
    for sb in (0, 1):
        eng = _engine(kv_alloc="full", small_burst=sb, jump_forward=True)
        got = []
        for c in chains:  # one chain in flight at a time
            r = eng.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=40)
            eng.run_until_idle()
            assert r.done_reason in ("stop", "length")
            got.append(r.out_ids)
        outs.append(got)
    assert outs[0] == outs[1]


@pytest.mark.parametrize("ah", [False, True])
def test_lazy_bound_covers_every_write_after_jumps(ah):
    """Engine.pos_hi is the host's upper bound on a row's next KV write position (the pending token's position,
    device s_pos): lazy growth allocates from it, so it must never fall below s_pos — in particular after a jump-forward
    forward, whose sampled token is written one past the run.  Checked after every step of a lazy run with a small
    lookahead (growth at nearly every block boundary), and the tokens must equal the full-reservation run's."""
    chains = synthetic_chains(6, seed=13, native=False)
    budgets = [48] * 6
    ref, _ = _run(_engine(kv_alloc="full", jump_forward=True, async_harvest=ah), chains, budgets)
    eng = _engine(kv_alloc="lazy", jump_forward=True, kv_lookahead=1, async_harvest=ah)
    reqs = [eng.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=n) for c, n in zip(chains, budgets)]
    bs = eng.blocks.block_size
    while eng.has_work():
        eng.step()
        for r in eng.running.values():
            assert r.pos_hi >= int(eng.s_pos[r.slot]), (r.rid, r.pos_hi, int(eng.s_pos[r.slot]))
            assert len(r.blocks) * bs >= min(r.kv_cap, int(eng.s_pos[r.slot])), (r.rid, len(r.blocks))
    assert eng.stats["jumps"] > 0 and eng.stats["kv_grow_blocks"] > 0
    assert [r.out_ids for r in reqs] == [r.out_ids for r in ref]
