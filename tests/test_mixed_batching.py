"""Mixed prefill + decode steps (steady-state continuous batching; Engine._mixed_step).

While sequences decode, arriving prompts are prefilled in the SAME forward as one decode token of every live row, so
a prompt never stalls the verdicts already in flight (the reference's README claims asynchronous many-in-flight
analysis, /root/reference/README.md:24, which its blocking call at chronos_sensor.py:147 never delivered)."""
from __future__ import annotations

import json

import pytest


def _engine(**kw):
    from chronos.brain.engine.engine import Engine, EngineConfig

    base = dict(model="tiny", device="cpu", max_slots=8, max_model_len=384, use_graphs=False, decode_burst=4,
                max_prefill_tokens=200, jump_forward=False)
    base.update(kw)
    return Engine(EngineConfig(**base))


def _chains(n, seed=4):
    from chronos.sensor.prompt import build_prompt
    from chronos.sensor.replay import synthetic_chains

    return [build_prompt(c.history) for c in synthetic_chains(n, seed=seed, native=False)]


def test_decode_rows_advance_while_prompts_keep_arriving():
    from chronos.sensor.prompt import VERDICT_SCHEMA

    eng = _engine(mixed_prefill_tokens=48, mixed_ratio=1)
    prompts = _chains(14)
    reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=30) for p in prompts[:3]]
    nxt, stalled, mixed_seen = 3, 0, 0
    while eng.has_work() or nxt < len(prompts):
        if nxt < len(prompts) and eng.running:  # a new chain arrives every step once decoding started
            reqs.append(eng.submit(prompts[nxt], fmt=VERDICT_SCHEMA, num_predict=30))
            nxt += 1
        running = dict(eng.running)
        before = {s: int(eng.s_nout[s]) for s in running}
        m0 = eng.stats["mixed_steps"]
        eng.step()
        mixed_seen += eng.stats["mixed_steps"] > m0
        # every row that was decoding before the step and is still decoding after it gained tokens
        for s, r in running.items():
            if eng.running.get(s) is r and int(eng.s_nout[s]) == before[s] and int(eng.s_state[s]) > 0:
                stalled += 1
    assert mixed_seen > 0
    assert stalled == 0
    assert eng.stats["mixed_steps"] >= 3
    for r in reqs:
        assert r.done_reason in ("stop", "length")
        if r.done_reason == "stop":
            assert set(json.loads(r.text)) == {"risk_score", "verdict", "reason"}


def test_mixed_steps_match_teacher_forcing_and_plain_scheduling():
    """A mixed step computes exactly what separate prefill and decode steps compute (reference ops are row-wise
    deterministic): same output ids as non-mixed scheduling, and every token the greedy choice of a fresh forward."""
    import sys
    import os

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_jump_forward import _teacher_forced_ok

    from chronos.sensor.prompt import VERDICT_SCHEMA

    prompts = _chains(10)
    outs = []
    for mixed in (False, True):
        eng = _engine(mixed_batching=mixed, mixed_prefill_tokens=64, mixed_ratio=2)
        reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=30) for p in prompts[:4]]
        eng.step()
        eng.step()
        reqs += [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=30) for p in prompts[4:]]
        eng.run_until_idle()
        assert (eng.stats["mixed_steps"] > 0) == mixed
        for r in reqs:
            _teacher_forced_ok(eng, r)
        outs.append([r.out_ids for r in reqs])
        assert eng.blocks.free == eng.blocks.num_blocks - 1 and not eng.running
    assert outs[0] == outs[1]


def test_wave_backlog_prefills_in_full_steps():
    """A wave (more queued prompts than mixed_max_backlog) is prefilled in full-size steps; mixing resumes once the
    backlog is a trickle."""
    from chronos.sensor.prompt import VERDICT_SCHEMA

    eng = _engine(max_slots=8, mixed_max_backlog=4, mixed_prefill_tokens=48, mixed_ratio=1)
    prompts = _chains(12)
    reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=20) for p in prompts]
    seen = []
    while eng.has_work():
        backlog = len(eng.waiting) + len(eng.prefilling)
        m0, p0 = eng.stats["mixed_steps"], eng.stats["prefill_steps"]
        eng.step()
        if eng.stats["mixed_steps"] > m0:
            seen.append(backlog)
    assert seen and max(seen) <= 4
    assert all(r.done_reason in ("stop", "length") for r in reqs)


def test_mixed_steps_with_jump_forward_apply_each_run_once():
    """Jump-forward parking together with mixed steps: a mixed step harvests the snapshot of the step
    before, which can still show a row parked whose run the previous harvest already appended.  Every run must be
    applied exactly once (spans strictly increasing, never overlapping) and the output must still be the greedy
    choice of a fresh forward at every position (teacher forcing)."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_jump_forward import _teacher_forced_ok

    from chronos.sensor.prompt import VERDICT_SCHEMA

    prompts = _chains(16, seed=9)
    eng = _engine(mixed_batching=True, jump_forward=True, mixed_prefill_tokens=48, mixed_ratio=1, decode_burst=1)
    reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=40) for p in prompts[:3]]
    nxt, it, stale = 3, 0, 0
    harvest = eng._harvest

    def counting_harvest(snap):  # count parked rows a lagging (mixed-step) harvest must skip
        nonlocal stale
        st = snap.state[:snap.n].tolist()
        stale += sum(1 for s, r in snap.owners.items() if eng.running.get(r.slot) is r and st[s] <= -2
                     and r.meta.get("jump_seq", 0) >= snap.seq)
        return harvest(snap)

    eng._harvest = counting_harvest
    # park in mixed steps too (production passes None there): every parked row is then seen by two lagging harvests
    sample = eng._sample
    eng._sample = lambda logits, jump: sample(logits, eng._jump_flags(len(eng.running) + 1))
    while eng.has_work() or nxt < len(prompts):
        # phases: a few plain decode steps (rows get parked by the decode sampler, jumps resample and park again),
        # then arrivals every step (mixed steps, whose harvests lag one step behind those parks)
        if nxt < len(prompts) and eng.running and it % 6 >= 3:
            reqs.append(eng.submit(prompts[nxt], fmt=VERDICT_SCHEMA, num_predict=40))
            nxt += 1
        eng.step()
        it += 1
    assert eng.stats["mixed_steps"] > 0 and eng.stats["jumps"] > 0
    assert stale > 0  # the lagging-harvest case was exercised
    for r in reqs:
        assert r.done_reason in ("stop", "length")
        spans = r.meta.get("jump_spans", [])
        for (a0, k0), (a1, _) in zip(spans, spans[1:]):
            assert a1 >= a0 + k0, spans  # a run applied twice would restart at (or before) its own start
        _teacher_forced_ok(eng, r)
