"""Jump-forward over grammar-forced token runs (brain/constrain GrammarBank.jumps, Engine._jump, sampler.hip parking).

The CPU engine (tiny model, reference ops) decodes verdicts with and without jump-forward.  Checks: the verdict
grammar has forced runs; jumps happen and every jumped span is exactly the grammar's run; the verdicts stay valid
JSON; and — the numerics check — every token the model chose is the greedy legal argmax of a from-scratch forward
over prompt + output (teacher forcing), so the KV and logits the jump path left behind are the ones plain decoding
would have produced.
"""
from __future__ import annotations

import json

import pytest
import torch

from chronos.brain.constrain import DONE
from chronos.models.llama import make_prefill_batch


@pytest.fixture(scope="module")
def tok():
    from chronos.brain.tokenizer import load_tokenizer

    return load_tokenizer(None)


def _engine(tok, jf: bool):
    from chronos.brain.engine.engine import Engine, EngineConfig

    return Engine(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False,
                               decode_burst=4, max_prefill_tokens=128, jump_forward=jf), tokenizer=tok)


def _prompts(n=3):
    from chronos.sensor.prompt import build_prompt
    from chronos.sensor.replay import synthetic_chains

    return [build_prompt(c.history) for c in synthetic_chains(n, seed=11, native=False)]


def _teacher_forced_ok(eng, req, tol: float = 1e-2) -> None:
    """Every model-chosen output token is the greedy legal choice of a fresh full-sequence forward."""
    seq = req.prompt_ids + req.out_ids
    blocks = eng.blocks.alloc(eng.blocks.blocks_for(len(seq)))
    try:
        sb = make_prefill_batch([seq], [0], [blocks], eng.model.cfg, eng.tp, eng.device,
                                max_blocks=eng.max_blocks_per_seq, nqt=eng.cfg.prefill_nqt)
        sb.last_idx = torch.arange(len(seq), dtype=torch.int64, device=eng.device)
        logits = eng.model.forward(sb, eng.kv).float()
    finally:
        eng.blocks.release(blocks)
    jumped = {j for n0, k in req.meta.get("jump_spans", []) for j in range(n0, n0 + k)}
    bank = eng.bank
    state = bank.get(req.fmt).start
    plen = len(req.prompt_ids)
    for j, t in enumerate(req.out_ids):
        nx = bank.next[state].long()
        if j not in jumped:
            budget = req.num_predict - j - 1
            legal = (nx >= 0) & (bank.dist[nx.clamp(min=0)].long() <= budget)
            lg = logits[plen + j - 1]
            best = float(lg.masked_fill(~legal, float("-inf")).max())
            assert bool(legal[t]), f"token {j} illegal"
            assert float(lg[t]) >= best - tol * (abs(best) + 1.0), f"token {j} is not the greedy choice"
        state = int(nx[t])
        assert state >= 0
    assert state != DONE or req.done_reason == "stop"


def test_verdict_grammar_has_forced_runs(tok):
    from chronos.sensor.prompt import VERDICT_SCHEMA

    eng = _engine(tok, True)
    cg = eng.bank.get(VERDICT_SCHEMA)
    runs = {s: v for s, v in eng.bank.jumps.items() if cg.start <= s < cg.start + cg.num_states}
    assert len(runs) >= 4
    tb = tok.token_bytes_list()
    texts = {b"".join(tb[t] for t in run if t < len(tb)) for run, _ in runs.values()}
    assert any(b"score" in t for t in texts) and any(b"reason" in t or b"on" in t for t in texts)
    for s, (run, end) in runs.items():  # walking the run through the device table lands on its end state
        st = s
        for t in run:
            st = int(eng.bank.next[st, t])
        assert st == end and bool(eng.bank.jump[s])


def test_jump_forward_matches_teacher_forcing(tok):
    from chronos.sensor.prompt import VERDICT_SCHEMA

    eng = _engine(tok, True)
    reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=40) for p in _prompts()]
    eng.run_until_idle()
    assert eng.stats["jumps"] > 0 and eng.stats["jump_tokens"] >= eng.stats["jumps"]
    for r in reqs:
        v = json.loads(r.text)
        assert set(v) == {"risk_score", "verdict", "reason"}
        assert r.meta.get("jump_spans")
        for n0, k in r.meta["jump_spans"]:
            assert n0 + k <= len(r.out_ids) + 1
        _teacher_forced_ok(eng, r)
    assert eng.blocks.free == eng.blocks.num_blocks - 1 and not eng.running


def test_no_jump_forward_also_teacher_forced(tok):
    """The checker itself on plain token-by-token decoding."""
    from chronos.sensor.prompt import VERDICT_SCHEMA

    eng = _engine(tok, False)
    reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=40) for p in _prompts(2)]
    eng.run_until_idle()
    assert eng.stats["jumps"] == 0
    for r in reqs:
        json.loads(r.text)
        _teacher_forced_ok(eng, r)


@pytest.mark.gpu
@pytest.mark.parametrize("asy", [False, True])
def test_jump_forward_gpu_graphs_teacher_forced(asy):
    """GPU engine, captured decode bursts, parking in the HIP sampler: the same properties as on the CPU (bf16 decode
    vs prefill rounding: looser tie tolerance); also with async harvest (single chains and a batch)."""
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA

    eng = Engine(EngineConfig(model="small", device="cuda", max_slots=4, max_model_len=256, decode_burst=4,
                              async_harvest=asy))
    reqs = []
    if asy:  # one chain at a time first (1-step bursts, the single-stream regime)
        for p in _prompts(2):
            reqs.append(eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=48))
            eng.run_until_idle()
    reqs += [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=48) for p in _prompts()]
    eng.run_until_idle()
    assert eng.stats["jumps"] > 0
    for r in reqs:
        assert set(json.loads(r.text)) == {"risk_score", "verdict", "reason"}
        _teacher_forced_ok(eng, r, tol=5e-2)
    off = Engine(EngineConfig(model="small", device="cuda", max_slots=4, max_model_len=256, decode_burst=4,
                              jump_forward=False))
    r0 = off.submit(_prompts(1)[0], fmt=VERDICT_SCHEMA, num_predict=48)
    off.run_until_idle()
    assert off.stats["jumps"] == 0
    json.loads(r0.text)


def _park_case(budget, need, dev="cpu"):
    """States: 0 -(tok 1)-> 1 -(tok 2)-> DONE(=3 here); state 1 starts a forced run needing `need` budget."""
    from chronos import ops

    V, done = 4, 3
    nxt = torch.full((4, V), -1, dtype=torch.int16)
    nxt[0, 1], nxt[1, 2] = 1, done
    dist = torch.tensor([2, 1, 32767, 0], dtype=torch.int16)
    jump = torch.tensor([0, need, 0, 0], dtype=torch.int16)
    i32 = lambda *v: torch.tensor(v, dtype=torch.int32, device=dev)  # noqa: E731
    state, rem = i32(0), i32(budget + 1)  # the sampled token costs 1: `budget` is what is left after it
    ids, pos, ctx, nout = i32(0), i32(5), i32(6), i32(0)
    out = torch.zeros(1, 8, dtype=torch.int32, device=dev)
    logits = torch.zeros(1, V, device=dev)
    ops.constrained_sample(logits, None, nxt.to(dev), dist.to(dev), done, state, rem,
                           torch.zeros(1, device=dev), i32(0), ids, pos, ctx, nout, out, None, None, jump.to(dev))
    return int(state[0])


def test_park_only_when_the_budget_takes_the_run():
    """The sampler parks a row entering a forced-run state only if its remaining budget covers the run plus the
    grammar's shortest finish after it (GrammarBank.jump); otherwise the row keeps decoding (a refused
    jump used to re-park at every state of the run, one token per burst)."""
    assert _park_case(budget=5, need=5) == -2 - 1
    assert _park_case(budget=4, need=5) == 1
    assert _park_case(budget=9, need=0) == 1


@pytest.mark.gpu
def test_park_only_when_the_budget_takes_the_run_gpu():
    from chronos import ops

    ops.load()
    assert _park_case(budget=5, need=5, dev="cuda") == -2 - 1
    assert _park_case(budget=4, need=5, dev="cuda") == 1


def test_tight_budget_never_parks_a_row_it_cannot_jump(tok):
    """num_predict at or just above the grammar's shortest verdict: a forced run the budget cannot take must not
    park the row (it would be refused and unparked at every state of the run, one token per burst)."""
    from chronos.sensor.prompt import VERDICT_SCHEMA

    eng = _engine(tok, True)
    cg = eng.bank.get(VERDICT_SCHEMA)
    need = eng.bank.min_tokens(cg.start)
    prompts = _prompts(2)
    for extra in (0, 1, 2, 4):
        reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=need + extra) for p in prompts]
        eng.run_until_idle()
        for r in reqs:
            assert r.done_reason in ("stop", "length")
            if r.done_reason == "stop":
                assert set(json.loads(r.text)) == {"risk_score", "verdict", "reason"}
    assert eng.stats["jump_refused"] == 0
    eng2 = _engine(tok, True)
    for r in [eng2.submit(p, fmt=VERDICT_SCHEMA, num_predict=40) for p in prompts]:
        pass
    eng2.run_until_idle()
    assert eng2.stats["jumps"] > 0 and eng2.stats["jump_refused"] == 0


@pytest.mark.gpu
def test_sampler_greedy_on_padded_logits_view():
    """A logits view whose row stride is not a multiple of 16 B must not take the 16-B vector path."""
    from chronos import ops

    ops.load()
    V, n = 64, 3
    g = torch.Generator(device="cuda").manual_seed(0)
    base = torch.randn(n, V + 3, device="cuda", generator=g).to(torch.bfloat16)
    logits = base[:, 1:V + 1]  # stride V + 3 elements, base offset 2 B: misaligned rows
    nxt = torch.zeros(1, V, dtype=torch.int16, device="cuda")  # one looping state, every token legal
    dist = torch.ones(1, dtype=torch.int16, device="cuda")
    i32 = lambda v: torch.tensor(v, dtype=torch.int32, device="cuda")  # noqa: E731
    state, rem = i32([0] * n), i32([10] * n)
    out = torch.zeros(n, 4, dtype=torch.int32, device="cuda")
    ops.constrained_sample(logits, None, nxt, dist, -5, state, rem, torch.zeros(n, device="cuda"), i32([0] * n),
                           i32([0] * n), i32([0] * n), i32([1] * n), i32([0] * n), out)
    assert out[:, 0].tolist() == logits.float().argmax(1).tolist()


@pytest.mark.parametrize("burst", [1, 4])
def test_jump_forward_with_async_harvest_teacher_forced(tok, burst):
    """Async harvest (burst k harvested while burst k+1 runs) with jump-forward: a parked row is seen one burst late,
    the stale snapshot taken before its jump is skipped, and every verdict is still the teacher-forced greedy one —
    the same tokens as the synchronous engine, one chain at a time and several in flight."""
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA

    outs = {}
    for asy in (False, True):
        eng = Engine(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False,
                                  decode_burst=burst, small_burst=0, max_prefill_tokens=128, jump_forward=True,
                                  async_harvest=asy), tokenizer=tok)
        single = []
        for p in _prompts(2):
            r = eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=40)
            eng.run_until_idle()
            single.append(r)
        batch = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=40) for p in _prompts(3)]
        eng.run_until_idle()
        for r in single + batch:
            json.loads(r.text)
            _teacher_forced_ok(eng, r)
        assert eng.stats["jumps"] > 0
        assert eng.blocks.free == eng.blocks.num_blocks - 1 and not eng.running
        outs[asy] = [r.out_ids for r in single + batch]
    assert outs[True] == outs[False]
