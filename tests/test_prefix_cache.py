"""Prefix caching: reusing the shared CHRONOS template block changes nothing but the work done."""
import pytest

from chronos.brain.engine.block_manager import BlockManager


def test_block_manager_refcounts_and_lru():
    bm = BlockManager(10, 4)
    toks = list(range(13))           # 3 full blocks + 1 token
    a = bm.alloc(4)
    bm.register(toks, a)
    assert bm.lookup(toks) == a[:3]  # never the block holding the last prompt token
    bm.release(a)                    # owner done; the 3 shared still referenced by the lookup
    assert bm.free == 9 - 3
    bm.release(a[:3])                # sharer done: cached blocks become evictable, still hit
    assert bm.free == 9 and bm.lookup(toks) == a[:3]
    bm.release(a[:3])
    taken = bm.alloc(9)              # pressure evicts the cached blocks (LRU) and forgets their hashes
    assert len(set(taken)) == 9 and bm.lookup(toks) == []


def test_partial_block_lookup_uses_only_computed_slots():
    bm = BlockManager(16, 4)
    a_toks = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10]       # 2 full blocks + 2 tokens
    a = bm.alloc(3)
    bm.register(a_toks, a)
    bm.note_prompt(a_toks, a)
    b_toks = [1, 2, 3, 4, 5, 6, 70, 80, 90, 100]    # shares block 0 and 2 slots of block 1
    assert bm.lookup_partial(b_toks, 1) is None      # nothing computed yet
    bm.mark_computed(a, 0, 10)
    got = bm.lookup_partial(b_toks, 1)
    assert got == (a[1], 2)
    bm.release([got[0]])
    c_toks = [1, 2, 3, 4, 5, 6, 7, 8, 9, 11, 12]   # block 2 matches 1 slot: below min_tokens
    assert bm.lookup_partial(c_toks, 2) is None
    assert bm.lookup_partial(c_toks, 2, min_tokens=1) == (a[2], 1)
    d_toks = [1, 2, 3, 4, 5, 6, 7]                   # prompt ends inside the block: its last token is recomputed
    assert bm.lookup_partial(d_toks, 1) == (a[1], 2)
    bm.release(a)
    bm.release([a[1], a[2]])                         # the partial last block is freed and stops being a source
    assert bm.lookup_partial(c_toks, 2, min_tokens=1) is None


def test_partial_source_maps_stay_bounded():
    """Unique prompts (argv makes deep parents unique) cycling through a small cache: the partial-block source maps
    must shrink as blocks are reused or freed, never grow with the number of requests."""
    import random

    rng = random.Random(0)
    bm = BlockManager(24, 4)
    for i in range(400):
        toks = [1, 2, 3, 4, 5, 6] + [rng.randrange(1000) for _ in range(rng.randrange(3, 15))]
        shared = bm.lookup(toks)
        blocks = shared + bm.alloc(bm.blocks_for(len(toks)) - len(shared))
        bm.note_prompt(toks, blocks, len(shared))
        bm.mark_computed(blocks, len(shared) * 4, len(toks))
        bm.register(toks, blocks)
        bm.release(blocks)
        assert len(bm._part) <= bm.num_blocks
        assert sum(len(v) for v in bm._children.values()) == len(bm._part)
        assert len(bm._children) <= bm.num_blocks
    off = BlockManager(8, 4, partial_prefix=False)
    b = off.alloc(2)
    off.note_prompt(list(range(8)), b)
    assert not off._part and not off._children and off.lookup_partial(list(range(8)), 1) is None


@pytest.mark.parametrize("partial", [False, True])
def test_engine_partial_prefix_same_outputs(partial):
    """Prompts arriving after earlier ones were prefilled reuse computed slots of partially matching blocks."""
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    chains = synthetic_chains(12, seed=11, native=False)
    outs, stats = [], []
    for pc in (False, True):
        # non-mixed scheduling: both runs batch every decode row identically, so outputs must match bit for bit
        eng = Engine(EngineConfig(model="tiny", device="cpu", max_slots=16, max_model_len=384, use_graphs=False,
                                  prefix_cache=pc, partial_prefix=partial, max_prefill_tokens=120, prefill_ramp=0,
                                  jump_forward=False, mixed_batching=False))
        reqs = [eng.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=20) for c in chains]
        eng.run_until_idle()
        outs.append([r.out_ids for r in reqs])
        stats.append(dict(eng.stats))
    assert outs[0] == outs[1]
    if partial:
        assert stats[1]["partial_prefix_tokens"] > 0


@pytest.mark.parametrize("chunk", [200, 40])
def test_engine_prefix_cache_same_outputs(chunk):
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    chains = synthetic_chains(10, seed=4, native=False)
    outs, stats = [], []
    for pc in (False, True):
        eng = Engine(EngineConfig(model="tiny", device="cpu", max_slots=8, max_model_len=384, use_graphs=False,
                                  prefix_cache=pc, max_prefill_tokens=chunk, mixed_batching=False))
        reqs = [eng.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=30) for c in chains]
        eng.run_until_idle()
        outs.append([r.out_ids for r in reqs])
        stats.append(dict(eng.stats))
    assert outs[0] == outs[1]
    assert stats[1]["prefix_hit_tokens"] >= 16 * 9 and stats[1]["prefill_tokens"] < stats[0]["prefill_tokens"]


def test_slot_compaction_preserves_outputs():
    """Verdicts of different lengths finish at different steps; compaction moves live rows down so the decode bucket
    shrinks — every sequence must still produce exactly what it produces alone."""
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    chains = synthetic_chains(12, seed=4, native=False)
    budgets = list(range(16, 40, 2))
    # jump-forward off: it only runs while <= jump_max_rows sequences decode, and its canonical tokenization of forced
    # runs would make the batch and the solo token ids differ by design (the verdict text of those runs is the same)
    mk = lambda: Engine(EngineConfig(model="tiny", device="cpu", max_slots=16, max_model_len=384,  # noqa: E731
                                     use_graphs=False, decode_burst=4, jump_forward=False))
    eng = mk()
    reqs = [eng.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=n) for c, n in zip(chains, budgets)]
    eng.run_until_idle()
    assert eng.stats["compactions"] >= 1
    solo_eng = mk()
    for c, n, r in zip(chains, budgets, reqs):
        s = solo_eng.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=n)
        solo_eng.run_until_idle()
        assert s.out_ids == r.out_ids


def test_async_harvest_matches_sync_with_refill_and_streaming():
    """Harvesting burst k while burst k+1 runs (GPU default) reads slot states one burst late, across compaction and
    slots refilled by later submissions: outputs, stream chunks and completion must equal the synchronous engine."""
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    chains = synthetic_chains(14, seed=9, native=False)
    budgets = [16 + 3 * (i % 7) for i in range(14)]

    def run(async_harvest):
        eng = Engine(EngineConfig(model="tiny", device="cpu", max_slots=8, max_model_len=384, use_graphs=False,
                                  decode_burst=3, async_harvest=async_harvest, jump_forward=False))
        streamed = {}
        reqs = []

        def submit(i):
            r = eng.submit(build_prompt(chains[i].history), fmt=VERDICT_SCHEMA, num_predict=budgets[i],
                           meta={"on_tokens": lambda ids, i=i: streamed.setdefault(i, []).extend(ids)})
            reqs.append(r)

        for i in range(6):
            submit(i)
        nxt, steps = 6, 0
        while eng.has_work() or nxt < len(chains):
            eng.step()
            steps += 1
            if steps % 2 == 0 and nxt < len(chains):  # arrivals mid-run land in freed (possibly compacted) slots
                submit(nxt)
                nxt += 1
        return reqs, streamed, eng.stats

    a_reqs, a_stream, a_stats = run(True)
    s_reqs, s_stream, _ = run(False)
    assert a_stats["compactions"] >= 1
    for a, s in zip(a_reqs, s_reqs):
        assert a.done_reason == s.done_reason and a.done_reason in ("stop", "length")
        assert a.out_ids == s.out_ids
    for i, a in enumerate(a_reqs):
        got = a_stream.get(i, [])
        assert got == a.out_ids or got[:-1] == a.out_ids  # the stream may include the stop token
