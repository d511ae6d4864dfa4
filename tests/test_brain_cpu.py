"""CPU tests of the Brain: grammars, tokenizer, grammar bank, model consistency, engine end-to-end, TP over gloo.

The CPU path runs the same model/engine code with the fp32 reference ops (chronos.ops.reference); the GPU path is
covered by tests/test_kernels_gpu.py.
"""
import json
import os
import socket

import pytest
import torch

from chronos.brain.constrain import grammar as G


# ---------------------------------------------------------------------------------------------------------------
# grammars
# ---------------------------------------------------------------------------------------------------------------

def test_verdict_schema_language():
    from chronos.sensor.prompt import VERDICT_SCHEMA

    d = G.compile_dfa(G.grammar_for_format(VERDICT_SCHEMA, max_string=40))
    good = [b'{"risk_score": 8, "verdict": "MALICIOUS", "reason": "curl then chmod"}',
            b'{"risk_score":0,"verdict":"SAFE","reason":""}',
            b' {"risk_score": 10, "verdict": "SAFE", "reason": "a \\"quoted\\" word"}\n']
    bad = [b'{"risk_score": 11, "verdict": "MALICIOUS", "reason": "x"}',
           b'{"verdict": "SAFE", "risk_score": 1, "reason": "x"}',
           b'{"risk_score": 1, "verdict": "MAYBE", "reason": "x"}',
           b'{"risk_score": 1, "verdict": "SAFE", "reason": "' + b"x" * 41 + b'"}',
           b'{"risk_score": 1, "verdict": "SAFE"}']
    for s in good:
        assert d.matches(s), s
        json.loads(s)
    for s in bad:
        assert not d.matches(s), s


def test_json_grammar_depth_and_validity():
    d = G.compile_dfa(G.grammar_for_format("json", json_depth=3))
    assert d.matches(b'{"a": [1, -2.5e3, {"b": null}], "c": "x", "d": true}')
    assert d.matches(b"{}")
    assert not d.matches(b'{"a": [1,}')
    assert not d.matches(b'[1, 2]')  # Ollama json mode: an object
    assert not d.matches(b'{"a": {"b": {"c": {"d": 1}}}}')  # deeper than 3


def test_schema_subset():
    sch = {"type": "object", "properties": {"n": {"type": "integer", "minimum": 1, "maximum": 3},
                                            "tags": {"type": "array", "items": {"type": "string", "enum": ["a", "b"]},
                                                     "maxItems": 2},
                                            "ok": {"type": "boolean"}},
           "required": ["n", "ok"]}
    d = G.compile_dfa(G.grammar_for_format(sch))
    assert d.matches(b'{"n": 2, "tags": ["a", "b"], "ok": true}')
    assert d.matches(b'{"n": 2, "ok": false}')
    assert not d.matches(b'{"n": 4, "ok": false}')
    assert not d.matches(b'{"n": 2, "tags": ["a", "b", "a"], "ok": true}')


# ---------------------------------------------------------------------------------------------------------------
# tokenizer + grammar bank
# ---------------------------------------------------------------------------------------------------------------

@pytest.fixture(scope="module")
def tok():
    from chronos.brain.tokenizer import ChronosBPE

    return ChronosBPE()


def test_tokenizer_roundtrip_and_template(tok):
    from chronos.brain.tokenizer import BOS_ID, END_HEADER_ID, EOT_ID, START_HEADER_ID
    from chronos.sensor.prompt import build_prompt

    p = build_prompt(["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"])
    ids = tok.encode(p)
    assert tok.decode(ids) == p
    assert 60 <= len(ids) <= 110  # realistic prompt lengths (Llama-3 would give ~80)
    chat = tok.chat_ids(p)
    assert chat[0] == BOS_ID and chat.count(START_HEADER_ID) == 2 and chat.count(END_HEADER_ID) == 2
    assert EOT_ID in chat and max(chat) < 128256
    tb = tok.token_bytes_list()
    assert len(tb) == 128256 and tb[BOS_ID] == b"" and b"".join(tb[i] for i in ids) == p.encode()


def test_piece_cached_encoding_is_exact(tok):
    from chronos.sensor.prompt import build_prompt
    from chronos.sensor.replay import synthetic_chains

    texts = ["\n\n" + build_prompt(c.history) for c in synthetic_chains(300, seed=21, native=False)]
    texts += ["hello   world\n\n  x", "a\tb  \n", "naïve café 日本語 123456", "  leading", "trailing  ", "''s 're",
              "x\n\n\n", '{"risk_score": 8, "verdict": "MALICIOUS"}']
    for t in texts + texts:  # second pass hits the cache
        assert tok.encode(t) == tok.encode_uncached(t)


def test_grammar_bank_walk(tok):
    from chronos.brain.constrain import DONE, GrammarBank
    from chronos.sensor.prompt import VERDICT_SCHEMA

    bank = GrammarBank(tok.token_bytes_list(), tok.stop_ids, 128256, capacity=1024)
    g = bank.get(VERDICT_SCHEMA)
    assert bank.get(dict(VERDICT_SCHEMA)) is g  # cached by content
    text = '{"risk_score": 8, "verdict": "MALICIOUS", "reason": "dropper pattern"}'
    s = g.start
    for i in tok.encode(text):
        s = bank.step(s, i)
        assert s > 0
    assert bank.step(s, tok.eot_id) == DONE
    assert bank.min_tokens(g.start) >= 10
    free = bank.get(None)
    assert bank.step(free.start, tok.encode("hello")[0]) == free.start
    assert bank.step(free.start, tok.eot_id) == DONE


# ---------------------------------------------------------------------------------------------------------------
# model consistency (reference ops)
# ---------------------------------------------------------------------------------------------------------------

def _logits(model, kv, prompts, starts, bts, split=1):
    from chronos.models.llama import make_prefill_batch

    sb = make_prefill_batch(prompts, starts, bts, model.cfg, model.tp, "cpu", max_blocks=8, split=split)
    return model.forward(sb, kv).float()


def test_chunked_prefill_equals_full():
    from chronos.models.llama import KVCache, build_model

    m = build_model("tiny", "cpu", seed=1)
    toks = list(range(200, 260))
    kv1 = KVCache(m.cfg, m.tp, 16, 16, "cpu")
    full = _logits(m, kv1, [toks], [0], [[3, 4, 5, 6]])
    kv2 = KVCache(m.cfg, m.tp, 16, 16, "cpu")
    _logits(m, kv2, [toks[:23]], [0], [[3, 4, 5, 6]])
    part = _logits(m, kv2, [toks[23:]], [23], [[3, 4, 5, 6]])
    assert torch.allclose(full, part, atol=2e-2, rtol=0)


def test_batched_equals_single():
    from chronos.models.llama import KVCache, build_model

    m = build_model("tiny", "cpu", seed=2)
    a, b = list(range(300, 337)), list(range(500, 509))
    kv = KVCache(m.cfg, m.tp, 16, 16, "cpu")
    both = _logits(m, kv, [a, b], [0, 0], [[1, 2, 3], [4]])
    kv = KVCache(m.cfg, m.tp, 16, 16, "cpu")
    only_b = _logits(m, kv, [b], [0], [[7]])
    assert torch.allclose(both[1], only_b[0], atol=2e-2)


def test_rope_llama31_scaling_matches_formula():
    from chronos.models.llama import get_config, rope_inv_freq

    base = rope_inv_freq(get_config("llama3-8b"))
    sc = rope_inv_freq(get_config("llama3.1-8b"))
    assert torch.allclose(sc[:10], base[:10])          # high-frequency dims untouched
    assert torch.allclose(sc[-5:], base[-5:] / 8.0)     # low-frequency dims divided by the factor


# ---------------------------------------------------------------------------------------------------------------
# engine
# ---------------------------------------------------------------------------------------------------------------

@pytest.fixture(scope="module")
def engine(tok):
    from chronos.brain.engine.engine import Engine, EngineConfig

    return Engine(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False,
                               decode_burst=4, max_prefill_tokens=96), tokenizer=tok)


def test_engine_verdicts_are_valid_json(engine):
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    chains = synthetic_chains(6, seed=11, native=False)  # 6 > 4 slots: exercises admission + slot reuse
    reqs = [engine.submit(build_prompt(c.history), fmt=VERDICT_SCHEMA, num_predict=32) for c in chains]
    engine.run_until_idle()
    for r in reqs:
        v = json.loads(r.text)
        assert set(v) == {"risk_score", "verdict", "reason"} and 0 <= v["risk_score"] <= 10
        assert v["verdict"] in ("SAFE", "MALICIOUS")
        assert r.done_reason == "stop" and len(r.out_ids) < 32
    assert engine.blocks.free == engine.blocks.num_blocks - 1
    assert not engine.running and not engine.prefilling


def test_engine_prefill_ramp(tok):
    """After an idle period the prefill steps grow prefill_ramp, 4x, 16x ... up to max_prefill_tokens, and the
    verdicts are the ones full-size chunks give."""
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    prompts = [build_prompt(c.history) for c in synthetic_chains(6, seed=5, native=False)]
    texts = {}
    for ramp in (0, 16):
        eng = Engine(EngineConfig(model="tiny", device="cpu", max_slots=8, max_model_len=384, use_graphs=False,
                                  decode_burst=4, max_prefill_tokens=256, prefix_cache=False, prefill_ramp=ramp),
                     tokenizer=tok)
        sizes = []
        for _ in range(2):  # the ramp restarts once the engine went idle
            reqs = [eng.submit(p, fmt=VERDICT_SCHEMA, num_predict=16) for p in prompts]
            while eng.has_work():
                before, pre = eng.stats["prefill_tokens"], bool(eng.prefilling or eng.waiting)
                eng.step()
                if pre:
                    sizes.append(eng.stats["prefill_tokens"] - before)
        texts[ramp] = [r.text for r in reqs]
        total = sum(len(r.prompt_ids) for r in reqs)
        if ramp:
            half = sizes[:len(sizes) // 2]
            assert half[:3] == [16, 64, 256] and sum(half) == total, sizes
            assert sizes[len(sizes) // 2] == 16
        else:
            assert sizes[0] == 256
    assert texts[0] == texts[16]


def test_engine_json_mode_and_budget(engine):
    r = engine.submit("anything", fmt="json", num_predict=12)
    r2 = engine.submit("free text", fmt=None, num_predict=5, temperature=0.9, seed=3)
    engine.run_until_idle()
    assert isinstance(json.loads(r.text), dict) and len(r.out_ids) <= 11
    assert len(r2.out_ids) <= 5


def test_engine_deterministic_greedy(engine):
    from chronos.sensor.prompt import VERDICT_SCHEMA

    a = engine.submit("same prompt", fmt=VERDICT_SCHEMA, num_predict=24)
    engine.run_until_idle()
    b = engine.submit("same prompt", fmt=VERDICT_SCHEMA, num_predict=24)
    engine.run_until_idle()
    assert a.out_ids == b.out_ids


def test_engine_long_prompt_chunked(engine):
    from chronos.sensor.prompt import VERDICT_SCHEMA

    hist = [f"[OPEN] app{i} -> /home/kali/file{i}.txt" for i in range(12)]
    r = engine.submit(str(hist), fmt=VERDICT_SCHEMA, num_predict=20)
    engine.run_until_idle()
    assert len(r.prompt_ids) > 96  # needed more than one prefill chunk
    json.loads(r.text)


def test_engine_rejects_oversized_and_bad_format(engine):
    r = engine.submit(list(range(1000)), fmt=None, num_predict=10)
    assert r.done_reason == "error" and "max_model_len" in r.error
    from chronos.sensor.prompt import VERDICT_SCHEMA

    r = engine.submit("x", fmt=VERDICT_SCHEMA, num_predict=4)  # the verdict needs >= 15 tokens
    assert r.done_reason == "error" and "num_predict" in r.error


# ---------------------------------------------------------------------------------------------------------------
# tensor parallelism over gloo (the multi-GPU code path without GPUs)
# ---------------------------------------------------------------------------------------------------------------

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_worker(rank, world, port, q):
    import torch.distributed as dist

    from chronos.models.llama import KVCache, build_model
    from chronos.parallel.tp import TPContext

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TPContext.from_group()
    m = build_model("tiny", "cpu", tp=tp, seed=4)
    kv = KVCache(m.cfg, tp, 16, 16, "cpu")
    out = _logits(m, kv, [list(range(40, 71)), list(range(90, 95))], [0, 0], [[1, 2], [3]])
    # the overlapped form: two micro-batches, async all-reduces interleaved with the other part's compute
    kv2 = KVCache(m.cfg, tp, 16, 16, "cpu")
    out2 = _logits(m, kv2, [list(range(40, 71)), list(range(90, 95)), list(range(7, 30))], [0, 0, 0],
                   [[1, 2], [3], [4, 5]], split=2)
    if rank == 0:  # numpy, pickled by value: a torch tensor would be shared through an fd the exiting worker owns
        q.put((out.numpy(), out2.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_tensor_parallel_matches_single():
    import torch.multiprocessing as mp

    from chronos.models.llama import KVCache, build_model

    m = build_model("tiny", "cpu", seed=4)
    kv = KVCache(m.cfg, m.tp, 16, 16, "cpu")
    ref = _logits(m, kv, [list(range(40, 71)), list(range(90, 95))], [0, 0], [[1, 2], [3]])
    kv2 = KVCache(m.cfg, m.tp, 16, 16, "cpu")
    ref2 = _logits(m, kv2, [list(range(40, 71)), list(range(90, 95)), list(range(7, 30))], [0, 0, 0],
                   [[1, 2], [3], [4, 5]])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_tp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out, out2 = (torch.from_numpy(a) for a in q.get(timeout=240))
    for p in ps:
        p.join(timeout=60)
    assert torch.allclose(out, ref, atol=3e-2), float((out - ref).abs().max())
    assert out2.shape == ref2.shape
    assert torch.allclose(out2, ref2, atol=3e-2), float((out2 - ref2).abs().max())
