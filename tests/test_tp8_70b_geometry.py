"""Tensor parallelism at W = 8 with the Llama-3-70B attention geometry, over gloo on the CPU (VERDICT r3 item 5;
SURVEY.md §2.4 C1-C5, §4.2 "distributed (CPU)").

The ``tiny70`` preset keeps what makes 70B TP=8 different from the W = 2 tests: 64 query / 8 KV heads, so every rank
holds ONE KV head with a GQA group of 8, and the real 128256-token vocabulary, so every rank's embedding / LM-head
shard is 16032 rows (not a multiple of 128).  Weights are fp32, so the only difference between TP = 8 and TP = 1 is
summation order (plus the bf16 KV cache both share):

* first-step logits of a 3-prompt prefill (odd token count) match TP = 1 within 1e-3 of max |logit|, in all four
  combinations of Megatron sequence parallelism (reduce-scatter / all-gather) and the two-micro-batch overlap split;
* a lockstep TP = 8 engine (leader schedules, 7 followers) produces exactly the TP = 1 engine's greedy tokens.
"""
import os
import socket

import pytest
import torch

PROMPTS = [[128000] + list(range(10, 47)), list(range(200, 219)), list(range(300, 305))]  # 61 tokens (odd)
BTS = [[1, 2, 3], [4, 5], [6]]
CHAINS = [["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"],
          ["[EXEC] bash -> cat", "[OPEN] cat -> /tmp/malware.bin", "[EXEC] bash -> nc"]]
SEED = 5


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(tp):
    from chronos.models.llama import LlamaModel, get_config, random_weights

    cfg = get_config("tiny70")
    return LlamaModel(cfg, random_weights(cfg, tp, "cpu", SEED, dtype=torch.float32), tp, "cpu")


def _prefill_logits(m, sp: bool, split: int):
    from chronos.models.llama import KVCache, make_prefill_batch

    m.sequence_parallel = sp
    kv = KVCache(m.cfg, m.tp, 12, 16, "cpu")
    sb = make_prefill_batch(PROMPTS, [0, 0, 0], BTS, m.cfg, m.tp, "cpu", max_blocks=3, split=split)
    out = m.forward(sb, kv, logits_dtype=torch.float32)
    m.sequence_parallel = False
    return out


def _ecfg():
    from chronos.brain.engine.engine import EngineConfig

    return EngineConfig(model="tiny70", device="cpu", max_slots=4, max_model_len=256, use_graphs=False,
                        decode_burst=4, max_prefill_tokens=256)


def _greedy_tp1():
    from chronos.brain.engine.engine import Engine
    from chronos.sensor.prompt import build_prompt

    eng = Engine(_ecfg(), model=_model(None))
    reqs = [eng.submit(build_prompt(c), num_predict=12) for c in CHAINS]
    eng.run_until_idle()
    return [list(r.out_ids) for r in reqs]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from chronos.parallel.tp import TPContext
    from chronos.parallel.tp_engine import TPEngine
    from chronos.sensor.prompt import build_prompt

    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TPContext.from_group()
    m = _model(tp)
    shard = (m.w.embed.shape[0], m.cfg.num_kv_heads // tp.world)
    logits = {f"{int(sp)}{split}": _prefill_logits(m, sp, split).numpy() for sp in (False, True) for split in (1, 2)}
    eng = TPEngine(_ecfg(), tp, ctrl_group=None, model=m)
    if rank == 0:
        res = {}
        for i, c in enumerate(CHAINS):
            eng.submit(build_prompt(c), num_predict=12, callback=lambda r, i=i: res.__setitem__(i, list(r.out_ids)))
        eng.run_until_idle()
        q.put((rank, shard, logits, [res[i] for i in range(len(CHAINS))]))
    else:
        eng.follower_loop()
        q.put((rank, shard, None, dict(eng.engine.stats)["completed"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_tp8_70b_geometry_matches_tp1():
    import torch.multiprocessing as mp

    torch.set_num_threads(2)
    ref = _prefill_logits(_model(None), False, 1)
    ref_ids = _greedy_tp1()
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        item = q.get(timeout=900)
        got[item[0]] = item
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r][1] == (16032, 1)  # vocab shard rows, KV heads per rank
        if r:
            assert got[r][3] == len(CHAINS)  # every follower completed the same requests in lockstep
    _, _, logits, ids = got[0]
    tol = 1e-3 * ref.abs().max().item()
    for key, lg in logits.items():
        err = (torch.from_numpy(lg) - ref).abs().max().item()
        assert err <= tol, f"sp/split {key}: max |TP8 - TP1| {err:.3g} > {tol:.3g}"
        assert (torch.from_numpy(lg).argmax(-1) == ref.argmax(-1)).all()
    assert ids == ref_ids  # identical greedy tokens through the lockstep TP engine
