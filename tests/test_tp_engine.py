"""Tensor-parallel engine over gloo (world 2): lockstep replicated scheduling produces the same verdicts on every rank
and matches the TP=1 engine (the multi-GPU serving path exercised without GPUs; SURVEY.md §4.2 "distributed")."""
import json
import os
import socket

import pytest


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CHAINS = [["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"],
          ["[EXEC] bash -> chmod", "[OPEN] chmod -> "],
          ["[EXEC] bash -> cat", "[OPEN] cat -> /tmp/malware.bin", "[EXEC] bash -> nc"]]


def _cfg():
    from chronos.brain.engine.engine import EngineConfig

    return EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False, decode_burst=4)


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from chronos.parallel.tp import TPContext
    from chronos.parallel.tp_engine import TPEngine
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TPContext.from_group()
    eng = TPEngine(_cfg(), tp, ctrl_group=None)
    if rank == 0:
        results = {}
        for i, c in enumerate(CHAINS):
            eng.submit(build_prompt(c), fmt=VERDICT_SCHEMA, num_predict=40,
                       callback=lambda r, i=i: results.__setitem__(i, (r.out_ids, r.text, r.done_reason)))
        # a cancellation is decided by the leader and applied on every rank in the same step
        tag = eng.submit(build_prompt(CHAINS[0]), fmt=VERDICT_SCHEMA, num_predict=40,
                         callback=lambda r: results.__setitem__(3, (r.out_ids, r.text, r.done_reason)))
        eng.cancel(tag)
        eng.run_until_idle()
        q.put(("leader", results))
    else:
        eng.follower_loop()
        q.put(("follower", dict(eng.engine.stats)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_tp2_engine_lockstep_matches_tp1():
    import torch.multiprocessing as mp

    from chronos.brain.engine.engine import Engine
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    ref = Engine(_cfg())
    reqs = [ref.submit(build_prompt(c), fmt=VERDICT_SCHEMA, num_predict=40) for c in CHAINS]
    ref.run_until_idle()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=600) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    res = got["leader"]
    assert sorted(res) == [0, 1, 2, 3]
    assert res[3][2] == "cancelled" and got["follower"]["cancelled"] == 1
    assert got["follower"]["completed"] == 3
    agree = 0
    for i, r in enumerate(reqs):
        ids, text, _ = res[i]
        assert set(json.loads(text)) == {"risk_score", "verdict", "reason"}
        # same model, different summation order across the TP shards: greedy paths agree on the prefix at least
        n = min(len(ids), len(r.out_ids))
        agree += sum(a == b for a, b in zip(ids[:n], r.out_ids[:n])) / max(1, n)
    assert agree / len(reqs) > 0.5
