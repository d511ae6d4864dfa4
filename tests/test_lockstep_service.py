"""The HTTP-facing lockstep service of a TP / CP group (brain/api/service.py LockstepService) over gloo, world 2:
requests submitted through the leader's asyncio API come back as valid verdicts (incl. a long prompt that takes the
context-parallel path), the follower stays in lockstep and is released when the leader's service closes."""
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


def _worker(rank, world, port, mode, q):
    import asyncio

    import torch.distributed as dist

    from chronos.brain.api.protocol import GenerateParams
    from chronos.brain.api.service import LockstepService
    from chronos.brain.engine.engine import EngineConfig
    from chronos.parallel.tp import TPContext
    from chronos.parallel.tp_engine import TPEngine
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grp = TPContext.from_group()
    cfg = EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=1024, use_graphs=False,
                       decode_burst=4, max_prefill_tokens=128, cp_min_tokens=64)
    tpe = TPEngine(cfg, grp, None) if mode == "tp" else TPEngine(cfg, TPContext.single(), None, cp=grp)
    if rank != 0:
        tpe.follower_loop()
        q.put((rank, dict(tpe.engine.stats)))
    else:
        svc = LockstepService(tpe, "llama3", idle_s=0.005)
        long_hist = [f"[OPEN] bash -> /var/lib/app/f{i}.dat" for i in range(30)] + ["[EXEC] bash -> curl"]
        prompts = [build_prompt(["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"]),
                   build_prompt(long_hist)]

        async def go():
            ps = [GenerateParams(model="llama3", prompt=p, format=VERDICT_SCHEMA, num_predict=24) for p in prompts]
            reqs = await asyncio.gather(*[svc.generate(p) for p in ps])
            chunks = [c async for c in svc.generate_stream(ps[0])]
            return reqs, chunks

        reqs, chunks = asyncio.run(go())
        svc.close()
        q.put((0, [r.text for r in reqs], chunks[-1][1].text, dict(tpe.engine.stats)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["tp", "cp"])
def test_lockstep_service_world2(mode):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        item = q.get(timeout=600)
        res[item[0]] = item
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, texts, streamed, stats = res[0]
    for t in texts + [streamed]:
        v = json.loads(t)
        assert {"risk_score", "verdict", "reason"} <= set(v)
    assert res[1][1]["completed"] == stats["completed"] == 3  # the follower ran the same requests in lockstep
    if mode == "cp":
        assert stats["cp_prefill_steps"] >= 1


def _fail_worker(rank, world, port, q):
    """Only the leader's engine raises (step 2): the leader must stop stepping and answer errors; the follower must
    not stay blocked in a collective once the leader's process is gone."""
    import asyncio
    import datetime

    import torch.distributed as dist

    from chronos.brain.api.protocol import GenerateParams
    from chronos.brain.api.service import LockstepService
    from chronos.brain.engine.engine import EngineConfig
    from chronos.parallel.tp import TPContext
    from chronos.parallel.tp_engine import TPEngine
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    grp = TPContext.from_group()
    cfg = EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=512, use_graphs=False,
                       decode_burst=4, max_prefill_tokens=128)
    tpe = TPEngine(cfg, grp, None)
    if rank != 0:
        try:
            tpe.follower_loop()
            q.put((1, "returned"))
        except Exception as e:  # noqa: BLE001 — expected: the leader's process left the group
            q.put((1, "raised", type(e).__name__))
        q.close()
        q.join_thread()  # os._exit skips the queue's feeder thread: flush first
        os._exit(0)
    fatal = []
    svc = LockstepService(tpe, "llama3", idle_s=0.005, on_fatal=lambda e: fatal.append(str(e)))
    orig, calls = tpe.engine.step, [0]

    def bad_step():
        # count only steps with work: the scheduler also steps while idle (the followers' heartbeat), and a fault
        # on an idle step would race the first submission
        if tpe.engine.has_work():
            calls[0] += 1
            if calls[0] == 2:
                raise RuntimeError("injected leader-only fault")
        return orig()

    tpe.engine.step = bad_step
    p = GenerateParams(model="llama3", prompt=build_prompt(["[EXEC] sh -> curl", "[OPEN] sh -> /tmp/x"]),
                       format=VERDICT_SCHEMA, num_predict=24)

    async def go():
        r1 = await asyncio.wait_for(svc.generate(p), 120.0)
        r2 = await asyncio.wait_for(svc.generate(p), 30.0)  # after the failure: answered, never left queued
        return r1, r2

    r1, r2 = asyncio.run(go())
    q.put((0, r1.done_reason, r2.done_reason, svc.broken, bool(fatal), calls[0]))
    svc.close()
    q.close()
    q.join_thread()
    os._exit(3)  # what the server's on_fatal hook does: the group restarts in fresh processes


@pytest.mark.slow
def test_lockstep_leader_only_failure_is_fatal_for_the_group():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        item = q.get(timeout=300)
        res[item[0]] = item
    for p in procs:
        p.join(timeout=60)
    _, d1, d2, broken, fatal, calls = res[0]
    assert d1 == "error" and d2 == "error" and broken and fatal
    assert calls == 2  # no step after the failure
    assert res[1][1] == "raised"  # the follower left its pending broadcast instead of hanging
    assert procs[0].exitcode == 3
