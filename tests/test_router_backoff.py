"""DP router supervisor (parallel/router.py): a replica that dies at start-up is respawned with an
exponential delay and, after ``max_start_failures`` consecutive start-up deaths, marked failed and retried only every
``failed_retry_s`` (or at once through ``reset_replica``) — the other replica keeps serving and /healthz stays
"degraded" (ADVICE r3/r4).  The fault is injected through the constructor, never the environment."""
import asyncio
import json
import os
import time

import pytest


@pytest.mark.slow
def test_startup_failure_respawns_are_bounded():
    from chronos.brain.api.protocol import GenerateParams
    from chronos.brain.engine.engine import EngineConfig
    from chronos.parallel.router import DPRouter
    from chronos.sensor.prompt import VERDICT_SCHEMA

    # replica 1's worker dies before it reports ready
    router = DPRouter(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False,
                                   decode_burst=4), 2, poll_s=0.05, respawn_base_s=0.2, respawn_cap_s=0.8,
                      max_start_failures=3, failed_retry_s=60.0, fault_start_ranks=(1,))
    try:
        t0 = time.time()
        while not router.failed[1]:
            time.sleep(0.1)
            assert time.time() - t0 < 120, router.health()
        elapsed = time.time() - t0
        n_restarts = router.restarts[1]
        assert n_restarts == 2  # 3 start-up deaths: the first two respawned, the third gives up
        assert elapsed >= 0.2 + 0.4 - 0.1  # the respawns waited 0.2 s then 0.4 s (no hot loop)
        time.sleep(1.0)
        assert router.restarts[1] == n_restarts  # a failed replica waits failed_retry_s, not a poll
        ok, h = router.health()
        assert ok and h["status"] == "degraded" and h["failed_replicas"] == [1] and h["serving_replicas"] == [0]
        assert h["start_failures"][1] == 3 and h["failed_retry_s"] == 60.0
        router.reset_replica(1)  # admin retry: respawned at once (and dies again: still the injected fault)
        t1 = time.time()
        while router.restarts[1] == n_restarts:
            time.sleep(0.05)
            assert time.time() - t1 < 30, router.health()

        async def go():
            p = GenerateParams(prompt="chain z", stream=False, format=VERDICT_SCHEMA, num_predict=24)
            return await asyncio.gather(*[router.generate(p) for _ in range(3)])

        for o in asyncio.run(go()):  # the survivor serves everything
            assert o.rank == 0 and set(json.loads(o.text)) == {"risk_score", "verdict", "reason"}
    finally:
        router.close()


@pytest.mark.slow
def test_failed_replica_is_retried_periodically():
    """A failed replica keeps being retried at failed_retry_s (a transient start-up cause must not remove
    it for the router's life)."""
    from chronos.brain.engine.engine import EngineConfig
    from chronos.parallel.router import DPRouter

    router = DPRouter(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False,
                                   decode_burst=4), 2, poll_s=0.05, respawn_base_s=0.1, respawn_cap_s=0.2,
                      max_start_failures=2, failed_retry_s=0.3, fault_start_ranks=(1,))
    try:
        t0 = time.time()
        while not router.failed[1]:
            time.sleep(0.05)
            assert time.time() - t0 < 120, router.health()
        r0 = router.restarts[1]
        t1 = time.time()
        while router.restarts[1] < r0 + 2:  # two more retries at the failed interval
            time.sleep(0.05)
            assert time.time() - t1 < 60, router.health()
        assert time.time() - t1 >= 0.3  # not a hot loop
        assert router.failed[1]
    finally:
        router.close()


def test_router_tokenizer_follows_config(tmp_path):
    """DPRouter.tok must load EngineConfig.tokenizer (the vocabulary the workers decode in), not the
    default — stop-cut contexts and streamed text are decoded with it."""
    from chronos.brain.engine.engine import EngineConfig
    from chronos.parallel.router import DPRouter

    seen = []
    import chronos.brain.tokenizer as tk

    orig = tk.load_tokenizer

    def spy(path=None):
        seen.append(path)
        return orig(None)

    r = DPRouter.__new__(DPRouter)  # no workers: only the tokenizer property is under test
    r._cfgd = {"tokenizer": str(tmp_path / "tokenizer.json")}
    tk.load_tokenizer = spy
    try:
        r.tok
    finally:
        tk.load_tokenizer = orig
    assert seen == [str(tmp_path / "tokenizer.json")]
