"""DP router supervisor (parallel/router.py): a replica that dies at start-up is respawned with an
exponential delay and, after ``max_start_failures`` consecutive start-up deaths, marked failed and left alone — the
other replica keeps serving and /healthz stays "degraded" (ADVICE r3)."""
import asyncio
import json
import os
import time

import pytest


@pytest.mark.slow
def test_startup_failure_respawns_are_bounded(monkeypatch):
    from chronos.brain.api.protocol import GenerateParams
    from chronos.brain.engine.engine import EngineConfig
    from chronos.parallel.router import DPRouter
    from chronos.sensor.prompt import VERDICT_SCHEMA

    monkeypatch.setenv("CHRONOS_FAULT_START_RANK", "1")  # replica 1's worker dies before it reports ready
    router = DPRouter(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False,
                                   decode_burst=4), 2, poll_s=0.05, respawn_base_s=0.2, respawn_cap_s=0.8,
                      max_start_failures=3)
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
        assert router.restarts[1] == n_restarts  # nothing respawns a failed replica
        ok, h = router.health()
        assert ok and h["status"] == "degraded" and h["failed_replicas"] == [1] and h["serving_replicas"] == [0]
        assert h["start_failures"][1] == 3

        async def go():
            p = GenerateParams(prompt="chain z", stream=False, format=VERDICT_SCHEMA, num_predict=24)
            return await asyncio.gather(*[router.generate(p) for _ in range(3)])

        for o in asyncio.run(go()):  # the survivor serves everything
            assert o.rank == 0 and set(json.loads(o.text)) == {"risk_score", "verdict", "reason"}
    finally:
        router.close()
