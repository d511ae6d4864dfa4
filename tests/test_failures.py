"""Failure detection / recovery: engine-level cancellation and request deadlines free slots and KV
blocks wherever the request is; the service watchdog flags a stalled step and /healthz reports it; a server-side
timeout cancels the engine request."""
import threading
import time

import pytest
import requests

from test_api import Server


def _engine(**kw):
    from chronos.brain.engine.engine import Engine, EngineConfig

    cfg = dict(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False, decode_burst=2,
               max_prefill_tokens=64)
    cfg.update(kw)
    return Engine(EngineConfig(**cfg))


def _prompt(i):
    from chronos.sensor.prompt import build_prompt

    return build_prompt([f"[OPEN] app{i} -> /tmp/f{i}.bin", f"[EXEC] app{i} -> curl", f"[EXEC] app{i} -> chmod"])


def test_cancel_everywhere_frees_resources():
    from chronos.sensor.prompt import VERDICT_SCHEMA

    eng = _engine()
    free0 = eng.blocks.free
    reqs = [eng.submit(_prompt(i), fmt=VERDICT_SCHEMA, num_predict=40) for i in range(6)]
    eng.step()  # admits up to the prefill budget: some prefilling, the rest waiting
    assert eng.prefilling and eng.waiting
    eng.cancel(reqs[0])   # prefilling: finishes its prefill first, then dropped
    eng.cancel(reqs[-1])  # waiting
    while not eng.running:
        eng.step()
    running = next(iter(eng.running.values()))
    eng.cancel(running)   # decoding
    eng.run_until_idle()
    assert reqs[0].done_reason == "cancelled" and reqs[-1].done_reason == "cancelled"
    assert running.done_reason == "cancelled" and running.error
    others = [r for r in reqs if r not in (reqs[0], reqs[-1], running)]
    assert all(r.done_reason in ("stop", "length") for r in others)
    assert eng.blocks.free == free0 and len(eng.free_slots) == 4 and not eng.running
    # the engine keeps serving normally afterwards
    r = eng.submit(_prompt(9), fmt=VERDICT_SCHEMA, num_predict=40)
    eng.run_until_idle()
    assert r.done_reason in ("stop", "length")


def test_request_deadline():
    from chronos.sensor.prompt import VERDICT_SCHEMA

    eng = _engine(request_timeout_s=0.05)
    r = eng.submit(_prompt(1), fmt=VERDICT_SCHEMA, num_predict=40)
    time.sleep(0.1)
    eng.run_until_idle()
    assert r.done_reason == "timeout" and eng.stats["timeout"] == 1 and len(eng.free_slots) == 4


class _SlowEngine:
    """Stands in for an Engine whose step hangs (a stuck kernel / collective)."""

    def __init__(self, hang):
        self.hang, self.stats, self.tok = hang, {}, None
        self.waiting, self.running = [1], {}

    def has_work(self):
        return True

    def step(self):
        self.hang.wait(30)
        raise RuntimeError("device lost")  # the step fails after the hang: health keeps reporting it

    def fail_all(self, error):
        self.waiting = []
        return []


def test_watchdog_flags_stalled_step_and_healthz_503():
    from chronos.brain.api.service import EngineService

    hang = threading.Event()
    svc = EngineService(_SlowEngine(hang), step_deadline_s=0.3)
    svc.info = lambda: {}
    s = Server(svc)
    try:
        t0 = time.time()
        while not svc.stalled and time.time() - t0 < 10:
            time.sleep(0.05)
        r = requests.get(f"{s.url}/healthz", timeout=10)
        assert r.status_code == 503 and r.json()["status"] == "stalled"
    finally:
        hang.set()
        s.close()
        svc.close()


def test_server_timeout_cancels_engine_request():
    from chronos.brain.api.service import EngineService
    from chronos.brain.engine.engine import EngineConfig

    svc = EngineService.from_config(EngineConfig(model="tiny", device="cpu", max_slots=2, max_model_len=384,
                                                 use_graphs=False, decode_burst=1))
    s = Server(svc, request_timeout=0.001)
    try:
        r = requests.post(f"{s.url}/api/generate", json={"prompt": "hello", "stream": False,
                                                         "options": {"num_predict": 200}}, timeout=60)
        assert r.status_code == 504
        t0 = time.time()
        while svc.engine.stats.get("cancelled", 0) == 0 and time.time() - t0 < 30:
            time.sleep(0.05)
        assert svc.engine.stats["cancelled"] == 1
        t0 = time.time()
        while svc.engine.has_work() and time.time() - t0 < 30:
            time.sleep(0.05)
        assert len(svc.engine.free_slots) == 2
        assert requests.get(f"{s.url}/healthz", timeout=10).status_code == 200
    finally:
        s.close()
        svc.close()


def test_roctx_ranges_are_noops_without_profiler():
    from chronos.utils import trace

    avail = trace.enable(True)
    with trace.range("unit-test"):
        trace.mark("inside")
    trace.enable(False)
    assert isinstance(avail, bool)


class _FaultyEngine:
    """A real CPU engine whose step raises while requests are queued / prefilling / decoding (a device fault)."""

    def __init__(self, fail_after: int):
        self.inner = _engine()
        self.fail_after = fail_after
        self.steps = 0

    def __getattr__(self, k):
        return getattr(self.inner, k)

    def step(self):
        self.steps += 1
        if self.steps > self.fail_after:
            raise RuntimeError("HIP error: device lost")
        return self.inner.step()


@pytest.mark.parametrize("fail_after", [0, 1, 3])
def test_step_exception_fails_inflight_requests_with_error(fail_after):
    """a raising step must answer every waiting / prefilling / running request with an error
    (HTTP 500), not leave them hanging while the scheduler hot-loops on the same exception."""
    from chronos.brain.api.service import EngineService

    eng = _FaultyEngine(fail_after)
    svc = EngineService(eng, step_deadline_s=60)
    s = Server(svc)
    try:
        import concurrent.futures as cf

        def post(i):
            return requests.post(f"{s.url}/api/generate", json={"prompt": _prompt(i), "stream": False,
                                                                 "format": "json",
                                                                 "options": {"num_predict": 40}}, timeout=60)

        with cf.ThreadPoolExecutor(6) as ex:
            rs = list(ex.map(post, range(6)))
        assert all(r.status_code in (200, 500) for r in rs)
        errs = [r for r in rs if r.status_code == 500]
        assert errs and all("device lost" in r.json()["error"] for r in errs)
        assert svc.stalled and svc.failures >= 1
        assert requests.get(f"{s.url}/healthz", timeout=10).status_code == 503
        # no hot loop: with nothing in flight the scheduler stops stepping
        n = eng.steps
        time.sleep(0.3)
        assert eng.steps == n
        # the engine state was reset: all slots free, nothing queued
        assert not eng.inner.has_work() and len(eng.inner.free_slots) == 4
    finally:
        s.close()
        svc.close()
