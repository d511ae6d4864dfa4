"""Sensor <-> Brain REST contract tests (SURVEY.md §4.2 "contract" row, App. A).

A real aiohttp server on 127.0.0.1 is driven by the sensor's own clients (chronos.sensor.client), so the bytes on the
wire are exactly what the reference sends (chronos_sensor.py:117-119) and reads (:120).
"""
import asyncio
import json
import socket
import threading
import time

import pytest
import requests

from chronos.brain.api.server import FakeBackend, make_app


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Server:
    def __init__(self, backend, **kw):
        from aiohttp import web

        self.port = _port()
        self.loop = asyncio.new_event_loop()
        self.backend = backend
        app = make_app(backend, **kw)
        self.runner = web.AppRunner(app)
        ready = threading.Event()

        def run():
            asyncio.set_event_loop(self.loop)
            self.loop.run_until_complete(self.runner.setup())
            site = web.TCPSite(self.runner, "127.0.0.1", self.port)
            self.loop.run_until_complete(site.start())
            ready.set()
            self.loop.run_forever()

        self.t = threading.Thread(target=run, daemon=True)
        self.t.start()
        ready.wait(10)
        self.url = f"http://127.0.0.1:{self.port}"

    def close(self):
        async def stop():
            await self.runner.cleanup()

        asyncio.run_coroutine_threadsafe(stop(), self.loop).result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(5)


@pytest.fixture
def fake():
    s = Server(FakeBackend("ok"))
    yield s
    s.close()


def test_reference_request_roundtrip(fake):
    """The exact reference call: requests.post(json={...,"stream": False,"format":"json"}) -> json.loads(response)."""
    from chronos.sensor.prompt import build_prompt

    prompt = build_prompt(["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"])
    resp = requests.post(f"{fake.url}/api/generate",
                         json={"model": "llama3", "prompt": prompt, "stream": False, "format": "json"}, timeout=30)
    body = resp.json()
    verdict = json.loads(body["response"])
    assert verdict["verdict"] == "MALICIOUS" and verdict["risk_score"] == 8
    for k in ("model", "created_at", "done", "done_reason", "total_duration", "prompt_eval_count", "eval_count",
              "eval_duration"):
        assert k in body
    seen = fake.backend.seen[-1]
    assert seen.prompt == prompt and seen.format == "json" and seen.stream is False


def test_sensor_clients_against_server(fake):
    from chronos.sensor.client import AsyncBrainClient, BrainClient, ClientConfig

    cfg = ClientConfig(url=f"{fake.url}/api/generate")
    v = BrainClient(cfg).analyze(["[EXEC] bash -> curl", "[OPEN] curl -> /tmp/x"])
    assert v["verdict"] == "MALICIOUS"

    async def many():
        c = AsyncBrainClient(cfg, max_inflight=16)
        out = await asyncio.gather(*[c.analyze([f"[EXEC] bash -> cat{i}", "[OPEN] cat -> /etc/passwd"])
                                     for i in range(40)])
        await c.close()
        return out

    out = asyncio.run(many())
    assert len(out) == 40 and all(o["verdict"] == "MALICIOUS" for o in out)


def test_streaming_and_endpoints(fake):
    r = requests.post(f"{fake.url}/api/generate", json={"prompt": "x", "format": "json"}, stream=True, timeout=30)
    lines = [json.loads(l) for l in r.iter_lines() if l]
    assert lines[-1]["done"] is True and all(not l["done"] for l in lines[:-1])
    text = "".join(l["response"] for l in lines)
    assert json.loads(text)["verdict"] == "MALICIOUS"
    chat = requests.post(f"{fake.url}/api/chat", json={"messages": [{"role": "user", "content": "hi"}],
                                                       "stream": False}, timeout=30).json()
    assert chat["message"]["role"] == "assistant"
    assert requests.get(f"{fake.url}/api/tags", timeout=5).json()["models"][0]["name"] == "llama3:latest"
    assert "version" in requests.get(f"{fake.url}/api/version", timeout=5).json()
    assert requests.get(f"{fake.url}/", timeout=5).text == "Ollama is running"
    assert requests.get(f"{fake.url}/healthz", timeout=5).json()["status"] == "ok"
    metrics = requests.get(f"{fake.url}/metrics", timeout=5).text
    for name in ("chronos_requests_total", "chronos_queued_requests", "chronos_generated_tokens_per_second",
                 "chronos_preemptions_total 0", "chronos_verdict_latency_seconds_bucket"):
        assert name in metrics
    bad = requests.post(f"{fake.url}/api/generate", json={"prompt": "x", "format": 7}, timeout=5)
    assert bad.status_code == 400
    bad = requests.post(f"{fake.url}/api/generate", data=b"{not json", timeout=5)
    assert bad.status_code == 400


@pytest.mark.parametrize("mode", ["stall", "badjson"])
def test_fault_injection_maps_to_error_verdict(mode):
    """Reference quirk Q2: any failure (timeout, bad JSON) becomes {"risk_score":0,"verdict":"ERROR",...}."""
    from chronos.sensor.client import BrainClient, ClientConfig

    s = Server(FakeBackend(mode, delay=3.0))
    try:
        v = BrainClient(ClientConfig(url=f"{s.url}/api/generate", timeout=1.0)).analyze(["[EXEC] bash -> nc"])
        assert v["verdict"] == "ERROR" and v["risk_score"] == 0 and v["reason"]
    finally:
        s.close()


@pytest.fixture(scope="module")
def tiny_service():
    from chronos.brain.api.service import EngineService
    from chronos.brain.engine.engine import EngineConfig

    svc = EngineService.from_config(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384,
                                                 use_graphs=False, decode_burst=4))
    s = Server(svc)
    yield s
    s.close()
    svc.close()


def test_real_engine_behind_api(tiny_service):
    from chronos.sensor.client import BrainClient, ClientConfig, schema_format

    url = f"{tiny_service.url}/api/generate"
    v = BrainClient(ClientConfig(url=url, fmt=schema_format(), options={"num_predict": 40})).analyze(
        ["[OPEN] attack_chain.sh -> /tmp/malware.bin", "[EXEC] attack_chain.sh -> curl"])
    assert set(v) == {"risk_score", "verdict", "reason"}
    body = requests.post(url, json={"prompt": "hi", "format": "json", "stream": False,
                                    "options": {"num_predict": 16}}, timeout=60).json()
    assert isinstance(json.loads(body["response"]), dict) and body["eval_count"] <= 16
    r = requests.post(url, json={"prompt": "hi", "format": "json", "options": {"num_predict": 16}}, stream=True,
                      timeout=60)
    lines = [json.loads(l) for l in r.iter_lines() if l]
    assert lines[-1]["done"] and isinstance(json.loads("".join(l["response"] for l in lines)), dict)


def test_dp_router_two_replicas():
    from chronos.brain.api.protocol import GenerateParams
    from chronos.brain.engine.engine import EngineConfig
    from chronos.parallel.router import DPRouter
    from chronos.sensor.prompt import VERDICT_SCHEMA

    router = DPRouter(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=384, use_graphs=False,
                                   decode_burst=4), 2)
    try:
        async def go():
            ps = [GenerateParams(prompt=f"chain {i}", stream=False, format=VERDICT_SCHEMA, num_predict=32)
                  for i in range(6)]
            return await asyncio.gather(*[router.generate(p) for p in ps])

        out = asyncio.run(go())
        assert {o.rank for o in out} == {0, 1}
        for o in out:
            assert set(json.loads(o.text)) == {"risk_score", "verdict", "reason"}
    finally:
        router.close()


def test_closed_loop_loadgen_against_fake_brain(fake):
    """scripts/loadgen.py (N8): closed-loop streams against the REST contract; ERROR verdicts are not counted."""
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location(
        "loadgen", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts", "loadgen.py"))
    lg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lg)
    rec = asyncio.run(lg.run_level(f"{fake.url}/api/generate", 8, 1.0, 0.2, True, 32, 0))
    assert rec["chains"] > 8 and rec["errors"] == 0 and rec["p50_latency_ms"] > 0
    bad = asyncio.run(lg.run_level("http://127.0.0.1:9/api/generate", 2, 0.5, 0.0, True, 32, 0))
    assert bad["chains"] == 0 and bad["errors"] > 0


@pytest.mark.slow
def test_dp_router_failover_and_respawn():
    """A replica process dies mid-request: its callers get an error reply within a second (not a hang), later
    requests succeed on the other replica and then on the respawned one, and health reports the transition
    (SURVEY.md §5.3)."""
    import os
    import signal
    import time

    from chronos.brain.api.protocol import GenerateParams
    from chronos.brain.engine.engine import EngineConfig
    from chronos.parallel.router import DPRouter
    from chronos.sensor.prompt import VERDICT_SCHEMA

    router = DPRouter(EngineConfig(model="tiny", device="cpu", max_slots=4, max_model_len=512, use_graphs=False,
                                   decode_burst=4, max_out=480, jump_forward=False), 2, poll_s=0.05)
    try:
        async def go():
            long = GenerateParams(prompt="chain x", stream=False, num_predict=400)  # free text: runs its budget
            tasks = [asyncio.ensure_future(router.generate(long)) for _ in range(4)]
            finished_at = {}
            for i, t in enumerate(tasks):
                t.add_done_callback(lambda _t, i=i: finished_at.setdefault(i, time.perf_counter()))
            await asyncio.sleep(0.5)
            victim = router._procs[0].pid
            t_kill = time.perf_counter()
            os.kill(victim, signal.SIGKILL)
            # the supervisor notices within a poll or two; under a loaded CPU (parallel test workers) allow a few
            # seconds — the fresh worker is still importing / building its engine for far longer than that
            await asyncio.sleep(0.3)
            ok_h, health = router.health()
            t_h = time.perf_counter()
            while health["status"] == "ok" and time.perf_counter() - t_h < 5.0:
                await asyncio.sleep(0.1)
                ok_h, health = router.health()
            done = []
            for t in tasks:
                done.append(await asyncio.wait_for(t, 600))  # the survivor runs 400-token requests on CPU
            failed = [i for i, d in enumerate(done) if d.done_reason == "error"]
            t_err = max(finished_at[i] for i in failed) - t_kill if failed else 99.0
            failed = [done[i] for i in failed]
            # later requests: served while replica 0 restarts, then by both once it is back
            p = GenerateParams(prompt="chain y", stream=False, format=VERDICT_SCHEMA, num_predict=32)
            later = await asyncio.gather(*[router.generate(p) for _ in range(3)])
            t0 = time.perf_counter()
            while not router.health()[0] or router.health()[1]["status"] != "ok":
                await asyncio.sleep(0.2)
                assert time.perf_counter() - t0 < 300
            after = await asyncio.gather(*[router.generate(p) for _ in range(6)])
            return failed, t_err, ok_h, health, later, after

        failed, t_err, ok_h, health, later, after = asyncio.run(go())
        assert failed and all("replica 0" in f.error for f in failed)
        # answered promptly after the kill (poll 50 ms), not at the request's own end: the survivors' 400-token CPU
        # decode takes far longer than this bound; CPU load from parallel test workers adds seconds of jitter
        assert t_err < 4.0
        assert ok_h and health["status"] == "degraded" and 0 not in health["serving_replicas"]
        for o in later + after:
            assert o.done_reason == "stop" and set(json.loads(o.text)) == {"risk_score", "verdict", "reason"}
        assert router.restarts[0] == 1 and 0 in {o.rank for o in after}
    finally:
        router.close()


def test_stop_filter_unit():
    from chronos.brain.api.protocol import StopFilter, apply_stop

    assert apply_stop("abc|STOPxyz", ("|STOP", "zz")) == ("abc", True)
    assert apply_stop("abc", ("q",)) == ("abc", False)
    f = StopFilter(("|STOP",))
    out = "".join(f.feed(c) for c in ["ab", "c|S", "TOPxyz", "more"]) + f.flush()
    assert out == "abc" and f.hit
    f = StopFilter(("END",))
    out = "".join(f.feed(c) for c in ["hello ", "wor", "ld E", "N"]) + f.flush()
    assert out == "hello world EN" and not f.hit


def test_ollama_options_stop_num_ctx_context(tiny_service):
    """options.stop (non-stream and stream), num_ctx (clamp + 400 when the prompt does not fit),
    keep_alive, context continuation and the reported ignored options."""
    from chronos.sensor.prompt import VERDICT_SCHEMA

    url = f"{tiny_service.url}/api/generate"
    base = {"prompt": "chain 1", "format": VERDICT_SCHEMA, "stream": False, "options": {"num_predict": 48}}
    full = requests.post(url, json=base, timeout=60).json()
    assert '"verdict"' in full["response"]
    cut = requests.post(url, json=dict(base, options={"num_predict": 48, "stop": ['"verdict"']}), timeout=60).json()
    assert cut["response"] == full["response"][:full["response"].index('"verdict"')]
    assert cut["done_reason"] == "stop"
    # the continuation context ends where the visible text ends: the stop string and what followed are not in it
    from chronos.brain.tokenizer import load_tokenizer

    tok = load_tokenizer(None)
    gen_ctx = cut["context"][cut["prompt_eval_count"]:]
    assert tok.decode(gen_ctx) == cut["response"]
    assert cut["context"][:cut["prompt_eval_count"]] == full["context"][:full["prompt_eval_count"]]
    r = requests.post(url, json=dict(base, stream=True, options={"num_predict": 48, "stop": '"verdict"'}),
                      stream=True, timeout=60)
    lines = [json.loads(l) for l in r.iter_lines() if l]
    assert lines[-1]["done"] and "".join(l["response"] for l in lines) == cut["response"]

    # num_ctx: a prompt that does not fit is the client's error; one that fits bounds the generation
    n_prompt = full["prompt_eval_count"]
    bad = requests.post(url, json=dict(base, options={"num_ctx": n_prompt - 1}), timeout=60)
    assert bad.status_code == 400 and "num_ctx" in bad.json()["error"]
    free = {"prompt": "chain 2", "stream": False, "options": {"num_predict": 64, "num_ctx": n_prompt + 6}}
    small = requests.post(url, json=free, timeout=60).json()
    assert small["eval_count"] <= n_prompt + 6 - small["prompt_eval_count"]
    assert requests.post(url, json=dict(base, options={"num_ctx": -1}), timeout=60).status_code == 400

    # context: the reply's token ids; sending them back continues the conversation (longer prompt)
    ctx = full["context"]
    assert len(ctx) == full["prompt_eval_count"] + full["eval_count"]
    more = requests.post(url, json=dict(base, context=ctx, keep_alive="5m"), timeout=60).json()
    assert more["prompt_eval_count"] > len(ctx) and set(json.loads(more["response"])) >= {"verdict"}
    assert requests.post(url, json=dict(base, context="nope"), timeout=60).status_code == 400

    ign = requests.post(url, json=dict(base, options={"num_predict": 48, "repeat_penalty": 1.3,
                                                      "presence_penalty": 0.0}), timeout=60).json()
    assert ign["ignored_options"] == ["repeat_penalty"]
