"""Ollama-compatible HTTP front door of the Brain (reference README.md:57-62 `ollama serve`).

Endpoints:
  POST /api/generate   the sensor contract (chronos_sensor.py:117-120): stream=false -> one JSON object whose
                       ``response`` is the (constrained) model text; stream=true -> NDJSON chunks (Ollama default)
  POST /api/chat       Llama-3 chat template over ``messages``
  GET  /api/tags, POST /api/show, GET /api/ps, GET /api/version, GET /      model listing / health (Ollama shapes)
  GET  /healthz        liveness + engine state;   GET /metrics   Prometheus text (utils/metrics.py)

Run: ``python -m chronos.brain.api --model llama3-8b --port 11434 [--dp N]`` (binds 0.0.0.0 like OLLAMA_HOST=0.0.0.0).
Backends: EngineService (one engine on this process's GPU), DPRouter (one engine process per GPU), FakeBackend
(tests / fault injection).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import threading
import time

from aiohttp import web

from ...utils import freeze_startup_objects
from ...utils.metrics import METRICS
from .protocol import (OLLAMA_VERSION, BadRequest, GenerateParams, StopFilter, apply_stop, chat_response,
                       stop_context_ids,
                       final_fields, generate_response, now_iso)

log = logging.getLogger("chronos.api")


def make_app(backend, model_name: str = "llama3", request_timeout: float | None = None) -> web.Application:
    app = web.Application(client_max_size=64 * 2**20)
    started = time.time()

    async def _params(request, chat=False) -> GenerateParams:
        try:
            body = await request.json()
        except Exception:
            raise web.HTTPBadRequest(text=json.dumps({"error": "invalid JSON body"}), content_type="application/json")
        try:
            return GenerateParams.parse(body, chat=chat)
        except (BadRequest, ValueError, TypeError) as e:
            raise web.HTTPBadRequest(text=json.dumps({"error": str(e)}), content_type="application/json")

    async def _run(params, chat: bool, request):
        model = params.model or model_name
        if not params.stream:
            try:
                coro = backend.generate(params)
                req = await (asyncio.wait_for(coro, request_timeout) if request_timeout else coro)
            except asyncio.TimeoutError:
                return web.json_response({"error": "generation timed out"}, status=504)
            if getattr(req, "error", None):
                # a request the engine rejected is the client's fault (400); a failed engine step is ours (500)
                internal = (getattr(req, "meta", None) or {}).get("internal_error", False)
                return web.json_response({"error": req.error}, status=500 if internal else 400)
            ctx = None
            if params.stop:  # checked on the finished text: cut at the first stop string, reason "stop"
                req.text, hit = apply_stop(req.text, params.stop)
                if hit:
                    req.done_reason = "stop"
                    tok = getattr(backend, "tok", None)
                    if tok is not None and not chat:
                        ctx = stop_context_ids(tok, req.prompt_ids, req.out_ids, req.text)
            if chat:
                return web.json_response(chat_response(model, req))
            body = generate_response(model, req, params.ignored)
            if ctx is not None:
                body["context"] = ctx
            return web.json_response(body)
        resp = web.StreamResponse(headers={"Content-Type": "application/x-ndjson"})
        await resp.prepare(request)
        sf = StopFilter(params.stop) if params.stop else None

        def piece(text: str, done: bool = False) -> dict:
            chunk = {"model": model, "created_at": now_iso()}
            if chat:
                chunk["message"] = {"role": "assistant", "content": text}
            else:
                chunk["response"] = text
            chunk["done"] = done
            return chunk

        gen = backend.generate_stream(params)
        async for text, final in gen:
            if sf is not None:
                text = sf.feed(text) if final is None else sf.flush()
                if final is not None and text:
                    await resp.write((json.dumps(piece(text)) + "\n").encode())
                    text = ""
                if final is None and sf.hit:
                    # stop string seen: emit what precedes it, end the reply, and close the generator, which
                    # cancels the engine request (its slot and KV blocks are freed at the next step)
                    if text:
                        await resp.write((json.dumps(piece(text)) + "\n").encode())
                    await gen.aclose()
                    await resp.write((json.dumps(dict(piece("", True), done_reason="stop")) + "\n").encode())
                    break
            if final is None:
                if not text:
                    continue
                chunk = piece(text)
            else:
                if getattr(final, "error", None):
                    chunk = {"error": final.error}
                else:
                    chunk = {"model": model, "created_at": now_iso()}
                    if chat:
                        chunk["message"] = {"role": "assistant", "content": ""}
                    else:
                        chunk["response"] = ""
                        chunk["context"] = [int(t) for t in list(final.prompt_ids) + list(final.out_ids)]
                    chunk.update(final_fields(final))
            await resp.write((json.dumps(chunk) + "\n").encode())
        await resp.write_eof()
        return resp

    async def generate(request):
        return await _run(await _params(request), False, request)

    async def chat(request):
        return await _run(await _params(request, chat=True), True, request)

    def _model_entry():
        info = backend.info() if hasattr(backend, "info") else {}
        return {"name": f"{model_name}:latest", "model": f"{model_name}:latest", "modified_at": now_iso(),
                "size": int(info.get("params", 0)) * 2, "digest": "chronos-random-init",
                "details": {"format": "safetensors", "family": "llama", "families": ["llama"],
                            "parameter_size": f"{info.get('params', 0) / 1e9:.1f}B", "quantization_level": "BF16"}}

    async def tags(request):
        return web.json_response({"models": [_model_entry()]})

    async def ps(request):
        e = _model_entry()
        e["expires_at"] = "2999-01-01T00:00:00Z"  # weights stay resident (no keep_alive unload, quirk X8)
        e["size_vram"] = e["size"]
        return web.json_response({"models": [e]})

    async def show(request):
        info = backend.info() if hasattr(backend, "info") else {}
        return web.json_response({"modelfile": "", "parameters": "", "template": "llama3",
                                  "details": _model_entry()["details"], "model_info": info})

    async def version(request):
        return web.json_response({"version": OLLAMA_VERSION})

    async def root(request):
        return web.Response(text="Ollama is running")

    async def healthz(request):
        info = backend.info() if hasattr(backend, "info") else {}
        ok, health = backend.health() if hasattr(backend, "health") else (True, {"status": "ok"})
        return web.json_response({**health, "uptime_s": time.time() - started, **info}, status=200 if ok else 503)

    async def metrics(request):
        return web.Response(text=METRICS.render(), content_type="text/plain")

    app.add_routes([
        web.post("/api/generate", generate), web.post("/api/chat", chat), web.get("/api/tags", tags),
        web.get("/api/ps", ps), web.post("/api/show", show), web.get("/api/version", version), web.get("/", root),
        web.get("/healthz", healthz), web.get("/metrics", metrics),
    ])
    return app


# ---------------------------------------------------------------------------------------------------------------
# fake backend (contract tests, fault injection: SURVEY.md §4.2 "contract" row, §5.3)
# ---------------------------------------------------------------------------------------------------------------


class FakeBackend:
    """Answers every request with a canned verdict.  ``mode``: "ok", "stall" (sleep ``delay`` s), "raise",
    "badjson" (response text that is not JSON), "error" (engine-level error)."""

    def __init__(self, mode: str = "ok", delay: float = 0.0, verdict: dict | None = None):
        self.mode, self.delay = mode, delay
        self.verdict = verdict or {"risk_score": 8, "verdict": "MALICIOUS", "reason": "curl -> chmod -> exec dropper"}
        self.seen: list[GenerateParams] = []

    def _req(self, params):
        from types import SimpleNamespace

        now = time.perf_counter()
        text = "not json {" if self.mode == "badjson" else json.dumps(self.verdict)
        return SimpleNamespace(text=text, error="engine failure" if self.mode == "error" else None,
                               prompt_ids=[0] * max(1, len(params.prompt) // 4), out_ids=[0] * 20, done_reason="stop",
                               t_submit=now - 0.01, t_admit=now - 0.01, t_first=now - 0.005, t_done=now)

    async def generate(self, params):
        self.seen.append(params)
        if self.mode == "stall":
            await asyncio.sleep(self.delay)
        if self.mode == "raise":
            raise RuntimeError("injected fault")
        return self._req(params)

    async def generate_stream(self, params):
        req = await self.generate(params)
        for i in range(0, len(req.text), 8):
            yield req.text[i:i + 8], None
        yield "", req

    def info(self):
        return {"engines": 0, "model": "fake", "params": 0}


# ---------------------------------------------------------------------------------------------------------------
# CLI
# ---------------------------------------------------------------------------------------------------------------


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="CHRONOS Brain: Ollama-compatible Llama-3 server on MI355X")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=11434)
    ap.add_argument("--model", default="llama3-8b", help="preset (random-init) when --checkpoint is not given")
    ap.add_argument("--checkpoint", default=None, help="HF or Meta Llama-3 checkpoint directory")
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("--served-name", default="llama3")
    ap.add_argument("--dp", type=int, default=1, help="engine replicas, one process per GPU")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree (launch with torchrun --nproc-per-node TP: rank 0 serves HTTP, the "
                         "other ranks follow the lockstep scheduler)")
    ap.add_argument("--sequence-parallel", action="store_true", help="with --tp: sequence-parallel prefill")
    ap.add_argument("--cp", type=int, default=1,
                    help="context-parallel degree for long kill-chain prefill (torchrun launch, full weights per rank)")
    ap.add_argument("--max-slots", type=int, default=512)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--fake", choices=["ok", "stall", "raise", "badjson"], default=None)
    ap.add_argument("--jsonl", default=None, help="append per-request records here")
    ap.add_argument("--request-timeout", type=float, default=0.0,
                    help="seconds; a slower generation answers 504 and is cancelled in the engine (0 = none)")
    ap.add_argument("--kv-dtype", choices=["bf16", "fp8"], default="bf16")
    ap.add_argument("--roctx", action="store_true", help="emit roctx ranges for rocprofv3 --marker-trace")
    a = ap.parse_args(argv)
    if a.roctx:
        from ...utils import trace

        trace.enable()
    logging.basicConfig(level=logging.INFO)
    METRICS.jsonl_path = a.jsonl
    if a.fake:
        backend = FakeBackend(a.fake, delay=60.0)
    else:
        from ..engine.engine import EngineConfig

        cfg = EngineConfig(model=a.model, checkpoint=a.checkpoint, tokenizer=a.tokenizer, device=a.device,
                           max_slots=a.max_slots, max_model_len=a.max_model_len, kv_dtype=a.kv_dtype,
                           request_timeout_s=a.request_timeout, tp_sequence_parallel=a.sequence_parallel)
        if a.tp > 1 or a.cp > 1:
            if a.tp > 1 and a.cp > 1:
                raise SystemExit("--tp and --cp are exclusive (CP ranks hold full weights)")
            from ...parallel.tp import TPContext
            from ...parallel.tp_engine import TPEngine, init_tp
            from .service import LockstepService

            if a.device == "cuda":  # before the process group: RCCL and the IPC all-reduce bind the current device
                import torch

                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
            grp, ctrl = init_tp("nccl" if a.device == "cuda" else "gloo", ipc_allreduce=None if a.tp > 1 else False)
            want = a.tp if a.tp > 1 else a.cp
            if grp.world != want:
                raise SystemExit(f"world size {grp.world} != {'--tp' if a.tp > 1 else '--cp'} {want}")
            tpe = TPEngine(cfg, grp, ctrl) if a.tp > 1 else TPEngine(cfg, TPContext.single(), ctrl, cp=grp)
            if grp.rank != 0:
                freeze_startup_objects()
                tpe.follower_loop()  # until the leader shuts down
                return 0
            def fatal(e):  # the group is out of lockstep: exit non-zero so the supervisor restarts every rank
                log.error("lockstep group failed (%s); exiting so the group restarts", e)
                threading.Timer(2.0, lambda: os._exit(3)).start()  # let /healthz answer 503 meanwhile

            backend = LockstepService(tpe, a.served_name, on_fatal=fatal)
        elif a.dp > 1:
            from ...parallel.router import DPRouter

            backend = DPRouter(cfg, a.dp)
        else:
            from .service import EngineService

            backend = EngineService.from_config(cfg, a.served_name)
    freeze_startup_objects()  # after the engine is built: no full-GC walks over start-up objects
    app = make_app(backend, a.served_name, a.request_timeout or None)
    web.run_app(app, host=a.host, port=a.port, access_log=None)
    return 0
