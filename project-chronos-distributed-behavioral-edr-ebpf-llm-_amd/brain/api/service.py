"""EngineService: runs one Engine on a dedicated scheduler thread and exposes an asyncio API to the HTTP layer.

Single-owner rule: only the scheduler thread touches the engine and its device state; the HTTP event
loop hands requests over through a queue and gets results back through ``loop.call_soon_threadsafe``.
"""
from __future__ import annotations

import asyncio
import queue
import threading
import time
from typing import Any, AsyncIterator, Optional

from ...utils.metrics import METRICS
from ..engine.engine import Engine, EngineConfig, Request
from .protocol import GenerateParams, chat_prompt_ids


class EngineService:
    def __init__(self, engine: Engine, model_name: str = "llama3"):
        self.engine = engine
        self.model_name = model_name
        self._q: "queue.Queue[tuple]" = queue.Queue()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="chronos-scheduler", daemon=True)
        self.started = time.time()
        self._thread.start()

    @classmethod
    def from_config(cls, cfg: EngineConfig, model_name: str = "llama3") -> "EngineService":
        return cls(Engine(cfg), model_name)

    # ---- scheduler thread ------------------------------------------------------------------------------------
    def _loop(self) -> None:
        eng = self.engine
        while not self._stop.is_set():
            try:
                block = not eng.has_work()
                item = self._q.get(timeout=0.05) if block else self._q.get_nowait()
            except queue.Empty:
                item = None
            while item is not None:
                self._admit(item)
                try:
                    item = self._q.get_nowait()
                except queue.Empty:
                    item = None
            if eng.has_work():
                t = time.perf_counter()
                done = eng.step()
                METRICS.observe_step(time.perf_counter() - t, eng)
                for r in done:
                    METRICS.observe_request(r)

    def _admit(self, item) -> None:
        params, ids, on_done, on_tokens = item
        self.engine.submit(ids, fmt=params.format, num_predict=params.num_predict, temperature=params.temperature,
                           seed=params.seed, top_k=params.top_k, top_p=params.top_p, callback=on_done, meta={"on_tokens": on_tokens} if on_tokens else None)

    def close(self) -> None:
        self._stop.set()
        self._thread.join(timeout=5)

    # ---- asyncio API -------------------------------------------------------------------------------------------
    def _ids(self, params: GenerateParams) -> list:
        tok = self.engine.tok
        if params.messages is not None:
            return chat_prompt_ids(tok, params.messages)
        return tok.chat_ids(params.prompt, system=params.system, raw=params.raw)

    async def generate(self, params: GenerateParams) -> Request:
        loop = asyncio.get_running_loop()
        fut: asyncio.Future = loop.create_future()

        def done(req: Request):
            loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(req))

        self._q.put((params, self._ids(params), done, None))
        return await fut

    async def generate_stream(self, params: GenerateParams) -> AsyncIterator[tuple[str, Optional[Request]]]:
        """Yields (text_delta, None) pieces, then ("", final_request)."""
        loop = asyncio.get_running_loop()
        aq: asyncio.Queue = asyncio.Queue()
        tok = self.engine.tok

        def on_tokens(new_ids: list):
            loop.call_soon_threadsafe(aq.put_nowait, ("tok", new_ids))

        def done(req: Request):
            loop.call_soon_threadsafe(aq.put_nowait, ("done", req))

        self._q.put((params, self._ids(params), done, on_tokens))
        pending = b""
        while True:
            kind, val = await aq.get()
            if kind == "tok":
                ids = [i for i in val if i not in tok.stop_ids]
                pending += b"".join(tok.token_bytes_list()[i] for i in ids)
                # emit only complete UTF-8 sequences
                try:
                    text = pending.decode("utf-8")
                    pending = b""
                except UnicodeDecodeError as e:
                    text = pending[:e.start].decode("utf-8")
                    pending = pending[e.start:]
                if text:
                    yield text, None
            else:
                if pending:
                    yield pending.decode("utf-8", errors="replace"), None
                yield "", val
                return

    def info(self) -> dict[str, Any]:
        eng = self.engine
        return {
            "engines": 1,
            "model": eng.model.cfg.name,
            "params": eng.model.cfg.param_count(),
            "kv_blocks": eng.blocks.num_blocks,
            "kv_free": eng.blocks.free,
            "slots": eng.cfg.max_slots,
            "running": len(eng.running),
            "waiting": len(eng.waiting),
            "stats": dict(eng.stats),
        }
