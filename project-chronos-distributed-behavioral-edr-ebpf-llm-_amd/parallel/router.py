"""Data-parallel replica router (SURVEY.md §2.5 "DP / replicas", §2.4 C7).

For Llama-3-8B the best MI355X layout is one full replica per GPU (16 GB of weights next to 270 GB of KV per GPU, no
collectives in steady state).  The router owns N worker processes — one per GPU, each with its own Engine, scheduler
loop and HIP context — and dispatches every request to the replica with the fewest outstanding requests; results
and streamed tokens come back over a multiprocessing queue.  The HTTP layer sees the same async interface as
EngineService.
"""
from __future__ import annotations

import asyncio
import itertools
import multiprocessing as mp
import queue
import threading
import time
from dataclasses import asdict
from types import SimpleNamespace
from typing import AsyncIterator, Optional


def _worker(rank: int, cfg_dict: dict, req_q, res_q, device: str) -> None:
    import torch

    from ..brain.api.protocol import GenerateParams, chat_prompt_ids
    from ..brain.engine.engine import Engine, EngineConfig

    if device == "cuda":
        torch.cuda.set_device(rank)
        cfg_dict = dict(cfg_dict, device=f"cuda:{rank}")
    eng = Engine(EngineConfig(**cfg_dict))
    res_q.put(("ready", rank, None))

    def finish(rid):
        def cb(r):
            res_q.put(("done", rid, dict(text=r.text, error=r.error, prompt_ids=len(r.prompt_ids),
                                         out_ids=len(r.out_ids), done_reason=r.done_reason, t_submit=r.t_submit,
                                         t_admit=r.t_admit, t_first=r.t_first, t_done=r.t_done, rank=rank)))
        return cb

    def tokens(rid):
        return lambda ids: res_q.put(("tok", rid, ids))

    live: dict = {}  # rid -> Request, for cancellations
    stop = False
    while not stop:
        try:
            item = req_q.get(timeout=0.05) if not eng.has_work() else req_q.get_nowait()
        except queue.Empty:
            item = None
        while item is not None:
            if item == "stop":
                stop = True
                break
            if item[0] == "cancel":
                r = live.pop(item[1], None)
                if r is not None and not r.done_reason:
                    eng.cancel(r)
                item = None if req_q.empty() else req_q.get_nowait()
                continue
            rid, pd, stream = item
            p = GenerateParams(**pd)
            ids = chat_prompt_ids(eng.tok, p.messages) if p.messages is not None else \
                eng.tok.chat_ids(p.prompt, system=p.system, raw=p.raw)
            live[rid] = eng.submit(ids, fmt=p.format, num_predict=p.num_predict, temperature=p.temperature,
                                   seed=p.seed, top_k=p.top_k, top_p=p.top_p, callback=finish(rid),
                                   meta={"rid": rid, **({"on_tokens": tokens(rid)} if stream else {})})
            try:
                item = req_q.get_nowait()
            except queue.Empty:
                item = None
        if eng.has_work():
            for r in eng.step():
                live.pop(r.meta.get("rid"), None)


class DPRouter:
    def __init__(self, cfg, replicas: int, device: str | None = None, start_timeout: float = 900.0):
        self.n = replicas
        dev = device or ("cuda" if str(cfg.device).startswith("cuda") else "cpu")
        ctx = mp.get_context("spawn")
        self._res = ctx.Queue()
        self._reqs = [ctx.Queue() for _ in range(replicas)]
        cfgd = asdict(cfg)
        self._procs = [ctx.Process(target=_worker, args=(r, cfgd, self._reqs[r], self._res, dev), daemon=True)
                       for r in range(replicas)]
        for p in self._procs:
            p.start()
        ready = 0
        t0 = time.time()
        while ready < replicas:
            kind, _, _ = self._res.get(timeout=max(1.0, start_timeout - (time.time() - t0)))
            ready += kind == "ready"
        self.outstanding = [0] * replicas
        self._waiters: dict[int, tuple] = {}
        self._rid = itertools.count()
        self._lock = threading.Lock()
        self._reader = threading.Thread(target=self._read, daemon=True)
        self._reader.start()

    def _read(self) -> None:
        while True:
            try:
                kind, rid, val = self._res.get()
            except (EOFError, OSError):
                return
            with self._lock:
                w = self._waiters.get(rid)
                if kind == "done":
                    self._waiters.pop(rid, None)
                    if w is not None:
                        self.outstanding[w[2]] -= 1
            if w is None:
                continue
            loop, sink, _ = w
            loop.call_soon_threadsafe(sink, kind, val)

    def _dispatch(self, params, stream: bool, sink) -> tuple[int, int]:
        loop = asyncio.get_running_loop()
        with self._lock:
            r = min(range(self.n), key=lambda i: self.outstanding[i])
            self.outstanding[r] += 1
            rid = next(self._rid)
            self._waiters[rid] = (loop, sink, r)
        self._reqs[r].put((rid, asdict(params), stream))
        return rid, r

    def _cancel(self, rid: int, r: int) -> None:
        with self._lock:
            if rid not in self._waiters:
                return  # already finished
        self._reqs[r].put(("cancel", rid))

    @staticmethod
    def _result(val: dict) -> SimpleNamespace:
        v = dict(val)
        v["prompt_ids"] = [0] * v["prompt_ids"]
        v["out_ids"] = [0] * v["out_ids"]
        return SimpleNamespace(**v)

    async def generate(self, params):
        fut = asyncio.get_running_loop().create_future()

        def sink(kind, val):
            if kind == "done" and not fut.done():
                fut.set_result(self._result(val))

        rid, r = self._dispatch(params, False, sink)
        try:
            return await fut
        except asyncio.CancelledError:  # HTTP timeout / disconnect: free the replica's slot
            self._cancel(rid, r)
            raise

    async def generate_stream(self, params) -> AsyncIterator[tuple[str, Optional[object]]]:
        aq: asyncio.Queue = asyncio.Queue()
        rid, r = self._dispatch(params, True, lambda kind, val: aq.put_nowait((kind, val)))
        from ..brain.tokenizer import load_tokenizer

        tok = getattr(self, "_tok", None) or load_tokenizer(None)
        self._tok = tok
        finished = False
        try:
            while True:
                kind, val = await aq.get()
                if kind == "tok":
                    text = tok.decode([i for i in val if i not in tok.stop_ids])
                    if text:
                        yield text, None
                else:
                    finished = True
                    yield "", self._result(val)
                    return
        finally:
            if not finished:
                self._cancel(rid, r)

    def health(self) -> tuple[bool, dict]:
        dead = [i for i, p in enumerate(self._procs) if not p.is_alive()]
        return not dead, {"status": "replica down" if dead else "ok", "dead_replicas": dead}

    def info(self) -> dict:
        return {"engines": self.n, "outstanding": list(self.outstanding)}

    def close(self) -> None:
        for q in self._reqs:
            q.put("stop")
        for p in self._procs:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()
