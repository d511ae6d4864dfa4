"""Data-parallel replica router (SURVEY.md §2.5 "DP / replicas", §2.4 C7).

For Llama-3-8B the best MI355X layout is one full replica per GPU (16 GB of weights next to 270 GB of KV per GPU, no
collectives in steady state).  The router owns N worker processes — one per GPU, each with its own Engine, scheduler
loop and HIP context — and dispatches every request to the replica with the fewest outstanding requests; results
and streamed tokens come back over a multiprocessing queue.  The HTTP layer sees the same async interface as
EngineService.

Failover: a supervisor thread watches every worker process.  When one exits (a crash, an OOM kill,
a GPU fault that took the process down), its in-flight requests are answered at once with an error reply — the
reference's ERROR verdict path (chronos_sensor.py:121-122) instead of a hang until the client's timeout — the replica
leaves the routing set, and a FRESH worker process is spawned in its place (never an exec of a process that touched
the GPU); it rejoins routing when its engine reports ready.  ``/healthz`` shows the transition: "degraded" (503 only
while no replica is serving) with the dead / restarting replicas and the restart counts.

Respawns are bounded: a worker that dies before reporting ready (OOM at model build, a GPU that fails to initialise)
is a start-up failure; consecutive ones are respawned after an exponential delay (``respawn_base_s`` doubling, capped
at ``respawn_cap_s``).  After ``max_start_failures`` in a row the replica is marked failed (``failed_replicas`` in
``/healthz``) and from then on retried only every ``failed_retry_s`` (default: ``respawn_cap_s``), so a transient
cause (GPU memory not yet released, a driver hiccup) does not remove it for the router's life while a persistent one
costs one GPU initialisation per interval, not one per poll.  ``reset_replica(r)`` retries a failed replica at once.
A replica that reports ready leaves the failed state; a death after ready resets the count (it had been serving).
"""
from __future__ import annotations

import asyncio
import itertools
import multiprocessing as mp
import os
import queue
import threading
import time
from dataclasses import asdict
from types import SimpleNamespace
from typing import AsyncIterator, Optional


def _worker(rank: int, cfg_dict: dict, req_q, res_q, device: str, fail_start: bool = False, replicas: int = 1) -> None:
    if fail_start:  # fault injection, set only through DPRouter(fault_start_ranks=...): die before ready
        print(f"[chronos router] replica {rank}: injected start-up fault (fault_start_ranks)", flush=True)
        raise SystemExit(7)
    import torch

    from ..brain.api.protocol import GenerateParams, chat_prompt_ids
    from ..brain.engine.engine import Engine, EngineConfig
    from ..utils import freeze_startup_objects

    if device == "cuda":
        torch.cuda.set_device(rank)
        cfg_dict = dict(cfg_dict, device=f"cuda:{rank}")
    else:  # CPU replicas share the host: split its cores instead of each oversubscribing all of them
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // max(1, replicas)))
    eng = Engine(EngineConfig(**cfg_dict))
    freeze_startup_objects()  # the replica process is an entry point of its own
    res_q.put(("ready", rank, None))

    def finish(rid):
        def cb(r):
            res_q.put(("done", rid, dict(text=r.text, error=r.error, prompt_ids=list(r.prompt_ids),
                                         out_ids=list(r.out_ids), done_reason=r.done_reason, t_submit=r.t_submit,
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
            if p.context and p.messages is None:
                ids = list(p.context) + (ids[1:] if ids and ids[0] == eng.tok.bos_id else ids)
            live[rid] = eng.submit(ids, fmt=p.format, num_predict=p.num_predict, temperature=p.temperature,
                                   seed=p.seed, top_k=p.top_k, top_p=p.top_p, callback=finish(rid),
                                   meta={"rid": rid, **({"on_tokens": tokens(rid)} if stream else {})},
                                   max_len=p.num_ctx or None)
            try:
                item = req_q.get_nowait()
            except queue.Empty:
                item = None
        if eng.has_work():
            for r in eng.step():
                live.pop(r.meta.get("rid"), None)


def _deliver(loop, sink, kind, val) -> None:
    """Hand a result to the caller's event loop; a caller whose loop has already closed (it gave up and returned) is
    simply gone — not an error in the reader / supervisor thread."""
    try:
        loop.call_soon_threadsafe(sink, kind, val)
    except RuntimeError:
        if not loop.is_closed():
            raise


class DPRouter:
    def __init__(self, cfg, replicas: int, device: str | None = None, start_timeout: float = 900.0,
                 respawn: bool = True, poll_s: float = 0.1, respawn_base_s: float = 1.0, respawn_cap_s: float = 60.0,
                 max_start_failures: int = 5, failed_retry_s: Optional[float] = None,
                 fault_start_ranks: tuple = ()):
        self.n = replicas
        self._fault_start = set(fault_start_ranks)  # tests: these ranks' workers die before ready
        self._dev = device or ("cuda" if str(cfg.device).startswith("cuda") else "cpu")
        self._ctx = mp.get_context("spawn")
        self._cfgd = asdict(cfg)
        self._res = self._ctx.Queue()
        self._reqs = [self._ctx.Queue() for _ in range(replicas)]
        self._ready_seen = [False] * replicas  # the current process of each replica reported ready
        self._procs = [self._spawn(r) for r in range(replicas)]
        t0 = time.time()
        # every replica ready, or dead before ready (the supervisor then owns its respawn / failure); none ready = error
        while not all(self._ready_seen[r] or not self._procs[r].is_alive() for r in range(replicas)):
            if time.time() - t0 > start_timeout:
                raise TimeoutError(f"replicas not ready after {start_timeout:.0f}s")
            try:
                kind, rank, _ = self._res.get(timeout=0.5)
            except queue.Empty:
                continue
            if kind == "ready":
                self._ready_seen[rank] = True
        if not any(self._ready_seen):
            codes = [p.exitcode for p in self._procs]
            for p in self._procs:
                p.join(timeout=5)
            raise RuntimeError(f"no replica started (exit codes {codes})")
        self.outstanding = [0] * replicas
        self.alive = list(self._ready_seen)  # in the routing set
        self.restarts = [0] * replicas
        self.start_failures = [0] * replicas  # consecutive deaths before ready
        self.failed = [False] * replicas      # given up on: never respawned again
        self._respawn_at: list = [None] * replicas
        self.respawn_base_s, self.respawn_cap_s = respawn_base_s, respawn_cap_s
        self.max_start_failures = max_start_failures
        self.failed_retry_s = respawn_cap_s if failed_retry_s is None else failed_retry_s
        self.failed_requests = 0
        self.respawn = respawn
        self._closing = False
        self._waiters: dict[int, tuple] = {}
        self._rid = itertools.count()
        self._lock = threading.Lock()
        self._reader = threading.Thread(target=self._read, daemon=True)
        self._reader.start()
        self._poll_s = poll_s
        self._handled: list = [None] * replicas  # the dead process each replica's last failover handled
        self._supervisor = threading.Thread(target=self._supervise, daemon=True)
        self._supervisor.start()

    def _spawn(self, r: int):
        self._ready_seen[r] = False
        p = self._ctx.Process(target=_worker, args=(r, self._cfgd, self._reqs[r], self._res, self._dev,
                                                    r in self._fault_start, self.n), daemon=True)
        p.start()
        return p

    def _read(self) -> None:
        while True:
            try:
                kind, rid, val = self._res.get()
            except (EOFError, OSError, ValueError):
                return
            if kind == "ready":  # a respawned replica rejoins the routing set
                with self._lock:
                    self.alive[rid] = True
                    self._ready_seen[rid] = True
                    self.start_failures[rid] = 0
                    self.failed[rid] = False
                continue
            with self._lock:
                w = self._waiters.get(rid)
                if kind == "done":
                    self._waiters.pop(rid, None)
                    if w is not None:
                        self.outstanding[w[2]] -= 1
            if w is None:
                continue
            loop, sink, _ = w
            _deliver(loop, sink, kind, val)

    def _error_result(self, r: int, msg: str) -> dict:
        now = time.perf_counter()
        return dict(text="", error=msg, prompt_ids=0, out_ids=0, done_reason="error", t_submit=now, t_admit=now,
                    t_first=now, t_done=now, rank=r, meta={"internal_error": True})

    def _supervise(self) -> None:
        while not self._closing:
            time.sleep(self._poll_s)
            for r in range(self.n):
                p = self._procs[r]
                if self._closing or p.is_alive():
                    continue
                if self._handled[r] is p:  # this death was already handled: a delayed respawn may be due
                    due = self._respawn_at[r]
                    if due is not None and time.time() >= due and not self._closing:
                        self._respawn_at[r] = None
                        self._reqs[r] = self._ctx.Queue()  # whatever the dead worker left queued was answered
                        self._procs[r] = self._spawn(r)
                        self.restarts[r] += 1
                    continue
                self._handled[r] = p
                if not self._ready_seen[r]:
                    self.start_failures[r] += 1
                with self._lock:
                    self.alive[r] = False
                    lost = [(rid, w) for rid, w in self._waiters.items() if w[2] == r]
                    for rid, _ in lost:
                        del self._waiters[rid]
                    self.outstanding[r] = 0
                    self.failed_requests += len(lost)
                code = p.exitcode
                for _, (loop, sink, _) in lost:  # answer at once: never leave a caller waiting for a dead replica
                    _deliver(loop, sink, "done", self._error_result(r, f"replica {r} exited ({code})"))
                if self.respawn and not self._closing:
                    sf = self.start_failures[r]
                    if sf >= self.max_start_failures:
                        # keeps dying before ready: failed, retried only every failed_retry_s (never a hot loop)
                        self.failed[r] = True
                        delay = self.failed_retry_s
                    else:  # the first respawn after a serving replica died is immediate, start-up failures back off
                        delay = 0.0 if sf == 0 else min(self.respawn_base_s * 2 ** (sf - 1), self.respawn_cap_s)
                    self._respawn_at[r] = time.time() + delay

    def reset_replica(self, r: int) -> None:
        """Admin path: retry a failed replica now (its start-up failure count starts over)."""
        with self._lock:
            self.start_failures[r] = 0
            if self.failed[r] and self._respawn_at[r] is not None:
                self._respawn_at[r] = time.time()

    def _dispatch(self, params, stream: bool, sink) -> tuple[int, int]:
        loop = asyncio.get_running_loop()
        with self._lock:
            live = [i for i in range(self.n) if self.alive[i]]
            rid = next(self._rid)
            if not live:
                r = -1
            else:
                r = min(live, key=lambda i: self.outstanding[i])
                self.outstanding[r] += 1
                self._waiters[rid] = (loop, sink, r)
                # queued under the lock: the supervisor cannot fail this request over and replace the queue in between
                # (the respawned worker would then run a request whose caller already got its error reply)
                self._reqs[r].put((rid, asdict(params), stream))
        if r < 0:  # every replica is down or restarting: the error verdict now, not a hang
            loop.call_soon(sink, "done", self._error_result(-1, "no replica available (restarting)"))
        return rid, r

    def _cancel(self, rid: int, r: int) -> None:
        with self._lock:
            if rid not in self._waiters or r < 0:
                return  # already finished (or failed over)
        self._reqs[r].put(("cancel", rid))

    @staticmethod
    def _result(val: dict) -> SimpleNamespace:
        v = dict(val)
        for key in ("prompt_ids", "out_ids"):
            if isinstance(v[key], int):
                v[key] = [0] * v[key]
        return SimpleNamespace(**v)

    @property
    def tok(self):
        if getattr(self, "_tok", None) is None:
            from ..brain.tokenizer import load_tokenizer

            # the replicas' own tokenizer (EngineConfig.tokenizer): stop-cut contexts and streamed text must be
            # decoded in the vocabulary the workers produced the ids in
            self._tok = load_tokenizer(self._cfgd.get("tokenizer"))
        return self._tok

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
        tok = self.tok
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
        with self._lock:
            serving = [i for i in range(self.n) if self.alive[i] and self._procs[i].is_alive()]
            dead = [i for i in range(self.n) if not self._procs[i].is_alive()]
            restarting = [i for i in range(self.n) if not self.alive[i] and self._procs[i].is_alive()]
            failed = [i for i in range(self.n) if self.failed[i]]
        status = "ok" if len(serving) == self.n else ("degraded" if serving else "down")
        return bool(serving), {"status": status, "serving_replicas": serving, "dead_replicas": dead,
                               "restarting_replicas": restarting, "failed_replicas": failed,
                               "restarts": list(self.restarts), "start_failures": list(self.start_failures),
                               "failed_retry_s": self.failed_retry_s,
                               "failed_over_requests": self.failed_requests}

    def info(self) -> dict:
        return {"engines": self.n, "outstanding": list(self.outstanding)}

    def close(self) -> None:
        self._closing = True
        for q in self._reqs:
            q.put("stop")
        for p in self._procs:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()
