"""Tensor-parallel Brain replica (Llama-3-70B TP=8 over xGMI; SURVEY.md §2.5 TP, §2.4 C1-C5).

One process per GPU of the TP group.  Every rank runs the SAME Engine (its weight shards, its KV-head shard) and the
SAME scheduler, in lockstep:

* the leader (TP rank 0) owns the request queue; once per step it broadcasts the requests that arrived since the
  previous step (C5 — a few hundred bytes over a host-side gloo group, never through the GPU stream);
* every rank submits them in the same order, so admission, KV block allocation, slot assignment and prefill packing
  are identical by construction;
* logits are all-gathered (vocab-parallel LM head), so the fused constrained sampler computes the same tokens and
  advances the same device state on every rank — no token broadcast, and the decode burst stays one captured graph
  per rank with the RCCL all-reduces inside it;
* finished requests are reported by the leader; followers just retire them;
* cancellations and request deadlines are decided by the leader alone and broadcast as (tag, reason) with the
  step's submissions — a rank-local clock check would let ranks drop different requests and fall out of lockstep.
"""
from __future__ import annotations

import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Optional

import torch.distributed as dist

from ..brain.engine.engine import Engine, EngineConfig, Request
from .tp import TPContext


@dataclass
class _Sub:
    ids: list
    fmt: Any = None
    num_predict: Optional[int] = None
    temperature: float = 0.0
    seed: int = 0
    tag: int = 0
    top_k: int = 0
    top_p: float = 1.0
    max_len: Optional[int] = None


@dataclass
class _Msg:
    subs: list = field(default_factory=list)
    cancels: list = field(default_factory=list)  # (tag, reason)
    stop: bool = False


class TPEngine:
    """Lockstep replicated scheduler over a TP group — or, with ``cp``, over a context-parallel group of full-weight
    ranks (parallel/context_parallel.py); the control plane is the same."""

    def __init__(self, cfg: EngineConfig, tp: TPContext, ctrl_group=None, cp: TPContext | None = None, model=None):
        """``model``: a prebuilt (already sharded) model for this rank instead of ``cfg.model`` (tests: fp32 weights)."""
        from dataclasses import replace

        self.tp = tp if cp is None else cp  # the lockstep group
        self.ctrl = ctrl_group  # gloo group spanning the lockstep ranks (host-side control plane)
        self.timeout_s = cfg.request_timeout_s  # enforced by the leader only (module docstring)
        if cp is None:
            self.engine = Engine(replace(cfg, request_timeout_s=0.0), tp=tp, model=model)
        else:
            self.engine = Engine(replace(cfg, request_timeout_s=0.0), cp=cp, model=model)
        self.leader = self.tp.rank == 0
        self._inbox: "queue.Queue[_Sub]" = queue.Queue()
        self._cancel_inbox: "queue.Queue[tuple[int, str]]" = queue.Queue()
        self._callbacks: dict[int, Callable[[Request], None]] = {}
        self._reqs: dict[int, Request] = {}  # tag -> live request (every rank)
        self._tag = 0
        self._lock = threading.Lock()

    # ---- leader API ----------------------------------------------------------------------------------------------
    def submit(self, prompt, fmt=None, num_predict: int | None = None, temperature: float = 0.0, seed: int = 0,
               callback: Callable[[Request], None] | None = None, top_k: int = 0, top_p: float = 1.0,
               max_len: int | None = None) -> int:
        assert self.leader, "requests enter through TP rank 0"
        ids = prompt if isinstance(prompt, list) else self.engine.tok.chat_ids(prompt)
        with self._lock:
            self._tag += 1
            tag = self._tag
            if callback is not None:
                self._callbacks[tag] = callback
        self._inbox.put(_Sub(ids, fmt, num_predict, temperature, seed, tag, top_k, top_p, max_len))
        return tag

    def cancel(self, tag: int, reason: str = "cancelled") -> None:
        assert self.leader, "cancellations enter through TP rank 0"
        self._cancel_inbox.put((tag, reason))

    def drop_callbacks(self) -> None:
        """Leader, after a failed step: requests still in the inbox never reached an engine; answer them with an
        error through their callbacks and forget every live request."""
        while True:
            try:
                s = self._inbox.get_nowait()
            except queue.Empty:
                break
            cb = self._callbacks.pop(s.tag, None)
            if cb is not None:
                r = Request(-1, list(s.ids), s.fmt, 0)
                r.done_reason, r.error = "error", "lockstep step failed"
                r.meta["internal_error"] = True
                cb(r)
        self._reqs.clear()

    def _exchange(self, stop: bool = False) -> _Msg:
        msg = _Msg()
        if self.leader:
            while True:
                try:
                    msg.subs.append(self._inbox.get_nowait())
                except queue.Empty:
                    break
            while True:
                try:
                    msg.cancels.append(self._cancel_inbox.get_nowait())
                except queue.Empty:
                    break
            if self.timeout_s > 0:
                dl = time.perf_counter() - self.timeout_s
                msg.cancels += [(t, "timeout") for t, r in self._reqs.items() if r.t_submit < dl]
            msg.stop = stop
        if self.tp.world > 1:
            box = [msg]
            dist.broadcast_object_list(box, src=dist.get_global_rank(self.ctrl, 0) if self.ctrl else 0,
                                       group=self.ctrl)
            msg = box[0]
        return msg

    def step(self, stop: bool = False) -> tuple[list[Request], bool]:
        """One lockstep iteration on every rank.  Returns (finished requests, stop flag)."""
        msg = self._exchange(stop)
        for s in msg.subs:
            cb = self._callbacks.pop(s.tag, None) if self.leader else None
            r = self.engine.submit(s.ids, fmt=s.fmt, num_predict=s.num_predict, temperature=s.temperature,
                                   seed=s.seed, callback=cb, meta={"tag": s.tag}, top_k=s.top_k, top_p=s.top_p,
                                   max_len=s.max_len)
            if not r.done_reason:
                self._reqs[s.tag] = r
        for tag, reason in msg.cancels:
            r = self._reqs.get(tag)
            if r is not None:
                self.engine.cancel(r, reason)
        done = self.engine.step() if self.engine.has_work() else []
        for r in done:
            self._reqs.pop(r.meta.get("tag"), None)
        return done, msg.stop

    def run_until_idle(self) -> list[Request]:
        """Leader: drive all ranks until every submitted request finished, then tell followers to stop serving."""
        out = []
        while True:
            pending = self.engine.has_work() or not self._inbox.empty()
            done, _ = self.step(stop=not pending)
            out += done
            if not pending:
                return out

    def follower_loop(self) -> None:
        while True:
            _, stop = self.step()
            if stop and not self.engine.has_work():
                return


def init_tp(backend: str = "nccl", ipc_allreduce: bool | None = None) -> tuple[TPContext, Any]:
    """Initialise the default process group (env:// rendezvous) + a gloo control group over the same ranks.  On GPUs
    the decode all-reduces go to the IPC one-shot kernel (K14) unless ``ipc_allreduce=False`` /
    CHRONOS_IPC_ALLREDUCE=0; if the IPC mapping cannot be set up the reason is logged and RCCL carries everything."""
    import logging
    import os

    if not dist.is_initialized():
        dist.init_process_group(backend)
    tp = TPContext.from_group()
    ctrl = dist.new_group(backend="gloo") if backend != "gloo" else None
    if ipc_allreduce is None:
        ipc_allreduce = backend == "nccl" and os.environ.get("CHRONOS_IPC_ALLREDUCE", "1") != "0"
    if ipc_allreduce and tp.world > 1:
        from .custom_ar import PeerAccessUnavailable

        try:  # collective: every rank gets the same outcome (custom_ar.peer_preflight)
            tp.enable_ipc_allreduce()
        except PeerAccessUnavailable as e:  # reported, and RCCL remains a complete implementation
            logging.getLogger("chronos.tp").warning("IPC all-reduce unavailable (%s); using RCCL only", e)
    return tp, ctrl
