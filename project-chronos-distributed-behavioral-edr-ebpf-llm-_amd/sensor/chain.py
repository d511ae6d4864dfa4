"""Stateful per-process kill-chain tracker ("short-term memory", reference chronos_sensor.py:105,124-157).

Semantics in compat mode (defaults), event by event:
  1. decode comm/argv/type as strict UTF-8; any error drops the event            (:127-131, quirk Q12)
  2. drop if any COMM_IGNORE word is a substring of comm                        (:133-135, quirk Q6)
  3. s = "[TYPE] comm -> argv"; append to the TGID's chain                     (:137-138)
  4. if any trigger keyword is a substring of s and the chain has >= 2 entries  (:141-142, quirk Q5)
     -> fire (pid, chain) and reset the chain                                   (:157)
Opt-in fixes: ``word_triggers`` (Q5), ``max_chain`` / ``max_pids`` bounded memory (Q4).

Two implementations share one interface: :class:`ChainTracker` (pure Python, the oracle) and
:class:`NativeChainTracker` (C++ ``_sensor_native``; batched record feeding with the GIL released).
"""
from __future__ import annotations

import re
from collections import OrderedDict
from dataclasses import dataclass, field

from . import abi
from .filters import COMM_IGNORE, MIN_CHAIN, TRIGGERS, open_is_noise


@dataclass
class TrackerConfig:
    ignore: tuple[str, ...] = COMM_IGNORE
    triggers: tuple[str, ...] = TRIGGERS
    min_len: int = MIN_CHAIN
    word_triggers: bool = False   # Q5 fix
    max_chain: int = 0            # Q4 fix: keep only the newest N events per PID (0 = unbounded, reference)
    max_pids: int = 0             # Q4 fix: LRU cap on tracked PIDs (0 = unbounded, reference)


@dataclass
class Trigger:
    pid: int
    history: list[str] = field(default_factory=list)


def format_event(etype: str, comm: str, argv: str) -> str:
    return f"[{etype}] {comm} -> {argv}"


class ChainTracker:
    def __init__(self, cfg: TrackerConfig | None = None):
        self.cfg = cfg or TrackerConfig()
        self._chains: OrderedDict[int, list[str]] = OrderedDict()
        self._word = [re.compile(r"(?<![A-Za-z0-9_])" + re.escape(t) + r"(?![A-Za-z0-9_])") for t in self.cfg.triggers]
        self.stats = dict(seen=0, dropped_kernel=0, dropped_decode=0, dropped_ignored=0, fired=0, evicted=0)

    def _hit(self, s: str) -> bool:
        if self.cfg.word_triggers:
            return any(r.search(s) for r in self._word)
        return any(t in s for t in self.cfg.triggers)

    def _chain(self, pid: int) -> list[str]:
        ch = self._chains.get(pid)
        if ch is not None:
            self._chains.move_to_end(pid)
            return ch
        if self.cfg.max_pids and len(self._chains) >= self.cfg.max_pids:
            self._chains.popitem(last=False)
            self.stats["evicted"] += 1
        ch = self._chains[pid] = []
        return ch

    def feed_event(self, pid: int, comm: bytes, argv: bytes, etype: bytes) -> Trigger | None:
        self.stats["seen"] += 1
        try:
            cmd, args, typ = comm.decode("utf-8"), argv.decode("utf-8"), etype.decode("utf-8")
        except UnicodeDecodeError:
            self.stats["dropped_decode"] += 1
            return None
        if any(x in cmd for x in self.cfg.ignore):
            self.stats["dropped_ignored"] += 1
            return None
        s = format_event(typ, cmd, args)
        ch = self._chain(pid)
        ch.append(s)
        if self.cfg.max_chain and len(ch) > self.cfg.max_chain:
            del ch[0]
        if self._hit(s) and len(ch) >= self.cfg.min_len:
            self.stats["fired"] += 1
            hist = list(ch)
            ch.clear()
            return Trigger(pid, hist)
        return None

    def feed_records(self, buf: bytes, kernel_filter: bool = False, strict: bool = False) -> list[Trigger]:
        out = []
        for ev in abi.iter_records(buf):
            if kernel_filter and ev.type == b"OPEN" and open_is_noise(ev.argv, strict):
                self.stats["dropped_kernel"] += 1
                continue
            t = self.feed_event(ev.pid, ev.comm, ev.argv, ev.type)
            if t is not None:
                out.append(t)
        return out

    def evict(self, pid: int) -> None:
        self._chains.pop(pid, None)

    def chain(self, pid: int) -> list[str]:
        return list(self._chains.get(pid, []))

    def num_pids(self) -> int:
        return len(self._chains)


class NativeChainTracker:
    """Same semantics as :class:`ChainTracker`, implemented in C++ (csrc/sensor_host/sensor_host.cpp)."""

    def __init__(self, cfg: TrackerConfig | None = None):
        from ..native import sensor_lib

        self.cfg = cfg or TrackerConfig()
        self._t = sensor_lib().ChainTracker(list(self.cfg.ignore), list(self.cfg.triggers), self.cfg.min_len,
                                            self.cfg.word_triggers, self.cfg.max_chain, self.cfg.max_pids)

    def feed_event(self, pid: int, comm: bytes, argv: bytes, etype: bytes) -> Trigger | None:
        r = self._t.feed_event(pid, comm, argv, etype)
        return None if r is None else Trigger(r[0], list(r[1]))

    def feed_records(self, buf: bytes, kernel_filter: bool = False, strict: bool = False) -> list[Trigger]:
        return [Trigger(p, list(h)) for p, h in self._t.feed_records(buf, kernel_filter, strict)]

    def evict(self, pid: int) -> None:
        self._t.evict(pid)

    def chain(self, pid: int) -> list[str]:
        return list(self._t.chain(pid))

    def num_pids(self) -> int:
        return self._t.num_pids()

    @property
    def stats(self) -> dict:
        return dict(self._t.stats())
