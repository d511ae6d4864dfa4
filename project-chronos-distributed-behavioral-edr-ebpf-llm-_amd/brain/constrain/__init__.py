"""Constrained decoding: grammar registry + device-resident token automaton (SURVEY.md §2.1 X6, §7.3 hard part 2).

All grammars live in ONE global state space so a decode batch can mix requests with different ``format`` values
(``"json"``, a JSON schema, or none) in a single sampler launch:

* global state 0 is DONE (every grammar's accepting path ends there through an EOS token);
* each grammar appends its states; a request starts in its grammar's start state;
* the device table ``next[cap, V]`` (int16) and ``dist[cap]`` are preallocated at a fixed capacity, so graphs captured
  against them stay valid when a new schema is registered at run time.

Jump-forward: given the tokenizer's ``encode``, every state from which the grammar forces a byte string (the bytes of
``, "verdict": "`` after a risk score) gets a canonical token run ``jumps[s] = (tokens, end_state)`` and the device
flag ``jump[s]``; the sampler parks a row entering such a state and the engine appends the run in one forward
instead of one decode step per token (Engine._jump).  The run's last token is left to the model (it may merge with
the free text that follows), except when the run ends the verdict: then it is completed through EOS to DONE.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass

import numpy as np
import torch

from . import grammar as G

DONE = 0

# process-wide cache of compiled token automata: (vocabulary fingerprint, grammar key) -> (next, dist, byte DFA).
# Engines in one process (DP replicas on one host, tests) share the ~seconds-long vocab walk per grammar.
_COMPILED: dict = {}
_COMPILED_LOCK = threading.Lock()


@dataclass
class CompiledGrammar:
    key: str
    start: int          # global start state
    num_states: int
    dfa: G.ByteDFA | None


class GrammarBank:
    def __init__(self, token_bytes: list[bytes], stop_ids: tuple[int, ...], vocab: int, capacity: int = 2048,
                 device="cpu", max_string: int = 160, json_depth: int = 3, max_ws: int = 1, encode=None,
                 jump_min: int = 2):
        self.token_bytes = token_bytes
        self.stop_ids = tuple(stop_ids)
        self.vocab = vocab
        self.capacity = capacity
        self.device = torch.device(device)
        self.max_string, self.json_depth, self.max_ws = max_string, json_depth, max_ws
        self.next = torch.full((capacity, vocab), -1, dtype=torch.int16, device=self.device)
        self.dist = torch.full((capacity,), 32767, dtype=torch.int16, device=self.device)
        self.dist[DONE] = 0
        self.encode, self.jump_min = encode, jump_min
        self.jump = torch.zeros((capacity,), dtype=torch.int16, device=self.device)  # budget a jump needs, 0 = none
        self.jumps: dict[int, tuple[tuple[int, ...], int]] = {}  # global state -> (forced tokens, state after them)
        self.used = 1
        self._host_dist: list[int] = [0]
        self._by_key: dict[str, CompiledGrammar] = {}
        self._last = None  # (format object, its grammar): identity hit for a repeated schema object (never mutated)
        self._lock = threading.Lock()
        sample = b"\x00".join(token_bytes[:: max(1, len(token_bytes) // 4096)])
        self._fp = (vocab, len(token_bytes), self.stop_ids, max_string, json_depth, max_ws, hash(sample))
        self._free_start = self._add_free()

    # ---- registration -------------------------------------------------------------------------------------------
    def _append(self, nxt: np.ndarray, dist: np.ndarray) -> int:
        """nxt/dist use local ids with the local DONE = last row; returns the global id of local state 0."""
        n = nxt.shape[0] - 1  # drop the local DONE row
        if self.used + n > self.capacity:
            raise RuntimeError(f"grammar bank full ({self.used}+{n} > {self.capacity} states)")
        base = self.used
        local_done = n
        g = nxt[:n].astype(np.int32)
        g = np.where(g < 0, -1, np.where(g == local_done, DONE, g + base)).astype(np.int16)
        self.next[base:base + n] = torch.from_numpy(g).to(self.device)
        self.dist[base:base + n] = torch.from_numpy(dist[:n].astype(np.int16)).to(self.device)
        self._host_dist += [int(x) for x in dist[:n]]
        self.used += n
        return base

    def _add_free(self) -> int:
        """Unconstrained text: one state, every non-special token loops, a stop token ends."""
        row = np.array([0 if b else -1 for b in self.token_bytes[: self.vocab]] + [-1] * max(0, self.vocab - len(self.token_bytes)),
                       dtype=np.int16)
        for s in self.stop_ids:
            if s < self.vocab:
                row[s] = 1
        nxt = np.stack([row, np.full(self.vocab, -1, np.int16)])
        dist = np.array([1, 0], dtype=np.int16)
        cg = CompiledGrammar("null", self._append(nxt, dist), 1, None)
        self._by_key["null"] = cg
        return cg.start

    def get(self, fmt) -> CompiledGrammar:
        # a wave submits the same schema object for every chain: skip its canonical-JSON key (half of submit's cost)
        last = self._last
        if last is not None and last[0] is fmt:
            return last[1]
        cg = self._get(fmt)
        if isinstance(fmt, dict):
            self._last = (fmt, cg)  # the reference keeps the id from being reused by another object
        return cg

    def _get(self, fmt) -> CompiledGrammar:
        key = G.format_key(fmt if fmt not in ("", False) else None)
        with self._lock:
            if key in self._by_key:
                return self._by_key[key]
            with _COMPILED_LOCK:
                hit = _COMPILED.get((self._fp, key))
            if hit is None:
                node = G.grammar_for_format(fmt, self.json_depth, self.max_ws, self.max_string)
                dfa = G.compile_dfa(node)
                from ...native import constrain_lib

                lib = constrain_lib()
                toks = list(self.token_bytes[: self.vocab]) + [b""] * max(0, self.vocab - len(self.token_bytes))
                nxt, dist, _live = lib.compile_token_dfa(dfa.trans, dfa.accept, toks, list(self.stop_ids), dfa.start)
                hit = (np.asarray(nxt), np.asarray(dist), dfa)
                with _COMPILED_LOCK:
                    _COMPILED[(self._fp, key)] = hit
            nxt, dist, dfa = hit
            cg = CompiledGrammar(key, self._append(nxt, dist), dfa.num_states, dfa)
            if self.encode is not None:
                self._add_jumps(cg.start, dfa, nxt, dist)
            self._by_key[key] = cg
            return cg

    def _add_jumps(self, base: int, dfa: "G.ByteDFA", nxt: np.ndarray, dist: np.ndarray) -> None:
        S = dfa.num_states  # local DONE = S
        trans = dfa.trans
        live = (trans >= 0) & (dist[np.clip(trans, 0, None)] < 32767)  # bytes that can still reach DONE
        nlive = live.sum(axis=1)
        eos = [e for e in self.stop_ids if 0 <= e < nxt.shape[1]]
        glob = lambda s: DONE if s == S else s + base  # noqa: E731
        flags, needs = [], []
        for q in range(S):
            data, cur = bytearray(), q
            while not dfa.accept[cur] and nlive[cur] == 1 and len(data) < 96:
                b = int(np.flatnonzero(live[cur])[0])
                data.append(b)
                cur = int(trans[cur, b])
            finishing = bool(dfa.accept[cur]) and nlive[cur] == 0
            try:
                toks = self.encode(data.decode("utf-8")) if data else []
            except UnicodeDecodeError:
                continue
            run, st = [], q
            for t in toks:
                ns = int(nxt[st, t]) if 0 <= t < nxt.shape[1] else -1
                if ns < 0:
                    break
                run.append(t)
                st = ns
            if finishing and st == cur and len(run) == len(toks) and eos:
                run.append(eos[0])
                st = S
            elif run:
                run.pop()  # leave the last token to the model: it may merge with what follows
                st = q
                for t in run:
                    st = int(nxt[st, t])
            if st == S or len(run) >= self.jump_min:
                if run:
                    self.jumps[q + base] = (tuple(run), glob(st))
                    flags.append(q + base)
                    needs.append(min(32767, len(run) + self.min_tokens(glob(st))))
        if flags:
            self.jump[torch.tensor(flags, dtype=torch.int64).to(self.device)] = torch.tensor(
                needs, dtype=torch.int16).to(self.device)

    # ---- host-side helpers (tests, CPU engine) -----------------------------------------------------------------
    def step(self, state: int, tok: int) -> int:
        return int(self.next[state, tok])

    def min_tokens(self, state: int) -> int:
        return self._host_dist[state]
