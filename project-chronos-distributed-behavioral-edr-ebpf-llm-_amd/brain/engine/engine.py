"""The Brain's serving engine: continuous batching over paged KV with graph-captured, grammar-constrained decode.

Replaces what Ollama + llama.cpp did for the reference:

* **admission**: a request gets a decode *slot* and the KV blocks of its prompt plus ``kv_lookahead`` generated
  tokens (``kv_alloc="lazy"``; ``"full"`` reserves prompt + num_predict up front as rounds 1-4 did; the default
  ``"auto"`` is full when the pool can hold every slot at max_model_len, lazy when it cannot).
  KV is sized from the HBM budget (288 GB per MI355X — 1-2 M tokens for 8B);
* **KV growth and preemption** (SURVEY.md §7.2 step 6): before every launch that writes generated-token KV (decode
  burst, mixed step, jump-forward) each running sequence's blocks are grown to cover the positions that launch can
  write (a host-side upper bound, ``Request.pos_hi``).  When the pool runs dry the NEWEST running sequences are
  preempted by recompute: their exact device state (generated ids, grammar state) is read back, their computed full
  blocks are published to the prefix cache, their blocks and slot are freed, and they go back to the FRONT of the
  queue with the generated ids appended to the prompt, the grammar resuming from the saved state.  A resumed greedy
  request produces the tokens an uninterrupted run would have (the re-prefill computes the pending token's logits
  exactly as the decode step would have);
* **prefill**: waiting prompts are packed into one flattened token stream (chunked to ``max_prefill_tokens``, so a
  128k-token chain context prefills in pieces that attend to the paged prefix);
* **decode**: all slots advance together; the step (32 layers + LM head + the constrained sampler, which also
  advances ids/positions/context/DFA state on device) is captured once per power-of-two slot bucket into a hipGraph
  holding ``decode_burst`` unrolled steps, so one host call runs e.g. 8 verdict tokens for every live stream;
* **harvest**: each decode burst ends with a copy of the slot states into pinned host memory, which the host reads
  to detokenize finished verdicts and free + compact slots (``async_harvest`` reads burst k while burst k+1 runs:
  less host time on the critical path, but compaction one burst later — measured slower on the 1024-stream wave).
  Prefill steps never sync and prompts are tokenized at admission one chunk ahead, so the host tokenizes and builds
  chunk i+1 while the GPU computes chunk i; after an idle period the chunks ramp up from ``prefill_ramp`` tokens so
  the GPU is not left waiting for the first chunk's tokenization.

The reference's ``analyze_sequence`` blocked the sensor for one chain at a time (quirk Q1); here thousands of chains
are in flight and each returns as soon as its own verdict closes.
"""
from __future__ import annotations

import collections
import itertools
import logging
import math
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Optional

import numpy as np
import torch

from ... import ops
from ...models.llama import KVCache, LlamaModel, StepBatch, build_model, h2d, make_prefill_batch
from ...parallel.tp import TPContext
from ...utils import trace
from ..constrain import DONE, GrammarBank
from ..tokenizer import load_tokenizer
from .block_manager import BlockManager

log = logging.getLogger("chronos.engine")
_PHASE_SYNC = os.environ.get("CHRONOS_PHASE_SYNC", "0") not in ("", "0")


@dataclass
class EngineConfig:
    model: str = "llama3-8b"
    checkpoint: Optional[str] = None
    tokenizer: Optional[str] = None
    device: str = "cuda"
    seed: int = 0
    max_slots: int = 256           # concurrent sequences in the decode batch
    block_size: int = 16
    max_model_len: int = 4096      # prompt + generated tokens per sequence
    kv_blocks: int = 0             # 0 = size from HBM (kv_fraction of free memory, capped at what max_slots can use)
    kv_fraction: float = 0.9
    reserve_gb: float = 12.0       # activations / graph pools / grammar table headroom
    max_prefill_tokens: int = 16384
    default_num_predict: int = 128
    max_out: int = 512             # hard cap on generated tokens per request
    decode_burst: int = 8
    # Shorter bursts once a large decode bucket has started to drain (<= tail_burst_fill of its rows live, >= 128
    # rows): compaction into a smaller bucket happens at harvests, so the tail of a wave sheds finished rows sooner.
    # 0 disables.
    tail_burst: int = 4
    tail_burst_fill: float = 0.9
    # Decode buckets of at most small_burst_rows rows (one or two sensor streams in flight) run bursts of small_burst
    # steps: the steps a burst runs after its row closed its verdict or parked on a grammar-forced run are gated but
    # not free, and the host harvest between bursts is cheap at this size (single stream, 24 chains: 2.85 ms/token at
    # 8 steps, 2.75 at 4, 2.73 at 2, 2.72 at 1; profiles/r5/single_stream_burst_ab*.json).  0 disables.
    small_burst: int = 1
    small_burst_rows: int = 2
    use_graphs: bool = True
    grammar_capacity: int = 2048
    max_string: int = 160          # default maxLength for schema strings without one (keeps verdicts short)
    prefix_cache: bool = True      # reuse KV blocks of identical prompt prefixes (the shared CHRONOS template head)
    partial_prefix: bool = True    # ... and the computed leading slots of a partially matching block (copied in)
    kv_dtype: str = "bf16"         # "bf16" or "fp8" (OCP e4m3fn, per-layer scale: half the KV bytes, 2x tokens/GPU)
    weight_dtype: str = "bf16"     # "bf16" or "fp8": W8A8 e4m3 projections on the block-scaled MFMA (csrc/kernels/fp8.hip)
    kv_scale: float = 1.0          # fp8 KV scale (stored = value / scale)
    prefill_nqt: int = 8           # 8 = flash prefill kernel (128 query rows / workgroup); 1-2 = split-K kernel
    async_harvest: bool = False    # harvest burst k while burst k+1 runs (hides host work, delays compaction)
    request_timeout_s: float = 0.0  # >0: a request not finished this long after submit is cancelled (reason "timeout")
    # KV reservation: "lazy" = prompt + kv_lookahead tokens at admission, grown per launch, recompute preemption of the
    # newest sequences when the pool runs dry; "full" = prompt + num_predict at admission (never preempts); "auto" =
    # full when the pool holds every slot at max_model_len (no pressure is possible: the per-launch growth bookkeeping
    # would be pure host overhead, ~0.4 % on the headline wave), lazy otherwise
    kv_alloc: str = "auto"
    kv_lookahead: int = 64         # generated-token headroom allocated per growth (amortises the block-table updates)
    kv_watermark: float = 0.01     # lazy admission leaves this fraction of the pool free for the running rows' growth
    tp_overlap: bool = True        # TP prefill: two micro-batches, each one's RCCL all-reduces overlap the other's compute
    tp_overlap_min_tokens: int = 1024
    tp_sequence_parallel: bool = False  # TP prefill: reduce-scatter / all-gather around the norms instead of all-reduce
    # TP decode: batches of at least this many rows run as two halves whose fused IPC all-reduce + norm launches
    # overlap the other half's compute on a second HIP stream (LlamaModel._forward_dec_overlap; 0 = off)
    tp_decode_overlap: int = 0
    decode_gate: bool = True       # small buckets: kernels of steps after the last live row finished return at once
    cp_min_tokens: int = 4096      # context parallel (Engine(cp=...)): prefill chunks at least this long are split
    cp_mode: str = "allgather"     # "allgather" (zigzag token pieces) or "ulysses" (head-sharded attention)
    # First prefill step after the engine was idle covers this many tokens, each later one 4x more, up to the chunk:
    # the GPU starts on a small chunk while the host tokenizes the next (0 = always full chunks).
    prefill_ramp: int = 2048
    # Jump-forward over grammar-forced token runs (brain/constrain GrammarBank.jumps) while at most jump_max_rows
    # sequences decode: a row entering a forced run parks, and the host appends the run in one prefill-mode forward
    # instead of one decode step per token.  Larger decode batches are compute-bound, where it would not pay.  The
    # forced run's token ids are its canonical tokenization, so a request's token ids (never the text of the forced
    # runs) can differ between a small batch and a large one; the GPU's batch-size-dependent GEMM kernels already make
    # outputs batch-dependent in the same way.
    jump_forward: bool = True
    jump_max_rows: int = 8
    # Mixed steps (steady-state continuous batching): while sequences decode, a waiting prompt's chunk joins the
    # decode rows in one forward instead of a prefill step that idles them.  Prefill tokens per mixed step: at most
    # max(mixed_prefill_tokens, mixed_ratio * decode rows) (and the admission ramp).
    mixed_batching: bool = True
    mixed_prefill_tokens: int = 2048
    mixed_ratio: int = 4
    # ... but only while the arrivals are a stream, not a wave: with more than this many prompts queued or
    # prefilling (a wave of chains arriving together) full-size prefill steps clear the backlog first — 2048-token
    # mixed chunks would re-stream every weight once per chunk (wave of 1024 chains: 17 forwards instead of 4, 575 vs
    # 620 chains/s), while the steady state gains from mixing (closed loop at 1024 streams: 691 vs 590 chains/s;
    # profiles/r3_bench_mixed_ab.txt).  A closed loop's harvests return ~100 completions (and as many arrivals) at
    # once; a limit of 64 turned most of them back into plain prefill steps (619 chains/s).
    mixed_max_backlog: int = 256
    # Cascade decode attention (csrc/kernels/attention.hip casc_prefix_kernel): when at least cascade_min_rows running
    # sequences hold the same leading prefix-cache blocks (the shared prompt template), their decode attention over
    # those blocks runs once per 16 / G rows as an MFMA pass and is merged into each row's walk over its own tokens.
    # Off by default: measured slower on the MI355X (profiles/r5/cascade_ab.md: the shared blocks are L2 hits for
    # the one-wave kernel, so skipping them saves little, and the extra pass costs ~10 us per layer at 1024 rows).
    cascade: bool = False
    cascade_min_rows: int = 32
    cascade_max_blocks: int = 8
    # token automata compiled at start-up (a first request must not pay the ~4 s vocab walk: the reference's cold-start
    # timeout): "verdict" = the CHRONOS verdict schema the sensor sends, "json" = format:"json"
    warm_formats: tuple = ("verdict", "json")


@dataclass
class Request:
    rid: int
    prompt_ids: list
    fmt: Any = None
    num_predict: int = 128
    temperature: float = 0.0
    seed: int = 0
    callback: Optional[Callable[["Request"], None]] = None
    meta: dict = field(default_factory=dict)
    top_k: int = 0                 # 0 = off
    top_p: float = 1.0             # 1.0 = off
    # runtime
    pending_text: Optional[tuple] = None  # (prompt, system, raw) until tokenized at admission
    slot: int = -1
    blocks: list = field(default_factory=list)
    prefilled: int = 0
    start_state: int = 0
    out_ids: list = field(default_factory=list)
    text: str = ""
    done_reason: str = ""
    error: Optional[str] = None
    t_submit: float = 0.0
    t_admit: float = 0.0
    t_first: float = 0.0
    t_done: float = 0.0
    # KV growth / preemption (lazy reservation): upper bound of the next KV position a queued launch may write, ids
    # generated before a preemption (the re-prefilled prompt carries them), prompt length as submitted
    pos_hi: int = 0
    resume_out: list = field(default_factory=list)
    orig_plen: int = -1
    preemptions: int = 0

    @property
    def kv_cap(self) -> int:
        """KV slots this request can ever write: prompt + num_predict (the last sampled token is never written)."""
        return len(self.prompt_ids) + self.num_predict

    @property
    def latency(self) -> float:
        return self.t_done - self.t_submit


def _bucket(n: int) -> int:
    """Decode batch rows for n live slots: powers of two up to 256, then multiples of 256.  Above 256 rows a decode
    step is GEMM-compute-bound with cost stepping at the library's 256-row M tile (896 rows cost what 1024 do, 768
    rows 15% less: profiles/), so 256-row steps let the tail of a wave shed cost as verdicts finish instead of only
    at each halving."""
    if n <= 256:
        return 1 << max(0, (n - 1).bit_length())
    return (n + 255) // 256 * 256


@dataclass
class _Snapshot:
    """Slot states copied (asynchronously) to pinned host memory at the end of a decode burst.  ``owners`` maps each
    slot to the request that occupied it when the copy was queued: slots can be freed, refilled or compacted before
    the snapshot is read, and those requests are matched by identity, never by slot number."""
    n: int
    event: Any
    state: torch.Tensor
    nout: torch.Tensor
    out: torch.Tensor
    owners: dict
    seq: int = 0  # order in which snapshots were queued (a jump applied after snapshot k makes k's parked rows stale)


class Engine:
    def __init__(self, cfg: EngineConfig, tp: TPContext | None = None, model: LlamaModel | None = None,
                 tokenizer=None, cp: TPContext | None = None):
        """``cp``: a context-parallel group (full weights on every rank, parallel/context_parallel.py).  Its ranks
        run this engine in lockstep (same submissions, same order); long prefill chunks are split across them and
        each prefill step covers ``max_prefill_tokens`` per rank."""
        self.cfg = cfg
        self.tp = tp or TPContext.single()
        self.cp = cp or TPContext.single()
        if self.cp.world > 1 and self.tp.world > 1:
            raise ValueError("context parallelism runs on full-weight (TP=1) ranks")
        self._chunk = cfg.max_prefill_tokens * self.cp.world
        self._ramp = self._chunk  # current prefill step size (see EngineConfig.prefill_ramp)
        self._check_parked = False  # a prefill / jump sampled with park flags since the last harvest
        self.device = torch.device(cfg.device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
            ops.load()  # the HIP library must load on a GPU engine — never a silent eager fallback
            ops.device_init()
        self.tok = tokenizer or load_tokenizer(cfg.tokenizer)
        t0 = time.perf_counter()
        self.model = model or build_model(cfg.model, self.device, self.tp, cfg.seed, cfg.checkpoint,
                                          max_position=cfg.max_model_len + 16, weight_dtype=cfg.weight_dtype)
        self.load_seconds = time.perf_counter() - t0
        self.model.sequence_parallel = cfg.tp_sequence_parallel and self.tp.world > 1
        self.model.decode_overlap_rows = cfg.tp_decode_overlap if self.tp.world > 1 else 0
        mc = self.model.cfg
        self.bank = GrammarBank(self.tok.token_bytes_list(), self.tok.stop_ids, mc.vocab_size, cfg.grammar_capacity,
                                self.device, max_string=cfg.max_string,
                                encode=self.tok.encode if cfg.jump_forward else None)
        for f in cfg.warm_formats:
            if f == "verdict":
                from ...sensor.prompt import VERDICT_SCHEMA

                f = VERDICT_SCHEMA
            self.bank.get(f)
        # ---- KV sizing ----
        bs = cfg.block_size
        self.max_blocks_per_seq = (cfg.max_model_len + bs - 1) // bs
        need = cfg.max_slots * self.max_blocks_per_seq + 1
        nb = cfg.kv_blocks
        if nb <= 0:
            if self.device.type == "cuda":
                free, _ = torch.cuda.mem_get_info(self.device)
                budget = max(0.0, free * cfg.kv_fraction - cfg.reserve_gb * 2**30)
                nb = int(budget // KVCache.bytes_per_block(mc, self.tp, bs, cfg.kv_dtype))
                nb = max(2, min(nb, need))
            else:
                nb = need
        for grp in (self.tp, self.cp):  # lockstep TP / CP scheduling needs the same block budget on every rank
            if grp.world > 1:
                import torch.distributed as dist

                t = torch.tensor([nb], dtype=torch.int64, device=self.device)
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=grp.group)
                nb = int(t.item())
        self.kv = KVCache(mc, self.tp, nb, bs, self.device, cfg.kv_dtype, cfg.kv_scale, cfg.kv_scale)
        if cfg.kv_alloc not in ("auto", "lazy", "full"):
            raise ValueError(f"kv_alloc must be auto, lazy or full, not {cfg.kv_alloc!r}")
        self.kv_alloc = cfg.kv_alloc if cfg.kv_alloc != "auto" else ("full" if nb >= need else "lazy")
        self.blocks = BlockManager(nb, bs, prefix_cache=cfg.prefix_cache, partial_prefix=cfg.partial_prefix)
        # ---- slot state (device) ----
        S, dev = cfg.max_slots, self.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.s_ids = torch.zeros(S, **i32)
        self.s_pos = torch.zeros(S, **i32)
        self.s_ctx = torch.ones(S, **i32)
        self.s_state = torch.full((S,), -1, **i32)
        self.s_rem = torch.zeros(S, **i32)
        self.s_nout = torch.zeros(S, **i32)
        self.s_seed = torch.zeros(S, **i32)
        self.s_temp = torch.zeros(S, dtype=torch.float32, device=dev)
        self.s_topk = torch.zeros(S, **i32)
        self.s_topp = torch.ones(S, dtype=torch.float32, device=dev)
        self.s_out = torch.zeros(S, cfg.max_out, **i32)
        self.s_bt = torch.zeros(S, self.max_blocks_per_seq, **i32)
        self.s_row = torch.full((S,), -1, **i32)
        self.ar = torch.arange(S + 1, **i32)
        self.ar64 = torch.arange(S, dtype=torch.int64, device=dev)
        # ---- scheduling state ----
        self.waiting: collections.deque[Request] = collections.deque()
        self.prefilling: list[Request] = []
        self._copies: list = []  # pending partial-prefix block copies (src, dst, request, start, j)
        self.running: dict[int, Request] = {}
        self.free_slots = list(range(S - 1, -1, -1))
        self._rid = itertools.count()
        self._graphs: dict[tuple[int, int, int], torch.cuda.CUDAGraph] = {}  # (rows, kv splits, steps) -> graph
        self._graph_pool = None
        self.stats = collections.Counter()
        # host wall seconds per scheduler phase (harvest includes harvest_gpu_wait: the wait for the burst to finish)
        self.phase_s: collections.Counter = collections.Counter()
        # re-entrant: request callbacks run on the scheduler thread and may submit follow-up requests (closed loop)
        self._lock = threading.RLock()
        self._cancels: list[tuple[Request, str]] = []
        # ---- harvest snapshots: two pinned host copies of (state, nout, out), alternated per burst ----
        pin = self.device.type == "cuda"
        self._snap_bufs = [tuple(torch.zeros(shape, dtype=torch.int32, pin_memory=pin)
                                 for shape in ((S,), (S,), (S, cfg.max_out))) for _ in range(2)]
        self._snap_i = 0
        self._snap_seq = 0
        self._pending: Optional[_Snapshot] = None
        self._ctx_need: Optional[int] = None  # _ctx_class's max(prompt + num_predict) over running rows
        self._deferred: list = []  # (request, reason) harvested, finished after the next launch (_flush_deferred)
        # cascade prefix state: device [P, block ids...] read by the decode graph, its O / lse scratch, host copy
        self._casc = None
        self._casc_cur: tuple = ()
        if self.device.type == "cuda" and cfg.cascade and self.model.hq % self.model.hkv == 0 and \
                16 % (self.model.hq // self.model.hkv) == 0:
            self._casc = (torch.zeros(1 + cfg.cascade_max_blocks, dtype=torch.int32, device=dev),
                          torch.empty(S, self.model.hq, 128, dtype=torch.bfloat16, device=dev),
                          torch.empty(S, self.model.hq, dtype=torch.float32, device=dev))
        self._async = cfg.async_harvest
        if self.device.type == "cuda":
            self._warmup()

    # ------------------------------------------------------------------------------------------------------------
    # public API
    # ------------------------------------------------------------------------------------------------------------
    def submit(self, prompt: str | list, fmt=None, num_predict: int | None = None, temperature: float = 0.0,
               seed: int = 0, raw: bool = False, system: str | None = None,
               callback: Callable[[Request], None] | None = None, meta: dict | None = None, top_k: int = 0,
               top_p: float = 1.0, max_len: int | None = None) -> Request:
        """Queue a request.  A text prompt is tokenized (chat template) lazily at admission, a prefill chunk's worth
        at a time, so host tokenization of a large wave overlaps the GPU prefill of the previous chunk."""
        n = num_predict if num_predict and num_predict > 0 else self.cfg.default_num_predict
        req = Request(next(self._rid), prompt if isinstance(prompt, list) else [], fmt, min(n, self.cfg.max_out),
                      float(temperature or 0.0), int(seed or 0), callback, meta or {})
        req.top_k, req.top_p = int(top_k or 0), float(top_p if top_p is not None else 1.0)
        if max_len:  # the request's own context window (Ollama options.num_ctx), within the engine's
            req.meta["max_len"] = min(int(max_len), self.cfg.max_model_len)
        req.t_submit = time.perf_counter()
        try:
            req.start_state = self.bank.get(fmt).start
        except Exception as e:  # bad schema: report, never crash the engine
            req.error = f"invalid format: {e}"
            self._finish(req, "error")
            return req
        if not isinstance(prompt, list):
            req.pending_text = (prompt, system, raw)
        if not self._check_length(req):  # a text prompt's length is re-checked once it is tokenized
            return req
        with self._lock:
            self.waiting.append(req)
        return req

    def _check_length(self, req: Request) -> bool:
        """Clamp num_predict to the context left after the prompt; finish the request with an error if nothing (or
        less than the format's shortest output) fits."""
        ids = req.prompt_ids
        limit = req.meta.get("max_len", self.cfg.max_model_len)
        req.num_predict = n = min(req.num_predict, limit - len(ids))
        if n <= 0:
            what = "num_ctx" if limit < self.cfg.max_model_len else "max_model_len"
            req.error = f"prompt of {len(ids)} tokens exceeds {what} {limit}"
        elif n < self.bank.min_tokens(req.start_state):
            need = self.bank.min_tokens(req.start_state)
            req.error = f"num_predict={n} cannot fit the shortest output of this format ({need} tokens)"
        if req.error:
            self._finish(req, "error")
            return False
        return True

    def has_work(self) -> bool:
        return bool(self.waiting or self.prefilling or self.running or self._deferred)

    def step(self) -> list[Request]:
        """One scheduling iteration: admit + prefill if anything is waiting, else one decode burst.

        A prefill step never syncs: its first tokens are sampled on device and a request that finishes on them is
        harvested after the next burst.  A decode burst queues its own snapshot and (async mode) harvests the previous
        one, which completed as soon as the GPU started on this burst."""
        pc, ph = time.perf_counter, self.phase_s
        t0 = pc()
        reaped = self._reap()
        with trace.range("admit"):
            self._admit()
        t1 = pc()
        ph["admit"] += t1 - t0
        if self.prefilling and self._mixable():
            with trace.range("mixed"):
                out = self._mixed_step()
            ph["mixed_host"] += pc() - t1
            return reaped + out + self._flush_deferred()
        if self.prefilling:
            with trace.range("prefill"):
                self._prefill_step()
            if _PHASE_SYNC and self.device.type == "cuda":
                torch.cuda.synchronize()  # attribute the prefill's GPU time to it (diagnostics only)
            ph["prefill_host"] += pc() - t1
            return reaped + self._flush_deferred()
        if self.running:
            if self._check_parked:
                # the last sampler launch (prefill / jump) may have parked every row: look before launching a burst
                # that would then run fully gated.  The fresh snapshot supersedes a mixed step's pending one (device
                # state only moves forward until a harvest resets it), whose pinned buffer the next snapshot reuses
                self._check_parked = False
                self._pending = None
                with trace.range("harvest"):
                    return reaped + self._harvest(self._snapshot(min(self._decode_rows(), self.cfg.max_slots)))
            with trace.range("decode_burst"):
                snap = self._decode_burst()
            reaped = reaped + self._flush_deferred()  # while the burst runs
            if snap is None:  # every row was preempted for KV: they re-prefill next step
                self._pending = None
                return reaped
            t2 = pc()
            ph["decode_launch"] += t2 - t1
            if not self._async:
                prev, self._pending = snap, None  # (a mixed step's pending snapshot is superseded by this one)
            else:
                prev, self._pending = self._pending, snap
            if prev is None:
                return reaped
            with trace.range("harvest"):
                out = reaped + self._harvest(prev)
            ph["harvest"] += pc() - t2
            return out
        self._pending = None
        return reaped + self._flush_deferred()

    def cancel(self, req: Request, reason: str = "cancelled") -> None:
        """Thread-safe: drop a request wherever it is (queued, prefilling or decoding) at the start of the next step;
        its slot and KV blocks are freed and its callback fires with ``done_reason == reason``."""
        with self._lock:
            self._cancels.append((req, reason))

    def _reap(self) -> list[Request]:
        with self._lock:
            todo, self._cancels = self._cancels, []
        if self.cfg.request_timeout_s > 0:
            dl = time.perf_counter() - self.cfg.request_timeout_s
            todo += [(r, "timeout") for r in (*self.waiting, *self.prefilling, *self.running.values())
                     if r.t_submit < dl]
        out, reset = [], []
        for req, reason in todo:
            if req.done_reason:
                continue  # already finished (or reaped twice)
            if req in self.prefilling:
                # Its prompt blocks are published in the prefix cache and may already be shared by a later request
                # that relies on this prefill computing them: finish the prefill, then drop it (_prefill_step).
                req.meta["cancel_reason"] = reason
                continue
            if self.running.get(req.slot) is req:
                del self.running[req.slot]
            else:
                with self._lock:
                    try:
                        self.waiting.remove(req)
                    except ValueError:
                        continue  # not known to this engine
            if req.slot >= 0:
                self.blocks.release(req.blocks)
                reset.append(req.slot)
                self.free_slots.append(req.slot)
                req.slot = -1
            req.error = f"request {reason}"
            self.stats[reason] += 1
            self._finish(req, reason)
            out.append(req)
        if reset:
            self.free_slots.sort(reverse=True)
            idx = h2d(torch.tensor(reset, dtype=torch.int64), self.device)
            self.s_state.index_fill_(0, idx, -1)
            self.s_bt.index_fill_(0, idx, 0)
            self.s_pos.index_fill_(0, idx, 0)
            self.s_ctx.index_fill_(0, idx, 1)
        return out

    def fail_all(self, error: str) -> list[Request]:
        """After a step raised: finish every queued, prefilling and decoding request with ``done_reason == 'error'``
        (callbacks fire, so HTTP callers get an error reply instead of hanging) and return the engine to empty.

        A faulted step may have left the block manager and the prefix cache half-updated, so both are rebuilt rather
        than patched; the device slot state is reset best-effort (the device itself may be gone)."""
        self._flush_deferred()  # verdicts harvested before the fault are complete: finish them normally
        with self._lock:
            reqs = [*self.waiting, *self.prefilling, *self.running.values()]
            self.waiting.clear()
            self._cancels = []
        self.prefilling = []
        self._copies = []
        self.running = {}
        self._pending = None
        self._check_parked = False
        S = self.cfg.max_slots
        self.free_slots = list(range(S - 1, -1, -1))
        self.blocks = BlockManager(self.blocks.num_blocks, self.blocks.block_size,
                                   prefix_cache=self.blocks.prefix_cache, partial_prefix=self.cfg.partial_prefix)
        self._casc_cur = ()
        try:
            if self._casc is not None:
                self._casc[0].zero_()
            self.s_state.fill_(-1)
            self.s_bt.zero_()
            self.s_pos.zero_()
            self.s_ctx.fill_(1)
        except Exception:  # noqa: BLE001 — a dead device must not stop the error replies below
            log.exception("slot state reset after a failed step")
        out = []
        for r in reqs:
            if r.done_reason:
                continue
            r.slot = -1
            r.error = error
            r.meta["internal_error"] = True
            self.stats["error"] += 1
            self._finish(r, "error")
            out.append(r)
        return out

    def run_until_idle(self, max_steps: int = 10**9) -> list[Request]:
        done = []
        for _ in range(max_steps):
            if not self.has_work():
                break
            done += self.step()
        return done

    def generate(self, prompts: list, fmt=None, num_predict: int | None = None, temperature: float = 0.0) -> list[Request]:
        reqs = [self.submit(p, fmt, num_predict, temperature) for p in prompts]
        self.run_until_idle()
        return reqs

    # ------------------------------------------------------------------------------------------------------------
    # scheduling
    # ------------------------------------------------------------------------------------------------------------
    def _admit(self) -> None:
        if self.waiting and self._deferred:
            # the KV blocks of requests the last harvest finished (their release is deferred past the GPU launch)
            for r, _ in self._deferred:
                self.blocks.release(r.blocks)
                r.blocks = []
        if not self.prefilling and not self.running and self.cfg.prefill_ramp > 0:
            # Idle engine: nothing is queued on the GPU, so the host's tokenization of a whole chunk would be exposed
            # (~50 ms for 16k tokens of chains).  Start small and grow 4x per step, so admitting the next step's
            # prompts always overlaps the current step's prefill.
            self._ramp = min(self.cfg.prefill_ramp, self._chunk)
        # admit about one prefill step ahead: the rest stays queued (and untokenized) while that step computes
        budget = self._ramp - sum(len(r.prompt_ids) - r.prefilled for r in self.prefilling)
        with self._lock:
            while self.waiting and self.free_slots and budget > 0:
                req = self.waiting[0]
                if req.pending_text is not None:
                    text, system, raw = req.pending_text
                    req.pending_text = None
                    req.prompt_ids = self.tok.chat_ids(text, system=system, raw=raw)
                    if not self._check_length(req):
                        self.waiting.popleft()
                        continue
                nblk, wm = self._admit_blocks(req)
                if nblk > self.blocks.num_blocks - 1:  # could never fit, even alone: an error, not a stalled queue
                    self.waiting.popleft()
                    req.error = (f"prompt of {len(req.prompt_ids)} tokens needs {nblk} KV blocks, the cache holds "
                                 f"{self.blocks.num_blocks - 1}")
                    self._finish(req, "error")
                    continue
                shared = self.blocks.lookup(req.prompt_ids)  # cached prefix blocks (already referenced)
                if not self.blocks.can_alloc(nblk - len(shared) + (wm if self.running else 0)):
                    self.blocks.release(shared)
                    break
                self.waiting.popleft()
                part = self.blocks.lookup_partial(req.prompt_ids, len(shared)) if self.cfg.partial_prefix else None
                if part is not None and not self.blocks.can_alloc(nblk - len(shared)):
                    self.blocks.release([part[0]])  # its reference took an evictable block out of the free pool
                    part = None
                req.blocks = shared + self.blocks.alloc(nblk - len(shared))
                req.meta["casc_n"] = len(shared)  # leading blocks shared through the prefix cache (cascade candidates)
                req.prefilled = len(shared) * self.blocks.block_size
                self.blocks.note_prompt(req.prompt_ids, req.blocks, len(shared))
                if part is not None:  # the first j slots of block len(shared) come from a computed block
                    src, j = part
                    self._copies.append((src, req.blocks[len(shared)], req, req.prefilled, j))
                    req.prefilled += j
                    self.stats["partial_prefix_tokens"] += j
                self.stats["prefix_hit_tokens"] += req.prefilled
                # Publish this prompt's full blocks right away: a request admitted later in this same round can
                # share them even before they are computed, because prefill packs requests in admission order and
                # every layer writes the step's K/V (rope_kv_write) before any of its attention reads it.
                self.blocks.register(req.prompt_ids, req.blocks)
                req.slot = self.free_slots.pop()
                req.t_admit = time.perf_counter()
                self.prefilling.append(req)
                budget -= len(req.prompt_ids) - req.prefilled
        # (the slots' block-table rows are published when their prompts finish: _init_slots)

    def _admit_blocks(self, req: Request) -> tuple[int, int]:
        """(KV blocks a request takes at admission, free blocks lazy admission leaves for the running rows)."""
        if self.kv_alloc == "full":
            return self.blocks.blocks_for(req.kv_cap), 0
        toks = min(req.kv_cap, len(req.prompt_ids) + self.cfg.kv_lookahead)
        return self.blocks.blocks_for(toks), int(self.cfg.kv_watermark * self.blocks.num_blocks)

    # ---- KV growth and recompute preemption (kv_alloc="lazy") -------------------------------------------------------
    def _ensure_kv(self, extra: list) -> None:
        """Grow running sequences' blocks so the launch about to be queued can write its KV.  ``extra``: (request,
        KV slots (positions + 1) that launch may write for it).  Oldest requests are served first; when the pool is
        short, the newest running requests are preempted (recompute) until it is not.  Updates the slot block
        tables of every grown row in one device write."""
        bs = self.blocks.block_size
        grown = []
        for r, need in sorted(extra, key=lambda e: e[0].rid):
            if self.running.get(r.slot) is not r:
                continue  # preempted as a victim of an older request's growth
            need = min(r.kv_cap, need)
            have = len(r.blocks) * bs
            if need <= have:
                continue
            want = self.blocks.blocks_for(need) - len(r.blocks)
            while not self.blocks.can_alloc(want):
                victim = max((q for q in self.running.values()), key=lambda q: q.rid)
                self._preempt(victim)
                if victim is r:
                    break
            if self.running.get(r.slot) is not r:
                continue
            more = self.blocks.blocks_for(min(r.kv_cap, need + self.cfg.kv_lookahead)) - len(r.blocks)
            take = max(want, min(more, self.blocks.free))
            old = len(r.blocks)
            r.blocks += self.blocks.alloc(take)
            grown.append((r, old))
            self.stats["kv_grow_blocks"] += take
        if grown:
            rows, cols, vals = [], [], []
            for r, old in grown:
                for j in range(old, len(r.blocks)):
                    rows.append(r.slot)
                    cols.append(j)
                    vals.append(r.blocks[j])
            dv = lambda t: h2d(t, self.device)  # noqa: E731
            self.s_bt[dv(torch.tensor(rows, dtype=torch.int64)), dv(torch.tensor(cols, dtype=torch.int64))] = dv(
                torch.tensor(vals, dtype=torch.int32))

    def _preempt(self, r: Request) -> None:
        """Recompute preemption of a running request: read its exact device state (a sync — preemption is rare),
        publish its computed full blocks to the prefix cache, free its blocks and slot, and queue it at the front
        with the generated ids appended to its prompt and its grammar resuming from the saved state.  A request whose
        verdict already closed on device is finished instead (nothing to recompute)."""
        s = r.slot
        st = int(self.s_state[s].item())
        n = min(int(self.s_nout[s].item()), self.cfg.max_out)
        out = self.s_out[s, :n].tolist() if n else []
        del self.running[s]
        r.slot = -1
        self._free_slots([s])
        if st == DONE:  # finished on device, not harvested yet: complete it now
            stop = bool(out) and out[-1] in self.tok.stop_ids
            r.out_ids = r.resume_out + (out[:-1] if stop else out)
            r.t_done = time.perf_counter()
            self.blocks.release(r.blocks)
            r.blocks = []
            self.stats["completed"] += 1
            self.stats["generated_tokens"] += len(r.out_ids)
            self._deferred.append((r, "stop" if stop else "length"))
            return
        on_tok = r.meta.get("on_tokens")
        if on_tok is not None:  # stream what this run produced before it is folded into the prompt
            e = r.meta.get("emitted", 0)
            if n > e:
                try:
                    on_tok(out[e:n])
                except Exception:
                    log.exception("stream callback failed")
            r.meta["emitted"] = 0
        plen = len(r.prompt_ids)
        if r.orig_plen < 0:
            r.orig_plen = plen
        ctx = r.prompt_ids + out
        # KV exists for positions < plen + n - 1 (the last sampled token is pending): publish those full blocks, so
        # the re-admission's prefix lookup finds them unless they are evicted first
        self.blocks.register(ctx[:plen + n - 1] if n else ctx, r.blocks)
        self.blocks.release(r.blocks)
        r.blocks = []
        r.prompt_ids = ctx
        r.resume_out = r.resume_out + out
        r.meta.setdefault("orig_num_predict", r.num_predict)
        r.num_predict -= n
        r.start_state = -2 - st if st <= -2 else st
        r.prefilled = 0
        r.preemptions += 1
        r.meta.pop("jump_seq", None)
        r.meta["preempt_seq"] = self._snap_seq  # snapshots queued so far hold this run's rows, not the next one's
        self.stats["preemptions"] += 1
        with self._lock:
            self.waiting.appendleft(r)

    def _update_casc(self) -> None:
        """Pick the cascade prefix for the next decode launch: the longest run of leading blocks held by at least
        cascade_min_rows sequences (block refcounts), taken from the latest running requests that share prefix-cache
        blocks.  Re-evaluated every launch (a few dozen dictionary lookups); the device copy is rewritten only on a
        change.  Rows that do not hold the prefix are unaffected (both kernels test membership per row)."""
        if self._casc is None:
            return
        ref, mn, pmax = self.blocks._ref, self.cfg.cascade_min_rows, self.cfg.cascade_max_blocks
        new: tuple = ()
        for r in list(self.running.values())[-32:]:  # the latest admissions (a wave's all share the template)
            k = min(r.meta.get("casc_n", 0), pmax, len(r.blocks))
            if k <= len(new):
                continue
            p = 0
            while p < k and ref.get(r.blocks[p], 0) >= mn:
                p += 1
            if p > len(new):
                new = tuple(r.blocks[:p])
        if new == self._casc_cur:
            return
        self._casc_cur = new
        v = [len(new)] + list(new) + [0] * (pmax - len(new))
        self._casc[0].copy_(h2d(torch.tensor(v, dtype=torch.int32), self.device))
        self.stats["cascade_updates"] += 1
        self.stats["cascade_max_blocks"] = max(self.stats["cascade_max_blocks"], len(new))

    def _free_slots(self, slots: list) -> None:
        """Return slots to the free list and park their device state (empty, scratch block table)."""
        self.free_slots.extend(slots)
        self.free_slots.sort(reverse=True)
        idx = h2d(torch.tensor(slots, dtype=torch.int64), self.device)
        self.s_state.index_fill_(0, idx, -1)
        self.s_bt.index_fill_(0, idx, 0)
        self.s_pos.index_fill_(0, idx, 0)
        self.s_ctx.index_fill_(0, idx, 1)

    def _grow_for(self, k: int) -> None:
        """Lazy KV: every running row may write k more KV positions in the launch about to be queued (a decode burst
        of k steps, or a mixed step's one): grow whoever needs it, then advance the bound."""
        if self.kv_alloc != "lazy" or not self.running:
            return
        bs = self.blocks.block_size
        extra = [(r, r.pos_hi + k) for r in self.running.values()
                 if r.pos_hi + k > len(r.blocks) * bs and len(r.blocks) * bs < r.kv_cap]
        if extra:
            self._ensure_kv(extra)
        for r in self.running.values():
            r.pos_hi += k

    def _copy_partial_blocks(self) -> None:
        """Batched copy of the partial-prefix source blocks into their new owners (every layer's K and V, whole
        blocks: the slots past j are rewritten by the owner's prefill before any attention reads them)."""
        jobs, self._copies = self._copies, []
        src = h2d(torch.tensor([c[0] for c in jobs], dtype=torch.int64), self.device)
        dst = h2d(torch.tensor([c[1] for c in jobs], dtype=torch.int64), self.device)
        for cache in (*self.kv.k, *self.kv.v):
            cache.index_copy_(0, dst, cache.index_select(0, src))
        for s, d, req, start, j in jobs:
            self.blocks.mark_computed(req.blocks, start, start + j)
            self.blocks.release([s])

    def _gather_prefill(self, budget: int):
        chunks, starts, bts, reqs = [], [], [], []
        for req in self.prefilling:
            if budget <= 0:
                break
            n = min(len(req.prompt_ids) - req.prefilled, budget)
            chunks.append(req.prompt_ids[req.prefilled:req.prefilled + n])
            starts.append(req.prefilled)
            bts.append(req.blocks)
            reqs.append(req)
            budget -= n
        return chunks, starts, bts, reqs

    def _prefill_done(self, reqs, chunks) -> tuple[list[int], list[Request]]:
        """Host bookkeeping after a prefill forward was queued: computed slots, finished prompts (their full blocks
        published, their slots initialised for decoding)."""
        done_rows, done_reqs = [], []
        for i, (req, ch) in enumerate(zip(reqs, chunks)):
            self.blocks.mark_computed(req.blocks, req.prefilled, req.prefilled + len(ch))
            req.prefilled += len(ch)
            if req.prefilled == len(req.prompt_ids):
                done_rows.append(i)
                done_reqs.append(req)
                req.pos_hi = len(req.prompt_ids)  # the first sampled token is written there by the next decode step
                self.blocks.register(req.prompt_ids, req.blocks)
        self.stats["prefill_tokens"] += sum(len(c) for c in chunks)
        self.stats["prefill_steps"] += 1
        if done_reqs:
            self._init_slots(done_reqs)
        return done_rows, done_reqs

    def _init_slots(self, done_reqs) -> None:
        """A finished prompt's slot state, ready for its first sampled token.  Its block-table row is published only
        now: until then the slot's row points at the scratch block, so a mixed step's decode rows (which cover every
        slot of the bucket) never write into a prompt that is still prefilling."""
        slots = torch.tensor([r.slot for r in done_reqs], dtype=torch.int64)
        plen = torch.tensor([len(r.prompt_ids) for r in done_reqs], dtype=torch.int32)
        dv = lambda t: h2d(t, self.device)  # noqa: E731
        sl = dv(slots)
        mb = self.max_blocks_per_seq
        self.s_bt[sl] = dv(torch.tensor([r.blocks + [0] * (mb - len(r.blocks)) for r in done_reqs], dtype=torch.int32))
        self.s_state[sl] = dv(torch.tensor([r.start_state for r in done_reqs], dtype=torch.int32))
        self.s_rem[sl] = dv(torch.tensor([r.num_predict for r in done_reqs], dtype=torch.int32))
        self.s_pos[sl] = dv(plen - 1)
        self.s_ctx[sl] = dv(plen)
        self.s_nout.index_fill_(0, sl, 0)
        self.s_temp[sl] = dv(torch.tensor([r.temperature for r in done_reqs], dtype=torch.float32))
        self.s_seed[sl] = dv(torch.tensor([r.seed for r in done_reqs], dtype=torch.int32))
        self.s_topk[sl] = dv(torch.tensor([r.top_k for r in done_reqs], dtype=torch.int32))
        self.s_topp[sl] = dv(torch.tensor([r.top_p for r in done_reqs], dtype=torch.float32))

    def _start_running(self, done_reqs) -> None:
        now = time.perf_counter()
        for r in done_reqs:
            r.t_first = now
            self.prefilling.remove(r)
            self.running[r.slot] = r
            self._ctx_need = None
            if "cancel_reason" in r.meta:  # cancelled mid-prefill: its blocks are computed now, drop it next step
                self.cancel(r, r.meta["cancel_reason"])

    def _sample(self, logits, jump) -> None:
        ops.constrained_sample(logits, self.s_row, self.bank.next, self.bank.dist, DONE, self.s_state, self.s_rem,
                               self.s_temp, self.s_seed, self.s_ids, self.s_pos, self.s_ctx, self.s_nout, self.s_out,
                               self.s_topk, self.s_topp, jump)

    def _prefill_step(self) -> None:
        if self._copies:
            self._copy_partial_blocks()
        budget = self._ramp
        self._ramp = min(4 * self._ramp, self._chunk)
        chunks, starts, bts, reqs = self._gather_prefill(budget)
        ntok = sum(len(c) for c in chunks)
        if (self.cp.world > 1 and len(chunks) == 1
                and ntok >= max(self.cfg.cp_min_tokens, 2 * self.cp.world)):  # context-parallel chunk
            from ...parallel.context_parallel import last_logits, make_cp_batch, make_ulysses_batch

            build = make_ulysses_batch if self.cfg.cp_mode == "ulysses" else make_cp_batch
            sb = build(chunks[0], starts[0], bts[0], self.model.cfg, self.cp, self.device,
                       self.max_blocks_per_seq, nqt=self.cfg.prefill_nqt)
            logits = last_logits(self.model.forward(sb, self.kv), self.cp, sb.cp)
            self.stats["cp_prefill_steps"] += 1
        else:
            chunks, starts, bts, reqs = self._fit(chunks, starts, bts, reqs)
            ntok = sum(len(c) for c in chunks)
            split = 2 if (self.tp.world > 1 and self.cfg.tp_overlap and ntok >= self.cfg.tp_overlap_min_tokens) else 1
            sb = make_prefill_batch(chunks, starts, bts, self.model.cfg, self.tp, self.device,
                                    max_blocks=self.max_blocks_per_seq, nqt=self.cfg.prefill_nqt, split=split)
            logits = self.model.forward(sb, self.kv)
        done_rows, done_reqs = self._prefill_done(reqs, chunks)
        if not done_reqs:
            return
        # sample the finished prompts' first token
        self.s_row.fill_(-1)
        self.s_row[h2d(torch.tensor([r.slot for r in done_reqs], dtype=torch.int64), self.device)] = h2d(
            torch.tensor(done_rows, dtype=torch.int32), self.device)
        jf = self._jump_flags(len(self.running) + len(done_reqs))
        self._sample(logits, jf)
        self._check_parked = jf is not None
        self._start_running(done_reqs)

    def _mixable(self) -> bool:
        return (self.cfg.mixed_batching and bool(self.running) and self.cp.world == 1
                and not self.model.sequence_parallel
                and len(self.waiting) + len(self.prefilling) <= self.cfg.mixed_max_backlog)

    def _mixed_step(self) -> list[Request]:
        """Continuous batching in steady state: ONE forward over a prefill chunk AND one decode token for every row
        of the live decode bucket (shared projections; prefill tiles and decode rows each on their own attention
        kernel), then one sampler launch that advances the decode rows and starts the prompts that finished.  An
        arriving chain therefore never stalls the verdicts already decoding.  The prefill share per step is bounded
        (``mixed_prefill_tokens``, or ``mixed_ratio`` per decode row) so the decode rows' per-token time stays close
        to a plain decode step.  Eager (the prefill part changes every step); the snapshot of step i is harvested
        after step i+1 was queued, so the host never waits for the GPU it is about to feed."""
        if self._copies:
            self._copy_partial_blocks()
        self._grow_for(1)  # (may preempt: the bucket below is sized after it)
        if not self.running:
            self._prefill_step()
            return []
        n = min(self._decode_rows(), self.cfg.max_slots)
        budget = min(self._ramp, max(self.cfg.mixed_prefill_tokens, self.cfg.mixed_ratio * n))
        self._ramp = min(4 * self._ramp, self._chunk)
        chunks, starts, bts, reqs = self._fit(*self._gather_prefill(budget))
        sb = make_prefill_batch(chunks, starts, bts, self.model.cfg, self.tp, self.device,
                                max_blocks=self.max_blocks_per_seq, nqt=self.cfg.prefill_nqt)
        tp_, bp = sum(len(c) for c in chunks), len(chunks)
        self._update_casc()
        sb.dec = StepBatch(self.s_ids[:n], self.s_pos[:n], self.ar[:n], self.s_bt[:n], self.ar[:n + 1], self.s_ctx[:n],
                           self.ar64[:n], None, n, 1, self._nsplit(n, self._ctx_class()), casc=self._casc)
        sb.last_idx = torch.cat([sb.last_idx, tp_ + self.ar64[:n]])
        logits = self.model.forward(sb, self.kv)
        done_rows, done_reqs = self._prefill_done(reqs, chunks)
        # logits rows: the prefill sequences' last tokens, then decode row i at bp + i
        self.s_row.fill_(-1)
        self.s_row[:n] = self.ar[:n] + bp
        if done_reqs:
            self.s_row[h2d(torch.tensor([r.slot for r in done_reqs], dtype=torch.int64), self.device)] = h2d(
                torch.tensor(done_rows, dtype=torch.int32), self.device)
        self._sample(logits, None)  # no jump-forward parking: this harvest lags one step
        self._start_running(done_reqs)
        self.stats["mixed_steps"] += 1
        self.stats["mixed_decode_rows"] += n
        self.stats["decode_row_steps"] += n
        snap = self._snapshot(min(self._decode_rows(), self.cfg.max_slots))
        prev, self._pending = self._pending, snap
        return self._harvest(prev) if prev is not None else []

    def _fit(self, chunks, starts, bts, reqs):
        """A replicated (non-CP) prefill step covers at most max_prefill_tokens: with CP the admission budget is
        W times that, so trim the packed chunks back to one rank's worth."""
        if self._chunk == self.cfg.max_prefill_tokens:
            return chunks, starts, bts, reqs
        out, left = ([], [], [], []), self.cfg.max_prefill_tokens
        for c, s0, bt, r in zip(chunks, starts, bts, reqs):
            if left <= 0:
                break
            c = c[:left]
            for lst, v in zip(out, (c, s0, bt, r)):
                lst.append(v)
            left -= len(c)
        return out

    def _decode_rows(self) -> int:
        return _bucket(max(self.running) + 1) if self.running else 0

    def _decode_once(self, n: int, nsplit: int) -> None:
        sb = StepBatch(self.s_ids[:n], self.s_pos[:n], self.ar[:n], self.s_bt[:n], self.ar[:n + 1], self.s_ctx[:n],
                       self.ar64[:n], None, n, 1, nsplit, casc=self._casc)
        logits = self.model.forward(sb, self.kv)
        ops.constrained_sample(logits, None, self.bank.next, self.bank.dist, DONE, self.s_state[:n], self.s_rem[:n],
                               self.s_temp[:n], self.s_seed[:n], self.s_ids[:n], self.s_pos[:n], self.s_ctx[:n],
                               self.s_nout[:n], self.s_out[:n], self.s_topk[:n], self.s_topp[:n], self._jump_flags(n))

    def _jump_flags(self, rows: int):
        """The sampler's park-on-forced-run flags for a decode batch of ``rows`` sequences (None = never park).  With
        async harvest the snapshot a row parked in is read one burst late: the burst launched meanwhile runs that row
        gated (the sampler leaves parked rows untouched), the jump's device writes queue behind it, and the next
        snapshot — taken before the jump — is recognised as stale by the row's ``jump_seq`` (``_harvest``)."""
        if self.cfg.jump_forward and self.bank.jumps and 0 < rows <= self.cfg.jump_max_rows:
            return self.bank.jump
        return None

    def _nsplit(self, n: int, ctx_cap: int | None = None) -> int:
        return ops.pick_nsplit(n * self.model.hkv, ctx_cap or self.cfg.max_model_len)

    def _ctx_class(self) -> int:
        """Power-of-two bound (>= 256, <= max_model_len) on every running sequence's context during the next burst:
        prompt + num_predict, known at admission.  The decode kv split (flash-decoding) is sized for it, so short
        verdict contexts decode with one split (no combine) instead of the split count max_model_len would ask for
        (single stream, 512-token engine: 3.71 -> 3.64 ms/token; profiles/r2_single_stream_split_ab.json), and a
        128k request still gets its 64."""
        # cached between admissions: rows only leave the running set while nothing is admitted, and a stale (larger)
        # bound only costs a split, so the 1024-row scan runs once per admission, not once per burst
        if self._ctx_need is None:
            self._ctx_need = max((len(r.prompt_ids) + r.num_predict for r in self.running.values()), default=1)
        need = self._ctx_need
        c = 256
        while c < need:
            c *= 2
        return min(c, self.cfg.max_model_len)

    def _burst_len(self, n: int) -> int:
        k, t = self.cfg.decode_burst, self.cfg.tail_burst
        if 0 < t < k and n >= 128 and len(self.running) <= self.cfg.tail_burst_fill * n:
            return t
        if 0 < self.cfg.small_burst < k and n <= self.cfg.small_burst_rows:
            return self.cfg.small_burst
        return k

    def _decode_burst(self) -> Optional[_Snapshot]:
        k = self._burst_len(min(self._decode_rows(), self.cfg.max_slots))
        self._grow_for(k)  # (may preempt: the bucket is sized after it)
        if not self.running:
            return None
        self._update_casc()
        n = min(self._decode_rows(), self.cfg.max_slots)
        ns = self._nsplit(n, self._ctx_class())
        if self.device.type == "cuda" and self.cfg.use_graphs:
            g = self._graphs.get((n, ns, k))
            if g is None:
                g = self._capture(n, ns, k)
            g.replay()
        else:
            self._gate(n)
            try:
                for _ in range(k):
                    self._decode_once(n, ns)
            finally:
                self._gate(0)
        self.stats["decode_steps"] += k
        self.stats[f"bursts@{n}"] += 1
        self.stats["decode_row_steps"] += k * n
        return self._snapshot(n)

    def _snapshot(self, n: int) -> _Snapshot:
        st, no, out = self._snap_bufs[self._snap_i]
        # two alternating pinned buffers: at most ONE snapshot (the pending one) may be outstanding when a new one is
        # queued, and never in the buffer about to be overwritten
        assert self._pending is None or self._pending.state is not st, "snapshot buffer still referenced"
        self._snap_i ^= 1
        self._snap_seq += 1
        st[:n].copy_(self.s_state[:n], non_blocking=True)
        no[:n].copy_(self.s_nout[:n], non_blocking=True)
        out[:n].copy_(self.s_out[:n], non_blocking=True)
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        return _Snapshot(n, ev, st, no, out, dict(self.running), self._snap_seq)

    def _gate(self, n: int) -> None:
        """Arm the decode early-exit gate for a small bucket (n <= 8 rows): the steps of a burst after every row's
        verdict closed skip all their kernels (csrc/include/chronos_hip.h).  Relies on DONE == 0, empty == -1."""
        if self.device.type == "cuda" and self.cfg.decode_gate:
            ops.set_decode_gate(self.s_state, n if 0 < n <= 8 else 0)

    def _capture(self, n: int, ns: int, k: int) -> "torch.cuda.CUDAGraph":
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        self._gate(n)
        try:
            with torch.cuda.graph(g, pool=self._graph_pool):
                for _ in range(k):
                    self._decode_once(n, ns)
        finally:
            self._gate(0)
        self._graphs[(n, ns, k)] = g
        self.stats["graphs_captured"] += 1
        return g

    def _warmup(self) -> None:
        """Initialise library handles / kernels with every slot empty (scratch block only), so graph capture later
        never has to run a lazily-initialising op."""
        n = self.cfg.max_slots
        self._decode_once(n, self._nsplit(n))
        torch.cuda.synchronize()

    def _harvest(self, snap: _Snapshot) -> list[Request]:
        if snap.event is not None:
            t = time.perf_counter()
            snap.event.synchronize()
            self.phase_s["harvest_gpu_wait"] += time.perf_counter() - t
        # (snapshot slot, request) for requests still running as the same object (identity, not slot number)
        # (a request preempted after this snapshot was queued may be running again in another slot: its row here
        # belongs to the run before the preemption).  The snapshot is read through numpy views of its pinned buffers
        # and only the rows that finished, parked or stream tokens get Python work: the full 1024-row scan and the
        # per-row tensor indexing it replaced were ~1 ms of GPU-idle host time per burst on the 1024-stream wave
        seq, owners, running = snap.seq, snap.owners, self.running

        def alive(s: int) -> Optional[Request]:
            r = owners.get(s)
            if r is not None and running.get(r.slot) is r and r.meta.get("preempt_seq", -1) < seq:
                return r
            return None

        st = snap.state[:snap.n].numpy()
        nout, outs = snap.nout.numpy(), snap.out.numpy()
        finished = [(s, r) for s in np.flatnonzero(st == DONE).tolist() if (r := alive(s)) is not None]
        # a parked row whose jump was already applied after this snapshot was queued (a mixed step harvests one step
        # late) is stale: applying its run again would rewind the row and duplicate the run
        parked = [(s, r) for s in np.flatnonzero(st <= -2).tolist()
                  if (r := alive(s)) is not None and r.meta.get("jump_seq", 0) < seq]
        streaming = [(s, r) for s, r in owners.items() if r.meta.get("on_tokens") and alive(s) is not None]
        ended = {}  # slot -> output ids of jumped runs that end the verdict
        if parked:
            t = time.perf_counter()
            ended = self._jump(parked, st, nout, outs)
            self.phase_s["jump"] += time.perf_counter() - t
        finished += [(s, r) for s, r in parked if s in ended]
        # (a jump's KV growth may have preempted some of these rows: they are queued again, not finished)
        finished = [(s, r) for s, r in finished if self.running.get(r.slot) is r]
        streaming = [(s, r) for s, r in streaming if self.running.get(r.slot) is r]
        if not finished and not streaming:
            return []
        for s, r in streaming:  # incremental tokens for stream=true clients
            src = ended.get(s)
            k = len(src) if src is not None else min(int(nout[s]), self.cfg.max_out)
            e = r.meta.get("emitted", 0)
            if k > e:
                r.meta["emitted"] = k
                try:
                    r.meta["on_tokens"](src[e:k] if src is not None else outs[s, e:k].tolist())
                except Exception:
                    log.exception("stream callback failed")
        if not finished:
            return []
        now = time.perf_counter()
        reset = []
        done = []
        for s, r in finished:
            done.append(r)
            k = int(nout[s])
            ids = ended[s] if s in ended else outs[s, :min(k, self.cfg.max_out)].tolist()
            stop = bool(ids) and ids[-1] in self.tok.stop_ids
            r.out_ids = r.resume_out + (ids[:-1] if stop else ids)
            r.t_done = now
            del self.running[r.slot]
            reset.append(r.slot)
            self.free_slots.append(r.slot)
            # KV block release, detokenisation and the callback run after the next GPU launch (_flush_deferred): ~60 us
            # per verdict, ~60 ms of host time per 1024-chain wave that the GPU otherwise sat idle for between bursts.
            # The row's slot is reset below, so no launch reads those blocks; they are free again before the next
            # admission (every step flushes its deferred requests before it returns)
            self._deferred.append((r, "stop" if stop else "length"))
        self.free_slots.sort(reverse=True)  # lowest slot first keeps the decode bucket small
        idx = h2d(torch.tensor(reset, dtype=torch.int64), self.device)
        self.s_state.index_fill_(0, idx, -1)
        self.s_bt.index_fill_(0, idx, 0)
        self.s_pos.index_fill_(0, idx, 0)
        self.s_ctx.index_fill_(0, idx, 1)
        self.stats["completed"] += len(done)
        self.stats["generated_tokens"] += sum(len(r.out_ids) for r in done)
        self._compact()
        return []  # reported by _flush_deferred once their text exists

    def _flush_deferred(self) -> list[Request]:
        """Finish the requests the last harvest completed: detokenise, fire callbacks.  Called right after a step's
        GPU work is queued, so this host work overlaps it instead of delaying the next launch."""
        if not self._deferred:
            return []
        out, self._deferred = self._deferred, []
        for r, reason in out:
            self.blocks.release(r.blocks)
            r.blocks = []
            r.text = self.tok.decode(r.out_ids)
            self._finish(r, reason, timed=False)
        return [r for r, _ in out]

    def _note_jump(self, r: Request, n0: int, k: int) -> None:
        r.meta.setdefault("jump_spans", []).append((len(r.resume_out) + n0, k))
        r.meta["jump_seq"] = self._snap_seq  # every snapshot queued so far predates this jump
        self.stats["jumps"] += 1
        self.stats["jump_tokens"] += k

    def _jump(self, parked, st, nout, outs) -> dict:
        """Append the grammar-forced token run of every parked row (sampler.hip parks a row entering a state with a
        run).  Each row's pending token and its run go through ONE prefill-mode forward (paged KV at their positions,
        logits of the last one), then the sampler picks the next token as after a prompt.  A run that ends the verdict
        (through EOS) needs no forward: those rows are returned as {snapshot slot: output ids} to finish now.  A row
        whose budget cannot take the run resumes token by token (unparked).

        Positions: a decoding row's pending token sits at prompt_len + nout - 1 (prefill leaves pos = len - 1 and
        every sampled token adds one to pos and nout), so after the run pos/ctx/nout/remaining all advance by k."""
        ended, unpark, rows = {}, [], []
        for s, r in parked:
            state = -2 - int(st[s])
            run, end = self.bank.jumps.get(state, ((), state))
            n0, k = int(nout[s]), len(run)
            if not run or n0 > self.cfg.max_out or n0 + k > self.cfg.max_out or \
                    r.num_predict - n0 - k < self.bank.min_tokens(end):
                # safety net only: the sampler parks a row only when its budget takes the run (GrammarBank.jump)
                unpark.append((r.slot, state))
                self.stats["jump_refused"] += 1
                continue
            ids = outs[s, :n0].tolist() + list(run)
            if end == DONE:
                self._note_jump(r, n0, k)
                ended[s] = ids
            else:
                rows.append((r, ids, end, n0, k))
        dv = lambda t: h2d(t, self.device)  # noqa: E731
        if unpark:
            self.s_state[dv(torch.tensor([u[0] for u in unpark], dtype=torch.int64))] = dv(
                torch.tensor([u[1] for u in unpark], dtype=torch.int32))
        if rows and self.kv_alloc == "lazy":
            # the forward writes positions pos0 .. pos0 + k: grow (preempting the newest rows if the pool is short)
            self._ensure_kv([(r, len(r.prompt_ids) + n0 + k) for r, _, _, n0, k in rows])
            rows = [x for x in rows if self.running.get(x[0].slot) is x[0]]
        for r, _, _, n0, k in rows:  # (recorded only for rows still running: a preempted row's jump never ran)
            self._note_jump(r, n0, k)
        if not rows:
            return ended
        pos0 = [len(r.prompt_ids) + n0 - 1 for r, _, _, n0, _ in rows]
        # Long contexts: nqt=2, the split-K paged kernel (32 query rows per tile, the KV range split over the chip).
        # The flash prefill kernel (nqt=8) runs one workgroup per (tile, kv head) over the whole context: at 128k
        # that is 8 workgroups streaming 16 GiB of KV per jump (14 ms/token decode instead of 6-7).
        nqt = 2 if max(pos0) > 4096 else self.cfg.prefill_nqt
        sb = make_prefill_batch([ids[n0 - 1:] for _, ids, _, n0, _ in rows], pos0, [r.blocks for r, *_ in rows],
                                self.model.cfg, self.tp, self.device, max_blocks=self.max_blocks_per_seq, nqt=nqt)
        logits = self.model.forward(sb, self.kv)
        i32 = lambda x: dv(torch.tensor(x, dtype=torch.int32))  # noqa: E731
        sl = dv(torch.tensor([r.slot for r, *_ in rows], dtype=torch.int64))
        oi = [(r.slot, n0 + j, t) for r, ids, _, n0, k in rows for j, t in enumerate(ids[n0:])]
        self.s_out[dv(torch.tensor([o[0] for o in oi], dtype=torch.int64)),
                   dv(torch.tensor([o[1] for o in oi], dtype=torch.int64))] = i32([o[2] for o in oi])
        self.s_nout[sl] = i32([n0 + k for _, _, _, n0, k in rows])
        self.s_rem[sl] = i32([r.num_predict - n0 - k for r, _, _, n0, k in rows])
        self.s_pos[sl] = i32([p + k for p, (*_, k) in zip(pos0, rows)])
        self.s_ctx[sl] = i32([p + k + 1 for p, (*_, k) in zip(pos0, rows)])
        self.s_state[sl] = i32([end for _, _, end, _, _ in rows])
        for p, (r, *_, k) in zip(pos0, rows):
            r.pos_hi = p + k + 1  # the run ends at p + k; the sampler's next token is written one past it
        self.s_row.fill_(-1)
        self.s_row[sl] = i32(list(range(len(rows))))
        ops.constrained_sample(logits, self.s_row, self.bank.next, self.bank.dist, DONE, self.s_state, self.s_rem,
                               self.s_temp, self.s_seed, self.s_ids, self.s_pos, self.s_ctx, self.s_nout, self.s_out,
                               self.s_topk, self.s_topp, self._jump_flags(len(self.running)))
        self._check_parked = self._jump_flags(len(self.running)) is not None
        return ended

    def _compact(self) -> None:
        """Move live decode rows into the lowest free slots so the decode bucket (and its captured graph) shrinks as
        verdicts finish: a wave of 1024 chains whose verdicts end at different lengths stops paying for finished
        rows.  Moving a sequence is a copy of its slot state rows; its KV blocks stay where they are."""
        if not self.running:
            return
        n = self._decode_rows()
        target = _bucket(len(self.running))
        if target >= n:
            return
        movers = sorted(r for r in self.running if r >= target)
        dst = sorted(s for s in self.free_slots if s < target)[:len(movers)]
        if len(dst) < len(movers):
            return
        si = h2d(torch.tensor(movers, dtype=torch.int64), self.device)
        di = h2d(torch.tensor(dst, dtype=torch.int64), self.device)
        for t in (self.s_ids, self.s_pos, self.s_ctx, self.s_state, self.s_rem, self.s_nout, self.s_seed, self.s_temp,
                  self.s_topk, self.s_topp, self.s_out, self.s_bt):
            t[di] = t[si]
        self.s_state.index_fill_(0, si, -1)
        self.s_bt.index_fill_(0, si, 0)
        self.s_pos.index_fill_(0, si, 0)
        self.s_ctx.index_fill_(0, si, 1)
        moved = {}
        for s, d in zip(movers, dst):
            r = self.running.pop(s)
            r.slot = d
            moved[d] = r
        self.running.update(moved)
        fs = set(self.free_slots) - set(dst) | set(movers)
        self.free_slots = sorted(fs, reverse=True)
        self.stats["compactions"] += 1

    def _finish(self, req: Request, reason: str, timed: bool = True) -> None:
        if req.orig_plen >= 0:  # preempted at least once: the prompt carried the generated ids while it re-prefilled
            req.prompt_ids = req.prompt_ids[:req.orig_plen]
            req.num_predict = req.meta.pop("orig_num_predict", req.num_predict)
            if not req.out_ids and req.resume_out:
                req.out_ids = list(req.resume_out)
        req.done_reason = reason
        if timed or not req.t_done:
            req.t_done = time.perf_counter()
        if req.callback is not None:
            try:
                req.callback(req)
            except Exception:  # a client callback must never take the engine down
                log.exception("request callback failed")

    def result_json(self, req: Request, model_name: str = "llama3") -> dict:
        """Ollama /api/generate (stream=false) response body."""
        ns = lambda s: int(max(0.0, s) * 1e9)  # noqa: E731
        return {
            "model": model_name,
            "created_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
            "response": req.text,
            "done": True,
            "done_reason": req.done_reason,
            "total_duration": ns(req.t_done - req.t_submit),
            "load_duration": 0,
            "prompt_eval_count": len(req.prompt_ids),
            "prompt_eval_duration": ns((req.t_first or req.t_done) - (req.t_admit or req.t_submit)),
            "eval_count": len(req.out_ids),
            "eval_duration": ns(req.t_done - (req.t_first or req.t_done)),
        }
