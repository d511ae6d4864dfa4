"""Brain observability: Prometheus text metrics + per-request JSONL records.

The reference had only print() (chronos_sensor.py:100,108,143-155).  Exposed at GET /metrics:
chains (requests) completed, verdict latency / TTFT histograms, generated tokens and tokens/s, engine step time,
batch size, queue depth, KV block usage, and the engine's own counters (prefix-cache hit tokens, prefill / decode steps,
decode row-steps, jumps, compactions, timeouts, cancellations) as ``chronos_engine_<name>_total``.  The engine never
preempts (a request's KV blocks are reserved at admission), so ``chronos_preemptions_total`` stays 0 by design.
"""
from __future__ import annotations

import json
import threading
import time


class _Hist:
    BUCKETS = (0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, float("inf"))

    def __init__(self):
        self.counts = [0] * len(self.BUCKETS)
        self.sum = 0.0
        self.n = 0

    def observe(self, v: float) -> None:
        for i, b in enumerate(self.BUCKETS):
            if v <= b:
                self.counts[i] += 1
        self.sum += v
        self.n += 1

    def lines(self, name: str) -> list[str]:
        out = []
        for b, c in zip(self.BUCKETS, self.counts):
            le = "+Inf" if b == float("inf") else repr(b)
            out.append(f'{name}_bucket{{le="{le}"}} {c}')
        out += [f"{name}_sum {self.sum}", f"{name}_count {self.n}"]
        return out


class Metrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.reset()
        self.jsonl_path: str | None = None

    def reset(self) -> None:
        self.requests = 0
        self.errors = 0
        self.gen_tokens = 0
        self.prompt_tokens = 0
        self.latency = _Hist()
        self.ttft = _Hist()
        self.step = _Hist()
        self.running = 0
        self.waiting = 0
        self.kv_usage = 0.0
        self.engine_stats: dict = {}
        self.t0 = time.time()

    def observe_request(self, r) -> None:
        with self._lock:
            self.requests += 1
            self.errors += int(r.done_reason == "error")
            self.gen_tokens += len(r.out_ids)
            self.prompt_tokens += len(r.prompt_ids)
            self.latency.observe(r.t_done - r.t_submit)
            if r.t_first:
                self.ttft.observe(r.t_first - r.t_submit)
        if self.jsonl_path:
            rec = dict(rid=r.rid, prompt_tokens=len(r.prompt_ids), gen_tokens=len(r.out_ids), reason=r.done_reason,
                       latency=r.t_done - r.t_submit, ttft=(r.t_first - r.t_submit) if r.t_first else None)
            with open(self.jsonl_path, "a") as fh:
                fh.write(json.dumps(rec) + "\n")

    def observe_step(self, seconds: float, engine) -> None:
        with self._lock:
            self.step.observe(seconds)
            self.running = len(engine.running)
            self.waiting = len(engine.waiting) + len(getattr(engine, "prefilling", ()))
            self.kv_usage = engine.blocks.usage()
            stats = getattr(engine, "stats", None)
            if stats:
                self.engine_stats = {k: v for k, v in stats.items() if isinstance(v, (int, float))}

    def render(self) -> str:
        with self._lock:
            up = max(1e-9, time.time() - self.t0)
            lines = [
                "# TYPE chronos_requests_total counter", f"chronos_requests_total {self.requests}",
                "# TYPE chronos_request_errors_total counter", f"chronos_request_errors_total {self.errors}",
                "# TYPE chronos_generated_tokens_total counter", f"chronos_generated_tokens_total {self.gen_tokens}",
                "# TYPE chronos_prompt_tokens_total counter", f"chronos_prompt_tokens_total {self.prompt_tokens}",
                "# TYPE chronos_chains_per_second gauge", f"chronos_chains_per_second {self.requests / up}",
                "# TYPE chronos_generated_tokens_per_second gauge",
                f"chronos_generated_tokens_per_second {self.gen_tokens / up}",
                "# TYPE chronos_running_sequences gauge", f"chronos_running_sequences {self.running}",
                "# TYPE chronos_queued_requests gauge", f"chronos_queued_requests {self.waiting}",
                "# TYPE chronos_preemptions_total counter", "chronos_preemptions_total 0",
                "# TYPE chronos_kv_usage_ratio gauge", f"chronos_kv_usage_ratio {self.kv_usage}",
                "# TYPE chronos_verdict_latency_seconds histogram", *self.latency.lines("chronos_verdict_latency_seconds"),
                "# TYPE chronos_ttft_seconds histogram", *self.ttft.lines("chronos_ttft_seconds"),
                "# TYPE chronos_engine_step_seconds histogram", *self.step.lines("chronos_engine_step_seconds"),
            ]
            for k in sorted(self.engine_stats):
                name = "chronos_engine_" + "".join(c if c.isalnum() else "_" for c in k) + "_total"
                lines += [f"# TYPE {name} counter", f"{name} {self.engine_stats[k]}"]
        return "\n".join(lines) + "\n"


METRICS = Metrics()
