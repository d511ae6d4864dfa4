"""Closed-loop sensor-fleet load generator for a running Brain.

N concurrent sensor streams, each a loop: take the next synthetic syscall chain (kernel filter -> chain tracker ->
reference prompt template), POST it to /api/generate exactly as the reference sensor does
(chronos_sensor.py:117-119, via sensor.client.AsyncBrainClient), wait for the verdict, repeat.  After a warm-up
window, chains completed in the measurement window give chains/s; per-chain wall latency gives p50/p99.  ERROR
verdicts (timeouts, HTTP errors, bad JSON) are counted separately, never as analysed chains.

  python -m chronos.brain.api --model llama3-8b --max-slots 1024 &      # or any Ollama-compatible Brain
  python scripts/loadgen.py --url http://127.0.0.1:11434/api/generate --streams 1,64,1024 --duration 30
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


async def run_level(url: str, streams: int, duration: float, warmup: float, schema: bool, num_predict: int,
                    seed: int) -> dict:
    from chronos.sensor.client import AsyncBrainClient, ClientConfig, schema_format
    from chronos.sensor.replay import synthetic_chains

    chains = synthetic_chains(max(256, 4 * streams), seed=seed, native=False)
    cfg = ClientConfig(url=url, fmt=schema_format() if schema else "json", timeout=max(30.0, duration * 2),
                       options={"num_predict": num_predict})
    client = AsyncBrainClient(cfg, max_inflight=streams)
    t_start = time.perf_counter()
    t_meas0 = t_start + warmup
    t_end = t_meas0 + duration
    lat: list[float] = []
    ok = err = 0

    async def stream(i: int):
        nonlocal ok, err
        k = i
        while True:
            t0 = time.perf_counter()
            if t0 >= t_end:
                return
            v = await client.analyze(chains[k % len(chains)].history)
            t1 = time.perf_counter()
            k += streams
            if t0 >= t_meas0 and t1 <= t_end:  # chains entirely inside the measurement window
                if v.get("verdict") == "ERROR":
                    err += 1
                else:
                    ok += 1
                    lat.append(t1 - t0)

    await asyncio.gather(*(stream(i) for i in range(streams)))
    await client.close()
    lat.sort()
    return {"streams": streams, "duration_s": duration, "chains": ok, "errors": err,
            "chains_per_s": round(ok / duration, 3),
            "p50_latency_ms": round(1000 * statistics.median(lat), 1) if lat else None,
            "p99_latency_ms": round(1000 * lat[max(0, -(-99 * len(lat) // 100) - 1)], 1) if lat else None}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="http://127.0.0.1:11434/api/generate")
    ap.add_argument("--streams", default="1,64,1024", help="comma list of concurrency levels (1 -> 1024)")
    ap.add_argument("--duration", type=float, default=30.0)
    ap.add_argument("--warmup", type=float, default=5.0)
    ap.add_argument("--num-predict", type=int, default=64)
    ap.add_argument("--json-mode", action="store_true", help='format "json" (reference) instead of the schema')
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None, help="append one JSON line per level")
    a = ap.parse_args(argv)
    for n in [int(s) for s in a.streams.split(",")]:
        rec = asyncio.run(run_level(a.url, n, a.duration, a.warmup, not a.json_mode, a.num_predict, a.seed))
        print(json.dumps(rec), flush=True)
        if a.out:
            with open(a.out, "a") as fh:
                fh.write(json.dumps(rec) + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
