"""BASELINE config 5: a 128k-token kill-chain context window (Llama-3.1-8B rope scaling, paged KV, chunked prefill,
optional fp8-e4m3 KV) on one MI355X.

Builds one CHRONOS prompt whose chain history holds thousands of syscall events (~--tokens tokens), prefills it in
--chunk-token pieces that attend to the growing paged prefix (flash prefill kernel), then decodes a schema-constrained
verdict with split-K decode attention over the full context.  Prints one JSON line: TTFT, prefill tokens/s, decode
ms/token, KV bytes.

  python scripts/long_context.py --tokens 131000 --kv-dtype fp8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--tokens", type=int, default=131000)
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--chunk", type=int, default=16384)
    ap.add_argument("--num-predict", type=int, default=64)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    eng = Engine(EngineConfig(model=a.model, device=a.device, max_slots=1, max_model_len=131072,
                              max_prefill_tokens=a.chunk, kv_dtype=a.kv_dtype, decode_burst=8, prefix_cache=False))
    # a very long chain: concatenated fleet histories (one process tree that never triggered a reset)
    hist = []
    for c in synthetic_chains(6000, seed=42):
        hist += c.history
    ids = eng.tok.chat_ids(build_prompt(hist))
    while len(ids) < a.tokens:
        hist = hist + hist
        ids = eng.tok.chat_ids(build_prompt(hist))
    # trim the history to the target length (keep the template tail intact)
    lo, hi = 1, len(hist)
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if len(eng.tok.chat_ids(build_prompt(hist[:mid]))) <= a.tokens:
            lo = mid
        else:
            hi = mid - 1
    ids = eng.tok.chat_ids(build_prompt(hist[:lo]))
    print(f"[long] prompt {len(ids)} tokens, {lo} events", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    req = eng.submit(ids, fmt=VERDICT_SCHEMA, num_predict=a.num_predict)
    while not req.t_first:
        eng.step()
        print(f"[long] prefilled {req.prefilled}/{len(ids)} at {time.perf_counter() - t0:.1f}s", file=sys.stderr,
              flush=True)
    torch.cuda.synchronize()
    ttft = time.perf_counter() - t0
    eng.run_until_idle()
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    v = json.loads(req.text)
    kv_bytes = eng.kv.buf.numel() * eng.kv.buf.element_size()
    print(json.dumps({
        "config": "128k-token kill-chain context", "model": a.model, "kv_dtype": a.kv_dtype,
        "prompt_tokens": len(ids), "ttft_s": round(ttft, 3), "prefill_tokens_per_s": round(len(ids) / ttft, 1),
        "verdict_tokens": len(req.out_ids), "decode_ms_per_token": round(1000 * (total - ttft) / max(1, len(req.out_ids)), 2),
        "kv_cache_gib": round(kv_bytes / 2**30, 2), "verdict_keys": sorted(v),
    }), flush=True)


if __name__ == "__main__":
    main()
