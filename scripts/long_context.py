"""BASELINE config 5: a 128k-token kill-chain context window (Llama-3.1-8B rope scaling, paged KV, chunked prefill,
optional fp8-e4m3 KV) on one MI355X.

Builds one CHRONOS prompt whose chain history holds thousands of syscall events (~--tokens tokens), prefills it in
--chunk-token pieces that attend to the growing paged prefix (flash prefill kernel), then decodes a schema-constrained
verdict with split-K decode attention over the full context.  Prints one JSON line: TTFT, prefill tokens/s, decode
ms/token, KV bytes.

  python scripts/long_context.py --tokens 131000 --kv-dtype fp8
  torchrun --nproc-per-node 8 scripts/long_context.py --cp 8      # context-parallel prefill over 8 GPUs (xGMI)

With ``--cp W`` (launched by torch.distributed.run, one rank per GPU) every rank holds the full model and the 16k-token
prefill chunks become W*16k-token context-parallel chunks: each rank projects and attends its zigzag share and the
K/V are all-gathered per layer over RCCL (parallel/context_parallel.py); rank 0 prints the JSON line.
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
    ap.add_argument("--weights", default="bf16", choices=["bf16", "fp8"],
                    help="fp8: W8A8 e4m3 projections on the block-scaled MFMA (the config's 'CDNA4 fp8 MFMA')")
    ap.add_argument("--chunk", type=int, default=16384)
    ap.add_argument("--num-predict", type=int, default=64)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--cp", type=int, default=1, help="context-parallel ranks (torch.distributed.run)")
    ap.add_argument("--repeat", type=int, default=1, help="run the long request this many times (first = cold)")
    ap.add_argument("--no-jump-forward", action="store_true")
    ap.add_argument("--knob", action="append", default=[], help="kernel knob name=value (torch.ops.chronos.set_knob)")
    a = ap.parse_args()
    from chronos.brain.engine.engine import Engine, EngineConfig
    from chronos.parallel.tp import TPContext

    cp = None
    if a.cp > 1:
        import torch.distributed as dist

        if a.device == "cuda":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl" if a.device == "cuda" else "gloo")
        cp = TPContext.from_group()
        assert cp.world == a.cp, f"--cp {a.cp} but world size {cp.world}"
    from chronos.sensor.prompt import VERDICT_SCHEMA, build_prompt
    from chronos.sensor.replay import synthetic_chains

    eng = Engine(EngineConfig(model=a.model, device=a.device, max_slots=1, max_model_len=131072,
                              max_prefill_tokens=a.chunk, kv_dtype=a.kv_dtype, decode_burst=8, prefix_cache=False,
                              cp_min_tokens=min(4096, a.chunk), weight_dtype=a.weights,
                              jump_forward=not a.no_jump_forward),
                 cp=cp)
    for kv in a.knob:
        name, val = kv.split("=")
        torch.ops.chronos.set_knob(name, int(val))
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
    sync = torch.cuda.synchronize if a.device == "cuda" else (lambda: None)
    for rep in range(a.repeat):
        sync()
        t0 = time.perf_counter()
        req = eng.submit(ids, fmt=VERDICT_SCHEMA, num_predict=a.num_predict)
        while not req.t_first and not req.done_reason:
            eng.step()
            print(f"[long] prefilled {req.prefilled}/{len(ids)} at {time.perf_counter() - t0:.1f}s", file=sys.stderr,
                  flush=True)
        if req.error:
            raise SystemExit(f"request failed: {req.error}")
        sync()
        ttft = time.perf_counter() - t0
        eng.run_until_idle()
        sync()
        total = time.perf_counter() - t0
        v = json.loads(req.text)
        kv_bytes = eng.kv.buf.numel() * eng.kv.buf.element_size()
        if cp is not None and cp.rank != 0:
            continue
        print(json.dumps({
            "config": "128k-token kill-chain context", "model": a.model, "kv_dtype": a.kv_dtype,
            "weights": a.weights, "cp": a.cp,
            "run": rep, "prompt_tokens": len(ids), "ttft_s": round(ttft, 3),
            "prefill_tokens_per_s": round(len(ids) / ttft, 1), "verdict_tokens": len(req.out_ids),
            "decode_ms_per_token": round(1000 * (total - ttft) / max(1, len(req.out_ids)), 2),
            "kv_cache_gib": round(kv_bytes / 2**30, 2), "verdict_keys": sorted(v),
        }), flush=True)


if __name__ == "__main__":
    main()
