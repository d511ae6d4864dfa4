"""Time one decode forward of a T-row bucket (Llama-3-8B bf16, random weights, ~200-token verdict contexts) the way
the engine runs it: a captured hipGraph of the forward, replayed; prints ms per forward and, with --prof, leaves the
kernels to rocprofv3.  VERDICT r4 item 5 measures the T = 128 bucket (the 70B-TP8 decode shape class).

    python scripts/fw_bucket.py --rows 128 [--model llama3-8b] [--ctx 200] [--iters 20]
    python scripts/fw_bucket.py --model llama3-70b --tp-rank-of 8 --rows 256     # one rank of 70B TP=8

``--tp-rank-of W`` builds rank 0's shard of a W-way tensor-parallel model (column-parallel QKV / gate_up / LM head,
row-parallel O / down: the plan's TP-shard GEMM shapes, 1/W of the heads for attention) on one GPU and replaces the
collectives by their local part (all-reduce = identity, the fused all-reduce + residual + RMSNorm = the local add +
RMSNorm, the logits all-gather = the rank's vocab shard): the per-rank compute of a TP decode step without xGMI.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_tp(world: int):
    """Rank 0 of a ``world``-way TP job with its collectives reduced to their local part (see module docstring)."""
    from chronos.parallel.tp import TPContext

    class RankTP(TPContext):
        def all_reduce(self, x):
            return x

        def all_reduce_async(self, x):
            return x, None

        def all_gather_last(self, x):
            return x

        def broadcast_obj(self, obj, src=0):
            return obj

    return RankTP(rank=0, world=world)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--rows", type=int, default=128)
    ap.add_argument("--ctx", type=int, default=200)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--weights", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--knob", action="append", default=[], help="kernel knob name=value (torch.ops.chronos.set_knob)")
    ap.add_argument("--tp-rank-of", type=int, default=1, help="W > 1: one rank of a W-way TP model, local collectives")
    a = ap.parse_args()
    from chronos import ops
    from chronos.models.llama import KVCache, StepBatch, build_model

    ops.load()
    for kv_ in a.knob:
        name, val = kv_.split("=")
        torch.ops.chronos.set_knob(name, int(val))
    dev = torch.device("cuda")
    tp = rank_tp(a.tp_rank_of) if a.tp_rank_of > 1 else None
    m = build_model(a.model, dev, tp=tp, weight_dtype=a.weights)
    n, bs = a.rows, 16
    nbs = (a.ctx + 1 + bs - 1) // bs
    kv = KVCache(m.cfg, m.tp, n * nbs + 1, bs, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    kv.buf.normal_(0, 0.5, generator=g)
    it = lambda v: torch.tensor(v, dtype=torch.int32, device=dev)  # noqa: E731
    bt = (torch.arange(n * nbs, dtype=torch.int32, device=dev) + 1).view(n, nbs)
    ctx = it([a.ctx - (i % 7) for i in range(n)])
    ar = torch.arange(n + 1, dtype=torch.int32, device=dev)
    sb = StepBatch(torch.randint(0, m.cfg.vocab_size, (n,), dtype=torch.int32, device=dev), ctx - 1, ar[:n], bt, ar,
                   ctx, torch.arange(n, dtype=torch.int64, device=dev), None, n, 1,
                   ops.pick_nsplit(n * m.hkv, a.ctx + 1))
    for _ in range(3):
        m.forward(sb, kv)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        m.forward(sb, kv)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        graph.replay()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    wbytes = m.w.nbytes()
    print(json.dumps({"model": a.model, "tp_rank_of": a.tp_rank_of, "weights": a.weights, "rows": n, "ctx": a.ctx,
                      "knobs": a.knob,
                      "ms_per_forward": round(ms, 3),
                      "weight_GB": round(wbytes / 1e9, 2), "weight_stream_TBps": round(wbytes / ms / 1e9, 2)}))


if __name__ == "__main__":
    main()
