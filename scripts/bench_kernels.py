"""Kernel micro-benchmarks on one MI355X (interleaved rounds in one process, median of N; random data).

Reports achieved HBM bandwidth / TFLOP/s of the hand-written kernels next to the vendor-library (hipBLASLt) path on
the Llama-3-8B decode / prefill shapes.  Usage: python scripts/bench_kernels.py [--out profiles/kernels.json]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, rounds=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters * 1e3)
    return statistics.median(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from chronos import ops
    from chronos.ops import gemm

    ops.load()
    dev = "cuda"
    out = {"gemv": [], "attention_decode": []}
    shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
              ("lm_head", 128256, 4096)]
    for m in (1, 2, 4, 8):
        for name, n, k in shapes:
            x = torch.randn(m, k, device=dev).to(torch.bfloat16)
            # cold weights: rotate over copies totalling >= 1 GiB so the 256 MiB Infinity Cache cannot serve them
            ncopy = max(1, -(-2**30 // (n * k * 2)))
            ws = [(torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % ncopy
                return ws[it[0]]

            t_h = timeit(lambda: gemm._gemv(x, nxt(), name == "gate_up"))
            t_b = timeit(lambda: torch.matmul(x, nxt().t()))
            del ws
            by = n * k * 2
            rec = dict(m=m, op=name, n=n, k=k, hip_us=round(t_h, 2), hipblaslt_us=round(t_b, 2),
                       hip_TBps=round(by / t_h / 1e6, 3), hipblaslt_TBps=round(by / t_b / 1e6, 3))
            out["gemv"].append(rec)
            print(json.dumps(rec), flush=True)
    # decode attention over the paged cache (8B shapes), KV bytes / time
    for B, ctx in ((1, 2048), (256, 160), (1024, 160), (16, 8192)):
        hq, hkv, bs = 32, 8, 16
        nbs = (ctx + bs - 1) // bs
        k = torch.randn(B * nbs + 1, hkv, bs, 128, device=dev).to(torch.bfloat16)
        v = torch.randn(B * nbs + 1, hkv, 128, bs, device=dev).to(torch.bfloat16)
        bt = torch.arange(B * nbs, device=dev, dtype=torch.int32).view(B, nbs)
        q = torch.randn(B, hq, 128, device=dev).to(torch.bfloat16)
        qs = torch.arange(B + 1, device=dev, dtype=torch.int32)
        cl = torch.full((B,), ctx, device=dev, dtype=torch.int32)
        ns = ops.pick_nsplit(B * hkv, ctx)
        t = timeit(lambda: ops.paged_attention(q, k, v, bt, qs, cl, None, B, 1, ns))
        by = B * ctx * hkv * 128 * 2 * 2
        rec = dict(batch=B, ctx=ctx, nsplit=ns, us=round(t, 2), TBps=round(by / t / 1e6, 3))
        out["attention_decode"].append(rec)
        print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
