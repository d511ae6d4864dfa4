"""Per-tile fixed cost vs per-slab cost of the 256 x 256 large-M kernels: time(K) at M = 16384, N = 4096 (1024 tiles =
4 rounds on 256 CUs) for K = 1024 .. 14336, fit t = rounds * (a + b * slabs).  Kernels: gemm_lg fp8 config 4 (F8HB),
hipBLASLt's fp8 GEMM (torch._scaled_mm), gemm_lg bf16 config 88 (HB) and hipBLASLt bf16.

  python scripts/f8hb_fixed_cost.py [--out gpurun_out/f8hb_fixed_cost.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t_us(fn, iters=10, rounds=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / iters * 1e3)
    return statistics.median(out)


def fit(ks, ts, per_slab_k):
    xs = [k / per_slab_k for k in ks]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ts) / n
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ts)) / sum((x - mx) ** 2 for x in xs)
    return my - b * mx, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--ks", default="1024,2048,4096,8192,14336")
    ap.add_argument("--out", default=None)
    ap.add_argument("--f8cfgs", default="4")
    ap.add_argument("--bfcfgs", default="88")
    a = ap.parse_args()
    from chronos import ops
    from chronos.ops import gemm as G

    ops.load()
    C = torch.ops.chronos
    dev = "cuda"
    m, n = a.m, a.n
    rounds = (-(-m // 256)) * (-(-n // 256)) / 256
    f8 = torch.float8_e4m3fn
    ks = [int(v) for v in a.ks.split(",")]
    res = {}
    g = torch.Generator(device=dev).manual_seed(0)
    for k in ks:
        xq = ((torch.rand(m, k, device=dev, generator=g) * 2 - 1) * 200).to(f8).view(torch.uint8)
        xs = torch.rand(m, device=dev, generator=g) * 1e-2 + 1e-3
        wq = ((torch.rand(n, k, device=dev, generator=g) * 2 - 1) * 200).to(f8).view(torch.uint8)
        ws = torch.rand(n, device=dev, generator=g) * 1e-3 + 1e-4
        x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        fns = {"f8_lib": lambda: ops._qlib(xq, xs, wq, ws), "bf16_lib": lambda: x @ w.t()}
        for c in (int(v) for v in a.f8cfgs.split(",") if v):
            fns[f"f8_lg{c}"] = (lambda c_: lambda: C.qgemm_lg(xq, xs, wq, ws, False, c_, 1))(c)
        for c in (int(v) for v in a.bfcfgs.split(",") if v):
            fns[f"bf16_lg{c}"] = (lambda c_: lambda: G.pp_gemm(x, w, 0, (c_, 1)))(c)
        rec = {"M": m, "N": n, "K": k}
        for name, fn in fns.items():
            us = t_us(fn)
            rec[name] = round(us, 1)
            res.setdefault(name, []).append(us)
        print(json.dumps(rec), flush=True)
        if a.out:
            with open(a.out, "a") as fh:
                fh.write(json.dumps(rec) + "\n")
        del xq, wq, x, w
    for name, ts in res.items():
        slab_k = 128 if name.startswith("f8") else 64
        a0, b0 = fit(ks, [t / rounds for t in ts], slab_k)
        rec = {"kernel": name, "per_round_fixed_us": round(a0, 2), "per_slab_us": round(b0, 4),
               "slab_k": slab_k, "rounds": rounds}
        print(json.dumps(rec), flush=True)
        if a.out:
            with open(a.out, "a") as fh:
                fh.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
