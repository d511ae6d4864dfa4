"""Does hipBLASLt / rocBLAS hold faster solutions than the default heuristic pick for the wave's library GEMMs?
Times y = x @ w.T (bf16) per shape with TunableOp off, then tunes it (TunableOp searches the hipBLASLt + rocBLAS
solutions) and times the tuned pick, cold weights (rotating copies).  Prints one JSON line per shape.

    python scripts/tunableop_probe.py --out gpurun_out/tunableop.jsonl
"""
import argparse
import json
import os

import torch

SHAPES = [("qkv", 16384, 6144, 4096), ("o", 16384, 4096, 4096), ("gate_up", 16384, 28672, 4096),
          ("down", 16384, 4096, 14336), ("qkv", 1024, 6144, 4096), ("gate_up", 2048, 28672, 4096),
          ("qkv", 8192, 6144, 4096)]


def bench(fn, iters=10, rounds=3):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(rounds):
        fn(0)
        torch.cuda.synchronize()
        st.record()
        for i in range(iters):
            fn(i)
        en.record()
        torch.cuda.synchronize()
        best = min(best, st.elapsed_time(en) * 1000 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--file", default="/tmp/tunableop_probe.csv")
    a = ap.parse_args()
    rows = []
    for name, m, n, k in SHAPES:
        ncopy = max(2, -(-(600 << 20) // (n * k * 2)))
        ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        fn = lambda i: x @ ws[i % ncopy].t()  # noqa: E731
        torch.cuda.tunable.enable(False)
        base = bench(fn)
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_filename(a.file)
        torch.cuda.tunable.set_max_tuning_duration(400)
        fn(0)  # tunes this (M, N, K)
        torch.cuda.synchronize()
        torch.cuda.tunable.tuning_enable(False)
        tuned = bench(fn)
        torch.cuda.tunable.enable(False)
        r = dict(op=name, m=m, n=n, k=k, default_us=round(base, 2), tuned_us=round(tuned, 2),
                 speedup=round(base / tuned, 3), TF_tuned=round(2 * m * n * k / tuned / 1e6, 1))
        rows.append(r)
        print(json.dumps(r), flush=True)
        del ws
        torch.cuda.empty_cache()
    res = torch.cuda.tunable.get_results()
    print("results:", len(res))
    for e in res:
        print("  ", e)
    if a.out:
        with open(a.out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
