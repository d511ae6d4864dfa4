"""Split-K on the vendor library for the under-filled decode projections (M = 256..1024, N = 4096 / 6144): the K range
is cut into S slices computed as ONE batched hipBLASLt GEMM with fp32 output (torch.bmm(..., out_dtype=float32)), so
S x more output tiles fill the 256 CUs; the S partial sums are reduced by the consumer (fused into the residual-add +
RMSNorm pass).  Prints library-GEMM time vs split-K GEMM time (+ a plain torch reduction for reference).

  python scripts/bench_splitk.py [--out gpurun_out/splitk.jsonl]
"""
import argparse
import json
import statistics

import torch


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
    dev = "cuda"
    shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)]
    out = []
    for m in (256, 512, 768, 1024):
        for name, n, k in shapes:
            x = torch.randn(m, k, device=dev).to(torch.bfloat16)
            w = (torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16)
            base = timeit(lambda: torch.matmul(x, w.t()))
            ref = (x.float() @ w.float().t())
            rec = dict(m=m, op=name, n=n, k=k, lib_us=round(base, 1))
            for S in (2, 3, 4, 7, 8):
                if k % S or (k // S) % 64:
                    continue
                xs = x.view(m, S, k // S).permute(1, 0, 2)           # [S, m, k/S] (strided view)
                ws = w.view(n, S, k // S).permute(1, 2, 0)           # [S, k/S, n]
                xs_c, ws_c = xs.contiguous(), ws.contiguous()
                t = timeit(lambda: torch.bmm(xs_c, ws_c, out_dtype=torch.float32))
                parts = torch.bmm(xs_c, ws_c, out_dtype=torch.float32)
                tr = timeit(lambda: parts.sum(0).to(torch.bfloat16))
                err = float((parts.sum(0) - ref).abs().max() / ref.abs().max())
                rec[f"s{S}_us"] = round(t, 1)
                rec[f"s{S}_reduce_us"] = round(tr, 1)
                rec[f"s{S}_relerr"] = round(err, 5)
            best = min((rec[f"s{S}_us"], S) for S in (2, 3, 4, 7, 8) if f"s{S}_us" in rec)
            rec["best_S"], rec["best_us"] = best[1], best[0]
            rec["speedup_gemm_only"] = round(base / best[0], 3)
            out.append(rec)
            print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
