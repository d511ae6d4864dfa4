"""hipBLASLt by weight layout / decomposition on the Llama-3-8B projection shapes (one MI355X, random data, weights
rotated over >= 1 GiB of copies so decode-sized calls meet them cold, variants interleaved in one process).

  nt      x @ W^T with W stored [N, K] (the HF layout, what models/llama.py uses)
  nn      x @ Wt  with Wt stored [K, N] (transposed once at load)
  split4  x @ W^T as 4 column blocks of W (N/4 each) written into one output (gate_up only)
  python scripts/bench_gemm_layout.py --ms 1024,16384 --out gpurun_out/gemm_layout.json
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
          ("lm_head", 128256, 4096)]


def timeit(fn, iters=10, rounds=5):
    for _ in range(2):
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
    ap.add_argument("--ms", default="512,1024,2048,16384")
    ap.add_argument("--ops", default="qkv,o,gate_up,down,lm_head")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = "cuda"
    out = []
    for name, n, k in SHAPES:
        if name not in a.ops.split(","):
            continue
        ncopy = max(2, -(-2**30 // (n * k * 2)))
        ws = [(torch.rand(n, k, device=dev) * 0.04 - 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        wts = [w.t().contiguous() for w in ws]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % ncopy
            return it[0]

        for m in [int(x) for x in a.ms.split(",")]:
            if name == "lm_head" and m > 2048:
                continue
            x = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
            y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
            ref = torch.matmul(x, ws[0].t())
            assert torch.equal(torch.matmul(x, wts[0]), ref) or \
                float((torch.matmul(x, wts[0]).float() - ref.float()).abs().max()) < 1e-2 * float(ref.abs().max())
            var = {
                "nt": lambda: torch.matmul(x, ws[nxt()].t(), out=y),
                "nn": lambda: torch.matmul(x, wts[nxt()], out=y),
            }
            if name == "gate_up":
                def split4():
                    i = nxt()
                    q = n // 4
                    for j in range(4):
                        torch.matmul(x, ws[i][j * q:(j + 1) * q].t(), out=y[:, j * q:(j + 1) * q])
                var["split4"] = split4
            ts = {kk: [] for kk in var}
            for _ in range(3):
                for kk, fn in var.items():
                    ts[kk].append(timeit(fn))
            t = {kk: statistics.median(v) for kk, v in ts.items()}
            flop = 2 * m * n * k
            rec = dict(op=name, m=m, n=n, k=k, **{f"{kk}_us": round(v, 1) for kk, v in t.items()},
                       **{f"{kk}_TF": round(flop / v / 1e6, 1) for kk, v in t.items()})
            out.append(rec)
            print(json.dumps(rec), flush=True)
        del ws, wts
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
