"""Hand-written MFMA GEMM (csrc/kernels/gemm.hip) vs hipBLASLt (torch.matmul) on the Llama-3-8B projection shapes.

Weights rotate over copies totalling >= 1 GiB (each decode layer meets its weights cold: 32 layers x 218 MB exceed
the 256 MB Infinity Cache); variants are interleaved in one process; median of rounds; random data.  Also checks
each kernel against an fp32 reference once per shape.
  python scripts/bench_gemm.py --ms 64,256,1024 --out gpurun_out/gemm.json
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
    ap.add_argument("--ms", default="64,128,256,512,768,1024,2048,16384")
    ap.add_argument("--ops", default="qkv,o,gate_up,down,lm_head")
    ap.add_argument("--stages", default="2,3,4")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from chronos import ops

    ops.load()
    C = torch.ops.chronos
    dev = "cuda"
    stages = [int(s) for s in a.stages.split(",")]
    out = []
    for name, n, k in SHAPES:
        if name not in a.ops.split(","):
            continue
        ncopy = max(2, -(-2**30 // (n * k * 2)))
        ws = [(torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % ncopy
            return ws[it[0]]

        sw = name == "gate_up"
        for m in [int(x) for x in a.ms.split(",")]:
            if name == "lm_head" and m > 2048:
                continue
            x = torch.randn(m, k, device=dev).to(torch.bfloat16)
            # correctness vs fp32
            w0 = ws[0]
            ref = x.float() @ w0.float().t()
            if sw:
                f = n // 2
                g, u = ref[:, :f].bfloat16().float(), ref[:, f:].bfloat16().float()
                ref = (torch.nn.functional.silu(g).bfloat16().float() * u)
            err = {}
            for s in stages:
                y = C.gemm(x, w0, sw, s).float()
                err[s] = float((y - ref).abs().max() / ref.abs().max())
            if sw:
                lib = lambda: C.silu_mul(torch.matmul(x, nxt().t()))  # noqa: E731
            else:
                lib = lambda: torch.matmul(x, nxt().t())  # noqa: E731
            t_lib = timeit(lib)
            t = {s: timeit(lambda s=s: C.gemm(x, nxt(), sw, s)) for s in stages}
            flop = 2 * m * n * k
            best = min(t, key=t.get)
            rec = dict(op=name, m=m, n=n, k=k, hipblaslt_us=round(t_lib, 1),
                       **{f"hip_s{s}_us": round(v, 1) for s, v in t.items()},
                       hipblaslt_TF=round(flop / t_lib / 1e6, 1), hip_best_TF=round(flop / t[best] / 1e6, 1),
                       best_stages=best, speedup=round(t_lib / t[best], 3),
                       max_rel_err=max(err.values()))
            out.append(rec)
            print(json.dumps(rec), flush=True)
        del ws
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
