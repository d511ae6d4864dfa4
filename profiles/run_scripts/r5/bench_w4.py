"""A/B of the experimental one-wave-per-SIMD GEMM (csrc/microbench/gemm_w4.hip) against hipBLASLt (torch.matmul) and
the production gemm_lg configs, interleaved in one process (cdna_hip_programming.md §5.4 rule 24), random operands.

    python scripts/r5/bench_w4.py --lib build/w4/libgemm_w4.so [--vars 4,5,12,13] [--shapes big|decode|all]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="build/w4/libgemm_w4.so")
    ap.add_argument("--vars", default="4,5,12,13")
    ap.add_argument("--lg", default="20", help="production gemm_lg configs to include (plain mode)")
    ap.add_argument("--shapes", default="all")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--gm", type=int, default=8)
    ap.add_argument("--gms", default="", help="also time every w4 variant at these tile-group sizes")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.abspath(a.lib))
    lib.gemm_w4.restype = ctypes.c_int
    lib.gemm_w4.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 5 + [ctypes.c_void_p]
    use_lg = bool(a.lg)
    if use_lg:
        from chronos import ops

        ops.load()
    dev = "cuda"
    if a.shapes == "sq":
        big = [(8192, 8192, 8192), (16384, 28672, 4096)]
    else:
        big = [(8192, 8192, 8192), (16384, 6144, 4096), (16384, 4096, 4096), (16384, 28672, 4096), (16384, 4096, 14336)]
    dec = [(1024, 6144, 4096), (1024, 4096, 4096), (1024, 28672, 4096), (1024, 4096, 14336), (1024, 128256, 4096)]
    shapes = {"big": big, "sq": big, "decode": dec, "all": big + dec}[a.shapes]
    vars_ = [int(v) for v in a.vars.split(",") if v]
    lgs = [int(v) for v in a.lg.split(",") if v]
    g = torch.Generator(device=dev).manual_seed(0)
    rows = []
    for (M, N, K) in shapes:
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        nw = max(1, min(4, int(2e9 // (N * K * 2))))  # rotate weight copies (cold-ish weights)
        ws = [((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(nw)]
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        st = torch.cuda.current_stream().cuda_stream
        ref = (x.float() @ ws[0].float().t())
        fns = {"lib": lambda w: torch.matmul(x, w.t())}
        gms = [a.gm] + [int(q) for q in a.gms.split(",") if q]
        for v in vars_:
            for gmv in gms:
                def f(w, v=v, gmv=gmv):
                    rc = lib.gemm_w4(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, N, K, v, gmv, st)
                    assert rc == 0, rc
                    return y
                fns[f"w4v{v}" + (f"g{gmv}" if gmv != a.gm else "")] = f
        for c in lgs:
            fns[f"lg{c}"] = lambda w, c=c: torch.ops.chronos.gemm_pp(x, w, 0, c, 1, None, None, 1e-5, False)[0]
        errs = {}
        for name, fn in fns.items():
            out = fn(ws[0]).float()
            errs[name] = float((out - ref).abs().max() / ref.abs().max())
        times = {k: [] for k in fns}
        for _ in range(a.rounds):
            for name, fn in fns.items():
                for i in range(2):
                    fn(ws[i % nw])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(a.iters):
                    fn(ws[i % nw])
                e1.record()
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) * 1000 / a.iters)
        row = {"M": M, "N": N, "K": K}
        for name in fns:
            t = statistics.median(times[name])
            row[name] = {"us": round(t, 1), "tflops": round(2 * M * N * K / t / 1e6, 1), "err": round(errs[name], 5),
                         "min_us": round(min(times[name]), 1)}
        row["best_own_vs_lib"] = round(row["lib"]["us"] / min(row[n]["us"] for n in fns if n != "lib"), 3)
        print(json.dumps(row), flush=True)
        rows.append(row)
        del x, ws, y, ref
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
