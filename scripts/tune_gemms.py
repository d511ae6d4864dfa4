"""Tune the vendor-library GEMMs the Brain issues (hipBLASLt / rocBLAS via PyTorch TunableOp) and report gains.

The projection GEMMs that stay on the vendor library are the batched ones (decode buckets M >= 4, prefill chunks);
M <= 2 goes to the hand-written GEMV.  TunableOp benchmarks every library solution for each (M, N, K) once and
writes the winners to a CSV that later runs load (PYTORCH_TUNABLEOP_FILENAME), so serving never tunes online.

  python scripts/tune_gemms.py --out assets/tunableop_mi355x.csv

Measured on MI355X (profiles/r1s4_tunableop_gemm_study.jsonl): the library's default choice is within a few percent at
the wave's M = 1024 decode bucket and at M = 16384 prefill (1.59 PF/s); the LM head gains 10-17 % at M = 512-1024 and
M = 256 QKV / down 17-29 % — about 1 % of a 1024-stream wave, so the engine does not load a tuning file by default.
"""
import argparse
import json
import os
import statistics
import sys

import torch

SHAPES_8B = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
             ("lm_head", 128256, 4096)]


def timeit(fn, iters=10, rounds=3):
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
    ap.add_argument("--out", default="gpurun_out/tunableop_mi355x.csv")
    ap.add_argument("--ms", default="4,8,16,32,64,128,256,512,1024,2048,16384")
    a = ap.parse_args()
    ms = [int(x) for x in a.ms.split(",")]
    dev = "cuda"
    x_cache = {}
    base = {}
    for m in ms:
        for name, n, k in SHAPES_8B:
            if name == "lm_head" and m > 2048:
                continue
            x = torch.randn(m, k, device=dev).to(torch.bfloat16)
            w = (torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16)
            x_cache[(m, name)] = (x, w)
            base[(m, name)] = timeit(lambda: torch.matmul(x, w.t()))
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_filename(a.out)
    tunable.set_max_tuning_duration(60)
    out = []
    for (m, name), (x, w) in x_cache.items():
        torch.matmul(x, w.t())  # tunes this shape
        torch.cuda.synchronize()
    tunable.tuning_enable(False)
    for (m, name), (x, w) in x_cache.items():
        t = timeit(lambda: torch.matmul(x, w.t()))
        flop = 2 * m * x.shape[1] * w.shape[0]
        rec = dict(m=m, op=name, default_us=round(base[(m, name)], 1), tuned_us=round(t, 1),
                   default_tflops=round(flop / base[(m, name)] / 1e6, 1), tuned_tflops=round(flop / t / 1e6, 1))
        out.append(rec)
        print(json.dumps(rec), flush=True)
    if hasattr(tunable, "write_file"):
        tunable.write_file()
    else:  # torch 2.10: results are flushed to the filename at exit
        tunable.set_filename(a.out)
    print(f"wrote {a.out}", file=sys.stderr)


if __name__ == "__main__":
    main()
