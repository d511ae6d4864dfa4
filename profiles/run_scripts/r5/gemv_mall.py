"""Decode GEMV (M = 1) on HBM-cold vs Infinity-Cache-warm weights: each 8B projection shape timed (a) cycling through
enough weight copies that every call streams from HBM, (b) on one copy reused (after the first call it sits in the
256 MB MALL when it fits).  If (b) is much faster the single-stream decode is bandwidth-bound and prefetching the next
projection's weights into the MALL would pay; if (a) ~ (b) the kernels are bound by their fill / drain latency."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from chronos import ops

    ops.load()
    C = torch.ops.chronos
    dev = "cuda"
    for name, n, k, swiglu in (("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("gate_up", 28672, 4096, True),
                               ("down", 4096, 14336, False)):
        wbytes = n * k * 2
        copies = max(2, int(2.5e9 // wbytes))  # > 2 GB of copies: nothing stays cached
        ws = [torch.randn(n, k, device=dev).to(torch.bfloat16) * 0.02 for _ in range(copies)]
        x = torch.randn(1, k, device=dev).to(torch.bfloat16)
        res = {}
        for mode in ("cold", "warm"):
            for _ in range(3):
                C.gemv(x, ws[0], swiglu)
            torch.cuda.synchronize()
            times = []
            for rep in range(5):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                iters = copies if mode == "cold" else 50
                s.record()
                for i in range(iters):
                    C.gemv(x, ws[i % copies] if mode == "cold" else ws[0], swiglu)
                e.record()
                torch.cuda.synchronize()
                times.append(s.elapsed_time(e) / iters * 1e3)
            res[mode] = statistics.median(times)
        print(json.dumps({"shape": name, "N": n, "K": k, "MB": round(wbytes / 1e6, 1),
                          "cold_us": round(res["cold"], 1), "warm_us": round(res["warm"], 1),
                          "cold_TBps": round(wbytes / res["cold"] / 1e6, 2),
                          "warm_TBps": round(wbytes / res["warm"] / 1e6, 2)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
