"""Decode GEMV by token rows M: Llama-3-8B projection shapes, M = 1, 2, 4, 8, cold weights (a rotating set of
weight copies larger than the 256 MB Infinity Cache), against torch.matmul (hipBLASLt).

    python scripts/bench_gemv_m.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from chronos import ops
    from chronos.ops import gemm

    ops.load()
    shapes = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, True),
              "down": (4096, 14336, False)}
    out = {}
    for name, (n, k, sw) in shapes.items():
        copies = max(2, int(1.2e9 // (n * k * 2)))
        ws = [torch.randn(n, k, device="cuda").to(torch.bfloat16) * 0.02 for _ in range(copies)]
        for m in [int(v) for v in os.environ.get("MS", "1,2,4,8").split(",")]:
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            impls = ["gemv", "hipblaslt"] + [f"gemv_persist={p}" for p in os.environ.get("PERSIST", "").split(",") if p]
            for impl in impls:
                if impl.startswith("gemv_persist="):
                    torch.ops.chronos.set_knob("gemv_persist", int(impl.split("=")[1]))
                def run(w):
                    if impl.startswith("gemv"):
                        return gemm._gemv(x, w, sw)
                    y = torch.matmul(x, w.t())
                    return ops.silu_mul(y) if sw else y
                for w in ws[:2]:
                    run(w)
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                reps = 4 * copies
                a.record()
                for i in range(reps):
                    run(ws[i % copies])
                b.record()
                b.synchronize()
                us = 1e3 * a.elapsed_time(b) / reps
                out[f"{name} M={m} {impl}"] = {"us": round(us, 2), "TB/s": round(n * k * 2 / us / 1e6, 2)}
                torch.ops.chronos.set_knob("gemv_persist", -1)
        del ws
    print(json.dumps(out))


if __name__ == "__main__":
    main()
