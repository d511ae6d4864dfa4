"""Skinny GEMM (gemm_skinny.hip) at M = 48-128 on the 8B projection shapes, the routed configs of ops/gemm_plan.json,
against hipBLASLt (+ its separate epilogue), cold weights.   python scripts/bench_skinny_m.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.bench_kernels import timeit  # noqa: E402

SHAPES = {"qkv": (6144, 4096, 0), "o": (4096, 4096, 2), "gate_up": (28672, 4096, 1), "down": (4096, 14336, 2)}
CANDS = {128: [(107, 1), (107, 2), (105, 1), (110, 1), (110, 2)], 64: [(105, 1), (105, 2), (110, 1), (110, 2), (106, 2)]}


def main():
    from chronos import ops

    ops.load()
    C = torch.ops.chronos
    for m, cands in CANDS.items():
        for name, (n, k, mode) in SHAPES.items():
            g = torch.Generator(device="cuda").manual_seed(1)
            x = (torch.rand(m, k, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
            nc = max(2, (600 << 20) // (n * k * 2))
            ws = [((torch.rand(n, k, device="cuda", generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(nc)]
            r = (torch.rand(m, n, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16) if mode == 2 else None
            it = [0]

            def lib():
                i = it[0] = (it[0] + 1) % nc
                y = x @ ws[i].t()
                return ops.silu_mul(y) if mode == 1 else (y + r if mode == 2 else y)

            ref = lib().float()
            row = [f"{name:8s} M={m:4d} lib {timeit(lib):7.1f}"]
            for cfg, sk in cands:
                def own():
                    i = it[0] = (it[0] + 1) % nc
                    return C.gemm_skinny(x, ws[i], mode, cfg - 100, sk, r, None, 1e-5)[0]
                try:
                    it[0] = -1
                    y = own().float()
                    it[0] = -1
                    ref = lib().float()
                    err = (y - ref).abs().max().item() / ref.abs().max().item()
                    row.append(f"c{cfg}s{sk} {timeit(own):7.1f}{'!' if err > 0.02 else ''}")
                except RuntimeError:
                    row.append(f"c{cfg}s{sk}   n/a")
            print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
