"""Run one gemm_pp configuration (or the hipBLASLt reference) back to back, for rocprofv3 kernel traces / PMC passes.

  python scripts/pp_one.py --op gate_up --m 1024 --cfg 0 --sk 1 --iters 20 [--lib]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.bench_gemm_pp import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="gate_up")
    ap.add_argument("--m", type=int, default=1024)
    ap.add_argument("--cfg", type=int, default=0)
    ap.add_argument("--sk", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", action="store_true")
    args = ap.parse_args()
    from chronos import ops

    ops.load()
    n, k, mode = SHAPES[args.op]
    if n is None:  # square
        n = k = args.m
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.rand(args.m, k, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    ncopy = max(2, -(-(600 << 20) // (n * k * 2)))
    ws = [((torch.rand(n, k, device="cuda", generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
    resid = (torch.rand(args.m, n, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16) if mode == 2 else None
    for i in range(args.iters):
        if args.lib:
            x @ ws[i % ncopy].t()
        else:
            torch.ops.chronos.gemm_pp(x, ws[i % ncopy], mode, args.cfg, args.sk, resid, None, 1e-5, False)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
