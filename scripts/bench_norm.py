"""RMSNorm (+ residual add) and SwiGLU elementwise kernels at the wave's shapes (M = 1024 decode rows, 16384-token
prefill chunks; d = 4096, F = 14336), cold operands rotated over several copies.  Prints us and TB/s per kernel.

  python scripts/bench_norm.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.bench_kernels import timeit  # noqa: E402


def main():
    from chronos import ops

    ops.load()
    d, f = 4096, 14336
    w = torch.rand(d, device="cuda").to(torch.bfloat16)
    for m in (1024, 16384):
        nc = max(2, (600 << 20) // (m * d * 2 * 2))
        xs = [torch.randn(m, d, device="cuda").to(torch.bfloat16) for _ in range(nc)]
        rs = [torch.randn(m, d, device="cuda").to(torch.bfloat16) for _ in range(nc)]
        it = [0]

        def norm():
            i = it[0] = (it[0] + 1) % nc
            ops.add_rmsnorm(xs[i], rs[i], w, 1e-5)

        us = timeit(norm)
        print(f"add_rmsnorm M={m}: {us:.1f} us, {4 * m * d * 2 / us / 1e6:.2f} TB/s", flush=True)
        del xs, rs
        nc = max(2, (600 << 20) // (m * 2 * f * 2))
        gus = [torch.randn(m, 2 * f, device="cuda").to(torch.bfloat16) for _ in range(nc)]

        def silu():
            i = it[0] = (it[0] + 1) % nc
            ops.silu_mul(gus[i])

        us = timeit(silu)
        print(f"silu_mul    M={m}: {us:.1f} us, {3 * m * f * 2 / us / 1e6:.2f} TB/s", flush=True)
        del gus


if __name__ == "__main__":
    main()
