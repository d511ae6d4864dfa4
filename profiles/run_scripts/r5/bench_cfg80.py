"""cfg 80 (gemm_lg slab schedule on 32x32x16 MFMAs) vs cfg 20 (the same on 16x16x32) vs hipBLASLt, interleaved in one
process on random data, at the large-M shapes (8192^3 and the 8B projections at M = 1024 / 16384).  JSON lines."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def t_us(fn, iters=10, rounds=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / iters * 1e3)
    return statistics.median(out)


def main():
    from chronos import ops

    ops.load()
    C = torch.ops.chronos
    dev = "cuda"
    shapes = [("sq8192", 8192, 8192, 8192, 0), ("qkv", 1024, 6144, 4096, 0), ("gate_up", 1024, 28672, 4096, 1),
              ("o", 1024, 4096, 4096, 2), ("qkv", 16384, 6144, 4096, 0), ("gate_up", 16384, 28672, 4096, 1),
              ("down", 16384, 4096, 14336, 2), ("o", 16384, 4096, 4096, 2)]
    for name, m, n, k, mode in shapes:
        g = torch.Generator(device=dev).manual_seed(m + n + k)
        x = (torch.randn(m, k, device=dev, generator=g)).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        r = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16) if mode == 2 else None
        res = {}
        outs = {}
        for cfg in (20, 80):
            fn = lambda cfg=cfg: C.gemm_pp(x, w, mode, cfg, 1, r, None, 1e-5, False)  # noqa: E731
            outs[cfg] = fn()[0]
            res[f"cfg{cfg}_us"] = round(t_us(fn), 1)
        lib = lambda: x @ w.t()  # noqa: E731
        res["lib_us"] = round(t_us(lib), 1)
        ref = outs[20].float()
        err = (outs[80].float() - ref).abs().max().item() / max(1e-6, ref.abs().max().item())
        fl = 2.0 * m * n * k
        print(json.dumps({"shape": name, "M": m, "N": n, "K": k, "mode": mode, **res,
                          "cfg80_TF": round(fl / res["cfg80_us"] / 1e6, 1), "cfg20_TF": round(fl / res["cfg20_us"] / 1e6, 1),
                          "lib_TF": round(fl / res["lib_us"] / 1e6, 1), "rel_diff_80_vs_20": err}), flush=True)


if __name__ == "__main__":
    main()
