"""gemm_lg / gemm_pp configs vs hipBLASLt (torch.matmul) at chosen shapes, interleaved in one process on random data.

Each config's output is checked against the fp32 product x.float() @ w.float().t() (relative max error), then timed
(median of rounds, operands resident: the prefill / wave shapes reuse one weight per call like the forward does).
  python scripts/bench_gemm_cfgs.py --cfgs 20,81 --shapes sq8192,qkv16k,o16k,gu16k,down16k,lm1k --out gpurun_out/x.jsonl
Shapes: name -> (M, N, K, mode); mode 0 plain, 1 SwiGLU (N = 2F), 2 residual (+ RMSNorm partials).
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "sq8192": (8192, 8192, 8192, 0),
    "sq4096": (4096, 4096, 4096, 0),
    "qkv16k": (16384, 6144, 4096, 0),
    "o16k": (16384, 4096, 4096, 2),
    "gu16k": (16384, 28672, 4096, 1),
    "down16k": (16384, 4096, 14336, 2),
    "qkv4k": (4096, 6144, 4096, 0),
    "o4k": (4096, 4096, 4096, 2),
    "gu4k": (4096, 28672, 4096, 1),
    "down4k": (4096, 4096, 14336, 2),
    "qkv2k": (2048, 6144, 4096, 0),
    "gu2k": (2048, 28672, 4096, 1),
    "lm1k": (1024, 128256, 4096, 0),
    "lm2k": (2048, 128256, 4096, 0),
    "lm768": (768, 128256, 4096, 0),
    "gu1k": (1024, 28672, 4096, 1),
    "gu768": (768, 28672, 4096, 1),
    "qkv1k": (1024, 6144, 4096, 0),
    "o1k": (1024, 4096, 4096, 2),
    "down1k": (1024, 4096, 14336, 2),
    "down2k": (2048, 4096, 14336, 2),
    "o2k": (2048, 4096, 4096, 2),
}


def t_us(fn, iters=10, rounds=7):
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


def lib_fn(x, ws, r, mode, wnext, normp=False):
    """The library path of the same epilogue (+ the standalone RMSNorm pass the folded-norm kernels save)."""
    from chronos import ops

    nw = torch.ones(x.shape[1], device=x.device, dtype=x.dtype)
    xin = (lambda: ops.rmsnorm(x, nw, 1e-5)) if normp else (lambda: x)  # noqa: E731
    if mode == 0:
        return lambda: xin() @ wnext().t()
    if mode == 1:
        return lambda: ops.silu_mul(xin() @ wnext().t())
    return lambda: x @ wnext().t() + r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="20,81")
    ap.add_argument("--shapes", default="sq8192,qkv16k,o16k,gu16k,down16k")
    ap.add_argument("--out", default=None)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--cold", type=int, default=0, help="1: rotate weight copies over >= 1 GiB (each call meets cold weights)")
    ap.add_argument("--normp", type=int, default=0, help="1: modes 0/1 with the folded-RMSNorm prologue (the decoder's call)")
    ap.add_argument("--gms", default="", help="comma list of pp_gm tile-group sizes to sweep (knob; default: as set)")
    a = ap.parse_args()
    from chronos import ops

    ops.load()
    C = torch.ops.chronos
    dev = "cuda"
    # "cfg" or "cfg:splitk"
    cfgs = [tuple(int(v) for v in (c.split(":") + ["1"])[:2]) for c in a.cfgs.split(",") if c]
    fh = open(a.out, "a") if a.out else None
    for name in a.shapes.split(","):
        m, n, k, mode = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(m + n + k)
        x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        ws = [w] + ([w.clone() for _ in range(max(1, -(-(1 << 30) // (n * k * 2))) - 1)] if a.cold else [])
        wi = [0]

        def wnext():
            wi[0] = (wi[0] + 1) % len(ws)
            return ws[wi[0]]
        r = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16) if mode == 2 else None
        rec = {"shape": name, "M": m, "N": n, "K": k, "mode": mode, "normp": bool(a.normp and mode != 2)}
        part = None
        xs = x.float()
        if a.normp and mode != 2:  # producer partials of x: 16 per row (any count works), the kernel scales rows
            part = torch.stack([(xs[:, i::16] ** 2).sum(1) for i in range(16)], 1).contiguous()
            xs = xs * torch.rsqrt((xs * xs).sum(1, keepdim=True) / k + 1e-5)
        ref = None
        if a.check:
            h = xs @ w.float().t()
            if mode == 1:
                f = n // 2
                ref = torch.nn.functional.silu(h[:, :f]) * h[:, f:]
            elif mode == 2:
                ref = h + r.float()
            else:
                ref = h
            del h
        fl = 2.0 * m * n * k
        gms = [int(v) for v in a.gms.split(",") if v] or [None]
        for gm in gms:
            if gm is not None:
                C.set_knob("pp_gm", gm)
            sfx = "" if gm is None else f"_gm{gm}"
            for cfg, sk in cfgs:
                tag = f"cfg{cfg}" + (f"sk{sk}" if sk > 1 else "")
                fn = lambda cfg=cfg, sk=sk: C.gemm_pp(x, wnext(), mode, cfg, sk, r, part, 1e-5, False)  # noqa: E731
                try:
                    y = fn()[0]
                except RuntimeError as e:  # config not valid at this shape
                    rec[tag] = str(e).splitlines()[0][:80]
                    continue
                if ref is not None and gm == gms[0]:
                    rec[f"{tag}_err"] = round(((y.float() - ref).abs().max() / ref.abs().max()).item(), 5)
                del y
                us = t_us(fn)
                rec[f"{tag}{sfx}_us"] = round(us, 1)
                rec[f"{tag}{sfx}_TF"] = round(fl / us / 1e6, 1)
        lf = lib_fn(x, ws, r, mode, wnext, part is not None)
        us = t_us(lf)
        rec["lib_us"] = round(us, 1)
        rec["lib_TF"] = round(fl / us / 1e6, 1)
        line = json.dumps(rec)
        print(line, flush=True)
        if fh:
            fh.write(line + "\n")
            fh.flush()
        del x, w, ws, r, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
