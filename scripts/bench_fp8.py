"""W8A8 fp8 projection GEMMs (csrc/kernels/fp8.hip) vs the bf16 paths the engine uses today, per Llama-3-8B shape.

bf16 side = what ops.linear / ops.gate_up_silu run (hand GEMV at M <= 2, hipBLASLt + silu_mul elsewhere).
fp8 side  = ops.qlinear on pre-quantised operands (the activation quantisation is timed separately: in the model it is
            fused into the RMSNorm or is one pass over the attention / SwiGLU output).
Weights rotate over enough copies to exceed the 256 MB Infinity Cache for decode-sized M (cold weights, as in
serving).  Interleaved rounds in one process; medians reported (cdna_hip_programming.md §5.4 rule 24).

  python scripts/bench_fp8.py --out gpurun_out/fp8_gemm.json
"""
import argparse
import json
import statistics
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("gate_up", 28672, 4096, True),
          ("down", 4096, 14336, False)]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,2,4,16,64,128,256,512,1024,2048,16384")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/fp8_gemm.json")
    a = ap.parse_args()
    from chronos import ops
    from chronos.ops import reference as ref

    ops.load()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    res = []
    for name, n, k, sw in SHAPES:
        copies = max(1, min(8, (600 << 20) // (n * k * 2)))
        wb = [(torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        wq = [ref.quantize_weight(w) for w in wb]
        for m in [int(x) for x in a.ms.split(",")]:
            x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
            xq, xs = ops.quant_rows(x)
            nc = copies if m <= 256 else 1
            fb = (lambda i: ops.gate_up_silu(x, wb[i % nc])) if sw else (lambda i: ops.linear(x, wb[i % nc]))
            fq = lambda i: ops.qlinear(xq, xs, wq[i % nc][0], wq[i % nc][1], sw)  # noqa: E731
            fz = lambda i: ops.quant_rows(x)  # noqa: E731
            iters = 20 if m <= 2048 else 5
            for f in (fb, fq, fz):
                f(0)
            torch.cuda.synchronize()
            tb, tq, tz, tg = [], [], [], {128: [], 256: []}
            for _ in range(a.rounds):
                tb.append(timed(fb, iters))
                tq.append(timed(fq, iters))
                tz.append(timed(fz, iters))
                if m > 4:
                    for geo in (128, 256):
                        torch.ops.chronos.set_knob("qgemm_tile", geo)
                        tg[geo].append(timed(fq, iters))
                    torch.ops.chronos.set_knob("qgemm_tile", 0)
            try:  # hipBLASLt's own fp8 (rowwise scales) as a library reference point
                xf8, wf8 = xq.view(torch.float8_e4m3fn), [q.view(torch.float8_e4m3fn) for q, _ in wq]
                fl8 = lambda i: torch._scaled_mm(xf8, wf8[i % nc].t(), scale_a=xs[:, None], scale_b=wq[i % nc][1][None, :],  # noqa: E731
                                                 out_dtype=torch.bfloat16)
                fl8(0)
                tl = statistics.median([timed(fl8, iters) for _ in range(a.rounds)])
            except Exception as e:  # noqa: BLE001
                tl = None
                print(f"_scaled_mm unavailable: {str(e)[:120]}", file=sys.stderr)
            yb, yq = fb(0).float(), fq(0).float()
            err = float(((yb - yq).norm() / yb.norm()).item())
            fl = 2.0 * m * n * k
            r = dict(op=name, m=m, n=n, k=k, bf16_us=round(statistics.median(tb), 1),
                     fp8_us=round(statistics.median(tq), 1), quant_us=round(statistics.median(tz), 1),
                     bf16_TF=round(fl / statistics.median(tb) / 1e6, 1), fp8_TF=round(fl / statistics.median(tq) / 1e6, 1),
                     speedup=round(statistics.median(tb) / statistics.median(tq), 3), rel_err_vs_bf16=round(err, 4),
                     tile128_us=round(statistics.median(tg[128]), 1) if tg[128] else None,
                     tile256_us=round(statistics.median(tg[256]), 1) if tg[256] else None,
                     hipblaslt_fp8_us=round(tl, 1) if tl else None)
            res.append(r)
            print(json.dumps(r), flush=True)
        del wb, wq
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
