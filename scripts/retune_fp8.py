"""Re-measure the W8A8 rows of ops/gemm_plan.json ("qplans") with gemm_lg.hip's fp8 config 4 (F8HB: the HB slab loop
on v_mfma_scale_f32_32x32x64_f8f6f4) among the candidates, and write the updated plan.

For every qplans key (N, K, SwiGLU) and every M row >= --min-m: the row's current route (hipBLASLt's fp8 GEMM through
torch._scaled_mm (+ silu_mul), fp8.hip's qlinear, or a gemm_lg fp8 config), fp8 config 4 at split-K 1 (and 2 / 4
while the 256 x 256 tile grid under-fills the chip) and the library, timed interleaved in one process with cold
weights (copies rotated over >= 1 GiB).  The fastest hand-written candidate wins the row unless the library is more
than --lib-margin faster (the plan's rule).  JSON lines per row go to --out-table.

  python scripts/retune_fp8.py --out-plan ops/gemm_plan.json --out-table gpurun_out/fp8_retune.jsonl
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HB8 = 4


def t_us(fn, iters=8, rounds=5):
    for _ in range(2):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--plan", default=None)
    ap.add_argument("--out-plan", default=None)
    ap.add_argument("--out-table", default=None)
    ap.add_argument("--min-m", type=int, default=256)
    ap.add_argument("--keys", default="")
    ap.add_argument("--lib-margin", type=float, default=0.03)
    a = ap.parse_args()
    from chronos import ops
    from chronos.ops import gemm as G

    ops.load()
    C = torch.ops.chronos
    path = a.plan or os.path.join(os.path.dirname(os.path.abspath(G.__file__)), "gemm_plan.json")
    plan = json.load(open(path))
    qp = plan["qplans"]
    keys = [k.replace(":", ",") for k in a.keys.split(",") if k] or list(qp)
    fh = open(a.out_table, "a") if a.out_table else None
    dev = "cuda"
    f8 = torch.float8_e4m3fn
    for key in keys:
        n, k, sw = (int(v) for v in key.split(","))
        swiglu = bool(sw)
        todo = [r for r in qp[key] if r[0] >= a.min_m]
        if not todo:
            continue
        ncopy = max(2, -(-(1 << 30) // (n * k)))
        g = torch.Generator(device=dev).manual_seed(n + k)
        wqs = [((torch.rand(n, k, device=dev, generator=g) * 2 - 1) * 200).to(f8).view(torch.uint8)
               for _ in range(ncopy)]
        wsc = torch.rand(n, device=dev, generator=g) * 1e-3 + 1e-4
        it = [0]

        def w_next():
            it[0] = (it[0] + 1) % ncopy
            return wqs[it[0]]

        for row in todo:
            m = row[0]
            xq = ((torch.rand(m, k, device=dev, generator=g) * 2 - 1) * 200).to(f8).view(torch.uint8)
            xs = torch.rand(m, device=dev, generator=g) * 1e-2 + 1e-3

            def lib(w):
                y = ops._qlib(xq, xs, w, wsc)
                return ops.silu_mul(y) if swiglu else y

            cands = {}
            code = row[1]
            if code == 1:
                cands["qlinear"] = lambda w: C.qlinear(xq, xs, w, wsc, swiglu)
            elif code >= G.QLG_BASE and code - G.QLG_BASE != HB8:
                c0, sk0 = code - G.QLG_BASE, row[2] if len(row) > 2 else 1
                cands[f"lg{c0}_sk{sk0}"] = (lambda c_, s_: lambda w: C.qgemm_lg(xq, xs, w, wsc, swiglu, c_, s_))(
                    c0, sk0)
            tiles = -(-m // 256) * (n // 256)
            for sk in (1, 2, 4):
                if (k // 128) % sk == 0 and (sk == 1 or tiles < 256) and (not swiglu or n % 256 == 0):
                    cands[f"lg{HB8}_sk{sk}"] = (lambda s_: lambda w: C.qgemm_lg(xq, xs, w, wsc, swiglu, HB8, s_))(sk)
            ref = lib(wqs[0]).float()  # (the accuracy check on one fixed weight copy; timing rotates them)
            rec = {"key": key, "M": m, "N": n, "K": k, "swiglu": swiglu, "was": row[1:]}
            best = None
            for name, fn in cands.items():
                err = (fn(wqs[0]).float() - ref).abs().max().item()
                if err > 0.03 * (ref.abs().max().item() + 1e-6):
                    rec[name] = f"error {err:.3g}"
                    continue
                us = t_us(lambda fn=fn: fn(w_next()))
                rec[name + "_us"] = round(us, 1)
                if best is None or us < best[0]:
                    best = (us, name)
            lus = t_us(lambda: lib(w_next()))
            rec["lib_us"] = round(lus, 1)
            flop = 2.0 * m * n * k
            rec["lib_TF"] = round(flop / lus / 1e6, 1)
            if best is None or lus * (1 + a.lib_margin) < best[0]:
                row[:] = [m, 0]
            elif best[1] == "qlinear":
                row[:] = [m, 1]
            else:
                c, sk = (int(v) for v in best[1][2:].split("_sk"))
                row[:] = [m, G.QLG_BASE + c, sk]
            if best:
                rec["own_TF"] = round(flop / best[0] / 1e6, 1)
                rec["own_vs_lib"] = round(lus / best[0], 3)
            rec["now"] = row[1:]
            line = json.dumps(rec)
            print(line, flush=True)
            if fh:
                fh.write(line + "\n")
                fh.flush()
        del wqs
        torch.cuda.empty_cache()
    if a.out_plan:
        plan.setdefault("meta", {})["r6_fp8_hb"] = (
            "W8A8 rows at M >= 256 re-measured with fp8 config 4 (F8HB: the HB slab loop on the 32x32x64 fp8 MFMA) "
            "among the candidates: scripts/retune_fp8.py (profiles/r6/fp8_hb_retune.jsonl)")
        with open(a.out_plan, "w") as fo:
            json.dump(plan, fo, indent=1)
            fo.write("\n")


if __name__ == "__main__":
    main()
