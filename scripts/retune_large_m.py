"""Re-measure the large-M rows of ops/gemm_plan.json with the HB configs of gemm_lg.hip (cfg 88 / 89: the 4-wave
three-barrier slab loop + LDS-staged epilogue, profiles/r6_gemm_isa_diff.md) among the candidates, and write the
updated plan.

For every plan key (N, K, epilogue) and every M row >= --min-m (plus --add-ms rows for keys whose table stops early):
the row's current hand-written config (if any), cfg 88, cfg 89 and the library path of the same epilogue (hipBLASLt +
silu_mul for SwiGLU, + the residual add for the residual epilogue), timed interleaved in one process on random data
with cold weights (copies rotated over >= 1 GiB).  The fastest hand-written config wins the row unless the library is
more than --lib-margin faster (the plan's rule since round 2).  JSON lines per row go to --out-table.

  python scripts/retune_large_m.py --out-plan ops/gemm_plan.json --out-table gpurun_out/x.jsonl
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HB_CFGS = (88, 89, 92, 93)  # 92 / 93: 88 / 89 with the square k-step-0 order (HB bit 7)


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
    ap.add_argument("--plan", default=None, help="input plan (default: the package's ops/gemm_plan.json)")
    ap.add_argument("--out-plan", default=None)
    ap.add_argument("--out-table", default=None)
    ap.add_argument("--min-m", type=int, default=512)
    ap.add_argument("--max-m", type=int, default=1 << 30)
    ap.add_argument("--extra-cfgs", default="",
                    help="more candidates for every row, 'cfg/splitk' comma-separated (e.g. 19/1,30/2)")
    ap.add_argument("--keys", default="", help="comma-separated 'N:K:mode' keys (default: every plan key)")
    ap.add_argument("--add-ms", default="", help="N:K:mode=M1/M2/.. rows to add before measuring (';'-separated)")
    ap.add_argument("--lib-margin", type=float, default=0.03)
    ap.add_argument("--hb-cfgs", default=",".join(str(c) for c in HB_CFGS))
    ap.add_argument("--own-only", action="store_true",
                    help="never route a row to the library (rows whose in-situ fused epilogue the bare A/B misses)")
    a = ap.parse_args()
    hb_cfgs = tuple(int(c) for c in a.hb_cfgs.split(",") if c)
    extra = [tuple(int(v) for v in c.split("/")) for c in a.extra_cfgs.split(",") if c]
    from chronos import ops
    from chronos.ops import gemm as G

    ops.load()
    C = torch.ops.chronos
    path = a.plan or os.path.join(os.path.dirname(os.path.abspath(G.__file__)), "gemm_plan.json")
    plan = json.load(open(path))
    rows_by_key = plan["plans"]
    for spec in [s for s in a.add_ms.split(";") if s]:
        key, ms = spec.split("=")
        kk = key.replace(":", ",")
        rows = rows_by_key.setdefault(kk, [])
        have = {r[0] for r in rows}
        for m in (int(v) for v in ms.split("/")):
            if m not in have:
                rows.append([m, -1, 1])
        rows.sort(key=lambda r: r[0])
    keys = [k.replace(":", ",") for k in a.keys.split(",") if k] or list(rows_by_key)
    fh = open(a.out_table, "a") if a.out_table else None
    dev = "cuda"
    for key in keys:
        n, k, mode = (int(v) for v in key.split(","))
        rows = rows_by_key[key]
        todo = [r for r in rows if a.min_m <= r[0] <= a.max_m]
        if not todo:
            continue
        wb = n * k * 2
        ncopy = max(2, -(-(1 << 30) // wb))
        g = torch.Generator(device=dev).manual_seed(n + k)
        ws = [(torch.randn(n, k, device=dev, generator=g) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        it = [0]

        def w_next():
            it[0] = (it[0] + 1) % ncopy
            return ws[it[0]]

        for row in todo:
            m = row[0]
            x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
            r = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16) if mode == 2 else None
            cands = []
            if row[1] >= 0 and row[1] not in hb_cfgs:
                cands.append((row[1], row[2]))
            for c in hb_cfgs:
                if G._pp_valid(c, n, k, mode, 1, m):
                    cands.append((c, 1))
            for c, sk in extra:
                if (c, sk) not in cands and G._pp_valid(c, n, k, mode, sk, m):
                    cands.append((c, sk))
            rec = {"key": key, "M": m, "N": n, "K": k, "mode": mode, "was": row[1:]}
            best = None
            for cfg, sk in cands:
                fn = lambda cfg=cfg, sk=sk: G.pp_gemm(x, w_next(), mode, (cfg, sk), r)  # noqa: E731
                try:
                    us = t_us(fn)
                except RuntimeError as e:
                    rec[f"cfg{cfg}_sk{sk}"] = str(e).splitlines()[0][:60]
                    continue
                rec[f"cfg{cfg}_sk{sk}_us"] = round(us, 1)
                if best is None or us < best[0]:
                    best = (us, cfg, sk)
            if mode == 0:
                lf = lambda: x @ w_next().t()  # noqa: E731
            elif mode == 1:
                lf = lambda: ops.silu_mul(x @ w_next().t())  # noqa: E731
            else:
                lf = lambda: torch.add(x @ w_next().t(), r)  # noqa: E731
            lib = t_us(lf)
            rec["lib_us"] = round(lib, 1)
            if best is None or (not a.own_only and lib * (1 + a.lib_margin) < best[0]):
                row[1], row[2] = -1, 1
            else:
                row[1], row[2] = best[1], best[2]
            rec["now"] = row[1:]
            rec["own_vs_lib"] = round(lib / best[0], 3) if best else None
            line = json.dumps(rec)
            print(line, flush=True)
            if fh:
                fh.write(line + "\n")
                fh.flush()
            del x, r
        del ws
        torch.cuda.empty_cache()
    if a.out_plan:
        meta = plan.setdefault("meta", {})
        meta["r6_hb"] = ("large-M rows re-measured with the HB configs 88 / 89 (4-wave three-barrier slab loop + "
                         "LDS-staged epilogue) among the candidates: scripts/retune_large_m.py "
                         "(profiles/r6/retune_large_m.jsonl)")
        with open(a.out_plan, "w") as fo:
            json.dump(plan, fo, indent=1)
            fo.write("\n")


if __name__ == "__main__":
    main()
