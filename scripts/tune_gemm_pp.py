"""Measure the hand-written GEMM families (gemm_skinny.hip for M <= 64, gemm_pp.hip) against hipBLASLt on every
projection shape of the served models and write the routing plan ops/gemm_plan.json (+ a per-shape table for
profiles/; M <= 2 rows record the decode GEMV, gemv.hip, which is always routed there).

For each (N, K, epilogue) and each M bucket: the fastest kernel / config / split-K among the cost model's candidates,
timed interleaved with the library path of the same epilogue (library GEMM + silu_mul for SwiGLU, + the residual add
for the residual epilogue) in one process on cold weights (cdna_hip_programming.md §5.4 rule 24).  The plan keeps
the hand-written kernel unless the library is more than 3 % faster (any shape left on the library needs a
recorded A/B where the hand-written kernel loses by > 3 %).

  python scripts/tune_gemm_pp.py [--models 8b,70b-tp8] [--ms 3,8,...] [--out-plan P] [--out-table T]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "8b": {"qkv": (6144, 4096, 0), "o": (4096, 4096, 2), "gate_up": (28672, 4096, 1), "down": (4096, 14336, 2),
           "lm_head": (128256, 4096, 0)},
    # Llama-3-70B, TP=8 shards (column-parallel QKV / gate_up / LM head, row-parallel O / down: plain epilogue, the
    # residual add follows the all-reduce)
    "70b-tp8": {"qkv": (1280, 8192, 0), "o": (8192, 1024, 0), "gate_up": (7168, 8192, 1), "down": (8192, 3584, 0),
                "lm_head": (16032, 8192, 0)},
    # Llama-3-70B on one GPU (141 GB of bf16 weights in HBM): TP = 1 shapes, residual epilogues on O / down
    "70b": {"qkv": (10240, 8192, 0), "o": (8192, 8192, 2), "gate_up": (57344, 8192, 1), "down": (8192, 28672, 2),
            "lm_head": (128256, 8192, 0)},
}
MS = [1, 2, 3, 4, 5, 8, 16, 32, 48, 64, 128, 256, 512, 768, 1024, 2048, 4096, 8192, 16384]


def skinny_candidates(m, n, k, mode, keep=10):
    """Skinny configs whose x tile covers M: every valid one without split-K, plus splits only while the grid is
    below two workgroups per CU (a split costs an L2 write-back per workgroup)."""
    from chronos.ops import gemm as G

    out = []
    for c, (rt, mt, nw) in G._SK.items():
        if m > 16 * mt or (mt > 1 and m <= 8 * mt and mt not in (2, 8)):
            continue
        groups = (n // 2) // (8 * rt) if mode == 1 else n // (16 * rt)
        for sk in (1, 2, 3, 4, 7, 8):
            if G._sk_valid(c, m, n, k, mode, sk) and (sk == 1 or groups * sk <= 512):
                out.append((sk > 1, -nw, G.SK_BASE + c, sk))
    out.sort()
    return [(c, sk) for _, _, c, sk in out[:keep]]


def tiny_candidates(m, n, k, mode):
    """M < 16: the 32-row-x-tile gemm_lg configs (72-75), split-K up to ~8 workgroups per CU (at this M the fp32
    partials are a few KB per task: the split buys load balance and loads in flight, not arithmetic)."""
    from chronos.ops import gemm as G

    out = []
    for cfg in (72, 73, 74, 75):
        tiles = -(-n // G._PP_BN[cfg])
        for sk in (1, 2, 4, 8):
            if G._pp_valid(cfg, n, k, mode, sk) and (sk == 1 or tiles * sk <= 2048):
                out.append((cfg, sk))
    return out


def candidates(m, n, k, mode, keep=6):
    from chronos.ops import gemm as G

    scored = []
    for cfg in [c for c in G._PP_BM if c < G.LG_FIRST]:
        bm, bn = G._PP_BM[cfg], G._PP_BN[cfg]
        tiles = -(-m // bm) * -(-n // bn)
        for sk in (1, 2, 4, 8):
            if not G._pp_valid(cfg, n, k, mode, sk) or (sk > 1 and (tiles >= 256 or tiles * sk > 512)):
                continue
            if m >= 4096 and sk > 1:
                continue
            rounds = -(-tiles * sk // 256)
            t = rounds * bm * bn * (k // sk) / G._PP_RATE[cfg] + (sk > 1) * tiles * sk * bm * bn * 4 * 2e3
            scored.append((t, cfg, sk))
    scored.sort()
    out = [(c, s) for _, c, s in scored[:keep]]
    for must in ((0, 1), (4, 1), (8, 1)):
        if must not in out and G._pp_valid(must[0], n, k, mode, 1):
            out.append(must)
    # the software-pipelined family (gemm_lg.hip): every slab / ring config that tiles the shape, split-K where the
    # tile grid under-fills the chip
    # (from M = 128: the wide-W-row tiles over the whole x panel, split-K to fill the chip — at mid-M the L2 -> LDS
    # feed, not HBM, bounds the stream, and x bytes per workgroup scale with x rows / W rows)
    # the HB configs (88 / 89: 4-wave three-barrier slab loop + staged epilogue; split-K only when the grid is small)
    if m >= 512:
        for cfg in (88, 89):
            tiles = -(-m // 256) * -(-n // 256)
            for sk in (1, 2):
                if G._pp_valid(cfg, n, k, mode, sk) and (sk == 1 or tiles < 128) and (cfg, sk) not in out:
                    out.append((cfg, sk))
    if m >= 128:
        for cfg in (20, 80, 29, 30, 19, 31, 23, 76, 77, 22):
            bm, bn = G._PP_BM[cfg], G._PP_BN[cfg]
            tiles = -(-m // bm) * -(-n // bn)
            for sk in (1, 2, 4):
                if G._pp_valid(cfg, n, k, mode, sk) and (sk == 1 or (tiles < 256 and tiles * sk <= 768)) \
                        and (cfg, sk) not in out:
                    out.append((cfg, sk))
    # mid-M weight streaming (gemm_lg.hip 32-39: 64 W rows, the x panel shared through LDS, 4-8 stage rings), split-K
    # until the grid covers the chip
    if 48 <= m <= 512:
        for cfg in (32, 33, 34, 35, 36, 37, 38, 39, 15):
            bm, bn = G._PP_BM[cfg], G._PP_BN[cfg]
            tiles = -(-m // bm) * -(-n // bn)
            if bm > 2 * m and cfg != 33 and cfg != 36 and cfg != 39:
                continue  # x tile far taller than M
            for sk in (1, 2, 4, 8):
                if G._pp_valid(cfg, n, k, mode, sk) and (sk == 1 or (tiles < 256 and tiles * sk <= 1024)) \
                        and (cfg, sk) not in out:
                    out.append((cfg, sk))
    # M <= 48: the same with 32-row x tiles (72-75); to M = 256 the deep-ring ones (78-79: W bytes in flight)
    if 2 <= m <= 256:
        for cfg in ((72, 73, 74, 75, 78, 79) if m <= 48 else (73, 75, 78, 79)):
            bm, bn = G._PP_BM[cfg], G._PP_BN[cfg]
            tiles = -(-m // bm) * -(-n // bn)
            for sk in (1, 2, 4, 8):
                if G._pp_valid(cfg, n, k, mode, sk) and (sk == 1 or (tiles < 256 and tiles * sk <= 1024)) \
                        and (cfg, sk) not in out:
                    out.append((cfg, sk))
    # split-K of the widest tiles where the tile grid under-fills the chip (the fence-free split costs ~2-5 us)
    for cfg in (0, 4, 3):
        bm, bn = G._PP_BM[cfg], G._PP_BN[cfg]
        tiles = -(-m // bm) * -(-n // bn)
        for sk in (2, 3, 4, 8):
            if tiles < 256 and tiles * sk <= 768 and G._pp_valid(cfg, n, k, mode, sk) and (cfg, sk) not in out:
                out.append((cfg, sk))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="8b,70b-tp8")
    ap.add_argument("--ms", default=",".join(str(m) for m in MS))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--out-plan", default="")
    ap.add_argument("--out-table", default="")
    ap.add_argument("--merge", default="", help="plan file whose rows at M not measured in this run are kept")
    ap.add_argument("--ops", default="", help="only these projections (e.g. qkv,lm_head)")
    ap.add_argument("--fp8", action="store_true", help="tune the W8A8 fp8 routing (qplans) instead of the bf16 plan")
    ap.add_argument("--own-only", action="store_true",
                    help="route the fastest hand-written candidate even where the library is faster (its margin is "
                         "still recorded in the table)")
    args = ap.parse_args()
    merged = {}
    if args.merge:
        with open(args.merge) as fh:
            merged = json.load(fh).get("plans", {})
    from chronos import ops
    from chronos.ops import gemm as G

    ops.load()
    if args.fp8:
        return tune_fp8(args, merged)
    dev = "cuda"
    ms = [int(v) for v in args.ms.split(",")]
    plans, table = {}, []
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for model in args.models.split(","):
        for op, (n, k, mode) in SHAPES[model].items():
            if args.ops and op not in args.ops.split(","):
                continue
            g = torch.Generator(device=dev).manual_seed(0)
            ncopy = max(2, -(-(600 << 20) // (n * k * 2)))
            ws = [((torch.rand(n, k, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
                  for _ in range(ncopy)]
            rows = []
            for m in ms:
                if op == "lm_head" and m > 2048:  # the LM head only sees the sampled rows (<= the decode batch)
                    continue
                x = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
                resid = (torch.rand(m, n, device=dev, generator=g) * 2 - 1).to(torch.bfloat16) if mode == 2 else None
                # TP=1 consumers (QKV, gate_up, LM head) read the residual stream with the norm folded in: the hand-
                # written kernels scale rows by the producer's partials (NORMP), the library path runs the RMSNorm
                # kernel first — time both as the model runs them
                normp = model == "8b" and mode in (0, 1)
                part = (x.float() ** 2).view(m, 64, -1).sum(-1).contiguous() if normp else None
                ones = torch.ones(k, device=dev, dtype=torch.bfloat16)

                def lib(i):
                    xin = ops.rmsnorm(x, ones, 1e-5) if normp else x
                    y = xin @ ws[i % ncopy].t()
                    return ops.silu_mul(y) if mode == 1 else (y + resid if mode == 2 else y)

                def own(i, c):
                    if c[0] == "gemv":
                        if mode == 2:
                            return G.gemv_resid(x, ws[i % ncopy], resid).s
                        if normp:
                            return torch.ops.chronos.gemv_normp(x, part, 1e-5, ws[i % ncopy], mode == 1)
                        return G._gemv(x, ws[i % ncopy], mode == 1)
                    if c[0] >= G.SK_BASE:
                        return torch.ops.chronos.gemm_skinny(x, ws[i % ncopy], mode, c[0] - G.SK_BASE, c[1], resid,
                                                             part, 1e-5)[0]
                    return torch.ops.chronos.gemm_pp(x, ws[i % ncopy], mode, c[0], c[1], resid, part, 1e-5, False)[0]

                if m == 1:
                    if not G.gemv_ok(m, n, k):
                        continue
                    cands = [("gemv", 1)]
                else:
                    cands = (skinny_candidates(m, n, k, mode) if m <= G.SKINNY_MAX_M else []) + \
                        (candidates(m, n, k, mode) if m >= 16 else tiny_candidates(m, n, k, mode))
                ref = lib(0).float()
                scale = ref.abs().max().item() + 1e-6
                bad = [c for c in cands if (own(0, c).float() - ref).abs().max().item() > 0.03 * scale]
                assert not bad, f"{op} M={m}: wrong results from {bad}"
                times = {c: [] for c in ["lib"] + cands}
                flop = 2.0 * m * n * k
                iters = max(2, min(args.iters, int(2e13 / flop) + 2))
                for _ in range(args.rounds):
                    for c in times:
                        fn = (lambda i: lib(i)) if c == "lib" else (lambda i, c=c: own(i, c))
                        fn(0)
                        torch.cuda.synchronize()
                        st.record()
                        for i in range(iters):
                            fn(i)
                        en.record()
                        torch.cuda.synchronize()
                        times[c].append(st.elapsed_time(en) * 1000 / iters)
                best = min(cands, key=lambda c: min(times[c]))
                lib_us, own_us = min(times["lib"]), min(times[best])
                use_lib = lib_us < own_us / 1.03 and not args.own_only
                if m > 1:
                    rows.append([m, -1 if use_lib else best[0], 1 if use_lib else best[1]])
                wbytes = n * k * 2
                rec = dict(model=model, op=op, m=m, n=n, k=k, mode=mode, lib_us=round(lib_us, 2),
                           own_us=round(own_us, 2), own=f"cfg{best[0]}_sk{best[1]}",
                           lib_TF=round(flop / lib_us / 1e6, 1), own_TF=round(flop / own_us / 1e6, 1),
                           own_weight_TBs=round(wbytes / own_us / 1e6, 2), lib_weight_TBs=round(wbytes / lib_us / 1e6, 2),
                           speedup=round(lib_us / own_us, 3), route="lib" if use_lib and m > 1 else "own",
                           all={f"cfg{c[0]}_sk{c[1]}": round(min(times[c]), 2) for c in cands})
                table.append(rec)
                print(json.dumps(rec), flush=True)
            # plan rows [measured M, cfg, split-K]: ops/gemm.py routes (previous measured M, M] by the row of M and
            # everything above the last row by the last row; rows of an earlier plan (--merge) at other M are kept
            key = f"{n},{k},{mode}"
            old = {r[0]: r for r in merged.get(key, []) if r[0] < (1 << 30)}
            old.update({r[0]: r for r in rows})
            plans[key] = [old[m] for m in sorted(old)]
            del ws
            torch.cuda.empty_cache()
    meta = {"device": torch.cuda.get_device_name(0),
            "note": "rows: [measured M, cfg (-1 = library, >= 100 = skinny config cfg - 100), split-K]"}
    if args.out_plan:
        for key, rows in merged.items():  # shapes not measured in this run
            plans.setdefault(key, rows)
        with open(args.out_plan, "w") as fh:
            out = {"meta": meta, "plans": plans}
            if args.merge:  # the fp8 routing rows (--fp8 runs) travel with the plan file
                with open(args.merge) as mf:
                    q = json.load(mf).get("qplans")
                if q:
                    out["qplans"] = q
            json.dump(out, fh, indent=1)
    if args.out_table:
        with open(args.out_table, "w") as fh:
            fh.writelines(json.dumps(r) + "\n" for r in table)
    won = sum(r["route"] == "own" for r in table)
    print(f"hand-written kernel routed on {won}/{len(table)} (shape, M) points", flush=True)


def tune_fp8(args, merged_unused):
    """W8A8: the hand-written fp8 kernels (qgemv / block-scaled MFMA qgemm, fused SwiGLU) against hipBLASLt's fp8 GEMM
    (+ silu_mul for gate_up), per 8B projection shape and M; rows [M, 1 own / 0 library] -> "qplans"."""
    from chronos import ops
    from chronos.ops import gemm as G

    G_F8 = G.QLG_GEO
    dev = "cuda"
    ms = [int(v) for v in args.ms.split(",")]
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    qplans, table = {}, []
    f8 = torch.float8_e4m3fn
    for op, (n, k, mode) in SHAPES["8b"].items():
        swiglu = mode == 1
        g = torch.Generator(device=dev).manual_seed(0)
        ncopy = max(2, -(-(600 << 20) // (n * k)))
        wqs = [((torch.rand(n, k, device=dev, generator=g) * 2 - 1) * 200).to(f8).view(torch.uint8)
               for _ in range(ncopy)]
        wsc = torch.rand(n, device=dev, generator=g) * 1e-3 + 1e-4
        rows = []
        for m in ms:
            if op == "lm_head":
                continue  # the LM head stays bf16 in the W8A8 model
            xq = ((torch.rand(m, k, device=dev, generator=g) * 2 - 1) * 200).to(f8).view(torch.uint8)
            xs = torch.rand(m, device=dev, generator=g) * 1e-2 + 1e-3

            def own(i):
                return torch.ops.chronos.qlinear(xq, xs, wqs[i % ncopy], wsc, swiglu)

            # gemm_lg.hip's fp8 configs (M >= 128): every config that tiles N, split-K while the grid under-fills
            lgc = []
            if m >= 128:
                for c in sorted(G_F8):
                    bm, bn = G_F8[c]
                    tiles = -(-m // bm) * (n // bn)
                    for sk in (1, 2, 4):
                        if (n % bn == 0) and (k // 128) % sk == 0 and (sk == 1 or tiles * sk <= 768):
                            lgc.append((c, sk))

            def lib(i):
                y = ops._qlib(xq, xs, wqs[i % ncopy], wsc)
                return ops.silu_mul(y) if swiglu else y

            ref = lib(0).float()
            fns = {"lib": lib, "own": own}
            for c, sk in lgc:
                fns[f"lg{c}_sk{sk}"] = (lambda c_, sk_: lambda i: torch.ops.chronos.qgemm_lg(
                    xq, xs, wqs[i % ncopy], wsc, swiglu, c_, sk_))(c, sk)
            for name, fn in fns.items():
                if name != "lib":
                    err = (fn(0).float() - ref).abs().max().item()
                    assert err <= 0.03 * (ref.abs().max().item() + 1e-6), f"fp8 {op} M={m} {name}: err {err}"
            flop = 2.0 * m * n * k
            iters = max(2, min(args.iters, int(4e13 / flop) + 2))
            t = {name: [] for name in fns}
            for _ in range(args.rounds):
                for name, fn in fns.items():
                    fn(0)
                    torch.cuda.synchronize()
                    st.record()
                    for i in range(iters):
                        fn(i)
                    en.record()
                    torch.cuda.synchronize()
                    t[name].append(st.elapsed_time(en) * 1000 / iters)
            best = min((v for v in t if v != "lib"), key=lambda v: min(t[v]))
            own_us, lib_us = min(t[best]), min(t["lib"])
            use_own = not lib_us < own_us / 1.03
            if not use_own:
                rows.append([m, 0])
            elif best == "own":
                rows.append([m, 1])
            else:
                c, sk = (int(v) for v in best[2:].split("_sk"))
                rows.append([m, G.QLG_BASE + c, sk])
            rec = dict(model="8b-fp8", op=op, m=m, n=n, k=k, mode=mode, lib_us=round(lib_us, 2),
                       own_us=round(own_us, 2), own="fp8.hip" if best == "own" else "gemm_lg fp8 " + best,
                       lib_TF=round(flop / lib_us / 1e6, 1),
                       own_TF=round(flop / own_us / 1e6, 1), own_weight_TBs=round(n * k / own_us / 1e6, 2),
                       speedup=round(lib_us / own_us, 3), route="own" if use_own else "lib",
                       all={v: round(min(ts), 2) for v, ts in t.items()})
            table.append(rec)
            print(json.dumps(rec), flush=True)
        if rows:
            qplans[f"{n},{k},{int(swiglu)}"] = rows
        del wqs
        torch.cuda.empty_cache()
    if args.out_plan:
        with open(args.out_plan, "w") as fh:
            json.dump({"meta": {"device": torch.cuda.get_device_name(0), "note": "qplans rows: [measured M, own]"},
                       "plans": {}, "qplans": qplans}, fh, indent=1)
    if args.out_table:
        with open(args.out_table, "w") as fh:
            fh.writelines(json.dumps(r) + "\n" for r in table)


if __name__ == "__main__":
    main()
