"""A/B of the hand-written projection GEMM family (gemm_pp.hip) against hipBLASLt (torch.matmul) on the Llama-3-8B
projection shapes, interleaved in one process (cdna_hip_programming.md §5.4 rule 24), random operands.

Weights rotate through enough copies to exceed the 256 MiB Infinity Cache ("cold", as in a decode step that streams
the whole model) unless --warm.  Prints one JSON line per (shape, candidate) and a summary table.

  python scripts/bench_gemm_pp.py [--m 1024] [--shapes qkv,o,gate_up,down,lm_head] [--rounds 3] [--out FILE]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (N, K, mode)  mode 1 = swiglu (N = 2F)
    "qkv": (6144, 4096, 0),
    "o": (4096, 4096, 2),
    "gate_up": (28672, 4096, 1),
    "down": (4096, 14336, 2),
    "lm_head": (128256, 4096, 0),
    "sq": (None, None, 0),  # square: N = K = M
}
BM = {0: 256, 1: 128, 2: 256, 3: 128, 4: 256, 5: 128, 6: 256, 7: 128, 8: 256, 9: 128, 10: 256, 11: 128,
      12: 256, 13: 128, 14: 256, 15: 128, 16: 256, 17: 128, 18: 256, 19: 128,
      20: 256, 21: 256, 22: 128, 23: 128, 24: 256, 25: 128, 26: 256, 27: 128, 28: 128, 29: 128, 30: 256, 31: 128,
      32: 128, 33: 64, 34: 128, 35: 256, 36: 64, 37: 128, 38: 64, 39: 64,
      72: 32, 73: 32, 74: 32, 75: 32}  # x rows per tile (12+: gemm_lg.hip)
BM.update({c: 256 for c in range(40, 72)})  # gemm_lg timing ablations (40 + 8 * (cfg == 16) + ABL)
BN = {0: 256, 1: 256, 2: 128, 3: 128, 4: 256, 5: 256, 6: 128, 7: 128, 8: 256, 9: 256, 10: 128, 11: 128,
      12: 256, 13: 256, 14: 128, 15: 128, 16: 256, 17: 256, 18: 128, 19: 128,
      20: 256, 21: 256, 22: 256, 23: 128, 24: 256, 25: 256, 26: 256, 27: 256, 28: 128, 29: 256, 30: 128, 31: 128,
      32: 64, 33: 64, 34: 64, 35: 64, 36: 64, 37: 64, 38: 128, 39: 64,
      72: 64, 73: 128, 74: 64, 75: 128}  # W rows per tile
BN.update({c: 256 for c in range(40, 72)})


def candidates(m, n, k, mode, cus=256):
    out = []
    for cfg in BM:
        if n % BN[cfg]:
            continue
        tiles = -(-m // BM[cfg]) * (n // BN[cfg])
        for sk in (1, 2, 3, 4, 7, 8):
            if (k // 64) % sk:
                continue
            if sk > 1 and tiles * sk > 3 * cus:
                continue
            if sk > 1 and tiles >= cus:
                continue
            out.append((cfg, sk))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="1024")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down,lm_head")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warm", action="store_true")
    ap.add_argument("--prio", action="store_true")
    ap.add_argument("--only", default="", help="cfg:sk list, e.g. 0:1,1:2")
    ap.add_argument("--gms", default="8", help="tile-order group sizes to sweep (knob pp_gm), e.g. 0,8")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    gms = [int(v) for v in args.gms.split(",")]
    from chronos import ops

    ops.load()
    dev = "cuda"
    results = []
    for mstr in args.m.split(","):
        m = int(mstr)
        for name in args.shapes.split(","):
            n, k, mode = SHAPES[name]
            if n is None:
                n = k = m
            g = torch.Generator(device=dev).manual_seed(0)
            x = ((torch.rand(m, k, device=dev, generator=g) * 2 - 1)).to(torch.bfloat16)
            wbytes = n * k * 2
            ncopy = 1 if args.warm else max(2, -(-(600 << 20) // wbytes))
            ws = [((torch.rand(n, k, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
            resid = ((torch.rand(m, n, device=dev, generator=g) * 2 - 1)).to(torch.bfloat16) if mode == 2 else None
            ref = None
            cands = candidates(m, n, k, mode)
            if args.only:
                keep = {tuple(int(v) for v in c.split(":")) for c in args.only.split(",")}
                cands = [c for c in cands if c in keep]
            cands = [(cfg, sk, gm) for cfg, sk in cands for gm in gms]

            def run_lib(i):
                y = x @ ws[i % ncopy].t()
                if mode == 1:
                    y = ops.silu_mul(y)
                elif mode == 2:
                    y = y + resid
                return y

            def run_pp(i, cfg, sk, gm):
                torch.ops.chronos.set_knob("pp_gm", gm)
                return torch.ops.chronos.gemm_pp(x, ws[i % ncopy], mode, cfg, sk, resid, None, 1e-5, args.prio)[0]

            # correctness first (vs the library, bf16 tolerance)
            ref = run_lib(0).float()
            scale = ref.abs().max().item()
            errs = {}
            for cfg, sk, gm in cands:
                y = run_pp(0, cfg, sk, gm).float()
                errs[(cfg, sk, gm)] = (y - ref).abs().max().item() / scale
            times = {("lib", 0): []}
            for c in cands:
                times[c] = []
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for r in range(args.rounds):
                for key in times:
                    for i in range(3):
                        run_lib(i) if key[0] == "lib" else run_pp(i, *key)
                    torch.cuda.synchronize()
                    st.record()
                    for i in range(args.iters):
                        run_lib(i) if key[0] == "lib" else run_pp(i, *key)
                    en.record()
                    torch.cuda.synchronize()
                    times[key].append(st.elapsed_time(en) * 1000 / args.iters)
            flop = 2.0 * m * n * k
            lib_us = min(times[("lib", 0)])
            for key, ts in times.items():
                us = min(ts)
                row = dict(op=name, m=m, n=n, k=k, cand="hipblaslt" if key[0] == "lib" else f"cfg{key[0]}_sk{key[1]}" + (f"_gm{key[2]}" if key[2] else ""),
                           us=round(us, 2), us_med=round(sorted(ts)[len(ts) // 2], 2),
                           TF=round(flop / us / 1e6, 1), vs_lib=round(lib_us / us, 3),
                           rel_err=None if key[0] == "lib" else round(errs[key], 5), cold=not args.warm)
                results.append(row)
                print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as fh:
            for r in results:
                fh.write(json.dumps(r) + "\n")
    # summary: best hand-written per shape
    best = {}
    for r in results:
        if r["cand"] == "hipblaslt":
            continue
        k = (r["op"], r["m"])
        if k not in best or r["us"] < best[k]["us"]:
            best[k] = r
    for (op, m), r in sorted(best.items()):
        lib = next(x for x in results if x["op"] == op and x["m"] == m and x["cand"] == "hipblaslt")
        print(f"{op:8s} M={m:6d}  best {r['cand']:10s} {r['us']:8.1f} us {r['TF']:7.1f} TF | hipBLASLt {lib['us']:8.1f} us"
              f" {lib['TF']:7.1f} TF | x{lib['us'] / r['us']:.2f}", flush=True)


if __name__ == "__main__":
    main()
