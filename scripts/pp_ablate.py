"""Ablation of the gemm_pp main loop (cdna_hip_programming.md §7 'The diagnostic loop', step 2): time the kernel with
the loop's LDS-DMA, LDS fragment reads or MFMAs skipped (knob pp_ablate bits 1/2/4; outputs are wrong, timing only),
plus the s_setprio variant, interleaved in one process on cold weights.

  python scripts/pp_ablate.py [--m 1024] [--n 28672] [--k 4096] [--cfgs 0,4]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1024)
    ap.add_argument("--n", type=int, default=28672)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--cfgs", default="0,4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("--abl", default="0,1,2,4,3,6")
    ap.add_argument("--warm", action="store_true")
    args = ap.parse_args()
    from chronos import ops

    ops.load()
    m, n, k = args.m, args.n, args.k
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.rand(m, k, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    ncopy = 1 if args.warm else max(2, -(-(600 << 20) // (n * k * 2)))
    ws = [((torch.rand(n, k, device="cuda", generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
    variants = []
    for cfg in [int(c) for c in args.cfgs.split(",")]:
        for abl in [int(v) for v in args.abl.split(",")]:
            variants.append((cfg, abl, False))
        variants.append((cfg, 0, True))
    times = {v: [] for v in variants}
    times["lib"] = []
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(args.rounds):
        for v in times:
            def run(i):
                if v == "lib":
                    return x @ ws[i % ncopy].t()
                torch.ops.chronos.set_knob("pp_ablate", v[1])
                return torch.ops.chronos.gemm_pp(x, ws[i % ncopy], 0, v[0], 1, None, None, 1e-5, v[2])
            for i in range(2):
                run(i)
            torch.cuda.synchronize()
            st.record()
            for i in range(args.iters):
                run(i)
            en.record()
            torch.cuda.synchronize()
            times[v].append(st.elapsed_time(en) * 1000 / args.iters)
    torch.ops.chronos.set_knob("pp_ablate", 0)
    flop = 2.0 * m * n * k
    rows = []
    for v, ts in times.items():
        us = min(ts)
        name = "hipblaslt" if v == "lib" else f"cfg{v[0]}_abl{v[1]}{'_prio' if v[2] else ''}"
        r = dict(m=m, n=n, k=k, warm=args.warm, variant=name, us=round(us, 1), TF=round(flop / us / 1e6, 1))
        rows.append(r)
        print(json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as fh:
            fh.writelines(json.dumps(r) + "\n" for r in rows)


if __name__ == "__main__":
    main()
