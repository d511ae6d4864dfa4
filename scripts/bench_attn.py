"""Decode attention variants A/B'd in one process (torch.ops.chronos.set_knob), 8B shapes, random data:
legacy split-over-waves kernel vs the one-wave-per-(seq, kv head) kernel with / without register prefetch.
Reports time and logical KV bytes / time.   python scripts/bench_attn.py [--out gpurun_out/attn.json]"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, rounds=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters * 1e3)
    return statistics.median(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from chronos import ops

    ops.load()
    C = torch.ops.chronos
    dev = "cuda"
    out = []
    base = dict(decode_attn_legacy=0, decode_pf=0)
    variants = {"legacy": dict(decode_attn_legacy=1, decode_pf=0),
                "wave": dict(base, decode_lean=0, decode_occ3=0),
                "wave_lean": dict(base, decode_lean=1, decode_occ3=0),
                "wave_occ3": dict(base, decode_lean=0, decode_occ3=1),
                "wave_lean_occ3": dict(base, decode_lean=1, decode_occ3=1),
                "wave_pf": dict(decode_attn_legacy=0, decode_pf=1)}
    ap_shared = int(os.environ.get("ATTN_SHARED_BLOCKS", "0"))
    cases = ((1024, 128, False), (1024, 200, False), (256, 160, False), (1024, 512, False), (64, 1024, False),
             (1024, 128, True))
    if os.environ.get("ATTN_CASES") == "wave":
        cases = ((1024, 128, False), (1024, 144, False))
    if os.environ.get("ATTN_CASES") == "long":  # split-K decode over long contexts (the 128k config's decode)
        cases = ((1, 131072, False), (1, 131072, True), (4, 32768, False), (16, 8192, False), (64, 1024, False))
        variants = {"split_pf": dict(split_lds=0, split_pf=1, attn_inkernel_combine=1),
                    "lds_nb1": dict(split_lds=1, split_lds_nb=1), "lds_nb2": dict(split_lds=1, split_lds_nb=2),
                    "lds_nb3": dict(split_lds=1, split_lds_nb=3), "lds_nb4": dict(split_lds=1, split_lds_nb=4),
                    "lds_inlaunch": dict(split_lds=1, split_lds_nb=0, sd_inkernel_max_split=1024),
                    "lds_sepcomb": dict(split_lds=1, split_lds_nb=0, sd_inkernel_max_split=4)}
    for B, ctx, fp8 in cases:
        hq, hkv, bs = 32, 8, 16
        nbs = (ctx + bs - 1) // bs
        nb = B * nbs + 1
        perm = torch.randperm(B * nbs, device=dev).to(torch.int32) + 1  # scattered pages, like a live cache
        if os.environ.get("ATTN_SEQ_PAGES"):  # pages in allocation order (a fresh engine's long sequence)
            perm = torch.arange(B * nbs, device=dev, dtype=torch.int32) + 1
        bt = perm.view(B, nbs).clone()
        if ap_shared:  # the chat-template prefix: the first blocks are the SAME pages for every sequence
            bt[:, :ap_shared] = bt[0, :ap_shared]
        if fp8:
            k = torch.randint(0, 120, (nb, hkv, bs, 128), device=dev, dtype=torch.uint8)
            v = torch.randint(0, 120, (nb, hkv, 128, bs), device=dev, dtype=torch.uint8)
        else:
            k = torch.randn(nb, hkv, bs, 128, device=dev).to(torch.bfloat16)
            v = torch.randn(nb, hkv, 128, bs, device=dev).to(torch.bfloat16)
        q = torch.randn(B, hq, 128, device=dev).to(torch.bfloat16)
        qs = torch.arange(B + 1, device=dev, dtype=torch.int32)
        cl = torch.randint(ctx // 2, ctx + 1, (B,), device=dev, dtype=torch.int32)
        if os.environ.get("ATTN_CASES") == "long":
            cl.fill_(ctx)
        ns = ops.pick_nsplit(B * hkv, ctx)
        res = {}
        outs = {}
        runs = [(name, kn, ns) for name, kn in variants.items()]
        if os.environ.get("ATTN_NSPLITS"):  # the split count itself (default kernel knobs, or ATTN_KNOBS sets)
            kn_sets = [dict(kv.split("=") for kv in ks.split("+")) if ks else {}
                       for ks in os.environ.get("ATTN_KNOBS", "").split(",")]
            runs = [(f"nsplit{n}" + ("_" + "_".join(f"{a}{b}" for a, b in kd.items()) if kd else ""),
                     {a: int(b) for a, b in kd.items()}, int(n))
                    for n in os.environ["ATTN_NSPLITS"].split(",") for kd in kn_sets]
        for name, kn, nsp in runs:
            for kk, vv in kn.items():
                C.set_knob(kk, vv)
            fn = lambda: ops.paged_attention(q, k, v, bt, qs, cl, None, B, 1, nsp)  # noqa: E731
            outs[name] = fn().float()
            res[name] = timeit(fn)
        ref = outs[next(iter(outs))]
        err = max(float((o - ref).abs().max()) for o in outs.values())
        by = int(cl.sum()) * hkv * 128 * 2 * (1 if fp8 else 2)
        rec = dict(batch=B, ctx=ctx, fp8=fp8, nsplit=ns, shared_blocks=ap_shared, **{f"{n}_us": round(t, 1) for n, t in res.items()},
                   **{f"{n}_TBps": round(by / t / 1e6, 2) for n, t in res.items()}, max_diff_vs_legacy=err)
        out.append(rec)
        print(json.dumps(rec), flush=True)
    C.set_knob("decode_attn_legacy", 0)
    C.set_knob("decode_pf", 0)
    C.set_knob("decode_lean", 1)
    C.set_knob("decode_occ3", 1)
    C.set_knob("split_pf", 1)
    C.set_knob("attn_inkernel_combine", 1)
    C.set_knob("split_lds", 1)
    C.set_knob("split_lds_nb", 0)
    C.set_knob("sd_inkernel_max_split", 4)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
