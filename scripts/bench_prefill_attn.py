"""Flash prefill attention (csrc/kernels/attention_prefill.hip) on long-context chunk shapes, Llama-3.1-8B heads
(32 q / 8 kv, D = 128), random data: one 16k-token chunk attending to a P-token paged prefix (the 128k config's
chunked prefill), plus the 1024-stream wave's short prompts.  Reports kernel time and attention TFLOP/s (causal FLOPs
actually needed: 4 * D * Hq * sum over query rows of keys visible), and checks one chunk against the fp32 reference.

  python scripts/bench_prefill_attn.py [--variants 0,1] [--out gpurun_out/prefill_attn.jsonl]
variants are values of the knob ``prefill_variant`` (torch.ops.chronos.set_knob), A/B'd in one process.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=5, rounds=3):
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


def case(q_lens, prefix, hq=32, hkv=8, bs=16, seed=0):
    """q_lens[b] new tokens of sequence b on top of prefix[b] cached tokens; returns op args + FLOPs."""
    from chronos import ops

    g = torch.Generator(device="cuda").manual_seed(seed)
    ctx = [p + n for p, n in zip(prefix, q_lens)]
    nbs = [(c + bs - 1) // bs for c in ctx]
    nb = sum(nbs) + 1
    k = (torch.randn(nb, hkv, bs, 128, device="cuda", generator=g)).to(torch.bfloat16)
    v = (torch.randn(nb, hkv, 128, bs, device="cuda", generator=g)).to(torch.bfloat16)
    mb = max(nbs)
    bt = torch.zeros(len(q_lens), mb, dtype=torch.int32)
    o = 1
    for b, n in enumerate(nbs):
        bt[b, :n] = torch.arange(o, o + n, dtype=torch.int32)
        o += n
    T = sum(q_lens)
    q = (torch.randn(T, hq, 128, device="cuda", generator=g)).to(torch.bfloat16)
    qs = [0]
    for n in q_lens:
        qs.append(qs[-1] + n)
    tiles = ops.attention_tiles(q_lens, hq, hkv, 8)
    tl = torch.tensor(tiles, dtype=torch.int32, device="cuda").view(-1, 2)
    vis = sum(sum(p + i + 1 for i in range(n)) for p, n in zip(prefix, q_lens))
    flops = 4 * 128 * hq * vis
    args = (q, k, v, bt.cuda(), torch.tensor(qs, dtype=torch.int32, device="cuda"),
            torch.tensor(ctx, dtype=torch.int32, device="cuda"), tl, len(tiles), 8, 1)
    return args, flops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0")
    ap.add_argument("--knob", default="prefill_variant", help="kernel knob the variants are values of")
    ap.add_argument("--out", default=None)
    ap.add_argument("--check", action="store_true", help="compare each variant with the fp32 reference (slow)")
    ap.add_argument("--cases", default=None, help="comma-separated subset of the case names")
    ap.add_argument("--fp8", action="store_true", help="fp8-e4m3 KV cache (k_scale 0.25, v_scale 0.5)")
    a = ap.parse_args()
    from chronos import ops
    from chronos.ops import reference as ref

    ops.load()
    cases = {
        "chunk16k_prefix0": ([16384], [0]),
        "chunk16k_prefix48k": ([16384], [49152]),
        "chunk16k_prefix112k": ([16384], [114688]),
        "wave_176x93": ([93] * 176, [0] * 176),
    }
    if a.cases:
        cases = {k: v for k, v in cases.items() if k in a.cases.split(",")}
    variants = [int(x) for x in a.variants.split(",")]
    out = []
    for name, (ql, pf) in cases.items():
        args, flops = case(ql, pf)
        if a.fp8:
            args = (args[0], ref.to_fp8_bytes(args[1], 4.0), ref.to_fp8_bytes(args[2], 2.0)) + args[3:] + (None, 0.25, 0.5)
        rec = dict(case=name, tflop=round(flops / 1e12, 2))
        base = None
        for var in variants:
            torch.ops.chronos.set_knob(a.knob, var)
            us = timeit(lambda: ops.paged_attention(*args))
            y = ops.paged_attention(*args)
            if base is None:
                base = y
            rec[f"v{var}_us"] = round(us, 1)
            rec[f"v{var}_TF"] = round(flops / us / 1e6, 1)
            rec[f"v{var}_maxdiff_vs_v{variants[0]}"] = float((y.float() - base.float()).abs().max())
        if a.check and name == "wave_176x93":
            r = ref.paged_attention(*args)
            rec["maxerr_vs_fp32"] = float((base.float() - r.float()).abs().max())
        torch.ops.chronos.set_knob(a.knob, variants[0])
        out.append(rec)
        print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
