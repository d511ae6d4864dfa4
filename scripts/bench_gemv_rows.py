"""Decode GEMV (csrc/kernels/gemv.hip) at M = 1, by rows per workgroup (knobs gemv_r_swiglu / gemv_r_plain /
gemv_r_resid), on the Llama-3-8B single-stream shapes.  Weights rotate over >= 1 GiB of copies (a decode step meets
every layer's weights cold), variants interleaved in one process, median of rounds; reports us and TB/s of weight
bytes.  Checks each variant's output against the default's.

  python scripts/bench_gemv_rows.py --out gpurun_out/gemv_rows.json
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, N, K, kind, knob, values); kind: swiglu | plain | resid
CASES = [("gate_up", 28672, 4096, "swiglu", "gemv_r_swiglu", (4, 2, 1)),
         ("down", 4096, 14336, "resid", "gemv_r_resid", (8, 4, 2)),
         ("o", 4096, 4096, "resid", "gemv_r_resid", (8, 4, 2)),
         ("lm_head", 128256, 4096, "plain", "gemv_r_plain", (8, 4, 2)),
         ("qkv_rope", 6144, 4096, "rope", "gemv_r_rope", (8, 4, 2))]


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
    for name, n, k, kind, kn, vals in CASES:
        ncopy = max(2, -(-2**30 // (n * k * 2)))
        ws = [(torch.rand(n, k, device=dev) * 0.04 - 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % ncopy
            return ws[it[0]]

        x = (torch.rand(1, k, device=dev) * 2 - 1).to(torch.bfloat16)
        rin = (torch.rand(1, n, device=dev) * 2 - 1).to(torch.bfloat16)
        rout = torch.empty_like(rin)
        if kind == "rope":
            pos = torch.tensor([100], dtype=torch.int32, device=dev)
            tseq = torch.zeros(1, dtype=torch.int32, device=dev)
            btab = torch.arange(1, 17, dtype=torch.int32, device=dev).view(1, -1)
            cs = torch.rand(256, 128, device=dev)
            qo = torch.empty(1, 32, 128, dtype=torch.bfloat16, device=dev)
            kc = torch.zeros(17, 8, 16, 128, dtype=torch.bfloat16, device=dev)
            vc = torch.zeros(17, 8, 128, 16, dtype=torch.bfloat16, device=dev)

            def fn(w):
                C.qkv_rope(x, None, 1e-5, w, pos, tseq, btab, cs, qo, kc, vc, 32, 8)
                return torch.cat([qo.flatten(), kc[7].flatten(), vc[7].flatten()])
        elif kind == "swiglu":
            fn = lambda w: C.gemv(x, w, True)  # noqa: E731
        elif kind == "plain":
            fn = lambda w: C.gemv(x, w, False)  # noqa: E731
        else:
            fn = lambda w: C.gemv_resid(x, w, rin, rout)  # noqa: E731
        outs, ts = {}, {v: [] for v in vals}
        for v in vals:
            C.set_knob(kn, v)
            r = fn(ws[0])
            outs[v] = (rout.clone() if kind == "resid" else r).float()
        for _ in range(3):
            for v in vals:
                C.set_knob(kn, v)
                ts[v].append(timeit(lambda: fn(nxt())))
        C.set_knob(kn, vals[0])
        t = {v: statistics.median(x) for v, x in ts.items()}
        by = n * k * 2
        rec = dict(op=name, n=n, k=k, knob=kn, **{f"r{v}_us": round(x, 2) for v, x in t.items()},
                   **{f"r{v}_TBps": round(by / x / 1e6, 2) for v, x in t.items()},
                   max_diff=max(float((outs[v] - outs[vals[0]]).abs().max()) for v in vals))
        out.append(rec)
        print(json.dumps(rec), flush=True)
        del ws
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
