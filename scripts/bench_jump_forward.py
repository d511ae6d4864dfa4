"""GPU time of a jump-forward step: one sequence, T = 2..6 new tokens over a ~200-token context, prefill-mode forward
(what Engine._jump runs), with the small-M projections on hipBLASLt / the MFMA GEMM (GEMV_MAX_M = 2, the default) or
on the decode GEMV (GEMV_MAX_M = 8).  Variants interleaved in one process.

    python scripts/bench_jump_forward.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from chronos.models.llama import KVCache, build_model, make_prefill_batch
    from chronos.ops import gemm

    model = build_model(os.environ.get("MODEL", "llama3-8b"), "cuda", seed=0)
    kv = KVCache(model.cfg, model.tp, 64, 16, "cuda")
    ctx0 = 200
    blocks = list(range(1, 17))
    prompt = [int(t) for t in torch.randint(0, 100000, (ctx0,))]
    model.forward(make_prefill_batch([prompt], [0], [blocks], model.cfg, model.tp, "cuda", max_blocks=16, nqt=8), kv)
    res = {}
    for T in (2, 3, 4, 5, 6):
        toks = [int(t) for t in torch.randint(0, 100000, (T,))]
        for mx in (2, 8):
            gemm.GEMV_MAX_M = mx
            sb = make_prefill_batch([toks], [ctx0], [blocks], model.cfg, model.tp, "cuda", max_blocks=16, nqt=8)
            for _ in range(3):
                model.forward(sb, kv)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            a.record()
            for _ in range(reps):
                model.forward(sb, kv)
            b.record()
            b.synchronize()
            res[f"T={T} gemv_max_m={mx}"] = round(a.elapsed_time(b) / reps, 3)
    gemm.GEMV_MAX_M = 2
    print(json.dumps({"ms_per_forward": res}))


if __name__ == "__main__":
    main()
