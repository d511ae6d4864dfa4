"""Is a decode GEMV faster when its weights were just read (Infinity Cache / MALL warm) than from cold HBM?
Times the M = 1 GEMV on one weight copy repeatedly (warm) against a rotation through copies that exceed the 256 MB
MALL (cold), per 8B projection — the question behind prefetching the next projection's weights during attention."""
import json
import sys

import torch

sys.path.insert(0, ".")
from chronos import ops  # noqa: E402
from chronos.ops import gemm as G  # noqa: E402

ops.load()
dev = "cuda"
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, n, k, sw in [("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("gate_up", 28672, 4096, True),
                       ("down", 4096, 14336, False)]:
    g = torch.Generator(device=dev).manual_seed(0)
    ncopy = max(2, -(-(1200 << 20) // (n * k * 2)))
    ws = [((torch.rand(n, k, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
    x = (torch.rand(1, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    res = {}
    for mode in ("cold", "warm"):
        best = 1e9
        for _ in range(3):
            G._gemv(x, ws[0], sw)
            torch.cuda.synchronize()
            st.record()
            for i in range(20):
                G._gemv(x, ws[i % ncopy] if mode == "cold" else ws[0], sw)
            en.record()
            torch.cuda.synchronize()
            best = min(best, st.elapsed_time(en) * 1000 / 20)
        res[mode] = round(best, 2)
    mb = n * k * 2 / 1e6
    print(json.dumps(dict(op=name, MB=round(mb, 1), cold_us=res["cold"], warm_us=res["warm"],
                          cold_TBs=round(mb / res["cold"] / 1e6 * 1e6 / 1e6, 2) if False else round(mb / res["cold"], 2),
                          warm_TBs=round(mb / res["warm"], 2))), flush=True)
    del ws
    torch.cuda.empty_cache()
