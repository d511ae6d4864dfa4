"""A/B of the batched GEMM's folded-norm (NORMP) prologue: the same config with and without part_in, cold weights,
8B gate_up / QKV / LM head at M = 1024 (profiles/r3_normp_ab.jsonl)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from chronos import ops  # noqa: E402

ops.load()
dev = "cuda"
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, n, k, mode, cfgs in [("gate_up", 28672, 4096, 1, (0, 4)), ("qkv", 6144, 4096, 0, (1, 2)),
                               ("lm_head", 128256, 4096, 0, (0,))]:
    g = torch.Generator(device=dev).manual_seed(0)
    ncopy = max(2, -(-(600 << 20) // (n * k * 2)))
    ws = [((torch.rand(n, k, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
    m = 1024
    x = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    part = (x.float() ** 2).view(m, 64, -1).sum(-1).contiguous()
    for cfg in cfgs:
        for use in (False, True):
            fn = lambda i: torch.ops.chronos.gemm_pp(x, ws[i % ncopy], mode, cfg, 1, None, part if use else None,  # noqa
                                                     1e-5, False)
            best = 1e9
            for _ in range(3):
                fn(0)
                torch.cuda.synchronize()
                st.record()
                for i in range(6):
                    fn(i)
                en.record()
                torch.cuda.synchronize()
                best = min(best, st.elapsed_time(en) * 1000 / 6)
            print(json.dumps(dict(op=name, m=m, cfg=cfg, normp=use, us=round(best, 2))), flush=True)
    lib = lambda i: ws[i % ncopy].new_empty(0) if False else x @ ws[i % ncopy].t()  # noqa
    best = 1e9
    for _ in range(3):
        lib(0)
        torch.cuda.synchronize()
        st.record()
        for i in range(6):
            lib(i)
        en.record()
        torch.cuda.synchronize()
        best = min(best, st.elapsed_time(en) * 1000 / 6)
    print(json.dumps(dict(op=name, m=m, cfg="lib", normp=False, us=round(best, 2))), flush=True)
    del ws
    torch.cuda.empty_cache()
