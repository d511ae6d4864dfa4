"""Cascade decode attention diagnostic: are member rows merged (outputs differ in rounding from the plain kernel), and
what do the producer / consumer cost against the plain kernel at the wave's shape (n rows, ~130-token contexts)."""
import sys
import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_cascade_gpu import _setup  # noqa: E402
from chronos import ops  # noqa: E402

ops.load()
for n, P in ((1024, 3), (1024, 2), (512, 3)):
    hq, hkv = 32, 8
    kc, vc, bt, ctx, pos, cos_sin, qkv, prefix, kinds = _setup(n, P, hq, hkv, seed=1)
    casc = torch.tensor([P] + prefix + [0] * (8 - P), dtype=torch.int32, device="cuda")
    co = torch.empty(n, hq, 128, dtype=torch.bfloat16, device="cuda")
    cl = torch.empty(n, hq, dtype=torch.float32, device="cuda")
    a = ops.decode_attention_rope(qkv, pos, cos_sin, kc.clone(), vc.clone(), bt, ctx, n, hq, 0.088, None)
    b = ops.decode_attention_rope(qkv, pos, cos_sin, kc.clone(), vc.clone(), bt, ctx, n, hq, 0.088, (casc, co, cl))
    mem = [i for i, k in enumerate(kinds) if k in (0, 1, 2, 5)]
    diff = (a[mem].float() - b[mem].float()).abs().amax(dim=(1, 2))
    print(f"n={n} P={P}: member rows {len(mem)}, rows whose output differs from plain {(diff > 0).sum().item()}, "
          f"max diff {diff.max().item():.3g}")
    k2, v2 = kc.clone(), vc.clone()
    for name, c in (("plain", None), ("casc", (casc, co, cl))):
        for _ in range(3):
            ops.decode_attention_rope(qkv, pos, cos_sin, k2, v2, bt, ctx, n, hq, 0.088, c)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.decode_attention_rope(qkv, pos, cos_sin, k2, v2, bt, ctx, n, hq, 0.088, c)
        e1.record()
        e1.synchronize()
        print(f"   {name}: {e0.elapsed_time(e1) / 20 * 1000:.1f} us")
