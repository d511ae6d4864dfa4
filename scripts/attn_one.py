"""One decode-attention configuration back to back (for rocprofv3 PMC passes): the production one-wave kernel at the
wave's shape (1024 sequences, 8B heads, bf16 KV, scattered pages), KV rotated over enough caches to stay cold.

  python scripts/attn_one.py [--ctx 144] [--shared 0] [--iters 40]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=144)
    ap.add_argument("--shared", type=int, default=0)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--copies", type=int, default=4, help="KV caches rotated (4 x ~0.5 GB: beyond the 256 MB MALL)")
    a = ap.parse_args()
    from chronos import ops

    ops.load()
    dev = "cuda"
    B, hq, hkv, bs = 1024, 32, 8, 16
    nbs = (a.ctx + bs - 1) // bs
    nb = B * nbs + 1
    caches = []
    for _ in range(a.copies):
        perm = torch.randperm(B * nbs, device=dev).to(torch.int32) + 1
        bt = perm.view(B, nbs).clone()
        if a.shared:
            bt[:, :a.shared] = bt[0, :a.shared]
        k = torch.randn(nb, hkv, bs, 128, device=dev).to(torch.bfloat16)
        v = torch.randn(nb, hkv, 128, bs, device=dev).to(torch.bfloat16)
        caches.append((k, v, bt))
    q = torch.randn(B, hq, 128, device=dev).to(torch.bfloat16)
    qs = torch.arange(B + 1, device=dev, dtype=torch.int32)
    cl = torch.randint(a.ctx // 2, a.ctx + 1, (B,), device=dev, dtype=torch.int32)
    ns = ops.pick_nsplit(B * hkv, a.ctx)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        k, v, bt = caches[i % a.copies]
        ops.paged_attention(q, k, v, bt, qs, cl, None, B, 1, ns)
    torch.cuda.synchronize()
    st.record()
    for i in range(a.iters):
        k, v, bt = caches[i % a.copies]
        ops.paged_attention(q, k, v, bt, qs, cl, None, B, 1, ns)
    en.record()
    torch.cuda.synchronize()
    by = int(cl.sum()) * hkv * 128 * 2 * 2
    us = st.elapsed_time(en) * 1e3 / a.iters
    print(f"ctx {a.ctx} shared {a.shared}: {us:.1f} us/call, {by / us / 1e6:.2f} TB/s logical KV")


if __name__ == "__main__":
    main()
