"""Context parallelism for long kill-chain prefill (SURVEY.md §2.4 C6, §2.5 "context parallel", §5.7).

The 128k-token config (BASELINE.json) fits one MI355X — 16 GiB of bf16 KV for Llama-3.1-8B — so CP here is a TTFT
tool, not a capacity tool: the W ranks of a CP group each hold the full (TP=1) weights and split a long prefill chunk
between them.

Per layer, rank r projects only its own tokens, then the ranks exchange K and V with ONE RCCL all-gather (GQA: the
8 KV heads are 1/4 of the QKV output, 4 KiB per token per layer — 64 MiB for a 16k-token slice, a bandwidth-optimal
ring over the xGMI links) and every rank writes the FULL chunk's K/V into its own paged cache (the rope_kv_write
kernel on the gathered [T, 2 * Hkv * 128] rows, positions carried along).  Attention is then the ordinary paged
prefill kernel: each local query row attends causally to the complete prefix.  This is the all-gather form of CP
(Llama 3's own long-context recipe) rather than a send/recv ring: for GQA the gathered K/V are small next to the
attention FLOPs, the collective is a single large RCCL call per layer, and every rank ends the prefill with the full
KV, so the verdict decode that follows runs on any rank (the engine runs it in lockstep on all of them).

Load balance: the chunk is cut into 2W pieces and rank r takes pieces r and 2W-1-r ("zigzag"), so every rank gets
one early and one late piece of the causal triangle.  The chunk's last token (whose logits start the verdict) is in
piece 2W-1, i.e. on CP rank 0, which broadcasts that row.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any

import torch
import torch.distributed as dist

from .tp import TPContext


@dataclass
class CPInfo:
    """What the model forward needs to all-gather and write the chunk's K/V (models/llama.py LlamaModel._attn)."""
    group: Any
    world: int
    rank: int
    tpad: int                 # per-rank padded token count of the gathered layout
    ntok: int                 # this rank's real token count
    pos_all: torch.Tensor     # [world * tpad] int32 positions of the gathered rows (pad rows: 0)
    seq_all: torch.Tensor     # [world * tpad] int32 row of ``bt`` per gathered row (pad rows -> the scratch row)
    bt: torch.Tensor          # [2, max_blocks] int32: the sequence's block table, then all-zero (scratch block 0)
    dummy_q: torch.Tensor     # rope_kv_write's q_out placeholder (no q is written for gathered rows)


def zigzag_pieces(n: int, world: int) -> list[tuple[int, int]]:
    """[0, n) cut into 2*world contiguous pieces whose sizes differ by at most one."""
    k = 2 * world
    b = [i * n // k for i in range(k + 1)]
    return [(b[i], b[i + 1]) for i in range(k)]


def rank_pieces(n: int, world: int, rank: int) -> list[tuple[int, int]]:
    pcs = zigzag_pieces(n, world)
    return [pcs[rank], pcs[2 * world - 1 - rank]]


def make_cp_batch(ids: list[int], start: int, blocks: list[int], cfg, cp: TPContext, device, max_blocks: int,
                  nqt: int = 8):
    """This rank's StepBatch for a CP prefill of ``ids`` (absolute positions start..start+len-1, KV blocks
    ``blocks``): its two zigzag pieces as two sequences sharing one block table, plus the gathered-write layout.
    Every rank must call it with the same arguments."""
    from ..models.llama import h2d, make_prefill_batch

    W, r, n = cp.world, cp.rank, len(ids)
    if n < 2 * W:
        raise ValueError(f"CP prefill needs at least {2 * W} tokens, got {n}")
    mine = rank_pieces(n, W, r)
    sb = make_prefill_batch([ids[a:b] for a, b in mine], [start + a for a, _ in mine], [blocks, blocks], cfg,
                            TPContext.single(), device, max_blocks=max_blocks, nqt=nqt)
    sizes = [sum(b - a for a, b in rank_pieces(n, W, q)) for q in range(W)]
    tpad = max(sizes)
    pos, seq = [], []
    for q in range(W):
        p = [start + t for a, b in rank_pieces(n, W, q) for t in range(a, b)]
        pos += p + [0] * (tpad - len(p))
        seq += [0] * len(p) + [1] * (tpad - len(p))
    bt = torch.zeros(2, max_blocks, dtype=torch.int32)
    bt[0, :len(blocks)] = torch.tensor(blocks, dtype=torch.int32)
    it = lambda x: h2d(torch.tensor(x, dtype=torch.int32), device)  # noqa: E731
    sb.cp = CPInfo(cp.group, W, r, tpad, sizes[r], it(pos), it(seq), h2d(bt, device),
                   torch.empty(1, 128, dtype=torch.bfloat16, device=device))
    return sb


def gather_kv(qkv: torch.Tensor, hq: int, cp: CPInfo) -> torch.Tensor:
    """All-gather the K/V columns of this rank's QKV rows: [world * tpad, 2 * hkv * 128] (rank-major, padded)."""
    kv = qkv[:, hq * 128:]
    send = torch.zeros(cp.tpad, kv.shape[1], dtype=kv.dtype, device=kv.device)
    send[:cp.ntok].copy_(kv)
    out = torch.empty(cp.world * cp.tpad, kv.shape[1], dtype=kv.dtype, device=kv.device)
    dist.all_gather_into_tensor(out, send, group=cp.group)
    return out


def last_logits(logits: torch.Tensor, cp: TPContext) -> torch.Tensor:
    """[1, V] logits of the chunk's last token on every rank: row 1 (piece 2W-1) of CP rank 0, broadcast."""
    row = logits[1:2].contiguous() if cp.rank == 0 else torch.empty_like(logits[:1])
    src = dist.get_global_rank(cp.group, 0) if cp.group is not None else 0
    dist.broadcast(row, src=src, group=cp.group)
    return row
