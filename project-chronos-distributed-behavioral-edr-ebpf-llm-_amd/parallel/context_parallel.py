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

Ulysses form (``EngineConfig.cp_mode = "ulysses"``, SURVEY.md §2.5 "Ulysses", optional): rank r projects a
CONTIGUOUS 1/W of the chunk; after the same K/V all-gather + full-chunk cache write (every rank must still end the
prefill with the whole KV, the lockstep decode needs it), the roped queries are re-sharded from tokens to heads by
one all-to-all, rank r runs the causal attention of the WHOLE chunk for query-head group r (Hq/W heads against its
Hkv/W KV heads, G stays Hq/Hkv), and a second all-to-all returns the outputs to token shards for the O projection.
Balance comes from the head split (every rank sees the full causal triangle), not from zigzag pieces; the price is
the two extra all-to-alls of Q and O per layer (``README.md``: strictly more xGMI bytes than the all-gather form,
which stays the default).  The head group's K/V are staged into a contiguous scratch cache (the paged kernels address
``blk * Hkv + h``), so the hand-written flash / split-K prefill kernels run unchanged.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Optional

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
    last_rank: int = 0        # CP rank holding the chunk's last token, and its row in that rank's logits
    last_row: int = 1
    ulysses: Optional["UlyssesInfo"] = None


@dataclass
class UlyssesInfo:
    """Head-sharded attention of the whole chunk on this rank (Ulysses form)."""
    sizes: list               # real token count of every rank's contiguous shard
    h0: int                   # first KV head of this rank's group (query heads h0 * G ...)
    hkv_g: int                # KV heads per group
    blk_idx: torch.Tensor     # [nblk] int64 the sequence's cache blocks covering start + n tokens
    bt: torch.Tensor          # [1, max_blocks] int32 block table of the staged scratch cache (0 .. nblk-1)
    q_start: torch.Tensor     # [2] int32
    ctx_len: torch.Tensor     # [1] int32
    tiles: torch.Tensor       # [ntiles, 2] int32 prefill tiles of the whole chunk for Hq/W query heads
    ntiles: int
    nqt: int
    nsplit: int


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


def contiguous_pieces(n: int, world: int) -> list[tuple[int, int]]:
    """[0, n) cut into ``world`` contiguous pieces whose sizes differ by at most one (Ulysses token shards)."""
    b = [i * n // world for i in range(world + 1)]
    return [(b[i], b[i + 1]) for i in range(world)]


def make_ulysses_batch(ids: list[int], start: int, blocks: list[int], cfg, cp: TPContext, device, max_blocks: int,
                       nqt: int = 8):
    """This rank's StepBatch for a Ulysses CP prefill of ``ids`` (see the module docstring); same contract as
    make_cp_batch: every rank calls it with the same arguments."""
    from .. import ops
    from ..models.llama import h2d, make_prefill_batch

    W, r, n = cp.world, cp.rank, len(ids)
    if cfg.num_heads % W or cfg.num_kv_heads % W:
        raise ValueError(f"Ulysses CP needs the head counts ({cfg.num_heads}, {cfg.num_kv_heads}) divisible by {W}")
    if n < W:
        raise ValueError(f"Ulysses CP prefill needs at least {W} tokens, got {n}")
    pcs = contiguous_pieces(n, W)
    a, b = pcs[r]
    sb = make_prefill_batch([ids[a:b]], [start + a], [blocks], cfg, TPContext.single(), device,
                            max_blocks=max_blocks, nqt=nqt)
    sizes = [e - s for s, e in pcs]
    tpad = max(sizes)
    pos, seq = [], []
    for s0, e0 in pcs:
        pos += [start + t for t in range(s0, e0)] + [0] * (tpad - (e0 - s0))
        seq += [0] * (e0 - s0) + [1] * (tpad - (e0 - s0))
    bt = torch.zeros(2, max_blocks, dtype=torch.int32)
    bt[0, :len(blocks)] = torch.tensor(blocks, dtype=torch.int32)
    it = lambda x: h2d(torch.tensor(x, dtype=torch.int32), device)  # noqa: E731
    hq_g, hkv_g = cfg.num_heads // W, cfg.num_kv_heads // W
    ctx = start + n
    nblk = -(-ctx // 16)
    tiles = ops.attention_tiles([n], hq_g, hkv_g, nqt)
    gbt = torch.zeros(1, max_blocks, dtype=torch.int32)
    gbt[0, :nblk] = torch.arange(nblk, dtype=torch.int32)
    uy = UlyssesInfo(sizes, r * hkv_g, hkv_g, h2d(torch.tensor(blocks[:nblk], dtype=torch.int64), device),
                     h2d(gbt, device), it([0, n]), it([ctx]), h2d(torch.tensor(tiles, dtype=torch.int32).view(-1, 2),
                                                                  device),
                     len(tiles), nqt, ops.pick_nsplit(len(tiles) * hkv_g, ctx))
    sb.cp = CPInfo(cp.group, W, r, tpad, sizes[r], it(pos), it(seq), h2d(bt, device),
                   torch.empty(1, 128, dtype=torch.bfloat16, device=device), last_rank=W - 1, last_row=0, ulysses=uy)
    return sb


def _a2a(x: torch.Tensor, cp: CPInfo) -> torch.Tensor:
    """all_to_all_single over dim 0 (one slice per rank); both buffers dense row-major (empty_like of a transposed
    view would keep its strides)."""
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    dist.all_to_all_single(out, x, group=cp.group)
    return out


def ulysses_attention(q_loc: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, cp: CPInfo, scale: float,
                      k_scale: float = 1.0, v_scale: float = 1.0) -> torch.Tensor:
    """Attention output [ntok, Hq * 128] of this rank's token shard, computed head-sharded: q_loc [ntok, Hq, 128]
    (roped) -> all-to-all -> [n, Hq/W, 128] of head group r -> causal paged attention over the whole chunk (the
    group's K/V staged contiguously) -> all-to-all back."""
    from .. import ops

    uy, W = cp.ulysses, cp.world
    hq, d = q_loc.shape[1], q_loc.shape[2]
    hq_g = hq // W
    send = torch.zeros(cp.tpad, W, hq_g, d, dtype=q_loc.dtype, device=q_loc.device)
    send[:cp.ntok] = q_loc.view(cp.ntok, W, hq_g, d)
    recv = _a2a(send.transpose(0, 1), cp)  # [W (token shard), tpad, hq_g, d]
    q_g = torch.cat([recv[i, :uy.sizes[i]] for i in range(W)])  # [n, hq_g, d] in chunk order
    kg = k_cache.index_select(0, uy.blk_idx)[:, uy.h0:uy.h0 + uy.hkv_g].contiguous()
    vg = v_cache.index_select(0, uy.blk_idx)[:, uy.h0:uy.h0 + uy.hkv_g].contiguous()
    o_g = ops.paged_attention(q_g, kg, vg, uy.bt, uy.q_start, uy.ctx_len, uy.tiles, uy.ntiles, uy.nqt, uy.nsplit,
                              scale, k_scale, v_scale).view(-1, hq_g, d)
    back = torch.zeros(W, cp.tpad, hq_g, d, dtype=o_g.dtype, device=o_g.device)
    off = 0
    for i in range(W):
        back[i, :uy.sizes[i]] = o_g[off:off + uy.sizes[i]]
        off += uy.sizes[i]
    mine = _a2a(back, cp)  # [W (head group), tpad, hq_g, d]
    return mine[:, :cp.ntok].transpose(0, 1).reshape(cp.ntok, hq * d)


def gather_kv(qkv: torch.Tensor, hq: int, cp: CPInfo) -> torch.Tensor:
    """All-gather the K/V columns of this rank's QKV rows: [world * tpad, 2 * hkv * 128] (rank-major, padded)."""
    kv = qkv[:, hq * 128:]
    send = torch.zeros(cp.tpad, kv.shape[1], dtype=kv.dtype, device=kv.device)
    send[:cp.ntok].copy_(kv)
    out = torch.empty(cp.world * cp.tpad, kv.shape[1], dtype=kv.dtype, device=kv.device)
    dist.all_gather_into_tensor(out, send, group=cp.group)
    return out


def last_logits(logits: torch.Tensor, cp: TPContext, info: CPInfo | None = None) -> torch.Tensor:
    """[1, V] logits of the chunk's last token on every rank, broadcast from the rank that holds it: zigzag — row 1
    (piece 2W-1) of CP rank 0; Ulysses — row 0 of the last rank."""
    lr, row_i = (info.last_rank, info.last_row) if info is not None else (0, 1)
    row = logits[row_i:row_i + 1].contiguous() if cp.rank == lr else torch.empty_like(logits[:1])
    src = dist.get_global_rank(cp.group, lr) if cp.group is not None else lr
    dist.broadcast(row, src=src, group=cp.group)
    return row
