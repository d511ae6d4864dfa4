"""Pure-PyTorch reference implementations of every HIP kernel (the numerics oracle, and the CPU execution path).

Each function mirrors the exact contract of its kernel in csrc/kernels (same layouts, same in-place semantics) and
computes in fp32, rounding to bf16 at the same points the kernel and HF Llama do.
"""
from __future__ import annotations

import math

import torch


def embedding(ids: torch.Tensor, table: torch.Tensor, vstart: int = 0) -> torch.Tensor:
    idx = ids.long() - vstart
    ok = (idx >= 0) & (idx < table.shape[0])
    out = table[idx.clamp(0, table.shape[0] - 1)]
    return out * ok[:, None].to(out.dtype)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * inv).to(torch.bfloat16).float().mul(w.float()).to(x.dtype)


def add_rmsnorm(x: torch.Tensor, resid: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    resid.copy_((x.float() + resid.float()).to(resid.dtype))
    return rmsnorm(resid, w, eps)


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    f = gu.shape[-1] // 2
    g, u = gu[..., :f].float(), gu[..., f:].float()
    return (torch.nn.functional.silu(g).to(torch.bfloat16).float() * u).to(gu.dtype)


FP8_MAX = 448.0


def to_fp8_bytes(x: torch.Tensor, inv_scale: float) -> torch.Tensor:
    """f32 -> OCP e4m3fn bytes with saturation (what the HIP kernels store)."""
    return (x.float() * inv_scale).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(torch.uint8)


def from_fp8_bytes(b: torch.Tensor, scale: float) -> torch.Tensor:
    return b.view(torch.float8_e4m3fn).float() * scale


def quant_rows(x: torch.Tensor, resid: torch.Tensor | None = None, w: torch.Tensor | None = None, eps: float = 1e-5,
               mode: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-row dynamic e4m3 quantisation (fp8.hip quant_rows_kernel): mode 0 = x, 1 = rmsnorm(x) * w,
    2 = resid <- bf16(x + resid), rmsnorm(resid) * w, 3 = silu(gate) * up of [gate | up] rows.
    Returns (bytes [rows, d] uint8, scale [rows] f32)."""
    d = x.shape[-1]
    if mode == 3:
        y = silu_mul(x)
        d = d // 2
    elif mode == 2:
        y = add_rmsnorm(x, resid, w, eps)
    elif mode == 1:
        y = rmsnorm(x, w, eps)
    else:
        y = x
    y = y.reshape(-1, d).float()
    amax = y.abs().amax(-1)
    s = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
    r = torch.where(amax > 0, FP8_MAX / amax, torch.ones_like(amax))
    q = (y * r[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(torch.uint8)
    return q, s


def qlinear(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor, swiglu: bool = False) -> torch.Tensor:
    """fp32 reference of the W8A8 GEMM: (dequant(xq) @ dequant(wq).T), bf16 out; swiglu: wq = [gate; up]."""
    x = xq.view(torch.float8_e4m3fn).float()
    wf = wq.view(torch.float8_e4m3fn).float()
    acc = x @ wf.t()
    y = acc * xs.float()[:, None] * ws.float()[None, :]
    if not swiglu:
        return y.to(torch.bfloat16)
    f = y.shape[-1] // 2
    g = y[:, :f].to(torch.bfloat16).float()
    u = y[:, f:].to(torch.bfloat16).float()
    return (torch.nn.functional.silu(g).to(torch.bfloat16).float() * u).to(torch.bfloat16)


def quantize_weight(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-output-channel e4m3 weight quantisation: (bytes [N, K] uint8, scale [N] f32), w ~= bytes * scale."""
    wf = w.float()
    amax = wf.abs().amax(-1).clamp_min(1e-12)
    s = amax / FP8_MAX
    q = (wf / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(torch.uint8)
    return q.contiguous(), s.contiguous()


def rope_kv_write(qkv, pos, tok_seq, block_table, cos_sin, q_out, k_cache, v_cache, hq: int, hkv: int,
                  write_q: bool = True, k_scale: float = 1.0, v_scale: float = 1.0) -> None:
    T = qkv.shape[0]
    D = 128
    x = qkv.view(T, hq + 2 * hkv, D).float()
    p = pos.long()
    cos = cos_sin[p, :64].float()[:, None, :]
    sin = cos_sin[p, 64:].float()[:, None, :]
    qk = x[:, : hq + hkv]
    x1, x2 = qk[..., :64], qk[..., 64:]
    rot = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(torch.bfloat16)
    if write_q:
        q_out.view(-1, hq, D)[:T].copy_(rot[:, :hq])
    bs = k_cache.shape[2]
    blk = block_table[tok_seq.long(), p // bs].long()
    off = p % bs
    v = x[:, hq + hkv:].to(torch.bfloat16)  # [T, hkv, D]
    if k_cache.dtype == torch.uint8:
        rotf = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)
        k_cache[blk, :, off, :] = to_fp8_bytes(rotf[:, hq:], 1.0 / k_scale)
        v_cache[blk, :, :, off] = to_fp8_bytes(v, 1.0 / v_scale)
    else:
        k_cache[blk, :, off, :] = rot[:, hq:]
        v_cache[blk, :, :, off] = v


def paged_attention(q, k_cache, v_cache, block_table, q_start, ctx_len, tiles=None, ntiles=0, nqt=1, nsplit=1,
                    scale: float | None = None, k_scale: float = 1.0, v_scale: float = 1.0,
                    max_q: int = 1) -> torch.Tensor:
    """Causal varlen attention over the paged cache.  q [T, Hq, 128]; seqs given by q_start/ctx_len.  Decode mode
    (tiles None): one token per sequence, or with max_q > 1 the q_start ranges (<= max_q tokens, the last at the end
    of the context) — the same causal semantics as a prefill chunk."""
    T, hq, D = q.shape
    hkv, bs = k_cache.shape[1], k_cache.shape[2]
    G = hq // hkv
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    out = torch.zeros_like(q)
    if tiles is None and max_q == 1:  # decode: one token per sequence, seq i = token i
        qs = list(range(ntiles + 1))
    elif tiles is None:
        qs = q_start[:ntiles + 1].tolist()
    else:
        qs = q_start.tolist()
    B = len(qs) - 1
    bt = block_table.long()
    for b in range(B):
        q0, q1 = qs[b], qs[b + 1]
        ql = q1 - q0
        if ql == 0:
            continue
        ctx = int(ctx_len[b])
        nblk = (ctx + bs - 1) // bs
        blks = bt[b, :nblk]
        kb, vb = k_cache[blks], v_cache[blks]
        if k_cache.dtype == torch.uint8:  # fp8 cache: dequantise like the kernel (value * scale, then bf16)
            kb = from_fp8_bytes(kb, k_scale).to(torch.bfloat16)
            vb = from_fp8_bytes(vb, v_scale).to(torch.bfloat16)
        K = kb.permute(1, 0, 2, 3).reshape(hkv, nblk * bs, D)[:, :ctx].float()
        V = vb.permute(1, 0, 3, 2).reshape(hkv, nblk * bs, D)[:, :ctx].float()
        qq = q[q0:q1].float().view(ql, hkv, G, D)
        s = torch.einsum("qhgd,hkd->hgqk", qq, K) * scale
        qpos = torch.arange(ctx - ql, ctx, device=q.device)
        kpos = torch.arange(ctx, device=q.device)
        mask = kpos[None, :] > qpos[:, None]
        s = s.masked_fill(mask[None, None], float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hgqk,hkd->qhgd", p, V)
        out[q0:q1] = o.reshape(ql, hq, D).to(q.dtype)
    return out


def ord_key(x: torch.Tensor) -> torch.Tensor:
    """Monotone 16-bit key of the bf16 rounding of x (the kernel's top-k/top-p ranking key)."""
    b = x.to(torch.bfloat16).view(torch.int16).to(torch.int32) & 0xFFFF
    return torch.where(b & 0x8000 != 0, (~b) & 0xFFFF, b | 0x8000)


def topkp_threshold(logits: torch.Tensor, legal: torch.Tensor, top_k: int, top_p: float) -> int:
    """Smallest key kept by top-k / top-p (llama.cpp order: raw logits), ties kept; 0 = no filtering."""
    x = logits.float()[legal]
    if x.numel() == 0:
        return 0
    keys = ord_key(x)
    thr = 0
    if top_k > 0:
        ks = torch.sort(keys, descending=True).values
        thr = max(thr, int(ks[min(top_k, ks.numel()) - 1]))
    if top_p < 1.0:
        mass = torch.exp(x - x.max())
        uk, inv = torch.unique(keys, return_inverse=True)          # ascending unique keys
        km = torch.zeros(uk.numel(), dtype=torch.float64).index_add_(0, inv, mass.double())
        cum = torch.flip(torch.cumsum(torch.flip(km, [0]), 0), [0])   # mass of keys >= uk[i]
        ok = (cum >= top_p * float(mass.sum())).nonzero()
        thr = max(thr, int(uk[int(ok.max())]) if ok.numel() else 0)
    return thr


def constrained_sample(logits, row_of_slot, next_tab, dist, done_state: int, state, remaining, temperature, seed,
                       ids, pos, ctx, nout, out_tokens, topk=None, topp=None, jump=None) -> None:
    """Greedy / Gumbel-max sampling restricted by the token DFA; advances the slot state in place (host loop).
    A row entering a state flagged in ``jump`` is parked as ``-2 - state``."""
    n = state.numel()
    V = next_tab.shape[1]
    for slot in range(n):
        s = int(state[slot])
        if s < 0 or s == done_state:
            continue
        row = int(row_of_slot[slot]) if row_of_slot is not None else slot
        if row < 0:
            continue
        nx = next_tab[s].long()
        budget = int(remaining[slot]) - 1
        legal = (nx >= 0)
        legal &= dist[nx.clamp(min=0)].long() <= budget
        if not bool(legal.any()):
            state[slot] = done_state
            continue
        sc = logits[row, :V].float()
        t = float(temperature[slot]) if temperature is not None else 0.0
        tk = int(topk[slot]) if topk is not None else 0
        tp = float(topp[slot]) if topp is not None else 1.0
        if t > 0 and (tk > 0 or tp < 1.0):
            thr = topkp_threshold(sc, legal, tk, tp)
            legal = legal & (ord_key(sc) >= thr)
        if t > 0:
            g = torch.Generator(device="cpu")
            g.manual_seed((int(seed[slot]) if seed is not None else 0) * 1000003 + int(nout[slot]) * 7919 + slot)
            u = torch.rand(V, generator=g).clamp_(1e-7, 1 - 1e-7).to(sc.device)
            sc = sc / t - torch.log(-torch.log(u))
        sc = sc.masked_fill(~legal, float("-inf"))
        tok = int(torch.argmax(sc))
        ns = int(nx[tok])
        k = int(nout[slot])
        if k < out_tokens.shape[1]:
            out_tokens[slot, k] = tok
        nout[slot] = k + 1
        remaining[slot] = budget
        park = jump is not None and ns != done_state and 0 < int(jump[ns]) <= budget
        state[slot] = -2 - ns if park else ns
        if ns != done_state:
            ids[slot] = tok
            pos[slot] += 1
            ctx[slot] += 1
