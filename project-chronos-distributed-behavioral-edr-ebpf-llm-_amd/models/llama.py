"""Llama-3 / 3.1 for the Brain: config presets, TP-sharded weights, random init,
HF-safetensors and Meta ``consolidated.*.pth`` loaders, and the varlen paged-KV forward.

The reference never holds a model: it POSTs to Ollama's ``llama3`` (chronos_sensor.py:10,118; README.md:21).  This is
the model Ollama served, re-built MI355X-first:

* weights in the layout the kernels want: fused ``wqkv`` [(Hq+2Hkv)*128, d] and ``w_gu`` [2F, d] (one GEMM each),
  bf16, resident for the life of the engine (no lazy load: reference quirk X8 / screenshot chain 1);
* one flattened token stream per step (prefill chunks and decode tokens alike) with per-sequence metadata, so
  continuous batching never pads;
* every non-GEMM op is a gfx950 HIP kernel (chronos.ops); TP collectives sit exactly after the row-parallel GEMMs
  (o_proj, down_proj), the vocab-parallel embedding and the LM head.
"""
from __future__ import annotations

import glob
import json
import math
import os
from dataclasses import asdict, dataclass, field, replace
from typing import Optional

import torch

from .. import ops
from ..parallel.tp import TPContext

# decode steps (T <= 2, TP=1): residual add + norm partials in the producing GEMV's epilogue, the norm in the consuming
# GEMV's prologue, RoPE + paged-KV write in the QKV GEMV's epilogue (CHRONOS_FUSE_NORM=0: the separate kernels)
_FUSE_NORM = os.environ.get("CHRONOS_FUSE_NORM", "1") != "0"
_FUSE_AR_NORM = os.environ.get("CHRONOS_FUSE_AR_NORM", "1") != "0"
# fp8-weight decode (T <= 2): W8A16 GEMVs on bf16 activations with the bf16 path's fused norm / RoPE + KV write /
# residual epilogues instead of W8A8 (an activation-quantisation launch per projection).  Not at T = 3-4: the GEMV's
# per-row-group overhead makes it slower there than the W8A8 GEMMs (gate_up 140 vs 27 us, profiles/r5/w8a16_*)
_W8A16_DECODE = os.environ.get("CHRONOS_W8A16_DECODE", "1") != "0"  # TP: fused IPC all-reduce + residual + RMSNorm
# batched decode (>= 1024 (row, kv head) items, bf16 KV): RoPE + paged-KV write fused into the decode attention
_FUSE_DECODE_ROPE = os.environ.get("CHRONOS_FUSE_DECODE_ROPE", "1") != "0"


@dataclass
class LlamaConfig:
    name: str = "llama3-8b"
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rms_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    max_position: int = 8192
    tie_word_embeddings: bool = False
    init_std: float = 0.02

    @property
    def group(self) -> int:
        return self.num_heads // self.num_kv_heads

    def param_count(self) -> int:
        d, f, v = self.hidden_size, self.intermediate_size, self.vocab_size
        qkv = d * (self.num_heads + 2 * self.num_kv_heads) * self.head_dim
        per = qkv + self.num_heads * self.head_dim * d + 3 * d * f + 2 * d
        return self.num_layers * per + v * d * (1 if self.tie_word_embeddings else 2) + d

    @classmethod
    def from_hf(cls, cfg: dict, name: str = "hf") -> "LlamaConfig":
        return cls(
            name=name,
            vocab_size=cfg["vocab_size"],
            hidden_size=cfg["hidden_size"],
            intermediate_size=cfg["intermediate_size"],
            num_layers=cfg["num_hidden_layers"],
            num_heads=cfg["num_attention_heads"],
            num_kv_heads=cfg.get("num_key_value_heads", cfg["num_attention_heads"]),
            head_dim=cfg.get("head_dim", cfg["hidden_size"] // cfg["num_attention_heads"]),
            rms_eps=cfg.get("rms_norm_eps", 1e-5),
            rope_theta=cfg.get("rope_theta", 10000.0),
            rope_scaling=cfg.get("rope_scaling"),
            max_position=cfg.get("max_position_embeddings", 8192),
            tie_word_embeddings=cfg.get("tie_word_embeddings", False),
        )

    @classmethod
    def from_meta(cls, params: dict, name: str = "meta") -> "LlamaConfig":
        d = params["dim"]
        nh = params["n_heads"]
        mult = params.get("ffn_dim_multiplier", 1.0)
        hidden = int(2 * (4 * d) / 3)
        hidden = int(mult * hidden)
        mo = params.get("multiple_of", 256)
        hidden = mo * ((hidden + mo - 1) // mo)
        scaling = None
        if params.get("use_scaled_rope"):
            scaling = dict(rope_type="llama3", factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0,
                           original_max_position_embeddings=8192)
        return cls(name=name, vocab_size=params.get("vocab_size", 128256), hidden_size=d, intermediate_size=hidden,
                   num_layers=params["n_layers"], num_heads=nh, num_kv_heads=params.get("n_kv_heads", nh),
                   head_dim=d // nh, rms_eps=params.get("norm_eps", 1e-5), rope_theta=params.get("rope_theta", 500000.0),
                   rope_scaling=scaling, max_position=131072 if scaling else 8192)


_LLAMA31_SCALING = dict(rope_type="llama3", factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0,
                        original_max_position_embeddings=8192)

PRESETS: dict[str, LlamaConfig] = {
    "llama3-8b": LlamaConfig(),
    "llama3-70b": LlamaConfig(name="llama3-70b", hidden_size=8192, intermediate_size=28672, num_layers=80,
                              num_heads=64, num_kv_heads=8),
    "llama3.1-8b": LlamaConfig(name="llama3.1-8b", rope_scaling=_LLAMA31_SCALING, max_position=131072),
    "llama3.1-70b": LlamaConfig(name="llama3.1-70b", hidden_size=8192, intermediate_size=28672, num_layers=80,
                                num_heads=64, num_kv_heads=8, rope_scaling=_LLAMA31_SCALING, max_position=131072),
    # test-sized models with the real vocabulary and head_dim (the kernels assume head_dim 128)
    "tiny": LlamaConfig(name="tiny", hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4,
                        num_kv_heads=2, max_position=4096),
    "small": LlamaConfig(name="small", hidden_size=1024, intermediate_size=2816, num_layers=4, num_heads=8,
                         num_kv_heads=2, max_position=8192),
    # the 70B attention geometry (64 q / 8 KV heads: at TP=8 one KV head per rank, GQA group 8) and the real vocab
    # (a 16032-row shard per rank at TP=8, not a multiple of 128) in a CPU-sized model (hidden 256, 2 layers)
    "tiny70": LlamaConfig(name="tiny70", hidden_size=256, intermediate_size=512, num_layers=2, num_heads=64,
                          num_kv_heads=8, max_position=4096),
}


def get_config(name: str) -> LlamaConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; have {sorted(PRESETS)}")
    return replace(PRESETS[name])


# -----------------------------------------------------------------------------------------------------------------
# RoPE tables
# -----------------------------------------------------------------------------------------------------------------


def rope_inv_freq(cfg: LlamaConfig) -> torch.Tensor:
    d = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, d, 2, dtype=torch.float64) / d))
    sc = cfg.rope_scaling
    if sc and sc.get("rope_type", sc.get("type")) == "llama3":
        factor = sc["factor"]
        lo, hi = sc["low_freq_factor"], sc["high_freq_factor"]
        old = sc["original_max_position_embeddings"]
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        inv_l = torch.where(wl > lo_wl, inv / factor, inv)
        smooth = (old / wl - lo) / (hi - lo)
        smoothed = (1 - smooth) * inv_l / factor + smooth * inv_l
        medium = ~(wl < hi_wl) & ~(wl > lo_wl)
        inv = torch.where(medium, smoothed, inv_l)
    return inv


def rope_table(cfg: LlamaConfig, max_pos: int, device=None) -> torch.Tensor:
    """cos_sin[p, 0:64] = cos(p * f), [64:128] = sin(p * f), f32 (consumed by the rope_kv_write kernel)."""
    inv = rope_inv_freq(cfg)
    p = torch.arange(max_pos, dtype=torch.float64)
    fr = torch.outer(p, inv)
    return torch.cat([fr.cos(), fr.sin()], dim=1).float().to(device)


# -----------------------------------------------------------------------------------------------------------------
# weights
# -----------------------------------------------------------------------------------------------------------------


@dataclass
class QTensor:
    """fp8-e4m3 (OCP) projection weight for the W8A8 path (csrc/kernels/fp8.hip): bytes [N, K] uint8 and a
    per-output-channel f32 scale [N], w ~= bytes * scale.  Quantised after TP sharding, so a row-parallel shard's
    scales cover exactly the K-slice it multiplies."""
    q: torch.Tensor
    s: torch.Tensor

    @property
    def shape(self):
        return self.q.shape

    def numel(self) -> int:
        return self.q.numel()

    def nbytes(self) -> int:
        return self.q.numel() + 4 * self.s.numel()


def quantize(w: torch.Tensor) -> QTensor:
    return QTensor(*ops.reference.quantize_weight(w))


@dataclass
class LayerWeights:
    attn_norm: torch.Tensor
    wqkv: "torch.Tensor | QTensor"
    wo: "torch.Tensor | QTensor"
    mlp_norm: torch.Tensor
    w_gu: "torch.Tensor | QTensor"
    w_down: "torch.Tensor | QTensor"


@dataclass
class LlamaWeights:
    embed: torch.Tensor            # [V_local, d] (vocab-parallel shard)
    layers: list
    norm: torch.Tensor
    lm_head: torch.Tensor          # [V_local, d]
    vocab_start: int = 0
    # RMSNorm weights folded into the following projections (W' = W diag(w), norms stored as ones): what the decode
    # GEMV's folded-norm prologue (csrc/kernels/gemv.hip NORMP) relies on
    norms_folded: bool = False

    def nbytes(self) -> int:
        n = 2 * (self.embed.numel() + self.norm.numel() + (0 if self.lm_head is self.embed else self.lm_head.numel()))
        for l in self.layers:
            for t in (l.attn_norm, l.wqkv, l.wo, l.mlp_norm, l.w_gu, l.w_down):
                n += t.nbytes() if isinstance(t, QTensor) else 2 * t.numel()
        return n

    @property
    def fp8(self) -> bool:
        return bool(self.layers) and isinstance(self.layers[0].wqkv, QTensor)


def _shard_rows(t: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    n = t.shape[0] // world
    return t[rank * n:(rank + 1) * n]


def _shard_cols(t: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    n = t.shape[1] // world
    return t[:, rank * n:(rank + 1) * n]


def _local_heads(cfg: LlamaConfig, tp: TPContext) -> tuple[int, int]:
    if cfg.num_heads % tp.world or cfg.num_kv_heads % tp.world:
        raise ValueError(f"TP={tp.world} must divide q heads {cfg.num_heads} and kv heads {cfg.num_kv_heads}")
    return cfg.num_heads // tp.world, cfg.num_kv_heads // tp.world


def fold_norm(wt: torch.Tensor, nw: torch.Tensor) -> torch.Tensor:
    """W diag(nw): an RMSNorm weight folded into the projection that consumes the norm (scales W's input columns, one
    bf16 rounding).  rmsnorm(x) * nw @ W^T == rmsnorm(x) @ (W diag(nw))^T.  A ones vector (random init) is a no-op."""
    if bool((nw == 1).all()):
        return wt
    return (wt.float() * nw.float().to(wt.device)).to(wt.dtype)


def assemble_layer(cfg: LlamaConfig, tp: TPContext, full: dict, device, dtype=torch.bfloat16,
                   weight_dtype: str = "bf16", fold_norms: bool = True) -> LayerWeights:
    """Full (unsharded) HF-named tensors of one layer -> this rank's fused shard (projections quantised to
    per-channel e4m3 when ``weight_dtype == "fp8"``; norms stay bf16).  ``fold_norms``: the input-norm weights are
    folded into QKV / gate_up (before quantisation) and stored as ones."""
    if fold_norms:
        full = dict(full)
        an, mn = full["attn_norm"], full["mlp_norm"]
        for n in ("q", "k", "v"):
            full[n] = fold_norm(full[n], an)
        for n in ("gate", "up"):
            full[n] = fold_norm(full[n], mn)
        full["attn_norm"] = torch.ones_like(an)
        full["mlp_norm"] = torch.ones_like(mn)
    r, w = tp.rank, tp.world
    D = cfg.head_dim
    q = full["q"].view(cfg.num_heads, D, -1)
    k = full["k"].view(cfg.num_kv_heads, D, -1)
    v = full["v"].view(cfg.num_kv_heads, D, -1)
    hq, hkv = _local_heads(cfg, tp)
    qs = q[r * hq:(r + 1) * hq].reshape(hq * D, -1)
    ks = k[r * hkv:(r + 1) * hkv].reshape(hkv * D, -1)
    vs = v[r * hkv:(r + 1) * hkv].reshape(hkv * D, -1)
    wqkv = torch.cat([qs, ks, vs], 0)
    wo = _shard_cols(full["o"], r, w)
    w_gu = torch.cat([_shard_rows(full["gate"], r, w), _shard_rows(full["up"], r, w)], 0)
    w_down = _shard_cols(full["down"], r, w)
    cv = lambda t: t.to(device=device, dtype=dtype).contiguous()  # noqa: E731
    if weight_dtype == "fp8":
        pj = lambda t: quantize(cv(t))  # noqa: E731
    elif weight_dtype == "bf16":
        pj = cv
    else:
        raise ValueError(f"weight_dtype must be 'bf16' or 'fp8', got {weight_dtype!r}")
    return LayerWeights(cv(full["attn_norm"]), pj(wqkv), pj(wo), cv(full["mlp_norm"]), pj(w_gu), pj(w_down))


def random_weights(cfg: LlamaConfig, tp: TPContext | None = None, device="cpu", seed: int = 0,
                   dtype=torch.bfloat16, weight_dtype: str = "bf16", fold_norms: bool = True) -> LlamaWeights:
    """Random-init weights with the real architecture (the benchmark's model; no checkpoints offline).

    Every rank draws the FULL tensor from the same seeded generator and keeps its shard, so a TP run is numerically
    the same model as TP=1.  Generation happens on ``device`` (GPU: ~1 s for 8B).
    """
    tp = tp or TPContext.single()
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    d, f, D = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    std = cfg.init_std

    def rnd(*shape):
        t = torch.empty(*shape, device=dev, dtype=dtype)
        t.normal_(0.0, std, generator=gen)
        return t

    def ones(n):
        return torch.ones(n, device=dev, dtype=dtype)

    gen.manual_seed(seed)
    embed_full = rnd(cfg.vocab_size, d)
    vs = cfg.vocab_size // tp.world
    embed = embed_full[tp.rank * vs:(tp.rank + 1) * vs].contiguous()
    del embed_full
    layers = []
    for i in range(cfg.num_layers):
        gen.manual_seed(seed * 1000003 + i + 1)
        full = dict(
            attn_norm=ones(d),
            q=rnd(cfg.num_heads * D, d), k=rnd(cfg.num_kv_heads * D, d), v=rnd(cfg.num_kv_heads * D, d),
            o=rnd(d, cfg.num_heads * D), mlp_norm=ones(d),
            gate=rnd(f, d), up=rnd(f, d), down=rnd(d, f),
        )
        layers.append(assemble_layer(cfg, tp, full, dev, dtype, weight_dtype, fold_norms))
        del full
    gen.manual_seed(seed * 1000003 + 999983)
    if cfg.tie_word_embeddings:
        lm_head = embed
    else:
        lm_full = rnd(cfg.vocab_size, d)
        lm_head = lm_full[tp.rank * vs:(tp.rank + 1) * vs].contiguous()
        del lm_full
    return LlamaWeights(embed, layers, ones(d), lm_head, vocab_start=tp.rank * vs, norms_folded=fold_norms)


# ---- checkpoint loaders ----------------------------------------------------------------------------------------


def _meta_permute(w: torch.Tensor, n_heads: int) -> torch.Tensor:
    """Meta's interleaved-pair rotary layout -> HF rotate-half layout (the transform convert_llama_weights applies)."""
    d1, d2 = w.shape
    return w.view(n_heads, d1 // n_heads // 2, 2, d2).transpose(1, 2).reshape(d1, d2)


def _final(norm: torch.Tensor, lm_head: torch.Tensor, fold: bool):
    """(norm, lm_head) with the final norm folded into the LM head (a tied head becomes its own copy)."""
    if not fold:
        return norm, lm_head
    return torch.ones_like(norm), fold_norm(lm_head, norm)


def load_hf(path: str, tp: TPContext | None = None, device="cpu", dtype=torch.bfloat16,
            weight_dtype: str = "bf16", fold_norms: bool = True) -> tuple[LlamaConfig, LlamaWeights]:
    """HF layout: config.json + model*.safetensors (tensor names: SURVEY.md App. B)."""
    from safetensors import safe_open

    tp = tp or TPContext.single()
    with open(os.path.join(path, "config.json")) as fh:
        cfg = LlamaConfig.from_hf(json.load(fh), name=os.path.basename(path.rstrip("/")))
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors in {path}")
    index: dict[str, str] = {}
    for fpath in files:
        with safe_open(fpath, framework="pt") as f:
            for k in f.keys():
                index[k] = fpath
    handles: dict[str, object] = {}

    def get(name):
        fp = index[name]
        if fp not in handles:
            handles[fp] = safe_open(fp, framework="pt")
        return handles[fp].get_tensor(name)

    vs = cfg.vocab_size // tp.world
    embed = get("model.embed_tokens.weight")[tp.rank * vs:(tp.rank + 1) * vs].to(device=device, dtype=dtype).contiguous()
    layers = []
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        full = dict(
            attn_norm=get(p + "input_layernorm.weight"), mlp_norm=get(p + "post_attention_layernorm.weight"),
            q=get(p + "self_attn.q_proj.weight"), k=get(p + "self_attn.k_proj.weight"),
            v=get(p + "self_attn.v_proj.weight"), o=get(p + "self_attn.o_proj.weight"),
            gate=get(p + "mlp.gate_proj.weight"), up=get(p + "mlp.up_proj.weight"), down=get(p + "mlp.down_proj.weight"),
        )
        layers.append(assemble_layer(cfg, tp, full, device, dtype, weight_dtype, fold_norms))
    norm = get("model.norm.weight").to(device=device, dtype=dtype)
    if cfg.tie_word_embeddings or "lm_head.weight" not in index:
        lm_head = embed
    else:
        lm_head = get("lm_head.weight")[tp.rank * vs:(tp.rank + 1) * vs].to(device=device, dtype=dtype).contiguous()
    norm, lm_head = _final(norm, lm_head, fold_norms)
    return cfg, LlamaWeights(embed, layers, norm, lm_head, vocab_start=tp.rank * vs, norms_folded=fold_norms)


def load_meta(path: str, tp: TPContext | None = None, device="cpu", dtype=torch.bfloat16,
              weight_dtype: str = "bf16", fold_norms: bool = True) -> tuple[LlamaConfig, LlamaWeights]:
    """Meta layout: params.json + consolidated.NN.pth (model-parallel shards are concatenated back first).
    Loaded with ``weights_only=True`` (no pickled code is ever executed)."""
    tp = tp or TPContext.single()
    with open(os.path.join(path, "params.json")) as fh:
        cfg = LlamaConfig.from_meta(json.load(fh), name=os.path.basename(path.rstrip("/")))
    shards = [torch.load(f, map_location="cpu", weights_only=True, mmap=True)
              for f in sorted(glob.glob(os.path.join(path, "consolidated.*.pth")))]
    if not shards:
        raise FileNotFoundError(f"no consolidated.*.pth in {path}")

    def cat(name, dim):
        ts = [s[name] for s in shards]
        return ts[0] if len(ts) == 1 or ts[0].dim() == 1 else torch.cat(ts, dim)

    vs = cfg.vocab_size // tp.world
    embed = cat("tok_embeddings.weight", 1)[tp.rank * vs:(tp.rank + 1) * vs].to(device=device, dtype=dtype).contiguous()
    layers = []
    for i in range(cfg.num_layers):
        p = f"layers.{i}."
        full = dict(
            attn_norm=cat(p + "attention_norm.weight", 0), mlp_norm=cat(p + "ffn_norm.weight", 0),
            q=_meta_permute(cat(p + "attention.wq.weight", 0), cfg.num_heads),
            k=_meta_permute(cat(p + "attention.wk.weight", 0), cfg.num_kv_heads),
            v=cat(p + "attention.wv.weight", 0), o=cat(p + "attention.wo.weight", 1),
            gate=cat(p + "feed_forward.w1.weight", 0), up=cat(p + "feed_forward.w3.weight", 0),
            down=cat(p + "feed_forward.w2.weight", 1),
        )
        layers.append(assemble_layer(cfg, tp, full, device, dtype, weight_dtype, fold_norms))
    norm = cat("norm.weight", 0).to(device=device, dtype=dtype)
    lm_head = cat("output.weight", 0)[tp.rank * vs:(tp.rank + 1) * vs].to(device=device, dtype=dtype).contiguous()
    norm, lm_head = _final(norm, lm_head, fold_norms)
    return cfg, LlamaWeights(embed, layers, norm, lm_head, vocab_start=tp.rank * vs, norms_folded=fold_norms)


def load_checkpoint(path: str, tp: TPContext | None = None, device="cpu", weight_dtype: str = "bf16",
                    fold_norms: bool = True):
    if os.path.exists(os.path.join(path, "config.json")):
        return load_hf(path, tp, device, weight_dtype=weight_dtype, fold_norms=fold_norms)
    if os.path.exists(os.path.join(path, "params.json")):
        return load_meta(path, tp, device, weight_dtype=weight_dtype, fold_norms=fold_norms)
    raise FileNotFoundError(f"{path}: neither an HF (config.json) nor a Meta (params.json) Llama checkpoint")


# -----------------------------------------------------------------------------------------------------------------
# KV cache + step metadata
# -----------------------------------------------------------------------------------------------------------------


class KVCache:
    """Paged KV: per layer K [NB, Hkv, BS, 128] (token rows) and V [NB, Hkv, 128, BS] (transposed, attention.hip).

    One allocation for all layers, sized from the HBM budget (288 GB per MI355X).
    """

    def __init__(self, cfg: LlamaConfig, tp: TPContext, num_blocks: int, block_size: int = 16, device="cpu",
                 dtype: str = "bf16", k_scale: float = 1.0, v_scale: float = 1.0):
        _, hkv = _local_heads(cfg, tp)
        self.num_blocks, self.block_size, self.hkv = num_blocks, block_size, hkv
        self.dtype = dtype
        per = hkv * block_size * cfg.head_dim
        tdt = torch.uint8 if dtype == "fp8" else torch.bfloat16  # fp8 = OCP e4m3fn bytes + per-layer scale
        self.buf = torch.zeros(cfg.num_layers, 2, num_blocks, per, device=device, dtype=tdt)
        self.k_scale = [float(k_scale)] * cfg.num_layers
        self.v_scale = [float(v_scale)] * cfg.num_layers
        self.k = [self.buf[l, 0].view(num_blocks, hkv, block_size, cfg.head_dim) for l in range(cfg.num_layers)]
        self.v = [self.buf[l, 1].view(num_blocks, hkv, cfg.head_dim, block_size) for l in range(cfg.num_layers)]

    @staticmethod
    def bytes_per_block(cfg: LlamaConfig, tp: TPContext, block_size: int = 16, dtype: str = "bf16") -> int:
        _, hkv = _local_heads(cfg, tp)
        return cfg.num_layers * 2 * hkv * block_size * cfg.head_dim * (1 if dtype == "fp8" else 2)


@dataclass
class StepBatch:
    """One forward step over a flattened token stream (any mix of prefill chunks and decode tokens)."""
    ids: torch.Tensor          # [T] int32
    pos: torch.Tensor          # [T] int32
    tok_seq: torch.Tensor      # [T] int32  token -> row of block_table / ctx_len
    block_table: torch.Tensor  # [B, max_blocks] int32
    q_start: torch.Tensor      # [B+1] int32
    ctx_len: torch.Tensor      # [B] int32 kv length after this step
    last_idx: torch.Tensor     # [B] int64 token index whose logits are wanted
    tiles: Optional[torch.Tensor]  # [ntiles, 2] int32, None = decode mode (one token per sequence, seq i = token i)
    ntiles: int
    nqt: int = 1
    nsplit: int = 1
    # micro-batches over contiguous sequence ranges (TP prefill): the forward interleaves them layer by layer so the
    # RCCL all-reduce of one runs on its stream while the other computes (LlamaModel.forward)
    parts: Optional[list] = None
    # context-parallel prefill (parallel/context_parallel.py): this rank holds part of a long chunk; K/V are
    # all-gathered per layer and written for every token of the chunk
    cp: Optional[object] = None
    # mixed step: decode rows (a decode-mode StepBatch over device slot state) appended after this batch's prefill
    # tokens — one forward, shared projections; ``last_idx`` then also lists the decode rows (after the prefill rows)
    dec: Optional["StepBatch"] = None
    # decode rows: cascade attention over a shared prompt prefix (ops.decode_attention_rope ``casc``), device tensors
    # owned by the engine and updated in place between graph replays
    casc: Optional[tuple] = None
    # a few tokens per sequence over long contexts (jump-forward forwards): (max tokens per sequence, kv splits) —
    # the split-K decode kernel with all of a sequence's tokens in one pass over its K/V (ops.paged_attention
    # max_q) instead of the prefill tiles, whose per-tile workgroups each stream the whole context
    rows_dec: Optional[tuple] = None


# decode-form attention for tiny chunks over long contexts (StepBatch.rows_dec): at least this much context (the
# chunk's tokens per sequence x GQA group must fit the kernel's 16 query rows)
ROWS_DEC_MIN_CTX = int(os.environ.get("CHRONOS_ROWS_DEC_MIN_CTX", "2048"))


def make_prefill_batch(prompts: list[list[int]], starts: list[int], block_tables: list[list[int]], cfg: LlamaConfig,
                       tp: TPContext, device, max_blocks: int | None = None, nqt: int = 2,
                       ctx_totals: list[int] | None = None, split: int = 1) -> StepBatch:
    """Host builder for a (chunked) prefill step.  prompts[b] are the tokens of this chunk, starts[b] the position of
    its first token (prefix already in the cache).  ``split > 1`` also builds that many token-balanced micro-batches
    of whole sequences (``StepBatch.parts``) for communication/compute overlap under tensor parallelism."""
    if split > 1 and len(prompts) >= split:
        total = sum(len(t) for t in prompts)
        cuts, acc, b0 = [], 0, 0
        for b, t in enumerate(prompts):
            acc += len(t)
            if len(cuts) < split - 1 and acc >= total * (len(cuts) + 1) / split and b + 1 < len(prompts):
                cuts.append(b + 1)
        bounds = [0] + cuts + [len(prompts)]
        whole = make_prefill_batch(prompts, starts, block_tables, cfg, tp, device, max_blocks, nqt, ctx_totals)
        whole.parts = [make_prefill_batch(prompts[a:b], starts[a:b], block_tables[a:b], cfg, tp, device, max_blocks,
                                          nqt) for a, b in zip(bounds, bounds[1:]) if b > a]
        if len(whole.parts) < 2:
            whole.parts = None
        return whole
    hq, hkv = _local_heads(cfg, tp)
    ids, pos, tok_seq, qs = [], [], [], [0]
    for b, (toks, s0) in enumerate(zip(prompts, starts)):
        ids += toks
        pos += list(range(s0, s0 + len(toks)))
        tok_seq += [b] * len(toks)
        qs.append(qs[-1] + len(toks))
    ctx = [s0 + len(t) for t, s0 in zip(prompts, starts)]
    mb = max_blocks or max(len(x) for x in block_tables)
    bt = torch.zeros(len(prompts), mb, dtype=torch.int32)
    for b, blks in enumerate(block_tables):
        bt[b, :len(blks)] = torch.tensor(blks, dtype=torch.int32)
    tiles = ops.attention_tiles([len(t) for t in prompts], hq, hkv, nqt)
    nsplit = ops.pick_nsplit(len(tiles) * hkv, max(ctx)) if prompts else 1
    last = torch.tensor([q - 1 for q in qs[1:]], dtype=torch.int64)
    it = lambda x: torch.tensor(x, dtype=torch.int32)  # noqa: E731
    sb = StepBatch(it(ids), it(pos), it(tok_seq), bt, it(qs), it(ctx), last,
                   torch.tensor(tiles, dtype=torch.int32).view(-1, 2), len(tiles), nqt, nsplit)
    mq = max((len(t) for t in prompts), default=0)
    if prompts and mq * (hq // hkv) <= 16 and max(ctx) >= ROWS_DEC_MIN_CTX and ctx_totals is None:
        sb.rows_dec = (mq, ops.pick_nsplit(len(prompts) * hkv, max(ctx)))
    return to_device(sb, device)


def h2d(t: torch.Tensor | None, device) -> torch.Tensor | None:
    """Host->device copy that never stalls the host: a pageable-memory copy waits for the stream to drain first, a
    pinned one (PyTorch's caching host allocator) is queued, so the host builds the next batch while the GPU runs."""
    if t is None:
        return None
    if torch.device(device).type == "cuda":
        t = t.pin_memory()
    return t.to(device, non_blocking=True)


def to_device(sb: StepBatch, device) -> StepBatch:
    mv = lambda t: h2d(t, device)  # noqa: E731
    return StepBatch(mv(sb.ids), mv(sb.pos), mv(sb.tok_seq), mv(sb.block_table), mv(sb.q_start), mv(sb.ctx_len),
                     mv(sb.last_idx), mv(sb.tiles), sb.ntiles, sb.nqt, sb.nsplit, sb.parts, sb.cp, sb.dec, sb.casc,
                     sb.rows_dec)


# -----------------------------------------------------------------------------------------------------------------
# model
# -----------------------------------------------------------------------------------------------------------------


class LlamaModel:
    def __init__(self, cfg: LlamaConfig, weights: LlamaWeights, tp: TPContext | None = None, device="cpu",
                 max_position: int | None = None):
        self.cfg, self.w = cfg, weights
        self.tp = tp or TPContext.single()
        self.device = torch.device(device)
        self.hq, self.hkv = _local_heads(cfg, self.tp)
        self.cos_sin = rope_table(cfg, max_position or cfg.max_position, self.device)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        # Megatron-style sequence parallelism for TP prefill (set by the engine, EngineConfig.tp_sequence_parallel)
        self.sequence_parallel = False
        # TP decode comm/compute overlap (set by the engine, EngineConfig.tp_decode_overlap): decode batches of at least
        # this many rows run as two row halves whose fused IPC all-reduce + residual + RMSNorm launches go to a second
        # HIP stream, each overlapping the other half's attention / MLP (0 = off)
        self.decode_overlap_rows = 0
        self._comm = None

    # ---- one micro-batch's pieces of a layer (bf16: x is a tensor; W8A8: x is (e4m3 bytes, row scales)) ----------
    def _norm(self, h, st: dict, w: torch.Tensor, first: bool = False, reduce: bool = False):
        """(st["resid"] <- h + st["resid"]) and the normalised projection input (first: the residual stream starts as
        h itself).  When h is an ops.ResidOut (a decode producer already added the residual and summed the squares)
        the result is an ops.LazyNorm that the consuming GEMV folds into its prologue: no norm launch.  ``reduce``: h
        is still this rank's partial sum; the TP all-reduce, residual add and norm run as one fused IPC launch."""
        eps = self.cfg.rms_eps
        if reduce:
            return self.tp.all_reduce_add_rmsnorm(h, st["resid"], w, eps)
        if isinstance(h, ops.ResidOut):
            st["resid"] = h.s
            return ops.LazyNorm(h.s, h.part, w, eps)
        resid = None if first else st["resid"]
        if self.w.fp8 and not st.get("w16"):
            return ops.quant_rows(h, resid, w, eps, 1 if resid is None else 2)
        return ops.rmsnorm(h, w, eps) if resid is None else ops.add_rmsnorm(h, resid, w, eps)

    def _out_proj(self, x: torch.Tensor, w: torch.Tensor, st: dict):
        """Row-parallel output projection (o_proj / down_proj).  TP=1: the producer that also adds the residual and
        emits the next RMSNorm's partial sums (ops.ResidOut: the decode GEMV at T <= 2, the batched GEMM's kResid
        epilogue above, prefill included) — the norm then costs no launch: its consumer (QKV / gate_up / LM head)
        applies it as a per-row scale."""
        T = st["T"]
        if (_FUSE_NORM and self.w.norms_folded and self.tp.world == 1 and x.is_cuda and st["sb"].cp is None
                and (st["sb"].tiles is None or T > 2) and ops.resid_ok(T, w.shape[0], w.shape[1], ops.is_q(w))):
            return ops.gemv_resid(x, w, st["resid"])
        return ops.linear(x, w)

    def _attn_rows(self, li: int, qkv: torch.Tensor, sb: StepBatch, q_buf: torch.Tensor, kv: KVCache) -> torch.Tensor:
        """RoPE + paged-KV write + attention for the rows of one step batch (prefill tiles or decode rows)."""
        T = qkv.shape[0]
        attn = None
        if _FUSE_DECODE_ROPE and sb.tiles is None and sb.cp is None and sb.nqt == 1 and sb.nsplit == 1:
            # batched decode: RoPE + KV write inside the one-wave decode attention (None off its shapes)
            attn = ops.decode_attention_rope(qkv, sb.pos, self.cos_sin, kv.k[li], kv.v[li], sb.block_table,
                                             sb.ctx_len, T, self.hq, self.scale, sb.casc)
        if attn is None:
            ops.rope_kv_write(qkv, sb.pos, sb.tok_seq, sb.block_table, self.cos_sin, q_buf, kv.k[li], kv.v[li],
                              self.hq, self.hkv, True, kv.k_scale[li], kv.v_scale[li])
        if sb.cp is not None:  # CP: every rank writes the whole chunk's K/V before any rank attends
            from ..parallel.context_parallel import gather_kv

            cp = sb.cp
            ops.rope_kv_write(gather_kv(qkv, self.hq, cp), cp.pos_all, cp.seq_all, cp.bt, self.cos_sin,
                              cp.dummy_q, kv.k[li], kv.v[li], 0, self.hkv, False, kv.k_scale[li], kv.v_scale[li])
        if sb.cp is not None and sb.cp.ulysses is not None:  # head-sharded attention of the whole chunk
            from ..parallel.context_parallel import ulysses_attention

            return ulysses_attention(q_buf, kv.k[li], kv.v[li], sb.cp, self.scale, kv.k_scale[li], kv.v_scale[li])
        if attn is None and sb.rows_dec is not None and sb.cp is None:
            mq, ns = sb.rows_dec  # every sequence's few tokens in one pass over its K/V
            attn = ops.paged_attention(q_buf, kv.k[li], kv.v[li], sb.block_table, sb.q_start, sb.ctx_len, None,
                                       sb.q_start.numel() - 1, 1, ns, self.scale, kv.k_scale[li], kv.v_scale[li],
                                       max_q=mq)
        if attn is None:
            attn = ops.paged_attention(q_buf, kv.k[li], kv.v[li], sb.block_table, sb.q_start, sb.ctx_len, sb.tiles,
                                       sb.ntiles, sb.nqt, sb.nsplit, self.scale, kv.k_scale[li], kv.v_scale[li])
        return attn.view(T, -1)

    def _attn(self, li: int, lw: LayerWeights, st: dict, kv: KVCache) -> torch.Tensor:
        """Attention block up to the row-parallel o_proj; returns this rank's partial sum.  A mixed step (``sb.dec``)
        runs the projections over prefill and decode rows together and the attention of each part with its own
        kernel (flash / split-K prefill tiles; the decode kernel for the one-token rows)."""
        sb, T, x = st["sb"], st["T"], st["x"]
        q8 = self.w.fp8 and not st.get("w16")  # W8A8: x is (e4m3 bytes, row scales)
        if (sb.dec is None and not q8 and _FUSE_NORM and ops.qkv_rope(
                x, lw.wqkv, sb.pos, sb.tok_seq, sb.block_table, self.cos_sin, st["q_buf"], kv.k[li], kv.v[li],
                self.hq, self.hkv, kv.k_scale[li], kv.v_scale[li])):
            # decode: QKV GEMV (+ folded norm) + RoPE / paged-KV write in one launch
            attn = ops.paged_attention(st["q_buf"], kv.k[li], kv.v[li], sb.block_table, sb.q_start, sb.ctx_len,
                                       sb.tiles, sb.ntiles, sb.nqt, sb.nsplit, self.scale, kv.k_scale[li],
                                       kv.v_scale[li]).view(T, -1)
        else:
            # a LazyNorm input goes straight to the projection (the batched GEMM applies the folded norm as a row
            # scale; anything else materialises it)
            qkv = ops.qlinear(*x, lw.wqkv.q, lw.wqkv.s) if q8 else ops.linear(x, lw.wqkv)
            if sb.dec is None:
                attn = self._attn_rows(li, qkv, sb, st["q_buf"], kv)
            else:
                tp_ = T - sb.dec.ntiles
                attn = torch.cat([self._attn_rows(li, qkv[:tp_], sb, st["q_buf"][:tp_], kv),
                                  self._attn_rows(li, qkv[tp_:], sb.dec, st["q_buf"][tp_:], kv)])
        if q8:
            return ops.qlinear(*ops.quant_rows(attn), lw.wo.q, lw.wo.s)
        return self._out_proj(attn, lw.wo, st)

    def _mlp(self, lw: LayerWeights, st: dict) -> torch.Tensor:
        """SwiGLU MLP up to the row-parallel down_proj; returns this rank's partial sum."""
        x = st["x"]
        if self.w.fp8 and not st.get("w16"):
            return ops.qlinear(*ops.qgate_up_quant(*x, lw.w_gu.q, lw.w_gu.s), lw.w_down.q, lw.w_down.s)
        return self._out_proj(ops.gate_up_silu(x, lw.w_gu), lw.w_down, st)

    def _forward_sp(self, sb: StepBatch, kv: KVCache, logits_dtype) -> torch.Tensor:
        """TP prefill with sequence parallelism (SURVEY.md §2.5 "Sequence parallel"): every row-parallel output is
        reduce-SCATTERED over the token rows instead of all-reduced, so the residual stream lives sharded ([T/W, d]
        per rank) and each rank adds + normalises only its own rows; the normalised rows are all-gathered in front
        of the next column-parallel GEMM.  Same bytes on the wire as the all-reduce form, 1/W of the norm/residual
        work and memory.  T is padded to a multiple of W with zero rows (dropped before the projections)."""
        cfg, w, tp = self.cfg, self.w, self.tp
        T = sb.ids.numel()
        Tp = -(-T // tp.world) * tp.world
        eps = cfg.rms_eps
        emb = ops.embedding(sb.ids, w.embed, w.vocab_start)
        resid = tp.reduce_scatter_rows(_pad_rows(emb, Tp))  # vocab-parallel embedding: partial rows -> shard
        st = dict(sb=sb, T=T, resid=resid, q_buf=torch.empty(T, self.hq, cfg.head_dim, device=emb.device,
                                                             dtype=emb.dtype))
        xs = ops.rmsnorm(resid, w.layers[0].attn_norm, eps)
        L = len(w.layers)
        for li, lw in enumerate(w.layers):
            st["x"] = tp.all_gather_rows(xs)[:T]
            o = tp.reduce_scatter_rows(_pad_rows(self._attn(li, lw, st, kv), Tp))
            st["x"] = tp.all_gather_rows(ops.add_rmsnorm(o, st["resid"], lw.mlp_norm, eps))[:T]
            dn = tp.reduce_scatter_rows(_pad_rows(self._mlp(lw, st), Tp))
            xs = ops.add_rmsnorm(dn, st["resid"], w.layers[li + 1].attn_norm if li + 1 < L else w.norm, eps)
        x = tp.all_gather_rows(xs)[:T].index_select(0, sb.last_idx)
        logits = tp.all_gather_last(ops.linear(x, w.lm_head))
        return logits if logits.dtype == logits_dtype else logits.to(logits_dtype)

    def _decode_halves(self, sb: StepBatch) -> list:
        """Two decode-mode StepBatches over rows [0, h) and [h, n) of a decode batch (views of the slot state: decode
        rows are seq i = token i, q_start / tok_seq / last_idx are aranges, so each half re-uses their prefix)."""
        n = sb.ntiles
        h = (n + 1) // 2
        halves = []
        for a, b in ((0, h), (h, n)):
            m = b - a
            halves.append(StepBatch(sb.ids[a:b], sb.pos[a:b], sb.tok_seq[:m], sb.block_table[a:b], sb.q_start[:m + 1],
                                    sb.ctx_len[a:b], sb.last_idx[:m], None, m, sb.nqt, sb.nsplit))
        return halves

    def _forward_dec_overlap(self, sb: StepBatch, kv: KVCache, logits_dtype) -> torch.Tensor:
        """TP decode with comm/compute overlap: the batch's two row halves A, B run
        layer by layer on the compute stream while every row-parallel projection's all-reduce — the fused IPC one-shot
        + residual add + RMSNorm — runs on a second stream (``self._comm``), ordered by events:

            compute: attn(A) | attn(B) | wait ARo(A) mlp(A) | wait ARo(B) mlp(B) | wait ARd(A) attn'(A) | wait ARd(B) ..
            comm:            ARo(A)   ARo(B)               ARd(A)             ARd(B)

        so half A's all-reduce hides behind half B's compute and vice versa.  All all-reduces share ONE stream, issued
        in the same order on every rank (the IPC kernel's epoch lives on the device: one sequence per rank).  Both
        streams are captured into the decode hipGraph (the side stream forks from and joins the compute stream through
        events).  Allocator safety without record_stream (which graph capture does not like): every comm-stream launch
        first waits for the compute stream's current tail, and a compute-stream tensor the comm stream reads (the
        partial sums) stays referenced until the compute stream has waited for that launch."""
        cfg, w, tp = self.cfg, self.w, self.tp
        main = torch.cuda.current_stream(self.device)
        if self._comm is None:
            self._comm = torch.cuda.Stream(self.device)
        comm = self._comm
        eps = cfg.rms_eps

        def ar_norm(st, hpart, wn):
            ev = torch.cuda.Event()
            ev.record(main)
            comm.wait_event(ev)
            with torch.cuda.stream(comm):
                x = tp.all_reduce_add_rmsnorm(hpart, st["resid"], wn, eps)
            done = torch.cuda.Event()
            done.record(comm)
            return x, done, hpart

        states = []
        for p in self._decode_halves(sb):
            h = tp.all_reduce(ops.embedding(p.ids, w.embed, w.vocab_start))
            T = p.ids.numel()
            st = dict(sb=p, T=T, resid=h, q_buf=torch.empty(T, self.hq, cfg.head_dim, device=h.device, dtype=h.dtype))
            st["x"] = self._norm(h, st, w.layers[0].attn_norm, first=True)
            states.append(st)
        L = len(w.layers)
        # each half waits for its own previous down all-reduce only right before its next attention, so half B's
        # down all-reduce runs beside half A's next attention (and half A's beside half B's MLP)
        pend_d = [None] * len(states)
        for li, lw in enumerate(w.layers):
            pend = []
            for i, st in enumerate(states):
                if pend_d[i] is not None:
                    x, done, _ = pend_d[i]
                    main.wait_event(done)
                    st["x"] = x
                    pend_d[i] = None
                pend.append(ar_norm(st, self._attn(li, lw, st, kv), lw.mlp_norm))
            for i, (st, (x, done, _)) in enumerate(zip(states, pend)):
                main.wait_event(done)
                st["x"] = x
                nxt = w.layers[li + 1].attn_norm if li + 1 < L else w.norm
                pend_d[i] = ar_norm(st, self._mlp(lw, st), nxt)
            del pend
        for i, st in enumerate(states):
            x, done, _ = pend_d[i]
            main.wait_event(done)
            st["x"] = x
        del pend_d
        logits = ops.linear(torch.cat([st["x"] for st in states]), w.lm_head)
        logits = tp.all_gather_last(logits)
        return logits if logits.dtype == logits_dtype else logits.to(logits_dtype)

    def forward(self, sb: StepBatch, kv: KVCache, logits_dtype=torch.bfloat16) -> torch.Tensor:
        """Returns logits [B, V] for the token at sb.last_idx of every sequence (full vocab on every TP rank).

        With TP and ``sb.parts`` (prefill), the micro-batches run interleaved: every layer issues each part's o_proj
        all-reduce asynchronously (RCCL runs it on its own HIP stream) and moves on to the next part's attention, then
        waits for it before that part's MLP, whose down_proj all-reduce in turn overlaps the next part's MLP / the next
        layer's attention — xGMI time hides behind compute instead of adding to it (SURVEY.md §5.8 overlap).
        Single part (decode, TP=1): the same ops in the same order with synchronous all-reduces (graph-capturable, the
        IPC one-shot kernel for decode-sized messages)."""
        cfg, w, tp = self.cfg, self.w, self.tp
        if (tp.world > 1 and sb.tiles is not None and self.sequence_parallel and not w.fp8 and sb.cp is None
                and sb.dec is None):
            return self._forward_sp(sb, kv, logits_dtype)
        if (0 < self.decode_overlap_rows and max(2, self.decode_overlap_rows) <= sb.ntiles and sb.tiles is None
                and sb.dec is None and sb.cp is None
                and tp.world > 1 and tp.fast_allreduce_norm is not None and not w.fp8 and _FUSE_AR_NORM
                and self.device.type == "cuda"):
            return self._forward_dec_overlap(sb, kv, logits_dtype)
        parts = sb.parts if (sb.parts and tp.world > 1) else [sb]
        overlap = len(parts) > 1
        # TP, one part: the all-reduce after o_proj / down_proj is fused with the residual add + RMSNorm that follows
        # (IPC kernel; tp.all_reduce_add_rmsnorm falls back to the two steps for messages it cannot take)
        fuse = (not overlap and tp.world > 1 and tp.fast_allreduce_norm is not None and not w.fp8 and _FUSE_AR_NORM)
        if overlap:
            ar = lambda t: tp.all_reduce_async(t)  # noqa: E731
        elif fuse:
            ar = lambda t: (t, None)  # noqa: E731 — reduced inside _norm
        else:
            ar = lambda t: (tp.all_reduce(t), None)  # noqa: E731
        states = []
        for p in parts:
            ids = p.ids if p.dec is None else torch.cat([p.ids, p.dec.ids])
            h = tp.all_reduce(ops.embedding(ids, w.embed, w.vocab_start))
            T = ids.numel()
            st = dict(sb=p, T=T, resid=h, q_buf=torch.empty(T, self.hq, cfg.head_dim, device=h.device, dtype=h.dtype),
                      w16=(w.fp8 and _W8A16_DECODE and T <= 2 and h.is_cuda and p.cp is None and p.dec is None
                           and cfg.hidden_size % 1024 == 0))
            st["x"] = self._norm(h, st, w.layers[0].attn_norm, first=True)
            states.append(st)
        L = len(w.layers)
        for li, lw in enumerate(w.layers):
            pend = [ar(self._attn(li, lw, st, kv)) for st in states]
            pend2 = []
            for st, (o, work) in zip(states, pend):
                if work is not None:
                    work.wait()
                st["x"] = self._norm(o, st, lw.mlp_norm, reduce=fuse)
                pend2.append(ar(self._mlp(lw, st)))
            for st, (dn, work) in zip(states, pend2):
                if work is not None:
                    work.wait()
                if li + 1 < L:
                    st["x"] = self._norm(dn, st, w.layers[li + 1].attn_norm, reduce=fuse)
                elif isinstance(dn, ops.ResidOut) and st["sb"].tiles is None:  # decode: every token is sampled
                    st["x"] = self._norm(dn, st, w.norm)
                elif fuse and st["sb"].tiles is None:  # TP decode: every token is sampled
                    st["x"] = self._norm(dn, st, w.norm, reduce=True)
                elif isinstance(dn, ops.ResidOut):  # prefill producer: the sampled rows' stream and partials
                    li_ = st["sb"].last_idx
                    st["x"] = ops.LazyNorm(dn.s.index_select(0, li_), dn.part.index_select(0, li_), w.norm,
                                           cfg.rms_eps)
                else:  # only the sampled rows need the final norm + LM head (bf16)
                    if fuse:
                        dn = tp.all_reduce(dn)
                    li_ = st["sb"].last_idx
                    st["x"] = ops.add_rmsnorm(dn.index_select(0, li_), st["resid"].index_select(0, li_), w.norm,
                                              cfg.rms_eps)
        x = states[0]["x"] if len(states) == 1 else torch.cat([ops.LazyNorm.force(st["x"]) for st in states])
        logits = ops.linear(x, w.lm_head)
        logits = tp.all_gather_last(logits)
        return logits if logits.dtype == logits_dtype else logits.to(logits_dtype)


def _pad_rows(x: torch.Tensor, rows: int) -> torch.Tensor:
    if x.shape[0] == rows:
        return x
    out = torch.zeros((rows,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    out[:x.shape[0]] = x
    return out


def build_model(preset: str | LlamaConfig = "tiny", device="cpu", tp: TPContext | None = None, seed: int = 0,
                checkpoint: str | None = None, max_position: int | None = None,
                weight_dtype: str = "bf16") -> LlamaModel:
    """``weight_dtype="fp8"``: projections as per-channel e4m3 + W8A8 fp8 MFMA GEMMs (embedding, norms, LM head, attention
    and the KV cache keep their own dtypes)."""
    tp = tp or TPContext.single()
    if checkpoint:
        cfg, w = load_checkpoint(checkpoint, tp, device, weight_dtype)
    else:
        cfg = preset if isinstance(preset, LlamaConfig) else get_config(preset)
        w = random_weights(cfg, tp, device, seed, weight_dtype=weight_dtype)
    return LlamaModel(cfg, w, tp, device, max_position)


def config_dict(cfg: LlamaConfig) -> dict:
    return asdict(cfg)
