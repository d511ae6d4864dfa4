"""Checkpoint loaders: HF safetensors and Meta consolidated.*.pth round-trip to the same model.

No Llama-3 weights exist offline, so the test writes tiny checkpoints in both layouts from one set of random tensors
(the Meta files get the interleaved-rotary q/k layout by inverting the HF conversion) and checks every loader
produces identical logits — including TP=2 sharding at load time.
"""
import json
import os

import torch

from chronos.models.llama import KVCache, LlamaConfig, LlamaModel, load_checkpoint, make_prefill_batch
from chronos.parallel.tp import TPContext


def get_config(_name):
    # head_dim 128 (the kernels' contract) must equal hidden / heads for the Meta format, which has no head_dim field
    return LlamaConfig(name="ckpt-test", vocab_size=4096, hidden_size=512, intermediate_size=1024, num_layers=2,
                       num_heads=4, num_kv_heads=2, max_position=4096)


def _hf_tensors(cfg, seed=0):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: (torch.randn(*s, generator=g) * 0.02).to(torch.bfloat16)  # noqa: E731
    d, f, D = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    t = {"model.embed_tokens.weight": r(cfg.vocab_size, d), "model.norm.weight": torch.ones(d, dtype=torch.bfloat16),
         "lm_head.weight": r(cfg.vocab_size, d)}
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        t[p + "input_layernorm.weight"] = (1 + torch.rand(d, generator=g) * 0.1).to(torch.bfloat16)
        t[p + "post_attention_layernorm.weight"] = (1 + torch.rand(d, generator=g) * 0.1).to(torch.bfloat16)
        t[p + "self_attn.q_proj.weight"] = r(cfg.num_heads * D, d)
        t[p + "self_attn.k_proj.weight"] = r(cfg.num_kv_heads * D, d)
        t[p + "self_attn.v_proj.weight"] = r(cfg.num_kv_heads * D, d)
        t[p + "self_attn.o_proj.weight"] = r(d, cfg.num_heads * D)
        t[p + "mlp.gate_proj.weight"] = r(f, d)
        t[p + "mlp.up_proj.weight"] = r(f, d)
        t[p + "mlp.down_proj.weight"] = r(d, f)
    return t


def _write_hf(path, cfg, t):
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as fh:
        json.dump({"vocab_size": cfg.vocab_size, "hidden_size": cfg.hidden_size,
                   "intermediate_size": cfg.intermediate_size, "num_hidden_layers": cfg.num_layers,
                   "num_attention_heads": cfg.num_heads, "num_key_value_heads": cfg.num_kv_heads,
                   "rms_norm_eps": cfg.rms_eps, "rope_theta": cfg.rope_theta, "max_position_embeddings": 4096}, fh)
    keys = sorted(t)
    half = len(keys) // 2  # two shards, like the real multi-file checkpoints
    save_file({k: t[k] for k in keys[:half]}, os.path.join(path, "model-00001-of-00002.safetensors"))
    save_file({k: t[k] for k in keys[half:]}, os.path.join(path, "model-00002-of-00002.safetensors"))


def _unpermute(w, n_heads):
    d1, d2 = w.shape
    return w.view(n_heads, 2, d1 // n_heads // 2, d2).transpose(1, 2).reshape(d1, d2)


def _write_meta(path, cfg, t):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "params.json"), "w") as fh:
        json.dump({"dim": cfg.hidden_size, "n_layers": cfg.num_layers, "n_heads": cfg.num_heads,
                   "n_kv_heads": cfg.num_kv_heads, "vocab_size": cfg.vocab_size, "multiple_of": 256,
                   "ffn_dim_multiplier": cfg.intermediate_size / int(2 * 4 * cfg.hidden_size / 3),
                   "norm_eps": cfg.rms_eps, "rope_theta": cfg.rope_theta}, fh)
    m = {"tok_embeddings.weight": t["model.embed_tokens.weight"], "norm.weight": t["model.norm.weight"],
         "output.weight": t["lm_head.weight"]}
    for i in range(cfg.num_layers):
        p, q = f"model.layers.{i}.", f"layers.{i}."
        m[q + "attention_norm.weight"] = t[p + "input_layernorm.weight"]
        m[q + "ffn_norm.weight"] = t[p + "post_attention_layernorm.weight"]
        m[q + "attention.wq.weight"] = _unpermute(t[p + "self_attn.q_proj.weight"], cfg.num_heads)
        m[q + "attention.wk.weight"] = _unpermute(t[p + "self_attn.k_proj.weight"], cfg.num_kv_heads)
        m[q + "attention.wv.weight"] = t[p + "self_attn.v_proj.weight"]
        m[q + "attention.wo.weight"] = t[p + "self_attn.o_proj.weight"]
        m[q + "feed_forward.w1.weight"] = t[p + "mlp.gate_proj.weight"]
        m[q + "feed_forward.w3.weight"] = t[p + "mlp.up_proj.weight"]
        m[q + "feed_forward.w2.weight"] = t[p + "mlp.down_proj.weight"]
    torch.save(m, os.path.join(path, "consolidated.00.pth"))


def _logits(cfg, w, tp=None):
    tp = tp or TPContext.single()
    model = LlamaModel(cfg, w, tp, "cpu")
    kv = KVCache(cfg, tp, 8, 16, "cpu")
    sb = make_prefill_batch([list(range(1000, 1037)), [5, 6, 7]], [0, 0], [[1, 2, 3], [4]], cfg, tp, "cpu",
                            max_blocks=3)
    return model.forward(sb, kv).float()


def test_hf_and_meta_loaders_agree(tmp_path):
    cfg = get_config("tiny")
    t = _hf_tensors(cfg)
    _write_hf(str(tmp_path / "hf"), cfg, t)
    _write_meta(str(tmp_path / "meta"), cfg, t)
    c1, w1 = load_checkpoint(str(tmp_path / "hf"))
    c2, w2 = load_checkpoint(str(tmp_path / "meta"))
    assert (c1.hidden_size, c1.intermediate_size, c1.num_kv_heads) == (c2.hidden_size, c2.intermediate_size,
                                                                       c2.num_kv_heads)
    for a, b in zip(w1.layers, w2.layers):
        assert torch.equal(a.wqkv, b.wqkv) and torch.equal(a.w_gu, b.w_gu) and torch.equal(a.w_down, b.w_down)
    l1, l2 = _logits(c1, w1), _logits(c2, w2)
    assert torch.equal(l1, l2)


def test_tp_sharded_load_is_a_partition(tmp_path):
    cfg = get_config("tiny")
    t = _hf_tensors(cfg, seed=3)
    _write_hf(str(tmp_path / "hf"), cfg, t)
    _, full = load_checkpoint(str(tmp_path / "hf"))
    shards = [load_checkpoint(str(tmp_path / "hf"), TPContext(rank=r, world=2))[1] for r in range(2)]
    D = cfg.head_dim
    for li in range(cfg.num_layers):
        f = full.layers[li]
        hq, hkv = cfg.num_heads // 2, cfg.num_kv_heads // 2
        q = torch.cat([s.layers[li].wqkv[: hq * D] for s in shards])
        assert torch.equal(q, f.wqkv[: cfg.num_heads * D])
        down = torch.cat([s.layers[li].w_down for s in shards], dim=1)
        assert torch.equal(down, f.w_down)
    emb = torch.cat([s.embed for s in shards])
    assert torch.equal(emb, full.embed) and shards[1].vocab_start == cfg.vocab_size // 2


def test_folded_norms_match_unfolded(tmp_path):
    """RMSNorm weights folded into QKV / gate_up / LM head (the decode GEMV's fused-norm layout) give the same logits
    as the unfolded model, to bf16 rounding of W diag(w); the folded model stores its norms as ones."""
    cfg = get_config("tiny")
    t = _hf_tensors(cfg, seed=5)
    t["model.norm.weight"] = (1 + torch.rand(cfg.hidden_size) * 0.2).to(torch.bfloat16)
    _write_hf(str(tmp_path / "hf"), cfg, t)
    c1, wf = load_checkpoint(str(tmp_path / "hf"))
    c2, wu = load_checkpoint(str(tmp_path / "hf"), fold_norms=False)
    assert wf.norms_folded and not wu.norms_folded
    assert bool((wf.layers[0].attn_norm == 1).all()) and bool((wf.norm == 1).all())
    assert not bool((wu.layers[0].attn_norm == 1).all())
    lf, lu = _logits(c1, wf), _logits(c2, wu)
    assert (lf - lu).abs().max() <= 0.02 * lu.abs().max() + 1e-3
    assert (lf.argmax(-1) == lu.argmax(-1)).float().mean() >= 0.9
