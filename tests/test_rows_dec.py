"""Decode-form attention for a few tokens over a long context (models/llama.py StepBatch.rows_dec: every token of a
jump-forward chunk attends as its own decode row, context pos + 1) against the prefill-tile path of the same chunk:
same logits, on the CPU references and on the GPU kernels (split-K decode vs the paged prefill tiles)."""
import pytest
import torch


def _run(device, min_ctx, prompt_len=2100, chunk=(5, 6, 7)):
    from chronos.models import llama
    from chronos.models.llama import KVCache, build_model, make_prefill_batch

    llama.ROWS_DEC_MIN_CTX = min_ctx
    try:
        m = build_model("tiny", device, seed=2)
        kv = KVCache(m.cfg, m.tp, 160, 16, device)
        bt = list(range(1, 1 + (prompt_len + len(chunk) + 15) // 16))
        prompt = [(i * 37) % 1000 + 3 for i in range(prompt_len)]
        m.forward(make_prefill_batch([prompt], [0], [bt], m.cfg, m.tp, device, max_blocks=160, nqt=8), kv)
        sb = make_prefill_batch([list(chunk)], [prompt_len], [bt], m.cfg, m.tp, device, max_blocks=160, nqt=2)
        assert (sb.rows_dec is not None) == (min_ctx <= prompt_len)
        return m.forward(sb, kv).float()
    finally:
        llama.ROWS_DEC_MIN_CTX = 2048


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_rows_dec_matches_prefill_tiles(device):
    if device == "cuda":
        from chronos import ops

        ops.load()
    a = _run(device, 1 << 30)  # prefill tiles
    b = _run(device, 2048)     # decode rows
    err = (a - b).abs().max().item()
    assert err <= 2e-2 * a.abs().max().item(), err
    assert torch.equal(a.argmax(-1), b.argmax(-1))
