"""LDS-staged split-K decode attention (csrc/kernels/attention.hip split_decode_kernel) against the
fp32 reference, bf16 and fp8-e4m3 KV, every ring depth, long and ragged contexts (splits with no keys, partial last
steps, contexts not a multiple of the 32-token step), the in-launch combine and the separate combine kernel."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from chronos import ops

    ops.load()
    yield
    torch.ops.chronos.set_knob("split_lds", 1)
    torch.ops.chronos.set_knob("split_lds_nb", -1)
    torch.ops.chronos.set_knob("attn_inkernel_combine", 1)
    torch.ops.chronos.set_knob("sd_inkernel_max_split", 4)


def _case(ctx, hq, hkv, fp8, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    bs = 16
    B = len(ctx)
    nbs = [(c + bs - 1) // bs for c in ctx]
    nb = sum(nbs) + 1
    perm = (torch.randperm(nb - 1, generator=torch.Generator().manual_seed(seed)) + 1).tolist()
    bt = torch.zeros(B, max(nbs), dtype=torch.int32)
    o = 0
    for b, n in enumerate(nbs):
        bt[b, :n] = torch.tensor(perm[o:o + n])
        o += n
    if fp8:
        from chronos.ops import reference as ref

        k = ref.to_fp8_bytes(torch.randn(nb, hkv, bs, 128, device=DEV, generator=g) * 1.5, 1.0 / 0.5)
        v = ref.to_fp8_bytes(torch.randn(nb, hkv, 128, bs, device=DEV, generator=g), 1.0 / 0.25)
    else:
        k = (torch.randn(nb, hkv, bs, 128, device=DEV, generator=g) * 0.7).to(torch.bfloat16)
        v = torch.randn(nb, hkv, 128, bs, device=DEV, generator=g).to(torch.bfloat16)
    q = (torch.randn(B, hq, 128, device=DEV, generator=g)).to(torch.bfloat16)
    qs = torch.arange(B + 1, dtype=torch.int32, device=DEV)
    return q, k, v, bt.to(DEV), qs, torch.tensor(ctx, dtype=torch.int32, device=DEV)


@pytest.mark.parametrize("fp8,nb", [(False, 1), (False, 2), (True, 2), (True, 3), (True, 4)])
@pytest.mark.parametrize("ctx,nsplit", [([33000], 32), ([8191, 100, 4097], 16), ([700, 33, 1, 480], 4),
                                        ([131072], 32)])
def test_split_lds_matches_reference(fp8, nb, ctx, nsplit):
    from chronos import ops
    from chronos.ops import reference as ref

    if ctx == [131072] and nb not in (2, 3):
        pytest.skip("the 128k case once per dtype")
    hq, hkv = 32, 8
    q, k, v, bt, qs, cl = _case(ctx, hq, hkv, fp8, seed=sum(ctx) + nb)
    ks, vs = (0.5, 0.25) if fp8 else (1.0, 1.0)
    torch.ops.chronos.set_knob("split_lds_nb", nb)
    outs = {}
    for lds in (1, 0):
        torch.ops.chronos.set_knob("split_lds", lds)
        for comb in (1, 0):
            torch.ops.chronos.set_knob("attn_inkernel_combine", comb)
            torch.ops.chronos.set_knob("sd_inkernel_max_split", 1024 if comb else 4)
            outs[(lds, comb)] = ops.paged_attention(q, k, v, bt, qs, cl, None, len(ctx), 1, nsplit, None, ks, vs).float()
    torch.ops.chronos.set_knob("split_lds", 1)
    torch.ops.chronos.set_knob("attn_inkernel_combine", 1)
    torch.ops.chronos.set_knob("sd_inkernel_max_split", 4)
    want = ref.paged_attention(q, k, v, bt, qs, cl, None, len(ctx), 1, nsplit, None, ks, vs).float()
    tol = 2e-2 * want.abs().max().item()
    for key, o in outs.items():
        assert (o - want).abs().max().item() <= tol, (key, (o - want).abs().max().item(), tol)
    # in-launch combine == separate combine kernel (same merge code)
    assert torch.equal(outs[(1, 1)], outs[(1, 0)])


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("qlens,ctx,nsplit", [([3], [33000], 32), ([4, 1, 2], [8191, 100, 4097], 16),
                                              ([2, 4], [700, 33], 4), ([4], [131072], 32), ([3, 3], [500, 37], 1)])
def test_split_decode_multi_token(fp8, qlens, ctx, nsplit):
    """Sequences of up to 4 query tokens (jump-forward chunks) in one pass over their K/V (max_q): against the fp32
    reference of the same causal chunk attention, with the in-launch and the separate combine."""
    from chronos import ops
    from chronos.ops import reference as ref

    hq, hkv = 32, 8
    _, k, v, bt, _, cl = _case(ctx, hq, hkv, fp8, seed=sum(ctx) + sum(qlens))
    T = sum(qlens)
    q = torch.randn(T, hq, 128, device=DEV, generator=torch.Generator(device=DEV).manual_seed(T)).to(torch.bfloat16)
    qs = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    ks, vs = (0.5, 0.25) if fp8 else (1.0, 1.0)
    B, mq = len(ctx), max(qlens)
    want = ref.paged_attention(q, k, v, bt, qs, cl, None, B, 1, nsplit, None, ks, vs, max_q=mq).float()
    outs = {}
    for comb in (1, 0):
        torch.ops.chronos.set_knob("attn_inkernel_combine", comb)
        torch.ops.chronos.set_knob("sd_inkernel_max_split", 1024 if comb else 4)
        outs[comb] = ops.paged_attention(q, k, v, bt, qs, cl, None, B, 1, nsplit, None, ks, vs, max_q=mq).float()
    torch.ops.chronos.set_knob("attn_inkernel_combine", 1)
    torch.ops.chronos.set_knob("sd_inkernel_max_split", 4)
    tol = 2e-2 * want.abs().max().item()
    for comb, o in outs.items():
        assert (o - want).abs().max().item() <= tol, (comb, (o - want).abs().max().item(), tol)
    assert torch.equal(outs[1], outs[0])
