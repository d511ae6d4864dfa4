"""The HB configs of gemm_lg.hip (81-90: one wave per SIMD, 128 x 128 outputs per wave, the three-barrier slab loop
of profiles/r6_gemm_isa_diff.md; 88-90 with the LDS-staged epilogue and split-K) against fp32, in every epilogue mode.

Shapes cover what the production plan never shows at once: M and N that are not tile multiples (partial x tiles,
partial W tiles in the plain epilogue), K of one slab, an odd number of slabs (the loop is unrolled by two), the
folded-RMSNorm prologue, the residual epilogue's RMSNorm partials, and split-K (slab hand-off + ticket, the tickets
left at zero for the next call).
"""
import pytest
import torch

DEV = "cuda"
HB = [81, 82, 83, 84, 85, 86, 87, 88, 89, 90, 91, 92, 93, 94]
STAGED = [88, 89, 90, 91, 92, 93, 94]


def _rand(shape, g, scale=1.0, shift=0.0):
    return ((torch.rand(shape, device=DEV, generator=g) * 2 - 1) * scale + shift).to(torch.bfloat16)


def _check(y, ref, tol):
    y = y.float()
    err = (y - ref).abs()
    scale = ref.abs().max().item() + 1e-6
    bad = err > tol * scale + (2.0 ** -7) * ref.abs()
    assert not bool(bad.any()), f"{int(bad.sum())} elements off; max err {err.max().item():.4g} vs max |ref| {scale:.4g}"


def _parts(s):
    sf = s.float()
    return torch.stack([(sf[:, i::16] ** 2).sum(1) for i in range(16)], 1).contiguous()


def _run(cfg, m, n, k, mode, sk=1, normp=False, seed=0):
    from chronos import ops
    from chronos.ops import gemm as G

    ops.load()
    g = torch.Generator(device=DEV).manual_seed(seed + 31 * cfg + m + n + k + mode)
    w = _rand((n, k), g, 0.5 / (k ** 0.5) * 8)
    if mode == G.PP_RESID:
        x = _rand((m, k), g, 1.0, 0.05)
        r = _rand((m, n), g, 2.0)
        s, part = G.pp_gemm(x, w, mode, (cfg, sk), r)
        ref = (x.float() @ w.float().t()).to(torch.bfloat16).float() + r.float()
        _check(s, ref, 1e-2)
        torch.testing.assert_close(part.sum(1), (s.float() ** 2).sum(1), rtol=1e-4, atol=1e-3)
        assert part.shape == (m, n // 128)
        return s
    s = _rand((m, k), g, 2.0, 0.2)
    sf = s.float()
    if normp:
        inv = torch.rsqrt((sf * sf).sum(1, keepdim=True) / k + 1e-5)
        h = (sf * inv) @ w.float().t()
        y, _ = G.pp_gemm(s, w, mode, (cfg, sk), None, _parts(s), 1e-5)
    else:
        h = sf @ w.float().t()
        y, _ = G.pp_gemm(s, w, mode, (cfg, sk))
    if mode == G.PP_SWIGLU:
        f = n // 2
        ref = torch.nn.functional.silu(h[:, :f].to(torch.bfloat16).float()) * h[:, f:].to(torch.bfloat16).float()
        _check(y, ref, 2e-2)
    else:
        _check(y, h, 1e-2)
    return y


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", HB)
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_hb_modes(cfg, mode):
    # M = 600: three x tiles, the last partial; K = 704: 11 slabs (odd: the two-slab loop's tail half)
    _run(cfg, 600, 512, 704, mode)
    if mode != 2:
        _run(cfg, 600, 512, 704, mode, normp=True)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [81, 86, 88, 89, 91, 92, 93, 94])
def test_hb_partial_w_tile_and_one_slab(cfg):
    _run(cfg, 300, 520, 64, 0)        # N = 520: two whole W tiles + 8 rows; K = 64: a single slab
    _run(cfg, 257, 1032, 128, 0)      # N % 8 == 0 but not % 16: the staged epilogue's 8-column tail store
    _run(cfg, 1, 256, 256, 0)         # one row


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", STAGED)
@pytest.mark.parametrize("mode,normp", [(0, False), (0, True), (1, True), (2, False)])
@pytest.mark.parametrize("sk", [2, 4])
def test_hb_splitk(cfg, mode, normp, sk):
    y1 = _run(cfg, 512, 1024, 1024, mode, sk=sk, normp=normp)
    y2 = _run(cfg, 512, 1024, 1024, mode, sk=sk, normp=normp)  # same seed: tickets back at zero, same bits
    assert torch.equal(y1, y2)
    y0 = _run(cfg, 512, 1024, 1024, mode, sk=1, normp=normp)
    # the slices are summed in slice order in fp32: close to the unsplit tile, not bit-equal
    torch.testing.assert_close(y1.float(), y0.float(), rtol=2e-2, atol=2e-2)


def test_hb_configs_reject_splitk_without_the_staged_epilogue():
    """CPU: the router never pairs an HB config without split-K support with split-K > 1."""
    from chronos.ops import gemm as G

    for c in HB:
        assert G._pp_valid(c, 4096, 4096, 0, 1, 1024)
        assert G._pp_valid(c, 4096, 4096, 0, 2, 1024) == (c in STAGED)
