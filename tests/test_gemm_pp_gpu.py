"""Numerics of the batched projection GEMM family (csrc/kernels/gemm_pp.hip) against an fp32 PyTorch reference.

Every tile config, split-K, and all three epilogues (plain, SwiGLU, residual + RMSNorm partials) plus the folded-norm
prologue, at ragged M (partial last tiles) with asymmetric random operands.  Run on an MI355X: ``pytest -m gpu``.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from chronos import ops

    ops.load()
    import chronos.native as n

    assert "_C" in n._loaded


def _rand(shape, g, scale=1.0, shift=0.0):
    return ((torch.rand(shape, device=DEV, generator=g) * 2 - 1) * scale + shift).to(torch.bfloat16)


def _pp(x, w, mode, cfg, splitk=1, resid=None, part=None, eps=1e-5):
    return torch.ops.chronos.gemm_pp(x, w, mode, cfg, splitk, resid, part, eps, False)


def _check(y, ref, tol=2e-2):
    err = (y.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err:.4g} vs max |ref| {scale:.4g}"


LG = [12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 72, 73, 74, 75, 78,
      79, 80]
# gemm_lg.hip configs (12-19 / 29-31 ring schedule, 20-28 slab schedule, 32-39 mid-M weight streaming); 76-77 (192 W
# rows: plain epilogue only at these toy N, whose SwiGLU / residual widths are not multiples of 192)
LG192 = [76, 77]
CFGS = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11] + LG + LG192


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("m", [3, 130, 257])
def test_plain(cfg, m):
    g = torch.Generator(device=DEV).manual_seed(7 * m + cfg)
    n, k = 512, 640
    x = _rand((m, k), g, 1.0, 0.1)
    w = _rand((n, k), g, 0.5)
    y, _ = _pp(x, w, 0, cfg)
    _check(y, x.float() @ w.float().t())


@pytest.mark.parametrize("cfg", [0, 3, 5, 8, 11] + LG + LG192)
def test_n_tail(cfg):
    """N not a multiple of the tile (the 70B TP=8 LM-head shard is N = 16032): the last W tile is partial."""
    g = torch.Generator(device=DEV).manual_seed(21 + cfg)
    m, n, k = 77, 16032 // 8, 256
    x = _rand((m, k), g)
    w = _rand((n, k), g, 0.5)
    y, _ = _pp(x, w, 0, cfg, 2)
    _check(y, x.float() @ w.float().t())


@pytest.mark.parametrize("cfg,splitk", [(0, 2), (1, 4), (3, 2), (2, 5), (4, 2), (5, 4), (7, 2), (8, 2), (9, 4), (10, 2), (11, 5),
                                        (12, 2), (13, 4), (14, 5), (15, 2), (16, 2), (17, 4), (18, 5), (19, 2), (20, 2), (21, 4), (22, 5), (23, 2), (24, 2), (25, 4), (26, 2), (27, 4), (28, 5), (29, 2), (30, 4), (31, 5), (32, 4), (33, 5), (34, 2), (35, 4), (36, 4), (37, 2), (38, 5), (39, 2), (72, 4), (73, 2), (74, 5), (75, 4), (76, 2), (77, 4)])
def test_splitk(cfg, splitk):
    g = torch.Generator(device=DEV).manual_seed(11 + cfg)
    m, n, k = 300, 512, 64 * 20
    x = _rand((m, k), g)
    w = _rand((n, k), g, 0.5, 0.05)
    ref = x.float() @ w.float().t()
    for _ in range(3):  # tickets must be left at zero by every call
        y, _ = _pp(x, w, 0, cfg, splitk)
        _check(y, ref)


@pytest.mark.parametrize("cfg", [0, 1, 3, 4, 5, 8, 9, 11] + LG)
def test_swiglu_normp(cfg):
    g = torch.Generator(device=DEV).manual_seed(3 + cfg)
    m, f, k = 200, 256, 512
    s = _rand((m, k), g, 2.0, 0.3)
    w = _rand((2 * f, k), g, 0.3)
    # partials of a producer: any split of sum(s^2) over columns works
    sf = s.float()
    part = torch.stack([(sf[:, i::8] ** 2).sum(1) for i in range(8)], 1).contiguous()
    inv = torch.rsqrt((sf * sf).sum(1, keepdim=True) / k + 1e-5)
    hv = (sf * inv) @ w.float().t()
    ref = torch.nn.functional.silu(hv[:, :f]) * hv[:, f:]
    y, _ = _pp(s, w, 1, cfg, 1, None, part)
    _check(y, ref, 3e-2)
    # plain + norm prologue
    y2, _ = _pp(s, w, 0, cfg, 1, None, part)
    _check(y2, hv)


@pytest.mark.parametrize("cfg,splitk", [(0, 1), (1, 2), (3, 1), (4, 1), (5, 2), (8, 1), (9, 2), (10, 1),
                                        (12, 1), (12, 2), (13, 1), (14, 2), (15, 1), (16, 1), (17, 2), (18, 1), (19, 2), (20, 1), (20, 2), (21, 1), (22, 2), (23, 1), (24, 1), (24, 2), (25, 1), (26, 1), (26, 2), (27, 1), (28, 2), (29, 1), (30, 2), (31, 1), (32, 1), (32, 4), (33, 2), (34, 1), (35, 2), (36, 4), (37, 1), (38, 2), (39, 1), (72, 2), (73, 1), (75, 2)])
def test_resid_partials(cfg, splitk):
    g = torch.Generator(device=DEV).manual_seed(5 + cfg)
    m, n, k = 259, 512, 768
    x = _rand((m, k), g)
    w = _rand((n, k), g, 0.2)
    r = _rand((m, n), g, 4.0)
    s, part = _pp(x, w, 2, cfg, splitk, r)
    ref = (x.float() @ w.float().t()).to(torch.bfloat16).float() + r.float()
    _check(s, ref)
    ss = (s.float() ** 2).sum(1)
    assert torch.allclose(part.sum(1), ss, rtol=1e-4, atol=1e-3)


def test_decode_shapes_vs_library():
    """One 8B decode-bucket shape per projection at M = 1024 against hipBLASLt, tight tolerance."""
    g = torch.Generator(device=DEV).manual_seed(1)
    for n, k, cfg, sk in [(6144, 4096, 1, 1), (4096, 14336, 1, 2), (4096, 4096, 3, 1), (6144, 4096, 12, 1),
                          (4096, 14336, 12, 4), (4096, 4096, 13, 2), (28672, 4096, 14, 1), (4096, 4096, 15, 1)]:
        x = _rand((1024, k), g)
        w = _rand((n, k), g, 0.05)
        y, _ = _pp(x, w, 0, cfg, sk)
        lib = x @ w.t()
        err = (y.float() - lib.float()).abs().max().item()
        assert err <= 2e-2 * lib.float().abs().max().item()
