"""Numerics of the skinny-M projection GEMM (csrc/kernels/gemm_skinny.hip) against an fp32 PyTorch reference.

Every config at ragged M up to its 16 MT bound, split-K (tickets reset, bitwise-reproducible slab order), and all
epilogues: plain, SwiGLU, residual add + RMSNorm partials, and the folded-norm (NORMP) prologue on plain / SwiGLU.
Run on an MI355X: ``pytest -m gpu``.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
# cfg -> (RT, MT, NW): csrc/kernels/gemm_skinny.hip SK_CONFIGS
CFGS = {0: (1, 1, 16), 1: (2, 1, 8), 2: (4, 1, 4), 3: (2, 2, 8), 4: (4, 2, 4), 5: (2, 4, 4), 6: (4, 4, 4),
        7: (2, 8, 4), 8: (1, 2, 16), 9: (1, 4, 16), 10: (2, 4, 8), 11: (1, 1, 8)}


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from chronos import ops

    ops.load()
    import chronos.native as n

    assert "_C" in n._loaded


def _rand(shape, g, scale=1.0, shift=0.0):
    return ((torch.rand(shape, device=DEV, generator=g) * 2 - 1) * scale + shift).to(torch.bfloat16)


def _sk(x, w, mode, cfg, splitk=1, resid=None, part=None, eps=1e-5):
    return torch.ops.chronos.gemm_skinny(x, w, mode, cfg, splitk, resid, part, eps)


def _check(y, ref, tol=2e-2):
    err = (y.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err:.4g} vs max |ref| {scale:.4g}"


@pytest.mark.parametrize("cfg", sorted(CFGS))
@pytest.mark.parametrize("splitk", [1, 2, 3])
def test_plain(cfg, splitk):
    rt, mt, nw = CFGS[cfg]
    g = torch.Generator(device=DEV).manual_seed(7 * cfg + splitk)
    n, k = 64 * 12, 64 * nw * splitk * 3
    for m in sorted({1, 3, 16 * mt - 5, 16 * mt}):
        x = _rand((m, k), g, 1.0, 0.1)
        w = _rand((n, k), g, 0.5)
        y, _ = _sk(x, w, 0, cfg, splitk)
        _check(y, x.float() @ w.float().t())


@pytest.mark.parametrize("cfg", sorted(CFGS))
def test_splitk_deterministic(cfg):
    """Split-K sums the slabs in slice order: repeated calls are bitwise equal (a replayed graph == the eager step),
    and the tickets are left at zero by every call."""
    rt, mt, nw = CFGS[cfg]
    g = torch.Generator(device=DEV).manual_seed(40 + cfg)
    m, n, k = 16 * mt - 1, 512, 64 * nw * 8
    x = _rand((m, k), g)
    w = _rand((n, k), g, 0.5, 0.05)
    first, _ = _sk(x, w, 0, cfg, 8)
    _check(first, x.float() @ w.float().t())
    for _ in range(4):
        y, _ = _sk(x, w, 0, cfg, 8)
        assert torch.equal(y, first)
    one, _ = _sk(x, w, 0, cfg, 1)
    _check(one, first.float())


@pytest.mark.parametrize("cfg", [c for c in sorted(CFGS) if CFGS[c][0] % 2 == 0])
@pytest.mark.parametrize("splitk", [1, 2])
def test_swiglu_normp(cfg, splitk):
    rt, mt, nw = CFGS[cfg]
    g = torch.Generator(device=DEV).manual_seed(3 + cfg)
    m, f, k = 16 * mt - 3, 256, 64 * nw * 2
    s = _rand((m, k), g, 2.0, 0.3)
    w = _rand((2 * f, k), g, 0.3)
    sf = s.float()
    part = torch.stack([(sf[:, i::8] ** 2).sum(1) for i in range(8)], 1).contiguous()
    inv = torch.rsqrt((sf * sf).sum(1, keepdim=True) / k + 1e-5)
    hv = (sf * inv) @ w.float().t()
    ref = torch.nn.functional.silu(hv[:, :f]) * hv[:, f:]
    y, _ = _sk(s, w, 1, cfg, splitk, None, part)
    _check(y, ref, 3e-2)
    y_plain_sw, _ = _sk(s, w, 1, cfg, splitk)  # no norm prologue
    hp = sf @ w.float().t()
    _check(y_plain_sw, torch.nn.functional.silu(hp[:, :f]) * hp[:, f:], 3e-2)
    y2, _ = _sk(s, w, 0, cfg, splitk, None, part)
    _check(y2, hv)


@pytest.mark.parametrize("cfg", sorted(CFGS))
def test_plain_normp_every_config(cfg):
    """Folded-norm prologue on every config (odd RT included): with many waves and a long K the first waves to finish
    write the norm scales while others still stream x through their LDS tiles (the XL configs alias the two)."""
    rt, mt, nw = CFGS[cfg]
    g = torch.Generator(device=DEV).manual_seed(90 + cfg)
    m, n, k = 16 * mt - 5, 16 * rt * 24, 64 * nw * 6
    s = _rand((m, k), g, 2.0, 0.3)
    w = _rand((n, k), g, 0.3)
    sf = s.float()
    part = torch.stack([(sf[:, i::8] ** 2).sum(1) for i in range(8)], 1).contiguous()
    inv = torch.rsqrt((sf * sf).sum(1, keepdim=True) / k + 1e-5)
    y, _ = _sk(s, w, 0, cfg, 1, None, part)
    _check(y, (sf * inv) @ w.float().t())


@pytest.mark.parametrize("cfg", sorted(CFGS))
@pytest.mark.parametrize("splitk", [1, 4])
def test_resid_partials(cfg, splitk):
    rt, mt, nw = CFGS[cfg]
    g = torch.Generator(device=DEV).manual_seed(5 + cfg)
    m, n, k = 16 * mt - 2, 512, 64 * nw * 4
    x = _rand((m, k), g)
    w = _rand((n, k), g, 0.2)
    r = _rand((m, n), g, 4.0)
    s, part = _sk(x, w, 2, cfg, splitk, r)
    ref = (x.float() @ w.float().t()).to(torch.bfloat16).float() + r.float()
    _check(s, ref)
    assert part.shape == (m, n // (16 * rt))
    ss = (s.float() ** 2).sum(1)
    assert torch.allclose(part.sum(1), ss, rtol=1e-4, atol=1e-3)


def test_decode_shapes_vs_library():
    """Llama-3-8B projection shapes at jump-forward / tail-bucket M against hipBLASLt, tight tolerance."""
    g = torch.Generator(device=DEV).manual_seed(1)
    for m, n, k, cfg, sk in [(4, 6144, 4096, 1, 1), (5, 4096, 14336, 2, 2), (32, 4096, 4096, 4, 4),
                             (64, 28672, 4096, 6, 1), (16, 128256, 4096, 2, 1), (128, 4096, 14336, 7, 2),
                             (3, 4096, 14336, 0, 1), (30, 6144, 4096, 8, 1), (60, 4096, 4096, 9, 1),
                             (3, 8192, 3584, 11, 1)]:
        x = _rand((m, k), g)
        w = _rand((n, k), g, 0.05)
        y, _ = _sk(x, w, 0, cfg, sk)
        lib = x @ w.t()
        err = (y.float() - lib.float()).abs().max().item()
        assert err <= 2e-2 * lib.float().abs().max().item()


def test_rejects_bad_shapes():
    g = torch.Generator(device=DEV).manual_seed(2)
    x = _rand((20, 512), g)
    w = _rand((256, 512), g)
    with pytest.raises(RuntimeError):
        _sk(x, w, 0, 0, 1)  # M = 20 > 16 MT for cfg 0
    with pytest.raises(RuntimeError):
        _sk(x[:8], w, 0, 0, 1)  # K % (64 * 16)
    with pytest.raises(RuntimeError):
        _sk(x[:8], w, 1, 0, 1)  # swiglu needs RT even
