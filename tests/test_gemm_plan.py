"""Routing of the projection GEMMs (ops/gemm.py): the measured plan file decides kernel / config / split-K by M range
(skinny kernel = cfg >= SK_BASE), invalid rows fall back to the library, and the cost models only return configs the
kernels accept.  CPU-only: the routing is pure Python."""
import pytest

from chronos.ops import gemm as G


@pytest.fixture
def plan(monkeypatch):
    table = {(4096, 4096, 2): [[5, 101, 2], [64, 106, 8], [256, 1, 2], [1024, -1, 1], [4096, 0, 1]],
             (6144, 4096, 0): [[8, 100, 3]]}  # split 3 does not divide 4096 / 1024: invalid -> library
    monkeypatch.setattr(G, "_plan_table", table)
    monkeypatch.setattr(G, "_plan_cache", {})
    monkeypatch.setattr(G, "PP_MODE", "auto")
    return table


def test_plan_rows_by_m(plan):
    assert G.pp_plan(1, 4096, 4096, G.PP_RESID) is None  # M = 1: the GEMV, never the plan
    assert G.pp_plan(2, 4096, 4096, G.PP_RESID) == (101, 2)  # M = 2: the first row
    assert G.pp_plan(3, 4096, 4096, G.PP_RESID) == (101, 2)
    assert G.pp_plan(5, 4096, 4096, G.PP_RESID) == (101, 2)
    assert G.pp_plan(6, 4096, 4096, G.PP_RESID) == (106, 8)
    assert G.pp_plan(64, 4096, 4096, G.PP_RESID) == (106, 8)
    assert G.pp_plan(65, 4096, 4096, G.PP_RESID) == (1, 2)
    assert G.pp_plan(1000, 4096, 4096, G.PP_RESID) is None
    assert G.pp_plan(4096, 4096, 4096, G.PP_RESID) == (0, 1)
    assert G.pp_plan(9000, 4096, 4096, G.PP_RESID) == (0, 1)  # above the last row: the last row
    assert G.pp_plan(4, 6144, 4096, G.PP_PLAIN) is None
    assert G.pp_plan(4, 1024, 4096, G.PP_PLAIN) is None  # unmeasured shape: library


def test_skinny_row_beyond_its_m_bound_is_rejected(monkeypatch):
    monkeypatch.setattr(G, "_plan_table", {(4096, 4096, 0): [[64, 100, 1]]})  # cfg 0: M <= 16 only
    monkeypatch.setattr(G, "_plan_cache", {})
    monkeypatch.setattr(G, "PP_MODE", "auto")
    assert G.pp_plan(16, 4096, 4096, 0) == (100, 1)
    assert G.pp_plan(17, 4096, 4096, 0) is None


@pytest.mark.parametrize("n,k,mode", [(6144, 4096, 0), (4096, 4096, 2), (28672, 4096, 1), (4096, 14336, 2),
                                      (128256, 4096, 0), (1280, 8192, 0), (7168, 8192, 1), (8192, 3584, 0),
                                      (16032, 8192, 0)])
@pytest.mark.parametrize("m", [3, 4, 5, 8, 16, 17, 32, 33, 48, 64])
def test_skinny_model_valid(m, n, k, mode):
    got = G._sk_model(m, n, k, mode)
    if got is None:
        return
    cfg, sk = got
    rt, mt, nw = G._SK[cfg - G.SK_BASE]
    assert m <= 16 * mt and k % (64 * nw * sk) == 0
    if mode == G.PP_SWIGLU:
        assert rt % 2 == 0 and (n // 2) % (8 * rt) == 0
    else:
        assert n % (16 * rt) == 0


def test_own_mode_uses_skinny_then_tiles(monkeypatch):
    monkeypatch.setattr(G, "_plan_cache", {})
    monkeypatch.setattr(G, "PP_MODE", "own")
    assert G.pp_plan(5, 4096, 4096, G.PP_PLAIN)[0] >= G.SK_BASE
    assert G.pp_plan(512, 4096, 4096, G.PP_PLAIN)[0] < G.SK_BASE


def test_fp8_qplan(monkeypatch):
    monkeypatch.setattr(G, "_plan_table", {})
    monkeypatch.setattr(G, "_qplan_table", {(28672, 4096, 1): [[4, 1], [128, 1], [1024, 0], [16384, 1]]})
    assert G.qplan_own(3, 28672, 4096, True) is True
    assert G.qplan_own(512, 28672, 4096, True) is False
    assert G.qplan_own(20000, 28672, 4096, True) is True
    assert G.qplan_own(5, 28672, 4096, False) is None
    from chronos import ops

    monkeypatch.setattr(ops, "_QGEMM", "auto")
    assert ops._qown(512, 28672, 4096, True) is False
    assert ops._qown(3, 4096, 4096, False) is True  # unmeasured: the round-1 rule (GEMV at M <= 4)
