"""GPU parity of the batched KB kernel (sssp_batch.hpp), fused and unfused.

KB with fused path attributes (sssp_batch_kernel<true>) writes the rows itself: parent
records in LDS, each target's tree path walked and its reliability folded source-first.
Its knobs: walks deeper than KB_MAXD arcs (slow path), several 8-source batches per
workgroup (the arc region is re-staged after each batch's walk arrays), sources whose
batch is partly empty, vertex loss, and the directed in-CSR.  Every case is bit-exact
against the oracle's engine tie rule and against the unfused KB + K2 pair.
"""
import numpy as np
import pytest

from shadow_amd.graph import config, internet_like
from tests.test_kd_gpu import _chain

pytestmark = pytest.mark.gpu


def _graph(name):
    from tests.golden import make_golden as mg
    if name == "chain":
        return _chain(600, 41)
    if name == "ba400":
        return internet_like(400, 4, seed=43, name="ba400")
    if name == "ties":
        return mg._ties(300, 45)
    if name == "dir":
        return mg._directed(200, 47)
    if name == "c2":
        return config("c2")
    if name == "c2v":
        return config("c2", vloss=True)
    raise KeyError(name)


def _rows(route, g, src, tgt, monkeypatch, fuse, grid=None):
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    monkeypatch.setenv("SHD_ROUTE_KBFUSE", "1" if fuse else "0")
    if grid:
        monkeypatch.setenv("SHD_ROUTE_KBGRID", str(grid))
    else:
        monkeypatch.delenv("SHD_ROUTE_KBGRID", raising=False)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 2
    assert eng.info["reserved"] == (1 if fuse else 0)
    return eng.rows(src, tgt, dispatch=False)


@pytest.fixture(scope="module")
def route():
    from shadow_amd import route as r
    r.load_library()
    return r


@pytest.mark.parametrize("name", ["chain", "ba400", "ties", "dir", "c2"])
@pytest.mark.parametrize("grid", [None, 3])
def test_kb_fused_bitexact(route, oracle_mod, monkeypatch, name, grid):
    g = _graph(name)
    T = g.targets()
    S = T if g.n <= 600 else T[::7]
    lat, rel, mn = _rows(route, g, S, T, monkeypatch, True, grid)
    og = oracle_mod.OracleGraph(g)
    olat, orel, _, _ = og.source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat), name
    assert np.array_equal(rel, orel), name
    assert np.array_equal(mn, olat.min(axis=1)), name


def test_kb_fused_equals_unfused_c2(route, monkeypatch):
    g = config("c2")
    T = g.targets()
    a = _rows(route, g, T, T, monkeypatch, True)
    b = _rows(route, g, T, T, monkeypatch, False)
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint64), y.view(np.uint64))


def test_kb_fused_vertex_loss(route, oracle_mod, monkeypatch):
    g = _graph("c2v")
    T = g.targets()
    S = T[5::61]
    lat, rel, mn = _rows(route, g, S, T, monkeypatch, True)
    _, urel, _ = _rows(route, g, S, T, monkeypatch, False)
    og = oracle_mod.OracleGraph(g)
    olat, orel, _, _ = og.source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    # KBF's walks fold from (1.0 * f_s) * f_t, the reference's order: bit-exact; K2's level
    # pass multiplies f_t last: within 1e-12
    assert np.array_equal(rel, orel)
    np.testing.assert_allclose(urel, orel, rtol=1e-12, atol=0)


def test_kb_fused_ragged_batches_and_subset_targets(route, oracle_mod, monkeypatch):
    """13 sources (a partly empty last batch), a permuted target subset, repeated targets."""
    g = _graph("ba400")
    rng = np.random.default_rng(7)
    S = rng.choice(g.n, 13, replace=False).astype(np.int32)
    T = np.concatenate([rng.permutation(g.n)[:150], [S[0], S[0]]]).astype(np.int32)
    lat, rel, mn = _rows(route, g, S, T, monkeypatch, True, grid=1)
    og = oracle_mod.OracleGraph(g)
    olat, orel, _, _ = og.source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))
