"""GPU parity of the KD delta-stepping kernel (sssp_delta.hpp) against the CPU oracle.

KD's correctness argument has three knobs that the default configs never stress:
the bucket width D (D = 1 is Dial's algorithm, every arc heavy; D above every latency
is one bucket, every arc light, so every parent comes from the phase-B pull fix-up),
the LDS queue capacity (overflowing vertices must stay pending), and directedness
(no fused parents).  Each case is bit-exact against the oracle's engine tie rule.
"""
import numpy as np
import pytest

from shadow_amd.graph import Graph, config, internet_like

pytestmark = pytest.mark.gpu


def _chain(n, seed):
    """A long path plus a few chords: tree depths far beyond the phase-C path walk's
    register window (KD_MAXD arcs), so the level sweep must take over."""
    rng = np.random.default_rng(seed)
    e = [(i, i + 1) for i in range(n - 1)]
    have = set(e) | {(b, a) for a, b in e}
    while len(e) < n - 1 + n // 20:  # simple graph: no parallel edges
        a, b = (int(x) for x in rng.integers(0, n, 2))
        if a != b and (a, b) not in have:
            have |= {(a, b), (b, a)}
            e.append((a, b))
    e = np.array(e, np.int32)
    k = len(e)
    loops = np.arange(n, dtype=np.int32)
    lat = np.concatenate([rng.integers(1, 20, size=k), rng.integers(1, 5, size=n)]).astype(np.float64)
    loss = np.concatenate([np.where(rng.random(k) < 0.3, 0.0, rng.integers(1, 50, size=k) * 1e-4), np.zeros(n)])
    return Graph(n=n, src=np.concatenate([e[:, 0], loops]), dst=np.concatenate([e[:, 1], loops]),
                 latency=lat, packetloss=loss, vertex_packetloss=np.zeros(n), name="chain")


def _graph(name):
    from tests.golden import make_golden as mg
    if name == "chain":
        return _chain(600, 37)
    if name == "ba400":
        return internet_like(400, 4, seed=31, name="ba400")
    if name == "ties":
        return mg._ties(300, 33)
    if name == "dir":
        return mg._directed(200, 35)
    if name == "c2":
        return config("c2")
    raise KeyError(name)


@pytest.fixture
def kd(monkeypatch):
    """Forced KD with a small grid: each workgroup runs many sources back to back, so any
    LDS state a phase fails to restore for the next source shows up as a mismatch."""
    monkeypatch.setenv("SHD_ROUTE_KERNEL", "kd")
    monkeypatch.setenv("SHD_ROUTE_KDGRID", "7")
    return monkeypatch


@pytest.mark.parametrize("walk", [None, "0"])
@pytest.mark.parametrize("name", ["ba400", "ties", "dir", "c2", "chain"])
@pytest.mark.parametrize("delta,qcap", [(None, None), (1, None), (7, 64), (100000, None), (None, 64)])
def test_kd_rows_bitexact(oracle_mod, kd, name, delta, qcap, walk):
    """walk None: phase C by LDS path walks (level sweep only for deep rows) over packed
    out-arc records (v | w << 16 | ridx << 24); "0": level sweeps only, unpacked records
    (the writer wave gathers each winner's parent and reliability index)."""
    from shadow_amd import route
    if walk is None:
        kd.delenv("SHD_ROUTE_KDWALK", raising=False)
        kd.delenv("SHD_ROUTE_KDPACK", raising=False)
    else:
        kd.setenv("SHD_ROUTE_KDWALK", walk)
        kd.setenv("SHD_ROUTE_KDPACK", "0")
    if delta is None:
        kd.delenv("SHD_ROUTE_DELTA", raising=False)
    else:
        kd.setenv("SHD_ROUTE_DELTA", str(delta))
    if qcap is None:
        kd.delenv("SHD_ROUTE_QCAP", raising=False)
    else:
        kd.setenv("SHD_ROUTE_QCAP", str(qcap))
    g = _graph(name)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 4
    og = oracle_mod.OracleGraph(g)
    T = g.targets()
    S = T[:: max(1, len(T) // 96)]
    lat, rel, mn = eng.rows(S, T, dispatch=False)
    olat, orel, _, _ = og.source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_kd_sources_subset(oracle_mod, kd, cfg):
    """C3/C4 (512- and 1024-thread workgroups): attached subset (|A| < n) as targets,
    sources in arbitrary order."""
    from shadow_amd import route
    g = config(cfg)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 4
    og = oracle_mod.OracleGraph(g)
    T = g.targets()
    rng = np.random.default_rng(5)
    S = rng.choice(T, 40, replace=False).astype(np.int32)
    lat, rel, mn = eng.rows(S, T, dispatch=False)
    olat, orel, _, _ = og.source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)


@pytest.mark.parametrize("nt", [1000, 70000])
def test_kd_unsorted_duplicate_targets(oracle_mod, kd, nt):
    """A caller's target list that is unsorted and repeats vertices: on the
    chain graph most chains outlive the capped first walk and go through the second pass's
    list.  nt = 1000 (<= 2n) lists them by 32-bit position; nt = 70000 (> 2n, and past
    the 16 bits the sorted list's entries spend on a position) walks uncapped in one pass."""
    from shadow_amd import route
    g = _chain(600, 41)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 4
    og = oracle_mod.OracleGraph(g)
    rng = np.random.default_rng(nt)
    T = rng.integers(0, g.n, size=nt).astype(np.int32)
    S = np.array([0, 299, 599, 17], np.int32)
    lat, rel, mn = eng.rows(S, T, dispatch=False)
    allv = np.arange(g.n, dtype=np.int32)
    olat, orel, _, _ = og.source_rows(S, allv, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat[:, T])
    assert np.array_equal(rel, orel[:, T])
    assert np.array_equal(mn, olat[:, T].min(axis=1))
