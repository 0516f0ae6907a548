"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle.

Latency must be bit-exact everywhere.  Reliability is bit-exact against the oracle's
engine tie rule (ORC_TIE_MINKEY) when vertex factors are 1.0/absent, and matches
igraph's tie rule wherever the shortest path is unique.  With non-unit vertex loss the
walk kernels (KBF, KD) fold from (1.0 * f_s) * f_t as the reference does (topology.c:
1443-1462, then :1499): bit-exact; the level-sweep kernels (K32, f64, KF) multiply f_t
last: tolerance REL_TOL relative (north_star: 1e-12).
"""
import numpy as np
import pytest

from shadow_amd.graph import Graph, complete_graph, config, example_one_vertex, internet_like

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12


@pytest.fixture(scope="module")
def route():
    from shadow_amd import route as r
    r.load_library()
    return r


KERNEL_ID = {"f64": 0, "k32": 1, "kb": 2, "k16": 3, "kd": 4, "kf": 5}


@pytest.fixture(params=["auto", "kd", "k32", "f64", "kf"])
def kernel(request, monkeypatch):
    """Run a test on the auto-selected kernel and on each forced kernel."""
    if request.param == "auto":
        monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    else:
        monkeypatch.setenv("SHD_ROUTE_KERNEL", request.param)
    return request.param


def _check_rows(eng, og, oracle_mod, src, tgt, rel_exact=True):
    lat, rel, mn = eng.rows(src, tgt, dispatch=False)
    olat, orel, ouq, _ = og.source_rows(src, tgt, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    if rel_exact:
        assert np.array_equal(rel, orel)
    else:
        np.testing.assert_allclose(rel, orel, rtol=REL_TOL, atol=0)
    assert np.array_equal(mn, olat.min(axis=1))
    ilat, irel, iuq, _ = og.source_rows(src, tgt, oracle_mod.TIE_IGRAPH)
    assert np.array_equal(lat, ilat)
    np.testing.assert_allclose(rel[iuq], irel[iuq], rtol=REL_TOL, atol=0)
    return lat, rel


def test_c2_rows_bitexact(route, oracle_mod, kernel):
    g = config("c2")
    eng = route.RouteEngine(g)
    assert eng.info["lds_resident"] == 1
    assert eng.info["kernel"] == (2 if kernel == "auto" else KERNEL_ID[kernel])
    og = oracle_mod.OracleGraph(g)
    src = np.arange(0, g.n, 13, dtype=np.int32)
    _check_rows(eng, og, oracle_mod, src, g.targets())


def test_c2_vertex_loss_within_tol(route, oracle_mod, kernel):
    g = config("c2", vloss=True)
    eng = route.RouteEngine(g)
    og = oracle_mod.OracleGraph(g)
    src = np.arange(3, g.n, 97, dtype=np.int32)
    # walk kernels (auto = KBF, KD): bit-exact; level sweeps: within REL_TOL
    _check_rows(eng, og, oracle_mod, src, g.targets(), rel_exact=kernel in ("auto", "kd"))


def test_hbm_resident_path(route, oracle_mod, monkeypatch):
    monkeypatch.setenv("SHD_ROUTE_KERNEL", "f64")
    g = internet_like(8000, 3, seed=5, name="hbm")
    eng = route.RouteEngine(g)
    assert eng.info["lds_resident"] == 0
    og = oracle_mod.OracleGraph(g)
    src = np.array([0, 1, 7, 4000, 7999], np.int32)
    _check_rows(eng, og, oracle_mod, src, g.targets())


def test_example_kat(route):
    # resource/examples/shadow.config.xml:2-24: lat 50.0, rel 0.99, runahead 50 ms
    eng = route.RouteEngine(example_one_vertex(0.0, 0.01, 50.0))
    assert eng.info["is_complete"] == 1
    lat, rel, mn = eng.rows([0], [0])
    assert lat[0, 0] == 50.0 and rel[0, 0] == 1.0 - 0.01 and mn[0] == 50.0
    # src/test/tcp/tcp-blocking-lossy: no vertex packetloss key, edge loss 0.25
    eng = route.RouteEngine(example_one_vertex(None, 0.25, 50.0))
    lat, rel, _ = eng.rows([0], [0])
    assert lat[0, 0] == 50.0 and rel[0, 0] == 0.75


def test_complete_direct_dispatch(route, oracle_mod):
    g = complete_graph(64, seed=3)
    eng = route.RouteEngine(g)
    assert eng.info["is_complete"] == 1
    og = oracle_mod.OracleGraph(g)
    t = np.arange(g.n, dtype=np.int32)
    lat, rel, _ = eng.rows(t, t, dispatch=True)
    for s in range(0, g.n, 9):
        for j in range(g.n):
            L, R = og.direct(s, j)
            assert lat[s, j] == L and rel[s, j] == R


def test_self_paths(route, oracle_mod):
    g = internet_like(200, 2, seed=9)
    eng = route.RouteEngine(g)
    og = oracle_mod.OracleGraph(g)
    v = np.arange(g.n, dtype=np.int32)
    lat, rel = eng.self_paths(v)
    for k in range(g.n):
        L, R = og.self_path(k)
        assert lat[k] == L and rel[k] == R


# ---------------------------------------------------------------------------
# full-size parity through the committed golden fixtures (tests/golden/)
import hashlib  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float64).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def digests():
    return json.load(open(os.path.join(GOLD, "rows_digests.json")))


def test_c2_full_table_matches_golden(route, digests, kernel):
    g = config("c2")
    eng = route.RouteEngine(g)
    T = g.targets()
    lat, rel, mn = eng.rows(T, T)
    rows = {r["src"]: r for r in digests["c2"]["rows"]}
    assert len(rows) == len(T)
    for i, s in enumerate(T):
        r = rows[int(s)]
        assert _sha(lat[i]) == r["lat_sha"] and _sha(rel[i]) == r["rel_sha"], s
        assert mn[i] == r["row_min"]
    # undirected, integer weights: the table is symmetric in latency
    assert np.array_equal(lat, lat.T)


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_sampled_rows_match_golden(route, digests, cfg, kernel):
    g = config(cfg)
    eng = route.RouteEngine(g)
    T = g.targets()
    S = np.array([r["src"] for r in digests[cfg]["rows"]], np.int32)
    lat, rel, mn = eng.rows(S, T)
    for i, r in enumerate(digests[cfg]["rows"]):
        assert _sha(lat[i]) == r["lat_sha"] and _sha(rel[i]) == r["rel_sha"], (cfg, r["src"])
        assert mn[i] == r["row_min"]


def test_bundled_topology_engine(route):
    z = np.load(os.path.join(GOLD, "bundled_topology.npz"))
    exp = json.load(open(os.path.join(GOLD, "bundled_expected.json")))
    g = Graph(n=int(z["n"]), src=z["src"], dst=z["dst"], latency=z["latency"], packetloss=z["packetloss"],
              vertex_packetloss=z["vertex_packetloss"], directed=bool(z["directed"]))
    eng = route.RouteEngine(g)
    assert eng.info["is_complete"] == 1
    A = np.arange(g.n, dtype=np.int32)
    lat, rel, mn = eng.rows(A, A, dispatch=True)
    assert _sha(lat) == exp["lat_sha"] and _sha(rel) == exp["rel_sha"]
    assert mn.min() == exp["min_latency"] == 5.0


def test_small_golden_tables_engine(route, kernel):
    z = np.load(os.path.join(GOLD, "small_tables.npz"))
    for name in z["names"]:
        p = f"{name}__"
        vl = z[p + "vertex_packetloss"]
        g = Graph(n=int(z[p + "n"]), src=z[p + "src"], dst=z[p + "dst"], latency=z[p + "latency"],
                  packetloss=z[p + "packetloss"], vertex_packetloss=vl if len(vl) else None,
                  directed=bool(z[p + "directed"]), prefer_direct=bool(z[p + "prefer_direct"]))
        eng = route.RouteEngine(g)
        A = z[p + "attached"].astype(np.int32)
        lat, rel, _ = eng.rows(A, A, dispatch=True)
        # eager cache: lookup(i, j) = the Path stored from row min(i, j) (first writer wins)
        iu = np.triu_indices(len(A))
        E_lat = np.zeros_like(lat); E_rel = np.zeros_like(rel)
        E_lat[iu] = lat[iu]; E_rel[iu] = rel[iu]
        E_lat.T[iu] = lat[iu]; E_rel.T[iu] = rel[iu]
        assert np.array_equal(E_lat, z[p + "lat"]), name
        uq = z[p + "unique"]
        np.testing.assert_allclose(E_rel[uq], z[p + "rel"][uq], rtol=REL_TOL, atol=0, err_msg=name)
        if not len(vl) or np.all(vl == 0):
            assert np.array_equal(E_rel[uq], z[p + "rel"][uq]), name
        if not (g.prefer_direct or eng.info["is_complete"]):
            # raw SOURCE rows against the golden raw rows too
            assert np.array_equal(lat, z[p + "raw_lat"]), name


def test_kernel_selection(route):
    g = config("c2")
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 2 and 0 < eng.info["dist_bound"] < 65535
    g2 = internet_like(300, 2, seed=3)
    g2.latency = g2.latency + 0.25  # fractional -> KF (LDS-resident f64 delta-stepping)
    assert route.RouteEngine(g2).info["kernel"] == 5
    g3 = internet_like(20000, 2, seed=3)
    g3.latency = g3.latency + 0.25  # fractional, past KF's LDS -> KFH (vertex state in HBM)
    e3 = route.RouteEngine(g3)
    assert e3.info["kernel"] == 5 and e3.info["lds_resident"] == 0
    g4 = internet_like(70000, 2, seed=3)
    g4.latency = g4.latency + 0.25  # past KFH's u16 ring ids -> the generic f64 kernel
    assert route.RouteEngine(g4).info["kernel"] == 0
