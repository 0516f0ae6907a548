"""KF (fractional-latency delta-stepping, sssp_f64d.hpp) against the oracle and the generic
f64 kernel.  Latency bit-exact (any relaxation order reaches the same left fold);
reliability bit-exact against the oracle's engine tie rule (ORC_TIE_MINKEY) with unit or
absent vertex factors, within REL_TOL with vertex loss (f_t multiplied last)."""
import numpy as np
import pytest

from shadow_amd.graph import Graph, config, fractional, internet_like

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12


@pytest.fixture(scope="module")
def route():
    from shadow_amd import route as r
    r.load_library()
    return r


def _rows(route, g, src, tgt, kernel, monkeypatch):
    monkeypatch.setenv("SHD_ROUTE_KERNEL", kernel)
    eng = route.RouteEngine(g)
    return eng, eng.rows(src, tgt, dispatch=False)


@pytest.mark.parametrize("cfg,step", [("c2f", 7), ("c3f", 211)])
def test_kf_fractional_bitexact(route, oracle_mod, monkeypatch, cfg, step):
    g = config(cfg)
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5  # KF is the fractional path at this size
    src = np.arange(0, g.n, step, dtype=np.int32)
    tgt = g.targets()
    lat, rel, mn = eng.rows(src, tgt, dispatch=False)
    og = oracle_mod.OracleGraph(g)
    olat, orel, _, _ = og.source_rows(src, tgt, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))


@pytest.mark.parametrize("kfh", [0, 1])
def test_kf_packed_arcs(route, oracle_mod, monkeypatch, kfh):
    """C2f's latencies have two decimals: KFH reads each arc as one u32 (head | k << 16,
    latency k / 100.0, the double the decimal parses to); the LDS kernel keeps f64 arcs.  The
    same rows as the f64 arcs (SHD_ROUTE_KFPK=0) and the oracle."""
    g = config("c2f")
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    if kfh:
        monkeypatch.setenv("SHD_ROUTE_KFH", "1")
    src = np.arange(0, g.n, 3, dtype=np.int32)
    tgt = g.targets()
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5 and eng.info["reserved"] == (100 if kfh else 0) and eng.info["lds_resident"] == 1 - kfh
    lat, rel, mn = eng.rows(src, tgt, dispatch=False)
    monkeypatch.setenv("SHD_ROUTE_KFPK", "0")
    e0 = route.RouteEngine(g)
    assert e0.info["reserved"] == 0
    l0, r0, m0 = e0.rows(src, tgt, dispatch=False)
    assert np.array_equal(lat, l0) and np.array_equal(rel, r0) and np.array_equal(mn, m0)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(src, tgt, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat) and np.array_equal(rel, orel)


def test_kf_many_sources_per_workgroup(route, monkeypatch):
    # every source of C2f in one launch (about two per workgroup) against KF one source per
    # workgroup: per-source state is reset between sources
    g = config("c2f")
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    eng = route.RouteEngine(g)
    tgt = g.targets()
    lat, rel, mn = eng.rows(tgt, tgt, dispatch=False)
    for part in (tgt[:200], tgt[1000:1100]):
        l2, r2, m2 = eng.rows(part, tgt, dispatch=False)
        assert np.array_equal(l2, lat[part]) and np.array_equal(r2, rel[part]) and np.array_equal(m2, mn[part])


def test_kf_repeated_launches_identical(route, monkeypatch):
    # every C2f source, three launches, against the generic f64 kernel's rows: the
    # workgroups' asynchronous rounds must give the same table every time
    g = config("c2f")
    tgt = g.targets()
    _, (l0, r0, m0) = _rows(route, g, tgt, tgt, "f64", monkeypatch)
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5
    for _ in range(3):
        lat, rel, mn = eng.rows(tgt, tgt, dispatch=False)
        assert np.array_equal(lat, l0) and np.array_equal(rel, r0) and np.array_equal(mn, m0)


def test_kf_equals_generic_f64(route, monkeypatch):
    g = config("c2f")
    src = np.arange(0, g.n, 5, dtype=np.int32)
    tgt = g.targets()
    e1, (l1, r1, m1) = _rows(route, g, src, tgt, "kf", monkeypatch)
    e0, (l0, r0, m0) = _rows(route, g, src, tgt, "f64", monkeypatch)
    assert e1.info["kernel"] == 5 and e0.info["kernel"] == 0
    assert np.array_equal(l1, l0) and np.array_equal(r1, r0) and np.array_equal(m1, m0)


def test_kf_forced_on_integer_graphs(route, oracle_mod, monkeypatch):
    # integer latencies through KF: the same rows as the oracle (and as KBF/KD)
    g = internet_like(1500, 4, 21, name="kf_int")
    src = np.arange(0, g.n, 11, dtype=np.int32)
    eng, (lat, rel, mn) = _rows(route, g, src, g.targets(), "kf", monkeypatch)
    assert eng.info["kernel"] == 5
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(src, g.targets(), oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat) and np.array_equal(rel, orel)


def test_kf_vertex_loss_and_subset_targets(route, oracle_mod, monkeypatch):
    g = fractional(internet_like(3000, 3, 5, vloss=True, hosts=2500, name="kf_vl"), 3)
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5
    tgt = g.targets()
    src = tgt[::37]
    lat, rel, mn = eng.rows(src, tgt, dispatch=False)
    og = oracle_mod.OracleGraph(g)
    olat, orel, _, _ = og.source_rows(src, tgt, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    np.testing.assert_allclose(rel, orel, rtol=REL_TOL, atol=0)
    # unique shortest paths: igraph's own tie rule agrees
    ilat, irel, iuq, _ = og.source_rows(src, tgt, oracle_mod.TIE_IGRAPH)
    np.testing.assert_allclose(rel[iuq], irel[iuq], rtol=REL_TOL, atol=0)


def test_kf_directed_and_ragged(route, oracle_mod, monkeypatch):
    rng = np.random.default_rng(9)
    n = 700
    # a directed ring (strongly connected) plus random chords, fractional latencies
    a = np.arange(n)
    src = np.concatenate([a, rng.integers(0, n, 3000), a]).astype(np.int32)
    dst = np.concatenate([(a + 1) % n, rng.integers(0, n, 3000), a]).astype(np.int32)
    keep = (src != dst) | (np.arange(len(src)) >= n + 3000)
    src, dst = src[keep], dst[keep]
    _, first = np.unique(src.astype(np.int64) * n + dst, return_index=True)  # a simple graph
    first = np.sort(first)
    src, dst = src[first], dst[first]
    lat = np.round(rng.uniform(0.5, 90.0, len(src)), 3)
    loss = np.where(rng.random(len(src)) < 0.7, 0.0, rng.integers(1, 50, len(src)) * 1e-3)
    g = Graph(n=n, src=src, dst=dst, latency=lat, packetloss=loss, directed=True, name="kf_dir")
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5
    for s_ in (np.array([0], np.int32), np.arange(0, n, 3, dtype=np.int32)):
        t = np.arange(n - 1, -1, -2, dtype=np.int32)  # unsorted, a subset
        lat_, rel_, mn_ = eng.rows(s_, t, dispatch=False)
        olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(s_, t, oracle_mod.TIE_MINKEY)
        assert np.array_equal(lat_, olat) and np.array_equal(rel_, orel)


def test_kf_limits_fall_back(route, monkeypatch):
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    # more than 254 distinct reliabilities: the generic f64 kernel
    g = fractional(internet_like(1000, 3, 8, name="kf_many_r"), 4)
    g.packetloss = np.random.default_rng(1).uniform(0.0, 0.5, g.m)
    assert route.RouteEngine(g).info["kernel"] == 0


@pytest.mark.parametrize("delta", ["1e9", "0.004", "1e-6"])
def test_kf_extreme_bucket_widths(route, oracle_mod, monkeypatch, delta):
    """Bucket width far above every distance (one bucket: the ring holds a Bellman-Ford
    frontier, the case where a push could find no free slot -- ADVICE r03) and far below
    the arc latencies (a bucket per distinct distance): bit-exact against the oracle, and
    the overflow path (pushes moved to the pending bitmask) leaves nothing behind."""
    g = config("c2f")
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    monkeypatch.setenv("SHD_ROUTE_KFDELTA", delta)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5
    src = np.arange(3, g.n, 97, dtype=np.int32)
    tgt = g.targets()
    lat, rel, mn = eng.rows(src, tgt, dispatch=False)
    og = oracle_mod.OracleGraph(g)
    olat, orel, _, _ = og.source_rows(src, tgt, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))


# ---- KFH: the vertex state in an HBM slice (n above KF's LDS limit; C4f) ----------------

def test_kfh_equals_kf_rows(route, monkeypatch):
    # KFH forced on C2f (which KF takes): every row bit-identical to KF's, three launches
    g = config("c2f")
    tgt = g.targets()
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    e0 = route.RouteEngine(g)
    assert e0.info["kernel"] == 5 and e0.info["lds_resident"] == 1
    l0, r0, m0 = e0.rows(tgt, tgt, dispatch=False)
    monkeypatch.setenv("SHD_ROUTE_KFH", "1")
    e1 = route.RouteEngine(g)
    assert e1.info["kernel"] == 5 and e1.info["lds_resident"] == 0
    for _ in range(3):
        lat, rel, mn = e1.rows(tgt, tgt, dispatch=False)
        assert np.array_equal(lat, l0) and np.array_equal(rel, r0) and np.array_equal(mn, m0)


@pytest.mark.parametrize("ring", ["64", "700"])
def test_kfh_small_ring(route, oracle_mod, monkeypatch, ring):
    # KFH's ring holds what LDS leaves (C4f: 19.6k of 50k vertices): a gather that finds more
    # vertices below the bucket bound than the ring holds leaves the rest pending, a push
    # past it moves the ring to the pending bitmask, a hub list past it leaves the hubs to
    # their threads.  A 64 / 700-entry ring on C2f (2000 vertices) takes all three paths
    g = config("c2f")
    monkeypatch.setenv("SHD_ROUTE_KFH", "1")
    monkeypatch.setenv("SHD_ROUTE_KFH_RING", ring)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5 and eng.info["lds_resident"] == 0
    tgt = g.targets()
    src = tgt[::13]
    lat, rel, mn = eng.rows(src, tgt, dispatch=False)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(src, tgt, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))


def test_kfh_vertex_loss_directed(route, oracle_mod, monkeypatch):
    g = fractional(internet_like(3000, 3, 5, vloss=True, hosts=2500, name="kfh_vl"), 3)
    monkeypatch.setenv("SHD_ROUTE_KFH", "1")
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5 and eng.info["lds_resident"] == 0
    tgt = g.targets()
    src = tgt[::41]
    lat, rel, mn = eng.rows(src, tgt, dispatch=False)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(src, tgt, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    # KFH's LDS walks fold from (1.0 * f_s) * f_t, the reference's order: bit-exact
    assert np.array_equal(rel, orel)


@pytest.mark.parametrize("lossy", [0.05, 1.0])
def test_kfh_walks_and_deep_paths(route, oracle_mod, monkeypatch, lossy):
    """KFH's reliability rows by LDS walks (round 5), and the level passes a row falls back
    to when a path has more than 16 lossy arcs: an undirected chain of 600 vertices with
    sparse chords (paths of hundreds of hops), every arc lossy (1.0: every row falls back)
    or 5% of them (0.05: most rows walk), with vertex loss."""
    rng = np.random.default_rng(21)
    n = 600
    a = np.arange(n - 1)
    ch = rng.integers(0, n, (40, 2))
    ch = ch[ch[:, 0] != ch[:, 1]]
    src = np.concatenate([a, ch[:, 0]]).astype(np.int32)
    dst = np.concatenate([a + 1, ch[:, 1]]).astype(np.int32)
    key = np.minimum(src, dst).astype(np.int64) * n + np.maximum(src, dst)
    _, first = np.unique(key, return_index=True)
    first = np.sort(first)
    src, dst = src[first], dst[first]
    lat = np.round(rng.uniform(0.5, 20.0, len(src)), 2)
    loss = np.where(rng.random(len(src)) < lossy, rng.integers(1, 40, len(src)) * 1e-3, 0.0)
    # self-loops: a row's own target takes one (topology.c:1471-1499)
    src = np.concatenate([src, np.arange(n, dtype=np.int32)])
    dst = np.concatenate([dst, np.arange(n, dtype=np.int32)])
    lat = np.concatenate([lat, np.full(n, 0.25)])
    loss = np.concatenate([loss, np.zeros(n)])
    vl = np.where(rng.random(n) < 0.2, rng.integers(1, 30, n) * 1e-3, np.nan)
    g = Graph(n=n, src=src, dst=dst, latency=lat, packetloss=loss, vertex_packetloss=vl, name="kfh_chain")
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    monkeypatch.setenv("SHD_ROUTE_KFH", "1")
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5 and eng.info["lds_resident"] == 0
    tgt = np.arange(n, dtype=np.int32)
    s_ = np.arange(0, n, 7, dtype=np.int32)
    lat_, rel_, mn_ = eng.rows(s_, tgt, dispatch=False)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(s_, tgt, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat_, olat)
    np.testing.assert_allclose(rel_, orel, rtol=REL_TOL, atol=0)
    # a walked row folds from (1.0 * f_s) * f_t, the reference's order: bit-exact against the
    # oracle; a row that fell back to the level passes multiplies f_t last, as the LDS kernel
    # (level passes only) does: bit-exact against it.  Every row is one of the two; with 5% lossy
    # arcs most rows walk, with every arc lossy every row falls back
    monkeypatch.delenv("SHD_ROUTE_KFH")
    e2 = route.RouteEngine(g)
    assert e2.info["lds_resident"] == 1
    l2, r2, _ = e2.rows(s_, tgt, dispatch=False)
    assert np.array_equal(l2, lat_)
    walked = np.array([np.array_equal(rel_[i], orel[i]) for i in range(len(s_))])
    level = np.array([np.array_equal(rel_[i], r2[i]) for i in range(len(s_))])
    assert np.all(walked | level)
    if lossy == 1.0:
        assert level.all()
    else:
        assert walked.mean() > 0.5, walked.mean()


def test_kfh_20k_vertices(route, oracle_mod, monkeypatch):
    # above KF's LDS limit: KFH by default, sampled rows bit-exact against the oracle
    g = fractional(internet_like(20000, 4, 6, name="kfh_20k"), 5)
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    monkeypatch.delenv("SHD_ROUTE_KFH", raising=False)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 5 and eng.info["lds_resident"] == 0
    tgt = g.targets()
    src = np.concatenate([tgt[:3], tgt[::977], tgt[-2:]]).astype(np.int32)
    lat, rel, mn = eng.rows(src, tgt, dispatch=False)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(src, tgt, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))
