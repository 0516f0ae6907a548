"""GPU: K4 blocked min-plus Floyd-Warshall (fw.hpp) and its SOURCE rows, and the f64
in-place variant, against the oracle.

K4 has no reference equivalent (complete graphs take the direct path in Shadow 1.14,
topology.c:1321-1323); its rows are held to the SOURCE(s,.) semantics of every other
rows kernel: latency bit-exact (integer latencies: FW sums are exact), reliability
bit-exact against the oracle's engine tie rule (vertex factors 1.0 here).
"""
import numpy as np
import pytest

from shadow_amd.graph import complete_graph, config, internet_like

pytestmark = pytest.mark.gpu


def _fw_rows(eng, S, T):
    import torch
    dev = torch.device("cuda", 0)
    d_src = torch.from_numpy(np.ascontiguousarray(S, np.int32)).to(dev)
    d_tgt = torch.from_numpy(np.ascontiguousarray(T, np.int32)).to(dev)
    lat = torch.empty((len(S), len(T)), dtype=torch.float64, device=dev)
    rel = torch.empty_like(lat)
    mn = torch.empty(len(S), dtype=torch.float64, device=dev)
    eng.fw_table_async()
    eng.fw_rows_async(d_src, d_tgt, lat, rel, mn)
    eng.sync()
    return lat.cpu().numpy(), rel.cpu().numpy(), mn.cpu().numpy()


@pytest.mark.parametrize("name", ["k200", "ba300", "ties", "k130_odd", "ba100"])
def test_fw_rows_bitexact(oracle_mod, name):
    from shadow_amd import route
    from tests.golden import make_golden as mg
    g = {"k200": lambda: complete_graph(200, seed=5), "ba300": lambda: internet_like(300, 3, seed=17),
         "ties": lambda: mg._ties(300, 33), "k130_odd": lambda: complete_graph(130, seed=6),
         "ba100": lambda: internet_like(100, 2, seed=9)}[name]()  # (2 pivot tiles)
    eng = route.RouteEngine(g)
    T = np.arange(g.n, dtype=np.int32)
    S = T[::3]
    lat, rel, mn = _fw_rows(eng, S, T)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))


def test_fw_rows_all_sources_sparse(oracle_mod):
    """Every source of a sparse 700-vertex graph (11 pivot tiles, multi-hop paths through
    each): the pivot tiles closed inside the rest launches give the oracle's full table."""
    from shadow_amd import route
    g = internet_like(700, 2, seed=23)
    eng = route.RouteEngine(g)
    T = np.arange(g.n, dtype=np.int32)
    lat, rel, _ = _fw_rows(eng, T, T)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(T, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)


@pytest.mark.parametrize("name", ["directed", "wide"])
def test_fw_rows_parent_search(oracle_mod, name):
    """The parent search's two start rules: the threshold table (w <= 255) and the binary
    search (distances past 255: weights up to 4000), and directed in-lists."""
    from shadow_amd import route
    from tests.golden import make_golden as mg
    if name == "directed":
        g = mg._directed(250, 21)
    else:
        g = complete_graph(180, seed=9)
        g.latency = np.where(g.src != g.dst, g.latency * 16 + 100, g.latency)
    eng = route.RouteEngine(g)
    T = np.arange(g.n, dtype=np.int32)
    S = T[::2]
    lat, rel, mn = _fw_rows(eng, S, T)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    if name == "wide":
        assert np.nanmax(olat) > 300 and np.nanmin(olat[olat > 20]) < 255  # both start rules


def test_fw_table_vs_oracle_floyd_warshall(oracle_mod):
    """The K4 table (every pair, self distance 0) against the oracle's plain FW, and the
    f64 in-place shd_route_fw_async against the same."""
    import torch
    from shadow_amd import route
    g = complete_graph(256, seed=12)
    d = np.full((g.n, g.n), np.inf)
    np.fill_diagonal(d, 0.0)
    for a, b, w in zip(g.src, g.dst, g.latency):
        if a != b:
            d[a, b] = min(d[a, b], w); d[b, a] = min(d[b, a], w)
    ref = oracle_mod.floyd_warshall(d)
    eng = route.RouteEngine(g)
    T = np.arange(g.n, dtype=np.int32)
    lat, _, _ = _fw_rows(eng, T, T)
    off = ~np.eye(g.n, dtype=bool)
    assert np.array_equal(lat[off], ref[off])
    dd = torch.from_numpy(d.copy()).cuda()
    eng.fw_async(dd)
    eng.sync()
    assert np.array_equal(dd.cpu().numpy(), ref)


def test_c5_fw_rows_sampled(oracle_mod):
    """C5 (complete K4000 + self-loops): the K4 table and rows of sampled sources against
    the oracle's Dijkstra rows (SOURCE semantics) and against the KD rows."""
    from shadow_amd import route
    g = config("c5")
    eng = route.RouteEngine(g)
    assert eng.info["is_complete"] == 1
    T = np.arange(g.n, dtype=np.int32)
    S = np.array([0, 1, 777, 2048, 3999], np.int32)
    lat, rel, mn = _fw_rows(eng, S, T)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    klat, krel, _ = eng.rows(S, T, dispatch=False)
    assert np.array_equal(lat, klat) and np.array_equal(rel, krel)


def test_fw_unsupported_fractional():
    from shadow_amd import route
    g = internet_like(120, 2, seed=3)
    g.latency = g.latency + 0.5
    eng = route.RouteEngine(g)
    with pytest.raises(route.RouteError) as e:
        eng.fw_table_async()
    assert e.value.code == route.EUNSUPPORTED


def test_fw_ineligible_stays_unsupported():
    """A graph whose K4 rows state overflows LDS (12 n + 4 (bound + 2) bytes): every
    fw_table call answers EUNSUPPORTED (nothing is half-built by the first), and rows
    from the table are refused."""
    import torch
    from shadow_amd import route
    g = internet_like(10000, 2, seed=31)
    g.latency = np.where(g.src != g.dst, g.latency * 40, g.latency)
    eng = route.RouteEngine(g)
    assert eng.info["integer_weights"] == 1 and 12 * g.n + 4 * (eng.info["dist_bound"] + 2) > 160 * 1024
    for _ in range(2):
        with pytest.raises(route.RouteError) as e:
            eng.fw_table_async()
        assert e.value.code == route.EUNSUPPORTED
    dev = torch.device("cuda", 0)
    S = torch.zeros(1, dtype=torch.int32, device=dev)
    lat = torch.empty((1, 1), dtype=torch.float64, device=dev)
    with pytest.raises(route.RouteError) as e:
        eng.fw_rows_async(S, S, lat, lat.clone(), None)
    assert e.value.code == route.EINVAL


def test_fw_on_side_stream(oracle_mod):
    """Table (with its first-call in-list build) and rows enqueued on a non-default torch
    stream: the in-lists are built on that stream, ahead of the kernels that read them."""
    import torch
    from shadow_amd import route
    g = internet_like(600, 3, seed=41)
    eng = route.RouteEngine(g)
    dev = torch.device("cuda", 0)
    T = np.arange(g.n, dtype=np.int32)
    S = T[::5]
    st = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(st):
        d_src = torch.from_numpy(S).to(dev)
        d_tgt = torch.from_numpy(T).to(dev)
        lat = torch.empty((len(S), len(T)), dtype=torch.float64, device=dev)
        rel = torch.empty_like(lat)
        eng.fw_table_async(st.cuda_stream)
        eng.fw_rows_async(d_src, d_tgt, lat, rel, None, stream=st.cuda_stream)
    eng.sync(st.cuda_stream)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat.cpu().numpy(), olat)
    assert np.array_equal(rel.cpu().numpy(), orel)


def test_c5_direct_table_full(oracle_mod):
    """C5's reference semantics on the whole table: K3 (direct_rows_kernel) over all
    4,000 x 4,000 pairs with the topology.c:2019 dispatch (complete graph -> every pair
    DIRECT, topology.c:1877-1927) against the oracle's eager direct-mode table, and K5
    (runahead min over the row minima, topology.c:1374-1385) against its min latency."""
    import torch
    from shadow_amd import route
    g = config("c5")
    eng = route.RouteEngine(g)
    assert eng.info["is_complete"] == 1
    T = np.arange(g.n, dtype=np.int32)
    dev = torch.device("cuda", 0)
    d_src = torch.from_numpy(T).to(dev)
    lat = torch.empty((g.n, g.n), dtype=torch.float64, device=dev)
    rel = torch.empty_like(lat)
    mn = torch.full((g.n,), float("inf"), dtype=torch.float64, device=dev)
    out = torch.full((1,), float("inf"), dtype=torch.float64, device=dev)
    eng.rows_async(d_src, d_src, lat, rel, mn, dispatch=True)
    eng.min_reduce_async(mn, out)
    eng.sync()
    tab = oracle_mod.OracleGraph(g).eager_table(T)
    assert tab["is_direct"].all()
    assert np.array_equal(lat.cpu().numpy(), tab["lat"])
    assert np.array_equal(rel.cpu().numpy(), tab["rel"])
    assert np.array_equal(mn.cpu().numpy(), tab["lat"].min(axis=1))
    assert float(out.item()) == tab["min_latency"]


@pytest.mark.parametrize("cfg", ["ba700", "c5"])
def test_fw_fused_panels_equal_separate_launches(monkeypatch, cfg):
    """The default K4 sequence (each rest launch also closes the next pivot and computes its
    panels, fw_restp_kernel) and its persistent-workgroup form (SHD_ROUTE_FWREST=3, the next
    tile prefetched during the product; 1024 and 7 workgroups) against the separate panel +
    rest launches (SHD_ROUTE_FWREST=1): every SOURCE row of every source bit-identical."""
    import torch
    from shadow_amd import route
    g = internet_like(700, 2, seed=23) if cfg == "ba700" else config("c5")
    T = np.arange(g.n, dtype=np.int32)
    dev = torch.device("cuda", 0)
    d_T = torch.from_numpy(T).to(dev)
    out = []
    for mode, P in (("1", "1024"), ("0", "1024"), ("3", "1024"), ("3", "7")):
        monkeypatch.setenv("SHD_ROUTE_FWREST", mode)
        monkeypatch.setenv("SHD_ROUTE_FWP", P)
        eng = route.RouteEngine(g)
        lat = torch.empty((g.n, g.n), dtype=torch.float64, device=dev)
        rel = torch.empty_like(lat)
        mn = torch.empty(g.n, dtype=torch.float64, device=dev)
        for _ in range(2):  # (a second table on the same context: flags re-armed)
            eng.fw_table_async()
            eng.fw_rows_async(d_T, d_T, lat, rel, mn)
        eng.sync()
        out.append((lat, rel, mn))
    for o in out[1:]:
        assert torch.equal(out[0][0], o[0]) and torch.equal(out[0][1], o[1]) and torch.equal(out[0][2], o[2])


@pytest.mark.parametrize("case", ["k200_dense_r", "manyrel"])
def test_fw_rows_reliability_paths(oracle_mod, monkeypatch, case):
    """fw_rows' two ways to a parent arc's reliability (round 5): by its index in a dense u8
    matrix into a table of the distinct reliabilities (<= 255 of them, the default) or by the
    dense n x n f64 table -- forced (SHD_ROUTE_FWDENSER=1), or because a graph has more distinct
    reliabilities than an index holds ("manyrel": a continuous loss per edge)."""
    import dataclasses
    from shadow_amd import route
    if case == "k200_dense_r":
        monkeypatch.setenv("SHD_ROUTE_FWDENSER", "1")
        g = complete_graph(200, seed=5)
    else:
        monkeypatch.delenv("SHD_ROUTE_FWDENSER", raising=False)
        g = internet_like(300, 3, seed=19)
        rng = np.random.default_rng(4)
        g = dataclasses.replace(g, packetloss=rng.random(g.m) * 0.01)
    eng = route.RouteEngine(g)
    T = np.arange(g.n, dtype=np.int32)
    S = T[::2]
    lat, rel, mn = _fw_rows(eng, S, T)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)


@pytest.mark.parametrize("fwp8", ["1", "0"])
@pytest.mark.parametrize("fwpk", ["1", "0"])
def test_fw_rows_key_forms(oracle_mod, monkeypatch, fwpk, fwp8):
    """The two in-list key forms (round 6): packed (every latency <= 255: (255 - w) << 24 |
    u << 8 | reliability index, the parent search hands the index to fw_rows) and wide
    ((0xFFFF - w) << 16 | u, the index gathered from the dense matrix; SHD_ROUTE_FWPK=0).
    A sparse graph with w <= 250 whose distances reach ~870, so most targets start the
    packed search at the list head (distance past 255) and the rest from the threshold
    table; lossy arcs, so the reliability index matters.  Both parent searches: eight
    sources per workgroup (fw_parent8_kernel) and one (fw_parent_kernel, SHD_ROUTE_FWP8=0)."""
    from shadow_amd import route
    monkeypatch.setenv("SHD_ROUTE_FWPK", fwpk)
    monkeypatch.setenv("SHD_ROUTE_FWP8", fwp8)
    g = internet_like(400, 2, seed=4)
    assert g.latency.max() <= 255
    eng = route.RouteEngine(g)
    T = np.arange(g.n, dtype=np.int32)
    S = T[::3]
    lat, rel, mn = _fw_rows(eng, S, T)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.nanmax(olat) > 255 and (olat[np.isfinite(olat)] < 255).any()
    assert (orel[np.isfinite(orel)] < 1.0).any()
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))
