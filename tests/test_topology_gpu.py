"""GPU: the C front end (topology.c semantics) end to end over the HIP engine."""
import json
import lzma
import os

import numpy as np
import pytest

from shadow_amd.graph import Graph, config, example_one_vertex, internet_like, to_graphml

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def topo():
    from shadow_amd import topology
    topology.load_library()
    return topology


def _small(name):
    z = np.load(os.path.join(GOLD, "small_tables.npz"))
    p = f"{name}__"
    vl = z[p + "vertex_packetloss"]
    g = Graph(n=int(z[p + "n"]), src=z[p + "src"], dst=z[p + "dst"], latency=z[p + "latency"],
              packetloss=z[p + "packetloss"], vertex_packetloss=vl if len(vl) else None,
              directed=bool(z[p + "directed"]), prefer_direct=bool(z[p + "prefer_direct"]))
    return g, z, p


@pytest.mark.parametrize("name", ["ba60", "ba80_prefer", "k24", "ba100_attached", "dir40", "ba90_frac"])
def test_cache_matches_golden_eager_table(topo, name):
    g, z, p = _small(name)
    A = z[p + "attached"]
    t = topo.Topology.from_graph(g)
    t.attach_all(A)
    lat, rel = t.table(A)
    assert np.array_equal(lat, z[p + "lat"]), name
    uq = z[p + "unique"]
    assert np.array_equal(rel[uq], z[p + "rel"][uq]), name
    assert t.min_path_latency() == float(z[p + "min_latency"])
    isd = np.array([[t.is_direct(a, b) for b in A] for a in A], bool)
    assert np.array_equal(isd, z[p + "is_direct"]), name


def test_example_config_graphml_kat(topo, tmp_path):
    # resource/examples/shadow.config.xml: 2 hosts on the single vertex
    g = example_one_vertex(0.0, 0.01, 50.0)
    pth = tmp_path / "ex.graphml.xml"
    to_graphml(g, str(pth))
    t = topo.Topology.new(str(pth))
    t.attach(0)
    assert t.get_latency(0, 0) == 50.0 and t.get_reliability(0, 0) == 0.99
    assert t.is_routable(0, 0) and t.is_direct(0, 0) == 1
    assert t.runahead_ns() == 50_000_000


def test_reference_bundled_file(topo):
    """topology_new on the reference's own resource/topology.graphml.xml.xz (committed
    byte for byte): complete -> every pair direct (topology.c:1877-1927); the whole
    lookup table equals the committed digests, runahead 5 ms."""
    import hashlib
    exp = json.load(open(os.path.join(GOLD, "bundled_expected.json")))
    t = topo.Topology.new(os.path.join(GOLD, "topology.graphml.xml.xz"))
    n = t.vertex_count()
    assert n == 183 and t.find_vertex("poi-112") == 0
    t.attach_all(range(n))
    lat, rel = t.table(range(n))
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a, np.float64).tobytes()).hexdigest()
    assert sha(lat) == exp["lat_sha"] and sha(rel) == exp["rel_sha"]
    assert t.min_path_latency() == exp["min_latency"] == 5.0 and t.runahead_ns() == 5_000_000


def test_late_attach_with_concurrent_lookups(topo):
    """Lookups running while another thread attaches vertices (a late attach retires the
    filled cache; readers holding it stay valid), and packet counters carried over."""
    import threading
    g = internet_like(60, 2, seed=10)
    t = topo.Topology.from_graph(g)
    t.attach_all(range(0, 60, 2))
    ref = {(a, b): t.get_latency(a, b) for a in range(0, 60, 6) for b in range(0, 60, 4)}
    for _ in range(5):
        t.increment_path_packet_counter(0, 4)
    stop = threading.Event()
    bad = []
    def reader():
        while not stop.is_set():
            for (a, b), L in ref.items():
                if t.get_latency(a, b) != L:
                    bad.append((a, b))
    th = [threading.Thread(target=reader) for _ in range(4)]
    [x.start() for x in th]
    for v in range(1, 60, 2):
        t.attach(v)
        t.get_latency(0, v)  # refills over the grown set
    stop.set(); [x.join() for x in th]
    assert not bad
    assert t.packet_count(0, 4) == 5 and t.packet_count(4, 0) == 5
    assert t.attached_count() == 60 and t.get_latency(1, 3) > 0


def test_bundled_topology_xz(topo, tmp_path):
    z = np.load(os.path.join(GOLD, "bundled_topology.npz"))
    g = Graph(n=int(z["n"]), src=z["src"], dst=z["dst"], latency=z["latency"], packetloss=z["packetloss"],
              vertex_packetloss=z["vertex_packetloss"], directed=bool(z["directed"]), ids=list(z["ids"]))
    pth = tmp_path / "topology.graphml.xml"
    to_graphml(g, str(pth))
    pxz = tmp_path / "topology.graphml.xml.xz"
    pxz.write_bytes(lzma.compress(pth.read_bytes()))
    t = topo.Topology.new(str(pxz))
    assert t.find_vertex("poi-112") == 0
    t.attach_all(range(g.n))
    lat, rel = t.table(range(g.n))
    w = {}
    for a, b, L in zip(g.src, g.dst, g.latency):
        w[(a, b)] = w[(b, a)] = L
    assert all(lat[s, d] == w[(s, d)] for s in range(0, g.n, 13) for d in range(g.n))
    assert np.all(rel == 1.0 - 0.005)
    assert t.min_path_latency() == 5.0 and t.runahead_ns() == 5_000_000


def test_unattached_and_counters(topo):
    g = internet_like(50, 2, seed=8)
    t = topo.Topology.from_graph(g)
    t.attach_all([1, 5, 9])
    assert t.get_latency(1, 2) == -1.0 and not t.is_routable(2, 1)
    for _ in range(3):
        t.increment_path_packet_counter(5, 9)
    t.increment_path_packet_counter(9, 5)  # same cached Path (reverse lookup)
    assert t.packet_count(5, 9) == 4 and t.packet_count(9, 5) == 4
    # attaching later refills over the grown set
    t.attach(2)
    assert t.get_latency(1, 2) > 0


def test_counters_concurrent(topo):
    """Worker threads count packets at once (worker.c:279 from every worker): the per-pair
    atomic counters lose nothing, either orientation lands on the same Path."""
    import threading
    g = internet_like(40, 2, seed=9)
    t = topo.Topology.from_graph(g)
    t.attach_all(range(g.n))
    pairs = [(a, b) for a in range(0, 40, 7) for b in range(0, 40, 5)]
    def work(seed):
        for k in range(4000):
            a, b = pairs[(seed * 31 + k) % len(pairs)]
            t.increment_path_packet_counter(a, b) if k & 1 else t.increment_path_packet_counter(b, a)
    th = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    [x.start() for x in th]; [x.join() for x in th]
    want = {}
    for i in range(8):
        for k in range(4000):
            a, b = pairs[(i * 31 + k) % len(pairs)]
            key = (min(a, b), max(a, b))
            want[key] = want.get(key, 0) + 1
    for (a, b), c in want.items():
        assert t.packet_count(a, b) == c and t.packet_count(b, a) == c


def test_multi_context_fill_equals_single(topo):
    g = config("c2")
    A = np.arange(0, g.n, 3)
    t1 = topo.Topology.from_graph(g)
    t2 = topo.Topology.from_graph(g, devices=(0, 0, 0))  # rows sharded over 3 contexts
    t1.attach_all(A); t2.attach_all(A)
    t1.fill(); t2.fill()
    sel = A[::17]
    l1, r1 = t1.table(sel)
    l2, r2 = t2.table(sel)
    assert np.array_equal(l1, l2) and np.array_equal(r1, r2)
    assert t1.min_path_latency() == t2.min_path_latency()


@pytest.mark.parametrize("devices", [(0,), (0, 0)])
def test_fill_c3_matches_golden_rows(topo, devices):
    """The eager fill at C3 (9,337 attached vertices, a 43.6M-pair triangle in pinned host
    memory) through shd_route_fill_triangle: one seeded plan per context (two contexts:
    the plan's forest partition, rows out of triangle order).  The golden-sampled rows
    read back through the getters: latency equal to the golden digests (the table is
    symmetric); reliability, on the pairs the row's own source wrote (targets at or after
    it in attach order, first writer wins: topology.c:1307-1336), equal to the engine
    rows, which must themselves hash to the golden digests."""
    import hashlib
    from shadow_amd import route
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a, np.float64).tobytes()).hexdigest()
    dig = json.load(open(os.path.join(GOLD, "rows_digests.json")))["c3"]
    g = config("c3")
    T = g.targets()
    t = topo.Topology.from_graph(g, devices=devices)
    t.attach_all(T)
    sec = t.fill()
    assert sec > 0
    rows = dig["rows"][::4]
    S = np.array([r["src"] for r in rows], np.int32)
    eng = route.RouteEngine(g)
    lat, rel, mn = eng.rows(S, T)
    pos = {int(v): i for i, v in enumerate(sorted(int(x) for x in T))}
    for k, r in enumerate(rows):
        assert sha(lat[k]) == r["lat_sha"] and sha(rel[k]) == r["rel_sha"]
        s = r["src"]
        fl = np.array([t.get_latency(s, int(d)) for d in T])
        assert sha(fl) == r["lat_sha"], s
        own = np.array([pos[int(d)] >= pos[s] for d in T])
        fr = np.array([t.get_reliability(s, int(d)) for d in T])
        assert np.array_equal(fr[own], rel[k][own]), s
    # minimumPathLatency (topology.c:1374-1385): a lightest arc between two attached
    # vertices is their shortest path, so the minimum is that arc or a self pair
    att = np.zeros(g.n, bool)
    att[T] = True
    both = att[g.src] & att[g.dst] & (g.src != g.dst)
    selfs = [t.get_latency(int(v), int(v)) for v in T]
    assert t.min_path_latency() == min(float(g.latency[both].min()), min(selfs))


def test_dump_paths(topo, tmp_path):
    import ctypes
    g = internet_like(12, 2, seed=2)
    t = topo.Topology.from_graph(g)
    t.attach_all(range(g.n))
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    out = tmp_path / "paths.txt"
    fp = libc.fopen(str(out).encode(), b"w")
    assert topo.load_library().shd_topology_dump_paths(t._h, fp) == 0
    libc.fclose(fp)
    lines = out.read_text().splitlines()
    assert len(lines) == g.n * (g.n + 1) // 2
    assert lines[0].startswith("Found path 0<->0 in cache: SourceIndex=0 DestinationIndex=0 Latency=")


def test_topology_attach_hosts(topo, tmp_path):
    """topology_attach (topology.c:2371-2439) end to end: the vertex as the restatement of
    _topology_findAttachmentVertex picks it, the vertex joins the routed set, and the
    default bandwidths come back as (guint64) casts of the vertex attributes."""
    import random
    from oracle.attach_ref import ShadowRandom, find_attachment_vertex
    from tests.test_attach import _graphml, _hints
    p = tmp_path / "hosts.xml"
    ips = _graphml(p, 60, 11)
    idx = topo.AttachIndex(str(p))
    attrs = idx.vertex_attrs()
    t = topo.Topology.new(str(p))
    rng = random.Random(5)
    r1, r2 = ShadowRandom(42), ShadowRandom(42)   # one pool across hosts, as Shadow's
    want_set = set()
    for _ in range(30):
        h = _hints(rng, ips)
        v, down, up = t.attach_host(r1.next_double, **h)
        w = find_attachment_vertex(attrs, 60, r2, ip_hint=h["ip"], citycode_hint=h["citycode"],
                                   countrycode_hint=h["countrycode"], geocode_hint=h["geocode"], type_hint=h["type"])
        assert v == w and (down, up) == (1000 + v, 2000 + 3 * v)
        want_set.add(v)
    assert r1.draws == r2.draws
    A = sorted(want_set)
    assert t.attached_count() == len(A)
    # the ring has no self-loops: the batch cannot store (a, a) (topology.c:1488-1495), so
    # the reference's (a, a) lookup computes the path to self, 2 * the lightest out-edge
    # (topology.c:1674-1676, 1545-1653); every other pair is the ring distance
    w = [1 + v % 7 for v in range(60)]   # edge v -- v+1 (mod 60)
    def ring(a, b):
        if a == b:
            return 2.0 * min(w[a], w[a - 1])
        lo, hi = min(a, b), max(a, b)
        d = float(sum(w[lo:hi]))
        return min(d, float(sum(w)) - d)
    for a in A:
        for b in A:
            assert t.is_routable(a, b)
            assert t.get_latency(a, b) == ring(a, b) and t.get_reliability(a, b) == 1.0
    assert t.min_path_latency() == min(ring(a, b) for a in A for b in A)
    idx.close()


@pytest.mark.parametrize("name", ["ba60", "ba80_prefer", "k24", "ba100_attached", "dir40", "ba120_vloss"])
def test_compact_triangle_equals_interleaved(topo, monkeypatch, name):
    """The compact fill layout (SHD_ROUTE_FILL_LAT16: six pairs per 64-byte line, u16
    latency widened exactly) against the interleaved doubles: every getter on every pair,
    the dump, the minimum and the self pairs agree bit for bit; single and sharded fills."""
    g, z, p = _small(name)
    A = z[p + "attached"]
    tabs = []
    for mode, devs in (("0", (0,)), ("1", (0,)), ("1", (0, 0, 0))):
        monkeypatch.setenv("SHD_TOPOLOGY_LAT16", mode)
        t = topo.Topology.from_graph(g, devices=devs)
        t.attach_all(A)
        lat, rel = t.table(A)
        cnt = [t.is_routable(int(a), int(b)) for a in A for b in A]
        tabs.append((lat, rel, t.min_path_latency(), cnt))
    for lat, rel, mn, cnt in tabs[1:]:
        assert np.array_equal(lat, tabs[0][0], equal_nan=True)
        assert np.array_equal(rel, tabs[0][1], equal_nan=True)
        assert mn == tabs[0][2] and cnt == tabs[0][3]
    assert np.array_equal(tabs[0][0], z[p + "lat"])


def test_compact_triangle_c3_sharded(topo, monkeypatch):
    """C3 (9,337 attached) filled in the compact layout over two contexts (rows out of
    triangle order, each row's lines disjoint) against the interleaved fill, on the
    golden-sampled rows through the getters."""
    g = config("c3")
    T = g.targets()
    dig = json.load(open(os.path.join(GOLD, "rows_digests.json")))["c3"]
    S = [r["src"] for r in dig["rows"][::6]]
    out = []
    for mode, devs in (("0", (0,)), ("1", (0, 0))):
        monkeypatch.setenv("SHD_TOPOLOGY_LAT16", mode)
        t = topo.Topology.from_graph(g, devices=devs)
        t.attach_all(T)
        t.fill()
        out.append((np.array([[t.get_latency(s, int(d)) for d in T] for s in S]),
                    np.array([[t.get_reliability(s, int(d)) for d in T] for s in S]), t.min_path_latency()))
        t.close()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1]) and out[0][2] == out[1][2]
