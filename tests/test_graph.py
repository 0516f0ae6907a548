"""CPU: synthetic topology generators and graphml output."""
import numpy as np

from shadow_amd.graph import barabasi_albert_edges, complete_graph, config, internet_like, to_graphml


def test_c2_shape_and_determinism():
    g1, g2 = config("c2"), config("c2")
    assert g1.n == 2000 and g1.m_nonloop == 9975 and g1.m == 9975 + 2000 and g1.nnz == 19950
    assert np.array_equal(g1.src, g2.src) and np.array_equal(g1.latency, g2.latency)
    nl = g1.src != g1.dst
    assert g1.latency[nl].min() >= 1 and g1.latency[nl].max() <= 250
    assert np.all(g1.latency == np.floor(g1.latency))
    assert np.all(g1.latency[~nl] <= 10)
    assert np.all((g1.packetloss >= 0) & (g1.packetloss <= 0.01 + 1e-12))


def test_ba_simple_and_counts():
    rng = np.random.default_rng(0)
    e = barabasi_albert_edges(500, 4, rng)
    assert len(e) == 4 * (500 - 4)
    key = set(map(tuple, np.sort(e, axis=1).tolist()))
    assert len(key) == len(e) and np.all(e[:, 0] != e[:, 1])


def test_c3_attached_subset():
    g = config("c3")
    A = g.targets()
    assert g.n == 10000 and g.m_nonloop == 39984
    assert 9000 < len(A) < 9700 and np.all(np.diff(A) > 0)


def test_complete_counts():
    g = complete_graph(50, seed=1)
    assert g.m == 50 * 49 // 2 + 50


def test_graphml_writer(tmp_path):
    g = internet_like(30, 2, seed=1, prefer_direct=True)
    p = tmp_path / "g.graphml.xml"
    to_graphml(g, str(p))
    txt = p.read_text()
    assert txt.count("<node ") == 30 and txt.count("<edge ") == g.m
    assert "preferdirectpaths" in txt
