"""CPU: host attachment (shadow_amd/csrc/attach.c) against the restatement of
_topology_findAttachmentVertex (oracle/attach_ref.py, topology.c:2094-2366).

The reference's own tests attach every host of a one-vertex graph (all configs under
src/test and resource/examples), so the only fixture-pinned answer is vertex 0; the
multi-vertex cases are parity against the restatement, with the same glibc rand_r
stream on both sides (Shadow's Random, random.c:29-43) and the same number of draws."""
import random

import pytest

from oracle.attach_ref import ShadowRandom, find_attachment_vertex, string_to_ip

CODES = ["us", "US", "de", "De", "fr", "jp", ""]
TYPES = ["relay", "client", "CLIENT", "server", ""]


@pytest.fixture(scope="module")
def topo():
    from shadow_amd import build, topology
    build.build()
    topology.load_library()
    return topology


def _graphml(path, n, seed, default_city=None, declare=("ip", "citycode", "countrycode", "geocode", "type")):
    rng = random.Random(seed)
    keys = ['<key attr.name="latency" attr.type="double" for="edge" id="el" />',
            '<key attr.name="packetloss" attr.type="double" for="edge" id="ep" />',
            '<key attr.name="bandwidthup" attr.type="int" for="node" id="bu" />',
            '<key attr.name="bandwidthdown" attr.type="int" for="node" id="bd" />']
    for a in declare:
        if a == "citycode" and default_city is not None:
            keys.append(f'<key attr.name="{a}" attr.type="string" for="node" id="{a}"><default>{default_city}</default></key>')
        else:
            keys.append(f'<key attr.name="{a}" attr.type="string" for="node" id="{a}" />')
    ips = [f"11.0.{rng.randrange(4)}.{rng.randrange(8)}" for _ in range(6)] + \
          ["0.0.0.0", "127.0.0.1", "1.0.0.127", "999.1.1.1", "", "255.255.255.255", "10.1.2.3"]
    nodes = []
    for v in range(n):
        d = [f'<data key="bd">{1000 + v}</data><data key="bu">{2000 + 3 * v}</data>']
        for a in declare:
            if rng.random() < 0.2:
                continue  # no <data>: key default or ""
            val = {"ip": lambda: rng.choice(ips), "citycode": lambda: rng.choice(CODES),
                   "countrycode": lambda: rng.choice(CODES), "geocode": lambda: rng.choice(CODES),
                   "type": lambda: rng.choice(TYPES)}[a]()
            d.append(f'<data key="{a}">{val}</data>')
        nodes.append(f'<node id="v{v}">{"".join(d)}</node>')
    edges = [f'<edge source="v{v}" target="v{(v + 1) % n}"><data key="el">{1 + v % 7}</data>'
             f'<data key="ep">0.0</data></edge>' for v in range(n)]
    path.write_text('<graphml xmlns="http://graphml.graphdrawing.org/xmlns">' + "".join(keys) +
                    '<graph edgedefault="undirected">' + "".join(nodes) + "".join(edges) + "</graph></graphml>")
    return ips


def _hints(rng, ips):
    pick = lambda xs: rng.choice(xs + [None, None])
    return dict(ip=pick(ips + ["11.0.3.200", "0.0.0.0", "127.0.0.1", "not-an-ip"]), citycode=pick(CODES),
                countrycode=pick(CODES), geocode=pick(CODES), type=pick(TYPES))


@pytest.mark.parametrize("seed,n,default_city,declare", [
    (1, 40, None, ("ip", "citycode", "countrycode", "geocode", "type")),
    (2, 300, "US", ("ip", "citycode", "countrycode", "geocode", "type")),
    (3, 120, None, ("citycode", "type")),          # no ip key: never longest-prefix
    (4, 200, None, ("ip",)),                        # ip only
    (5, 1, None, ("ip", "citycode", "countrycode", "geocode", "type")),
])
def test_attach_matches_restatement(topo, tmp_path, seed, n, default_city, declare):
    p = tmp_path / "g.xml"
    ips = _graphml(p, n, seed, default_city, declare)
    idx = topo.AttachIndex(str(p))
    attrs = idx.vertex_attrs()
    rng = random.Random(100 + seed)
    for trial in range(400):
        h = _hints(rng, ips)
        r1, r2 = ShadowRandom(7 + trial), ShadowRandom(7 + trial)
        got = idx.find(r1.next_double, **h)
        want = find_attachment_vertex(attrs, n, r2, ip_hint=h["ip"], citycode_hint=h["citycode"],
                                      countrycode_hint=h["countrycode"], geocode_hint=h["geocode"],
                                      type_hint=h["type"])
        assert got == want, (trial, h)
        assert r1.draws == r2.draws, (trial, h)  # random_nextDouble consumed exactly as the reference
    idx.close()


def test_attach_many_distinct_codes(topo, tmp_path):
    """Every vertex with its own geocode and most with their own citycode (the interning
    table at its fullest), hints drawn from those codes in mixed case."""
    n = 500
    rng = random.Random(77)
    keys = ''.join(f'<key attr.name="{a}" attr.type="string" for="node" id="{a}" />'
                   for a in ("ip", "citycode", "geocode", "type"))
    keys += ('<key attr.name="latency" attr.type="double" for="edge" id="el" />'
             '<key attr.name="packetloss" attr.type="double" for="edge" id="ep" />'
             '<key attr.name="bandwidthup" attr.type="int" for="node" id="bu" />'
             '<key attr.name="bandwidthdown" attr.type="int" for="node" id="bd" />')
    city = [f"c{rng.randrange(400)}" for _ in range(n)]
    nodes = "".join(f'<node id="v{v}"><data key="bd">1</data><data key="bu">1</data>'
                    f'<data key="ip">11.{v % 7}.{v % 5}.{v % 250}</data><data key="citycode">{city[v]}</data>'
                    f'<data key="geocode">g{v}</data><data key="type">{rng.choice(TYPES)}</data></node>'
                    for v in range(n))
    edges = "".join(f'<edge source="v{v}" target="v{(v + 1) % n}"><data key="el">1</data><data key="ep">0</data></edge>'
                    for v in range(n))
    p = tmp_path / "many.xml"
    p.write_text(f'<graphml xmlns="http://graphml.graphdrawing.org/xmlns">{keys}<graph edgedefault="undirected">'
                 f'{nodes}{edges}</graph></graphml>')
    idx = topo.AttachIndex(str(p))
    attrs = idx.vertex_attrs()
    for trial in range(300):
        v = rng.randrange(n)
        h = {"citycode": rng.choice([city[v], city[v].upper(), "nowhere", None]),
             "geocode": rng.choice([f"G{v}", f"g{rng.randrange(n)}", None]),
             "type": rng.choice(TYPES + [None]),
             "ip": rng.choice([None, f"11.{v % 7}.{v % 5}.{v % 250}", f"11.{v % 7}.9.9"])}
        r1, r2 = ShadowRandom(trial), ShadowRandom(trial)
        want = find_attachment_vertex(attrs, n, r2, ip_hint=h["ip"], citycode_hint=h["citycode"],
                                      geocode_hint=h["geocode"], type_hint=h["type"])
        assert idx.find(r1.next_double, **h) == want and r1.draws == r2.draws, (trial, h)
    idx.close()


def test_attach_reference_configs_one_vertex(topo, tmp_path):
    """Every host of the reference's test/example configs joins vertex 0 (1-vertex graphs,
    e.g. src/test/tcp/tcp-blocking-lossy.test.shadow.config.xml with countrycode US)."""
    p = tmp_path / "one.xml"
    p.write_text('''<graphml xmlns="http://graphml.graphdrawing.org/xmlns">
  <key attr.name="packetloss" attr.type="double" for="edge" id="d4" />
  <key attr.name="latency" attr.type="double" for="edge" id="d3" />
  <key attr.name="bandwidthup" attr.type="int" for="node" id="d2" />
  <key attr.name="bandwidthdown" attr.type="int" for="node" id="d1" />
  <key attr.name="countrycode" attr.type="string" for="node" id="d0" />
  <graph edgedefault="undirected">
    <node id="poi-1"><data key="d0">US</data><data key="d1">10240</data><data key="d2">10240</data></node>
    <edge source="poi-1" target="poi-1"><data key="d3">50.0</data><data key="d4">0.25</data></edge>
  </graph></graphml>''')
    idx = topo.AttachIndex(str(p))
    r = ShadowRandom(1)
    for h in ({}, {"countrycode": "us"}, {"ip": "11.0.0.1", "type": "client"}, {"countrycode": "DE"}):
        assert idx.find(r.next_double, **h) == 0
    idx.close()


def test_attach_quirks(topo, tmp_path):
    """Exact IP match beats every code filter; longest-prefix on network-order values;
    127.0.0.1 stays usable (the host-order INADDR_LOOPBACK compare), 1.0.0.127 does not."""
    assert string_to_ip("127.0.0.1") == 0x0100007F and string_to_ip("1.0.0.127") == 0x7F000001
    p = tmp_path / "q.xml"
    keys = ('<key attr.name="latency" attr.type="double" for="edge" id="el" />'
            '<key attr.name="packetloss" attr.type="double" for="edge" id="ep" />'
            '<key attr.name="bandwidthup" attr.type="int" for="node" id="bu" />'
            '<key attr.name="bandwidthdown" attr.type="int" for="node" id="bd" />'
            '<key attr.name="ip" attr.type="string" for="node" id="ip" />'
            '<key attr.name="citycode" attr.type="string" for="node" id="cc" />')
    rows = [("10.0.0.1", "nyc"), ("10.0.0.2", "sfo"), ("127.0.0.1", "sfo"), ("1.0.0.127", "sfo"), ("10.0.1.9", "NYC")]
    nodes = "".join(f'<node id="n{i}"><data key="bd">1</data><data key="bu">1</data><data key="ip">{ip}</data>'
                    f'<data key="cc">{cc}</data></node>' for i, (ip, cc) in enumerate(rows))
    edges = "".join(f'<edge source="n{i}" target="n{(i + 1) % 5}"><data key="el">1</data><data key="ep">0</data></edge>'
                    for i in range(5))
    p.write_text(f'<graphml xmlns="http://graphml.graphdrawing.org/xmlns">{keys}<graph edgedefault="undirected">'
                 f'{nodes}{edges}</graph></graphml>')
    idx = topo.AttachIndex(str(p))
    attrs = idx.vertex_attrs()
    r = ShadowRandom(3)
    assert idx.find(r.next_double, ip="10.0.0.2", citycode="nyc") == 1      # exact IP wins
    assert idx.find(r.next_double, ip="127.0.0.1") == 2                      # loopback usable
    for h in ({"ip": "10.0.1.200", "citycode": "nyc"}, {"ip": "10.0.0.3"}, {"ip": "1.0.0.127"},
              {"ip": "0.0.0.0"}, {"ip": ""}, {"citycode": "NYC"}):
        r1, r2 = ShadowRandom(9), ShadowRandom(9)
        want = find_attachment_vertex(attrs, 5, r2, ip_hint=h.get("ip"), citycode_hint=h.get("citycode"))
        assert idx.find(r1.next_double, **h) == want and r1.draws == r2.draws, h
    idx.close()
