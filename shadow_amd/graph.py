"""Topology container and seeded synthetic topologies.

A ``Graph`` holds exactly what igraph holds after ``igraph_read_graph_graphml``
for the attributes Shadow reads (reference topology.c:565-722): vertices and edges
numbered in graphml document order, edge ``latency`` / ``packetloss`` and the
optional vertex ``packetloss`` (NaN = attribute absent, topology.c:330-347).
"""
from __future__ import annotations

import dataclasses
import math
import xml.sax.saxutils as _sx
from typing import Optional

import numpy as np


@dataclasses.dataclass
class Graph:
    n: int
    src: np.ndarray          # int32 [m]
    dst: np.ndarray          # int32 [m]
    latency: np.ndarray      # float64 [m], ms
    packetloss: np.ndarray   # float64 [m]
    vertex_packetloss: Optional[np.ndarray] = None  # float64 [n], NaN = absent
    directed: bool = False
    prefer_direct: bool = False
    ids: Optional[list] = None
    attached: Optional[np.ndarray] = None  # vertices with >= 1 attached host (sorted)
    name: str = "graph"

    @property
    def m(self) -> int:
        return int(len(self.src))

    @property
    def m_nonloop(self) -> int:
        return int(np.count_nonzero(self.src != self.dst))

    @property
    def nnz(self) -> int:
        """SSSP arcs: 2 per undirected non-loop edge (self-loops never relax)."""
        k = self.m_nonloop
        return k if self.directed else 2 * k

    def targets(self) -> np.ndarray:
        if self.attached is not None:
            return np.asarray(self.attached, np.int32)
        return np.arange(self.n, dtype=np.int32)

    def vertex_id(self, v: int) -> str:
        return self.ids[v] if self.ids is not None else f"poi-{v}"


# ---------------------------------------------------------------------------
# generators

def barabasi_albert_edges(n: int, m: int, rng: np.random.Generator) -> np.ndarray:
    """Preferential attachment (Barabasi-Albert) as networkx.barabasi_albert_graph:
    a star on m+1 vertices, then each new vertex attaches to m distinct targets
    drawn proportionally to degree.  Returns [k,2] int32 edges (m*(n-m) of them)."""
    if not (1 <= m < n):
        raise ValueError("need 1 <= m < n")
    edges = [(0, t) for t in range(1, m + 1)]
    repeated = np.empty(2 * m * n, np.int64)
    rl = 0
    for t in range(1, m + 1):
        repeated[rl] = 0; repeated[rl + 1] = t; rl += 2
    for src in range(m + 1, n):
        chosen = set()
        while len(chosen) < m:
            draws = rng.integers(0, rl, size=2 * m)
            for d in draws:
                chosen.add(int(repeated[d]))
                if len(chosen) == m:
                    break
        tg = sorted(chosen)
        for t in tg:
            edges.append((src, t))
            repeated[rl] = t; repeated[rl + 1] = src; rl += 2
    return np.asarray(edges, np.int32)


def _edge_attrs(rng, k, lo=1, hi=250):
    lat = rng.integers(lo, hi + 1, size=k).astype(np.float64)
    lossy = rng.random(k) >= 0.8
    loss = np.where(lossy, rng.integers(1, 101, size=k) * 1e-4, 0.0)
    return lat, loss


def internet_like(n: int, m_ba: int, seed: int, *, exact_edges: Optional[int] = None,
                  vloss: bool = False, hosts: Optional[int] = None, name: str = "synthetic",
                  prefer_direct: bool = False) -> Graph:
    """BA graph, integer-ms latency U[1,250], self-loop on
    every vertex with latency U[1,10], edge loss 0 (p=0.8) else k*1e-4 (k in U[1,100]),
    vertex loss 0.0 (or U{0..10}*1e-4 with vloss=True)."""
    rng = np.random.default_rng(seed)
    e = barabasi_albert_edges(n, m_ba, rng)
    if exact_edges is not None and exact_edges > len(e):
        have = set(map(tuple, np.sort(e, axis=1).tolist()))
        extra = []
        while len(have) < exact_edges:
            a, b = (int(x) for x in rng.integers(0, n, size=2))
            if a == b:
                continue
            key = (min(a, b), max(a, b))
            if key in have:
                continue
            have.add(key)
            extra.append(key)
        e = np.concatenate([e, np.asarray(extra, np.int32).reshape(-1, 2)])
    lat, loss = _edge_attrs(rng, len(e))
    loops = np.arange(n, dtype=np.int32)
    llat = rng.integers(1, 11, size=n).astype(np.float64)
    _, lloss = _edge_attrs(rng, n)
    vl = (rng.integers(0, 11, size=n) * 1e-4) if vloss else np.zeros(n)
    attached = None
    if hosts is not None:
        attached = np.unique(rng.integers(0, n, size=hosts)).astype(np.int32)
    return Graph(n=n,
                 src=np.concatenate([e[:, 0], loops]).astype(np.int32),
                 dst=np.concatenate([e[:, 1], loops]).astype(np.int32),
                 latency=np.concatenate([lat, llat]),
                 packetloss=np.concatenate([loss, lloss]),
                 vertex_packetloss=vl.astype(np.float64),
                 attached=attached, name=name, prefer_direct=prefer_direct)


def complete_graph(n: int, seed: int, name: str = "complete") -> Graph:
    """C5: K_n + self-loops, integer latency U[1,250], same loss distributions."""
    rng = np.random.default_rng(seed)
    iu, ju = np.triu_indices(n, 1)
    k = len(iu)
    lat, loss = _edge_attrs(rng, k)
    loops = np.arange(n, dtype=np.int32)
    llat = rng.integers(1, 11, size=n).astype(np.float64)
    _, lloss = _edge_attrs(rng, n)
    return Graph(n=n, src=np.concatenate([iu, loops]).astype(np.int32),
                 dst=np.concatenate([ju, loops]).astype(np.int32),
                 latency=np.concatenate([lat, llat]), packetloss=np.concatenate([loss, lloss]),
                 vertex_packetloss=np.zeros(n), name=name)


def fractional(g: Graph, seed: int = 0, name: Optional[str] = None) -> Graph:
    """The same topology with two-decimal latencies (the format of the reference's own
    resource/topology.graphml.xml.xz, e.g. 2293.85 ms): latency + U{0..99} / 100, each the
    double its decimal text parses to (strtod: the nearest double, here (100 latency + k) /
    100.0, one correctly rounded division; until round 5 the sum latency + k / 100.0, one ulp
    off that for ~0.2% of the arcs).  No integer kernel applies; the fractional path (KF, or
    the generic f64 kernel) does."""
    rng = np.random.default_rng(10_000 + seed)
    lat = (np.rint(g.latency * 100.0) + rng.integers(0, 100, size=g.m)) / 100.0
    return dataclasses.replace(g, latency=lat, name=name or (g.name + "_frac"))


CONFIGS = {
    # name: (builder, kwargs)  -- BASELINE.md section 3
    "c2": lambda vloss=False: internet_like(2000, 5, 1, vloss=vloss, name="c2_ba2k"),
    "c3": lambda vloss=False: internet_like(10000, 4, 2, vloss=vloss, hosts=27000, name="c3_ba10k_tor"),
    "c4": lambda vloss=False: internet_like(50000, 10, 3, exact_edges=500000, vloss=vloss, name="c4_as50k"),
    "c5": lambda vloss=False: complete_graph(4000, 4, name="c5_k4000"),
    # fractional-latency variants of C2 / C3 (no integer kernel applies)
    "c2f": lambda vloss=False: fractional(internet_like(2000, 5, 1, vloss=vloss, name="c2_ba2k"), 1),
    "c3f": lambda vloss=False: fractional(internet_like(10000, 4, 2, vloss=vloss, hosts=27000, name="c3_ba10k_tor"), 2),
    "c4f": lambda vloss=False: fractional(internet_like(50000, 10, 3, exact_edges=500000, vloss=vloss,
                                                        name="c4_as50k"), 3),
}


def config(name: str, **kw) -> Graph:
    return CONFIGS[name](**kw)


def example_one_vertex(vertex_loss: Optional[float] = 0.0, edge_loss: float = 0.01,
                       latency: float = 50.0) -> Graph:
    """resource/examples/shadow.config.xml:2-24 (and the src/test/*.config.xml family):
    one vertex, one self-loop."""
    vl = None if vertex_loss is None else np.array([vertex_loss], np.float64)
    return Graph(n=1, src=np.array([0], np.int32), dst=np.array([0], np.int32),
                 latency=np.array([latency]), packetloss=np.array([edge_loss]),
                 vertex_packetloss=vl, name="example_1v")


# ---------------------------------------------------------------------------
# graphml writer (for loader tests and for feeding the C front end)

def to_graphml(g: Graph, path: str) -> None:
    def f(x):
        return repr(float(x))
    with open(path, "w") as fh:
        fh.write('<?xml version="1.0" encoding="utf-8"?><graphml xmlns="http://graphml.graphdrawing.org/xmlns">\n')
        fh.write('  <key attr.name="packetloss" attr.type="double" for="edge" id="d9" />\n')
        fh.write('  <key attr.name="latency" attr.type="double" for="edge" id="d7" />\n')
        fh.write('  <key attr.name="bandwidthup" attr.type="int" for="node" id="d4" />\n')
        fh.write('  <key attr.name="bandwidthdown" attr.type="int" for="node" id="d3" />\n')
        if g.vertex_packetloss is not None:
            fh.write('  <key attr.name="packetloss" attr.type="double" for="node" id="d0" />\n')
        if g.prefer_direct:
            fh.write('  <key attr.name="preferdirectpaths" attr.type="string" for="graph" id="g0" />\n')
        fh.write('  <graph edgedefault="%s">\n' % ("directed" if g.directed else "undirected"))
        if g.prefer_direct:
            fh.write('    <data key="g0">true</data>\n')
        out = []
        for v in range(g.n):
            vid = _sx.quoteattr(g.vertex_id(v))
            s = f'    <node id={vid}><data key="d3">10240</data><data key="d4">10240</data>'
            if g.vertex_packetloss is not None and not math.isnan(g.vertex_packetloss[v]):
                s += f'<data key="d0">{f(g.vertex_packetloss[v])}</data>'
            out.append(s + "</node>\n")
        fh.write("".join(out))
        out = []
        for e in range(g.m):
            a, b = _sx.quoteattr(g.vertex_id(int(g.src[e]))), _sx.quoteattr(g.vertex_id(int(g.dst[e])))
            out.append(f'    <edge source={a} target={b}><data key="d7">{f(g.latency[e])}</data>'
                       f'<data key="d9">{f(g.packetloss[e])}</data></edge>\n')
            if len(out) > 65536:
                fh.write("".join(out)); out = []
        fh.write("".join(out))
        fh.write("  </graph>\n</graphml>\n")
