#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ (run in the dev container,
where /root/reference exists; the GPU box only reads the committed outputs).

Fixtures are DATA: inputs and expected outputs.
  ref_kat.json            every 1-vertex topology embedded in the reference's own test
                          and example configs (src/test/**/*.config.xml,
                          resource/examples/shadow.config.xml) with the Path the
                          reference caches for (0,0) (complete -> direct,
                          topology.c:1877-1927) and the runahead (master.c:153)
  bundled_topology.npz    resource/topology.graphml.xml.xz as igraph numbers it
                          (document order), plus expected direct-mode digests
  small_tables.npz        oracle eager tables (igraph tie rule) for small synthetic
                          graphs in every routing mode, latency cross-checked against
                          networkx at generation time
  rows_digests.json       per-row SHA-256 of the C2 latency/reliability rows (engine tie
                          rule) and the row minima; c3/c4 sampled rows likewise; every
                          row pinned by networkx at generation time (nx_pin.py: latency
                          on every pair, rel along networkx's path on unique pairs), the
                          counts in stats
"""
from __future__ import annotations

import glob
import hashlib
import json
import lzma
import math
import os
import sys
import xml.etree.ElementTree as ET

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from shadow_amd.graph import Graph, complete_graph, config, internet_like  # noqa: E402
from oracle import oracle as O  # noqa: E402

REF = "/root/reference"
NS = "{http://graphml.graphdrawing.org/xmlns}"


def parse_graphml_text(text: str) -> Graph:
    """igraph_read_graphml semantics for the attributes Shadow reads: vertices/edges in
    document order, missing numeric attribute = NaN."""
    root = ET.fromstring(text.strip().encode())
    def tag(e):
        return e.tag.replace(NS, "")
    keys = {}
    for k in root:
        if tag(k) == "key":
            keys[k.get("id")] = (k.get("for"), k.get("attr.name"), k.get("attr.type"))
    graph = [c for c in root if tag(c) == "graph"][0]
    directed = graph.get("edgedefault", "directed") == "directed"
    ids, vidx, vloss = [], {}, []
    has_vloss = any(f == "node" and nm == "packetloss" for f, nm, _ in keys.values())
    gattr = {}
    for c in graph:
        if tag(c) == "data":
            gattr[keys[c.get("key")][1]] = c.text
    for c in graph:
        if tag(c) == "node":
            vidx[c.get("id")] = len(ids)
            ids.append(c.get("id"))
            p = math.nan
            for d in c:
                f, nm, _ = keys[d.get("key")]
                if nm == "packetloss" and f == "node":
                    p = float(d.text)
            vloss.append(p)
    src, dst, lat, loss = [], [], [], []
    for c in graph:
        if tag(c) == "edge":
            src.append(vidx[c.get("source")]); dst.append(vidx[c.get("target")])
            L = P = math.nan
            for d in c:
                f, nm, _ = keys[d.get("key")]
                if f == "edge" and nm == "latency":
                    L = float(d.text)
                if f == "edge" and nm == "packetloss":
                    P = float(d.text)
            lat.append(L); loss.append(P)
    pd = str(gattr.get("preferdirectpaths", "")).lower()
    return Graph(n=len(ids), src=np.array(src, np.int32), dst=np.array(dst, np.int32),
                 latency=np.array(lat), packetloss=np.array(loss),
                 vertex_packetloss=np.array(vloss) if has_vloss else None,
                 directed=directed, prefer_direct=pd.startswith(("true", "yes", "1")), ids=ids)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, np.float64).tobytes()).hexdigest()


def _embedded_graphml(f):
    """The graphml a reference file embeds: a config's CDATA block, the first xml block of
    a markdown doc, or the CDATA block inside a C string literal (escaped quotes, backslash
    line continuations)."""
    text = open(f).read()
    if f.endswith(".md"):
        i = text.find("<graphml")
        j = text.find("</graphml>", i)
        return None if i < 0 or j < 0 else text[text.rfind("<?xml", 0, i):j + len("</graphml>")]
    if f.endswith(".c"):
        text = text.replace("\\\n", "\n").replace('\\"', '"')
    i = text.find("<![CDATA[")
    if i < 0:
        return None
    return text[i + 9:text.find("]]>", i)]


def ref_kats():
    out = []
    files = sorted(glob.glob(f"{REF}/src/test/**/*.config.xml", recursive=True))
    files += [f"{REF}/resource/examples/shadow.config.xml",
              f"{REF}/docs/3.2-Network-Config.md",           # the documented example topology
              f"{REF}/src/main/core/support/examples.c"]     # example_getTestContents()
    for f in files:
        xml = _embedded_graphml(f)
        if xml is None:
            continue
        g = parse_graphml_text(xml)
        og = O.OracleGraph(g)
        complete = og.is_complete()
        lat, rel = og.direct(0, 0) if complete else (None, None)
        out.append(dict(config=os.path.relpath(f, REF), n=g.n, m=g.m, directed=g.directed,
                        edge_latency=g.latency.tolist(), edge_packetloss=g.packetloss.tolist(),
                        vertex_packetloss=None if g.vertex_packetloss is None else
                        [None if math.isnan(x) else x for x in g.vertex_packetloss],
                        complete=complete, lat=lat, rel=rel, runahead_ns=O.runahead_ns(lat)))
    return out


def bundled():
    text = lzma.open(f"{REF}/resource/topology.graphml.xml.xz").read().decode()
    g = parse_graphml_text(text)
    og = O.OracleGraph(g)
    A = np.arange(g.n, dtype=np.int32)
    tab = og.eager_table(A)
    exp = dict(complete=og.is_complete(), min_latency=tab["min_latency"],
               runahead_ns=O.runahead_ns(tab["min_latency"]),
               lat_sha=sha(tab["lat"]), rel_sha=sha(tab["rel"]),
               all_direct=bool(tab["is_direct"].all()))
    np.savez_compressed(os.path.join(HERE, "bundled_topology.npz"), n=g.n, src=g.src, dst=g.dst,
                        latency=g.latency, packetloss=g.packetloss,
                        vertex_packetloss=g.vertex_packetloss, ids=np.array(g.ids),
                        directed=g.directed)
    return exp


SMALL = [
    # name, builder
    ("ba60", lambda: internet_like(60, 2, seed=101)),
    ("ba120_vloss", lambda: internet_like(120, 3, seed=102, vloss=True)),
    ("ba80_prefer", lambda: internet_like(80, 2, seed=103, prefer_direct=True)),
    ("k24", lambda: complete_graph(24, seed=104)),
    ("ba100_attached", lambda: internet_like(100, 2, seed=105, hosts=60)),
    ("ba64_ties", lambda: _ties(64, 106)),
    ("dir40", lambda: _directed(40, 107)),
    ("ba90_frac", lambda: _fractional(90, 108)),
]


def _ties(n, seed):
    g = internet_like(n, 3, seed=seed)
    rng = np.random.default_rng(seed)
    g.latency = np.where(g.src != g.dst, rng.integers(1, 4, size=g.m), g.latency).astype(np.float64)
    g.name = "ties"
    return g


def _fractional(n, seed):
    g = internet_like(n, 2, seed=seed)
    rng = np.random.default_rng(seed)
    g.latency = np.round(rng.uniform(0.5, 300.0, size=g.m), 3)
    return g


def _directed(n, seed):
    """Strongly connected directed graph: a ring both ways plus random chords, self-loops."""
    rng = np.random.default_rng(seed)
    e = [(i, (i + 1) % n) for i in range(n)] + [((i + 1) % n, i) for i in range(0, n, 2)]
    have = set(e)
    while len(e) < 4 * n:
        a, b = (int(x) for x in rng.integers(0, n, 2))
        if a != b and (a, b) not in have:
            have.add((a, b)); e.append((a, b))
    e = np.array(e, np.int32)
    k = len(e)
    lat = rng.integers(1, 100, size=k).astype(np.float64)
    loss = np.where(rng.random(k) < 0.5, 0.0, rng.integers(1, 100, size=k) * 1e-4)
    loops = np.arange(n, dtype=np.int32)
    return Graph(n=n, src=np.concatenate([e[:, 0], loops]), dst=np.concatenate([e[:, 1], loops]),
                 latency=np.concatenate([lat, rng.integers(1, 5, size=n).astype(np.float64)]),
                 packetloss=np.concatenate([loss, np.zeros(n)]), vertex_packetloss=np.zeros(n),
                 directed=True, name="dir")


def small_tables():
    import networkx as nx
    blobs = {}
    for name, mk in SMALL:
        g = mk()
        og = O.OracleGraph(g)
        A = g.targets()
        tab = og.eager_table(A, prefer_direct=g.prefer_direct)
        raw_lat, raw_rel, raw_uq, _ = og.source_rows(A, A)
        # networkx cross-check (latency, non-complete, non-direct pairs)
        if not og.is_complete():
            G = nx.DiGraph() if g.directed else nx.Graph()
            for a, b, w in zip(g.src, g.dst, g.latency):
                if a != b:
                    G.add_edge(int(a), int(b), weight=float(w))
            for i, s in enumerate(A):
                d = nx.single_source_dijkstra_path_length(G, int(s))
                ref = np.array([d[int(t)] for t in A])
                mask = A != s
                assert np.array_equal(ref[mask], raw_lat[i][mask]), name
        p = f"{name}__"
        blobs.update({p + "n": g.n, p + "src": g.src, p + "dst": g.dst, p + "latency": g.latency,
                      p + "packetloss": g.packetloss,
                      p + "vertex_packetloss": g.vertex_packetloss if g.vertex_packetloss is not None
                      else np.array([]), p + "directed": g.directed, p + "prefer_direct": g.prefer_direct,
                      p + "attached": A, p + "lat": tab["lat"], p + "rel": tab["rel"],
                      p + "is_direct": tab["is_direct"], p + "unique": tab["unique"],
                      p + "min_latency": tab["min_latency"], p + "raw_lat": raw_lat, p + "raw_rel": raw_rel,
                      p + "raw_unique": raw_uq})
    np.savez_compressed(os.path.join(HERE, "small_tables.npz"), names=np.array([s for s, _ in SMALL]), **blobs)


def row_digests():
    from tests.golden.nx_pin import nx_graph, pin_row
    out = {}
    for cfg, picks in (("c2", None), ("c3", 48), ("c4", 12)):
        g = config(cfg)
        og = O.OracleGraph(g)
        G = nx_graph(g)
        T = g.targets()
        if picks is None:
            S = T
        else:
            S = T[np.linspace(0, len(T) - 1, num=picks).astype(int)]
        rows = []
        stats = dict(pairs=0, unique=0, rel_diff_on_ties=0, nx_latency_pairs_equal=0, nx_unique_rel_pairs_equal=0)
        for s in S:
            lat, rel, uq, hops = og.source_row(int(s), T, O.TIE_MINKEY)
            ilat, irel, iuq, _ = og.source_row(int(s), T, O.TIE_IGRAPH)
            assert np.array_equal(lat, ilat)
            # independent pin: networkx latency (every t != s) and rel along its path on
            # unique-shortest-path pairs; any mismatch stops the generator
            nl, nr = pin_row(G, g, int(s), T, lat, rel, uq)
            stats["nx_latency_pairs_equal"] += nl; stats["nx_unique_rel_pairs_equal"] += nr
            stats["pairs"] += len(T); stats["unique"] += int(uq.sum())
            stats["rel_diff_on_ties"] += int((rel != irel).sum())
            rows.append(dict(src=int(s), lat_sha=sha(lat), rel_sha=sha(rel), row_min=float(lat.min()),
                             max_hops=int(hops.max()), sample=[[int(T[j]), float(lat[j]), float(rel[j]),
                                                                bool(uq[j])] for j in range(0, len(T), max(1, len(T) // 16))]))
        out[cfg] = dict(n=g.n, m=g.m, targets=len(T), rows=rows, stats=stats)
        print(cfg, stats, flush=True)
    json.dump(out, open(os.path.join(HERE, "rows_digests.json"), "w"))


if __name__ == "__main__":
    O.build()
    if "--rows-only" not in sys.argv:
        json.dump(ref_kats(), open(os.path.join(HERE, "ref_kat.json"), "w"), indent=1)
        json.dump(bundled(), open(os.path.join(HERE, "bundled_expected.json"), "w"), indent=1)
        small_tables()
    if "--no-rows" not in sys.argv:
        row_digests()
