"""Independent pins of SOURCE rows by networkx (test infrastructure).

igraph, where the reference's Dijkstra lives, is absent here, so the
multi-vertex goldens come from the CPU restatement (oracle/).  networkx is an
independent implementation of the same two things the rows carry:
  * latency: single_source_dijkstra_path_length.  Every relaxation-based SSSP reaches
    the same left-fold minimum (fl(a + w) is monotone in a), so the row must equal
    networkx's bit for bit on every t != s (the (s,s) entry is the self-loop hop);
  * reliability on unique-shortest-path pairs: networkx's path is then THE path, and
    Shadow's product along it (topology.c:1430-1499: rel = 1.0, times f_s if present,
    times f_t if present and t != s, then r_e = 1 - loss_e hop by hop from the source,
    topology.c:437) must equal the row's entry bit for bit.
"""
from __future__ import annotations

import math

import numpy as np


def nx_graph(g):
    import networkx as nx
    G = nx.DiGraph() if g.directed else nx.Graph()
    G.add_nodes_from(range(g.n))
    for e, (a, b, w) in enumerate(zip(g.src, g.dst, g.latency)):
        if a != b:
            G.add_edge(int(a), int(b), weight=float(w), r=1.0 - float(g.packetloss[e]))
    return G


def pin_row(G, g, s, targets, lat, rel, unique):
    """Check one row against networkx; returns (latency pairs, unique-pair rel checks).
    Raises AssertionError on any mismatch."""
    import networkx as nx
    dist, paths = nx.single_source_dijkstra(G, int(s), weight="weight")
    vf = g.vertex_packetloss
    fs = None if vf is None or math.isnan(vf[s]) else 1.0 - float(vf[s])
    n_lat = n_rel = 0
    for j, t in enumerate(targets):
        t = int(t)
        if t == s:
            continue
        assert dist[t] == lat[j], (s, t, dist[t], lat[j])
        n_lat += 1
        if not unique[j]:
            continue
        P = paths[t]
        r = 1.0
        if fs is not None:
            r *= fs
        if vf is not None and not math.isnan(vf[t]):
            r *= 1.0 - float(vf[t])
        for a, b in zip(P[:-1], P[1:]):
            r *= G[a][b]["r"]
        assert r == rel[j], (s, t, r, rel[j])
        n_rel += 1
    return n_lat, n_rel
