#!/usr/bin/env python3
"""Offline (CPU) measure of the round-3 "seed rel row reuse" idea: a seeded
row s whose seed arc (s,u) is lossless (r = 1.0, no vertex factors) could copy rel_u(t)
from u's finished output row for every target t whose tree path from s is s -> u -> (u's
tree path to t): the products are then the same left folds (1.0 * x == x).  For sampled
rows, with exact trees from the oracle (engine tie rule), this reports the share of rows
whose primary seed qualifies and the share of targets below u in s's tree, and checks that
rel_s(t) == rel_u(t) bit-exactly on those targets.

  python tools/rel_reuse.py --config c4 --samples 100
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--samples", type=int, default=100)
a = ap.parse_args()

from seed_locality import load, topk  # noqa: E402
from shadow_amd.graph import config  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (test infrastructure: the checker, offline only)

g = config(a.config)
A, n, hubs, close, rk = load(a.config)
og = orc.OracleGraph(g)
loss = {}
for x, y, pl in zip(g.src, g.dst, g.packetloss):
    loss[(int(x), int(y))] = min(loss.get((int(x), int(y)), 1.0), float(pl))
    loss[(int(y), int(x))] = loss[(int(x), int(y))]
S = np.random.default_rng(3).choice(n, a.samples, replace=False)
T = np.arange(n, dtype=np.int32)
qual, below, checked, mism = 0, [], 0, 0
for s in S:
    sd = topk(A, rk, close, int(s), None, 1)
    if not sd:
        continue
    u = sd[0][0]
    if loss.get((int(s), u), 1.0) != 0.0:
        continue
    dist, pe = og.dijkstra(int(s), orc.TIE_MINKEY)  # (parent edge ids)
    ok = pe >= 0
    par = np.full(n, -1, np.int64)
    e = pe[ok]
    vv = np.nonzero(ok)[0]
    par[ok] = np.where(g.dst[e] == vv, g.src[e], g.dst[e])
    if par[u] != s:
        continue
    qual += 1
    order = np.argsort(dist, kind="stable")
    anc = np.zeros(n, bool)
    anc[u] = True
    for v in order:
        if v != u and v != s and par[v] >= 0 and anc[par[v]]:
            anc[v] = True
    below.append(anc.mean())
    if checked < 10:
        _, rs_, _, _ = og.source_row(int(s), T, orc.TIE_MINKEY)
        _, ru_, _, _ = og.source_row(int(u), T, orc.TIE_MINKEY)
        mism += int(np.count_nonzero(rs_[anc] != ru_[anc]))
        checked += 1
b = np.array(below) if below else np.zeros(1)
print(f"{a.config}: {len(S)} sampled rows; primary seed lossless with parent(u) = s: {qual} ({qual / len(S):.1%}); "
      f"targets below u in s's tree: mean {b.mean():.1%} p50 {np.median(b):.1%}; reusable share of all pairs "
      f"{qual / len(S) * b.mean():.1%}; rel_s == rel_u bit-exact on those targets in {checked} checked rows: "
      f"{'yes' if mism == 0 else f'no ({mism} differ)'}")
