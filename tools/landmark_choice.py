#!/usr/bin/env python3
"""Offline (CPU) model of landmark-only plans: the share of vertices a
row improves on its landmark bound D0(v) = min over its k nearest landmarks L of
d(s, L) + d_L(v) (the share that drives phase A), under different landmark sets, with exact
distances from scipy's Dijkstra on the same graph.
  python tools/landmark_choice.py --config c3 --count 512 --samples 200"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--count", type=int, default=512)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--samples", type=int, default=200)
    ap.add_argument("--rules", action="store_true", help="top-degree landmarks under several choice rules")
    a = ap.parse_args()
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra
    from shadow_amd.graph import config
    g = config(a.config)
    n = g.n
    m = g.src != g.dst
    s_, d_, w_ = g.src[m], g.dst[m], g.latency[m]
    A = sp.coo_matrix((np.concatenate([w_, w_]), (np.concatenate([s_, d_]), np.concatenate([d_, s_]))), shape=(n, n)).tocsr()
    A.sum_duplicates()
    deg = np.diff(A.indptr)
    rng = np.random.default_rng(7)
    T = g.targets()
    S = np.sort(rng.choice(T, size=min(a.samples, len(T)), replace=False))
    DS = dijkstra(A, indices=S)
    byd = np.lexsort((np.arange(n), -deg))

    def farthest(k, start):
        sel = list(start)
        dmin = dijkstra(A, indices=sel).min(axis=0) if sel else np.full(n, np.inf)
        while len(sel) < k:
            v = int(np.argmax(np.where(np.isfinite(dmin), dmin, -1)))
            sel.append(v)
            dmin = np.minimum(dmin, dijkstra(A, indices=[v])[0])
        return np.array(sel)

    sets = {
        "top-degree": byd[:a.count],
        "random": rng.choice(n, a.count, replace=False),
        "half degree + half farthest": farthest(a.count, byd[:a.count // 2]),
        "farthest (k-center from the top hub)": farthest(a.count, byd[:1]),
    }
    if a.rules:
        sets = {"top-degree": sets["top-degree"]}
    for name, L in sets.items():
        DL = dijkstra(A, indices=L)  # d_L(v), undirected: d(s, L) = d_L(s)
        closeL = DL[:, byd[:16]].mean(axis=1)  # each landmark's mean distance to the 16 top hubs
        rules = {"nearest": lambda s: DL[:, s]}
        if a.rules:
            rules.update({
                "nearest + 0.25 closeness(L)": lambda s: DL[:, s] + 0.25 * closeL,
                "nearest + 0.375 closeness(L)": lambda s: DL[:, s] + 0.375 * closeL,
                "nearest + 0.5 closeness(L)": lambda s: DL[:, s] + 0.5 * closeL,
                "nearest + 0.625 closeness(L)": lambda s: DL[:, s] + 0.625 * closeL,
                "nearest + 0.75 closeness(L)": lambda s: DL[:, s] + 0.75 * closeL,
                "nearest + 1.0 closeness(L)": lambda s: DL[:, s] + 1.0 * closeL,
                "nearest, one per gateway": None,
                "greedy diverse g=0.375": ("div", 0.375),
                "greedy diverse g=0.625": ("div", 0.625),
                "greedy diverse g=0.75": ("div", 0.75),
                "greedy diverse g=0.5": ("div", 0.5),
                "greedy diverse g=1.0": ("div", 1.0),
            })
        for rname, rule in rules.items():
            shares = []
            for i, s in enumerate(S):
                if isinstance(rule, tuple):
                    # greedy: each next landmark minimises d(s,L) + 0.5 closeness(L) minus gamma x
                    # its distance to the nearest landmark already picked (spread the seeds)
                    gam = rule[1]
                    base = DL[:, s] + 0.5 * closeL
                    near = [int(np.argmin(base))]
                    LL = DL[:, L]  # [landmark, landmark vertex] distances
                    while len(near) < a.k:
                        sep = LL[near][:, np.arange(len(L))].min(axis=0)
                        sc = base - gam * sep
                        sc[near] = np.inf
                        near.append(int(np.argmin(sc)))
                    near = np.array(near)
                elif rule is None:
                    # the nearest landmark to each of s's k lightest neighbours (by w + d to it)
                    ip, ix, dat = A.indptr, A.indices, A.data
                    us, ws = ix[ip[s]:ip[s + 1]], dat[ip[s]:ip[s + 1]]
                    cand = (ws[None, :] + DL[:, us])  # [L, nbr]: via neighbour u to landmark
                    near = []
                    for j in np.argsort(cand.min(axis=0), kind="stable"):
                        for l in np.argsort(cand[:, j], kind="stable"):
                            if l not in near:
                                near.append(int(l))
                                break
                        if len(near) == a.k:
                            break
                    near = np.array(near)
                else:
                    near = np.argsort(rule(s), kind="stable")[:a.k]
                D0 = (DL[near, s][:, None] + DL[near]).min(axis=0)
                shares.append(np.mean(DS[i] < D0))
            print(f"{a.config} {a.count} landmarks, {name:28s} {rname:28s} k={a.k}: improved share "
                  f"{100 * np.mean(shares):.2f}% (p90 {100 * np.quantile(shares, 0.9):.1f}%)", flush=True)


if __name__ == "__main__":
    main()
