#!/usr/bin/env python3
"""Offline (CPU) model of seed quality for multi-GPU plans.

A seeded row s expands only the vertices v whose true distance beats the seeds' bound
D0(v) = min_j w(s,u_j) + d_{u_j}(v) (sssp_delta.hpp, seeded rows); that "improved" share
drives phase A's cost (stamps: ~19 k cycles per percent at C4).  This tool measures the
improved share of sampled rows under several seed sets and partitions, with exact
distances from scipy's Dijkstra on the same graph:

  gateways   the planner's rule on one GPU: the k neighbours of smaller closeness rank
             with the smallest w(s,u) + closeness(u) (k = 1, 2, 3), and landmark seeds
             (the k nearest of L hub rows)
  partition  rank 0 of a W-way split: the engine's seed-forest partition (each row's best
             gateway on its rank, subtrees by LPT), a label-propagation refinement of it over
             the top-3 gateway graph, and a Louvain partition of that graph; rows seeded by
             their 2 best local gateways (then two-hop rows), roots by 2 landmarks

  python tools/seed_locality.py gateways --config c4
  python tools/seed_locality.py partition --config c4 --world 8
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(cfg):
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra
    from shadow_amd.graph import config
    g = config(cfg)
    n = g.n
    m = g.src != g.dst
    a, b, w = g.src[m], g.dst[m], g.latency[m]
    A = sp.coo_matrix((np.concatenate([w, w]), (np.concatenate([a, b]), np.concatenate([b, a]))), shape=(n, n)).tocsr()
    A.sum_duplicates()
    deg = np.diff(A.indptr)
    hubs = np.lexsort((np.arange(n), -deg))[:256]  # the planner's hub rows: degree, then id
    close = dijkstra(A, indices=hubs[:16]).mean(axis=0)  # closeness: mean distance to 16 hubs
    rk = np.empty(n, np.int64)
    rk[np.lexsort((np.arange(n), close))] = np.arange(n)
    return A, n, hubs, close, rk


def topk(A, rk, close, s, avail, k):
    ip, ix, dat = A.indptr, A.indices, A.data
    us, ws = ix[ip[s]:ip[s + 1]], dat[ip[s]:ip[s + 1]]
    sel = rk[us] < rk[s]
    if avail is not None:
        sel &= avail[us]
    us, ws = us[sel], ws[sel]
    o = np.lexsort((us, ws + close[us]))[:k]
    return [(int(u), float(x)) for u, x in zip(us[o], ws[o])]


def improved(D, idx, s, seeds, n):
    if not seeds:
        return 1.0
    D0 = np.min([wu + D[idx[u]] for u, wu in seeds], axis=0)
    return np.count_nonzero(D[idx[s]] < D0) / n


def gateways(a):
    from scipy.sparse.csgraph import dijkstra
    A, n, hubs, close, rk = load(a.config)
    S = np.random.default_rng(0).choice(n, a.samples, replace=False)
    plans = {(s, k): topk(A, rk, close, s, None, k) for s in S for k in (1, 2, 3)}
    need = sorted(set(S.tolist()) | set(hubs.tolist()) | {u for v in plans.values() for u, _ in v})
    D = dijkstra(A, indices=need)
    idx = {v: i for i, v in enumerate(need)}
    for k in (3, 2, 1):
        v = np.array([improved(D, idx, s, plans[(s, k)], n) for s in S])
        print(f"top-{k} gateways: improved mean {v.mean():.4f} p50 {np.median(v):.4f} p90 {np.percentile(v, 90):.4f}")
    # three gateways picked spread apart: each next one minimises w(s,u) + closeness(u) - g x sep,
    # sep = the distance to the nearest picked gateway, exact or its landmark lower bound
    # max_L |d_L(u) - d_L(u')| over the 16 closeness rows (what a planner has)
    H16 = dijkstra(A, indices=hubs[:16])
    ip, ix, dat = A.indptr, A.indices, A.data
    cand = {}
    for s in S:
        us, ws = ix[ip[s]:ip[s + 1]], dat[ip[s]:ip[s + 1]]
        sel = rk[us] < rk[s]
        cand[s] = (us[sel], ws[sel])
    need2 = sorted(set(need) | {int(u) for s in S for u in cand[s][0]})
    if len(need2) > len(need):
        D = dijkstra(A, indices=need2)
        idx = {v: i for i, v in enumerate(need2)}
    for exact in (True, False):
        for gam in (0.25, 0.5, 1.0):
            v = []
            for s in S:
                us, ws = cand[s]
                if len(us) == 0:
                    v.append(1.0)
                    continue
                base = ws + close[us]
                picked = []
                for _ in range(3):
                    if len(picked) == len(us):
                        break
                    sc = base.copy()
                    if picked:
                        if exact:
                            sep = np.min([D[idx[int(us[p])]][us] for p in picked], axis=0)
                        else:
                            sep = np.min([np.abs(H16[:, us] - H16[:, [us[p]]]).max(axis=0) for p in picked], axis=0)
                        sc = sc - gam * sep
                    sc[picked] = np.inf
                    picked.append(int(np.argmin(sc)))
                v.append(improved(D, idx, s, [(int(us[p]), float(ws[p])) for p in picked], n))
            print(f"3 gateways spread ({'exact' if exact else 'landmark bound'} separation, g={gam}): "
                  f"improved mean {np.mean(v):.4f} p50 {np.median(v):.4f}")
    # two gateways + a landmark spread from them (engine lm_pick rule) as the third seed
    for nl in (16, 256, 1024):
        Lh = hubs[:nl] if nl <= len(hubs) else np.lexsort((np.arange(n), -np.diff(A.indptr)))[:nl]
        DLm = dijkstra(A, indices=Lh)
        bias = 0.5 * DLm[:, Lh[:16]].mean(axis=1)
        v = []
        for s in S:
            sd = plans[(s, 2)]
            sc = DLm[:, s] + bias
            if sd:
                sc = sc - 0.5 * np.min(DLm[:, [u for u, _ in sd]], axis=1)
            q = int(np.argmin(sc))
            seeds = sd + [(int(Lh[q]), float(DLm[q, s]))]
            D0 = np.min([wu + (D[idx[u]] if u in idx else DLm[list(Lh).index(u)]) for u, wu in seeds], axis=0)
            v.append(np.count_nonzero(D[idx[s]] < D0) / n)
        print(f"top-2 gateways + spread landmark of {nl}: improved mean {np.mean(v):.4f} p50 {np.median(v):.4f}")
    for L in (16, 64, 256):
        for k in (1, 2, 3):
            v = []
            for s in S:
                dsl = np.array([D[idx[int(h)]][s] for h in hubs[:L]])
                o = np.argsort(dsl)[:k]
                v.append(improved(D, idx, s, [(int(hubs[q]), dsl[q]) for q in o], n))
            print(f"landmarks L={L} k={k}: improved mean {np.mean(v):.4f} p50 {np.median(v):.4f}")


def forest_owner(A, n, rk, close, W):
    gw = np.array([([u for u, _ in topk(A, rk, close, s, None, 3)] + [-1, -1, -1])[:3] for s in range(n)])
    pos = np.argsort(rk)
    bu = gw[:, 0]
    sub = np.ones(n, np.int64)
    for s in pos[::-1]:
        if bu[s] >= 0:
            sub[bu[s]] += sub[s]
    cap = max(1, n // (4 * W))
    top = [s for s in pos if sub[s] > cap]
    heads = sorted([s for s in pos if sub[s] <= cap and (bu[s] < 0 or sub[bu[s]] > cap)], key=lambda s: -sub[s])
    owner = np.full(n, -1)
    load_ = np.zeros(W)
    for h in heads:
        r = int(np.argmin(load_)); owner[h] = r; load_[r] += sub[h]
    for p in top:
        r = int(np.argmin(load_)); owner[p] = r; load_[r] += 1
    for s in pos:
        if owner[s] < 0 and bu[s] >= 0:
            owner[s] = owner[bu[s]]
    topset = np.zeros(n, bool)
    topset[top] = True
    return owner, topset, gw


def lp_refine(owner, gw, n, W, passes=6, slack=0.01):
    import scipy.sparse as sp
    wt = np.array([4.0, 2.0, 1.0])
    rows, cols, vals = [], [], []
    for k in range(3):
        sel = gw[:, k] >= 0
        s, u = np.where(sel)[0], gw[sel, k]
        rows += [s, u]; cols += [u, s]; vals += [np.full(len(s), wt[k])] * 2
    G = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n)).tocsr()
    owner = owner.copy()
    rng = np.random.default_rng(0)
    hi = n / W * (1 + slack)
    for _ in range(passes):
        load_ = np.bincount(owner, minlength=W).astype(float)
        moved = 0
        for v in rng.permutation(n):
            nb, ww = G.indices[G.indptr[v]:G.indptr[v + 1]], G.data[G.indptr[v]:G.indptr[v + 1]]
            gain = np.bincount(owner[nb], weights=ww, minlength=W)
            cur = owner[v]
            best = int(np.argmax(gain - 1e9 * (load_ + 1 > hi) * (np.arange(W) != cur)))
            if best != cur and gain[best] > gain[cur]:
                owner[v] = best; load_[cur] -= 1; load_[best] += 1; moved += 1
        if not moved:
            break
    return owner


def eval_rank(A, n, hubs, close, rk, owner, topset, label, samples):
    from scipy.sparse.csgraph import dijkstra
    ip, ix, dat = A.indptr, A.indices, A.data
    avail = (owner == 0) | topset
    rows = np.where(owner == 0)[0]
    jobs = np.where(avail)[0]
    roots = set(jobs[np.argsort(rk[jobs])][:256].tolist())
    samp = np.random.default_rng(1).choice(rows, samples, replace=False)
    plans = {}
    for s in samp:
        if s in roots:
            plans[s] = None
            continue
        sd = topk(A, rk, close, s, avail, 2)
        if len(sd) < 2:  # two-hop rows s -> x -> u (deg x <= 256), as the planner
            best = []
            for x, wx in zip(ix[ip[s]:ip[s + 1]], dat[ip[s]:ip[s + 1]]):
                if ip[x + 1] - ip[x] > 256:
                    continue
                for u, wu in zip(ix[ip[x]:ip[x + 1]], dat[ip[x]:ip[x + 1]]):
                    if u != s and u != x and rk[u] < rk[s] and avail[u] and all(u != q for q, _ in sd):
                        best.append((wx + wu + close[u], int(u), wx + wu))
            best.sort()
            seen = set()
            for _, u, off in best:
                if len(sd) >= 2:
                    break
                if u not in seen:
                    seen.add(u); sd.append((u, off))
        plans[s] = sd
    nl = getattr(eval_rank, "landmarks", 0)
    mode = getattr(eval_rank, "lmmode", "nearest-weak")
    if nl:  # rows also take a landmark seed: nearest, or spread from their seeds (engine lm_pick)
        from scipy.sparse.csgraph import dijkstra as _dj
        L = np.lexsort((np.arange(n), -np.diff(A.indptr)))[:nl]
        DL = _dj(A, indices=L)
        bias = 0.5 * DL[:, L[:16]].mean(axis=1)
        direct = {s: sum(1 for u, _ in (plans[s] or []) if A[s, u] != 0) for s in samp}
        for s in samp:
            if plans[s] is None or (mode.endswith("weak") and direct[s] > 1):
                continue
            if mode.startswith("nearest"):
                q = int(np.argmin(DL[:, s]))
            else:
                sc = DL[:, s] + bias
                if plans[s]:
                    sc = sc - 0.5 * np.min(DL[:, [u for u, _ in plans[s]]], axis=1)
                q = int(np.argmin(sc))
            plans[s] = plans[s] + [(int(L[q]), float(DL[q, s]))]
    need = sorted(set(samp.tolist()) | set(hubs[:16].tolist()) | {u for v in plans.values() if v for u, _ in v})
    D = dijkstra(A, indices=need)
    idx = {v: i for i, v in enumerate(need)}
    v = []
    for s in samp:
        if plans[s] is None:
            dsl = np.array([D[idx[int(h)]][s] for h in hubs[:16]])
            o = np.argsort(dsl)[:2]
            v.append(improved(D, idx, s, [(int(hubs[q]), dsl[q]) for q in o], n))
        else:
            v.append(improved(D, idx, s, plans[s], n))
    v = np.array(v)
    print(f"{label}: rank 0 improved mean {v.mean():.4f} p50 {np.median(v):.4f} (sample {len(samp)}, "
          f"{sum(plans[s] is None for s in samp)} roots)", flush=True)


def partition(a):
    A, n, hubs, close, rk = load(a.config)
    W = a.world
    t0 = time.time()
    owner, topset, gw = forest_owner(A, n, rk, close, W)

    def loc(o):
        return [float(np.mean(o[gw[gw[:, k] >= 0, k]] == o[gw[:, k] >= 0])) for k in range(3)]
    print(f"forest partition ({time.time() - t0:.1f} s): gateway k=1,2,3 on the row's rank: "
          + ", ".join(f"{x:.3f}" for x in loc(owner)), flush=True)
    eval_rank(A, n, hubs, close, rk, owner, topset, "forest", a.samples)
    ref = lp_refine(owner, gw, n, W)
    print("label-propagation refinement: gateway k=1,2,3 local: " + ", ".join(f"{x:.3f}" for x in loc(ref)), flush=True)
    eval_rank(A, n, hubs, close, rk, ref, np.zeros(n, bool), "forest + LP refinement", a.samples)
    if a.louvain:
        import networkx as nx
        G = nx.Graph()
        G.add_nodes_from(range(n))
        for s in range(n):
            for q, u in enumerate(gw[s]):
                if u >= 0:
                    G.add_edge(s, int(u), weight=float(3 - q))
        comms = sorted(nx.community.louvain_communities(G, weight="weight", seed=1), key=len, reverse=True)
        lo = np.full(n, -1)
        load_ = np.zeros(W)
        cap = n / W
        for c in comms:
            c = sorted(c, key=lambda v: rk[v])
            while c:
                r = int(np.argmin(load_))
                take = c[:max(1, int(min(len(c), cap - load_[r])))]
                lo[take] = r; load_[r] += len(take); c = c[len(take):]
        cut = np.mean([lo[u] != lo[v] for u, v in G.edges()])
        print(f"Louvain ({len(comms)} communities, binned): gateway-graph cut {cut:.3f}; gateway k=1,2,3 local: "
              + ", ".join(f"{x:.3f}" for x in loc(lo)), flush=True)
        eval_rank(A, n, hubs, close, rk, lo, np.zeros(n, bool), "Louvain", a.samples)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["gateways", "partition"])
    ap.add_argument("--config", default="c4")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--samples", type=int, default=150)
    ap.add_argument("--louvain", action="store_true")
    ap.add_argument("--landmarks", type=int, default=0, help="partition: rows with <= 1 direct gateway add their nearest of L hub rows")
    ap.add_argument("--lmmode", default="nearest-weak", choices=["nearest-weak", "spread-weak", "spread-all", "nearest-all"])
    a = ap.parse_args()
    eval_rank.landmarks = a.landmarks
    eval_rank.lmmode = a.lmmode
    gateways(a) if a.mode == "gateways" else partition(a)
