import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
os.environ["SHD_ROUTE_KERNEL"] = "k16"
from shadow_amd.graph import internet_like, config
from shadow_amd.route import RouteEngine, RouteError
from oracle.oracle import OracleGraph, TIE_MINKEY
for g in [internet_like(100, 2, seed=1), internet_like(1000, 3, seed=2), config("c2")]:
    eng = RouteEngine(g)
    print("n", g.n, "kernel", eng.info["kernel"], "bound", eng.info["dist_bound"], flush=True)
    T = g.targets(); S = T[:5]
    try:
        lat, rel, mn = eng.rows(S, T, dispatch=False)
    except RouteError as e:
        print("ERR", e); continue
    og = OracleGraph(g)
    ol, orl, _, _ = og.source_rows(S, T, TIE_MINKEY)
    bad = np.argwhere(lat != ol)
    print("lat mismatches", len(bad), bad[:5], lat[tuple(bad[0])] if len(bad) else None, ol[tuple(bad[0])] if len(bad) else None)
    badr = np.argwhere(rel != orl)
    print("rel mismatches", len(badr), badr[:5], rel[tuple(badr[0])] if len(badr) else None, orl[tuple(badr[0])] if len(badr) else None)
