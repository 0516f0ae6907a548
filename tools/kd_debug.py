import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SHD_ROUTE_KERNEL"] = "kd"
import numpy as np
from shadow_amd import route
from shadow_amd.graph import internet_like, config
from oracle.oracle import OracleGraph, TIE_MINKEY
for name, g in [("ba400", internet_like(400, 4, seed=31, name="ba400")), ("c2", config("c2"))]:
    eng = route.RouteEngine(g)
    T = g.targets(); S = T[:8]
    L = route.load_library()
    t0 = time.time()
    try:
        lat, rel, mn = eng.rows(S, T, dispatch=False)
        og = OracleGraph(g); olat, orel, _, _ = og.source_rows(S, T, TIE_MINKEY)
        print(name, "ok", time.time() - t0, np.array_equal(lat, olat), np.array_equal(rel, orel), flush=True)
    except Exception as e:
        print(name, "ERR", e, time.time() - t0, flush=True)
