import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from shadow_amd import route
from shadow_amd.graph import complete_graph, internet_like
g = complete_graph(200, seed=5) if sys.argv[1] == "k200" else internet_like(700, 2, seed=23)
T = np.arange(g.n, dtype=np.int32)
dev = torch.device("cuda", 0)
d_T = torch.from_numpy(T).to(dev)
res = {}
for mode in ("1", "0"):
    os.environ["SHD_ROUTE_FWREST"] = mode
    eng = route.RouteEngine(g)
    lat = torch.empty((g.n, g.n), dtype=torch.float64, device=dev); rel = torch.empty_like(lat); mn = torch.empty(g.n, dtype=torch.float64, device=dev)
    eng.fw_table_async(); eng.fw_rows_async(d_T, d_T, lat, rel, mn)
    try:
        eng.sync(); print(mode, "ok")
    except Exception as e:
        print(mode, "err", e)
    res[mode] = lat.cpu().numpy()
a, b = res["1"], res["0"]
bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
print("bad", bad.sum())
if bad.any():
    ii, jj = np.nonzero(bad)
    tiles = sorted(set(zip((ii // 64).tolist(), (jj // 64).tolist())))
    print("tiles", tiles[:40])
    print(a[ii[:5], jj[:5]], b[ii[:5], jj[:5]])
