import os, sys, time
sys.path.insert(0, os.getcwd())
os.environ["SHD_ROUTE_PLAN_DEBUG"] = "1"
import numpy as np, torch
torch.cuda.init()
from shadow_amd.route import RouteEngine
from shadow_amd.graph import config
g = config("c4")
eng = RouteEngine(g)
T = np.sort(g.targets()).astype(np.int32)
for W, r in [(1, 0), (8, 0), (8, 3), (2, 1)]:
    for rep in range(2):
        t0 = time.perf_counter(); p = eng.plan(T, W, r); dt = time.perf_counter() - t0
        print(f"W={W} rank={r} rep={rep} plan {dt*1e3:.1f} ms rows {p.info['rows']}", flush=True)
        p.close()
