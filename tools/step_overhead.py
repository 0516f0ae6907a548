"""Step-time overhead probe (GPU box): C2 rows + runahead min per step, timed as
(a) bench.py does (HIP events around the rows kernel every step), (b) without per-step
events, (c) replaying a captured HIP graph of the step."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd.graph import config  # noqa: E402
from shadow_amd.route import RouteEngine  # noqa: E402

g = config("c2")
eng = RouteEngine(g)
dev = torch.device("cuda", 0)
T = g.targets()
d_src = torch.from_numpy(T.astype(np.int32)).to(dev)
d_tgt = d_src.clone()
ns = nt = len(T)
d_lat = torch.empty((ns, nt), dtype=torch.float64, device=dev)
d_rel = torch.empty_like(d_lat)
d_rmin = torch.empty(ns, dtype=torch.float64, device=dev)
d_min = torch.empty(1, dtype=torch.float64, device=dev)
K = 50


def run(stream, events):
    sh = stream.cuda_stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for _ in range(5):
        eng.rows_async(d_src, d_tgt, d_lat, d_rel, d_rmin, stream=sh)
        eng.min_reduce_async(d_rmin, d_min, stream=sh)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        if events:
            ev[k][0].record(stream)
        eng.rows_async(d_src, d_tgt, d_lat, d_rel, d_rmin, stream=sh)
        if events:
            ev[k][1].record(stream)
        eng.min_reduce_async(d_rmin, d_min, stream=sh)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e3
    km = np.mean([a.elapsed_time(b) for a, b in ev]) if events else float("nan")
    return dt, km


s = torch.cuda.current_stream()
print("events      ms/step %.4f kernel %.4f" % run(s, True), flush=True)
print("no events   ms/step %.4f" % run(s, False)[0], flush=True)
side = torch.cuda.Stream()
print("side stream ms/step %.4f kernel %.4f" % run(side, True), flush=True)
# graph of one step
cs = torch.cuda.Stream()
graph = torch.cuda.CUDAGraph()
torch.cuda.synchronize()
with torch.cuda.graph(graph, stream=cs):
    eng.rows_async(d_src, d_tgt, d_lat, d_rel, d_rmin, stream=cs.cuda_stream)
    eng.min_reduce_async(d_rmin, d_min, stream=cs.cuda_stream)
for _ in range(5):
    graph.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    graph.replay()
torch.cuda.synchronize()
print("graph       ms/step %.4f" % ((time.perf_counter() - t0) / K * 1e3), flush=True)
lat = d_lat.cpu().numpy()
print("graph rows finite:", bool(np.isfinite(lat).all()))
