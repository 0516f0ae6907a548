#!/usr/bin/env python3
"""Per-phase cycle breakdown of the K32 kernel from a diagnostic (SHD_STAMPS) build.
Run on the GPU box:  SHD_ROUTE_LIB=shadow_amd/libshd_route_diag.so python tools/stamps.py --config c2"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SHD_ROUTE_LIB", os.path.join(ROOT, "shadow_amd", "libshd_route_diag.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from shadow_amd import route  # noqa: E402
from shadow_amd.graph import config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--sources", type=int, default=0)
ap.add_argument("--plan", action="store_true", help="seeded plan over the sources (rows in source order)")
ap.add_argument("--world", type=int, default=1, help="with --plan: rank --rank of a W-way split")
ap.add_argument("--rank", type=int, default=0)
a = ap.parse_args()
g = config(a.config)
eng = route.RouteEngine(g)
L = route.load_library()
T = g.targets()
S = T if not a.sources else T[: a.sources]
dev = torch.device("cuda", 0)
d_src = torch.from_numpy(S.astype(np.int32)).to(dev)
d_tgt = torch.from_numpy(T.astype(np.int32)).to(dev)
lat = torch.empty((len(S), len(T)), dtype=torch.float64, device=dev)
rel = torch.empty_like(lat)
mn = torch.empty(len(S), dtype=torch.float64, device=dev)
nwg = (len(S) + 7) // 8
dbg = torch.zeros((len(S) + nwg) * 40, dtype=torch.int64, device=dev)
L.shd_route_debug_buffer.argtypes = [C.c_void_p, C.c_void_p]
L.shd_route_debug_buffer(eng._h, C.c_void_p(dbg.data_ptr()))
plan = eng.plan(S, a.world, a.rank) if a.plan else None
if plan is not None and a.world > 1:
    S = plan.sources
    lat = torch.empty((len(S), len(T)), dtype=torch.float64, device=dev)
    rel = torch.empty_like(lat)
    mn = torch.empty(len(S), dtype=torch.float64, device=dev)
for rep in range(3):
    dbg.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    if plan is not None:
        plan.rows_async(d_tgt, lat, rel, mn)
    else:
        eng.rows_async(d_src, d_tgt, lat, rel, mn)
    e1.record()
    eng.sync()
    torch.cuda.synchronize()
print(f"launch time (diag build, last rep): {e0.elapsed_time(e1):.3f} ms")
if plan is not None:
    print("plan", plan.info)
d_all = dbg.cpu().numpy().astype(np.int64).reshape(-1, 40 if eng.info["kernel"] == 4 else 8)
d = d_all[: len(S)]
if eng.info["kernel"] == 2:
    flat = dbg.cpu().numpy().astype(np.int64)
    fused = eng.info["reserved"] == 1
    w = 16 if fused else 8
    kb = flat[len(S) * 8: len(S) * 8 + nwg * w].reshape(nwg, w)
    print(f"config {a.config} n={g.n} nnz={g.nnz} sources={len(S)} kernel=KB{' fused' if fused else '+K2'}")
    print(f"  KB stage+init mean {np.mean(kb[:,1]-kb[:,0]):10.0f} cyc")
    print(f"  KB sweeps  mean {np.mean(kb[:,2]-kb[:,1]):10.0f} cyc  max {np.max(kb[:,2]-kb[:,1])}  rounds mean {kb[:,4].mean():.1f} max {kb[:,4].max():.0f}")
    if fused:
        print(f"  KB parents mean {np.mean(kb[:,5]-kb[:,2]):10.0f} cyc")
        print(f"  KB convert mean {np.mean(kb[:,6]-kb[:,5]):10.0f} cyc")
        print(f"  KB rows    mean {np.mean(kb[:,3]-kb[:,6]):10.0f} cyc  max {np.max(kb[:,3]-kb[:,6])}")
        tr = max(kb[:, 11].mean(), 1)
        print(f"  rows wave0: {tr:.1f} trips, {kb[:,12].mean()/tr:.1f} steps/trip; walk {kb[:,8].mean()/tr:.0f}  fold {kb[:,9].mean()/tr:.0f}  output {kb[:,10].mean()/tr:.0f} cyc/trip")
        t0 = kb[:, 0] - kb[:, 0].min()
        print(f"  total      mean {np.mean(kb[:,3]-kb[:,0]):10.0f} cyc  start spread max {t0.max()}  end max {(kb[:,3]-kb[:,0].min()).max()}")
        sys.exit(0)
    print(f"  KB parents mean {np.mean(kb[:,3]-kb[:,2]):10.0f} cyc")
    print(f"  K2 phaseB  mean {np.mean(d[:,1]-d[:,0]):10.0f} cyc")
    print(f"  K2 sweeps  mean {np.mean(d[:,2]-d[:,1]):10.0f} cyc  sweeps mean {d[:,5].mean():.1f}")
    print(f"  K2 output  mean {np.mean(d[:,3]-d[:,2]):10.0f} cyc")
    t0 = d[:, 0] - d[:, 0].min()
    print(f"  K2 start spread p50 {np.median(t0):.0f} max {t0.max()}")
    sys.exit(0)
if eng.info["kernel"] == 4:
    ph = np.diff(d[:, :5], axis=1)
    print(f"config {a.config} n={g.n} nnz={g.nnz} sources={len(S)} kernel=KD block={eng.info['block']} delta={eng.info['reserved']}")
    for k, nm in enumerate(["A_delta", "B_fixup", "C_lat+par+rel", "D_out"]):
        print(f"  {nm:14s} mean {ph[:, k].mean():10.0f} cyc  p50 {np.median(ph[:, k]):10.0f}  max {ph[:, k].max():10.0f}")
    tot = d[:, 4] - d[:, 0]
    print(f"  total          mean {tot.mean():10.0f} cyc")
    pa = ph[:, 0]
    q = np.percentile(pa, [50, 90, 99, 99.9])
    print(f"  A percentiles p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} p99.9 {q[3]:.0f}; rows > 1M cyc: {(pa > 1e6).sum()}, "
          f"their share of A cycles {pa[pa > 1e6].sum() / max(pa.sum(), 1):.3f}; top rows {np.argsort(pa)[-8:][::-1].tolist()}")
    print(f"  sweeps mean/max        {d[:, 5].mean():.1f} / {d[:, 5].max()}   C sweeps {d[:, 12].mean():.1f}")
    print(f"  queued vertices / n    {d[:, 6].mean() / g.n:.3f}")
    print(f"  arcs expanded / nnz    {d[:, 7].mean() / g.nnz:.3f}")
    print(f"  slices/source {d[:, 20].mean():.0f}  avg slice {d[:, 6].mean() / max(d[:, 20].mean(), 1):.1f} vertices  idle spins/source {d[:, 21].mean():.0f}")
    ns0 = max(d[:, 26].mean(), 1)
    print(f"  wave0 slices {ns0:.0f}: setup {d[:, 22].mean() / ns0:.0f}  groups {d[:, 23].mean() / ns0:.0f} ({d[:, 25].mean() / ns0:.2f} groups/slice)  records {d[:, 24].mean() / ns0:.0f} cyc/slice")
    ng = max(d[:, 25].mean(), 1)
    print(f"  wave0 per group: owners {d[:, 30].mean() / ng:.0f}  owners+loads {d[:, 27].mean() / ng:.0f}  process {d[:, 28].mean() / ng:.0f} (relax {d[:, 29].mean() / ng:.0f}) cyc")
    print(f"  queue overflow/source: pushes to pending {d[:, 14].mean():.0f}  gathered past capacity {d[:, 15].mean():.0f}")
    print(f"  drain of the previous row's stores {d[:, 9].mean():.0f}")
    print(f"  seeded init {d[:, 29].mean():.0f} (seed wait {d[:, 31].mean():.0f}, {100 * d[:, 31].mean() / max(d[:, 29].mean(), 1):.0f}% of it; "
          f"seeds dropped {d[:, 36].mean():.3f}/row)  A' copy {d[:, 27].mean():.0f}  A' events {d[:, 28].mean():.0f} cyc/source")
    for k, nm in [(11, "minreduce"), (8, "gather"), (9, "prep"), (10, "expand"), (16, "B.short"), (17, "B.long"),
                  (18, "lat row+drain"), (19, "par copy"), (13, "C.compute")]:
        print(f"  A.{nm:10s} mean {d[:, k].mean():10.0f} cyc  ({d[:, k].mean() / max(d[:, 5].mean(), 1):.0f}/sweep)")
    print(f"  pre-init: walk (wave 0) {d[:, 32].mean():.0f}  barrier wait {d[:, 33].mean():.0f}  pre-init wave {d[:, 34].mean():.0f} cyc/row; "
          f"rows started pre-initialised {d[:, 35].sum():.0f} of {len(d)}")
    t0 = d[:, 0] - d[:, 0].min()
    print(f"  start spread (cyc): p50 {np.median(t0):.0f} max {t0.max()}  end max {(d[:, 4] - d[:, 0].min()).max()}")
    sys.exit(0)
ph = np.diff(d[:, :5], axis=1)
names = ["A_bf", "B_parent", "C_rel", "D_out"]
print(f"config {a.config} n={g.n} nnz={g.nnz} sources={len(S)} kernel={eng.info['kernel']} block={eng.info['block']}")
for k, nm in enumerate(names):
    print(f"  {nm:10s} mean {ph[:, k].mean():10.0f} cyc  p50 {np.median(ph[:, k]):10.0f}  max {ph[:, k].max():10.0f}")
tot = d[:, 4] - d[:, 0]
print(f"  total      mean {tot.mean():10.0f} cyc")
print(f"  arcs expanded / nnz   {d[:, 5].mean() / g.nnz:.2f}")
print(f"  BF rounds mean/max    {d[:, 6].mean():.1f} / {d[:, 6].max()}")
print(f"  rel sweeps mean/max   {d[:, 7].mean():.1f} / {d[:, 7].max()}")
t0 = d[:, 0] - d[:, 0].min()
print(f"  start spread (cyc): p50 {np.median(t0):.0f} max {t0.max()}  end max {(d[:, 4] - d[:, 0].min()).max()}")
