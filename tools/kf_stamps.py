#!/usr/bin/env python3
"""Per-phase cycles of KF (sssp_f64d_kernel) rows from the diagnostic (SHD_STAMPS) build:
SHD_ROUTE_LIB=shadow_amd/libshd_route_diag.so python tools/kf_stamps.py --config c3f"""
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
ap.add_argument("--config", default="c3f")
ap.add_argument("--sources", type=int, default=0)
a = ap.parse_args()
g = config(a.config)
eng = route.RouteEngine(g)
assert eng.info["kernel"] == 5, eng.info
L = route.load_library()
T = g.targets()
S = T if not a.sources else T[: a.sources]
dev = torch.device("cuda", 0)
d_src = torch.from_numpy(S.astype(np.int32)).to(dev)
d_tgt = torch.from_numpy(T.astype(np.int32)).to(dev)
lat = torch.empty((len(S), len(T)), dtype=torch.float64, device=dev)
rel = torch.empty_like(lat)
mn = torch.empty(len(S), dtype=torch.float64, device=dev)
dbg = torch.zeros(len(S) * 16, dtype=torch.int64, device=dev)
L.shd_route_debug_buffer.argtypes = [C.c_void_p, C.c_void_p]
L.shd_route_debug_buffer(eng._h, C.c_void_p(dbg.data_ptr()))
for rep in range(2):
    dbg.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.rows_async(d_src, d_tgt, lat, rel, mn)
    e1.record()
    eng.sync()
    torch.cuda.synchronize()
print(f"{a.config}: n={g.n} sources={len(S)} block={eng.info['block']} launch {e0.elapsed_time(e1):.3f} ms")
d = dbg.cpu().numpy().astype(np.int64).reshape(-1, 16)
ph = np.diff(d[:, :6], axis=1)
for k, nm in enumerate(["A delta-stepping", "B parents", "C lat row", "C level passes", "D rel row + min"]):
    print(f"  {nm:18s} mean {ph[:, k].mean():10.0f} cyc  p50 {np.median(ph[:, k]):10.0f}  max {ph[:, k].max():10.0f}")
print(f"  A: gathers {d[:, 10].mean():.1f} ({d[:, 8].mean():.0f} cyc), rounds {d[:, 6].mean():.1f} (expansion {d[:, 9].mean():.0f} cyc, "
      f"{d[:, 9].mean() / max(d[:, 6].mean(), 1):.0f}/round)")
ns_ = max(d[:, 11].mean(), 1)
print(f"  wave 0: {ns_:.1f} slices/row; per slice: setup {d[:, 12].mean() / ns_:.0f}, owners {d[:, 13].mean() / ns_:.0f}, "
      f"arc loads {d[:, 14].mean() / ns_:.0f}, relax (+ next grab) {d[:, 9].mean() / ns_:.0f} cyc")
print(f"  total mean {(d[:, 5] - d[:, 0]).mean():.0f} cyc; level passes {d[:, 7].mean():.1f}")
