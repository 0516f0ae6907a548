#!/usr/bin/env python3
"""Per-phase cycles of KBF (sssp_batch_rows_kernel) workgroups from the diagnostic
(SHD_STAMPS) build: SHD_ROUTE_LIB=shadow_amd/libshd_route_diag.so python tools/kb_stamps.py --config c2
Slots (sssp_batch.hpp): 0 kernel start, 1 sweeps start (CSR staged, D initialised), 2 sweeps
done, 5 parents done, 6 walk records done, 3 rows done; 4 the sweep count."""
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
a = ap.parse_args()
g = config(a.config)
eng = route.RouteEngine(g)
L = route.load_library()
T = g.targets()
S = T
dev = torch.device("cuda", 0)
d_src = torch.from_numpy(S.astype(np.int32)).to(dev)
d_tgt = torch.from_numpy(T.astype(np.int32)).to(dev)
lat = torch.empty((len(S), len(T)), dtype=torch.float64, device=dev)
rel = torch.empty_like(lat)
mn = torch.empty(len(S), dtype=torch.float64, device=dev)
# (the KB kernels index the buffer past ns * 8 entries: room for both layouts)
dbg = torch.zeros(len(S) * 8 + len(S) * 16 + 4096, dtype=torch.int64, device=dev)
L.shd_route_debug_buffer.argtypes = [C.c_void_p, C.c_void_p]
L.shd_route_debug_buffer(eng._h, C.c_void_p(dbg.data_ptr()))
for rep in range(3):
    dbg.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.rows_async(d_src, d_tgt, lat, rel, mn)
    e1.record()
    eng.sync()
    torch.cuda.synchronize()
print(f"{a.config}: n={g.n} sources={len(S)} kernel={eng.info['kernel']} launch {e0.elapsed_time(e1):.3f} ms")
d = dbg.cpu().numpy().astype(np.int64)[len(S) * 8:len(S) * 8 + len(S) * 16].reshape(-1, 16)
d = d[d[:, 0] > 0]
print(f"  workgroups stamped {len(d)}")
order = [(0, 1, "init (CSR to LDS, D)"), (1, 2, "sweeps"), (2, 5, "parents"), (5, 6, "walk records"), (6, 3, "rows (walks + stores)")]
for s0, s1, nm in order:
    x = d[:, s1] - d[:, s0]
    print(f"  {nm:24s} mean {x.mean():9.0f} cyc  p50 {np.median(x):9.0f}  max {x.max():9.0f}")
print(f"  sweeps per batch mean {d[:, 4].mean():.1f} max {d[:, 4].max()}; total mean {(d[:, 3] - d[:, 0]).mean():.0f} cyc "
      f"(s_memtime: shader cycles)")
