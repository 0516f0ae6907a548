"""End-to-end eager fill through the C front end (shd_topology_fill: every attached pair's
Path, topology.c:1284-1386 + 1407-1523 for all sources) at C3 / C4 on the GPU box.

Reports, per config: attach time, fill wall time (plan + rows on the device + pack +
D2H into the pinned triangle), the triangle's bytes and the rate they land in host
memory at, and the process's peak host RSS.  The reference's equivalent is one igraph
Dijkstra per source on one CPU core.

  python tools/fill_bench.py --configs c3,c4 [--devices 0] [--out profiles/r02_fill.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rss_gb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6  # kB -> GB


def breakdown(g, T, dev):
    """The same fill straight through the engine (shd_route_fill_triangle), split into:
    pinning the triangle, planning, the rows on the device into HBM, and the whole fill
    (plan + rows + pack + D2H) twice: the first into freshly pinned pages, then warm; and
    the front end's path, a lazily pinned buffer (chunks registered while the rows run and
    the first chunks copy: shd_route_host_alloc_lazy), timed from the allocation.  The
    layout is the front end's: compact when the engine reports lat16."""
    import numpy as np
    import torch
    from shadow_amd import route
    eng = route.RouteEngine(g, device=dev)
    A = np.sort(T).astype(np.int32)
    na = len(A)
    l16 = bool(eng.info["lat16"]) and float(g.latency.max()) < 65535.0
    nbytes = 64 * route.tri16_lines(na) if l16 else 16 * (na * (na + 1) // 2)
    t0 = time.perf_counter()
    buf = route.PinnedBuffer(nbytes)
    pin_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    plan = eng.plan(A)
    plan_s = time.perf_counter() - t0
    d = torch.device("cuda", dev)
    d_tgt = torch.from_numpy(A).to(d)
    lat = torch.empty((na, na), dtype=torch.float64, device=d)
    rel = torch.empty_like(lat)
    plan.rows_async(d_tgt, lat, rel, None)
    eng.sync()
    t0 = time.perf_counter()
    plan.rows_async(d_tgt, lat, rel, None)
    eng.sync()
    rows_s = time.perf_counter() - t0
    del lat, rel
    plan.close()
    torch.cuda.empty_cache()
    _, cold = eng.fill_triangle(A, buf, lat16=l16)
    _, warm = eng.fill_triangle(A, buf, lat16=l16)
    ref = np.frombuffer((C.c_char * nbytes).from_address(buf.ptr), np.uint8).copy()
    buf.close()
    t0 = time.perf_counter()
    lz = route.PinnedBuffer(nbytes, lazy=True)
    eng.fill_triangle(A, lz, lat16=l16)
    lz.wait()
    lazy_s = time.perf_counter() - t0
    same = bool(np.array_equal(ref, np.frombuffer((C.c_char * nbytes).from_address(lz.ptr), np.uint8)))
    lz.close()
    eng.close()
    return {"layout_bytes": nbytes, "pin_s": round(pin_s, 4), "plan_s": round(plan_s, 4),
            "rows_hbm_s": round(rows_s, 4), "fill_cold_s": round(cold, 4), "fill_warm_s": round(warm, 4),
            "d2h_GBps_warm": round(nbytes / max(1e-9, warm - plan_s - rows_s) / 1e9, 2),
            "lazy_alloc_plus_fill_s": round(lazy_s, 4), "lazy_equals_eager": same}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c4")
    ap.add_argument("--devices", default="0", help="comma list of device ids (one context each)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    torch.cuda.init()  # torch's HIP runtime first (tests/conftest.py)
    from shadow_amd import topology
    from shadow_amd.graph import config
    topology.load_library()
    devs = tuple(int(x) for x in a.devices.split(","))
    out = []
    for cfg in a.configs.split(","):
        g = config(cfg)
        T = g.targets()
        t0 = time.perf_counter()
        t = topology.Topology.from_graph(g, devices=devs)
        t_new = time.perf_counter() - t0
        t0 = time.perf_counter()
        t.attach_all(T)
        t_att = time.perf_counter() - t0
        rss0 = rss_gb()
        t0 = time.perf_counter()
        sec = t.fill()
        wall = time.perf_counter() - t0
        na = len(T)
        pairs = na * (na + 1) // 2
        tri_bytes = t.triangle_bytes()
        lat = t.get_latency(int(T[0]), int(T[-1]))
        rec = {"config": cfg, "n": g.n, "attached": na, "contexts": len(devs), "new_s": round(t_new, 3),
               "attach_s": round(t_att, 3), "fill_s": round(sec, 4), "fill_wall_s": round(wall, 4),
               "triangle_pairs": pairs, "triangle_bytes": tri_bytes,
               "layout": "compact u16 lat + f64 rel, 6 pairs per 64-B line" if tri_bytes < 16 * pairs
                         else "interleaved f64 (lat, rel)", "bytes_per_pair": round(tri_bytes / pairs, 3),
               "host_write_GBps": round(tri_bytes / sec / 1e9, 2), "pairs_per_s": round(pairs / sec),
               "peak_rss_gb_before_fill": round(rss0, 2), "peak_rss_gb": round(rss_gb(), 2),
               "min_path_latency": t.min_path_latency(), "probe_latency": lat}
        t.close()
        del t
        if len(devs) == 1:
            rec["engine"] = breakdown(g, T, devs[0])
        print(json.dumps(rec), flush=True)
        out.append(rec)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
