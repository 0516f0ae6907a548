#!/usr/bin/env python3
"""Compute time of every rank of a W-way strong split of one config, each rank's plan run in
turn on this one GPU (diagnostic for the multi-GPU partition: the slowest rank sets N>1 time).
  python tools/emul_ranks.py --config c4 --world 8 [--reps 3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from shadow_amd.graph import config  # noqa: E402
from shadow_amd.route import REFRESH_JOBS, REFRESH_MINE, RouteEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--world", type=int, nargs="+", default=[8])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--shared", action="store_true",
                help="one context for every rank (else each rank builds its own, so its plan pays "
                     "for its own hub rows, as a real rank's would)")
a = ap.parse_args()
g = config(a.config)
eng = RouteEngine(g)
T = g.targets()
dev = torch.device("cuda", 0)
d_tgt = torch.from_numpy(np.ascontiguousarray(T, np.int32)).to(dev)
st = torch.cuda.current_stream(dev)
for W in a.world:
    res = []
    ttt = []
    for r in range(W):
        if not a.shared and (r > 0 or W != a.world[0]):
            eng.close()
            eng = RouteEngine(g)
        t0 = time.perf_counter()
        plan = eng.plan(T, W, r)
        tp = time.perf_counter() - t0
        ns = len(plan.sources)
        lat = torch.empty((max(ns, 1), len(T)), dtype=torch.float64, device=dev)
        rel = torch.empty_like(lat)
        mn = torch.full((max(ns, 1),), float("inf"), dtype=torch.float64, device=dev)
        # a landmark-only plan's rank computes its share of the landmark rows and receives the
        # rest (the all-gather is not run here: the other shares stay in the store from the
        # plan's creation; its bytes are reported)
        lm = plan.landmarks()
        split = W > 1 and lm is not None

        def run():
            if split:
                plan.refresh_async(stream=st.cuda_stream, what=REFRESH_MINE)
                plan.refresh_async(stream=st.cuda_stream, what=REFRESH_JOBS)
            plan.rows_async(d_tgt, lat, rel, mn, stream=st.cuda_stream, reuse=split)
        run()
        eng.sync(st.cuda_stream)
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run()
            e1.record(st)
            eng.sync(st.cuda_stream)
            ms.append(e0.elapsed_time(e1))
        info = plan.info
        res.append(min(ms))
        ttt.append(tp * 1e3 + min(ms))
        print(f"W={W} rank {r}: rows {ns} helpers {info['helpers']} roots {info['roots']} levels {info['levels']} "
              f"launches {info['launches']} step {min(ms):.2f} ms (plan {tp * 1e3:.1f} ms, time to table "
              f"{ttt[-1]:.2f} ms)" + (f" landmarks {lm['count']} of {lm['nland']}, exchange "
                                      f"{(W - 1) * -(-lm['nland'] // W) * lm['row_stride'] * 6 / 1e6:.1f} MB in"
                                      if split else ""), flush=True)
        del lat, rel, plan
        torch.cuda.empty_cache()
    print(f"W={W}: max {max(res):.2f} ms  mean {np.mean(res):.2f} ms  time-to-table max {max(ttt):.2f} ms",
          flush=True)
