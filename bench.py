#!/usr/bin/env python3
"""Benchmark: all-pairs topology routing (source-paths/s, GTEPS) on MI355X.

One step = the hot path over one synthetic topology: every attached source's
SOURCE(s,.) row (batched SSSP + path attributes, K1+K2) written to HBM, plus the
device-wide runahead min (K5).  Inputs (graph, source/target lists) are resident in
HBM before the timed region; outputs stay in HBM.

Default workload (N=1): BASELINE.json configs[1] = C2, a 2,000-vertex Barabasi-Albert
Internet-like topology, all 2,000 vertices attached, full 2,000 x 2,000 table.

Multi-GPU (one process per GPU, launched by torch.distributed.run):
  --scaling weak   (default) every rank computes the full table of its own C2-shaped
                   topology (seed 1 + rank; rank 0 is exactly C2): independent objects,
                   no data-path collective.
  --scaling strong one topology, attached sources sharded in contiguous blocks; the
                   runahead min is combined with an RCCL all-reduce(MIN) each step and,
                   with --allgather, the row shards are all-gathered over xGMI.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def b_src(n, nnz, nt):
    """SURVEY 8(d) algorithmic bytes per source row:
    4(n+1) row_ptr + 12 nnz (col i32 + lat f64) + 12 n (parent i32 + r f64) + 16 |T| (lat+rel out)."""
    return 4 * (n + 1) + 12 * nnz + 12 * n + 16 * nt


def workload_graph(cfg: str, seed_offset: int):
    from shadow_amd import graph as G
    if seed_offset == 0:
        return G.config(cfg)
    base = {"c2": (2000, 5, 1, None, None), "c3": (10000, 4, 2, None, 27000),
            "c4": (50000, 10, 3, 500000, None)}[cfg]
    n, m, seed, exact, hosts = base
    return G.internet_like(n, m, seed + seed_offset, exact_edges=exact, hosts=hosts,
                           name=f"{cfg}_rank{seed_offset}")


def cpu_baseline(g, sources, targets, budget_s: float):
    """Oracle port timed on this box's host cores (rank 0, N=1 only)."""
    from oracle.oracle import OracleGraph
    og = OracleGraph(g)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    # parallel restatement: the whole source set if it fits the budget, else a prefix sample
    probe = sources[: max(1, min(len(sources), 64))]
    dt, _, used = og.bench_parallel(probe, targets, threads)
    per_src = dt / len(probe)
    k = int(min(len(sources), max(len(probe), budget_s / max(per_src, 1e-9))))
    sample = sources[:k]
    dt, _, used = og.bench_parallel(sample, targets, threads)
    par = {"value": k / dt, "unit": "source-paths/s", "cores": int(used), "kind": "port",
           "sample": f"{k} of {len(sources)} sources x {len(targets)} targets (oracle/oracle.c "
                     f"orc_bench_parallel: OpenMP binary-heap Dijkstra + forward-order path products)",
           "cpu": platform.processor() or platform.machine()}
    # reference-faithful: 1 thread, igraph-order Dijkstra + per-hop get_eid + string formatting
    kf = max(1, min(len(sources), int(0.25 * budget_s / max(per_src * used, 1e-9))))
    dtf, _ = og.bench_faithful(sources[:kf], targets)
    faithful = {"value": kf / dtf, "unit": "source-paths/s", "cores": 1, "kind": "port",
                "sample": f"{kf} sources x {len(targets)} targets, igraph-0.7.1-order Dijkstra with "
                          "topology.c:1449,1502,1831 path/log formatting, serialised as under graphLock"}
    return par, faithful


def load_traffic(cfg: str, n_src: int):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary
    (profiles/*pmc*<cfg>*.json written by tools/pmc_traffic.py), or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc*{cfg}*.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        if int(d.get("sources_per_launch", -1)) != n_src:
            return None
        return float(d["hbm_bytes_per_launch"])
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--allgather", action="store_true", help="strong: all-gather row shards each step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work")
    ap.add_argument("--verify", type=int, default=8, help="rows checked against the oracle after timing")
    ap.add_argument("--sources", type=int, default=0, help="limit sources per rank (0 = all)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "f64", "k32", "kb", "k16", "kd"], help="force an SSSP kernel")
    args = ap.parse_args()
    if args.kernel != "auto":
        os.environ["SHD_ROUTE_KERNEL"] = args.kernel

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("launch N>1 with torch.distributed.run (one process per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    from shadow_amd.route import RouteEngine

    weak = args.scaling == "weak"
    g = workload_graph(args.config, rank if weak else 0)
    targets = g.targets()
    all_sources = targets.copy()
    if args.sources:
        all_sources = all_sources[: args.sources]
    from shadow_amd.shard import allgather_rows, runahead_min, shard_range
    if weak or world == 1:
        my_sources = all_sources
    else:
        lo, hi = shard_range(len(all_sources), world, rank)
        my_sources = all_sources[lo:hi]
    ns, nt = len(my_sources), len(targets)

    eng = RouteEngine(g, device=local)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    d_src = torch.from_numpy(np.ascontiguousarray(my_sources, np.int32)).to(dev)
    d_tgt = torch.from_numpy(np.ascontiguousarray(targets, np.int32)).to(dev)
    d_lat = torch.empty((max(ns, 1), nt), dtype=torch.float64, device=dev)
    d_rel = torch.empty((max(ns, 1), nt), dtype=torch.float64, device=dev)
    d_rmin = torch.empty(max(ns, 1), dtype=torch.float64, device=dev)
    d_min = torch.empty(1, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    k_start = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k_end = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    def step(t=None):
        if t is not None:
            k_start[t].record(stream)
        eng.rows_async(d_src, d_tgt, d_lat, d_rel, d_rmin, stream=sh)
        if t is not None:
            k_end[t].record(stream)
        eng.min_reduce_async(d_rmin, d_min, stream=sh)
        if world > 1 and not weak:
            runahead_min(d_min, dist)                         # RCCL all-reduce MIN
            if args.allgather:                                # full latency table on every GPU
                allgather_rows(d_lat[:ns], len(all_sources), dist)

    for _ in range(args.warmup):
        step()
    eng.sync(sh)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    eng.sync(sh)  # raises on any device-side error
    # dominant-kernel duration: HIP events on the launch stream around the rows kernel, in
    # a second pass of the same K steps (an event pair per step costs ~10 us of stream time
    # on this stack, so the throughput pass above carries none)
    for t in range(args.steps):
        step(t)
    torch.cuda.synchronize()
    eng.sync(sh)
    kms = [k_start[t].elapsed_time(k_end[t]) for t in range(args.steps)]
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    total_src = ns * world if weak else len(all_sources)

    # correctness spot check against the oracle, outside the timed region
    verified = None
    if args.verify and rank == 0 and ns:
        from oracle.oracle import OracleGraph, TIE_MINKEY
        og = OracleGraph(g)
        pick = np.linspace(0, ns - 1, num=min(args.verify, ns)).astype(int)
        lat_h = d_lat[torch.from_numpy(pick).to(dev)].cpu().numpy()
        rel_h = d_rel[torch.from_numpy(pick).to(dev)].cpu().numpy()
        olat, orel, _, _ = og.source_rows(my_sources[pick], targets, TIE_MINKEY)
        verified = bool(np.array_equal(lat_h, olat) and np.array_equal(rel_h, orel))

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    n, nnz = g.n, g.nnz
    kavg_s = float(np.mean(kms)) / 1e3
    alg_bytes = ns * b_src(n, nnz, nt)
    achieved = alg_bytes / kavg_s / 1e9
    peak = 8000.0
    res = {
        "metric": "source-paths/sec",
        "value": total_src * args.steps / dt,
        "unit": "source-paths/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"{g.name}: Barabasi-Albert Internet-like topology, all-pairs latency/reliability "
                        f"table (BASELINE.json configs[{ {'c2': 1, 'c3': 2, 'c4': 3}[args.config] }])",
            "n_vertices": n, "n_edges": g.m, "n_edges_nonloop": g.m_nonloop, "csr_arcs": nnz,
            "sources_per_gpu": ns, "targets": nt,
            "parallelism": (f"replicas x{world} (independent topologies)" if weak else f"sources sharded /{world}"),
        },
        "gteps": total_src * g.m_nonloop * args.steps / dt / 1e9,
        "pairs_per_s": total_src * nt * args.steps / dt,
        "kernel_ms": float(np.mean(kms)),
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s", "frac": achieved / peak,
            "traffic": load_traffic(args.config, ns),
            "kernel": {0: "sssp_rows_kernel", 1: "sssp_k32_kernel",
                       2: ("sssp_batch_rows_kernel" if eng.info["reserved"] == 1
                           else "sssp_batch_kernel+path_attr_kernel"),
                       3: "sssp_k16_kernel", 4: "sssp_delta_kernel"}[eng.info["kernel"]],
            "bytes_per_source": b_src(n, nnz, nt),
        },
        "verified_rows_vs_oracle": verified,
    }
    if not args.no_cpu_baseline and world == 1:
        par, faithful = cpu_baseline(g, all_sources, targets, args.cpu_budget)
        res["cpu_baseline"] = par
        res["cpu_baseline_faithful"] = faithful
    else:
        res["cpu_baseline"] = None
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
