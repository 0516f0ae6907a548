#!/usr/bin/env python3
"""Benchmark: all-pairs topology routing (source-paths/s, GTEPS) on MI355X.

One step = the hot path over one synthetic topology: every attached source's
SOURCE(s,.) row (batched SSSP + path attributes) written to HBM, plus the device-wide
runahead min (K5).  Inputs (graph, source/target lists) are resident in HBM before the
timed region; outputs stay in HBM.

Default workload: BASELINE.json configs[3] = C4, the 50,000-vertex / 500,000-edge
synthetic AS graph, all 50,000 vertices attached: the full 50k x 50k latency and
reliability table (2.5e9 pairs, 40 GB of f64 in HBM) per step.  --config c2 / c3
select the smaller configs, --config c5 the dense complete graph (K3 direct fill + K5,
with the K4 Floyd-Warshall timed beside it).

Multi-GPU (one process per GPU, launched by torch.distributed.run):
  --scaling strong (default) one topology, attached sources sharded over the ranks
                   by the seeded plan (whole subtrees of the seed forest per rank, its top
                   levels computed on every rank as helper rows); the runahead min is
                   combined with an RCCL all-reduce(MIN) each step.  The all-gather of the latency AND reliability row shards into
                   the full table on every GPU is timed separately (it is needed only
                   where a device-resident full matrix is; Shadow's host cache is filled
                   per rank by D2H of its own shard); --allgather puts it in every step.
  --scaling weak   every rank computes the full table of its own topology (seed 1 +
                   rank): independent objects, no data-path collective.
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

CFG_INDEX = {"c2": 1, "c3": 2, "c4": 3, "c5": 4, "c2f": 1, "c3f": 2, "c4f": 3}


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


def cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count()
    quota = None
    try:  # cgroup v2 CPU quota of this job ("max" = none)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        pass
    try:
        out = subprocess.run(["ldconfig", "-p"], capture_output=True, text=True, timeout=20).stdout
        igraph = "libigraph present: " + ",".join(sorted({l.split()[0] for l in out.splitlines() if "igraph" in l})) \
            if "igraph" in out else "libigraph absent (ldconfig -p): reference not linkable, oracle port timed"
    except Exception as e:  # noqa: BLE001
        igraph = f"ldconfig probe failed: {e}"
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "igraph_probe": igraph}


def all_cores():
    """every host core this process may run on (nproc)."""
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def thread_counts(info):
    """CPU thread counts a baseline is tried at: every core this process may run on (nproc),
    the job's cgroup CPU quota, 16 (the box's nominal CPU share)."""
    counts = []
    for c in (all_cores(), int(math.ceil(info["cgroup_cpu_quota"])) if info.get("cgroup_cpu_quota") else None, 16):
        if c and min(c, all_cores()) not in counts:
            counts.append(min(c, all_cores()))
    return counts


def cpu_baseline(g, sources, targets, budget_s: float):
    """Oracle port timed on this box's host cores (rank 0, N=1 only), on a bounded seeded
    sample of the same workload; the rate is per source row, so it extrapolates to the
    full table linearly (every row is one full SSSP + |T| path products).  B2 (BASELINE.md
    3): the best rate over nproc threads, the cgroup quota and 16 threads, with the
    winning thread count as `cores` and every count tried beside it."""
    from oracle.oracle import OracleGraph
    og = OracleGraph(g)
    rng = np.random.default_rng(12345)
    info = cpu_info()

    def run(threads, budget):
        probe = np.sort(rng.choice(sources, size=min(len(sources), 2 * threads), replace=False)).astype(np.int32)
        dt, _, used = og.bench_parallel(probe, targets, threads)
        per_src = dt / len(probe)
        k = int(min(len(sources), max(len(probe), budget / max(per_src, 1e-9))))
        sample = np.sort(rng.choice(sources, size=k, replace=False)).astype(np.int32) if k < len(sources) else sources
        dt, _, used = og.bench_parallel(sample, targets, threads)
        return {"value": k / dt, "unit": "source-paths/s", "cores": int(used), "kind": "port",
                "sample": f"{k} of {len(sources)} sources (seeded uniform sample) x {len(targets)} targets, "
                          f"{dt:.2f} s on {used} threads (oracle/oracle.c orc_bench_parallel: OpenMP binary-heap "
                          f"Dijkstra + forward-order path products); full table extrapolated "
                          f"{len(sources) / (k / dt):.1f} s",
                "extrapolated": k < len(sources)}, sample

    # thread counts tried: every core this process may run on (nproc), the job's cgroup CPU
    # quota, 16 (the box's nominal CPU share); the best rate is the baseline, and the thread
    # count that produced it is its `cores` (nproc threads on a 16-CPU quota run oversubscribed)
    counts = thread_counts(info)
    tried, sample = [], None
    for c in counts:
        r, smp = run(c, 0.8 * budget_s / len(counts))
        tried.append(r)
        sample = smp if sample is None else sample
    par = dict(max(tried, key=lambda r: r["value"]))
    par.update(info)
    par["threads_tried"] = [{k: r[k] for k in ("value", "cores", "sample")} for r in tried]
    par["selection"] = "best rate over the thread counts tried (nproc, cgroup quota, 16)"
    # reference-faithful: 1 thread, igraph-order Dijkstra + per-hop get_eid + string formatting
    t1, _ = og.bench_faithful(sample[:1], targets)
    kf = int(max(1, min(len(sources), 0.15 * budget_s / max(t1, 1e-9))))
    dtf, _ = og.bench_faithful(sample[:kf], targets)
    faithful = {"value": kf / dtf, "unit": "source-paths/s", "cores": 1, "kind": "port",
                "sample": f"{kf} sources x {len(targets)} targets in {dtf:.2f} s, igraph-0.7.1-order Dijkstra "
                          "with topology.c:1449,1502,1831 path/log formatting, serialised as under graphLock",
                "extrapolated": kf < len(sources)}
    return par, faithful


def build_id():
    """This engine build's identity (shadow_amd/build.py source_id: flags + sources)."""
    from shadow_amd import build
    return build.source_id()


def load_pmc(cfg: str, n_src: int, kernel: str):
    """The newest committed PMC summary (profiles/<round>_pmc_<cfg>.json, tools/pmc_traffic.py)
    for this config and launch size that was profiled on THIS build and holds `kernel`: its
    per-launch bytes (fetch + write) of that kernel only.  None when there is none; the reason
    is in the returned note."""
    # (exactly <round>_pmc_<cfg>.json: "c3" must not pick up a c3f summary)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{cfg}.json")))
    bid = build_id()
    note = f"no PMC summary for {cfg} at {n_src} sources per launch"
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if int(d.get("sources_per_launch", -1)) != n_src:
            continue
        if d.get("build_id") != bid:
            note = (f"newest PMC summary {os.path.relpath(f, ROOT)} was profiled on build "
                    f"{d.get('build_id')}, not this build {bid}: traffic not reported")
            break  # (an older file is older still)
        ks = {k: v for k, v in d.get("kernels", {}).items() if kernel in k}
        if not ks:
            note = f"{os.path.relpath(f, ROOT)} holds no {kernel} entry"
            break
        fetch = sum(float(v["fetch_bytes"]) for v in ks.values())
        fetch_lo = sum(float(v.get("fetch_bytes_uncorrected", v["fetch_bytes"])) for v in ks.values())
        write = sum(float(v.get("write_bytes", 0.0)) for v in ks.values())
        return {"file": os.path.relpath(f, ROOT), "build_id": bid, "kernels": sorted(ks),
                "bytes": fetch + write, "bytes_range": [fetch_lo + write, fetch + write],
                "read_bytes": fetch, "write_bytes": write}, None
    return None, note


def physical(cfg: str, n_src: int, n_tgt: int, kernel_s: float, peak_gbps: float, kernel: str):
    """What the counters say beside the algorithmic model: HBM bytes the line's kernel
    actually moved per launch and their rate, the writes against the compulsory output (16 B
    per pair), and the time the output write alone needs at peak."""
    out = 16.0 * n_src * n_tgt
    res = {"output_bytes": out, "output_floor_ms": out / (peak_gbps * 1e9) * 1e3}
    d, note = load_pmc(cfg, n_src, kernel)
    if d:
        tot = d["bytes"]
        res.update({"pmc_file": d["file"], "pmc_kernels": d["kernels"], "pmc_build_id": d["build_id"],
                    "traffic_bytes": tot, "traffic_bytes_range": d["bytes_range"],
                    "traffic_GBps": tot / kernel_s / 1e9, "traffic_frac": tot / kernel_s / 1e9 / peak_gbps,
                    "read_bytes": d["read_bytes"], "write_bytes": d["write_bytes"],
                    "write_amplification": d["write_bytes"] / out if out else None})
    else:
        res["pmc_note"] = note
    return res


def timed(fn, reps, sync, barrier=None):
    """Wall time of `reps` calls bracketed by barrier + device sync on both sides."""
    if barrier:
        barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    if barrier:
        barrier()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=25)  # C4: ~1.2 s timed
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4", choices=["c2", "c3", "c4", "c5", "c2f", "c3f", "c4f"])
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"])
    ap.add_argument("--allgather", action="store_true", help="strong: all-gather lat+rel shards in every step")
    ap.add_argument("--gather-reps", type=int, default=2, help="strong, N>1: separately timed all-gathers")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work")
    ap.add_argument("--verify", type=int, default=8, help="rows checked against the oracle after timing")
    ap.add_argument("--sources", type=int, default=0, help="limit sources (0 = all)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "f64", "k32", "kb", "kd"], help="force an SSSP kernel")
    ap.add_argument("--no-seed", action="store_true", help="plain KD rows (no seeded plan)")
    ap.add_argument("--emulate", default="", help="W:R = one GPU runs rank R's plan of a W-GPU strong split "
                    "(diagnostic: that rank's compute time; no collectives)")
    args = ap.parse_args()
    if args.kernel != "auto":
        os.environ["SHD_ROUTE_KERNEL"] = args.kernel
    if args.no_seed:
        os.environ["SHD_ROUTE_SEED"] = "0"

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1:
        raise SystemExit("launch N>1 with torch.distributed.run (one process per GPU)")
    # (rehearsals of N ranks on a smaller box share its GPUs: SHD_BENCH_BACKEND=gloo)
    gpu = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("SHD_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    barrier = dist.barrier if world > 1 else None

    if args.config == "c5":
        return bench_c5(args, torch, dist, world, rank, dev, barrier)

    from shadow_amd.route import RouteEngine
    from shadow_amd.shard import runahead_min

    weak = args.scaling == "weak"
    g = workload_graph(args.config, rank if weak else 0)
    targets = g.targets()
    all_sources = targets.copy()
    if args.sources:
        all_sources = all_sources[: args.sources]
    eng = RouteEngine(g, device=gpu)
    # the rows of this rank (strong: a contiguous block of the source list) under one
    # seeded plan: rows whose source has an already-computed neighbour start from it
    t_plan = time.perf_counter()
    if args.emulate and world == 1:
        ew, er = (int(x) for x in args.emulate.split(":"))
        plan = eng.plan(all_sources, ew, er)
    else:
        plan = eng.plan(all_sources, 1 if weak else world, 0 if weak else rank)
    t_plan = time.perf_counter() - t_plan
    my_sources = plan.sources
    ns, nt = len(my_sources), len(targets)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    d_tgt = torch.from_numpy(np.ascontiguousarray(targets, np.int32)).to(dev)
    gather = world > 1 and not weak
    d_lat = torch.empty((max(ns, 1), nt), dtype=torch.float64, device=dev)
    d_rel = torch.empty((max(ns, 1), nt), dtype=torch.float64, device=dev)
    if gather:
        # table assembly payload: each rank packs the upper triangles of its rows (the Path
        # cache holds each unordered pair once, topology.c:1307-1336), latency as u16 where
        # exact, and all-gathers the packed segments (padded to the largest rank's)
        from shadow_amd.shard import tri_offsets, allgather_payload, TriangleIndex
        lat16 = bool(eng.info["lat16"])  # integer latencies and self-loops below 0xFFFF
        pos = np.asarray(plan.positions, np.int64)  # attached positions (sources = the sorted targets)
        off, tot = tri_offsets(pos, nt)
        seg_t = torch.tensor([tot], dtype=torch.int64, device=dev)
        dist.all_reduce(seg_t, op=dist.ReduceOp.MAX)
        seg = int(seg_t.item())
        d_pos = torch.from_numpy(pos.astype(np.int32)).to(dev)
        d_off = torch.from_numpy(off[:-1].copy()).to(dev)
        p_lat = torch.empty(max(seg, 1), dtype=torch.int16 if lat16 else torch.float64, device=dev)
        p_rel = torch.empty(max(seg, 1), dtype=torch.float64, device=dev)
        pos_by_rank = [None] * world
        dist.all_gather_object(pos_by_rank, pos)
        tindex = TriangleIndex(pos_by_rank, nt, seg)
        gathered = {}
    # landmark-only plans split over ranks (C3-class): each rank computes its share of the
    # landmark rows and the shares are all-gathered in the step (an emulated rank, one GPU:
    # its share only, the others' rows present from the plan's creation, exchange unmeasured)
    from shadow_amd.route import REFRESH_MINE, REFRESH_JOBS
    from shadow_amd.shard import bind_landmark_store, exchange_landmarks, landmark_exchange_bytes
    ew = int(args.emulate.split(":")[0]) if args.emulate and world == 1 else world
    lm_split = ew > 1 and not weak and ns > 0 and plan.landmarks() is not None
    lm_store = bind_landmark_store(plan, world, dev) if lm_split and world > 1 else None
    # +inf: a rank with an empty shard contributes nothing to the runahead MIN
    d_rmin = torch.full((max(ns, 1),), float("inf"), dtype=torch.float64, device=dev)
    d_min = torch.full((1,), float("inf"), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    l_start = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k_start = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k_end = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    def gather_tables():
        if ns:
            eng.tri_payload_async(d_lat, d_rel, d_pos, d_off, nt, p_lat, p_rel, lat16=lat16, stream=sh)
        gathered["lat"], gathered["rel"] = allgather_payload(p_lat[:seg], p_rel[:seg], seg, dist)

    def step(t=None):
        # a step is every SSSP of the table: a landmark-only plan (C3) recomputes its landmark
        # rows, queue order and jobs first, inside rows_async.  The kernel-timing pass (t set)
        # runs that part ahead of the events and the rows launch alone inside them, so that
        # kernel_ms / roofline.achieved describe the rows kernel (landmark_ms beside it).
        if t is not None:
            l_start[t].record(stream)
        if lm_split:
            plan.refresh_async(stream=sh, what=REFRESH_MINE)
            exchange_landmarks(lm_store, dist)
            plan.refresh_async(stream=sh, what=REFRESH_JOBS)
        elif t is not None and ns:
            plan.refresh_async(stream=sh)
        if t is not None:
            k_start[t].record(stream)
        if ns:
            plan.rows_async(d_tgt, d_lat, d_rel, d_rmin, stream=sh, reuse=(t is not None) or lm_split)
        if t is not None:
            k_end[t].record(stream)
        eng.min_reduce_async(d_rmin, d_min, stream=sh)
        if world > 1 and not weak:
            runahead_min(d_min, dist)                         # RCCL all-reduce MIN
            if args.allgather:
                gather_tables()

    for _ in range(args.warmup):
        step()
    eng.sync(sh)
    dt = timed(step, args.steps, torch.cuda.synchronize, barrier)
    eng.sync(sh)  # raises on any device-side error
    # dominant-kernel duration: HIP events on the launch stream around the rows launch, in
    # a second pass of the same K steps (the throughput pass above carries no events)
    for t in range(args.steps):
        step(t)
    torch.cuda.synchronize()
    eng.sync(sh)
    kms = [k_start[t].elapsed_time(k_end[t]) for t in range(args.steps)]
    lms = [l_start[t].elapsed_time(k_start[t]) for t in range(args.steps)]  # (0 unless landmark-only)
    split = None
    if gather:
        # compute / collective split: the runahead all-reduce and the table
        # all-gather, each timed on its own
        ar_s = timed(lambda: runahead_min(d_min, dist), 20, torch.cuda.synchronize, barrier) / 20
        ag_s = None
        if not args.allgather and args.gather_reps > 0:
            gather_tables()
            ag_s = timed(gather_tables, args.gather_reps, torch.cuda.synchronize, barrier) / args.gather_reps
        split = torch.tensor([float(np.mean(kms)) / 1e3, ar_s, ag_s or 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(split, op=dist.ReduceOp.MAX)
        gathered_ok = None
        if args.verify and rank == 0 and gathered:
            # rows computed on the LAST rank, read back out of rank 0's gathered payload
            from oracle.oracle import OracleGraph, TIE_MINKEY
            og = OracleGraph(g)
            mine = np.asarray(pos_by_rank[world - 1])
            pick = mine[np.linspace(0, len(mine) - 1, num=min(3, len(mine))).astype(int)]
            from shadow_amd.shard import decode_lat16
            gl, gr = gathered["lat"].cpu().numpy(), gathered["rel"].cpu().numpy()
            gathered_ok = True
            for i in pick:
                olat, orel, _, _ = og.source_row(int(targets[i]), targets, TIE_MINKEY)
                k = tindex.index(np.full(nt - i, i), np.arange(i, nt))
                L = decode_lat16(gl[k]) if lat16 else gl[k]
                gathered_ok &= bool(np.array_equal(L, olat[i:], equal_nan=True) and
                                    np.array_equal(gr[k], orel[i:], equal_nan=True))
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    total_src = ns * world if weak else (ns if args.emulate else len(all_sources))

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
    runahead = float(d_min.item())

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    n, nnz = g.n, g.nnz
    kavg_s = float(np.mean(kms)) / 1e3
    peak = 8000.0
    # roofline: the bytes the launch MUST move (its output rows, 16 B per pair) over the
    # kernel's HIP-event time; the counters' bytes beside it (traffic, traffic_frac)
    out_bytes = 16.0 * ns * nt
    achieved = out_bytes / kavg_s / 1e9
    kname = {0: "sssp_rows_kernel", 1: "sssp_k32_kernel",
             2: ("sssp_batch_rows_kernel" if eng.info["reserved"] == 1 else "sssp_batch_kernel"),
             4: "sssp_delta_kernel", 5: "sssp_f64d_kernel"}.get(eng.info["kernel"], str(eng.info["kernel"]))
    phys = physical(args.config, ns, nt, kavg_s, peak, kname)
    model_bytes = ns * b_src(n, nnz, nt)
    res = {
        "metric": "source-paths/sec",
        "build_id": build_id(),
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
                        f"table (BASELINE.json configs[{CFG_INDEX[args.config]}]"
                        + (", two-decimal fractional latencies)" if args.config.endswith("f") else ")"),
            "n_vertices": n, "n_edges": g.m, "n_edges_nonloop": g.m_nonloop, "csr_arcs": nnz,
            "sources_total": total_src, "sources_per_gpu": ns, "targets": nt,
            "table_bytes": 16 * total_src * nt,
            "parallelism": (f"replicas x{world} (independent topologies)" if weak
                            else (f"sources sharded /{world}: seed-forest subtrees per rank, "
                                  f"top levels replicated as helper rows" if world > 1 else "one GPU")),
        },
        "gteps": total_src * g.m_nonloop * args.steps / dt / 1e9,
        "pairs_per_s": total_src * nt * args.steps / dt,
        "kernel_ms": float(np.mean(kms)),
        "landmark_ms": float(np.mean(lms)),
        "step_contents": (("this rank's share of the landmark rows + their all-gather over the ranks + the job records "
                           "(1 kernel) + the rows launch + runahead min" if lm_split else
                           "landmark rows (hub-row launch) + the job records derived from them (1 kernel) + the "
                           "rows launch + runahead min: every SSSP of the table") if plan.info["launches"] > 1 else
                          "the rows launch (every row of the table) + runahead min"),
        "time_to_table_ms": t_plan * 1e3 + dt / args.steps * 1e3,
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s", "frac": achieved / peak,
            "traffic": phys.get("traffic_bytes"),
            "traffic_frac": phys.get("traffic_frac"),
            "kernel": kname,
            "model": "compulsory bytes per launch = the lat + rel output rows (16 B per source-target pair); "
                     "achieved = those bytes / the rows kernel's HIP-event time; traffic = PMC HBM bytes per "
                     "launch (profiles/), traffic_frac = traffic / kernel time / peak",
            "compulsory_bytes_per_launch": out_bytes,
            "launches_per_step": plan.info["launches"],
            "physical": phys,
            "work_avoided": {
                "survey_model": "SURVEY 8(d) B_src = 4(n+1) + 12 nnz + 12 n + 16 |T| per source row "
                                "(every row a full CSR pass)",
                "bytes_per_source": b_src(n, nnz, nt),
                "model_rate_GBps": model_bytes / kavg_s / 1e9,
                "model_over_peak": model_bytes / kavg_s / 1e9 / peak,
                "note": "above 1 means seeded rows skip most of the per-row CSR pass the model charges; "
                        "it measures work avoided, not bandwidth used"},
        },
        "plan": {**plan.info, "plan_seconds": t_plan},
        "landmark_split": ({**plan.landmarks(), "exchange_bytes_per_rank": (world - 1) * -(-plan.landmarks()["nland"] // ew)
                            * plan.landmarks()["row_stride"] * 6 if world > 1 else None,
                            "emulated_exchange_bytes": (ew - 1) * -(-plan.landmarks()["nland"] // ew)
                            * plan.landmarks()["row_stride"] * 6,
                            "note": "emulated rank: the exchange is not run (unmeasured on hardware)"
                            if world == 1 else "exchange inside the step"} if lm_split else None),
        "runahead_min_latency_ms": runahead,
        "verified_rows_vs_oracle": verified,
    }
    if split is not None:
        c_s, ar_s, ag_s = (float(x) for x in split.tolist())
        gb = (world - 1) * seg * ((2 if lat16 else 8) + 8)  # received per GPU
        full_gb = 16 * len(all_sources) * nt * (world - 1) / world
        res["split"] = {"compute_ms": c_s * 1e3, "allreduce_min_ms": ar_s * 1e3,
                        "allgather_lat_rel_ms": (ag_s * 1e3) if ag_s else None,
                        "allgather_in_step": bool(args.allgather),
                        "allgather_payload": ("upper-triangle rows, lat u16 + rel f64" if lat16
                                              else "upper-triangle rows, lat f64 + rel f64"),
                        "allgather_bytes_per_gpu": gb,
                        "full_f64_table_bytes_per_gpu": full_gb,
                        "payload_over_full_table": gb / full_gb,
                        "allgather_GBps_per_gpu": (gb / ag_s / 1e9) if ag_s else None,
                        "gathered_rows_verified_vs_oracle": gathered_ok}
    if not args.no_cpu_baseline and world == 1:
        par, faithful = cpu_baseline(g, all_sources, targets, args.cpu_budget)
        res["cpu_baseline"] = par
        res["cpu_baseline_faithful"] = faithful
    else:
        res["cpu_baseline"] = None
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_c5(g, T, budget_s: float):
    """the reference semantics (every pair DIRECT, topology.c:1877-1927)
    filled on all nproc cores, timed in full; and Floyd-Warshall in f64 on all cores over a
    sample of k-phases, extrapolated x n / k (the CPU counterpart of K4)."""
    from oracle.oracle import OracleGraph, bench_fw_phases
    og = OracleGraph(g)
    info = cpu_info()
    tried = []
    for c in thread_counts(info):  # the best rate over nproc / quota / 16 threads (as for C4)
        dt, used = og.bench_direct(T, c)
        tried.append({"value": len(T) / dt, "cores": int(used),
                      "sample": f"full direct fill {len(T)} x {len(T)} pairs in {dt:.3f} s on {used} threads "
                                "(oracle/oracle.c orc_bench_direct: get_eid + factor products per pair, rows "
                                "written to per-thread buffers)"})
    best = max(tried, key=lambda r: r["value"])
    direct = {"value": best["value"], "unit": "source-paths/s", "cores": best["cores"], "kind": "port",
              "sample": best["sample"], "extrapolated": False, **info, "threads_tried": tried,
              "selection": "best rate over the thread counts tried (nproc, cgroup quota, 16)"}
    n = g.n
    W = np.full((n, n), np.inf)
    W[g.src, g.dst] = np.minimum(W[g.src, g.dst], g.latency)
    if not g.directed:
        W[g.dst, g.src] = np.minimum(W[g.dst, g.src], g.latency)
    np.fill_diagonal(W, 0.0)
    # the best rate over nproc / quota / 16 threads, as for the direct fill (round 4 ran it on
    # nproc = 256 threads against a 16-CPU quota, oversubscribed)
    fw_tried = []
    for c in thread_counts(info):
        t1, used = bench_fw_phases(W, 0, 8, c)  # probe 8 phases (oversubscribed barriers vary)
        nk = int(max(1, min(n - 8, 0.1 * budget_s / max(t1 / 8, 1e-9))))
        dtk, used = bench_fw_phases(W, 8, nk, c)
        fw_tried.append({"value": len(T) / (dtk * n / nk), "cores": int(used),
                         "sample": f"{nk} of {n} k-phases of f64 Floyd-Warshall (oracle/oracle.c orc_bench_fw_phases) "
                                   f"in {dtk:.2f} s on {used} threads; full table extrapolated {dtk * n / nk:.1f} s",
                         "extrapolated": nk < n})
    fb = max(fw_tried, key=lambda r: r["value"])
    fw = {"value": fb["value"], "unit": "source-paths/s (FW table only)", "cores": fb["cores"], "kind": "port",
          "sample": fb["sample"], "extrapolated": fb["extrapolated"], "threads_tried": fw_tried,
          "selection": "best rate over the thread counts tried (nproc, cgroup quota, 16)"}
    return direct, fw


def bench_c5(args, torch, dist, world, rank, dev, barrier):
    """C5: dense K4000 + self-loops.  A step is the reference semantics for a complete
    graph: every pair DIRECT (K3 direct fill, topology.c:1877-1927) + the runahead
    min (K5).  Beside it, the K4 path: the blocked min-plus Floyd-Warshall table
    (G-relax/s against the packed-u16 VALU rate it runs at) and the SOURCE rows of
    every vertex from it (parents by the engine tie rule, rel down the tree)."""
    from shadow_amd import graph as G
    from shadow_amd.route import RouteEngine
    g = G.config("c5")
    T = g.targets()
    eng = RouteEngine(g, device=int(os.environ.get("LOCAL_RANK", "0")))
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    n = g.n
    d_src = torch.from_numpy(T.astype(np.int32)).to(dev)
    d_tgt = d_src
    d_lat = torch.empty((n, n), dtype=torch.float64, device=dev)
    d_rel = torch.empty_like(d_lat)
    d_rmin = torch.full((n,), float("inf"), dtype=torch.float64, device=dev)
    d_min = torch.full((1,), float("inf"), dtype=torch.float64, device=dev)

    def step():
        eng.rows_async(d_src, d_tgt, d_lat, d_rel, d_rmin, stream=sh, dispatch=True)  # complete -> K3
        eng.min_reduce_async(d_rmin, d_min, stream=sh)

    for _ in range(args.warmup):
        step()
    eng.sync(sh)
    dt = timed(step, args.steps, torch.cuda.synchronize, barrier)
    eng.sync(sh)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        eng.rows_async(d_src, d_tgt, d_lat, d_rel, d_rmin, stream=sh, dispatch=True)
    e1.record(stream)
    torch.cuda.synchronize()
    k3_s = e0.elapsed_time(e1) / 1e3 / args.steps
    runahead = float(d_min.item())
    verified = None
    if args.verify and rank == 0:
        from oracle.oracle import OracleGraph
        og = OracleGraph(g)
        lat_h = d_lat[:2].cpu().numpy(); rel_h = d_rel[:2].cpu().numpy()
        verified = all(og.direct(s, t) == (lat_h[s, t], rel_h[s, t]) for s in range(2) for t in range(0, n, 97))
    # K4: the FW table, then the SOURCE rows of every vertex from it
    reps = max(1, min(args.steps, 5))
    eng.fw_table_async(sh)
    eng.sync(sh)
    e0.record(stream)
    for _ in range(reps):
        eng.fw_table_async(sh)
    e1.record(stream)
    torch.cuda.synchronize()
    fw_s = e0.elapsed_time(e1) / 1e3 / reps
    # rows: one untimed call first (it allocates the parent-key buffer), then reps timed
    eng.fw_rows_async(d_src, d_tgt, d_lat, d_rel, d_rmin, stream=sh)
    eng.sync(sh)
    e0.record(stream)
    for _ in range(reps):
        eng.fw_rows_async(d_src, d_tgt, d_lat, d_rel, d_rmin, stream=sh)
    e1.record(stream)
    torch.cuda.synchronize()
    eng.sync(sh)
    fwr_s = e0.elapsed_time(e1) / 1e3 / reps
    fw_ok = None
    if args.verify and rank == 0:
        from oracle.oracle import OracleGraph, TIE_MINKEY
        pick = np.array([0, n // 2, n - 1])
        olat, orel, _, _ = OracleGraph(g).source_rows(T[pick], T, TIE_MINKEY)
        fw_ok = bool(np.array_equal(d_lat[torch.from_numpy(pick).to(dev)].cpu().numpy(), olat) and
                     np.array_equal(d_rel[torch.from_numpy(pick).to(dev)].cpu().numpy(), orel))
    if rank != 0:
        return
    relax = float(n) ** 3
    k3_phys = physical("c5", n, n, k3_s, 8000.0, "direct_rows_kernel")
    # packed u16 min-plus: one v_pk_add_u16 + one v_pk_min_u16 per 2 relaxations, i.e. one packed
    # instruction per relaxation.  Nominal: 32 lanes/cycle/SIMD at 2.4 GHz; measured on MI355X
    # (tools/micro/pk_rate.hip, 8 waves/SIMD, independent chains: profiles/r03_pk_rate.txt):
    # 35.8 T packed instructions/s (u32 adds 50.0 T/s), the roof the kernel can reach
    peak_nominal = 256 * 4 * 32 * 2.4e9
    peak_relax = 35.8e12
    res = {
        "metric": "source-paths/sec", "build_id": build_id(), "value": n * args.steps / dt, "unit": "source-paths/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{g.name}: complete K{n} + self-loops, reference semantics = every pair DIRECT "
                               "(K3) + runahead min (K5) (BASELINE.json configs[4])",
                   "n_vertices": n, "n_edges": g.m, "sources_total": n, "targets": n, "parallelism": "one GPU"},
        "pairs_per_s": n * n * args.steps / dt,
        "kernel_ms": k3_s * 1e3,
        "roofline": {"bound": "hbm", "achieved": 32.0 * n * n / k3_s / 1e9, "peak": 8000.0, "unit": "GB/s",
                     "frac": 32.0 * n * n / k3_s / 1e9 / 8000.0, "traffic": k3_phys.get("traffic_bytes"),
                     "traffic_frac": k3_phys.get("traffic_frac"), "physical": k3_phys,
                     "kernel": "direct_rows_kernel", "bytes_per_pair": 32,
                     "model": "SURVEY 8(d) K3: read lat + r (16 B) and write lat + rel (16 B) per pair"},
        "k4": {"fw_table_ms": fw_s * 1e3, "grelax_per_s": relax / fw_s / 1e9,
               "peak_grelax_per_s": peak_relax / 1e9, "frac": relax / fw_s / peak_relax,
               "peak_source": "measured packed-u16 VALU rate (tools/micro/pk_rate.hip, profiles/r03_pk_rate.txt)",
               "nominal_peak_grelax_per_s": peak_nominal / 1e9, "frac_of_nominal": relax / fw_s / peak_nominal,
               "bound": "valu (packed u16 min-plus: v_pk_add_u16 + v_pk_min_u16 per 2 relaxations)",
               "fp64_equivalent_peak_grelax_per_s": 39.3e12 / 1e9,
               "fw_rows_ms": fwr_s * 1e3, "rows_verified_vs_oracle": fw_ok,
               "fw_plus_rows_source_paths_per_s": n / (fw_s + fwr_s)},
        "runahead_min_latency_ms": runahead, "verified_rows_vs_oracle": verified, "cpu_baseline": None,
    }
    if not args.no_cpu_baseline and world == 1:
        res["cpu_baseline"], res["cpu_baseline_fw"] = cpu_baseline_c5(g, T, args.cpu_budget)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
