"""Two processes on the one GPU of the box, gloo between them: each rank computes its
plan rows with the HIP engine (seeded, multi-GPU plan), the rows and the runahead min go
through torch.distributed, and rank 0 checks the gathered latency AND reliability tables
against the oracle.  (The 8-GPU runs use the same plumbing over RCCL.)"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    torch.cuda.init()  # torch's HIP runtime before the engine's (see conftest)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["SHD_ROUTE_KERNEL"] = "kd"
    os.environ["SHD_ROUTE_KDGRID"] = "7"  # few workgroup slots: few forced roots, deep seed chains
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from shadow_amd import route
    from shadow_amd.graph import internet_like
    from shadow_amd.shard import allgather_rows, runahead_min
    g = internet_like(300, 3, seed=41, name="mp")
    T = g.targets()
    eng = route.RouteEngine(g)
    plan = eng.plan(T, world, rank)
    dev = torch.device("cuda", 0)
    nr = plan.info["rows"]
    d_tgt = torch.from_numpy(T.astype(np.int32)).to(dev)
    d_lat = torch.empty((max(nr, 1), len(T)), dtype=torch.float64, device=dev)
    d_rel = torch.empty_like(d_lat)
    d_min = torch.full((max(nr, 1),), float("inf"), dtype=torch.float64, device=dev)
    plan.rows_async(d_tgt, d_lat, d_rel, d_min, dispatch=False)
    eng.sync()
    m = torch.tensor([float(d_min[:nr].min().item()) if nr else float("inf")], dtype=torch.float64)
    runahead_min(m, dist)
    blk = torch.tensor([nr], dtype=torch.int64)
    dist.all_reduce(blk, op=dist.ReduceOp.MAX)
    n_total = int(blk.item()) * world
    lat = allgather_rows(d_lat[:nr].cpu(), n_total, dist)
    rel = allgather_rows(d_rel[:nr].cpu(), n_total, dist)
    pos = allgather_rows(torch.from_numpy(np.pad(plan.positions.astype(np.int64), (0, int(blk.item()) - nr),
                                                 constant_values=-1)).reshape(-1, 1), n_total, dist)
    if rank == 0:
        q.put((lat.numpy(), rel.numpy(), pos.numpy().ravel(), float(m.item()), int(plan.info["seeded"])))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_hip_rows_gathered(oracle_mod):
    import torch.multiprocessing as mp
    from shadow_amd.graph import internet_like
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    lat, rel, pos, mn, seeded = q.get(timeout=180)
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    assert seeded == 1
    g = internet_like(300, 3, seed=41, name="mp")
    T = g.targets()
    keep = pos >= 0
    assert sorted(pos[keep].tolist()) == list(range(len(T)))
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(T[pos[keep]], T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat[keep], olat) and np.array_equal(rel[keep], orel)
    assert mn == olat.min()


def _lm_worker(rank, world, port, q):
    """A landmark-only plan split over the ranks (round 6): each rank computes its share of
    the landmark rows, the shares are all-gathered (gloo here, staged through host memory;
    RCCL in place on the GPU nodes), then the job records and the rows."""
    import torch
    import torch.distributed as dist
    torch.cuda.init()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["SHD_ROUTE_KERNEL"] = "kd"  # (a 3000-vertex graph would take KBF)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from shadow_amd import route
    from shadow_amd.graph import internet_like
    from shadow_amd.shard import allgather_rows, bind_landmark_store, exchange_landmarks
    g = internet_like(3000, 3, seed=77, name="ba3000")
    T = g.targets()
    eng = route.RouteEngine(g)
    plan = eng.plan(T, world, rank)
    dev = torch.device("cuda", 0)
    lm = plan.landmarks()
    assert lm is not None and plan.info["launches"] == 4, plan.info
    store = bind_landmark_store(plan, world, dev)
    # poison the other ranks' shares: only the exchange can restore them
    cnt = store["share"]
    for k in range(world):
        if k != rank:
            store["drow"][k * cnt:(k + 1) * cnt] = 7
    nr = plan.info["rows"]
    d_tgt = torch.from_numpy(T.astype(np.int32)).to(dev)
    d_lat = torch.empty((max(nr, 1), len(T)), dtype=torch.float64, device=dev)
    d_rel = torch.empty_like(d_lat)
    d_min = torch.full((max(nr, 1),), float("inf"), dtype=torch.float64, device=dev)
    plan.refresh_async(what=route.REFRESH_MINE)
    eng.sync()
    exchange_landmarks(store, dist)
    plan.refresh_async(what=route.REFRESH_JOBS)
    plan.rows_async(d_tgt, d_lat, d_rel, d_min, dispatch=False, reuse=True)
    eng.sync()
    blk = torch.tensor([nr], dtype=torch.int64)
    dist.all_reduce(blk, op=dist.ReduceOp.MAX)
    n_total = int(blk.item()) * world
    lat = allgather_rows(d_lat[:nr].cpu(), n_total, dist)
    rel = allgather_rows(d_rel[:nr].cpu(), n_total, dist)
    pos = allgather_rows(torch.from_numpy(np.pad(plan.positions.astype(np.int64), (0, int(blk.item()) - nr),
                                                 constant_values=-1)).reshape(-1, 1), n_total, dist)
    if rank == 0:
        q.put((lat.numpy(), rel.numpy(), pos.numpy().ravel(), lm["count"], lm["nland"]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_landmark_split(oracle_mod):
    import torch.multiprocessing as mp
    from shadow_amd.graph import internet_like
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    lat, rel, pos, cnt, nland = q.get(timeout=240)
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert cnt == nland // 2
    g = internet_like(3000, 3, seed=77, name="ba3000")
    T = g.targets()
    keep = pos >= 0
    assert sorted(pos[keep].tolist()) == list(range(len(T)))
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(T[pos[keep]], T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat[keep], olat) and np.array_equal(rel[keep], orel)
