"""CPU, world_size 2 over gloo: source sharding, runahead all-reduce MIN and the row
all-gather (latency and reliability, also in the bench's in-place form) reproduce the single-process table (rows computed by the oracle here; on
the GPU box the same plumbing carries the HIP rows over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from shadow_amd.graph import internet_like
from shadow_amd.shard import allgather_rows, runahead_min, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import OracleGraph, TIE_MINKEY
    g = internet_like(90, 2, seed=21)
    T = g.targets()
    lo, hi = shard_range(len(T), world, rank)
    og = OracleGraph(g)
    lat, rel, _, _ = og.source_rows(T[lo:hi], T, TIE_MINKEY)
    local_min = torch.tensor([lat.min() if len(lat) else np.inf], dtype=torch.float64)
    runahead_min(local_min, dist)
    full = allgather_rows(torch.from_numpy(lat), len(T), dist)
    # the bench's in-place form: rows written into this rank's block of the full tables
    from shadow_amd.shard import allgather_inplace, full_table
    f_lat, s_lat = full_table(len(T), len(T), world, rank, torch.empty(0, dtype=torch.float64))
    f_rel, s_rel = full_table(len(T), len(T), world, rank, torch.empty(0, dtype=torch.float64))
    s_lat[:hi - lo] = torch.from_numpy(lat)
    s_rel[:hi - lo] = torch.from_numpy(rel)
    allgather_inplace(f_lat, dist)
    allgather_inplace(f_rel, dist)
    if rank == 0:
        q.put((full.numpy(), float(local_min.item()), f_lat[:len(T)].numpy(), f_rel[:len(T)].numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_rows_allgather_and_min(world, oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, mn, glat, grel = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = internet_like(90, 2, seed=21)
    T = g.targets()
    og = oracle_mod.OracleGraph(g)
    ref, rref, _, _ = og.source_rows(T, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(full, ref)
    assert np.array_equal(glat, ref) and np.array_equal(grel, rref)
    assert mn == ref.min()


def test_shard_ranges_cover():
    for n in (1, 7, 2000, 9337):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
