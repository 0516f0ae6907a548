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


def _payload_worker(rank, world, port, q):
    """Each rank owns an arbitrary (interleaved) set of rows, as a seed-forest partition
    does; packs their upper triangles (u16 latency + f64 rel), all-gathers the segments
    (padded to the largest) and rank 0 reads every pair back through TriangleIndex."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import OracleGraph, TIE_MINKEY
    from shadow_amd.shard import TriangleIndex, allgather_payload, pack_triangle_host, tri_offsets
    g = internet_like(90, 2, seed=21)
    T = g.targets()
    na = len(T)
    rng = np.random.default_rng(7)
    owner = rng.integers(0, world, size=na)
    pos = np.flatnonzero(owner == rank)[::-1].copy()  # any row order
    lat, rel, _, _ = OracleGraph(g).source_rows(T[pos], T, TIE_MINKEY)
    L, R = pack_triangle_host(lat, rel, pos, na, lat16=True)
    _, tot = tri_offsets(pos, na)
    seg_t = torch.tensor([tot], dtype=torch.int64)
    dist.all_reduce(seg_t, op=dist.ReduceOp.MAX)
    seg = int(seg_t.item())
    pos_by_rank = [None] * world
    dist.all_gather_object(pos_by_rank, pos)
    gl, gr = allgather_payload(torch.from_numpy(L.view(np.int16)), torch.from_numpy(R), seg, dist)
    if rank == 0:
        idx = TriangleIndex(pos_by_rank, na, seg)
        q.put((gl.numpy().view(np.uint16), gr.numpy(), idx.start, seg, tot))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_triangle_payload_gather(world, oracle_mod):
    """The reduced table-assembly payload (bench.py --gpus N strong): every unordered
    pair of the attached set arrives once, latency exact as u16, reliability bit-exact,
    and each pair's value is the row of its smaller position (first writer over both
    directions, topology.c:1307-1336)."""
    from shadow_amd.shard import TriangleIndex, decode_lat16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_payload_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gl, gr, start, seg, _ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = internet_like(90, 2, seed=21)
    T = g.targets()
    na = len(T)
    ref, rref, _, _ = oracle_mod.OracleGraph(g).source_rows(T, T, oracle_mod.TIE_MINKEY)
    ii, jj = np.triu_indices(na)
    k = start[ii] + (jj - ii)
    assert len(np.unique(k)) == len(k) and k.max() < world * seg
    assert np.array_equal(decode_lat16(gl[k]), ref[ii, jj], equal_nan=True)
    assert np.array_equal(gr[k], rref[ii, jj])
    assert gl.nbytes + gr.nbytes <= 0.5 * 16 * na * na * world / world + 16 * world * na
