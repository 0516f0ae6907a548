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


def _lm_worker(rank, world, port, q):
    """Each rank fills only its share of a landmark store (the hub vertices' exact distance
    rows as u16, a per-vertex record word), then exchange_landmarks all-gathers the shares."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import OracleGraph, TIE_MINKEY
    from shadow_amd.shard import exchange_landmarks, landmark_exchange_bytes
    g = internet_like(120, 2, seed=23)
    T = g.targets()
    nland = 10  # (not a multiple of 3: the padded last share)
    deg = np.bincount(np.concatenate([g.src, g.dst]), minlength=g.n)
    hubs = sorted(range(g.n), key=lambda v: (-deg[v], v))[:nland]
    rs = (g.n + 2 + 7) & ~7
    cnt = -(-nland // world)
    store = {"drow": torch.full((cnt * world, rs), -1, dtype=torch.int16),
             "prow": torch.full((cnt * world, rs), -1, dtype=torch.int32),
             "share": cnt, "nland": nland, "row_stride": rs}
    og = OracleGraph(g)
    for k in range(rank * cnt, min(nland, (rank + 1) * cnt)):
        lat, _, _, _ = og.source_rows(np.array([hubs[k]], np.int32), T, TIE_MINKEY)
        store["drow"][k, :g.n] = torch.from_numpy(lat[0].astype(np.int32)).to(torch.int16)
        store["prow"][k, :g.n] = torch.arange(g.n, dtype=torch.int32) + 1000 * k
    exchange_landmarks(store, dist)
    q.put((rank, store["drow"][:nland, :g.n].numpy().copy(), store["prow"][:nland, :g.n].numpy().copy(),
           landmark_exchange_bytes(store, world)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_landmark_store_exchange(world, oracle_mod):
    """Round 6, multi-GPU landmark-only plans (C3 split over ranks): every rank ends with all
    landmark rows although it computed only its share (bench.py: REFRESH_MINE, then this
    exchange, then REFRESH_JOBS; RCCL all-gather in place on the GPU nodes)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    g = internet_like(120, 2, seed=23)
    T = g.targets()
    deg = np.bincount(np.concatenate([g.src, g.dst]), minlength=g.n)
    hubs = sorted(range(g.n), key=lambda v: (-deg[v], v))[:10]
    og = oracle_mod.OracleGraph(g)
    want, _, _, _ = og.source_rows(np.array(hubs, np.int32), T, oracle_mod.TIE_MINKEY)
    rs = (g.n + 2 + 7) & ~7
    for rank, drow, prow, nbytes in got:
        assert np.array_equal(drow.astype(np.int64), want.astype(np.int64)), rank
        assert np.array_equal(prow, np.arange(g.n)[None, :] + 1000 * np.arange(10)[:, None]), rank
        assert nbytes == (world - 1) * -(-10 // world) * rs * 6
