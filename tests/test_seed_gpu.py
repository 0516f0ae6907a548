"""GPU parity of seeded KD rows (shd_route_plan_* / sssp_delta.hpp seeded mode).

A seeded row starts from w(s,u) + d_u(v) for a neighbour u whose row is already in the
row store, and settles the parents of the vertices that keep that distance from u's
parent records plus the tie events of the expansion.  Everything must stay bit-exact
against the oracle (engine tie rule), including: many launches (deep seed forests),
workgroups running many rows back to back (small grid), tie-event lists that overflow
(the row reruns unseeded), directed graphs (plans fall back to plain rows), rows seeded
from host-computed landmark rows or two-hop rows, and the full C3/C4 tables against the
committed golden row digests.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from shadow_amd.graph import config

from tests.test_kd_gpu import _graph

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture
def kd(monkeypatch):
    monkeypatch.setenv("SHD_ROUTE_KERNEL", "kd")
    monkeypatch.setenv("SHD_ROUTE_KDGRID", "7")
    monkeypatch.delenv("SHD_ROUTE_SEED", raising=False)
    monkeypatch.delenv("SHD_ROUTE_EVCAP", raising=False)
    monkeypatch.delenv("SHD_ROUTE_SEEDS", raising=False)
    return monkeypatch


@pytest.mark.parametrize("seeds,evcap", [(None, None), ("1", None), ("3", None), (None, "0"), ("3", "2")])
@pytest.mark.parametrize("name", ["ba400", "ties", "chain", "c2"])
def test_seeded_rows_bitexact(oracle_mod, kd, name, seeds, evcap):
    """seeds: rows started from 1..3 neighbour rows (default 2); evcap 0 / 2: every row
    with more tie events than that reruns unseeded."""
    from shadow_amd import route
    if evcap is not None:
        kd.setenv("SHD_ROUTE_EVCAP", evcap)
    if seeds is not None:
        kd.setenv("SHD_ROUTE_SEEDS", seeds)
    g = _graph(name)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 4
    T = g.targets()
    S = T if name != "c2" else T[::3]
    plan = eng.plan(S)
    assert plan.info["seeded"] == 1 and plan.info["levels"] > 2 and plan.info["stored_rows"] > 0
    assert np.array_equal(plan.positions, np.arange(len(S)))
    lat, rel, mn = eng.rows(S, T, dispatch=False)  # host rows take the seeded plan
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(S, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))


@pytest.mark.parametrize("pdelta", ["1", "7", "1000"])
@pytest.mark.parametrize("name", ["ba400", "c2"])
def test_plan_bucket_width_bitexact(oracle_mod, kd, name, pdelta):
    """A plan's rows may take a narrower bucket width than the context's (round 6: ranks of a
    split of 1024-thread rows take the 12th percentile); any width up to the context's is
    exact (the light in-CSR holds the in-arcs below the context's width, a superset), and a
    wider request is clamped to the context's."""
    from shadow_amd import route
    kd.setenv("SHD_ROUTE_PLAN_DELTA", pdelta)
    g = _graph(name)
    eng = route.RouteEngine(g)
    T = g.targets()
    S = T if name != "c2" else T[::3]
    plan = eng.plan(S)
    assert plan.info["seeded"] == 1
    assert plan.info["delta"] == min(int(pdelta), eng.info["reserved"]), (plan.info, eng.info["reserved"])
    lat, rel, mn = _plan_rows(eng, plan, T)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(S[plan.positions], T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))


def test_seeded_equals_unseeded_shuffled_sources(kd):
    """Sources in arbitrary order with repeats: seeding picks seeds among the listed rows."""
    from shadow_amd import route
    g = _graph("ba400")
    T = g.targets()
    rng = np.random.default_rng(3)
    S = np.concatenate([rng.permutation(T), T[:17]]).astype(np.int32)
    lat, rel, mn = route.RouteEngine(g).rows(S, T, dispatch=False)
    kd.setenv("SHD_ROUTE_SEED", "0")
    lat0, rel0, mn0 = route.RouteEngine(g).rows(S, T, dispatch=False)
    assert np.array_equal(lat, lat0) and np.array_equal(rel, rel0) and np.array_equal(mn, mn0)


def test_plans_independent_of_host_workers(oracle_mod, kd):
    """The plan does not depend on where its seed choices are made: on the device (default),
    on the host workers with the sequential pass consuming them as they finish
    (SHD_ROUTE_GPUCHOICE=0), choices first and the pass after them (SHD_ROUTE_PIPE=0), and two
    host-choice plans at once on two contexts (the second finds the shared workers busy and
    starts its own)."""
    import threading
    from shadow_amd import route
    g = _graph("c2")
    T = g.targets()
    eng = route.RouteEngine(g)
    ref = eng.plan(T).info
    assert ref["seeded"] == 1
    kd.setenv("SHD_ROUTE_GPUCHOICE", "0")  # seed choices on the host workers, not the device
    assert eng.plan(T).info == ref
    kd.setenv("SHD_ROUTE_PIPE", "0")
    assert eng.plan(T).info == ref
    kd.delenv("SHD_ROUTE_PIPE")
    engs = [route.RouteEngine(g) for _ in range(2)]
    out = [None, None]

    def run(i):
        out[i] = engs[i].plan(T).info

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert out[0] == ref and out[1] == ref
    lat, rel, _ = engs[1].rows(T[::5], T, dispatch=False)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(T[::5], T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat) and np.array_equal(rel, orel)


@pytest.mark.parametrize("cfg,world", [("c2", 3), ("c3", 8)])
def test_partition_forest_device_equals_host(kd, cfg, world):
    """A multi-GPU plan's seed forest (every row's best seed, which decides the partition) is
    computed on the device by default; SHD_ROUTE_GPUCHOICE=0 computes it (and the seed
    choices) with the host scan.  Every rank's rows and plan shape must be the same."""
    from shadow_amd import route
    g = config(cfg)
    T = g.targets()
    eng = route.RouteEngine(g)
    dev = []
    for r in range(world):
        p = eng.plan(T, world, r)
        dev.append((p.info, p.positions.copy()))
        p.close()
    kd.setenv("SHD_ROUTE_GPUCHOICE", "0")

    def shape(info):  # (a device-built landmark-only plan recomputes its landmark rows in its
        return {k: v for k, v in info.items() if k not in ("store_bytes", "launches")}  # launches
    for r in range(world):
        p = eng.plan(T, world, r)
        assert shape(p.info) == shape(dev[r][0])
        assert np.array_equal(p.positions, dev[r][1])
        p.close()


def test_directed_plan_falls_back(oracle_mod, kd):
    from shadow_amd import route
    g = _graph("dir")
    eng = route.RouteEngine(g)
    T = g.targets()
    plan = eng.plan(T)
    assert plan.info["seeded"] == 0 and plan.info["levels"] == 1
    lat, rel, _ = eng.rows(T, T, dispatch=False)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(T, T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat) and np.array_equal(rel, orel)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float64).tobytes()).hexdigest()


def _digest16(row):
    return hashlib.sha256(row.tobytes()).digest()[:16]


def _check_every_row(d_lat, d_rel, d_min, row_src, gold, block=2048):
    """Every row of the device table against the golden digests (tests/golden/
    full_digests.npz: first 16 bytes of SHA-256 of each oracle row): rows come over in
    pinned blocks and are hashed on host threads (hashlib releases the GIL)."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    src = gold["src"]
    k_of = {int(v): k for k, v in enumerate(src)}
    ks = np.array([k_of[int(s)] for s in row_src])
    nr, nt = len(row_src), d_lat.shape[1]
    assert np.array_equal(d_min[:nr].cpu().numpy(), gold["row_min"][ks])
    bl = torch.empty((block, nt), dtype=torch.float64, pin_memory=True)
    br = torch.empty((block, nt), dtype=torch.float64, pin_memory=True)
    bad = []
    with ThreadPoolExecutor(16) as ex:
        for r0 in range(0, nr, block):
            r1 = min(nr, r0 + block)
            bl[: r1 - r0].copy_(d_lat[r0:r1])
            br[: r1 - r0].copy_(d_rel[r0:r1])
            L, R = bl.numpy(), br.numpy()
            dl = list(ex.map(lambda i: _digest16(L[i]), range(r1 - r0)))
            dr = list(ex.map(lambda i: _digest16(R[i]), range(r1 - r0)))
            for i in range(r1 - r0):
                k = ks[r0 + i]
                if dl[i] != gold["lat_d"][k].tobytes() or dr[i] != gold["rel_d"][k].tobytes():
                    bad.append(int(row_src[r0 + i]))
    assert not bad, (len(bad), bad[:16])
    return nr


def _gold(cfg):
    z = np.load(os.path.join(GOLD, "full_digests.npz"))
    return {k: z[f"{cfg}__{k}"] for k in ("src", "lat_d", "rel_d", "row_min")}


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_full_table_every_row(monkeypatch, cfg):
    """The whole C3 (9,337 x 9,337) / C4 (50k x 50k, 40 GB) table by one seeded plan in
    HBM: EVERY row's latency and reliability against the oracle's row digests (C3 9,337
    rows, C4 50,000 rows), every row minimum, the sampled rows' SHA-256 of
    rows_digests.json, and the whole latency table's symmetry (undirected graph)."""
    import torch
    from shadow_amd import route
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    monkeypatch.delenv("SHD_ROUTE_KDGRID", raising=False)
    monkeypatch.delenv("SHD_ROUTE_SEED", raising=False)
    gold = _gold(cfg)
    dig = json.load(open(os.path.join(GOLD, "rows_digests.json")))[cfg]
    g = config(cfg)
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 4
    T = g.targets()
    assert np.array_equal(T, gold["src"])
    plan = eng.plan(T)
    assert plan.info["seeded"] == 1 and np.array_equal(plan.positions, np.arange(len(T)))
    dev = torch.device("cuda", 0)
    d_tgt = torch.from_numpy(T.astype(np.int32)).to(dev)
    d_lat = torch.empty((len(T), len(T)), dtype=torch.float64, device=dev)
    d_rel = torch.empty_like(d_lat)
    d_min = torch.empty(len(T), dtype=torch.float64, device=dev)
    plan.rows_async(d_tgt, d_lat, d_rel, d_min, dispatch=False)
    eng.sync()
    assert _check_every_row(d_lat, d_rel, d_min, plan.sources, gold) == len(T)
    row_of = {int(v): i for i, v in enumerate(T)}
    idx = torch.tensor([row_of[r["src"]] for r in dig["rows"]], device=dev)
    lat, rel = d_lat[idx].cpu().numpy(), d_rel[idx].cpu().numpy()
    for k, r in enumerate(dig["rows"]):
        assert _sha(lat[k]) == r["lat_sha"] and _sha(rel[k]) == r["rel_sha"], (cfg, r["src"])
    # undirected: lat(s,t) == lat(t,s) over the whole table, tile against transposed tile
    tb = 8192
    for i0 in range(0, len(T), tb):
        for j0 in range(i0, len(T), tb):
            a = d_lat[i0:i0 + tb, j0:j0 + tb]
            b = d_lat[j0:j0 + tb, i0:i0 + tb]
            assert torch.equal(a, b.t()), (i0, j0)
    del d_lat, d_rel
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cfg,mask", [("c3", 2), ("c3", 4), ("c3", 6), ("c4", 2), ("c4", 4)])
def test_seed_subsets_every_row(monkeypatch, cfg, mask):
    """Seed dropping (KD_SEEDSPIN: a seed after the first not ready in time leaves the job)
    claims ANY subset of a row's seeds gives exact rows.  SHD_ROUTE_SEEDDROP forces a chosen
    subset on every seeded job -- bit 1 drops the second seed, bit 2 the third, 6 both --
    and every row of the C3 / C4 table must still equal the oracle's digests."""
    import torch
    from shadow_amd import route
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    monkeypatch.delenv("SHD_ROUTE_KDGRID", raising=False)
    monkeypatch.delenv("SHD_ROUTE_SEED", raising=False)
    monkeypatch.setenv("SHD_ROUTE_SEEDDROP", str(mask))
    gold = _gold(cfg)
    g = config(cfg)
    eng = route.RouteEngine(g)
    T = g.targets()
    plan = eng.plan(T)
    assert plan.info["seeded"] == 1
    dev = torch.device("cuda", 0)
    d_tgt = torch.from_numpy(T.astype(np.int32)).to(dev)
    d_lat = torch.empty((len(T), len(T)), dtype=torch.float64, device=dev)
    d_rel = torch.empty_like(d_lat)
    d_min = torch.empty(len(T), dtype=torch.float64, device=dev)
    plan.rows_async(d_tgt, d_lat, d_rel, d_min, dispatch=False)
    eng.sync()
    assert _check_every_row(d_lat, d_rel, d_min, plan.sources, gold) == len(T)
    del d_lat, d_rel
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,landmarks", [(20, None), (40, None), (300, "1"), (300, "64"), (300, "0")])
def test_landmark_seeded_roots(oracle_mod, monkeypatch, n, landmarks):
    """Full grid (every workgroup slot starts with a landmark-seeded row): graphs smaller
    than the landmark set (every vertex a landmark: roots seeded by their own exact row),
    one landmark, many, none; two-hop fills.  Bit-exact against the oracle."""
    from shadow_amd import route
    from shadow_amd.graph import internet_like
    monkeypatch.setenv("SHD_ROUTE_KERNEL", "kd")
    monkeypatch.delenv("SHD_ROUTE_KDGRID", raising=False)
    monkeypatch.delenv("SHD_ROUTE_SEED", raising=False)
    if landmarks is not None:
        monkeypatch.setenv("SHD_ROUTE_LANDMARKS", landmarks)
    g = internet_like(n, 2, seed=40 + n, name=f"ba{n}")
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 4
    T = g.targets()
    plan = eng.plan(T)
    if landmarks != "0":
        # every row is a first row here (the grid has more slots than there are rows): all
        # seeded from landmark rows
        assert plan.info["seeded"] == 1 and plan.info["roots"] == 0
    else:
        assert plan.info["seeded"] == 0  # all rows unseeded: no row store, plain rows
    lat, rel, mn = _plan_rows(eng, plan, T)
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(T[plan.positions], T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat)
    assert np.array_equal(rel, orel)
    assert np.array_equal(mn, olat.min(axis=1))


def test_c3_writer_ring_no_stall(monkeypatch):
    """256-thread rows (three compute waves + the writer wave, a 256-record ring): with
    bucket width 60 on C3 the writer's full 256-record pass used to wait on a reservation
    whose owner waited for ring space, both spinning to their caps (~110 ms per launch in
    2 of 3 runs).  The kernel's wait counters must stay far below a stall's, and the
    golden rows must hold."""
    import torch
    from shadow_amd import route
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    monkeypatch.delenv("SHD_ROUTE_KDGRID", raising=False)
    monkeypatch.delenv("SHD_ROUTE_SEED", raising=False)
    monkeypatch.setenv("SHD_ROUTE_DELTA", "60")
    dig = json.load(open(os.path.join(GOLD, "rows_digests.json")))["c3"]
    g = config("c3")
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 4 and eng.info["block"] == 256
    T = g.targets()
    plan = eng.plan(T)
    dev = torch.device("cuda", 0)
    d_tgt = torch.from_numpy(T.astype(np.int32)).to(dev)
    d_lat = torch.empty((len(T), len(T)), dtype=torch.float64, device=dev)
    d_rel = torch.empty_like(d_lat)
    d_min = torch.empty(len(T), dtype=torch.float64, device=dev)
    plan.rows_async(d_tgt, d_lat, d_rel, d_min, dispatch=False)
    eng.sync()
    eng.kd_stats(reset=True)
    for _ in range(6):
        plan.rows_async(d_tgt, d_lat, d_rel, d_min, dispatch=False)
        eng.sync()
    # the kernel's own longest waits (s_sleep rounds), box-independent: a stall spins both
    # sides of the ring to their 2^22 caps (~110 ms each); a healthy wait is hundreds
    ring, writer, slot = eng.kd_stats(reset=True)
    assert max(ring, writer, slot) < 1 << 16, (ring, writer, slot)
    row_of = {int(v): i for i, v in enumerate(T)}
    idx = torch.tensor([row_of[r["src"]] for r in dig["rows"]], device=dev)
    lat, rel = d_lat[idx].cpu().numpy(), d_rel[idx].cpu().numpy()
    for k, r in enumerate(dig["rows"]):
        assert _sha(lat[k]) == r["lat_sha"] and _sha(rel[k]) == r["rel_sha"], r["src"]


def _plan_rows(eng, plan, T, reuse=False):
    import torch
    dev = torch.device("cuda", 0)
    d_tgt = torch.from_numpy(np.ascontiguousarray(T, np.int32)).to(dev)
    nr = max(1, plan.info["rows"])
    d_lat = torch.empty((nr, len(T)), dtype=torch.float64, device=dev)
    d_rel = torch.empty_like(d_lat)
    d_min = torch.empty(nr, dtype=torch.float64, device=dev)
    plan.rows_async(d_tgt, d_lat, d_rel, d_min, dispatch=False, reuse=reuse)
    eng.sync()
    k = plan.info["rows"]
    return d_lat[:k].cpu().numpy(), d_rel[:k].cpu().numpy(), d_min[:k].cpu().numpy()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("name", ["ba400", "c2"])
def test_partitioned_plans_cover_and_match(kd, name, world):
    """Multi-GPU plans (one per rank, all run here on device 0): the ranks' rows cover the
    source list exactly once, every rank's seeds are its own rows or its helper rows
    (top of the seed forest), and each row equals the single-GPU table's row."""
    from shadow_amd import route
    g = _graph(name)
    eng = route.RouteEngine(g)
    T = g.targets()
    ref_lat, ref_rel, ref_mn = eng.rows(T, T, dispatch=False)
    seen = []
    for r in range(world):
        plan = eng.plan(T, world, r)
        assert plan.info["seeded"] == 1 and plan.info["world"] == world and plan.info["rank"] == r
        assert plan.info["helpers"] > 0
        lat, rel, mn = _plan_rows(eng, plan, T)
        pos = plan.positions
        assert np.array_equal(lat, ref_lat[pos]) and np.array_equal(rel, ref_rel[pos]) and np.array_equal(mn, ref_mn[pos])
        seen.extend(pos.tolist())
    assert sorted(seen) == list(range(len(T)))


def test_c4_eight_rank_plans_balanced_and_golden(monkeypatch):
    """C4 split over 8 ranks: blocks within 10% of 6,250 rows, few helper rows, and the
    golden sampled rows come out of whichever rank owns them bit-exact."""
    from shadow_amd import route
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    monkeypatch.delenv("SHD_ROUTE_KDGRID", raising=False)
    dig = json.load(open(os.path.join(GOLD, "rows_digests.json")))["c4"]
    g = config("c4")
    eng = route.RouteEngine(g)
    T = g.targets()
    want = {r["src"]: r for r in dig["rows"]}
    found = 0
    for r in range(8):
        plan = eng.plan(T, 8, r)
        assert abs(plan.info["rows"] - 6250) <= 625, plan.info
        # (every plan takes the context's bucket width: 38 on C4, round 6 A/B in DESIGN 6)
        assert plan.info["delta"] == 38 and eng.info["reserved"] == 38, (plan.info, eng.info["reserved"])
        assert plan.info["helpers"] <= 2500, plan.info
        mine = [k for k, s in enumerate(plan.sources) if int(s) in want]
        if not mine:
            continue
        lat, rel, mn = _plan_rows(eng, plan, T)
        for k in mine:
            w = want[int(plan.sources[k])]
            assert _sha(lat[k]) == w["lat_sha"] and _sha(rel[k]) == w["rel_sha"] and mn[k] == w["row_min"]
            found += 1
    assert found == len(want)


def test_c3_eight_rank_plans_every_row(monkeypatch):
    """BASELINE configs[2] (Tor-scale C3, "sources sharded across 8 GPUs"): the 8 ranks'
    plans, all run here on device 0, cover the 9,337 sources exactly once, and EVERY row
    of every rank equals the oracle's row digest (full_digests.npz), row minimum included."""
    import torch
    from shadow_amd import route
    monkeypatch.delenv("SHD_ROUTE_KERNEL", raising=False)
    monkeypatch.delenv("SHD_ROUTE_KDGRID", raising=False)
    monkeypatch.delenv("SHD_ROUTE_SEED", raising=False)
    gold = _gold("c3")
    g = config("c3")
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 4
    T = g.targets()
    dev = torch.device("cuda", 0)
    d_tgt = torch.from_numpy(T.astype(np.int32)).to(dev)
    seen = []
    for r in range(8):
        plan = eng.plan(T, 8, r)
        assert plan.info["seeded"] == 1 and plan.info["world"] == 8 and plan.info["rank"] == r
        assert abs(plan.info["rows"] - len(T) / 8) <= 0.15 * len(T) / 8, plan.info
        nr = max(1, plan.info["rows"])
        d_lat = torch.empty((nr, len(T)), dtype=torch.float64, device=dev)
        d_rel = torch.empty_like(d_lat)
        d_min = torch.empty(nr, dtype=torch.float64, device=dev)
        plan.rows_async(d_tgt, d_lat, d_rel, d_min, dispatch=False)
        eng.sync()
        assert _check_every_row(d_lat, d_rel, d_min, plan.sources, gold) == plan.info["rows"]
        seen.extend(plan.positions.tolist())
    assert sorted(seen) == list(range(len(T)))


@pytest.mark.parametrize("world,vloss", [(1, False), (1, True), (3, False)])
def test_landmark_only_plans(oracle_mod, monkeypatch, world, vloss):
    """Landmark-only plans (round 5: 256-thread contexts with n >= 2048, and ranks with at
    most 1.5 rows per workgroup slot): every row seeded from its 3 nearest of the landmark
    rows (1024 of the 3000 vertices), all at level 0, a rank taking every
    world-th row.  Bit-exact against the oracle,
    the ranks covering the source list exactly once; the device-built plan (order and jobs
    on the device, the landmark rows borrowed as the store) gives the rows of the host builds
    (SHD_ROUTE_GPUCHOICE=0: host seeds; SHD_ROUTE_PLANDEV=0: device seeds, host jobs)."""
    from shadow_amd import route
    from shadow_amd.graph import internet_like
    monkeypatch.setenv("SHD_ROUTE_KERNEL", "kd")  # (a 3000-vertex graph would take KBF)
    monkeypatch.delenv("SHD_ROUTE_KDGRID", raising=False)
    monkeypatch.delenv("SHD_ROUTE_SEED", raising=False)
    monkeypatch.delenv("SHD_ROUTE_LANDMARKS", raising=False)
    g = internet_like(3000, 3, seed=77, vloss=vloss, name="ba3000")
    eng = route.RouteEngine(g)
    assert eng.info["kernel"] == 4 and eng.info["block"] == 256
    T = g.targets()
    og = oracle_mod.OracleGraph(g)
    seen = []
    for r in range(world):
        plan = eng.plan(T, world, r)
        info = dict(plan.info)
        assert info["seeded"] == 1 and info["levels"] == 1 and info["helpers"] == 0 and info["stored_rows"] == 0, info
        lat, rel, mn = _plan_rows(eng, plan, T)
        pos = plan.positions.copy()
        olat, orel, _, _ = og.source_rows(T[pos], T, oracle_mod.TIE_MINKEY)
        assert np.array_equal(lat, olat) and np.array_equal(mn, olat.min(axis=1))
        if vloss:
            # vertex factors: the walks fold from (1.0 * f_s) * f_t, the reference's order
            # (topology.c:1443-1462, then :1499): bit-exact against the oracle, and against
            # the engine's unseeded rows
            assert np.array_equal(rel, orel, equal_nan=True)
            monkeypatch.setenv("SHD_ROUTE_SEED", "0")
            _, rel0, _ = route.RouteEngine(g).rows(T[pos][::7], T, dispatch=False)
            monkeypatch.delenv("SHD_ROUTE_SEED")
            assert np.array_equal(rel[::7], rel0)
        else:
            assert np.array_equal(rel, orel)
        seen.extend(pos.tolist())
        # the device-built plan (default) recomputes its landmark rows, queue order and jobs
        # in every rows call (round 6: four launches); reusing the last refresh, or refreshing
        # explicitly first, gives the same rows
        assert info["launches"] == 4 and info["store_bytes"] > 0, info
        lat_r, rel_r, _ = _plan_rows(eng, plan, T, reuse=True)
        assert np.array_equal(lat_r, lat) and np.array_equal(rel_r, rel, equal_nan=True)
        plan.refresh_async()
        lat_r, rel_r, _ = _plan_rows(eng, plan, T, reuse=True)
        assert np.array_equal(lat_r, lat) and np.array_equal(rel_r, rel, equal_nan=True)
        plan.close()
        # the host builds (host seeds, or device seeds with host jobs) take the landmark rows
        # computed when the plan is made into their own store
        for knob in ("SHD_ROUTE_GPUCHOICE", "SHD_ROUTE_PLANDEV"):
            monkeypatch.setenv(knob, "0")
            plan = eng.plan(T, world, r)
            i2 = dict(plan.info)
            skip = ("store_bytes", "launches")
            assert i2["launches"] == 1 and i2["store_bytes"] > 0, (knob, i2)
            assert {k: v for k, v in i2.items() if k not in skip} == {k: v for k, v in info.items() if k not in skip}, (knob, i2)
            assert np.array_equal(plan.positions, pos)
            lat2, rel2, _ = _plan_rows(eng, plan, T)
            assert np.array_equal(lat2, lat) and np.array_equal(rel2, rel)
            plan.close()
            monkeypatch.delenv(knob)
    assert sorted(seen) == list(range(len(T)))


@pytest.mark.parametrize("lm2", ["64", "256"])
def test_landmark_rows_two_levels(oracle_mod, monkeypatch, lm2):
    """SHD_ROUTE_LM2=k: a landmark-only plan's landmark rows in two levels (the first k
    unseeded, the rest seeded from their nearest of those): the landmark rows are exact
    either way, so the table is the oracle's."""
    from shadow_amd import route
    from shadow_amd.graph import internet_like
    monkeypatch.setenv("SHD_ROUTE_KERNEL", "kd")
    monkeypatch.delenv("SHD_ROUTE_KDGRID", raising=False)
    monkeypatch.delenv("SHD_ROUTE_SEED", raising=False)
    monkeypatch.setenv("SHD_ROUTE_LM2", lm2)
    g = internet_like(3000, 3, seed=77, name="ba3000")
    eng = route.RouteEngine(g)
    T = g.targets()
    plan = eng.plan(T)
    assert plan.info["launches"] == 4, plan.info
    lat, rel, mn = _plan_rows(eng, plan, T)
    pos = plan.positions
    olat, orel, _, _ = oracle_mod.OracleGraph(g).source_rows(T[pos], T, oracle_mod.TIE_MINKEY)
    assert np.array_equal(lat, olat) and np.array_equal(rel, orel) and np.array_equal(mn, olat.min(axis=1))
