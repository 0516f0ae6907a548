"""shd_route_tri_payload_async (the multi-GPU table-assembly payload) on the device against
its host statement shard.pack_triangle_host, and the LAT16 eligibility: the table's
diagonal holds self-loop latencies, which the CSR's shortest-path bound does not cover, so
a self-loop at or above 0xFFFF ms makes info["lat16"] 0 and a LAT16 request
EUNSUPPORTED (no truncated latency, no collision with the NaN code 0xFFFF)."""
import numpy as np
import pytest

from shadow_amd.graph import Graph, internet_like

pytestmark = pytest.mark.gpu


def _with_self_loops(g: Graph, w):
    """g with every self-loop replaced by one of latency w (a second loop would make it a
    multigraph)."""
    v = np.arange(g.n, dtype=np.int32)
    keep = g.src != g.dst
    return Graph(n=g.n, src=np.concatenate([g.src[keep], v]), dst=np.concatenate([g.dst[keep], v]),
                 latency=np.concatenate([g.latency[keep], np.full(g.n, float(w))]),
                 packetloss=np.concatenate([g.packetloss[keep], np.full(g.n, 0.01)]), name=g.name + "_loops")


def _payload(eng, g, lat16):
    import torch
    from shadow_amd.shard import tri_offsets
    T = g.targets()
    na = len(T)
    dev = torch.device("cuda", 0)
    pos = np.arange(na - 1, -1, -3, dtype=np.int32)  # any row order
    lat, rel, _ = eng.rows(T[pos], T, dispatch=False)
    off, tot = tri_offsets(pos, na)
    d_lat = torch.from_numpy(lat).to(dev)
    d_rel = torch.from_numpy(rel).to(dev)
    out_l = torch.empty(max(tot, 1), dtype=torch.int16 if lat16 else torch.float64, device=dev)
    out_r = torch.empty(max(tot, 1), dtype=torch.float64, device=dev)
    eng.tri_payload_async(d_lat, d_rel, torch.from_numpy(pos).to(dev), torch.from_numpy(off[:-1].copy()).to(dev),
                          na, out_l, out_r, lat16=lat16)
    eng.sync()
    return lat, rel, pos, na, out_l.cpu().numpy()[:tot], out_r.cpu().numpy()[:tot]


@pytest.mark.parametrize("lat16", [True, False])
def test_payload_matches_host_statement(lat16):
    from shadow_amd import route
    from shadow_amd.shard import decode_lat16, pack_triangle_host
    g = _with_self_loops(internet_like(300, 2, seed=5), 40)
    eng = route.RouteEngine(g)
    assert eng.info["lat16"] == 1
    lat, rel, pos, na, L, R = _payload(eng, g, lat16)
    hl, hr = pack_triangle_host(lat, rel, pos, na, lat16=lat16)
    if lat16:
        assert np.array_equal(L.view(np.uint16), hl)
        assert np.array_equal(decode_lat16(L), decode_lat16(hl), equal_nan=True)
    else:
        assert np.array_equal(L, hl, equal_nan=True)
    assert np.array_equal(R, hr, equal_nan=True)


def test_payload_lat16_refused_for_wide_self_loops():
    from shadow_amd import route
    g = _with_self_loops(internet_like(300, 2, seed=5), 70000)
    eng = route.RouteEngine(g)
    assert eng.info["integer_weights"] == 1 and 0 < eng.info["dist_bound"] < 0xFFFF
    assert eng.info["lat16"] == 0  # the diagonal (70000 ms) does not fit u16
    with pytest.raises(route.RouteError):
        _payload(eng, g, True)
    lat, rel, pos, na, L, R = _payload(eng, g, False)  # f64 latencies stay exact
    i = int(np.flatnonzero(pos == na - 1)[0])
    assert lat[i, na - 1] == 70000.0
