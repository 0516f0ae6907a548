"""GPU: the runahead min-reduce (K5, topology.c:1374-1385 minimumPathLatency) through the
C-ABI, on both launch shapes (one workgroup up to 2^20 values, grid + atomics above)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from shadow_amd import route
    from shadow_amd.graph import internet_like
    return route.RouteEngine(internet_like(200, 2, seed=5))


@pytest.mark.parametrize("count", [1, 7, 2000, 50_000, (1 << 20), (1 << 20) + 1, 3_000_000])
def test_min_reduce_sizes(eng, count):
    import torch
    rng = np.random.default_rng(count)
    v = rng.integers(1, 100_000, size=count).astype(np.float64) + 0.5
    v[rng.integers(0, count, size=max(1, count // 100))] = np.nan  # unreachable rows
    k = int(rng.integers(0, count))
    v[k] = 0.25
    d = torch.from_numpy(v).cuda()
    out = torch.empty(1, dtype=torch.float64, device="cuda")
    eng.min_reduce_async(d, out)
    eng.sync()
    assert out.item() == np.nanmin(v) == 0.25


def test_min_reduce_no_finite_values(eng):
    import torch
    for v in (np.array([], np.float64), np.full(5, np.inf), np.full(3, np.nan)):
        d = torch.from_numpy(v).cuda() if len(v) else torch.empty(0, dtype=torch.float64, device="cuda")
        out = torch.zeros(1, dtype=torch.float64, device="cuda")
        eng.min_reduce_async(d, out)
        eng.sync()
        assert out.cpu().numpy().view(np.uint64)[0] == np.uint64(0xFFFFFFFFFFFFFFFF)
