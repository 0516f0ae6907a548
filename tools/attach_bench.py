"""Host attachment throughput at Tor scale (CPU, no GPU): 27,000 hosts onto a
10,000-vertex graphml with ip/citycode/countrycode/geocode/type attributes, through the
C index (shd_attach_find_vertex) and, on a sample, through the restatement of the
reference's per-host scan (oracle/attach_ref.py, the GQueue structure of
topology.c:2094-2366; the reference itself also pays 5 igraph attribute lookups per
vertex under the graph lock, so this is a lower bound on its cost)."""
import os
import pathlib
import random
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle.attach_ref import ShadowRandom, find_attachment_vertex  # noqa: E402
from shadow_amd import topology  # noqa: E402
from test_attach import _graphml, _hints  # noqa: E402

topology.load_library()
with tempfile.TemporaryDirectory() as d:
    p = pathlib.Path(d) / "tor.xml"
    ips = _graphml(p, 10_000, 2024)
    idx = topology.AttachIndex(str(p))
    attrs = idx.vertex_attrs()
    rng = random.Random(1)
    hints = [_hints(rng, ips) for _ in range(27_000)]
    r = ShadowRandom(1)
    t0 = time.perf_counter()
    got = [idx.find(r.next_double, **h) for h in hints]
    dt = time.perf_counter() - t0
    k = 60
    r2 = ShadowRandom(1)
    t0 = time.perf_counter()
    ref = [find_attachment_vertex(attrs, 10_000, r2, ip_hint=h["ip"], citycode_hint=h["citycode"],
                                  countrycode_hint=h["countrycode"], geocode_hint=h["geocode"],
                                  type_hint=h["type"]) for h in hints[:k]]
    dtr = time.perf_counter() - t0
    assert got[:k] == ref
    print(f"C index: {len(hints)} hosts in {dt:.3f} s = {len(hints) / dt:,.0f} hosts/s (1 thread)")
    print(f"restatement: {k} hosts in {dtr:.3f} s = {k / dtr:,.1f} hosts/s (1 thread, sample)")
