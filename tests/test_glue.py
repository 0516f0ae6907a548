"""The topology.c drop-in (integration/topology.c): Shadow's public routing API
(topology.h:17-28) over libshd_topology, compiled against GLib and run the way Shadow
drives it (integration/glue_main.c)."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GLUE = os.path.join(ROOT, "integration")


def _build():
    from shadow_amd import build
    build.build()
    subprocess.run(["make", "-s", "-C", GLUE], check=True)
    return os.path.join(GLUE, "glue_test")


def test_glue_compiles_and_links():
    exe = _build()
    assert os.access(exe, os.X_OK)
    out = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True, check=True).stdout
    for sym in ("shd_topology_new", "shd_topology_attach", "shd_topology_get_latency", "shd_topology_free",
                "g_hash_table_lookup_extended"):
        assert sym in out, sym


@pytest.mark.gpu
def test_glue_runs_shadow_call_sequence():
    """Bundled reference topology (complete K183, every edge loss 0.005): 200 hosts
    attached by seeded random draws, 200k packets through the worker.c:267-279 calls,
    then one detach.  Every pair is routable, rel = 1 - 0.005 everywhere, the runahead
    is reported once (>= the 5 ms minimum edge), a detached address is unroutable."""
    exe = _build()
    topo = os.path.join(HERE, "golden", "topology.graphml.xml.xz")
    r = subprocess.run([exe, topo, "200", "200000", "3"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["routable"] == d["packets"] == 200000
    assert d["rel_min"] == d["rel_max"] == 1.0 - 0.005
    assert d["lat_min"] >= 5.0 and d["runahead_reported_ms"] >= 5.0
    assert d["runahead_reported_ms"] <= d["lat_min"]
    assert d["detached_latency"] == -1.0 and d["detached_routable"] == 0
    assert d["bw_sum"] > 0
