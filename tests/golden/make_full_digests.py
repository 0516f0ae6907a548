#!/usr/bin/env python3
"""Regenerate tests/golden/full_digests.npz: a digest of EVERY source row of C3 and C4
(test infrastructure; runs in the dev container, the GPU box only reads the output).

For every attached source s (C3: 9,337 rows, C4: 50,000 rows) the oracle's SOURCE(s,.)
row (oracle/oracle.c orc_source_row, engine tie rule; topology.c:1655-1875 +
1407-1523) over all targets is hashed:
  lat_d[k], rel_d[k]  first 16 bytes of SHA-256 over the row's float64 bytes
  row_min[k]          min over the row (the per-row runahead candidate, topology.c:1374-1385)
The GPU test (tests/test_seed_gpu.py::test_full_table_every_row) hashes every row of the
planned table the same way, so every row of both tables is compared, not a sample.

The oracle itself is pinned by networkx (an independent SSSP, tests/golden/nx_pin.py)
on a stratified C4 sample of 512 sources: the 64 highest-degree vertices (the plan's
roots and landmark rows are the most central), 64 degree-m leaves, and 384 seeded-
uniform others; latency on every target and reliability on every unique-shortest-path
target must match bit for bit or the generator stops.  The counts go to `nx_stats`.

Usage: python tests/golden/make_full_digests.py [--threads 8] [--no-nx]
"""
from __future__ import annotations

import argparse
import hashlib
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor, ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from shadow_amd.graph import config  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(HERE, "full_digests.npz")


def digest16(a: np.ndarray) -> bytes:
    return hashlib.sha256(np.ascontiguousarray(a, np.float64).tobytes()).digest()[:16]


def table_digests(cfg: str, threads: int):
    g = config(cfg)
    og = O.OracleGraph(g)
    T = g.targets()
    ns = len(T)
    lat_d = np.zeros((ns, 16), np.uint8)
    rel_d = np.zeros((ns, 16), np.uint8)
    mn = np.zeros(ns, np.float64)

    def one(k):
        # orc_source_row without the uniqueness pass is re-entrant (per-call scratch);
        # ctypes and hashlib release the GIL, so the threads run in parallel
        lat, rel, _, _ = og.source_row(int(T[k]), T, O.TIE_MINKEY)
        lat_d[k] = np.frombuffer(digest16(lat), np.uint8)
        rel_d[k] = np.frombuffer(digest16(rel), np.uint8)
        mn[k] = lat.min()

    t0 = time.time()
    with ThreadPoolExecutor(threads) as ex:
        for i, _ in enumerate(ex.map(one, range(ns), chunksize=16)):
            if i % 2000 == 0:
                print(f"{cfg}: {i}/{ns} rows, {time.time() - t0:.0f} s", flush=True)
    print(f"{cfg}: {ns} rows in {time.time() - t0:.0f} s", flush=True)
    return T.astype(np.int32), lat_d, rel_d, mn


_NX = {}


def _nx_init(cfg):
    from tests.golden.nx_pin import nx_graph
    g = config(cfg)
    _NX.update(g=g, G=nx_graph(g), og=O.OracleGraph(g), T=g.targets())


def _nx_one(s):
    from tests.golden.nx_pin import pin_row
    g, G, og, T = _NX["g"], _NX["G"], _NX["og"], _NX["T"]
    lat, rel, uq, _ = og.source_row(int(s), T, O.TIE_MINKEY)
    nl, nr = pin_row(G, g, int(s), T, lat, rel, uq)
    return int(s), nl, nr, digest16(lat), digest16(rel)


def nx_sample(cfg: str, k: int = 512):
    g = config(cfg)
    T = g.targets()
    deg = np.bincount(np.concatenate([g.src[g.src != g.dst], g.dst[g.src != g.dst]]), minlength=g.n)
    order = np.argsort(-deg[T], kind="stable")
    hubs = T[order[:64]]
    leaves = T[order[::-1][:64]]
    rng = np.random.default_rng(2026)
    rest = np.setdiff1d(T, np.concatenate([hubs, leaves]))
    uni = rng.choice(rest, size=k - 128, replace=False)
    return np.sort(np.concatenate([hubs, leaves, uni])).astype(np.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--no-nx", action="store_true")
    ap.add_argument("--nx-procs", type=int, default=4)
    a = ap.parse_args()
    O.build()
    blobs = {}
    for cfg in ("c3", "c4"):
        T, ld, rd, mn = table_digests(cfg, a.threads)
        blobs.update({f"{cfg}__src": T, f"{cfg}__lat_d": ld, f"{cfg}__rel_d": rd, f"{cfg}__row_min": mn})
    if not a.no_nx:
        S = nx_sample("c4")
        T = blobs["c4__src"]
        row = {int(v): i for i, v in enumerate(T)}
        t0 = time.time()
        nl = nr = 0
        with ProcessPoolExecutor(a.nx_procs, initializer=_nx_init, initargs=("c4",)) as ex:
            for i, (s, l, r, dl, dr) in enumerate(ex.map(_nx_one, S.tolist(), chunksize=4)):
                # the networkx-pinned row is the row the table digests hold
                assert dl == blobs["c4__lat_d"][row[s]].tobytes() and dr == blobs["c4__rel_d"][row[s]].tobytes(), s
                nl += l
                nr += r
                if i % 64 == 0:
                    print(f"nx c4: {i}/{len(S)} rows, {time.time() - t0:.0f} s", flush=True)
        blobs["c4__nx_src"] = S
        blobs["c4__nx_stats"] = np.array([len(S), nl, nr], np.int64)
        print(f"nx c4: {len(S)} rows, {nl} latency pairs, {nr} unique-path rel pairs equal", flush=True)
    np.savez_compressed(OUT, **blobs)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
