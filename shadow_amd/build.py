"""Build the HIP engine in-tree for gfx950 (no JIT cache: the .so travels with the repo)."""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = [os.path.join(HERE, "csrc", "engine.hip")]
# every kernel header the engine includes (a glob: a new header cannot be left out of the
# staleness check, as sssp_f64d.hpp was in round 3)
HEADERS = sorted(glob.glob(os.path.join(HERE, "csrc", "*.hpp")))
OUT = os.path.join(HERE, "libshd_route.so")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-result"]


FRONT_SOURCES = [os.path.join(HERE, "csrc", "graphml.c"), os.path.join(HERE, "csrc", "topology_front.c"),
                 os.path.join(HERE, "csrc", "attach.c")]
FRONT_OUT = os.path.join(HERE, "libshd_topology.so")
CC = os.environ.get("CC", "gcc")


def build_front(verbose: bool = False) -> str:
    """C front end (topology.c semantics + graphml loader), linked against the engine."""
    cmd = [CC, "-O2", "-std=gnu11", "-fPIC", "-shared", "-Wall", "-I/usr/include/libxml2",
           "-o", FRONT_OUT, *FRONT_SOURCES, "-L" + HERE, "-lshd_route", "-lxml2", "-lpthread", "-lm",
           "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return FRONT_OUT


def source_id() -> str:
    """Identity of the engine build: a hash of its compile flags and every source it is built
    from.  bench.py writes it into its line and the PMC summaries carry the one they were
    profiled under, so a line's counter bytes are only ever taken from the same build."""
    import hashlib
    h = hashlib.sha256(" ".join(FLAGS).encode())
    for p in SOURCES + HEADERS + [os.path.join(ROOT, "include", "shd_route.h")]:
        h.update(os.path.basename(p).encode())
        h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SOURCES + HEADERS + [os.path.join(ROOT, "include", "shd_route.h")]
    return any(os.path.getmtime(p) > t for p in deps)


def build_diag(verbose: bool = False) -> str:
    """Diagnostic build with per-phase s_memtime stamps (tools/stamps.py); never shipped."""
    out = os.path.join(HERE, "libshd_route_diag.so")
    cmd = [HIPCC, *FLAGS, "-DSHD_STAMPS", "-DSHD_DIAG", "-o", out, *SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    if force or needs_build():
        cmd = [HIPCC, *FLAGS, "-o", OUT, *SOURCES]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    front_deps = FRONT_SOURCES + [os.path.join(ROOT, "include", f) for f in ("shd_topology.h", "shd_route.h")] + [OUT]
    if force or not os.path.exists(FRONT_OUT) or any(os.path.getmtime(p) > os.path.getmtime(FRONT_OUT)
                                                     for p in front_deps):
        build_front(verbose)
    return OUT


if __name__ == "__main__":
    if "--diag" in sys.argv:
        build_diag(verbose=True)
    else:
        build(force="--force" in sys.argv, verbose=True)
