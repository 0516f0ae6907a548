"""ctypes wrapper for the CPU oracle (oracle/oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product (shadow_amd/).  See
oracle/oracle.h for what each function restates (topology.c file:line) and the
parity status (igraph 0.7.1 restated, not linked).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

TIE_IGRAPH = 0
TIE_MINKEY = 1


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "oracle.c")
        ):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C")
        f64p = np.ctypeslib.ndpointer(np.float64, flags="C")
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C")
        i64p = np.ctypeslib.ndpointer(np.int64, flags="C")
        L.orc_graph_new.restype = P
        L.orc_graph_new.argtypes = [C.c_int32, C.c_int32, i32p, i32p, f64p, f64p, P, C.c_int32]
        L.orc_graph_free.argtypes = [P]
        L.orc_is_complete.restype = C.c_int32
        L.orc_is_complete.argtypes = [P]
        L.orc_get_eid.restype = C.c_int64
        L.orc_get_eid.argtypes = [P, C.c_int32, C.c_int32]
        L.orc_dijkstra.restype = C.c_int32
        L.orc_dijkstra.argtypes = [P, C.c_int32, C.c_int32, f64p, i64p]
        L.orc_source_row.restype = C.c_int32
        L.orc_source_row.argtypes = [P, C.c_int32, i32p, C.c_int32, C.c_int32, f64p, f64p, P, P]
        L.orc_direct.restype = C.c_int32
        L.orc_direct.argtypes = [P, C.c_int32, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.orc_self_path.restype = C.c_int32
        L.orc_self_path.argtypes = [P, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.orc_eager_table.restype = C.c_int32
        L.orc_eager_table.argtypes = [P, i32p, C.c_int32, C.c_int32, C.c_int32, f64p, f64p, P, P,
                                      C.POINTER(C.c_double)]
        L.orc_runahead_ns.restype = C.c_uint64
        L.orc_runahead_ns.argtypes = [C.c_double]
        L.orc_bench_faithful.restype = C.c_double
        L.orc_bench_faithful.argtypes = [P, i32p, C.c_int32, i32p, C.c_int32, C.POINTER(C.c_double)]
        L.orc_bench_parallel.restype = C.c_double
        L.orc_bench_parallel.argtypes = [P, i32p, C.c_int32, i32p, C.c_int32, C.c_int32,
                                         C.POINTER(C.c_double), C.POINTER(C.c_int32)]
        L.orc_floyd_warshall.argtypes = [C.c_int32, f64p]
        L.orc_bench_direct.restype = C.c_double
        L.orc_bench_direct.argtypes = [P, i32p, C.c_int32, C.c_int32, C.POINTER(C.c_double),
                                       C.POINTER(C.c_int32)]
        L.orc_bench_fw_phases.restype = C.c_double
        L.orc_bench_fw_phases.argtypes = [C.c_int32, f64p, C.c_int32, C.c_int32, C.c_int32,
                                          C.POINTER(C.c_int32)]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OracleGraph:
    """An igraph-0.7.1-shaped graph plus Shadow's attribute semantics."""

    def __init__(self, g):
        """g: shadow_amd.graph.Graph-like (n, src, dst, latency, packetloss, vertex_packetloss, directed)."""
        L = lib()
        self.n = int(g.n)
        self._keep = (
            np.ascontiguousarray(g.src, np.int32),
            np.ascontiguousarray(g.dst, np.int32),
            np.ascontiguousarray(g.latency, np.float64),
            np.ascontiguousarray(g.packetloss, np.float64),
            None if g.vertex_packetloss is None else np.ascontiguousarray(g.vertex_packetloss, np.float64),
        )
        s, d, lat, loss, vl = self._keep
        self.h = L.orc_graph_new(self.n, len(s), s, d, lat, loss, _ptr(vl), int(bool(g.directed)))
        if not self.h:
            raise ValueError("orc_graph_new rejected the graph")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_graph_free(self.h)
            self.h = None

    def is_complete(self) -> bool:
        return bool(lib().orc_is_complete(self.h))

    def get_eid(self, a, b) -> int:
        return int(lib().orc_get_eid(self.h, int(a), int(b)))

    def dijkstra(self, s, tiebreak=TIE_IGRAPH):
        dist = np.empty(self.n, np.float64)
        par = np.empty(self.n, np.int64)
        lib().orc_dijkstra(self.h, int(s), tiebreak, dist, par)
        return dist, par

    def source_row(self, s, targets, tiebreak=TIE_IGRAPH):
        t = np.ascontiguousarray(targets, np.int32)
        lat = np.empty(len(t), np.float64)
        rel = np.empty(len(t), np.float64)
        uniq = np.empty(len(t), np.uint8)
        hops = np.empty(len(t), np.int32)
        r = lib().orc_source_row(self.h, int(s), t, len(t), tiebreak, lat, rel, _ptr(uniq), _ptr(hops))
        if r != 0:
            raise RuntimeError(f"orc_source_row failed for source {s}")
        return lat, rel, uniq.astype(bool), hops

    def source_rows(self, sources, targets, tiebreak=TIE_IGRAPH):
        ns, nt = len(sources), len(targets)
        lat = np.empty((ns, nt)); rel = np.empty((ns, nt))
        uniq = np.empty((ns, nt), bool); hops = np.empty((ns, nt), np.int32)
        for i, s in enumerate(sources):
            lat[i], rel[i], uniq[i], hops[i] = self.source_row(s, targets, tiebreak)
        return lat, rel, uniq, hops

    def direct(self, s, t):
        a, b = C.c_double(), C.c_double()
        if lib().orc_direct(self.h, int(s), int(t), C.byref(a), C.byref(b)) != 0:
            raise RuntimeError("no edge")
        return a.value, b.value

    def self_path(self, s):
        a, b = C.c_double(), C.c_double()
        if lib().orc_self_path(self.h, int(s), C.byref(a), C.byref(b)) != 0:
            raise RuntimeError("no incident edge")
        return a.value, b.value

    def eager_table(self, attached, prefer_direct=False, tiebreak=TIE_IGRAPH):
        A = np.ascontiguousarray(np.sort(np.asarray(attached)), np.int32)
        na = len(A)
        lat = np.empty(na * na); rel = np.empty(na * na)
        isd = np.empty(na * na, np.uint8); uq = np.empty(na * na, np.uint8)
        mn = C.c_double()
        r = lib().orc_eager_table(self.h, A, na, int(bool(prefer_direct)), tiebreak, lat, rel,
                                  _ptr(isd), _ptr(uq), C.byref(mn))
        if r != 0:
            raise RuntimeError("orc_eager_table failed")
        sh = (na, na)
        return dict(attached=A, lat=lat.reshape(sh), rel=rel.reshape(sh), is_direct=isd.reshape(sh).astype(bool),
                    unique=uq.reshape(sh).astype(bool), min_latency=mn.value)

    def bench_faithful(self, sources, targets):
        s = np.ascontiguousarray(sources, np.int32); t = np.ascontiguousarray(targets, np.int32)
        cs = C.c_double()
        dt = lib().orc_bench_faithful(self.h, s, len(s), t, len(t), C.byref(cs))
        return dt, cs.value

    def bench_parallel(self, sources, targets, threads=0):
        s = np.ascontiguousarray(sources, np.int32); t = np.ascontiguousarray(targets, np.int32)
        cs = C.c_double(); used = C.c_int32()
        dt = lib().orc_bench_parallel(self.h, s, len(s), t, len(t), int(threads), C.byref(cs), C.byref(used))
        return dt, cs.value, used.value

    def bench_direct(self, attached, threads=0):
        a = np.ascontiguousarray(attached, np.int32)
        cs = C.c_double(); used = C.c_int32()
        dt = lib().orc_bench_direct(self.h, a, len(a), int(threads), C.byref(cs), C.byref(used))
        return dt, used.value


def bench_fw_phases(d: np.ndarray, k0: int, nk: int, threads: int = 0):
    """nk k-phases of f64 Floyd-Warshall over d (in place); returns (seconds, threads)."""
    used = C.c_int32()
    dt = lib().orc_bench_fw_phases(d.shape[0], d, int(k0), int(nk), int(threads), C.byref(used))
    return dt, used.value


def runahead_ns(min_latency: float) -> int:
    return int(lib().orc_runahead_ns(float(min_latency)))


def floyd_warshall(d: np.ndarray) -> np.ndarray:
    d = np.ascontiguousarray(d, np.float64).copy()
    lib().orc_floyd_warshall(d.shape[0], d)
    return d
