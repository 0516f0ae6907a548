"""ctypes binding of the C front end (shadow_amd/libshd_topology.so, include/shd_topology.h).

Mirrors Shadow's routing API (reference src/main/routing/topology.h:17-28) keyed by
vertex index: ``Topology.new(path)`` ~ ``topology_new``, ``get_latency`` ~
``topology_getLatency`` (-1 on error), ``get_reliability``, ``is_routable``,
``increment_path_packet_counter``; plus the runahead the cache implies.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np

from .graph import Graph
from .route import _Graph, load_library as _load_engine

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libshd_topology.so")

EXPORTS = (
    "shd_graphml_load", "shd_graphml_free", "shd_topology_new", "shd_topology_new_from_graph",
    "shd_topology_free", "shd_topology_vertex_count", "shd_topology_find_vertex",
    "shd_topology_attach_vertex", "shd_topology_attached_count", "shd_topology_get_latency",
    "shd_topology_get_reliability", "shd_topology_is_routable",
    "shd_topology_increment_path_packet_counter", "shd_topology_get_path_packet_count",
    "shd_topology_is_direct_path", "shd_topology_min_path_latency", "shd_topology_runahead_ns",
    "shd_topology_fill", "shd_topology_dump_paths", "shd_topology_triangle_bytes",
    "shd_attach_create", "shd_attach_find_vertex", "shd_attach_destroy", "shd_topology_attach",
)

VATTRS = ("ip", "citycode", "countrycode", "geocode", "type")  # SHD_VATTR_* order
_NEXT_DOUBLE = C.CFUNCTYPE(C.c_double, C.c_void_p)


class _GraphML(C.Structure):
    _fields_ = [("graph", _Graph), ("vertex_ids", C.POINTER(C.c_char_p)),
                ("bandwidth_down", C.POINTER(C.c_double)), ("bandwidth_up", C.POINTER(C.c_double)),
                ("has_vertex_packetloss", C.c_int32), ("has_vertex_str", C.c_int32 * 5),
                ("vertex_str", C.POINTER(C.c_char_p) * 5)]


_lib = None


def load_library():
    global _lib
    if _lib is not None:
        return _lib
    _load_engine()
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"front end not built: {LIB_PATH} missing (run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P, I32, D = C.c_void_p, C.c_int32, C.c_double
    L.shd_graphml_load.restype = C.c_int
    L.shd_graphml_load.argtypes = [C.c_char_p, C.POINTER(_GraphML), C.c_char_p, C.c_size_t]
    L.shd_graphml_free.argtypes = [C.POINTER(_GraphML)]
    L.shd_topology_new.restype = P
    L.shd_topology_new.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.c_int]
    L.shd_topology_new_from_graph.restype = P
    L.shd_topology_new_from_graph.argtypes = [C.POINTER(_Graph), C.POINTER(C.c_int), C.c_int]
    L.shd_topology_free.argtypes = [P]
    L.shd_topology_vertex_count.restype = I32
    L.shd_topology_vertex_count.argtypes = [P]
    L.shd_topology_find_vertex.restype = I32
    L.shd_topology_find_vertex.argtypes = [P, C.c_char_p]
    L.shd_topology_attach_vertex.restype = C.c_int
    L.shd_topology_attach_vertex.argtypes = [P, I32]
    L.shd_topology_attached_count.restype = I32
    L.shd_topology_attached_count.argtypes = [P]
    for f in ("get_latency", "get_reliability"):
        getattr(L, "shd_topology_" + f).restype = D
        getattr(L, "shd_topology_" + f).argtypes = [P, I32, I32]
    L.shd_topology_is_routable.restype = C.c_int
    L.shd_topology_is_routable.argtypes = [P, I32, I32]
    L.shd_topology_is_direct_path.restype = C.c_int
    L.shd_topology_is_direct_path.argtypes = [P, I32, I32]
    L.shd_topology_increment_path_packet_counter.argtypes = [P, I32, I32]
    L.shd_topology_get_path_packet_count.restype = C.c_uint64
    L.shd_topology_get_path_packet_count.argtypes = [P, I32, I32]
    L.shd_topology_min_path_latency.restype = D
    L.shd_topology_min_path_latency.argtypes = [P]
    L.shd_topology_runahead_ns.restype = C.c_uint64
    L.shd_topology_runahead_ns.argtypes = [P]
    L.shd_topology_fill.restype = C.c_int
    L.shd_topology_fill.argtypes = [P, C.POINTER(D)]
    L.shd_topology_triangle_bytes.restype = C.c_uint64
    L.shd_topology_triangle_bytes.argtypes = [P]
    L.shd_topology_dump_paths.restype = C.c_int
    L.shd_topology_dump_paths.argtypes = [P, P]
    S = C.c_char_p
    L.shd_attach_create.restype = C.c_int
    L.shd_attach_create.argtypes = [C.POINTER(P), C.POINTER(_GraphML)]
    L.shd_attach_find_vertex.restype = I32
    L.shd_attach_find_vertex.argtypes = [P, _NEXT_DOUBLE, P, S, S, S, S, S]
    L.shd_attach_destroy.argtypes = [P]
    L.shd_topology_attach.restype = I32
    L.shd_topology_attach.argtypes = [P, _NEXT_DOUBLE, P, S, S, S, S, S, C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64)]
    _lib = L
    return L


def load_graphml(path: str) -> Graph:
    """Parse + validate graphml with the C loader (no GPU needed)."""
    L = load_library()
    out = _GraphML()
    err = C.create_string_buffer(512)
    rc = L.shd_graphml_load(path.encode(), C.byref(out), err, 512)
    if rc != 0:
        raise ValueError(err.value.decode() or f"graphml load failed ({rc})")
    try:
        g = out.graph
        n, m = g.n_vertices, g.n_edges
        arr = lambda p, cnt, ct, dt: np.ctypeslib.as_array(C.cast(p, C.POINTER(ct)), shape=(cnt,)).astype(dt).copy() \
            if cnt else np.zeros(0, dt)
        src = arr(g.edge_src, m, C.c_int32, np.int32)
        dst = arr(g.edge_dst, m, C.c_int32, np.int32)
        lat = arr(g.edge_latency, m, C.c_double, np.float64)
        loss = arr(g.edge_packetloss, m, C.c_double, np.float64)
        vl = arr(g.vertex_packetloss, n, C.c_double, np.float64) if g.vertex_packetloss else None
        ids = [out.vertex_ids[v].decode() for v in range(n)]
        return Graph(n=n, src=src, dst=dst, latency=lat, packetloss=loss, vertex_packetloss=vl,
                     directed=bool(g.directed), prefer_direct=bool(g.prefer_direct), ids=ids,
                     name=os.path.basename(path))
    finally:
        L.shd_graphml_free(C.byref(out))


def _enc(x):
    return None if x is None else x.encode()


class AttachIndex:
    """Host attachment over a graphml file (shd_attach_*, no GPU): the vertex a host
    with these hints joins, as _topology_findAttachmentVertex (topology.c:2245-2366).
    ``next_double`` is called where the reference draws random_nextDouble."""

    def __init__(self, path: str):
        L = load_library()
        self._gml = _GraphML()
        err = C.create_string_buffer(512)
        rc = L.shd_graphml_load(path.encode(), C.byref(self._gml), err, 512)
        if rc != 0:
            raise ValueError(err.value.decode() or f"graphml load failed ({rc})")
        self._h = C.c_void_p()
        rc = L.shd_attach_create(C.byref(self._h), C.byref(self._gml))
        if rc != 0:
            L.shd_graphml_free(C.byref(self._gml))
            raise ValueError(f"shd_attach_create failed ({rc})")
        self.n = self._gml.graph.n_vertices

    def vertex_attrs(self):
        """{name: [value or None per vertex] or None when the key is not declared}."""
        out = {}
        for a, name in enumerate(VATTRS):
            if not self._gml.has_vertex_str[a]:
                out[name] = None
                continue
            col = self._gml.vertex_str[a]
            out[name] = [None if col[v] is None else col[v].decode() for v in range(self.n)]
        return out

    def find(self, next_double=None, ip=None, citycode=None, countrycode=None, geocode=None, type=None) -> int:
        cb = _NEXT_DOUBLE((lambda _ctx: float(next_double()))) if next_double else _NEXT_DOUBLE()
        return int(load_library().shd_attach_find_vertex(self._h, cb, None, _enc(ip), _enc(citycode),
                                                          _enc(countrycode), _enc(geocode), _enc(type)))

    def close(self):
        if getattr(self, "_h", None):
            L = load_library()
            L.shd_attach_destroy(self._h)
            L.shd_graphml_free(C.byref(self._gml))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Topology:
    """topology.h over the GPU engine, vertex-indexed (one object per simulation)."""

    def __init__(self, handle, keep=None):
        if not handle:
            raise RuntimeError("topology creation failed")
        self._h = C.c_void_p(handle)
        self._keep = keep

    @classmethod
    def new(cls, path: str, devices=(0,)):
        L = load_library()
        dv = (C.c_int * len(devices))(*devices)
        return cls(L.shd_topology_new(path.encode(), dv, len(devices)))

    @classmethod
    def from_graph(cls, g: Graph, devices=(0,)):
        L = load_library()
        keep = (np.ascontiguousarray(g.src, np.int32), np.ascontiguousarray(g.dst, np.int32),
                np.ascontiguousarray(g.latency, np.float64), np.ascontiguousarray(g.packetloss, np.float64),
                None if g.vertex_packetloss is None else np.ascontiguousarray(g.vertex_packetloss, np.float64))
        s, d, lat, loss, vl = keep
        desc = _Graph(int(g.n), len(s), s.ctypes.data, d.ctypes.data, lat.ctypes.data, loss.ctypes.data,
                      None if vl is None else vl.ctypes.data, int(bool(g.directed)), int(bool(g.prefer_direct)))
        dv = (C.c_int * len(devices))(*devices)
        return cls(L.shd_topology_new_from_graph(C.byref(desc), dv, len(devices)), keep)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            load_library().shd_topology_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def vertex_count(self):
        return load_library().shd_topology_vertex_count(self._h)

    def find_vertex(self, graphml_id: str) -> int:
        return load_library().shd_topology_find_vertex(self._h, graphml_id.encode())

    def attach(self, vertex: int):
        rc = load_library().shd_topology_attach_vertex(self._h, int(vertex))
        if rc:
            raise ValueError(f"attach failed ({rc})")

    def attach_host(self, next_double=None, ip=None, citycode=None, countrycode=None, geocode=None, type=None):
        """topology_attach (topology.c:2371-2439): (vertex, bandwidth down, bandwidth up)."""
        cb = _NEXT_DOUBLE((lambda _ctx: float(next_double()))) if next_double else _NEXT_DOUBLE()
        down, up = C.c_uint64(), C.c_uint64()
        v = load_library().shd_topology_attach(self._h, cb, None, _enc(ip), _enc(citycode), _enc(countrycode),
                                               _enc(geocode), _enc(type), C.byref(down), C.byref(up))
        if v < 0:
            raise ValueError("attach failed (topology not loaded from graphml?)")
        return int(v), int(down.value), int(up.value)

    def attached_count(self) -> int:
        return int(load_library().shd_topology_attached_count(self._h))

    def attach_all(self, vertices):
        for v in vertices:
            self.attach(v)

    def fill(self) -> float:
        t = C.c_double()
        rc = load_library().shd_topology_fill(self._h, C.byref(t))
        if rc:
            raise RuntimeError(f"fill failed ({rc})")
        return t.value

    def triangle_bytes(self) -> int:
        """Host bytes of the filled triangle (16 per pair, or the compact u16 layout)."""
        return int(load_library().shd_topology_triangle_bytes(self._h))

    def get_latency(self, s, d) -> float:
        return load_library().shd_topology_get_latency(self._h, int(s), int(d))

    def get_reliability(self, s, d) -> float:
        return load_library().shd_topology_get_reliability(self._h, int(s), int(d))

    def is_routable(self, s, d) -> bool:
        return bool(load_library().shd_topology_is_routable(self._h, int(s), int(d)))

    def is_direct(self, s, d) -> int:
        return load_library().shd_topology_is_direct_path(self._h, int(s), int(d))

    def increment_path_packet_counter(self, s, d):
        load_library().shd_topology_increment_path_packet_counter(self._h, int(s), int(d))

    def packet_count(self, s, d) -> int:
        return int(load_library().shd_topology_get_path_packet_count(self._h, int(s), int(d)))

    def min_path_latency(self) -> float:
        return load_library().shd_topology_min_path_latency(self._h)

    def runahead_ns(self) -> int:
        return int(load_library().shd_topology_runahead_ns(self._h))

    def table(self, vertices):
        """Dense lookup(i, j) table (lat, rel) for a vertex list, via the public getters."""
        k = len(vertices)
        lat = np.empty((k, k)); rel = np.empty((k, k))
        L = load_library()
        for a, s in enumerate(vertices):
            for b, d in enumerate(vertices):
                lat[a, b] = L.shd_topology_get_latency(self._h, int(s), int(d))
                rel[a, b] = L.shd_topology_get_reliability(self._h, int(s), int(d))
        return lat, rel
