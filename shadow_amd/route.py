"""ctypes binding of the HIP engine (shadow_amd/libshd_route.so, include/shd_route.h).

This is the same binding a maintainer would add on the reference side (see
INTEGRATION.md); Python is only the test/bench driver.  There is no CPU fallback:
if the HIP library is missing, importing the engine raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .graph import Graph

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SHD_ROUTE_LIB") or os.path.join(_HERE, "libshd_route.so")

OK = 0
EINVAL = -1
ENOMEM = -2
EDEVICE = -3
ENOEDGE = -4
EUNREACH = -5
EUNSUPPORTED = -6
DISPATCH = 0x1
PLAN_REUSE = 0x200  # shd_route.h SHD_ROUTE_PLAN_REUSE
REFRESH_ALL, REFRESH_MINE, REFRESH_JOBS = 0x1, 0x2, 0x4  # SHD_ROUTE_REFRESH_*
PAYLOAD_LAT16 = 0x1
FILL_LAT16 = 0x100


class RouteError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})")


class _Graph(C.Structure):
    _fields_ = [
        ("n_vertices", C.c_int32), ("n_edges", C.c_int32),
        ("edge_src", C.c_void_p), ("edge_dst", C.c_void_p),
        ("edge_latency", C.c_void_p), ("edge_packetloss", C.c_void_p),
        ("vertex_packetloss", C.c_void_p),
        ("directed", C.c_int32), ("prefer_direct", C.c_int32),
    ]


class _Info(C.Structure):
    _fields_ = [
        ("n_vertices", C.c_int32), ("n_edges", C.c_int32), ("n_arcs", C.c_int32),
        ("is_complete", C.c_int32), ("directed", C.c_int32), ("prefer_direct", C.c_int32),
        ("integer_weights", C.c_int32), ("multigraph", C.c_int32), ("device", C.c_int32),
        ("lds_resident", C.c_int32), ("device_bytes", C.c_uint64), ("min_edge_latency", C.c_double),
        ("kernel", C.c_int32), ("dist_bound", C.c_int32), ("block", C.c_int32), ("reserved", C.c_int32),
        ("lat16", C.c_int32),
    ]


class _PlanInfo(C.Structure):
    _fields_ = [
        ("rows", C.c_int32), ("seeded", C.c_int32), ("launches", C.c_int32), ("levels", C.c_int32),
        ("roots", C.c_int32),
        ("helpers", C.c_int32), ("stored_rows", C.c_int32), ("world", C.c_int32), ("rank", C.c_int32),
        ("store_bytes", C.c_uint64), ("delta", C.c_int32), ("pad_", C.c_int32),
    ]


# every symbol include/shd_route.h declares
EXPORTS = (
    "shd_route_create", "shd_route_destroy", "shd_route_get_info", "shd_route_strerror",
    "shd_route_rows", "shd_route_rows_async", "shd_route_sync", "shd_route_direct",
    "shd_route_self", "shd_route_min_reduce_async", "shd_route_fw_async",
    "shd_route_plan_create", "shd_route_plan_destroy", "shd_route_plan_get_info", "shd_route_plan_rows",
    "shd_route_rows_planned_async", "shd_route_fw_table_async", "shd_route_fw_rows_async",
    "shd_route_fill_triangle", "shd_route_host_alloc", "shd_route_host_free", "shd_route_tri_payload_async",
    "shd_route_kd_stats", "shd_route_host_alloc_lazy", "shd_route_host_wait",
    "shd_route_host_unpinned", "shd_route_plan_refresh_async", "shd_route_plan_landmarks",
    "shd_route_plan_bind_store",
)

_lib = None


def load_library():
    """Load libshd_route.so (fails loudly if the HIP build is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP engine not built: {LIB_PATH} missing (run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P, I32, I64, U32 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32
    L.shd_route_strerror.restype = C.c_char_p
    L.shd_route_strerror.argtypes = [C.c_int]
    L.shd_route_create.restype = C.c_int
    L.shd_route_create.argtypes = [C.POINTER(P), C.POINTER(_Graph), C.c_int]
    L.shd_route_destroy.argtypes = [P]
    L.shd_route_get_info.restype = C.c_int
    L.shd_route_get_info.argtypes = [P, C.POINTER(_Info)]
    L.shd_route_rows.restype = C.c_int
    L.shd_route_rows.argtypes = [P, P, I32, P, I32, U32, P, P, P]
    L.shd_route_rows_async.restype = C.c_int
    L.shd_route_rows_async.argtypes = [P, P, I32, P, I32, I64, U32, P, P, P, P]
    L.shd_route_sync.restype = C.c_int
    L.shd_route_sync.argtypes = [P, P]
    L.shd_route_direct.restype = C.c_int
    L.shd_route_direct.argtypes = [P, P, I32, P, I32, P, P, P]
    L.shd_route_self.restype = C.c_int
    L.shd_route_self.argtypes = [P, P, I32, P, P]
    L.shd_route_min_reduce_async.restype = C.c_int
    L.shd_route_min_reduce_async.argtypes = [P, P, I64, P, P]
    L.shd_route_fw_async.restype = C.c_int
    L.shd_route_fw_async.argtypes = [P, P, P]
    L.shd_route_fill_triangle.restype = C.c_int
    L.shd_route_fill_triangle.argtypes = [P, P, I32, I32, I32, U32, P, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.shd_route_host_alloc.restype = P
    L.shd_route_host_alloc.argtypes = [C.c_size_t]
    L.shd_route_host_free.argtypes = [P]
    L.shd_route_host_alloc_lazy.restype = P
    L.shd_route_host_alloc_lazy.argtypes = [C.c_size_t]
    L.shd_route_host_wait.restype = C.c_int
    L.shd_route_host_wait.argtypes = [P]
    L.shd_route_host_unpinned.restype = C.c_int64
    L.shd_route_host_unpinned.argtypes = [P]
    L.shd_route_fw_table_async.restype = C.c_int
    L.shd_route_fw_table_async.argtypes = [P, P]
    L.shd_route_fw_rows_async.restype = C.c_int
    L.shd_route_fw_rows_async.argtypes = [P, P, I32, P, I32, I64, P, P, P, P]
    L.shd_route_tri_payload_async.restype = C.c_int
    L.shd_route_tri_payload_async.argtypes = [P, P, P, I64, P, P, I32, I32, U32, P, P, P]
    L.shd_route_plan_create.restype = C.c_int
    L.shd_route_plan_create.argtypes = [P, P, I32, I32, I32, C.POINTER(P)]
    L.shd_route_plan_destroy.argtypes = [P]
    L.shd_route_plan_get_info.restype = C.c_int
    L.shd_route_plan_get_info.argtypes = [P, C.POINTER(_PlanInfo)]
    L.shd_route_plan_rows.restype = C.c_int
    L.shd_route_plan_rows.argtypes = [P, P]
    L.shd_route_rows_planned_async.restype = C.c_int
    L.shd_route_rows_planned_async.argtypes = [P, P, P, I32, I64, U32, P, P, P, P]
    L.shd_route_plan_refresh_async.restype = C.c_int
    L.shd_route_plan_refresh_async.argtypes = [P, P, U32, P]
    L.shd_route_plan_landmarks.restype = C.c_int
    L.shd_route_plan_landmarks.argtypes = [P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                           C.POINTER(C.c_int64)]
    L.shd_route_plan_bind_store.restype = C.c_int
    L.shd_route_plan_bind_store.argtypes = [P, P, P, P]
    L.shd_route_kd_stats.restype = C.c_int
    L.shd_route_kd_stats.argtypes = [P, P, I32]
    _lib = L
    return L


def strerror(code: int) -> str:
    try:
        return load_library().shd_route_strerror(int(code)).decode()
    except RuntimeError:
        return f"error {code}"


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _check(rc, what):
    if rc != OK:
        raise RouteError(rc, what)


class RouteEngine:
    """One routing context on one GPU (one process per GPU)."""

    def __init__(self, g: Graph, device: int = 0):
        L = load_library()
        self.graph = g
        self._arrays = (
            np.ascontiguousarray(g.src, np.int32), np.ascontiguousarray(g.dst, np.int32),
            np.ascontiguousarray(g.latency, np.float64), np.ascontiguousarray(g.packetloss, np.float64),
            None if g.vertex_packetloss is None else np.ascontiguousarray(g.vertex_packetloss, np.float64),
        )
        s, d, lat, loss, vl = self._arrays
        desc = _Graph(int(g.n), len(s), s.ctypes.data, d.ctypes.data, lat.ctypes.data, loss.ctypes.data,
                      None if vl is None else vl.ctypes.data, int(bool(g.directed)), int(bool(g.prefer_direct)))
        h = C.c_void_p()
        _check(L.shd_route_create(C.byref(h), C.byref(desc), int(device)), "shd_route_create")
        self._h = h
        self.device = device
        # plans made on this context (a plan must be destroyed before its context: when both
        # become garbage together, the collector may finalise them in either order)
        import weakref
        self._plans = weakref.WeakSet()
        inf = _Info()
        _check(L.shd_route_get_info(self._h, C.byref(inf)), "shd_route_get_info")
        self.info = {k: getattr(inf, k) for k, _ in _Info._fields_}

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            for p in list(getattr(self, "_plans", ())):
                p.close()
            load_library().shd_route_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host-pointer API -----------------------------------------------------
    def rows(self, sources, targets, dispatch: bool = True):
        s = np.ascontiguousarray(sources, np.int32)
        t = np.ascontiguousarray(targets, np.int32)
        lat = np.empty((len(s), len(t))); rel = np.empty((len(s), len(t))); mn = np.empty(len(s))
        rc = load_library().shd_route_rows(self._h, _p(s), len(s), _p(t), len(t),
                                           DISPATCH if dispatch else 0, _p(lat), _p(rel), _p(mn))
        _check(rc, "shd_route_rows")
        return lat, rel, mn

    def direct(self, sources, targets):
        s = np.ascontiguousarray(sources, np.int32)
        t = np.ascontiguousarray(targets, np.int32)
        lat = np.empty((len(s), len(t))); rel = np.empty((len(s), len(t))); mn = np.empty(len(s))
        _check(load_library().shd_route_direct(self._h, _p(s), len(s), _p(t), len(t), _p(lat), _p(rel), _p(mn)),
               "shd_route_direct")
        return lat, rel, mn

    def self_paths(self, vertices):
        v = np.ascontiguousarray(vertices, np.int32)
        lat = np.empty(len(v)); rel = np.empty(len(v))
        _check(load_library().shd_route_self(self._h, _p(v), len(v), _p(lat), _p(rel)), "shd_route_self")
        return lat, rel

    # -- device-pointer API (torch tensors as HBM plumbing) --------------------
    def rows_async(self, d_src, d_tgt, d_lat, d_rel, d_rowmin, stream=None, dispatch=True, ld=None):
        ns, nt = int(d_src.numel()), int(d_tgt.numel())
        ld = nt if ld is None else int(ld)
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        rc = load_library().shd_route_rows_async(
            self._h, ptr(d_src), ns, ptr(d_tgt), nt, ld, DISPATCH if dispatch else 0,
            ptr(d_lat), ptr(d_rel), ptr(d_rowmin), C.c_void_p(stream) if stream else None)
        _check(rc, "shd_route_rows_async")

    def sync(self, stream=None):
        _check(load_library().shd_route_sync(self._h, C.c_void_p(stream) if stream else None), "shd_route_sync")

    def min_reduce_async(self, d_vals, d_out, stream=None):
        rc = load_library().shd_route_min_reduce_async(self._h, C.c_void_p(d_vals.data_ptr()), int(d_vals.numel()),
                                                       C.c_void_p(d_out.data_ptr()),
                                                       C.c_void_p(stream) if stream else None)
        _check(rc, "shd_route_min_reduce_async")

    def fw_table_async(self, stream=None):
        """K4: the all-pairs u16 table by blocked min-plus Floyd-Warshall (kept on the device)."""
        _check(load_library().shd_route_fw_table_async(self._h, C.c_void_p(stream) if stream else None),
               "shd_route_fw_table_async")

    def fw_rows_async(self, d_src, d_tgt, d_lat, d_rel, d_rowmin, stream=None, ld=None):
        ns, nt = int(d_src.numel()), int(d_tgt.numel())
        ld = nt if ld is None else int(ld)
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        _check(load_library().shd_route_fw_rows_async(self._h, ptr(d_src), ns, ptr(d_tgt), nt, ld, ptr(d_lat),
                                                      ptr(d_rel), ptr(d_rowmin), C.c_void_p(stream) if stream else None),
               "shd_route_fw_rows_async")

    def fill_triangle(self, attached, out, world: int = 1, rank: int = 0, dispatch: bool = True,
                      lat16: bool = False):
        """shd_route_fill_triangle: this rank's rows of the front end's upper-triangle cache
        over the sorted `attached` vertices into `out` (a PinnedBuffer or any object with
        .ptr; 16 * na * (na + 1) / 2 bytes, or 64 * tri16_lines(na) with lat16: the compact
        layout).  Returns (min latency written, seconds)."""
        A = np.ascontiguousarray(attached, np.int32)
        mn, sec = C.c_double(), C.c_double()
        flags = (DISPATCH if dispatch else 0) | (FILL_LAT16 if lat16 else 0)
        rc = load_library().shd_route_fill_triangle(self._h, _p(A), len(A), int(world), int(rank),
                                                   flags, C.c_void_p(out.ptr),
                                                   C.byref(mn), C.byref(sec))
        if rc not in (OK, ENOEDGE, EUNREACH):
            raise RouteError(rc, "shd_route_fill_triangle")
        return mn.value, sec.value

    def tri_payload_async(self, d_lat, d_rel, d_pos, d_off, na, out_lat, out_rel, lat16=True, stream=None, ld=None):
        """shd_route_tri_payload_async: the upper-triangle payload of this rank's rows
        (row r = attached position d_pos[r], targets j >= it) at offsets d_off - d_off[0]."""
        nrows = int(d_pos.numel())
        ld = int(d_lat.shape[1]) if ld is None else int(ld)
        ptr = lambda t: C.c_void_p(t.data_ptr())
        _check(load_library().shd_route_tri_payload_async(
            self._h, ptr(d_lat), ptr(d_rel), ld, ptr(d_pos), ptr(d_off), nrows, int(na),
            PAYLOAD_LAT16 if lat16 else 0, ptr(out_lat), ptr(out_rel), C.c_void_p(stream) if stream else None),
            "shd_route_tri_payload_async")

    def kd_stats(self, reset: bool = True):
        """shd_route_kd_stats: the longest KD waits (s_sleep rounds) since the last reset:
        ring space, writer on an unwritten record, slice on an unwritten queue entry."""
        out = np.zeros(4, np.uint64)
        _check(load_library().shd_route_kd_stats(self._h, _p(out), int(reset)), "shd_route_kd_stats")
        return [int(x) for x in out[:3]]

    def plan(self, sources, world: int = 1, rank: int = 0) -> "RoutePlan":
        return RoutePlan(self, sources, world, rank)

    def fw_async(self, d_dist, stream=None):
        _check(load_library().shd_route_fw_async(self._h, C.c_void_p(d_dist.data_ptr()),
                                                 C.c_void_p(stream) if stream else None), "shd_route_fw_async")


class RoutePlan:
    """A seeded plan over a source list (shd_route_plan_*): this rank's output rows, the
    launches that compute them and the device row store.  Keep it for repeated fills."""

    def __init__(self, eng: RouteEngine, sources, world: int = 1, rank: int = 0):
        L = load_library()
        self.eng = eng
        src = np.ascontiguousarray(sources, np.int32)
        h = C.c_void_p()
        _check(L.shd_route_plan_create(eng._h, _p(src), len(src), int(world), int(rank), C.byref(h)),
               "shd_route_plan_create")
        self._h = h
        eng._plans.add(self)
        inf = _PlanInfo()
        _check(L.shd_route_plan_get_info(self._h, C.byref(inf)), "shd_route_plan_get_info")
        self.info = {k: getattr(inf, k) for k, _ in _PlanInfo._fields_ if not k.endswith("_")}
        pos = np.empty(max(1, self.info["rows"]), np.int32)
        _check(L.shd_route_plan_rows(self._h, _p(pos)), "shd_route_plan_rows")
        self.positions = pos[: self.info["rows"]]
        self.sources = src[self.positions]

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            load_library().shd_route_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def rows_async(self, d_tgt, d_lat, d_rel, d_rowmin, stream=None, dispatch=True, ld=None, reuse=False):
        """The plan's rows (shd_route_rows_planned_async).  A device-built landmark-only plan
        recomputes its landmark rows and job records first, unless reuse=True
        (SHD_ROUTE_PLAN_REUSE: the last refresh_async's, for timing the rows launch alone)."""
        nt = int(d_tgt.numel())
        ld = nt if ld is None else int(ld)
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        flags = (DISPATCH if dispatch else 0) | (PLAN_REUSE if reuse else 0)
        rc = load_library().shd_route_rows_planned_async(
            self.eng._h, self._h, ptr(d_tgt), nt, ld, flags, ptr(d_lat), ptr(d_rel),
            ptr(d_rowmin), C.c_void_p(stream) if stream else None)
        _check(rc, "shd_route_rows_planned_async")

    def refresh_async(self, stream=None, what: int = 0):
        """The landmark rows, queue order and job records of a device-built landmark-only
        plan (shd_route_plan_refresh_async; what: REFRESH_ALL / REFRESH_MINE / REFRESH_JOBS,
        0 = all landmark rows + jobs); nothing for other plans."""
        rc = load_library().shd_route_plan_refresh_async(self.eng._h, self._h, int(what),
                                                         C.c_void_p(stream) if stream else None)
        _check(rc, "shd_route_plan_refresh_async")

    def landmarks(self):
        """The landmark store of a device-built landmark-only plan: {nland, first, count,
        row_stride} (this rank's share = slots [first, first + count)), or None."""
        a, b, c, d = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
        rc = load_library().shd_route_plan_landmarks(self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(d))
        if rc == EUNSUPPORTED:
            return None
        _check(rc, "shd_route_plan_landmarks")
        return {"nland": a.value, "first": b.value, "count": c.value, "row_stride": d.value}

    def bind_store(self, d_drow, d_prow):
        """Move the landmark store into caller tensors (int16 / int32, nland x row_stride at
        least), which the plan keeps a reference to."""
        rc = load_library().shd_route_plan_bind_store(self.eng._h, self._h, C.c_void_p(d_drow.data_ptr()),
                                                      C.c_void_p(d_prow.data_ptr()))
        _check(rc, "shd_route_plan_bind_store")
        self._store = (d_drow, d_prow)


def tri16_lines(na: int, i: int | None = None) -> int:
    """shd_route_tri16_line: first 64-byte line of row i of the compact triangle (i = na, the
    default: the line count)."""
    na = int(na)
    i = na if i is None else int(i)
    pad = (i // 6) * 15 + sum((6 - (na - t) % 6) % 6 for t in range(i % 6))
    return (i * na - i * (i - 1) // 2 + pad) // 6


class PinnedBuffer:
    """Pinned host memory (shd_route_host_alloc) viewed as float64.  lazy: pinned in the
    background (shd_route_host_alloc_lazy); hand it to the device only through fill_triangle
    until wait() returns."""

    def __init__(self, nbytes: int, lazy: bool = False):
        self.nbytes = int(nbytes)
        name = "shd_route_host_alloc_lazy" if lazy else "shd_route_host_alloc"
        self.ptr = getattr(load_library(), name)(self.nbytes)
        if not self.ptr:
            raise RouteError(ENOMEM, name)

    def wait(self):
        _check(load_library().shd_route_host_wait(C.c_void_p(self.ptr)), "shd_route_host_wait")

    def unpinned(self) -> int:
        """Bytes of the buffer the runtime refused to register (pageable: still usable)."""
        n = int(load_library().shd_route_host_unpinned(C.c_void_p(self.ptr)))
        if n < 0:
            _check(n, "shd_route_host_unpinned")
        return n

    def array(self):
        buf = (C.c_double * (self.nbytes // 8)).from_address(self.ptr)
        return np.frombuffer(buf, dtype=np.float64)

    def close(self):
        if getattr(self, "ptr", None):
            load_library().shd_route_host_free(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
