"""CPU: the C-ABI library loads and exports every symbol include/shd_route.h declares
(no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(ROOT, "include", "shd_route.h")).read()
    return sorted(set(re.findall(r"\b(shd_route_[a-z_]+)\s*\(", text)))


def test_header_matches_binding_exports():
    from shadow_amd import route
    assert sorted(route.EXPORTS) == header_symbols()


def test_library_exports_all_symbols():
    from shadow_amd import build, route
    if not os.path.exists(route.LIB_PATH):
        build.build()
    lib = ctypes.CDLL(route.LIB_PATH)
    for sym in header_symbols():
        assert hasattr(lib, sym), sym
    # pure host function: safe without a GPU
    route.load_library()
    assert route.strerror(route.ENOEDGE).startswith("path hop")
    assert route.strerror(0) == "success"


def test_no_cpu_fallback_when_missing(tmp_path, monkeypatch):
    from shadow_amd import route
    monkeypatch.setattr(route, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(route, "_lib", None)
    with pytest.raises(RuntimeError, match="not built"):
        route.load_library()


def test_product_does_not_import_oracle():
    """Only tests/, smoke() and bench.py's cpu_baseline may touch oracle/."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "shadow_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".c", ".cpp", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in txt.replace("oracle/", "").lower() or f == "__init__.py", f


def test_front_end_exports():
    import re
    from shadow_amd import build, topology
    build.build()
    text = open(os.path.join(ROOT, "include", "shd_topology.h")).read()
    declared = sorted(set(re.findall(r"\b(shd_(?:topology|graphml|attach)_[a-z_]+)\s*\(", text)))
    assert sorted(topology.EXPORTS) == declared
    lib = ctypes.CDLL(topology.LIB_PATH)
    for sym in declared:
        assert hasattr(lib, sym), sym
