"""shadow_amd -- MI355X-native routing engine for Shadow's topology shortest-path hot path.

Product: the HIP/C-ABI library shadow_amd/libshd_route.so (include/shd_route.h).
Python modules here are the host-side driver: graph container and generators,
the ctypes binding, the eager path cache mirror of topology.c and multi-GPU sharding.
"""
from .graph import Graph, config, example_one_vertex, internet_like, complete_graph  # noqa: F401

__all__ = ["Graph", "config", "example_one_vertex", "internet_like", "complete_graph"]
