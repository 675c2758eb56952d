"""mi355_mp — MI355X-native message-passing aggregation engine.

HIP kernels for gfx950 (csrc/) behind the C-ABI of include/mi355_mp.h,
bound with ctypes (``_lib``); torch-facing ops with autograd (``ops``);
CSR/schedule caches (``graph``); synthetic graph generators (``graphgen``);
destination-range sharding with RCCL halo exchange (``dist``).
"""
from . import _lib  # noqa: F401
from .graph import CSR, Graph, graph_for, csr_for_index, clear_caches  # noqa: F401

__all__ = ["CSR", "Graph", "graph_for", "csr_for_index", "clear_caches", "load_native"]


def load_native():
    """Load libmi355_mp.so (raises if it was not built)."""
    return _lib.load()
