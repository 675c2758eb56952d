"""Cached self-loop rewrites of a user's edge_index (structure only).

GCNConv/GATConv rewrite edge_index on every forward upstream;
the rewritten tensor is a new object each time, which would force a new CSR
sort per forward.  The rewrite depends only on the input tensor, so it is
cached on that tensor (identity + version, dropped with it) -- results are
identical to recomputing it.  The rewrite itself is native (mp_self_loops).
"""
from mi355_mp import ops as _ops
from mi355_mp.graph import _Cache

_cache = _Cache()


def remaining_loops_structure(edge_index, num_nodes):
    """(edge_index with remaining self loops, pos): the structure half of
    add_remaining_self_loops; pos[k] = input edge whose weight edge k carries
    (its own, or for a loop the node's LAST pre-existing loop), -1 = fill."""
    return _cache.get(edge_index, ("remaining", int(num_nodes)),
                      lambda: _ops.self_loops(edge_index, num_nodes, "add_remaining"))


def remaining_loops_weight(edge_weight, pos, fill_value):
    """The weight half of add_remaining_self_loops (same order and values)."""
    return _ops.gather_fill(edge_weight, pos, fill_value)


def gat_loops(edge_index, num_nodes):
    """remove_self_loops + add_self_loops(num_nodes) (GATConv.forward), cached:
    the same edge list as the structure of add_remaining_self_loops."""
    return remaining_loops_structure(edge_index, num_nodes)[0]


def cached_value(key_tensor, tag, factory):
    return _cache.get(key_tensor, tag, factory)
