"""Self-loop utilities (PyG 1.4.3 utils.loop [U4]).

Edge-list rewrites feeding the aggregation; the output order matters for the
fp32 summation order, so it follows upstream exactly: kept edges in original
order, then the N loop edges 0..N-1.  They run on the native engine
(mi355_mp.ops.self_loops -> mp_self_loops: stable compaction + loop append,
loop weights by a position gather); like every hot-path op they need device
tensors (no CPU fallback).
"""
from mi355_mp import ops as _ops

from .num_nodes import maybe_num_nodes


def contains_self_loops(edge_index):
    row, col = edge_index
    return bool((row == col).sum() > 0)


def remove_self_loops(edge_index, edge_attr=None):
    ei, pos = _ops.self_loops(edge_index, maybe_num_nodes(edge_index), "remove")
    return ei, (None if edge_attr is None else edge_attr[pos])


def add_self_loops(edge_index, edge_weight=None, fill_value=1, num_nodes=None):
    num_nodes = maybe_num_nodes(edge_index, num_nodes)
    ei, pos = _ops.self_loops(edge_index, num_nodes, "add")
    if edge_weight is not None:
        assert edge_weight.numel() == edge_index.size(1)
        edge_weight = _ops.gather_fill(edge_weight, pos, fill_value)
    return ei, edge_weight


def add_remaining_self_loops(edge_index, edge_weight=None, fill_value=1, num_nodes=None):
    """Drop existing loops, append one loop per node; a node's loop keeps the
    weight of its LAST pre-existing loop (upstream's sequential CPU index_put_),
    else `fill_value`."""
    num_nodes = maybe_num_nodes(edge_index, num_nodes)
    ei, pos = _ops.self_loops(edge_index, num_nodes, "add_remaining")
    if edge_weight is not None:
        assert edge_weight.numel() == edge_index.size(1)
        edge_weight = _ops.gather_fill(edge_weight, pos, fill_value)
    return ei, edge_weight
