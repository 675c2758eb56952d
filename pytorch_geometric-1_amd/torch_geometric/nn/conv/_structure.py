"""Cached self-loop rewrites of a user's edge_index (structure only).

GCNConv/GATConv rewrite edge_index on every forward upstream;
the rewritten tensor is a new object each time, which would force a new CSR
sort per forward.  The rewrite depends only on the input tensor, so it is
cached on that tensor (identity + version, dropped with it) -- results are
identical to recomputing it.
"""
import torch

from mi355_mp.graph import _Cache

from ...utils.loop import add_self_loops, remove_self_loops

_cache = _Cache()


def last_loop_edge(edge_index, mask, num_nodes):
    """For every node with a pre-existing self loop: (nodes, position of its
    LAST loop edge).  Upstream's `loop_weight[row[inv_mask]] = w[inv_mask]`
    is a sequential index_put_ on the CPU, so with duplicate loops the last
    one wins; a device index_put_ with duplicates would pick any of them."""
    row = edge_index[0]
    pos = torch.nonzero(~mask).view(-1)
    last = torch.full((num_nodes,), -1, dtype=torch.long, device=row.device)
    if pos.numel():
        last.scatter_reduce_(0, row[pos], pos, "amax", include_self=True)
    nodes = torch.nonzero(last >= 0).view(-1)
    return nodes, last[nodes]


def remaining_loops_structure(edge_index, num_nodes):
    """(edge_index with remaining self loops, kept-edge mask, (loop nodes,
    their last loop edge)) -- the structure half of add_remaining_self_loops."""

    def build():
        row, col = edge_index
        mask = row != col
        loop_index = torch.arange(0, num_nodes, dtype=row.dtype, device=row.device)
        loop_index = loop_index.unsqueeze(0).repeat(2, 1)
        ei = torch.cat([edge_index[:, mask], loop_index], dim=1)
        return ei, mask, last_loop_edge(edge_index, mask, num_nodes)

    return _cache.get(edge_index, ("remaining", int(num_nodes)), build)


def remaining_loops_weight(edge_weight, mask, loops, num_nodes, fill_value):
    """The weight half of add_remaining_self_loops (same order and values)."""
    loop_weight = torch.full((num_nodes,), fill_value, dtype=edge_weight.dtype, device=edge_weight.device)
    nodes, last = loops
    if nodes.numel() > 0:
        loop_weight[nodes] = edge_weight[last]
    return torch.cat([edge_weight[mask], loop_weight], dim=0)


def gat_loops(edge_index, num_nodes):
    """remove_self_loops + add_self_loops(num_nodes) (GATConv.forward), cached."""

    def build():
        ei, _ = remove_self_loops(edge_index)
        ei, _ = add_self_loops(ei, num_nodes=num_nodes)
        return ei

    return _cache.get(edge_index, ("gat", int(num_nodes)), build)


def cached_value(key_tensor, tag, factory):
    return _cache.get(key_tensor, tag, factory)
