"""Self-loop utilities (PyG 1.4.3 utils.loop [U4]).

Edge-list rewrites feeding the aggregation; the output order matters for the
fp32 summation order, so it follows upstream exactly: kept edges in original
order, then the N loop edges 0..N-1.
"""
import torch

from .num_nodes import maybe_num_nodes


def contains_self_loops(edge_index):
    row, col = edge_index
    return bool((row == col).sum() > 0)


def remove_self_loops(edge_index, edge_attr=None):
    row, col = edge_index
    mask = row != col
    edge_attr = edge_attr if edge_attr is None else edge_attr[mask]
    edge_index = edge_index[:, mask]
    return edge_index, edge_attr


def add_self_loops(edge_index, edge_weight=None, fill_value=1, num_nodes=None):
    num_nodes = maybe_num_nodes(edge_index, num_nodes)
    loop_index = torch.arange(0, num_nodes, dtype=torch.long, device=edge_index.device)
    loop_index = loop_index.unsqueeze(0).repeat(2, 1)
    if edge_weight is not None:
        assert edge_weight.numel() == edge_index.size(1)
        loop_weight = edge_weight.new_full((num_nodes,), fill_value)
        edge_weight = torch.cat([edge_weight, loop_weight], dim=0)
    edge_index = torch.cat([edge_index, loop_index], dim=1)
    return edge_index, edge_weight


def add_remaining_self_loops(edge_index, edge_weight=None, fill_value=1, num_nodes=None):
    """Drop existing loops, append one loop per node; a node's loop keeps the
    weight of its (last) pre-existing loop, else `fill_value`."""
    num_nodes = maybe_num_nodes(edge_index, num_nodes)
    row, col = edge_index
    mask = row != col
    inv_mask = ~mask
    loop_weight = torch.full((num_nodes,), fill_value,
                             dtype=None if edge_weight is None else edge_weight.dtype,
                             device=edge_index.device)
    if edge_weight is not None:
        assert edge_weight.numel() == edge_index.size(1)
        # sequential semantics of the CPU index_put_: with duplicate self
        # loops the LAST one's weight wins (deterministic on the device too)
        pos = torch.nonzero(inv_mask).view(-1)
        if pos.numel() > 0:
            last = torch.full((num_nodes,), -1, dtype=torch.long, device=row.device)
            last.scatter_reduce_(0, row[pos], pos, "amax", include_self=True)
            has = last >= 0
            loop_weight[has] = edge_weight[last[has]]
        edge_weight = torch.cat([edge_weight[mask], loop_weight], dim=0)
    loop_index = torch.arange(0, num_nodes, dtype=row.dtype, device=row.device)
    loop_index = loop_index.unsqueeze(0).repeat(2, 1)
    edge_index = torch.cat([edge_index[:, mask], loop_index], dim=1)
    return edge_index, edge_weight
