"""Self-loop utilities (PyG 1.4.3 utils.loop [U4]).

Edge-list rewrites feeding the aggregation; the output order matters for the
fp32 summation order, so it follows upstream exactly: kept edges in original
order, then the N loop edges 0..N-1.  Device tensors run on the native engine
(mi355_mp.ops.self_loops -> mp_self_loops: stable compaction + loop append,
loop weights by a position gather).  Host tensors -- one-off preprocessing
such as a CPU dataset transform (the reference's examples/qm9_nn_conv.py:43
`Complete` calls remove_self_loops before any .to(device)) -- take the same
rewrite in torch ops; the aggregation itself has no CPU path.
"""
import torch

from mi355_mp import ops as _ops

from .num_nodes import maybe_num_nodes


def contains_self_loops(edge_index):
    row, col = edge_index
    return bool((row == col).sum() > 0)


def _host_loops(edge_index, num_nodes, mode):
    """The host form of ops.self_loops: (edge_index_out, pos), pos[k] = input
    position whose weight output edge k carries (-1: the fill value)."""
    row, col = edge_index[0], edge_index[1]
    E = row.numel()
    ar = torch.arange(E, dtype=torch.int64)
    if mode == "add":
        keep = torch.ones(E, dtype=torch.bool)
    else:
        keep = row != col
    out = [edge_index[:, keep]]
    pos = [ar[keep]]
    if mode != "remove":
        N = int(num_nodes)
        loop = torch.arange(N, dtype=edge_index.dtype)
        out.append(torch.stack([loop, loop]))
        lpos = torch.full((N,), -1, dtype=torch.int64)
        if mode == "add_remaining":
            lr = row[~keep]
            if lr.numel() and (int(lr.min()) < 0 or int(lr.max()) >= N):
                raise IndexError("self loops name a node outside [0, %d)" % N)
            # upstream's sequential index_put_: the LAST loop of a node wins
            lpos.scatter_reduce_(0, lr.to(torch.int64), ar[~keep], "amax")
        pos.append(lpos)
    return torch.cat(out, dim=1), torch.cat(pos)


def _loops(edge_index, num_nodes, mode):
    if edge_index.is_cuda:
        return _ops.self_loops(edge_index, num_nodes, mode)
    return _host_loops(edge_index, num_nodes, mode)


def _weights(edge_weight, pos, fill_value):
    if edge_weight.is_cuda:
        return _ops.gather_fill(edge_weight, pos, fill_value)
    # gather only where an input edge exists: with no input edges (E == 0) the
    # weights are all fill values, as upstream's concatenation gives
    out = torch.full((pos.numel(),) + tuple(edge_weight.shape[1:]), fill_value, dtype=edge_weight.dtype)
    has = pos >= 0
    out[has] = edge_weight[pos[has]]
    return out


def remove_self_loops(edge_index, edge_attr=None):
    ei, pos = _loops(edge_index, maybe_num_nodes(edge_index), "remove")
    return ei, (None if edge_attr is None else edge_attr[pos])


def add_self_loops(edge_index, edge_weight=None, fill_value=1, num_nodes=None):
    num_nodes = maybe_num_nodes(edge_index, num_nodes)
    ei, pos = _loops(edge_index, num_nodes, "add")
    if edge_weight is not None:
        assert edge_weight.numel() == edge_index.size(1)
        edge_weight = _weights(edge_weight, pos, fill_value)
    return ei, edge_weight


def add_remaining_self_loops(edge_index, edge_weight=None, fill_value=1, num_nodes=None):
    """Drop existing loops, append one loop per node; a node's loop keeps the
    weight of its LAST pre-existing loop (upstream's sequential CPU index_put_),
    else `fill_value`."""
    num_nodes = maybe_num_nodes(edge_index, num_nodes)
    ei, pos = _loops(edge_index, num_nodes, "add_remaining")
    if edge_weight is not None:
        assert edge_weight.numel() == edge_index.size(1)
        edge_weight = _weights(edge_weight, pos, fill_value)
    return ei, edge_weight
