import torch

from .num_nodes import maybe_num_nodes


def degree(index, num_nodes=None, dtype=None):
    """Number of occurrences of each index value (PyG 1.4.3 utils.degree)."""
    num_nodes = maybe_num_nodes(index, num_nodes)
    out = torch.zeros((num_nodes,), dtype=dtype, device=index.device)
    return out.scatter_add_(0, index, out.new_ones((index.size(0),)))
