"""get_laplacian (PyG 1.4.3 torch_geometric.utils.get_laplacian [U]; the
normalisation ChebConv applies before it propagates, ConvexPruning.py:259-264).

    None : L = D - A            (loops appended with weight deg)
    'sym': L = I - D^-1/2 A D^-1/2
    'rw' : L = I - D^-1 A

Self loops are removed first; the Laplacian's diagonal is appended as loops
0..N-1 after the remaining edges (upstream's order, which fixes the fp32
summation order of every later propagate).  deg = scatter_add(w, row) runs on
the native serial segment sum (edge order per node, the CPU scatter_add_'s
arithmetic bit for bit), deg^-1/2 on mp_gcn_norm_from_deg_f32 (torch's CPU
pow(-0.5) rounding), the loop rewrites on mp_self_loops.
"""
import torch

import torch_scatter
from mi355_mp import ops as _ops
from mi355_mp.graph import csr_for_index

from .loop import remove_self_loops, add_self_loops
from .num_nodes import maybe_num_nodes


def get_laplacian(edge_index, edge_weight=None, normalization=None, dtype=None, num_nodes=None):
    assert normalization in [None, "sym", "rw"], "Invalid normalization"
    edge_index, edge_weight = remove_self_loops(edge_index, edge_weight)
    if edge_weight is None:
        edge_weight = torch.ones((edge_index.size(1),), dtype=dtype, device=edge_index.device)
    num_nodes = maybe_num_nodes(edge_index, num_nodes)
    row, col = edge_index
    exact = edge_index.is_cuda and not edge_weight.requires_grad and edge_weight.dtype == torch.float32
    if exact:
        # the reference's edge-order scatter_add_, bit for bit (serial segment sum)
        deg = _ops.segment_sum_serial(csr_for_index(row, num_nodes), edge_weight)
    else:
        deg = torch_scatter.scatter_add(edge_weight, row, dim=0, dim_size=num_nodes)
    if normalization is None:
        # L = D - A
        edge_index, _ = add_self_loops(edge_index, num_nodes=num_nodes)
        edge_weight = torch.cat([-edge_weight, deg], dim=0)
    elif normalization == "sym":
        # A_norm = -D^-1/2 A D^-1/2, L = I - A_norm
        if exact:   # deg^-1/2 with torch's CPU pow(-0.5) rounding (gfx950's sqrt is not correctly rounded)
            edge_weight = _ops.norm_from_degree(row, col, deg.clone(), edge_weight)
        else:
            deg_inv_sqrt = deg.pow(-0.5)
            deg_inv_sqrt[deg_inv_sqrt == float("inf")] = 0
            edge_weight = deg_inv_sqrt[row] * edge_weight * deg_inv_sqrt[col]
        edge_index, edge_weight = add_self_loops(edge_index, -edge_weight, fill_value=1, num_nodes=num_nodes)
    else:
        # A_norm = -D^-1 A, L = I - A_norm
        deg_inv = 1.0 / deg
        deg_inv[deg_inv == float("inf")] = 0
        edge_weight = deg_inv[row] * edge_weight
        edge_index, edge_weight = add_self_loops(edge_index, -edge_weight, fill_value=1, num_nodes=num_nodes)
    return edge_index, edge_weight
