"""torch_geometric.utils.softmax (PyG 1.4.3 [U3]):

    out = exp(src - scatter_max(src, index)[0][index])
    out = out / (scatter_add(out, index)[index] + 1e-16)

Sparse (segment-wise) softmax over the rows grouped by `index`; every
scatter/gather step runs on the native engine.  (GATConv itself does not
call this: its softmax is fused into mp_gat_aggregate_f32.)
"""
import math as _math
from mi355_mp import ops as _ops

from .num_nodes import maybe_num_nodes


def softmax(src, index, num_nodes=None):
    num_nodes = maybe_num_nodes(index, num_nodes)
    flat = src.reshape(src.shape[0], _math.prod(src.shape[1:]))
    mx, _ = _ops.segment_reduce(flat, index, num_nodes, "max")
    out = (flat - _ops.index_select_rows(mx, index)).exp()
    den, _ = _ops.segment_reduce(out, index, num_nodes, "sum")
    out = out / (_ops.index_select_rows(den, index) + 1e-16)
    return out.reshape(src.shape)
