"""torch_geometric.utils.scatter_ (PyG 1.4.3 [U2]).

Dispatches to torch_scatter.scatter_{add,mean,min,max}, keeps the first
element of tuple results, and masks max -> out < -10000 := 0,
min -> out > 10000 := 0.  Here the mask is fused into the native reduction
(MP_FLAG_PYG_MASK) for every device dtype the engine takes.
"""
import math as _math
import torch_scatter

from mi355_mp import ops as _ops


def scatter_(name, src, index, dim=0, dim_size=None):
    assert name in ["add", "mean", "min", "max"]
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() > 0 else 0
    d = dim % src.dim()
    if d == 0 and index.dim() == 1:
        flat = src.reshape(src.shape[0], _math.prod(src.shape[1:]))
        out, _ = _ops.segment_reduce(flat, index, dim_size, name, pyg_mask=name in ("min", "max"))
        return out.reshape((out.shape[0],) + tuple(src.shape[1:]))
    op = getattr(torch_scatter, "scatter_{}".format(name))
    out = op(src, index, dim, None, dim_size)
    out = out[0] if isinstance(out, tuple) else out
    if name == "max":
        out = out.masked_fill(out < -10000, 0)
    elif name == "min":
        out = out.masked_fill(out > 10000, 0)
    return out
