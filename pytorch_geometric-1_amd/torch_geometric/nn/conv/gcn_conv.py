"""GCNConv (PyG 1.4.3 [U5]; callers /root/reference/examples/gcn.py:18-19,
/root/reference/ConvexPruning.py:180-185 with cached=True).

    x' = D^-1/2 (A + I) D^-1/2 X W + b

forward: X W on hipBLASLt (torch.matmul), then the normalised aggregation
+ bias as one fused HIP kernel (mi355_mp).  The normalisation (deg over
edge_index[0] after add_remaining_self_loops, deg^-1/2 with inf -> 0,
norm = dinv[row] * w * dinv[col]) is the native mp_gcn_norm_f32.

``aggregate_first=True`` (an extension; default False keeps the reference's
order and results): when in_channels < out_channels the layer computes
(Â X) W + b instead of Â (X W) + b -- the aggregation then moves
in_channels-wide rows instead of out_channels-wide ones.  The
two orders agree to rounding, not bit for bit.
"""
import torch
from torch.nn import Parameter

import torch_scatter

from mi355_mp import ops as _ops
from mi355_mp.graph import graph_for

from ..inits import glorot, zeros
from .message_passing import MessagePassing
from ._structure import remaining_loops_structure, remaining_loops_weight, cached_value


class GCNConv(MessagePassing):
    r"""The graph convolutional operator from the `"Semi-supervised
    Classification with Graph Convolutional Networks"
    <https://arxiv.org/abs/1609.02907>`_ paper.

    Args:
        in_channels (int): Size of each input sample.
        out_channels (int): Size of each output sample.
        improved (bool): use A + 2I. (default: False)
        cached (bool): cache the normalised edge_index/norm of the first call.
        bias (bool): learn an additive bias. (default: True)
        normalize (bool): apply the symmetric normalisation. (default: True)
        aggregate_first (bool): aggregate before the feature transform when
            in_channels < out_channels. (default: False)
    """

    def __init__(self, in_channels, out_channels, improved=False, cached=False, bias=True,
                 normalize=True, aggregate_first=False, **kwargs):
        super(GCNConv, self).__init__(aggr="add", **kwargs)
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.improved = improved
        self.cached = cached
        self.normalize = normalize
        self.aggregate_first = aggregate_first
        self.weight = Parameter(torch.Tensor(in_channels, out_channels))
        if bias:
            self.bias = Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        glorot(self.weight)
        zeros(self.bias)
        self.cached_result = None
        self.cached_num_edges = None

    @staticmethod
    def norm(edge_index, num_nodes, edge_weight=None, improved=False, dtype=None):
        fill_value = 1 if not improved else 2
        ei, pos = remaining_loops_structure(edge_index, num_nodes)
        if edge_weight is None:
            if dtype in (None, torch.float32):
                # depends on the structure only: cache it with the structure
                def build():
                    ones = torch.ones((edge_index.size(1),), dtype=torch.float32, device=edge_index.device)
                    w = remaining_loops_weight(ones, pos, fill_value)
                    return _ops.gcn_norm_weights(ei, num_nodes, w, integer_weights=True)
                norm = cached_value(edge_index, ("gcn_norm", int(num_nodes), fill_value), build)
                return ei, norm
            edge_weight = torch.ones((edge_index.size(1),), dtype=dtype, device=edge_index.device)
        w = remaining_loops_weight(edge_weight, pos, fill_value)
        if w.dtype != torch.float32 or (torch.is_grad_enabled() and w.requires_grad):
            # a float64 / half model, or learned edge weights: upstream's form in the
            # weights' dtype and differentiable, so the gradient reaches edge_weight
            # through deg and norm (the degree's scatter_add on the native segmented
            # sum of that dtype, in edge order, with its autograd)
            row, col = ei
            deg = torch_scatter.scatter_add(w, row, dim=0, dim_size=num_nodes)
            deg_inv_sqrt = deg.pow(-0.5)
            deg_inv_sqrt = deg_inv_sqrt.masked_fill(deg_inv_sqrt == float("inf"), 0)
            return ei, deg_inv_sqrt[row] * w * deg_inv_sqrt[col]
        return ei, _ops.gcn_norm_weights(ei, num_nodes, w)

    def forward(self, x, edge_index, edge_weight=None):
        """"""
        reorder = self.aggregate_first and self.in_channels < self.out_channels
        if not reorder:
            x = _ops.feature_transform(x, self.weight)

        if self.cached and self.cached_result is not None:
            if edge_index.size(1) != self.cached_num_edges:
                raise RuntimeError(
                    "Cached {} number of edges, but found {}. Please disable the caching behavior "
                    "of this layer by removing the `cached=True` argument in its constructor."
                    .format(self.cached_num_edges, edge_index.size(1)))

        if not self.cached or self.cached_result is None:
            self.cached_num_edges = edge_index.size(1)
            if self.normalize:
                edge_index, norm = self.norm(edge_index, x.size(self.node_dim), edge_weight,
                                             self.improved, x.dtype)
            else:
                norm = edge_weight
            self.cached_result = edge_index, norm

        edge_index, norm = self.cached_result
        if reorder:
            n = x.size(self.node_dim)
            graph = graph_for(edge_index, n, n, self.flow)
            h = _ops.fused_propagate(graph, x, edge_index, edge_weight=norm, reduce="sum")
            out = _ops.feature_transform(h, self.weight)
            return out + self.bias if self.bias is not None else out
        return self.propagate(edge_index, x=x, norm=norm)

    def message(self, x_j, norm):
        return norm.view(-1, 1) * x_j if norm is not None else x_j

    def update(self, aggr_out):
        if self.bias is not None:
            aggr_out = aggr_out + self.bias
        return aggr_out

    # fused form: message = norm * x_j, update = + bias
    def _fused_message(self, kwargs):
        if type(self).message is GCNConv.message:
            return "x", kwargs.get("norm", None)
        return None

    def _fused_bias(self):
        if type(self).update is GCNConv.update:
            return self.bias, True
        return None, False

    def __repr__(self):
        return "{}({}, {})".format(self.__class__.__name__, self.in_channels, self.out_channels)

