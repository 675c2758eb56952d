"""SAGEConv (PyG 1.4.3 nn.conv.sage_conv [U7], mean aggregation).

    x'_i = W * mean_{j in N(i) u {i}} x_j     (concat=False, loops added)
    x'_i = W * [x_i || mean_{j in N(i)} x_j]   (concat=True)

The mean over x_j (optionally edge-weighted) is the fused native path.
"""
import torch
import torch.nn.functional as F
from torch.nn import Parameter

from ..inits import uniform
from .message_passing import MessagePassing
from ._structure import remaining_loops_structure, remaining_loops_weight


class SAGEConv(MessagePassing):
    def __init__(self, in_channels, out_channels, normalize=False, concat=False, bias=True, **kwargs):
        super(SAGEConv, self).__init__(aggr="mean", **kwargs)
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.normalize = normalize
        self.concat = concat
        in_channels = 2 * in_channels if concat else in_channels
        self.weight = Parameter(torch.Tensor(in_channels, out_channels))
        if bias:
            self.bias = Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        uniform(self.weight.size(0), self.weight)
        uniform(self.weight.size(0), self.bias)

    def forward(self, x, edge_index, edge_weight=None, size=None, res_n_id=None):
        """"""
        if not self.concat and torch.is_tensor(x):
            # add_remaining_self_loops(edge_index, edge_weight, 1, N), structure cached on edge_index
            N = x.size(self.node_dim)
            ei, pos = remaining_loops_structure(edge_index, N)
            if edge_weight is not None:
                edge_weight = remaining_loops_weight(edge_weight, pos, 1)
            edge_index = ei
        return self.propagate(edge_index, size=size, x=x, edge_weight=edge_weight, res_n_id=res_n_id)

    def message(self, x_j, edge_weight):
        return x_j if edge_weight is None else edge_weight.view(-1, 1) * x_j

    def update(self, aggr_out, x, res_n_id):
        if self.concat and torch.is_tensor(x):
            aggr_out = torch.cat([x, aggr_out], dim=-1)
        elif self.concat and (isinstance(x, tuple) or isinstance(x, list)):
            if res_n_id is not None:
                aggr_out = torch.cat([x[0][res_n_id], aggr_out], dim=-1)
            else:
                aggr_out = torch.cat([x[1], aggr_out], dim=-1)
        aggr_out = torch.matmul(aggr_out, self.weight)
        if self.bias is not None:
            aggr_out = aggr_out + self.bias
        if self.normalize:
            aggr_out = F.normalize(aggr_out, p=2, dim=-1)
        return aggr_out

    def _fused_message(self, kwargs):
        if type(self).message is SAGEConv.message:
            return "x", kwargs.get("edge_weight", None)
        return None

    def __repr__(self):
        return "{}({}, {})".format(self.__class__.__name__, self.in_channels, self.out_channels)
