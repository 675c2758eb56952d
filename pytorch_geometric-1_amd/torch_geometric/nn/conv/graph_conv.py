"""GraphConv (PyG 1.4.3 nn.conv.graph_conv [U7]): the aggr='max' user on the path.

    x'_i = Theta_1 x_i + AGGR_{j in N(i)} e_ji * Theta_2 x_j

With aggr='max' this is the segmented max + first-index argmax kernel
(torch_scatter scatter_max semantics + scatter_'s -10000 mask).
"""
import torch
from torch.nn import Parameter

from ..inits import uniform
from .message_passing import MessagePassing


class GraphConv(MessagePassing):
    def __init__(self, in_channels, out_channels, aggr="add", bias=True, **kwargs):
        super(GraphConv, self).__init__(aggr=aggr, **kwargs)
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.weight = Parameter(torch.Tensor(in_channels, out_channels))
        self.lin = torch.nn.Linear(in_channels, out_channels, bias=bias)
        self.reset_parameters()

    def reset_parameters(self):
        uniform(self.in_channels, self.weight)
        self.lin.reset_parameters()

    def forward(self, x, edge_index, edge_weight=None, size=None):
        """"""
        h = torch.matmul(x, self.weight)
        return self.propagate(edge_index, size=size, x=x, h=h, edge_weight=edge_weight)

    def message(self, h_j, edge_weight):
        return h_j if edge_weight is None else edge_weight.view(-1, 1) * h_j

    def update(self, aggr_out, x):
        return aggr_out + self.lin(x)

    def _fused_message(self, kwargs):
        if type(self).message is GraphConv.message:
            return "h", kwargs.get("edge_weight", None)
        return None

    def __repr__(self):
        return "{}({}, {})".format(self.__class__.__name__, self.in_channels, self.out_channels)
