"""GINConv (PyG 1.4.3 nn.conv.gin_conv [U]; upstream example
examples/mutag_gin.py in the reference tree).

    x'_i = h_Theta( (1 + eps) x_i + sum_{j in N(i)} x_j )

Self loops are removed first; the neighbour sum is one fused gather ->
segment-sum HIP kernel (message x_j, no weight), the MLP stays torch.
"""
import torch

from ..inits import reset
from ...utils import remove_self_loops
from .message_passing import MessagePassing


class GINConv(MessagePassing):
    def __init__(self, nn, eps=0, train_eps=False, **kwargs):
        super(GINConv, self).__init__(aggr="add", **kwargs)
        self.nn = nn
        self.initial_eps = eps
        if train_eps:
            self.eps = torch.nn.Parameter(torch.Tensor([eps]))
        else:
            self.register_buffer("eps", torch.Tensor([eps]))
        self.reset_parameters()

    def reset_parameters(self):
        reset(self.nn)
        self.eps.data.fill_(self.initial_eps)

    def forward(self, x, edge_index):
        """"""
        x = x.unsqueeze(-1) if x.dim() == 1 else x
        edge_index, _ = remove_self_loops(edge_index)
        out = self.nn((1 + self.eps) * x + self.propagate(edge_index, x=x))
        return out

    def message(self, x_j):
        return x_j

    def _fused_message(self, kwargs):
        if type(self).message is GINConv.message:
            return "x", None
        return None

    def __repr__(self):
        return "{}(nn={})".format(self.__class__.__name__, self.nn)
