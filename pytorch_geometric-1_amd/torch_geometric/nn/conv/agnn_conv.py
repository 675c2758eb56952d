"""AGNNConv (PyG 1.4.3 nn.conv.agnn_conv [U]; caller
/root/reference/ConvexPruning.py:236-237, `AGNNConv(requires_grad=True)`).

    x'_i = sum_{j in N(i) u {i}} P_ij x_j,
    P_ij = softmax_j( beta * cos(x_i, x_j) )

forward: self loops removed then added, x_norm = F.normalize(x, p=2, dim=-1),
propagate(edge_index, x=x, x_norm=x_norm, num_nodes=N).  The message reads
x_norm at both ends, so it runs on the generic path: native row gathers of
x_j / x_norm_i / x_norm_j, the per-edge score, utils.softmax on the native
segment max / sum (+1e-16), and the native segmented sum of x_j * alpha.
"""
import torch
import torch.nn.functional as F
from torch.nn import Parameter

from ...utils import remove_self_loops, add_self_loops, softmax
from .message_passing import MessagePassing


class AGNNConv(MessagePassing):
    def __init__(self, requires_grad=True, **kwargs):
        super(AGNNConv, self).__init__(aggr="add", **kwargs)
        self.requires_grad = requires_grad
        if requires_grad:
            self.beta = Parameter(torch.Tensor(1))
        else:
            self.register_buffer("beta", torch.ones(1))
        self.reset_parameters()

    def reset_parameters(self):
        if self.requires_grad:
            self.beta.data.fill_(1)

    def forward(self, x, edge_index):
        """"""
        edge_index, _ = remove_self_loops(edge_index)
        edge_index, _ = add_self_loops(edge_index, num_nodes=x.size(self.node_dim))
        x_norm = F.normalize(x, p=2, dim=-1)
        return self.propagate(edge_index, x=x, x_norm=x_norm, num_nodes=x.size(self.node_dim))

    def message(self, edge_index_i, x_j, x_norm_i, x_norm_j, num_nodes):
        beta = self.beta if self.requires_grad else self._buffers["beta"]
        alpha = beta * (x_norm_i * x_norm_j).sum(dim=-1)
        alpha = softmax(alpha, edge_index_i, num_nodes)
        return x_j * alpha.view(-1, 1)

    def __repr__(self):
        return "{}()".format(self.__class__.__name__)
