"""ChebConv (PyG 1.4.3 nn.conv.cheb_conv [U]; caller
/root/reference/ConvexPruning.py:259-264, `ChebConv(in, out, K=1)`).

    X' = sum_k T_k(L_hat) X Theta_k,   L_hat = 2 L / lambda_max - I
    T_0 = X, T_1 = L_hat X, T_k = 2 L_hat T_{k-1} - T_{k-2}

norm(): self loops removed, get_laplacian, the weights scaled by
2 / lambda_max (inf -> 0), then add_self_loops with fill -1 (the "- I") --
the Laplacian's own diagonal loops and the -1 loops stay separate edges,
summed in that order, as upstream.  Every L_hat X is one propagate with
message norm * x_j: the fused gather * weight -> segment-sum HIP kernel.
"""
import torch
from torch.nn import Parameter

from ..inits import glorot, zeros
from ...utils import remove_self_loops, add_self_loops, get_laplacian
from .message_passing import MessagePassing


class ChebConv(MessagePassing):
    def __init__(self, in_channels, out_channels, K, normalization="sym", bias=True, **kwargs):
        super(ChebConv, self).__init__(aggr="add", **kwargs)
        assert K > 0
        assert normalization in [None, "sym", "rw"], "Invalid normalization"
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.normalization = normalization
        self.weight = Parameter(torch.Tensor(K, in_channels, out_channels))
        if bias:
            self.bias = Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        glorot(self.weight)
        zeros(self.bias)

    @staticmethod
    def norm(edge_index, num_nodes, edge_weight, normalization, lambda_max, dtype=None, batch=None):
        edge_index, edge_weight = remove_self_loops(edge_index, edge_weight)
        edge_index, edge_weight = get_laplacian(edge_index, edge_weight, normalization, dtype, num_nodes)
        if batch is not None and torch.is_tensor(lambda_max):
            lambda_max = lambda_max[batch[edge_index[0]]]
        edge_weight = (2.0 * edge_weight) / lambda_max
        edge_weight.masked_fill_(edge_weight == float("inf"), 0)
        edge_index, edge_weight = add_self_loops(edge_index, edge_weight, fill_value=-1, num_nodes=num_nodes)
        return edge_index, edge_weight

    def forward(self, x, edge_index, edge_weight=None, batch=None, lambda_max=None):
        """"""
        if self.normalization != "sym" and lambda_max is None:
            raise ValueError("You need to pass `lambda_max` to `forward() in`"
                             "case the normalization is non-symmetric.")
        lambda_max = 2.0 if lambda_max is None else lambda_max
        edge_index, norm = self.norm(edge_index, x.size(0), edge_weight, self.normalization, lambda_max,
                                     dtype=x.dtype, batch=batch)
        Tx_0 = x
        out = torch.matmul(Tx_0, self.weight[0])
        if self.weight.size(0) > 1:
            Tx_1 = self.propagate(edge_index, x=x, norm=norm)
            out = out + torch.matmul(Tx_1, self.weight[1])
        for k in range(2, self.weight.size(0)):
            Tx_2 = 2 * self.propagate(edge_index, x=Tx_1, norm=norm) - Tx_0
            out = out + torch.matmul(Tx_2, self.weight[k])
            Tx_0, Tx_1 = Tx_1, Tx_2
        if self.bias is not None:
            out = out + self.bias
        return out

    def message(self, x_j, norm):
        return norm.view(-1, 1) * x_j

    # fused form: message = norm * x_j, default aggregate / update
    def _fused_message(self, kwargs):
        if type(self).message is ChebConv.message:
            return "x", kwargs.get("norm", None)
        return None

    def __repr__(self):
        return "{}({}, {}, K={}, normalization={})".format(self.__class__.__name__, self.in_channels,
                                                           self.out_channels, self.weight.size(0),
                                                           self.normalization)
