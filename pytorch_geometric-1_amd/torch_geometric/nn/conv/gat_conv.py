"""GATConv (PyG 1.4.3 [U6]; callers /root/reference/ConvexPruning.py:209-214,
/root/reference/examples/ppi.py:22-28).

    alpha_ij = softmax_i(leaky_relu(a^T [W x_i || W x_j]))
    x'_i     = sum_j alpha_ij W x_j        (per head; concat or mean)

forward: x W on hipBLASLt; per-node scores a_dst = <Wx, att[:C]>,
a_src = <Wx, att[C:]> (a split of the reference's (cat[x_i,x_j]*att).sum(-1));
then leaky_relu + segment softmax (+1e-16) + weighted aggregation + bias in
ONE online-softmax HIP kernel (mp_gat_aggregate_f32).  Attention dropout in
training mode (dropout > 0) runs in the same fused training kernels: the keep
mask of (edge, head) is a hash of a seed drawn from torch's generator and the
edge's CSR slot, evaluated again by the backward, never stored
(mp_gat_aggregate_train_drop_f32; shapes outside mi355_mp.ops.gat_dropout_ok
take the generic message path).

Heads of any width: out_channels not a multiple of 4 are padded per head to
the next multiple of 4 (zero columns of W, att and bias; the padded output
columns are dropped), so the 16-byte row kernels apply; heads whose C/4 is not
a power of two <= 64 (the reference's own GAT stacks, heads=1 with random
widths) run the wide forms (mp_gat_node_scores_wide_f32, the training forward
reading a_src from the node-score array, mp_gat_backward_wide_f32).
"""
import torch
import torch.nn.functional as F
from torch.nn import Parameter

from mi355_mp import ops as _ops
from mi355_mp.graph import GAT_TARGET_TASKS, graph_for

from ...utils import softmax
from ..inits import glorot, zeros
from .message_passing import MessagePassing
from ._structure import gat_loops


class GATConv(MessagePassing):
    r"""The graph attentional operator from the `"Graph Attention Networks"
    <https://arxiv.org/abs/1710.10903>`_ paper.

    Args:
        in_channels (int), out_channels (int), heads (int, default 1),
        concat (bool, default True), negative_slope (float, default 0.2),
        dropout (float, default 0), bias (bool, default True).
    """

    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2, dropout=0,
                 bias=True, **kwargs):
        super(GATConv, self).__init__(aggr="add", **kwargs)
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.heads = heads
        self.concat = concat
        self.negative_slope = negative_slope
        self.dropout = dropout
        self.weight = Parameter(torch.Tensor(in_channels, heads * out_channels))
        self.att = Parameter(torch.Tensor(1, heads, 2 * out_channels))
        if bias and concat:
            self.bias = Parameter(torch.Tensor(heads * out_channels))
        elif bias and not concat:
            self.bias = Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.alpha = None
        self.reset_parameters()

    def reset_parameters(self):
        glorot(self.weight)
        glorot(self.att)
        zeros(self.bias)

    def _padded_channels(self):
        return (self.out_channels + 3) // 4 * 4

    def _can_fuse(self, x, size):
        return (size is None and torch.is_tensor(x) and x.is_cuda and x.dtype == torch.float32
                and type(self).message is GATConv.message and type(self).update is GATConv.update
                and type(self).aggregate is MessagePassing.aggregate and self.node_dim == 0
                and (self.dropout == 0 or not self.training
                     or _ops.gat_dropout_ok(self.heads, self._padded_channels(), self.dropout)))

    def forward(self, x, edge_index, size=None, return_attention_weights=False):
        """"""
        if size is None and torch.is_tensor(x):
            edge_index = gat_loops(edge_index, x.size(self.node_dim))

        if self._can_fuse(x, size):
            weight, att, fused_bias, C4 = self._fused_operands()
            xw = _ops.feature_transform(x, weight, row_exact=_ops.GAT_ROW_EXACT_GEMM)
            N = xw.size(0)
            graph = graph_for(edge_index, N, N, self.flow, target_tasks=GAT_TARGET_TASKS)
            drop = self.dropout if self.training else 0.0
            out, alpha = _ops.gat_propagate(graph, edge_index, xw, att, self.heads, C4, self.negative_slope,
                                            fused_bias, return_attention_weights, dropout=drop)
            out = self._finish(out, C4)
            if return_attention_weights:
                return out, (edge_index, alpha)
            return out

        # generic path (bipartite inputs, attention dropout, overridden hooks)
        if torch.is_tensor(x):
            x = torch.matmul(x, self.weight)
        else:
            x = (None if x[0] is None else torch.matmul(x[0], self.weight),
                 None if x[1] is None else torch.matmul(x[1], self.weight))
        out = self.propagate(edge_index, size=size, x=x, return_attention_weights=return_attention_weights)
        if return_attention_weights:
            alpha, self.alpha = self.alpha, None
            return out, (edge_index, alpha)
        return out

    def _fused_operands(self):
        """(weight, att, bias for the kernel or None, C4): per head, out_channels
        padded with zero columns to C4 (a multiple of 4) so the 16-byte row
        kernels apply; the concat bias is added in the kernel."""
        H, C = self.heads, self.out_channels
        C4 = (C + 3) // 4 * 4
        weight, att = self.weight, self.att
        fused_bias = self.bias if self.concat else None
        if C4 != C:
            weight = F.pad(weight.view(-1, H, C), (0, C4 - C)).view(-1, H * C4)
            att = F.pad(att.view(1, H, 2, C), (0, C4 - C)).view(1, H, 2 * C4)
            if fused_bias is not None:
                fused_bias = F.pad(fused_bias.view(H, C), (0, C4 - C)).view(H * C4)
        return weight, att, fused_bias, C4

    def _finish(self, out, C4):
        """The fused output [n, H*C4] -> GATConv.update's: padding dropped, heads
        concatenated (bias already in) or averaged (+ bias)."""
        H, C = self.heads, self.out_channels
        if C4 != C:
            out = out.view(-1, H, C4)[:, :, :C].reshape(-1, H * C).contiguous()
        if not self.concat:
            out = out.view(-1, H, C).mean(dim=1)
            if self.bias is not None:
                out = out + self.bias
        return out

    def message(self, edge_index_i, x_i, x_j, size_i, return_attention_weights):
        # Compute attention coefficients.
        x_j = x_j.view(-1, self.heads, self.out_channels)
        if x_i is None:
            alpha = (x_j * self.att[:, :, self.out_channels:]).sum(dim=-1)
        else:
            x_i = x_i.view(-1, self.heads, self.out_channels)
            alpha = (torch.cat([x_i, x_j], dim=-1) * self.att).sum(dim=-1)
        alpha = F.leaky_relu(alpha, self.negative_slope)
        alpha = softmax(alpha, edge_index_i, size_i)
        if return_attention_weights:
            self.alpha = alpha
        # Sample attention coefficients stochastically.
        alpha = F.dropout(alpha, p=self.dropout, training=self.training)
        return x_j * alpha.view(-1, self.heads, 1)

    def update(self, aggr_out):
        if self.concat is True:
            aggr_out = aggr_out.view(-1, self.heads * self.out_channels)
        else:
            aggr_out = aggr_out.mean(dim=1)
        if self.bias is not None:
            aggr_out = aggr_out + self.bias
        return aggr_out

    def _fused_message(self, kwargs):
        return None  # the fused GAT path is taken in forward()

    def __repr__(self):
        return "{}({}, {}, heads={})".format(self.__class__.__name__, self.in_channels, self.out_channels,
                                            self.heads)
