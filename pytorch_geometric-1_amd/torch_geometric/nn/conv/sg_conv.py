"""SGConv (PyG 1.4.3 nn.conv.sg_conv [U]; upstream example examples/sgc.py
in the reference tree).

    X' = (D^-1/2 (A + I) D^-1/2)^K X Theta

K propagates of GCNConv's normalised graph (GCNConv.norm: native loop rewrite
+ mp_gcn_norm_f32), each one fused gather * norm -> segment-sum HIP kernel,
then the linear layer.  cached=True keeps the propagated features (upstream
caches S^K X, not only the normalisation).
"""
from torch.nn import Linear

from .gcn_conv import GCNConv
from .message_passing import MessagePassing


class SGConv(MessagePassing):
    def __init__(self, in_channels, out_channels, K=1, cached=False, bias=True, **kwargs):
        super(SGConv, self).__init__(aggr="add", **kwargs)
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.K = K
        self.cached = cached
        self.lin = Linear(in_channels, out_channels, bias=bias)
        self.reset_parameters()

    def reset_parameters(self):
        self.lin.reset_parameters()
        self.cached_result = None
        self.cached_num_edges = None

    def forward(self, x, edge_index, edge_weight=None):
        """"""
        if self.cached and self.cached_result is not None:
            if edge_index.size(1) != self.cached_num_edges:
                raise RuntimeError(
                    "Cached {} number of edges, but found {}. Please disable the caching behavior "
                    "of this layer by removing the `cached=True` argument in its constructor."
                    .format(self.cached_num_edges, edge_index.size(1)))
        if not self.cached or self.cached_result is None:
            self.cached_num_edges = edge_index.size(1)
            edge_index, norm = GCNConv.norm(edge_index, x.size(self.node_dim), edge_weight, dtype=x.dtype)
            for k in range(self.K):
                x = self.propagate(edge_index, x=x, norm=norm)
            self.cached_result = x
        return self.lin(self.cached_result)

    def message(self, x_j, norm):
        return norm.view(-1, 1) * x_j

    def _fused_message(self, kwargs):
        if type(self).message is SGConv.message:
            return "x", kwargs.get("norm", None)
        return None

    def __repr__(self):
        return "{}({}, {}, K={})".format(self.__class__.__name__, self.in_channels, self.out_channels, self.K)
