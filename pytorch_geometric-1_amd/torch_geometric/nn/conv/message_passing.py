"""MessagePassing (PyG 1.4.3 API [U1]; usage text /root/reference/README.md:35-49,
subclass example /root/reference/gmm_conv.py:58,131-144).

``propagate(edge_index, size=None, **kwargs)``:
  * kwargs named ``foo_i`` / ``foo_j`` in message/aggregate/update signatures
    are gathered from ``foo`` at the target / source node of every edge
    (flow='source_to_target': j = edge_index[0], i = edge_index[1]);
    a tuple ``foo=(foo_src, foo_dst)`` selects bipartite mode;
  * special args: edge_index, edge_index_i, edge_index_j, size, size_i,
    size_j, index (= edge_index_i), dim_size (= size_i);
  * message(...) -> aggregate(inputs, index, dim_size) -> update(inputs, ...).

MI355X engine:
  * Fused path -- when the layer's message is ``x_j`` or ``w.view(-1,1)*x_j``
    (default message, GCNConv, SAGEConv, GraphConv) and ``aggregate`` is not
    overridden, gather + message + reduce (+ bias) run as ONE HIP kernel over
    a cached destination-sorted CSR (mi355_mp.ops.fused_propagate); x_j is
    never materialised.
  * Generic path -- any other message: the gathers of __collect__ and the
    reduction of aggregate still run on native kernels (row gather and
    segmented reduce), the user's message runs as ordinary torch code.
"""
import math as _math
import inspect
from collections import OrderedDict

import torch

from mi355_mp import ops as _ops
from mi355_mp.graph import graph_for

from ...utils.scatter import scatter_

special_args = ["edge_index", "edge_index_i", "edge_index_j", "size", "size_i", "size_j", "index",
                "dim_size"]
__size_error_msg__ = ("All tensors which should get mapped to the same source or target nodes must "
                      "be of same size in dimension 0.")


def _params(fn, drop_first):
    p = OrderedDict(inspect.signature(fn).parameters)
    if drop_first and p:
        p.popitem(last=False)
    return p


class MessagePassing(torch.nn.Module):
    r"""Base class for message passing layers

    .. math::
        \mathbf{x}_i^{\prime} = \gamma_{\mathbf{\Theta}} \left( \mathbf{x}_i,
        \square_{j \in \mathcal{N}(i)} \, \phi_{\mathbf{\Theta}}
        \left(\mathbf{x}_i, \mathbf{x}_j,\mathbf{e}_{i,j}\right) \right),

    Args:
        aggr (string): "add", "mean" or "max". (default: "add")
        flow (string): "source_to_target" or "target_to_source".
        node_dim (int): the axis along which to propagate. (default: 0)
    """

    def __init__(self, aggr="add", flow="source_to_target", node_dim=0):
        super(MessagePassing, self).__init__()
        self.aggr = aggr
        assert self.aggr in ["add", "mean", "max"]
        self.flow = flow
        assert self.flow in ["source_to_target", "target_to_source"]
        self.node_dim = node_dim
        assert self.node_dim >= 0

        self.__msg_params__ = _params(self.message, False)
        self.__aggr_params__ = _params(self.aggregate, True)
        self.__update_params__ = _params(self.update, True)
        msg_args = set(self.__msg_params__.keys()) - set(special_args)
        aggr_args = set(self.__aggr_params__.keys()) - set(special_args)
        update_args = set(self.__update_params__.keys()) - set(special_args)
        self.__args__ = set().union(msg_args, aggr_args, update_args)

    # -- argument plumbing -------------------------------------------------

    def __set_size__(self, size, index, tensor):
        if not torch.is_tensor(tensor):
            return
        if size[index] is None:
            size[index] = tensor.size(self.node_dim)
        elif size[index] != tensor.size(self.node_dim):
            raise ValueError(__size_error_msg__)

    def _ij(self):
        return (0, 1) if self.flow == "target_to_source" else (1, 0)

    def _gather(self, data, idx_vec):
        if (self.node_dim == 0 and data.dim() >= 1 and data.dtype == torch.float32 and data.is_cuda
                and data.dim() <= 2):
            flat = data if data.dim() == 2 else data.view(-1, 1)
            out = _ops.index_select_rows(flat, idx_vec)
            return out if data.dim() == 2 else out.view(-1)
        if self.node_dim == 0 and data.dtype == torch.float32 and data.is_cuda:
            flat = data.reshape(data.shape[0], _math.prod(data.shape[1:]))
            return _ops.index_select_rows(flat, idx_vec).view((-1,) + tuple(data.shape[1:]))
        return data.index_select(self.node_dim, idx_vec)

    def __collect__(self, edge_index, size, kwargs):
        i, j = self._ij()
        ij = {"_i": i, "_j": j}
        out = {}
        for arg in self.__args__:
            if arg[-2:] not in ij.keys():
                out[arg] = kwargs.get(arg, inspect.Parameter.empty)
            else:
                idx = ij[arg[-2:]]
                data = kwargs.get(arg[:-2], inspect.Parameter.empty)
                if data is inspect.Parameter.empty:
                    out[arg] = data
                    continue
                if isinstance(data, tuple) or isinstance(data, list):
                    assert len(data) == 2
                    self.__set_size__(size, 1 - idx, data[1 - idx])
                    data = data[idx]
                if not torch.is_tensor(data):
                    out[arg] = data
                    continue
                self.__set_size__(size, idx, data)
                out[arg] = self._gather(data, edge_index[idx])

        size[0] = size[1] if size[0] is None else size[0]
        size[1] = size[0] if size[1] is None else size[1]

        out["edge_index"] = edge_index
        out["edge_index_i"] = edge_index[i]
        out["edge_index_j"] = edge_index[j]
        out["size"] = size
        out["size_i"] = size[i]
        out["size_j"] = size[j]
        out["index"] = out["edge_index_i"]
        out["dim_size"] = out["size_i"]
        return out

    def __distribute__(self, params, kwargs):
        out = {}
        for key, param in params.items():
            data = kwargs[key]
            if data is inspect.Parameter.empty:
                if param.default is inspect.Parameter.empty:
                    raise TypeError("Required parameter {} is empty.".format(key))
                data = param.default
            out[key] = data
        return out

    # -- fused fast path ---------------------------------------------------

    def _fused_message(self, kwargs):
        """(name of the gathered node tensor, per-edge weight or None) if this
        layer's message is ``weight.view(-1,1) * <name>_j``; None otherwise."""
        if type(self).message is MessagePassing.message:
            return "x", None
        return None

    def _fused_bias(self):
        """(bias to add inside the kernel, skip update()) -- subclasses override."""
        return None, False

    def _try_fused(self, edge_index, size, kwargs):
        if self.node_dim != 0 or type(self).aggregate is not MessagePassing.aggregate:
            return None
        spec = self._fused_message(kwargs)
        if spec is None:
            return None
        name, weight = spec
        data = kwargs.get(name, None)
        i, j = self._ij()
        if isinstance(data, (tuple, list)):
            if len(data) != 2:
                return None
            src, dst = data[j], data[i]
        else:
            src, dst = data, None
        if not (torch.is_tensor(src) and src.dim() == 2 and src.dtype == torch.float32 and src.is_cuda):
            return None
        if weight is not None and not (torch.is_tensor(weight) and weight.dim() == 1 and weight.is_cuda):
            return None
        if any(k[-2:] in ("_i", "_j") for k in self.__update_params__):
            return None
        size = list(size)
        self.__set_size__(size, j, src)
        if dst is not None:
            self.__set_size__(size, i, dst)
        size[0] = size[1] if size[0] is None else size[0]
        size[1] = size[0] if size[1] is None else size[1]
        graph = graph_for(edge_index, size[i], size[j], self.flow)
        bias, skip_update = self._fused_bias()
        out = _ops.fused_propagate(graph, src, edge_index, edge_weight=weight, reduce=self.aggr,
                                   bias=bias, pyg_mask=self.aggr == "max")
        if skip_update:
            return out
        kw = dict(kwargs)
        kw.update({"edge_index": edge_index, "edge_index_i": edge_index[i], "edge_index_j": edge_index[j],
                   "size": size, "size_i": size[i], "size_j": size[j], "index": edge_index[i],
                   "dim_size": size[i]})
        for key in self.__update_params__:
            kw.setdefault(key, inspect.Parameter.empty)
        update_kwargs = self.__distribute__(self.__update_params__, kw)
        return self.update(out, **update_kwargs)

    # -- public API ----------------------------------------------------------

    def propagate(self, edge_index, size=None, **kwargs):
        r"""The initial call to start propagating messages.

        Args:
            edge_index (Tensor): [2, E] indices.
            size (list or tuple, optional): (N, M) for bipartite graphs.
            **kwargs: all data needed to construct messages and updates.
        """
        size = [None, None] if size is None else list(size)
        assert len(size) == 2

        fused = self._try_fused(edge_index, size, kwargs)
        if fused is not None:
            return fused

        kwargs = self.__collect__(edge_index, size, kwargs)
        msg_kwargs = self.__distribute__(self.__msg_params__, kwargs)
        out = self.message(**msg_kwargs)
        aggr_kwargs = self.__distribute__(self.__aggr_params__, kwargs)
        out = self.aggregate(out, **aggr_kwargs)
        update_kwargs = self.__distribute__(self.__update_params__, kwargs)
        out = self.update(out, **update_kwargs)
        return out

    def message(self, x_j):  # pragma: no cover
        r"""Constructs messages from node j to node i (default: x_j)."""
        return x_j

    def aggregate(self, inputs, index, dim_size):  # pragma: no cover
        r"""Aggregates messages from neighbors (scatter_ of self.aggr)."""
        return scatter_(self.aggr, inputs, index, self.node_dim, dim_size)

    def update(self, inputs):  # pragma: no cover
        r"""Updates node embeddings (default: identity)."""
        return inputs
