"""Global pooling (PyG 1.4.3 nn.glob [U]; callers /root/reference/ConvexPruningBatchSize.py:230,
/root/reference/examples/MyGCN.py:143-151):

    global_add_pool(x, batch, size=None)  = scatter_('add',  x, batch, dim_size=size)
    global_mean_pool(x, batch, size=None) = scatter_('mean', x, batch, dim_size=size)
    global_max_pool(x, batch, size=None)  = scatter_('max',  x, batch, dim_size=size)

The `batch` vector maps nodes to graphs; the same destination-sorted segment
kernels reduce it (a sorted batch vector makes the CSR build trivial).
"""
from ...utils.scatter import scatter_


def _size(batch, size):
    return int(batch.max().item()) + 1 if size is None else size


def global_add_pool(x, batch, size=None):
    return scatter_("add", x, batch, dim=0, dim_size=_size(batch, size))


def global_mean_pool(x, batch, size=None):
    return scatter_("mean", x, batch, dim=0, dim_size=_size(batch, size))


def global_max_pool(x, batch, size=None):
    return scatter_("max", x, batch, dim=0, dim_size=_size(batch, size))


__all__ = ["global_add_pool", "global_mean_pool", "global_max_pool"]
