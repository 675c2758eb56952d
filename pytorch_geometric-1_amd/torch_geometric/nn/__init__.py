from .conv import MessagePassing, GCNConv, GATConv, SAGEConv, GraphConv, ChebConv, AGNNConv, SGConv, GINConv
from .glob import global_add_pool, global_mean_pool, global_max_pool
from .data_parallel import DataParallel
from . import inits  # noqa: F401

__all__ = ["MessagePassing", "GCNConv", "GATConv", "SAGEConv", "GraphConv", "ChebConv", "AGNNConv", "SGConv",
           "GINConv", "global_add_pool", "global_mean_pool", "global_max_pool", "DataParallel"]
