from .conv import MessagePassing, GCNConv, GATConv, SAGEConv, GraphConv
from . import inits  # noqa: F401

__all__ = ["MessagePassing", "GCNConv", "GATConv", "SAGEConv", "GraphConv"]
