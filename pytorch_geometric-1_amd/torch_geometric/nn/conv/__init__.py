from .message_passing import MessagePassing
from .gcn_conv import GCNConv
from .gat_conv import GATConv
from .sage_conv import SAGEConv
from .graph_conv import GraphConv

__all__ = ["MessagePassing", "GCNConv", "GATConv", "SAGEConv", "GraphConv"]
