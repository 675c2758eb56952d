from .message_passing import MessagePassing
from .gcn_conv import GCNConv
from .gat_conv import GATConv
from .sage_conv import SAGEConv
from .graph_conv import GraphConv
from .cheb_conv import ChebConv
from .agnn_conv import AGNNConv
from .sg_conv import SGConv
from .gin_conv import GINConv

__all__ = ["MessagePassing", "GCNConv", "GATConv", "SAGEConv", "GraphConv", "ChebConv", "AGNNConv", "SGConv", "GINConv"]
