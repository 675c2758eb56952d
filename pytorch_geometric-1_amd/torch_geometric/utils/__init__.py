from .num_nodes import maybe_num_nodes
from .scatter import scatter_
from .softmax import softmax
from .loop import (contains_self_loops, remove_self_loops, add_self_loops,
                   add_remaining_self_loops)
from .degree import degree
from .get_laplacian import get_laplacian

__all__ = ["maybe_num_nodes", "scatter_", "softmax", "contains_self_loops", "remove_self_loops",
           "add_self_loops", "add_remaining_self_loops", "degree", "get_laplacian"]
