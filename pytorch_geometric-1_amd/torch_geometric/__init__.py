"""Drop-in ``torch_geometric`` (PyG 1.4.3 API surface of the message-passing hot path).

Pinned at /root/reference/requirement.txt:7 (torch-geometric==1.4.3); the
reference tree only calls it (examples/gcn.py:5-7, ConvexPruning.py:12-19).
Only the aggregation path is provided here: ``nn.MessagePassing``,
``nn.GCNConv``, ``nn.GATConv``, ``nn.SAGEConv``, ``nn.GraphConv``, global
pooling, ``nn.DataParallel`` with the ``data`` containers it batches, and the
``utils`` they use.  Every aggregation runs on the MI355X engine
(``mi355_mp``); there is no CPU fallback.
"""
from . import debug as _debug_mod
from .debug import is_debug_enabled, debug, set_debug  # noqa: F401
from . import utils  # noqa: F401
from . import data  # noqa: F401
from . import nn  # noqa: F401

__version__ = "1.4.3"

__all__ = ["is_debug_enabled", "debug", "set_debug", "__version__"]
