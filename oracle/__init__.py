"""CPU oracle for the message-passing hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / the timed CPU baseline.  The
product path (pytorch_geometric-1_amd/) never imports it.

What it restates (the reference's algorithm for this path lives in
unvendored third-party packages pinned at /root/reference/requirement.txt:
torch-scatter==2.0.4 (:3) and torch-geometric==1.4.3 (:7); neither is in
/root/reference nor installed here -- SURVEY.md 8c):
  * scatter_ref.py   torch_scatter 2.0.4 scatter_sum/mean/max/min (torch CPU
                     ops for sum/mean = the literal `scatter_add_` it calls;
                     max/min through scatter_loop.c, a serial restatement of
                     csrc/cpu/scatter_cpu.cpp's b/e/k loop)
  * pyg_ref.py       PyG 1.4.3 utils.scatter_, utils.softmax, self-loop
                     utilities, GCNConv.norm/forward, GATConv.forward,
                     GraphConv(aggr='max'), generic MessagePassing
  * scatter_loop.c   the serial C loop (also the CPU baseline of bench.py)

PARITY UNPINNED: the reference tree holds no tests, fixtures or golden
vectors for this path and its dependencies cannot be
imported or built here (ModuleNotFoundError; sources absent).  The oracle is
pinned only by hand-derived known-answer tests of the published semantics
(tests/test_oracle.py) and by agreement between its two independent forms
(torch ops vs the C loop); golden fixtures in tests/golden/ are generated
from it by tests/golden/make_golden.py.
"""
