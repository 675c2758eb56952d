import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    sys.path.insert(0, p)
import torch
from oracle import pyg_ref as P, scatter_ref as S
from mi355_mp import _lib
from mi355_mp.graph import graph_for
N = 3000
g = torch.Generator().manual_seed(5)
E = 60_000
src = torch.cat([torch.zeros(20_000, dtype=torch.int64), torch.randint(N, (E - 20_000,), generator=g)])
ei = torch.stack([src, torch.randint(N, (E,), generator=g)])
w = torch.rand(E, generator=g) * 3
ei2, w2 = P.add_remaining_self_loops(ei, w, 1, N)
deg_ref = S.scatter_sum(w2, ei2[0], N)
eid, wd = ei2.cuda(), w2.cuda()
lib = _lib.load()
rows = graph_for(eid, N, N, "source_to_target").src
deg = torch.empty(N, device="cuda")
_lib.check(lib.mp_segment_sum_serial_f32(rows.rowptr.data_ptr(), rows.eid.data_ptr(), wd.data_ptr(), N, deg.data_ptr(), _lib.stream_ptr()), "x")
dc = deg.cpu()
bad = (dc != deg_ref).nonzero().view(-1)
print("deg mismatches", bad.numel(), bad[:10].tolist(), (dc - deg_ref).abs().max().item())
# order check
rp = rows.rowptr.cpu(); e_ = rows.eid.cpu()
r0 = e_[rp[0]:rp[1]]
print("row0 sorted", bool((r0[1:] > r0[:-1]).all()), r0.numel())
dinv = deg.clone()
norm = torch.empty(ei2.shape[1], device="cuda")
r, c = eid[0].contiguous(), eid[1].contiguous()
_lib.check(lib.mp_gcn_norm_from_deg_f32(r.data_ptr(), c.data_ptr(), wd.data_ptr(), ei2.shape[1], N, dinv.data_ptr(), norm.data_ptr(), _lib.stream_ptr()), "y")
dref = deg_ref.pow(-0.5)
print("dinv mismatches", (dinv.cpu() != dref).sum().item())
_, nref = P.gcn_norm(ei, N, w)
print("norm mismatches", (norm.cpu() != nref).sum().item())
# dinv from the correct deg
d2 = deg_ref.cuda().clone()
_lib.check(lib.mp_gcn_norm_from_deg_f32(r.data_ptr(), c.data_ptr(), wd.data_ptr(), ei2.shape[1], N, d2.data_ptr(), norm.data_ptr(), _lib.stream_ptr()), "y")
print("dinv(from ref deg) mismatches", (d2.cpu() != dref).sum().item(), "norm", (norm.cpu() != nref).sum().item())
