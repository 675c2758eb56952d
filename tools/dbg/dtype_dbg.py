import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    sys.path.insert(0, p)
import torch
import torch_scatter
from oracle import scatter_ref as S
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_parity import _dtype_case
src, idx, N = _dtype_case(torch.int64, 31)
base = (torch.arange(N * src.shape[1]).view(N, -1) % 5).to(torch.int64)
o = base.clone().cuda()
torch_scatter.scatter_mean(src.cuda(), idx.cuda(), 0, out=o)
ref, _ = S.scatter_loop_any(src, idx, N, "mean", out=base)
bad = (o.cpu() != ref).nonzero()
print(bad.shape, bad[:5].tolist())
for r, f in bad[:5].tolist():
    sel = idx == r
    print(r, f, "got", o[r, f].item(), "ref", ref[r, f].item(), "base", base[r, f].item(), "sum", src[sel, f].sum().item(), "cnt", int(sel.sum()))
