"""Config-2 gather stream for tools/sim_l2.c: the RMAT21 graph (same generator
and seed as bench.py, on the CPU), add_remaining_self_loops, stable sort by
destination -> /tmp/sim/col.bin (int32 CSR columns), plus the source-popularity
curve (share of all gathers that hit the top-k source rows)."""
import os
import sys, torch, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pytorch_geometric-1_amd"))
from mi355_mp.graphgen import rmat_edge_index
torch.set_num_threads(8)
ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device="cpu")
N = 1 << 21
src, dst = ei[0], ei[1]
keep = src != dst
src, dst = src[keep], dst[keep]
loop = torch.arange(N)
src = torch.cat([src, loop]); dst = torch.cat([dst, loop])
order = torch.sort(dst, stable=True).indices
col = src[order].to(torch.int32).numpy()
rowptr = np.zeros(N + 1, dtype=np.int64)
np.cumsum(np.bincount(dst.numpy(), minlength=N), out=rowptr[1:])
os.makedirs("/tmp/sim", exist_ok=True)
col.tofile("/tmp/sim/col.bin"); rowptr.astype(np.int32).tofile("/tmp/sim/rowptr.bin")
deg = np.bincount(col, minlength=N)
s = np.sort(deg)[::-1]; cs = np.cumsum(s) / s.sum()
for k in [640, 1280, 4096, 8192, 16384, 32768, 65536, 131072, 262144, 1048576]:
    print(k, round(float(cs[k-1]), 3))
print("E", col.size, "rows with deg<=32 share", float(deg[deg<=32].sum())/col.size)
