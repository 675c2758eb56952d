"""Upper bound of locality-aware relabelling on the config-2 workload: the
main kernel on the bench's label-permuted RMAT graph vs the same RMAT sample
with its natural (recursive-quadrant) labels, plus a BFS relabelling of the
permuted graph.  Same edge multiset, same kernel; interleaved rounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def bfs_order(ei, N):
    """Node order by BFS levels from the max-degree node (unreached last),
    ties inside a level by parent order (torch ops on the GPU)."""
    dev = ei.device
    from mi355_mp.graph import CSR
    csr = CSR(ei[0], ei[1], N, N)   # out-neighbours
    rp = csr.rowptr.long()
    col = csr.col[:csr.n_edges].long()
    deg = rp[1:] - rp[:-1]
    order = torch.full((N,), -1, dtype=torch.long, device=dev)
    seen = torch.zeros(N, dtype=torch.bool, device=dev)
    frontier = torch.argmax(deg).view(1)
    seen[frontier] = True
    pos = 0
    while frontier.numel():
        order[pos:pos + frontier.numel()] = frontier
        pos += frontier.numel()
        d = deg[frontier]
        starts = rp[frontier]
        idx = torch.repeat_interleave(starts - torch.cumsum(d, 0) + d, d) + torch.arange(int(d.sum()), device=dev)
        nb = col[idx]
        nb = nb[~seen[nb]]
        # first occurrence keeps parent order
        uniq, inv = torch.unique(nb, return_inverse=True)
        first = torch.full((uniq.numel(),), nb.numel(), dtype=torch.long, device=dev)
        first.scatter_reduce_(0, inv, torch.arange(nb.numel(), device=dev), "amin")
        nxt = uniq[torch.argsort(first)]
        seen[nxt] = True
        frontier = nxt
    rest = torch.nonzero(~seen).view(-1)
    order[pos:] = rest
    return order   # new -> old


def main():
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, F = 1 << 21, 256
    x = torch.randn(N, F, device=dev)
    setups = {}
    for name, permute in (("permuted", True), ("natural", False)):
        ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev, permute=permute)
        ei2, norm = GCNConv.norm(ei, N)
        setups[name] = (ei2, norm)
    ei2, norm = setups["permuted"]
    order = bfs_order(ei2, N)
    new_id = torch.empty_like(order)
    new_id[order] = torch.arange(N, device=dev)
    setups["permuted+bfs"] = (new_id[ei2], norm)
    runs = {}
    for name, (e, w) in setups.items():
        g = Graph(e, N, N)
        csr = g.dst
        runs[name] = (csr, csr.to_csr_order(w), torch.empty(N, F, device=dev))
    times = {n: [] for n in runs}
    for _ in range(4):
        for n, (csr, w, out) in runs.items():
            from mi355_mp import ops
            ops._aggregate(csr, "other", x, w, "sum", 0, None, out=out, stages=_lib.MP_STAGE_MAIN)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                ops._aggregate(csr, "other", x, w, "sum", 0, None, out=out, stages=_lib.MP_STAGE_MAIN)
            b.record()
            torch.cuda.synchronize()
            times[n].append(a.elapsed_time(b) / 10)
    for n in runs:
        t = sorted(times[n])
        print("%-14s main kernel median %.3f ms  (E=%d, n_split=%d)" % (n, t[len(t) // 2], runs[n][0].n_edges,
                                                                          runs[n][0].n_split), flush=True)


if __name__ == "__main__":
    main()
