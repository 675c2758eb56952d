"""What a finished row costs k_agg_flat (config 2 sum kernel), apart from its
gathers: the same 62M slots in the same CSR order, grouped into rows k at a
time (k = 2, 4, 8: consecutive rows merged) or each row cut in two halves
(k = 0.5), so only the number of row ends changes.  The main kernel is timed
with HIP events (chunk fixed at 1024, the config-2 value); T(k) = A + B / k
gives the cost of one row end B / N.  One JSON line per k.
    python tools/exp_row_cost.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    from mi355_mp import _lib, ops
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N, F = 1 << 21, 256
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    ei = ei[:, ei[0] != ei[1]]
    loops = torch.arange(N, device=dev)
    ei = torch.cat([ei, torch.stack([loops, loops])], 1)
    g0 = Graph(ei, N, N, chunk=1024)
    csr0 = g0.dst
    E = csr0.n_edges
    # CSR slot order as an edge list (row of each slot, its column)
    rowptr = csr0.rowptr.long()
    deg = rowptr[1:] - rowptr[:-1]
    row_of_slot = torch.repeat_interleave(torch.arange(N, device=dev), deg)
    col = csr0.col[:E].long()
    x = torch.randn(N, F, device=dev)
    w_slot = torch.rand(E, device=dev)
    del ei
    res = []
    for k in (0.5, 1, 2, 4, 8):
        if k == 0.5:
            pos = torch.arange(E, device=dev) - rowptr[row_of_slot]
            dst = 2 * row_of_slot + (2 * pos >= deg[row_of_slot]).long()
            n_rows = 2 * N
        else:
            dst = row_of_slot // k
            n_rows = (N + k - 1) // k
        g = Graph(torch.stack([col, dst]), n_rows, N, chunk=1024)
        csr = g.dst                       # stable sort by dst: the slots keep their order
        w = csr.to_csr_order(w_slot)
        out = torch.empty(n_rows, F, device=dev)
        for _ in range(3):
            ops._aggregate(csr, "other", x, w, "sum", 0, None, out=out, stages=_lib.MP_STAGE_MAIN)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(10):
            ops._aggregate(csr, "other", x, w, "sum", 0, None, out=out, stages=_lib.MP_STAGE_MAIN)
        ev[1].record()
        ev[1].synchronize()
        ms = ev[0].elapsed_time(ev[1]) / 10
        same_order = bool(torch.equal(csr.col[:E].long(), col))
        line = {"k": k, "rows": n_rows, "slots": E, "main_ms": ms, "slot_order_unchanged": same_order}
        res.append(line)
        print(json.dumps(line), flush=True)
        del g, csr, w, out, dst
        torch.cuda.empty_cache()
    # least squares T = A + B * rows over the points
    xs = torch.tensor([r["rows"] for r in res], dtype=torch.float64)
    ys = torch.tensor([r["main_ms"] for r in res], dtype=torch.float64)
    M = torch.stack([torch.ones_like(xs), xs], 1)
    sol = torch.linalg.lstsq(M, ys.unsqueeze(1)).solution.view(-1)
    print(json.dumps({"fit": "main_ms = A + B * rows", "A_ms": float(sol[0]), "B_ns_per_row": float(sol[1]) * 1e6,
                      "row_ends_share_at_k1": float(sol[1]) * N / float(ys[1])}), flush=True)


if __name__ == "__main__":
    main()
