"""Merge-path task size on the per-rank graphs of the sharded config-2 bench:
rank 0's local graph of a P-way destination-range partition (P = 2, 4, 8) and
its interior / boundary halves (OverlappedAggregation), aggregated alone on one
GPU (no exchange) at several chunks.  auto_chunk's 50K-task target was tuned
on the whole 62M-edge graph; a rank's graph is P times smaller.
Prints ms per aggregation (main + fix-up, median of interleaved rounds)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    import mi355_mp
    from mi355_mp import dist as mdist, ops
    from mi355_mp.graph import Graph, auto_chunk
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, F = 1 << 21, 256
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    ei2, norm = GCNConv.norm(ei, N)
    chunks = [int(c) for c in os.environ.get("EXP_CHUNKS", "128,256,512,1024").split(",")]
    for P in (2, 4, 8):
        plan = mdist.ShardPlan(ei2, N, 0, P)
        lei = plan.local_edge_index
        w = norm[plan.edge_pos]
        interior = lei[0] < plan.n_own
        parts = {"local": (lei, w, plan.n_local_src),
                 "interior": (lei[:, interior], w[interior], plan.n_own),
                 "boundary": (lei[:, ~interior], w[~interior], plan.n_local_src)}
        x = torch.randn(plan.n_local_src, F, device=dev)
        for name, (e, ww, n_src) in parts.items():
            auto = auto_chunk(plan.n_own, e.shape[1])
            runs = {}
            for c in sorted(set(chunks + [auto])):
                g = Graph(e, plan.n_own, n_src, chunk=c)
                runs[c] = (g.dst, g.dst.to_csr_order(ww.contiguous()), torch.empty(plan.n_own, F, device=dev))
            times = {c: [] for c in runs}
            for _ in range(5):
                for c, (csr, wc, out) in runs.items():
                    ops._aggregate(csr, "other", x, wc, "sum", 0, None, out=out)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(10):
                        ops._aggregate(csr, "other", x, wc, "sum", 0, None, out=out)
                    b.record()
                    torch.cuda.synchronize()
                    times[c].append(a.elapsed_time(b) / 10)
            ref = runs[auto][2]
            line = []
            for c in runs:
                t = sorted(times[c])
                line.append("%d%s: %.3f" % (c, "*" if c == auto else "", t[len(t) // 2]))
                assert torch.allclose(runs[c][2], ref, rtol=1e-5, atol=1e-5)
            print("P=%d %-9s E=%9d rows=%8d  %s ms  (* = auto_chunk)" % (
                P, name, e.shape[1], plan.n_own, "  ".join(line)), flush=True)


if __name__ == "__main__":
    main()
