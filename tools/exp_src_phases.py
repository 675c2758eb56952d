"""Source-range phases on the config-2 workload: does splitting the gathered
rows into Infinity-Cache-sized source ranges pay for the partial-output
re-read it costs?

Variants (same x, weights, output layout; interleaved rounds; main + fix-up):
  base         one launch, 4 feature tiles on XCD pairs (the bench step)
  tiles        one launch per 64-feature tile (each tile over all 8 XCDs)
  phases S     per tile, S launches over the edges whose source lies in range
               s of S equal id ranges; launch s > 0 accumulates into the
               output (MP_FLAG_INIT_FROM_OUT), the last adds the bias.
               A row's sum becomes (range-0 part) + (range-1 part) + ...:
               within the 1e-5 bound, not bitwise the edge-order sum.
  phases_full S  S launches over the full 256-feature rows (tiles concurrent)
Prints the median ms per step and max |out - base| / max(1, sum|w x|)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    import mi355_mp
    from mi355_mp import _lib, ops
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, F, T = 1 << 21, 256, 64
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    ei2, norm = GCNConv.norm(ei, N)
    x = torch.randn(N, F, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    bias = torch.randn(F, device=dev) * 0.1
    g = Graph(ei2, N, N)
    w = g.dst.to_csr_order(norm)

    def seg_graphs(S):
        res = []
        bounds = [(N * s) // S for s in range(S + 1)]
        for s in range(S):
            m = (ei2[0] >= bounds[s]) & (ei2[0] < bounds[s + 1])
            gs = Graph(ei2[:, m], N, N)
            res.append((gs.dst, gs.dst.to_csr_order(norm[m].contiguous())))
        return res

    segs = {S: seg_graphs(S) for S in (2, 3, 4)}
    outs = {}

    def run(name, out):
        if name == "base":
            ops._aggregate(g.dst, "other", x, w, "sum", 0, bias, out=out)
        elif name == "tiles":
            for t in range(0, F, T):
                ops._aggregate(g.dst, "other", x[:, t:t + T], w, "sum", 0, bias[t:t + T], out=out[:, t:t + T])
        elif name.startswith("phases_full"):
            S = int(name.split("_")[-1])
            for s, (c, ws) in enumerate(segs[S]):
                ops._aggregate(c, "other", x, ws, "sum", _lib.MP_FLAG_INIT_FROM_OUT if s else 0,
                               bias if s == S - 1 else None, out=out)
        else:
            S = int(name.split("_")[-1])
            for t in range(0, F, T):
                for s, (c, ws) in enumerate(segs[S]):
                    ops._aggregate(c, "other", x[:, t:t + T], ws, "sum", _lib.MP_FLAG_INIT_FROM_OUT if s else 0,
                                   bias[t:t + T] if s == S - 1 else None, out=out[:, t:t + T])

    names = ["base", "tiles", "phases_2", "phases_3", "phases_4", "phases_full_2", "phases_full_4"]
    for n in names:
        outs[n] = torch.empty(N, F, device=dev)
        run(n, outs[n])
    torch.cuda.synchronize()
    # tolerance reference: sum |w x_j| per row (float64 not needed for the scale)
    absum = torch.zeros(N, F, device=dev)
    for s in range(0, ei2.shape[1], 8_000_000):
        e = slice(s, s + 8_000_000)
        absum.index_add_(0, ei2[1, e], (norm[e].view(-1, 1) * x[ei2[0, e]]).abs())
    base = outs["base"]
    times = {n: [] for n in names}
    for _ in range(5):
        for n in names:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                run(n, outs[n])
            b.record()
            torch.cuda.synchronize()
            times[n].append(a.elapsed_time(b) / 5)
    for n in names:
        t = sorted(times[n])
        d = ((outs[n] - base).abs() / absum.clamp(min=1)).max().item()
        eq = torch.equal(outs[n], base)
        print("%-14s %.3f ms/step (min %.3f)  max|d|/max(1,sum|wx|) %.2e  bitwise=%s" % (
            n, t[len(t) // 2], t[0], d, eq), flush=True)


if __name__ == "__main__":
    main()
