"""bench.py's single-GPU step (GCN-normalised weighted sum + bias, F=256,
main + fix-up timed with HIP events per launch) on other synthetic graphs, for
dispatch A/B runs in separate processes (tools/ab_bench_u.sh):
    python tools/bench_graph.py --graph rmat20_deg58
Prints one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402

GRAPHS = {
    # name: (generator, args)
    "rmat21": ("rmat", dict(scale=21, n_samples=30_000_000)),
    "rmat21_deg15": ("rmat", dict(scale=21, n_samples=15_000_000)),
    "rmat21_flat": ("rmat", dict(scale=21, n_samples=30_000_000, abcd=(0.45, 0.22, 0.22, 0.11))),
    "rmat20_deg58": ("rmat", dict(scale=20, n_samples=30_000_000)),
    "rmat21_deg45": ("rmat", dict(scale=21, n_samples=45_000_000)),
    "products": ("powerlaw", dict(num_nodes=2_449_029, num_edges=123_718_280)),
    "products_deg25": ("powerlaw", dict(num_nodes=2_449_029, num_edges=61_859_140)),
    "rmat22": ("rmat", dict(scale=22, n_samples=30_000_000)),
    "rmat22_deg30": ("rmat", dict(scale=22, n_samples=60_000_000)),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="rmat21", choices=sorted(GRAPHS))
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import mi355_mp
    from mi355_mp import _lib, ops
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index, powerlaw_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    kind, kw = GRAPHS[args.graph]
    if kind == "rmat":
        ei = rmat_edge_index(seed=1, device=dev, **kw)
        N = 1 << kw["scale"]
    else:
        ei = powerlaw_edge_index(seed=4, device=dev, **kw)
        N = kw["num_nodes"]
    F = 256
    ei2, norm = GCNConv.norm(ei, N)
    csr = Graph(ei2, N, N).dst
    w = csr.to_csr_order(norm)
    # share of slots gathering one of the 16K most-gathered rows (the 256-B tiles an XCD's L2 holds)
    cnt = torch.bincount(csr.col[:csr.n_edges], minlength=N)
    share = float(cnt.topk(min(16384, N), sorted=False).values.sum()) / csr.n_edges
    x = torch.randn(N, F, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    bias = torch.randn(F, device=dev, generator=torch.Generator(device=dev).manual_seed(7)) * 0.1
    out = torch.empty(N, F, device=dev)
    slab = torch.empty(_lib.load().mp_aggregate_slab_bytes(csr.struct("other"), F, 0), dtype=torch.uint8,
                       device=dev)

    def agg(stages):
        ops._aggregate(csr, "other", x, w, "sum", 0, bias, out=out, stages=stages, slab=slab)
    for _ in range(5):
        agg(_lib.MP_STAGE_ALL)
    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    for a, b, c in ev:
        a.record()
        agg(_lib.MP_STAGE_MAIN)
        b.record()
        agg(_lib.MP_STAGE_FIXUP)
        c.record()
    torch.cuda.synchronize()
    main_ms = sorted(a.elapsed_time(b) for a, b, _ in ev)
    fix_ms = sorted(b.elapsed_time(c) for _, b, c in ev)
    kernel = _lib.kernel_name(csr.struct("other"), w.data_ptr(), x.data_ptr(), x.stride(0), F, "sum",
                              bias.data_ptr(), out.data_ptr(), out.stride(0), dev)
    print(json.dumps({"graph": args.graph, "num_nodes": N, "num_edges": csr.n_edges,
                      "avg_degree": csr.n_edges / N, "main_ms": main_ms[len(main_ms) // 2],
                      "fixup_ms": fix_ms[len(fix_ms) // 2], "hot_share": share, "kernel": kernel}))


if __name__ == "__main__":
    main()
