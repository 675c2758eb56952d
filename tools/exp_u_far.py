"""Row loads in flight (U) of the scalar-batch sum kernel over an x beyond the
Infinity Cache, on several graphs, against a per-graph statistic the CSR
build could compute: the share of slots whose source is among the 16K hottest
(by out-degree) -- what one XCD's L2 can hold at 256-B tiles.
Variants: tools/variants/lib_far<U>.so (make variant NAME=far6
DEFS=-DMP_U_VEC1_FAR=6; EXP_U lists them) and the default build, interleaved
in one process, outputs checked bitwise."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index, powerlaw_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    F = 256
    us = [int(u) for u in os.environ.get("EXP_U", "4,5,6,7,8,10").split(",")]
    libs = {"default": _lib.load()}
    for u in us:
        libs["u%d" % u] = _lib.load(os.path.join(ROOT, "tools", "variants", "lib_far%d.so" % u))
    graphs = {
        "rmat21": lambda: (rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev), 1 << 21),
        "products": lambda: (powerlaw_edge_index(2_449_029, 123_718_280, seed=4, device=dev), 2_449_029),
        "rmat21_flat": lambda: (rmat_edge_index(scale=21, n_samples=30_000_000, abcd=(0.45, 0.22, 0.22, 0.11),
                                                seed=1, device=dev), 1 << 21),
        "rmat20_deg57": lambda: (rmat_edge_index(scale=20, n_samples=30_000_000, seed=1, device=dev), 1 << 20),
        "rmat21_deg15": lambda: (rmat_edge_index(scale=21, n_samples=15_000_000, seed=1, device=dev), 1 << 21),
    }
    st = torch.cuda.current_stream().cuda_stream
    for name, make in graphs.items():
        ei, N = make()
        ei2, norm = GCNConv.norm(ei, N)
        del ei
        csr = Graph(ei2, N, N).dst
        w = csr.to_csr_order(norm)
        del ei2, norm
        col = csr.col[:csr.n_edges].long()
        outdeg = torch.bincount(col, minlength=N)
        top = torch.topk(outdeg, min(16384, N)).values.sum().item()
        hot = top / csr.n_edges
        x = torch.randn(N, F, device=dev)
        g = csr.struct("other")
        sb = libs["default"].mp_aggregate_slab_bytes(g, F, 0)
        slab = torch.empty(sb, dtype=torch.uint8, device=dev)
        outs = {n: torch.empty(N, F, device=dev) for n in libs}

        def launch(lib, out, stages):
            _lib.check(lib.mp_aggregate_f32(g, w.data_ptr(), x.data_ptr(), x.stride(0), F, 0, 0, None,
                                            out.data_ptr(), out.stride(0), None, slab.data_ptr(), sb, stages, st),
                       "agg")
        for n, lib in libs.items():
            launch(lib, outs[n], _lib.MP_STAGE_ALL)
        torch.cuda.synchronize()
        same = all(torch.equal(outs[n], outs["default"]) for n in libs)
        times = {n: [] for n in libs}
        for _ in range(5):
            for n, lib in libs.items():
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(5):
                    launch(lib, outs[n], _lib.MP_STAGE_MAIN)
                b.record()
                torch.cuda.synchronize()
                times[n].append(a.elapsed_time(b) / 5)
        med = {n: sorted(t)[2] for n, t in times.items()}
        print("%-13s N=%8d E=%9d deg=%5.1f hot16K=%.3f x=%.2f GB  %s  bitwise=%s" % (
            name, N, csr.n_edges, csr.n_edges / N, hot, N * F * 4 / 1e9,
            "  ".join("%s %.3f" % (n, med[n]) for n in libs), same), flush=True)
        del csr, w, x, outs, slab, col, outdeg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
