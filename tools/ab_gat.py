"""In-process A/B of GAT aggregation variants (tools/variants/lib_*.so) on config 3."""
import glob
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
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv._structure import gat_loops
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, H, C = 1 << 21, 8, 32
    ei = gat_loops(rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev), N)
    csr = Graph(ei, N, N).dst
    xw = torch.randn(N, H * C, device=dev)
    a_src = torch.randn(N, H, device=dev)
    a_dst = torch.randn(N, H, device=dev)
    vdir = os.path.join(ROOT, "tools", "variants")
    names = sorted(os.path.basename(f)[4:-3] for f in glob.glob(os.path.join(vdir, "lib_*.so")))
    libs = {n: _lib.load(os.path.join(vdir, "lib_%s.so" % n)) for n in names}
    g = csr.struct("other")
    sb = libs[names[0]].mp_gat_slab_bytes(g, H, C)
    slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    outs = {n: torch.empty(N, H * C, device=dev) for n in names}
    st = torch.cuda.current_stream().cuda_stream

    def launch(n, stages):
        _lib.check(libs[n].mp_gat_aggregate_f32(g, xw.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(), H, C, 0.2,
                                                None, outs[n].data_ptr(), H * C, None, slab.data_ptr(), sb,
                                                stages, st), "gat")
    for n in names:
        launch(n, 3)
    torch.cuda.synchronize()
    times = {n: [] for n in names}
    for _ in range(5):
        for n in names:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                launch(n, 1)
            b.record()
            torch.cuda.synchronize()
            times[n].append(a.elapsed_time(b) / 10)
    for n in names:
        t = sorted(times[n])
        print(n, "median %.3f ms" % t[2], "max|diff| vs %s %.3g" % (names[0], (outs[n] - outs[names[0]]).abs().max().item()))


if __name__ == "__main__":
    main()
