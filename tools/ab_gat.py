"""In-process A/B of GAT variants (tools/variants/lib_*.so) on config 3: the
fused forward aggregation (mp_gat_aggregate_f32) and the fused backward pass
over the transposed CSR (mp_gat_backward_f32), main stage only, interleaved."""
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
    graph = Graph(ei, N, N)
    csr = graph.dst
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
        print(n, "forward median %.3f ms" % t[2], "max|diff| vs %s %.3g" % (names[0], (outs[n] - outs[names[0]]).abs().max().item()))
    # backward pass (random but well-formed inputs)
    src = graph.src_with_dst_slots()
    gs = src.struct("dst_slot")
    E = src.n_edges
    gen = torch.Generator(device=dev).manual_seed(5)
    gout = torch.randn(N, H * C, device=dev, generator=gen)
    pack = torch.stack([torch.randn(N, H, device=dev, generator=gen), torch.rand(N, H, device=dev, generator=gen) + 2,
                        torch.rand(N, H, device=dev, generator=gen) * 0.1, torch.randn(N, H, device=dev, generator=gen)],
                       -1).contiguous()
    att = torch.randn(H, 2 * C, device=dev, generator=gen) * 0.1
    sbb = libs[names[0]].mp_gat_slab_bytes(gs, H, C)
    slabb = torch.empty(sbb, dtype=torch.uint8, device=dev)
    gx = {n: torch.empty(N, H * C, device=dev) for n in names}
    gas = torch.empty(N, H, device=dev)
    de = torch.empty(E, H, device=dev)

    def launch_b(n, stages):
        _lib.check(libs[n].mp_gat_backward_f32(gs, gout.data_ptr(), H * C, xw.data_ptr(), a_src.data_ptr(),
                                               pack.data_ptr(), att.data_ptr(), H, C, 0.2, gx[n].data_ptr(),
                                               gas.data_ptr(), de.data_ptr(), slabb.data_ptr(), sbb, stages, st),
                   "gat_bwd")
    for n in names:
        launch_b(n, 3)
    torch.cuda.synchronize()
    times = {n: [] for n in names}
    for _ in range(5):
        for n in names:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                launch_b(n, 1)
            b.record()
            torch.cuda.synchronize()
            times[n].append(a.elapsed_time(b) / 10)
    for n in names:
        t = sorted(times[n])
        print(n, "backward median %.3f ms" % t[2], "max|diff| vs %s %.3g" % (names[0], (gx[n] - gx[names[0]]).abs().max().item()))


if __name__ == "__main__":
    main()
