"""Locality experiments on the config-2 graph (main kernel only, in-process
interleaved rounds): baseline vs all-nt x loads vs degree-relabelled node ids
(hub rows contiguous; permutation cost NOT included -- an upper bound)."""
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
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, F = 1 << 21, 256
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    ei2, norm = GCNConv.norm(ei, N)
    x = torch.randn(N, F, device=dev)
    bias = torch.zeros(F, device=dev)
    vdir = os.path.join(ROOT, "tools", "variants")
    libs = {n: _lib.load(os.path.join(vdir, "lib_%s.so" % n)) for n in ["base", "ntx"]}
    # degree relabelling: rank by out-degree (gather frequency), hubs first
    deg = torch.bincount(ei2[0], minlength=N)
    perm = torch.argsort(deg, descending=True)          # new -> old
    new_id = torch.empty_like(perm)
    new_id[perm] = torch.arange(N, device=dev)
    ei_r = new_id[ei2]
    x_r = x[perm].contiguous()
    setups = {}
    for name, e, xx in (("orig", ei2, x), ("relabel", ei_r, x_r)):
        csr = Graph(e, N, N).dst
        w = csr.to_csr_order(norm)
        setups[name] = (csr, w, xx)
    out = torch.empty(N, F, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    slab = torch.empty(1 << 30, dtype=torch.uint8, device=dev)

    def launch(lib, s):
        csr, w, xx = s
        g = csr.struct("other")
        sb = lib.mp_aggregate_slab_bytes(g, F, 0)
        _lib.check(lib.mp_aggregate_f32(g, w.data_ptr(), xx.data_ptr(), F, F, 0, 0, bias.data_ptr(),
                                        out.data_ptr(), F, None, slab.data_ptr(), sb, 1, st), "agg")
    combos = [(ln, sn) for ln in libs for sn in setups]
    times = {c: [] for c in combos}
    for _ in range(5):
        for c in combos:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            launch(libs[c[0]], setups[c[1]])
            a.record()
            for _ in range(10):
                launch(libs[c[0]], setups[c[1]])
            b.record()
            torch.cuda.synchronize()
            times[c].append(a.elapsed_time(b) / 10)
    for c in combos:
        t = sorted(times[c])
        print(c, "median %.3f ms  min %.3f" % (t[2], t[0]))
    # cost of the permutation itself (x[perm])
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        x[perm]
    b.record()
    torch.cuda.synchronize()
    print("x[perm] gather: %.3f ms" % (a.elapsed_time(b) / 10))


if __name__ == "__main__":
    main()
