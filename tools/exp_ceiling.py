"""Calibrates the main kernel's ceilings on the config-2 CSR by rewriting the
gather columns: all rows in a 4 MB set (L2-resident), a 128 MB set (Infinity
Cache), uniformly random over N (no reuse), and the real graph."""
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
    lib = mi355_mp.load_native()
    if os.environ.get("EXP_LIB"):   # a build variant (tools/variants/lib_*.so)
        lib = _lib.load(os.environ["EXP_LIB"])
    dev = torch.device("cuda", 0)
    N = 1 << 21
    F = int(os.environ.get("EXP_F", "256"))
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    ei2, norm = GCNConv.norm(ei, N)
    x = torch.randn(N, F, device=dev)
    bias = torch.zeros(F, device=dev)
    csr = Graph(ei2, N, N).dst
    w = csr.to_csr_order(norm)
    E = csr.n_edges
    # proxy for an LDS cache of the K hottest source rows: their slots are
    # rewritten to the single hottest row (served by L1 instead of the miss queue)
    outdeg = torch.bincount(csr.col.long(), minlength=N)
    order = torch.argsort(outdeg, descending=True)
    hot = {}
    for K in (640, 1280, 4096):
        is_hot = torch.zeros(N, dtype=torch.bool, device=dev)
        is_hot[order[:K]] = True
        hot["hot%d_to_one" % K] = torch.where(is_hot[csr.col.long()], order[0].to(torch.int32), csr.col)
    # cold rows flagged in the column's sign bit (variant libraries built with
    # -DMP_COLD_FLAG=1 load them with the MP_COLD_AUX cache-policy bits)
    cold = {}
    for t in [int(v) for v in os.environ.get("EXP_COLD", "").split(",") if v]:
        is_cold = (outdeg <= t)[csr.col.long()]
        cold["cold_deg%d" % t] = torch.where(is_cold, csr.col.long() - (1 << 31), csr.col.long()).to(torch.int32)
        print("cold_deg%d: %.1f%% of slots" % (t, 100.0 * float(is_cold.float().mean())))
    cols = {
        "real": csr.col,
        **cold,
        **hot,
        "l2_4MB": (csr.col % 4096).to(torch.int32),
        "mall_128MB": (csr.col % 131072).to(torch.int32),
        "mall_32MB": (csr.col % 32768).to(torch.int32),
        "uniform_2GB": torch.randint(N, (E,), device=dev, dtype=torch.int32),
        "sequential": (torch.arange(E, device=dev) % N).to(torch.int32),
    }
    out = torch.empty(N, F, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    g0 = csr.struct("other")
    sb = lib.mp_aggregate_slab_bytes(g0, F, 0)
    slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    structs = {}
    for k, c in cols.items():
        structs[k] = _lib.MpCsr(csr.rowptr.data_ptr(), c.data_ptr(), csr.eid.data_ptr(), csr.wave_row.data_ptr(),
                                csr.wave_slot.data_ptr(), csr.split_waves.data_ptr(), N, E, csr.chunk,
                                csr.n_waves, csr.n_split, N)  # n_cols = N: the VEC=1 shape of the real launch

    def launch(s):
        _lib.check(lib.mp_aggregate_f32(s, w.data_ptr(), x.data_ptr(), F, F, 0, 0, bias.data_ptr(),
                                        out.data_ptr(), F, None, slab.data_ptr(), sb, 1, st), "agg")
    times = {k: [] for k in cols}
    for _ in range(5):
        for k in cols:
            launch(structs[k])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                launch(structs[k])
            b.record()
            torch.cuda.synchronize()
            times[k].append(a.elapsed_time(b) / 10)
    alg = E * (4 * F + 8) + N * (4 * F + 4)
    only = os.environ.get("EXP_ONLY")
    for k in cols:
        if only and k not in only.split(","):
            continue
        t = sorted(times[k])[2]
        print("%-12s %.3f ms  %.0f GB/s algorithmic" % (k, t, alg / t / 1e6))


if __name__ == "__main__":
    main()
