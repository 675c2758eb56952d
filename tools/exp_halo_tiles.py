"""Per-rank compute of the sharded bench step by halo-tile width, on one GPU
(no exchange: the halo rows are random): rank 0's interior + boundary passes
of OverlappedAggregation over whole 256-feature rows (step) and over
tile-major buffers of 128 / 64 features (step_tiled's launches), at P = 2 / 4
/ 8 on the config-2 graph.  HIP events around back-to-back repetitions."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    import mi355_mp
    from mi355_mp import _lib, ops, dist as mdist
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, F = 1 << 21, 256
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    ei2, norm = GCNConv.norm(ei, N)
    del ei
    bias = torch.randn(F, device=dev)
    for P in (2, 4, 8):
        plan = mdist.ShardPlan(ei2, N, 0, P)
        ov = mdist.OverlappedAggregation(plan, norm)
        out = torch.empty(plan.n_own, F, device=dev)
        res = {}
        for tile in (256, 128, 64):
            xs = [torch.randn(plan.n_local_src, min(tile, F - c0), device=dev) for c0 in range(0, F, tile)]
            offs = [0]
            for xt in xs:
                offs.append(offs[-1] + xt.shape[1])

            def run():
                for t, xt in enumerate(xs):
                    ops._aggregate(ov.g_int.dst, "other", xt[:plan.n_own], ov.w_int, "sum", 0, None,
                                   out=out[:, offs[t]:offs[t + 1]])
                for t, xt in enumerate(xs):
                    ops._aggregate(ov.g_bnd.dst, "other", xt, ov.w_bnd, "sum", _lib.MP_FLAG_INIT_FROM_OUT,
                                   bias[offs[t]:offs[t + 1]], out=out[:, offs[t]:offs[t + 1]])
            for _ in range(3):
                run()
            per = []
            for _ in range(3):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(10):
                    run()
                b.record()
                torch.cuda.synchronize()
                per.append(a.elapsed_time(b) / 10)
            res[tile] = min(per)
            del xs
        print("P=%d rank0 edges %d (interior %d) halo rows %d: compute per step  256: %.3f  128: %.3f  64: %.3f ms"
              % (P, ov.n_interior + ov.n_boundary, ov.n_interior, plan.n_local_src - plan.n_own,
                 res[256], res[128], res[64]), flush=True)
        del ov, plan, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
