"""In-process A/B of the fused GAT forward's feature-tile width on config 3
(RMAT21, heads=8, C=32): one 256-feature tile per task (VEC=4, k_agg_main)
against 64- and 128-feature tiles holding whole heads (k_agg_flat with scalar
slot batches, MP_TUNE_GAT_TILE_VEC = 1 / 2).  Same per-head arithmetic, so
the outputs and row statistics must be bitwise equal.  Main stage timed with
HIP events, variants interleaved.
    python tools/ab_gat_tile.py [--heads 8 --C 32 --vecs 0,1,2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--heads", type=int, default=8)
    ap.add_argument("--C", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--vecs", default="0,1,2")
    ap.add_argument("--graph", default="rmat21", choices=["rmat21", "small"])
    args = ap.parse_args()
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graph import Graph, GAT_TARGET_TASKS
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv._structure import gat_loops
    lib = mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    H, C = args.heads, args.C
    if args.graph == "rmat21":
        N = 1 << 21
        ei = gat_loops(rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev), N)
    else:
        N = 1 << 14
        ei = gat_loops(rmat_edge_index(scale=14, n_samples=200_000, seed=1, device=dev), N)
    csr = Graph(ei, N, N, target_tasks=GAT_TARGET_TASKS).dst
    n_edges = ei.shape[1]
    del ei
    gen = torch.Generator(device=dev).manual_seed(2)
    xw = torch.randn(N, H * C, device=dev, generator=gen)
    att = torch.randn(H, 2 * C, device=dev, generator=gen) * 0.1
    a_src = torch.empty(N, H, device=dev)
    a_dst = torch.empty(N, H, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.mp_gat_node_scores_f32(xw.data_ptr(), N, H, C, att.data_ptr(), a_src.data_ptr(),
                                          a_dst.data_ptr(), st), "scores")
    g = csr.struct("other")
    sb = lib.mp_gat_slab_bytes(g, H, C)
    slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    vecs = [int(v) for v in args.vecs.split(",")]
    outs = {v: torch.empty(N, H * C, device=dev) for v in vecs}
    stats = {v: torch.empty(N, H, 2, device=dev) for v in vecs}
    old = lib.mp_tune(_lib.MP_TUNE_GAT_TILE_VEC, -1)

    def launch(v, stages):
        lib.mp_tune(_lib.MP_TUNE_GAT_TILE_VEC, v)
        _lib.check(lib.mp_gat_aggregate_att_f32(g, xw.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                att.data_ptr(), H, C, 0.2, None, outs[v].data_ptr(), H * C,
                                                stats[v].data_ptr(), slab.data_ptr(), sb, stages, st), "gat")
    for v in vecs:
        launch(v, _lib.MP_STAGE_ALL)
    torch.cuda.synchronize()
    base = vecs[0]
    same = {v: bool(torch.equal(outs[v], outs[base])) and bool(torch.equal(stats[v], stats[base])) for v in vecs}
    diff = {v: float((outs[v] - outs[base]).abs().max()) for v in vecs}
    times = {v: [] for v in vecs}
    fix = {v: [] for v in vecs}
    for _ in range(args.rounds):
        for v in vecs:
            for stage, acc in ((_lib.MP_STAGE_MAIN, times), (_lib.MP_STAGE_FIXUP, fix)):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(10):
                    launch(v, stage)
                b.record()
                torch.cuda.synchronize()
                acc[v].append(a.elapsed_time(b) / 10)
    lib.mp_tune(_lib.MP_TUNE_GAT_TILE_VEC, old)
    for v in vecs:
        t = sorted(times[v])
        fx = sorted(fix[v])
        print(json.dumps({"gat_tile_vec": v, "graph": args.graph, "heads": H, "C": C, "edges": n_edges,
                          "median_ms": round(t[len(t) // 2], 4), "min_ms": round(t[0], 4),
                          "fixup_ms": round(fx[len(fx) // 2], 4),
                          "bitwise_equal_to_first": same[v], "max_abs_diff": diff[v]}), flush=True)


if __name__ == "__main__":
    main()
