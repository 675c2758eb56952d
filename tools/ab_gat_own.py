"""In-process A/B of the fused GAT forward on config 3 (RMAT21, heads=8, C=32):
a_src gathered per slot (mp_gat_aggregate_f32, LDS-staged windows) against
a_src recomputed from each gathered xw row (mp_gat_aggregate_att_f32).  a_src /
a_dst come from mp_gat_node_scores_f32 on the same xw and att, so the two
outputs must be bitwise equal.  Main stage timed with HIP events, interleaved.
    python tools/ab_gat_own.py [--heads 8 --C 32]
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
    args = ap.parse_args()
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv._structure import gat_loops
    lib = mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, H, C = 1 << 21, args.heads, args.C
    ei = gat_loops(rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev), N)
    from mi355_mp.graph import GAT_TARGET_TASKS
    csr = Graph(ei, N, N, target_tasks=GAT_TARGET_TASKS).dst
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
    outs = {n: torch.empty(N, H * C, device=dev) for n in ("gather", "own")}
    stats = {n: torch.empty(N, H, 2, device=dev) for n in outs}

    def launch(n, stages):
        _lib.check(lib.mp_gat_aggregate_att_f32(g, xw.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                att.data_ptr() if n == "own" else None, H, C, 0.2, None,
                                                outs[n].data_ptr(), H * C, stats[n].data_ptr(), slab.data_ptr(), sb,
                                                stages, st), "gat")
    for n in outs:
        launch(n, _lib.MP_STAGE_ALL)
    torch.cuda.synchronize()
    same = bool(torch.equal(outs["own"], outs["gather"])) and bool(torch.equal(stats["own"], stats["gather"]))
    times = {n: [] for n in outs}
    for _ in range(args.rounds):
        for n in outs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                launch(n, _lib.MP_STAGE_MAIN)
            b.record()
            torch.cuda.synchronize()
            times[n].append(a.elapsed_time(b) / 10)
    for n in outs:
        t = sorted(times[n])
        print(json.dumps({"config": n, "heads": H, "C": C, "median_ms": round(t[len(t) // 2], 4),
                          "min_ms": round(t[0], 4), "bitwise_equal": same}))


if __name__ == "__main__":
    main()
