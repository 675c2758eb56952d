"""Ceiling of an LDS hub-row cache for the config-4 max kernel (timing only).

The max kernel over the Reddit-scale first-occurrence graph is bound by the
texture-address unit, so a gather served from LDS instead of the
vector memory pipeline saves its whole TA cost.  The ceiling of that idea is
the kernel's time with the gathers of the K hottest sources removed: the same
graph minus every edge whose source is among the top K by out-degree.  Prints
the main-kernel time per K (K = 0 is the real graph).
    python tools/exp_hot_lds.py [--ks 0,160,320,640,1280]
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
    ap.add_argument("--ks", default="0,160,320,640,1280")
    ap.add_argument("--reduce", default="max")
    args = ap.parse_args()
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import powerlaw_edge_index
    mi355_mp.load_native()
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    N, E, F = 232_965, 114_615_892, 256
    ei = powerlaw_edge_index(N, E, seed=3, device=dev)
    # first occurrences of (dst, src), in edge order (what the layer gathers)
    key = ei[1] * N + ei[0]
    order = torch.sort(key, stable=True).indices
    ks = key[order]
    first = torch.ones_like(ks, dtype=torch.bool)
    first[1:] = ks[1:] != ks[:-1]
    keep = torch.zeros(E, dtype=torch.bool, device=dev)
    keep[order[first]] = True
    ei = ei[:, keep]
    del key, order, ks, first, keep
    deg = torch.bincount(ei[0], minlength=N)
    rank = torch.argsort(deg, descending=True)
    x = torch.randn(N, F, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    out = torch.empty(N, F, device=dev)
    arg = torch.empty(N, F, dtype=torch.int64, device=dev)
    red = _lib.MP_REDUCE[args.reduce]
    st = torch.cuda.current_stream().cuda_stream
    for k in [int(v) for v in args.ks.split(",")]:
        if k:
            hot = torch.zeros(N, dtype=torch.bool, device=dev)
            hot[rank[:k]] = True
            e_k = ei[:, ~hot[ei[0]]]
        else:
            e_k = ei
        csr = Graph(e_k, N, N).dst
        s = csr.struct("other")
        sb = lib.mp_aggregate_slab_bytes(s, F, red)
        slab = torch.empty(sb, dtype=torch.uint8, device=dev)

        def agg(stages):
            _lib.check(lib.mp_aggregate_f32(s, None, x.data_ptr(), F, F, red, 0, None, out.data_ptr(), F,
                                            arg.data_ptr() if red >= 2 else None, slab.data_ptr(), sb, stages, st),
                       "agg")
        agg(_lib.MP_STAGE_ALL)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                agg(_lib.MP_STAGE_MAIN)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / 10)
        ts.sort()
        print(json.dumps({"hot_rows_removed": k, "gathers": int(e_k.shape[1]),
                          "share_removed": 1 - e_k.shape[1] / ei.shape[1], "main_ms": round(ts[2], 4)}), flush=True)
        del csr, s, slab, e_k


if __name__ == "__main__":
    main()
