"""In-process A/B of aggregation-kernel build variants (tools/variants/lib_*.so).

Rule 24 of the CDNA guide: variants are timed in interleaved rounds inside
ONE process on ONE device.  Each variant's output is checked bitwise against
the first variant.  Usage (GPU box):
    python tools/ab_bench.py [--chunks 256,512] [--variants base,u16,...] [--rounds 5]
"""
import argparse
import glob
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
    ap.add_argument("--chunks", default="256")
    ap.add_argument("--variants", default="")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--F", type=int, default=256)
    ap.add_argument("--reduce", default="sum")
    ap.add_argument("--graph", default="rmat21", choices=["rmat21", "reddit"])
    args = ap.parse_args()
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    if args.graph == "reddit":   # config 4: Reddit-scale power law (x fits the Infinity Cache)
        from mi355_mp.graphgen import powerlaw_edge_index
        N = 232_965
        ei2 = powerlaw_edge_index(N, 114_615_892, seed=3, device=dev)
        norm = torch.rand(ei2.shape[1], device=dev)
    else:
        N = 1 << 21
        ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
        ei2, norm = GCNConv.norm(ei, N)
    x = torch.randn(N, args.F, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    bias = torch.randn(args.F, device=dev) * 0.1
    vdir = os.path.join(ROOT, "tools", "variants")
    names = args.variants.split(",") if args.variants else sorted(
        os.path.basename(f)[4:-3] for f in glob.glob(os.path.join(vdir, "lib_*.so")))
    libs = {n: _lib.load(os.path.join(vdir, "lib_%s.so" % n)) for n in names}
    red = _lib.MP_REDUCE[args.reduce]
    results = {}
    for chunk in [int(c) for c in args.chunks.split(",")]:
        csr = Graph(ei2, N, N, chunk=chunk).dst
        w = csr.to_csr_order(norm) if args.reduce in ("sum", "mean") else None
        g = csr.struct("other")
        outs = {n: torch.empty(N, args.F, device=dev) for n in names}
        args_out = {n: torch.empty(N, args.F, dtype=torch.int64, device=dev) if red >= 2 else None for n in names}
        sb = libs[names[0]].mp_aggregate_slab_bytes(g, args.F, red)
        slab = torch.empty(sb, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream().cuda_stream

        def launch(lib, out, stages, arg=None):
            _lib.check(lib.mp_aggregate_f32(g, _lib.ptr(w), x.data_ptr(), x.stride(0), args.F, red, 0,
                                            bias.data_ptr(), out.data_ptr(), out.stride(0), _lib.ptr(arg),
                                            slab.data_ptr(), sb, stages, st), "agg")
        for n in names:
            launch(libs[n], outs[n], _lib.MP_STAGE_ALL, args_out[n])
        torch.cuda.synchronize()
        same = {n: bool(torch.equal(outs[n], outs[names[0]])) and
                (args_out[n] is None or bool(torch.equal(args_out[n], args_out[names[0]]))) for n in names}
        times = {n: [] for n in names}
        ftimes = {n: [] for n in names}
        for _ in range(args.rounds):
            for n in names:
                for stage, acc in ((_lib.MP_STAGE_MAIN, times), (_lib.MP_STAGE_FIXUP, ftimes)):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(args.reps):
                        launch(libs[n], outs[n], stage, args_out[n])
                    b.record()
                    torch.cuda.synchronize()
                    acc[n].append(a.elapsed_time(b) / args.reps)
        for n in names:
            t = sorted(times[n])
            ft = sorted(ftimes[n])
            results["%s/chunk%d" % (n, chunk)] = {"median_ms": t[len(t) // 2], "min_ms": t[0],
                                                  "fixup_ms": ft[len(ft) // 2],
                                                  "bitwise_equal_to_%s" % names[0]: same[n],
                                                  "n_split": csr.n_split, "n_waves": csr.n_waves}
    for k, v in results.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main()
