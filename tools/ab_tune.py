"""In-process A/B of aggregation dispatch settings (mp_tune keys) and build variants.

Rule 24 of the CDNA guide: variants are timed in interleaved rounds inside ONE
process on ONE device.  Every configuration's output (and argmax) is checked
bitwise against the first one.  Usage (GPU box):

    python tools/ab_tune.py --configs "base;pair:flat_pair=1;p32@upair32:flat_pair=1" \
        [--graph rmat21|reddit|products] [--F 256] [--reduce sum] [--rounds 5]

A config is  name[@variant]:key=value,key=value  -- keys are mp_tune names
without the MP_TUNE_ prefix (lower case); @variant loads
tools/variants/lib_<variant>.so (make -C pytorch_geometric-1_amd/csrc variant
NAME=<variant> DEFS=...) instead of the in-tree library.
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


def parse_configs(text):
    out = []
    for item in text.split(";"):
        item = item.strip()
        if not item:
            continue
        head, _, kv = item.partition(":")
        name, _, variant = head.partition("@")
        keys = {}
        for pair in filter(None, kv.split(",")):
            k, v = pair.split("=")
            keys[k.strip()] = int(v)
        out.append((name, variant or None, keys))
    return out


def make_graph(kind, dev):
    from mi355_mp.graphgen import rmat_edge_index, powerlaw_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    if kind == "reddit":    # config 4: x fits the Infinity Cache
        N = 232_965
        ei = powerlaw_edge_index(N, 114_615_892, seed=3, device=dev)
        return N, ei, torch.rand(ei.shape[1], device=dev)
    if kind == "products":  # config 5 on one GPU
        N = 2_449_029
        ei = powerlaw_edge_index(N, 123_718_280, seed=4, device=dev)
    else:                   # config 2
        N = 1 << 21
        ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    ei2, norm = GCNConv.norm(ei, N)
    return N, ei2, norm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="base")
    ap.add_argument("--graph", default="rmat21", choices=["rmat21", "reddit", "products"])
    ap.add_argument("--F", type=int, default=256)
    ap.add_argument("--reduce", default="sum")
    ap.add_argument("--weighted", type=int, default=1)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graph import Graph
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, ei, norm = make_graph(args.graph, dev)
    csr = Graph(ei, N, N, chunk=args.chunk or None).dst
    del ei
    x = torch.randn(N, args.F, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    bias = torch.randn(args.F, device=dev) * 0.1
    w = csr.to_csr_order(norm) if args.weighted else None
    del norm
    red = _lib.MP_REDUCE[args.reduce]
    g = csr.struct("other")
    st = torch.cuda.current_stream().cuda_stream
    configs = parse_configs(args.configs)
    libs = {}
    for name, variant, _ in configs:
        path = os.path.join(ROOT, "tools", "variants", "lib_%s.so" % variant) if variant else None
        libs[name] = _lib.load(path) if path else _lib.load()
    sb = max(libs[n].mp_aggregate_slab_bytes(g, args.F, red) for n in libs)
    slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    outs = {n: torch.empty(N, args.F, device=dev) for n, _, _ in configs}
    arg_outs = {n: torch.empty(N, args.F, dtype=torch.int64, device=dev) if red >= 2 else None
                for n, _, _ in configs}

    def with_keys(lib, keys, fn):
        prev = {}
        for k, v in keys.items():
            prev[k] = lib.mp_tune(getattr(_lib, "MP_TUNE_" + k.upper()), v)
        try:
            return fn()
        finally:
            for k, v in prev.items():
                lib.mp_tune(getattr(_lib, "MP_TUNE_" + k.upper()), v)

    def launch(name, keys, stages):
        lib = libs[name]
        _lib.check(lib.mp_aggregate_f32(g, _lib.ptr(w), x.data_ptr(), x.stride(0), args.F, red, 0, bias.data_ptr(),
                                        outs[name].data_ptr(), outs[name].stride(0), _lib.ptr(arg_outs[name]),
                                        slab.data_ptr(), sb, stages, st), "mp_aggregate_f32")

    kernel = {}
    for name, _, keys in configs:
        with_keys(libs[name], keys, lambda: launch(name, keys, _lib.MP_STAGE_ALL))
        buf = __import__("ctypes").create_string_buffer(1024)
        with_keys(libs[name], keys, lambda: libs[name].mp_aggregate_kernel_name(
            g, _lib.ptr(w), x.data_ptr(), x.stride(0), args.F, red, bias.data_ptr(), outs[name].data_ptr(),
            outs[name].stride(0), buf, 1024, st))
        kernel[name] = buf.value.decode()
    torch.cuda.synchronize()
    first = configs[0][0]
    same = {n: bool(torch.equal(outs[n], outs[first])) and
            (arg_outs[n] is None or bool(torch.equal(arg_outs[n], arg_outs[first]))) for n, _, _ in configs}
    times = {n: [] for n, _, _ in configs}
    ftimes = {n: [] for n, _, _ in configs}
    for _ in range(args.rounds):
        for name, _, keys in configs:
            for stage, acc in ((_lib.MP_STAGE_MAIN, times), (_lib.MP_STAGE_FIXUP, ftimes)):
                def run():
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(args.reps):
                        launch(name, keys, stage)
                    b.record()
                    torch.cuda.synchronize()
                    return a.elapsed_time(b) / args.reps
                acc[name].append(with_keys(libs[name], keys, run))
    for name, variant, keys in configs:
        t = sorted(times[name])
        ft = sorted(ftimes[name])
        print(json.dumps({"config": name, "variant": variant, "keys": keys, "graph": args.graph, "F": args.F,
                          "reduce": args.reduce, "weighted": bool(args.weighted), "chunk": csr.chunk,
                          "median_ms": round(t[len(t) // 2], 4), "min_ms": round(t[0], 4),
                          "fixup_ms": round(ft[len(ft) // 2], 4),
                          "bitwise_equal_to_%s" % first: same[name], "kernel": kernel[name]}))


if __name__ == "__main__":
    main()
