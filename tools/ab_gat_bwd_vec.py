"""In-process A/B of the GAT backward's feature-tile width (MP_TUNE_GAT_BWD_VEC
4 / 2 / 1: 256- / 128- / 64-feature tiles of the transposed pass) on config 3
(RMAT21 + GAT loops, GATConv(256, 32, heads=8), training forward + backward).
Variants interleaved per round; each round times the layer step (forward +
backward) with HIP events; gradients of every variant are compared with the
default's (max |diff| / max |ref| per tensor).
    python tools/ab_gat_bwd_vec.py [--vecs 4,2,1] [--rounds 5] [--dropout 0]
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
    ap.add_argument("--vecs", default="4,2,1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--dropout", type=float, default=0.0)
    args = ap.parse_args()
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn import GATConv
    lib = mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, H, C, Fi = 1 << 21, 8, 32, 256
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    gen = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn(N, Fi, device=dev, generator=gen)
    gout = torch.randn(N, H * C, device=dev, generator=gen)
    torch.manual_seed(0)
    conv = GATConv(Fi, C, heads=H, dropout=args.dropout).to(dev).train()
    vecs = [int(v) for v in args.vecs.split(",")]
    old = lib.mp_tune(_lib.MP_TUNE_GAT_BWD_VEC, -1)

    def run(v):
        assert lib.mp_tune(_lib.MP_TUNE_GAT_BWD_VEC, v) >= 0
        conv.zero_grad()
        xd = x.clone().requires_grad_(True)
        torch.cuda.manual_seed(5)
        out = conv(xd, ei)
        out.backward(gout)
        return [xd.grad, conv.weight.grad.clone(), conv.att.grad.clone(), conv.bias.grad.clone()]

    ref = {v: run(v) for v in vecs}
    torch.cuda.synchronize()
    diffs = {v: [float((a - b).abs().max() / b.abs().max()) for a, b in zip(ref[v], ref[vecs[0]])] for v in vecs}
    del ref
    times = {v: [] for v in vecs}
    for _ in range(args.rounds):
        for v in vecs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(v)
            b.record()
            torch.cuda.synchronize()
            times[v].append(a.elapsed_time(b))
    lib.mp_tune(_lib.MP_TUNE_GAT_BWD_VEC, old)
    for v in vecs:
        t = sorted(times[v])
        print(json.dumps({"gat_bwd_vec": v, "dropout": args.dropout, "layer_fwd_bwd_median_ms": t[len(t) // 2],
                          "min_ms": t[0], "rel_diff_vs_first[gx,gW,gatt,gb]": diffs[v]}), flush=True)


if __name__ == "__main__":
    main()
