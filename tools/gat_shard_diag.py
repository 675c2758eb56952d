"""Diagnostic (round 5): sharded GATConv (3 gloo ranks sharing one GPU) vs the
single-GPU GATConv vs a float64 CPU oracle, per seed; prints one JSON line per
(seed, rank).  python tools/gat_shard_diag.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tests._ranks import run_ranks  # noqa: E402


def worker(rank, world, port, q, seeds):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mi355_mp import dist as mdist
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn import GATConv
        from oracle import pyg_ref as P
        dev = torch.device("cuda", 0)
        N, E, Fi, H, C = 3000, 60000, 64, 8, 32
        ei = powerlaw_edge_index(N, E, seed=47).to(dev)
        gen = torch.Generator().manual_seed(47)
        x = torch.randn(N, Fi, generator=gen).to(dev)
        gout = torch.randn(N, H * C, generator=gen).to(dev)
        out_l = []
        for seed in seeds:
            torch.manual_seed(seed)
            ref = GATConv(Fi, C, heads=H).to(dev)
            with torch.no_grad():
                ref.bias.normal_()
            mdist.broadcast_parameters(ref)
            xr = x.clone().requires_grad_(True)
            out_ref = ref(xr, ei)
            (out_ref * gout).sum().backward()
            sgs = mdist.ShardedGraph.for_gat_from_slices(ei[:, rank * E // world:(rank + 1) * E // world].clone(),
                                                         rank * E // world, N, rank, world)
            conv = mdist.ShardedGATConv(Fi, C, heads=H).to(dev)
            conv.load_state_dict(ref.state_dict())
            lo, hi = sgs.lo, sgs.hi
            xo = x[lo:hi].clone().requires_grad_(True)
            out = conv(xo, sgs)
            (out * gout[lo:hi]).sum().backward()
            mdist.allreduce_gradients(conv)
            # float64 oracle on the CPU
            x64 = x.cpu().double().requires_grad_(True)
            W64, a64, b64 = (t.detach().cpu().double().requires_grad_(True) for t in (ref.weight, ref.att, ref.bias))
            o64 = P.gat_conv(x64, ei.cpu(), W64, a64, b64, H, C)
            (o64 * gout.cpu().double()).sum().backward()
            gx64 = x64.grad[lo:hi]
            m = float(x64.grad.abs().max())
            out_l.append({"seed": seed, "rank": rank,
                          "shard_vs_single_gx": float((xo.grad - xr.grad[lo:hi]).abs().max()) / m,
                          "shard_vs_f64_gx": float((xo.grad.cpu().double() - gx64).abs().max()) / m,
                          "single_vs_f64_gx": float((xr.grad[lo:hi].cpu().double() - gx64).abs().max()) / m,
                          "shard_vs_f64_gatt": float((conv.att.grad.cpu().double() - a64.grad).abs().max()
                                                     / a64.grad.abs().max()),
                          "single_vs_f64_gatt": float((ref.att.grad.cpu().double() - a64.grad).abs().max()
                                                      / a64.grad.abs().max()),
                          "bias_absmax": float(ref.bias.abs().max()),
                          "out_absmax": float(out_ref.abs().max())})
        q.put((rank, out_l))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    res = run_ranks(worker, 3, timeout=400, args=(list(range(6)),))
    for rank, lst in res:
        for d in lst:
            print(json.dumps(d), flush=True)
