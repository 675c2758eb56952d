"""Repro of the GAT-dropout fuzz example (N=121, deg=23.82, H=4, C=64, p=0.9,
seed=121): per gradient, the engine's and the fp32 reference's max error
against float64 autograd of the reference formula."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")]
from oracle import pyg_ref as P  # noqa: E402
from mi355_mp import ops  # noqa: E402
from mi355_mp.graph import Graph  # noqa: E402

DEV = "cuda"
for (N, deg, H, C, p, chunk, seed) in [(121, 23.8203125, 4, 64, 0.9, 16, 121), (121, 23.8203125, 4, 64, 0.9, 256, 121)]:
    g = torch.Generator().manual_seed(seed)
    E = int(N * deg)
    dst = torch.randint(N, (E,), generator=g)
    ei = torch.stack([torch.randint(N, (E,), generator=g), dst])
    ei_l = P.add_self_loops(P.remove_self_loops(ei)[0], num_nodes=N)[0]
    xw = torch.randn(N, H * C, generator=g)
    att = torch.randn(1, H, 2 * C, generator=g) * 0.3
    bias = torch.randn(H * C, generator=g)
    gout = torch.randn(N, H * C, generator=g)
    graph = Graph(ei_l.to(DEV), N, N, chunk=chunk)
    xd = xw.to(DEV).requires_grad_(True)
    ad = att.to(DEV).requires_grad_(True)
    bd = bias.to(DEV).requires_grad_(True)
    seed_d = seed * 7919 + 13
    out, _ = ops.gat_propagate(graph, ei_l.to(DEV), xd, ad, H, C, 0.2, bd, False, dropout=p, seed=seed_d)
    out.backward(gout.to(DEV))
    keep = ops.gat_dropout_keep(graph, seed_d, p, H).cpu()
    res = {}
    for dt in (torch.float64, torch.float32):
        x_ = xw.to(dt).requires_grad_(True)
        a_ = att.to(dt).requires_grad_(True)
        b_ = bias.to(dt).requires_grad_(True)
        w = P.gat_conv(x_, ei_l, torch.eye(H * C, dtype=dt), a_, b_, H, C, drop_keep=keep, drop_p=p)
        w.backward(gout.to(dt))
        res[dt] = (w.detach(), x_.grad, a_.grad, b_.grad)
    r64, r32 = res[torch.float64], res[torch.float32]
    got = (out.detach().cpu(), xd.grad.cpu(), ad.grad.cpu(), bd.grad.cpu())
    for k, name in enumerate(("out", "d xw", "d att", "d bias")):
        e_eng = (got[k].double() - r64[k]).abs()
        e_ref = (r32[k].double() - r64[k]).abs()
        i = int(e_eng.argmax())
        print("chunk %d %-7s engine err %.3g at |ref| %.3g (tol %.3g) | fp32 reference err %.3g | max|ref| %.3g"
              % (chunk, name, float(e_eng.max()), float(r64[k].reshape(-1)[i].abs()),
                 1e-4 + 1e-4 * float(r64[k].reshape(-1)[i].abs()), float(e_ref.max()), float(r64[k].abs().max())))
