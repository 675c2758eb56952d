"""Why a sharded step's short-row passes run slower than the same shape alone
(round 6): rank 0 of a P = 8 split of the config-2 graph (rmat21,
GCN norm, edge-balanced cut) taken apart on ONE GPU -- its interior edges
(own -> own), its pulled boundary edges (halo -> own, halo rows compacted)
and its pushed edges (own -> peer rows, the send packing's shape) -- each
pass timed (a) warm: 20 launches back to back, (b) cold: the L2 / Infinity
Cache flushed (1 GiB written) before every launch, (c) in the step's order
(pack, interior, boundary) and with the interior first; the interior also
as the step launches it (+ bias on the rows without a boundary edge), and
on a stream of its own (the step's compute stream).  Plus the interior's
edge count with uniform sources, for the distribution's share.
Usage: python tools/exp_interior.py   (one JSON line per measurement)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")]

import torch  # noqa: E402


def main():
    from mi355_mp import _lib, ops
    from mi355_mp import dist as mdist
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    dev = torch.device("cuda", 0)
    N, F, P = 1 << 21, 256, 8
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    ei2, norm = GCNConv.norm(ei, N)
    del ei
    cuts = mdist.balanced_cut_points(torch.bincount(ei2[1], minlength=N), P)
    c1 = int(cuts[1])
    src, dst = ei2[0], ei2[1]
    g = torch.Generator(device=dev).manual_seed(5)
    x_own = torch.randn(c1, F, device=dev, generator=g)
    flush = torch.empty(1 << 28, device=dev)          # 1 GiB

    def graph_of(mask, rows_of, srcs_of):
        s, d, w = src[mask], dst[mask], norm[mask]
        d_u, d_c = torch.unique(d, return_inverse=True) if rows_of is None else (None, d)
        s_u, s_c = torch.unique(s, return_inverse=True) if srcs_of is None else (None, s)
        n_rows = d_u.numel() if d_u is not None else rows_of
        n_x = s_u.numel() if s_u is not None else srcs_of
        gr = Graph(torch.stack([s_c, d_c]), n_rows, n_x)
        return gr, gr.dst.to_csr_order(w), n_rows, n_x

    own_d, own_s = dst < c1, src < c1
    shapes = {}
    shapes["interior"] = graph_of(own_d & own_s, c1, c1)
    shapes["boundary_pull"] = graph_of(own_d & ~own_s, c1, None)
    shapes["send_pack"] = graph_of(~own_d & own_s, None, c1)
    E_int = int((own_d & own_s).sum())
    us = torch.randint(0, c1, (E_int,), device=dev, generator=g)
    ud = torch.sort(torch.randint(0, c1, (E_int,), device=dev, generator=g)).values
    gu = Graph(torch.stack([us, ud]), c1, c1)
    shapes["interior_uniform_src"] = (gu, gu.dst.to_csr_order(torch.rand(E_int, device=dev, generator=g)), c1, c1)
    del ei2, norm, src, dst

    # the step's own interior launch: + bias on the rows without a boundary edge
    shapes["interior_bias_rows"] = shapes["interior"]
    shapes["interior_bias"] = shapes["interior"]           # bias on every row, no flags
    shapes["interior_main"] = shapes["interior"]           # the main launch alone (no split-row fix-up)
    shapes["interior_bias_rows_main"] = shapes["interior"]
    rp = shapes["boundary_pull"][0].dst.rowptr
    no_bnd = (rp[1:] == rp[:-1]).to(torch.int32)
    bias = torch.randn(F, device=dev, generator=g) * 0.1
    xs, outs, runs = {}, {}, {}
    for k, (gr, w, n_rows, n_x) in shapes.items():
        xs[k] = x_own if n_x == c1 else torch.randn(n_x, F, device=dev, generator=g)
        outs[k] = torch.empty(n_rows, F, device=dev)
        b, br = {"interior_bias_rows": (bias, no_bnd), "interior_bias": (bias, None),
                 "interior_bias_rows_main": (bias, no_bnd)}.get(k, (None, None))
        st = _lib.MP_STAGE_MAIN if k.endswith("_main") else _lib.MP_STAGE_ALL
        runs[k] = (lambda gr=gr, w=w, k=k, b=b, br=br, st=st: ops.aggregate_tiles(
            gr.dst, "other", xs[k], w, F, outs[k], "sum", 0, b, bias_rows=br, stages=st))
        runs[k]()
    torch.cuda.synchronize()

    def ev():
        return torch.cuda.Event(enable_timing=True)

    for k, (gr, w, n_rows, n_x) in shapes.items():
        E = gr.dst.n_edges if hasattr(gr.dst, "n_edges") else int(w.numel())
        warm = []
        for _ in range(5):
            a, b = ev(), ev()
            a.record()
            for _ in range(20):
                runs[k]()
            b.record()
            torch.cuda.synchronize()
            warm.append(a.elapsed_time(b) / 20)
        cold = []
        for _ in range(9):
            flush.fill_(1.0)
            a, b = ev(), ev()
            a.record()
            runs[k]()
            b.record()
            torch.cuda.synchronize()
            cold.append(a.elapsed_time(b))
        wm, cm = sorted(warm)[2], sorted(cold)[4]
        print(json.dumps({"pass": k, "rows": n_rows, "x_rows": n_x, "edges": E, "warm_ms": wm, "cold_ms": cm,
                          "warm_edges_per_s": E / (wm * 1e-3), "cold_edges_per_s": E / (cm * 1e-3)}), flush=True)

    for order in (("send_pack", "interior", "boundary_pull"), ("interior", "send_pack", "boundary_pull"),
                  ("send_pack", "interior_bias_rows", "boundary_pull")):
        t = {k: [] for k in order}
        for _ in range(9):
            e = [ev() for _ in range(len(order) + 1)]
            e[0].record()
            for i, k in enumerate(order):
                runs[k]()
                e[i + 1].record()
            torch.cuda.synchronize()
            for i, k in enumerate(order):
                t[k].append(e[i].elapsed_time(e[i + 1]))
        med = {k: sorted(v)[4] for k, v in t.items()}
        print(json.dumps({"sequence": list(order), "ms": med, "total_ms": sum(med.values())}), flush=True)

    # the step's order on a non-default stream (OverlappedAggregation's compute stream)
    side = torch.cuda.Stream(device=dev)
    order = ("send_pack", "interior_bias_rows", "boundary_pull")
    t = {k: [] for k in order}
    with torch.cuda.stream(side):
        for _ in range(9):
            e = [ev() for _ in range(len(order) + 1)]
            e[0].record()
            for i, k in enumerate(order):
                runs[k]()
                e[i + 1].record()
            side.synchronize()
            for i, k in enumerate(order):
                t[k].append(e[i].elapsed_time(e[i + 1]))
    med = {k: sorted(v)[4] for k, v in t.items()}
    print(json.dumps({"sequence": list(order), "stream": "non-default", "ms": med,
                      "total_ms": sum(med.values())}), flush=True)


if __name__ == "__main__":
    main()
