"""How a short-row sum pass's time scales with its size (round 6): the P = 8
interior shape (4.6 edges a row, x ~ 257 MB of 1 KB rows, F = 256) at 1x, 2x,
4x, 8x the rows and edges, one launch each (mp_aggregate_tiles_f32, row-major
operands), HIP events over back-to-back launches.  A fixed cost per launch
(launch + tail) shows as the intercept of time against size.
Usage: python tools/exp_pass_scale.py   (one JSON line per size)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")]

import torch  # noqa: E402


def main():
    from mi355_mp import ops
    from mi355_mp.graph import Graph
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    n_x, F = 263_000, 256
    x = torch.randn(n_x, F, device=dev, generator=g)
    for s in (1, 2, 4, 8):
        n, E = 263_000 * s, 1_210_000 * s
        dst = torch.randint(0, n, (E,), device=dev, generator=g)
        u = torch.rand(E, device=dev, generator=g)
        src = (u.pow(2.0) * n_x).to(torch.int64).clamp(max=n_x - 1)
        gr = Graph(torch.stack([src, dst]), n, n_x)
        w = gr.dst.to_csr_order(torch.rand(E, device=dev, generator=g))
        out = torch.empty(n, F, device=dev)

        def run():
            ops.aggregate_tiles(gr.dst, "other", x, w, F, out, "sum", 0, None)
        run()
        per = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                run()
            b.record()
            torch.cuda.synchronize()
            per.append(a.elapsed_time(b) / 20)
        ms = sorted(per)[2]
        print(json.dumps({"scale": s, "rows": n, "edges": E, "chunk": gr.dst.chunk, "tasks": gr.dst.n_waves,
                          "ms": ms, "edges_per_s": E / (ms * 1e-3)}), flush=True)
        del gr, w, out, dst, src, u


if __name__ == "__main__":
    main()
