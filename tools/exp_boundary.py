"""A/B of the sharded step's boundary-pass shape on one GPU (round 6).

A synthetic graph with the shape of config 2's P = 4 boundary pass (rank 0 of
profiles/r05_bench_rmat21_gloo4_rehearsal.json): 530K own rows, 47 % of them
without boundary edges, 1.51M boundary edges over 347K halo rows (a hub-heavy
source draw), F = 256.  Each variant is timed with HIP events over
back-to-back launches (median of rounds); every variant's output is checked
bitwise against the plain INIT_FROM_OUT launch:

  plain        sum into a fresh out (no read of out)          -- the floor
  init         MP_FLAG_INIT_FROM_OUT (every row's out read when it opens)
  skip         + MP_FLAG_SKIP_EMPTY (rows without slots untouched; their bias
               comes with the interior pass's per-row flags)
  *_u16        the same with 16 row loads in flight per wave (the near-x batch)
  chunk C      skip at merge-path chunk C

Usage: python tools/exp_boundary.py [--rows 530000] [--edges 1510000] ...
Prints one JSON line per variant."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=530_000)
    ap.add_argument("--halo", type=int, default=347_000)
    ap.add_argument("--edges", type=int, default=1_510_000)
    ap.add_argument("--empty", type=float, default=0.47)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--tiles-only", action="store_true",
                    help="only the feature-tile order A/B (XCD-affine vs one tile after another) of plain sums")
    args = ap.parse_args()
    from mi355_mp import _lib, ops
    from mi355_mp.graph import Graph
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    n, h, E, F = args.rows, args.halo, args.edges, 256
    # destination rows: a non-empty subset, sizes ~ geometric; sources hub-heavy
    nonempty = torch.randperm(n, device=dev, generator=g)[:int(n * (1 - args.empty))]
    dst = nonempty[torch.randint(0, nonempty.numel(), (E,), device=dev, generator=g)]
    u = torch.rand(E, device=dev, generator=g)
    src = (u.pow(3.0) * h).to(torch.int64).clamp(max=h - 1)
    ei = torch.stack([src, dst])
    x = torch.randn(h, F, device=dev, generator=g)
    w = torch.rand(E, device=dev, generator=g)
    bias = torch.randn(F, device=dev, generator=g)
    out0 = torch.randn(n, F, device=dev, generator=g)

    def make(chunk=None):
        gr = Graph(ei, n, h, chunk=chunk)
        return gr, gr.dst.to_csr_order(w)

    def timed(fn):
        per = []
        fn()
        for _ in range(args.rounds):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                fn()
            b.record()
            torch.cuda.synchronize()
            per.append(a.elapsed_time(b) / args.reps)
        return sorted(per)[len(per) // 2]

    gr, wc = make()
    out = out0.clone()
    if args.tiles_only:
        res = {"rows": n, "edges": E, "x_rows": h, "x_MB": h * F * 4 / 2**20}
        for seq in (0, 1):
            prev = lib.mp_tune(_lib.MP_TUNE_FLAT_SEQ_TILES, seq)
            try:
                res["seq_tiles_%d_ms" % seq] = timed(lambda: ops.aggregate_tiles(gr.dst, "other", x, wc, F, out, "sum",
                                                                               0, bias))
            finally:
                lib.mp_tune(_lib.MP_TUNE_FLAT_SEQ_TILES, prev)
        # the XR kernel instance (per-row bias flags: every row flagged) against the plain launch
        ones = torch.ones(n, dtype=torch.int32, device=dev)
        res["plain_bias_ms"] = timed(lambda: ops.aggregate_tiles(gr.dst, "other", x, wc, F, out, "sum", 0, bias))
        res["xr_bias_rows_ms"] = timed(lambda: ops.aggregate_tiles(gr.dst, "other", x, wc, F, out, "sum", 0, bias,
                                                                   bias_rows=ones))
        # XR without the bias flags (MP_FLAG_SKIP_EMPTY alone forces the XR instance)
        res["xr_skip_only_ms"] = timed(lambda: ops.aggregate_tiles(gr.dst, "other", x, wc, F, out, "sum",
                                                                   _lib.MP_FLAG_SKIP_EMPTY, bias))
        print(json.dumps(res), flush=True)
        return
    INIT, SKIP = _lib.MP_FLAG_INIT_FROM_OUT, _lib.MP_FLAG_SKIP_EMPTY

    def run(flags, chunk_graph=None, u16=False):
        G, W = chunk_graph or (gr, wc)
        prev = lib.mp_tune(_lib.MP_TUNE_FLAT_FAR_MIN_BYTES, 1 << 40) if u16 else None
        try:
            ops.aggregate_tiles(G.dst, "other", x, W, F, out, "sum", flags, bias)
        finally:
            if prev is not None:
                lib.mp_tune(_lib.MP_TUNE_FLAT_FAR_MIN_BYTES, prev)

    # reference: INIT, from out0 (one launch)
    out.copy_(out0)
    run(INIT)
    ref = out.clone()
    deg = gr.dst.degree()
    rows_nonempty = int((deg > 0).sum())
    base = {"rows": n, "rows_with_slots": rows_nonempty, "edges": E, "halo_rows": h, "chunk": gr.dst.chunk,
            "tasks": gr.dst.n_waves, "split_rows": gr.dst.n_split, "x_MB": h * F * 4 / 2**20}
    print(json.dumps(dict(base, variant="shape")), flush=True)
    for name, flags, u16 in (("plain", 0, False), ("init", INIT, False), ("skip", INIT | SKIP, False),
                             ("plain_u16", 0, True), ("skip_u16", INIT | SKIP, True)):
        ms = timed(lambda: run(flags, u16=u16))
        out.copy_(out0)
        run(flags, u16=u16)
        if flags & INIT:
            want = ref if not flags & SKIP else torch.where((deg > 0).view(-1, 1), ref, out0)
            same = bool(torch.equal(out, want))
        else:
            same = None
        print(json.dumps({"variant": name, "ms": ms, "edges_per_s": E / (ms * 1e-3), "bitwise_vs_init": same}),
              flush=True)
    for chunk in (64, 256, 512):
        cg = make(chunk)
        ms = timed(lambda: run(INIT | SKIP, chunk_graph=cg))
        print(json.dumps({"variant": "skip chunk %d" % chunk, "ms": ms, "tasks": cg[0].dst.n_waves,
                          "edges_per_s": E / (ms * 1e-3)}), flush=True)
    # the interior pass's per-row bias (the boundary's empty rows) against a plain bias
    flags_rows = (deg == 0).to(torch.int32)
    for name, br in (("bias_all_rows", None), ("bias_rows_flags", flags_rows)):
        ms = timed(lambda: ops.aggregate_tiles(gr.dst, "other", x, wc, F, out, "sum", 0, bias, bias_rows=br))
        print(json.dumps({"variant": name, "ms": ms}), flush=True)
    ops.aggregate_tiles(gr.dst, "other", x, wc, F, out, "sum", 0, bias, bias_rows=flags_rows)
    o1 = out.clone()
    ops.aggregate_tiles(gr.dst, "other", x, wc, F, out, "sum", 0, None)
    want = torch.where((deg == 0).view(-1, 1), out + bias, out)
    print(json.dumps({"variant": "bias_rows_check", "bitwise": bool(torch.equal(o1, want))}), flush=True)


if __name__ == "__main__":
    main()
