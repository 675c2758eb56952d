"""The hybrid halo cover (dist.HaloCover) against the pull exchange on the
config-2 graph at P ranks sharing one GPU (gloo; the exchange is staged
through the host, so only the compute is timed):

  1. full-size check: one real step of both exchanges; every rank's rows of the
     cover within 1e-5 * sum|w x| of the pull step (which equals one GPU's
     kernel per row order);
  2. per rank, one rank at a time (barriers between): HIP events around the
     compute of a step with 128-feature tiles -- send pack (pull: row gather;
     cover: the send-graph aggregation), interior passes, boundary passes --
     and the rows / bytes each rank receives and sends.

  python tools/exp_halo_cover_gpu.py --parts 2     (one JSON line per rank)
"""
import argparse
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        t = a.elapsed_time(b) / reps
        best = t if best is None else min(best, t)
    return best


def worker(rank, world, port, scale, samples, cpu_peers=False):
    import time
    t0 = time.time()

    def log(msg):   # progress on stderr (a long silent setup looks hung to the runner)
        print("[P=%d rank %d %.0fs] %s" % (world, rank, time.time() - t0, msg), file=sys.stderr, flush=True)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mi355_mp
    from mi355_mp import _lib, ops, dist as mdist
    from mi355_mp.graphgen import rmat_edge_index
    on_gpu = rank == 0 or not cpu_peers
    dev = torch.device("cuda", 0) if on_gpu else torch.device("cpu")
    if on_gpu:
        mi355_mp.load_native()
        torch.cuda.set_device(dev)
    N, F = 1 << scale, 256
    if cpu_peers:
        # every rank generates on the host (one RNG stream for all); only rank 0 runs on the GPU
        ei = rmat_edge_index(scale=scale, n_samples=samples, seed=1, device="cpu").to(dev)
    else:
        ei = rmat_edge_index(scale=scale, n_samples=samples, seed=1, device=dev)
    E_raw = ei.shape[1]
    s0, s1 = rank * E_raw // world, (rank + 1) * E_raw // world
    sl = ei[:, s0:s1].clone()
    del ei
    log("graph generated")
    sg = mdist.ShardedGraph.for_gcn_from_slices(sl, s0, N, rank, world)
    plan = sg.fwd
    log("shards built")
    if not on_gpu:
        # a host peer: its share of the cover's request exchange, then the barriers
        mdist.HaloCover(plan, sg.norm_fwd)
        log("cover requests answered")
        for _ in range(world):
            dist.barrier()
            dist.barrier()
        dist.destroy_process_group()
        return
    ov_p = mdist.OverlappedAggregation(plan, sg.norm_fwd, local_weights=True)
    log("pull exchange built")
    ov_c = mdist.OverlappedAggregation(plan, sg.norm_fwd, local_weights=True, cover=True)
    log("pull + cover exchanges built")
    gen = torch.Generator(device=dev).manual_seed(1)
    x_full = torch.randn(N, F, device=dev, generator=gen)
    bias = torch.randn(F, device=dev, generator=gen) * 0.1
    lo, hi = plan.lo, plan.hi

    def tiles_of(ov):
        ts = ov.local_tiles(F, 128)
        for t, xt in enumerate(ts):
            xt[:plan.n_own].copy_(x_full[lo:hi, 128 * t:128 * t + xt.shape[1]])
        return ts
    tp, tc = tiles_of(ov_p), tiles_of(ov_c)
    out_p = torch.empty(plan.n_own, F, device=dev)
    out_c = torch.empty_like(out_p)
    excess = None
    if not cpu_peers:
        ov_p.step_tiled(tp, out_p, bias)
        ov_c.step_tiled(tc, out_c, bias)
        torch.cuda.synchronize()
        log("one step of each exchange done")
        # |w x| sums over the rank's in-edges (pull layout: the received halo rows are exact copies)
        xa = plan.local_buffer(F)
        xa[:plan.n_own].copy_(x_full[lo:hi])
        plan.exchange_into(xa, ops.gather_rows)
        terms = ops._aggregate(sg.g_fwd.dst, "other", xa.abs(), sg._w[0].abs(), "sum", 0, None)[0]
        excess = float(((out_c - out_p).abs() - 1e-5 * terms.clamp(min=1.0)).max()) if plan.n_own else -1.0
        del xa, terms
        torch.cuda.empty_cache()

    def pieces(ov, ts):
        out = out_p
        offs = [0]
        for xt in ts:
            offs.append(offs[-1] + xt.shape[1])

        def send():
            for xt in ts:
                ov._send(xt[:plan.n_own])

        def interior():
            for t, xt in enumerate(ts):
                ops._aggregate(ov.g_int.dst, "other", xt[:plan.n_own], ov.w_int, "sum", 0, None,
                               out=out[:, offs[t]:offs[t + 1]])

        def boundary():
            for t, xt in enumerate(ts):
                ops._aggregate(ov.g_bnd.dst, "other", xt, ov.w_bnd, "sum", _lib.MP_FLAG_INIT_FROM_OUT,
                               bias[offs[t]:offs[t + 1]], out=out[:, offs[t]:offs[t + 1]])
        return {"send_ms": _ms(send), "interior_ms": _ms(interior), "boundary_ms": _ms(boundary)}

    res = None
    for r in range(world):
        dist.barrier()
        if r == rank:
            res = {"P": world, "rank": rank, "rows": plan.n_own, "edges": int(plan.edge_pos.numel()),
                   "cover_vs_pull_bound_excess": excess,
                   "within_1e-5_bound": None if excess is None else excess <= 0,
                   "pull": dict(rows_in=ov_p.n_local_src - plan.n_own, rows_out=ov_p.n_send,
                                peers_in=ov_p.recv_counts, **pieces(ov_p, tp)),
                   "cover": dict(rows_in=ov_c.n_local_src - plan.n_own, rows_out=ov_c.n_send,
                                 peers_in=ov_c.recv_counts, pulled_rows=ov_c.cover.n_pull_rows,
                                 partial_rows=ov_c.cover.n_push_rows, push_edges=ov_c.cover.n_push_edges,
                                 **pieces(ov_c, tc))}
            print(json.dumps(res), flush=True)
        dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=2)
    ap.add_argument("--scale", type=int, default=21)
    ap.add_argument("--samples", type=int, default=30_000_000)
    ap.add_argument("--cpu-peers", action="store_true",
                    help="ranks > 0 build on the host and only answer the cover's requests; rank 0 alone runs "
                         "on the GPU (no full-size check; P ranks sharing one GPU oversubscribe its queues)")
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    import threading
    import time

    def beat():   # the runner kills a call that writes nothing for 3 minutes
        while True:
            time.sleep(50)
            print("[alive]", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    procs = [ctx.Process(target=worker, args=(r, a.parts, port, a.scale, a.samples, a.cpu_peers)) for r in range(a.parts)]
    for p in procs:
        p.start()
    rc = 0
    for p in procs:
        p.join()
        rc = rc or p.exitcode
    sys.exit(rc)


if __name__ == "__main__":
    main()
