"""Benchmark: GCNConv F=256 aggregation (PyG 1.4.3 propagate, fused on MI355X).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload rmat21|products]
    torchrun --nproc-per-node N bench.py --gpus N ...     (driver, N > 1)

--gpus N > 1 without a launcher (RANK unset): bench.py starts the N rank
processes itself -- a `python -m torch.distributed.run` child, started before
this process touches the GPU, whose exit code it returns -- the way the
reference's own multi-GPU entry takes --gpus directly
(/root/reference/ConvexPruning.py:613).  Every rank checks that the job has
exactly N ranks and exits non-zero otherwise; the process group has an
explicit collective timeout, and each rank logs its stages to stderr.

Workloads (one GCNConv propagate per step, F = 256, fp32):
  rmat21   (default; BASELINE.json configs[1]) RMAT scale 21 (N = 2,097,152),
           (a,b,c,d) = (.57,.19,.19,.05), 30M samples symmetrised (E = 60M),
           add_remaining_self_loops (E' = 62,094,512), x ~ N(0,1), seed 1.
  products (BASELINE.json configs[4], the 8 x MI355X configuration)
           ogbn-products scale power-law graph, N = 2,449,029,
           E = 123,718,280 (E' = 126,163,923), x ~ N(0,1), seed 4.
  reddit   (BASELINE.json configs[3], one GPU) Reddit-scale power-law graph,
           N = 232,965, E = 114,615,892, seed 3, F = 256: one step = the fused
           segmented max + int64 first-index argmax (+ PyG's -10000 mask) over
           every edge -- metric: edges aggregated/s with argmax.
  gat      (BASELINE.json configs[2]) the rmat21 graph, GATConv 8 heads x 32:
           one step = the fused node scores + leaky_relu + softmax + aggregate +
           bias (mp_gat_forward_f32); N > 1: the X W halo rows over the pull
           plan, then the fused kernels on the rank's local graph
           (ShardedGraph.gat_propagate) -- metric: GAT edges/s.
One step = the fused gather * norm -> segment-sum + bias HIP kernel (plus its
split-row fix-up) over all E' edges.  The CSR / schedule / norm build
(one-time, cached=True semantics) and the x @ W GEMM are timed separately and
reported beside the metric.

N > 1: the graph is sharded by destination range (edge balanced), built from
per-rank slices of the edge list (ShardedGraph.for_gcn_from_slices: no rank
holds the whole list); a step is the halo all_to_all (RCCL) overlapped with
the interior edges, then the boundary edges, on every rank.  The exchange is
the hybrid cover (dist.HaloCover: a remote source row is pulled, or its owner
pushes a partial row of the destination, whichever covers the cross edges
with fewer rows); --no-halo-cover pulls every remote source.  value = E' /
max-over-ranks step time (strong scaling).  extra.per_rank carries each
rank's halo bytes, the interior / exposed-exchange / boundary split of its
timed steps, and the same step taken apart after the timed region: the
exchange alone, the compute alone and the exchange-then-compute step.

Prints ONE JSON line on rank 0.
"""
import argparse
import datetime
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402

F_DIM = 256
# step forms the N>1 warm-up times (--halo-tile -1), each with the interior pass after
# and beside the send packing (split_interior): (tile width, boundary as ONE launch after
# the last tile arrives).  One launch per pass is the compute-bound P = 8 form; tiles whose
# boundary pass runs per tile as it arrives pipeline the link-bound P = 2 chain
# pack + exchange + boundary_last
# (tile width, boundary in one launch, send rows packed per tile)
GAT_DROP_SEED = 1234          # --gat-dropout's key
HALO_FORMS = ((256, True, False), (128, True, False), (128, False, False), (64, False, False),
              (128, True, True), (128, False, True), (64, False, True))
HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md chip table)
# SURVEY 8(d) / BASELINE.md section 2 algorithmic bytes: every gathered x_j row
# counted at full size, no cache-reuse credit.  Reported, but its ratio to the
# peak is NOT a roofline fraction (hub rows are re-served from L2 / Infinity
# Cache, so it can exceed 1).
BYTES_PER_EDGE = 4 * F_DIM + 4 + 4   # x_j row + col + norm
BYTES_PER_NODE = 4 * F_DIM + 4       # out row + rowptr
COLLECTIVE_TIMEOUT_S = 300
COMM_INIT_S = [None]     # the process group's first collectives (setup_dist), seconds
T_START = time.perf_counter()


def _rmat21(dev):
    from mi355_mp.graphgen import rmat_edge_index
    return rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)


def _products(dev):
    from mi355_mp.graphgen import powerlaw_edge_index
    return powerlaw_edge_index(2_449_029, 123_718_280, seed=4, device=dev)


def _reddit(dev):
    from mi355_mp.graphgen import powerlaw_edge_index
    return powerlaw_edge_index(232_965, 114_615_892, seed=3, device=dev)


WORKLOADS = {
    "gat": {"name": "rmat21_gat_h8c32", "num_nodes": 1 << 21, "seed": 2, "gen": _rmat21,
            "baseline_config": 3,
            "graph": "RMAT scale 21 (.57,.19,.19,.05) 30M samples symmetrised + remove/add self loops (GATConv)"},
    "rmat21": {"name": "rmat21_gcn_f256", "num_nodes": 1 << 21, "seed": 1, "gen": _rmat21,
               "baseline_config": 2,
               "graph": "RMAT scale 21 (.57,.19,.19,.05) 30M samples symmetrised + add_remaining_self_loops"},
    "reddit": {"name": "reddit_max_f256", "num_nodes": 232_965, "seed": 3, "gen": _reddit,
               "baseline_config": 4,
               "graph": "Reddit-scale power-law (RMAT into [0, N)), 114,615,892 directed edges, aggr='max' + "
                        "int64 first-index argmax + utils.scatter_'s -10000 mask"},
    "products": {"name": "products_gcn_f256", "num_nodes": 2_449_029, "seed": 4, "gen": _products,
                 "baseline_config": 5,
                 "graph": "ogbn-products-scale power-law (RMAT into [0, N)), 123,718,280 directed edges "
                          "+ add_remaining_self_loops"},
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="rmat21")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ref-paths", action="store_true",
                    help="skip timing the reference's ATen device path and the vendor SpMM")
    ap.add_argument("--verify", action="store_true",
                    help="after the timed region, hold every output row to |out - ref| <= 1e-5 * max(1, "
                         "sum|w x_j|) against a float64 reference over the rank's own edges")
    ap.add_argument("--cpu-sample-edges", type=int, default=48_000_000)
    ap.add_argument("--chunk", type=int, default=0, help="merge-path task size (0: auto_chunk)")
    ap.add_argument("--no-overlap", action="store_true", help="N>1: exchange, then aggregate (no overlap)")
    ap.add_argument("--no-halo-cover", action="store_true",
                    help="N>1: pull exchange (every remote source row) instead of the hybrid pull / push "
                         "cover (dist.HaloCover)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the N>1 sharded path (shards, plans, halo exchange, per-rank split) even at "
                         "one rank -- under torch.distributed.run --nproc-per-node 1 it rehearses the "
                         "driver's multi-GPU code path on the RCCL backend with empty halos")
    ap.add_argument("--emulate-peers", type=str, default="", metavar="P[,P..]",
                    help="with --sharded at one rank (RCCL): also measure RCCL beside the aggregation -- rank 0 "
                         "of a P-way partition of the graph aggregates its in-edges while a world-1 "
                         "all_to_all_single moves that rank's halo volume as a self split (extra.per_rank[0]"
                         ".rccl_contention: exchange alone, compute alone, overlapped, hidden_frac)")
    ap.add_argument("--no-build-split", action="store_true",
                    help="N>1: do not take the one-time build apart into device-busy and host time")
    ap.add_argument("--halo-tile", type=int, default=-1,
                    help="N>1: exchange feature tiles of this width (64 / 128 / 256; 256 = whole rows), the "
                         "boundary pass as one launch (see --boundary-per-tile); 0 = the unfused step of "
                         "[own ; halo] rows; -1 (default) = the form chosen in the warm-up among HALO_FORMS "
                         "by timing each on this job's links (max over ranks)")
    ap.add_argument("--boundary-per-tile", action="store_true",
                    help="with --halo-tile W: the boundary pass per tile as its halo arrives")
    ap.add_argument("--gat-dropout", type=float, default=0.0,
                    help="--workload gat: GATConv's training-mode attention dropout p in every step")
    ap.add_argument("--pack-per-tile", action="store_true",
                    help="with --halo-tile W: the send rows packed per tile, each tile's exchange started "
                         "right after its packing")
    return ap.parse_args(argv)


_LAST_STAGE = ["start"]
_JSON_OUT = []


def claim_stdout():
    """Keep file descriptor 1 for the one JSON line: everything else this
    process writes to stdout -- Python prints and native libraries alike (RCCL
    prints a version banner on every rank, gloo its connection lines) -- goes
    to stderr from here on."""
    if not _JSON_OUT:
        sys.stdout.flush()
        _JSON_OUT.append(os.fdopen(os.dup(1), "w"))
        os.dup2(2, 1)


def emit(obj):
    """The JSON line, alone on the real stdout."""
    out = _JSON_OUT[0] if _JSON_OUT else sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def stage(rank, msg):
    """One progress line per stage on stderr (the JSON line stays alone on stdout)."""
    _LAST_STAGE[0] = msg[:80]
    print("[bench rank %s +%.1fs] %s" % (rank, time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


def start_heartbeat(rank, every_s=60.0):
    """Rank 0 prints one line a minute while it runs (a daemon thread): a long
    one-time build still shows progress to whoever watches the log."""
    import threading
    if rank != 0:
        return

    def beat():
        while True:
            time.sleep(every_s)
            print("[bench rank %s +%.1fs] running; last stage: %s" % (rank, time.perf_counter() - T_START,
                                                                       _LAST_STAGE[0]), file=sys.stderr, flush=True)
    threading.Thread(target=beat, name="bench-heartbeat", daemon=True).start()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """--gpus N > 1 and no launcher: run N ranks under a torch.distributed.run
    CHILD process (this process has not touched the GPU, and is not replaced:
    it waits and returns the child's exit code; a failing rank makes
    torch.distributed.run stop the others and exit non-zero)."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    stage("-", "no launcher for --gpus %d: starting %d ranks (torch.distributed.run, port %d)"
          % (args.gpus, args.gpus, port))
    return subprocess.call(cmd, env=env, cwd=ROOT)


def setup_dist(args):
    """(rank, world, local device index).  Single process unless launched as
    ranks (RANK set) -- then the job must have exactly --gpus ranks."""
    if "RANK" not in os.environ:
        if args.sharded and args.gpus == 1:
            # one rank of the sharded path with no launcher: this process is the
            # whole job (a world-1 process group over 127.0.0.1), so it can run
            # directly under rocprofv3
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(_free_port()))
        elif args.sharded:
            raise SystemExit("bench.py --sharded with --gpus > 1 needs a launcher (torch.distributed.run)")
        else:
            return 0, 1, 0
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if world != args.gpus:
        stage(rank, "ERROR: the job has %d ranks but --gpus %d" % (world, args.gpus))
        raise SystemExit(3)
    timeout = datetime.timedelta(seconds=COLLECTIVE_TIMEOUT_S)
    if os.environ.get("MP_BENCH_LAUNCH_PROBE"):
        # CPU test of the launch path (tests/test_host.py): the ranks meet over
        # gloo without touching a GPU, report themselves and stop
        dist.init_process_group("gloo", timeout=timeout)
        ok = dist.get_world_size() == args.gpus
        got = [None] * dist.get_world_size()
        dist.all_gather_object(got, {"rank": rank, "local_rank": local, "world": dist.get_world_size()})
        stage(rank, "launch probe: %s" % got[rank])
        if rank == 0:
            emit({"launch_probe": got, "gpus": args.gpus})
        dist.destroy_process_group()
        raise SystemExit(0 if ok else 3)
    if world == 1 and not args.sharded:
        return 0, 1, local
    backend = os.environ.get("MP_BENCH_BACKEND", "nccl")
    # the node's host threads are shared by its ranks: each rank's intra-op pool
    # gets its share of OMP_NUM_THREADS (eight ranks x 16 spinning OpenMP threads
    # on a 16-thread share stalled the shared-GPU rehearsal's builds)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    if local_world > 1:
        share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        torch.set_num_threads(max(1, share // local_world))
    if backend == "gloo":
        # rehearsal of the multi-GPU path on a box with fewer GPUs than ranks:
        # ranks share devices, halo rows are staged through the host
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group("gloo", timeout=timeout)
    else:
        n_dev = torch.cuda.device_count()
        if local >= n_dev:
            stage(rank, "ERROR: local rank %d but only %d visible GPUs (RCCL ranks cannot share a device)"
                  % (local, n_dev))
            raise SystemExit(3)
        torch.cuda.set_device(local)
        # RCCL on high-priority streams: HIP gives them hardware queues of their own.  With
        # normal priority the communicator's stream is dealt a queue round-robin among
        # GPU_MAX_HW_QUEUES (4) and may share one with the aggregation's stream -- measured
        # at one RCCL rank: an all_to_all on the default stream's queue never ran beside the
        # aggregation (hidden_frac -0.03), on a queue of its own it hid half the exchange
        # (0.58; profiles/r05_queue_probe.jsonl).  Priority also lets RCCL's few blocks
        # start before the aggregation's waves.
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout, pg_options=opts)
    if dist.get_world_size() != args.gpus:
        stage(rank, "ERROR: process group has %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus))
        raise SystemExit(3)
    # the communicator is set up here, before the one-time build (whose split
    # would otherwise charge its creation to the first collective it makes):
    # one all_reduce, all_gather and all_to_all of a few bytes on every rank
    t0 = time.perf_counter()
    dev = torch.device("cuda", local) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.ones(world, dtype=torch.int64, device=dev)
    dist.all_reduce(t)
    g = torch.empty(world * world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(g, t)
    r = torch.empty_like(t)
    dist.all_to_all_single(r, t)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    COMM_INIT_S[0] = time.perf_counter() - t0
    stage(rank, "process group up: backend %s, world %d, device cuda:%d (communicator set up in %.2f s)"
          % (dist.get_backend(), world, local, COMM_INIT_S[0]))
    return rank, world, local


def barrier(world):
    if world > 1 or dist.is_initialized():
        dist.barrier()


def cpu_info():
    """(CPU model, threads available to this process).  The thread count is the
    affinity mask, capped by a cgroup CPU quota when one is set: on the GPU box
    os.cpu_count() reports the whole machine while the job gets a share of it,
    and more threads than that share would only oversubscribe it."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = max(1, min(n, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return model, n, os.cpu_count() or 1


def cpu_baseline(ei_loops, norm, x, sample_edges):
    """The reference algorithm on the host (oracle, kind 'port'): index_select
    -> norm * x_j -> scatter_add_ (torch_scatter scatter_sum), timed on a
    bounded sample of the same edges in their original order, in 4M-edge
    chunks (the materialised x_j of all edges is 64-130 GB)."""
    from oracle import pyg_ref  # noqa: F401  (checker/baseline only)
    model, threads, machine = cpu_info()
    torch.set_num_threads(threads)
    E = min(sample_edges, ei_loops.shape[1])
    ei = ei_loops[:, :E].cpu()
    w = norm[:E].cpu()
    xc = x.cpu()
    out = torch.zeros_like(xc)
    chunk = 4_000_000
    t0 = time.perf_counter()
    for s in range(0, E, chunk):
        e = min(E, s + chunk)
        x_j = xc.index_select(0, ei[0, s:e])
        msg = w[s:e].view(-1, 1) * x_j
        out.scatter_add_(0, ei[1, s:e].view(-1, 1).expand_as(msg), msg)
    dt = time.perf_counter() - t0
    del out, xc
    return {"value": E / dt, "unit": "edges/s", "cores": threads, "kind": "port",
            "cpu_model": model, "machine_cpus": machine,
            "sample": "first %d of the %d edges (original order), F=%d, torch CPU index_select+mul+"
                      "scatter_add_ in 4M-edge chunks, %d threads (the CPUs this job may use; the machine "
                      "has %d), %.1f s" % (E, ei_loops.shape[1], F_DIM, threads, machine, dt)}


def _ev_ms(fn, reps):
    """Average ms of fn() over `reps` runs, HIP events on the current stream
    (one warm-up run first)."""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def device_reference_paths(ei, norm, x, csr, w_csr, bias, fused_out, terms, reps=3):
    """The same GCNConv propagate + bias on the same MI355X by two other routes,
    timed beside the fused kernel and checked against its output:

      reference_path: what the reference runs on a GPU (examples/gcn.py:31-32
        moves the model and data to CUDA): PyG 1.4.3 __collect__'s
        x.index_select(0, edge_index[0]) -> GCNConv.message norm.view(-1, 1) * x_j
        -> torch_scatter 2.0.4 scatter_sum = zeros.scatter_add_(0, broadcast
        index, msg) (ATen atomics) -> update + bias.  The [E', 256] x_j and
        message tensors are materialised at full size (63.6 GB each on rmat21).
      vendor_spmm: torch.sparse_csr_tensor(rowptr, col, norm) @ x on the same
        CSR and weights (rocSPARSE / hipSPARSE SpMM) + bias.

    Each output is compared with the fused kernel's: within
    1e-5 * max(1, sum_e |w_e x_j|) (terms), plus the bitwise-equal fraction."""
    res = {}
    N, F = x.shape
    E = ei.shape[1]

    def check(out):
        d = (out - fused_out).abs()
        excess = float((d - 1e-5 * terms.clamp(min=1.0)).max())
        return {"max_abs_diff": float(d.max()), "bound_excess": excess, "within_1e-5_bound": excess <= 0,
                "bitwise_equal_frac": float((out == fused_out).float().mean())}
    try:
        idx = ei[1].view(-1, 1).expand(E, F)
        bufs = {}

        # (each piece frees its previous output first: x_j and msg are 63.6 GB apiece)
        def gather():
            bufs.pop("x_j", None)
            bufs["x_j"] = x.index_select(0, ei[0])

        def message():
            bufs.pop("msg", None)
            bufs["msg"] = norm.view(-1, 1) * bufs["x_j"]

        def scatter():
            bufs.pop("out", None)
            bufs["out"] = torch.zeros(N, F, device=x.device).scatter_add_(0, idx, bufs["msg"]) + bias

        def whole():
            bufs.clear()
            gather()
            message()
            scatter()
        ms = _ev_ms(whole, reps)
        piece = {"index_select_ms": _ev_ms(gather, reps), "mul_ms": _ev_ms(message, reps),
                 "scatter_add_plus_bias_ms": _ev_ms(scatter, reps)}
        res["reference_path"] = dict(ms=ms, **piece, **check(bufs["out"]),
                                     desc="ATen index_select -> norm*x_j -> zeros.scatter_add_ -> +bias, fp32, "
                                          "full size (x_j and msg materialised)")
        bufs.clear()
        del idx
    except RuntimeError as exc:   # e.g. out of memory on a smaller part
        res["reference_path"] = {"error": str(exc)[:200]}
    torch.cuda.empty_cache()
    try:
        A = torch.sparse_csr_tensor(csr.rowptr, csr.col[:csr.n_edges], w_csr[:csr.n_edges], size=(N, N))
        box = {}

        def spmm():
            box["out"] = torch.mm(A, x) + bias
        ms = _ev_ms(spmm, reps)
        res["vendor_spmm"] = dict(ms=ms, **check(box["out"]),
                                  desc="torch.sparse_csr_tensor(rowptr, col, norm; int32 indices) @ x "
                                       "(rocSPARSE/hipSPARSE SpMM) + bias")
        del A, box
    except RuntimeError as exc:
        res["vendor_spmm"] = {"error": str(exc)[:200]}
    torch.cuda.empty_cache()
    return res


def verify_f64(out, x_src, src, dst, w, bias, step=4_000_000):
    """|out - ref| <= 1e-5 * max(1, sum|w x_j|) per element, ref = a float64
    index_add of w_e x[src_e] (+ bias) over the given edges in edge chunks (the
    whole [E, F] message tensor does not fit).  Returns a small report."""
    n, F = out.shape
    ref = torch.zeros(n, F, device=out.device, dtype=torch.float64)
    terms = torch.zeros(n, F, device=out.device, dtype=torch.float64)
    for s in range(0, src.numel(), step):
        msg = w[s:s + step].double().view(-1, 1) * x_src[src[s:s + step]].double()
        ref.index_add_(0, dst[s:s + step], msg)
        terms.index_add_(0, dst[s:s + step], msg.abs())
        del msg
    if bias is not None:
        ref += bias.double()
    excess = float(((out.double() - ref).abs() - 1e-5 * terms.clamp(min=1.0)).max()) if n else -1.0
    res = {"rows": n, "edges": int(src.numel()), "max_abs_diff": float((out.double() - ref).abs().max()) if n else 0.0,
           "bound_excess": excess, "within_1e-5_bound": excess <= 0,
           "reference": "float64 index_add of w * x_j over the same edges (+ bias)"}
    del ref, terms
    torch.cuda.empty_cache()
    return res


def find_pmc(workload, kernel, src_hash, full=False):
    """The newest committed PMC summary (profiles/r*_pmc_traffic*.json) of THIS
    build's dispatched kernel on this workload: (hbm bytes per launch, path)
    (+ the summary itself with full=True).  kernel=None: the summary's own
    dominant kernel (the GAT workload, whose dispatch has no name query)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic*.json")), reverse=True):
        try:
            with open(path) as f:
                pmc = json.load(f)
        except (OSError, ValueError):
            continue
        if (pmc.get("workload") == workload and kernel in (None, pmc.get("kernel"))
                and pmc.get("source_hash") == src_hash):
            res = (pmc.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT))
            return res + (pmc,) if full else res
    res = (None, "no committed profile of this build's kernel on %s" % workload)
    return res + (None,) if full else res


def cpu_gat_baseline(ei, xw, att, H, C, sample):
    """GATConv's reference pipeline after x @ W on the host (oracle, kind
    'port'): x_i / x_j index_select, (cat[x_i, x_j] * att).sum(-1), leaky_relu,
    utils.softmax (serial scatter_max loop + scatter_add_), x_j * alpha,
    scatter_add_ -- on the first `sample` edges."""
    import torch.nn.functional as Fn
    from oracle import pyg_ref as P, scatter_ref as S  # checker/baseline only
    model, threads, machine = cpu_info()
    torch.set_num_threads(threads)
    E = min(sample, ei.shape[1])
    eic, h, a = ei[:, :E].cpu(), xw.cpu(), att.cpu()
    N = h.shape[0]
    t0 = time.perf_counter()
    x_i = h.index_select(0, eic[1]).view(-1, H, C)
    x_j = h.index_select(0, eic[0]).view(-1, H, C)
    alpha = Fn.leaky_relu((torch.cat([x_i, x_j], dim=-1) * a).sum(dim=-1), 0.2)
    alpha = P.softmax(alpha, eic[1], N)
    out = S.scatter_sum(x_j * alpha.view(-1, H, 1), eic[1], N)
    dt = time.perf_counter() - t0
    del out, x_i, x_j
    return {"value": E / dt, "unit": "edges/s", "cores": threads, "kind": "port", "cpu_model": model,
            "machine_cpus": machine, "sample": "first %d of %d edges, oracle GATConv pipeline (torch CPU ops + "
            "serial scatter_max loop in the softmax), %d threads, %.1f s" % (E, ei.shape[1], threads, dt)}


def main_gat(args, rank, world, local):
    """--workload gat: BASELINE config 3 (GATConv 8 heads x 32 on the rmat21
    graph), one step = one fused GAT propagate over all E' edges (N = 1), or
    per rank the pull exchange of the X W halo rows then the fused kernels on
    the rank's local graph (N > 1)."""
    from mi355_mp import ops
    from mi355_mp.graph import GAT_TARGET_TASKS, Graph
    from torch_geometric.nn.conv._structure import gat_loops
    import mi355_mp
    mi355_mp.load_native()
    wl = WORKLOADS["gat"]
    sharded = dist.is_initialized()
    dev = torch.device("cuda", local)
    N, H, C = wl["num_nodes"], 8, 32
    F = H * C
    # --gat-dropout p: GATConv's training-mode attention dropout in every step (one
    # fixed key, so --verify can apply the same keep mask in float64)
    drop_p = float(args.gat_dropout)
    t0 = time.perf_counter()
    ei = wl["gen"](dev)
    g = torch.Generator(device=dev).manual_seed(wl["seed"])
    xw_full = torch.randn(N, F, device=dev, generator=g)
    att = torch.randn(1, H, 2 * C, device=dev, generator=g) * 0.1
    bias = torch.randn(F, device=dev, generator=g) * 0.1
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    stage(rank, "gat graph generated (%.1f s)" % t_gen)
    t0 = time.perf_counter()
    if not sharded:
        ei2 = gat_loops(ei, N)
        del ei
        graph = Graph(ei2, N, N, target_tasks=GAT_TARGET_TASKS)     # as GATConv builds it
        graph.dst                                                     # the one-time build
        E2 = E_local = ei2.shape[1]
        xw = xw_full
        n_rows, n_src = N, N

        def step():
            return ops.gat_propagate(graph, ei2, xw, att, H, C, 0.2, bias, dropout=drop_p, seed=GAT_DROP_SEED)[0]
    else:
        from mi355_mp import dist as mdist
        E_raw = ei.shape[1]
        s0, s1 = rank * E_raw // world, (rank + 1) * E_raw // world
        sg = mdist.ShardedGraph.for_gat_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
        del ei
        E2, E_local = sg.n_edges, int(sg.fwd.edge_pos.numel())
        xw = xw_full[sg.lo:sg.hi].contiguous()
        n_rows, n_src = sg.n_own, sg.fwd.n_local_src
        cover_stats = None
        if not args.no_halo_cover:
            # the hybrid cover: a remote source row is pulled, or its owner pushes its
            # online-softmax piece of the destination row (mi355_mp.gat_cover)
            sg.enable_gat_halo_cover()
            sg.gat_cover.graphs()                                     # the one-time build
            cover_stats = sg.gat_cover.stats()
        else:
            sg.g_fwd.dst                                              # the one-time build
        stage(rank, "gat shards built: %d rows, %d in-edges, %d pull-halo rows%s"
              % (n_rows, E_local, n_src - n_rows, "" if cover_stats is None else
                 ", cover: %d rows in (%d pulled + %d pieces)" % (cover_stats["halo_rows"],
                                                                  cover_stats["cover_pulled_rows"],
                                                                  cover_stats["cover_partial_rows"])))

        def step():
            return sg.gat_propagate(xw, att, H, C, 0.2, bias, dropout=drop_p, seed=GAT_DROP_SEED)[0]
    del xw_full
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        barrier(world)
        stage(rank, "warm-up done (%d steps)" % args.warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        dt_local = dt = time.perf_counter() - t0
        if sharded:
            tt = torch.tensor([dt], dtype=torch.float64)
            tt = tt.to(dev) if dist.get_backend() == "nccl" else tt
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        stage(rank, "timed steps done: %.3f ms/step (max over ranks)" % (dt / args.steps * 1e3))
        # the step's kernel time on this rank (HIP events over back-to-back steps; N > 1:
        # the exchange alone and the local fused kernels alone, in the same process)
        reps = max(args.steps, 10)
        split = {}
        if sharded:
            xl = mdist.halo_rows(xw, sg.fwd, sg.group)      # pull halo: the verify reference's inputs
            if cover_stats is not None:
                split = sg.gat_cover.decompose(xw, att, H, C, 0.2, bias, reps, barrier=lambda: barrier(world))
            else:
                def exchange():
                    mdist.halo_rows(xw, sg.fwd, sg.group)

                def local():
                    ops.gat_propagate(sg.g_fwd, sg.fwd.local_edge_index, xl, att, H, C, 0.2, bias)
                for name, fn in (("exchange_only_ms", exchange), ("compute_only_ms", local)):
                    barrier(world)
                    torch.cuda.synchronize()
                    t1 = time.perf_counter()
                    for _ in range(reps):
                        fn()
                    torch.cuda.synchronize()
                    split[name] = (time.perf_counter() - t1) / reps * 1e3
            kern_ms = split["compute_only_ms"]
        else:
            kern_ms = _ev_ms(step, reps)
        verify = None
        if args.verify:
            # alpha (by global edge id) and the rows against the single-GPU fused kernel's
            # formula in float64 over this rank's edges (edge chunks)
            ei_l = sg.fwd.local_edge_index if sharded else ei2
            xs = xl if sharded else xw
            src, dst = ei_l[0], ei_l[1]
            x3 = xs.view(-1, H, C).double()
            a_dst = (x3 * att[:, :, :C].double()).sum(-1)
            a_src = (x3 * att[:, :, C:].double()).sum(-1)
            del x3
            keep = None
            if drop_p > 0:       # the kernels' keep mask of these edges (global edge ids on a shard)
                keep = ops.gat_dropout_keep(sg.g_fwd if sharded else graph, GAT_DROP_SEED, drop_p, H).double() \
                    / (1.0 - drop_p)
            m = torch.full((n_rows, H), float("-inf"), device=dev, dtype=torch.float64)
            den = torch.zeros(n_rows, H, device=dev, dtype=torch.float64)
            ref = torch.zeros(n_rows, H, C, device=dev, dtype=torch.float64)
            terms = torch.zeros_like(ref)
            step_e = 4_000_000
            for pss in range(3):
                for s in range(0, src.numel(), step_e):
                    sl = slice(s, s + step_e)
                    sc = torch.nn.functional.leaky_relu(a_dst[dst[sl]] + a_src[src[sl]], 0.2)
                    if pss == 0:
                        m.scatter_reduce_(0, dst[sl].view(-1, 1).expand(-1, H), sc, "amax")
                    elif pss == 1:
                        den.index_add_(0, dst[sl], torch.exp(sc - m[dst[sl]]))
                    else:
                        a = torch.exp(sc - m[dst[sl]]) / (den[dst[sl]] + 1e-16)
                        if keep is not None:
                            a = a * keep[sl]
                        msg = a.unsqueeze(-1) * xs.view(-1, H, C)[src[sl]].double()
                        ref.index_add_(0, dst[sl], msg)
                        terms.index_add_(0, dst[sl], msg.abs())
                        del msg
            ref = ref.view(n_rows, F) + bias.double()
            excess = float(((out.double() - ref).abs() - 1e-5 * terms.view(n_rows, F).clamp(min=1.0)).max())
            verify = {"rows": n_rows, "edges": int(src.numel()), "bound_excess": excess,
                      "within_1e-5_bound": excess <= 0,
                      "reference": "float64 GATConv formula over the rank's edges (edge chunks)"}
            del ref, terms
            stage(rank, "verify: %s" % json.dumps(verify))
    comp = n_src * F * 4 + n_rows * F * 4 + E_local * 4 + (n_rows + 1) * 4
    # counter traffic of the fused GAT kernel from a committed profile of this build
    # (tools/profile.sh with BENCH_ARGS="--workload gat"), per launch of its main kernel
    src_hash = mi355_mp.load_native().mp_source_hash().decode()
    traffic, traffic_src, pmc = (None, "N>1: per-rank graphs are not profiled", None) if sharded else \
        find_pmc(wl["name"], None, src_hash, full=True)
    ranks = None
    if sharded:
        if cover_stats is None:
            mine = {"rank": rank, "rows": n_rows, "edges": E_local, "exchange": "pull", "halo_rows": n_src - n_rows,
                    "halo_bytes_in": (n_src - n_rows) * F * 4,
                    "halo_bytes_out": int(sg.fwd.send_idx.numel()) * F * 4}
        else:
            gc = sg.gat_cover
            mine = {"rank": rank, "rows": n_rows, "edges": E_local,
                    "exchange": "cover (pulled rows + pushed online-softmax pieces)",
                    "halo_rows": gc.n_halo, "pull_halo_rows": n_src - n_rows,
                    "cover_over_pull_rows": gc.n_halo / max(1, n_src - n_rows),
                    "halo_bytes_in": gc.n_halo * (F + 2 * H) * 4 + sum(gc.adst_send_counts) * H * 4,
                    "halo_bytes_out": gc.n_send * (F + 2 * H) * 4 + sum(gc.adst_recv_counts) * H * 4,
                    "peers_in": list(gc.recv_counts), "peers_out": list(gc.send_counts), **cover_stats}
        mine.update({"step_ms_this_rank": dt_local / args.steps * 1e3, **split, "verify": verify})
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        if verify is not None:
            verify = {"all_ranks_within_1e-5_bound": all(r["verify"]["within_1e-5_bound"] for r in ranks),
                      "max_bound_excess": max(r["verify"]["bound_excess"] for r in ranks)}
    cpu = None
    if rank == 0 and not sharded and not args.no_cpu_baseline:
        cpu = cpu_gat_baseline(ei2, xw, att, H, C, 3_000_000)
    if rank == 0:
        line = {
            "metric": "edges aggregated/sec (GATConv 8x32 propagate: fused node scores + leaky_relu + "
                      "softmax(+1e-16) + aggregate + bias)",
            "value": E2 * args.steps / dt, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic rmat21 graph (seeded, generated on device), random X W / att / bias",
            "config": {"workload": wl["name"], "baseline_config": wl["baseline_config"], "graph": wl["graph"],
                       "num_nodes": N, "num_edges": E2, "heads": H, "out_channels": C, "seed": wl["seed"],
                       "attention_dropout": drop_p,
                       "parallelism": ("dst-range shards x%d, RCCL halo all_to_all (%s)"
                                       % (world, "pull" if args.no_halo_cover else "hybrid cover")) if sharded
                       else "single GPU"},
            "roofline": {"bound": "hbm", "achieved": comp / (kern_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": comp / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_frac": (traffic / (pmc["kernel_trace_avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS)
                         if traffic else None,
                         "traffic_source": traffic_src, "kernel": pmc["kernel"] if pmc else None,
                         "kernel_trace_avg_ms": pmc["kernel_trace_avg_ms"] if pmc else None,
                         "source_hash": src_hash,
                         "bytes": "compulsory: xw rows read once, out written once, col + rowptr",
                         "compulsory_bytes_per_step": comp, "kernel_ms": kern_ms,
                         "algorithmic_bytes_per_step": E_local * (4 * F + 4 + 4 * H) + n_rows * (4 * F + 4 * H + 4)},
            "cpu_baseline": cpu,
            "extra": {"one_time_build_s": t_build, "graph_gen_s": t_gen, "per_rank": ranks, "verify": verify,
                      "collective_timeout_s": COLLECTIVE_TIMEOUT_S if sharded else None},
        }
        emit(line)
    stage(rank, "done")
    if dist.is_initialized():
        dist.destroy_process_group()


def cpu_max_baseline(ei, x, sample):
    """max + argmax on the host (oracle, kind 'port'): torch index_select, then
    torch_scatter 2.0.4's serial CPU scatter_max loop (scatter_cpu.cpp, restated
    in oracle/scatter_loop.c), on the first `sample` edges in 4M-edge chunks
    accumulated through `out` (the loop's has_out path)."""
    from oracle import scatter_ref as S  # checker/baseline only
    model, threads, machine = cpu_info()
    torch.set_num_threads(threads)
    E = min(sample, ei.shape[1])
    eic, xc = ei[:, :E].cpu(), x.cpu()
    N, F = xc.shape
    out = torch.full((N, F), -3.4028234663852886e38)
    t0 = time.perf_counter()
    for s0 in range(0, E, 4_000_000):
        e1 = min(E, s0 + 4_000_000)
        msg = xc.index_select(0, eic[0, s0:e1])
        out, _ = S.scatter_loop(msg, eic[1, s0:e1], N, "max", out=out)
    dt = time.perf_counter() - t0
    return {"value": E / dt, "unit": "edges/s", "cores": threads, "kind": "port", "cpu_model": model,
            "machine_cpus": machine,
            "sample": "first %d of %d edges: torch index_select (%d threads) + the serial scatter_max loop "
                      "(1 thread, oracle/scatter_loop.c), %.1f s" % (E, ei.shape[1], threads, dt)}


def verify_max(out, arg, x, src, dst, step=2_000_000):
    """Exact check of a max + first-index argmax aggregation: the max by
    torch's scatter_reduce('amax') and the arg as the smallest edge id whose
    message equals it (scatter_reduce('amin') over edge ids), in edge chunks;
    empty rows (0, E); the PyG -10000 mask.  Bitwise, values and args."""
    n, F = out.shape
    E = src.numel()
    ref = torch.full((n, F), float("-inf"), device=out.device)
    for s in range(0, E, step):
        ref.scatter_reduce_(0, dst[s:s + step].view(-1, 1).expand(-1, F), x[src[s:s + step]], "amax")
    ids = torch.full((n, F), E, dtype=torch.int64, device=out.device)
    for s in range(0, E, step):
        d = dst[s:s + step]
        hit = x[src[s:s + step]] == ref[d]
        cand = torch.where(hit, torch.arange(s, s + d.numel(), device=out.device).view(-1, 1), E)
        ids.scatter_reduce_(0, d.view(-1, 1).expand(-1, F), cand, "amin")
    ref = torch.where(torch.isinf(ref) | (ref < -10000), torch.zeros_like(ref), ref)
    return {"rows": n, "edges": E, "values_bitwise_equal": bool(torch.equal(out, ref)),
            "args_bitwise_equal": bool(torch.equal(arg, ids)),
            "reference": "torch scatter_reduce amax + smallest edge id attaining it (amin), edge chunks"}


def main_reddit(args, rank, world, local):
    """--workload reddit: BASELINE config 4 (one GPU), aggr='max' with int64
    first-index argmax and PyG's -10000 mask over every edge of the
    Reddit-scale graph; one step = the fused main launch + its fix-up."""
    import mi355_mp
    from mi355_mp import _lib, ops
    from mi355_mp.graph import Graph
    wl = WORKLOADS["reddit"]
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    lib = mi355_mp.load_native()
    N, F = wl["num_nodes"], F_DIM
    t0 = time.perf_counter()
    ei = wl["gen"](dev)
    x = torch.randn(N, F, device=dev, generator=torch.Generator(device=dev).manual_seed(wl["seed"]))
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    stage(rank, "reddit graph generated (%.1f s)" % t_gen)
    t0 = time.perf_counter()
    graph = Graph(ei, N, N)
    csr = graph.dst
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    E = csr.n_edges
    out = torch.empty(N, F, device=dev)
    arg = torch.empty(N, F, dtype=torch.int64, device=dev)
    st_main = csr.struct("other")
    slab = torch.empty(lib.mp_aggregate_slab_bytes(st_main, F, _lib.MP_REDUCE["max"]), dtype=torch.uint8, device=dev)

    def aggregate(stages):
        # stage by stage: every edge is gathered (the one-off form of a layer's
        # first two calls; ops' first-occurrence CSR engages from the third)
        ops._aggregate(csr, "other", x, None, "max", _lib.MP_FLAG_PYG_MASK, None, out=out, stages=stages,
                       slab=slab, arg=arg)

    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    for _ in range(args.warmup):
        aggregate(_lib.MP_STAGE_MAIN)
        aggregate(_lib.MP_STAGE_FIXUP)
    torch.cuda.synchronize()
    stage(rank, "warm-up done (%d steps)" % args.warmup)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record()
        aggregate(_lib.MP_STAGE_MAIN)
        ev[i][1].record()
        aggregate(_lib.MP_STAGE_FIXUP)
        ev[i][2].record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stage(rank, "timed steps done: %.3f ms/step" % (dt / args.steps * 1e3))
    main_ms = sorted(a.elapsed_time(b) for a, b, _ in ev)
    fix_ms = sorted(b.elapsed_time(c) for _, b, c in ev)
    main_avg, fix_avg = sum(main_ms) / len(main_ms), sum(fix_ms) / len(fix_ms)
    verify = verify_max(out, arg, x, ei[0], ei[1]) if args.verify else None
    if verify is not None:
        stage(rank, "verify: %s" % json.dumps(verify))
    kernel = _lib.kernel_name(st_main, None, x.data_ptr(), F, F, "max", None, out.data_ptr(), F, dev)
    src_hash = lib.mp_source_hash().decode()
    traffic, traffic_src = find_pmc(wl["name"], kernel, src_hash)
    # compulsory: x once, col + eid per slot, rowptr, out and the int64 arg once
    comp = N * F * 4 + E * 8 + (N + 1) * 4 + N * F * 12
    alg = E * (4 * F + 4) + N * (4 * F + 8 * F + 4)       # 1028 B/edge + 3076 B/node
    cpu = cpu_max_baseline(ei, x, 12_000_000) if not args.no_cpu_baseline else None
    line = {
        "metric": "edges aggregated/sec (aggr='max' + int64 first-index argmax, PyG -10000 mask, F=256)",
        "value": E * args.steps / dt, "unit": "edges/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic Reddit-scale power-law graph (seeded, generated on device), random features",
        "config": {"workload": wl["name"], "baseline_config": wl["baseline_config"], "graph": wl["graph"],
                   "num_nodes": N, "num_edges": E, "features": F, "seed": wl["seed"], "parallelism": "single GPU",
                   "chunk": csr.chunk},
        "roofline": {"bound": "hbm", "achieved": comp / (main_avg * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": comp / (main_avg * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_frac": (traffic / (main_avg * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                     "traffic_source": traffic_src,
                     "bytes": "achieved = compulsory bytes (x read once, col + eid, rowptr, out and int64 arg "
                              "written once) / avg launch time",
                     "compulsory_bytes_per_launch": comp, "algorithmic_bytes_per_launch": alg,
                     "algorithmic_GBps_no_cache_credit": alg / (main_avg * 1e-3) / 1e9,
                     "kernel": kernel, "source_hash": src_hash, "avg_launch_ms": main_avg,
                     "median_launch_ms": main_ms[len(main_ms) // 2], "fixup_avg_ms": fix_avg,
                     "timing": "HIP events around each main / fix-up launch inside the timed steps"},
        "cpu_baseline": cpu,
        "extra": {"one_time_build_s": t_build, "graph_gen_s": t_gen, "n_split_rows": csr.n_split,
                  "n_wave_tasks": csr.n_waves, "verify": verify,
                  "note": "x is 238 MB: it fits the 256 MB Infinity Cache"},
    }
    emit(line)
    stage(rank, "done")


LINK_GBS = (60.0, 77.0, 100.0)   # xGMI per link direction: low / nominal / high


class BuildMeter:
    """Takes a one-time build phase apart on this rank (N > 1 lines, the
    driver's first 8-GPU run): wall time, the time the device was busy (union
    of the kernel / copy intervals the torch profiler records, device activity
    only), the rest = host work and host-device round trips, and the number of
    synchronising calls (torch's sync debug mode, counted as warnings, with
    the source line of each: sync_sites).  The gloo rehearsal stages every
    all_to_all through host memory: those syncs (mdist._stage_to_host) and the
    host time inside the staged all_to_alls are given apart -- over RCCL
    neither exists.  The profiler's start-up and trace processing lie outside
    the wall time.  enabled=False: wall time only."""

    def __init__(self, enabled):
        self.enabled = enabled
        self.res = {}

    def run(self, name, fn):
        import warnings
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if not self.enabled:
            out = fn()
            torch.cuda.synchronize()
            self.res[name] = {"wall_s": time.perf_counter() - t0}
            return out
        from torch.profiler import ProfilerActivity, profile
        import inspect
        import mi355_mp.dist as mdist
        prof = profile(activities=[ProfilerActivity.CUDA])
        try:
            prof.start()            # the profiler's own start-up is not charged to the phase
        except Exception as ex:  # pragma: no cover - a profiler that cannot start: wall time only
            out = fn()
            torch.cuda.synchronize()
            self.res[name] = {"wall_s": time.perf_counter() - t0, "note": "profiler did not start: %s" % ex}
            return out
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            torch.cuda.synchronize()
            staged0 = mdist.GLOO_STAGED_S[0]
            t0 = time.perf_counter()
            torch.cuda.set_sync_debug_mode("warn")
            try:
                out = fn()
            finally:
                torch.cuda.set_sync_debug_mode("default")    # the phase's end below is not one of its syncs
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0           # before the profiler's stop / trace processing
            prof.stop()
        src, first = inspect.getsourcelines(mdist._stage_to_host)
        stage_lines = set(range(first, first + len(src)))
        sites = {}
        n_stage = 0
        for w in caught:
            if "synchroniz" not in str(w.message).lower():
                continue
            where = "%s:%d" % (os.path.basename(w.filename), w.lineno)
            sites[where] = sites.get(where, 0) + 1
            if os.path.basename(w.filename) == "dist.py" and w.lineno in stage_lines:
                n_stage += 1
        syncs = sum(sites.values())
        spans, longest = [], []
        try:
            for e in prof.events():
                if getattr(e, "device_type", None) == torch.autograd.DeviceType.CUDA:
                    spans.append((e.time_range.start, e.time_range.end))
                    longest.append(((e.time_range.end - e.time_range.start) * 1e-3, e.name[:90]))
        except Exception as ex:  # pragma: no cover - profiler without device events
            self.res[name] = {"wall_s": wall, "host_syncs": syncs, "device_busy_s": None,
                              "note": "profiler gave no device events: %s" % ex}
            return out
        spans.sort()
        busy, cur_s, cur_e = 0.0, None, None
        for a, b in spans:
            if cur_e is None or a > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = a, b
            else:
                cur_e = max(cur_e, b)
        if cur_e is not None:
            busy += cur_e - cur_s
        busy_s = busy * 1e-6
        self.res[name] = {"wall_s": wall, "device_busy_s": busy_s if spans else None,
                          "host_and_sync_s": (wall - busy_s) if spans else None,
                          "device_ops": len(spans), "host_syncs": syncs,
                          "host_syncs_without_gloo_staging": syncs - n_stage,
                          "gloo_staged_all_to_all_s": mdist.GLOO_STAGED_S[0] - staged0,
                          "sync_sites": dict(sorted(sites.items(), key=lambda kv: -kv[1])),
                          "longest_device_ops_ms": [[round(ms, 3), nm] for ms, nm in sorted(longest, reverse=True)[:4]]}
        return out


def form_name(width, one_boundary, split, pack_per_tile=False):
    """Name of a fused step form in the bench line / autotune table."""
    return "%d-wide tiles, %sboundary %s%s" % (width, "packed per tile, " if pack_per_tile else "",
                                               "in one launch" if one_boundary else "per tile",
                                               ", interior beside the packing" if split else "")


def link_model(mine, rank, n_tiles, fused=False, boundary_per_tile=True, pack_per_tile=False):
    """The link-bandwidth model of this rank's step, from its own
    per-peer halo bytes and the compute it measured: each peer pair has its own
    xGMI link, so the exchange takes max over peers of max(bytes in, bytes out)
    / link rate; the step is the longer of the compute (pack + interior +
    boundary, measured alone) and the chain pack(first tile) + exchange +
    boundary(last tile) -- in the fused step every tile is packed by one launch
    (the first exchange starts after the whole pack) and, with the boundary in
    one launch, the whole boundary pass follows the last tile.  Predicted at
    60 / 77 / 100 GB/s per link direction, next to the measured overlapped
    step, with the verdict which piece sets it."""
    row = F_DIM * 4
    peers = [q for q in range(len(mine["peers_in"])) if q != rank]
    per_peer = max([max(mine["peers_in"][q], mine["peers_out"][q]) * row for q in peers] or [0])
    dec = mine.get("decomposed") or {}
    comp = dec.get("compute_only_ms")
    if comp is None:
        return None
    T = max(1, n_tiles)
    Tp = 1 if fused and not pack_per_tile else T
    Tb = T if boundary_per_tile else 1
    pack_first = mine.get("send_pack_ms", 0.0) / Tp
    bnd_last = mine.get("boundary_ms", 0.0) / Tb
    pred = {}
    for gbs in LINK_GBS:
        ex = per_peer / (gbs * 1e9) * 1e3
        pred["%g" % gbs] = {"exchange_ms": ex, "step_ms": max(comp, pack_first + ex + bnd_last)}
    meas = dec.get("overlapped_step_ms")
    ex_meas = dec.get("exchange_only_ms")
    nominal = pred["77"]["step_ms"]
    res = {"max_peer_bytes": per_peer, "compute_only_ms": comp, "pack_first_tile_ms": pack_first,
           "boundary_last_tile_ms": bnd_last, "predicted": pred, "measured_step_ms": meas,
           "measured_exchange_ms": ex_meas,
           "measured_link_GBps": (per_peer / (ex_meas * 1e-3) / 1e9) if ex_meas and per_peer else None,
           "measured_over_predicted_77": (meas / nominal) if meas and nominal else None}
    cit = mine.get("compute_in_turn")
    if cit:
        # the same model on the compute each rank measured with the GPU to
        # itself (ranks sharing one GPU in a rehearsal: the node's compute), in
        # the form the step runs (interior beside the send packing or after it)
        c_pf, c_bl = cit["send_pack_ms"] / Tp, cit["boundary_ms"] / Tb
        c_all = cit["compute_alone_split_ms"] if mine.get("split_interior") else cit["compute_alone_ms"]
        res["predicted_in_turn"] = {
            "%g" % gbs: max(c_all, c_pf + per_peer / (gbs * 1e9) * 1e3 + c_bl) for gbs in LINK_GBS}
    if meas is not None and ex_meas is not None:
        longer = max(comp, ex_meas)
        res["contention_ms"] = meas - longer     # beyond a perfect overlap of the two measured pieces
        res["sets_the_step"] = ("exchange" if ex_meas > comp else "compute") + \
            (" + contention" if meas > 1.1 * longer else "")
    return res


# rank 0's halo rows in under the hybrid cover: the exchange volume
# --emulate-peers moves -- config 2 (profiles/r03_halo_cover_p{2,4,8}.jsonl) and
# config 5 (profiles/r06_bench_products_gloo{2,4,8}_rehearsal.json)
EMULATED_COVER_ROWS = {"rmat21": {2: 288_668, 4: 346_920, 8: 313_427},
                       "products": {2: 508_972, 4: 619_964, 8: 570_164}}


def rccl_contention(sg, P, bias, reps=10, rounds=3, workload="rmat21"):
    """RCCL beside the aggregation on one GPU (world 1, RCCL): rank 0 of a P-way
    destination-range partition (edge-balanced cuts of this graph) aggregates
    its in-edges over [own rows ; halo rows] while all_to_all_single moves that
    rank's halo volume (EMULATED_COVER_ROWS, 1 KB rows) as the world's one self
    split -- RCCL's copy kernels then share the CUs, L2 and HBM with k_agg_flat,
    as on the 8-GPU node (the xGMI transfer itself is not modelled: a self
    split is a device-local copy).  Times (ms, median of `rounds` x `reps`):
    exchange alone, compute alone, the two in a row, and overlapped (the
    collective started async, the aggregation on the compute stream, then its
    wait) -- from the legacy default stream and, as OverlappedAggregation
    issues them, from the device's compute stream (dist.compute_stream);
    hidden_frac as OverlappedAggregation.decompose; two aggregations on two
    streams show whether the aggregation leaves any bandwidth to share."""
    from mi355_mp import dist as mdist, ops
    from mi355_mp.graph import Graph
    dev = bias.device
    ei = sg.fwd.local_edge_index          # world 1: the global edge list, global ids
    w = sg.norm_fwd
    N = sg.num_nodes
    deg = torch.bincount(ei[1], minlength=N)
    cuts = mdist.edge_balanced_cuts(deg, P)
    lo, hi = int(cuts[0]), int(cuts[1])
    sel = (ei[1] >= lo) & (ei[1] < hi)
    src, dst, wl = ei[0][sel], ei[1][sel] - lo, w[sel].contiguous()
    remote = (src < lo) | (src >= hi)
    halo = torch.unique(src[remote])
    n_own = hi - lo
    local_src = torch.where(remote, n_own + torch.searchsorted(halo, src), src - lo)
    g = Graph(torch.stack([local_src, dst]), n_own, n_own + halo.numel())
    w_csr = g.dst.to_csr_order(wl)
    gen = torch.Generator(device=dev).manual_seed(11)
    x_loc = torch.randn(n_own + halo.numel(), F_DIM, device=dev, generator=gen)
    out = torch.empty(n_own, F_DIM, device=dev)
    rows = EMULATED_COVER_ROWS.get(workload, {}).get(P, int(halo.numel()))
    send = torch.randn(rows, F_DIM, device=dev, generator=gen)
    recv = torch.empty_like(send)

    side = torch.cuda.Stream(device=dev)
    out2 = torch.empty_like(out)
    assert torch.cuda.current_stream(dev) == torch.cuda.default_stream(dev), "the probe starts on the default stream"

    def compute():
        ops._aggregate(g.dst, "other", x_loc, w_csr, "sum", 0, bias, out=out)

    def exchange():
        dist.all_to_all_single(recv, send)

    def serial():
        exchange()
        compute()

    def overlapped():
        work = dist.all_to_all_single(recv, send, async_op=True)
        compute()
        work.wait()

    def overlapped_side():
        # what OverlappedAggregation does (dist.compute_stream): the collective
        # and the aggregation issued from the device's compute stream, not from
        # the legacy default stream
        with mdist.compute_stream(dev):
            work = dist.all_to_all_single(recv, send, async_op=True)
            compute()
            work.wait()

    def two_aggregations():
        # two aggregations on two streams: whether this GPU runs kernels of
        # different streams side by side at all
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            ops._aggregate(g.dst, "other", x_loc, w_csr, "sum", 0, bias, out=out2)
        compute()
        cur.wait_stream(side)

    def timed(fn):
        per = []
        fn()
        for _ in range(rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            per.append((time.perf_counter() - t0) / reps * 1e3)
        return sorted(per)[len(per) // 2]

    res = {"P": P, "rank_rows": n_own, "rank_edges": int(src.numel()), "pull_halo_rows": int(halo.numel()),
           "exchange_rows": rows, "exchange_bytes": rows * F_DIM * 4, "reps": reps, "rounds": rounds,
           "exchange_only_ms": timed(exchange), "compute_only_ms": timed(compute),
           "serial_step_ms": timed(serial), "overlapped_default_stream_ms": timed(overlapped),
           "overlapped_step_ms": timed(overlapped_side),
           "two_aggregations_two_streams_ms": timed(two_aggregations)}
    shorter = min(res["exchange_only_ms"], res["compute_only_ms"])
    for k, v in (("hidden_frac", "overlapped_step_ms"), ("hidden_frac_default_stream", "overlapped_default_stream_ms")):
        res[k] = (res["exchange_only_ms"] + res["compute_only_ms"] - res[v]) / shorter
    res["overlap_loss_vs_compute"] = res["overlapped_step_ms"] / res["compute_only_ms"] - 1.0
    res["contention_ms"] = res["overlapped_step_ms"] - max(res["exchange_only_ms"], res["compute_only_ms"])
    res["note"] = ("self split on one GPU: RCCL's kernels contend with the aggregation for CUs / L2 / HBM; "
                   "the xGMI transfer time is not part of it")
    return res


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.workload == "reddit" and (args.gpus > 1 or args.sharded):
        # BASELINE config 4 is a one-GPU configuration (x is 238 MB: it fits one
        # GPU's Infinity Cache); the sharded max path is ShardedGraph.propagate
        stage("-", "ERROR: --workload reddit is BASELINE config 4, a one-GPU configuration")
        sys.exit(2)
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(args, argv))
    claim_stdout()
    rank, world, local = setup_dist(args)
    sharded = dist.is_initialized()
    if sharded:
        start_heartbeat(rank)
    if args.workload == "gat":
        return main_gat(args, rank, world, local)
    if args.workload == "reddit":
        return main_reddit(args, rank, world, local)
    wl = WORKLOADS[args.workload]
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import mi355_mp
    from mi355_mp import _lib, ops
    from mi355_mp.graph import Graph
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    mi355_mp.load_native()

    N = wl["num_nodes"]
    t0 = time.perf_counter()
    ei = wl["gen"](dev)
    if sharded:
        # each rank keeps only its contiguous 1/world slice of the edge list (the
        # generator, deterministic on every rank, stands in for reading the rank's
        # shard of an edge file): loops, norm, cuts and plans are built from the
        # slices with all_to_alls -- no rank holds or sorts the whole list
        E_raw = ei.shape[1]
        s0, s1 = rank * E_raw // world, (rank + 1) * E_raw // world
        ei_slice = ei[:, s0:s1].clone()
        del ei
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    stage(rank, "%s graph generated (%.1f s)" % (args.workload, t_gen))

    # one-time build: loops + norm (GCNConv.norm), CSR + schedule
    t0 = time.perf_counter()
    bias = torch.randn(F_DIM, device=dev, generator=torch.Generator(device=dev).manual_seed(7)) * 0.1
    g = torch.Generator(device=dev).manual_seed(wl["seed"])
    t_shards = t_exchange_plan = None
    t_warm = 0.0
    if not sharded:
        ei2, norm = GCNConv.norm(ei, N)
        del ei
        E2 = ei2.shape[1]
        graph = Graph(ei2, N, N, chunk=args.chunk or None)
        csr = graph.dst
        w_csr = csr.to_csr_order(norm)
        x = torch.randn(N, F_DIM, device=dev, generator=g)
        n_rows = N
        E_local = E2
    else:
        from mi355_mp import dist as mdist
        # more than two ranks per GPU with the default four hardware queues per
        # process: the queues oversubscribe the GPU's queue slots and the build
        # crawls (61 s instead of 1.1 s at 4 ranks) -- wall time only
        # there; the rehearsals run with GPU_MAX_HW_QUEUES=1 and are profiled
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        crowded = (local_world > 2 * max(1, torch.cuda.device_count())
                   and os.environ.get("GPU_MAX_HW_QUEUES") != "1")
        meter = BuildMeter(not args.no_build_split and not crowded)
        sg = meter.run("shards", lambda: mdist.ShardedGraph.for_gcn_from_slices(ei_slice, s0, N, rank, world,
                                                                               chunk=args.chunk or None))
        torch.cuda.synchronize()
        t_shards = time.perf_counter() - t0
        if world == 1 and meter.enabled:
            # one rank: the same build once more, warm -- the first one also pays the
            # process's one-time costs (first launch of every kernel, the pinned
            # staging pool), the second shows the build's own host / device split
            # (not counted in the build times)
            tw = time.perf_counter()
            meter.run("shards_warm", lambda: mdist.ShardedGraph.for_gcn_from_slices(
                ei_slice, s0, N, rank, world, chunk=args.chunk or None))
            t_warm += time.perf_counter() - tw
        del ei_slice
        stage(rank, "shards built: %d rows, %d in-edges, %d pull-halo rows (%.1f s)"
              % (sg.n_own, sg.fwd.edge_pos.numel(), sg.fwd.n_local_src - sg.n_own, t_shards))
        E2 = sg.n_edges
        plan = sg.fwd
        x_full = torch.randn(N, F_DIM, device=dev, generator=g)
        x_local = plan.local_buffer(F_DIM)
        x_local[:plan.n_own].copy_(x_full[plan.lo:plan.hi])
        x = x_local[:plan.n_own]
        overlap = meter.run("exchange_plan", lambda: mdist.OverlappedAggregation(
            plan, sg.norm_fwd, chunk=args.chunk or None, local_weights=True,
            cover=not (args.no_halo_cover or args.no_overlap)))
        torch.cuda.synchronize()
        t_exchange_plan = time.perf_counter() - t0 - t_shards - t_warm
        if world == 1 and meter.enabled:
            tw = time.perf_counter()
            meter.run("exchange_plan_warm", lambda: mdist.OverlappedAggregation(
                plan, sg.norm_fwd, chunk=args.chunk or None, local_weights=True,
                cover=not (args.no_halo_cover or args.no_overlap)))
            t_warm += time.perf_counter() - tw
        bufs = x_ov = None
        tile_tune = None
        if args.halo_tile != 0 and not args.no_overlap:
            if args.halo_tile > 0:
                form = (args.halo_tile, not args.boundary_per_tile, args.pack_per_tile)
            else:
                # warm-up autotune: every rank times each step form (tile width x
                # boundary as one launch or per tile x send rows packed in one launch
                # or per tile), with the interior pass after and beside the send
                # packing (split_interior), one untimed step then 3; the max over
                # ranks decides -- the same choice on every rank.  A gloo rehearsal
                # (ranks sharing a GPU, every exchange staged through host memory)
                # ranks the forms by the node step its own measurements predict
                # instead: the longer of its compute in turn and the link chain
                # pack(first) + exchange at 77 GB/s + boundary(last) (link_model) --
                # its step time is the host staging's, not the forms'.  With one
                # hardware queue per process (the rehearsals' GPU_MAX_HW_QUEUES=1,
                # DESIGN 5.5) the side stream cannot run beside the compute stream,
                # so the split forms are left out there.
                tune_out = torch.empty((plan.n_own, F_DIM), device=dev)
                tile_tune = {}
                staged = dist.get_backend() == "gloo"
                one_queue = os.environ.get("GPU_MAX_HW_QUEUES") == "1"
                peer_bytes = max([max(overlap.recv_counts[q], overlap.send_counts[q]) * F_DIM * 4
                                  for q in range(world) if q != rank] or [0])
                forms = [(c, sp) for c in HALO_FORMS for sp in ((False,) if one_queue else (False, True))]
                for (width, one, ppt), split in forms:
                    if staged and split:
                        continue                  # timed with its non-split twin below
                    tb = overlap.halo_buffers(F_DIM, width)
                    overlap.split_interior, overlap.one_boundary_launch, overlap.pack_per_tile = split, one, ppt
                    if staged:
                        cit = overlap.compute_in_turn((x, tb), tune_out, bias, reps=5, barrier=lambda: barrier(world))
                        T = tb.n_tiles
                        chain = (cit["send_pack_ms"] / (T if ppt else 1) + peer_bytes / 77e9 * 1e3
                                 + cit["boundary_ms"] / (1 if one else T))
                        tt = torch.tensor([max(cit["compute_alone_ms"], chain),
                                           max(cit["compute_alone_split_ms"], chain)], dtype=torch.float64)
                        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                        tile_tune[form_name(width, one, False, ppt)] = float(tt[0])
                        if not one_queue:
                            tile_tune[form_name(width, one, True, ppt)] = float(tt[1])
                        del tb
                        continue
                    overlap.step_fused(x, tb, tune_out, bias)
                    torch.cuda.synchronize()
                    barrier(world)
                    t1 = time.perf_counter()
                    for _ in range(3):
                        overlap.step_fused(x, tb, tune_out, bias)
                    torch.cuda.synchronize()
                    tt = torch.tensor([(time.perf_counter() - t1) / 3 * 1e3], dtype=torch.float64)
                    tt = tt.to(dev) if dist.get_backend() == "nccl" else tt
                    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                    tile_tune[form_name(width, one, split, ppt)] = float(tt.item())
                    del tb
                del tune_out
                best = min(tile_tune, key=tile_tune.get)
                (width, one, ppt), split = next(f for f in [(c, sp) for c in HALO_FORMS for sp in (False, True)]
                                                if form_name(f[0][0], f[0][1], f[1], f[0][2]) == best)
                form = (width, one, ppt)
                overlap.split_interior = split
                stage(rank, "step form chosen in the warm-up: %s (max over ranks, %s: %s)"
                      % (best, "predicted node step from the compute in turn, ms" if staged else "ms/step",
                         json.dumps(tile_tune)))
            overlap.one_boundary_launch, overlap.pack_per_tile = form[1], form[2]
            bufs = overlap.halo_buffers(F_DIM, form[0])
        elif not args.no_overlap:
            x_ov = overlap.local_buffer(F_DIM)
            x_ov[:plan.n_own].copy_(x_full[plan.lo:plan.hi])
        del x_full
        graph = sg.g_fwd
        csr = graph.dst
        w_csr = sg._w[0]
        n_rows = plan.n_own
        E_local = plan.local_edge_index.shape[1]
        stage(rank, "exchange plan built: %s, %d interior / %d boundary edges (%.1f s)"
              % ("cover" if overlap.cover is not None else "pull", overlap.n_interior, overlap.n_boundary,
                 t_exchange_plan))
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0 - t_warm

    lib = _lib.load()
    st_main = csr.struct("other")

    slab = torch.empty(lib.mp_aggregate_slab_bytes(st_main, F_DIM, _lib.MP_REDUCE["sum"]),
                       dtype=torch.uint8, device=dev)

    def aggregate(x_src, stages=_lib.MP_STAGE_ALL, out=None):
        return ops._aggregate(csr, "other", x_src, w_csr, "sum", 0, bias, out=out, stages=stages,
                              slab=slab)[0]

    out_buf = torch.empty((n_rows, F_DIM), device=dev)

    # dominant-kernel timing inside the timed region (N=1): HIP events on the
    # stream the kernels run on (torch's current stream), around the main
    # launch and the fix-up launch of every timed step
    ev = None

    def step(i=None):
        if not sharded:
            if i is None or ev is None:
                aggregate(x, out=out_buf)
            else:
                ev[i][0].record()
                aggregate(x, stages=_lib.MP_STAGE_MAIN, out=out_buf)
                ev[i][1].record()
                aggregate(x, stages=_lib.MP_STAGE_FIXUP, out=out_buf)
                ev[i][2].record()
        elif args.no_overlap:
            aggregate(plan.exchange_into(x_local, ops.gather_rows), out=out_buf)
        elif bufs is not None:
            overlap.step_fused(x, bufs, out_buf, bias, events=None if i is None else step_events[i])
        else:
            overlap.step(x_ov, out_buf, bias)

    step_events = [dict() for _ in range(args.steps)]
    for _ in range(args.warmup):
        step()
    if not sharded:
        ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    barrier(world)
    stage(rank, "warm-up done (%d steps)" % args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    dt_local = dt = time.perf_counter() - t0
    if sharded:
        tt = torch.tensor([dt], dtype=torch.float64)
        tt = tt.to(dev) if dist.get_backend() == "nccl" else tt
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    stage(rank, "timed steps done: %d steps, %.3f ms/step (max over ranks)" % (args.steps, dt / args.steps * 1e3))
    ms_per_step = dt / args.steps * 1e3
    value = E2 * args.steps / dt    # whole-job edges aggregated per second

    # the step once more, outside the timed region, for --verify
    verify = None
    if args.verify:
        step()
        torch.cuda.synchronize()
        if not sharded:
            verify = verify_f64(out_buf, x, ei2[0], ei2[1], norm, bias)
        else:
            # the rank's own edges over [own rows ; pulled halo rows] (plan order =
            # global edge order), whatever exchange (pull / cover, tiled) the step used
            xv = plan.local_buffer(F_DIM)
            xv[:plan.n_own].copy_(x)
            plan.exchange_into(xv, ops.gather_rows)
            lei = plan.local_edge_index
            verify = verify_f64(out_buf, xv, lei[0], lei[1], sg.norm_fwd, bias)
            del xv
        stage(rank, "verify: %s" % json.dumps(verify))

    # dominant kernel (main aggregation launch) timed with HIP events on the
    # stream it runs on (torch's current stream): `reps` back-to-back launches
    # between two events (host launch latency amortised), averaged
    x_src = x if not sharded else plan.exchange_into(x_local, ops.gather_rows)
    reps = max(args.steps, 10)

    def timed(stages, rounds=3):
        per = []
        for _ in range(rounds):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                aggregate(x_src, stages=stages, out=out_buf)
            b.record()
            torch.cuda.synchronize()
            per.append(a.elapsed_time(b) / reps)
        return sorted(per)

    if not sharded:
        main_ms = sorted(a.elapsed_time(b) for a, b, _ in ev)
        fix_ms = sorted(b.elapsed_time(c) for _, b, c in ev)
        timing_src = "HIP events around each main / fix-up launch inside the timed steps"
    else:
        # N>1: a step is several launches (per tile, interior + boundary); the
        # per-rank kernel rate is timed on the rank's full local graph instead
        main_ms = timed(_lib.MP_STAGE_MAIN)
        fix_ms = timed(_lib.MP_STAGE_FIXUP)
        timing_src = "HIP events over back-to-back launches on the rank's local graph (after the timed region)"
    # the kernel the library dispatches for exactly these arguments (no heuristic copy)
    kernel = _lib.kernel_name(st_main, w_csr.data_ptr(), x_src.data_ptr(), x_src.stride(0), F_DIM, "sum",
                              bias.data_ptr(), out_buf.data_ptr(), out_buf.stride(0), dev)
    main_avg = sum(main_ms) / len(main_ms)
    fix_avg = sum(fix_ms) / len(fix_ms)
    alg_bytes = E_local * BYTES_PER_EDGE + n_rows * BYTES_PER_NODE
    # compulsory bytes: every input read once and the output written once
    # (x, col, norm, rowptr, out) -- the least any implementation must move,
    # so achieved / peak <= 1 is a true HBM-roofline fraction
    n_src_rows = x_src.shape[0]
    comp_bytes = n_src_rows * F_DIM * 4 + E_local * 8 + (n_rows + 1) * 4 + n_rows * F_DIM * 4
    achieved = comp_bytes / (main_avg * 1e-3) / 1e9

    # GEMM (reported separately, the only MFMA work)
    W = torch.randn(F_DIM, F_DIM, device=dev) * 0.06
    for _ in range(3):
        torch.matmul(x, W)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.matmul(x, W)
    e1.record()
    torch.cuda.synchronize()
    gemm_ms = e0.elapsed_time(e1) / 10

    # counter traffic (FETCH_SIZE + WRITE_SIZE, corrected) of THIS build's
    # dispatched kernel, from a committed profile summary -- used only when the
    # summary names the same workload, kernel and native source hash
    src_hash = lib.mp_source_hash().decode()   # the LOADED library's build (load() checks it against the tree)
    traffic, traffic_src = (None, "N>1: per-rank graphs are not profiled") if sharded else \
        find_pmc(wl["name"], kernel, src_hash)

    # the reference's own device path and a vendor SpMM on the same GPU, same
    # CSR / weights (outside the timed region; checked against the fused output)
    ref_paths = None
    if not sharded and not args.no_ref_paths:
        aggregate(x, out=out_buf)
        fused_out = out_buf.clone()
        terms = ops._aggregate(csr, "other", x.abs(), w_csr.abs(), "sum", 0, None)[0]
        ref_paths = device_reference_paths(ei2, norm, x, csr, w_csr, bias, fused_out, terms)
        ref_paths["fused_ms"] = main_avg + fix_avg
        del fused_out, terms
        torch.cuda.empty_cache()
        stage(rank, "same-GPU reference paths timed")

    # per-rank exchange / compute split (N > 1): of the timed steps (tiled
    # overlap: HIP events on the compute stream around the interior passes,
    # around each tile's work.wait() -- exchange time the compute stream is
    # exposed to -- and around each boundary pass), then the step taken apart:
    # the exchange alone, the compute alone, exchange-then-compute; gathered to rank 0
    ranks = None
    if sharded:
        def span(evs, k):
            lst = evs.get(k, [])
            return sum(lst[j].elapsed_time(lst[j + 1]) for j in range(0, len(lst) - 1, 2))
        torch.cuda.synchronize()
        mine = {"rank": rank, "build_shards_s": t_shards, "build_exchange_s": t_exchange_plan,
                "rows": plan.n_own, "edges": E_local, "interior_edges": overlap.n_interior,
                "boundary_edges": overlap.n_boundary,
                "exchange": "pull" if args.no_overlap or overlap.cover is None else "cover (pull + push partials)",
                "halo_rows": (plan.n_local_src if args.no_overlap else overlap.n_local_src) - plan.n_own,
                "halo_bytes_in": ((plan.n_local_src if args.no_overlap else overlap.n_local_src) - plan.n_own)
                * F_DIM * 4,
                "halo_bytes_out": (int(plan.send_idx.numel()) if args.no_overlap else overlap.n_send) * F_DIM * 4,
                "pull_exchange_rows_in": plan.n_local_src - plan.n_own,
                "peers_in": [int(c) for c in (plan.recv_counts if args.no_overlap else overlap.recv_counts)],
                "peers_out": [int(c) for c in (plan.send_counts if args.no_overlap else overlap.send_counts)],
                "build_split": meter.res, "build_split_profiled": meter.enabled,
                "step_ms_this_rank": dt_local / args.steps * 1e3}
        if overlap.cover is not None:
            mine.update({"cover_pulled_rows": overlap.cover.n_pull_rows,
                         "cover_partial_rows": overlap.cover.n_push_rows,
                         "cover_push_edges": overlap.cover.n_push_edges})
        if bufs is not None:
            n = max(1, len(step_events))
            mine.update({"send_pack_ms": sum(span(e, "send") for e in step_events) / n,
                         "interior_ms": sum(span(e, "interior") for e in step_events) / n,
                         "exchange_exposed_ms": sum(span(e, "wait") for e in step_events) / n,
                         "boundary_ms": sum(span(e, "boundary") for e in step_events) / n})
        if not args.no_overlap:
            form = (x, bufs) if bufs is not None else [x_ov]
            reps_d = max(3, min(args.steps, 10))
            mine["decomposed"] = overlap.decompose(form, out_buf, bias, reps_d, barrier=lambda: barrier(world))
            stage(rank, "step decomposition: %s" % json.dumps(mine["decomposed"]))
            mine["split_interior"] = bool(overlap.split_interior)
            mine["one_boundary_launch"] = bool(overlap.one_boundary_launch) if bufs is not None else None
            mine["compute_in_turn"] = overlap.compute_in_turn(form, out_buf, bias, max(7, reps_d),
                                                              barrier=lambda: barrier(world))
            stage(rank, "compute in turn: %s" % json.dumps(mine["compute_in_turn"]))
            mine["link_model"] = link_model(mine, rank, bufs.n_tiles if bufs is not None else 1,
                                            fused=bufs is not None,
                                            boundary_per_tile=bufs is not None and not overlap.one_boundary_launch,
                                            pack_per_tile=bufs is not None and overlap.pack_per_tile)
            stage(rank, "link model: %s" % json.dumps(mine["link_model"]))
        if args.emulate_peers:
            if world != 1 or dist.get_backend() != "nccl":
                raise SystemExit("--emulate-peers needs --sharded at one RCCL rank")
            mine["rccl_contention"] = []
            for P in [int(p) for p in args.emulate_peers.split(",") if p]:
                r = rccl_contention(sg, P, bias, workload=args.workload)
                mine["rccl_contention"].append(r)
                stage(rank, "RCCL beside the aggregation (P = %d): %s" % (P, json.dumps(r)))
        if verify is not None:
            mine["verify"] = verify
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        if verify is not None:
            verify = {"all_ranks_within_1e-5_bound": all(r["verify"]["within_1e-5_bound"] for r in ranks),
                      "max_bound_excess": max(r["verify"]["bound_excess"] for r in ranks),
                      "rows": sum(r["verify"]["rows"] for r in ranks),
                      "reference": ranks[0]["verify"]["reference"] + ", per rank over its own edges"}

    cpu = None
    if rank == 0 and not sharded and not args.no_cpu_baseline:
        cpu = cpu_baseline(ei2, norm, x, args.cpu_sample_edges)
        stage(rank, "cpu baseline done")

    if rank == 0:
        line = {
            "metric": "edges aggregated/sec (GCNConv F=256 propagate, fused gather*norm->segment-sum+bias)",
            "value": value,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic %s graph (seeded, generated on device), random-init features" % args.workload,
            "config": {"workload": wl["name"], "baseline_config": wl["baseline_config"], "graph": wl["graph"],
                       "num_nodes": N, "num_edges": E2, "features": F_DIM, "seed": wl["seed"],
                       "parallelism": "dst-range shards x%d, RCCL halo all_to_all" % world if sharded
                       else "single GPU", "chunk": csr.chunk},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_frac": (traffic / (main_avg * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
                         "traffic_source": traffic_src,
                         "bytes": "achieved = compulsory bytes (x read once, out written once, col + norm + "
                                  "rowptr) / avg launch time",
                         "compulsory_bytes_per_launch": comp_bytes,
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "algorithmic_GBps_no_cache_credit": alg_bytes / (main_avg * 1e-3) / 1e9,
                         "kernel": kernel, "source_hash": src_hash,
                         "avg_launch_ms": main_avg, "median_launch_ms": main_ms[len(main_ms) // 2],
                         "fixup_avg_ms": fix_avg, "timing": timing_src},
            "cpu_baseline": cpu,
            "extra": {"gemm_xW_ms": gemm_ms, "layer_ms_est": gemm_ms + main_avg + fix_avg,
                      "one_time_build_s": t_build, "graph_gen_s": t_gen,
                      "edges_local_rank0": E_local, "n_split_rows": csr.n_split,
                      "halo_rows_rank0": ((plan.n_local_src if args.no_overlap else overlap.n_local_src)
                                          - plan.n_own) if sharded else 0,
                      "halo_cover": sharded and not args.no_overlap and not args.no_halo_cover,
                      "interior_edges_rank0": overlap.n_interior if sharded else E_local,
                      "overlap": sharded and not args.no_overlap,
                      "halo_tile": args.halo_tile if sharded and not args.no_overlap else None,
                      "halo_tiles": [bufs.width] * bufs.n_tiles if sharded and bufs is not None else None,
                      "step_form": ("fused: one launch per pass, %s" % form_name(bufs.width, overlap.one_boundary_launch,
                                                                          overlap.split_interior, overlap.pack_per_tile))
                      if sharded and bufs is not None else None,
                      "halo_tile_autotune_ms": tile_tune if sharded else None,
                      "halo_tile_autotune_basis": (None if not sharded or tile_tune is None else
                                                   "max over ranks of max(compute in turn, link chain at 77 GB/s)"
                                                   " (gloo rehearsal)"
                                                   if dist.get_backend() == "gloo" else "step time, max over ranks"),
                      "split_interior": bool(overlap.split_interior) if sharded and overlap is not None else None,
                      "collective_timeout_s": COLLECTIVE_TIMEOUT_S if sharded else None,
                      "comm_init_s": COMM_INIT_S[0] if sharded else None,
                      "n_wave_tasks": csr.n_waves,
                      "per_rank": ranks,
                      "verify": verify,
                      "gpu_reference_path_ms": ((ref_paths or {}).get("reference_path") or {}).get("ms"),
                      "hipsparse_spmm_ms": ((ref_paths or {}).get("vendor_spmm") or {}).get("ms"),
                      "same_gpu_paths": ref_paths,
                      "agg_only_GBps_incl_fixup": alg_bytes / ((main_avg + fix_avg) * 1e-3) / 1e9},
        }
        emit(line)
    stage(rank, "done")
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
