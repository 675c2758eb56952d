"""Which streams let RCCL run beside the aggregation on one MI355X (round 5).

HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 on the pool),
round-robin as they are created; two streams on one queue run their kernels
one after the other.  At one RCCL rank with a non-empty self split (the P = 8
volume of bench.py --emulate-peers), an all_to_all started async and the
P = 8 rank's aggregation are timed from: the default stream, normal-priority
side streams created before and after the communicator, and a high-priority
side stream.  Prints one JSON line per variant (hidden_frac as
OverlappedAggregation.decompose); run under rocprofv3 --kernel-trace to see
the queue of every kernel.
    python tools/queue_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from mi355_mp import ops
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29577"), RANK="0",
                      WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    early = torch.cuda.Stream(device=dev)                  # created before the communicator
    dist.init_process_group("nccl", device_id=dev)
    F, N, P = 256, 1 << 21, 8
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    # rank 0 of a P-way edge-balanced destination split, sources renumbered [own ; halo]
    deg = torch.bincount(ei[1], minlength=N)
    csum = torch.cumsum(deg, 0)
    hi = int(torch.searchsorted(csum, csum[-1] // P, right=True))
    sel = ei[1] < hi
    src, dst = ei[0][sel], ei[1][sel]
    remote = src >= hi
    halo = torch.unique(src[remote])
    lsrc = torch.where(remote, hi + torch.searchsorted(halo, src), src)
    g = Graph(torch.stack([lsrc, dst]), hi, hi + halo.numel())
    del ei, src, dst, lsrc
    x = torch.randn(hi + halo.numel(), F, device=dev)
    w = g.dst.to_csr_order(torch.rand(g.dst.n_edges, device=dev))
    out = torch.empty(hi, F, device=dev)
    send = torch.randn(313_427, F, device=dev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)                     # communicator + its streams
    late = torch.cuda.Stream(device=dev)                   # created after it
    high = torch.cuda.Stream(device=dev, priority=-1)

    def compute():
        ops._aggregate(g.dst, "other", x, w, "sum", 0, None, out=out)

    def on(stream, fn):
        if stream is None:
            fn()
            return
        cur = torch.cuda.current_stream(dev)
        stream.wait_stream(cur)
        with torch.cuda.stream(stream):
            fn()
        cur.wait_stream(stream)

    def overlapped(stream):
        def body():
            work = dist.all_to_all_single(recv, send, async_op=True)
            compute()
            work.wait()
        on(stream, body)

    def timed(fn, reps=10, rounds=3):
        fn()
        per = []
        for _ in range(rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            per.append((time.perf_counter() - t0) / reps * 1e3)
        return sorted(per)[len(per) // 2]

    ex = timed(lambda: dist.all_to_all_single(recv, send))
    comp = timed(compute)
    for name, s in (("default", None), ("early", early), ("late", late), ("high_priority", high)):
        ov = timed(lambda: overlapped(s))
        print(json.dumps({"variant": name, "stream_id": None if s is None else s.stream_id,
                          "exchange_only_ms": ex, "compute_only_ms": comp, "overlapped_ms": ov,
                          "hidden_frac": (ex + comp - ov) / min(ex, comp),
                          "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                          "torch_nccl_high_priority": os.environ.get("TORCH_NCCL_HIGH_PRIORITY")}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
