import os, sys, socket
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    sys.path.insert(0, p)
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mi355_mp import dist as mdist, ops
    from torch_geometric.nn import GCNConv
    from mi355_mp.graphgen import powerlaw_edge_index
    dev = torch.device("cuda", 0)
    N, E, Fi, Fo = 3000, 60000, 64, 256
    ei = powerlaw_edge_index(N, E, seed=41).to(dev)
    gen = torch.Generator().manual_seed(41)
    x = torch.randn(N, Fi, generator=gen).to(dev)
    ref = GCNConv(Fi, Fo).to(dev)
    with torch.no_grad():
        ref.bias.normal_()
    print(rank, "W sum", float(ref.weight.sum()), "b sum", float(ref.bias.sum()), flush=True)
    out_ref = ref(x, ei)
    sg = mdist.ShardedGraph.for_gcn(ei, N, rank, world)
    xw = x @ ref.weight
    lo, hi = sg.lo, sg.hi
    p = sg.propagate(xw[lo:hi]) + ref.bias
    print(rank, "err", float((p - out_ref[lo:hi]).abs().max()), flush=True)
    plan = sg.fwd
    xl = plan.local_buffer(Fo, device=dev)
    xl[:plan.n_own].copy_(xw[lo:hi])
    plan.exchange_into(xl, ops.gather_rows)
    print(rank, "halo err", float((xl[plan.n_own:] - xw[plan.halo_nodes]).abs().max()), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(worker, args=(2, port), nprocs=2)
