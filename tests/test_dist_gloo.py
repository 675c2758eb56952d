"""Multi-process (gloo, CPU) tests of the destination-range sharding + halo
exchange (mi355_mp.dist).  The local aggregation is the CPU oracle here (the
GPU runs the same plan with the native kernel and RCCL); every rank's rows
must equal the single-process oracle bit for bit, because a rank keeps its
edges in global order and so sums every row in the same order."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, result_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mi355_mp import dist as mdist
        from mi355_mp.graphgen import powerlaw_edge_index
        from oracle import scatter_ref as S
        N, E, F = 900, 12000, 7
        ei = powerlaw_edge_index(N, E, seed=21)
        g = torch.Generator().manual_seed(21)
        x = torch.randn(N, F, generator=g)
        w = torch.rand(E, generator=g)
        plan = mdist.ShardPlan(ei, N, rank, world).exchange_requests()

        def local_aggregate(xl, lei, n_dst, n_src, wl):
            return S.gather_sum(xl, lei[0], lei[1], wl, n_dst)

        out = mdist.sharded_propagate(plan, x[plan.lo:plan.hi].contiguous(), local_aggregate,
                                      lambda t, idx: t[idx], edge_weight=w)
        want = S.gather_sum(x, ei[0], ei[1], w, N)[plan.lo:plan.hi]
        ok = torch.equal(out, want)
        # edge balance: every rank holds about E / world edges
        result_q.put((rank, ok, plan.lo, plan.hi, int(plan.edge_pos.numel()), plan.recv_counts))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gcn_aggregation_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert all(r[1] for r in res), res
    # contiguous cover of [0, N)
    assert res[0][2] == 0 and all(res[k][3] == res[k + 1][2] for k in range(world - 1))
    edges = [r[4] for r in res]
    assert sum(edges) == 12000
    assert max(edges) < 1.5 * 12000 / world + 200


def test_edge_balanced_cuts():
    from mi355_mp.dist import edge_balanced_cuts
    deg = torch.tensor([100, 1, 1, 1, 1, 1, 1, 94])
    cuts = edge_balanced_cuts(deg, 2)
    assert cuts[0] == 0 and cuts[-1] == 8
    assert cuts[1] in (1, 2, 7)
    cuts = edge_balanced_cuts(torch.ones(10, dtype=torch.long), 5)
    assert cuts == [0, 2, 4, 6, 8, 10]
