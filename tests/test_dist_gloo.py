"""Multi-process (gloo, CPU) tests of the destination-range sharding + halo
exchange (mi355_mp.dist).  The local aggregation is the CPU oracle here (the
GPU runs the same plan with the native kernel and RCCL); every rank's rows
must equal the single-process oracle bit for bit, because a rank keeps its
edges in global order and so sums every row in the same order: sum, max/min
with global argmax ids, and the backward of the sum (a forward over the
transposed plan)."""
import os

import pytest
import torch
import torch.distributed as dist

from tests._ranks import run_ranks


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
        from tests import _host_twins
        _host_twins.install()   # host twins of the native kernels (no CPU fallback in mi355_mp)
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

        rows = lambda t, idx: t[idx]  # noqa: E731
        out = mdist.sharded_propagate(plan, x[plan.lo:plan.hi].contiguous(), local_aggregate, rows, edge_weight=w)
        want = S.gather_sum(x, ei[0], ei[1], w, N)[plan.lo:plan.hi]
        ok = torch.equal(out, want)
        # max / min + arg: local args map to GLOBAL edge ids, first maximal edge wins
        # (tie-heavy small integers, duplicate edges)
        xi = torch.randint(-3, 4, (N, F), generator=g).to(torch.float32)
        for red in ("max", "min"):
            def local_arg(xl, lei, n_dst, n_src, wl, red=red):
                return S.scatter_loop(xl[lei[0]], lei[1], n_dst, red)
            o, a = mdist.sharded_propagate(plan, xi[plan.lo:plan.hi].contiguous(), local_arg, rows,
                                           n_edges_global=E)
            wo, wa = S.scatter_loop(xi[ei[0]], ei[1], N, red)
            ok = ok and torch.equal(o, wo[plan.lo:plan.hi]) and torch.equal(a, wa[plan.lo:plan.hi])
        # backward of the sum = a forward over the transposed plan: d x_j summed by
        # j's owner in global edge order (bit-equal to the single-process transpose)
        plan_t = mdist.transposed_plan(ei, N, rank, world, plan.cuts)
        gout = torch.randn(N, F, generator=torch.Generator().manual_seed(99))

        def local_t(xl, lei, n_dst, n_src, wl):
            return S.gather_sum(xl, lei[1], lei[0], wl, n_dst)
        gx = mdist.sharded_propagate(plan_t, gout[plan.lo:plan.hi].contiguous(), local_t, rows, edge_weight=w)
        gwant = S.gather_sum(gout, ei[1], ei[0], w, N)[plan.lo:plan.hi]
        ok_bwd = torch.equal(gx, gwant)
        # return_halo: every halo row goes back to its owner, aligned with send_idx
        back = plan.return_halo(x[plan.halo_nodes])
        ok_ret = torch.equal(back, x[plan.send_idx + plan.lo])
        # edge balance: every rank holds about E / world edges
        result_q.put((rank, ok and ok_bwd and ok_ret, plan.lo, plan.hi, int(plan.edge_pos.numel()),
                      plan.recv_counts, (ok, ok_bwd, ok_ret)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_sharded_gcn_aggregation_matches_single_process(world):
    res = run_ranks(_worker, world, timeout=120)
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


def _slices_worker(rank, world, port, result_q):
    """gcn_shards_from_slices / ShardedGraph.for_gcn_from_slices: every rank
    holds only its contiguous slice of the edge list; the cuts, the rank's local
    edge lists (in-edges and out-edges, global order), their global ids and the
    GCN norms must equal the plans built from the full list and the oracle's
    norm bit for bit -- weighted, with duplicate pre-existing self loops (the
    last one's weight wins) -- and the sharded propagate must equal the
    single-process oracle."""
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
        from tests import _host_twins
        _host_twins.install()   # host twins of the native kernels (no CPU fallback in mi355_mp)
        from mi355_mp.graphgen import powerlaw_edge_index
        from oracle import pyg_ref as P, scatter_ref as S
        N, E, F = 700, 9000, 5
        ei = powerlaw_edge_index(N, E, seed=23)
        g = torch.Generator().manual_seed(23)
        loops = torch.randint(N, (40,), generator=g)
        loops = torch.cat([loops, loops[:10]])                       # duplicate loops of some nodes
        ei = torch.cat([ei, torch.stack([loops, loops])], 1)
        ei = ei[:, torch.randperm(ei.shape[1], generator=g)]
        E = ei.shape[1]
        w = torch.rand(E, generator=g) * 2
        ok = {}
        for improved, weighted in ((False, False), (True, True), (False, True)):
            ww = w if weighted else None
            s0, s1 = rank * E // world, (rank + 1) * E // world
            sg = mdist.ShardedGraph.for_gcn_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world, improved=improved,
                                                         edge_weight=None if ww is None else ww[s0:s1].clone())
            ei2, norm = P.gcn_norm(ei, N, ww, improved)
            cuts = mdist.edge_balanced_cuts(torch.bincount(ei2[1], minlength=N), world)
            rf = mdist.ShardPlan(ei2, N, rank, world, cuts=cuts)
            rb = mdist.ShardPlan(ei2, N, rank, world, cuts=cuts, flow="target_to_source")
            key = (improved, weighted)
            ok[key] = (sg.fwd.cuts == cuts and sg.n_edges == ei2.shape[1]
                       and torch.equal(sg.fwd.local_edge_index, rf.local_edge_index)
                       and torch.equal(sg.fwd.edge_gid, rf.edge_pos)
                       and torch.equal(sg.bwd.local_edge_index, rb.local_edge_index)
                       and torch.equal(sg.bwd.edge_gid, rb.edge_pos)
                       and torch.equal(sg.norm_fwd, norm[rf.edge_pos])
                       and torch.equal(sg.norm_bwd, norm[rb.edge_pos]))
            # the sharded propagate over the slice-built plan == the single-process oracle
            x = torch.randn(N, F, generator=torch.Generator().manual_seed(5))

            def local_aggregate(xl, lei, n_dst, n_src, wl):
                return S.gather_sum(xl, lei[0], lei[1], wl, n_dst)
            out = mdist.sharded_propagate(sg.fwd, x[sg.lo:sg.hi].contiguous(), local_aggregate,
                                          lambda t, idx: t[idx], edge_weight=sg.norm_fwd)
            want = S.gather_sum(x, ei2[0], ei2[1], norm, N)[sg.lo:sg.hi]
            ok[key] = ok[key] and torch.equal(out, want)
        result_q.put((rank, all(ok.values()), {str(k): v for k, v in ok.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_gcn_shards_from_edge_slices_match_full_list(world):
    res = run_ranks(_slices_worker, world, timeout=180)
    assert all(r[1] for r in res), res


def _cover_worker(rank, world, port, result_q, cuts):
    """HaloCover (hybrid pull / push halo exchange) against the single-process
    oracle: float data within 1e-5 * sum|w x| (rows regrouped), integer-valued
    data bit for bit (every regrouping is exact there), and never more rows
    over the links than the pull exchange."""
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
        from tests import _host_twins
        _host_twins.install()   # host twins of the native kernels (no CPU fallback in mi355_mp)
        from mi355_mp.graphgen import powerlaw_edge_index
        from oracle import scatter_ref as S
        N, E, F = 1200, 30000, 6
        ei = powerlaw_edge_index(N, E, seed=41)
        g = torch.Generator().manual_seed(41)
        w = torch.rand(E, generator=g) + 0.1
        plan = mdist.ShardPlan(ei, N, rank, world, cuts=cuts).exchange_requests()
        hc = mdist.HaloCover(plan, w[plan.edge_pos])

        def agg(xs, s, d, ws, n):
            return S.gather_sum(xs, s, d, ws, n)
        x = torch.randn(N, F, generator=g)
        out = _host_twins.host_step(hc, x[plan.lo:plan.hi].contiguous(), agg)
        want = S.gather_sum(x, ei[0], ei[1], w, N)[plan.lo:plan.hi]
        terms = S.gather_sum(x.abs(), ei[0], ei[1], w, N)[plan.lo:plan.hi]
        ok_f = bool(((out - want).abs() <= 1e-5 * terms.clamp(min=1.0)).all())
        xi = torch.randint(-8, 9, (N, F), generator=g).to(torch.float32)
        wi = torch.randint(1, 4, (E,), generator=g).to(torch.float32)
        hci = mdist.HaloCover(plan, wi[plan.edge_pos])
        outi = _host_twins.host_step(hci, xi[plan.lo:plan.hi].contiguous(), agg)
        ok_i = torch.equal(outi, S.gather_sum(xi, ei[0], ei[1], wi, N)[plan.lo:plan.hi])
        pull_rows = plan.n_local_src - plan.n_own
        edges_ok = (hc.n_pull_edges + hc.n_push_edges + int(hc.int_src.numel()) == int(plan.edge_pos.numel()))
        result_q.put((rank, ok_f and ok_i and edges_ok and hc.n_halo <= pull_rows,
                       (ok_f, ok_i, edges_ok), hc.n_halo, pull_rows, hc.n_push_rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,cuts", [(1, None), (2, None), (3, None), (4, None), (3, [0, 600, 600, 1200])])
def test_halo_cover_matches_single_process(world, cuts):
    res = run_ranks(_cover_worker, world, timeout=180, args=(cuts,))
    assert all(r[1] for r in res), res
    if world > 1:
        # fewer rows than the pull exchange (this small graph is dense: ~0.86x; RMAT21 0.57x)
        assert sum(r[3] for r in res) < 0.95 * sum(r[4] for r in res), res
        assert any(r[5] > 0 for r in res), res


def _cover_fuzz_worker(rank, world, port, result_q, n_cases):
    """Random graphs and cuts (empty ranks, isolated nodes, duplicate edges,
    self loops, star hubs, a fully-connected tail): the cover's step on
    integer-valued data equals the oracle bit for bit, every in-edge is
    accounted for exactly once, and the cover never ships more rows than the
    pull halo.  Every rank draws the same cases from the same seeds."""
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
        from tests import _host_twins
        _host_twins.install()   # host twins of the native kernels (no CPU fallback in mi355_mp)
        from oracle import scatter_ref as S
        bad = []
        for case in range(n_cases):
            g = torch.Generator().manual_seed(1000 + case)
            N = int(torch.randint(1, 300, (1,), generator=g))
            E = int(torch.randint(0, 3000, (1,), generator=g))
            kind = case % 3
            if kind == 0:      # uniform
                ei = torch.randint(N, (2, E), generator=g)
            elif kind == 1:    # star hubs: a few sources / destinations carry most edges
                hubs = torch.randint(N, (3,), generator=g)
                src = torch.where(torch.rand(E, generator=g) < 0.5, hubs[torch.randint(3, (E,), generator=g)],
                                  torch.randint(N, (E,), generator=g))
                dst = torch.where(torch.rand(E, generator=g) < 0.5, hubs[torch.randint(3, (E,), generator=g)],
                                  torch.randint(N, (E,), generator=g))
                ei = torch.stack([src, dst])
            else:              # dense tail block + duplicates
                k = max(1, min(N, 20))
                a = torch.arange(N - k, N)
                blk = torch.stack([a.repeat_interleave(k), a.repeat(k)])
                ei = torch.cat([torch.randint(N, (2, E), generator=g), blk, blk[:, :E % (k * k + 1)]], 1)
            cuts = sorted(int(c) for c in torch.randint(0, N + 1, (world - 1,), generator=g))
            cuts = [0] + cuts + [N]
            w = torch.randint(1, 4, (ei.shape[1],), generator=g).to(torch.float32)
            x = torch.randint(-8, 9, (N, 3), generator=g).to(torch.float32)
            plan = mdist.ShardPlan(ei, N, rank, world, cuts=cuts).exchange_requests()
            hc = mdist.HaloCover(plan, w[plan.edge_pos])
            out = _host_twins.host_step(hc, x[plan.lo:plan.hi].contiguous(),
                               lambda xs, s, d, ws, n: S.gather_sum(xs, s, d, ws, n))
            want = S.gather_sum(x, ei[0], ei[1], w, N)[plan.lo:plan.hi]
            n_edges = hc.n_pull_edges + hc.n_push_edges + int(hc.int_src.numel())
            if not (torch.equal(out, want) and n_edges == int(plan.edge_pos.numel())
                    and hc.n_halo <= plan.n_local_src - plan.n_own):
                bad.append((case, N, ei.shape[1], cuts))
        result_q.put((rank, bad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_halo_cover_fuzz(world):
    res = run_ranks(_cover_fuzz_worker, world, timeout=300, args=(30,))
    assert all(not r[1] for r in res), res


def _host_gat(graph, ei, xw, att, H, C, slope, bias, return_alpha, dropout):
    """GATConv.message + utils.softmax + scatter_add + update on a rank's local
    graph, in the oracle's own arithmetic ((cat[x_i, x_j] * att).sum(-1), the
    serial CPU segment max / sum): the local op the HIP path runs on the GPU."""
    import torch.nn.functional as F
    from oracle import pyg_ref as P, scatter_ref as S
    n = graph.n_dst
    x_i = xw.index_select(0, ei[1]).view(-1, H, C)
    x_j = xw.index_select(0, ei[0]).view(-1, H, C)
    alpha = F.leaky_relu((torch.cat([x_i, x_j], dim=-1) * att).sum(dim=-1), slope)
    alpha = P.softmax(alpha, ei[1], n)
    out = S.scatter_sum(x_j * alpha.view(-1, H, 1), ei[1], n).view(-1, H * C)
    if bias is not None:
        out = out + bias
    return out, (alpha if return_alpha else None)


def _gat_worker(rank, world, port, result_q):
    """Sharded GATConv (ShardedGraph.for_gat / for_gat_from_slices +
    ShardedGATConv) on the CPU: every rank's output rows and attention weights
    (by GLOBAL edge id) bit-equal to the single-process oracle (a rank holds all
    in-edges of its rows, in global order), and the backward (halo gradients
    returned to their owners) within 1e-5 of the single-process autograd."""
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
        from tests import _host_twins
        _host_twins.install()   # host twins of the native kernels (no CPU fallback in mi355_mp)
        from mi355_mp.graphgen import powerlaw_edge_index
        from oracle import pyg_ref as P
        N, E, Fi, H, C = 600, 8000, 6, 3, 4
        ei = powerlaw_edge_index(N, E, seed=61)
        g = torch.Generator().manual_seed(61)
        ei = torch.cat([ei, torch.stack([torch.arange(5), torch.arange(5)])], 1)   # pre-existing loops
        ei = ei[:, torch.randperm(ei.shape[1], generator=g)]
        E = ei.shape[1]
        x = torch.randn(N, Fi, generator=g)
        gout = torch.randn(N, H * C, generator=g)
        conv = mdist.ShardedGATConv(Fi, C, heads=H)
        with torch.no_grad():
            conv.bias.normal_(generator=g)
        mdist.broadcast_parameters(conv)
        W, att, b = conv.weight.detach(), conv.att.detach(), conv.bias.detach()
        res = {}
        sg = mdist.ShardedGraph.for_gat(ei, N, rank, world)
        s0, s1 = rank * E // world, (rank + 1) * E // world
        sgs = mdist.ShardedGraph.for_gat_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
        res["slices_equal"] = (sgs.fwd.cuts == sg.fwd.cuts and sgs.n_edges == sg.n_edges
                               and torch.equal(sgs.fwd.local_edge_index, sg.fwd.local_edge_index)
                               and torch.equal(sgs.fwd.edge_gid, sg.fwd.edge_pos))
        lo, hi = sg.lo, sg.hi
        # forward rows and alpha (global edge ids) vs the single-process oracle
        want, ei_l, alpha_want = P.gat_conv(x, ei, W, att, b, H, C, return_alpha=True)
        xo = x[lo:hi].clone().requires_grad_(True)
        out, (gid, alpha) = conv(xo, sgs, return_attention_weights=True, local_gat=_host_gat)
        res["out_equal"] = bool(torch.equal(out.detach(), want[lo:hi]))
        res["alpha_equal"] = bool(torch.equal(alpha.detach(), alpha_want[gid]))
        # backward: d x (halo gradients returned to their owners), d W / d att / d b all-reduced
        (out * gout[lo:hi]).sum().backward()
        mdist.allreduce_gradients(conv)
        xr = x.clone().requires_grad_(True)
        Wr, attr, br = (t.clone().requires_grad_(True) for t in (W, att, b))
        (P.gat_conv(xr, ei, Wr, attr, br, H, C) * gout).sum().backward()

        # d x element-wise; the replicated parameters' gradients are sums over all
        # rows regrouped by rank (then all-reduced): normwise, as ShardedGCNConv's
        res["gx"] = float(((xo.grad - xr.grad[lo:hi]).abs() - 1e-5 * xr.grad[lo:hi].abs().clamp(min=1.0)).max())
        for k, a, r in (("gw", conv.weight.grad, Wr.grad), ("gatt", conv.att.grad, attr.grad),
                        ("gb", conv.bias.grad, br.grad)):
            res[k] = float((a - r).abs().max() - 1e-5 * r.abs().max())
        result_q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_sharded_gat_matches_single_process(world):
    res = run_ranks(_gat_worker, world, timeout=180)
    for rank, r in res:
        assert r["slices_equal"] and r["out_equal"] and r["alpha_equal"], r
        assert r["gx"] <= 0 and r["gw"] <= 0 and r["gatt"] <= 0 and r["gb"] <= 0, r


def _bad_slice_worker(rank, world, port, result_q):
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
        from tests import _host_twins
        _host_twins.install()   # host twins of the native kernels (no CPU fallback in mi355_mp)
        N = 50
        ei = torch.randint(N, (2, 400), generator=torch.Generator().manual_seed(3))
        ei[1, 390] = N + 4                          # only the LAST rank's slice holds the bad id
        s0, s1 = rank * 400 // world, (rank + 1) * 400 // world
        raised = []
        for fn in (mdist.ShardedGraph.for_gcn_from_slices, mdist.ShardedGraph.for_gat_from_slices):
            try:
                fn(ei[:, s0:s1].clone(), s0, N, rank, world)
                raised.append(False)
            except IndexError:
                raised.append(True)
        # a slice offset that does not follow the earlier slices (only the last
        # rank's is off by one): every rank raises, none waits in a collective
        ei[1, 390] = 1
        off = s0 + (1 if rank == world - 1 else 0)
        for fn in (mdist.ShardedGraph.for_gcn_from_slices, mdist.ShardedGraph.for_gat_from_slices):
            try:
                fn(ei[:, s0:s1].clone(), off, N, rank, world)
                raised.append(False)
            except ValueError as e:
                raised.append("rank %d's slice offset" % (world - 1) in str(e))
        result_q.put((rank, raised))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_slice_build_rejects_out_of_range_ids_on_every_rank(world):
    """An edge id outside [0, N) in one rank's slice: every rank raises
    IndexError before the first collective whose size depends on N (no hang, no
    all_reduce of vectors of different lengths).  A slice offset out of step
    with the earlier slices on one rank: every rank raises ValueError naming
    that rank (the offsets travel with the slice sizes)."""
    res = run_ranks(_bad_slice_worker, world, timeout=120)
    assert all(r[1] == [True, True, True, True] for r in res), res


def _tiny_worker(rank, world, port, result_q, N, edges):
    """Degenerate shards built from per-rank slices: fewer edges than ranks
    (empty slices), ranks that own no rows, a graph with no edges at all."""
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
        from tests import _host_twins
        _host_twins.install()   # host twins of the native kernels (no CPU fallback in mi355_mp)
        from oracle import pyg_ref as P, scatter_ref as S
        ei = torch.tensor(edges, dtype=torch.long).view(2, -1)
        E = ei.shape[1]
        s0, s1 = rank * E // world, (rank + 1) * E // world
        sg = mdist.ShardedGraph.for_gcn_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
        ei2, norm = P.gcn_norm(ei, N, None, False)
        x = torch.randn(N, 3, generator=torch.Generator().manual_seed(7))

        def local_aggregate(xl, lei, n_dst, n_src, wl):
            return S.gather_sum(xl, lei[0], lei[1], wl, n_dst)
        out = mdist.sharded_propagate(sg.fwd, x[sg.lo:sg.hi].contiguous(), local_aggregate,
                                      lambda t, idx: t[idx], edge_weight=sg.norm_fwd)
        want = S.gather_sum(x, ei2[0], ei2[1], norm, N)[sg.lo:sg.hi]
        result_q.put((rank, bool(torch.equal(out, want)) and sg.n_edges == ei2.shape[1], sg.lo, sg.hi))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,edges", [
    (4, 5, [[0, 3], [1, 4]]),          # 2 edges over 4 ranks: empty slices
    (3, 4, [[], []]),                  # no edges at all: loops only
    (3, 1, [[0], [0]]),                # one node: two ranks own nothing
    (2, 6, [[5, 5, 5, 4], [0, 1, 2, 5]]),
])
def test_slice_built_shards_degenerate_graphs(world, N, edges):
    res = run_ranks(_tiny_worker, world, timeout=120, args=(N, edges,))
    assert all(r[1] for r in res), res
    assert sum(r[3] - r[2] for r in res) == N


def _grad_flags_worker(rank, world, port, result_q):
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
        from tests import _host_twins
        _host_twins.install()   # host twins of the native kernels (no CPU fallback in mi355_mp)
        m = torch.nn.Linear(3, 2)
        m.extra = torch.nn.Parameter(torch.ones(4))      # no rank forms a gradient for it
        m.only0 = torch.nn.Parameter(torch.ones(2))      # only rank 0 does
        x = torch.full((5, 3), float(rank + 1))
        loss = m(x).sum()
        if rank == 0:
            loss = loss + (m.only0 * 3).sum()
        loss.backward()
        mdist.allreduce_gradients(m)
        result_q.put((rank, m.extra.grad is None, m.only0.grad.tolist(), m.bias.grad.tolist(),
                      m.weight.grad.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allreduce_gradients_keeps_unused_parameters_gradless(world):
    """allreduce_gradients: a parameter no rank has a gradient for
    keeps grad None on every rank (an optimizer with weight decay / momentum
    leaves it alone, as on one GPU); one some ranks lack is summed with zeros
    from those ranks; the rest are plain sums."""
    res = run_ranks(_grad_flags_worker, world, timeout=120)
    s = sum(range(1, world + 1))
    for rank, extra_none, only0, b, w in res:
        assert extra_none
        assert only0 == [3.0, 3.0]
        assert b == [5.0 * world] * 2
        assert w == [[5.0 * s] * 3] * 2


def _gat_cover_worker(rank, world, port, result_q, from_slices, cuts):
    """Sharded GATConv over the hybrid halo cover (mi355_mp.gat_cover) on the
    CPU in float64: the host form of the distributed algorithm (a_dst requests,
    pushed online-softmax pieces, the merge; autograd through a differentiable
    all_to_all) against the single-process oracle, forward rows and every
    gradient; the cover ships no more rows than the pull plan."""
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
        from tests import _host_twins
        _host_twins.install()   # host twins of the native kernels (no CPU fallback in mi355_mp)
        from mi355_mp.graphgen import powerlaw_edge_index
        from oracle import pyg_ref as P
        torch.set_default_dtype(torch.float64)
        N, E, Fi = 700, 9000, 6
        ei = powerlaw_edge_index(N, E, seed=67)
        g = torch.Generator().manual_seed(67)
        # hub destinations and hub sources: rows both pushed and pulled
        ei = torch.cat([ei, torch.stack([torch.randint(0, N, (600,), generator=g), torch.full((600,), 5)]),
                        torch.stack([torch.full((400,), 650), torch.randint(0, N, (400,), generator=g)])], 1)
        ei = ei[:, torch.randperm(ei.shape[1], generator=g)]
        E = ei.shape[1]
        x = torch.randn(N, Fi, generator=g)
        res = {}
        for H, C, concat in ((3, 4, True), (2, 8, False), (1, 6, True)):
            conv = mdist.ShardedGATConv(Fi, C, heads=H, concat=concat)
            with torch.no_grad():
                conv.bias.normal_(generator=g)
                conv.att.mul_(3.0)          # sharper softmax: the pieces' maxima differ
            mdist.broadcast_parameters(conv)
            W, att, b = conv.weight.detach(), conv.att.detach(), conv.bias.detach()
            if from_slices:
                s0, s1 = rank * E // world, (rank + 1) * E // world
                sg = mdist.ShardedGraph.for_gat_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
            else:
                sg = mdist.ShardedGraph.for_gat(ei, N, rank, world, cuts=cuts)
            pull_rows = sg.fwd.n_local_src - sg.n_own
            sg.enable_gat_halo_cover()
            st = sg.gat_cover.stats()
            lo, hi = sg.lo, sg.hi
            Fo = H * C if concat else C
            gout = torch.randn(N, Fo, generator=g)
            xo = x[lo:hi].clone().requires_grad_(True)
            out = conv(xo, sg)
            (out * gout[lo:hi]).sum().backward()
            mdist.allreduce_gradients(conv)
            xr = x.clone().requires_grad_(True)
            Wr, attr, br = (t.clone().requires_grad_(True) for t in (W, att, b))
            want = P.gat_conv(xr, ei, Wr, attr, br, H, C, concat=concat)
            (want * gout).sum().backward()
            tol = 1e-10
            r = {"out": float(((out.detach() - want.detach()[lo:hi]).abs()
                               - tol * want.detach()[lo:hi].abs().clamp(min=1.0)).max()) if hi > lo else -1.0,
                 "gx": float(((xo.grad - xr.grad[lo:hi]).abs() - tol * xr.grad[lo:hi].abs().clamp(min=1.0)).max())
                 if hi > lo else -1.0,
                 "halo_rows": st["halo_rows"], "pull_rows": pull_rows, "pushed": st["cover_partial_rows"]}
            for k, a, rr in (("gw", conv.weight.grad, Wr.grad), ("gatt", conv.att.grad, attr.grad),
                             ("gb", conv.bias.grad, br.grad)):
                r[k] = float((a - rr).abs().max() - tol * rr.abs().max())
            res[(H, C, concat)] = r
        result_q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,from_slices,cuts", [(1, False, None), (2, False, None), (3, True, None),
                                                     (3, False, [0, 0, 350, 700]), (4, False, None)])
def test_sharded_gat_over_halo_cover_matches_single_process(world, from_slices, cuts):
    """GAT over the hybrid cover, float64 on the CPU: every rank's rows and the
    all-reduced d W / d att / d b, and d x of its rows, within 1e-10 of the
    single-process oracle (pieces merge exactly up to rounding); ranks that own
    no rows take part; pieces are pushed (the cover is not the pull plan) and
    the halo is never larger than the pull plan's."""
    res = run_ranks(_gat_cover_worker, world, timeout=300, args=(from_slices, cuts))
    pushed = 0
    for rank, r in res:
        for key, v in r.items():
            for k in ("out", "gx", "gw", "gatt", "gb"):
                assert v[k] <= 0, (rank, key, k, v)
            assert v["halo_rows"] <= v["pull_rows"], (rank, key, v)
            pushed += v["pushed"]
    if world > 1:
        assert pushed > 0, res
