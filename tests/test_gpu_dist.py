"""Sharded aggregation on the GPU with two ranks sharing one device (gloo:
halo rows staged through the host -- the RCCL call is the only part not
exercised).  Checks the overlapped interior/boundary path and the plain
exchange-then-aggregate path against the single-GPU result."""
import datetime
import os
import socket

import pytest
import torch
import torch.distributed as dist

from tests._ranks import DEFAULT_TIMEOUT, run_ranks

# gloo process groups of the spawned ranks: rendezvous and collectives give up
# after this (a lost peer fails the test instead of stalling the suite)
_PG_TIMEOUT = datetime.timedelta(seconds=240)

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _fused_forms_equal(ov, x_own, out_ref, bias, F):
    """step_fused over every (tile width, boundary in one launch / per tile,
    interior after / beside the packing, send rows packed in one launch / per
    tile) form: bitwise out_ref (step()'s output).  Returns the list of forms
    that differ (empty: all equal)."""
    bad = []
    for width in (64, 128, 256):
        bufs = ov.halo_buffers(F, width)
        for one in (True, False):
            for split in (False, True):
                for ppt in ((False, True) if width < F else (False,)):
                    ov.one_boundary_launch, ov.split_interior, ov.pack_per_tile = one, split, ppt
                    for _ in range(2):   # twice: the result never depends on the buffers' last contents
                        o = torch.full_like(out_ref, float("nan"))
                        ov.step_fused(x_own, bufs, o, bias)
                        if not torch.equal(o, out_ref):
                            bad.append((width, one, split, ppt))
                            break
    ov.one_boundary_launch, ov.split_interior, ov.pack_per_tile = True, False, False
    return bad


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import Graph
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn.conv.gcn_conv import GCNConv
        dev = torch.device("cuda", 0)
        N, E, F = 3000, 60000, 256
        ei = powerlaw_edge_index(N, E, seed=31).to(dev)
        ei2, norm = GCNConv.norm(ei, N)
        x = torch.randn(N, F, generator=torch.Generator().manual_seed(31)).to(dev)
        bias = torch.randn(F, generator=torch.Generator().manual_seed(32)).to(dev)
        g = Graph(ei2, N, N, chunk=64)
        ref = ops._aggregate(g.dst, "other", x, g.dst.to_csr_order(norm), "sum", 0, bias)[0]
        plan = mdist.ShardPlan(ei2, N, rank, world).exchange_requests()
        xl = plan.local_buffer(F)
        xl[:plan.n_own].copy_(x[plan.lo:plan.hi])
        ov = mdist.OverlappedAggregation(plan, norm, chunk=64)
        out = torch.empty(plan.n_own, F, device=dev)
        ov.step(xl, out, bias)
        want = ref[plan.lo:plan.hi]
        err = (out - want).abs().max().item()
        # plain path: bit-equal to the single-GPU kernel (same per-row order)
        gl = Graph(plan.local_edge_index, plan.n_own, plan.n_local_src, chunk=64)
        xl2 = plan.exchange_into(xl, ops.gather_rows)
        out2 = ops._aggregate(gl.dst, "other", xl2, gl.dst.to_csr_order(norm[plan.edge_pos]), "sum", 0, bias)[0]
        # feature-tile pipeline: bitwise the same as step()
        tiles = plan.local_tiles(F, 128)
        for t, xt in enumerate(tiles):
            xt[:plan.n_own].copy_(x[plan.lo:plan.hi, 128 * t:128 * t + xt.shape[1]])
        out3 = torch.empty(plan.n_own, F, device=dev)
        ov.step_tiled(tiles, out3, bias)
        assert torch.equal(out3, out), "step_tiled must equal step"
        # the interior passes on the side stream beside the send packing: the same
        # arithmetic, so bitwise the same output, every time (ordering, not luck)
        ov.split_interior = True
        for _ in range(3):
            out4 = torch.full_like(out, float("nan"))
            ov.step_tiled(tiles, out4, bias)
            assert torch.equal(out4, out), "split_interior must equal step"
        ov.split_interior = False
        # the fused step (one launch per pass, own rows read in place, tile-major halo
        # buffers, out values prefetched with the batch's gathers, rows without
        # boundary edges skipped): bitwise step()'s output in every form
        bad = _fused_forms_equal(ov, xl[:plan.n_own], out, bias, F)
        assert not bad, ("step_fused differs from step", bad)
        # ... and without a bias (the skipped rows keep the interior sums as they are)
        out_nb = torch.empty_like(out)
        ov.step(xl, out_nb, None)
        assert not _fused_forms_equal(ov, xl[:plan.n_own], out_nb, None, F)
        q.put((rank, err, bool(torch.equal(out2, want)), ov.n_interior, ov.n_boundary))
    finally:
        dist.destroy_process_group()


def test_overlapped_sharded_gcn_on_one_gpu():
    res = _spawn(_worker, world=2, timeout=300)
    for rank, err, exact, n_int, n_bnd in res:
        assert err < 1e-5, res
        assert n_int > 0 and n_bnd > 0
    # unsplit rows bit-exact; split hub rows may differ in the last bits
    assert all(r[2] or r[1] < 1e-6 for r in res), res


def _layer_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import Graph
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn import GCNConv
        dev = torch.device("cuda", 0)
        N, E, Fi, Fo = 3000, 60000, 64, 256
        ei = powerlaw_edge_index(N, E, seed=41).to(dev)
        gen = torch.Generator().manual_seed(41)
        x = torch.randn(N, Fi, generator=gen).to(dev)
        gout = torch.randn(N, Fo, generator=gen).to(dev)
        ref = GCNConv(Fi, Fo).to(dev)
        with torch.no_grad():
            ref.bias.normal_()
        mdist.broadcast_parameters(ref)   # replicated weights: rank 0's values everywhere
        xr = x.clone().requires_grad_(True)
        out_ref = ref(xr, ei)
        (out_ref * gout).sum().backward()
        sg = mdist.ShardedGraph.for_gcn(ei, N, rank, world)
        # the same shards built from per-rank slices of the edge list (native
        # serial degree, exact deg^-1/2, degree halo exchange): bit-equal plans and norms
        s0, s1 = rank * ei.shape[1] // world, (rank + 1) * ei.shape[1] // world
        sgs = mdist.ShardedGraph.for_gcn_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
        slices_equal = (sgs.fwd.cuts == sg.fwd.cuts and sgs.n_edges == sg.n_edges
                        and torch.equal(sgs.fwd.local_edge_index, sg.fwd.local_edge_index)
                        and torch.equal(sgs.fwd.edge_gid, sg.fwd.edge_pos)
                        and torch.equal(sgs.bwd.local_edge_index, sg.bwd.local_edge_index)
                        and torch.equal(sgs._w[0], sg._w[0]) and torch.equal(sgs._w[1], sg._w[1]))
        conv = mdist.ShardedGCNConv(Fi, Fo).to(dev)
        conv.load_state_dict(ref.state_dict())
        lo, hi = sg.lo, sg.hi
        xo = x[lo:hi].clone().requires_grad_(True)
        out = conv(xo, sg)
        (out * gout[lo:hi]).sum().backward()
        mdist.allreduce_gradients(conv)
        out, out_ref = out.detach(), out_ref.detach()
        res = {
            "out": float((out - out_ref[lo:hi]).abs().max()),
            "out_bitwise_frac": float((out == out_ref[lo:hi]).float().mean()),
            "gx": float((xo.grad - xr.grad[lo:hi]).abs().max()),
            "gx_bitwise_frac": float((xo.grad == xr.grad[lo:hi]).float().mean()),
            "gw": float((conv.weight.grad - ref.weight.grad).abs().max() / ref.weight.grad.abs().max()),
            "gb": float((conv.bias.grad - ref.bias.grad).abs().max() / ref.bias.grad.abs().max()),
        }
        # max / min with GLOBAL edge ids through the sharded graph, vs the single-GPU kernel
        xi = torch.randint(-3, 4, (N, Fo), generator=gen).to(torch.float32).to(dev)
        from torch_geometric.nn.conv.gcn_conv import GCNConv as G
        ei2, _ = G.norm(ei, N)
        sgm = mdist.ShardedGraph(ei2, N, rank, world)
        g1 = Graph(ei2, N, N)
        exact = True
        for red in ("max", "min"):
            o, a = sgm.propagate(xi[lo:hi], red)
            wo, wa = ops._aggregate(g1.dst, "other", xi, None, red, 0, None)
            exact = exact and bool(torch.equal(o, wo[lo:hi])) and bool(torch.equal(a, wa[lo:hi]))
        # max backward: gradient reaches remote argmax sources through return_halo.
        # Gradients on a 1/8 grid keep every partial sum exact, so the sharded
        # order (local edge order, then the peers' rows in peer order) must give
        # the single-GPU result bit for bit; random ones must repeat bit for bit.
        gq = torch.round(gout * 8) / 8
        grads = []
        for gg in (gq, gq, gout, gout):
            xm = xi[lo:hi].clone().requires_grad_(True)
            om, _ = sgm.propagate(xm, "max")
            (om * gg[lo:hi]).sum().backward()
            grads.append(xm.grad)
        xf = xi.clone().requires_grad_(True)
        of = ops.fused_propagate(Graph(ei2, N, N), xf, ei2, None, "max")
        (of * gq).sum().backward()
        res["gmax_exact"] = bool(torch.equal(grads[0], xf.grad[lo:hi]))
        res["gmax_repeat"] = bool(torch.equal(grads[0], grads[1])) and bool(torch.equal(grads[2], grads[3]))
        res["max_exact"] = exact
        res["slices_equal"] = bool(slices_equal)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _spawn(target, world=2, timeout=None, args=()):
    """tests._ranks.run_ranks: the ranks' own deadline (below pytest.ini's
    session-aborting backstop), every rank terminated when one fails."""
    return run_ranks(target, world, timeout=timeout or DEFAULT_TIMEOUT, args=args)


def test_sharded_gcnconv_forward_backward_on_one_gpu():
    """ShardedGCNConv over a ShardedGraph (2 ranks sharing the device, halo
    rows staged through gloo): forward rows, d x (backward = transposed-plan
    propagate) and the all-reduced d W / d b against the single-GPU GCNConv;
    sharded max / min values and GLOBAL argmax ids bit-equal to the single-GPU
    kernel, and the max backward through return_halo."""
    res = _spawn(_layer_worker)
    for rank, r in res:
        # tolerance only: the rank's x @ W has M = n_own rows, and hipBLASLt picks
        # its GEMM kernel (and so its k-order) by M; d x also sums the local and the
        # returned halo contributions separately.  The bitwise fractions are
        # reported, not asserted (round 2 saw 0.93 / 0.70 on a fresh box).
        assert r["out"] < 1e-5 and r["gx"] < 1e-5, r
        assert r["gw"] < 1e-5 and r["gb"] < 1e-5, r
        assert r["max_exact"], r
        assert r["slices_equal"], r
        assert r["gmax_exact"] and r["gmax_repeat"], r   # deterministic on both sides (round 3)


def _learn_w_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import Graph
        from mi355_mp.graphgen import powerlaw_edge_index
        dev = torch.device("cuda", 0)
        N, E, F = 2000, 30000, 32
        ei = powerlaw_edge_index(N, E, seed=57).to(dev)
        gen = torch.Generator().manual_seed(57)
        x = torch.randn(N, F, generator=gen).to(dev)
        w0 = torch.rand(E, generator=gen).to(dev) + 0.5
        gout = torch.randn(N, F, generator=gen).to(dev)
        g1 = Graph(ei, N, N)
        res = {}
        for red in ("sum", "mean", "max", "min"):
            # single GPU: the fused propagate with the weights differentiated
            xr, wr = x.clone().requires_grad_(True), w0.clone().requires_grad_(True)
            ref = ops.fused_propagate(g1, xr, ei, wr, red)
            ref = ref[0] if isinstance(ref, tuple) else ref
            (ref * gout).sum().backward()
            sg = mdist.ShardedGraph(ei, N, rank, world)
            lo, hi = sg.lo, sg.hi
            xo, w = x[lo:hi].clone().requires_grad_(True), w0.clone().requires_grad_(True)
            o = sg.propagate(xo, red, edge_weight=w)
            o = o[0] if isinstance(o, tuple) else o
            (o * gout[lo:hi]).sum().backward()
            # regrouped sums on hub rows (the two graphs' merge-path tasks split them
            # differently): relative to the largest magnitude; max / min bit-exact
            sc_o = float(ref.detach().abs().max().clamp(min=1.0))
            sc_g = float(xr.grad.abs().max().clamp(min=1.0))
            res[red] = {"out": float((o.detach() - ref.detach()[lo:hi]).abs().max()) / sc_o if hi > lo else 0.0,
                        "gx": float((xo.grad - xr.grad[lo:hi]).abs().max()) / sc_g if hi > lo else 0.0,
                        "out_exact": bool(torch.equal(o.detach(), ref.detach()[lo:hi]))}
            # the rank's own in-edges carry its share; the sum over ranks is the full gradient
            gw_h = w.grad.cpu()
            dist.all_reduce(gw_h)
            res[red]["gw"] = float((gw_h.to(dev) - wr.grad).abs().max() / wr.grad.abs().max().clamp(min=1e-30))
            res[red]["own_edges_only"] = bool((w.grad[~torch.isin(torch.arange(E, device=dev), sg.fwd.edge_pos)]
                                               == 0).all())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_sharded_propagate_learnable_edge_weights():
    """ShardedGraph.propagate(x, reduce, edge_weight=w) with w requiring grad
    (VERDICT r05 missing 5): forward rows and d x against the single-GPU fused
    propagate with the same weights differentiated; each rank writes d w on its
    own in-edges only, and their sum over the ranks is the single-GPU d w --
    sum, mean and max / min (winning edges), 2 ranks sharing the GPU."""
    res = _spawn(_learn_w_worker)
    for rank, r in res:
        for red, v in r.items():
            assert v["out"] < 1e-5 and v["gx"] < 1e-5, (rank, red, v)
            assert v["gw"] < 1e-5, (rank, red, v)
            assert v["own_edges_only"], (rank, red, v)
            if red in ("max", "min"):
                assert v["out_exact"], (rank, red, v)


def _gat_alpha_cover_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn import GATConv
        dev = torch.device("cuda", 0)
        N, Fi = 1500, 24
        ei = powerlaw_edge_index(N, 20000, seed=83).to(dev)
        gen = torch.Generator().manual_seed(83)
        x = _gauss_(torch.empty(N, Fi), gen, 4.0).to(dev)
        res = {}
        for H, C in ((4, 16), (2, 24)):
            ref = GATConv(Fi, C, heads=H).to(dev)
            _gauss_(ref.weight, gen, 16.0)             # the same weights on every rank
            with torch.no_grad():
                ref.att.copy_(torch.randn(ref.att.shape, generator=gen) * 0.3)
                ref.bias.copy_(torch.randn(ref.bias.shape, generator=gen))
            out_ref, (_, a_ref) = ref(x, ei, return_attention_weights=True)
            conv = mdist.ShardedGATConv(Fi, C, heads=H).to(dev)
            conv.load_state_dict(ref.state_dict())
            for cover in (False, True):
                sg = mdist.ShardedGraph.for_gat(ei, N, rank, world)
                if cover:
                    sg.enable_gat_halo_cover()
                xo = x[sg.lo:sg.hi].clone().requires_grad_(True)
                out, (gid, alpha) = conv(xo, sg, return_attention_weights=True)
                out.sum().backward()           # the training path (autograd Function) returns alpha too
                with torch.no_grad():
                    out2, (gid2, alpha2) = conv(xo, sg, return_attention_weights=True)
                res["%dx%d %s" % (H, C, "cover" if cover else "pull")] = {
                    "alpha": float((alpha - a_ref[gid]).abs().max()) if alpha.numel() else 0.0,
                    "alpha_nograd_equal": bool(torch.equal(alpha, alpha2)) and bool(torch.equal(gid, gid2)),
                    "n": int(alpha.shape[0]), "rows_ok": bool(torch.equal(gid, sg.fwd.edge_gid))}
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gatconv_return_alpha_over_cover(world):
    """ShardedGATConv(return_attention_weights=True) over the hybrid cover
    (VERDICT r05 item 4): every in-edge's alpha -- the local piece's from the
    merged row statistics, a pushed edge's evaluated by its pusher with the
    destination's merged statistics and sent back -- within 1e-5 of the
    single-GPU layer's alpha at the same global edge id, as over the pull
    exchange; fused and wide heads; the training and no-grad paths agree."""
    res = _spawn(_gat_alpha_cover_worker, world=world)
    for rank, r in res:
        for key, v in r.items():
            assert v["alpha"] < 1e-5 and v["alpha_nograd_equal"] and v["rows_ok"], (rank, key, v)


def _unsplit_equal(sg, g1, alpha, alpha_ref, out, out_ref):
    """Bit-equality of the sharded GAT and the single-GPU kernel where both
    schedules keep a row whole: a row of <= snap in-edges is never split across
    merge-path tasks (graph.default_snap), so its softmax and weighted sum run
    in one task in global edge order on both sides.  Hub rows above either
    schedule's snap may be cut at different slots (partials merged by the
    fix-up), and are held to the tolerance only.  Returns (every alpha of the
    rank's edges into such rows equal, every such output row equal)."""
    loc = sg.g_fwd.dst
    deg = (loc.rowptr[1:] - loc.rowptr[:-1]).long()
    whole = deg <= min(loc.snap, g1.dst.snap)
    dst = sg.fwd.local_edge_index[1].long()
    ok_e = whole[dst]
    a_eq = bool(torch.equal(alpha[ok_e], alpha_ref[ok_e])) and int(ok_e.sum()) > 0
    o_eq = bool(torch.equal(out[whole], out_ref[whole])) and int(whole.sum()) > 0
    return a_eq, o_eq


def _gat_layer_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import GAT_TARGET_TASKS, Graph
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn import GATConv
        from torch_geometric.nn.conv._structure import gat_loops
        dev = torch.device("cuda", 0)
        N, E, Fi = 3000, 60000, 64
        ei = powerlaw_edge_index(N, E, seed=47).to(dev)
        gen = torch.Generator().manual_seed(47)
        # Gaussian x and W: the row-exact GEMM gives the rank the single-GPU rows of X W (_gauss_)
        x = _gauss_(torch.empty(N, Fi), gen, 4.0).to(dev)
        res = {}
        # (heads, out_channels, concat): config 3's shape, the reference's heads=1 stacks
        # (ConvexPruning.py:209-214, a wide head), a padded width, and ppi's mean head
        for H, C, concat in ((8, 32, True), (1, 96, True), (2, 10, True), (3, 8, False)):
            Fo = H * C if concat else C
            gout = torch.randn(N, Fo, generator=gen).to(dev)
            ref = GATConv(Fi, C, heads=H, concat=concat).to(dev)
            _gauss_(ref.weight, gen, 16.0)
            with torch.no_grad():
                ref.att.copy_(torch.randn(ref.att.shape, generator=gen) * 0.3)
                ref.bias.copy_(torch.randn(ref.bias.shape, generator=gen))
            mdist.broadcast_parameters(ref)
            xr = x.clone().requires_grad_(True)
            out_ref = ref(xr, ei)
            (out_ref * gout).sum().backward()
            sg = mdist.ShardedGraph.for_gat(ei, N, rank, world)
            s0, s1 = rank * E // world, (rank + 1) * E // world
            sgs = mdist.ShardedGraph.for_gat_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
            same = (sgs.fwd.cuts == sg.fwd.cuts and torch.equal(sgs.fwd.local_edge_index, sg.fwd.local_edge_index)
                    and torch.equal(sgs.fwd.edge_gid, sg.fwd.edge_pos))
            conv = mdist.ShardedGATConv(Fi, C, heads=H, concat=concat).to(dev)
            conv.load_state_dict(ref.state_dict())
            lo, hi = sg.lo, sg.hi
            xo = x[lo:hi].clone().requires_grad_(True)
            out = conv(xo, sgs)
            (out * gout[lo:hi]).sum().backward()
            mdist.allreduce_gradients(conv)
            r = {"slices_equal": bool(same),
                 "out": float((out.detach() - out_ref.detach()[lo:hi]).abs().max()),
                 "gx": float((xo.grad - xr.grad[lo:hi]).abs().max() / xr.grad.abs().max())}
            for k in ("weight", "att", "bias"):
                a, b = getattr(conv, k).grad, getattr(ref, k).grad
                r["g" + k] = float((a - b).abs().max() / b.abs().max())
            res[(H, C, concat)] = r
        # propagate level, the same X W on both sides: alpha by global edge id and the
        # output rows equal the single-GPU fused kernel except on rows a merge-path
        # task boundary splits (different on the rank's local CSR)
        H, C = 8, 32
        xw = torch.randn(N, H * C, generator=gen).to(dev)
        att = torch.randn(1, H, 2 * C, generator=gen).to(dev) * 0.2
        ei2 = gat_loops(ei, N)
        g1 = Graph(ei2, N, N, target_tasks=GAT_TARGET_TASKS)
        o1, a1 = ops.gat_propagate(g1, ei2, xw, att, H, C, return_alpha=True)
        sg = mdist.ShardedGraph.for_gat(ei, N, rank, world)
        o2, (gid, a2) = sg.gat_propagate(xw[sg.lo:sg.hi].contiguous(), att, H, C, return_alpha=True)
        a_eq, o_eq = _unsplit_equal(sg, g1, a2, a1[gid], o2, o1[sg.lo:sg.hi])
        res["prop"] = {"out": float((o2 - o1[sg.lo:sg.hi]).abs().max()),
                       "alpha": float((a2 - a1[gid]).abs().max()),
                       "alpha_unsplit_bitwise": a_eq, "out_unsplit_bitwise": o_eq}
        # ABI 6: the round-4 fault's sizing -- d att partials for the rank's own rows
        # while the finish pass covers own + halo rows -- is now MP_ERR_ARG from the
        # library, raised before any launch, instead of a device write past the end.
        # (The rank's local GAT backward only: no collective, so every rank checks alone.)
        xl = torch.randn(sg.fwd.n_local_src, H * C, generator=gen).to(dev).requires_grad_(True)
        at = att.clone().requires_grad_(True)
        gl = torch.randn(sg.n_own, H * C, generator=gen).to(dev)
        good = ops._att_part_blocks
        ops._att_part_blocks = lambda n_rows, n_dst: good(n_dst, n_dst)   # the r04 sizing
        rejected = ""
        try:
            o, _ = ops.gat_propagate(sg.g_fwd, sg.fwd.local_edge_index, xl, at, H, C)
            (o * gl).sum().backward()
        except RuntimeError as e:
            rejected = str(e)
        finally:
            ops._att_part_blocks = good
        o, _ = ops.gat_propagate(sg.g_fwd, sg.fwd.local_edge_index, xl, at, H, C)
        (o * gl).sum().backward()
        torch.cuda.synchronize()
        res["short_att_part"] = {"rejected": rejected, "n_local": int(sg.fwd.n_local_src), "n_own": int(sg.n_own),
                                 "finite_after": bool(torch.isfinite(at.grad).all())}
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gatconv_forward_backward_on_one_gpu(world):
    """ShardedGATConv over ShardedGraph.for_gat / for_gat_from_slices (ranks
    sharing the device, halo rows of X W staged through gloo): forward rows,
    d x (the halo rows' gradients returned to their owners) and the all-reduced
    d W / d att / d b against the single-GPU GATConv -- config 3's 8 x 32 heads,
    a heads=1 wide head, a padded width and a mean-of-heads layer; at the
    propagate level, with the same X W, alpha (by global edge id) and the
    output rows bit-equal to the single-GPU kernel on all but split rows."""
    res = _spawn(_gat_layer_worker, world=world)
    for rank, r in res:
        for key, v in r.items():
            if key == "short_att_part":
                # an att_part sized for the own rows is refused whenever the halo adds blocks
                assert v["n_local"] > v["n_own"], v
                assert "mp_gat_backward_finish_f32" in v["rejected"] and "code 1" in v["rejected"], v
                assert "att_part holds" in v["rejected"], v
                assert v["finite_after"], v
                continue
            if key == "prop":
                assert v["out"] < 1e-5 and v["alpha"] < 1e-6, (key, v)
                assert v["out_unsplit_bitwise"] and v["alpha_unsplit_bitwise"], (key, v)
                continue
            assert v["slices_equal"], (key, v)
            # tolerance: the rank's X W GEMM has M = n_own rows (hipBLASLt picks its kernel by M)
            assert v["out"] < 1e-5 and v["gx"] < 1e-5, (key, v)
            assert v["gweight"] < 1e-5 and v["gatt"] < 1e-5 and v["gbias"] < 1e-5, (key, v)


def _gat_uneven_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn import GATConv
        dev = torch.device("cuda", 0)
        N, Fi, H, C = 1500, 24, 4, 16
        ei = powerlaw_edge_index(N, 20000, seed=71).to(dev)
        gen = torch.Generator().manual_seed(71)
        x = _gauss_(torch.empty(N, Fi), gen, 4.0).to(dev)       # X W bitwise on both sides (_gauss_)
        gout = torch.randn(N, H * C, generator=gen).to(dev)
        res = {}
        # an empty rank (cuts [0, N, N]) and a rank holding a single row
        for name, cuts in (("empty_rank", [0, N, N]), ("one_row", [0, 1, N])):
            ref = GATConv(Fi, C, heads=H).to(dev)
            _gauss_(ref.weight, gen, 16.0)
            with torch.no_grad():
                ref.att.copy_(torch.randn(ref.att.shape, generator=gen) * 0.3)
                ref.bias.copy_(torch.randn(ref.bias.shape, generator=gen))
            mdist.broadcast_parameters(ref)
            xr = x.clone().requires_grad_(True)
            out_ref = ref(xr, ei)
            (out_ref * gout).sum().backward()
            sg = mdist.ShardedGraph.for_gat(ei, N, rank, world, cuts=cuts)
            conv = mdist.ShardedGATConv(Fi, C, heads=H).to(dev)
            conv.load_state_dict(ref.state_dict())
            lo, hi = sg.lo, sg.hi
            xo = x[lo:hi].clone().requires_grad_(True)
            out = conv(xo, sg)
            (out * gout[lo:hi]).sum().backward()
            mdist.allreduce_gradients(conv)
            r = {"rows": hi - lo, "out": float((out.detach() - out_ref.detach()[lo:hi]).abs().max()) if hi > lo else 0.0,
                 "gx": float((xo.grad - xr.grad[lo:hi]).abs().max()) if hi > lo else 0.0}
            for k in ("weight", "att", "bias"):
                a, b = getattr(conv, k).grad, getattr(ref, k).grad
                r["g" + k] = float((a - b).abs().max() / b.abs().max())
            res[name] = r
            # GCN on the same cuts: the layer (pull plan), then the hybrid halo cover, then
            # max with global argmax ids, against the single-GPU layer / kernel
            from torch_geometric.nn import GCNConv
            from mi355_mp import ops
            gref = GCNConv(Fi, 32).to(dev)
            with torch.no_grad():
                gref.bias.normal_()
            mdist.broadcast_parameters(gref)
            xr = x.clone().requires_grad_(True)
            gref(xr, ei).square().sum().backward()
            sgc = mdist.ShardedGraph.for_gcn(ei, N, rank, world, cuts=cuts)
            gconv = mdist.ShardedGCNConv(Fi, 32).to(dev)
            gconv.load_state_dict(gref.state_dict())
            xo = x[lo:hi].clone().requires_grad_(True)
            go = gconv(xo, sgc)
            go.square().sum().backward()
            mdist.allreduce_gradients(gconv)
            want = gref(x, ei).detach()[lo:hi]
            r2 = {"rows": hi - lo, "out": float((go.detach() - want).abs().max()) if hi > lo else 0.0,
                  "gx": float((xo.grad - xr.grad[lo:hi]).abs().max()) if hi > lo else 0.0,
                  "gweight": float((gconv.weight.grad - gref.weight.grad).abs().max() / gref.weight.grad.abs().max()),
                  "gatt": 0.0,
                  "gbias": float((gconv.bias.grad - gref.bias.grad).abs().max() / gref.bias.grad.abs().max())}
            h = x @ gref.weight.detach()
            oc = sgc.enable_halo_cover().propagate(h[lo:hi].contiguous())
            r2["cover"] = float((oc - (want - gref.bias.detach())).abs().max()) if hi > lo else 0.0
            sgm = mdist.ShardedGraph(ei, N, rank, world, cuts=cuts)
            om, am = sgm.propagate(h[lo:hi].contiguous(), "max")
            from mi355_mp.graph import Graph
            o1, a1 = ops._aggregate(Graph(ei, N, N).dst, "other", h, None, "max", 0, None)
            r2["max_exact"] = bool(torch.equal(om, o1[lo:hi]) and torch.equal(am, a1[lo:hi]))
            res[name + "_gcn"] = r2
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_sharded_gatconv_uneven_cuts_on_one_gpu():
    """Sharded layers when a rank owns no rows (its local graph has no
    destinations but still sends halo rows and joins every collective) and
    when a rank owns one row: ShardedGATConv and ShardedGCNConv outputs, d x
    and the all-reduced parameter gradients against the single-GPU layers;
    the GCN propagate over the hybrid halo cover; max with global argmax ids
    bit-equal to the single-GPU kernel."""
    res = _spawn(_gat_uneven_worker, world=2)
    for rank, r in res:
        for name, v in r.items():
            assert v["out"] < 1e-5 and v["gx"] < 1e-5, (rank, name, v)
            assert v["gweight"] < 1e-5 and v["gatt"] < 1e-5 and v["gbias"] < 1e-5, (rank, name, v)
            if name.endswith("_gcn"):
                assert v["cover"] < 1e-4 and v["max_exact"], (rank, name, v)
        assert sorted(v["rows"] for k, v in r.items() if k in ("empty_rank", "one_row")) == sorted(
            ({0: 1500, 1: 0}[rank], {0: 1, 1: 1499}[rank]))



def _gat_dropout_worker(rank, world, port, q, cut_sets):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn import GATConv
        dev = torch.device("cuda", 0)
        N, Fi, p = 1500, 24, 0.3
        ei = powerlaw_edge_index(N, 20000, seed=73).to(dev)
        gen = torch.Generator().manual_seed(73)
        x = _gauss_(torch.empty(N, Fi), gen, 4.0).to(dev)
        res = {}
        # heads 4 x 16 (the fused transposed pass) and 2 x 24 (the wide kernels), over
        # the pull exchange and over the hybrid cover
        for H, C in ((4, 16), (2, 24)):
            gout = torch.randn(N, H * C, generator=gen).to(dev)
            for ci, cuts in enumerate(cut_sets):
                for cover in (False, True):
                    ref = GATConv(Fi, C, heads=H, dropout=p).to(dev).train()
                    _gauss_(ref.weight, gen, 16.0)
                    with torch.no_grad():
                        ref.att.copy_(torch.randn(ref.att.shape, generator=gen) * 0.3)
                        ref.bias.copy_(torch.randn(ref.bias.shape, generator=gen))
                    xr = x.clone().requires_grad_(True)
                    torch.manual_seed(11 + ci)                 # the dropout key both layers draw
                    out_ref = ref(xr, ei)
                    (out_ref * gout).sum().backward()
                    if cuts is None:
                        E = ei.shape[1]
                        s0, s1 = rank * E // world, (rank + 1) * E // world
                        sg = mdist.ShardedGraph.for_gat_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
                    else:
                        sg = mdist.ShardedGraph.for_gat(ei, N, rank, world, cuts=cuts)
                    if cover:
                        sg.enable_gat_halo_cover()
                    conv = mdist.ShardedGATConv(Fi, C, heads=H, dropout=p).to(dev).train()
                    conv.load_state_dict(ref.state_dict())
                    lo, hi = sg.lo, sg.hi
                    xo = x[lo:hi].clone().requires_grad_(True)
                    torch.manual_seed(11 + ci)
                    out = conv(xo, sg)
                    (out * gout[lo:hi]).sum().backward()
                    mdist.allreduce_gradients(conv)
                    o, w = out.detach(), out_ref.detach()[lo:hi]
                    r = {"rows": hi - lo,
                         "out": float(((o - w).abs() - 1e-5 * w.abs().clamp(min=1.0)).max()) if hi > lo else -1.0,
                         "gx": float((xo.grad - xr.grad[lo:hi]).abs().max() / xr.grad.abs().max()) if hi > lo else 0.0}
                    for k in ("weight", "att", "bias"):
                        a, b = getattr(conv, k).grad, getattr(ref, k).grad
                        r["g" + k] = float((a - b).abs().max() / b.abs().max())
                    if cover:
                        st = sg.gat_cover.stats()
                        r["cover_rows"], r["pull_rows"] = st["halo_rows"], st["pull_halo_rows"]
                    else:
                        # the rank's keep mask IS the single-GPU mask on its edges (global edge ids)
                        from mi355_mp.graph import GAT_TARGET_TASKS, Graph
                        from torch_geometric.nn.conv._structure import gat_loops
                        g1 = Graph(gat_loops(ei, N), N, N, target_tasks=GAT_TARGET_TASKS)
                        k1 = ops.gat_dropout_keep(g1, 99, p, H)
                        kr = ops.gat_dropout_keep(sg.g_fwd, 99, p, H)
                        r["mask_equal"] = bool(torch.equal(kr, k1[sg.fwd.edge_gid]))
                        r["dropped_frac"] = float(1.0 - kr.float().mean()) if kr.numel() else p
                    res["%dx%d cuts %d %s" % (H, C, ci, "cover" if cover else "pull")] = r
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gatconv_attention_dropout_matches_one_gpu(world):
    """ShardedGATConv(dropout=0.3) in training mode against the single-GPU
    GATConv under one seed: the attention-dropout mask is
    keyed on the GLOBAL edge id (ABI 7 drop_ids), so every rank drops exactly
    the single-GPU layer's (edge, head) pairs -- its keep mask equals the
    single-GPU mask on its edges, and the forward rows, d x and the all-reduced
    d W / d att / d b agree within the bound, over the pull exchange AND over
    the hybrid halo cover (pieces with the dropped weights, keys sent with the
    push edges), fused (4 x 16) and wide (2 x 24) heads.  Slice-built shards,
    edge-balanced cuts, and a rank that owns no rows."""
    N = 1500
    cut_sets = [None, [0, N // 3, N] if world == 2 else [0, N // 3, 2 * N // 3, N],
                [0, N, N] if world == 2 else [0, 0, N // 2, N]]
    res = _spawn(_gat_dropout_worker, world=world, args=(cut_sets,))
    covered = 0
    for rank, r in res:
        for key, v in r.items():
            if "mask_equal" in v:
                assert v["mask_equal"], (rank, key, v)
                assert abs(v["dropped_frac"] - 0.3) < 0.05, (rank, key, v)
            assert v["out"] <= 0 and v["gx"] < 1e-5, (rank, key, v)
            assert v["gweight"] < 1e-5 and v["gatt"] < 1e-5 and v["gbias"] < 1e-5, (rank, key, v)
            if "cover_rows" in v:
                assert v["cover_rows"] <= v["pull_rows"], (rank, key, v)
                covered += v["pull_rows"] > 0
    assert covered > 0

def _products_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import Graph
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn.conv.gcn_conv import GCNConv
        dev = torch.device("cuda", 0)
        N, E, F = 2_449_029, 123_718_280, 256
        ei = powerlaw_edge_index(N, E, seed=4, device=dev)
        x = torch.randn(N, F, device=dev, generator=torch.Generator(device=dev).manual_seed(4))
        sg = mdist.ShardedGraph.for_gcn(ei, N, rank, world)
        lo, hi = sg.lo, sg.hi
        out = sg.propagate(x[lo:hi])
        # single-GPU kernel on the whole graph, and the bound's sum of |terms|
        ei2, norm = GCNConv.norm(ei, N)
        del ei
        g1 = Graph(ei2, N, N)
        w1 = g1.dst.to_csr_order(norm)
        ref = ops._aggregate(g1.dst, "other", x, w1, "sum", 0, None)[0][lo:hi]
        terms = ops._aggregate(g1.dst, "other", x.abs(), w1.abs(), "sum", 0, None)[0][lo:hi]
        excess = float(((out - ref).abs() - 1e-5 * terms.clamp(min=1)).max())
        excess_c, rows_c = None, None
        if world == 2:   # the hybrid halo cover at full size (8 ranks on one GPU oversubscribe its queues)
            out_c = sg.enable_halo_cover().propagate(x[lo:hi])
            excess_c = float(((out_c - ref).abs() - 1e-5 * terms.clamp(min=1)).max())
            rows_c = sg.cover.n_halo
        q.put((rank, excess, float((out == ref).float().mean()), hi - lo, int(sg.fwd.edge_pos.numel()),
               int(sg.fwd.halo_nodes.numel()), excess_c, rows_c))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_full_size_products_sharded_rehearsal(world):
    """Config 5 at full size (N=2,449,029, E=123,718,280 + self loops, F=256),
    destination-range sharded over 2 ranks, and over 8 -- config 5's own
    partition count -- sharing the device (gloo staging of the halo rows; the
    RCCL call is covered by test_sharded_path_over_rccl_world_one): every
    rank's owned rows within 1e-5 * sum|w x| of the single-GPU kernel; at 2
    ranks also over the hybrid halo cover (ShardedGraph.enable_halo_cover),
    which must receive fewer rows than the pull halo."""
    res = _spawn(_products_worker, world=world, timeout=540)
    assert sum(r[3] for r in res) == 2_449_029
    for rank, excess, frac, n_own, n_edges, n_halo, excess_c, rows_c in res:
        assert excess <= 0, res
        assert frac > 0.95, res   # rows split across merge-path tasks differ in the last bits
        assert n_halo > 0
        if world == 2:
            assert excess_c <= 0 and rows_c < n_halo, res


def _gat_full_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import GAT_TARGET_TASKS, Graph
        from mi355_mp.graphgen import rmat_edge_index
        from torch_geometric.nn.conv._structure import gat_loops
        dev = torch.device("cuda", 0)
        N, H, C = 1 << 21, 8, 32
        ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
        g = torch.Generator(device=dev).manual_seed(2)
        xw = torch.randn(N, H * C, device=dev, generator=g) * 0.5
        att = torch.randn(1, H, 2 * C, device=dev, generator=g) * 0.2
        E_raw = ei.shape[1]
        s0, s1 = rank * E_raw // world, (rank + 1) * E_raw // world
        sg = mdist.ShardedGraph.for_gat_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
        lo, hi = sg.lo, sg.hi
        out, (gid, alpha) = sg.gat_propagate(xw[lo:hi].contiguous(), att, H, C, return_alpha=True)
        # the single-GPU fused kernel on the whole graph, and the bound's sum |alpha x_j|
        ei2 = gat_loops(ei, N)
        del ei
        g1 = Graph(ei2, N, N, target_tasks=GAT_TARGET_TASKS)
        out1, alpha1 = ops.gat_propagate(g1, ei2, xw, att, H, C, return_alpha=True)
        eid = g1.dst.eid[:g1.dst.n_edges].long()
        terms = ops._heads_aggregate(g1.dst, "other", alpha1[eid].contiguous(), H, xw.abs())[lo:hi]
        excess = float(((out - out1[lo:hi]).abs() - 1e-5 * terms.clamp(min=1.0)).max())
        da = (alpha - alpha1[gid]).abs()
        a_eq, o_eq = _unsplit_equal(sg, g1, alpha, alpha1[gid], out, out1[lo:hi])
        q.put((rank, excess, float(da.max()), a_eq, o_eq, sg.n_edges == ei2.shape[1], hi - lo))
    finally:
        dist.destroy_process_group()


def test_full_size_gat_sharded_rehearsal():
    """Config 3 at full size (RMAT21 + self loops, 8 heads x 32) sharded over 2
    ranks sharing the device, built from per-rank edge slices: every rank's
    rows within 1e-5 * max(1, sum|alpha x_j|) of the single-GPU fused kernel and
    every (edge, head) alpha within 1e-5 of it (bit-equal on all but the rows a
    task boundary splits)."""
    res = _spawn(_gat_full_worker, world=2, timeout=540)
    assert sum(r[6] for r in res) == 1 << 21
    for rank, excess, dalpha, a_eq, o_eq, edges_ok, _ in res:
        assert excess <= 0 and dalpha <= 1e-5 and edges_ok, res
        assert a_eq and o_eq, res


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("flow", ["source_to_target", "target_to_source"])
def test_native_shard_plan_matches_torch_plan(world, flow):
    """mp_shard_plan (flag + scan on the device) vs the torch-op plan, bitwise:
    edge positions, local ids, halo nodes and per-owner counts, for every rank
    of a power-law graph with duplicate edges, self loops, isolated nodes and
    (world 8) an empty shard."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from mi355_mp import dist as mdist
    from mi355_mp.graphgen import powerlaw_edge_index
    dev = torch.device("cuda", 0)
    N, E = 5000, 80000
    ei = powerlaw_edge_index(N - 100, E, seed=41)        # nodes N-100.. are isolated
    ei = torch.cat([ei, ei[:, :500], torch.arange(7).repeat(2, 1)], 1).to(dev)
    key = ei[1] if flow == "source_to_target" else ei[0]
    cuts = mdist.edge_balanced_cuts(torch.bincount(key, minlength=N), world)
    if world == 8:
        cuts[3] = cuts[2]                                  # rank 2 owns no rows
    for rank in range(world):
        plan = mdist.ShardPlan(ei, N, rank, world, cuts=cuts, flow=flow)
        i, j = (1, 0) if flow == "source_to_target" else (0, 1)
        from tests import _host_twins
        want = _host_twins.plan(ei[i], ei[j], N, cuts, rank, world)
        assert torch.equal(plan.edge_pos, want[0])
        loc = plan.local_edge_index
        lk, lo_ = (loc[1], loc[0]) if flow == "source_to_target" else (loc[0], loc[1])
        assert torch.equal(lk, want[1]) and torch.equal(lo_, want[2])
        assert torch.equal(plan.halo_nodes, want[3])
        assert plan.recv_counts == want[4]
        assert plan.n_local_src == plan.n_own + want[3].numel()


def test_native_shard_plan_rejects_out_of_range_endpoint():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from mi355_mp import dist as mdist
    dev = torch.device("cuda", 0)
    ei = torch.tensor([[0, 1, 2, 99], [1, 2, 0, 1]], device=dev)   # source 99 >= N
    with pytest.raises(IndexError):
        mdist.ShardPlan(ei, 4, 0, 2, cuts=[0, 2, 4])


def _rccl_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import Graph
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn import GCNConv
        N, E, Fi, F = 3000, 60000, 64, 256
        ei = powerlaw_edge_index(N, E, seed=51).to(dev)
        gen = torch.Generator().manual_seed(51)
        x = torch.randn(N, F, generator=gen).to(dev)
        bias = torch.randn(F, generator=gen).to(dev)
        ei2, norm = GCNConv.norm(ei, N)
        g1 = Graph(ei2, N, N, chunk=64)
        ref = ops._aggregate(g1.dst, "other", x, g1.dst.to_csr_order(norm), "sum", 0, bias)[0]
        res = {}
        # the bench's step: async all_to_all_single on the RCCL stream + work.wait()
        plan = mdist.ShardPlan(ei2, N, rank, world).exchange_requests()
        ov = mdist.OverlappedAggregation(plan, norm, chunk=64)
        xl = plan.local_buffer(F)
        xl[:plan.n_own].copy_(x)
        out = torch.empty(plan.n_own, F, device=dev)
        ov.step(xl, out, bias)
        tiles = plan.local_tiles(F, 128)
        for t, xt in enumerate(tiles):
            xt[:plan.n_own].copy_(x[:, 128 * t:128 * t + xt.shape[1]])
        out_t = torch.empty(plan.n_own, F, device=dev)
        ov.step_tiled(tiles, out_t, bias)
        res["step"] = float((out - ref).abs().max())
        res["tiled_eq_step"] = bool(torch.equal(out_t, out))
        # the halo cover's collective build and step over RCCL (empty exchanges at one rank)
        ovc = mdist.OverlappedAggregation(plan, norm, chunk=64, cover=True)
        tc = ovc.local_tiles(F, 128)
        for t, xt in enumerate(tc):
            xt[:plan.n_own].copy_(x[:, 128 * t:128 * t + xt.shape[1]])
        out_c = torch.empty(plan.n_own, F, device=dev)
        ovc.step_tiled(tc, out_c, bias)
        res["cover_step"] = float((out_c - ref).abs().max())
        ovc.split_interior = True       # interior passes beside the send packing: bitwise the same
        out_cs = torch.full_like(out_c, float("nan"))
        ovc.step_tiled(tc, out_cs, bias)
        res["cover_split_eq"] = bool(torch.equal(out_cs, out_c))
        ovc.split_interior = False
        # the fused step over RCCL (async all_to_all per tile into tile-major buffers)
        res["fused_eq"] = not _fused_forms_equal(ovc, x.contiguous(), out_c, bias, F) and \
            not _fused_forms_equal(ov, x.contiguous(), out, bias, F)
        # sharded GCNConv forward + backward, RCCL broadcast / all_reduce of the weights
        gout = torch.randn(N, F, generator=gen).to(dev)
        xi = torch.randn(N, Fi, generator=gen).to(dev)
        conv_ref = GCNConv(Fi, F).to(dev)
        with torch.no_grad():
            conv_ref.bias.normal_()
        xr = xi.clone().requires_grad_(True)
        (conv_ref(xr, ei) * gout).sum().backward()
        sg = mdist.ShardedGraph.for_gcn(ei, N, rank, world)
        # the slice-built shards over RCCL (all_gather_object, all_reduce, all_to_all of edges)
        sgs = mdist.ShardedGraph.for_gcn_from_slices(ei.clone(), 0, N, rank, world)
        slices_equal = (sgs.n_edges == sg.n_edges and torch.equal(sgs.fwd.local_edge_index, sg.fwd.local_edge_index)
                        and torch.equal(sgs._w[0], sg._w[0]) and torch.equal(sgs._w[1], sg._w[1]))
        conv = mdist.ShardedGCNConv(Fi, F).to(dev)
        conv.load_state_dict(conv_ref.state_dict())
        mdist.broadcast_parameters(conv)
        xo = xi.clone().requires_grad_(True)
        o = conv(xo, sg)
        (o * gout).sum().backward()
        mdist.allreduce_gradients(conv)
        res["layer_out"] = float((o.detach() - conv_ref(xi, ei).detach()).abs().max())
        res["layer_gx"] = float((xo.grad - xr.grad).abs().max())
        res["layer_gw"] = float((conv.weight.grad - conv_ref.weight.grad).abs().max()
                                / conv_ref.weight.grad.abs().max())
        sgc = mdist.ShardedGraph.for_gcn(ei, N, rank, world).enable_halo_cover()
        xc = xi.clone().requires_grad_(True)
        oc = conv(xc, sgc)
        (oc * gout).sum().backward()
        res["cover_layer_out"] = float((oc.detach() - o.detach()).abs().max())
        res["cover_layer_gx"] = float((xc.grad - xo.grad).abs().max())
        # max / min with global edge ids
        xm = torch.randint(-3, 4, (N, F), generator=gen).to(torch.float32).to(dev)
        sgm = mdist.ShardedGraph(ei2, N, rank, world)
        exact = True
        for red in ("max", "min"):
            om, am = sgm.propagate(xm, red)
            wo, wa = ops._aggregate(g1.dst, "other", xm, None, red, 0, None)
            exact = exact and bool(torch.equal(om, wo)) and bool(torch.equal(am, wa))
        res["max_exact"] = exact
        res["slices_equal"] = bool(slices_equal)
        # sharded GATConv forward + backward over RCCL (plan exchange, halo rows and
        # their gradients' return, replicated parameters)
        from torch_geometric.nn import GATConv
        gref = GATConv(Fi, 32, heads=8).to(dev)
        xg = xi.clone().requires_grad_(True)
        (gref(xg, ei) * gout).sum().backward()
        sgg = mdist.ShardedGraph.for_gat_from_slices(ei.clone(), 0, N, rank, world)
        gconv = mdist.ShardedGATConv(Fi, 32, heads=8).to(dev)
        gconv.load_state_dict(gref.state_dict())
        mdist.broadcast_parameters(gconv)
        xs = xi.clone().requires_grad_(True)
        og = gconv(xs, sgg)
        (og * gout).sum().backward()
        mdist.allreduce_gradients(gconv)
        res["gat_out"] = float((og.detach() - gref(xi, ei).detach()).abs().max())
        res["gat_gx"] = float((xs.grad - xg.grad).abs().max() / xg.grad.abs().max())
        res["gat_gatt"] = float((gconv.att.grad - gref.att.grad).abs().max() / gref.att.grad.abs().max())
        torch.cuda.synchronize()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_sharded_path_over_rccl_world_one():
    """The sharded path on the RCCL backend ("nccl" = RCCL on ROCm) itself:
    one rank on the box's one GPU (two ranks cannot share a device under RCCL,
    profiles/r02_rccl_one_gpu_probe.log).  Runs every RCCL call the multi-GPU
    bench makes -- communicator setup with device_id, async all_to_all_single
    with split sizes on device tensors + work.wait() (OverlappedAggregation
    step / step_tiled), the blocking exchanges of ShardPlan / ShardedGraph,
    broadcast and all_reduce of the replicated GCNConv weights, the halo
    cover's collective build, step and autograd, the sharded GATConv (halo
    rows of X W and their gradients' return) -- with empty halo splits,
    against the single-GPU kernel, GCNConv and GATConv."""
    (rank, r), = _spawn(_rccl_worker, world=1, timeout=300)
    assert r["step"] < 1e-5 and r["tiled_eq_step"] and r["cover_split_eq"] and r["fused_eq"], r
    assert r["layer_out"] < 1e-5 and r["layer_gx"] < 1e-5 and r["layer_gw"] < 1e-5, r
    assert r["max_exact"], r
    assert r["slices_equal"], r
    assert r["cover_step"] < 1e-5 and r["cover_layer_out"] < 1e-6 and r["cover_layer_gx"] < 1e-6, r
    assert r["gat_out"] < 1e-5 and r["gat_gx"] < 1e-5 and r["gat_gatt"] < 1e-5, r


def _run_bench(args, env_extra=None, timeout=540):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", **(env_extra or {}))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MP_BENCH_LAUNCH_PROBE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable] + args, cwd=root, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    # stdout holds the JSON line and nothing else (gloo's and RCCL's own prints go to stderr)
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    return json.loads(lines[0]), r.stderr


def test_bench_multi_rank_path_end_to_end():
    """bench.py --gpus 2 with NO launcher (the driver's plain call): bench.py
    starts its two ranks itself; here they are gloo ranks sharing the box's GPU
    (MP_BENCH_BACKEND=gloo stages the halo rows through the host; the timing is
    meaningless, the line's shape, the shard bookkeeping, the per-rank stage
    markers and the step decomposition are what is checked).  --verify holds
    every rank's rows to the float64 bound over its own edges."""
    d, err = _run_bench(["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                         "--no-ref-paths", "--verify"], {"MP_BENCH_BACKEND": "gloo"})
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    assert d["config"]["num_edges"] == 62_094_512 and d["cpu_baseline"] is None
    assert d["config"]["workload"] == "rmat21_gcn_f256"
    ex = d["extra"]
    assert ex["overlap"] and ex["halo_rows_rank0"] > 0
    # the warm-up times every fused step form (max over ranks) and keeps the fastest
    import bench
    tune = ex["halo_tile_autotune_ms"]
    forms = {bench.form_name(w, one, sp, ppt) for (w, one, ppt) in bench.HALO_FORMS for sp in (False, True)}
    assert set(tune) == forms and len(forms) == 2 * len(bench.HALO_FORMS)
    assert all(v > 0 for v in tune.values())
    best = min(tune, key=tune.get)    # tile width, boundary in one launch or per tile, interior beside the packing
    assert ex["step_form"].endswith(best), (ex["step_form"], best)
    assert best.startswith("%d-wide" % ex["halo_tiles"][0]) and sum(ex["halo_tiles"]) == 256
    assert ex["split_interior"] == best.endswith("interior beside the packing")
    assert ex["comm_init_s"] is not None
    assert ex["collective_timeout_s"] == 300
    assert 0 < ex["interior_edges_rank0"] < ex["edges_local_rank0"] < d["config"]["num_edges"]
    assert ex["verify"]["all_ranks_within_1e-5_bound"], ex["verify"]
    pr = ex["per_rank"]
    assert [p["rank"] for p in pr] == [0, 1] and sum(p["edges"] for p in pr) == d["config"]["num_edges"]
    for p in pr:
        assert p["halo_bytes_in"] == p["halo_rows"] * 256 * 4 and p["halo_bytes_out"] > 0
        assert p["interior_ms"] > 0 and p["boundary_ms"] > 0 and p["exchange_exposed_ms"] >= 0
        dc = p["decomposed"]
        assert dc["exchange_only_ms"] > 0 and dc["compute_only_ms"] > 0
        assert dc["serial_step_ms"] > 0 and dc["overlapped_step_ms"] > 0
        # host-staged gloo exchanges: hidden_frac is not reported as a number
        assert dc["hidden_frac"] is None and not dc["hidden_frac_valid"] and dc["hidden_frac_note"], dc
        # the compute timed one rank at a time (the GPU to itself): its parts add up
        cit = p["compute_in_turn"]
        assert cit["compute_alone_split_ms"] > 0
        parts = cit["send_pack_ms"] + cit["interior_ms"] + cit["boundary_ms"]
        assert min(cit["send_pack_ms"], cit["interior_ms"], cit["boundary_ms"]) > 0, cit
        assert abs(parts - cit["compute_alone_ms"]) < 1e-6 * max(1.0, parts), cit
        assert set(p["link_model"]["predicted_in_turn"]) == {"60", "77", "100"}
    for r in (0, 1):
        for marker in ("process group up", "shards built", "warm-up done", "timed steps done", "done"):
            assert ("[bench rank %d " % r) in err and marker in err, marker


def test_bench_products_workload_one_gpu():
    """--workload products (BASELINE config 5, N = 2,449,029, E' = 126,163,923)
    on one GPU: the line names the workload, and --verify holds every output
    row to test_full_size_products_gcn's bound (|out - ref| <= 1e-5 *
    max(1, sum|w x_j|) against a float64 reference over all edges)."""
    d, _ = _run_bench(["bench.py", "--workload", "products", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                       "--no-ref-paths", "--verify"])
    assert d["n_gpus"] == 1 and d["config"]["workload"] == "products_gcn_f256"
    assert d["config"]["num_nodes"] == 2_449_029 and d["config"]["num_edges"] == 126_163_923
    assert d["config"]["baseline_config"] == 5
    v = d["extra"]["verify"]
    assert v["within_1e-5_bound"] and v["rows"] == 2_449_029 and v["edges"] == 126_163_923, v
    assert d["value"] > 4e9 and d["roofline"]["frac"] > 0


def test_bench_products_workload_two_ranks():
    """The config-5 workload under bench.py's own N-rank launch: 2 gloo ranks
    sharing the GPU, slice-built shards, hybrid-cover tiled overlap, every
    rank's rows within the float64 bound."""
    d, _ = _run_bench(["bench.py", "--gpus", "2", "--workload", "products", "--steps", "2", "--warmup", "1",
                       "--no-cpu-baseline", "--no-ref-paths", "--verify"], {"MP_BENCH_BACKEND": "gloo"})
    assert d["n_gpus"] == 2 and d["config"]["workload"] == "products_gcn_f256"
    assert d["config"]["num_edges"] == 126_163_923
    assert d["extra"]["verify"]["all_ranks_within_1e-5_bound"], d["extra"]["verify"]
    assert sum(p["rows"] for p in d["extra"]["per_rank"]) == 2_449_029


def test_bench_reddit_workload_one_gpu():
    """--workload reddit (BASELINE config 4: N = 232,965, E = 114,615,892,
    aggr='max' + int64 first-index argmax + the -10000 mask) on one GPU:
    --verify holds every value and every argmax bit-equal to torch's
    scatter_reduce amax and the smallest edge id attaining it."""
    d, _ = _run_bench(["bench.py", "--workload", "reddit", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                       "--verify"])
    assert d["n_gpus"] == 1 and d["config"]["workload"] == "reddit_max_f256"
    assert d["config"]["num_edges"] == 114_615_892 and d["config"]["baseline_config"] == 4
    v = d["extra"]["verify"]
    assert v["values_bitwise_equal"] and v["args_bitwise_equal"], v
    assert d["value"] > 5e9 and "ArgRed" in d["roofline"]["kernel"]


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_gat_workload(gpus):
    """--workload gat (BASELINE config 3: the rmat21 graph, GATConv 8 heads x 32)
    at one GPU and as 2 gloo ranks sharing the device (bench.py's own launch):
    every rank's rows within 1e-5 * max(1, sum|alpha x_j|) of a float64 GATConv
    formula over its own edges; per-rank exchange-only / compute-only times."""
    args = ["bench.py", "--workload", "gat", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--verify"]
    if gpus > 1:
        d, _ = _run_bench(args[:1] + ["--gpus", str(gpus)] + args[1:], {"MP_BENCH_BACKEND": "gloo"})
        assert d["extra"]["verify"]["all_ranks_within_1e-5_bound"], d["extra"]["verify"]
        pr = d["extra"]["per_rank"]
        assert len(pr) == gpus and sum(p["rows"] for p in pr) == 1 << 21
        assert all(p["exchange_only_ms"] > 0 and p["compute_only_ms"] > 0 for p in pr)
    else:
        d, _ = _run_bench(args)
        assert d["extra"]["verify"]["within_1e-5_bound"], d["extra"]["verify"]
    assert d["n_gpus"] == gpus and d["config"]["workload"] == "rmat21_gat_h8c32"
    assert d["config"]["num_edges"] == 62_094_512      # remove + add self loops: GCN's E'
    assert d["value"] > 0 and d["roofline"]["frac"] > 0


def test_bench_sharded_path_over_rccl_one_rank():
    """bench.py's N > 1 code path on the RCCL backend -- the one the driver's
    8-GPU run takes -- as ONE rank (two ranks cannot share a device under
    RCCL): `--sharded` routes the one-rank job through the slice-built shards,
    the collective plan / halo-cover build, the tiled overlapped step with its
    (empty) all_to_all_single per tile, the max-over-ranks all_reduce and the
    per-rank all_gather_object; the rate must match the single-GPU kernel's
    order of magnitude and every edge must be interior."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("MP_BENCH_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
           "--sharded", "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    # the one JSON line alone on stdout: RCCL's version banner goes to stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["config"]["num_edges"] == 62_094_512 and d["cpu_baseline"] is None
    assert d["config"]["parallelism"].startswith("dst-range shards x1")
    ex = d["extra"]
    assert ex["overlap"] and ex["halo_cover"] and ex["halo_rows_rank0"] == 0
    assert ex["halo_tiles"] in ([256], [128, 128], [64] * 4) and ex["step_form"].startswith("fused")
    assert ex["interior_edges_rank0"] == ex["edges_local_rank0"] == d["config"]["num_edges"]
    (p,) = ex["per_rank"]
    assert p["rank"] == 0 and p["halo_bytes_in"] == 0 and p["peers_in"] == [0]
    assert p["interior_ms"] > 0 and p["exchange_exposed_ms"] >= 0
    dc = p["decomposed"]   # one rank: empty splits, the exchange alone costs ~nothing
    assert dc["exchange_only_ms"] < 0.2 * dc["compute_only_ms"], dc
    cit = p["compute_in_turn"]   # one rank: the same compute, timed with events
    assert 0.5 * dc["compute_only_ms"] < cit["compute_alone_ms"] < 2.0 * dc["compute_only_ms"], (cit, dc)
    # the same kernels over the whole graph: within 2x of the single-GPU step
    assert d["value"] > 4e9, d["value"]
    # the line explains itself: link model and build split per rank
    assert p["link_model"]["sets_the_step"].startswith("compute"), p["link_model"]
    # one rank also rebuilds both warm: the build itself is device-bound
    bs = p["build_split"]
    assert set(bs) == {"shards", "exchange_plan", "shards_warm", "exchange_plan_warm"}
    assert all(v["wall_s"] > 0 for v in bs.values())
    for k in ("shards_warm", "exchange_plan_warm"):
        assert bs[k]["host_and_sync_s"] < bs[k]["device_busy_s"], (k, bs[k])
        assert bs[k]["host_syncs"] <= bs[k.replace("_warm", "")]["host_syncs"], bs


def test_rccl_runs_beside_the_aggregation_one_rank():
    """RCCL's kernels next to k_agg_flat: one RCCL rank, no
    launcher (`--sharded` at --gpus 1 makes its own world-1 group), a self
    split of the P = 8 rank's cover volume started async beside that rank's
    aggregation.  Issued as OverlappedAggregation issues it (its compute stream,
    RCCL on high-priority streams with hardware queues of their own) the
    exchange must partly hide behind the aggregation: round 5 measured 0.54
    there and -0.03 while RCCL's stream shared the default stream's queue."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MP_BENCH_BACKEND"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--sharded", "--emulate-peers", "8", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-ref-paths", "--no-build-split"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    (c,) = d["extra"]["per_rank"][0]["rccl_contention"]
    assert c["P"] == 8 and c["exchange_rows"] == 313_427, c
    assert c["serial_step_ms"] > c["overlapped_step_ms"], c
    assert c["hidden_frac"] > 0.2, c


def _cover_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import Graph
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn.conv.gcn_conv import GCNConv
        dev = torch.device("cuda", 0)
        N, E, F = 4000, 80000, 256
        ei = powerlaw_edge_index(N, E, seed=37).to(dev)
        ei2, norm = GCNConv.norm(ei, N)
        gen = torch.Generator().manual_seed(37)
        x = torch.randn(N, F, generator=gen).to(dev)
        bias = torch.randn(F, generator=gen).to(dev)
        g = Graph(ei2, N, N, chunk=64)
        wc = g.dst.to_csr_order(norm)
        ref = ops._aggregate(g.dst, "other", x, wc, "sum", 0, bias)[0]
        terms = ops._aggregate(g.dst, "other", x.abs(), wc.abs(), "sum", 0, None)[0]
        plan = mdist.ShardPlan(ei2, N, rank, world).exchange_requests()
        ov = mdist.OverlappedAggregation(plan, norm, chunk=64, cover=True)
        xl = ov.local_buffer(F)
        xl[:plan.n_own].copy_(x[plan.lo:plan.hi])
        out = torch.empty(plan.n_own, F, device=dev)
        ov.step(xl, out, bias)
        lo, hi = plan.lo, plan.hi
        ok_f = bool(((out - ref[lo:hi]).abs() <= 1e-5 * terms[lo:hi].clamp(min=1.0)).all())
        tiles = ov.local_tiles(F, 128)
        for t, xt in enumerate(tiles):
            xt[:plan.n_own].copy_(x[lo:hi, 128 * t:128 * t + xt.shape[1]])
        out_t = torch.empty_like(out)
        ov.step_tiled(tiles, out_t, bias)
        ok_t = torch.equal(out_t, out) and not _fused_forms_equal(ov, x[lo:hi].contiguous(), out, bias, F)
        # integer-valued features and weights: every regrouping is exact -> bitwise
        xi = torch.randint(-8, 9, (N, F), generator=gen).to(torch.float32).to(dev)
        wi = torch.randint(1, 4, (ei2.shape[1],), generator=gen).to(torch.float32).to(dev)
        refi = ops._aggregate(g.dst, "other", xi, g.dst.to_csr_order(wi), "sum", 0, None)[0]
        ovi = mdist.OverlappedAggregation(plan, wi, chunk=64, cover=True)
        xli = ovi.local_buffer(F)
        xli[:plan.n_own].copy_(xi[lo:hi])
        outi = torch.empty_like(out)
        ovi.step(xli, outi, None)
        ok_i = torch.equal(outi, refi[lo:hi])
        q.put((rank, ok_f, ok_t, ok_i, ov.n_local_src - plan.n_own, plan.n_local_src - plan.n_own,
               ov.cover.n_push_rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_overlapped_halo_cover_on_one_gpu(world):
    """The hybrid pull / push exchange (dist.HaloCover) on the native kernels,
    ranks sharing the GPU over gloo: every rank's rows within 1e-5 * sum|w x|
    of the single-GPU kernel, step_tiled bitwise step, integer-valued data
    bitwise the single-GPU kernel, fewer rows than the pull exchange."""
    res = _spawn(_cover_worker, world=world, timeout=300)
    assert all(r[1] and r[2] and r[3] for r in res), res
    assert sum(r[4] for r in res) < sum(r[5] for r in res), res
    assert any(r[6] > 0 for r in res), res


def _cover_layer_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import Graph
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn import GCNConv
        from torch_geometric.nn.conv.gcn_conv import GCNConv as G
        dev = torch.device("cuda", 0)
        N, E, Fi, Fo = 3000, 60000, 64, 128
        ei = powerlaw_edge_index(N, E, seed=43).to(dev)
        gen = torch.Generator().manual_seed(43)
        x = torch.randn(N, Fi, generator=gen).to(dev)
        gout = torch.randn(N, Fo, generator=gen).to(dev)
        ref = GCNConv(Fi, Fo).to(dev)
        with torch.no_grad():
            ref.bias.normal_()
        mdist.broadcast_parameters(ref)
        xr = x.clone().requires_grad_(True)
        out_ref = ref(xr, ei)
        (out_ref * gout).sum().backward()
        sg = mdist.ShardedGraph.for_gcn(ei, N, rank, world).enable_halo_cover()
        conv = mdist.ShardedGCNConv(Fi, Fo).to(dev)
        conv.load_state_dict(ref.state_dict())
        lo, hi = sg.lo, sg.hi
        xo = x[lo:hi].clone().requires_grad_(True)
        out = conv(xo, sg)
        (out * gout[lo:hi]).sum().backward()
        mdist.allreduce_gradients(conv)
        r = {"out": float((out.detach() - out_ref.detach()[lo:hi]).abs().max()),
             "gx": float((xo.grad - xr.grad[lo:hi]).abs().max()),
             "gw": float((conv.weight.grad - ref.weight.grad).abs().max() / ref.weight.grad.abs().max()),
             "rows_cover": sg.cover.n_halo, "rows_pull": sg.fwd.n_local_src - sg.n_own}
        # integer-valued data and weights: every regrouping is exact, so forward and
        # backward equal the single-GPU fused aggregation bit for bit (sum and mean)
        ei2, _ = G.norm(ei, N)
        wi = torch.randint(1, 4, (ei2.shape[1],), generator=gen).to(torch.float32).to(dev)
        sgi = mdist.ShardedGraph(ei2, N, rank, world).set_edge_weight(wi).enable_halo_cover()
        g1 = Graph(ei2, N, N)
        xi = torch.randint(-8, 9, (N, Fo), generator=gen).to(torch.float32).to(dev)
        gi = torch.randint(-4, 5, (N, Fo), generator=gen).to(torch.float32).to(dev)
        exact = {}
        for red in ("sum", "mean"):
            xs = xi[lo:hi].clone().requires_grad_(True)
            o = sgi.propagate(xs, red)
            (o * gi[lo:hi]).sum().backward()
            xf = xi.clone().requires_grad_(True)
            of = ops.fused_propagate(g1, xf, ei2, wi, red)
            (of * gi).sum().backward()
            if red == "sum":
                exact[red] = bool(torch.equal(o, of[lo:hi])) and bool(torch.equal(xs.grad, xf.grad[lo:hi]))
            else:
                # forward: the same exact sum divided once by the same degree; backward: g / deg is
                # not integer-valued, so the regrouped sums agree to rounding (relative bound)
                o, of = o.detach(), of.detach()
                r["mean_fwd_diff"] = float((o - of[lo:hi]).abs().max())
                gref = xf.grad[lo:hi]
                r["mean_bwd_excess"] = float(((xs.grad - gref).abs() - 1e-5 * gref.abs().clamp(min=1.0)).max())
                exact[red] = bool(torch.equal(o, of[lo:hi])) and r["mean_bwd_excess"] <= 0
        r["exact"] = exact
        q.put((rank, r))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gcnconv_over_halo_cover_on_one_gpu(world):
    """ShardedGraph.enable_halo_cover(): ShardedGCNConv forward + backward over the
    hybrid cover (ranks sharing the GPU over gloo) within 1e-5 of the single-GPU
    GCNConv, integer-valued sum / mean forward and backward equal to the
    single-GPU kernel, fewer rows than the pull exchange."""
    res = _spawn(_cover_layer_worker, world=world)
    for rank, r in res:
        assert r["out"] < 1e-5 and r["gx"] < 1e-5 and r["gw"] < 1e-5, r
        assert r["exact"]["sum"] and r["exact"]["mean"], r
    assert sum(r["rows_cover"] for _, r in res) < sum(r["rows_pull"] for _, r in res), res


def _tiny_gpu_worker(rank, world, port, q, N, edges):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import Graph
        from torch_geometric.nn.conv.gcn_conv import GCNConv
        dev = torch.device("cuda", 0)
        ei = torch.tensor(edges, dtype=torch.long).view(2, -1).to(dev)
        E = ei.shape[1]
        s0, s1 = rank * E // world, (rank + 1) * E // world
        sg = mdist.ShardedGraph.for_gcn_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
        x = torch.randn(N, 64, generator=torch.Generator().manual_seed(7)).to(dev)
        ei2, norm = GCNConv.norm(ei, N)
        g1 = Graph(ei2, N, N)
        want = ops._aggregate(g1.dst, "other", x, g1.dst.to_csr_order(norm), "sum", 0, None)[0][sg.lo:sg.hi]
        res = {"rows": sg.hi - sg.lo}
        po = sg.propagate(x[sg.lo:sg.hi].contiguous())     # every rank: the exchange is collective
        res["pull"] = float((po - want).abs().max()) if sg.n_own else 0.0
        # the bench's overlapped tiled step (hybrid cover) on the same shards
        ov = mdist.OverlappedAggregation(sg.fwd, sg.norm_fwd, local_weights=True, cover=True)
        tiles = ov.local_tiles(64, 32)
        for t, xt in enumerate(tiles):
            xt[:sg.n_own].copy_(x[sg.lo:sg.hi, 32 * t:32 * (t + 1)])
        out = torch.empty((sg.n_own, 64), device=dev)
        ov.step_tiled(tiles, out)
        res["cover"] = float((out - want).abs().max()) if sg.n_own else 0.0
        # the fused step on the same degenerate shards (empty buffers, ranks without rows)
        of = torch.full_like(out, float("nan"))
        ov.step_fused(x[sg.lo:sg.hi].contiguous(), ov.halo_buffers(64, 64), of)
        res["fused_eq"] = bool(torch.equal(of, out))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,edges", [
    (4, 5, [[0, 3], [1, 4]]),          # 2 edges over 4 ranks: empty slices
    (3, 4, [[], []]),                  # no edges at all: loops only
    (3, 1, [[0], [0]]),                # one node: two ranks own nothing
])
def test_slice_built_shards_degenerate_graphs_on_one_gpu(world, N, edges):
    """The native slice build, the sharded propagate and the bench's overlapped
    tiled step over the hybrid cover on degenerate graphs (empty slices, ranks
    owning no rows, no edges at all), against the single-GPU kernel."""
    res = _spawn(_tiny_gpu_worker, world=world, timeout=300, args=(N, edges))
    assert sum(r["rows"] for _, r in res) == N
    for rank, r in res:
        assert r["pull"] < 1e-6 and r["cover"] < 1e-6 and r["fused_eq"], (rank, r)


def _sharded_fuzz_worker(rank, world, port, q, seeds):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist, ops
        from mi355_mp.graph import Graph
        from torch_geometric.nn import GATConv, GCNConv
        dev = torch.device("cuda", 0)
        res = []
        for seed in seeds:
            g = torch.Generator().manual_seed(seed)       # the same draws on every rank
            N = int(torch.randint(1, 2000, (1,), generator=g))
            E = int(torch.randint(0, 12 * N + 1, (1,), generator=g))
            hub = torch.randint(0, N, (1,), generator=g)
            src = torch.where(torch.rand(E, generator=g) < 0.3, hub.expand(E), torch.randint(0, N, (E,), generator=g))
            dst = torch.randint(0, N, (E,), generator=g)
            ei = torch.stack([src, dst]).to(dev)
            inner = sorted(int(c) for c in torch.randint(0, N + 1, (world - 1,), generator=g))
            cuts = [0] + inner + [N]                    # random ranges, empty ones included
            Fi = int(torch.randint(1, 40, (1,), generator=g))
            x = torch.randn(N, Fi, generator=g).to(dev)
            kind = ["gcn", "gcn_cover", "gat", "max", "gat_cover"][seed % 5]
            r = {"seed": seed, "kind": kind, "N": N, "E": E, "cuts": cuts}
            torch.manual_seed(seed)
            if kind in ("gcn", "gcn_cover"):
                ref = GCNConv(Fi, 24).to(dev)
                sg = mdist.ShardedGraph.for_gcn(ei, N, rank, world, cuts=cuts)
                if kind == "gcn_cover":
                    sg.enable_halo_cover()
                conv = mdist.ShardedGCNConv(Fi, 24).to(dev)
            elif kind in ("gat", "gat_cover"):
                H = int(torch.randint(1, 5, (1,), generator=g))
                Cg = 8 if kind == "gat" else int(torch.randint(1, 41, (1,), generator=g))   # cover: any width
                ref = GATConv(Fi, Cg, heads=H).to(dev)
                if kind == "gat_cover":
                    # Gaussian x and W: the row-exact GEMM keeps X W bitwise on both sides, so no leaky_relu branch flips
                    x = _gauss_(torch.empty(N, Fi), g, 4.0).to(dev)
                    _gauss_(ref.weight, g, 16.0)
                sg = mdist.ShardedGraph.for_gat(ei, N, rank, world, cuts=cuts)
                if kind == "gat_cover":
                    sg.enable_gat_halo_cover()
                conv = mdist.ShardedGATConv(Fi, Cg, heads=H).to(dev)
            if kind != "max":
                with torch.no_grad():
                    ref.bias.normal_(generator=None)
                mdist.broadcast_parameters(ref)
                conv.load_state_dict(ref.state_dict())
                gout = torch.randn(N, ref.bias.shape[0], generator=g).to(dev)
                xr = x.clone().requires_grad_(True)
                out_ref = ref(xr, ei)
                (out_ref * gout).sum().backward()
                lo, hi = sg.lo, sg.hi
                xo = x[lo:hi].clone().requires_grad_(True)
                out = conv(xo, sg)
                (out * gout[lo:hi]).sum().backward()
                mdist.allreduce_gradients(conv)
                scale = max(1.0, float(out_ref.abs().max()))
                r["out"] = float((out.detach() - out_ref.detach()[lo:hi]).abs().max()) / scale if hi > lo else 0.0
                gs = max(1.0, float(xr.grad.abs().max()))
                r["gx"] = float((xo.grad - xr.grad[lo:hi]).abs().max()) / gs if hi > lo else 0.0
                r["gparams"] = max(float((getattr(conv, k).grad - getattr(ref, k).grad).abs().max())
                                   / max(1.0, float(getattr(ref, k).grad.abs().max()))
                                   for k in ("weight", "bias") + (("att",) if kind.startswith("gat") else ()))
            else:
                sgm = mdist.ShardedGraph(ei, N, rank, world, cuts=cuts)
                om, am = sgm.propagate(x[sgm.lo:sgm.hi].contiguous(), "max")
                wo, wa = ops._aggregate(Graph(ei, N, N).dst, "other", x, None, "max", 0, None)
                r["exact"] = bool(torch.equal(om, wo[sgm.lo:sgm.hi]) and torch.equal(am, wa[sgm.lo:sgm.hi]))
            res.append(r)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_sharded_layers_fuzz_random_cuts_on_one_gpu():
    """48 random graphs (hub-heavy sources, 0..12N edges, 1..2000 nodes) at 3
    ranks with random row ranges (empty ranks included): ShardedGCNConv over
    the pull plan and over the halo cover, ShardedGATConv (1-4 heads) over the
    pull plan and over the GAT halo cover, each
    forward + backward within 1e-5 (relative to max(1, |ref|)) of the
    single-GPU layer with all-reduced parameter gradients; sharded max with
    global argmax ids bit-equal to the single-GPU kernel."""
    res = _spawn(_sharded_fuzz_worker, world=3, timeout=300, args=(list(range(100, 148)),))
    assert len(res) == 3
    for rank, rows in res:
        assert len(rows) == 48 and {r["kind"] for r in rows} == {"gcn", "gcn_cover", "gat", "max", "gat_cover"}
        for r in rows:
            if r["kind"] == "max":
                assert r["exact"], (rank, r)
            else:
                assert r["out"] < 1e-5 and r["gx"] < 1e-5 and r["gparams"] < 1e-5, (rank, r)


def _gauss_(t, gen, scale):
    """Fill t with N(0, 1) / (2 scale) draws.  Round 5 drew X and W on a dyadic
    grid here, so that X W came out exact whatever GEMM kernel computed it
    (hipBLASLt picks its kernel, and so its rounding, by the row count M, and a
    rank's M is n_own): a score within rounding of 0 would otherwise flip
    leaky' between 1 and the slope on one side only.  GATConv and
    ShardedGATConv now compute X W with the row-exact GEMM (ops.gemm_rows:
    each output row a function of its own input row), so Gaussian inputs give
    a rank bitwise the single-GPU rows of X W."""
    with torch.no_grad():
        t.copy_(torch.randn(tuple(t.shape), generator=gen).to(t.dtype) / (2.0 * scale))
    return t


def _gat_cover_gpu_worker(rank, world, port, q, cut_sets):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "pytorch_geometric-1_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=_PG_TIMEOUT)
    try:
        from mi355_mp import dist as mdist
        from mi355_mp.graph import GAT_TARGET_TASKS, Graph
        from mi355_mp.graphgen import powerlaw_edge_index
        from torch_geometric.nn import GATConv
        from torch_geometric.nn.conv._structure import gat_loops
        dev = torch.device("cuda", 0)
        N, E, Fi = 2500, 40000, 48
        gen = torch.Generator().manual_seed(83)
        ei = powerlaw_edge_index(N, E, seed=83)
        # a hub destination and a hub source: rows both pushed and pulled
        ei = torch.cat([ei, torch.stack([torch.randint(0, N, (2000,), generator=gen), torch.full((2000,), 7)]),
                        torch.stack([torch.full((1500,), N - 3), torch.randint(0, N, (1500,), generator=gen)])], 1)
        ei = ei[:, torch.randperm(ei.shape[1], generator=gen)].to(dev)
        E = ei.shape[1]
        x = _gauss_(torch.empty(N, Fi), gen, 4.0).to(dev)
        res = {}
        for ci, cuts in enumerate(cut_sets):
            # fused-pass heads (C/4 a power of two) and wide ones (a heads=1 stack's 96, a
            # padded 10 -> 12: the wide kernels, d a_dst shares from the pieces' out2 / s2);
            # heads that cross the merge kernel's 256-feature chunks: PPI's conv3
            # (examples/ppi.py: 6 heads of 121 -> 124, concat=False) and one head of 512
            for H, C, concat in ((8, 32, True), (3, 8, False), (2, 4, True), (1, 96, True), (2, 10, True),
                                 (6, 121, False), (1, 512, True)):
                Fo = H * C if concat else C
                gout = torch.randn(N, Fo, generator=gen).to(dev)
                ref = GATConv(Fi, C, heads=H, concat=concat).to(dev)
                _gauss_(ref.weight, gen, 16.0)
                with torch.no_grad():
                    ref.att.copy_(torch.randn(ref.att.shape, generator=gen) * 0.3)
                    ref.bias.copy_(torch.randn(ref.bias.shape, generator=gen))
                xr = x.clone().requires_grad_(True)
                out_ref = ref(xr, ei)
                (out_ref * gout).sum().backward()
                if cuts is None:
                    s0, s1 = rank * E // world, (rank + 1) * E // world
                    sg = mdist.ShardedGraph.for_gat_from_slices(ei[:, s0:s1].clone(), s0, N, rank, world)
                else:
                    sg = mdist.ShardedGraph.for_gat(ei, N, rank, world, cuts=cuts)
                pull_rows = sg.fwd.n_local_src - sg.n_own
                sg.enable_gat_halo_cover()
                conv = mdist.ShardedGATConv(Fi, C, heads=H, concat=concat).to(dev)
                conv.load_state_dict(ref.state_dict())
                lo, hi = sg.lo, sg.hi
                xo = x[lo:hi].clone().requires_grad_(True)
                out = conv(xo, sg)
                (out * gout[lo:hi]).sum().backward()
                mdist.allreduce_gradients(conv)
                o, w = out.detach(), out_ref.detach()[lo:hi]
                r = {"rows": hi - lo, "halo_rows": sg.gat_cover.n_halo, "pull_rows": pull_rows,
                     "pieces": sg.gat_cover.n_push_rows,
                     "out": float(((o - w).abs() - 1e-5 * w.abs().clamp(min=1.0)).max()) if hi > lo else -1.0,
                     "gx": float((xo.grad - xr.grad[lo:hi]).abs().max() / xr.grad.abs().max()) if hi > lo else 0.0}
                for k in ("weight", "att", "bias"):
                    a, b = getattr(conv, k).grad, getattr(ref, k).grad
                    r["g" + k] = float((a - b).abs().max() / b.abs().max())
                if concat and hi > lo:
                    # rows no peer pushes a piece of, whole on both schedules: the single-GPU
                    # kernel's rows bit for bit (same edges, same order, same kernel)
                    gl = sg.gat_cover.graphs()[0].dst
                    ei_l = gat_loops(ei, N)
                    g1 = Graph(ei_l, N, N, target_tasks=GAT_TARGET_TASKS).dst    # as GATConv builds it
                    deg_l = (gl.rowptr[1:] - gl.rowptr[:-1]).long()
                    deg_1 = (g1.rowptr[1:] - g1.rowptr[:-1]).long()[lo:hi]
                    merged = torch.zeros(hi - lo, dtype=torch.bool, device=dev)
                    merged[sg.gat_cover.part_dst] = True
                    plain = (~merged) & (deg_l == deg_1) & (deg_l <= min(gl.snap, g1.snap))
                    r["plain_rows"] = int(plain.sum())
                    r["plain_bitwise"] = bool(torch.equal(o[plain], w[plain]))
                res[(ci, H, C, concat)] = r
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gatconv_over_halo_cover_on_one_gpu(world):
    """ShardedGATConv over the hybrid halo cover (mi355_mp.gat_cover: pulled rows
    + pushed online-softmax pieces, merged by mp_gat_merge_partials_f32; the
    native backward returns g and the pack of every pushed row to its pusher):
    forward rows, d x and the all-reduced d W / d att / d b against the
    single-GPU GATConv -- slice-built shards, an empty rank, a one-row rank;
    config 3's 8 x 32 heads, a mean of heads, C = 4, and wide heads (one head
    of 96, two padded heads of 10), and heads that cross the merge kernel's
    256-feature chunks (PPI conv3's 6 x 121 -> 124 mean, one head of 512).  Rows no peer pushes a
    piece of are the single-GPU rows bit for bit; the cover never receives
    more rows than the pull plan, and pieces are pushed."""
    N = 2500
    cut_sets = [None, [0, N, N] if world == 2 else [0, 0, N // 2, N], [0, 1, N] if world == 2 else [0, 1, N // 2, N]]
    res = _spawn(_gat_cover_gpu_worker, world=world, args=(cut_sets,))
    pieces = 0
    for rank, r in res:
        for key, v in r.items():
            assert v["out"] <= 0 and v["gx"] < 1e-5, (rank, key, v)
            assert v["gweight"] < 1e-5 and v["gatt"] < 1e-5 and v["gbias"] < 1e-5, (rank, key, v)
            assert v["halo_rows"] <= v["pull_rows"], (rank, key, v)
            if "plain_bitwise" in v:
                assert v["plain_bitwise"], (rank, key, v)
            pieces += v["pieces"]
    assert pieces > 0


def test_host_tensors_raise_without_twins():
    """No CPU fallback in the product package: a shard
    plan, the GAT cover step and the ordered segment sum on host tensors raise
    RuntimeError in a process that has not installed the gloo tests' host twins
    (tests/_host_twins.py) -- this GPU suite's process."""
    from mi355_mp import dist as mdist
    from mi355_mp.gat_cover import gat_cover_propagate
    assert mdist._HOST_TWINS is None
    ei = torch.tensor([[0, 1, 2], [1, 2, 0]])
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        mdist.ShardPlan(ei, 3, 0, 1)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        mdist._segment_sum_in_order(torch.zeros(3, dtype=torch.long), torch.zeros(3), 2)

    class _Cover:
        n_own = 3
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        gat_cover_propagate(_Cover(), torch.zeros(3, 8), torch.zeros(1, 1, 16), 1, 8)
    # the same calls on the device run the engine
    plan = mdist.ShardPlan(ei.cuda(), 3, 0, 1)
    assert plan.n_own == 3 and plan.halo_nodes.numel() == 0
