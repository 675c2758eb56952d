"""Destination-range graph sharding with a halo exchange.

The reference's only multi-GPU mechanism is torch_geometric.nn.DataParallel
(replicas over a list of small graphs; /root/reference/ConvexPruning.py:530,
examples/data_parallel.py:35-49).  One large graph is sharded here instead:

  * rank p owns the destination rows [lo_p, hi_p); cut points come from the
    in-degree prefix sum so every rank gets ~E/P edges (power-law safe);
  * rank p also owns the node features of [lo_p, hi_p) (it computes its own
    X W rows);
  * halo plan (built once, cached like GCNConv(cached=True)): the sorted
    unique remote source nodes of p's in-edges, grouped by owner; local
    column ids are renumbered into [0, n_own + n_halo);
  * per layer: every rank packs the rows its peers requested (native row
    gather), one all_to_all_single moves them (RCCL over xGMI: each peer pair
    on its own link), then the local fused aggregation runs on
    [own rows ; halo rows];
  * HaloCover (the bench's exchange): a cross edge is covered either by
    pulling its source row or by its source's owner pushing a partial row of
    the destination, whichever covers the pair's cross edges with fewer rows
    (0.57x the pull rows on RMAT21); the sender fills its send buffer with one
    aggregation over a send graph.

The plan is built natively on the device (mp_shard_plan: flag + scan, no
sort).  The data path calls the native kernels; a host tensor raises unless a
test installed host twins of them (install_host_twins: the gloo tests run the
distributed logic of this module on CPU that way).
"""
import torch
import torch.distributed as dist


GLOO_STAGED_S = [0.0]     # host time inside staged (gloo) all_to_alls: copies + host transfer


def _stage_to_host(t):
    """gloo staging (the multi-process rehearsal of the RCCL path on a shared
    GPU): a device tensor's copy in host memory -- the one host sync of a
    staged collective (bench.py's build split counts the syncs on this line
    apart).  A host tensor is returned as it is."""
    return t.cpu()


def _a2a(out, inp, out_splits=None, in_splits=None, group=None):
    """all_to_all_single; with the gloo backend (CPU-only collectives) device
    tensors are staged through host memory: one device-to-host copy of the
    input, the result lands in pinned memory and goes back without a sync."""
    if out.is_cuda and dist.get_backend(group) == "gloo":
        import time
        t0 = time.perf_counter()
        o = torch.empty(out.shape, dtype=out.dtype, pin_memory=True)
        dist.all_to_all_single(o, _stage_to_host(inp), output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=group)
        out.copy_(o, non_blocking=True)
        GLOO_STAGED_S[0] += time.perf_counter() - t0
        return out
    dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=group)
    return out


def _device_collectives(dev, group=None):
    """True when collectives of `group` take tensors on `dev` (RCCL); gloo
    takes host tensors."""
    return dev.type != "cpu" and dist.get_backend(group) != "gloo"


def _exchange_counts(send, group=None):
    """all_to_all of per-peer counts: send [world] or [world, k] int64 (device
    or host).  Returns (send, recv) as host lists (of lists for k > 1) with ONE
    host sync -- the splits of the exchanges that follow need them on the host."""
    world = dist.get_world_size(group)
    k = 1 if send.dim() == 1 else send.shape[1]
    if _device_collectives(send.device, group):
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv.view(-1), send.reshape(-1).contiguous(), group=group)
        both = torch.stack([send.reshape(world, k), recv.reshape(world, k)]).tolist()
    else:
        sh = _stage_to_host(send.reshape(world, k))
        rh = torch.empty_like(sh)
        dist.all_to_all_single(rh.view(-1), sh.reshape(-1).contiguous(), group=group)
        both = [sh.tolist(), rh.tolist()]
    if send.dim() == 1:
        return [r[0] for r in both[0]], [r[0] for r in both[1]]
    return both[0], both[1]


def _dev_ints(lists, dev):
    """Host int lists -> int64 tensors on `dev` in ONE asynchronous copy
    (pinned staging: no synchronising host-to-device memcpy per small tensor).
    Returns one tensor per list (views of one buffer)."""
    flat = [int(v) for lst in lists for v in lst]
    buf = torch.tensor(flat if flat else [0], dtype=torch.int64)
    if dev.type == "cuda":
        buf = buf.pin_memory().to(dev, non_blocking=True)
    out, o = [], 0
    for lst in lists:
        out.append(buf[o:o + len(lst)])
        o += len(lst)
    return out


def _nonzero_n(mask, n):
    """Positions of the n true entries of a 1-D mask, n known on the host: no
    read-back of the count (torch.nonzero_static)."""
    return torch.nonzero_static(mask, size=int(n)).view(-1)


def _count_by(idx, n):
    """Integer histogram of idx over [0, n) without a host sync (torch.bincount
    reads the maximum back): exact in any order."""
    return torch.zeros(n, dtype=torch.int64, device=idx.device).scatter_add_(0, idx, torch.ones_like(idx))


def tile_widths(F, tile):
    """Feature-tile widths covering F: `tile` wide each (the last takes the
    rest), or an explicit list of widths summing to F."""
    if isinstance(tile, (list, tuple)):
        widths = [int(w) for w in tile]
        if sum(widths) != F or min(widths) <= 0:
            raise ValueError("tile widths %s do not cover %d features" % (widths, F))
        return widths
    return [min(int(tile), F - c0) for c0 in range(0, F, int(tile))]


def balanced_cut_points(in_degree, parts):
    """edge_balanced_cuts on the device, without a read-back: an int64 tensor
    [0 = c_0 <= ... <= c_P = N] (the targets E * p // parts searched in the
    in-degree prefix sum, made monotone)."""
    N = in_degree.numel()
    dev = in_degree.device
    if N == 0 or parts <= 1:
        return _dev_ints([[0] * parts + [N]], dev)[0]
    csum = torch.cumsum(in_degree.to(torch.int64), 0)
    p = torch.arange(1, parts, dtype=torch.int64, device=dev)
    found = torch.searchsorted(csum, (csum[-1] * p) // parts, right=True)
    found = torch.cummax(found, 0).values
    ends = torch.tensor([0, N], dtype=torch.int64, device=dev)
    return torch.cat([ends[:1], found, ends[1:]])


def edge_balanced_cuts(in_degree, parts):
    """Row cut points [0=c_0 <= ... <= c_P = N] with ~equal edges per part
    (balanced_cut_points, read back with one host sync)."""
    return [int(c) for c in balanced_cut_points(in_degree, parts).tolist()]


# ---------------------------------------------------------------------------
# host tensors: no CPU fallback.  The gloo tests (tests/test_dist_gloo.py) run
# this module's distributed logic -- plans, covers, slice builds, exchanges --
# on CPU with host twins of the native kernels they install themselves
# (tests/_host_twins.py); without them a host tensor raises.
# ---------------------------------------------------------------------------
_HOST_TWINS = None


def install_host_twins(twins):
    """Test hook: `twins` provides host forms of the native pieces (plan,
    gather_rows, sum_returned_rows, segment_sum_in_order, norm_local,
    gat_loops, gat_cover_forward).  None removes them."""
    global _HOST_TWINS
    _HOST_TWINS = twins


def _host(what):
    if _HOST_TWINS is None:
        raise RuntimeError("mi355_mp.dist: %s on host tensors -- there is no CPU fallback: the engine runs on ROCm "
                           "device tensors" % what)
    return getattr(_HOST_TWINS, what)


def _plan_launch(key, other, num_nodes, cuts, cuts_d, rank, world):
    """mp_shard_plan of rank `rank` on the device, without a read-back: the
    full-size outputs (edge_pos, local key, local other, halo_nodes) and the
    device count vector [n edges, n halo, per-owner halo counts...]."""
    from . import _lib
    lib = _lib.load()
    dev = key.device
    key = key.to(torch.int64).contiguous()
    other = other.to(torch.int64).contiguous()
    E = key.numel()
    edge_pos = torch.empty(E, dtype=torch.int64, device=dev)
    lkey = torch.empty_like(edge_pos)
    lother = torch.empty_like(edge_pos)
    halo = torch.empty(num_nodes, dtype=torch.int64, device=dev)
    counts = torch.empty(2 + world, dtype=torch.int64, device=dev)
    ws = torch.empty(lib.mp_shard_plan_workspace(E, num_nodes), dtype=torch.uint8, device=dev)
    _lib.check(lib.mp_shard_plan(key.data_ptr(), other.data_ptr(), E, num_nodes, cuts_d.data_ptr(), world, rank,
                                 cuts[rank], cuts[rank + 1], edge_pos.data_ptr(), lkey.data_ptr(),
                                 lother.data_ptr(), halo.data_ptr(), counts.data_ptr(), ws.data_ptr(),
                                 ws.numel(), _lib.stream_ptr(dev)), "mp_shard_plan")
    return edge_pos, lkey, lother, halo, counts


def _plan_finish(launched, c, num_nodes):
    """The compact plan from _plan_launch's outputs and its counts read back."""
    if c[1] < 0:
        raise IndexError("mi355_mp.dist: an edge endpoint lies outside [0, %d)" % num_nodes)
    edge_pos, lkey, lother, halo, _ = launched
    n = c[0]
    return edge_pos[:n].clone(), lkey[:n].clone(), lother[:n].clone(), halo[:c[1]].clone(), list(c[2:])


def _plan_native(key, other, num_nodes, cuts, rank, world):
    """The plan of rank `rank` on the device by mp_shard_plan (flag + scan, no
    sort): (edge_pos, local key, local other, halo_nodes, recv_counts) -- the
    positions of the rank's edges in the list's order, its destinations and
    sources renumbered [own rows ; sorted halo rows], the halo's global ids and
    their count per owner.  One host sync (the sizes)."""
    launched = _plan_launch(key, other, num_nodes, cuts, _dev_ints([cuts], key.device)[0], rank, world)
    return _plan_finish(launched, launched[4].tolist(), num_nodes)


class ShardPlan:
    """Everything rank `rank` needs to aggregate its destination rows."""

    def __init__(self, edge_index, num_nodes, rank, world, cuts=None, flow="source_to_target", edge_ids=None,
                 _planned=None):
        """edge_index: the global edge list, or any list holding (at least) this
        rank's edges in global order -- e.g. the rank's own in-edges from
        scatter_edges_by_owner; edge_ids then gives each listed edge's GLOBAL id
        (argmax ids stay global).  edge_pos indexes the list passed in."""
        i, j = (1, 0) if flow == "source_to_target" else (0, 1)
        dst_all, src_all = edge_index[i], edge_index[j]
        if cuts is None:
            deg = torch.bincount(dst_all, minlength=num_nodes)
            cuts = edge_balanced_cuts(deg, world)
        self.cuts = cuts
        self.rank, self.world = rank, world
        lo, hi = cuts[rank], cuts[rank + 1]
        self.lo, self.hi, self.n_own = lo, hi, hi - lo
        if _planned is None:
            plan = _plan_native if edge_index.is_cuda else _host("plan")
            _planned = plan(dst_all, src_all, num_nodes, cuts, rank, world)
        self.edge_pos, dst, local_src, halo_nodes, self.recv_counts = _planned
        self.halo_nodes = halo_nodes
        self.edge_gid = edge_ids[self.edge_pos] if edge_ids is not None else self.edge_pos
        self.local_edge_index = torch.stack([local_src, dst]) if i == 1 else torch.stack([dst, local_src])
        self.n_local_src = self.n_own + halo_nodes.numel()
        self.send_idx = None
        self.send_counts = None

    @classmethod
    def many(cls, edge_lists, num_nodes, rank, world, cuts, flows, edge_ids, group=None):
        """Several plans of one partition (e.g. GCN's forward and backward
        plans) built and their requests exchanged together: every plan's sizes
        and the peers' request counts come back in ONE host read, and all the
        requests travel in one all_to_all (per peer: plan 0's, plan 1's, ...).
        Each plan equals ShardPlan(...).exchange_requests(group)."""
        K = len(edge_lists)
        specs = []
        for ei, flow in zip(edge_lists, flows):
            i, j = (1, 0) if flow == "source_to_target" else (0, 1)
            specs.append((ei[i], ei[j]))
        dev = edge_lists[0].device
        if dev.type == "cuda":
            cuts_d = _dev_ints([cuts], dev)[0]
            launched = [_plan_launch(k, o, num_nodes, cuts, cuts_d, rank, world) for k, o in specs]
            cnt = torch.stack([l[4] for l in launched])                 # [K, 2 + world]
        else:
            host = [_host("plan")(k, o, num_nodes, cuts, rank, world) for k, o in specs]
            cnt = torch.tensor([[h[0].numel(), h[3].numel()] + list(h[4]) for h in host], dtype=torch.int64)
        W = 2 + world
        if _device_collectives(dev, group):
            rc_d = cnt[:, 2:].t().contiguous()                          # [world, K] rows requested per owner
            sc_d = torch.empty_like(rc_d)
            dist.all_to_all_single(sc_d.view(-1), rc_d.view(-1), group=group)
            allv = torch.cat([cnt.view(-1), sc_d.view(-1)]).tolist()
        else:
            ch = _stage_to_host(cnt)
            rc_h = ch[:, 2:].t().contiguous()
            sc_h = torch.empty_like(rc_h)
            dist.all_to_all_single(sc_h.view(-1), rc_h.view(-1), group=group)
            allv = ch.view(-1).tolist() + sc_h.view(-1).tolist()
        plans = []
        for k in range(K):
            c = allv[k * W:(k + 1) * W]
            planned = _plan_finish(launched[k], c, num_nodes) if dev.type == "cuda" else host[k]
            plans.append(cls(edge_lists[k], num_nodes, rank, world, cuts=cuts, flow=flows[k],
                             edge_ids=edge_ids[k], _planned=planned))
        sc = [allv[K * W + q * K:K * W + (q + 1) * K] for q in range(world)]    # [peer][plan]
        for k, p in enumerate(plans):
            p.send_counts = [sc[q][k] for q in range(world)]
        segs, offs = [], [0] * K
        for q in range(world):
            for k, p in enumerate(plans):
                segs.append(p.halo_nodes[offs[k]:offs[k] + p.recv_counts[q]])
                offs[k] += p.recv_counts[q]
        send = torch.cat(segs) if segs else torch.empty(0, dtype=torch.int64, device=dev)
        requests = torch.empty(sum(map(sum, sc)), dtype=torch.int64, device=dev)
        _a2a(requests, send.contiguous(), [sum(r) for r in sc],
             [sum(p.recv_counts[q] for p in plans) for q in range(world)], group)
        got, pos = [[] for _ in range(K)], 0
        for q in range(world):
            for k in range(K):
                got[k].append(requests[pos:pos + sc[q][k]])
                pos += sc[q][k]
        for k, p in enumerate(plans):
            p.send_idx = torch.cat(got[k]) - p.lo      # rows of my own block that peers need
        return plans

    def exchange_requests(self, group=None):
        """All-to-all of the requested node ids (once per plan; one host sync
        for the counts)."""
        dev = self.halo_nodes.device
        _, self.send_counts = _exchange_counts(_dev_ints([self.recv_counts], dev)[0], group)
        requests = torch.empty(sum(self.send_counts), dtype=torch.int64, device=dev)
        _a2a(requests, self.halo_nodes.contiguous(), self.send_counts, self.recv_counts, group)
        self.send_idx = requests - self.lo     # rows of my own block that peers need
        return self

    def local_buffer(self, F, dtype=torch.float32, device=None):
        """[n_own + n_halo, F] buffer: the owner writes rows [:n_own] (e.g. its
        X W GEMM output), exchange_into() fills the halo rows [n_own:]."""
        return torch.empty((self.n_local_src, F), dtype=dtype, device=device or self.halo_nodes.device)

    def exchange_into(self, x_local, gather_rows, group=None):
        """Pack the rows peers requested from x_local[:n_own] (native row
        gather) and receive this rank's halo rows straight into
        x_local[n_own:] (one all_to_all_single, no concatenation)."""
        F = x_local.shape[1]
        own = x_local[:self.n_own]
        send = gather_rows(own, self.send_idx) if self.send_idx.numel() else x_local.new_empty((0, F))
        _a2a(x_local[self.n_own:], send.contiguous(), self.recv_counts, self.send_counts, group)
        return x_local

    def local_tiles(self, F, tile=128, dtype=torch.float32, device=None):
        """Tile-major [n_own + n_halo, width] buffers covering F features, for
        OverlappedAggregation.step_tiled: each tile's halo rows are contiguous,
        so every tile is exchanged (and received in place) on its own.  tile:
        one width (the last tile takes the rest) or the list of widths."""
        dev = device or self.halo_nodes.device
        return [torch.empty((self.n_local_src, w), dtype=dtype, device=dev) for w in tile_widths(F, tile)]

    def halo_exchange(self, x_own, gather_rows, group=None):
        """[own rows ; halo rows] for this rank (allocating form)."""
        x_local = self.local_buffer(x_own.shape[1], x_own.dtype, x_own.device)
        x_local[:self.n_own].copy_(x_own)
        return self.exchange_into(x_local, gather_rows, group)

    def return_halo(self, halo_rows, group=None):
        """The reverse of exchange_into: rows living in this rank's halo
        ([n_halo, F], halo order) go back to their owners.  Returns the rows
        this rank receives, [len(send_idx), F], aligned with send_idx (peer
        order, then each peer's request order) -- the caller adds them into
        its own rows (a row requested by several peers appears once per peer)."""
        F = halo_rows.shape[1]
        out = halo_rows.new_empty((int(self.send_idx.numel()), F))
        _a2a(out, halo_rows.contiguous(), self.send_counts, self.recv_counts, group)
        return out

    def global_edge_ids(self, arg_local, n_edges_global):
        """Arg of a max/min over this rank's edges (local positions; the local
        edge list is the global one restricted, in global order, so the first
        maximal local edge IS the first maximal global edge) -> global edge
        ids; the empty-row sentinel (number of local edges) becomes the
        reference's sentinel, the global edge count (edge ids stay
        global, argmax bit-exact)."""
        n_local = int(self.edge_pos.numel())
        if n_local == 0:
            return torch.full_like(arg_local, n_edges_global)
        ids = self.edge_gid[arg_local.clamp(max=n_local - 1)]
        return torch.where(arg_local >= n_local, torch.full_like(ids, n_edges_global), ids)


def _sum_returned_rows(plan, back):
    """Rows returned by the peers (plan.return_halo: aligned with send_idx, peer
    order, then each peer's request order) summed into this rank's own rows in
    that fixed order: the native segmented sum keyed on send_idx.
    Deterministic."""
    if not back.is_cuda:
        return _host("sum_returned_rows")(plan, back)
    from . import ops
    from .graph import csr_for_index
    return ops._aggregate(csr_for_index(plan.send_idx, plan.n_own), "eid", back.contiguous(), None, "sum", 0,
                          None)[0]


class _HaloRows(torch.autograd.Function):
    """x_own [n_own, F] -> [own rows ; halo rows] over a pull plan; the backward
    sends the halo rows' gradients back to their owners (return_halo), which add
    them to their own rows' gradients (_sum_returned_rows)."""

    @staticmethod
    def forward(ctx, x_own, plan, group):
        ctx.plan, ctx.group = plan, group
        x_local = plan.local_buffer(x_own.shape[1], dtype=x_own.dtype, device=x_own.device)
        x_local[:plan.n_own].copy_(x_own)
        if x_own.is_cuda:
            from . import ops
            plan.exchange_into(x_local, ops.gather_rows, group)
        else:
            plan.exchange_into(x_local, _host("gather_rows"), group)
        return x_local

    @staticmethod
    def backward(ctx, g):
        plan = ctx.plan
        g = g.contiguous()
        gx = g[:plan.n_own]
        back = plan.return_halo(g[plan.n_own:], ctx.group)
        if back.shape[0]:
            gx = gx + _sum_returned_rows(plan, back)
        return gx.contiguous(), None, None


def halo_rows(x_own, plan, group=None):
    """Differentiable [own rows ; halo rows] of x over a pull plan (after
    plan.exchange_requests()): one all_to_all forward, the reverse one backward."""
    if x_own.shape[0] != plan.n_own:
        raise ValueError("mi355_mp.dist: x_own has %d rows, this rank owns %d" % (x_own.shape[0], plan.n_own))
    return _HaloRows.apply(x_own, plan, group)


def sharded_propagate(plan, x_own, local_aggregate, gather_rows, edge_weight=None, group=None, n_edges_global=None):
    """One sharded aggregation: halo exchange then local aggregation.

    local_aggregate(x_local, local_edge_index, n_dst, n_src, edge_weight) ->
    [n_own, F], or (out, arg) for max/min with arg in LOCAL edge positions:
    then arg is returned as global edge ids (n_edges_global = the sentinel).
    edge_weight: per-edge weights in GLOBAL edge order (sliced by the plan).
    The backward of a sum is the same call on the transposed plan (see
    ShardedGraph): the gradient rows of remote destinations come in as halo
    rows, so every source row is summed in global edge order by its owner.
    """
    x_local = plan.halo_exchange(x_own, gather_rows, group)
    w = edge_weight[plan.edge_pos] if edge_weight is not None else None
    res = local_aggregate(x_local, plan.local_edge_index, plan.n_own, plan.n_local_src, w)
    if isinstance(res, tuple):
        out, arg = res
        if n_edges_global is None:
            raise ValueError("sharded_propagate: a max/min aggregation needs n_edges_global "
                             "(the global edge count, the empty-row argmax sentinel)")
        return out, plan.global_edge_ids(arg, n_edges_global)
    return res


# ---------------------------------------------------------------------------
# building the shards from per-rank slices of the edge list (no rank holds it all)
# ---------------------------------------------------------------------------

def scatter_edges_by_owner(key, cuts, payloads, group=None):
    """Route the entries of `payloads` (1-D int64 / float32 tensors aligned with
    `key`) to the rank owning key (range partition `cuts`): the counts, then
    every payload in ONE all_to_all (int64 columns; a float32 payload travels
    as its bits), one host sync.  The result is the concatenation over sender
    ranks in rank order, each sender's entries in their original order -- so
    when every rank holds a contiguous slice of the global edge list (rank r
    before rank r + 1), each rank receives its edges in GLOBAL order."""
    return scatter_edges_by_owner_many([(key, payloads)], cuts, group)[0]


def scatter_edges_by_owner_many(jobs, cuts, group=None):
    """scatter_edges_by_owner for several (key, payloads) jobs in one exchange:
    one all_to_all of the counts ([world, jobs], one host sync) and one of all
    the payloads (columns padded to the widest job; to each peer the jobs
    follow one another).  Returns one list of payloads per job, each exactly
    what scatter_edges_by_owner(key, cuts, payloads) returns."""
    world = len(cuts) - 1
    K = len(jobs)
    dev = jobs[0][0].device
    ncol = max(len(p) for _, p in jobs)
    cuts_t, bins = _dev_ints([cuts[1:], range(world * K + 1)], dev)
    keys, packs = [], []
    for k, (key, payloads) in enumerate(jobs):
        cols = []
        for p in payloads:
            if p.dtype == torch.float32:
                cols.append(p.view(torch.int32).to(torch.int64))
            elif p.dtype == torch.int64:
                cols.append(p)
            else:
                raise TypeError("scatter_edges_by_owner: payloads are int64 or float32 (got %s)" % p.dtype)
        cols += [key.new_zeros(key.shape, dtype=torch.int64)] * (ncol - len(cols))
        keys.append(torch.searchsorted(cuts_t, key, right=True) * K + k)
        packs.append(torch.stack(cols, 1) if ncol else key.new_empty((key.numel(), 0), dtype=torch.int64))
    ck = torch.cat(keys) if K > 1 else keys[0]
    srt = torch.sort(ck, stable=True)      # by owner, then job; each job's entries keep their order
    # per (owner, job) counts from the sorted keys (no atomics on world * K bins)
    bounds = torch.searchsorted(srt.values, bins)
    sc, rc = _exchange_counts((bounds[1:] - bounds[:-1]).view(world, K), group)
    packed = (torch.cat(packs) if K > 1 else packs[0])[srt.indices].contiguous()
    buf = packed.new_empty((sum(map(sum, rc)), ncol))
    _a2a(buf, packed, [sum(r) for r in rc], [sum(r) for r in sc], group)
    outs, pos = [[] for _ in range(K)], 0
    for q in range(world):            # from sender q: job 0's entries, job 1's, ...
        for k in range(K):
            outs[k].append(buf[pos:pos + rc[q][k]])
            pos += rc[q][k]
    res = []
    for k, (key, payloads) in enumerate(jobs):
        got = torch.cat(outs[k]) if world > 1 else outs[k][0]
        one = []
        for j, p in enumerate(payloads):
            c = got[:, j].contiguous()
            one.append(c.to(torch.int32).view(torch.float32) if p.dtype == torch.float32 else c)
        res.append(one)
    return res


def _segment_sum_in_order(index, values, n):
    """out[k] = sum of values[index == k] left to right (the CPU scatter_add_'s
    order): the transposed CSR's serial segment sum (mp_segment_sum_serial_f32)."""
    if not values.is_cuda:
        return _host("segment_sum_in_order")(index, values, n)
    from . import ops
    from .graph import CSR
    return ops.segment_sum_serial(CSR(index, None, n, index.numel()), values)


def gcn_shards_from_slices(edge_slice, slice_offset, num_nodes, rank, world, group=None, edge_weight=None,
                           improved=False, structure_only=False):
    """GCNConv's graph (add_remaining_self_loops + deg over row + norm, PyG 1.4.3
    [U5]) for a graph held as per-rank slices: rank r holds the global edges
    [slice_offset, slice_offset + n_r) (slices contiguous, in rank order).  No
    rank ever holds the whole edge list:

      1. self loops are dropped locally; kept-edge global ids follow from the
         kept counts of the earlier ranks (one all_gather of two ints);
      2. cuts: the in-degree (integer, so exact under any reduction order; +1
         for the appended loops) is all-reduced, then edge-balanced;
      3. a node's pre-existing loops go to its owner, the LAST one's weight wins
         (upstream's sequential index_put_);
      4. the out-edges of each rank's rows come to it in global order
         (scatter_edges_by_owner by source): the degree is their edge-order sum,
         then + the loop weight -- the reference's scatter_add arithmetic;
      5. the in-edges of each rank's rows come to it in global order (by
         destination); the N loops are appended last with ids E_kept + v;
      6. the norm needs deg of remote endpoints: it travels over each plan's
         halo exchange (ShardedGraph.for_gcn_from_slices).

    Returns a dict: cuts, E (total edges after the loops), deg (own rows),
    fwd = (edge_index [2, m] global ids, global edge ids, weights) of the
    in-edges, bwd = the same for the out-edges.

    structure_only=True (GATConv: remove_self_loops + add_self_loops gives the
    same edge list): steps 3 and 4 are skipped; deg and bwd are None and the
    fwd weights are ones."""
    row, col = edge_slice[0].to(torch.int64), edge_slice[1].to(torch.int64)
    dev = row.device
    N = int(num_nodes)
    n = row.numel()
    keep = row != col
    # 1-2. one gather of (slice size, kept edges, offset, bad-id flag) from every
    # rank and the all-reduced in-degree (+1 for every node's loop) -> cuts, all
    # read back with ONE host sync: every rank learns whether ANY rank holds an
    # id outside [0, N) before the first collective whose size depends on the
    # data, and all of them raise together (a lone raising rank would leave its
    # peers waiting in the next collective); every rank checks every offset the
    # same way.  Ids outside [0, N) are counted in a spare bin of the degree.
    if n:
        bad_t = ((torch.minimum(row.min(), col.min()) < 0) | (torch.maximum(row.max(), col.max()) >= N))
        n_off = _dev_ints([[n, int(slice_offset)]], dev)[0]
        mine = torch.stack([n_off[0], keep.sum(), n_off[1], bad_t.to(torch.int64)])
        inr = keep & (col >= 0) & (col < N)
        deg_in = _count_by(torch.where(inr, col, torch.full_like(col, N)), N + 1)[:N]
    else:
        mine = torch.tensor([0, 0, int(slice_offset), 0], dtype=torch.int64, device=dev)
        deg_in = torch.zeros(N, dtype=torch.int64, device=dev)
    if _device_collectives(dev, group):
        got = torch.empty((world, 4), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(got.view(-1), mine, group=group)
        dist.all_reduce(deg_in, group=group)
        allv = torch.cat([got.view(-1), balanced_cut_points(deg_in + 1, world)]).tolist()
        sizes = [allv[4 * r:4 * r + 4] for r in range(world)]
        cuts = allv[4 * world:]
    else:
        h = _stage_to_host(torch.cat([mine, deg_in]))
        got = torch.empty((world, 4), dtype=torch.int64)
        dist.all_gather_into_tensor(got.view(-1), h[:4].clone(), group=group)
        deg_h = h[4:].clone()
        dist.all_reduce(deg_h, group=group)
        sizes = got.tolist()
        cuts = edge_balanced_cuts(deg_h + 1, world)
    del deg_in
    if any(sz[3] for sz in sizes):
        raise IndexError("mi355_mp.dist: an edge of some rank's slice names a node outside [0, %d)" % N)
    for r, sz in enumerate(sizes):
        if sz[2] != sum(t[0] for t in sizes[:r]):
            raise ValueError("gcn_shards_from_slices: rank %d's slice offset %d does not follow the earlier slices"
                             % (r, sz[2]))
    n_kept = sizes[rank][1]
    w = (edge_weight.to(torch.float32) if edge_weight is not None
         else torch.ones(n, dtype=torch.float32, device=dev))
    fill = 2.0 if improved else 1.0
    kept = _nonzero_n(keep, n_kept)
    k_off = sum(sz[1] for sz in sizes[:rank])
    E_kept = sum(sz[1] for sz in sizes)
    kr, kc, kw = row[kept], col[kept], w[kept]
    kgid = k_off + torch.arange(n_kept, dtype=torch.int64, device=dev)
    lo, hi = cuts[rank], cuts[rank + 1]
    own = torch.arange(lo, hi, dtype=torch.int64, device=dev)
    if structure_only:
        f_row, f_col, f_gid = scatter_edges_by_owner(kc, cuts, [kr, kc, kgid], group)
        fwd = (torch.stack([torch.cat([f_row, own]), torch.cat([f_col, own])]), torch.cat([f_gid, E_kept + own]),
               torch.ones(f_row.numel() + hi - lo, dtype=torch.float32, device=dev))
        return {"cuts": cuts, "E": E_kept + N, "deg": None, "fwd": fwd, "bwd": None}
    # 3-5 in ONE exchange: the pre-existing loops to the node's owner, the
    # out-edges of each rank's rows (by source) and its in-edges (by destination),
    # each in global order
    lidx = _nonzero_n(~keep, n - n_kept)
    lv, lw = row[lidx], w[lidx]
    (rv, rpos, rw), (b_row, b_col, b_gid, b_w), (f_row, f_col, f_gid, f_w) = scatter_edges_by_owner_many(
        [(lv, [lv, lidx + slice_offset, lw]), (kr, [kr, kc, kgid, kw]), (kc, [kr, kc, kgid, kw])], cuts, group)
    # 3. pre-existing loops -> the node's owner; the last one (largest position) wins
    loop_w = torch.full((hi - lo,), fill, dtype=torch.float32, device=dev)
    if rv.numel():
        best = torch.full((hi - lo,), -1, dtype=torch.int64, device=dev)
        best.scatter_reduce_(0, rv - lo, rpos, "amax")
        last = rpos == best[rv - lo]
        # the winners' weights into their rows; the other entries land in a spare slot
        slot = torch.where(last, rv - lo, torch.full_like(rv, hi - lo))
        lw_ext = torch.cat([loop_w, loop_w.new_zeros(1)])
        lw_ext.scatter_(0, slot, torch.where(last, rw, torch.zeros_like(rw)))
        loop_w = lw_ext[:hi - lo]
    # 4. out-edges of my rows, global order -> deg = scatter_add(w, row) in edge order, then the loop
    deg = _segment_sum_in_order(b_row - lo, b_w, hi - lo)
    deg = deg + loop_w
    # 5. in-edges of my rows, global order; the loops last
    loop_gid = E_kept + own
    fwd = (torch.stack([torch.cat([f_row, own]), torch.cat([f_col, own])]), torch.cat([f_gid, loop_gid]),
           torch.cat([f_w, loop_w]))
    bwd = (torch.stack([torch.cat([b_row, own]), torch.cat([b_col, own])]), torch.cat([b_gid, loop_gid]),
           torch.cat([b_w, loop_w]))
    return {"cuts": cuts, "E": E_kept + N, "deg": deg, "fwd": fwd, "bwd": bwd}


def _exchange_into_many(plans, bufs, gather_rows, group=None):
    """exchange_into() of several plans of one group in ONE all_to_all (per
    peer: plan 0's rows, plan 1's, ...): bufs[k] is plans[k]'s [n_local_src, F]
    buffer, its own rows filled; its halo rows are written."""
    world = plans[0].world
    sends = [gather_rows(b[:p.n_own], p.send_idx) if p.send_idx.numel() else b.new_empty((0, b.shape[1]))
             for p, b in zip(plans, bufs)]
    segs, offs = [], [0] * len(plans)
    for q in range(world):
        for k, p in enumerate(plans):
            segs.append(sends[k][offs[k]:offs[k] + p.send_counts[q]])
            offs[k] += p.send_counts[q]
    recv = bufs[0].new_empty((sum(p.n_local_src - p.n_own for p in plans), bufs[0].shape[1]))
    _a2a(recv, torch.cat(segs).contiguous(), [sum(p.recv_counts[q] for p in plans) for q in range(world)],
         [sum(p.send_counts[q] for p in plans) for q in range(world)], group)
    pos, offs = 0, [p.n_own for p in plans]
    for q in range(world):
        for k, p in enumerate(plans):
            n = p.recv_counts[q]
            if n:
                bufs[k][offs[k]:offs[k] + n].copy_(recv[pos:pos + n])
            pos += n
            offs[k] += n
    return bufs


def _norms_over_plans(plans, deg_own, w_locals, group=None):
    """GCN norm dinv[row] * w * dinv[col] of each plan's local edges: the
    degrees of the halo endpoints come over the plans' exchanges (one float
    per halo node, all plans in one all_to_all), dinv = deg^-1/2 with inf -> 0
    (torch's CPU pow(-0.5) rounding: the native mp_gcn_norm_from_deg_f32 on
    the device)."""
    bufs = []
    for p in plans:
        degl = deg_own.new_empty((p.n_local_src, 1))
        degl[:p.n_own, 0] = deg_own
        bufs.append(degl)
    if deg_own.is_cuda:
        from . import ops
        _exchange_into_many(plans, bufs, ops.gather_rows, group)
        # local ids < n_own + n_halo by the plans' construction: no range read-back
        return [ops.norm_from_degree(p.local_edge_index[0], p.local_edge_index[1], b.view(-1).clone(), w,
                                     trusted=True) for p, b, w in zip(plans, bufs, w_locals)]
    _exchange_into_many(plans, bufs, _host("gather_rows"), group)
    return [_host("norm_local")(p.local_edge_index[0], p.local_edge_index[1], b.view(-1), w)
            for p, b, w in zip(plans, bufs, w_locals)]


class HaloCover:
    """Hybrid halo exchange of a sum aggregation: fewer rows over the links.

    The pull exchange (ShardPlan) ships x_j of every remote source of the
    rank's in-edges.  A cross edge j -> i (j owned by q, i by p) can equally be
    covered by q shipping its PARTIAL row of i, sum over its own sources j of
    w_ji x_j.  Covering every cross edge of the pair (q, p) with the fewest rows
    is a minimum vertex cover of the bipartite cross-edge graph; on power-law
    graphs a hub source is best pulled and a hub destination best pushed.
    Rule (one-time, on the receiver p, from its own in-edges): an edge goes to
    the endpoint with the larger cross-degree of the pair (ties: pull), then two
    clean-ups -- an edge whose source is pulled anyway is pulled, an edge whose
    destination is pushed anyway is pushed; per owner the fewest rows of that
    cover, pull only and push only is kept (on a dense pair the degree rule can
    lose to either), so the cover never ships more rows than the pull halo.  On
    RMAT graphs it ships 0.56-0.57x the pull rows, within 2 % of the exact
    minimum cover (Konig / Hopcroft-Karp; tools/exp_halo_cover.py,
    profiles/r03_halo_cover_model.log).

    Per step the sender fills its whole send buffer with ONE aggregation over a
    "send graph": a pulled row is a row with one edge of weight 1.0 (an exact
    copy), a pushed row sums its push edges in global edge order.  The receiver
    aggregates its boundary edges over [own rows ; received rows]: the pulled
    edges with their weights plus one weight-1.0 edge per received partial.
    Rows sum the same terms as the single-GPU kernel, regrouped: within the
    1e-5 * sum|w x| bound, not bit-identical (exact on integer-valued data).

    Built from a forward ShardPlan (flow source_to_target) and the plan's local
    edge weights; every rank of `group` builds its cover together (three
    all_to_alls of the requests)."""

    def __init__(self, plan, w_local, group=None, edge_ids=False):
        dev = plan.halo_nodes.device
        world, rank = plan.world, plan.rank
        n_own = plan.n_own
        lei = plan.local_edge_index
        src_l, dst_l = lei[0], lei[1]
        E_l = src_l.numel()
        if w_local is None:
            w_local = torch.ones(E_l, dtype=torch.float32, device=dev)
        w_local = w_local.to(torch.float32)
        N = plan.cuts[-1]
        cut_all = _dev_ints([plan.cuts], dev)[0]
        cuts_t = cut_all[1:]
        stride = max(n_own, 1)
        nkey = world * stride
        # Every edge of the plan stays in place and the remote ones are masked (no
        # compaction before the sizes are known): the whole cover is computed on the
        # device and its sizes come back in ONE host read, with the request counts
        # of the peers (three host syncs for the build in all, whatever the graph).
        remm = src_l >= n_own                                  # remote source (a halo slot)
        if plan.halo_nodes.numel():
            gsrc = torch.where(remm, plan.halo_nodes[(src_l - n_own).clamp(min=0)], torch.zeros_like(src_l))
        else:
            gsrc = torch.zeros_like(src_l)
        r_own = torch.searchsorted(cuts_t, gsrc, right=True)   # owner of the source (remote edges)
        key = r_own * stride + dst_l                           # (owner, destination) of a cross edge

        spread = torch.arange(E_l, device=dev) & 1023

        def count(idx, mask, n):
            # masked-out entries go to 1024 spare bins (not all onto one bin: an
            # atomic hot spot that held the P = 2 build's device for 1.6 s)
            i = torch.where(mask, idx, n + spread)
            return torch.zeros(n + 1024, dtype=torch.int64, device=dev).scatter_add_(0, i, torch.ones_like(i))[:n]

        def per_owner_nodes(flags):      # flagged global nodes per owner (contiguous ranges)
            cz = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(flags.to(torch.int64), 0)])
            return cz[cut_all[1:]] - cz[cut_all[:-1]]

        def per_owner_keys(flags):       # flagged (owner, destination) keys per owner
            return flags.to(torch.int64).view(world, stride).sum(1)

        # --- the cover: larger cross-degree endpoint, then the two clean-ups, then per
        # owner the fewest rows of {this cover, pull only, push only}
        cs = count(gsrc, remm, N)                              # cross out-degree of each remote source
        cd = count(key, remm, nkey)                            # cross in-degree per (owner, destination)
        pick = cs[gsrc] >= cd[key]
        in_s = count(gsrc, remm & pick, N) > 0
        push = remm & ~in_s[gsrc]
        in_d = count(key, push, nkey) > 0
        push = remm & in_d[key]
        in_s = count(gsrc, remm & ~push, N) > 0
        cover_q = per_owner_nodes(in_s) + per_owner_keys(in_d)
        pull_q = per_owner_nodes(cs > 0)
        push_q = per_owner_keys(cd > 0)
        mode = torch.where((pull_q <= cover_q) & (pull_q <= push_q), 0, torch.where(push_q < cover_q, 1, 2))
        m = mode[r_own]
        push = remm & torch.where(m == 0, torch.zeros_like(push), torch.where(m == 1, torch.ones_like(push), push))
        pull = remm & ~push
        in_s = count(gsrc, pull, N) > 0
        in_d = count(key, push, nkey) > 0
        del cs, cd, pick
        nS = per_owner_nodes(in_s)                             # pulled rows per owner
        nD = per_owner_keys(in_d)                              # pushed rows per owner
        nP = per_owner_keys(count(key, push, nkey))            # push edges per owner
        cnt = torch.stack([nS, nD, nP], 1).contiguous()
        extra = torch.stack([(~remm).sum(), pull.sum(), push.sum()])
        # host read 1 (+ the peers' counts): sizes of everything below
        if _device_collectives(dev, group):
            cnt_in = torch.empty_like(cnt)
            dist.all_to_all_single(cnt_in.view(-1), cnt.view(-1), group=group)
            allv = torch.cat([cnt.view(-1), cnt_in.view(-1), extra]).tolist()
            mine_c, peer_c = allv[:3 * world], allv[3 * world:6 * world]
            n_int, n_pull, n_push = allv[6 * world:]
        else:
            allv = torch.cat([cnt.view(-1), extra]).tolist()
            mine_c = allv[:3 * world]
            n_int, n_pull, n_push = allv[3 * world:]
            ch = torch.tensor(mine_c, dtype=torch.int64).view(world, 3)
            rh = torch.empty_like(ch)
            dist.all_to_all_single(rh.view(-1), ch.view(-1), group=group)
            peer_c = rh.view(-1).tolist()
        nS_l, nD_l, nP_l = mine_c[0::3], mine_c[1::3], mine_c[2::3]
        snS, snD, snP = peer_c[0::3], peer_c[1::3], peer_c[2::3]
        nS_tot, nD_tot = sum(nS_l), sum(nD_l)
        # --- the plan's edges by class in plan (= global edge) order: interior,
        # pulled, pushed (a stable partition: each class's positions ascending, the
        # sizes known from the read above -- no sort)
        idx_int = _nonzero_n(~remm, n_int)
        idx_pull = _nonzero_n(remm & ~push, n_pull)
        idx_push = _nonzero_n(push, n_push)
        self.int_src, self.int_dst, self.int_w = src_l[idx_int], dst_l[idx_int], w_local[idx_int]
        S = _nonzero_n(in_s, nS_tot)                           # ascending node ids: grouped by owner
        D = _nonzero_n(in_d, nD_tot)                           # ascending (owner, destination) keys
        s_rank = torch.cumsum(in_s, 0) - 1                    # position of a pulled node in S
        d_rank = torch.cumsum(in_d, 0) - 1                    # position of a pushed key in D
        del in_s, in_d
        S_own = torch.searchsorted(cuts_t, S, right=True)
        D_own = D // stride
        self.recv_counts = [a_ + b_ for a_, b_ in zip(nS_l, nD_l)]
        off = [0]
        for c in self.recv_counts:
            off.append(off[-1] + c)
        off_t, nS_t, S_start, D_start = _dev_ints([off[:-1], nS_l, [sum(nS_l[:q]) for q in range(world)],
                                                   [sum(nD_l[:q]) for q in range(world)]], dev)
        # halo slot of each pulled source / pushed destination row: per owner q,
        # [its pulled rows ; its partial rows]
        s_pos = s_rank[gsrc[idx_pull]]
        s_q = S_own[s_pos]
        pull_halo = n_own + off_t[s_q] + (s_pos - S_start[s_q])
        d_q = D_own
        d_halo = n_own + off_t[d_q] + nS_t[d_q] + (torch.arange(nD_tot, device=dev) - D_start[d_q])
        self.bnd_src = torch.cat([pull_halo, d_halo])
        self.bnd_dst = torch.cat([dst_l[idx_pull], D - d_q * stride])
        self.bnd_w = torch.cat([w_local[idx_pull], torch.ones(nD_tot, dtype=torch.float32, device=dev)])
        # kept for GatHaloCover: plan positions of the interior and pulled edges, the
        # halo slot of each pulled one, and per pushed row its destination
        self.int_pos, self.pull_pos, self.pull_halo = idx_int, idx_pull, pull_halo
        self.push_dst, self.push_halo = D - d_q * stride, d_halo
        self.n_push_rows_to = list(nD_l)     # pushed rows this rank receives, per owner
        self.n_halo = off[-1]
        self.n_local_src = n_own + self.n_halo
        self.n_pull_rows, self.n_push_rows = nS_tot, nD_tot
        self.n_pull_edges, self.n_push_edges = n_pull, n_push
        # --- requests to the owners: pulled ids, and the push edges (source, partial
        # row, weight) grouped by owner, global edge order inside (a stable sort)
        p_own = r_own[idx_push]
        p_key = key[idx_push]
        p_row = d_rank[p_key] - D_start[p_own]
        del s_rank, d_rank
        # grouped by owner, each group in edge order (per-owner counts known: no sort)
        ord_p = torch.cat([_nonzero_n(p_own == q, nP_l[q]) for q in range(world)]) if world else p_own
        # the push edges in the order they go out (plan positions), and their counts
        # per owner both ways (GatHaloCover's alpha travels back along them)
        self.push_pos = idx_push[ord_p]
        self.push_edges_to, self.push_edges_from = list(nP_l), list(snP)
        req = S.new_empty(sum(snS))
        _a2a(req, S.contiguous(), snS, nS_l, group)
        lo = plan.lo
        # the push edges' (source, partial row, weight bits[, global edge id]) in one all_to_all
        cols = [gsrc[idx_push], p_row, w_local[idx_push].view(torch.int32).to(torch.int64)]
        if edge_ids:
            cols.append(plan.edge_gid[idx_push].to(torch.int64))
        pk = torch.stack(cols, 1)[ord_p]
        pk_in = pk.new_empty((sum(snP), len(cols)))
        _a2a(pk_in, pk.contiguous(), snP, nP_l, group)
        ps, pr = pk_in[:, 0], pk_in[:, 1]
        pw = pk_in[:, 2].to(torch.int32).view(torch.float32)
        # edge_ids: the GLOBAL id of every push edge this rank sums for its peers, in
        # send-graph order (the attention-dropout key of a pushed GAT piece's edges)
        self.push_gid = pk_in[:, 3].contiguous() if edge_ids else None
        # --- the send graph: rows = this rank's send buffer (per peer: pulled rows, then partial rows)
        self.send_counts = [a_ + b_ for a_, b_ in zip(snS, snD)]
        self.send_pull_counts, self.send_push_counts = snS, snD
        base = [0]
        for c in self.send_counts:
            base.append(base[-1] + c)
        ar = torch.arange(world, device=dev)
        snS_t, snP_t, base_t, sS_start = _dev_ints([snS, snP, base[:-1], [sum(snS[:k]) for k in range(world)]], dev)
        peer_s = torch.repeat_interleave(ar, snS_t, output_size=sum(snS))
        peer_p = torch.repeat_interleave(ar, snP_t, output_size=sum(snP))
        pull_rows = base_t[peer_s] + (torch.arange(req.numel(), device=dev) - sS_start[peer_s])
        push_rows = base_t[peer_p] + snS_t[peer_p] + pr
        # every requested row is one of this rank's own rows by construction (the
        # requests name sources in [lo, hi) of the shared cuts)
        self.send_src = torch.cat([req - lo, ps - lo])
        self.send_dst = torch.cat([pull_rows, push_rows])
        self.send_w = torch.cat([torch.ones(req.numel(), dtype=torch.float32, device=dev), pw])
        self.n_send = base[-1]
        self.n_own = n_own


_COMPUTE_STREAMS = {}


class compute_stream:
    """Context: run the enclosed device work on this process's compute stream
    of the device (one non-default HIP stream per device), ordered after
    everything already queued on the caller's current stream, and make the
    caller's stream wait for it on exit.

    Why: on ROCm, kernels on the legacy default stream never ran beside
    RCCL's kernels -- measured at one RCCL rank with a non-empty self split
    (bench.py --emulate-peers, profiles/r05_rccl_stream_probe.json): an
    all_to_all started async next to an aggregation on the default stream took
    as long as the two in a row (hidden_frac -0.05, no concurrent kernel in the
    trace), while the same aggregation on a stream of its own hid half the
    exchange (hidden_frac 0.51 / 0.54 at P = 8 / 2, RCCL and k_agg_flat
    intervals overlapping in the trace).  Host tensors: no-op."""

    def __init__(self, device):
        self.dev = torch.device(device)
        self.cs = self.cur = self.ctx = None

    def __enter__(self):
        if self.dev.type != "cuda":
            return None
        idx = self.dev.index if self.dev.index is not None else torch.cuda.current_device()
        cs = _COMPUTE_STREAMS.get(idx)
        if cs is None:
            cs = _COMPUTE_STREAMS[idx] = torch.cuda.Stream(device=idx)
        self.cur = torch.cuda.current_stream(idx)
        if self.cur == cs:
            return cs                     # already on it (nested)
        self.cs = cs
        cs.wait_stream(self.cur)
        self.ctx = torch.cuda.stream(cs)
        self.ctx.__enter__()
        return cs

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
            self.cur.wait_stream(self.cs)
        return False


_SIDE_STREAMS = {}


def _side_stream(device):
    """A second non-default stream per device: OverlappedAggregation's interior
    passes beside its send packing (split_interior)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _SIDE_STREAMS.get(idx)
    if st is None:
        st = _SIDE_STREAMS[idx] = torch.cuda.Stream(device=idx)
    return st


class OverlappedAggregation:
    """GCN-style sharded aggregation with the halo exchange hidden behind the
    interior edges.

    The rank's in-edges split into interior edges (source owned by this rank)
    and boundary edges (source in the halo), each a cached CSR in global edge
    order.  One step:
      1. pack the rows peers asked for (native row gather),
      2. start the all_to_all (RCCL runs on its own stream),
      3. aggregate the interior edges into `out` meanwhile,
      4. wait for the halo, then aggregate the boundary edges on top of `out`
         (MP_FLAG_INIT_FROM_OUT) and add the bias once.
    A row's sum is (interior part) + (boundary part, in order): within the
    1e-5 bound of the single-GPU order, not bit-identical to it.
    """

    def __init__(self, plan, edge_weight=None, chunk=None, local_weights=False, cover=False, group=None):
        """edge_weight: per-edge weights of the list the plan was built from
        (indexed by plan.edge_pos); local_weights=True: already in the plan's
        local edge order.  cover=True: the hybrid pull / push exchange of
        HaloCover (fewer rows over the links; built collectively over `group`),
        else the plan's pull exchange."""
        from .graph import Graph
        self.plan = plan
        self.n_own = plan.n_own
        lei = plan.local_edge_index
        src_local = lei[0]
        interior = src_local < plan.n_own
        w = None
        if edge_weight is not None:
            w = edge_weight if local_weights else edge_weight[plan.edge_pos]
        self.cover = None
        if cover:
            hc = HaloCover(plan, w, group)
            self.cover = hc
            ei_int = torch.stack([hc.int_src, hc.int_dst])
            ei_bnd = torch.stack([hc.bnd_src, hc.bnd_dst])
            w_int, w_bnd = hc.int_w, hc.bnd_w
            self.recv_counts, self.send_counts = hc.recv_counts, hc.send_counts
            self.n_local_src = hc.n_local_src
            self.n_send = hc.n_send
            self.g_send = Graph(torch.stack([hc.send_src, hc.send_dst]), hc.n_send, plan.n_own, chunk=chunk)
            self.w_send = self.g_send.dst.to_csr_order(hc.send_w.contiguous())
        else:
            ei_int = lei[:, interior]
            ei_bnd = lei[:, ~interior]
            w_int = w[interior] if w is not None else None
            w_bnd = w[~interior] if w is not None else None
            self.recv_counts, self.send_counts = plan.recv_counts, plan.send_counts
            self.n_local_src = plan.n_local_src
            self.n_send = int(plan.send_idx.numel())
        self.g_int = Graph(ei_int, plan.n_own, plan.n_own, chunk=chunk)
        self.g_bnd = Graph(ei_bnd, plan.n_own, self.n_local_src, chunk=chunk)
        self.w_int = self.g_int.dst.to_csr_order(w_int.contiguous()) if w_int is not None else None
        self.w_bnd = self.g_bnd.dst.to_csr_order(w_bnd.contiguous()) if w_bnd is not None else None
        self.n_interior = int(ei_int.shape[1])
        self.n_boundary = int(ei_bnd.shape[1])
        self.n_halo = self.n_local_src - plan.n_own
        self._chunk = chunk
        self._ei_bnd = ei_bnd
        self._fused = None
        # step_tiled / step_fused: run the interior pass(es) on a second stream
        # beside the send packing (both read only the rank's own rows); the
        # boundary passes wait for them.  Off by default; bench.py's warm-up times
        # both and keeps the faster (the two streams may land on one hardware queue).
        self.split_interior = False
        # step_fused: the boundary pass as one launch over every tile after the
        # last tile's halo arrived (True), or one launch per tile as its halo
        # arrives (False: tile t's boundary pass overlaps tile t+1's exchange)
        self.one_boundary_launch = True
        # step_fused: the send rows packed by one launch over every tile (False),
        # or one launch per tile with that tile's all_to_all started right after
        # it (True: the exchange starts after 1/T of the packing instead of all
        # of it -- the link chain pack + exchange + boundary is shorter, the
        # compute a few launches longer)
        self.pack_per_tile = False

    def local_buffer(self, F, dtype=torch.float32, device=None):
        """[n_own + n_halo, F]: the owner writes rows [:n_own], the exchange the rest."""
        return torch.empty((self.n_local_src, F), dtype=dtype, device=device or self.plan.halo_nodes.device)

    def local_tiles(self, F, tile=128, dtype=torch.float32, device=None):
        """Tile-major buffers for step_tiled (see ShardPlan.local_tiles)."""
        dev = device or self.plan.halo_nodes.device
        return [torch.empty((self.n_local_src, w), dtype=dtype, device=dev) for w in tile_widths(F, tile)]

    def _send(self, own):
        """This rank's send buffer: the requested rows (pull), or with a cover
        one aggregation over the send graph (copies + partial rows)."""
        from . import ops
        F = own.shape[1]
        if self.n_send == 0:
            return own.new_empty((0, F))
        if self.cover is not None:
            return ops._aggregate(self.g_send.dst, "other", own, self.w_send, "sum", 0, None)[0]
        return ops.gather_rows(own, self.plan.send_idx)

    def step(self, x_local, out, bias=None, group=None):
        """(see the class docstring) -- on the device's compute stream
        (compute_stream: RCCL overlaps it, unlike the default stream)."""
        with compute_stream(out.device):
            return self._step(x_local, out, bias, group)

    def _step(self, x_local, out, bias=None, group=None):
        from . import _lib, ops
        plan = self.plan
        own = x_local[:plan.n_own]
        send = self._send(own)
        halo = x_local[plan.n_own:]
        work = None
        if x_local.is_cuda and dist.get_backend(group) == "gloo":
            _a2a(halo, send, self.recv_counts, self.send_counts, group)
        else:
            work = dist.all_to_all_single(halo, send, output_split_sizes=self.recv_counts,
                                          input_split_sizes=self.send_counts, group=group, async_op=True)
        # no boundary edge (one rank, or rows fed only by local sources): the
        # interior pass is the whole row and adds the bias itself
        last = self.n_boundary == 0
        ops._aggregate(self.g_int.dst, "other", own, self.w_int, "sum", 0, bias if last else None, out=out)
        if work is not None:
            work.wait()
        if not last:
            ops._aggregate(self.g_bnd.dst, "other", x_local, self.w_bnd, "sum", _lib.MP_FLAG_INIT_FROM_OUT, bias,
                           out=out)
        return out

    def step_tiled(self, x_tiles, out, bias=None, group=None, events=None):
        """step() pipelined over feature tiles (x_tiles from plan.local_tiles):
          1. pack every tile's requested rows and start its all_to_all (RCCL
             runs them back to back on its stream while the compute stream
             packs the next tile),
          2. aggregate the interior edges of every tile,
          3. per tile, wait for ITS halo only, then aggregate its boundary
             edges on top (MP_FLAG_INIT_FROM_OUT) plus that tile's bias.
        Tile t's boundary pass overlaps tile t+1's exchange.  Per row and
        feature the arithmetic is that of step(): bitwise the same output.
        events (optional dict of lists): HIP events recorded on the compute
        stream -- 'send' (start, end) of packing every tile's send buffer (the
        cover's send graph: copies + partial rows), 'interior' (start, end) of
        the interior passes, 'wait'
        (before, after) around each tile's wait (the exchange time the compute
        stream is exposed to), 'boundary' (start, end) of each boundary pass.
        The whole step runs on the device's compute stream (compute_stream),
        ordered after the caller's stream and waited for by it."""
        with compute_stream(out.device):
            return self._step_tiled(x_tiles, out, bias, group, events)

    def _step_tiled(self, x_tiles, out, bias=None, group=None, events=None):
        def rec(name):
            if events is None:
                return None
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            events.setdefault(name, []).append(e)
            return e
        from . import _lib, ops
        plan = self.plan
        gloo = out.is_cuda and dist.get_backend(group) == "gloo"
        offs = [0]
        for xt in x_tiles:
            offs.append(offs[-1] + xt.shape[1])
        if offs[-1] != out.shape[1]:
            raise ValueError("step_tiled: tiles cover %d features, out has %d" % (offs[-1], out.shape[1]))
        for xt in x_tiles:
            if xt.shape[0] != self.n_local_src:
                raise ValueError("step_tiled: tiles have %d rows, this exchange needs %d (use local_tiles())"
                                 % (xt.shape[0], self.n_local_src))
        last = self.n_boundary == 0   # the interior pass is the whole row (see step)
        split = self.split_interior and out.is_cuda
        if split:
            start = torch.cuda.current_stream(out.device).record_event()
        pending = []
        rec("send")
        for xt in x_tiles:
            own = xt[:plan.n_own]
            send = self._send(own)
            halo = xt[plan.n_own:]
            if gloo:
                _a2a(halo, send, self.recv_counts, self.send_counts, group)
                pending.append((None, send))
            else:
                work = dist.all_to_all_single(halo, send, output_split_sizes=self.recv_counts,
                                              input_split_sizes=self.send_counts, group=group, async_op=True)
                pending.append((work, send))
        rec("send")
        if split:
            # the interior passes on the side stream, ordered after what preceded
            # the sends only: they run beside the send packing (the sends were
            # queued first, so the exchange's inputs are not held back)
            side = _side_stream(out.device)
            side.wait_event(start)
            with torch.cuda.stream(side):
                rec("interior")
                self._passes(x_tiles, out, bias, boundary=False)
                rec("interior")
            torch.cuda.current_stream(out.device).wait_stream(side)
        else:
            rec("interior")
            self._passes(x_tiles, out, bias, boundary=False)
            rec("interior")
        for t, xt in enumerate(x_tiles):
            work, _send = pending[t]
            rec("wait")
            if work is not None:
                work.wait()
            rec("wait")
            rec("boundary")
            if not last:
                b = bias[offs[t]:offs[t + 1]] if bias is not None else None
                ops._aggregate(self.g_bnd.dst, "other", xt, self.w_bnd, "sum", _lib.MP_FLAG_INIT_FROM_OUT, b,
                               out=out[:, offs[t]:offs[t + 1]])
            rec("boundary")
        return out

    def _exchange_async(self, xt, send, group=None):
        """Start one tile's all_to_all into its halo rows; returns the work
        handle (None: gloo with device tensors, done synchronously)."""
        halo = xt[self.plan.n_own:]
        if xt.is_cuda and dist.get_backend(group) == "gloo":
            _a2a(halo, send, self.recv_counts, self.send_counts, group)
            return None
        return dist.all_to_all_single(halo, send, output_split_sizes=self.recv_counts,
                                      input_split_sizes=self.send_counts, group=group, async_op=True)

    def _passes(self, x_tiles, out, bias, interior=True, boundary=True):
        """The interior and / or boundary aggregations of every tile (as step_tiled)."""
        from . import _lib, ops
        n_own = self.plan.n_own
        last = self.n_boundary == 0
        offs = [0]
        for xt in x_tiles:
            offs.append(offs[-1] + xt.shape[1])
        if interior:
            for t, xt in enumerate(x_tiles):
                b = bias[offs[t]:offs[t + 1]] if (last and bias is not None) else None
                ops._aggregate(self.g_int.dst, "other", xt[:n_own], self.w_int, "sum", 0, b,
                               out=out[:, offs[t]:offs[t + 1]])
        if boundary and not last:
            for t, xt in enumerate(x_tiles):
                b = bias[offs[t]:offs[t + 1]] if bias is not None else None
                ops._aggregate(self.g_bnd.dst, "other", xt, self.w_bnd, "sum", _lib.MP_FLAG_INIT_FROM_OUT, b,
                               out=out[:, offs[t]:offs[t + 1]])

    # ------------------------------------------------------------------
    # the fused step: own rows from the caller's row-major tensor, tile-major
    # buffers holding only the exchanged rows, one launch per pass
    # ------------------------------------------------------------------
    def halo_buffers(self, F, width=128, device=None):
        """HaloBuffers for step_fused: the send rows and the received halo rows,
        tile-major ([T, rows, width], T = F / width), so each tile's rows are
        contiguous and go over the links on their own, while each pass reads or
        writes every tile in one launch.  width: 64, 128 or 256 (one tile:
        whole rows), dividing F."""
        dev = device or self.plan.halo_nodes.device
        return HaloBuffers(self.n_send, self.n_halo, F, width, dev)

    def _fused_graphs(self):
        """(boundary graph over the halo rows alone -- columns = halo slot, the
        same edges in the same order as g_bnd --, the send graph of the pull
        exchange: one unweighted edge per requested row, the per-row flags
        of the own rows with no boundary edge, int32), built once."""
        if self._fused is None:
            from .graph import Graph
            n_own = self.plan.n_own
            ei = self._ei_bnd
            g_bh = Graph(torch.stack([ei[0] - n_own, ei[1]]), n_own, max(self.n_halo, 1), chunk=self._chunk)
            g_sp = None
            if self.cover is None and self.n_send:
                si = self.plan.send_idx
                g_sp = Graph(torch.stack([si, torch.arange(si.numel(), dtype=si.dtype, device=si.device)]),
                             self.n_send, n_own, chunk=self._chunk)
            rp = g_bh.dst.rowptr
            no_bnd = (rp[1:] == rp[:-1]).to(torch.int32)     # per own row: 1 = no boundary edge
            self._fused = (g_bh, g_sp, no_bnd)
        return self._fused

    def _pack_fused(self, x_own, bufs):
        """Every tile's send rows in ONE launch: the cover's send graph (copies +
        partial rows) or the pull requests, written tile-major into bufs.send."""
        from . import ops
        if self.n_send == 0:
            return
        g_bh, g_sp, _ = self._fused_graphs()
        if self.cover is not None:
            g, w = self.g_send.dst, self.w_send
        else:
            g, w = g_sp.dst, None
        if bufs.n_tiles == 1:        # whole rows: the send buffer is row-major
            ops.aggregate_tiles(g, "other", x_own, w, bufs.F, bufs.send[0], "sum", 0, None)
        else:
            ops.aggregate_tiles(g, "other", x_own, w, bufs.F, bufs.send, "sum", 0, None,
                                out_tiles=(bufs.width, bufs.n_send * bufs.width))

    def _pack_tile(self, x_own, bufs, t):
        """Tile t's send rows alone (pack_per_tile): features [t*width, (t+1)*width)
        of x_own's rows into bufs.send[t], the same per-row arithmetic."""
        from . import ops
        if self.n_send == 0:
            return
        g_bh, g_sp, _ = self._fused_graphs()
        g, w = (self.g_send.dst, self.w_send) if self.cover is not None else (g_sp.dst, None)
        c0 = t * bufs.width
        ops.aggregate_tiles(g, "other", x_own[:, c0:c0 + bufs.width], w, bufs.width, bufs.send[t], "sum", 0, None)

    def _pack_and_exchange(self, x_own, bufs, group=None):
        """The send packing and every tile's all_to_all: one packing launch then
        the tiles' exchanges, or (pack_per_tile) tile by tile."""
        if self.pack_per_tile and bufs.n_tiles > 1:
            works = []
            for t in range(bufs.n_tiles):
                self._pack_tile(x_own, bufs, t)
                works += self._start_exchange(bufs, group, tiles=[t])
            return works
        self._pack_fused(x_own, bufs)
        return self._start_exchange(bufs, group)

    def _interior_fused(self, x_own, out, bias):
        """The interior edges of every feature in one launch, with the bias of
        the rows the boundary pass leaves untouched (no boundary edge: a per-row
        flag; every row when no boundary edge follows at all)."""
        from . import ops
        if self.n_boundary == 0:
            ops._aggregate(self.g_int.dst, "other", x_own, self.w_int, "sum", 0, bias, out=out)
            return
        F = x_own.shape[1]
        ops.aggregate_tiles(self.g_int.dst, "other", x_own, self.w_int, F, out, "sum", 0, bias,
                            bias_rows=self._fused_graphs()[2] if bias is not None else None)

    def _boundary_fused(self, bufs, out, bias, tile=None):
        """The boundary edges over the received halo rows on top of out
        (MP_FLAG_INIT_FROM_OUT) + bias, rows without boundary edges untouched
        (MP_FLAG_SKIP_EMPTY: their bias came with the interior pass): every tile
        in one launch (tile None), or tile `tile` alone.  Each row's out values
        are loaded with the gathers of its first slot's batch (the kernel's
        out prefetch), not when the row opens."""
        from . import _lib, ops
        if self.n_boundary == 0:
            return
        g_bh, _, _ = self._fused_graphs()
        flags = _lib.MP_FLAG_INIT_FROM_OUT | _lib.MP_FLAG_SKIP_EMPTY
        if tile is None:
            if bufs.n_tiles == 1:    # whole rows: the halo buffer is row-major
                ops.aggregate_tiles(g_bh.dst, "other", bufs.recv[0], self.w_bnd, bufs.F, out, "sum", flags, bias)
            else:
                ops.aggregate_tiles(g_bh.dst, "other", bufs.recv, self.w_bnd, bufs.F, out, "sum", flags, bias,
                                    x_tiles=(bufs.width, bufs.n_halo * bufs.width))
            return
        c0, c1 = tile * bufs.width, (tile + 1) * bufs.width
        b = bias[c0:c1] if bias is not None else None
        ops.aggregate_tiles(g_bh.dst, "other", bufs.recv[tile], self.w_bnd, bufs.width, out[:, c0:c1], "sum", flags, b)

    def _start_exchange(self, bufs, group=None, tiles=None):
        """Every tile's all_to_all (or those of `tiles`), started in tile order
        (RCCL runs them back to back on its stream); returns one work handle per
        tile (None: gloo with device tensors, done synchronously)."""
        gloo = bufs.recv.is_cuda and dist.get_backend(group) == "gloo"
        works = []
        for t in (range(bufs.n_tiles) if tiles is None else tiles):
            if gloo:
                _a2a(bufs.recv[t], bufs.send[t], self.recv_counts, self.send_counts, group)
                works.append(None)
            else:
                works.append(dist.all_to_all_single(bufs.recv[t], bufs.send[t], output_split_sizes=self.recv_counts,
                                                    input_split_sizes=self.send_counts, group=group, async_op=True))
        return works

    def step_fused(self, x_own, bufs, out, bias=None, group=None, events=None):
        """The step with one launch per pass:
          1. pack every tile's send rows in one launch (tile-major bufs.send),
             then start each tile's all_to_all into bufs.recv (pack_per_tile:
             one launch per tile, its all_to_all started right after it),
          2. the interior edges in one launch over x_own (the caller's
             row-major [n_own, F] rows: no copy into a tile buffer), beside the
             packing on a second stream when split_interior,
          3. the boundary edges over the received halo rows on top (INIT_FROM_OUT)
             + bias: one launch after the last tile arrived
             (one_boundary_launch), or per tile as each tile arrives.
        Per row and feature the arithmetic is step()'s: bitwise the same output.
        events: as step_tiled ('send', 'interior', 'wait', 'boundary')."""
        if x_own.shape != (self.n_own, bufs.F) or x_own.stride(1) != 1:
            raise ValueError("step_fused: x_own must be this rank's [%d, %d] rows (row-major)" % (self.n_own, bufs.F))
        with compute_stream(out.device):
            return self._step_fused(x_own, bufs, out, bias, group, events)

    def _step_fused(self, x_own, bufs, out, bias=None, group=None, events=None):
        def rec(name):
            if events is None:
                return None
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            events.setdefault(name, []).append(e)
            return e
        split = self.split_interior and out.is_cuda
        if split:
            start = torch.cuda.current_stream(out.device).record_event()
        rec("send")
        works = self._pack_and_exchange(x_own, bufs, group)
        rec("send")
        if split:
            side = _side_stream(out.device)
            side.wait_event(start)
            with torch.cuda.stream(side):
                rec("interior")
                self._interior_fused(x_own, out, bias)
                rec("interior")
            torch.cuda.current_stream(out.device).wait_stream(side)
        else:
            rec("interior")
            self._interior_fused(x_own, out, bias)
            rec("interior")
        if self.one_boundary_launch:
            rec("wait")
            for w in works:
                if w is not None:
                    w.wait()
            rec("wait")
            rec("boundary")
            self._boundary_fused(bufs, out, bias)
            rec("boundary")
        else:
            for t, w in enumerate(works):
                rec("wait")
                if w is not None:
                    w.wait()
                rec("wait")
                rec("boundary")
                self._boundary_fused(bufs, out, bias, tile=t)
                rec("boundary")
        return out

    # ------------------------------------------------------------------
    # the step's pieces, for either form (step_tiled's list of [own ; halo]
    # tiles, or step_fused's (x_own, HaloBuffers)): timing and decomposition
    # ------------------------------------------------------------------
    def _pieces(self, form, out, bias):
        """(pack, interior, boundary, exchange(group) -> works) of one form."""
        n_own = self.plan.n_own
        if isinstance(form, tuple):
            x_own, bufs = form

            def boundary():
                if self.one_boundary_launch:
                    self._boundary_fused(bufs, out, bias)
                else:
                    for t in range(bufs.n_tiles):
                        self._boundary_fused(bufs, out, bias, tile=t)
            def pack():
                if self.pack_per_tile and bufs.n_tiles > 1:
                    for t in range(bufs.n_tiles):
                        self._pack_tile(x_own, bufs, t)
                else:
                    self._pack_fused(x_own, bufs)
            return (pack, lambda: self._interior_fused(x_own, out, bias), boundary,
                    lambda group: self._start_exchange(bufs, group))
        x_tiles = form
        sends = {}

        def pack():
            sends["s"] = [self._send(xt[:n_own]) for xt in x_tiles]

        def exchange(group):
            if "s" not in sends:
                pack()
            return [self._exchange_async(xt, s, group) for xt, s in zip(x_tiles, sends["s"])]
        return (pack, lambda: self._passes(x_tiles, out, bias, boundary=False),
                lambda: self._passes(x_tiles, out, bias, interior=False), exchange)

    def _compute(self, form, out, bias, split=None):
        """The step's device work without the exchange: send packing, interior
        and boundary passes (the interior beside the packing on the side stream
        when split, default self.split_interior), on the current stream."""
        split = self.split_interior if split is None else split
        pack, interior, boundary, _ = self._pieces(form, out, bias)
        if not (split and out.is_cuda):
            pack()
            interior()
            boundary()
            return
        cur = torch.cuda.current_stream(out.device)
        start = cur.record_event()
        pack()
        side = _side_stream(out.device)
        side.wait_event(start)
        with torch.cuda.stream(side):
            interior()
        cur.wait_stream(side)
        boundary()

    def _step_form(self, form, out, bias, group=None):
        if isinstance(form, tuple):
            return self.step_fused(form[0], form[1], out, bias, group)
        return self.step_tiled(form, out, bias, group)

    def compute_in_turn(self, form, out, bias=None, reps=5, group=None, barrier=None):
        """decompose()'s compute alone, one rank at a time: rank r times its
        send pack, interior and boundary passes with HIP events on the compute
        stream while every other rank waits at `barrier`.  Ranks that share
        one GPU (the gloo rehearsal) get the compute time each rank would have
        on a GPU of its own; on a node it equals compute_only_ms.  Also the
        same work with the interior pass(es) beside the send packing
        (compute_alone_split_ms, split_interior).  form: step_tiled's tile
        list, or (x_own, HaloBuffers) of step_fused.  Collective over `group`
        (every rank calls it)."""
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        pack, interior, boundary, _ = self._pieces(form, out, bias)
        res = None
        for r in range(world):
            if barrier is not None:
                barrier()
            if r != rank:
                continue
            with compute_stream(out.device):
                self._compute(form, out, bias, split=False)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                parts = [[], [], []]
                for _ in range(reps):
                    ev[0].record()
                    pack()
                    ev[1].record()
                    interior()
                    ev[2].record()
                    boundary()
                    ev[3].record()
                    ev[3].synchronize()
                    for j in range(3):
                        parts[j].append(ev[j].elapsed_time(ev[j + 1]))
                # the same work with the interior pass(es) on the side stream beside
                # the send packing (split_interior), timed on the compute stream
                split = []
                for _ in range(reps):
                    ev[0].record()
                    self._compute(form, out, bias, split=True)
                    ev[3].record()
                    ev[3].synchronize()
                    split.append(ev[0].elapsed_time(ev[3]))
            # medians over the repetitions: ranks time-sharing one GPU see rare
            # multi-ms stalls while the others sit idle at the barrier
            med = [sorted(v)[len(v) // 2] for v in parts]
            res = {"reps": reps, "send_pack_ms": med[0], "interior_ms": med[1], "boundary_ms": med[2],
                   "compute_alone_ms": sum(med), "compute_alone_split_ms": sorted(split)[len(split) // 2],
                   "statistic": "median over reps (per part)"}
        if barrier is not None:
            barrier()
        return res

    def decompose(self, form, out, bias=None, reps=5, group=None, barrier=None):
        """The overlapped step taken apart on this rank, each piece timed alone
        (wall clock over `reps` repetitions, the device synchronised after
        them, the ranks lined up by `barrier` before each piece):
          exchange_only_ms   every tile's all_to_all and its wait, the send
                             buffers packed beforehand: the links alone
                             (at one rank the splits are empty: ~0);
          compute_only_ms    packing + interior + boundary passes and no
                             exchange (the halo rows keep their last values;
                             the interior beside the packing when
                             split_interior, as the step runs them);
          serial_step_ms     pack, exchange and wait, then the interior and
                             boundary passes: the step without overlap;
          overlapped_step_ms the step itself, timed the same way.
        hidden_frac = (exchange + compute - overlapped) / min(exchange, compute)
        is the share of the shorter piece the overlap hides (1 = all of it;
        below 0, the overlapped step is slower than the two pieces in a row,
        e.g. RCCL's kernels contending with the aggregation for CUs / L2).  It
        is reported only where the pieces are comparable (hidden_frac_valid):
        when the exchange alone takes longer than the whole serial step (the
        gloo rehearsal, whose host staging makes exchange timings swing from
        one measurement to the next) or the ratio leaves [-1, 1], it is None
        with the reason in hidden_frac_note.  form: as compute_in_turn."""
        import time
        pack, interior, boundary, exchange_start = self._pieces(form, out, bias)

        def timed(fn):
            if barrier is not None:
                barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with compute_stream(out.device):      # where the step runs its work
                for _ in range(reps):
                    fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps * 1e3

        with compute_stream(out.device):
            pack()

        def exchange_only():
            for w in exchange_start(group):
                if w is not None:
                    w.wait()

        def compute_only():
            self._compute(form, out, bias)

        def serial():
            pack()
            for w in exchange_start(group):
                if w is not None:
                    w.wait()
            interior()
            boundary()

        res = {"reps": reps,
               "exchange_only_ms": timed(exchange_only),
               "compute_only_ms": timed(compute_only),
               "serial_step_ms": timed(serial),
               "overlapped_step_ms": timed(lambda: self._step_form(form, out, bias, group))}
        res.update(hidden_fraction(res, staged=out.is_cuda and dist.get_backend(group) == "gloo"))
        return res


def hidden_fraction(res, staged=False):
    """hidden_frac of a decomposition {exchange_only_ms, compute_only_ms,
    serial_step_ms, overlapped_step_ms} (OverlappedAggregation.decompose), or
    None with the reason when the pieces are not comparable: device tensors
    exchanged over gloo (staged: the host copies make the exchange a blocking
    call that cannot overlap, and its time swings between measurements), the
    exchange alone longer than the serial step that contains it, a shorter
    piece of ~0 ms (one rank), or a ratio outside [-1, 1]."""
    if staged:
        return {"hidden_frac": None, "hidden_frac_valid": False,
                "hidden_frac_note": "host-staged gloo exchange (a rehearsal): blocking, not the node's links"}
    ex, co = res["exchange_only_ms"], res["compute_only_ms"]
    shorter = min(ex, co)
    if shorter <= 1e-3:
        return {"hidden_frac": None, "hidden_frac_valid": False,
                "hidden_frac_note": "the shorter piece takes ~0 ms (empty splits): nothing to hide"}
    if "serial_step_ms" in res and ex > res["serial_step_ms"]:
        return {"hidden_frac": None, "hidden_frac_valid": False,
                "hidden_frac_note": "exchange alone (%.3f ms) exceeds the serial step (%.3f ms): the exchange "
                                    "timings are not comparable (host-staged gloo)" % (ex, res["serial_step_ms"])}
    h = (ex + co - res.get("overlapped_step_ms", res.get("step_ms"))) / shorter
    if not -1.0 <= h <= 1.0:
        return {"hidden_frac": None, "hidden_frac_valid": False,
                "hidden_frac_note": "ratio %.3f outside [-1, 1]: the pieces are not comparable" % h}
    return {"hidden_frac": h, "hidden_frac_valid": True, "hidden_frac_note": None}


class HaloBuffers:
    """The fused step's exchange buffers (OverlappedAggregation.halo_buffers):
    send [T, n_send, width] and recv [T, n_halo, width], T = F / width,
    tile-major -- tile t's rows contiguous (one all_to_all per tile), every
    tile addressed by the kernel in one launch (mp_aggregate_tiles_f32).  The
    rank's own rows stay in the caller's row-major tensor."""

    def __init__(self, n_send, n_halo, F, width, device):
        width = int(width)
        if width not in (64, 128, 256) or F % width:
            raise ValueError("HaloBuffers: width %d must be 64, 128 or 256 and divide F = %d" % (width, F))
        self.F, self.width, self.n_tiles = int(F), width, int(F) // width
        self.n_send, self.n_halo = int(n_send), int(n_halo)
        self.send = torch.empty((self.n_tiles, self.n_send, width), dtype=torch.float32, device=device)
        self.recv = torch.empty((self.n_tiles, self.n_halo, width), dtype=torch.float32, device=device)

    def halo_rows(self):
        """The received halo rows as one row-major [n_halo, F] tensor (a copy)."""
        return self.recv.permute(1, 0, 2).reshape(self.n_halo, self.F)


def transposed_plan(edge_index, num_nodes, rank, world, cuts, group=None):
    """The plan of the backward pass: rank p owns the SOURCE rows [lo_p, hi_p)
    of the same cuts, its edges are the out-edges of those rows (global order)
    and its halo the remote destinations whose gradient rows it gathers."""
    return ShardPlan(edge_index, num_nodes, rank, world, cuts=cuts, flow="target_to_source").exchange_requests(group)


class ShardedGraph:
    """One graph sharded by destination-node range over the ranks of `group`
    (SURVEY 8e), with everything a layer needs for forward AND backward:

      fwd : ShardPlan of the in-edges of this rank's rows (halo = remote sources)
      bwd : ShardPlan of the out-edges of this rank's rows (halo = remote
            destinations), same cuts: the backward of the aggregation is a
            forward over the transposed graph, so d x_j is summed by j's owner
            in global edge order -- no partial sums cross ranks.
      g_fwd / g_bwd : native CSR graphs of the rank's local edge lists.

    Built once per (edge_index, weights) like GCNConv(cached=True).  Every rank
    passes the full edge_index (one-time plan construction)."""

    def __init__(self, edge_index, num_nodes, rank, world, group=None, cuts=None, chunk=None):
        from .graph import Graph
        self.group = group
        self.num_nodes = int(num_nodes)
        self.n_edges = int(edge_index.shape[1])
        if cuts is None:
            cuts = edge_balanced_cuts(_count_by(edge_index[1].to(torch.int64), num_nodes), world)
        self.fwd, self.bwd = ShardPlan.many([edge_index, edge_index], num_nodes, rank, world, cuts,
                                            ["source_to_target", "target_to_source"], [None, None], group)
        self.lo, self.hi, self.n_own = self.fwd.lo, self.fwd.hi, self.fwd.n_own
        self.g_fwd = Graph(self.fwd.local_edge_index, self.n_own, self.fwd.n_local_src, chunk=chunk)
        # bwd.local_edge_index = [local row (= source j), local column (= destination i)]
        self.g_bwd = Graph(self.bwd.local_edge_index, self.n_own, self.bwd.n_local_src,
                           flow="target_to_source", chunk=chunk)
        self._w = None
        self.cover = None
        self._chunk = chunk

    @classmethod
    def for_gcn(cls, edge_index, num_nodes, rank, world, group=None, improved=False, edge_weight=None, chunk=None,
                cuts=None):
        """GCNConv's graph (add_remaining_self_loops + symmetric norm, [U5]),
        built from the full edge list, sharded, with the norm as edge weight
        (cuts: explicit row ranges, else edge-balanced)."""
        from torch_geometric.nn.conv.gcn_conv import GCNConv
        ei2, norm = GCNConv.norm(edge_index, num_nodes, edge_weight, improved)
        return cls(ei2, num_nodes, rank, world, group=group, chunk=chunk, cuts=cuts).set_edge_weight(norm)

    @classmethod
    def for_gcn_from_slices(cls, edge_slice, slice_offset, num_nodes, rank, world, group=None, improved=False,
                            edge_weight=None, chunk=None):
        """for_gcn() for a graph held as per-rank slices of its edge list (rank r:
        the global edges [slice_offset, slice_offset + n_r), slices contiguous in
        rank order; edge_weight aligned with the slice): the loops, degrees and
        both plans are built from the slices with all_to_alls (gcn_shards_from_slices);
        the local edge lists, global edge ids and norms are those of for_gcn()
        bit for bit."""
        from .graph import Graph
        d = gcn_shards_from_slices(edge_slice, slice_offset, num_nodes, rank, world, group, edge_weight, improved)
        self = cls.__new__(cls)
        self.group = group
        self.num_nodes = int(num_nodes)
        self.n_edges = int(d["E"])
        f_ei, f_gid, f_w = d["fwd"]
        b_ei, b_gid, b_w = d["bwd"]
        self.fwd, self.bwd = ShardPlan.many([f_ei, b_ei], num_nodes, rank, world, d["cuts"],
                                            ["source_to_target", "target_to_source"], [f_gid, b_gid], group)
        self.lo, self.hi, self.n_own = self.fwd.lo, self.fwd.hi, self.fwd.n_own
        self.g_fwd = Graph(self.fwd.local_edge_index, self.n_own, self.fwd.n_local_src, chunk=chunk)
        self.g_bwd = Graph(self.bwd.local_edge_index, self.n_own, self.bwd.n_local_src,
                           flow="target_to_source", chunk=chunk)
        self.deg = d["deg"]
        self.cover = None
        self._chunk = chunk
        self.norm_fwd, self.norm_bwd = _norms_over_plans([self.fwd, self.bwd], d["deg"],
                                                         [f_w[self.fwd.edge_pos], b_w[self.bwd.edge_pos]], group)
        self._w = None
        if self.norm_fwd.is_cuda:
            self._set_local_weights(self.norm_fwd, self.norm_bwd)
        return self

    @classmethod
    def for_gat(cls, edge_index, num_nodes, rank, world, group=None, cuts=None):
        """GATConv's graph (remove_self_loops + add_self_loops, PyG 1.4.3 [U6])
        from the full edge list, sharded: the forward plan only -- the GAT
        backward runs over the rank's local transposed CSR, and the gradients of
        its halo rows go back to their owners (halo_rows)."""
        from torch_geometric.nn.conv._structure import gat_loops
        ei = gat_loops(edge_index, num_nodes) if edge_index.is_cuda else _host("gat_loops")(edge_index, num_nodes)
        plan = ShardPlan(ei, num_nodes, rank, world, cuts=cuts).exchange_requests(group)
        return cls._for_gat_plan(plan, ei.shape[1], group)

    @classmethod
    def for_gat_from_slices(cls, edge_slice, slice_offset, num_nodes, rank, world, group=None):
        """for_gat() for a graph held as per-rank slices of its edge list (as
        for_gcn_from_slices; the loops are the same edge list GCN's
        add_remaining_self_loops gives, so gcn_shards_from_slices builds it,
        structure only).  Local edge lists and global edge ids equal for_gat()'s."""
        d = gcn_shards_from_slices(edge_slice, slice_offset, num_nodes, rank, world, group, structure_only=True)
        f_ei, f_gid, _ = d["fwd"]
        plan = ShardPlan(f_ei, num_nodes, rank, world, cuts=d["cuts"], edge_ids=f_gid).exchange_requests(group)
        return cls._for_gat_plan(plan, d["E"], group)

    @classmethod
    def _for_gat_plan(cls, plan, n_edges, group):
        from .graph import GAT_TARGET_TASKS, Graph
        self = cls.__new__(cls)
        self.group = group
        self.num_nodes = int(plan.cuts[-1])
        self.n_edges = int(n_edges)
        self.fwd, self.bwd = plan, None
        self.lo, self.hi, self.n_own = plan.lo, plan.hi, plan.n_own
        # destination rows = own rows, sources = [own rows ; halo rows]: the fused
        # GAT kernels' sharded form (ops._gat_rows_ok); built lazily on first use
        self.g_fwd = Graph(plan.local_edge_index, self.n_own, plan.n_local_src, target_tasks=GAT_TARGET_TASKS)
        # attention dropout keyed on the GLOBAL edge id: the single-GPU layer's mask
        self.g_fwd.edge_key = plan.edge_gid
        self.g_bwd = None
        self.deg = None
        self._w = None
        self.cover = None
        self.gat_cover = None
        self._chunk = None
        return self

    def gat_propagate(self, xw_own, att, heads, out_channels, negative_slope=0.2, bias=None,
                      return_alpha=False, dropout=0.0, local_gat=None, seed=None):
        """Sharded fused GATConv aggregation (GATConv.message + utils.softmax +
        scatter_add + update, [U3, U6]): this rank's rows [n_own, H*C] (+ bias).

        xw_own: the rank's rows of X W.  Their halo rows arrive over the pull
        plan (halo_rows: differentiable, the backward returns the halo rows'
        gradients to their owners).  A destination row's score a_dst comes from
        its own xw row, a_src is recomputed from each gathered row, and every
        in-edge of a destination row lives on its owner -- the softmax and the
        weighted sum of a row run over the same edges in the same (global)
        order as on one GPU: no extra collective, alpha bit-equal on rows no
        merge-path task splits.  return_alpha: (global edge ids, alpha [m, H])
        of this rank's in-edges (pull or cover).  dropout: the fused attention
        dropout, its keep mask keyed on the GLOBAL edge ids -- the single-GPU
        layer's mask (over the cover too).
        local_gat(graph, edge_index, xw_local, att, H, C, slope, bias,
        return_alpha, dropout) -> (out, alpha): default the HIP path
        (ops.gat_propagate); the gloo CPU tests pass the oracle.  seed: the
        dropout key (default: drawn from the device's generator)."""
        from .gat_cover import cover_ok
        gc = getattr(self, "gat_cover", None)
        if gc is not None and local_gat is None:
            if not xw_own.is_cuda:
                if not dropout and not return_alpha:
                    return _host("gat_cover_forward")(gc, xw_own, att, heads, out_channels, negative_slope, bias), None
            elif cover_ok(heads, out_channels):
                from .gat_cover import gat_cover_propagate
                res = gat_cover_propagate(gc, xw_own, att, heads, out_channels, negative_slope, bias, dropout, seed,
                                          return_alpha)
                if return_alpha:
                    return res[0], (self.fwd.edge_gid, res[1])
                return res, None
        if local_gat is None:
            from . import ops
            local_gat = ops.gat_propagate
            if seed is not None:
                def local_gat(*a, _seed=seed):
                    return ops.gat_propagate(*a, seed=_seed)
        xw_local = halo_rows(xw_own, self.fwd, self.group)
        out, alpha = local_gat(self.g_fwd, self.fwd.local_edge_index, xw_local, att, heads, out_channels,
                               negative_slope, bias, return_alpha, dropout)
        return out, ((self.fwd.edge_gid, alpha) if return_alpha else None)

    def enable_gat_halo_cover(self):
        """Run gat_propagate (forward AND backward) over the hybrid halo cover
        (mi355_mp.gat_cover.GatHaloCover: a remote source row is pulled, or its
        owner pushes its online-softmax piece of the destination row -- 0.57x
        the pull rows on the config-2 graph) instead of the pull exchange.
        Attention dropout (keys: global edge ids) and return_alpha run over the
        cover too; heads of any width (C % 4 == 0, GATConv pads to it) take the
        cover.  Collective, once (every rank of the group)."""
        from .gat_cover import GatHaloCover
        if self.bwd is not None:
            raise ValueError("mi355_mp.dist: enable_gat_halo_cover needs a graph made by for_gat / "
                             "for_gat_from_slices")
        self.gat_cover = GatHaloCover(self.fwd, self.group)
        return self

    def _set_local_weights(self, w_fwd, w_bwd):
        """Per-edge weights already in each plan's local edge order."""
        self._w = (self.g_fwd.dst.to_csr_order(w_fwd.contiguous()), self.g_bwd.dst.to_csr_order(w_bwd.contiguous()),
                   w_fwd.contiguous())
        return self

    def set_edge_weight(self, edge_weight):
        """Per-edge weights in GLOBAL edge order (e.g. the GCN norm), permuted
        once into both local CSR orders."""
        if edge_weight is None:
            self._w = None
            return self
        if edge_weight.requires_grad:
            raise ValueError("mi355_mp.dist: set_edge_weight fixes the weights (e.g. a norm); pass learnable "
                             "weights to propagate(x_own, reduce, edge_weight=w) instead")
        w = edge_weight.to(torch.float32)
        return self._set_local_weights(w[self.fwd.edge_pos], w[self.bwd.edge_pos])

    def enable_halo_cover(self):
        """Run sum / mean propagate (forward AND backward) over the hybrid halo
        cover (HaloCover, 0.57x the pull rows on the config-2 graph) instead of
        the pull exchange.  Forward: send graph -> all_to_all -> one aggregation
        over the rank's interior + boundary edges.  Backward (its transpose): the
        transposed local graph gives the gradient of every local row, the halo
        rows' gradients go back over the reverse all_to_all, and the transposed
        send graph folds them into the owned rows.  Both directions move the
        cover's rows; deterministic; within 1e-5 of the pull form (regrouped
        sums).  max / min keep the pull exchange (arg ids).  Collective, once;
        call after the edge weights are set."""
        from .graph import Graph
        w = self._w[2] if self._w is not None else None        # the plan's local edge order
        hc = HaloCover(self.fwd, w, self.group)
        self.cover = hc
        ch = self._chunk
        self.g_cov = Graph(torch.stack([torch.cat([hc.int_src, hc.bnd_src]), torch.cat([hc.int_dst, hc.bnd_dst])]),
                           self.n_own, hc.n_local_src, chunk=ch)
        w_cov = torch.cat([hc.int_w, hc.bnd_w]).contiguous()
        self.w_cov = (self.g_cov.dst.to_csr_order(w_cov), self.g_cov.src.to_csr_order(w_cov))
        self.g_send = Graph(torch.stack([hc.send_src, hc.send_dst]), hc.n_send, self.n_own, chunk=ch)
        ws = hc.send_w.contiguous()
        self.w_send = (self.g_send.dst.to_csr_order(ws), self.g_send.src.to_csr_order(ws))
        return self

    def propagate(self, x_own, reduce="sum", edge_weight=None):
        """Sharded MessagePassing.propagate for message = w * x_j: this rank's
        rows of REDUCE_{e: dst(e) = i} w_e x[src(e)] (autograd included).
        max/min return (out, arg) with arg = GLOBAL edge ids.

        edge_weight: per-edge weights in GLOBAL edge order that the call
        differentiates (a learnable edge weight held by every rank, like a
        replicated parameter): they replace the weights set_edge_weight fixed,
        run over the pull exchange (the cover regroups each edge's term into a
        peer's partial row), and this rank's backward writes d w_e = <g_i, x_j>
        for its own in-edges only -- all-reduce the gradient over the ranks
        (allreduce_gradients does, for a module parameter) to get the full
        one, as for a layer weight."""
        from . import ops
        reduce = "sum" if reduce == "add" else reduce
        if reduce not in ("sum", "mean", "max", "min"):
            raise ValueError("unknown reduce %r" % (reduce,))
        x_own = ops._f32_2d(x_own, "x")
        if x_own.shape[0] != self.n_own:
            raise ValueError("mi355_mp.dist: x_own has %d rows, this rank owns %d" % (x_own.shape[0], self.n_own))
        w_fwd = w_bwd = None
        if edge_weight is not None:
            if edge_weight.dim() != 1 or edge_weight.numel() != self.n_edges:
                raise ValueError("mi355_mp.dist: edge_weight must hold the %d global edges" % self.n_edges)
            if not (edge_weight.is_cuda and x_own.is_cuda):
                raise RuntimeError("mi355_mp.dist: learnable edge weights on host tensors -- there is no CPU "
                                   "fallback: the engine runs on ROCm device tensors")
            w = edge_weight.to(torch.float32)
            w_fwd = w[self.fwd.edge_pos]                        # differentiable: d w lands on these edges
            w_bwd = w.detach()[self.bwd.edge_pos] if self.bwd is not None else None
        out, arg = _ShardedAggregate.apply(x_own, w_fwd, w_bwd, self, reduce)
        return (out, arg) if reduce in ("max", "min") else out


class _ShardedAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_own, w_fwd, w_bwd, sg, reduce):
        """w_fwd / w_bwd: learnable weights in the two plans' local edge orders
        (None: the weights set_edge_weight fixed); with them the pull form."""
        from . import ops
        from .graph import in_csr_order
        ctx.sg, ctx.reduce = sg, reduce
        ctx.learn = w_fwd is not None
        if sg.cover is not None and reduce in ("sum", "mean") and not ctx.learn:
            hc = sg.cover
            F = x_own.shape[1]
            x_local = x_own.new_empty((hc.n_local_src, F))
            x_local[:hc.n_own].copy_(x_own)
            send = (ops._aggregate(sg.g_send.dst, "other", x_own, sg.w_send[0], "sum", 0, None)[0]
                    if hc.n_send else x_own.new_empty((0, F)))
            _a2a(x_local[hc.n_own:], send, hc.recv_counts, hc.send_counts, sg.group)
            out, _ = ops._aggregate(sg.g_cov.dst, "other", x_local, sg.w_cov[0], "sum", 0, None)
            if reduce == "mean":   # the true in-degree (a partial row stands for several edges)
                out = out / sg.g_fwd.dst.degree().clamp(min=1).to(torch.float32).view(-1, 1)
            return out, None
        plan = sg.fwd
        F = x_own.shape[1]
        x_local = plan.local_buffer(F, device=x_own.device)
        x_local[:plan.n_own].copy_(x_own)
        plan.exchange_into(x_local, ops.gather_rows, sg.group)
        if ctx.learn:
            wl = w_fwd.detach().contiguous()
            w_csr = in_csr_order(sg.g_fwd.dst, wl)
            ctx.w_bwd_csr = in_csr_order(sg.g_bwd.dst, w_bwd.contiguous()) if w_bwd is not None else None
        else:
            wl = sg._w[2] if sg._w is not None else None
            w_csr = sg._w[0] if sg._w is not None else None
        out, arg = ops._aggregate(sg.g_fwd.dst, "other", x_local, w_csr, reduce, 0, None)
        arg_g = None
        ctx.save_for_backward(arg, wl, x_local if ctx.learn else None)
        if arg is not None:
            arg_g = plan.global_edge_ids(arg, sg.n_edges)
            ctx.mark_non_differentiable(arg_g)
        return out, arg_g

    @staticmethod
    def backward(ctx, grad_out, _grad_arg=None):
        from . import ops
        sg, reduce = ctx.sg, ctx.reduce
        g = grad_out.contiguous()
        F = g.shape[1]
        want_w = ctx.learn and ctx.needs_input_grad[1]
        if reduce in ("max", "min"):
            # gradient lands on the argmax edge's source, which may live in the halo:
            # accumulate per local column, then return the halo rows to their owners
            # (deterministic: the local transposed CSR adds each column's winning
            # terms in local = global edge order; the rows returned by several
            # peers are summed by a segmented sum keyed on send_idx, in peer order)
            arg, w, x_local = ctx.saved_tensors      # w: local edge order, the arg's positions
            plan = sg.fwd
            gl, gw = ops.arg_backward(sg.g_fwd, arg, g, plan.n_local_src, w, x_local, True, want_w)
            gx = gl[:plan.n_own]
            back = plan.return_halo(gl[plan.n_own:], sg.group)
            if back.shape[0]:
                gx = gx + _sum_returned_rows(plan, back)
            return gx.contiguous(), gw, None, None, None
        if reduce == "mean":
            g = g / sg.g_fwd.dst.degree().clamp(min=1).to(torch.float32).view(-1, 1)
        gw = None
        if want_w:       # d w_e = <g_i, x_j> over this rank's in-edges, local edge order
            _, _, x_local = ctx.saved_tensors
            gw = ops._edge_dot(sg.g_fwd.dst, g.contiguous(), x_local)
        if sg.cover is not None and not ctx.learn:
            # transpose of the cover forward: local rows' gradients over the transposed
            # local graph, the halo part back to its senders, the transposed send graph
            hc = sg.cover
            gl, _ = ops._aggregate(sg.g_cov.src, "other", g.contiguous(), sg.w_cov[1], "sum", 0, None)
            back = g.new_empty((hc.n_send, F))
            _a2a(back, gl[hc.n_own:].contiguous(), hc.send_counts, hc.recv_counts, sg.group)
            gx = gl[:hc.n_own]
            if hc.n_send:
                gx = gx + ops._aggregate(sg.g_send.src, "other", back, sg.w_send[1], "sum", 0, None)[0]
            return gx.contiguous(), None, None, None, None
        plan = sg.bwd
        g_local = plan.local_buffer(F, device=g.device)
        g_local[:plan.n_own].copy_(g)
        plan.exchange_into(g_local, ops.gather_rows, sg.group)
        if ctx.learn:
            w_bwd = ctx.w_bwd_csr
        else:
            w_bwd = sg._w[1] if sg._w is not None else None
        gx, _ = ops._aggregate(sg.g_bwd.dst, "other", g_local, w_bwd, "sum", 0, None)
        return gx, gw, None, None, None


def broadcast_parameters(module, src=0, group=None):
    """Give every rank rank `src`'s parameter values (replicated layer weights,
    as DDP does at construction)."""
    for p in module.parameters():
        with torch.no_grad():
            if p.is_cuda and dist.get_backend(group) == "gloo":
                t = p.detach().cpu()
                dist.broadcast(t, src, group=group)
                p.copy_(t)
            else:
                dist.broadcast(p.data, src, group=group)


def allreduce_gradients(module, group=None):
    """Sum the gradients of replicated parameters over the ranks (each rank's
    weight gradient covers its own rows only), as DDP would, in ONE bucketed
    all_reduce: [one has-grad flag per parameter ; every gradient flattened].
    A parameter some rank has no gradient for contributes zeros there (e.g. a
    rank that owns no rows, whose empty output does not involve GATConv's
    att), so every rank reduces the same bucket; a parameter NO rank has a
    gradient for keeps grad None on every rank (an optimizer with momentum or
    weight decay leaves it alone, as on one GPU) -- only a rank that lacks a
    gradient reads the summed flags back (the host waits for the reduction
    there and nowhere else; with every gradient present nothing syncs)."""
    params = [p for p in module.parameters() if p.requires_grad]
    if not params:
        return
    gloo = dist.get_backend(group) == "gloo"
    dev = params[0].device
    dtype = params[0].dtype
    if any(p.dtype != dtype or p.device != dev for p in params):
        raise ValueError("mi355_mp.dist.allreduce_gradients: replicated parameters of one dtype and device")
    have = [p.grad is not None for p in params]
    # flags built on the device (fills, no host-to-device copy)
    parts = [torch.full((1,), 1.0 if h else 0.0, dtype=dtype, device=dev) for h in have]
    parts += [(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params]
    flat = torch.cat(parts)
    if flat.is_cuda and gloo:
        t = _stage_to_host(flat)
        dist.all_reduce(t, group=group)
        flat.copy_(t)
    else:
        dist.all_reduce(flat, group=group)
    k = len(params)
    flags = flat[:k].tolist() if not all(have) else None
    o = k
    for i, p in enumerate(params):
        n = p.numel()
        if flags is not None and flags[i] == 0:
            o += n
            continue                           # no rank formed it: None everywhere
        g = flat[o:o + n].view_as(p)
        if p.grad is None:
            p.grad = g.clone()
        else:
            p.grad.copy_(g)
        o += n


class ShardedGCNConv(torch.nn.Module):
    """GCNConv [U5] over a ShardedGraph: this rank's rows of
    D^-1/2 (A+I) D^-1/2 (X W) + b.  x_own holds the rank's rows of X; the X W
    GEMM is local (hipBLASLt), the aggregation exchanges halo rows of X W
    (forward) and of the output gradient (backward).  Parameters are
    replicated: broadcast_parameters(module) once at setup, and after backward
    allreduce_gradients(module) sums the weight and bias gradients over the
    ranks.  Same parameter names and init as
    GCNConv, so a GCNConv state_dict loads unchanged."""

    def __init__(self, in_channels, out_channels, bias=True):
        super().__init__()
        from torch.nn import Parameter
        from torch_geometric.nn.inits import glorot, zeros
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight = Parameter(torch.Tensor(in_channels, out_channels))
        self.bias = Parameter(torch.Tensor(out_channels)) if bias else None
        glorot(self.weight)
        zeros(self.bias)

    def forward(self, x_own, sg):
        from . import ops
        out = sg.propagate(ops.feature_transform(x_own, self.weight), "sum")
        return out + self.bias if self.bias is not None else out

    def __repr__(self):
        return "{}({}, {})".format(self.__class__.__name__, self.in_channels, self.out_channels)


class ShardedGATConv(torch.nn.Module):
    """GATConv [U6] over a ShardedGraph made by ShardedGraph.for_gat /
    for_gat_from_slices: this rank's rows of the layer's output.  x_own holds
    the rank's rows of X; the X W GEMM is local (hipBLASLt), the halo rows of
    X W come over the plan's exchange (forward) and their gradients go back to
    their owners (backward); the fused GAT kernels run on the rank's local
    graph.  Same parameters, names, init and options as GATConv (a GATConv
    state_dict loads unchanged); replicated like ShardedGCNConv:
    broadcast_parameters once, allreduce_gradients after backward."""

    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2, dropout=0, bias=True):
        super().__init__()
        from torch.nn import Parameter
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope, self.dropout = concat, negative_slope, dropout
        self.weight = Parameter(torch.Tensor(in_channels, heads * out_channels))
        self.att = Parameter(torch.Tensor(1, heads, 2 * out_channels))
        if bias:
            self.bias = Parameter(torch.Tensor(heads * out_channels if concat else out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        from torch_geometric.nn.inits import glorot, zeros
        glorot(self.weight)
        glorot(self.att)
        zeros(self.bias)

    def forward(self, x_own, sg, return_attention_weights=False, local_gat=None):
        from torch_geometric.nn.conv.gat_conv import GATConv
        from . import ops
        weight, att, fused_bias, C4 = GATConv._fused_operands(self)
        xw = ops.feature_transform(x_own, weight, row_exact=ops.GAT_ROW_EXACT_GEMM)
        drop = self.dropout if self.training else 0.0
        out, aw = sg.gat_propagate(xw, att, self.heads, C4, self.negative_slope, fused_bias,
                                   return_attention_weights, drop, local_gat=local_gat)
        out = GATConv._finish(self, out, C4)
        return (out, aw) if return_attention_weights else out

    def __repr__(self):
        return "{}({}, {}, heads={})".format(self.__class__.__name__, self.in_channels, self.out_channels,
                                            self.heads)
