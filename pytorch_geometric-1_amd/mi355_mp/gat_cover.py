"""Sharded GATConv over the hybrid halo cover (callers
/root/reference/ConvexPruning.py:209-224, examples/ppi.py:22-28).

The pull form (ShardedGraph.gat_propagate without a cover) ships X W of every
remote source of the rank's in-edges.  A GAT destination row is a softmax-
weighted sum, and softmax sums split into online-softmax pieces that merge
exactly (GatRed::merge): a cross edge j -> i (j owned by q, i by p) can be
covered by q pushing its PIECE of row i -- the state (m, den, acc / den) of
the softmax over q's own sources of i's in-edges -- instead of p pulling
x_j.  Which edges are pushed is HaloCover's rule (the endpoint with the larger
cross-degree; on RMAT graphs 0.56-0.57x the pull rows).  One step:

  forward (rank p; every rank is also the "q" of its peers)
    1. node scores of the own rows; a_dst of every destination some peer pushes
       a piece of goes to that peer (H floats per row, one all_to_all)
    2. the send rows: ONE fused GAT aggregation over the send graph (a pulled
       row is a one-edge row: alpha = 1, the row itself bit for bit; a pushed
       row is the piece over the push edges, with the received a_dst), then
       the rows and their (m, den) go out (two all_to_alls)
    3. the local piece of every own row: the fused GAT aggregation over the
       interior and pulled edges (global edge order), node scores of the
       received rows first
    4. mp_gat_merge_partials_f32: the pieces of each row, local first, then the
       peers' in rank order, plus the bias.  A row no peer pushes a piece of is
       the single-GPU kernel's row bit for bit (same edges, same order); merged
       rows are within the 1e-5 bound (regrouped softmax sums).
  backward (the global softmax gradient, split by where each edge lives)
    p: pack (a_dst, M, 1/den, rs) per own row from the MERGED stats (rs over
       out - bias), the node-wise d a_dst of the local edges (the training
       forward's agg2 / s2 scaled to the merged rows), the transposed pass
       over the local edges; then ONE reverse all_to_all of [n_halo, H*C]:
       a pulled row's slot carries its gradient back to its owner, a pushed
       piece's slot carries the gradient g_i of its destination (and a second,
       its pack).
    q: a pulled row's gradient folds into the own row it copied; the pushed
       pieces' edges take the GAT backward over the transposed push graph
       (mp_gat_backward_f32: d xw_j, d a_src_j, de per edge), and the per-row
       sums of de -- the peer's share of d a_dst_i -- go back to p (one
       all_to_all of H floats per pushed row).
    p: d a_dst_i complete; its att_dst term of d xw and the d att partials.
  Every collective runs in the same order on every rank.

Device path: the HIP kernels (GatHaloCover.forward_device / backward_device,
wrapped by _GatCoverFn); no CPU fallback.  The gloo CPU tests check the
distributed algorithm, forward and backward, against the single-process
oracle with a host twin of the same data flow in differentiable torch ops
(tests/_host_twins.py, installed through dist.install_host_twins).  Heads of any width (GATConv pads C to a
multiple of 4): C / 4 a power of two <= 64 takes the fused transposed pass,
whose per-edge d score gives a pusher its share of d a_dst; other widths the
wide kernels, the share then node-wise from the pieces' training accumulators
(out2, s2) rescaled to the merged row.

Attention dropout (training) keys its hashed keep mask on each edge's GLOBAL
id, as the single-GPU layer does (ABI 7 drop_ids): the local piece's edges
carry their plan's global ids, the pushed pieces' edges the ids their owner
sent with them (HaloCover(edge_ids=True)).  A piece keeps the undropped
softmax statistics and the dropped weights on its sum, so the merge rule is
unchanged; the pulled rows are plain copies (no attention edge, no mask);
a pusher's share of d a_dst comes node-wise from its pieces' (out2, s2)
whatever the head width.

return_alpha: the alpha of every in-edge of the rank's rows, in the plan's
local edge order, from the MERGED row statistics: the local piece's edges
directly; for a pushed edge the destination's merged (max, denominator) go
back to the pusher (one all_to_all of H pairs per piece), which evaluates the
edge's alpha with the a_dst it received and returns it (one all_to_all of H
floats per push edge).
"""
import torch

from .dist import HaloCover, _a2a


def fused_heads(H, C):
    """Heads whose C/4 is a power of two <= 64 (mp_gat_train_ok): the fused
    transposed pass with per-edge d score serves the pushed pieces' edges.
    Other widths take the wide kernels (any C % 4 == 0)."""
    q = C // 4
    return H > 0 and C % 4 == 0 and 1 <= q <= 64 and (q & (q - 1)) == 0


def cover_ok(H, C):
    """Head shapes the device path takes: any C % 4 == 0 (GATConv pads every
    head to it); fused_heads picks the kernels."""
    return H > 0 and C > 0 and C % 4 == 0


def _cat_ranges(starts, lengths, dev):
    """concatenation of arange(s, s + n) over (s, n) pairs, as an int64 tensor."""
    parts = [torch.arange(s, s + n, dtype=torch.int64, device=dev) for s, n in zip(starts, lengths) if n]
    return torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int64, device=dev)


class GatHaloCover:
    """The GAT form of HaloCover for one rank of a ShardedGraph.for_gat plan
    (built collectively over `group`, like HaloCover).  Index structures:

      loc_src / loc_dst   the local piece's edges, global edge order: interior
                          edges and pulled edges (source = its halo slot)
      part_row / part_dst per received piece: its row in the receive buffer and
                          the own destination row (the merge list)
      adst_rows           own destination rows whose a_dst the peers need, in
                          the order of their pushed rows (per owner)
      send graph          copy edges (own row -> send row) and push edges (own
                          source -> pushed send row), rows = this rank's send
                          buffer (per peer: pulled rows, then pieces)
    Graphs are built lazily on the device of the plan."""

    def __init__(self, plan, group=None):
        hc = HaloCover(plan, None, group, edge_ids=True)
        self.hc, self.plan, self.group = hc, plan, group
        dev = plan.halo_nodes.device
        n_own = plan.n_own
        self.n_own = n_own
        self.n_halo, self.n_local_src, self.n_send = hc.n_halo, hc.n_local_src, hc.n_send
        self.recv_counts, self.send_counts = hc.recv_counts, hc.send_counts
        self.n_pull_rows, self.n_push_rows = hc.n_pull_rows, hc.n_push_rows
        self.n_pull_edges, self.n_push_edges = hc.n_pull_edges, hc.n_push_edges
        # the local piece: plan order (= global edge order), pushed edges left out,
        # a pulled edge's source replaced by its halo slot
        lei = plan.local_edge_index
        src, dst = lei[0].clone(), lei[1]
        src[hc.pull_pos] = hc.pull_halo
        loc = torch.sort(torch.cat([hc.int_pos, hc.pull_pos])).values
        self.loc_pos = loc                                     # plan positions of the local piece's edges
        self.loc_src, self.loc_dst = src[loc].contiguous(), dst[loc].contiguous()
        self.loc_gid = plan.edge_gid[loc].contiguous()        # attention-dropout keys
        self.push_gid = hc.push_gid
        # return_alpha: the push edges' plan positions in the order they went out, and
        # the per-owner push-edge counts both ways
        self.push_pos = hc.push_pos
        self.push_edges_to, self.push_edges_from = hc.push_edges_to, hc.push_edges_from
        self.n_interior = int(hc.int_pos.numel())
        # received pieces -> own destination (the merge list)
        self.part_row = (hc.push_halo - n_own).contiguous()
        self.part_dst = hc.push_dst.contiguous()
        # a_dst requests: the destinations of the pieces this rank receives, grouped by
        # the pushing owner in its row order (ascending destination within an owner)
        self.adst_rows = hc.push_dst.contiguous()
        self.adst_send_counts = list(hc.n_push_rows_to)
        self.adst_recv_counts = list(hc.send_push_counts)
        # send buffer positions of this rank's pushed rows, per peer after its pulled rows
        base = [0]
        for c in self.send_counts:
            base.append(base[-1] + c)
        self.send_push_rows = _cat_ranges([b + s for b, s in zip(base[:-1], hc.send_pull_counts)],
                                          hc.send_push_counts, dev)
        n_copy = sum(hc.send_pull_counts)
        self.copy_src, self.copy_dst = hc.send_src[:n_copy].contiguous(), hc.send_dst[:n_copy].contiguous()
        self.push_src, self.push_dst = hc.send_src[n_copy:].contiguous(), hc.send_dst[n_copy:].contiguous()
        self.send_src = hc.send_src.contiguous()
        self.send_dst = hc.send_dst.contiguous()
        self._graphs = None

    # ------------------------------------------------------------------ graphs
    def graphs(self):
        """(local piece, send graph, merge list, transposed copy graph, push
        graph) as native Graphs, built once."""
        if self._graphs is None:
            from .graph import GAT_TARGET_TASKS, Graph
            n_own = self.n_own
            g_loc = Graph(torch.stack([self.loc_src, self.loc_dst]), n_own, self.n_local_src,
                          target_tasks=GAT_TARGET_TASKS)
            g_send = Graph(torch.stack([self.send_src, self.send_dst]), self.n_send, n_own,
                           target_tasks=GAT_TARGET_TASKS)
            g_merge = Graph(torch.stack([self.part_row, self.part_dst]), n_own, max(self.n_halo, 1))
            g_copy_t = Graph(torch.stack([self.copy_dst, self.copy_src]), n_own, max(self.n_send, 1))
            g_push = Graph(torch.stack([self.push_src, self.push_dst]), self.n_send, n_own,
                           target_tasks=GAT_TARGET_TASKS)
            # attention dropout keyed on the global edge ids (Graph.drop_ids)
            g_loc.edge_key, g_push.edge_key = self.loc_gid, self.push_gid
            self._graphs = (g_loc, g_send, g_merge, g_copy_t, g_push)
        return self._graphs

    def stats(self):
        return {"cover_pulled_rows": self.n_pull_rows, "cover_partial_rows": self.n_push_rows,
                "cover_push_edges": self.n_push_edges, "halo_rows": self.n_halo,
                "pull_halo_rows": self.plan.n_local_src - self.plan.n_own,
                "send_rows": self.n_send, "local_piece_edges": int(self.loc_src.numel())}

    # ---------------------------------------------------------- device (HIP)
    def forward_device(self, xw_own, att_c, H, C, slope, bias, train, exchange=True, drop=None, keep=False):
        """The step on the fused kernels.  Returns (out [n_own, H*C] with bias,
        saved) -- saved holds what backward_device needs when train.
        exchange=False: the compute alone (no collective; the receive buffers
        hold zeros), for decompose().  drop = (seed, p): attention dropout
        (training form).  keep: return saved outside training too (alpha)."""
        from . import _lib
        lib = _lib.load()
        g_loc, g_send, g_merge, _, g_push = self.graphs()
        train = train or drop is not None
        dev = xw_own.device
        st = _lib.stream_ptr(dev)
        n_own, F = self.n_own, H * C
        grp = self.group
        fused = fused_heads(H, C)
        node_scores = lib.mp_gat_node_scores_f32 if fused else lib.mp_gat_node_scores_wide_f32
        xl = torch.empty((self.n_local_src, F), dtype=torch.float32, device=dev)
        xl[:n_own].copy_(xw_own)
        a_src = torch.empty((self.n_local_src, H), dtype=torch.float32, device=dev)
        a_dst = torch.empty((self.n_local_src, H), dtype=torch.float32, device=dev)
        if n_own:
            _lib.check(node_scores(xl.data_ptr(), n_own, H, C, att_c.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                   st), "mp_gat_node_scores (own rows)")
        # 1. a_dst of the rows the peers push pieces of
        a2a = _a2a if exchange else (lambda o, *a: o.zero_())
        adst_in = torch.empty((sum(self.adst_recv_counts), H), dtype=torch.float32, device=dev)
        a2a(adst_in, a_dst[self.adst_rows].contiguous(), self.adst_recv_counts, self.adst_send_counts, grp)
        send_adst = torch.zeros((max(self.n_send, 1), H), dtype=torch.float32, device=dev)
        if adst_in.shape[0]:
            send_adst[self.send_push_rows] = adst_in
        # 2. the send rows: one fused aggregation over the send graph, then rows + stats out
        #    (wide heads in training: the training form, whose out2 / s2 of the pushed
        #    pieces give this rank's share of d a_dst node-wise in the backward)
        send = torch.empty((self.n_send, F), dtype=torch.float32, device=dev)
        send_st = torch.empty((self.n_send, H, 2), dtype=torch.float32, device=dev)
        send2 = send_s2 = None
        if self.n_send and drop is not None:
            # the pushed pieces over the push graph with the keep mask of their
            # global edge ids (training form: out2 / s2 give this rank's share of
            # d a_dst), then the pulled rows copied in -- a copy is not an
            # attention edge; alpha = 1 would give the row itself bit for bit
            send2 = torch.zeros((self.n_send, F), dtype=torch.float32, device=dev)
            send_s2 = torch.zeros((self.n_send, H), dtype=torch.float32, device=dev)
            if self.push_src.numel():
                gp = g_push.dst.struct("other")
                sb = lib.mp_gat_train_slab_bytes(gp, H, C)
                slab = torch.empty(sb, dtype=torch.uint8, device=dev)
                _lib.check(lib.mp_gat_aggregate_train_drop_f32(gp, xl.data_ptr(), a_src.data_ptr(),
                                                               send_adst.data_ptr(), att_c.data_ptr(), H, C,
                                                               float(slope), None, send.data_ptr(), F, None,
                                                               send_st.data_ptr(), send2.data_ptr(),
                                                               send_s2.data_ptr(), int(drop[0]), float(drop[1]),
                                                               g_push.drop_ids("dst").data_ptr(), slab.data_ptr(), sb,
                                                               _lib.MP_STAGE_ALL, st),
                           "mp_gat_aggregate_train_drop_f32 (pushed pieces)")
                del slab
            else:
                send.zero_()
                send_st.zero_()
            if self.copy_src.numel():
                send[self.copy_dst] = xl[self.copy_src]
        elif self.n_send:
            gs = g_send.dst.struct("other")
            if train and not fused:
                send2 = torch.empty((self.n_send, F), dtype=torch.float32, device=dev)
                send_s2 = torch.empty((self.n_send, H), dtype=torch.float32, device=dev)
                sb = lib.mp_gat_train_slab_bytes(gs, H, C)
                slab = torch.empty(sb, dtype=torch.uint8, device=dev)
                _lib.check(lib.mp_gat_aggregate_train_f32(gs, xl.data_ptr(), a_src.data_ptr(), send_adst.data_ptr(),
                                                          att_c.data_ptr(), H, C, float(slope), None, send.data_ptr(),
                                                          F, None, send_st.data_ptr(), send2.data_ptr(),
                                                          send_s2.data_ptr(), slab.data_ptr(), sb, _lib.MP_STAGE_ALL,
                                                          st), "mp_gat_aggregate_train_f32 (send rows)")
            else:
                sb = lib.mp_gat_slab_bytes(gs, H, C)
                slab = torch.empty(sb, dtype=torch.uint8, device=dev)
                _lib.check(lib.mp_gat_aggregate_att_f32(gs, xl.data_ptr(), a_src.data_ptr(), send_adst.data_ptr(),
                                                        att_c.data_ptr(), H, C, float(slope), None, send.data_ptr(),
                                                        F, send_st.data_ptr(), slab.data_ptr(), sb, _lib.MP_STAGE_ALL,
                                                        st), "mp_gat_aggregate_att_f32 (send rows)")
            del slab
        r_st = torch.empty((self.n_halo, H, 2), dtype=torch.float32, device=dev)
        a2a(xl[n_own:], send, self.recv_counts, self.send_counts, grp)
        a2a(r_st, send_st, self.recv_counts, self.send_counts, grp)
        if self.n_halo:
            _lib.check(node_scores(xl[n_own:].data_ptr(), self.n_halo, H, C, att_c.data_ptr(),
                                   a_src[n_own:].data_ptr(), a_dst[n_own:].data_ptr(), st),
                       "mp_gat_node_scores (received rows)")
        # 3. the local piece (no bias: the merge adds it)
        out = torch.empty((n_own, F), dtype=torch.float32, device=dev)
        stats = torch.empty((n_own, H, 2), dtype=torch.float32, device=dev)
        agg2 = s2 = None
        if n_own:
            gl = g_loc.dst.struct("other")
            if drop is not None:
                agg2 = torch.empty((n_own, F), dtype=torch.float32, device=dev)
                s2 = torch.empty((n_own, H), dtype=torch.float32, device=dev)
                sb = lib.mp_gat_train_slab_bytes(gl, H, C)
                slab = torch.empty(sb, dtype=torch.uint8, device=dev)
                _lib.check(lib.mp_gat_aggregate_train_drop_f32(gl, xl.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                               att_c.data_ptr(), H, C, float(slope), None,
                                                               out.data_ptr(), F, None, stats.data_ptr(),
                                                               agg2.data_ptr(), s2.data_ptr(), int(drop[0]),
                                                               float(drop[1]), g_loc.drop_ids("dst").data_ptr(),
                                                               slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
                           "mp_gat_aggregate_train_drop_f32 (local piece)")
            elif train:
                agg2 = torch.empty((n_own, F), dtype=torch.float32, device=dev)
                s2 = torch.empty((n_own, H), dtype=torch.float32, device=dev)
                sb = lib.mp_gat_train_slab_bytes(gl, H, C)
                slab = torch.empty(sb, dtype=torch.uint8, device=dev)
                _lib.check(lib.mp_gat_aggregate_train_f32(gl, xl.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                          att_c.data_ptr(), H, C, float(slope), None, out.data_ptr(),
                                                          F, None, stats.data_ptr(), agg2.data_ptr(), s2.data_ptr(),
                                                          slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
                           "mp_gat_aggregate_train_f32 (local piece)")
            else:
                sb = lib.mp_gat_slab_bytes(gl, H, C)
                slab = torch.empty(sb, dtype=torch.uint8, device=dev)
                _lib.check(lib.mp_gat_aggregate_att_f32(gl, xl.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                        att_c.data_ptr(), H, C, float(slope), None, out.data_ptr(), F,
                                                        stats.data_ptr(), slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
                           "mp_gat_aggregate_att_f32 (local piece)")
            del slab
            # 4. merge the pieces (+ bias; agg2 / s2 scaled to the merged rows)
            m = g_merge.dst
            merged = self.part_row.numel() > 0
            n_parts = self.n_halo if merged else 0       # rows of the receive buffer the merge list names
            _lib.check(lib.mp_gat_merge_partials_f32(n_own, H, C, m.rowptr.data_ptr(),
                                                     m.col.data_ptr() if merged else None, n_parts,
                                                     xl[n_own:].data_ptr() if merged else None,
                                                     _lib.nbytes(xl[n_own:]), F,
                                                     r_st.data_ptr() if merged else None, _lib.nbytes(r_st),
                                                     _lib.ptr(bias),
                                                     out.data_ptr(), F, stats.data_ptr(), _lib.ptr(agg2),
                                                     _lib.ptr(s2), st), "mp_gat_merge_partials_f32")
        saved = (xl, a_src, a_dst, stats, agg2, s2, send_st, send2, send_s2, drop, send_adst) if (train or keep) else None
        return out, saved

    def decompose(self, xw_own, att, H, C, slope, bias, reps=10, barrier=None):
        """The forward step taken apart on this rank (wall clock over `reps`,
        the device synchronised after them, ranks lined up by `barrier`):
        exchange_only_ms -- the three all_to_alls (a_dst requests, rows, stats)
        with packed buffers; compute_only_ms -- node scores, send rows, local
        piece and merge with no collective; step_ms -- the step itself;
        hidden_frac as OverlappedAggregation.decompose (the GAT step runs its
        pieces in order, so ~0 means nothing is hidden)."""
        import time
        H, C = int(H), int(C)
        att_c = att.reshape(H, 2 * C).contiguous().to(torch.float32)
        dev = xw_own.device
        F = H * C
        grp = self.group
        adst_s = torch.zeros((sum(self.adst_send_counts), H), dtype=torch.float32, device=dev)
        adst_r = torch.empty((sum(self.adst_recv_counts), H), dtype=torch.float32, device=dev)
        rows_s = torch.zeros((self.n_send, F), dtype=torch.float32, device=dev)
        rows_r = torch.empty((self.n_halo, F), dtype=torch.float32, device=dev)
        st_s = torch.zeros((self.n_send, H, 2), dtype=torch.float32, device=dev)
        st_r = torch.empty((self.n_halo, H, 2), dtype=torch.float32, device=dev)

        def exchange():
            _a2a(adst_r, adst_s, self.adst_recv_counts, self.adst_send_counts, grp)
            _a2a(rows_r, rows_s, self.recv_counts, self.send_counts, grp)
            _a2a(st_r, st_s, self.recv_counts, self.send_counts, grp)

        def timed(fn):
            fn()
            if barrier is not None:
                barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps * 1e3

        res = {"exchange_only_ms": timed(exchange),
               "compute_only_ms": timed(lambda: self.forward_device(xw_own, att_c, H, C, slope, bias, False,
                                                                   exchange=False)),
               "step_ms": timed(lambda: self.forward_device(xw_own, att_c, H, C, slope, bias, False))}
        import torch.distributed as tdist
        from .dist import hidden_fraction
        res.update(hidden_fraction(res, staged=xw_own.is_cuda and tdist.get_backend(grp) == "gloo"))
        return res

    def alpha(self, saved, H, slope):
        """alpha [m, H] of this rank's in-edges, in the plan's local edge order
        (GATConv's return_attention_weights: the undropped softmax), from the
        forward's node scores and merged row statistics (saved of
        forward_device).  Collective over the group (two all_to_alls)."""
        from . import _lib
        lib = _lib.load()
        xl, a_src, a_dst, stats, _, _, _, _, _, _, send_adst = saved
        dev = xl.device
        st = _lib.stream_ptr(dev)
        E_l = int(self.plan.local_edge_index.shape[1])
        alpha = torch.zeros((E_l, H), dtype=torch.float32, device=dev)
        n_loc = int(self.loc_src.numel())
        if n_loc:
            a_loc = torch.empty((n_loc, H), dtype=torch.float32, device=dev)
            _lib.check(lib.mp_gat_alpha_f32(self.loc_src.data_ptr(), self.loc_dst.data_ptr(), n_loc, H,
                                            a_src.data_ptr(), a_dst.data_ptr(), float(slope), stats.data_ptr(),
                                            a_loc.data_ptr(), st), "mp_gat_alpha_f32 (local piece)")
            alpha[self.loc_pos] = a_loc
        # the merged (max, denominator) of each pushed destination back to its pusher
        rev_st = torch.zeros((self.n_halo, H, 2), dtype=torch.float32, device=dev)
        if self.part_row.numel():
            rev_st[self.part_row] = stats[self.part_dst]
        back_st = torch.zeros((self.n_send, H, 2), dtype=torch.float32, device=dev)
        _a2a(back_st, rev_st, self.send_counts, self.recv_counts, self.group)
        # the pusher evaluates its push edges' alpha, which return to the destination's owner
        E_push = int(self.push_src.numel())
        a_push = torch.empty((E_push, H), dtype=torch.float32, device=dev)
        if E_push:
            _lib.check(lib.mp_gat_alpha_f32(self.push_src.data_ptr(), self.push_dst.data_ptr(), E_push, H,
                                            a_src.data_ptr(), send_adst.data_ptr(), float(slope), back_st.data_ptr(),
                                            a_push.data_ptr(), st), "mp_gat_alpha_f32 (pushed pieces)")
        got = torch.empty((sum(self.push_edges_to), H), dtype=torch.float32, device=dev)
        _a2a(got, a_push, self.push_edges_to, self.push_edges_from, self.group)
        if got.shape[0]:
            alpha[self.push_pos] = got
        return alpha

    def backward_device(self, g, out, bias, att_c, H, C, slope, saved, want_att, want_bias):
        """d xw_own, d att (or None), d bias (or None) of forward_device (see the
        module docstring for the split)."""
        from . import _lib, ops
        lib = _lib.load()
        g_loc, _, g_merge, g_copy_t, g_push = self.graphs()
        xl, a_src, a_dst, stats, agg2, s2, send_st, send2, send_s2, drop, _ = saved
        seed, p_drop = (0, 0.0) if drop is None else (int(drop[0]), float(drop[1]))
        dev = g.device
        st = _lib.stream_ptr(dev)
        n_own, F, grp = self.n_own, H * C, self.group
        nl = self.n_local_src
        fused = fused_heads(H, C)

        def wide_pass(gt_struct, n_rows, grad_out, pack_, xw_rows, gx_out, graph):
            """mp_gat_backward_wide_f32 + its epilogue over a transposed graph of
            n_rows source rows (graph: its Graph, for the dropout keys):
            gx_out += sum alpha g + d a_src att_src; returns d a_src."""
            acc2 = torch.zeros((n_rows, F), dtype=torch.float32, device=dev)
            sc = torch.zeros((n_rows, H), dtype=torch.float32, device=dev)
            sb = lib.mp_gat_train_slab_bytes(gt_struct, H, C)
            slab = torch.empty(sb, dtype=torch.uint8, device=dev)
            _lib.check(lib.mp_gat_backward_wide_f32(gt_struct, grad_out.data_ptr(), F, a_src.data_ptr(),
                                                    pack_.data_ptr(), H, C, float(slope), seed, p_drop,
                                                    graph.drop_ids("src").data_ptr() if drop is not None else None,
                                                    gx_out.data_ptr(),
                                                    acc2.data_ptr(), _lib.nbytes(acc2), sc.data_ptr(),
                                                    _lib.nbytes(sc), slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
                       "mp_gat_backward_wide_f32 (cover)")
            del slab
            zero_gd = torch.zeros((n_rows, H), dtype=torch.float32, device=dev)
            _lib.check(lib.mp_gat_backward_epilogue_wide_f32(gx_out.data_ptr(), acc2.data_ptr(), xw_rows.data_ptr(),
                                                             att_c.data_ptr(), zero_gd.data_ptr(), sc.data_ptr(),
                                                             n_rows, H, C, st), "mp_gat_backward_epilogue_wide_f32")
            return sc

        # p: pack from the merged stats, node-wise d a_dst of the local edges
        pack = torch.zeros((max(n_own, 1), H, 4), dtype=torch.float32, device=dev)
        ga_dst = torch.zeros((max(n_own, 1), H), dtype=torch.float32, device=dev)
        if n_own:
            if fused:
                _lib.check(lib.mp_gat_backward_prep_train_f32(g.data_ptr(), F, out.data_ptr(), F, _lib.ptr(bias),
                                                              agg2.data_ptr(), s2.data_ptr(), a_dst.data_ptr(),
                                                              stats.data_ptr(), n_own, H, C, pack.data_ptr(),
                                                              _lib.nbytes(pack), None, 0, ga_dst.data_ptr(), st),
                           "mp_gat_backward_prep_train_f32 (cover)")
            else:
                _lib.check(lib.mp_gat_backward_prep_wide_f32(g.data_ptr(), F, out.data_ptr(), F, _lib.ptr(bias),
                                                             agg2.data_ptr(), s2.data_ptr(), a_dst.data_ptr(),
                                                             stats.data_ptr(), n_own, H, C, pack.data_ptr(),
                                                             _lib.nbytes(pack), ga_dst.data_ptr(), st),
                           "mp_gat_backward_prep_wide_f32 (cover)")
        # p: the transposed pass over the local edges (the att_dst term comes last)
        gx_l = torch.zeros((nl, F), dtype=torch.float32, device=dev)
        ga_src_l = torch.zeros((nl, H), dtype=torch.float32, device=dev)
        if n_own and g_loc.dst.n_edges:
            gt = g_loc.src_with_dst_slots()
            gs = gt.struct("dst_slot")
            if fused and drop is not None:
                zero_gd = torch.zeros((nl, H), dtype=torch.float32, device=dev)
                sb = lib.mp_gat_slab_bytes(gs, H, C)
                slab = torch.empty(sb, dtype=torch.uint8, device=dev)
                _lib.check(lib.mp_gat_backward_train_drop_f32(gs, g.data_ptr(), F, xl.data_ptr(), a_src.data_ptr(),
                                                              pack.data_ptr(), att_c.data_ptr(), H, C, float(slope),
                                                              zero_gd.data_ptr(), seed, p_drop,
                                                              g_loc.drop_ids("src").data_ptr(), gx_l.data_ptr(),
                                                              ga_src_l.data_ptr(), slab.data_ptr(), sb,
                                                              _lib.MP_STAGE_ALL, st),
                           "mp_gat_backward_train_drop_f32 (local piece)")
                del slab, zero_gd
            elif fused:
                zero_gd = torch.zeros((nl, H), dtype=torch.float32, device=dev)
                sb = lib.mp_gat_slab_bytes(gs, H, C)
                slab = torch.empty(sb, dtype=torch.uint8, device=dev)
                _lib.check(lib.mp_gat_backward_train_f32(gs, g.data_ptr(), F, xl.data_ptr(), a_src.data_ptr(),
                                                         pack.data_ptr(), att_c.data_ptr(), H, C, float(slope),
                                                         zero_gd.data_ptr(), gx_l.data_ptr(), ga_src_l.data_ptr(),
                                                         slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
                           "mp_gat_backward_train_f32 (local piece)")
                del slab, zero_gd
            else:
                ga_src_l = wide_pass(gs, nl, g, pack, xl, gx_l, g_loc)
        # reverse exchange: a pulled slot returns its row's gradient to the owner, a
        # piece's slot carries its destination's g and pack to the peer that pushed it
        rev = gx_l[n_own:]
        rev_pack = torch.zeros((self.n_halo, H * 4), dtype=torch.float32, device=dev)
        if self.part_row.numel():
            rev[self.part_row] = g[self.part_dst]
            rev_pack[self.part_row] = pack.view(-1, H * 4)[self.part_dst]
        back = torch.empty((self.n_send, F), dtype=torch.float32, device=dev)
        back_pack = torch.empty((self.n_send, H * 4), dtype=torch.float32, device=dev)
        _a2a(back, rev.contiguous(), self.send_counts, self.recv_counts, grp)
        _a2a(back_pack, rev_pack, self.send_counts, self.recv_counts, grp)
        # q: pulled rows' gradients fold into the rows they copied
        gx = gx_l[:n_own].clone()
        if self.copy_src.numel():
            gx += ops._aggregate(g_copy_t.dst, "other", back, None, "sum", 0, None)[0]
        # q: the pushed pieces' edges (global softmax gradient with p's pack)
        ga_src_push = torch.zeros((max(n_own, 1), H), dtype=torch.float32, device=dev)
        ga_back = torch.zeros((self.n_send, H), dtype=torch.float32, device=dev)
        E_push = int(self.push_src.numel())
        if E_push and (not fused or drop is not None):
            # wide heads (the fused pass's per-edge d score needs C/4 a power of two) and
            # attention dropout (that pass has no dropout form): this rank's share of
            # d a_dst comes node-wise from its pieces' training accumulators instead:
            # with c = den_q e^(m_q - M) / den the piece's weight in the merged row,
            # share = c (<g, out2_q> - rs s2_q)
            gt = g_push.src_with_dst_slots()
            gx_push = torch.zeros((n_own, F), dtype=torch.float32, device=dev)
            ga_src_push = wide_pass(gt.struct("dst_slot"), n_own, back, back_pack, xl[:n_own], gx_push, g_push)
            gx += gx_push
            pk = back_pack.view(-1, H, 4)
            c = send_st[..., 1] * torch.exp(send_st[..., 0] - pk[..., 1]) * pk[..., 2]
            dot = (back.view(-1, H, C) * send2.view(-1, H, C)).sum(-1)
            share = c * (dot - pk[..., 3] * send_s2)
            ga_back = torch.zeros_like(share)
            ga_back[self.send_push_rows] = share[self.send_push_rows]
        elif E_push:
            gt = g_push.src_with_dst_slots()
            gs = gt.struct("dst_slot")
            gx_push = torch.empty((n_own, F), dtype=torch.float32, device=dev)
            de = torch.empty((E_push, H), dtype=torch.float32, device=dev)
            sb = lib.mp_gat_slab_bytes(gs, H, C)
            slab = torch.empty(sb, dtype=torch.uint8, device=dev)
            _lib.check(lib.mp_gat_backward_f32(gs, back.data_ptr(), F, xl.data_ptr(), a_src.data_ptr(),
                                               back_pack.data_ptr(), att_c.data_ptr(), H, C, float(slope),
                                               gx_push.data_ptr(), ga_src_push.data_ptr(), de.data_ptr(),
                                               _lib.nbytes(de), slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
                       "mp_gat_backward_f32 (pushed pieces)")
            del slab
            gx += gx_push
            ga_back = ops._aggregate(g_push.dst, "slot", de, None, "sum", 0, None)[0]
        # the peers' shares of d a_dst come home
        ga_in = torch.empty((self.n_halo, H), dtype=torch.float32, device=dev)
        _a2a(ga_in, ga_back.contiguous(), self.recv_counts, self.send_counts, grp)
        if n_own and self.part_row.numel():
            ga_dst = ga_dst + ops._aggregate(g_merge.dst, "other", ga_in, None, "sum", 0, None)[0]
        ga_dst = ga_dst[:n_own]
        if n_own:
            _lib.check(lib.mp_heads_outer_add_f32(gx.data_ptr(), F, ga_dst.contiguous().data_ptr(), n_own, H, C,
                                                  att_c.data_ptr(), 2 * C, st), "mp_heads_outer_add_f32")
        gatt = None
        if want_att:
            x_own3 = xl[:n_own].view(n_own, H, C)
            d_dst = torch.einsum("nh,nhc->hc", ga_dst, x_own3)
            d_src = (torch.einsum("nh,nhc->hc", ga_src_l, xl.view(nl, H, C))
                     + torch.einsum("nh,nhc->hc", ga_src_push[:n_own], x_own3))
            gatt = torch.cat([d_dst, d_src], dim=-1)
        gb = ops.col_sums(g) if want_bias else None
        return gx, gatt, gb


class _GatCoverFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xw_own, att, bias, cover, H, C, slope, drop, holder):
        att_c = att.reshape(H, 2 * C).contiguous().to(torch.float32)
        out, saved = cover.forward_device(xw_own.contiguous(), att_c, H, C, slope, bias, True, drop=drop)
        if holder is not None:           # return_alpha: the caller evaluates alpha from them
            holder["saved"] = saved
        ctx.cover, ctx.H, ctx.C, ctx.slope = cover, H, C, slope
        ctx.saved = saved
        ctx.save_for_backward(out, bias, att_c)
        return out

    @staticmethod
    def backward(ctx, g):
        out, bias, att_c = ctx.saved_tensors
        g = g.contiguous()
        if g.data_ptr() % 16:
            g = g.clone()
        gx, gatt, gb = ctx.cover.backward_device(g, out, bias, att_c, ctx.H, ctx.C, ctx.slope, ctx.saved,
                                                 ctx.needs_input_grad[1], bias is not None and ctx.needs_input_grad[2])
        ctx.saved = None
        if gatt is not None:
            gatt = gatt.view(1, ctx.H, 2 * ctx.C)
        return gx, gatt, gb, None, None, None, None, None, None


def gat_cover_propagate(cover, xw_own, att, heads, out_channels, negative_slope=0.2, bias=None, dropout=0.0,
                        seed=None, return_alpha=False):
    """This rank's rows of the fused GATConv aggregation over the cover (+ bias)
    on the HIP path with its native backward; a host tensor raises.
    dropout > 0: GATConv's training-mode attention dropout, its keep mask keyed
    on the global edge ids (seed from the device's generator unless given):
    the single-GPU layer's mask.  return_alpha: (out, alpha [m, H] of this
    rank's in-edges in the plan's local edge order) (GatHaloCover.alpha)."""
    H, C = int(heads), int(out_channels)
    if xw_own.shape[0] != cover.n_own:
        raise ValueError("mi355_mp.gat_cover: xw_own has %d rows, this rank owns %d" % (xw_own.shape[0], cover.n_own))
    if not xw_own.is_cuda:
        raise RuntimeError("mi355_mp.gat_cover: host tensors -- there is no CPU fallback: the engine runs on ROCm "
                           "device tensors")
    if not cover_ok(H, C):
        raise ValueError("mi355_mp.gat_cover: heads of %d features need C %% 4 == 0 (GATConv pads them)" % C)
    drop = None
    if dropout > 0:
        from . import ops
        if not ops.gat_dropout_ok(H, C, dropout):
            raise ValueError("mi355_mp.gat_cover: attention dropout needs 0 < p < 1 and H <= 32 (got p=%g, H=%d)"
                             % (dropout, H))
        if seed is None:
            seed = ops.dropout_seed(xw_own.device)
        drop = (int(seed) & 0xFFFFFFFFFFFFFFFF, float(dropout))
    needs = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (xw_own, att, bias))
    if not needs:
        att_c = att.reshape(H, 2 * C).contiguous().to(torch.float32)
        out, saved = cover.forward_device(xw_own.contiguous(), att_c, H, C, float(negative_slope), bias, False,
                                          drop=drop, keep=return_alpha)
    else:
        holder = {} if return_alpha else None
        out = _GatCoverFn.apply(xw_own, att, bias, cover, H, C, float(negative_slope), drop, holder)
        saved = holder["saved"] if return_alpha else None
    if not return_alpha:
        return out
    with torch.no_grad():
        return out, cover.alpha(saved, H, float(negative_slope))
