"""Host twins of mi355_mp's native pieces -- TEST INFRASTRUCTURE, never part of
the product path (mi355_mp has no CPU fallback: a host tensor raises there).

The gloo tests (tests/test_dist_gloo.py) run the distributed logic of
mi355_mp.dist on CPU: plans, slice builds, the halo covers, their collectives.
The local compute of those runs -- a shard plan, row gathers, the ordered
segment sums, the GCN norm of a plan's local edges, GATConv's loops and the
GAT cover's step -- comes from here, installed per rank process with
mi355_mp.dist.install_host_twins(tests._host_twins).  Each twin is the
reference's own torch-op arithmetic (PyG 1.4.3 / torch_scatter 2.0.4 on the
CPU), so the gloo results are checked against the single-process oracle.
"""
import sys

import torch
import torch.distributed as dist


def plan(key, other, num_nodes, cuts, rank, world):
    """The plan of rank `rank` in torch ops (mp_shard_plan's host twin; also
    the GPU tests' checker of it).  Returns (edge_pos, local key, local other,
    halo_nodes, recv_counts)."""
    dev = key.device
    lo, hi = cuts[rank], cuts[rank + 1]
    mine = (key >= lo) & (key < hi)
    edge_pos = torch.nonzero(mine).view(-1)                  # positions in the global edge order
    k = key[edge_pos] - lo
    o = other[edge_pos]
    if o.numel() and (int(o.min()) < 0 or int(o.max()) >= num_nodes):
        raise IndexError("mi355_mp.dist: an edge endpoint lies outside [0, %d)" % num_nodes)
    owner = torch.searchsorted(torch.tensor(cuts[1:], device=dev), o, right=True)
    remote = owner != rank
    halo_nodes = torch.unique(o[remote])                     # sorted, hence grouped by owner
    halo_owner = torch.searchsorted(torch.tensor(cuts[1:], device=dev), halo_nodes, right=True)
    recv_counts = [int((halo_owner == q).sum()) for q in range(world)]
    # local column ids: own rows first, then halo rows in sorted order
    local_o = torch.empty_like(o)
    local_o[~remote] = o[~remote] - lo
    local_o[remote] = (hi - lo) + torch.searchsorted(halo_nodes, o[remote])
    return edge_pos, k, local_o, halo_nodes, recv_counts


def gather_rows(t, idx):
    """x[idx] (mp_gather_rows_f32)."""
    return t[idx]


def sum_returned_rows(plan, back):
    """The returned halo rows summed into the own rows, torch's serial CPU
    index_add_ (the native segmented sum keyed on send_idx)."""
    return torch.zeros((plan.n_own, back.shape[1]), dtype=back.dtype).index_add_(0, plan.send_idx, back)


def segment_sum_in_order(index, values, n):
    """torch's serial CPU scatter_add_ (mp_segment_sum_serial_f32)."""
    return torch.zeros(n, dtype=values.dtype).scatter_add_(0, index, values)


def norm_local(row, col, deg, w):
    """dinv[row] * w * dinv[col], dinv = deg^-1/2 with inf -> 0 (GCNConv.norm,
    PyG 1.4.3; mp_gcn_norm_from_deg_f32)."""
    dinv = deg.pow(-0.5)
    dinv[dinv == float("inf")] = 0
    return dinv[row] * w * dinv[col]


def gat_loops(edge_index, num_nodes):
    """remove_self_loops + add_self_loops (GATConv, PyG 1.4.3; mp_self_loops)."""
    keep = edge_index[0] != edge_index[1]
    loops = torch.arange(int(num_nodes), dtype=edge_index.dtype).view(1, -1).repeat(2, 1)
    return torch.cat([edge_index[:, keep], loops], 1)


def host_step(hc, x_own, aggregate, group=None):
    """One step of a HaloCover on host tensors: aggregate(x_src, src_idx,
    dst_idx, w, n_dst) is the serial edge-order sum (the oracle).  Returns the
    rank's [n_own, F] sum over all its in-edges."""
    from mi355_mp.dist import _a2a
    F = x_own.shape[1]
    send = aggregate(x_own, hc.send_src, hc.send_dst, hc.send_w, hc.n_send)
    xl = x_own.new_empty((hc.n_local_src, F))
    xl[:hc.n_own] = x_own
    _a2a(xl[hc.n_own:], send.contiguous(), hc.recv_counts, hc.send_counts, group)
    out = aggregate(x_own, hc.int_src, hc.int_dst, hc.int_w, hc.n_own)
    return out + aggregate(xl, hc.bnd_src, hc.bnd_dst, hc.bnd_w, hc.n_own)


class _A2A(torch.autograd.Function):
    """Differentiable all_to_all_single of rows: forward send -> recv with the
    given splits, backward the reverse exchange of the gradient."""

    @staticmethod
    def forward(ctx, send, recv_counts, send_counts, group):
        from mi355_mp.dist import _a2a
        ctx.counts, ctx.group = (recv_counts, send_counts), group
        recv = send.new_empty((sum(recv_counts),) + tuple(send.shape[1:]))
        _a2a(recv, send.contiguous(), recv_counts, send_counts, group)
        return recv

    @staticmethod
    def backward(ctx, g):
        from mi355_mp.dist import _a2a
        recv_counts, send_counts = ctx.counts
        gs = g.new_empty((sum(send_counts),) + tuple(g.shape[1:]))
        _a2a(gs, g.contiguous(), send_counts, recv_counts, ctx.group)
        return gs, None, None, None


def gat_cover_forward(self, xw_own, att, H, C, slope=0.2, bias=None):
    """GatHaloCover's step with differentiable torch ops (self: the cover; any
    float dtype): the data flow of forward_device / backward_device that the
    gloo CPU tests hold to the single-process oracle, forward and backward
    (autograd through a differentiable all_to_all).  Returns the rank's rows
    [n_own, H*C] (+ bias)."""
    n_own, F = self.n_own, H * C
    g = self.group
    att2 = att.reshape(H, 2 * C)

    def scores(x):
        x3 = x.view(-1, H, C)
        return (x3 * att2[:, :C]).sum(-1), (x3 * att2[:, C:]).sum(-1)     # a_dst, a_src

    def piece(x_src, a_src, a_dst_rows, src, dst, n_rows):
        """(out = acc / den, m, den) of the softmax over each row's edges."""
        e = torch.nn.functional.leaky_relu(a_src[src] + a_dst_rows[dst], slope)
        m = torch.full((n_rows, H), float("-inf"), dtype=x_src.dtype, device=x_src.device)
        m = m.scatter_reduce(0, dst.view(-1, 1).expand(-1, H), e.detach(), "amax", include_self=True)
        p = torch.exp(e - m[dst])
        den = torch.zeros((n_rows, H), dtype=x_src.dtype, device=x_src.device).index_add(0, dst, p) + 1e-16
        msg = x_src[src].view(-1, H, C) * p.unsqueeze(-1)
        acc = torch.zeros((n_rows, H, C), dtype=x_src.dtype, device=x_src.device).index_add(0, dst, msg)
        return acc / den.unsqueeze(-1), m, den

    a_dst_own, a_src_own = scores(xw_own)
    # 1. a_dst of the rows the peers push pieces of
    adst_in = _A2A.apply(a_dst_own[self.adst_rows], self.adst_recv_counts, self.adst_send_counts, g)
    send_adst = a_dst_own.new_zeros((self.n_send, H)).index_copy(0, self.send_push_rows, adst_in)
    # 2. the send rows and their stats
    s_out, s_m, s_den = piece(xw_own, a_src_own, send_adst, self.send_src, self.send_dst, self.n_send)
    recv = _A2A.apply(s_out.reshape(self.n_send, F), self.recv_counts, self.send_counts, g)
    r_m = _A2A.apply(s_m, self.recv_counts, self.send_counts, g)
    r_den = _A2A.apply(s_den, self.recv_counts, self.send_counts, g)
    # 3. the local piece over [own ; received rows]
    x_loc = torch.cat([xw_own, recv])
    _, a_src_loc = scores(x_loc)
    o, m, den = piece(x_loc, a_src_loc, a_dst_own, self.loc_src, self.loc_dst, n_own)
    # 4. merge: local piece, then the peers' pieces
    pm, pden, po = r_m[self.part_row], r_den[self.part_row], recv[self.part_row].view(-1, H, C)
    M = m.detach().scatter_reduce(0, self.part_dst.view(-1, 1).expand(-1, H), pm.detach(), "amax",
                                  include_self=True)
    w_loc = den * torch.exp(m - M)
    w_p = pden * torch.exp(pm - M[self.part_dst])
    tot = w_loc.index_add(0, self.part_dst, w_p)
    out = o * (w_loc / tot).unsqueeze(-1)
    out = out.index_add(0, self.part_dst, po * (w_p / tot[self.part_dst]).unsqueeze(-1))
    out = out.reshape(n_own, F)
    return out + bias if bias is not None else out


def install():
    """Install these twins in this process's mi355_mp.dist."""
    from mi355_mp import dist as mdist
    mdist.install_host_twins(sys.modules[__name__])
