"""Torch-facing ops over the native engine (autograd included).

Every function here launches HIP kernels from libmi355_mp.so on the current
stream; inputs must already live on the GPU.  Backward passes reuse the same
kernels on the transposed CSR.

Reference semantics (all [U], restated from torch_scatter 2.0.4 /
torch_geometric 1.4.3; see oracle/ for the CPU restatement used as checker):
  * sum/add   : scatter_sum = zeros(...).scatter_add_(0, index, src)
  * mean      : scatter_sum / count.clamp(1)
  * max/min   : (out, arg); strict compare, first edge wins ties, empty row
                -> (0, src.size(0)); scatter_(...) also masks <-10000 / >10000
"""
import os

import torch

from . import _lib
from .graph import _Cache, csr_for_index, in_csr_order

_REDUCES = ("sum", "add", "mean", "max", "min")


def _any_2d(x, what):
    """A 2-D row-major tensor of a dtype the native reductions take (fp32 hot
    path; float64 / float16 / bfloat16 / int64 breadth path, mp_segment_reduce)."""
    if x.dtype not in _lib.MP_DTYPE:
        raise TypeError("mi355_mp: %s dtype %s is not supported (float32, float64, float16, bfloat16, int64)"
                        % (what, x.dtype))
    if x.dim() != 2:
        raise ValueError("mi355_mp: %s must be 2-D [rows, features]" % what)
    if x.stride(1) != 1 or x.stride(0) < max(x.shape[1], 1):
        x = x.contiguous()
    return x


def _aggregate_any(csr, gather, src, reduce, flags, out=None):
    """mp_segment_reduce: any supported dtype, every row in edge order (not
    split).  Returns (out, arg_or_None)."""
    lib = _lib.load()
    F = src.shape[1]
    dev = src.device
    if out is None:
        out = torch.empty((csr.n_rows, F), dtype=src.dtype, device=dev)
    arg = torch.empty((csr.n_rows, F), dtype=torch.int64, device=dev) if reduce in ("max", "min") else None
    if csr.n_rows == 0 or F == 0:
        return out, arg
    _lib.check(lib.mp_segment_reduce(csr.struct(gather), _lib.MP_DTYPE[src.dtype], src.data_ptr(), src.stride(0), F,
                                     _lib.MP_REDUCE[reduce], flags, out.data_ptr(), out.stride(0), _lib.ptr(arg),
                                     _lib.stream_ptr(dev)), "mp_segment_reduce")
    return out, arg


def _f32_2d(x, what):
    if x.dtype != torch.float32:
        raise TypeError("mi355_mp: %s must be float32 (got %s)" % (what, x.dtype))
    if x.dim() != 2:
        raise ValueError("mi355_mp: %s must be 2-D [rows, features]" % what)
    if x.stride(1) != 1:
        x = x.contiguous()
    return x


# Unweighted max / min over x[col] read each (row, column) pair once: from the
# (FIRST_OCCURRENCE_AFTER + 1)-th such aggregation over one CSR on, the CSR's
# first-occurrence form (graph.CSR.first_occurrences: bit-identical results,
# no repeated gathers) is built once and used.  A one-off aggregation never
# pays for its sort; a layer reused every epoch does.  None disables it.
FIRST_OCCURRENCE_AFTER = 2


def _max_csr(csr):
    if FIRST_OCCURRENCE_AFTER is None:
        return csr
    n = getattr(csr, "_max_uses", 0) + 1
    csr._max_uses = n
    return csr.first_occurrences() if n > FIRST_OCCURRENCE_AFTER else csr


def _aggregate(csr, gather, x, w_csr, reduce, flags, bias, out=None, stages=_lib.MP_STAGE_ALL, slab=None,
               arg=None):
    """Launch mp_aggregate_f32; returns (out, arg_or_None)."""
    lib = _lib.load()
    if reduce in ("max", "min") and w_csr is None and gather == "other" and stages == _lib.MP_STAGE_ALL:
        csr = _max_csr(csr)
    F = x.shape[1]
    dev = x.device
    if out is None:
        out = torch.empty((csr.n_rows, F), dtype=torch.float32, device=dev)
    is_arg = reduce in ("max", "min")
    if is_arg and arg is None:
        arg = torch.empty((csr.n_rows, F), dtype=torch.int64, device=dev)
    if csr.n_rows == 0 or F == 0:
        return out, arg
    g = csr.struct(gather)
    red = _lib.MP_REDUCE[reduce]
    sb = lib.mp_aggregate_slab_bytes(g, F, red)
    if slab is None or slab.numel() < sb:
        slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    _lib.check(lib.mp_aggregate_f32(g, _lib.ptr(w_csr), x.data_ptr(), x.stride(0), F, red, flags,
                                    _lib.ptr(bias), out.data_ptr(), out.stride(0), _lib.ptr(arg),
                                    slab.data_ptr(), sb, stages, _lib.stream_ptr(dev)),
               "mp_aggregate_f32")
    return out, arg


def aggregate_tiles(csr, gather, x, w_csr, F, out, reduce="sum", flags=0, bias=None, x_tiles=None, out_tiles=None,
                    slab=None, stages=_lib.MP_STAGE_ALL, bias_rows=None):
    """One sum / mean launch (mp_aggregate_tiles_f32) over operands held
    tile-major: x_tiles / out_tiles = (width, stride in elements) when x / out
    is a [T, rows, width] buffer (feature f of row r at
    [f // width][r][f % width]), None when row-major (then x / out is a 2-D
    tensor and its row stride is used).  bias_rows: None, or int32 [rows]
    flags -- the bias goes only to rows whose flag is nonzero.  Bitwise the
    arithmetic of _aggregate on the same values laid out row-major.  Returns
    out."""
    lib = _lib.load()
    dev = out.device
    if csr.n_rows == 0:
        return out
    g = csr.struct(gather)
    red = _lib.MP_REDUCE[reduce]
    sb = lib.mp_aggregate_slab_bytes(g, F, red)
    if slab is None or slab.numel() < sb:
        slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    xw, xs = x_tiles if x_tiles is not None else (0, 0)
    ow, os_ = out_tiles if out_tiles is not None else (0, 0)
    ldx = 0 if x_tiles is not None else x.stride(0)
    ldo = 0 if out_tiles is not None else out.stride(0)
    _lib.check(lib.mp_aggregate_tiles_f32(g, _lib.ptr(w_csr), x.data_ptr() if x.numel() else None, ldx, xw, xs, F, red,
                                          flags, _lib.ptr(bias), _lib.ptr(bias_rows), out.data_ptr(), ldo, ow, os_,
                                          slab.data_ptr(), sb,
                                          stages, _lib.stream_ptr(dev)), "mp_aggregate_tiles_f32")
    return out


def gather_rows(x, idx):
    """out = x[idx] via the native row gather (no autograd; see GatherRows)."""
    lib = _lib.load()
    x = _any_2d(x, "x")
    idx = idx.to(torch.int64).contiguous()
    out = torch.empty((idx.numel(), x.shape[1]), dtype=x.dtype, device=x.device)
    if idx.numel() and x.shape[1]:
        if x.dtype == torch.float32:
            _lib.check(lib.mp_gather_rows_f32(x.data_ptr(), x.stride(0), idx.data_ptr(), idx.numel(),
                                              x.shape[1], out.data_ptr(), out.stride(0),
                                              _lib.stream_ptr(x.device)), "mp_gather_rows_f32")
        else:
            _lib.check(lib.mp_gather_rows_any(x.element_size(), x.data_ptr(), x.stride(0), idx.data_ptr(),
                                              idx.numel(), x.shape[1], out.data_ptr(), out.stride(0),
                                              _lib.stream_ptr(x.device)), "mp_gather_rows_any")
    return out


def col_sums(g):
    """sum over rows of a [n, F] fp32 gradient (a bias gradient): native
    per-block partials (mp_col_sums_f32) where the row fits 256 features,
    else torch's reduction."""
    n, F = g.shape
    if g.is_cuda and 0 < F <= 256 and F % 4 == 0 and g.stride(1) == 1 and g.stride(0) % 4 == 0 \
            and g.data_ptr() % 16 == 0 and g.dtype == torch.float32:
        lib = _lib.load()
        part = torch.empty((int(lib.mp_gat_bwd_blocks(n)), F), dtype=torch.float32, device=g.device)
        _lib.check(lib.mp_col_sums_f32(g.data_ptr(), g.stride(0), n, F, part.data_ptr(), _lib.nbytes(part),
                                       _lib.stream_ptr(g.device)), "mp_col_sums_f32")
        return part.sum(0)
    return g.sum(0)


def arg_backward(graph, arg, g, n_src, edge_weight=None, x=None, want_gx=True, want_gw=False):
    """ScatterMax / ScatterMin backward of the fused message w_e * x[src_e]
    (torch_scatter 2.0.4 [U8]: grad_msg = zeros(E+1, F).scatter_(0, arg, g)[:E],
    then the message's backward and index_select's backward, an index_add_ by
    source in edge order), deterministic and in the reference's order: a winner
    bit mask in the transposed CSR's slot order, then one pass over the
    transposed CSR that adds each source row's winning terms slot by slot
    (mp_scatter_arg_backward_csr_f32) -- no float atomics.  `arg` holds original
    edge ids of graph.dst's edges (E = no edge).  Returns (gx or None, gw or None)."""
    lib = _lib.load()
    dev = g.device
    st = _lib.stream_ptr(dev)
    src = graph.src
    E = src.n_edges
    F = g.shape[1]
    inv = src.inverse_eid()
    W = int(lib.mp_arg_mask_words(F))
    mask = torch.empty(max(E * W, 2), dtype=torch.int32, device=dev)
    _lib.check(lib.mp_arg_winner_mask(arg.data_ptr(), g.shape[0], F, E, inv.data_ptr(), mask.data_ptr(),
                                      _lib.nbytes(mask), st), "mp_arg_winner_mask")
    w = edge_weight.to(torch.float32).contiguous() if edge_weight is not None else None
    gx = gw = None
    if want_gx:
        gx = torch.empty((int(n_src), F), dtype=torch.float32, device=dev)
        _lib.check(lib.mp_scatter_arg_backward_csr_f32(src.struct("other"), mask.data_ptr(), _lib.nbytes(mask),
                                                       g.data_ptr(), g.stride(0), F, _lib.ptr(w), gx.data_ptr(),
                                                       gx.stride(0), st),
                   "mp_scatter_arg_backward_csr_f32")
    if want_gw:
        ei = graph._edge_index()
        srcs = ei[graph.j].contiguous()
        dsts = ei[graph.i].contiguous()
        gw = torch.empty(max(E, 1), dtype=torch.float32, device=dev)[:E]
        _lib.check(lib.mp_scatter_arg_grad_w_f32(srcs.data_ptr(), dsts.data_ptr(), E, inv.data_ptr(), mask.data_ptr(),
                                                 _lib.nbytes(mask), F, g.data_ptr(), g.stride(0), x.data_ptr(),
                                                 x.stride(0),
                                                 gw.data_ptr(), st), "mp_scatter_arg_grad_w_f32")
    return gx, gw


# ---------------------------------------------------------------------------
# fused gather -> weight -> reduce over a Graph (MessagePassing fast path)
# ---------------------------------------------------------------------------

class _FusedPropagate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, edge_weight, bias, graph, edge_index, reduce, pyg_mask, weight_csr):
        csr = graph.dst
        w_csr = weight_csr
        if w_csr is None and edge_weight is not None:
            w_csr = in_csr_order(csr, edge_weight)
        is_arg = reduce in ("max", "min")
        need_mask_grad = is_arg and pyg_mask and ctx.needs_input_grad[0]
        flags = _lib.MP_FLAG_PYG_MASK if (pyg_mask and not need_mask_grad) else 0
        fuse_bias = bias if not need_mask_grad else None
        out, arg = _aggregate(csr, "other", x, w_csr, reduce, flags, fuse_bias)
        keep = None
        if need_mask_grad:
            keep = ~((out < -10000) if reduce == "max" else (out > 10000))
            out = out.masked_fill(~keep, 0.0)
            if bias is not None:
                out = out + bias
        ctx.graph = graph
        ctx.reduce = reduce
        ctx.n_src = x.shape[0]
        ctx.save_for_backward(x, edge_weight, edge_index, arg, keep)
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, edge_weight, edge_index, arg, keep = ctx.saved_tensors
        graph, reduce = ctx.graph, ctx.reduce
        grad_out = grad_out.contiguous()
        gx = gw = gb = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = col_sums(grad_out)
        if reduce in ("max", "min"):
            want_w = ctx.needs_input_grad[1] and edge_weight is not None
            if ctx.needs_input_grad[0] or want_w:
                # message = w_e * x[src_e] at the argmax edge e: d x[src_e] += w_e g,
                # d w_e += <g, x[src_e]> over the features whose argmax is e
                g = (grad_out * keep if keep is not None else grad_out).contiguous()
                gx, gw = arg_backward(graph, arg, g, ctx.n_src, edge_weight, x, ctx.needs_input_grad[0], want_w)
                if gw is not None and gw.dtype != edge_weight.dtype:
                    gw = gw.to(edge_weight.dtype)
            return gx, gw, gb, None, None, None, None, None
        g = grad_out
        if reduce == "mean":
            deg = graph.dst.degree().clamp(min=1).to(torch.float32)
            g = g / deg.view(-1, 1)
        if ctx.needs_input_grad[0]:
            src = graph.src  # transposed CSR: rows = source nodes, gathers destination rows
            w_src = in_csr_order(src, edge_weight) if edge_weight is not None else None
            gx, _ = _aggregate(src, "other", g, w_src, "sum", 0, None)
        if ctx.needs_input_grad[1] and edge_weight is not None:
            gw = _edge_dot(graph.dst, g.contiguous(), x).to(edge_weight.dtype)
        return gx, gw, gb, None, None, None, None, None


def _edge_dot(csr, g, x):
    """d w_e = <g[dst_e], x[src_e]> for every edge, in original edge order: one
    CSR SDDMM over the destination CSR (mp_gat_sddmm_f32 with one head of width
    F), then a permutation by eid -- no [E, F] gathers of x_j and g_i."""
    E = csr.n_edges
    F = g.shape[1]
    dev = g.device
    out = torch.zeros(E, dtype=torch.float32, device=dev)
    if E == 0 or F == 0:
        return out
    sr = csr.slot_rows()
    d = torch.empty(E, dtype=torch.float32, device=dev)
    _lib.check(_lib.load().mp_gat_sddmm_f32(csr.struct("other"), sr.data_ptr(), g.data_ptr(), g.stride(0),
                                            x.data_ptr(), x.stride(0), 1, F, d.data_ptr(), _lib.stream_ptr(dev)),
               "mp_gat_sddmm_f32")
    out[csr.eid[:E].long()] = d
    return out


def fused_propagate(graph, x, edge_index, edge_weight=None, reduce="sum", bias=None, pyg_mask=False,
                    weight_csr=None):
    """out[i] = REDUCE_{e : index[e] == i} (w[e] * x[other[e]]) (+ bias).

    The fused form of ``propagate`` for message(x_j) / message(x_j, norm)
    (PyG 1.4.3 MessagePassing [U1] + GCNConv.message [U5]).
    """
    if reduce not in _REDUCES:
        raise ValueError("unknown reduce %r" % (reduce,))
    reduce = "sum" if reduce == "add" else reduce
    _lib.require_device(x, edge_index, edge_weight, bias)
    x = _f32_2d(x, "x")
    return _FusedPropagate.apply(x, edge_weight, bias, graph, edge_index, reduce, pyg_mask, weight_csr)


# ---------------------------------------------------------------------------
# materialised-message path (torch_scatter semantics)
# ---------------------------------------------------------------------------

class _SegmentReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, index, dim_size, reduce, pyg_mask):
        csr = csr_for_index(index, dim_size)
        need_mask_grad = pyg_mask and reduce in ("max", "min") and ctx.needs_input_grad[0]
        flags = _lib.MP_FLAG_PYG_MASK if (pyg_mask and not need_mask_grad) else 0
        if src.dtype == torch.float32:
            out, arg = _aggregate(csr, "eid", src, None, reduce, flags, None)
        else:
            out, arg = _aggregate_any(csr, "eid", src, reduce, flags)
        ctx.reduce = reduce
        ctx.csr = csr
        ctx.n_src = src.shape[0]
        keep = None
        if need_mask_grad:
            keep = ~((out < -10000) if reduce == "max" else (out > 10000))
            out = out.masked_fill(~keep, 0.0)
        ctx.save_for_backward(index, arg, keep)
        if arg is not None:
            ctx.mark_non_differentiable(arg)
        return out, arg

    @staticmethod
    def backward(ctx, grad_out, _grad_arg=None):
        index, arg, keep = ctx.saved_tensors
        grad_out = grad_out.contiguous()
        reduce = ctx.reduce
        if reduce in ("max", "min"):
            lib = _lib.load()
            g = (grad_out * keep if keep is not None else grad_out).contiguous()
            gs = torch.zeros((ctx.n_src, g.shape[1]), dtype=g.dtype, device=g.device)
            if g.dtype == torch.float32:
                _lib.check(lib.mp_scatter_arg_backward_f32(g.data_ptr(), arg.data_ptr(), g.shape[0], g.shape[1],
                                                           ctx.n_src, gs.data_ptr(), gs.stride(0),
                                                           _lib.stream_ptr(g.device)), "mp_scatter_arg_backward_f32")
            else:
                _lib.check(lib.mp_scatter_arg_any(g.element_size(), g.data_ptr(), arg.data_ptr(), g.shape[0],
                                                  g.shape[1], ctx.n_src, gs.data_ptr(), gs.stride(0),
                                                  _lib.stream_ptr(g.device)), "mp_scatter_arg_any")
            return gs, None, None, None, None
        g = grad_out
        if reduce == "mean":
            g = g / ctx.csr.degree().clamp(min=1).to(g.dtype).view(-1, 1)
        return gather_rows(g, index), None, None, None, None


def segment_reduce(src, index, dim_size, reduce="sum", pyg_mask=False):
    """torch_scatter.scatter_{sum,mean,max,min}(src, index, 0, dim_size=...) on 2-D src.

    Returns (out, arg) with arg None for sum/mean.
    """
    if reduce not in _REDUCES:
        raise ValueError("unknown reduce %r" % (reduce,))
    reduce = "sum" if reduce == "add" else reduce
    _lib.require_device(src, index)
    src = _any_2d(src, "src")
    if index.dim() != 1 or index.numel() != src.shape[0]:
        raise ValueError("mi355_mp: index must be 1-D with src.size(0) entries")
    return _SegmentReduce.apply(src, index, int(dim_size), reduce, pyg_mask)


def _reduce_into_native(src, index, out, reduce):
    csr = csr_for_index(index, out.shape[0])
    if src.dtype == torch.float32:
        res, arg = _aggregate(csr, "eid", src, None, reduce, _lib.MP_FLAG_INIT_FROM_OUT, None, out=out)
    else:
        res, arg = _aggregate_any(csr, "eid", src, reduce, _lib.MP_FLAG_INIT_FROM_OUT, out=out)
    return res, arg, csr


class _SegmentReduceInto(torch.autograd.Function):
    """torch_scatter 2.0.4's ``out=`` forms with autograd, as upstream
    differentiates them: scatter_sum is ``out.scatter_add_(dim, index, src)``
    (d src = gather(g), d out = g), scatter_mean divides that by the clamped
    count in place (d src = gather(g / count), d out = g / count), and the
    C++ ScatterMax / ScatterMin give src its winners' gradients and out none.
    Out of place here (the result a fresh tensor); segment_reduce_into copies
    it into the caller's out."""

    @staticmethod
    def forward(ctx, src, index, out_old, reduce):
        res = out_old.clone(memory_format=torch.contiguous_format)
        res, arg, csr = _reduce_into_native(src, index, res, reduce)
        ctx.reduce, ctx.csr, ctx.n_src = reduce, csr, src.shape[0]
        ctx.save_for_backward(index, arg)
        if arg is not None:
            ctx.mark_non_differentiable(arg)
        return res, arg

    @staticmethod
    def backward(ctx, g, _grad_arg=None):
        index, arg = ctx.saved_tensors
        g = g.contiguous()
        if ctx.reduce in ("max", "min"):
            lib = _lib.load()
            gs = torch.zeros((ctx.n_src, g.shape[1]), dtype=g.dtype, device=g.device)
            if g.dtype == torch.float32:
                _lib.check(lib.mp_scatter_arg_backward_f32(g.data_ptr(), arg.data_ptr(), g.shape[0], g.shape[1],
                                                           ctx.n_src, gs.data_ptr(), gs.stride(0),
                                                           _lib.stream_ptr(g.device)), "mp_scatter_arg_backward_f32")
            else:
                _lib.check(lib.mp_scatter_arg_any(g.element_size(), g.data_ptr(), arg.data_ptr(), g.shape[0],
                                                  g.shape[1], ctx.n_src, gs.data_ptr(), gs.stride(0),
                                                  _lib.stream_ptr(g.device)), "mp_scatter_arg_any")
            return gs, None, None, None
        if ctx.reduce == "mean":
            g = g / ctx.csr.degree().clamp(min=1).to(g.dtype).view(-1, 1)
        return gather_rows(g, index), None, g, None


def segment_reduce_into(src, index, out, reduce="sum"):
    """torch_scatter ``out=`` semantics: reduce into (and return) the given out
    tensor; differentiable in src and out as upstream (_SegmentReduceInto)."""
    reduce = "sum" if reduce == "add" else reduce
    _lib.require_device(src, index, out)
    src = _any_2d(src, "src")
    # (a one-feature out may carry any stride on its size-1 dim: torch calls it contiguous)
    if out.dtype != src.dtype or out.dim() != 2 or (out.shape[1] > 1 and out.stride(1) != 1):
        raise ValueError("mi355_mp: out must be a row-major [dim_size, F] tensor of src's dtype")
    if torch.is_grad_enabled() and (src.requires_grad or out.requires_grad):
        res, arg = _SegmentReduceInto.apply(src, index, out, reduce)
        out.copy_(res)
        return out, arg
    res, arg, _ = _reduce_into_native(src, index, out, reduce)
    return res, arg


class GatherRows(torch.autograd.Function):
    """x[idx] with backward = segment-sum of the row gradients by idx (native)."""

    @staticmethod
    def forward(ctx, x, idx):
        ctx.n = x.shape[0]
        ctx.save_for_backward(idx)
        return gather_rows(x, idx)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        csr = csr_for_index(idx, ctx.n)
        g = g.contiguous()
        if g.dtype == torch.float32:
            gx, _ = _aggregate(csr, "eid", g, None, "sum", 0, None)
        else:
            gx, _ = _aggregate_any(csr, "eid", g, "sum", 0)
        return gx, None


_range_cache = _Cache()


def index_range(idx):
    """(min, max) of an index tensor: one aminmax and one host read the first
    time, then cached on the tensor (identity + version counter + data pointer,
    dropped with it -- graph._Cache), so the per-forward checks of a reused
    edge_index cost a dictionary lookup, not a device sync.

    Limitation (the same contract as the per-edge_index CSR cache, graph_for):
    a write that does not bump the version counter -- through ``.data``, a
    DLPack / from_blob alias, or a raw-pointer kernel -- is not seen.  After such
    a write call forget_index(idx) (or mutate through ordinary in-place ops)."""
    def compute():
        mn, mx = torch.aminmax(idx)
        return tuple(torch.stack([mn, mx]).tolist())
    return _range_cache.get(idx, ("range", idx.data_ptr()), compute)


def forget_index(idx):
    """Drop every cached fact about idx (its range and CSR graphs): for index
    tensors written behind autograd's back (see index_range)."""
    from .graph import _graph_cache, _index_cache
    base = idx._base if idx._base is not None else idx
    for c in (_range_cache, _graph_cache, _index_cache):
        c._drop(id(base))


def check_row_index(idx, n, what="index_select"):
    """IndexError when an index falls outside [0, n), as x.index_select(0, idx)
    raises on the CPU (the native row gather reads whatever row it is given, so
    a bad index must never reach it).  The range is cached per index tensor
    (index_range); skipped while a HIP graph is being captured (the captured
    call was checked when it ran eagerly before capture, and a capture cannot
    read values back)."""
    if idx.numel() == 0 or (idx.is_cuda and torch.cuda.is_current_stream_capturing()):
        return
    lo, hi = index_range(idx)
    if lo < 0 or hi >= n:
        raise IndexError("%s: index %d out of range for %d rows" % (what, lo if lo < 0 else hi, n))


def index_select_rows(x, idx):
    """Differentiable native replacement of x.index_select(0, idx) for 2-D x
    (fp32 / fp64 / fp16 / bf16 / int64); an index outside [0, x.size(0))
    raises IndexError (check_row_index)."""
    _lib.require_device(x, idx)
    x = _any_2d(x, "x")
    check_row_index(idx, x.shape[0])
    return GatherRows.apply(x, idx)


# ---------------------------------------------------------------------------
# self-loop rewrites (PyG 1.4.3 utils.loop [U4])
# ---------------------------------------------------------------------------

_LOOP_MODES = {"remove": _lib.MP_LOOPS_REMOVE, "add": _lib.MP_LOOPS_ADD,
               "add_remaining": _lib.MP_LOOPS_ADD_REMAINING}


def self_loops(edge_index, num_nodes, mode):
    """Native loop rewrite of a [2, E] int64 device edge_index (mp_self_loops).

    Returns (edge_index_out, pos): the kept edges in original order, then (for
    'add' / 'add_remaining') the loops 0..N-1; pos[k] = input position whose
    weight output edge k carries (-1: fill value).  One host sync reads the
    number of self loops (the output size), like upstream's boolean-mask
    indexing."""
    _lib.require_device(edge_index)
    lib = _lib.load()
    dev = edge_index.device
    st = _lib.stream_ptr(dev)
    N = int(num_nodes)
    E = int(edge_index.shape[1])
    row = edge_index[0].to(torch.int64).contiguous()
    col = edge_index[1].to(torch.int64).contiguous()
    m = _LOOP_MODES[mode]
    n_kept = E
    if m != _lib.MP_LOOPS_ADD and E:
        cnt = torch.empty(2, dtype=torch.int64, device=dev)
        _lib.check(lib.mp_self_loop_count(row.data_ptr(), col.data_ptr(), E, N, cnt.data_ptr(), st),
                   "mp_self_loop_count")
        n_loops, n_bad = cnt.tolist()
        if n_bad and m == _lib.MP_LOOPS_ADD_REMAINING:
            # upstream: loop_weight[row[inv_mask]] = ... raises for these
            raise IndexError("mi355_mp: %d self loops name a node outside [0, %d)" % (n_bad, N))
        n_kept = E - n_loops
    n_out = n_kept + (0 if m == _lib.MP_LOOPS_REMOVE else N)
    out = torch.empty((2, n_out), dtype=torch.int64, device=dev)
    pos = torch.empty(max(n_out, 1), dtype=torch.int64, device=dev)
    wsb = lib.mp_self_loops_workspace(E, N)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    _lib.check(lib.mp_self_loops(row.data_ptr(), col.data_ptr(), E, N, m, n_kept, out[0].data_ptr(),
                                 out[1].data_ptr(), pos.data_ptr(), ws.data_ptr(), wsb, st), "mp_self_loops")
    return out, pos[:n_out]


class _GatherFill(torch.autograd.Function):
    """out[k] = w[pos[k]] if pos[k] >= 0 else fill (native); every input
    position appears at most once in pos, so the backward is a plain scatter."""

    @staticmethod
    def forward(ctx, w, pos, fill):
        ctx.n = w.shape[0]
        ctx.save_for_backward(pos)
        out = torch.empty(pos.shape[0], dtype=torch.float32, device=w.device)
        _lib.check(_lib.load().mp_gather_fill_f32(w.data_ptr(), pos.data_ptr(), pos.shape[0], float(fill),
                                                  out.data_ptr(), _lib.stream_ptr(w.device)), "mp_gather_fill_f32")
        return out

    @staticmethod
    def backward(ctx, g):
        (pos,) = ctx.saved_tensors
        keep = pos >= 0
        gw = torch.zeros(ctx.n, dtype=g.dtype, device=g.device)
        gw[pos[keep]] = g[keep]
        return gw, None, None


def gather_fill(w, pos, fill):
    """Per-edge weights of a loop rewrite: w[pos] with `fill` where pos < 0."""
    _lib.require_device(w, pos)
    if w.dtype != torch.float32:
        v = w[pos.clamp(min=0)]
        return torch.where(pos >= 0, v, torch.full_like(v, fill))
    return _GatherFill.apply(w.contiguous(), pos, fill)


# ---------------------------------------------------------------------------
# GCN normalisation (GCNConv.norm [U5])
# ---------------------------------------------------------------------------

def segment_sum_serial(csr, values, out=None):
    """out[r] = sum over the slots of row r, in slot order, of values[eid[k]]
    (mp_segment_sum_serial_f32): a 1-D scatter_add_ in the reference's edge
    order, bit for bit (csr keyed on the scatter index; values in original
    edge order, fp32)."""
    _lib.require_device(values)
    v = values.to(torch.float32).contiguous()
    if out is None:
        out = torch.empty(max(csr.n_rows, 1), dtype=torch.float32, device=v.device)[:csr.n_rows]
    _lib.check(_lib.load().mp_segment_sum_serial_f32(csr.rowptr.data_ptr(), csr.eid.data_ptr(), v.data_ptr(),
                                                     csr.n_rows, out.data_ptr(), _lib.stream_ptr(v.device)),
               "mp_segment_sum_serial_f32")
    return out


def norm_from_degree(row, col, deg, edge_weight, trusted=False):
    """dinv = deg^-1/2 (inf -> 0, torch's CPU pow(-0.5) rounding), then
    dinv[row] * w * dinv[col] (mp_gcn_norm_from_deg_f32).  deg is consumed.
    The kernel reads deg[row[e]] and deg[col[e]]: an id outside [0, deg.numel())
    raises IndexError first, as the reference's deg_inv_sqrt[row] / [col] does.
    trusted=True (ids the caller built in range, e.g. a shard plan's local
    edges): no range check, so no host read-back."""
    _lib.require_device(row, col, deg, edge_weight)
    if not trusted:
        check_row_index(row, deg.numel(), "gcn_norm (row)")
        check_row_index(col, deg.numel(), "gcn_norm (col)")
    E = row.numel()
    w = edge_weight.to(torch.float32).contiguous() if edge_weight is not None else None
    norm = torch.empty(E, dtype=torch.float32, device=row.device)
    d = deg.to(torch.float32).contiguous()
    row, col = row.contiguous(), col.contiguous()  # named: a temporary copy could be freed before the launch
    _lib.check(_lib.load().mp_gcn_norm_from_deg_f32(row.data_ptr(), col.data_ptr(),
                                                    _lib.ptr(w), E, d.numel(), d.data_ptr(), norm.data_ptr(),
                                                    _lib.stream_ptr(row.device)), "mp_gcn_norm_from_deg_f32")
    return norm


def gcn_norm_weights(edge_index, num_nodes, edge_weight=None, integer_weights=False):
    """norm[e] = deg^-1/2[row] * w[e] * deg^-1/2[col], deg = scatter_add(w, row).

    edge_index must already carry the self loops (add_remaining_self_loops).
    integer_weights: the caller guarantees integer-valued weights (GCNConv's
    structure-only norm: ones and the loop fill 1 / 2): the degree is then
    exact in any order and mp_gcn_norm_f32 sums it with atomics.  Otherwise the
    degree is the transposed CSR's serial segment sum
    (mp_segment_sum_serial_f32): the reference's edge-order sum bit for bit,
    deterministic; that CSR is the one the layer's backward uses anyway.
    """
    _lib.require_device(edge_index, edge_weight)
    lib = _lib.load()
    E = edge_index.shape[1]
    N = int(num_nodes)
    # the degree kernel adds at deg[row[e]]: a node id outside [0, N) raises
    # here, as the reference's scatter_add(edge_weight, row, dim_size=N) does
    check_row_index(edge_index, N, "gcn_norm")
    dev = edge_index.device
    st = _lib.stream_ptr(dev)
    row = edge_index[0].contiguous()
    col = edge_index[1].contiguous()
    w = edge_weight.to(torch.float32).contiguous() if edge_weight is not None else None
    deg = torch.empty(max(N, 1), dtype=torch.float32, device=dev)
    norm = torch.empty(E, dtype=torch.float32, device=dev)
    if w is None or integer_weights or E == 0:
        _lib.check(lib.mp_gcn_norm_f32(row.data_ptr(), col.data_ptr(), _lib.ptr(w), E, N,
                                       deg.data_ptr(), norm.data_ptr(), st), "mp_gcn_norm_f32")
        return norm
    from .graph import graph_for
    rows = graph_for(edge_index, N, N, "source_to_target").src   # CSR keyed on edge_index[0]
    segment_sum_serial(rows, w, out=deg[:N])
    _lib.check(lib.mp_gcn_norm_from_deg_f32(row.data_ptr(), col.data_ptr(), w.data_ptr(), E, N, deg.data_ptr(),
                                            norm.data_ptr(), st), "mp_gcn_norm_from_deg_f32")
    return norm


# ---------------------------------------------------------------------------
# GATConv fused attention aggregation (GATConv.message + utils.softmax [U3,U6])
# ---------------------------------------------------------------------------

# GAT forward form.  Default: one online-softmax pass (mp_gat_aggregate_f32).
# GAT_TWO_PASS = True selects mp_gat_softmax_aggregate_f32, which follows the
# reference's operation order (softmax row max, then the denominator summed in
# edge order, then alpha * x_j summed in edge order) at a cost: on config 3 its
# two statistics passes take 3.6 ms and its 64-feature-tile aggregation 10.6 ms
# (one a_src gather per slot per tile), against 8.6 ms for the single pass
# (DESIGN.md section 3.3).
GAT_TWO_PASS = False
# The single pass recomputes a_src[j] from each gathered xw row (bitwise the
# node-score kernel's value) instead of gathering it: mp_gat_aggregate_att_f32.
GAT_OWN_A_SRC = True


def gat_two_pass(csr, H, C):
    return GAT_TWO_PASS and bool(_lib.load().mp_gat_two_pass_ok(H, C))


# Training forward: the fused pass also leaves sum_j alpha leaky' xw_j and
# sum_j alpha leaky' per (row, head) (mp_gat_aggregate_train_f32), which make the
# backward's d a_dst node-wise: no per-edge d score array, no segmented pass.
GAT_TRAIN_FWD = True
# The fused forward computes each row's node scores (a_src, a_dst) from the
# row's own xw (mp_gat_forward_f32 / mp_gat_forward_train_f32, bitwise the
# node-score kernel's values) instead of running mp_gat_node_scores_f32 first.
# Config 3 (inference): main 7.78 ms, no 0.50 ms node-score pass -> 7.85 vs 8.30 ms.
GAT_NODE_SCORES_IN_KERNEL = os.environ.get("MP_GAT_ND", "1") != "0"   # MP_GAT_ND=0: A/B runs
# The training forward with in-kernel scores needs 92 VGPRs (5 waves / SIMD
# instead of 6): GATConv forward + backward 26.49 vs 26.28 ms on config 3, so
# training keeps the separate node-score pass (MP_GAT_ND_TRAIN=1 selects it).
GAT_NODE_SCORES_IN_KERNEL_TRAIN = os.environ.get("MP_GAT_ND_TRAIN", "0") == "1"


def _gat_nd_ok(graph, xw, H, C, bias):
    return (GAT_NODE_SCORES_IN_KERNEL and GAT_OWN_A_SRC and bool(_lib.load().mp_gat_train_ok(H, C))
            and not gat_two_pass(graph.dst, H, C) and xw.data_ptr() % 16 == 0 and graph.n_dst == xw.shape[0]
            and graph.n_src == xw.shape[0] and (bias is None or bias.data_ptr() % 16 == 0))


def _gat_train_fwd_ok(graph, xw, H, C):
    """The training forward (mp_gat_aggregate_train_f32) applies: C % 4 == 0
    (a_src from the gathered rows when C/4 is a power of two <= 64, else from
    the node-score array)."""
    return (GAT_TRAIN_FWD and GAT_OWN_A_SRC and gat_wide_ok(H, C)
            and not gat_two_pass(graph.dst, H, C) and xw.data_ptr() % 16 == 0 and _gat_rows_ok(graph, xw))


def _gat_rows_ok(graph, xw):
    """The fused GAT kernels take a square graph (n_dst == n_src == xw rows) or a
    sharded rank's local graph: n_src == xw rows and destination row i's own xw
    row is row i of xw (the rank's own rows first, then its halo rows:
    mi355_mp.dist.ShardedGraph.gat_propagate), so n_dst <= n_src."""
    return graph.n_src == xw.shape[0] and graph.n_dst <= xw.shape[0]


def _pad_rows(t, n):
    """t [m, ...] -> [n, ...] with zero rows appended (node-wise gradients of the
    destination rows, extended over the halo rows of a sharded local graph)."""
    if t.shape[0] == n:
        return t
    out = t.new_zeros((n,) + tuple(t.shape[1:]))
    out[:t.shape[0]] = t
    return out


def gat_wide_ok(H, C):
    """Heads of any width with C % 4 == 0 (GATConv pads C to it): the fused
    training forward reads a_src from the node-score array when C/4 is not a
    power of two <= 64, and the backward runs the wide form (mp_gat_backward_wide_f32)."""
    return bool(_lib.load().mp_gat_wide_ok(H, C))


def gat_dropout_ok(H, C, p):
    """The fused path carries GATConv's attention dropout (training, 0 < p < 1):
    the training forward and its transposed backward evaluate one hashed keep
    mask per (edge, head) (mp_gat_aggregate_train_drop_f32; the edge's key is
    its id -- the global id on a shard: Graph.drop_ids)."""
    return (0.0 < float(p) < 1.0 and GAT_TRAIN_FWD and GAT_OWN_A_SRC and 1 <= H <= 32 and gat_wide_ok(H, C))


def gat_dropout_keep(graph, seed, p, H):
    """The attention-dropout keep mask [E, H] (bool, the graph's edge order) that
    the fused GAT kernels apply for (seed, p): mp_gat_dropout_keep over the
    destination-CSR slots with their keys (Graph.drop_ids), mapped back through
    the CSR's edge ids."""
    lib = _lib.load()
    csr = graph.dst
    E = csr.n_edges
    dev = csr.rowptr.device
    bits = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
    _lib.check(lib.mp_gat_dropout_keep(int(seed) & 0xFFFFFFFFFFFFFFFF, float(p), int(H), E,
                                       graph.drop_ids("dst").data_ptr(), bits.data_ptr(),
                                       _lib.stream_ptr(dev)), "mp_gat_dropout_keep")
    shifts = torch.arange(H, dtype=torch.int32, device=dev)
    keep_slot = ((bits[:E].unsqueeze(1) >> shifts) & 1).bool()
    keep = torch.empty_like(keep_slot)
    keep[csr.eid[:E].long()] = keep_slot
    return keep


def _gat_forward(graph, edge_index, xw, att, H, C, slope, bias, want_alpha, train2=False, drop=None):
    """Returns (out, alpha, a_src, a_dst, stats, extra).  train2 (callers check
    _gat_train_fwd_ok first): the training forward, out = aggregate + bias and
    extra = (agg2, s2); else extra = None.  No pre-bias copy of the aggregate
    is written: the backward prologues take rs over out - bias (ABI 6).
    drop = (seed, p): attention dropout on the messages (train2 only)."""
    lib = _lib.load()
    dev = xw.device
    N = xw.shape[0]
    csr = graph.dst
    st = _lib.stream_ptr(dev)
    if not _gat_rows_ok(graph, xw):
        raise ValueError("mi355_mp: fused GAT needs n_src == x.size(0) >= n_dst (a square graph, or a sharded "
                         "rank's own rows followed by its halo rows)")
    att_c = att.reshape(H, 2 * C).contiguous().to(torch.float32)
    a_src = torch.empty((N, H), dtype=torch.float32, device=dev)
    a_dst = torch.empty((N, H), dtype=torch.float32, device=dev)
    if drop is not None and not train2:
        raise ValueError("mi355_mp: fused attention dropout runs in the training forward only")
    nd = (_gat_nd_ok(graph, xw, H, C, bias) and (GAT_NODE_SCORES_IN_KERNEL_TRAIN or not train2)
          and drop is None)
    if N and not nd:
        _lib.check(lib.mp_gat_node_scores_f32(xw.data_ptr(), N, H, C, att_c.data_ptr(), a_src.data_ptr(),
                                              a_dst.data_ptr(), st), "mp_gat_node_scores_f32")
    out = torch.empty((graph.n_dst, H * C), dtype=torch.float32, device=dev)
    stats = torch.empty((graph.n_dst, H, 2), dtype=torch.float32, device=dev)
    g = csr.struct("other")
    extra = None
    if train2 and nd:
        agg2 = torch.empty((graph.n_dst, H * C), dtype=torch.float32, device=dev)
        s2 = torch.empty((graph.n_dst, H), dtype=torch.float32, device=dev)
        sb = lib.mp_gat_train_slab_bytes(g, H, C)
        slab = torch.empty(sb, dtype=torch.uint8, device=dev)
        _lib.check(lib.mp_gat_forward_train_f32(g, xw.data_ptr(), att_c.data_ptr(), H, C, float(slope), _lib.ptr(bias),
                                                out.data_ptr(), out.stride(0), None, stats.data_ptr(),
                                                agg2.data_ptr(), s2.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st), "mp_gat_forward_train_f32")
        extra = (agg2, s2)
    elif train2:
        agg2 = torch.empty((graph.n_dst, H * C), dtype=torch.float32, device=dev)
        s2 = torch.empty((graph.n_dst, H), dtype=torch.float32, device=dev)
        sb = lib.mp_gat_train_slab_bytes(g, H, C)
        slab = torch.empty(sb, dtype=torch.uint8, device=dev)
        if drop is not None:
            _lib.check(lib.mp_gat_aggregate_train_drop_f32(g, xw.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                           att_c.data_ptr(), H, C, float(slope), _lib.ptr(bias),
                                                           out.data_ptr(), out.stride(0), None,
                                                           stats.data_ptr(), agg2.data_ptr(), s2.data_ptr(),
                                                           int(drop[0]), float(drop[1]),
                                                           graph.drop_ids("dst").data_ptr(), slab.data_ptr(), sb,
                                                           _lib.MP_STAGE_ALL, st), "mp_gat_aggregate_train_drop_f32")
        else:
            _lib.check(lib.mp_gat_aggregate_train_f32(g, xw.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                      att_c.data_ptr(), H, C, float(slope), _lib.ptr(bias),
                                                      out.data_ptr(), out.stride(0), None, stats.data_ptr(),
                                                      agg2.data_ptr(), s2.data_ptr(), slab.data_ptr(), sb,
                                                      _lib.MP_STAGE_ALL, st), "mp_gat_aggregate_train_f32")
        extra = (agg2, s2)
    if extra is None:
        sb = lib.mp_gat_slab_bytes(g, H, C)
        slab = torch.empty(sb, dtype=torch.uint8, device=dev)
        if nd:
            _lib.check(lib.mp_gat_forward_f32(g, xw.data_ptr(), att_c.data_ptr(), H, C, float(slope), _lib.ptr(bias),
                                              out.data_ptr(), out.stride(0), a_src.data_ptr(), a_dst.data_ptr(),
                                              stats.data_ptr(), slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
                       "mp_gat_forward_f32")
        elif gat_two_pass(csr, H, C):
            _lib.check(lib.mp_gat_softmax_aggregate_f32(g, csr.slot_rows().data_ptr(), xw.data_ptr(), a_src.data_ptr(),
                                                        a_dst.data_ptr(), H, C, float(slope), _lib.ptr(bias),
                                                        out.data_ptr(), out.stride(0), stats.data_ptr(), slab.data_ptr(),
                                                        sb, _lib.MP_STAGE_ALL, st), "mp_gat_softmax_aggregate_f32")
        else:
            _lib.check(lib.mp_gat_aggregate_att_f32(g, xw.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                    att_c.data_ptr() if GAT_OWN_A_SRC else None, H, C, float(slope),
                                                    _lib.ptr(bias), out.data_ptr(), out.stride(0), stats.data_ptr(),
                                                    slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
                       "mp_gat_aggregate_att_f32")
    alpha = None
    if want_alpha:
        E = edge_index.shape[1]
        alpha = torch.empty((E, H), dtype=torch.float32, device=dev)
        src = edge_index[graph.j].contiguous()
        dst = edge_index[graph.i].contiguous()
        _lib.check(lib.mp_gat_alpha_f32(src.data_ptr(), dst.data_ptr(), E, H, a_src.data_ptr(),
                                        a_dst.data_ptr(), float(slope), stats.data_ptr(), alpha.data_ptr(), st),
                   "mp_gat_alpha_f32")
    return out, alpha, a_src, a_dst, stats, extra


def _heads_aggregate(csr, gather, w_slot, H, x):
    """out[r, h*C+c] = sum_k w_slot[k, h] * x[col_k, h*C+c] (mp_aggregate_heads_f32)."""
    lib = _lib.load()
    F = x.shape[1]
    out = torch.empty((csr.n_rows, F), dtype=torch.float32, device=x.device)
    if csr.n_rows == 0:
        return out
    g = csr.struct(gather)
    sb = lib.mp_aggregate_slab_bytes(g, F, 0)
    slab = torch.empty(sb, dtype=torch.uint8, device=x.device)
    _lib.check(lib.mp_aggregate_heads_f32(g, w_slot.data_ptr(), H, x.data_ptr(), x.stride(0), F, out.data_ptr(),
                                          out.stride(0), slab.data_ptr(), sb, _lib.MP_STAGE_ALL,
                                          _lib.stream_ptr(x.device)), "mp_aggregate_heads_f32")
    return out


def _gat_bwd_fused_ok(C):
    """mp_gat_backward_f32 reduces a head's dot product over C/4 (or C) lanes."""
    def pow2(q):
        return 1 <= q <= 64 and (q & (q - 1)) == 0
    return (C % 4 == 0 and pow2(C // 4)) or pow2(C)


def _gat_backward_wide(graph, g, xw, att, a_src, a_dst, stats, agg, agg_bias, extra, H, C, slope, want_att,
                       want_bias, drop=None):
    """GATConv backward for heads of any width (C % 4 == 0), after the training
    forward: prep (pack + node-wise d a_dst), one pass over the transposed CSR
    with no per-slot dot product (mp_gat_backward_wide_f32: sum alpha g_i,
    sum lk alpha g_i, sum lk alpha rs_i per source row), then the node-wise
    epilogue (d a_src = <acc2, xw> - sc, the att terms of d xw).  agg: the
    forward's output, agg_bias the bias inside it (None: none).
    Returns (d xw, d att or None, d bias or None)."""
    lib = _lib.load()
    dev = xw.device
    st = _lib.stream_ptr(dev)
    N = xw.shape[0]
    F = H * C
    att_c = att.reshape(H, 2 * C).contiguous()
    if N == 0:
        return (torch.zeros_like(xw), torch.zeros_like(att) if want_att else None,
                g.new_zeros(F) if want_bias else None)
    agg2, s2 = extra
    n_dst = graph.n_dst            # < N on a sharded rank's local graph (halo rows receive no edges)
    pack = torch.empty((max(n_dst, 1), H, 4), dtype=torch.float32, device=dev)
    ga_dst = (torch.empty if n_dst == N else torch.zeros)((N, H), dtype=torch.float32, device=dev)
    if n_dst:
        _lib.check(lib.mp_gat_backward_prep_wide_f32(g.data_ptr(), g.stride(0), agg.data_ptr(), agg.stride(0),
                                                     _lib.ptr(agg_bias), agg2.data_ptr(), s2.data_ptr(),
                                                     a_dst.data_ptr(), stats.data_ptr(), n_dst, H, C, pack.data_ptr(),
                                                     _lib.nbytes(pack), ga_dst.data_ptr(), st),
                   "mp_gat_backward_prep_wide_f32")
    src = graph.src_with_dst_slots()
    gs = src.struct("dst_slot")
    gx = torch.empty((N, F), dtype=torch.float32, device=dev)
    acc2 = torch.empty((N, F), dtype=torch.float32, device=dev)
    sc = torch.empty((N, H), dtype=torch.float32, device=dev)
    sb = lib.mp_gat_train_slab_bytes(gs, H, C)
    slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    seed, p = (0, 0.0) if drop is None else (int(drop[0]), float(drop[1]))
    ids = graph.drop_ids("src").data_ptr() if drop is not None else None
    _lib.check(lib.mp_gat_backward_wide_f32(gs, g.data_ptr(), g.stride(0), a_src.data_ptr(), pack.data_ptr(), H, C,
                                            float(slope), seed, p, ids, gx.data_ptr(), acc2.data_ptr(),
                                            _lib.nbytes(acc2),
                                            sc.data_ptr(), _lib.nbytes(sc), slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
               "mp_gat_backward_wide_f32")
    del slab, pack
    _lib.check(lib.mp_gat_backward_epilogue_wide_f32(gx.data_ptr(), acc2.data_ptr(), xw.data_ptr(), att_c.data_ptr(),
                                                     ga_dst.data_ptr(), sc.data_ptr(), N, H, C, st),
               "mp_gat_backward_epilogue_wide_f32")
    del acc2
    ga_src = sc
    gatt = None
    if want_att:
        x3 = xw.view(N, H, C)
        gatt = torch.cat([torch.einsum("nh,nhc->hc", ga_dst, x3), torch.einsum("nh,nhc->hc", ga_src, x3)],
                         dim=-1).view_as(att)
    gb = col_sums(g) if want_bias else None
    return gx, gatt, gb


def _att_part_blocks(n_rows, n_dst):
    """Blocks of the d att partials of mp_gat_backward_finish_f32: the pass runs
    over all n_rows rows of xw (own + halo rows on a sharded rank's local graph,
    n_dst of them own), one partial per block of mp_gat_bwd_blocks(n_rows).
    (Round 4 sized this for n_dst: the library now rejects such a buffer --
    ABI 6 extents -- instead of writing past it; tests/test_gpu_dist.py.)"""
    return int(_lib.load().mp_gat_bwd_blocks(n_rows))


def _gat_backward_fused(graph, g, xw, att, a_src, a_dst, stats, agg, agg_bias, H, C, slope, want_att, want_bias,
                        extra=None, drop=None):
    """GATConv backward: prep (packed destination terms + bias-grad partials),
    one gather pass over the transposed CSR (mp_gat_backward_f32), the d a_dst
    row sums over the dst CSR (reading the per-edge d score through the
    src-slot map), and the epilogue (att_dst term + att-grad partials).  agg:
    the forward's output, agg_bias the bias inside it (None: none).
    Returns (d xw, d att or None, d bias or None)."""
    lib = _lib.load()
    dev = xw.device
    st = _lib.stream_ptr(dev)
    N = xw.shape[0]
    F = H * C
    att_c = att.reshape(H, 2 * C).contiguous()
    if N == 0:
        return (torch.zeros_like(xw), torch.zeros_like(att) if want_att else None,
                g.new_zeros(F) if want_bias else None)
    epi = C % 4 == 0 and F <= 256
    n_dst = graph.n_dst            # < N on a sharded rank's local graph (halo rows receive no edges)
    nb = int(lib.mp_gat_bwd_blocks(n_dst))
    pack = torch.empty((max(n_dst, 1), H, 4), dtype=torch.float32, device=dev)
    gpart = torch.empty((nb, F), dtype=torch.float32, device=dev) if (want_bias and epi and n_dst) else None
    ga_dst = None
    if extra is not None:
        # d a_dst[n,h] = <g_n, agg2_n>_h - rs_n,h s2_n,h: node-wise, no per-edge d score
        agg2, s2 = extra
        ga_dst = (torch.empty if n_dst == N else torch.zeros)((N, H), dtype=torch.float32, device=dev)
        if n_dst:
            _lib.check(lib.mp_gat_backward_prep_train_f32(g.data_ptr(), g.stride(0), agg.data_ptr(), agg.stride(0),
                                                          _lib.ptr(agg_bias), agg2.data_ptr(), s2.data_ptr(),
                                                          a_dst.data_ptr(), stats.data_ptr(), n_dst, H, C,
                                                          pack.data_ptr(),
                                                          _lib.nbytes(pack), _lib.ptr(gpart), _lib.nbytes(gpart),
                                                          ga_dst.data_ptr(), st),
                       "mp_gat_backward_prep_train_f32")
    elif n_dst:
        _lib.check(lib.mp_gat_backward_prep_f32(g.data_ptr(), g.stride(0), agg.data_ptr(), agg.stride(0),
                                                _lib.ptr(agg_bias), a_dst.data_ptr(), stats.data_ptr(), n_dst, H, C,
                                                pack.data_ptr(), _lib.nbytes(pack), _lib.ptr(gpart), _lib.nbytes(gpart),
                                                st),
                   "mp_gat_backward_prep_f32")
    gb = None
    if want_bias:
        gb = gpart.sum(0) if gpart is not None else g.sum(0)
    src = graph.src_with_dst_slots()
    E = src.n_edges
    gx = torch.empty((N, F), dtype=torch.float32, device=dev)
    ga_src = torch.empty((N, H), dtype=torch.float32, device=dev)
    # per-edge d score in dst-CSR slot order (only without the training forward's extras)
    de = torch.empty((max(E, 1), H), dtype=torch.float32, device=dev) if ga_dst is None else None
    gs = src.struct("dst_slot")
    sb = lib.mp_gat_slab_bytes(gs, H, C)
    slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    fused_dst = ga_dst is not None
    if drop is not None:
        if not fused_dst:
            raise ValueError("mi355_mp: the attention-dropout backward needs the training forward's extras")
        _lib.check(lib.mp_gat_backward_train_drop_f32(gs, g.data_ptr(), g.stride(0), xw.data_ptr(), a_src.data_ptr(),
                                                      pack.data_ptr(), att_c.data_ptr(), H, C, float(slope),
                                                      ga_dst.data_ptr(), int(drop[0]), float(drop[1]),
                                                      graph.drop_ids("src").data_ptr(), gx.data_ptr(),
                                                      ga_src.data_ptr(), slab.data_ptr(), sb, _lib.MP_STAGE_ALL, st),
                   "mp_gat_backward_train_drop_f32")
    elif fused_dst:
        # the transposed pass also adds d a_dst (x) att_dst to each row's d xw
        _lib.check(lib.mp_gat_backward_train_f32(gs, g.data_ptr(), g.stride(0), xw.data_ptr(), a_src.data_ptr(),
                                                 pack.data_ptr(), att_c.data_ptr(), H, C, float(slope),
                                                 ga_dst.data_ptr(), gx.data_ptr(), ga_src.data_ptr(), slab.data_ptr(),
                                                 sb, _lib.MP_STAGE_ALL, st), "mp_gat_backward_train_f32")
    else:
        _lib.check(lib.mp_gat_backward_f32(gs, g.data_ptr(), g.stride(0), xw.data_ptr(), a_src.data_ptr(),
                                           pack.data_ptr(), att_c.data_ptr(), H, C, float(slope), gx.data_ptr(),
                                           ga_src.data_ptr(), _lib.ptr(de), _lib.nbytes(de), slab.data_ptr(), sb,
                                           _lib.MP_STAGE_ALL, st), "mp_gat_backward_f32")
    del slab, pack
    if ga_dst is None:
        ga_dst, _ = _aggregate(graph.dst, "slot", de, None, "sum", 0, None)
        ga_dst = _pad_rows(ga_dst, N)
        del de
    gatt = None
    if epi:
        if want_att or not fused_dst:
            # att_dst term of d xw (unless the transposed pass added it) + d att partials:
            # the finish pass runs over all N rows (own + halo on a sharded rank's
            # local graph), one partial per block of mp_gat_bwd_blocks(N)
            apart = torch.empty((_att_part_blocks(N, n_dst), 2, F), dtype=torch.float32, device=dev)
            _lib.check(lib.mp_gat_backward_finish_f32(None if fused_dst else gx.data_ptr(), xw.data_ptr(),
                                                      ga_dst.data_ptr(), ga_src.data_ptr(), att_c.data_ptr(), N, H, C,
                                                      apart.data_ptr(), _lib.nbytes(apart), st),
                       "mp_gat_backward_finish_f32")
        if want_att:
            p = apart.sum(0).view(2, H, C)
            gatt = torch.cat([p[0], p[1]], dim=-1).view_as(att)
    else:
        if not fused_dst:
            _lib.check(lib.mp_heads_outer_add_f32(gx.data_ptr(), gx.stride(0), ga_dst.data_ptr(), N, H, C,
                                                  att_c.data_ptr(), 2 * C, st), "mp_heads_outer_add_f32")
        if want_att:
            x3 = xw.view(N, H, C)
            gatt = torch.cat([torch.einsum("nh,nhc->hc", ga_dst, x3), torch.einsum("nh,nhc->hc", ga_src, x3)],
                             dim=-1).view_as(att)
    return gx, gatt, gb


class _GatPropagate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xw, att, bias, graph, edge_index, H, C, slope, want_alpha, train, drop=None):
        # attention dropout (drop = (seed, p)) runs in the training forward, with
        # or without a backward to follow (training mode under no_grad)
        wide = not _gat_bwd_fused_ok(C) and gat_wide_ok(H, C)
        fused = (train or drop is not None) and (_gat_bwd_fused_ok(C) or wide)
        # the fused backward's rs_i = <g_i, agg_i> comes from the saved output
        # (agg + bias, bias fused into the forward) and the bias: the prologue
        # takes rs over out - bias, so no pre-bias copy is written (ABI 6).  The
        # output is saved, so an in-place change of it before backward raises
        # torch's usual "modified by an inplace operation" error.
        train2 = fused and _gat_train_fwd_ok(graph, xw, H, C)
        if wide and fused and not train2:
            fused = False  # the wide backward needs the training forward's extras
        if drop is not None and not train2:
            raise ValueError("mi355_mp: fused attention dropout needs the training forward (gat_dropout_ok)")
        out, alpha, a_src, a_dst, stats, extra = _gat_forward(graph, edge_index, xw, att, H, C, slope, bias,
                                                              want_alpha, train2=train2, drop=drop)
        ctx.graph, ctx.H, ctx.C, ctx.slope, ctx.drop = graph, H, C, slope, drop
        ctx.wide = wide
        ctx.has_bias = bias is not None
        ctx.fused = fused
        ctx.has_extra = extra is not None
        ctx.save_for_backward(xw, att, edge_index, a_src, a_dst, stats, out if fused else None,
                              bias if fused else None, *(extra if extra is not None else ()))
        if alpha is not None:
            ctx.mark_non_differentiable(alpha)
        return out, alpha

    @staticmethod
    def backward(ctx, grad_out, _ga=None):
        """Native GAT backward over the two CSRs of the graph:
          dx_j   = sum_i alpha_ij g_i          (per-head weighted transposed aggregation)
          dalpha = <g_i, xw_j> per head        (CSR SDDMM)
          ds     = alpha (dalpha - sum_row alpha dalpha)   (softmax backward)
          de     = ds * leaky'(s);  d a_dst = row sums, d a_src = column sums of de
          dxw   += d a_src (x) att_src + d a_dst (x) att_dst;  d att = sum_n d a (x) xw
        Only [E, H]-sized arrays are materialised, never [E, H*C]."""
        lib = _lib.load()
        xw, att, edge_index, a_src, a_dst, stats, agg, agg_bias = ctx.saved_tensors[:8]
        extra = tuple(ctx.saved_tensors[8:10]) if ctx.has_extra else None
        graph, H, C, slope = ctx.graph, ctx.H, ctx.C, ctx.slope
        dev = xw.device
        st = _lib.stream_ptr(dev)
        g = grad_out.contiguous()
        if g.data_ptr() % 16:
            g = g.clone()  # a view at an odd offset: the 4-wide transposed pass (the dropout form has no other) needs 16-B rows
        N = xw.shape[0]
        if ctx.fused and ctx.wide:
            gx, gatt, gb = _gat_backward_wide(graph, g, xw, att, a_src, a_dst, stats, agg, agg_bias, extra, H, C,
                                              slope, ctx.needs_input_grad[1], ctx.has_bias and ctx.needs_input_grad[2],
                                              ctx.drop)
            return gx, gatt, gb, None, None, None, None, None, None, None, None
        if ctx.fused:
            gx, gatt, gb = _gat_backward_fused(graph, g, xw, att, a_src, a_dst, stats, agg, agg_bias, H, C, slope,
                                               ctx.needs_input_grad[1], ctx.has_bias and ctx.needs_input_grad[2],
                                               extra, ctx.drop)
            return gx, gatt, gb, None, None, None, None, None, None, None, None
        gb = col_sums(g) if ctx.has_bias and ctx.needs_input_grad[2] else None
        dst, src = graph.dst, graph.src
        E = dst.n_edges
        sr = dst.slot_rows()
        alpha = torch.empty((max(E, 1), H), dtype=torch.float32, device=dev)
        score = torch.empty_like(alpha)
        _lib.check(lib.mp_gat_alpha_csr_f32(dst.struct("other"), sr.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                            H, float(slope), stats.data_ptr(), alpha.data_ptr(), score.data_ptr(),
                                            st), "mp_gat_alpha_csr_f32")
        eid_d = dst.eid[:E].long()
        # message part of d xw: alpha in the transposed CSR's slot order
        alpha_orig = torch.empty_like(alpha)
        alpha_orig[eid_d] = alpha
        alpha_src = alpha_orig[src.eid[:E].long()].contiguous()
        gx = _heads_aggregate(src, "other", alpha_src, H, g)
        # d alpha (CSR order) and the softmax backward
        dalpha = torch.empty_like(alpha)
        _lib.check(lib.mp_gat_sddmm_f32(dst.struct("other"), sr.data_ptr(), g.data_ptr(), g.stride(0), xw.data_ptr(),
                                        xw.stride(0), H, C, dalpha.data_ptr(), st), "mp_gat_sddmm_f32")
        t = (alpha * dalpha)[:E].contiguous()
        rs, _ = _aggregate(dst, "slot", t, None, "sum", 0, None)             # sum over each row's slots
        ds = alpha[:E] * (dalpha[:E] - rs[sr[:E].long()])
        de = (ds * torch.where(score[:E] > 0, torch.ones_like(ds), torch.full_like(ds, slope))).contiguous()
        ga_dst, _ = _aggregate(dst, "slot", de, None, "sum", 0, None)
        ga_dst = _pad_rows(ga_dst, N)
        de_orig = torch.empty_like(de)
        de_orig[eid_d] = de
        ga_src, _ = _aggregate(src, "eid", de_orig, None, "sum", 0, None)
        att3 = att.reshape(H, 2 * C)
        x3 = xw.view(N, H, C)
        gx = gx.view(N, H, C) + ga_src.unsqueeze(-1) * att3[:, C:].unsqueeze(0) \
            + ga_dst.unsqueeze(-1) * att3[:, :C].unsqueeze(0)
        gatt = None
        if ctx.needs_input_grad[1]:
            gd = torch.einsum("nh,nhc->hc", ga_dst, x3)
            gs = torch.einsum("nh,nhc->hc", ga_src, x3)
            gatt = torch.cat([gd, gs], dim=-1).view_as(att)
        return gx.reshape(N, H * C), gatt, gb, None, None, None, None, None, None, None, None


_MASK64 = 0xFFFFFFFFFFFFFFFF
_seed_calls = {}


def _mix64(z):
    """splitmix64 finaliser: spreads (seed, offset) pairs over the 64-bit keys."""
    z = (z + 0x9E3779B97F4A7C15) & _MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    return z ^ (z >> 31)


def dropout_seed(device):
    """A fresh attention-dropout key from the device's default generator, with
    no device read: (its seed, its Philox offset) mixed on the host, and the
    offset advanced, as a device dropout mask draw advances it -- so
    torch.cuda.manual_seed(s) makes the key sequence repeat, the CPU generator
    stays untouched, and nothing blocks on the device (a training step of every
    sharded rank issues no sync for it).  During HIP-graph capture, or on a
    generator without offsets, a host counter per (device, seed) replaces the
    offset (the captured replay reuses the captured key, as any captured
    constant)."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    gen = torch.cuda.default_generators[idx]
    base = gen.initial_seed()
    if not torch.cuda.is_current_stream_capturing() and hasattr(gen, "get_offset"):
        try:
            off = gen.get_offset()
            gen.set_offset(off + 4)
            return _mix64(_mix64(base) ^ off)
        except RuntimeError:
            pass
    k = (idx, base)
    n = _seed_calls.get(k, 0)
    _seed_calls[k] = n + 1
    return _mix64(_mix64(base ^ 0x5EED) ^ n)


def gat_propagate(graph, edge_index, xw, att, heads, out_channels, negative_slope=0.2, bias=None,
                  return_alpha=False, dropout=0.0, seed=None):
    """Fused GATConv aggregation: returns (out [N, H*C], alpha [E, H] or None).
    dropout > 0: GATConv's training-mode attention dropout on the messages
    (callers check gat_dropout_ok); the keep mask is a hash of (seed, slot, head),
    seed drawn from the device's default generator unless given
    (gat_dropout_keep returns the mask).  alpha is the undropped softmax, as upstream's."""
    _lib.require_device(xw, edge_index, att, bias)
    xw = _f32_2d(xw, "x@W").contiguous()
    H, C = int(heads), int(out_channels)
    if xw.shape[0] == 0:
        # no nodes (hence no edges): an empty output, still connected to xw / bias
        # for autograd -- the kernels are not launched
        out = xw * 0.0 if bias is None else xw * 0.0 + bias
        return out, (xw.new_zeros((edge_index.shape[1], H)) if return_alpha else None)
    drop = None
    if dropout > 0:
        if not (gat_dropout_ok(H, C, dropout) and _gat_train_fwd_ok(graph, xw, H, C)):
            raise ValueError("mi355_mp: fused attention dropout needs 0 < p < 1, H <= 32, C %% 4 == 0 and C/4 a "
                             "power of two <= 64 (got p=%g, H=%d, C=%d)" % (dropout, H, C))
        if seed is None:
            seed = dropout_seed(xw.device)
        drop = (int(seed) & 0xFFFFFFFFFFFFFFFF, float(dropout))
    # autograd.Function.forward always runs with grad disabled: decide here whether
    # a backward can follow (then the forward keeps the pre-bias aggregate)
    train = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (xw, att, bias))
    return _GatPropagate.apply(xw, att, bias, graph, edge_index, H, C, float(negative_slope), bool(return_alpha),
                               train, drop)


class _FeatureTransform(torch.autograd.Function):
    """x @ W with a split-K weight gradient.

    Forward is torch.matmul (hipBLASLt), identical to the reference's
    ``torch.matmul(x, self.weight)`` (GCNConv/GATConv [U5, U6]).  The weight
    gradient x^T g reduces over all N rows into a small [F_in, F_out] matrix:
    as one GEMM it has a handful of output tiles (a few dozen workgroups on
    256 CUs), so it is computed as a batched GEMM over row chunks of
    SPLIT_ROWS (one output tile set per chunk) plus a sum over chunks."""
    SPLIT_ROWS = 8192

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return torch.matmul(x, w)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = torch.matmul(g, w.t())
        if ctx.needs_input_grad[1]:
            n = x.shape[0]
            k = _FeatureTransform.SPLIT_ROWS
            s = n // k
            if s >= 8:
                m = s * k
                xs = x[:m].view(s, k, x.shape[1]).transpose(1, 2)
                gs = g[:m].view(s, k, g.shape[1])
                gw = torch.bmm(xs, gs).sum(0)
                if m < n:
                    gw = gw + torch.matmul(x[m:].t(), g[m:])
            else:
                gw = torch.matmul(x.t(), g)
        return gx, gw


def gemm_rows(x, w, force_generic=False):
    """x @ w (fp32, device) with every output row the k-ordered fmaf chain of
    its own input row (mp_gemm_rows_f32): bitwise independent of how many rows
    x has -- a shard's rows equal the single-GPU rows.  No autograd."""
    lib = _lib.load()
    _lib.require_device(x)
    if x.dim() != 2 or w.dim() != 2 or x.shape[1] != w.shape[0]:
        raise ValueError("gemm_rows: x [M, K] and w [K, N] (got %s and %s)" % (tuple(x.shape), tuple(w.shape)))
    if x.dtype != torch.float32 or w.dtype != torch.float32 or w.device != x.device:
        raise TypeError("gemm_rows: fp32 x and w on one device (got %s / %s on %s / %s)"
                        % (x.dtype, w.dtype, x.device, w.device))
    x = x if (x.stride(1) == 1 and x.stride(0) >= x.shape[1]) else x.contiguous()
    w = w.contiguous()
    M, K = x.shape
    N = w.shape[1]
    out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    if M and K and N:
        _lib.check(lib.mp_gemm_rows_f32(x.data_ptr(), x.stride(0), M, K, w.data_ptr(), 0, N, out.data_ptr(), N,
                                        int(bool(force_generic)), _lib.stream_ptr(x.device)), "mp_gemm_rows_f32")
    elif M and N:
        out.zero_()
    return out


class _FeatureTransformRows(_FeatureTransform):
    """_FeatureTransform with the row-exact forward (gemm_rows); the backward is
    _FeatureTransform's."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return gemm_rows(x, w)


# GATConv / ShardedGATConv: x @ W with the row-exact GEMM, so a sharded layer's
# scores are bitwise the single-GPU layer's
GAT_ROW_EXACT_GEMM = True


def feature_transform(x, w, row_exact=False):
    """``torch.matmul(x, w)`` for a 2-D fp32 device x (split-K weight gradient);
    row_exact: the forward by gemm_rows (each output row a function of its own
    input row, whatever the row count)."""
    if not (torch.is_tensor(x) and x.dim() == 2 and x.is_cuda and x.dtype == torch.float32 and w.dim() == 2):
        return torch.matmul(x, w)
    if not (torch.is_grad_enabled() and (w.requires_grad or x.requires_grad)):
        return gemm_rows(x, w) if row_exact else torch.matmul(x, w)
    if row_exact:
        return _FeatureTransformRows.apply(x, w)
    if not w.requires_grad:
        return torch.matmul(x, w)
    return _FeatureTransform.apply(x, w)
