"""torch_scatter 2.0.4-compatible front door over the MI355X engine.

Same names, argument order and results as torch_scatter 2.0.4
(pinned at /root/reference/requirement.txt:3; the package itself is not in
the reference tree -- see SURVEY.md 2b U8/U9):

    scatter_sum / scatter_add(src, index, dim=-1, out=None, dim_size=None)
    scatter_mean(src, index, dim=-1, out=None, dim_size=None)
    scatter_max / scatter_min(src, index, dim=-1, out=None, dim_size=None) -> (out, arg)
    scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum")
    segment_csr(src, indptr, out=None, reduce="sum"), gather_csr(src, indptr, out=None)
    segment_coo(src, index, out=None, dim_size=None, reduce="sum"), gather_coo(src, index, out=None)
    segment_{sum,add,mean,min,max}_{csr,coo}   (the named forms)
    scatter_softmax / scatter_log_softmax(src, index, dim=-1, eps=1e-12)
    scatter_logsumexp(src, index, dim=-1, out=None, dim_size=None, eps=1e-12)
    scatter_std(src, index, dim=-1, out=None, dim_size=None, unbiased=True)
      (torch_scatter/composite/: restated from the published 2.0.4 source, the
      reductions on the native kernels, the elementwise steps as device ops)

The compiled package's dispatcher ops are registered too (torch.ops.torch_scatter.
scatter_max/min, segment_{sum,mean,min,max}_{csr,coo}, gather_{csr,coo}; the
schemas of torch_scatter 2.0.4's csrc), so TorchScript-visible callers resolve.

All reductions run as destination-sorted segmented reductions in HIP
(mi355_mp.ops) on a ROCm device -- there is no CPU path.  float32 takes the
fused hot-path kernels; float64 / float16 / bfloat16 / int64 the
mp_segment_reduce kernels (every row in edge order: float64 and int64 bit for
bit, the half types accumulated in fp32).
"""
import math as _math
import torch

from mi355_mp import ops as _ops
from mi355_mp import _lib

__version__ = "2.0.4"

__all__ = ["scatter", "scatter_sum", "scatter_add", "scatter_mean", "scatter_max", "scatter_min",
           "segment_csr", "gather_csr", "segment_coo", "gather_coo",
           "segment_sum_csr", "segment_add_csr", "segment_mean_csr", "segment_min_csr", "segment_max_csr",
           "segment_sum_coo", "segment_add_coo", "segment_mean_coo", "segment_min_coo", "segment_max_coo",
           "scatter_softmax", "scatter_log_softmax", "scatter_logsumexp", "scatter_std"]


def _broadcast(index, src, dim):
    """torch_scatter.utils.broadcast: a 1-D index is laid along `dim`, missing
    trailing dims are appended, then the index is expanded to src's shape."""
    if index.dim() == 1:
        for _ in range(dim):
            index = index.unsqueeze(0)
    while index.dim() < src.dim():
        index = index.unsqueeze(-1)
    return index.expand_as(src)


def _index_1d(src, index, dim):
    """The 1-D index along `dim` when torch_scatter's broadcast index is the
    same for every position of the other dims (PyG's case); None when the
    index is element-wise (handled by the general path)."""
    if index.dim() == 1:
        if index.numel() != src.size(dim):
            raise ValueError("index of size %d does not match src.size(%d) = %d"
                             % (index.numel(), dim, src.size(dim)))
        return index
    if index.dim() > src.dim():
        raise ValueError("index has more dimensions than src")
    while index.dim() < src.dim():
        index = index.unsqueeze(-1)
    sl = [0] * index.dim()
    sl[dim] = slice(None)
    first = index[tuple(sl)]
    if all(index.stride(d) == 0 or index.size(d) == 1 for d in range(index.dim()) if d != dim):
        return first
    view = [1] * index.dim()
    view[dim] = -1
    if bool((index == first.view(view)).all()):
        return first
    return None


def _check_dtype(src):
    if src.dtype not in _lib.MP_DTYPE:
        raise TypeError("mi355_mp: scatter ops take float32, float64, float16, bfloat16 or int64 (got %s)" % src.dtype)


def _prepare(src, index, dim, dim_size):
    _lib.require_device(src, index)
    _check_dtype(src)
    dim = dim % src.dim() if src.dim() else 0
    idx = _index_1d(src, index, dim).to(torch.int64)
    if dim_size is None:
        dim_size = int(idx.max()) + 1 if idx.numel() > 0 else 0
    moved = src.movedim(dim, 0)
    rest = moved.shape[1:]
    src2 = moved.reshape(moved.shape[0], _math.prod(moved.shape[1:]))
    return dim, idx, int(dim_size), src2, rest


def _finish(out2, dim, rest):
    out = out2.reshape((out2.shape[0],) + tuple(rest))
    return out.movedim(0, dim)


def _reduce_general(src, index, dim, out, dim_size, reduce):
    """Element-wise index: out[..., index[..., e, ...], ...] over every position.
    Flattened to one 1-D segmented reduction: key = (position of the other
    dims) * dim_size + index, one feature per element; the stable CSR sort keeps
    each output's elements in their original order along `dim`."""
    idx = _broadcast(index, src, dim).to(torch.int64)
    if out is not None:
        dim_size = out.size(dim)
    elif dim_size is None:
        dim_size = int(idx.max()) + 1 if idx.numel() > 0 else 0
    s = src.movedim(dim, -1)
    ix = idx.movedim(dim, -1)
    lead = tuple(s.shape[:-1])
    L = s.shape[-1]
    B = s.numel() // L if L else 0
    keys = (torch.arange(B, device=src.device).view(-1, 1) * dim_size + ix.reshape(B, L)).reshape(-1)
    vals = s.reshape(-1, 1)
    if out is not None:
        o = out.movedim(dim, -1).reshape(B * dim_size, 1).clone(memory_format=torch.contiguous_format)
        res, arg = _ops.segment_reduce_into(vals, keys, o, reduce)
        out.copy_(res.view(lead + (dim_size,)).movedim(-1, dim))
        res_t = out
    else:
        res, arg = _ops.segment_reduce(vals, keys, B * dim_size, reduce)
        res_t = res.view(lead + (dim_size,)).movedim(-1, dim)
    arg_t = None
    if arg is not None:   # flat element position -> position along dim (empty: src.size(dim))
        a = arg.view(-1)
        a = torch.where(a >= B * L, torch.full_like(a, L), a % max(L, 1))
        arg_t = a.view(lead + (dim_size,)).movedim(-1, dim)
    return res_t, arg_t


def _reduce(src, index, dim, out, dim_size, reduce):
    _lib.require_device(src, index)
    _check_dtype(src)
    d = dim % src.dim() if src.dim() else 0
    if _index_1d(src, index, d) is None:
        if out is not None:
            _lib.require_device(out)
        return _reduce_general(src, index, d, out, dim_size, reduce)
    if out is not None:
        dim = dim % src.dim()
        dim_size = out.size(dim)
    dim, idx, dim_size, src2, rest = _prepare(src, index, dim, dim_size)
    if out is not None:
        _lib.require_device(out)
        o2 = out.movedim(dim, 0).reshape(dim_size, -1)
        # reduce straight into out when the [dim_size, F] form is a row-major view of
        # it (the reshape did not copy); otherwise into a fresh row-major copy, then
        # copied back (never a copy that aliases out: size-1 dims make torch call
        # odd strides contiguous)
        F2 = o2.shape[1] if o2.dim() == 2 else 0
        in_place = (o2.untyped_storage().data_ptr() == out.untyped_storage().data_ptr()
                    and (F2 <= 1 or o2.stride(1) == 1) and (dim_size <= 1 or o2.stride(0) >= F2))
        buf = o2 if in_place else o2.clone(memory_format=torch.contiguous_format)
        res, arg = _ops.segment_reduce_into(src2, idx, buf, reduce)
        if not in_place:
            out.copy_(_finish(res, dim, rest))
        arg_full = _finish(arg, dim, rest) if arg is not None else None
        return out, arg_full
    res, arg = _ops.segment_reduce(src2, idx, dim_size, reduce)
    return _finish(res, dim, rest), (_finish(arg, dim, rest) if arg is not None else None)


def scatter_sum(src, index, dim=-1, out=None, dim_size=None):
    return _reduce(src, index, dim, out, dim_size, "sum")[0]


def scatter_add(src, index, dim=-1, out=None, dim_size=None):
    return scatter_sum(src, index, dim, out, dim_size)


def scatter_mean(src, index, dim=-1, out=None, dim_size=None):
    return _reduce(src, index, dim, out, dim_size, "mean")[0]


def scatter_max(src, index, dim=-1, out=None, dim_size=None):
    return _reduce(src, index, dim, out, dim_size, "max")


def scatter_min(src, index, dim=-1, out=None, dim_size=None):
    return _reduce(src, index, dim, out, dim_size, "min")


def scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum"):
    if reduce in ("sum", "add"):
        return scatter_sum(src, index, dim, out, dim_size)
    if reduce == "mean":
        return scatter_mean(src, index, dim, out, dim_size)
    if reduce == "max":
        return scatter_max(src, index, dim, out, dim_size)[0]
    if reduce == "min":
        return scatter_min(src, index, dim, out, dim_size)[0]
    raise ValueError("unknown reduce %r" % (reduce,))


def segment_csr(src, indptr, out=None, reduce="sum"):
    """torch_scatter.segment_csr for 1-D indptr along dim 0 (sum/mean/max/min)."""
    _lib.require_device(src, indptr)
    counts = indptr[1:] - indptr[:-1]
    index = torch.repeat_interleave(torch.arange(counts.numel(), device=src.device), counts)
    res = _reduce(src, index, 0, out, counts.numel(), "sum" if reduce == "add" else reduce)
    return res if reduce in ("max", "min") else res[0]


def gather_csr(src, indptr, out=None):
    """torch_scatter.gather_csr along dim 0: out[e] = src[segment(e)]."""
    _lib.require_device(src, indptr)
    counts = indptr[1:] - indptr[:-1]
    index = torch.repeat_interleave(torch.arange(counts.numel(), device=src.device), counts)
    res = _ops.index_select_rows(src.reshape(src.shape[0], _math.prod(src.shape[1:])), index).reshape((-1,) + tuple(src.shape[1:]))
    if out is not None:
        out.copy_(res)
        return out
    return res


def segment_coo(src, index, out=None, dim_size=None, reduce="sum"):
    """torch_scatter.segment_coo for a sorted 1-D index along dim 0: the same
    reduction as scatter (each segment in edge order, first-index argmax)."""
    _lib.require_device(src, index)
    if index.numel() > 1 and bool((index[1:] < index[:-1]).any()):
        raise ValueError("segment_coo: index must be sorted")
    res = _reduce(src, index, 0, out, dim_size, "sum" if reduce == "add" else reduce)
    return res if reduce in ("max", "min") else res[0]


def gather_coo(src, index, out=None):
    """torch_scatter.gather_coo along dim 0: out[e] = src[index[e]]."""
    _lib.require_device(src, index)
    res = _ops.index_select_rows(src.reshape(src.shape[0], _math.prod(src.shape[1:])), index).reshape((-1,) + tuple(src.shape[1:]))
    if out is not None:
        out.copy_(res)
        return out
    return res


def segment_sum_csr(src, indptr, out=None):
    return segment_csr(src, indptr, out, "sum")


def segment_add_csr(src, indptr, out=None):
    return segment_csr(src, indptr, out, "sum")


def segment_mean_csr(src, indptr, out=None):
    return segment_csr(src, indptr, out, "mean")


def segment_min_csr(src, indptr, out=None):
    return segment_csr(src, indptr, out, "min")


def segment_max_csr(src, indptr, out=None):
    return segment_csr(src, indptr, out, "max")


def segment_sum_coo(src, index, out=None, dim_size=None):
    return segment_coo(src, index, out, dim_size, "sum")


def segment_add_coo(src, index, out=None, dim_size=None):
    return segment_coo(src, index, out, dim_size, "sum")


def segment_mean_coo(src, index, out=None, dim_size=None):
    return segment_coo(src, index, out, dim_size, "mean")


def segment_min_coo(src, index, out=None, dim_size=None):
    return segment_coo(src, index, out, dim_size, "min")


def segment_max_coo(src, index, out=None, dim_size=None):
    return segment_coo(src, index, out, dim_size, "max")


# ---------------------------------------------------------------------------
# composite ops (torch_scatter 2.0.4 composite/{softmax,logsumexp,std}.py)
# ---------------------------------------------------------------------------

def _gather_back(t, index, dim):
    """t.gather(dim, broadcast(index)) -- each element's segment value.  A 1-D
    index (PyG's form) takes the native row gather."""
    d = dim % t.dim()
    if index.dim() == 1:
        moved = t.movedim(d, 0)
        rows = _ops.index_select_rows(moved.reshape(moved.shape[0], _math.prod(moved.shape[1:])).contiguous(), index.to(torch.int64))
        return rows.reshape((index.numel(),) + tuple(moved.shape[1:])).movedim(0, d)
    size = list(t.shape)
    size[d] = index.size(d) if index.dim() > d else index.size(-1)
    return t.gather(d, _broadcast(index, torch.empty(size, device="meta"), d))


def _check_float(src, name):
    if not torch.is_floating_point(src):
        raise ValueError("`%s` can only be computed over tensors with floating point data types." % name)


def scatter_softmax(src, index, dim=-1, eps=1e-12):
    """exp(src - max_seg) / (sum_seg exp(src - max_seg) + eps), per element."""
    _check_float(src, "scatter_softmax")
    dim = dim % src.dim()
    # the shift carries no gradient (softmax is shift-invariant: upstream's
    # gradient through the max cancels), so the max runs without autograd
    max_per_index = scatter_max(src.detach(), index, dim=dim)[0]
    recentered = src - _gather_back(max_per_index, index, dim)
    e = recentered.exp()
    den = scatter_sum(e, index, dim, dim_size=max_per_index.size(dim)) + eps
    return e / _gather_back(den, index, dim)


def scatter_log_softmax(src, index, dim=-1, eps=1e-12):
    """(src - max_seg) - log(sum_seg exp(src - max_seg) + eps), per element."""
    _check_float(src, "scatter_log_softmax")
    dim = dim % src.dim()
    max_per_index = scatter_max(src.detach(), index, dim=dim)[0]
    recentered = src - _gather_back(max_per_index, index, dim)
    den = scatter_sum(recentered.exp(), index, dim, dim_size=max_per_index.size(dim)) + eps
    return recentered - _gather_back(den.log(), index, dim)


def scatter_logsumexp(src, index, dim=-1, out=None, dim_size=None, eps=1e-12):
    """log(sum_seg exp(src - max_seg) + eps) + max_seg; the max starts from -inf
    (scatter_max into a -inf tensor: empty segments stay -inf), NaN
    differences count as -inf; a given `out` enters as exp(out - max)."""
    _check_float(src, "scatter_logsumexp")
    dim = dim % src.dim()
    if out is not None:
        dim_size = out.size(dim)
    elif dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() else 0
    size = list(src.size())
    size[dim] = dim_size
    max_per_index = torch.full(size, float("-inf"), dtype=src.dtype, device=src.device)
    scatter_max(src.detach(), index, dim, max_per_index, dim_size=dim_size)   # shift: no gradient (cancels)
    recentered = src - _gather_back(max_per_index, index, dim)
    recentered = recentered.masked_fill(torch.isnan(recentered), float("-inf"))
    if out is not None:
        out = out.sub_(max_per_index).exp_()
    s = scatter_sum(recentered.exp(), index, dim, out, dim_size)
    return s.add_(eps).log_().add_(max_per_index)


def scatter_std(src, index, dim=-1, out=None, dim_size=None, unbiased=True):
    """sqrt(sum_seg (src - mean_seg)^2 / (c + 1e-6)), mean = sum / max(count, 1),
    c = max(max(count, 1) - 1, 1) when unbiased else max(count, 1)."""
    if out is not None:
        dim_size = out.size(dim)
    dim = dim % src.dim()
    idx = _index_1d(src, index, dim)
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() else 0
    if idx is not None:
        ones = torch.ones(idx.numel(), 1, dtype=src.dtype, device=src.device)
        count = scatter_sum(ones, idx, 0, dim_size=dim_size).view(-1)
        shape = [1] * src.dim()
        shape[dim] = dim_size
        count = count.view(shape)
    else:
        ones = torch.ones(src.size(), dtype=src.dtype, device=src.device)
        count = scatter_sum(ones, index, dim, dim_size=dim_size)
    tmp = scatter_sum(src, index, dim, dim_size=dim_size)
    count = count.clamp(min=1)
    mean = tmp / count
    var = src - _gather_back(mean, index, dim)
    var = var * var
    res = scatter_sum(var, index, dim, out, dim_size)
    if unbiased:
        count = (count - 1).clamp(min=1)
    res = res / (count + 1e-6)
    res = res.sqrt()
    if out is not None:
        out.copy_(res)
        return out
    return res


# ---------------------------------------------------------------------------
# dispatcher registration (torch.ops.torch_scatter.*)
# ---------------------------------------------------------------------------

def _out_rows(*cands):
    """First known row count among cands (None = unknown), else a data-dependent
    size from the fake-tensor context (like nonzero's)."""
    for c in cands:
        if c is not None:
            return int(c)
    return torch.library.get_ctx().new_dynamic_size()


def _with_rows(t, rows, dim=0):
    size = list(t.shape)
    size[dim] = rows
    return size


def _arg_grad(grad, arg, src_shape, dim):
    """torch_scatter's ScatterMax / SegmentMax backward: grad_src =
    zeros(size with src.size(dim) + 1).scatter_(dim, arg, grad).narrow(dim, 0,
    src.size(dim)) -- the extra slice absorbs the empty-segment sentinel; each
    (position, column) is stored at most once (plain stores, deterministic)."""
    size = list(src_shape)
    n = size[dim]
    size[dim] = n + 1
    return grad.new_zeros(size).scatter_(dim, arg, grad).narrow(dim, 0, n)


def _csr_counts(indptr):
    return indptr[1:] - indptr[:-1]


def _register_ops():
    """torch_scatter 2.0.4's compiled ops on the dispatcher, split by key like a
    compiled extension: the HIP engine on CUDA (ROCm) tensors; CPU tensors
    raise (no CPU path); a fake (meta) kernel per op for shape propagation
    under FakeTensor / torch.compile tracing (torch.library.register_fake);
    and each op's backward (torch.library.register_autograd) on the same
    native ops -- scatter / segment min-max by their arg, sums and means by the
    matching gather, gathers by the matching segment sum."""
    try:
        lib = torch.library.Library("torch_scatter", "DEF")
    except RuntimeError:  # namespace already defined by another loader
        return None

    def arg_op(reduce):
        return lambda s, i, d, o, n: _reduce(s, i, d, o, n, reduce)

    defs = {
        "scatter_max": ("(Tensor src, Tensor index, int dim, Tensor? optional_out, int? dim_size) -> (Tensor, Tensor)",
                        arg_op("max")),
        "scatter_min": ("(Tensor src, Tensor index, int dim, Tensor? optional_out, int? dim_size) -> (Tensor, Tensor)",
                        arg_op("min")),
        "segment_sum_csr": ("(Tensor src, Tensor indptr, Tensor? optional_out) -> Tensor",
                            lambda s, p, o: segment_csr(s, p, o, "sum")),
        "segment_mean_csr": ("(Tensor src, Tensor indptr, Tensor? optional_out) -> Tensor",
                             lambda s, p, o: segment_csr(s, p, o, "mean")),
        "segment_min_csr": ("(Tensor src, Tensor indptr, Tensor? optional_out) -> (Tensor, Tensor)",
                            lambda s, p, o: segment_csr(s, p, o, "min")),
        "segment_max_csr": ("(Tensor src, Tensor indptr, Tensor? optional_out) -> (Tensor, Tensor)",
                            lambda s, p, o: segment_csr(s, p, o, "max")),
        "gather_csr": ("(Tensor src, Tensor indptr, Tensor? optional_out) -> Tensor",
                       lambda s, p, o: gather_csr(s, p, o)),
        "segment_sum_coo": ("(Tensor src, Tensor index, Tensor? optional_out, int? dim_size) -> Tensor",
                            lambda s, i, o, n: segment_coo(s, i, o, n, "sum")),
        "segment_mean_coo": ("(Tensor src, Tensor index, Tensor? optional_out, int? dim_size) -> Tensor",
                             lambda s, i, o, n: segment_coo(s, i, o, n, "mean")),
        "segment_min_coo": ("(Tensor src, Tensor index, Tensor? optional_out, int? dim_size) -> (Tensor, Tensor)",
                            lambda s, i, o, n: segment_coo(s, i, o, n, "min")),
        "segment_max_coo": ("(Tensor src, Tensor index, Tensor? optional_out, int? dim_size) -> (Tensor, Tensor)",
                            lambda s, i, o, n: segment_coo(s, i, o, n, "max")),
        "gather_coo": ("(Tensor src, Tensor index, Tensor? optional_out) -> Tensor",
                       lambda s, i, o: gather_coo(s, i, o)),
    }

    # --- fake kernels: output shapes only (no data_ptr, no launch)
    def fake_scatter(src, index, dim, out, dim_size):
        d = dim % src.dim()
        rows = _out_rows(out.size(d) if out is not None else None, dim_size)
        size = _with_rows(src, rows, d)
        return src.new_empty(size), src.new_empty(size, dtype=torch.int64)

    def fake_seg_csr(src, indptr, out):
        size = _with_rows(src, indptr.numel() - 1)
        return src.new_empty(size)

    def fake_seg_csr_arg(src, indptr, out):
        size = _with_rows(src, indptr.numel() - 1)
        return src.new_empty(size), src.new_empty(size, dtype=torch.int64)

    def fake_gather_csr(src, indptr, out):
        return src.new_empty(_with_rows(src, _out_rows(out.size(0) if out is not None else None)))

    def fake_seg_coo(src, index, out, dim_size):
        return src.new_empty(_with_rows(src, _out_rows(out.size(0) if out is not None else None, dim_size)))

    def fake_seg_coo_arg(src, index, out, dim_size):
        size = _with_rows(src, _out_rows(out.size(0) if out is not None else None, dim_size))
        return src.new_empty(size), src.new_empty(size, dtype=torch.int64)

    def fake_gather_coo(src, index, out):
        return src.new_empty(_with_rows(src, index.numel()))

    fakes = {"scatter_max": fake_scatter, "scatter_min": fake_scatter, "segment_sum_csr": fake_seg_csr,
             "segment_mean_csr": fake_seg_csr, "segment_min_csr": fake_seg_csr_arg,
             "segment_max_csr": fake_seg_csr_arg, "gather_csr": fake_gather_csr, "segment_sum_coo": fake_seg_coo,
             "segment_mean_coo": fake_seg_coo, "segment_min_coo": fake_seg_coo_arg,
             "segment_max_coo": fake_seg_coo_arg, "gather_coo": fake_gather_coo}

    # --- autograd: d src only (index / indptr carry none); through optional_out unsupported
    def make_setup(name):
        scatter = name.startswith("scatter")

        def setup(ctx, inputs, output):
            ctx.src_shape = tuple(inputs[0].shape)
            ctx.index = inputs[1]
            ctx.dim = inputs[2] % max(1, inputs[0].dim()) if scatter else 0
            ctx.has_out = (inputs[3] if scatter else inputs[2]) is not None
            pair = isinstance(output, (tuple, list))
            ctx.arg = output[1] if pair else None
            ctx.out_rows = (output[0] if pair else output).shape[0]
        return setup

    def no_out(ctx, name):
        if ctx.has_out:
            raise NotImplementedError("torch_scatter::%s: autograd through optional_out is not supported" % name)

    def bwd_arg(name):
        def f(ctx, grad, _grad_arg=None):
            no_out(ctx, name)
            g = _arg_grad(grad.contiguous(), ctx.arg, ctx.src_shape, ctx.dim)
            return (g,) + (None,) * (4 if name.startswith("scatter") else (3 if name.endswith("coo") else 2))
        return f

    def bwd_sum_csr(ctx, grad):
        no_out(ctx, "segment_sum_csr")
        return gather_csr(grad.contiguous(), ctx.index), None, None

    def bwd_mean_csr(ctx, grad):
        no_out(ctx, "segment_mean_csr")
        cnt = _csr_counts(ctx.index).clamp(min=1).to(grad.dtype).view((-1,) + (1,) * (grad.dim() - 1))
        return gather_csr((grad / cnt).contiguous(), ctx.index), None, None

    def bwd_gather_csr(ctx, grad):
        no_out(ctx, "gather_csr")
        return segment_csr(grad.contiguous(), ctx.index, None, "sum"), None, None

    def bwd_sum_coo(ctx, grad):
        no_out(ctx, "segment_sum_coo")
        return gather_coo(grad.contiguous(), ctx.index), None, None, None

    def bwd_mean_coo(ctx, grad):
        no_out(ctx, "segment_mean_coo")
        cnt = torch.bincount(ctx.index, minlength=ctx.out_rows)[:ctx.out_rows].clamp(min=1).to(grad.dtype)
        cnt = cnt.view((-1,) + (1,) * (grad.dim() - 1))
        return gather_coo((grad / cnt).contiguous(), ctx.index), None, None, None

    def bwd_gather_coo(ctx, grad):
        no_out(ctx, "gather_coo")
        return scatter_sum(grad.contiguous(), ctx.index, 0, dim_size=ctx.src_shape[0]), None, None

    bwds = {"scatter_max": bwd_arg("scatter_max"), "scatter_min": bwd_arg("scatter_min"),
            "segment_sum_csr": bwd_sum_csr, "segment_mean_csr": bwd_mean_csr,
            "segment_min_csr": bwd_arg("segment_min_csr"), "segment_max_csr": bwd_arg("segment_max_csr"),
            "gather_csr": bwd_gather_csr, "segment_sum_coo": bwd_sum_coo, "segment_mean_coo": bwd_mean_coo,
            "segment_min_coo": bwd_arg("segment_min_coo"), "segment_max_coo": bwd_arg("segment_max_coo"),
            "gather_coo": bwd_gather_coo}

    def below_autograd(fn):
        # the kernel runs below autograd (the op's backward is registered below):
        # the engine's own autograd Functions only run their forward here
        def k(*args):
            with torch.no_grad():
                return fn(*args)
        return k

    for name, (schema, fn) in defs.items():
        lib.define(name + schema)
        lib.impl(name, below_autograd(fn), "CUDA")
        lib.impl(name, below_autograd(fn), "CPU")   # raises: mi355_mp has no CPU fallback (_lib.require_device)
        torch.library.register_fake("torch_scatter::" + name, fakes[name], lib=lib)
        torch.library.register_autograd("torch_scatter::" + name, bwds[name], setup_context=make_setup(name), lib=lib)
    return lib


_LIB = _register_ops()
