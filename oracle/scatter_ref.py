"""torch_scatter 2.0.4 semantics on the CPU -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates, for 2-D src and a 1-D index along dim 0 (the only form PyG 1.4.3's
MessagePassing produces):
  scatter_sum  [U8] torch_scatter/scatter.py: broadcast(index) then
               `src.new_zeros(size).scatter_add_(dim, index, src)`
  scatter_mean [U8]: scatter_sum / scatter_sum(ones).clamp_(1) (true_divide)
  scatter_max/min [U9] csrc/cpu/scatter_cpu.cpp: serial strict-compare loop,
               first edge wins ties, empty row -> (0, E)   (scatter_loop.c)
"""
import ctypes
import os
import subprocess

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle_scatter.so")
_lib = None

R_SUM, R_MEAN, R_MAX, R_MIN = 0, 1, 2, 3


def build():
    """Compile scatter_loop.c with gcc (oracle/Makefile)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _c():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        p = ctypes.c_void_p
        i64 = ctypes.c_int64
        lib.oracle_scatter_f32.argtypes = [p, p, i64, i64, i64, ctypes.c_int, ctypes.c_int, p, p]
        lib.oracle_gather_sum_f32.argtypes = [p, p, p, p, i64, i64, i64, p]
        lib.oracle_gather_max_f32.argtypes = [p, p, p, i64, i64, i64, p, p]
        _lib = lib
    return _lib


def _np(t, dtype):
    return np.ascontiguousarray(t.detach().cpu().numpy().astype(dtype, copy=False))


def _addr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _flat2(src):
    """[E, ...] -> [E, prod(...)] (also for E = 0, where reshape(E, -1) is ambiguous)."""
    f = 1
    for d in src.shape[1:]:
        f *= int(d)
    return src.reshape(src.shape[0], f)


# --- torch-op forms (the literal upstream calls) ---------------------------

def scatter_sum(src, index, dim_size):
    """zeros(dim_size, F).scatter_add_(0, index broadcast, src) (edge order)."""
    src2 = _flat2(src)
    out = torch.zeros((dim_size, src2.shape[1]), dtype=src.dtype)
    if src2.numel():
        out.scatter_add_(0, index.view(-1, 1).expand_as(src2), src2)
    return out.reshape((dim_size,) + tuple(src.shape[1:]))


def scatter_mean(src, index, dim_size):
    out = scatter_sum(src, index, dim_size)
    ones = torch.ones(index.size(), dtype=src.dtype)
    count = torch.zeros(dim_size, dtype=src.dtype).scatter_add_(0, index, ones)
    count.clamp_(1)
    return out / count.view((-1,) + (1,) * (out.dim() - 1))


# --- serial-loop forms (scatter_cpu.cpp) ---------------------------------

def scatter_loop(src, index, dim_size, reduce, out=None):
    """Serial loop in C; returns (out, arg or None).  fp32 only."""
    red = {"sum": R_SUM, "add": R_SUM, "mean": R_MEAN, "max": R_MAX, "min": R_MIN}[reduce]
    s = _np(_flat2(src), np.float32)
    E, F = s.shape
    idx = _np(index, np.int64)
    has_out = out is not None
    o = _np(out, np.float32).copy() if has_out else np.empty((dim_size, F), np.float32)
    a = np.empty((dim_size, F), np.int64) if red in (R_MAX, R_MIN) else None
    _c().oracle_scatter_f32(_addr(s), _addr(idx), E, F, dim_size, red, int(has_out), _addr(o), _addr(a))
    shape = (dim_size,) + tuple(src.shape[1:])
    ot = torch.from_numpy(o).reshape(shape)
    at = torch.from_numpy(a).reshape(shape) if a is not None else None
    return ot, at


def scatter_max(src, index, dim_size, out=None):
    return scatter_loop(src, index, dim_size, "max", out)


def scatter_min(src, index, dim_size, out=None):
    return scatter_loop(src, index, dim_size, "min", out)


def gather_sum(x, other, index, weight, dim_size):
    """out[index[e]] += weight[e] * x[other[e]] in edge order (C loop)."""
    xs = _np(x, np.float32)
    F = xs.shape[1]
    o = np.empty((dim_size, F), np.float32)
    w = _np(weight, np.float32) if weight is not None else None
    oth = _np(other, np.int64)
    idx = _np(index, np.int64)
    _c().oracle_gather_sum_f32(_addr(xs), _addr(oth), _addr(idx), _addr(w), idx.shape[0], F, dim_size,
                               _addr(o))
    return torch.from_numpy(o)


def gather_max(x, other, index, dim_size):
    xs = _np(x, np.float32)
    F = xs.shape[1]
    o = np.empty((dim_size, F), np.float32)
    a = np.empty((dim_size, F), np.int64)
    oth = _np(other, np.int64)
    idx = _np(index, np.int64)
    _c().oracle_gather_max_f32(_addr(xs), _addr(oth), _addr(idx), idx.shape[0], F, dim_size, _addr(o),
                               _addr(a))
    return torch.from_numpy(o), torch.from_numpy(a)


# --- any dtype (scatter_cpu.cpp's loop for float64 / float16 / int64) -------

_LOWEST = {np.dtype(np.float64): np.finfo(np.float64).min, np.dtype(np.float32): np.finfo(np.float32).min,
           np.dtype(np.float16): np.finfo(np.float16).min, np.dtype(np.int64): np.iinfo(np.int64).min}
_HIGHEST = {np.dtype(np.float64): np.finfo(np.float64).max, np.dtype(np.float32): np.finfo(np.float32).max,
            np.dtype(np.float16): np.finfo(np.float16).max, np.dtype(np.int64): np.iinfo(np.int64).max}


def scatter_loop_any(src, index, dim_size, reduce, out=None):
    """scatter_cpu.cpp's serial loop (torch_scatter 2.0.4 [U9]) in numpy for
    any of float64 / float32 / float16 / int64, sequential over edges,
    vectorised over features: sums in the source dtype in edge order (numpy
    float16 rounds after every add, as the CPU Half kernel does), max / min with
    a strict compare from lowest() / max() (first edge wins; rows that keep the
    init value -> 0, arg = E unless `out` was given), mean = sum / max(count, 1)
    with integer division truncating toward zero.  Returns (out, arg or None)
    as torch tensors.  Small inputs only (a Python loop over edges)."""
    s = src.detach().cpu().numpy()
    s2 = s.reshape(s.shape[0], -1)
    E, F = s2.shape
    idx = index.cpu().numpy().astype(np.int64)
    dt = s2.dtype
    has_out = out is not None
    if has_out:
        o = out.detach().cpu().numpy().reshape(dim_size, F).copy()
    elif reduce == "max":
        o = np.full((dim_size, F), _LOWEST[dt], dt)
    elif reduce == "min":
        o = np.full((dim_size, F), _HIGHEST[dt], dt)
    else:
        o = np.zeros((dim_size, F), dt)
    a = np.full((dim_size, F), E, np.int64) if reduce in ("max", "min") else None
    cnt = np.zeros(dim_size, np.int64)
    with np.errstate(over="ignore"):
        for e in range(E):
            r = idx[e]
            cnt[r] += 1
            if reduce in ("sum", "add", "mean"):
                o[r] = o[r] + s2[e]
            else:
                better = s2[e] > o[r] if reduce == "max" else s2[e] < o[r]
                o[r] = np.where(better, s2[e], o[r])
                a[r] = np.where(better, e, a[r])
    if reduce == "mean":
        c = np.maximum(cnt, 1).reshape(-1, 1)
        if np.issubdtype(dt, np.integer):
            q = o // c                                   # floor; then toward zero (no abs: INT64_MIN)
            o = q + ((q * c != o) & (o < 0))
        else:
            o = (o / c.astype(dt)).astype(dt)
    if reduce in ("max", "min") and not has_out:
        init = _LOWEST[dt] if reduce == "max" else _HIGHEST[dt]
        o = np.where(o == init, np.zeros_like(o), o)
    shape = (dim_size,) + tuple(src.shape[1:])
    ot = torch.from_numpy(np.ascontiguousarray(o)).reshape(shape)
    at = torch.from_numpy(a).reshape(shape) if a is not None else None
    return ot, at


# --- composites (torch_scatter 2.0.4 composite/softmax.py, logsumexp.py, std.py) ---
# The published 2.0.4 composites restated for 2-D src and a 1-D index along dim
# 0, on the serial-loop max and the edge-order scatter_add above (the package
# is not in the reference tree: parity unpinned).

def scatter_softmax(src, index, eps=1e-12):
    """softmax.py: max_seg, recentre, exp, sum_seg + eps, divide."""
    n = int(index.max()) + 1 if index.numel() else 0
    mx = scatter_loop(src, index, n, "max")[0]
    e = (src - mx[index]).exp()
    return e / (scatter_sum(e, index, n) + eps)[index]


def scatter_log_softmax(src, index, eps=1e-12):
    n = int(index.max()) + 1 if index.numel() else 0
    mx = scatter_loop(src, index, n, "max")[0]
    rc = src - mx[index]
    return rc - torch.log(scatter_sum(rc.exp(), index, n) + eps)[index]


def scatter_logsumexp(src, index, dim_size, eps=1e-12):
    """logsumexp.py: scatter_max into a -inf tensor (out given: no init, no
    masking), recentre, NaN -> -inf, log(sum exp + eps) + max."""
    mx = torch.full((dim_size, src.shape[1]), float("-inf"), dtype=torch.float32)
    mx = scatter_loop(src, index, dim_size, "max", out=mx)[0]
    rc = src - mx[index]
    rc = rc.masked_fill(torch.isnan(rc), float("-inf"))
    return torch.log(scatter_sum(rc.exp(), index, dim_size) + eps) + mx


def scatter_std(src, index, dim_size, unbiased=True):
    """std.py: count = scatter_sum(ones) clamped to 1, mean = sum / count,
    sum of squared deviations / (count' + 1e-6), sqrt; count' = max(count - 1,
    1) when unbiased."""
    count = torch.zeros(dim_size, dtype=src.dtype).scatter_add_(0, index, torch.ones(index.numel(), dtype=src.dtype))
    count = count.clamp(min=1).view(-1, 1)
    mean = scatter_sum(src, index, dim_size) / count
    var = (src - mean[index]) ** 2
    out = scatter_sum(var, index, dim_size)
    if unbiased:
        count = (count - 1).clamp(min=1)
    return (out / (count + 1e-6)).sqrt()
