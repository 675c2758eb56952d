"""Destination-sorted CSR graphs + merge-path schedules, built and cached on the GPU.

PyG 1.4.3 keeps a graph as ``edge_index`` [2, E] int64 and, on every
``propagate``, gathers ``x[edge_index[j]]`` and scatter-adds into
``edge_index[i]``.  The engine instead sorts the edges by the
aggregation index once (stable: each row keeps its edges in original order)
and reuses that CSR for every aggregation over the same ``edge_index``
tensor.  Caches are keyed on the tensor object (identity + version counter)
and dropped when the tensor dies, mirroring GCNConv's ``cached=True`` idea
without changing its semantics.
"""
import weakref

import torch

from . import _lib

DEFAULT_CHUNK = None   # auto: see auto_chunk()
# Per-slot arrays (col, eid, CSR-order weights) are allocated this many
# elements past their end: scalar slot batches may read whole batches there.
SLOT_PAD = 64
MIN_CHUNK, MAX_CHUNK = 16, 1024
# auto_chunk: the best task size grows like sqrt(units): c with 56 c^2 <= units
CHUNK_SQRT_K = 56
# An explicit task-count target (the rule before the sqrt fit; GAT's graphs):
# GAT's per-slot softmax work favours more, shorter tasks: its fused backward
# pass over the transposed CSR runs 1.9 ms longer at chunk 1024 than at 512 on
# RMAT21 (layer forward + backward 32.0 vs 33.9 ms, profiles/r02_ab_chunk_train.log)
GAT_TARGET_TASKS = 100_000


def auto_chunk(n_rows, n_edges, target=None):
    """Merge-path task size in work units (rows + slots), a power of two in
    [16, 1024].

    Default: the largest c with 56 c^2 <= units -- a fit of the measured best
    chunk on graphs of 1.5M to 128M units (tools/exp_shard_chunk.py,
    profiles/r02_exp_shard_chunk.log, profiles/r02_ab_chunk.log): the per-rank
    graphs of the sharded config-2 bench (interior edges at P = 8, 1.5M units:
    128, 0.231 ms vs 0.323 ms at the old 50K-task rule's 16; boundary edges at
    P = 4, 11.8M units: 256, 1.160 vs 1.224 ms at 128), RMAT21 (64M units:
    1024, main + fix-up 6.57 ms vs 6.59 at 512 and 6.65 at 2048), the
    products-scale (128M) and Reddit-scale (115M) graphs 1024.  Bigger tasks
    mean fewer rows cut by a task boundary (a smaller fix-up, more rows summed
    in one task: bit-identical to the sequential order) and less per-task
    overhead; small graphs keep enough tasks to spread over 256 CUs (Cora, 13K
    units: 16 -> 829 tasks).

    target: the largest c <= units / target instead (GAT_TARGET_TASKS)."""
    units = int(n_rows) + int(n_edges)
    c = MIN_CHUNK
    if target is None:
        while c * 2 <= MAX_CHUNK and CHUNK_SQRT_K * (c * 2) ** 2 <= units:
            c *= 2
        return c
    target = int(target)
    while c * 2 <= MAX_CHUNK and units // (c * 2) >= target:
        c *= 2
    return c


def default_snap(chunk):
    """Rows of up to chunk/2 slots are never split across tasks."""
    return chunk // 2


class CSR:
    """One stable CSR of ``key`` (int64 [E]) with gather column ``other``.

    rowptr[n_rows+1], col[E] (= other[eid] or eid), eid[E] : int32 on device.
    """

    def __init__(self, key, other, n_rows, n_other, chunk=DEFAULT_CHUNK, snap=None, target_tasks=None):
        _lib.require_device(key)
        lib = _lib.load()
        dev = key.device
        key = key.contiguous()
        other = other.contiguous() if other is not None else None
        E = key.numel()
        self.n_rows = int(n_rows)
        self.n_edges = int(E)
        self.n_other = int(n_other)
        self.device = dev
        self.chunk = auto_chunk(self.n_rows, E, target_tasks) if chunk is None else int(chunk)
        self.snap = default_snap(self.chunk) if snap is None else int(snap)
        self.rowptr = torch.empty(self.n_rows + 1, dtype=torch.int32, device=dev)
        self.col = torch.zeros(E + SLOT_PAD, dtype=torch.int32, device=dev)
        self.eid = torch.zeros(E + SLOT_PAD, dtype=torch.int32, device=dev)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        st = _lib.stream_ptr(dev)
        ws_bytes = lib.mp_csr_build_workspace(E, self.n_rows)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        _lib.check(lib.mp_csr_build(key.data_ptr(), _lib.ptr(other), E, self.n_rows, self.n_other,
                                    self.rowptr.data_ptr(), self.col.data_ptr(), self.eid.data_ptr(),
                                    bad.data_ptr(), ws.data_ptr(), ws_bytes, st), "mp_csr_build")
        # the bad-index count is read together with the schedule's split-row count:
        # one host sync per CSR (the schedule over a rowptr that skipped bad ids is
        # still well formed, and is dropped with the raise)
        self._build_schedule(bad)
        del ws

    def _build_schedule(self, bad=None):
        """Merge-path schedule over rowptr (tasks of `chunk` rows + slots); bad:
        the CSR build's out-of-range count, read in the same host sync."""
        lib = _lib.load()
        dev, E = self.device, self.n_edges
        st = _lib.stream_ptr(dev)
        self.n_waves = int(lib.mp_schedule_n_waves(self.n_rows, E, self.chunk))
        self.wave_row = torch.empty(self.n_waves + 1, dtype=torch.int32, device=dev)
        self.wave_slot = torch.empty(self.n_waves + 1, dtype=torch.int32, device=dev)
        self.split_waves = torch.empty(self.n_waves, dtype=torch.int32, device=dev)
        n_split = torch.zeros(1, dtype=torch.int32, device=dev)
        sws = lib.mp_schedule_workspace(self.n_waves)
        ws = torch.empty(sws, dtype=torch.uint8, device=dev)
        _lib.check(lib.mp_schedule_build(self.rowptr.data_ptr(), self.n_rows, E, self.chunk, self.snap,
                                         self.wave_row.data_ptr(), self.wave_slot.data_ptr(),
                                         self.split_waves.data_ptr(), n_split.data_ptr(),
                                         ws.data_ptr(), sws, st), "mp_schedule_build")
        if bad is None:
            self.n_split = int(n_split.item())
        else:
            nbad, self.n_split = torch.cat([bad, n_split]).tolist()
            if nbad:
                raise IndexError("mi355_mp: %d edge indices out of range (rows %d, columns %d)"
                                 % (nbad, self.n_rows, self.n_other))
        self._structs = {}
        self._deg = None

    @classmethod
    def from_slots(cls, rowptr, col, eid, n_rows, n_other, chunk=DEFAULT_CHUNK):
        """A CSR over explicit int32 arrays (rowptr [n_rows+1], col / eid [E])."""
        self = cls.__new__(cls)
        E = int(col.numel())
        self.n_rows, self.n_edges, self.n_other = int(n_rows), E, int(n_other)
        self.device = col.device
        self.chunk = auto_chunk(self.n_rows, E) if chunk is None else int(chunk)
        self.snap = default_snap(self.chunk)
        self.rowptr = rowptr.to(torch.int32).contiguous()
        self.col = torch.zeros(E + SLOT_PAD, dtype=torch.int32, device=self.device)
        self.eid = torch.zeros(E + SLOT_PAD, dtype=torch.int32, device=self.device)
        self.col[:E] = col
        self.eid[:E] = eid
        self._build_schedule()
        return self

    def first_occurrences(self):
        """The CSR without repeated (row, column) slots: of the slots of one row
        that gather the same source, only the first (in original edge order) is
        kept, with its original edge id.  For an unweighted max / min this is
        the same reduction bit for bit -- a repeat contributes the same value,
        and torch_scatter's strict compare keeps the first edge's
        id on ties -- with fewer gathers (the Reddit-scale power-law graph of
        config 4 repeats 31% of its edges).  Returns self when nothing repeats;
        built once and cached."""
        u = getattr(self, "_first", None)
        if u is not None:
            return u
        E = self.n_edges
        if E < 2 or self.col is None:
            self._first = self
            return self
        rows = self.slot_rows()[:E].to(torch.int64)
        key = rows * max(self.n_other, 1) + self.col[:E].to(torch.int64)
        order = torch.sort(key, stable=True).indices       # equal keys keep slot (= edge) order
        ks = key[order]
        first = torch.ones(E, dtype=torch.bool, device=self.device)
        first[1:] = ks[1:] != ks[:-1]
        keep = torch.zeros(E, dtype=torch.bool, device=self.device)
        keep[order[first]] = True
        del key, order, ks, first
        n_keep = int(keep.sum().item())
        if n_keep == E:
            self._first = self
            return self
        counts = torch.bincount(rows[keep], minlength=self.n_rows)
        rowptr = torch.zeros(self.n_rows + 1, dtype=torch.int64, device=self.device)
        torch.cumsum(counts, 0, out=rowptr[1:])
        self._first = CSR.from_slots(rowptr, self.col[:E][keep], self.eid[:E][keep], self.n_rows, self.n_other,
                                     self.chunk)
        self._first.n_ids = E       # empty rows still report arg = E
        return self._first

    def add_gather(self, name, col, n_cols, eid=None):
        """Register a struct variant under ``name`` for struct(): a custom gather
        column (int32 [E]; None = identity, rows in slot order) and optionally a
        custom per-slot id array in place of eid."""
        self._extra = getattr(self, "_extra", {})
        self._extra[name] = (None if col is None else col.contiguous(), int(n_cols),
                             None if eid is None else eid.contiguous())
        self._structs.pop(name, None)

    def struct(self, gather="other"):
        """ctypes mp_csr; gather='other' reads x[other] rows, 'eid' reads message
        rows (original edge order), 'slot' reads rows already in CSR slot order
        (identity column: col = NULL); other names are variants registered with
        add_gather()."""
        s = self._structs.get(gather)
        if s is None:
            extra = getattr(self, "_extra", {})
            eid = self.eid
            if gather in extra:
                col, n_cols, e2 = extra[gather]
                if e2 is not None:
                    eid = e2
            elif gather == "slot":
                col, n_cols = None, self.n_edges
            else:
                col = self.col if gather == "other" else self.eid
                n_cols = self.n_other if gather == "other" else self.n_edges
            s = _lib.MpCsr(self.rowptr.data_ptr(), _lib.ptr(col), eid.data_ptr(),
                           self.wave_row.data_ptr(), self.wave_slot.data_ptr(),
                           self.split_waves.data_ptr(), self.n_rows, self.n_edges, self.chunk,
                           self.n_waves, self.n_split, n_cols, getattr(self, "n_ids", 0))
            self._structs[gather] = s
        return s

    def slot_rows(self):
        """int32 [E]: the row owning each CSR slot (cached)."""
        if getattr(self, "_slot_rows", None) is None:
            sr = torch.empty(max(self.n_edges, 1), dtype=torch.int32, device=self.device)
            _lib.check(_lib.load().mp_csr_slot_rows(self.struct("other"), sr.data_ptr(),
                                                    _lib.stream_ptr(self.device)), "mp_csr_slot_rows")
            self._slot_rows = sr
        return self._slot_rows

    def inverse_eid(self):
        """int32 [E]: inv[e] = the slot of edge id e in this CSR (cached)."""
        if getattr(self, "_inv", None) is None:
            inv = torch.empty(max(self.n_edges, 1), dtype=torch.int32, device=self.device)
            _lib.check(_lib.load().mp_csr_inverse_eid(self.struct("other"), inv.data_ptr(),
                                                      _lib.stream_ptr(self.device)), "mp_csr_inverse_eid")
            self._inv = inv
        return self._inv

    def degree(self):
        """In-degree per row (int64), from rowptr."""
        if self._deg is None:
            rp = self.rowptr.to(torch.int64)
            self._deg = rp[1:] - rp[:-1]
        return self._deg

    def to_csr_order(self, edge_values):
        """Permute a per-edge fp32 vector (original order) into CSR slot order."""
        lib = _lib.load()
        edge_values = edge_values.contiguous()
        out = torch.zeros(edge_values.numel() + SLOT_PAD, dtype=edge_values.dtype,
                          device=edge_values.device)[:edge_values.numel()]
        if self.n_edges:
            _lib.check(lib.mp_permute_f32(edge_values.data_ptr(), self.eid.data_ptr(), self.n_edges,
                                          out.data_ptr(), _lib.stream_ptr(self.device)),
                       "mp_permute_f32")
        return out


class Graph:
    """Both directions of one edge_index for a given flow.

    ``dst`` : CSR keyed on the aggregation index edge_index[i] (gathers edge_index[j])
    ``src`` : CSR keyed on edge_index[j] (transpose; used by backward passes)

    A Graph made by the cache (``graph_for``) holds only a weak reference to
    ``edge_index`` (the cache must not keep the user's tensor alive; callers
    keep it alive while a direction is first built -- autograd saves it for
    backward); one constructed directly holds a strong reference.
    """

    def __init__(self, edge_index, n_dst, n_src, flow="source_to_target", chunk=DEFAULT_CHUNK,
                 weak=False, target_tasks=None):
        self.i, self.j = (1, 0) if flow == "source_to_target" else (0, 1)
        if weak:
            self._ei = weakref.ref(edge_index)
        else:
            self._ei = lambda ei=edge_index: ei
        self.n_dst, self.n_src = int(n_dst), int(n_src)
        self.chunk = chunk
        self.target_tasks = target_tasks
        self._dst = None
        self._src = None
        # attention-dropout keys: None = the edge's id in this edge list; a
        # shard's local graph sets the GLOBAL edge ids (dist.ShardedGraph)
        self.edge_key = None
        self._drop_ids = {}

    def drop_ids(self, side):
        """Per-slot attention-dropout keys (int32) of the 'dst' CSR (the forward)
        or the 'src' CSR (the transposed backward): each slot's edge id in this
        edge list, or edge_key of it.  The keep mask is then a function of the
        edge, not of where a CSR puts it (ABI 7 drop_ids)."""
        ids = self._drop_ids.get(side)
        if ids is None:
            csr = self.dst if side == "dst" else self.src
            E = csr.n_edges
            if self.edge_key is None:
                ids = csr.eid                                    # int32 edge ids, slot order
            else:
                ids = self.edge_key[csr.eid[:E].long()].to(torch.int32).contiguous() if E else csr.eid
            self._drop_ids[side] = ids
        return ids

    def _edge_index(self):
        ei = self._ei()
        if ei is None:
            raise RuntimeError("mi355_mp: edge_index was freed before its CSR was built")
        return ei

    @property
    def dst(self):
        if self._dst is None:
            ei = self._edge_index()
            self._dst = CSR(ei[self.i], ei[self.j], self.n_dst, self.n_src, self.chunk,
                            target_tasks=self.target_tasks)
        return self._dst

    @property
    def src(self):
        if self._src is None:
            ei = self._edge_index()
            self._src = CSR(ei[self.j], ei[self.i], self.n_src, self.n_dst, self.chunk,
                            target_tasks=self.target_tasks)
        return self._src

    def src_with_dst_slots(self):
        """The src CSR with the struct variant 'dst_slot': its per-slot id array
        holds, for each src slot, the slot of the same edge in the dst CSR, so a
        pass over the src CSR can write per-edge values straight into dst-CSR
        order (mp_gat_backward_f32's de)."""
        src = self.src
        if "dst_slot" not in getattr(src, "_extra", {}):
            dst = self.dst
            E = dst.n_edges
            inv = torch.empty(max(E, 1), dtype=torch.int32, device=dst.device)
            if E:
                inv[dst.eid[:E].long()] = torch.arange(E, dtype=torch.int32, device=dst.device)
            pos = src.to_csr_order(inv.view(torch.float32)).view(torch.int32)  # bit copy: pos[k] = inv[eid[k]]
            src.add_gather("dst_slot", src.col, src.n_other, eid=pos)
        return src


class _Cache:
    """id(tensor) -> value, invalidated by the tensor's version counter or death."""

    def __init__(self):
        self._d = {}

    def get(self, t, extra, factory, valid=None):
        if t._base is not None:  # a view (e.g. edge_index[1]): key on its base tensor
            extra = (extra, t.storage_offset(), tuple(t.stride()), tuple(t.shape))
            t = t._base
        k = (id(t), extra)
        hit = self._d.get(k)
        if hit is not None and hit[0] == t._version and (valid is None or valid(hit[1])):
            return hit[1]
        val = factory()
        if hit is None:
            try:
                weakref.finalize(t, self._drop, id(t))
            except TypeError:  # pragma: no cover - non-weakrefable input
                return val
        self._d[k] = (t._version, val)
        return val

    def _drop(self, tid):
        for k in [k for k in self._d if k[0] == tid]:
            del self._d[k]

    def clear(self):
        self._d.clear()


_graph_cache = _Cache()
_index_cache = _Cache()


def graph_for(edge_index, n_dst, n_src, flow="source_to_target", target_tasks=None):
    """Cached Graph for an edge_index tensor (rebuilt if it is modified in place)."""
    return _graph_cache.get(edge_index, (int(n_dst), int(n_src), flow, target_tasks),
                            lambda: Graph(edge_index, n_dst, n_src, flow, weak=True, target_tasks=target_tasks))


def csr_for_index(index, n_rows):
    """Cached CSR of a bare 1-D index (torch_scatter path: gathers message rows)."""
    return _index_cache.get(index, int(n_rows),
                            lambda: CSR(index.to(torch.int64), None, n_rows, index.numel()))


_order_cache = _Cache()


def in_csr_order(csr, edge_values):
    """Per-edge fp32 values permuted into ``csr``'s slot order, cached on the
    value tensor (identity + version) for this CSR: a cached GCN norm is
    permuted once, not on every forward and backward."""
    v = edge_values.to(torch.float32)
    if v is not edge_values or v.requires_grad:
        return csr.to_csr_order(v.detach())
    ref = weakref.ref(csr)
    val = _order_cache.get(v, (id(csr), csr.n_edges), lambda: (ref, csr.to_csr_order(v.detach())),
                           valid=lambda h: h[0]() is csr)
    return val[1]


def clear_caches():
    _graph_cache.clear()
    _index_cache.clear()
    _order_cache.clear()
