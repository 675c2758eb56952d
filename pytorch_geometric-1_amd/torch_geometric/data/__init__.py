"""Graph containers and mini-batching for the replica path.

PyG 1.4.3's ``torch_geometric.data`` is out of scope as a subsystem (datasets,
downloads, transforms).  What the reference's multi-GPU path needs is kept:
``Data`` (attribute container), ``Batch.from_data_list`` (block-diagonal
mini-batch: node tensors concatenated, ``edge_index`` offset by the running
node count, a ``batch`` vector of graph ids), ``DataLoader`` (yields
``Batch``) and ``DataListLoader`` (yields lists, for ``nn.DataParallel``).
Callers: /root/reference/ConvexPruning.py:12,460-517,530 and
/root/reference/examples/data_parallel.py:25-49.

Batching semantics follow PyG 1.4.3: a key is concatenated along dim -1 when
its name contains ``index`` or ``face`` (and offset by ``num_nodes``),
along dim 0 otherwise; bool tensors are never offset.
"""
import re

import torch
import torch.utils.data

__all__ = ["Data", "Batch", "DataLoader", "DataListLoader"]


class Data(object):
    """A graph: ``x`` [N, F], ``edge_index`` [2, E], optional ``edge_attr``,
    ``y``, ``pos`` and any other attribute passed as a keyword."""

    def __init__(self, x=None, edge_index=None, edge_attr=None, y=None, pos=None, norm=None, face=None,
                 **kwargs):
        self.x = x
        self.edge_index = edge_index
        self.edge_attr = edge_attr
        self.y = y
        self.pos = pos
        self.norm = norm
        self.face = face
        for key, item in kwargs.items():
            if key == "num_nodes":
                self.__num_nodes__ = item
            else:
                self[key] = item

    @classmethod
    def from_dict(cls, dictionary):
        data = cls()
        for key, item in dictionary.items():
            data[key] = item
        return data

    def __getitem__(self, key):
        return getattr(self, key, None)

    def __setitem__(self, key, value):
        setattr(self, key, value)

    @property
    def keys(self):
        return [k for k in self.__dict__.keys() if self[k] is not None and not k.startswith("__")]

    def __len__(self):
        return len(self.keys)

    def __contains__(self, key):
        return key in self.keys

    def __iter__(self):
        for key in sorted(self.keys):
            yield key, self[key]

    def __call__(self, *keys):
        for key in sorted(self.keys) if not keys else keys:
            if key in self:
                yield key, self[key]

    def __cat_dim__(self, key, value):
        return -1 if re.search("(index|face)", key) else 0

    def __inc__(self, key, value):
        return self.num_nodes if re.search("(index|face)", key) else 0

    @property
    def num_nodes(self):
        n = self.__dict__.get("__num_nodes__")
        if n is not None:
            return n
        for key, item in self("x", "pos", "norm", "batch"):
            return item.size(self.__cat_dim__(key, item))
        if self.face is not None:
            return int(self.face.max()) + 1
        if self.edge_index is not None:
            return int(self.edge_index.max()) + 1 if self.edge_index.numel() else 0
        return None

    @num_nodes.setter
    def num_nodes(self, num_nodes):
        self.__num_nodes__ = num_nodes

    @property
    def num_edges(self):
        for key, item in self("edge_index", "edge_attr"):
            return item.size(self.__cat_dim__(key, item))
        return None

    @property
    def num_node_features(self):
        if self.x is None:
            return 0
        return 1 if self.x.dim() == 1 else self.x.size(1)

    @property
    def num_features(self):
        return self.num_node_features

    @property
    def num_edge_features(self):
        if self.edge_attr is None:
            return 0
        return 1 if self.edge_attr.dim() == 1 else self.edge_attr.size(1)

    def is_coalesced(self):
        ei = self.edge_index
        n = self.num_nodes
        key = ei[0] * n + ei[1]
        return bool((key[1:] > key[:-1]).all()) if key.numel() > 1 else True

    def contains_self_loops(self):
        return bool((self.edge_index[0] == self.edge_index[1]).any())

    def contains_isolated_nodes(self):
        n = self.num_nodes
        seen = torch.zeros(n, dtype=torch.bool, device=self.edge_index.device)
        seen[self.edge_index.reshape(-1)] = True
        return not bool(seen.all())

    def is_undirected(self):
        ei = self.edge_index
        n = self.num_nodes
        a = torch.unique(ei[0] * n + ei[1])
        b = torch.unique(ei[1] * n + ei[0])
        return a.numel() == b.numel() and bool((a == b).all())

    def apply(self, func, *keys):
        for key, item in self(*keys):
            if torch.is_tensor(item):
                self[key] = func(item)
        return self

    def contiguous(self, *keys):
        return self.apply(lambda x: x.contiguous(), *keys)

    def to(self, device, *keys, **kwargs):
        return self.apply(lambda x: x.to(device, **kwargs), *keys)

    def clone(self):
        return self.__class__.from_dict({k: v.clone() if torch.is_tensor(v) else v for k, v in self.__dict__.items()})

    def __repr__(self):
        info = ["{}={}".format(key, list(item.size()) if torch.is_tensor(item) else item) for key, item in self]
        return "{}({})".format(self.__class__.__name__, ", ".join(info))


class Batch(Data):
    """A block-diagonal mini-batch of graphs with a ``batch`` vector mapping
    every node to its graph."""

    def __init__(self, batch=None, **kwargs):
        super(Batch, self).__init__(**kwargs)
        self.batch = batch

    @staticmethod
    def from_data_list(data_list, follow_batch=(), device=None):
        """device (extension, e.g. a replica's ``cuda:k``): collate straight onto
        that device -- each key's raw items concatenated and copied once, the
        per-graph index offsets and the batch vectors applied there by
        ``mp_segment_offset_i64`` / ``mp_segment_ids_i64`` -- with the same
        result as ``from_data_list(data_list, follow_batch).to(device)``."""
        keys = []
        for data in data_list:
            for k in data.keys:
                if k not in keys:
                    keys.append(k)
        assert "batch" not in keys
        if device is not None and torch.device(device).type == "cuda":
            return _collate_on_device(data_list, keys, follow_batch, torch.device(device))
        batch = Batch()
        parts = {k: [] for k in keys}
        for k in follow_batch:
            parts["{}_batch".format(k)] = []
        inc = {k: 0 for k in keys}
        graph_ids = []
        for i, data in enumerate(data_list):
            for k in keys:
                item = data[k]
                if item is None:
                    continue
                if torch.is_tensor(item) and item.dtype != torch.bool:
                    item = item + inc[k]
                inc[k] = inc[k] + data.__inc__(k, item)
                parts[k].append(item)
                if k in follow_batch:
                    size = item.size(data.__cat_dim__(k, item))
                    parts["{}_batch".format(k)].append(torch.full((size,), i, dtype=torch.long))
            n = data.num_nodes
            if n is not None:
                graph_ids.append(torch.full((n,), i, dtype=torch.long))
        ref = data_list[0] if data_list else Data()
        for k, items in parts.items():
            if not items:
                continue
            first = items[0]
            if torch.is_tensor(first):
                dim = ref.__cat_dim__(k, first) if not k.endswith("_batch") else 0
                batch[k] = torch.cat(items, dim=dim)
            elif isinstance(first, (int, float)):
                batch[k] = torch.tensor(items)
            else:
                batch[k] = items
        batch.batch = torch.cat(graph_ids) if graph_ids else torch.empty(0, dtype=torch.long)
        return batch.contiguous()

    @property
    def num_graphs(self):
        return int(self.batch[-1]) + 1 if self.batch is not None and self.batch.numel() else 0

    def to_data_list(self):
        raise NotImplementedError("mi355_mp: Batch.to_data_list is not part of the replica path")


def _seg_starts(sizes, dev):
    starts = torch.zeros(len(sizes) + 1, dtype=torch.int64)
    if sizes:
        starts[1:] = torch.tensor(sizes, dtype=torch.int64).cumsum(0)
    # a blocking copy: an asynchronous one from this pageable temporary could
    # read it after it is freed
    return starts.to(dev)


def _graph_ids(sizes, dev, lib, st):
    """torch.cat([torch.full((n_g,), g) for g, n_g in enumerate(sizes)]) on dev."""
    from mi355_mp import _lib
    n = int(sum(sizes))
    ids = torch.empty(n, dtype=torch.long, device=dev)
    if n:
        starts = _seg_starts(sizes, dev)
        _lib.check(lib.mp_segment_ids_i64(ids.data_ptr(), n, starts.data_ptr(), len(sizes), st), "mp_segment_ids_i64")
    return ids


def _to_dev(t, dev):
    if t.device == dev:
        return t.contiguous()
    if t.device.type == "cpu" and t.numel():
        return t.contiguous().pin_memory().to(dev, non_blocking=True)
    return t.to(dev)


def _collate_on_device(data_list, keys, follow_batch, dev):
    """Batch.from_data_list(data_list, follow_batch).to(dev), collated on dev
    (see Batch.from_data_list)."""
    from mi355_mp import _lib
    lib = _lib.load()
    st = _lib.stream_ptr(dev)
    batch = Batch()
    ref = data_list[0] if data_list else Data()
    for k in keys:
        items, incs, gids = [], [], []
        inc = 0
        for i, data in enumerate(data_list):
            item = data[k]
            if item is None:
                continue
            items.append(item)
            incs.append(inc)
            gids.append(i)
            inc = inc + data.__inc__(k, item)
        if not items:
            continue
        first = items[0]
        if not torch.is_tensor(first):
            batch[k] = torch.tensor(items, device=dev) if isinstance(first, (int, float)) else items
            continue
        dim = ref.__cat_dim__(k, first)
        d = _to_dev(torch.cat([t if t.device == items[0].device else t.to(items[0].device) for t in items], dim=dim),
                    dev)
        dim = dim % d.dim() if d.dim() else 0
        sizes = [int(t.size(dim)) if t.dim() else 1 for t in items]
        if first.dtype != torch.bool:
            if any(incs):
                if d.dtype == torch.int64 and d.dim() in (1, 2) and dim == d.dim() - 1 and d.is_contiguous():
                    # item + cumsum[key] per graph, on the device
                    rows = 1 if d.dim() == 1 else d.shape[0]
                    n = d.shape[-1]
                    # both held in names until the launch is queued (a temporary's block
                    # would go back to the caching allocator before the next allocation)
                    starts = _seg_starts(sizes, dev)
                    inc_d = torch.tensor(incs, dtype=torch.int64).to(dev)
                    _lib.check(lib.mp_segment_offset_i64(d.data_ptr(), n, rows, n, starts.data_ptr(), inc_d.data_ptr(),
                                                         len(items), st), "mp_segment_offset_i64")
                else:
                    offs = torch.repeat_interleave(torch.tensor(incs, device=dev), torch.tensor(sizes, device=dev))
                    shape = [1] * d.dim()
                    shape[dim] = -1
                    d = d + offs.view(shape).to(d.dtype)
            elif d.is_floating_point() or d.is_complex():
                d = d + 0  # the reference's item + 0 (-0.0 becomes +0.0)
        batch[k] = d
        if k in follow_batch:
            fb = [0] * len(data_list)
            for g, sz in zip(gids, sizes):
                fb[g] = sz
            # graphs without the key contribute no entries (as upstream's per-item torch.full)
            batch["{}_batch".format(k)] = _graph_ids(fb, dev, lib, st)
    counts = [0] * len(data_list)
    for i, data in enumerate(data_list):
        n = data.num_nodes
        counts[i] = 0 if n is None else int(n)
    batch.batch = _graph_ids(counts, dev, lib, st)
    return batch.contiguous()


class DataLoader(torch.utils.data.DataLoader):
    """Mini-batches of graphs as ``Batch`` objects."""

    def __init__(self, dataset, batch_size=1, shuffle=False, follow_batch=(), **kwargs):
        super(DataLoader, self).__init__(
            dataset, batch_size, shuffle, collate_fn=lambda data_list: Batch.from_data_list(data_list, follow_batch),
            **kwargs)


class DataListLoader(torch.utils.data.DataLoader):
    """Mini-batches as plain lists of ``Data`` (for ``nn.DataParallel``)."""

    def __init__(self, dataset, batch_size=1, shuffle=False, **kwargs):
        super(DataListLoader, self).__init__(dataset, batch_size, shuffle,
                                             collate_fn=lambda data_list: data_list, **kwargs)
