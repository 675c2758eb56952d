"""``torch_geometric.nn.DataParallel``: replicas over a list of small graphs
(/root/reference/ConvexPruning.py:530,559 and
/root/reference/examples/data_parallel.py:35-49).

Same contract as PyG 1.4.3: ``model(data_list)`` splits the list into one
contiguous chunk per device, balanced by node count, batches each chunk with
``Batch.from_data_list`` on that device (collated there: one copy per key,
index offsets and batch vectors by device kernels), runs the replicas
(``torch.nn.DataParallel`` machinery: parameters broadcast over RCCL, one host
thread per device) and gathers the outputs on ``output_device``.  Every
replica's aggregations run on the native kernels of its own device.

This is the reference's single-process API, kept for drop-in use.  The
MI355X scaling path for one large graph is one process per GPU
(``mi355_mp.dist``); for many small graphs, one process per GPU with a
``DistributedSampler`` over the graph list avoids the per-step parameter
broadcast this class performs.
"""
import torch
from torch.nn.parallel import DataParallel as _TorchDataParallel

from ..data import Batch


class DataParallel(_TorchDataParallel):
    def __init__(self, module, device_ids=None, output_device=None):
        super(DataParallel, self).__init__(module, device_ids, output_device)
        self.src_device = torch.device("cuda:{}".format(self.device_ids[0])) if self.device_ids else None

    def forward(self, data_list):
        if len(data_list) == 0:
            raise ValueError("DataParallel received an empty data list")
        if not self.device_ids or len(self.device_ids) == 1:
            dev = self.src_device if self.src_device is not None else torch.device("cpu")
            return self.module(Batch.from_data_list(data_list, device=dev))
        for t in self.module.parameters():
            if t.device != self.src_device:
                raise RuntimeError("module must have its parameters on device {} (device_ids[0]) but found one "
                                   "on device {}".format(self.src_device, t.device))
        inputs = self.scatter(data_list, self.device_ids)
        replicas = self.replicate(self.module, self.device_ids[:len(inputs)])
        outputs = self.parallel_apply(replicas, inputs, None)
        return self.gather(outputs, self.output_device)

    def scatter(self, data_list, device_ids):
        """Contiguous chunks with ~equal node counts, one per device (at most
        one chunk per graph)."""
        split = split_points([d.num_nodes for d in data_list], len(device_ids))
        chunks = []
        for k in range(len(split) - 1):
            lo, hi = split[k], split[k + 1]
            if hi > lo:  # non-empty chunks take consecutive devices (replicas live on device_ids[:len])
                dev = torch.device("cuda:{}".format(device_ids[len(chunks)]))
                chunks.append((Batch.from_data_list(data_list[lo:hi], device=dev),))
        return chunks


def split_points(num_nodes, n_dev):
    """Boundaries [0 = s_0 <= ... <= s_k = len] of contiguous chunks: graph i
    goes to the device whose share of the running node count contains the
    graph's midpoint."""
    n_dev = max(1, min(n_dev, len(num_nodes)))
    counts = torch.tensor(num_nodes, dtype=torch.float64)
    if counts.numel() == 0:
        return [0, 0]
    cum = counts.cumsum(0)
    total = float(cum[-1]) if float(cum[-1]) > 0 else 1.0
    owner = ((cum - 0.5 * counts) / total * n_dev).floor().clamp(0, n_dev - 1).to(torch.long)
    return [0] + [int((owner < k).sum()) for k in range(1, n_dev)] + [len(num_nodes)]
