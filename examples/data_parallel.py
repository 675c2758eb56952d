"""The reference's examples/data_parallel.py pattern: nn.DataParallel over the
lists a DataListLoader yields, global mean pooling, graph classification.
The reference model uses SplineConv on MNISTSuperpixels (neither is on this
engine's path nor downloadable offline); the same loop runs here with a GCN
on synthetic superpixel-sized graphs (75 nodes, 1 feature, 10 classes).

    PYTHONPATH=pytorch_geometric-1_amd python examples/data_parallel.py [--epochs 3]
"""
import argparse
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_ROOT, "pytorch_geometric-1_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch_geometric.data import Data, DataListLoader  # noqa: E402
from torch_geometric.nn import DataParallel, GCNConv, global_mean_pool  # noqa: E402
from mi355_mp.graphgen import powerlaw_edge_index  # noqa: E402


def superpixel_like(n_graphs, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(n_graphs):
        y = int(torch.randint(0, 10, (1,), generator=g))
        x = torch.rand(75, 1, generator=g) + 0.1 * y
        out.append(Data(x=x, edge_index=powerlaw_edge_index(75, 600, seed=seed * 100000 + i), y=torch.tensor([y])))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--graphs", type=int, default=2048)
    args = ap.parse_args(argv)
    dataset = superpixel_like(args.graphs, 7)
    loader = DataListLoader(dataset, batch_size=256, shuffle=True)

    class Net(torch.nn.Module):
        def __init__(self):
            super(Net, self).__init__()
            self.conv1 = GCNConv(1, 32)
            self.conv2 = GCNConv(32, 64)
            self.lin1 = torch.nn.Linear(64, 128)
            self.lin2 = torch.nn.Linear(128, 10)

        def forward(self, data):
            x = F.elu(self.conv1(data.x, data.edge_index))
            x = F.elu(self.conv2(x, data.edge_index))
            x = global_mean_pool(x, data.batch)
            x = F.elu(self.lin1(x))
            return F.log_softmax(self.lin2(x), dim=1)

    model = Net()
    print("Let's use", torch.cuda.device_count(), "GPUs!")
    model = DataParallel(model)
    device = torch.device("cuda:0")
    model = model.to(device)
    optimizer = torch.optim.Adam(model.parameters(), lr=0.01)
    losses = []
    for _ in range(args.epochs):
        for data_list in loader:
            optimizer.zero_grad()
            output = model(data_list)
            y = torch.cat([data.y for data in data_list]).to(output.device)
            loss = F.nll_loss(output, y)
            loss.backward()
            optimizer.step()
            losses.append(float(loss.detach()))
        print("Outside Model: num graphs: {}, loss {:.4f}".format(output.size(0), losses[-1]))
    return losses


if __name__ == "__main__":
    main()
