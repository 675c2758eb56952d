"""The reference's examples/ppi.py (3-layer GAT with skip connections, multi-
label BCE), unchanged in its model and training loop, on PPI-shaped synthetic
graphs (the PPI download is not available offline): 20 train / 2 val / 2 test
graphs of ~2,245 nodes, ~28 in-edges per node, 50 features, 121 binary labels.
Exercises the fused GAT forward and backward with heads=4 x 256 (concat) and
heads=6 x 121 (mean: the unfused backward form, C=121).

    PYTHONPATH=pytorch_geometric-1_amd python examples/ppi.py [--epochs 100]
"""
import argparse
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_ROOT, "pytorch_geometric-1_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch_geometric.data import Data, DataLoader  # noqa: E402
from torch_geometric.nn import GATConv  # noqa: E402
from mi355_mp.graphgen import powerlaw_edge_index  # noqa: E402


def ppi_like(n_graphs, seed, num_features=50, num_classes=121):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(n_graphs):
        n = int(torch.randint(1800, 2700, (1,), generator=g))
        ei = powerlaw_edge_index(n, 28 * n, seed=seed * 1000 + i)
        x = torch.randn(n, num_features, generator=g)
        y = (torch.rand(n, num_classes, generator=g) < 0.3).to(torch.float32)
        out.append(Data(x=x, edge_index=ei, y=y))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--train-graphs", type=int, default=20)
    args = ap.parse_args(argv)
    train_dataset = ppi_like(args.train_graphs, 1)
    val_dataset = ppi_like(2, 2)
    test_dataset = ppi_like(2, 3)
    num_features, num_classes = 50, 121
    train_loader = DataLoader(train_dataset, batch_size=1, shuffle=True)
    val_loader = DataLoader(val_dataset, batch_size=2, shuffle=False)
    test_loader = DataLoader(test_dataset, batch_size=2, shuffle=False)

    class Net(torch.nn.Module):
        def __init__(self):
            super(Net, self).__init__()
            self.conv1 = GATConv(num_features, 256, heads=4)
            self.lin1 = torch.nn.Linear(num_features, 4 * 256)
            self.conv2 = GATConv(4 * 256, 256, heads=4)
            self.lin2 = torch.nn.Linear(4 * 256, 4 * 256)
            self.conv3 = GATConv(4 * 256, num_classes, heads=6, concat=False)
            self.lin3 = torch.nn.Linear(4 * 256, num_classes)

        def forward(self, x, edge_index):
            x = F.elu(self.conv1(x, edge_index) + self.lin1(x))
            x = F.elu(self.conv2(x, edge_index) + self.lin2(x))
            x = self.conv3(x, edge_index) + self.lin3(x)
            return x

    device = torch.device("cuda")
    model = Net().to(device)
    loss_op = torch.nn.BCEWithLogitsLoss()
    optimizer = torch.optim.Adam(model.parameters(), lr=0.005)

    def train():
        model.train()
        total_loss = 0
        for data in train_loader:
            num_graphs = data.num_graphs
            data.batch = None
            data = data.to(device)
            optimizer.zero_grad()
            loss = loss_op(model(data.x, data.edge_index), data.y)
            total_loss += loss.item() * num_graphs
            loss.backward()
            optimizer.step()
        return total_loss / len(train_loader.dataset)

    def test(loader):
        model.eval()
        ys, preds = [], []
        for data in loader:
            ys.append(data.y)
            with torch.no_grad():
                out = model(data.x.to(device), data.edge_index.to(device))
            preds.append((out > 0).float().cpu())
        y, pred = torch.cat(ys, dim=0), torch.cat(preds, dim=0)
        tp = float((y * pred).sum())
        return 2 * tp / max(1.0, float(y.sum() + pred.sum()))   # micro-F1

    losses = []
    for epoch in range(1, args.epochs + 1):
        losses.append(train())
        val_f1 = test(val_loader)
        test_f1 = test(test_loader)
        print("Epoch: {:02d}, Loss: {:.4f}, Val: {:.4f}, Test: {:.4f}".format(epoch, losses[-1], val_f1, test_f1))
    return losses


if __name__ == "__main__":
    main()
