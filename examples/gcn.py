"""The reference's examples/gcn.py (2-layer GCN on Cora, cached=True), unchanged
in its model and training loop, on a Cora-shaped synthetic graph: the
Planetoid download is not available offline (mi355_mp.graphgen.cora_like has
Cora's sizes: 2708 nodes, 10556 directed edges, 1433 row-normalised bag-of-
words features, 7 classes, the 140/500/1000 split).

    PYTHONPATH=pytorch_geometric-1_amd python examples/gcn.py [--epochs 200]
"""
import argparse
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_ROOT, "pytorch_geometric-1_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch_geometric.data import Data  # noqa: E402
from torch_geometric.nn import GCNConv  # noqa: E402
from mi355_mp.graphgen import cora_like  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=200)
    args = ap.parse_args(argv)
    d = cora_like()
    data = Data(x=d["x"], edge_index=d["edge_index"], y=d["y"], train_mask=d["train_mask"],
                val_mask=d["val_mask"], test_mask=d["test_mask"])
    num_features, num_classes = data.num_features, int(data.y.max()) + 1

    class Net(torch.nn.Module):
        def __init__(self):
            super(Net, self).__init__()
            self.conv1 = GCNConv(num_features, 16, cached=True)
            self.conv2 = GCNConv(16, num_classes, cached=True)

        def forward(self):
            x, edge_index = data.x, data.edge_index
            x = F.relu(self.conv1(x, edge_index))
            x = F.dropout(x, training=self.training)
            x = self.conv2(x, edge_index)
            return F.log_softmax(x, dim=1)

    device = torch.device("cuda")
    model, data = Net().to(device), data.to(device)
    optimizer = torch.optim.Adam(model.parameters(), lr=0.01, weight_decay=5e-4)

    def train():
        model.train()
        optimizer.zero_grad()
        loss = F.nll_loss(model()[data.train_mask], data.y[data.train_mask])
        loss.backward()
        optimizer.step()
        return float(loss.detach())

    def test():
        model.eval()
        logits, accs = model(), []
        for _, mask in data("train_mask", "val_mask", "test_mask"):
            pred = logits[mask].max(1)[1]
            accs.append(pred.eq(data.y[mask]).sum().item() / mask.sum().item())
        return accs

    best_val_acc = test_acc = 0
    losses = []
    for epoch in range(1, args.epochs + 1):
        losses.append(train())
        train_acc, val_acc, tmp_test_acc = test()
        if val_acc > best_val_acc:
            best_val_acc = val_acc
            test_acc = tmp_test_acc
        print("Epoch: {:03d}, Train: {:.4f}, Val: {:.4f}, Test: {:.4f}".format(epoch, train_acc, best_val_acc,
                                                                              test_acc))
    return losses


if __name__ == "__main__":
    main()
