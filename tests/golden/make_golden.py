"""Generates the golden fixtures in tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

Each fixture stores its INPUTS and the oracle's OUTPUTS; `compute(name,
inputs)` recomputes the outputs (tests/test_oracle.py checks the committed
files reproduce bit for bit; the GPU parity tests compare the HIP path with
them).  The oracle is the repo's own restatement (parity unpinned by the
reference, see oracle/__init__.py).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle import scatter_ref as S  # noqa: E402
from oracle import pyg_ref as P  # noqa: E402

OUTPUT_KEYS = {
    "kat_scatter": ["sum", "mean", "max", "argmax", "min", "argmin"],
    "powerlaw_agg": ["gsum", "gmean", "gmax", "gargmax", "gcn", "gat", "gat_alpha"],
    "cora_gcn": ["logp"],
}


def _t(a):
    return torch.from_numpy(np.asarray(a))


def compute(name, d):
    out = {}
    if name == "kat_scatter":
        src, idx, n = _t(d["src"]), _t(d["index"]), int(d["dim_size"])
        out["sum"] = S.scatter_sum(src, idx, n).numpy()
        out["mean"] = S.scatter_mean(src, idx, n).numpy()
        m, a = S.scatter_max(src, idx, n)
        out["max"], out["argmax"] = m.numpy(), a.numpy()
        m, a = S.scatter_min(src, idx, n)
        out["min"], out["argmin"] = m.numpy(), a.numpy()
    elif name == "powerlaw_agg":
        x, ei, w = _t(d["x"]), _t(d["edge_index"]), _t(d["w"])
        N = x.shape[0]
        out["gsum"] = S.gather_sum(x, ei[0], ei[1], w, N).numpy()
        out["gmean"] = S.scatter_mean(x[ei[0]], ei[1], N).numpy()
        m, a = S.gather_max(x, ei[0], ei[1], N)
        out["gmax"], out["gargmax"] = m.numpy(), a.numpy().astype(np.int32)
        out["gcn"] = P.gcn_conv(x, ei, _t(d["gcn_w"]), _t(d["gcn_b"])).numpy()
        o, _, alpha = P.gat_conv(x, ei, _t(d["gat_w"]), _t(d["gat_att"]), _t(d["gat_b"]),
                                 int(d["heads"]), int(d["out_channels"]), return_alpha=True)
        out["gat"], out["gat_alpha"] = o.numpy(), alpha.numpy()
    elif name == "cora_gcn":
        N, Fdim = int(d["num_nodes"]), int(d["num_features"])
        x = torch.zeros(N * Fdim, dtype=torch.float32)
        x[_t(d["x_flat_idx"])] = _t(d["x_val"])
        x = x.view(N, Fdim)
        ei = _t(d["edge_index"])
        h = torch.relu(P.gcn_conv(x, ei, _t(d["w1"]), _t(d["b1"])))
        h = P.gcn_conv(h, ei, _t(d["w2"]), _t(d["b2"]))
        out["logp"] = torch.log_softmax(h, dim=1).numpy()
    else:
        raise KeyError(name)
    return out


def make_inputs(name):
    if name == "kat_scatter":
        return dict(src=np.array([[1., -2.], [3., 5.], [-1., 0.], [3., 7.], [2., -3.]], np.float32),
                    index=np.array([0, 2, 0, 2, 3], np.int64), dim_size=np.array(5))
    if name == "powerlaw_agg":
        from mi355_mp.graphgen import powerlaw_edge_index
        g = torch.Generator().manual_seed(11)
        N, E, F, H, C = 1024, 16384, 64, 4, 16
        ei = powerlaw_edge_index(N, E, seed=11)
        x = torch.randn(N, F, generator=g)
        w = torch.rand(E, generator=g)
        gcn_w = (torch.rand(F, F, generator=g) * 2 - 1) * (6 / (2 * F)) ** 0.5
        gcn_b = torch.randn(F, generator=g) * 0.1
        gat_w = (torch.rand(F, H * C, generator=g) * 2 - 1) * (6 / (F + H * C)) ** 0.5
        gat_att = (torch.rand(1, H, 2 * C, generator=g) * 2 - 1) * (6 / (H + 2 * C)) ** 0.5
        gat_b = torch.randn(H * C, generator=g) * 0.1
        return dict(x=x.numpy(), edge_index=ei.numpy(), w=w.numpy(), gcn_w=gcn_w.numpy(),
                    gcn_b=gcn_b.numpy(), gat_w=gat_w.numpy(), gat_att=gat_att.numpy(),
                    gat_b=gat_b.numpy(), heads=np.array(H), out_channels=np.array(C))
    if name == "cora_gcn":
        from mi355_mp.graphgen import cora_like
        data = cora_like(seed=0)
        g = torch.Generator().manual_seed(12)
        Fdim, hid, K = data["x"].shape[1], 16, data["num_classes"]
        w1 = (torch.rand(Fdim, hid, generator=g) * 2 - 1) * (6 / (Fdim + hid)) ** 0.5
        w2 = (torch.rand(hid, K, generator=g) * 2 - 1) * (6 / (hid + K)) ** 0.5
        b1 = torch.randn(hid, generator=g) * 0.1
        b2 = torch.randn(K, generator=g) * 0.1
        flat = data["x"].reshape(-1)
        nz = torch.nonzero(flat).view(-1)
        return dict(num_nodes=np.array(data["x"].shape[0]), num_features=np.array(Fdim),
                    x_flat_idx=nz.numpy(), x_val=flat[nz].numpy(), edge_index=data["edge_index"].numpy(),
                    w1=w1.numpy(), b1=b1.numpy(), w2=w2.numpy(), b2=b2.numpy())
    raise KeyError(name)


def main():
    torch.set_num_threads(1)
    for name in OUTPUT_KEYS:
        inputs = make_inputs(name)
        outputs = compute(name, inputs)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **inputs, **outputs)
        size = os.path.getsize(os.path.join(HERE, name + ".npz"))
        print("%s: %d bytes" % (name, size))


if __name__ == "__main__":
    main()
