"""The examples/ scripts (the reference's example programs on synthetic data of
the same shapes) run end to end on the engine and learn."""
import importlib.util
import math
import os

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location("example_" + name, os.path.join(ROOT, "examples", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_example_gcn_cora_shaped():
    import torch
    torch.manual_seed(0)   # weights and dropout masks (the example itself is unseeded, as the reference's)
    losses = _load("gcn").main(["--epochs", "100"])
    # the Cora-shaped graph has random labels: the model can only fit the training
    # split, and dropout keeps the per-epoch loss noisy -- judge the last 10 epochs
    assert all(math.isfinite(v) for v in losses) and min(losses[-10:]) < 0.85 * losses[0], losses[::10]


def test_example_ppi_gat():
    import torch
    torch.manual_seed(0)
    losses = _load("ppi").main(["--epochs", "2", "--train-graphs", "3"])
    assert all(math.isfinite(v) for v in losses) and losses[-1] < losses[0]


def test_example_data_parallel():
    import torch
    torch.manual_seed(0)
    losses = _load("data_parallel").main(["--epochs", "3", "--graphs", "512"])
    assert all(math.isfinite(v) for v in losses) and losses[-1] < losses[0]
