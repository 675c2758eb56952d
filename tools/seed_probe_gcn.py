"""Seed sensitivity of examples/gcn.py (the GPU example test's criterion):
first loss, best of the last 10 epochs, ratio."""
import contextlib
import importlib.util
import io
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch_geometric-1_amd"))
import torch  # noqa: E402

for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    torch.manual_seed(seed)
    spec = importlib.util.spec_from_file_location("g", os.path.join(ROOT, "examples", "gcn.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    with contextlib.redirect_stdout(io.StringIO()):
        losses = m.main(["--epochs", "100"])
    print(seed, round(losses[0], 3), round(min(losses[-10:]), 3), round(min(losses[-10:]) / losses[0], 3), flush=True)
