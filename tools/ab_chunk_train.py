"""GCN / GAT layer forward + backward at two merge-path task targets (the
default auto_chunk rule replaced by a task-count target), one process:
python tools/ab_chunk_train.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    import mi355_mp
    from mi355_mp import graph
    import bench_configs
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    orig = graph.auto_chunk
    for target in (100_000, 50_000, 100_000, 50_000):
        graph.auto_chunk = lambda r, e, t=None, _T=target: orig(r, e, _T if t is None else t)
        graph.clear_caches()
        print("TARGET_TASKS", target, flush=True)
        for c in ("c3train", "c2train"):
            getattr(bench_configs, c)(dev)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
