"""FETCH_SIZE calibration for the aggregation kernel's own access pattern
(MI355X_MICROARCH.md 'HBM': widths other than 16 B/lane are uncalibrated).

Known byte count: N = 2^21 rows, each with exactly ONE in-edge from a
distinct source (a random permutation), F = 256: one launch reads every x row
exactly once (2 GiB, far beyond L2 and the Infinity Cache) plus col, weight,
rowptr and the schedule (~30 MB), and writes out (2 GiB).  Run under
  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_agg_(main|flat)" -- python3 tools/pmc_calibrate.py
with EXP_LIB=<variant .so> to pick the kernel shape; the expected bytes are
printed for the summary."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graph import Graph
    lib = mi355_mp.load_native()
    if os.environ.get("EXP_LIB"):
        lib = _lib.load(os.environ["EXP_LIB"])
    dev = torch.device("cuda", 0)
    N, F = 1 << 21, 256
    g = torch.Generator(device=dev).manual_seed(5)
    src = torch.randperm(N, generator=g, device=dev)
    ei = torch.stack([src, torch.arange(N, device=dev)])
    csr = Graph(ei, N, N).dst
    w = torch.rand(N, device=dev, generator=g)
    x = torch.randn(N, F, device=dev, generator=g)
    out = torch.empty(N, F, device=dev)
    s = csr.struct("other")
    sb = lib.mp_aggregate_slab_bytes(s, F, 0)
    slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    flush = torch.empty(1 << 29, dtype=torch.uint8, device=dev)   # 512 MiB: evicts the Infinity Cache
    for _ in range(5):
        flush.fill_(1)
        _lib.check(lib.mp_aggregate_f32(s, w.data_ptr(), x.data_ptr(), F, F, 0, 0, None, out.data_ptr(), F, None,
                                        slab.data_ptr(), sb, _lib.MP_STAGE_MAIN, st), "agg")
    torch.cuda.synchronize()
    x_bytes = N * F * 4
    idx_bytes = N * 4 * 3 + (csr.n_waves + 1) * 8
    print(json.dumps({"x_read_bytes": x_bytes, "index_bytes": idx_bytes, "expected_read_bytes": x_bytes + idx_bytes,
                      "out_write_bytes": N * F * 4}))


if __name__ == "__main__":
    main()
