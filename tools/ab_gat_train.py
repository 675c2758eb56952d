"""In-process A/B of the GAT training forward (mp_gat_aggregate_train_f32) over
build variants (tools/variants/lib_*.so) on config 3 (RMAT21, heads=8, C=32),
next to the inference forward (mp_gat_aggregate_att_f32) of the first
variant.  Outputs, row statistics, out2 and row_s2 must be bitwise equal
across variants (rows in flight do not change the arithmetic); the inference
output must equal the training one.  Main stage timed with HIP events,
variants interleaved.
    python tools/ab_gat_train.py [--variants a,b,...]
"""
import argparse
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import mi355_mp
    from mi355_mp import _lib
    from mi355_mp.graph import Graph, GAT_TARGET_TASKS
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv._structure import gat_loops
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    N, H, C = 1 << 21, 8, 32
    ei = gat_loops(rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev), N)
    csr = Graph(ei, N, N, target_tasks=GAT_TARGET_TASKS).dst
    del ei
    vdir = os.path.join(ROOT, "tools", "variants")
    names = args.variants.split(",") if args.variants else sorted(
        os.path.basename(f)[4:-3] for f in glob.glob(os.path.join(vdir, "lib_*.so")))
    libs = {n: _lib.load(os.path.join(vdir, "lib_%s.so" % n)) for n in names}
    lib0 = libs[names[0]]
    gen = torch.Generator(device=dev).manual_seed(2)
    xw = torch.randn(N, H * C, device=dev, generator=gen)
    att = torch.randn(H, 2 * C, device=dev, generator=gen) * 0.1
    a_src = torch.empty(N, H, device=dev)
    a_dst = torch.empty(N, H, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    _lib.check(lib0.mp_gat_node_scores_f32(xw.data_ptr(), N, H, C, att.data_ptr(), a_src.data_ptr(),
                                           a_dst.data_ptr(), st), "scores")
    g = csr.struct("other")
    sb = lib0.mp_gat_train_slab_bytes(g, H, C)
    slab = torch.empty(sb, dtype=torch.uint8, device=dev)
    res = {n: (torch.empty(N, H * C, device=dev), torch.empty(N, H, 2, device=dev), torch.empty(N, H * C, device=dev),
               torch.empty(N, H, device=dev)) for n in names}
    inf = (torch.empty(N, H * C, device=dev), torch.empty(N, H, 2, device=dev))

    def launch(n, stages):
        o, s_, o2, s2 = res[n]
        _lib.check(libs[n].mp_gat_aggregate_train_f32(g, xw.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                      att.data_ptr(), H, C, 0.2, None, o.data_ptr(), H * C, None,
                                                      s_.data_ptr(),
                                                      o2.data_ptr(), s2.data_ptr(), slab.data_ptr(), sb, stages, st),
                   "train")

    def launch_inf(stages):
        _lib.check(lib0.mp_gat_aggregate_att_f32(g, xw.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(), att.data_ptr(),
                                                 H, C, 0.2, None, inf[0].data_ptr(), H * C, inf[1].data_ptr(),
                                                 slab.data_ptr(), sb, stages, st), "inference")
    for n in names:
        launch(n, _lib.MP_STAGE_ALL)
    launch_inf(_lib.MP_STAGE_ALL)
    torch.cuda.synchronize()
    same = {n: all(torch.equal(a, b) for a, b in zip(res[n], res[names[0]])) for n in names}
    inf_same = torch.equal(inf[0], res[names[0]][0]) and torch.equal(inf[1], res[names[0]][1])
    times = {n: [] for n in names + ["inference"]}
    for _ in range(args.rounds):
        for n in names + ["inference"]:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                if n == "inference":
                    launch_inf(_lib.MP_STAGE_MAIN)
                else:
                    launch(n, _lib.MP_STAGE_MAIN)
            b.record()
            torch.cuda.synchronize()
            times[n].append(a.elapsed_time(b) / 10)
    for n in names + ["inference"]:
        t = sorted(times[n])
        print(json.dumps({"variant": n, "median_ms": round(t[len(t) // 2], 4), "min_ms": round(t[0], 4),
                          "bitwise_equal_to_first": same.get(n, inf_same)}), flush=True)


if __name__ == "__main__":
    main()
