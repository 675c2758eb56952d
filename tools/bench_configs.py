"""Measures the BASELINE.md configs other than the bench.py headline:

  c3  same RMAT graph, GATConv heads=8 C=32 (fused online-softmax aggregation)
  c4  Reddit-scale power-law N=232,965 E=114,615,892, F=256, aggr='max'
      (segmented max + int64 first-index argmax)
  c5  ogbn-products-scale N=2,449,029 E=123,718,280 GCNConv F=256 (1 GPU)

For each: dominant-kernel time (HIP events over back-to-back launches),
edges/s, algorithmic GB/s with BASELINE.md's byte formulas (no cache
credit), compulsory-byte HBM fraction, and -- with --cpu-baseline -- the
reference algorithm timed on the host on a bounded sample of the same edges
(the CPU baseline leg, like bench.py's, is the only
place the oracle is used).  One JSON line per config.
    python tools/bench_configs.py [--configs c3,c4,c5] [--cpu-baseline]
"""
import argparse
import time
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch_geometric-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from bench import cpu_info  # noqa: E402

PEAK = 8000.0
CPU_BASELINE = False


def timed(fn, reps=10, rounds=3):
    fn()
    torch.cuda.synchronize()
    per = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        per.append(a.elapsed_time(b) / reps)
    return sorted(per)[len(per) // 2]


def report(name, desc, E, N, bpe, bpn, ms_main, ms_total, extra=None, comp_bytes=None, cpu=None):
    alg = E * bpe + N * bpn
    gbs = alg / (ms_main * 1e-3) / 1e9
    line = {"config": name, "desc": desc, "num_nodes": N, "num_edges": E,
            "edges_per_s": E / (ms_total * 1e-3), "main_kernel_ms": ms_main, "aggregate_ms": ms_total,
            "algorithmic_bytes": alg, "algorithmic_GBps_no_cache_credit": gbs}
    if comp_bytes is not None:
        line["compulsory_bytes"] = comp_bytes
        line["roofline_frac_compulsory"] = comp_bytes / (ms_main * 1e-3) / 1e9 / PEAK
    if extra:
        line.update(extra)
    if cpu is not None:
        line["cpu_baseline"] = cpu
        line["gpu_over_cpu"] = line["edges_per_s"] / cpu["value"]
    print(json.dumps(line), flush=True)


def _cpu_threads():
    model, threads, machine = cpu_info()
    torch.set_num_threads(threads)
    return model, threads, machine


def cpu_sum_baseline(ei, w, x, sample):
    """GCN sum: index_select -> norm * x_j -> scatter_add_,
    4M-edge chunks in original edge order."""
    import time
    model, threads, machine = _cpu_threads()
    E = min(sample, ei.shape[1])
    eic, wc, xc = ei[:, :E].cpu(), w[:E].cpu(), x.cpu()
    out = torch.zeros_like(xc)
    t0 = time.perf_counter()
    for s0 in range(0, E, 4_000_000):
        e1 = min(E, s0 + 4_000_000)
        msg = wc[s0:e1].view(-1, 1) * xc.index_select(0, eic[0, s0:e1])
        out.scatter_add_(0, eic[1, s0:e1].view(-1, 1).expand_as(msg), msg)
    dt = time.perf_counter() - t0
    return {"value": E / dt, "unit": "edges/s", "cores": threads, "kind": "port", "cpu_model": model,
            "machine_cpus": machine, "sample": "first %d of %d edges, torch CPU index_select+mul+scatter_add_ "
            "(4M-edge chunks), %.1f s" % (E, ei.shape[1], dt)}


def cpu_max_baseline(ei, x, sample):
    """max + argmax: index_select (threaded) then torch_scatter 2.0.4's serial
    CPU loop (scatter_cpu.cpp, restated in oracle/scatter_loop.c), 4M-edge chunks
    accumulated through `out` (the loop's has_out path)."""
    import time
    from oracle import scatter_ref as S  # CPU-baseline leg only
    model, threads, machine = _cpu_threads()
    E = min(sample, ei.shape[1])
    eic, xc = ei[:, :E].cpu(), x.cpu()
    N, F = xc.shape
    out = torch.full((N, F), -3.4028234663852886e38)
    t_sel = t_loop = 0.0
    for s0 in range(0, E, 4_000_000):
        e1 = min(E, s0 + 4_000_000)
        t0 = time.perf_counter()
        msg = xc.index_select(0, eic[0, s0:e1])
        t1 = time.perf_counter()
        out, _ = S.scatter_loop(msg, eic[1, s0:e1], N, "max", out=out)
        t_loop += time.perf_counter() - t1
        t_sel += t1 - t0
    dt = t_sel + t_loop
    return {"value": E / dt, "unit": "edges/s", "cores": threads, "kind": "port", "cpu_model": model,
            "machine_cpus": machine, "index_select_s": t_sel, "serial_loop_s": t_loop,
            "sample": "first %d of %d edges: torch index_select (%d threads) + serial scatter_max loop "
            "(1 thread, oracle/scatter_loop.c), %.1f s" % (E, ei.shape[1], threads, dt)}


def cpu_gat_baseline(ei, xw, att, H, C, sample):
    """GATConv's reference pipeline (oracle/pyg_ref.gat_conv after x @ W):
    x_i / x_j index_select, (cat[x_i, x_j] * att).sum(-1), leaky_relu,
    utils.softmax (serial scatter_max loop + scatter_add_), x_j * alpha,
    scatter_add_ -- on the first `sample` edges."""
    import time
    import torch.nn.functional as Fn
    from oracle import pyg_ref as P, scatter_ref as S  # CPU-baseline leg only
    model, threads, machine = _cpu_threads()
    E = min(sample, ei.shape[1])
    eic, h = ei[:, :E].cpu(), xw.cpu()
    N = h.shape[0]
    a = att.cpu()
    t0 = time.perf_counter()
    x_i = h.index_select(0, eic[1]).view(-1, H, C)
    x_j = h.index_select(0, eic[0]).view(-1, H, C)
    alpha = (torch.cat([x_i, x_j], dim=-1) * a).sum(dim=-1)
    alpha = Fn.leaky_relu(alpha, 0.2)
    alpha = P.softmax(alpha, eic[1], N)
    out = S.scatter_sum(x_j * alpha.view(-1, H, 1), eic[1], N)
    dt = time.perf_counter() - t0
    del out, x_i, x_j
    return {"value": E / dt, "unit": "edges/s", "cores": threads, "kind": "port", "cpu_model": model,
            "machine_cpus": machine, "sample": "first %d of %d edges, oracle GATConv pipeline (torch CPU ops + "
            "serial scatter_max loop in the softmax), %.1f s" % (E, ei.shape[1], dt)}


def c3(dev):
    from mi355_mp import _lib, ops
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn.conv._structure import gat_loops
    N, H, C = 1 << 21, 8, 32
    from mi355_mp.graph import GAT_TARGET_TASKS
    ei = gat_loops(rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev), N)
    graph = Graph(ei, N, N, target_tasks=GAT_TARGET_TASKS)   # as GATConv builds it
    csr = graph.dst
    g = torch.Generator(device=dev).manual_seed(2)
    xw = torch.randn(N, H * C, device=dev, generator=g)
    att = torch.randn(1, H, 2 * C, device=dev, generator=g) * 0.1
    bias = torch.randn(H * C, device=dev, generator=g) * 0.1
    lib = _lib.load()
    a_src = torch.empty(N, H, device=dev)
    a_dst = torch.empty(N, H, device=dev)
    att_c = att.reshape(H, 2 * C).contiguous()
    out = torch.empty(N, H * C, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    s = csr.struct("other")
    sb = lib.mp_gat_slab_bytes(s, H, C)
    slab = torch.empty(sb, dtype=torch.uint8, device=dev)

    def scores():
        _lib.check(lib.mp_gat_node_scores_f32(xw.data_ptr(), N, H, C, att_c.data_ptr(), a_src.data_ptr(),
                                              a_dst.data_ptr(), st), "scores")

    def agg(stages):
        # the GATConv forward path: a_src recomputed from the gathered rows (ops.GAT_OWN_A_SRC)
        _lib.check(lib.mp_gat_aggregate_att_f32(s, xw.data_ptr(), a_src.data_ptr(), a_dst.data_ptr(),
                                                att_c.data_ptr() if ops.GAT_OWN_A_SRC else None, H, C, 0.2,
                                                bias.data_ptr(), out.data_ptr(), H * C, None, slab.data_ptr(), sb,
                                                stages, st), "gat")
    stats = torch.empty(N, H, 2, device=dev)
    sr = csr.slot_rows()

    def agg2(stages):
        _lib.check(lib.mp_gat_softmax_aggregate_f32(s, sr.data_ptr(), xw.data_ptr(), a_src.data_ptr(),
                                                    a_dst.data_ptr(), H, C, 0.2, bias.data_ptr(), out.data_ptr(),
                                                    H * C, stats.data_ptr(), slab.data_ptr(), sb, stages, st),
                   "gat2")
    a_src2 = torch.empty(N, H, device=dev)
    a_dst2 = torch.empty(N, H, device=dev)

    def agg_nd(stages):
        # the node scores reduced in-kernel from each row's own xw (mp_gat_forward_f32, ops.GAT_NODE_SCORES_IN_KERNEL)
        _lib.check(lib.mp_gat_forward_f32(s, xw.data_ptr(), att_c.data_ptr(), H, C, 0.2, bias.data_ptr(),
                                          out.data_ptr(), H * C, a_src2.data_ptr(), a_dst2.data_ptr(), None,
                                          slab.data_ptr(), sb, stages, st), "gat_nd")
    scores()
    ms_scores = timed(scores)
    E = csr.n_edges
    # one pass (online softmax, one 256-feature tile)
    ms_main1 = timed(lambda: agg(_lib.MP_STAGE_MAIN))
    ms_fix1 = timed(lambda: agg(_lib.MP_STAGE_FIXUP))
    agg(_lib.MP_STAGE_ALL)
    one = out.clone()
    ms_main_nd = timed(lambda: agg_nd(_lib.MP_STAGE_MAIN))
    ms_fix_nd = timed(lambda: agg_nd(_lib.MP_STAGE_FIXUP))
    agg_nd(_lib.MP_STAGE_ALL)
    nd_equal = bool(torch.equal(out, one)) and bool(torch.equal(a_src2, a_src)) and bool(torch.equal(a_dst2, a_dst))
    # two pass (row statistics, then 64-feature tiles with the reference's alpha)
    ms_stats = timed(lambda: agg2(_lib.MP_STAGE_STATS))
    ms_main = timed(lambda: agg2(_lib.MP_STAGE_MAIN))
    ms_fix = timed(lambda: agg2(_lib.MP_STAGE_FIXUP))
    agg2(_lib.MP_STAGE_ALL)
    diff = ((out - one).abs().max() / one.abs().max()).item()
    del one
    path = "two_pass" if ops.gat_two_pass(csr, H, C) else "one_pass"
    tot1 = ms_main1 + ms_fix1 + ms_scores
    tot2 = ms_stats + ms_main + ms_fix + ms_scores
    tot_nd = ms_main_nd + ms_fix_nd
    nd_info = {"main_kernel_ms": ms_main_nd, "fixup_ms": ms_fix_nd, "aggregate_ms": tot_nd,
               "bitwise_equal_to_separate_scores": nd_equal}
    # compulsory: xw read once + a_src/a_dst + col + rowptr + out written once
    comp = N * H * C * 4 * 2 + N * H * 8 + E * 4 + (N + 1) * 4
    cpu = cpu_gat_baseline(ei, xw, att, H, C, 3_000_000) if CPU_BASELINE else None
    if path == "two_pass":
        report("c3", "RMAT21 GATConv heads=8 C=32: softmax row-stat passes + 64-feature-tile aggregation with the "
               "reference's alpha + bias (GATConv forward path)",
               E, N, 4 * H * C + 8 + 4 * H, 4 * H * C + 12 * H + 4, ms_main, tot2,
               {"stats_ms": ms_stats, "fixup_ms": ms_fix, "node_scores_ms": ms_scores, "n_split": csr.n_split,
                "one_pass": {"main_kernel_ms": ms_main1, "fixup_ms": ms_fix1, "aggregate_ms": tot1},
                "max_rel_diff_two_vs_one_pass": diff}, comp, cpu)
    elif ops.GAT_NODE_SCORES_IN_KERNEL:
        report("c3", "RMAT21 GATConv heads=8 C=32, fused node scores + leaky_relu+softmax(+1e-16)+aggregate+bias "
               "(mp_gat_forward_f32, the GATConv forward path)",
               E, N, 4 * H * C + 4 + 4 * H, 4 * H * C + 4 * H + 4, ms_main_nd, tot_nd,
               {"fixup_ms": ms_fix_nd, "n_split": csr.n_split, "bitwise_equal_to_separate_scores": nd_equal,
                "separate_node_scores": {"node_scores_ms": ms_scores, "main_kernel_ms": ms_main1, "fixup_ms": ms_fix1,
                                         "aggregate_ms": tot1},
                "two_pass": {"stats_ms": ms_stats, "main_kernel_ms": ms_main, "fixup_ms": ms_fix,
                             "aggregate_ms": tot2}}, comp, cpu)
    else:
        report("c3", "RMAT21 GATConv heads=8 C=32, fused leaky_relu+softmax(+1e-16)+aggregate+bias",
               E, N, 4 * H * C + 4 + 4 * H, 4 * H * C + 4 * H + 4, ms_main1, tot1,
               {"fixup_ms": ms_fix1, "node_scores_ms": ms_scores, "n_split": csr.n_split,
                "node_scores_in_kernel": nd_info,
                "two_pass": {"stats_ms": ms_stats, "main_kernel_ms": ms_main, "fixup_ms": ms_fix,
                             "aggregate_ms": tot2}}, comp, cpu)
    # parity spot check against the generic PyG formula on identical inputs (one row block)
    del graph


def c4(dev):
    from mi355_mp import _lib, ops
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import powerlaw_edge_index
    N, E, F = 232_965, 114_615_892, 256
    ei = powerlaw_edge_index(N, E, seed=3, device=dev)
    graph = Graph(ei, N, N)
    csr = graph.dst
    x = torch.randn(N, F, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    out = torch.empty(N, F, device=dev)
    arg = torch.empty(N, F, dtype=torch.int64, device=dev)
    lib = _lib.load()
    # the layer's path from its third aggregation on (ops.FIRST_OCCURRENCE_AFTER):
    # repeated (row, source) edges dropped once, bit-identical max + argmax
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fo = csr.first_occurrences()
    torch.cuda.synchronize()
    t_first = time.perf_counter() - t0
    red = _lib.MP_REDUCE["max"]
    st = torch.cuda.current_stream().cuda_stream

    def agg_on(c, stages):
        s = c.struct("other")
        sb = lib.mp_aggregate_slab_bytes(s, F, red)
        slab = agg_on.slabs.get(id(c))
        if slab is None:
            slab = agg_on.slabs[id(c)] = torch.empty(sb, dtype=torch.uint8, device=dev)
        _lib.check(lib.mp_aggregate_f32(s, None, x.data_ptr(), F, F, red, _lib.MP_FLAG_PYG_MASK, None,
                                        out.data_ptr(), F, arg.data_ptr(), slab.data_ptr(), sb, stages, st),
                   "max")
    agg_on.slabs = {}
    # a one-off aggregation (the layer's first two calls over a CSR) gathers every edge
    ms_main_full = timed(lambda: agg_on(csr, _lib.MP_STAGE_MAIN))
    ms_fix_full = timed(lambda: agg_on(csr, _lib.MP_STAGE_FIXUP))
    # from the third call on (ops.FIRST_OCCURRENCE_AFTER): the first-occurrence CSR
    ms_main = timed(lambda: agg_on(fo, _lib.MP_STAGE_MAIN))
    ms_fix = timed(lambda: agg_on(fo, _lib.MP_STAGE_FIXUP))
    comp = N * F * 4 + csr.n_edges * 4 + (N + 1) * 4 + N * F * 12
    cpu = cpu_max_baseline(ei, x, 12_000_000) if CPU_BASELINE else None
    # headline: the one-off form, every edge gathered (edges/s == gathers/s there)
    report("c4", "Reddit-scale power-law, aggr='max' + int64 first-index argmax, PyG -10000 mask; "
           "headline = one aggregation gathering every edge",
           csr.n_edges, N, 4 * F + 4, 4 * F + 8 * F + 4, ms_main_full, ms_main_full + ms_fix_full,
           {"fixup_ms": ms_fix_full, "n_split": csr.n_split, "gathers_per_s": csr.n_edges / ((ms_main_full + ms_fix_full) * 1e-3),
            "repeated_layer_first_occurrences": {
                "engages": "from the 3rd unweighted max/min aggregation over one CSR (ops.FIRST_OCCURRENCE_AFTER = 2); "
                           "one-time build %.3f s" % t_first,
                "main_kernel_ms": ms_main, "fixup_ms": ms_fix, "aggregate_ms": ms_main + ms_fix,
                "gathers_per_aggregation": fo.n_edges,
                "gathers_per_s": fo.n_edges / ((ms_main + ms_fix) * 1e-3),
                "edges_reduced_per_s": csr.n_edges / ((ms_main + ms_fix) * 1e-3)},
            "note": "x is 238 MB: it fits the 256 MB Infinity Cache, so gathers are mostly on-die.  Of the %d edges, "
                    "%d are first occurrences of their (row, source) pair; a repeat changes neither value nor argmax "
                    "(max is idempotent, the first edge wins ties), so a layer reused every epoch drops them once "
                    "and gathers only the first occurrences" % (csr.n_edges, fo.n_edges)}, comp, cpu)


def c5(dev):
    from mi355_mp import _lib, ops
    from mi355_mp.graph import Graph
    from mi355_mp.graphgen import powerlaw_edge_index
    from torch_geometric.nn.conv.gcn_conv import GCNConv
    N, E, F = 2_449_029, 123_718_280, 256
    ei = powerlaw_edge_index(N, E, seed=4, device=dev)
    ei2, norm = GCNConv.norm(ei, N)
    graph = Graph(ei2, N, N)
    csr = graph.dst
    w = csr.to_csr_order(norm)
    x = torch.randn(N, F, device=dev, generator=torch.Generator(device=dev).manual_seed(4))
    bias = torch.zeros(F, device=dev)
    out = torch.empty(N, F, device=dev)
    slab = torch.empty(_lib.load().mp_aggregate_slab_bytes(csr.struct("other"), F, 0), dtype=torch.uint8,
                       device=dev)

    def agg(stages):
        ops._aggregate(csr, "other", x, w, "sum", 0, bias, out=out, stages=stages, slab=slab)
    ms_main = timed(lambda: agg(_lib.MP_STAGE_MAIN))
    ms_fix = timed(lambda: agg(_lib.MP_STAGE_FIXUP))
    comp = N * F * 8 + csr.n_edges * 8 + (N + 1) * 4
    # the reference's own device path and a vendor SpMM, same GPU / CSR / weights
    from bench import device_reference_paths
    agg(_lib.MP_STAGE_ALL)
    fused_out = out.clone()
    terms = ops._aggregate(csr, "other", x.abs(), w.abs(), "sum", 0, None)[0]
    paths = device_reference_paths(ei2, norm, x, csr, w, bias, fused_out, terms)
    del fused_out, terms
    cpu = cpu_sum_baseline(ei2, norm, x, 40_000_000) if CPU_BASELINE else None
    report("c5", "ogbn-products-scale power-law GCNConv F=256 on ONE GPU", csr.n_edges, N,
           4 * F + 8, 4 * F + 4, ms_main, ms_main + ms_fix,
           {"fixup_ms": ms_fix, "n_split": csr.n_split,
            "gpu_reference_path_ms": (paths.get("reference_path") or {}).get("ms"),
            "hipsparse_spmm_ms": (paths.get("vendor_spmm") or {}).get("ms"), "same_gpu_paths": paths}, comp,
           cpu)


def _train_step_ms(conv, x, ei):
    # one training step of the layer as an optimizer loop runs it: gradients
    # reset to None first (zero_grad(set_to_none=True), so no accumulation
    # pass), a fixed upstream gradient allocated once
    gout = [None]

    def step():
        conv.zero_grad(set_to_none=True)
        x.grad = None
        out = conv(x, ei)
        if gout[0] is None:
            gout[0] = torch.ones_like(out)
        out.backward(gout[0])
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        step()
    b.record()
    torch.cuda.synchronize()
    fwd_a, fwd_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.no_grad():
        conv(x, ei)
        fwd_a.record()
        for _ in range(5):
            conv(x, ei)
        fwd_b.record()
    torch.cuda.synchronize()
    return fwd_a.elapsed_time(fwd_b) / 5, a.elapsed_time(b) / 5


def c2train(dev):
    """Full GCNConv(256, 256) layer on config 2: x@W + fused aggregation (+ backward:
    transposed-CSR aggregation, GEMM grads)."""
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn import GCNConv
    N = 1 << 21
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    x = torch.randn(N, 256, device=dev).requires_grad_(True)
    conv = GCNConv(256, 256, cached=True).to(dev)
    fwd, step = _train_step_ms(conv, x, ei)
    print(json.dumps({"config": "c2train", "desc": "GCNConv(256,256) layer on RMAT21, cached=True",
                      "forward_ms": fwd, "forward_backward_ms": step}), flush=True)


def c3train(dev):
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn import GATConv
    N = 1 << 21
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    x = torch.randn(N, 256, device=dev).requires_grad_(True)
    conv = GATConv(256, 32, heads=8).to(dev)
    fwd, step = _train_step_ms(conv, x, ei)
    print(json.dumps({"config": "c3train", "desc": "GATConv(256, 32, heads=8) layer on RMAT21",
                      "forward_ms": fwd, "forward_backward_ms": step}), flush=True)


def c3train_drop(dev):
    """GATConv(256, 32, heads=8, dropout=0.6) training step on config 3: the
    attention dropout runs in the fused kernels (hashed keep mask)."""
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn import GATConv
    N = 1 << 21
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    x = torch.randn(N, 256, device=dev).requires_grad_(True)
    conv = GATConv(256, 32, heads=8, dropout=0.6).to(dev).train()
    _, step = _train_step_ms(conv, x, ei)
    print(json.dumps({"config": "c3train_drop", "desc": "GATConv(256, 32, heads=8, dropout=0.6) training step "
                      "on RMAT21, attention dropout fused", "forward_backward_ms": step}), flush=True)


def c3train_h1(dev):
    """The reference's own GAT stacks (ConvexPruning.py:209-214) use heads=1 and
    arbitrary widths: GATConv(256, C, heads=1) training steps on the config-3
    graph for C = 256 (C/4 a power of two: fused backward) and C = 200 / 255
    (C % 4 padded, the wide forms for C/4 not a power of two)."""
    from mi355_mp.graphgen import rmat_edge_index
    from torch_geometric.nn import GATConv
    N = 1 << 21
    ei = rmat_edge_index(scale=21, n_samples=30_000_000, seed=1, device=dev)
    x = torch.randn(N, 256, device=dev).requires_grad_(True)
    for C in (256, 200, 255, 100, 731):
        conv = GATConv(256, C, heads=1).to(dev)
        fwd, step = _train_step_ms(conv, x, ei)
        print(json.dumps({"config": "c3train_h1", "desc": "GATConv(256, %d, heads=1) layer on RMAT21" % C,
                          "C": C, "forward_ms": fwd, "forward_backward_ms": step}), flush=True)
        del conv
        torch.cuda.empty_cache()


def c5reorder(dev):
    """ogbn-products-shaped first layer GCNConv(100, 256): reference order
    A (X W) vs aggregate_first (A X) W, forward + backward."""
    from mi355_mp.graphgen import powerlaw_edge_index
    from torch_geometric.nn import GCNConv
    N, E = 2_449_029, 123_718_280
    ei = powerlaw_edge_index(N, E, seed=4, device=dev)
    x = torch.randn(N, 100, device=dev)
    res = {}
    for name, af in (("reference_order", False), ("aggregate_first", True)):
        torch.manual_seed(0)
        conv = GCNConv(100, 256, cached=True, aggregate_first=af).to(dev)
        fwd, step = _train_step_ms(conv, x, ei)
        res[name] = {"forward_ms": fwd, "forward_backward_ms": step}
        del conv
        torch.cuda.empty_cache()
    print(json.dumps({"config": "c5reorder", "desc": "GCNConv(100, 256) on ogbn-products-scale power law",
                      **res}), flush=True)


def c1graph(dev):
    """Config 1 (Cora-shaped 2-layer GCN 1433-16-7, cached=True): forward and one
    training step (forward + backward + Adam), eager vs HIP-graph replay
    (torch.cuda.graph / make_graphed_callables over the native kernels)."""
    import torch.nn.functional as Fn
    from mi355_mp.graphgen import cora_like
    from torch_geometric.nn import GCNConv
    d = cora_like()
    x, ei, y = d["x"].to(dev), d["edge_index"].to(dev), d["y"].to(dev)

    class Net(torch.nn.Module):
        def __init__(self):
            super(Net, self).__init__()
            self.c1 = GCNConv(1433, 16, cached=True)
            self.c2 = GCNConv(16, 7, cached=True)

        def forward(self, x):
            return Fn.log_softmax(self.c2(Fn.relu(self.c1(x, ei)), ei), dim=1)

    def per_call(fn, n=200):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / n

    torch.manual_seed(0)
    net = Net().to(dev)
    with torch.no_grad():
        fwd_eager = per_call(lambda: net(x))
        static_x = x.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                net(static_x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            net(static_x)
        fwd_graph = per_call(g.replay)
    opt = torch.optim.Adam(net.parameters(), lr=0.01)

    def step(m):
        opt.zero_grad()
        Fn.nll_loss(m(x), y).backward()
        opt.step()
    train_eager = per_call(lambda: step(net), 100)
    graphed = torch.cuda.make_graphed_callables(net, (x.clone(),))
    train_graph = per_call(lambda: step(graphed), 100)
    print(json.dumps({"config": "c1graph", "desc": "Cora-shaped 2-layer GCN 1433-16-7 (cached), per call",
                      "forward_eager_ms": fwd_eager, "forward_hipgraph_ms": fwd_graph,
                      "train_step_eager_ms": train_eager, "train_step_graphed_ms": train_graph}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c4,c5,c2train,c3train,c1graph")
    ap.add_argument("--cpu-baseline", action="store_true")
    args = ap.parse_args()
    global CPU_BASELINE
    CPU_BASELINE = args.cpu_baseline
    import mi355_mp
    mi355_mp.load_native()
    dev = torch.device("cuda", 0)
    for c in args.configs.split(","):
        globals()[c](dev)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
