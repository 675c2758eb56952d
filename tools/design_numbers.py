"""Print the current-state numbers DESIGN.md section 2 quotes, read from the
committed round files (profiles/<round>_bench_*.json, _bench_configs.jsonl,
_pmc_traffic*.json), so every number in those tables can be traced to a file;
and section 5.4's predicted multi-GPU curve from the gloo rehearsals'
per-rank compute and the one-GPU RCCL contention.
    python tools/design_numbers.py [r04]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(name):
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        if name.endswith(".jsonl"):
            return {d["config"]: d for d in map(json.loads, f)}
        text = f.read()
        try:
            return json.loads(text)
        except ValueError:     # a bench line saved with a library's banner above it
            return json.loads([ln for ln in text.splitlines() if ln.startswith("{")][-1])


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r06"
    out = {}
    for wl, f in (("c2", "bench_rmat21"), ("c5", "bench_products_n1"), ("c3", "bench_gat_n1"),
                  ("c5_gloo2", "bench_products_gloo2")):
        d = load("%s_%s.json" % (rnd, f))
        if not d:
            continue
        r, ex = d["roofline"], d.get("extra", {})
        out[wl] = {"edges_per_s": d["value"], "ms_per_step": d["ms_per_step"], "frac_compulsory": r["frac"],
                   "kernel_ms": r.get("avg_launch_ms", r.get("kernel_ms")), "fixup_ms": r.get("fixup_avg_ms"),
                   "traffic": r.get("traffic"), "cpu": (d.get("cpu_baseline") or {}).get("value"),
                   "gemm_ms": ex.get("gemm_xW_ms"), "ref_path_ms": ex.get("gpu_reference_path_ms"),
                   "spmm_ms": ex.get("hipsparse_spmm_ms"), "verify": ex.get("verify")}
    for wl, suffix in (("c2", ""), ("c5", "_products"), ("c3", "_gat")):
        p = load("%s_pmc_traffic%s.json" % (rnd, suffix))
        if p:
            out.setdefault(wl, {})["pmc"] = {"bytes_per_launch": p["hbm_bytes_per_launch"],
                                             "l2_hit": p["l2_hit_rate"], "kernel_trace_ms": p["kernel_trace_avg_ms"],
                                             "TBps": p["hbm_bytes_per_launch"] / p["kernel_trace_avg_ms"] / 1e9,
                                             "source_hash": p["source_hash"],
                                             "ta_busy": (p.get("stall") or {}).get("ta_busy_frac"),
                                             "l1_queue_stall": (p.get("stall") or {}).get("tcp_pending_stall_frac")}
    cfg = load("%s_bench_configs.jsonl" % rnd) or {}
    for k, d in cfg.items():
        out["cfg_" + k] = {kk: v for kk, v in d.items() if not isinstance(v, (dict, list)) and kk != "desc"}
        if "repeated_layer_first_occurrences" in d:
            out["cfg_" + k]["first_occurrences"] = d["repeated_layer_first_occurrences"]
    # the predicted multi-GPU curve from the rehearsals' per-rank compute
    # (GPU to itself), the one-GPU RCCL contention and the link model at 77 GB/s:
    # per rank the bench's link_model.predicted_in_turn["77"] = max(compute in turn
    # of the chosen form, pack(first) + exchange + boundary(last)), max over ranks,
    # + the contention; config 2 (rmat21) and config 5 (products)
    conts = {}
    for wl, f in (("c2", "bench_sharded_rccl_one_rank"), ("c5", "bench_sharded_rccl_one_rank_products")):
        rc = load("%s_%s.json" % (rnd, f))
        conts[wl] = {}
        if rc:
            for r in rc["extra"]["per_rank"][0].get("rccl_contention", []):
                conts[wl][r["P"]] = r["contention_ms"]
    for wl, one_name, pre in (("c2", "bench_rmat21", "bench_rmat21_gloo"),
                              ("c5", "bench_products_n1", "bench_products_gloo")):
        # config 5 without its own contention run: config 2's at the same P
        cont = {**conts["c2"], **conts[wl]}
        one = load("%s_%s.json" % (rnd, one_name)) or load("r05_%s.json" % one_name)
        for P in (2, 4, 8):
            d = load("%s_%s%d_rehearsal.json" % (rnd, pre, P))
            if not d or "compute_in_turn" not in d["extra"]["per_rank"][0]:
                continue
            ranks = d["extra"]["per_rank"]
            slow = max(ranks, key=lambda p: p["compute_in_turn"]["compute_alone_ms"])
            c = slow["compute_in_turn"]
            pred = max(p["link_model"]["predicted_in_turn"]["77"] for p in ranks)
            form = d["extra"].get("step_form") or ""
            T = len(d["extra"]["halo_tiles"])
            tp = T if "packed per tile" in form else 1
            tb = 1 if "boundary in one launch" in form else T
            chain = max(p["compute_in_turn"]["send_pack_ms"] / tp + p["link_model"]["max_peer_bytes"] / 77e9 * 1e3
                        + p["compute_in_turn"]["boundary_ms"] / tb for p in ranks)
            step = pred + cont.get(P, 0.0)
            out["curve_%s_P%d" % (wl, P)] = {
                "step_form": d["extra"].get("step_form"),
                "compute_in_turn_slowest_ms": c["compute_alone_ms"],
                "slowest_parts_ms": [c["send_pack_ms"], c["interior_ms"], c["boundary_ms"]],
                "compute_split_slowest_ms": max(p["compute_in_turn"]["compute_alone_split_ms"] for p in ranks),
                "link_chain_77_ms": chain, "predicted_in_turn_77_ms": pred,
                "contention_ms": cont.get(P), "predicted_step_ms": step,
                "one_gpu_ms": one["ms_per_step"] if one else None,
                "ideal_split_ms": one["ms_per_step"] / P if one else None,
                "speedup_vs_1gpu": (one["ms_per_step"] / step) if one else None,
                "verify": (d["extra"].get("verify") or {}).get("all_ranks_within_1e-5_bound"),
                "build_s": d["extra"].get("one_time_build_s")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
