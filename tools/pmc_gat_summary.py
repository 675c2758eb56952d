"""Summarise tools/profile_gat.sh into profiles/<round>_pmc_gat_bwd.json: per
fused GAT main kernel (forward GatRed, backward GatBwdRed) the kernel-trace
average, FETCH_SIZE (x2, the gfx950 correction of MI355X_MICROARCH.md 'HBM'),
WRITE_SIZE, L2 hit rate, L1 miss-queue stall, TA busy, VALU busy, L1->L2
lines per cycle per CU (GRBM_GUI_ACTIVE summed over the 8 XCDs; 256 CUs).
    python tools/pmc_gat_summary.py gpurun_out/prof_gat r03"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pytorch_geometric-1_amd"))
from mi355_mp._lib import source_hash  # noqa: E402


def counters(path):
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        rows[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {n: sum(v) / len(v) for n, v in c.items()} for k, c in rows.items()}


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv")))}
    m = collections.defaultdict(dict)
    for name in ("pmc_fetch", "pmc_write", "pmc_l2", "pmc_stall"):
        for k, c in counters(os.path.join(src, name, "pmc_counter_collection.csv")).items():
            m[k].update(c)
    out = {"workload": "c3train: GATConv(256, 32, heads=8) forward + backward on RMAT21 (+ loops)",
           "source_hash": source_hash(), "kernels": {}}
    for k, c in m.items():
        st = stats.get(k)
        avg_ns = float(st["AverageNs"]) if st else None
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        fetch = 2.0 * c.get("FETCH_SIZE", 0) * 1024
        write = c.get("WRITE_SIZE", 0) * 1024
        hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        out["kernels"][k] = {
            "avg_ms": avg_ns / 1e6 if avg_ns else None, "calls": int(st["Calls"]) if st else None,
            "fetch_bytes_x2": fetch, "write_bytes": write, "fabric_bytes": fetch + write,
            "fabric_TBps": (fetch + write) / (avg_ns * 1e-9) / 1e12 if avg_ns else None,
            "l2_hit": hit / (hit + miss) if hit + miss else None,
            "l1_miss_queue_stalled": c.get("TCP_PENDING_STALL_CYCLES_sum", 0) / (256 * cyc) if cyc else None,
            "ta_busy": c.get("TA_BUSY_avr", 0) / cyc if cyc else None,
            "valu_busy_per_simd": c.get("SQ_ACTIVE_INST_VALU", 0) / (1024 * cyc) if cyc else None,
            "waves_waiting": c.get("SQ_WAIT_ANY", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0)),
            "l1_to_l2_read_req": c.get("TCP_TCC_READ_REQ_sum"),
            "lines_per_cycle_per_cu": c.get("TCP_TCC_READ_REQ_sum", 0) / (256 * cyc) if cyc else None,
            "cycles": cyc}
    path = os.path.join("profiles", "%s_pmc_gat_bwd.json" % rnd)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    import shutil
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join("profiles", "%s_gat_train_kernel_stats.csv" % rnd))
    for k, v in out["kernels"].items():
        print(k[:80], json.dumps({a: (round(b, 4) if isinstance(b, float) else b) for a, b in v.items()}))


if __name__ == "__main__":
    main()
