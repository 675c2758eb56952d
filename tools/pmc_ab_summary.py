"""Per-kernel averages of the counters collected by tools/pmc_ab.sh.
    python tools/pmc_ab_summary.py gpurun_out/pmc_<tag>
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        cyc = d.get("GRBM_GUI_ACTIVE", 0) / 8 or None
        if "TCC_HIT_sum" in d:
            d["l2_hit"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        if cyc:
            d["kernel_cycles"] = cyc
            if "TCP_PENDING_STALL_CYCLES_sum" in d:
                d["tcp_pending_stall_frac"] = d["TCP_PENDING_STALL_CYCLES_sum"] / (256 * cyc)
            if "TA_BUSY_avr" in d:
                d["ta_busy_frac"] = d["TA_BUSY_avr"] / cyc
        if d.get("SQ_WAVE_CYCLES"):
            d["wave_waiting_frac"] = d.get("SQ_WAIT_ANY", 0) / d["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in d:
            d["fetch_bytes_x2"] = 2 * d["FETCH_SIZE"] * 1024
        out[k] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
