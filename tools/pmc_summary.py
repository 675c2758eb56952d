"""Summarise rocprofv3 output of tools/profile.sh into profiles/<round>_*.

  python tools/pmc_summary.py gpurun_out/prof r01

Writes profiles/<round>_kernel_stats.csv (copy of the --stats summary),
profiles/<round>_pmc_traffic.json: per-launch FETCH_SIZE / WRITE_SIZE of the
dominant kernel, corrected as MI355X_MICROARCH.md 'HBM' prescribes
(FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reads half the bytes
of a 16 B/lane coalesced stream -> doubled, and profiles/r01_pmc_calibration.json
measures the same factor for this kernel's 8 B/lane loads; WRITE_SIZE exact
for 16 B/lane stores), plus the L2 hit rate.  bench.py reads the json for roofline.traffic.
"""
import csv
import json
import os
import shutil
import sys

KERNEL = "k_agg_flat<mp::SumRed<2, true, false>, 2, 16, 64, false>"


def per_launch(path, counter):
    vals = []
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    os.makedirs("profiles", exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), "profiles/%s_kernel_stats.csv" % rnd)
    avg_ns = None
    for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))):
        if KERNEL in r["Name"]:
            avg_ns = float(r["AverageNs"])
    fetch, nf = per_launch(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write, nw = per_launch(os.path.join(src, "pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE")
    hit, _ = per_launch(os.path.join(src, "pmc_l2", "pmc_counter_collection.csv"), "TCC_HIT_sum")
    miss, _ = per_launch(os.path.join(src, "pmc_l2", "pmc_counter_collection.csv"), "TCC_MISS_sum")
    read_b = 2.0 * fetch * 1024
    write_b = write * 1024
    out = {
        "workload": "rmat21_gcn_f256",
        "kernel": KERNEL,
        "launches": {"fetch": nf, "write": nw},
        "FETCH_SIZE_KiB_raw": fetch,
        "WRITE_SIZE_KiB_raw": write,
        "read_bytes_corrected": read_b,
        "write_bytes": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "l2_hit_rate": hit / (hit + miss) if hit is not None and miss else None,
        "kernel_trace_avg_ms": avg_ns / 1e6 if avg_ns else None,
        "note": "FETCH_SIZE counts L2->fabric reads (Infinity-Cache hits included): an upper bound "
                "on HBM reads; doubled per the gfx950 correction (calibrated for this kernel's 8 B/lane "
                "loads in profiles/r01_pmc_calibration.json)",
    }
    with open("profiles/%s_pmc_traffic.json" % rnd, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
