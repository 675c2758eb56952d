"""Summarise rocprofv3 output of tools/profile.sh into profiles/<round>_*.

  python tools/pmc_summary.py gpurun_out/prof r01 [workload] [calib_dir]

Writes profiles/<round>_kernel_stats.csv (copy of the --stats summary),
profiles/<round>_pmc_traffic.json: per-launch FETCH_SIZE / WRITE_SIZE of the
dominant kernel, corrected as MI355X_MICROARCH.md 'HBM' prescribes
(FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reads half the bytes
of a 16 B/lane coalesced stream -> doubled, and profiles/r01_pmc_calibration.json
measures the same factor for this kernel's 8 B/lane loads; WRITE_SIZE exact
for 16 B/lane stores), plus the L2 hit rate.  bench.py reads the json for
roofline.traffic only when its kernel name and native source hash match the
running build.  Run it on the tree the profile was taken from.
"""
import csv
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pytorch_geometric-1_amd"))
from mi355_mp._lib import source_hash  # noqa: E402

N_CU = 256      # MI355X compute units (one TCP each)
N_XCD = 8
KERNEL = None   # the dominant k_agg_flat / k_agg_main instance, from the kernel-trace stats


def per_launch(path, counter):
    vals = []
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else "rmat21_gcn_f256"
    calib_dir = sys.argv[4] if len(sys.argv) > 4 else src
    suffix = "" if workload == "rmat21_gcn_f256" else "_" + ("gat" if "_gat" in workload else workload.split("_")[0])
    os.makedirs("profiles", exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), "profiles/%s_kernel_stats%s.csv" % (rnd, suffix))
    global KERNEL
    avg_ns, best = None, -1.0
    for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))):
        if ("k_agg_flat" in r["Name"] or "k_agg_main" in r["Name"]) and float(r["TotalDurationNs"]) > best:
            best = float(r["TotalDurationNs"])
            KERNEL, avg_ns = r["Name"], float(r["AverageNs"])
    fetch, nf = per_launch(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write, nw = per_launch(os.path.join(src, "pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE")
    hit, _ = per_launch(os.path.join(src, "pmc_l2", "pmc_counter_collection.csv"), "TCC_HIT_sum")
    miss, _ = per_launch(os.path.join(src, "pmc_l2", "pmc_counter_collection.csv"), "TCC_MISS_sum")
    read_b = 2.0 * fetch * 1024
    # this kernel's own FETCH_SIZE ratio, measured on a known byte count by
    # tools/pmc_calibrate.py in the same profile run (pass pmc_calib)
    ratio = None
    calib = os.path.join(calib_dir, "pmc_calib", "pmc_counter_collection.csv")
    if os.path.exists(calib):
        cv, _ = per_launch(calib, "FETCH_SIZE")
        if cv:
            ratio = cv * 1024 / 2172780552.0   # expected_read_bytes printed by pmc_calibrate.py
    write_b = write * 1024
    # where the kernel waits: L1 (TCP) input stalled on misses pending from L2
    stall = {}
    sp = os.path.join(src, "pmc_stall", "pmc_counter_collection.csv")
    if os.path.exists(sp):
        for c in ("GRBM_GUI_ACTIVE", "TCP_PENDING_STALL_CYCLES_sum", "TCP_TCC_READ_REQ_sum", "TA_BUSY_avr",
                  "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"):
            stall[c], _ = per_launch(sp, c)
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD active cycles = kernel clocks
        cyc = stall["GRBM_GUI_ACTIVE"] / N_XCD if stall.get("GRBM_GUI_ACTIVE") else None
        stall["kernel_cycles"] = cyc
        if cyc:
            stall["tcp_pending_stall_frac"] = stall["TCP_PENDING_STALL_CYCLES_sum"] / (N_CU * cyc)
            stall["ta_busy_frac"] = stall["TA_BUSY_avr"] / cyc
        if stall.get("SQ_WAVE_CYCLES"):
            stall["wave_waiting_frac"] = stall["SQ_WAIT_ANY"] / stall["SQ_WAVE_CYCLES"]
    # memory side of the L2 (tools/profile.sh passes pmc_ea, pmc_lat)
    mem = {}
    for sub, names in (("pmc_ea", ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum",
                                   "TCC_READ_REQ_LATENCY_sum")),
                       ("pmc_lat", ("TCC_READ_REQ_sum", "TCC_TAG_STALL_sum", "TCC_LATENCY_FIFO_FULL_sum",
                                    "TCC_BUSY_sum"))):
        path = os.path.join(src, sub, "pmc_counter_collection.csv")
        if os.path.exists(path):
            for c in names:
                mem[c], _ = per_launch(path, c)
    if mem.get("TCC_READ_REQ_LATENCY_sum") and mem.get("TCC_READ_REQ_sum"):
        mem["avg_l2_read_latency_cycles"] = mem["TCC_READ_REQ_LATENCY_sum"] / mem["TCC_READ_REQ_sum"]
    if mem.get("TCC_EA0_RDREQ_DRAM_sum") and mem.get("TCC_EA0_RDREQ_sum"):
        mem["dram_share_of_fabric_reads"] = mem["TCC_EA0_RDREQ_DRAM_sum"] / mem["TCC_EA0_RDREQ_sum"]
    cyc = stall.get("kernel_cycles") if stall else None
    if cyc and mem.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum") is not None:
        # summed over the 16 L2 channels of each of the 8 XCDs
        mem["dram_credit_stall_frac_per_channel"] = mem["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / (128 * cyc)
    out = {
        "workload": workload,
        "kernel": KERNEL,
        "source_hash": source_hash(),
        "launches": {"fetch": nf, "write": nw},
        "FETCH_SIZE_KiB_raw": fetch,
        "WRITE_SIZE_KiB_raw": write,
        "read_bytes_corrected": read_b,
        "fetch_ratio_calibrated": ratio,
        "read_bytes_calibrated": fetch * 1024 / ratio if ratio else None,
        "write_bytes": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "l2_hit_rate": hit / (hit + miss) if hit is not None and miss else None,
        "kernel_trace_avg_ms": avg_ns / 1e6 if avg_ns else None,
        "stall": stall or None,
        "memory_side": mem or None,
        "note": "FETCH_SIZE counts L2->fabric reads (Infinity-Cache hits included): an upper bound "
                "on HBM reads; doubled per the gfx950 correction (calibrated for this kernel's own "
                "load width in profiles/r01_pmc_calibration.json)",
    }
    with open("profiles/%s_pmc_traffic%s.json" % (rnd, suffix), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
