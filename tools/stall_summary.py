"""Per-kernel summary of tools/pmc_stall.sh output: L1 miss-queue stall and
issue fractions (GRBM_GUI_ACTIVE is summed over the 8 XCDs; 256 CUs, 1024 SIMDs).
    python tools/stall_summary.py gpurun_out/stall_<name>"""
import collections
import csv
import os
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(os.path.join(sys.argv[1], "pmc_counter_collection.csv"))):
    rows[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = []
for k, c in rows.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc < 1e5:
        continue
    out.append((cyc, k, m))
for cyc, k, m in sorted(out, reverse=True)[:12]:
    print("%-90s cyc/launch %9.0f  tcp_pending %.2f  ta_busy %.2f  valu/simd %.2f  vmem/cu %.3f  waiting %.2f" % (
        k[:90], cyc, m["TCP_PENDING_STALL_CYCLES_sum"] / (256 * cyc), m["TA_BUSY_avr"] / cyc,
        m["SQ_ACTIVE_INST_VALU"] / (1024 * cyc), m["SQ_ACTIVE_INST_VMEM"] / (256 * cyc),
        m["SQ_WAIT_ANY"] / max(1.0, m["SQ_WAVE_CYCLES"])))
