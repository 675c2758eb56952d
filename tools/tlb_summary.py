"""Per-kernel summary of tools/pmc_tlb.sh output (every pass directory under the
given one): each counter's per-launch mean, and the per-cycle / per-request
ratios (GRBM_GUI_ACTIVE is summed over the 8 XCDs; 256 CUs).
    python tools/tlb_summary.py gpurun_out/tlb_<name>"""
import collections
import csv
import glob
import os
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    tag = os.path.relpath(f, sys.argv[1]).split(os.sep)[0]
    for r in csv.DictReader(open(f)):
        name = r["Counter_Name"] if r["Counter_Name"] != "GRBM_GUI_ACTIVE" else "GRBM_GUI_ACTIVE@" + tag
        rows[r["Kernel_Name"]][name].append(float(r["Counter_Value"]))
out = []
for k, c in rows.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    cyc = max(v for n, v in m.items() if n.startswith("GRBM_GUI_ACTIVE")) / 8
    if cyc < 1e5:
        continue
    out.append((cyc, k, m))
for cyc, k, m in sorted(out, reverse=True)[:6]:
    print("%s\n  cycles/launch %.0f" % (k[:120], cyc))
    for n in sorted(m):
        if n.startswith("GRBM_GUI_ACTIVE"):
            continue
        v = m[n]
        print("  %-45s %14.0f  per-CU-cycle %.4f" % (n, v, v / (256 * cyc)))
    req = m.get("TCP_UTCL1_REQUEST_sum")
    if req:
        print("  UTCL1 hit rate %.4f, miss rate %.4f" % (
            m.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0) / req, m.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0) / req))
