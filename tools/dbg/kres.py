"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin):
one line per kernel: VGPRs, AGPRs, spills, occupancy.  Optional argv[1]: a
substring filter on the demangled name."""
import re, subprocess, sys
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split()[0] + ("_spill" if "Spill" in k else "")] = v
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r, n in zip(rows, names):
    if flt in n:
        print("%4s vgpr %3s spill occ %s  %s" % (r.get("VGPRs"), r.get("VGPRs_spill"), r.get("Occupancy"), n))
