"""Concurrency of RCCL kernels and the aggregation kernels in a rocprofv3
kernel trace (tools/gpu_round.sh step `rccl`: bench.py --sharded
--emulate-peers at one RCCL rank).  Prints one JSON object:
  rccl_kernels      instances, total ms, and the ms during which at least one
                    k_agg_* kernel ran at the same time (from the start / end
                    timestamps), per kernel name
  queues            instances per (kind, hardware queue, stream): kernels on one
                    queue run one after the other, whatever their streams
  agg_kernels       k_agg_* instances that overlap an RCCL kernel: their
                    duration next to the median duration of the same-named
                    instances in the same duration band that overlap none
                    (the slowdown of sharing the GPU with RCCL)
    python tools/kernel_overlap.py <rocprofv3 -d directory>
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def load(root):
    files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r.get("Queue_Id"), r.get("Stream_Id")))
    return files, rows


def is_rccl(name):
    n = name.lower()
    return "nccl" in n or "rccl" in n


def is_agg(name):
    return "k_agg_" in name


def overlap_ns(a, b, spans):
    """ns of [a, b) covered by the union of spans (sorted, possibly overlapping)."""
    tot, cur = 0, a
    for s, e in spans:
        if e <= cur:
            continue
        if s >= b:
            break
        lo, hi = max(s, cur), min(e, b)
        if hi > lo:
            tot += hi - lo
            cur = hi
    return tot


def main(root):
    files, rows = load(root)
    queues = collections.Counter()
    for n, s, e, qid, sid in rows:
        kind = "rccl" if is_rccl(n) else ("agg" if is_agg(n) else "other")
        queues["%s queue %s stream %s" % (kind, qid, sid)] += 1
    rccl = sorted((s, e, n) for n, s, e, _, _ in rows if is_rccl(n))
    agg = sorted((s, e, n) for n, s, e, _, _ in rows if is_agg(n))
    agg_spans = [(s, e) for s, e, _ in agg]
    rccl_spans = [(s, e) for s, e, _ in rccl]
    per = collections.defaultdict(lambda: {"instances": 0, "total_ms": 0.0, "concurrent_with_agg_ms": 0.0})
    for s, e, n in rccl:
        d = per[n[:120]]
        d["instances"] += 1
        d["total_ms"] += (e - s) * 1e-6
        d["concurrent_with_agg_ms"] += overlap_ns(s, e, agg_spans) * 1e-6
    shared, alone = [], collections.defaultdict(list)
    for s, e, n in agg:
        ov = overlap_ns(s, e, rccl_spans)
        if ov > 0:
            shared.append((n, (e - s) * 1e-6, ov * 1e-6))
        else:
            alone[n].append((e - s) * 1e-6)
    agg_out = []
    for n, dur, ov in shared:
        band = [d for d in alone.get(n, []) if 0.5 * dur <= d <= 2.0 * dur]
        base = statistics.median(band) if band else None
        agg_out.append({"kernel": n[:120], "ms": dur, "ms_sharing_with_rccl": ov,
                        "median_ms_same_band_alone": base,
                        "slowdown": (dur / base - 1.0) if base else None})
    res = {"trace_files": [os.path.relpath(f, root) for f in files],
           "queues": dict(sorted(queues.items())),
           "rccl_kernels": dict(per),
           "rccl_total_ms": sum(d["total_ms"] for d in per.values()),
           "rccl_concurrent_with_agg_ms": sum(d["concurrent_with_agg_ms"] for d in per.values()),
           "agg_instances": len(agg), "agg_instances_sharing_with_rccl": len(shared),
           "agg_kernels_sharing": agg_out}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
