"""Summarise rocprofv3 CSV output directories into a compact JSON/text report.

usage: python tools/prof_summary.py OUT.json DIR [DIR ...]
For each DIR: kernel-trace stats (per kernel name: calls, total/avg ns) and,
when present, PMC counters summed per kernel name.  Keeps only what profiles/
needs so the raw CSVs can be deleted on the GPU box.
"""
import collections
import csv
import glob
import json
import os
import sys


def summarize(d):
    out = {"dir": os.path.basename(d.rstrip("/"))}
    stats = glob.glob(os.path.join(d, "*kernel_stats.csv"))
    if stats:
        rows = list(csv.DictReader(open(stats[0])))
        out["kernel_stats"] = [{"name": r["Name"][:120], "calls": int(r["Calls"]),
                                "total_ns": float(r["TotalDurationNs"]), "avg_ns": float(r["AverageNs"]),
                                "pct": float(r["Percentage"])} for r in rows[:12]]
    trace = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    if trace:
        agg = collections.defaultdict(lambda: [0, 0.0])
        for r in csv.DictReader(open(trace[0])):
            k = r["Kernel_Name"][:80]
            agg[k][0] += 1
            agg[k][1] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        out["trace_by_kernel"] = {k: {"calls": v[0], "total_ms": round(v[1] / 1e6, 3)} for k, v in
                                  sorted(agg.items(), key=lambda kv: -kv[1][1])[:12]}
    cc = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if cc:
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        calls = collections.Counter()
        for r in csv.DictReader(open(cc[0])):
            k = r["Kernel_Name"][:80]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == next(iter(agg[k])):
                calls[k] += 1
        out["counters_by_kernel"] = {k: dict(v, dispatches=calls[k]) for k, v in agg.items()
                                     if "rt_" in k or "wf_" in k}
    return out


if __name__ == "__main__":
    res = [summarize(d) for d in sys.argv[2:] if os.path.isdir(d)]
    with open(sys.argv[1], "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1)[:4000])
