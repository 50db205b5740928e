"""Sum rocprofv3 counter_collection CSVs per kernel (name substring) and
print ratios.  usage: python tools/pmc_finisher.py DIR [kernel-substring]"""
import csv
import glob
import json
import sys
from collections import defaultdict

d = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else "wf_finish_bvh"
tot = defaultdict(float)
n = 0
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if ksub in row.get("Kernel_Name", ""):
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            n += 1
out = dict(tot)
if tot.get("SQ_WAVE_CYCLES"):
    w = tot["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if k in tot:
            out[k + "/WAVE_CYCLES"] = round(tot[k] / w, 4)
if tot.get("SQ_ACTIVE_INST_VALU") and tot.get("SQ_THREAD_CYCLES_VALU"):
    out["valu_lane_util"] = round(tot["SQ_THREAD_CYCLES_VALU"] / (64 * tot["SQ_ACTIVE_INST_VALU"]), 4)
if tot.get("SQC_ICACHE_HITS") is not None and tot.get("SQC_ICACHE_MISSES") is not None:
    out["icache_miss_rate"] = round(tot["SQC_ICACHE_MISSES"] / max(tot["SQC_ICACHE_HITS"] + tot["SQC_ICACHE_MISSES"], 1), 4)
out["rows"] = n
print(json.dumps(out))
