#!/bin/bash
# Memory-pipeline occupancy of the bulk finisher (TA / TD busy, L1 stalls), room2m 1080p one 32-pass call
# with paths cut at 64 bounces (tools/ab.py), one counter pass each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_ta; mkdir -p $O
cd /tmp && export TMPDIR=/tmp AB_NO_COUNT=1
timeout -s KILL 120 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
i=0
for set in "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TD_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d /tmp/pmc_ta_$i -o run --output-format csv -- python3 $R/tools/ab.py room2m 32 64 1 1 > $O/run_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/run_$i.log; }
  cp $(find /tmp/pmc_ta_$i -name "*counter_collection.csv" | head -1) $O/pass_$i.csv 2>/dev/null
done
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ["GRAFT_REPO_ROOT"]
for f in sorted(glob.glob(R + "/gpurun_out/pmc_ta/pass_*.csv")):
    tot = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:30]
        tot[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in tot.items():
        if "finish_bvh" in k:
            print(os.path.basename(f), k, {c: (sum(x) if not c.endswith("_avr") else sum(x) / len(x)) for c, x in v.items()})
PY
