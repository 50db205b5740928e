#!/bin/bash
# Issue / VALU-busy counters of the wavefront kernels over one room2m render (16 passes).
# PMC dispatches are serialised by the profiler: per-dispatch values are one kernel alone on the GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_issue
cd /tmp && export TMPDIR=/tmp AB_NO_COUNT=1
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
    --kernel-trace -d /tmp/pmc_issue -o run --output-format csv -- python3 $R/tools/ab.py room2m 16 0 1 1 > $R/gpurun_out/pmc_issue/run.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob, json, collections
cc = glob.glob('/tmp/pmc_issue/**/*counter_collection.csv', recursive=True)
tot = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in cc:
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '')[:40]
        tot[k][r['Counter_Name']] += float(r['Counter_Value'])
        n[(k, r['Counter_Name'])] += 1
out = {k: dict(v) for k, v in tot.items()}
json.dump(out, open('/root/repo/gpurun_out/pmc_issue/summary.json', 'w'), indent=1)
for k, v in out.items():
    if 'trace_coop' in k or 'shade' in k or 'finish' in k:
        print(k, json.dumps({a: round(b) for a, b in v.items()}))
PY
exit $rc
