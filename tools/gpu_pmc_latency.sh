#!/bin/bash
# Mean VMEM / LDS / SMEM instruction latency of the wavefront kernels (SQ_INST_LEVEL_x accumulated by
# SQ_ACCUM_PREV_HIRES, divided by the instruction count), one room2m render of 16 passes per pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_lat
cd /tmp && export TMPDIR=/tmp AB_NO_COUNT=1
for kind in VMEM LDS SMEM; do
  timeout -s KILL 200 rocprofv3 --pmc SQ_INST_LEVEL_$kind SQ_ACCUM_PREV_HIRES SQ_INSTS_$kind SQ_WAVE_CYCLES SQ_WAIT_ANY \
      --kernel-trace -d /tmp/pmc_lat_$kind -o run --output-format csv -- python3 $R/tools/ab.py room2m 16 0 1 1 \
      > $R/gpurun_out/pmc_lat/run_$kind.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, json, collections
out = {}
for kind in ("VMEM", "LDS", "SMEM"):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f'/tmp/pmc_lat_{kind}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '')[:40]
            tot[k][r['Counter_Name']] += float(r['Counter_Value'])
    for k, v in tot.items():
        if v.get(f'SQ_INSTS_{kind}'):
            out.setdefault(k, {})[kind] = {"insts": v[f'SQ_INSTS_{kind}'], "accum": v['SQ_ACCUM_PREV_HIRES'],
                                           "latency": v['SQ_ACCUM_PREV_HIRES'] / v[f'SQ_INSTS_{kind}'],
                                           "wave_cycles": v['SQ_WAVE_CYCLES'], "wait_any": v['SQ_WAIT_ANY']}
json.dump(out, open('/root/repo/gpurun_out/pmc_lat/summary.json', 'w'), indent=1)
for k, v in out.items():
    if 'trace_coop' in k or 'shade' in k:
        print(k, {a: (round(b['latency'], 1), round(b['insts'])) for a, b in v.items()})
PY
