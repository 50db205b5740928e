# per-iteration timeline of one 64-spp room2m call (RT_WF_TRACE_ITERS): when the pipelines finish vs the long-path slices
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RT_WF_TRACE_ITERS=1 timeout -k 10 300 python -u tools/ab.py room2m 64 0 1 1 > gpurun_out/tail_probe.json 2> gpurun_out/tail_probe.log || { tail -20 gpurun_out/tail_probe.log; exit 1; }
grep -E "pipelines done|long paths" gpurun_out/tail_probe.log | head -8
python3 - <<'PY'
import re
L = open("gpurun_out/tail_probe.log").read().splitlines()
t0 = None; last = {}
for l in L:
    m = re.match(r"\[wf\] pipe (\d+) it (\d+) live (\d+) t ([\d.]+)", l)
    if m:
        p, it, live, t = int(m[1]), int(m[2]), int(m[3]), float(m[4])
        t0 = t if t0 is None else min(t0, t)
        last[p] = (it, live, t)
for p, (it, live, t) in sorted(last.items()): print("pipe", p, "last it", it, "live", live, "t", round(t - t0, 3))
for l in L:
    m = re.search(r"t ([\d.]+)$", l)
    if ("done" in l or "long" in l or "finished" in l) and m: print(l.split(" t ")[0], round(float(m[1]) - t0, 3))
PY
