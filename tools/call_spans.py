"""Where a chained small call's time goes: N chained calls of `pc` passes
(room2m 1080p) with RtOptions.profile, then the finisher spans on the device
(rt_profile_history: start relative to the first, length) and the host's
issue time per rt_render call.  usage: python tools/call_spans.py [calls] [passes per call]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pc = int(sys.argv[2]) if len(sys.argv) > 2 else 1
long_depth = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # RtOptions.wf_long_depth (0: the library's default)
W, H = 1920, 1080
rt.check(rt.lib().rt_set_device(0))
run = helpers.GpuRun("room2m")
g = rt.GBuffer(W, H)
rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 16, adaptive=False, kernel=rt.KERNEL_WAVEFRONT))
rt.join()
rt.profile_history(reset=True)
issue = []
t0 = time.perf_counter()
for _ in range(N):
    t = time.perf_counter()
    rt.render(run.dev, g, run.camera, 1, rt.options(W, H, pc, adaptive=False, kernel=rt.KERNEL_WAVEFRONT,
                                                     overlap=True, profile=True, wf_long_depth=long_depth))
    issue.append(time.perf_counter() - t)
t_issued = time.perf_counter() - t0
rt.join()
wall = time.perf_counter() - t0
h = rt.profile_history(reset=True)
starts = np.array([p["start_ms"] for p in h])
lens = np.array([p["finish_ms"] for p in h])
gaps = starts[1:] - (starts[:-1] + lens[:-1]) if len(h) > 1 else np.array([0.0])
print(json.dumps({"calls": N, "passes_per_call": pc, "wf_long_depth": long_depth, "wall_s": round(wall, 4), "issued_s": round(t_issued, 4),
                  "Msamples_per_s": round(W * H * pc * N / wall / 1e6, 1),
                  "host_issue_ms": {"mean": round(1e3 * float(np.mean(issue)), 3), "max": round(1e3 * float(np.max(issue)), 3)},
                  "finisher_ms": {"mean": round(float(lens.mean()), 3), "min": round(float(lens.min()), 3),
                                  "max": round(float(lens.max()), 3)},
                  "gap_ms": {"mean": round(float(gaps.mean()), 3), "max": round(float(gaps.max()), 3)},
                  "span_total_ms": round(float(starts[-1] + lens[-1] - starts[0]), 2), "profiles": len(h)}), flush=True)
