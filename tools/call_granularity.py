"""Msamples/s of room2m 1920x1080 (adaptive off, unbounded depth) by passes
per rt_render call, chained (RtOptions.overlap = 1) and unchained: the
reference calls render() once per pass (rt/main.cu:114-155).  Each row renders
`total` passes after a warm-up, in calls of `per_call` passes, and ends with
rt_join.  usage: python tools/call_granularity.py [total passes] [per-call passes ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

total = int(sys.argv[1]) if len(sys.argv) > 1 else 256
per_calls = [int(x) for a in sys.argv[2:] for x in a.split(",")] or [1, 16, 64, 256]
scene = os.environ.get("RT_SCENE", "room2m")
long_depth = int(os.environ.get("RT_LONG_DEPTH", "0"))  # RtOptions.wf_long_depth (0 = default)
coalesce = int(os.environ.get("RT_COALESCE", "0"))  # RtOptions.coalesce_passes (0 = default 256, -1 = off)
overlaps = (1,) if os.environ.get("RT_CHAINED_ONLY") else (1, 0)
W, H = 1920, 1080
rt.check(rt.lib().rt_set_device(0))
run = helpers.GpuRun(scene)
g = rt.GBuffer(W, H)
rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 16, adaptive=False, kernel=rt.KERNEL_WAVEFRONT))
rt.join()
for pc in per_calls:
    for overlap in overlaps:
        if pc == 1 and not overlap and total > 64:
            continue  # (unchained 1-pass calls: every call waits for its longest deep path)
        n_calls = total // pc
        rt.check(rt.lib().rt_synchronize())
        t = time.perf_counter()
        for _ in range(n_calls):
            rt.render(run.dev, g, run.camera, 1, rt.options(W, H, pc, adaptive=False, kernel=rt.KERNEL_WAVEFRONT,
                                                             overlap=bool(overlap), wf_long_depth=long_depth,
                                                             coalesce_passes=coalesce))
        rt.join()
        dt = time.perf_counter() - t
        print(json.dumps({"scene": scene, "passes_per_call": pc, "calls": n_calls, "overlap": overlap, "long_depth": long_depth,
                          "coalesce_passes": coalesce,
                          "seconds": round(dt, 3), "Msamples_per_s": round(W * H * pc * n_calls / dt / 1e6, 1)}),
              flush=True)
