"""A/B of the two bounded-traversal call shapes on one frame: the whole call
in the persistent finisher (default) against trace / shade queue iterations
(wf_tail = 1: wf_trace_bvh_dyn, per-lane ray refill) — call wall time and the
queue path's kernel times (RtProfile).  usage: python tools/queue_vs_whole.py
[scene] [passes] [rounds] [max_depth]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "room2m"
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 32
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
max_depth = int(sys.argv[4]) if len(sys.argv) > 4 else 0
W, H = 1920, 1080
rt.check(rt.lib().rt_set_device(0))
run = helpers.GpuRun(scene)
g = rt.GBuffer(W, H)
rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 2, adaptive=False, kernel=rt.KERNEL_WAVEFRONT))
rt.join()
for r in range(rounds):
    for name, kw in (("whole", {}), ("queue_dyn", {"wf_tail": 1})):
        rt.check(rt.lib().rt_synchronize())
        t = time.perf_counter()
        rt.render(run.dev, g, run.camera, 1, rt.options(W, H, passes, adaptive=False, kernel=rt.KERNEL_WAVEFRONT,
                                                         profile=True, max_depth=max_depth, **kw))
        rt.join()
        dt = time.perf_counter() - t
        p = rt.last_profile()
        print(json.dumps({"round": r, "mode": name, "passes": passes, "max_depth": max_depth, "s": round(dt, 4),
                          "Msamples_s": round(W * H * passes / dt / 1e6, 1),
                          "profile": {k: round(v, 2) if isinstance(v, float) else v for k, v in p.items()}}),
              flush=True)
