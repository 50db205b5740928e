"""Phase profile of the whole-call finisher (wf_finish_bvh): wave time in the
loop overhead (path fetch, returns, leave checks), the BVH query, the KD
phase and shading (+ guard + hand-off), and the active lanes per ray query.
Needs the -DRT_PHASE_PROF build: bash tools/mkvariant.sh phase -DRT_PHASE_PROF,
then ISAKLM_RT_LIB_OVERRIDE=ab_libs/phase.so python tools/phase_profile.py [scene] [passes]."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "room2m"
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 64
W, H = 1920, 1080
L = rt.lib()
L.rt_debug_phase_profile.argtypes = [ctypes.c_void_p, ctypes.c_int]
rt.check(L.rt_set_device(0))
run = helpers.GpuRun(scene)
g = rt.GBuffer(W, H)
opt = rt.options(W, H, 8, adaptive=False, kernel=rt.KERNEL_WAVEFRONT)
rt.render(run.dev, g, run.camera, 0, opt)
buf = (ctypes.c_ulonglong * 8)()
rt.check(L.rt_debug_phase_profile(buf, 1))
for long_depth in (0, -1):  # with the deep-path hand-off (default) and with deep paths kept in the finisher
    t = time.perf_counter()
    rt.render(run.dev, g, run.camera, 1, rt.options(W, H, passes, adaptive=False, kernel=rt.KERNEL_WAVEFRONT,
                                                     wf_long_depth=long_depth, profile=True))
    rt.join()
    wall = time.perf_counter() - t
    prof = rt.last_profile()
    rt.check(L.rt_debug_phase_profile(buf, 1))
    v = list(buf)
    tot = sum(v[:4]) or 1
    out = {"scene": scene, "passes": passes, "wf_long_depth": long_depth, "wall_s": round(wall, 3),
           "finish_ms": round(prof["finish_ms"], 1),
           "share": {k: round(v[i] / tot, 4) for i, k in enumerate(["overhead", "bvh_query", "kd_phase", "shade"])},
           "iterations": v[4], "lanes_per_query": round(v[5] / max(v[4], 1), 2),
           "lanes_in_trace": round(v[6] / max(v[4], 1), 2)}
    print(json.dumps(out), flush=True)
