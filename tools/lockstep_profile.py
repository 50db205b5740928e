"""Lockstep profile of the whole-call finisher's ray queries (wf_finish_bvh):
each lane runs its own path, but a wave's BVH query and its KD phase each run
until the wave's slowest lane is done.  Reports, over one counted call (the
finisher's COUNT instantiation, RT_TRAVERSAL_BOUNDED_COUNTED), the lane steps
the rays need (BVH / KD nodes, plane records in batches of 4) against the
lane-steps the waves spend (64 x the slowest lane's steps per query), per
phase: the SIMT efficiency of the one-ray-per-lane query.
Needs the -DRT_LOCKSTEP_PROF build: bash tools/mkvariant.sh lockstep -DRT_LOCKSTEP_PROF, then
ISAKLM_RT_LIB_OVERRIDE=ab_libs/lockstep.so python tools/lockstep_profile.py [scene] [passes] [W] [H]."""
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
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 16
W = int(sys.argv[3]) if len(sys.argv) > 3 else 1920
H = int(sys.argv[4]) if len(sys.argv) > 4 else 1080
L = rt.lib()
L.rt_debug_phase_profile.argtypes = [ctypes.c_void_p, ctypes.c_int]
rt.check(L.rt_set_device(0))
run = helpers.GpuRun(scene)
g = rt.GBuffer(W, H)
rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 2, adaptive=False, kernel=rt.KERNEL_WAVEFRONT))
buf = (ctypes.c_ulonglong * 8)()
rt.check(L.rt_debug_phase_profile(buf, 1))
cnt = rt.DeviceCounters()
t = time.perf_counter()
rt.render(run.dev, g, run.camera, 1, rt.options(W, H, passes, adaptive=False, kernel=rt.KERNEL_WAVEFRONT,
                                                 counters=cnt.p, traversal=rt.TRAVERSAL_BOUNDED_COUNTED,
                                                 profile=True))
rt.join()
wall = time.perf_counter() - t
prof = rt.last_profile()
rt.check(L.rt_debug_phase_profile(buf, 1))
v = [int(x) for x in buf]
c = cnt.read(finisher=True)
out = {"scene": scene, "W": W, "H": H, "passes": passes, "wall_s": round(wall, 3),
       "finish_ms": round(prof["finish_ms"], 1), "finish_launches": prof["finish_launches"],
       "queries": c["ray"],
       "efficiency_total": round(v[1] / max(v[2] + v[4], 1), 4),
       "efficiency_bvh": round(v[3] / max(v[2], 1), 4),
       "efficiency_kd": round(v[5] / max(v[4], 1), 4),
       "lane_steps_per_ray": {"bvh": round(v[3] / max(c["ray"], 1), 2), "kd": round(v[5] / max(c["ray"], 1), 2)},
       "wave_steps_per_query": {"bvh": round(v[2] / 64 / max(v[0], 1), 2), "kd": round(v[4] / 64 / max(v[0], 1), 2)},
       "active_lanes_per_query": round(v[6] / max(v[0], 1), 2),
       "cycles_per_wave_query": round(v[7] / max(v[0], 1), 1),
       "raw": v,
       "trace_wave_cycles": v[7]}
print(json.dumps(out), flush=True)
