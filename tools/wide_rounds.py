"""Where a deep bounce's time goes in wf_long's wide KD traversal (the verdict's
per-round split): one counted room2m call (RtOptions.counters: the counting
build, KD traversal, deep paths in wf_long<true>) and the wide traversal's own
counters — calls (= bounces traced wide), frontier rounds, and s_memtime
cycles in the frontier + node load wait, the cooperative leaf batch and the
expansion (RT_CNT_WIDE_*, RT_CNT_T_WIDE_*; the counting build waits for each
phase's loads, so the split is of that build).  usage: python tools/wide_rounds.py [passes] [scene]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

passes = int(sys.argv[1]) if len(sys.argv) > 1 else 8
scene = sys.argv[2] if len(sys.argv) > 2 else "room2m"
W, H = 1920, 1080
rt.check(rt.lib().rt_set_device(0))
run = helpers.GpuRun(scene)
g = rt.GBuffer(W, H)
cnt = rt.DeviceCounters()
rt.render(run.dev, g, run.camera, 0, rt.options(W, H, passes, adaptive=False, kernel=rt.KERNEL_WAVEFRONT,
                                                 counters=cnt.p))
rt.join()
a = np.zeros(rt.N_COUNTERS, dtype=np.uint64)
rt.check(rt.lib().rt_download(rt._ptr(a), cnt.p, a.nbytes))
calls, rounds, t, tl, tf, te = (int(a[i]) for i in (22, 23, 24, 25, 26, 27))
print(json.dumps({"scene": scene, "passes": passes, "wide_calls": calls, "rounds": rounds,
                  "rounds_per_call": round(rounds / max(calls, 1), 2),
                  "cycles_per_call": round(t / max(calls, 1), 1), "cycles_per_round": round(t / max(rounds, 1), 1),
                  "share": {"frontier_and_load_wait": round(tl / max(t, 1), 3), "leaf_batch": round(tf / max(t, 1), 3),
                            "expansion": round(te / max(t, 1), 3)},
                  "note": "s_memtime shader cycles; counting build (each phase waits for its loads)"}), flush=True)
