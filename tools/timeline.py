"""Per-launch timeline of wf_trace_coop (debug): how much of each trace
launch runs after its ray queue is exhausted (the launch's tail, when waves
only finish the rays they hold).

usage: python tools/timeline.py SCENE PASSES
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("isaklm-raytracer_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import helpers  # noqa: E402
import rt  # noqa: E402

N = 4096


def main():
    scene, P = sys.argv[1], int(sys.argv[2])
    W, H = 1920, 1080
    run = helpers.GpuRun(scene)
    g = rt.GBuffer(W, H)
    buf = ctypes.c_void_p()
    rt.check(rt.lib().rt_device_alloc(ctypes.byref(buf), 3 * N * 8))
    out = {}
    for rep in range(2):
        rt.check(rt.lib().rt_memset(buf, 0xFF, 3 * N * 8))
        opt = rt.options(W, H, P, adaptive=False, kernel=rt.KERNEL_WAVEFRONT, profile=True, wave_times=buf)
        rt.render(run.dev, g, run.camera, 0, opt)
        prof = rt.last_profile()
        a = np.zeros(3 * N, np.uint64)
        rt.check(rt.lib().rt_download(a.ctypes.data, buf, a.nbytes))
        a = a.reshape(N, 3)[:prof["iterations"]]
        start, exh, end = a[:, 0].astype(np.float64), a[:, 1].astype(np.float64), (~a[:, 2]).astype(np.float64)
        dur = (end - start) / 1e5  # 100 MHz ticks -> ms
        tail = (end - exh) / 1e5
        out[rep] = {"iterations": prof["iterations"], "trace_ms_events": round(prof["trace_ms"], 1),
                    "sum_launch_ms": round(float(dur.sum()), 1), "sum_tail_ms": round(float(tail.sum()), 1),
                    "tail_share": round(float(tail.sum() / dur.sum()), 3),
                    "first_launches": [(round(float(d), 2), round(float(t), 2)) for d, t in zip(dur[:6], tail[:6])],
                    "last_launches": [(round(float(d), 2), round(float(t), 2)) for d, t in zip(dur[-6:], tail[-6:])]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
