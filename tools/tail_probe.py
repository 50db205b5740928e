"""Probe the per-launch tail of the megakernel: per-wave durations
(s_memrealtime, 100 MHz) and path-length extremes on a scene.

usage: python tools/tail_probe.py [scene] [passes] [max_depth]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "isaklm-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import helpers  # noqa: E402
import rt  # noqa: E402


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "room2m"
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    maxd = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    W, H = 1920, 1080
    run = helpers.GpuRun(scene)
    g = rt.GBuffer(W, H)
    waves = ((W + 15) // 16) * ((H + 15) // 16) * 4
    wt = ctypes.c_void_p()
    rt.check(rt.lib().rt_device_alloc(ctypes.byref(wt), waves * 16))
    res = {}
    for kernel in (rt.KERNEL_MEGA, rt.KERNEL_WAVEFRONT):
        cnt = rt.DeviceCounters()
        rt.check(rt.lib().rt_memset(wt, 0, waves * 16))
        opt = rt.options(W, H, P, adaptive=False, max_depth=maxd, counters=cnt.p, kernel=kernel)
        opt.wave_times_device = wt
        t = time.perf_counter()
        rt.render(run.dev, g, run.camera, 0, opt)
        dt = time.perf_counter() - t
        c = cnt.read()
        r = {"wall_s": round(dt, 4), "msamples_s": round(W * H * P / dt / 1e6, 3), "counters": c}
        if kernel == rt.KERNEL_MEGA:
            a = np.zeros(waves * 2, dtype=np.uint64)
            rt.check(rt.lib().rt_download(ctypes.c_void_p(a.ctypes.data), wt, a.nbytes))
            a = a.reshape(-1, 2).astype(np.float64)
            t0 = a[:, 0].min()
            start, end = (a[:, 0] - t0) / 1e5, (a[:, 1] - t0) / 1e5  # ms
            dur = end - start
            r["wave_ms_percentiles"] = {p: round(float(np.percentile(dur, p)), 2) for p in (50, 90, 99, 99.9, 100)}
            r["kernel_span_ms"] = round(float(end.max()), 2)
            for frac in (0.5, 0.9, 0.99):
                r[f"t_{int(frac*100)}pct_waves_done_ms"] = round(float(np.quantile(end, frac)), 2)
        res["mega" if kernel == rt.KERNEL_MEGA else "wavefront"] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
