"""Where a lone deep path's time goes: the glass light guide at a handful of
pixels, 1 pass, the counting build (wf_long traces with the 64-lane wide KD
traversal; its s_memtime phase counters: RT_CNT_T_WIDE = cycles inside
wide_trace, RT_CNT_WIDE_CALLS = rays, RT_CNT_WIDE_ROUNDS = frontier rounds).

usage: python tools/deep_profile.py [pixels]
"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("isaklm-raytracer_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import helpers  # noqa: E402
import rt  # noqa: E402


def main():
    npx = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    d = tempfile.mkdtemp(prefix="deepprof_")
    run = helpers.GpuRun(helpers.make_trap_scene(d, length=60.0))
    W, H = npx, 1
    out = []
    for r in range(3):
        g = rt.GBuffer(W, H, r * W * H)
        cnt = rt.DeviceCounters()
        rt.deviation_stats(reset=True)
        rt.check(rt.lib().rt_synchronize())
        t = time.perf_counter()
        rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 1, adaptive=False, kernel=rt.KERNEL_WAVEFRONT,
                                                         counters=cnt.p))
        rt.check(rt.lib().rt_synchronize())
        dt = time.perf_counter() - t
        c = cnt.read(finisher=True)
        dev = rt.deviation_stats()
        calls = max(c["wide_calls"], 1)
        res = {"call_ms": round(dt * 1e3, 2), "max_depth": dev["max_deep_depth"], "rays": c["ray"],
               "wide_calls": c["wide_calls"], "rounds_per_wide_call": round(c["wide_rounds"] / calls, 2),
               "wide_cycles_per_call": round(c["t_wide"] / calls), "load_cycles_per_call": round(c["t_wide_load"] / calls),
               "leaf_cycles_per_call": round(c["t_wide_leaf"] / calls),
               "expand_cycles_per_call": round(c["t_wide_expand"] / calls),
               "us_per_bounce_wall": round(dt * 1e6 / max(dev["max_deep_depth"], 1), 2)}
        out.append(res)
        print(res, file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
