"""Per-bounce latency of a lone deep path: the glass light guide
(tests/helpers.make_trap_scene: total internal reflection down a 60-unit rod)
rendered at a handful of pixels, 1 pass, so every path is deep and the call
time is the longest path's chain.  Prints call time / longest path (from the
always-on deviation statistics) for the ways a deep path can run:
wf_long (64 lanes, wide KD traversal), the bounded finisher's own lane
(wf_long off) and the bounded megakernel.

usage: python tools/deep_latency.py [pixels] [rounds]
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
    npx = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    d = tempfile.mkdtemp(prefix="deeplat_")
    run = helpers.GpuRun(helpers.make_trap_scene(d, length=60.0))
    W, H = npx, 2
    variants = {"wf_long (wide KD)": dict(kernel=rt.KERNEL_WAVEFRONT),
                "finisher lane (bounded)": dict(kernel=rt.KERNEL_WAVEFRONT, wf_long_depth=-1),
                "megakernel (bounded)": dict(kernel=rt.KERNEL_MEGA)}
    out = {}
    for name, kw in variants.items():
        res = []
        for r in range(rounds):
            g = rt.GBuffer(W, H, r * W * H)
            rt.deviation_stats(reset=True)
            rt.check(rt.lib().rt_synchronize())
            t = time.perf_counter()
            rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 1, adaptive=False, **kw))
            rt.check(rt.lib().rt_synchronize())
            dt = time.perf_counter() - t
            dev = rt.deviation_stats()
            res.append({"call_ms": round(dt * 1e3, 2), "max_depth": dev["max_deep_depth"],
                        "us_per_bounce": round(dt * 1e6 / max(dev["max_deep_depth"], 1), 2)})
            print(name, res[-1], file=sys.stderr, flush=True)
        out[name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
