"""Deep-sample log (RtOptions.debug = RT_DEBUG_LONG_LOG) of unchained room2m
1920x1080 calls: per call, the latest-ending deep samples, the longest ones
and the pixels whose deep samples end last (stderr).
usage: python tools/deep_log.py [calls] [passes per call]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 256
W, H = 1920, 1080
rt.check(rt.lib().rt_set_device(0))
run = helpers.GpuRun(os.environ.get("RT_SCENE", "room2m"))
g = rt.GBuffer(W, H)
rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 16, adaptive=False, kernel=rt.KERNEL_WAVEFRONT))
rt.join()
for i in range(calls):
    print(f"call {i}", file=sys.stderr, flush=True)
    rt.render(run.dev, g, run.camera, 1, rt.options(W, H, passes, adaptive=False, kernel=rt.KERNEL_WAVEFRONT,
                                                     debug=2))  # RT_DEBUG_LONG_LOG
    rt.join()
