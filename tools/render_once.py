"""One room2m render of PASSES passes after a warm-up call (profiler target:
rocprofv3 kernel traces / counter passes / PC sampling of the default render).
usage: python tools/render_once.py [SCENE] [PASSES] [W] [H]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("isaklm-raytracer_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import helpers  # noqa: E402
import rt  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "room2m"
P = int(sys.argv[2]) if len(sys.argv) > 2 else 16
W = int(sys.argv[3]) if len(sys.argv) > 3 else 1920
H = int(sys.argv[4]) if len(sys.argv) > 4 else 1080
run = helpers.GpuRun(scene)
g = rt.GBuffer(W, H)
rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 2, adaptive=False, kernel=rt.KERNEL_WAVEFRONT))
rt.join()
t = time.perf_counter()
rt.render(run.dev, g, run.camera, 1, rt.options(W, H, P, adaptive=False, kernel=rt.KERNEL_WAVEFRONT))
rt.join()
dt = time.perf_counter() - t
print(f"{scene} {W}x{H} {P} passes: {dt:.3f} s, {W * H * P / dt / 1e6:.1f} Msamples/s", flush=True)
