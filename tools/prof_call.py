"""One profiled whole-call render (room2m 1080p, unchained, `passes` passes)
after a 2-pass warm-up, for rocprofv3 counter passes on wf_finish_bvh.
usage: rocprofv3 --pmc ... -- python3 tools/prof_call.py [passes] [scene]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

passes = int(sys.argv[1]) if len(sys.argv) > 1 else 16
scene = sys.argv[2] if len(sys.argv) > 2 else "room2m"
W, H = 1920, 1080
import threading  # noqa: E402
import time  # noqa: E402


def heartbeat():  # (under counter collection a call runs for minutes: show it is alive)
    t0 = time.time()
    while True:
        time.sleep(20)
        print(f"[prof_call] running {time.time() - t0:.0f} s", file=sys.stderr, flush=True)


threading.Thread(target=heartbeat, daemon=True).start()
rt.check(rt.lib().rt_set_device(0))
run = helpers.GpuRun(scene)
g = rt.GBuffer(W, H)
dbg = int(os.environ.get("PROF_CALL_DEBUG", "0"))
extra = dict(check_interval=int(os.environ.get("PROF_CALL_CHECK", "0")),
             wf_long_depth=int(os.environ.get("PROF_CALL_LONG", "0")))
rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 2, adaptive=False, kernel=rt.KERNEL_WAVEFRONT, debug=dbg,
                                                **extra))
print("warm-up call issued", file=sys.stderr, flush=True)
rt.join()
print("warm-up call joined", file=sys.stderr, flush=True)
rt.render(run.dev, g, run.camera, 1, rt.options(W, H, passes, adaptive=False, kernel=rt.KERNEL_WAVEFRONT, debug=dbg,
                                                 **extra))
rt.join()
print("done", flush=True)
