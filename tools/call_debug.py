"""Consecutive room2m calls with the wavefront debug log (RT_WF_TRACE_ITERS=1):
per call, the wall time and the library's [wf] lines with their timestamps
made relative to the call's start (time.monotonic = CLOCK_MONOTONIC).  Used
to see where an outlier call's time goes (finishers, long-path slices).

usage: RT_WF_TRACE_ITERS=1 python tools/call_debug.py [passes] [calls]
"""
import os
import re
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("isaklm-raytracer_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import helpers  # noqa: E402
import rt  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    W, H = 1920, 1080
    run = helpers.GpuRun("room2m")
    g = rt.GBuffer(W, H)
    tmp = tempfile.NamedTemporaryFile(mode="w+", suffix=".log", delete=False)
    saved = os.dup(2)
    for c in range(calls):
        os.dup2(tmp.fileno(), 2)
        tmp.seek(0)
        tmp.truncate()
        t0 = time.monotonic()
        rt.render(run.dev, g, run.camera, 0 if c == 0 else 1,
                  rt.options(W, H, P, adaptive=False, kernel=rt.KERNEL_WAVEFRONT))
        t1 = time.monotonic()
        os.dup2(saved, 2)
        tmp.seek(0)
        lines = []
        for ln in tmp.read().splitlines():
            if " it " in ln:
                continue
            m = re.search(r"t ([0-9]+\.[0-9]+)$", ln)
            lines.append(re.sub(r"t [0-9]+\.[0-9]+$", f"t +{float(m.group(1)) - t0:.3f}", ln) if m else ln)
        print(f"call {c}: {t1 - t0:.3f} s", flush=True)
        for ln in lines:
            print("   " + ln, flush=True)


if __name__ == "__main__":
    main()
