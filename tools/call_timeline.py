"""Where does a wavefront call's wall time go?  Renders room2m calls with
RT_WF_TRACE_ITERS=1 (per-iteration host timestamps on stderr, CLOCK_MONOTONIC
= time.monotonic) and reports per pipeline: the end of its queue iterations,
its finisher time (RtProfile), and the call's end — at unbounded depth and
with max_depth capped (deep total-internal-reflection chains removed; the
image differs, only the timing is of interest).

usage: RT_WF_TRACE_ITERS=1 python tools/call_timeline.py [scene] [passes] [rounds]
"""
import json
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
    scene = sys.argv[1] if len(sys.argv) > 1 else "room2m"
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    W, H = 1920, 1080
    run = helpers.GpuRun(scene)
    g = rt.GBuffer(W, H)
    out = []
    # stderr of the library (fd 2) into a file we can read back
    tmp = tempfile.NamedTemporaryFile(mode="w+", suffix=".log", delete=False)
    saved = os.dup(2)
    for r in range(rounds):
        for maxd in (0, 64):
            os.dup2(tmp.fileno(), 2)
            tmp.seek(0)
            tmp.truncate()
            t0 = time.monotonic()
            rt.render(run.dev, g, run.camera, 0,
                      rt.options(W, H, P, adaptive=False, max_depth=maxd, kernel=rt.KERNEL_WAVEFRONT, profile=True))
            t1 = time.monotonic()
            os.dup2(saved, 2)
            prof = rt.last_profile()
            tmp.seek(0)
            last = {}
            for ln in tmp.read().splitlines():
                m = re.match(r"\[wf\] pipe (\d+) it (\d+) live (\d+) t ([0-9.]+)", ln)
                if m:
                    last[int(m.group(1))] = (int(m.group(2)), int(m.group(3)), float(m.group(4)) - t0)
            out.append({"round": r, "max_depth": maxd, "call_s": round(t1 - t0, 3),
                        "pipes_iter_end_s": {k: round(v[2], 3) for k, v in sorted(last.items())},
                        "pipes_iterations": {k: v[0] + 1 for k, v in sorted(last.items())},
                        "pipes_live_at_handover": {k: v[1] for k, v in sorted(last.items())},
                        "finish_ms_sum": round(prof["finish_ms"], 1), "trace_ms_sum": round(prof["trace_ms"], 1),
                        "shade_ms_sum": round(prof["shade_ms"], 1), "call_ms": round(prof["call_ms"], 1)})
            print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
