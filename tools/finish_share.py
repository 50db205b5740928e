"""Share of the work done by the cooperative finisher (debug): one counted
call of PASSES on SCENE at 1920x1080; prints rays / node visits / triangle
tests of the whole call and of the finisher, and the profile split.
usage: python tools/finish_share.py SCENE PASSES"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("isaklm-raytracer_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import helpers  # noqa: E402
import rt  # noqa: E402


def main():
    scene, P = sys.argv[1], int(sys.argv[2])
    W, H = 1920, 1080
    run = helpers.GpuRun(scene)
    g = rt.GBuffer(W, H)
    out = {}
    for counted in (False, True):
        cnt = rt.DeviceCounters() if counted else None
        opt = rt.options(W, H, P, adaptive=False, kernel=rt.KERNEL_WAVEFRONT, profile=not counted,
                         counters=cnt.p if cnt else None)
        rt.render(run.dev, g, run.camera, 1, opt)
        if counted:
            c = cnt.read(finisher=True)
            out["counters"] = {k: c[k] for k in ("ray", "node", "tri", "finish_ray", "finish_node", "finish_tri",
                                                 "sample", "maxdepth")}
            out["finisher_share"] = {k: round(c["finish_" + k] / max(c[k], 1), 4) for k in ("ray", "node", "tri")}
        else:
            out["profile"] = {k: v for k, v in rt.last_profile().items()}
        print(json.dumps(out), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
