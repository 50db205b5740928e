"""Debug: the light-guide trap (600 long) against the oracle under several settings; prints mismatching pixels."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

rt.check(rt.lib().rt_set_device(0))
path = helpers.make_trap_scene("/tmp/trap600", 600.0)
run = helpers.GpuRun(path)
W, H, P = 64, 48, 4
ref, _ = helpers.oracle_render(path, W, H, P, calls=2)
cases = [dict(), dict(wf_long_depth=-1), dict(overlap=True), dict(traversal=rt.TRAVERSAL_KD),
         dict(kernel=rt.KERNEL_MEGA), dict(wf_long_depth=1000000)]
for kw in cases:
    k = dict(kernel=rt.KERNEL_WAVEFRONT)
    k.update(kw)
    gpu, _, _ = run.render(W, H, P, calls=2, **k)
    bad = np.nonzero((gpu[0].view(np.uint32) != ref[0].view(np.uint32)).any(axis=1) |
                     (gpu[3] != ref[3]))[0]
    print(kw, "mismatching pixels:", len(bad), bad[:10].tolist(), flush=True)
