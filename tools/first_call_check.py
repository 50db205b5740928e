"""One process = one first call: test_gpu_chain's room2m case as the test
runs it at the start of a process (an unchained 64-pass call, then 4 chained
16-pass calls on a user stream), then a second unchained call; prints which
frames differ bitwise (NaN-safe) and where — for an intermittent first-call
difference.  usage: python tools/first_call_check.py"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

W, H = 1920, 1080
rt.check(rt.lib().rt_set_device(0))
hip = ctypes.CDLL("libamdhip64.so")
s = ctypes.c_void_p()
assert hip.hipStreamCreate(ctypes.byref(s)) == 0
run = helpers.GpuRun("room2m")
one = run.render(W, H, [64], kernel=rt.KERNEL_WAVEFRONT, overlap=False)[0]
ch = run.render(W, H, [16, 16, 16, 16], kernel=rt.KERNEL_WAVEFRONT, overlap=True, stream=s)[0]
two = run.render(W, H, [64], kernel=rt.KERNEL_WAVEFRONT, overlap=False)[0]


def diff(a, b):
    bad = np.zeros(W * H, bool)
    for x, y in zip(a, b):
        bad |= np.any(x.reshape(W * H, -1).view(np.uint32) != y.reshape(W * H, -1).view(np.uint32), axis=1)
    idx = np.nonzero(bad)[0]
    return {"n": int(len(idx)), "px": [int(i) for i in idx[:6]],
            "a": [a[0].reshape(-1, 3)[i].tolist() + [int(a[2].reshape(-1)[i])] for i in idx[:3]],
            "b": [b[0].reshape(-1, 3)[i].tolist() + [int(b[2].reshape(-1)[i])] for i in idx[:3]]}


print(json.dumps({"one_vs_chained": diff(one, ch), "one_vs_two": diff(one, two), "chained_vs_two": diff(ch, two)}),
      flush=True)
