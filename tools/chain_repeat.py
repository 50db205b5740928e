"""Repeat test_gpu_chain's room2m case in ONE process: one unchained 64-pass
call as the reference frame, then N rounds of 4 chained 16-pass calls (and an
unchained repeat every other round), printing the differing pixels per round
— a rate for an intermittent difference.  usage: python tools/chain_repeat.py [N]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers  # noqa: E402
import rt  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
scene = sys.argv[2] if len(sys.argv) > 2 else "room2m"
W, H = (1920, 1080) if scene == "room2m" else (640, 360)
rt.check(rt.lib().rt_set_device(0))
hip = ctypes.CDLL("libamdhip64.so")
s = ctypes.c_void_p()
assert hip.hipStreamCreate(ctypes.byref(s)) == 0
run = helpers.GpuRun(scene)
one = run.render(W, H, [64], kernel=rt.KERNEL_WAVEFRONT, overlap=False)[0]
two = run.render(W, H, [64], kernel=rt.KERNEL_WAVEFRONT, overlap=False)[0]


def diff(a, b):
    bad = np.nonzero(np.any(a[0].reshape(-1, 3) != b[0].reshape(-1, 3), axis=1) |
                     (a[2].reshape(-1) != b[2].reshape(-1)))[0]
    return [int(x) for x in bad[:8]], int(len(bad))


f, nb = diff(one, two)
print(json.dumps({"first_vs_second_call": nb, "first": f,
                  "pixels": [{"px": k, "fb1": one[0].reshape(-1, 3)[k].tolist(), "fb2": two[0].reshape(-1, 3)[k].tolist(),
                              "count1": int(one[2].reshape(-1)[k]), "count2": int(two[2].reshape(-1)[k]),
                              "sq1": float(one[1].reshape(-1)[k]), "sq2": float(two[1].reshape(-1)[k])} for k in f[:4]]}),
      flush=True)
if f:
    ref, _ = helpers.oracle_render(run.path, W, H, 64, pixels=np.array(f[:4], np.int32))
    print(json.dumps({"oracle": [{"px": k, "fb": ref[0][k].tolist(), "count": int(ref[2][k]),
                                  "first_ok": bool(np.array_equal(ref[0][k], one[0].reshape(-1, 3)[k])),
                                  "second_ok": bool(np.array_equal(ref[0][k], two[0].reshape(-1, 3)[k]))}
                                 for k in f[:4]]}), flush=True)
one = two
for i in range(N):
    ch = run.render(W, H, [16, 16, 16, 16], kernel=rt.KERNEL_WAVEFRONT, overlap=True, stream=s)[0]
    first, nb = diff(ch, one)
    out = {"round": i, "chained_vs_one": nb, "first": first}
    if i % 2 == 1:
        un = run.render(W, H, [64], kernel=rt.KERNEL_WAVEFRONT, overlap=False)[0]
        out["unchained_repeat_vs_one"] = diff(un, one)[1]
    print(json.dumps(out), flush=True)
