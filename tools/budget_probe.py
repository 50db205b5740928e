import sys, os, json, numpy as np
ROOT = "/root/repo" if os.path.exists("/root/repo/tests") else os.getcwd()
sys.path[:0] = [os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import helpers, rt
rt.check(rt.lib().rt_set_device(0))
run = helpers.GpuRun("room2m")
W, H = 1920, 1080
for calls in ([256, 256], [256, 256, 256], [256] * 4, [64] * 4):
    rt.deviation_stats(reset=True)
    gpu, _, _ = run.render(W, H, calls, kernel=rt.KERNEL_WAVEFRONT)
    st = rt.deviation_stats(reset=True)
    c = gpu[2]
    print(json.dumps({"calls": calls, "count_min": int(c.min()), "count_max": int(c.max()), "count_mean": float(c.mean()),
                      "n_bad": int((c != sum(calls)).sum()), "owed": st["owed_pixels"], "stranded": st["stranded_pixels"],
                      "deep": st["deep_paths"]}), flush=True)
