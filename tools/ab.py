"""A/B kernel variants in ONE process, interleaved rounds (guide §5.4 rule 24).
Round r renders the same samples (seeds = mt19937 outputs [r*W*H, (r+1)*W*H))
for every variant, so the work is identical and only the timing differs.

usage: python tools/ab.py SCENE PASSES MAX_DEPTH ROUNDS VARIANT[,VARIANT...]
  VARIANT = KERNEL[:WF_TAIL[:WF_FINISH_WAVES[:DESCENT_CAP[:POSTPONE[:WIDE[:PIPES[:LONG_DEPTH]]]]]]]; KERNEL 0 mega,
            1 wavefront
            (cooperative leaves), 2 wavefront static, 3 wavefront lane fetch
Prints per-variant Msamples/s (median, min, max) at 1920x1080 and the work
counters of one counted run.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("isaklm-raytracer_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import helpers  # noqa: E402
import rt  # noqa: E402


def main():
    scene, P, maxd, rounds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    variants = sys.argv[5].split(",")

    def opts(v, **kw):
        f = [int(x) for x in v.split(":")] + [0, 0, 0, 0, 0, 0, 0]
        return rt.options(W, H, P, adaptive=False, max_depth=maxd, kernel=f[0], wf_tail=f[1], wf_finish_waves=f[2],
                          wf_descent_cap=f[3], wf_postpone=f[4], wf_wide=f[5], wf_pipelines=f[6],
                          wf_long_depth=f[7], **kw)

    W, H = int(os.environ.get("AB_W", 1920)), int(os.environ.get("AB_H", 1080))
    run = helpers.GpuRun(scene)
    g = rt.GBuffer(W, H)
    n = W * H
    zf3, zf, zi = np.zeros((n, 3), np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32)
    times = {v: [] for v in variants}
    profs = {v: [] for v in variants}
    for r in range(rounds):
        seeds = rt.seeds(n, r * n)  # every variant renders the same samples in round r
        for v in variants:
            g.upload(zf3, zf, zi, seeds)
            opt = opts(v, profile=True)
            rt.check(rt.lib().rt_synchronize())
            t = time.perf_counter()
            rt.render(run.dev, g, run.camera, 0, opt)
            times[v].append(time.perf_counter() - t)
            print(f"round {r} {v} {times[v][-1]:.3f} s", file=sys.stderr, flush=True)  # progress (gpurun: silence kills)
            if v.split(":")[0] != "0":
                profs[v].append(rt.last_profile())
    out = {}
    if os.environ.get("AB_NO_COUNT"):  # timing only (tools/gpu_ab_libs.sh)
        for v in variants:
            ts = np.array(times[v])
            out[v] = {"msamples_s_median": round(W * H * P / np.median(ts) / 1e6, 3), "s": [round(x, 3) for x in ts]}
        print(json.dumps({"scene": scene, "passes": P, "max_depth": maxd, "variants": out}, indent=1))
        return
    for v in variants:
        cnt = rt.DeviceCounters()
        g.upload(zf3, zf, zi, rt.seeds(n, 0))
        opt = opts(v, counters=cnt.p)
        rt.render(run.dev, g, run.camera, 0, opt)
        c = cnt.read(finisher=True)
        ts = np.array(times[v])
        out[v] = {"msamples_s_median": round(W * H * P / np.median(ts) / 1e6, 3),
                  "msamples_s_best": round(W * H * P / ts.min() / 1e6, 3),
                  "s": [round(x, 3) for x in ts], "maxdepth": c["maxdepth"],
                  "trace_ms": [round(p["trace_ms"]) for p in profs[v]],
                  "shade_ms": [round(p["shade_ms"]) for p in profs[v]],
                  "finish_ms": [round(p["finish_ms"]) for p in profs[v]],
                  "iterations": [p["iterations"] for p in profs[v]],
                  "per_sample": {k: round(c[k] / max(c["sample"], 1), 2) for k in ("ray", "node", "tri", "cand", "plane", "rounds", "chunks", "bary", "t_descend", "t_leaves", "t_fetch", "finish_node", "finish_tri", "finish_ray",
                                                                                          "t_leaf_wait", "t_leaf_setup", "t_leaf_test", "t_leaf_bary",
                                                                                          "spill_push", "spill_pop", "pend_lanes", "leaf_tests",
                                                                                          "t_desc_wait")},
                  "wide": {"calls": c["wide_calls"], "rounds_per_call": round(c["wide_rounds"] / max(c["wide_calls"], 1), 2),
                           "clk_per_call": round(c["t_wide"] / max(c["wide_calls"], 1)),
                           "clk_per_round": {k: round(c[k] / max(c["wide_rounds"], 1))
                                             for k in ("t_wide_load", "t_wide_leaf", "t_wide_expand")}},
                  "wave_time_split": {k: round(c[k] / max(c["t_descend"] + c["t_leaves"] + c["t_fetch"], 1), 3)
                                      for k in ("t_descend", "t_leaves", "t_fetch")}}
    print(json.dumps({"scene": scene, "passes": P, "max_depth": maxd, "variants": out}, indent=1))


if __name__ == "__main__":
    main()
