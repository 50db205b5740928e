"""bench.py's measurement code on CPU: the counter-window parser and the
counter-measured roofline arithmetic (FETCH_SIZE x2 + WRITE_SIZE per sample x
samples/s), on synthetic rocprofv3 CSVs."""
import csv
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]


def _csv(path, rows, fields=FIELDS):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(fields, r)))


def _pass(tmp_path, tag, counter, per_kernel):
    """Dispatches: warm-up trace (outside), marker, trace, shade, long, marker, trace (outside)."""
    rows = [(1, "void wf_trace_coop<false>(...)", counter, 999.0), (2, "rt_tonemap_kernel(...)", counter, 0.0)]
    i = 3
    for k, v in per_kernel.items():
        rows.append((i, f"void {k}(RtDevScene, ...)", counter, v))
        i += 1
    rows += [(i, "rt_tonemap_kernel(...)", counter, 0.0), (i + 1, "void wf_trace_coop<false>(...)", counter, 777.0)]
    cc = tmp_path / f"{tag}_counter_collection.csv"
    _csv(cc, rows)
    trace = tmp_path / f"{tag}_kernel_trace.csv"
    _csv(trace, [(r[0], r[1], 1000 * r[0], 1000 * r[0] + 500) for r in rows],
         ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
    return str(cc), str(trace)


def test_window_sums_take_only_the_marked_call(tmp_path):
    cc, tr = _pass(tmp_path, "f", "FETCH_SIZE", {"wf_trace_coop<false>": 100.0, "wf_shade<false>": 10.0})
    total, per_kernel, n, kt = bench._window_sums(cc, tr)
    assert total == {"FETCH_SIZE": 110.0}
    assert n == 2
    assert per_kernel["wf_trace_coop<false>"]["FETCH_SIZE"] == 100.0
    assert kt["wf_shade<false>"]["dispatches"] == 1


def test_roofline_from_counters(tmp_path):
    fetch = {"wf_trace_coop<false>": 1000.0, "wf_shade<false>": 50.0, "wf_long<false>": 1.0}
    write = {"wf_trace_coop<false>": 10.0, "wf_shade<false>": 40.0, "wf_long<false>": 0.0}
    sq = {"wf_trace_coop<false>": 0.0}
    passes = {}
    for tag, ctr, vals in (("fetch", "FETCH_SIZE", fetch), ("write", "WRITE_SIZE", write)):
        cc, tr = _pass(tmp_path, tag, ctr, vals)
        total, per_kernel, n, kt = bench._window_sums(cc, tr)
        passes[tag] = {"counters": total, "per_kernel": per_kernel, "dispatches": n, "kernel_trace": kt,
                       "wall_s": 1.0, "samples": 1000}
    sq_rows = []
    for k, (wc, wait, inst, valu, thr) in {"wf_trace_coop<false>": (1000.0, 600.0, 300.0, 100.0, 4800.0),
                                            "wf_long<false>": (9000.0, 8900.0, 10.0, 5.0, 64.0)}.items():
        sq_rows.append((k, {"SQ_WAVE_CYCLES": wc, "SQ_WAIT_ANY": wait, "SQ_ACTIVE_INST_ANY": inst,
                            "SQ_ACTIVE_INST_VALU": valu, "SQ_THREAD_CYCLES_VALU": thr}))
    sq_total = {c: sum(v[c] for _, v in sq_rows) for c in sq_rows[0][1]}
    passes["sq"] = {"counters": sq_total, "per_kernel": dict(sq_rows), "dispatches": 2, "kernel_trace": {},
                    "wall_s": 1.0, "samples": 1000}
    achieved, d = bench.roofline_from_pmc({"passes": passes}, samples_per_s=1e6)
    fetch_b = 2 * 1024 * sum(fetch.values())
    write_b = 1024 * sum(write.values())
    assert d["hbm_bytes_per_sample"] == pytest.approx((fetch_b + write_b) / 1000, rel=1e-3)
    assert d["hbm_bytes_per_sample_raw"] == pytest.approx((fetch_b / 2 + write_b) / 1000, rel=1e-3)
    assert achieved == pytest.approx((fetch_b + write_b) / 1000 * 1e6 / 1e9)
    # the dominant kernel moves the most bytes (wf_long's slices only poll)
    assert d["dominant_kernel"] == "wf_trace_coop<false>"
    assert d["latency"]["scope"] == "wf_trace_coop<false>"
    assert d["latency"]["wait_frac"] == pytest.approx(0.6)
    assert d["latency"]["valu_lane_util"] == pytest.approx(4800.0 / (64 * 100.0), abs=1e-3)


def test_metric_names_the_rendered_frame():
    assert "1920×1080" in bench.METRIC


def test_call_plan_groups_steps_into_calls():
    # the driver's --steps 20 --warmup 5 with the default 4 steps per call
    assert bench.call_plan(0, 5, 4) == [(0, 4), (4, 1)]
    assert bench.call_plan(5, 20, 4) == [(5, 4), (9, 4), (13, 4), (17, 4), (21, 4)]
    # every step rendered exactly once, only the first call starts at step 0
    for first, count, per in ((0, 1, 4), (1, 4, 4), (0, 7, 3), (3, 0, 4), (2, 9, 1)):
        plan = bench.call_plan(first, count, per)
        covered = [s for start, k in plan for s in range(start, start + k)]
        assert covered == list(range(first, first + count))
        assert all(1 <= k <= per for _, k in plan)
    args = bench.parse_args([])
    assert args.passes * args.steps_per_call == 256
