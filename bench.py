"""Bench: Msamples/s of the render hot path at 1920x1080 (BASELINE.json metric).

Workload (BASELINE.json configs[2]): the README-like 2M-triangle synthetic
room ("room2m": room + 1,997,568-triangle displaced gold mesh + two glass
spheres + emissive quad), 1920x1080, adaptive sampling off.  One step = one
`--passes` passes (spp) over the full frame (default 64: 16 steps are the
config's 1024 spp), inputs resident in HBM.  The renderer is called with up
to `--steps-per-call` steps at once (default 4: rt_render calls of 256
passes; RtOptions batches passes per call, SURVEY §3 "passes batched in one
launch").  Each pixel's passes are a serial chain (its RNG state runs from
one pass into the next), so a call ends with a tail in which only the
pixels with the longest chains are still running; longer calls amortise it
(room2m 1080p: 36.7 / 38.1 / 39.4 Msamples/s at 64 / 128 / 256 passes per
call, profiles/r02/passes_per_call.json).  The image is bit-identical for any
split of the passes into calls (tests/test_gpu_parity.py).

Multi-GPU (`--gpus N`): one process per GPU.  Without WORLD_SIZE in the
environment this script starts the N ranks itself (children with RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 set, before any GPU call in
the parent); under torch.distributed.run it is one of them.  Rank r renders
its spp slice (seeds = mt19937 outputs [r*W*H, (r+1)*W*H)) and
the timed region closes with the product's ONE RCCL reduce of fb/sq/count
into rank 0 (rt_reduce_shards, csrc/shards.hip) plus the tonemap.  value =
samples of all ranks / max-over-ranks wall time.  The host-side barrier and
the max use a gloo process group (no data moves through it).

Roofline (north_star: "achieved HBM GB/s vs peak"): measured, not modelled.
Before this process touches the GPU (rank 0, N=1), the same render runs in
child processes under `rocprofv3 --pmc` (FETCH_SIZE; WRITE_SIZE; SQ
counters), one call of the bench's passes between two tonemap marker
dispatches; HBM bytes per sample = the sum of FETCH_SIZE (x2 on gfx950,
MI355X_MICROARCH.md HBM section; the raw figure is reported beside it) and
WRITE_SIZE over EVERY dispatch of that call / its samples.  achieved = those
bytes per sample x the timed samples/s: chip-wide, call-level, <= peak by
construction of the counters.  The SURVEY §8d algorithmic bytes (which the
caches serve, mostly) are reported separately as `algorithmic_GBps`.

cpu_baseline: the C oracle (OpenMP) on the host cores of the GPU box on
BASELINE.md's budget (the full frame x 1 spp; the whole job for the Cornell
config), beside the reference's own single-core rate measured in the survey
container.

deviations: the always-on statistics of the timed kernels over the whole
timed region (rt_deviation_stats): watchdog / depth-limit cuts, longest path,
histogram of paths deeper than 64 bounces.
"""
import argparse
import csv
import ctypes
import glob
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

METRIC = "Msamples/sec (W×H×spp/s) at 1920×1080; achieved HBM GB/s vs peak"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# the reference's own source compiled for the CPU (g++ -O2,
# -ffp-contract=off) in the survey container, 1 core, 2.0M-tri displaced
# mesh room, 255x255 x 1 spp
REF_SINGLE_CORE = {"value": 0.0054, "unit": "Msamples/s", "cores": 1,
                   "source": "SURVEY.md §6: reference source built for the CPU, Intel Xeon (family 6 model 207), "
                             "1 thread, 2.0M-triangle synthetic room, 255x255 x 1 spp"}
SQ_COUNTERS = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
               "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU"]
MARKER = "rt_tonemap_kernel"


def algorithmic_bytes(c):
    """bytes the reference's algorithm reads/writes, layout-independent."""
    return (8 * c["node"] + 40 * c["tri"] + 116 * c["hit"] + 4 * c["texel"] + 40 * c["nee"] + 48 * c["sample"] +
            20 * c["skip"])


def call_plan(first, count, per_call):
    """(first step, steps) of each rt_render call rendering steps
    [first, first + count) in calls of up to per_call steps; the call that
    renders step 0 resets the G-buffer (sample_count 0)"""
    plan, done = [], 0
    while done < count:
        k = min(per_call, count - done)
        plan.append((first + done, k))
        done += k
    return plan


def traversal_of(args, rt):
    return rt.TRAVERSAL_BOUNDED if args.traversal == "bounded" else rt.TRAVERSAL_KD


def bounded_kernel_bytes(c):
    """Bytes the bounded finisher's algorithm reads / writes (counters of a
    RT_TRAVERSAL_BOUNDED_COUNTED call; DESIGN.md "Roofline"): per ray query
    112 B per 4-wide BVH node (4 child boxes + references), 16 B per plane
    test (BVH or KD), 56 B per barycentric record read, 8 B per KD node; per
    hit its 112-B shading record and 64-B material; per sample the pixel's
    fb / sq / count read and written (40 B)."""
    return (112 * c["b_bvh_node"] + 16 * (c["b_bvh_tri"] + c["tri"]) + 56 * c["b_bary"] + 8 * c["node"] +
            176 * c["hit"] + 40 * c["sample"])


def call_steps(args):
    """steps per timed rt_render call (the first, largest call of the plan)"""
    return max(1, min(args.steps_per_call, args.steps))


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--passes", type=int, default=64, help="spp per step")
    ap.add_argument("--steps-per-call", type=int, default=4,
                    help="steps rendered by one rt_render call (passes per call = passes x this)")
    ap.add_argument("--scene", default="room2m")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cpu-seconds", type=float, default=240.0,
                    help="cap on the CPU baseline (full frame x 1 spp unless predicted above this)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 counter passes (roofline traffic)")
    ap.add_argument("--pmc-save", default=None, help="directory to keep the parsed counter summaries in")
    ap.add_argument("--pmc-child", default=None, help=argparse.SUPPRESS)  # internal: the profiled render
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rank wiring only (no GPU): ranks meet over gloo, rank 0 prints the line")
    ap.add_argument("--kernel", choices=["mega", "wavefront"], default="wavefront")
    ap.add_argument("--traversal", choices=["bounded", "kd"], default="bounded",
                    help="ray queries: the BVH-bounded KD traversal (default) or the KD traversal alone "
                         "(RtOptions.traversal; identical images)")
    ap.add_argument("--adaptive", action="store_true", help="adaptive sampling (configs[4]); value stays nominal "
                    "W*H*spp/s, value_actual = accumulated samples/s")
    ap.add_argument("--overlap", type=int, choices=[0, 1], default=1,
                    help="chained rt_render calls (RtOptions.overlap): a call's deep-path tail overlaps the next "
                         "call; the timed region ends with the tonemap, which joins them (identical images)")
    ap.add_argument("--debug", type=int, default=0,
                    help="RtOptions.debug (diagnostics: 1 = per-call hand-off log on stderr)")
    ap.add_argument("--check-interval", type=int, default=0,
                    help="the bounded traversal's run-time guard: 1 ray in N re-traced by the KD traversal "
                         "(RtOptions.check_interval; 0 = the library default 4096, < 0 off)")
    ap.add_argument("--min-samples", type=int, default=100)
    ap.add_argument("--max-depth", type=int, default=0, help="0 = unbounded (reference)")
    ap.add_argument("--scene-dir", default=os.environ.get("RT_SCENE_DIR", os.path.join(ROOT, "build", "scenes")))
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """Start n ranks of this script (one per GPU) and wait for them.  Runs in
    a parent that never touches the GPU; rank 0 prints the JSON line."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:  # a failed rank leaves the others waiting in a collective
                    q.terminate()
        time.sleep(0.2)
    return rc


# ------------------------------------------------------------------ counters
def _collect_csv(d, name):
    hits = glob.glob(os.path.join(d, "**", f"*{name}.csv"), recursive=True)
    return hits[0] if hits else None


def _window_sums(cc_csv, trace_csv):
    """Counter sums over the dispatches strictly between the two marker
    dispatches (the profiled call), per counter and per kernel."""
    rows = list(csv.DictReader(open(cc_csv)))
    marks = sorted({int(r["Dispatch_Id"]) for r in rows if MARKER in r["Kernel_Name"]})
    if len(marks) < 2 and trace_csv:
        marks = sorted({int(r["Dispatch_Id"]) for r in csv.DictReader(open(trace_csv)) if MARKER in r["Kernel_Name"]})
    if len(marks) < 2:
        raise RuntimeError(f"marker dispatches not found in {cc_csv}")
    lo, hi = marks[-2], marks[-1]
    total, per_kernel, dispatches = {}, {}, set()
    for r in rows:
        i = int(r["Dispatch_Id"])
        if lo < i < hi:
            v = float(r["Counter_Value"])
            c = r["Counter_Name"]
            total[c] = total.get(c, 0.0) + v
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
            per_kernel.setdefault(k, {}).setdefault(c, 0.0)
            per_kernel[k][c] += v
            dispatches.add(i)
    kt = {}
    if trace_csv:
        for r in csv.DictReader(open(trace_csv)):
            i = int(r["Dispatch_Id"])
            if lo < i < hi:
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
                e = kt.setdefault(k, {"dispatches": 0, "ns": 0.0, "vgpr": None, "lds": None})
                e["dispatches"] += 1
                e["ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                for key, col in (("vgpr", "Arch_VGPR_Count"), ("lds", "LDS_Block_Size")):
                    if col in r and r[col] != "":
                        e[key] = int(float(r[col]))
    return total, per_kernel, len(dispatches), kt


PMC_PASS_LIMIT_S = 120  # a counter pass of the default bench takes 5-6 s (profiles/r05/bench_pmc_summary.json)
PMC_SETTLE_S = 30


def measure_pmc(args, save_dir):
    """rocprofv3 counter passes over one render call (child processes, run
    before this process initialises the GPU).  Returns a dict or an error."""
    # the profiled call has the timed calls' shape: passes x steps-per-call
    child = ["--pmc-child", "1", "--passes", str(args.passes * call_steps(args)), "--scene", args.scene,
             "--width", str(args.width),
             "--height", str(args.height), "--scene-dir", args.scene_dir, "--kernel", args.kernel,
             "--traversal", args.traversal, "--max-depth", str(args.max_depth), "--min-samples", str(args.min_samples)]
    if args.adaptive:
        child.append("--adaptive")
    res = {"passes": {}}
    env = dict(os.environ, TMPDIR="/tmp")
    for tag, ctrs in (("fetch", ["FETCH_SIZE"]), ("write", ["WRITE_SIZE"]), ("sq", SQ_COUNTERS)):
        d = tempfile.mkdtemp(prefix=f"rtpmc_{tag}_", dir="/tmp")
        cmd = ["timeout", "-s", "KILL", str(PMC_PASS_LIMIT_S), "rocprofv3", "--pmc", *ctrs, "--kernel-trace", "-d", d, "-o", "run",
               "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__)] + child
        t = time.perf_counter()
        print(f"[bench] counter pass '{tag}' ({' '.join(ctrs)})", file=sys.stderr, flush=True)
        # stderr passes through (rocprofv3's log and the child's progress lines: a
        # pass of a 256-pass call runs for minutes); stdout carries the child's result
        r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, text=True)
        if r.returncode != 0:
            shutil.rmtree(d, ignore_errors=True)
            # (a pass killed at its limit: round 5's two such runs read 420-446 in the timed region
            # right after it, normal rates minutes later — give the killed process's GPU work time to
            # drain before this process starts its own)
            print(f"[bench] counter pass '{tag}' failed (rc={r.returncode}): skipping the rest, "
                  f"{PMC_SETTLE_S} s settle before the timed region", file=sys.stderr, flush=True)
            time.sleep(PMC_SETTLE_S)
            return {"error": f"rocprofv3 {tag} pass rc={r.returncode} (its log: this run's stderr): {r.stdout[-300:]}",
                    "settle_s": PMC_SETTLE_S}
        cc, kt = _collect_csv(d, "counter_collection"), _collect_csv(d, "kernel_trace")
        try:
            total, per_kernel, ndisp, ktrace = _window_sums(cc, kt)
            info = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{\"pmc_child\"")][-1])
        except Exception as e:  # noqa: BLE001
            shutil.rmtree(d, ignore_errors=True)
            return {"error": f"parsing the {tag} pass: {e}"}
        res["passes"][tag] = {"counters": total, "per_kernel": per_kernel, "dispatches": ndisp,
                              "kernel_trace": ktrace, "wall_s": round(time.perf_counter() - t, 1), **info}
        shutil.rmtree(d, ignore_errors=True)
    if save_dir:
        os.makedirs(save_dir, exist_ok=True)
        with open(os.path.join(save_dir, "bench_pmc_summary.json"), "w") as f:
            json.dump(res, f, indent=1)
    return res


def pmc_child(args, rt):
    """The profiled render: warm-up call, marker, ONE call of the timed calls'
    passes (the parent passes passes x steps-per-call), marker.  Prints the
    call's sample count."""
    rt.check(rt.lib().rt_set_device(0))
    scene_file = ensure_scene(args, rt)
    host = rt.HostScene(scene_file)
    dscene = rt.DeviceScene(host)
    W, H = args.width, args.height
    g = rt.GBuffer(W, H)
    kernel = rt.KERNEL_WAVEFRONT if args.kernel == "wavefront" else rt.KERNEL_MEGA
    kw = dict(adaptive=args.adaptive, min_samples=args.min_samples, max_depth=args.max_depth, kernel=kernel,
              traversal=traversal_of(args, rt))
    rt.render(dscene, g, host.camera, 0, rt.options(W, H, 8, **kw))
    print("[bench pmc child] warm-up call done", file=sys.stderr, flush=True)
    rgba = ctypes.c_void_p()
    rt.check(rt.lib().rt_device_alloc(ctypes.byref(rgba), W * H * 4))
    rt.check(rt.lib().rt_synchronize())
    before = int(g.download()[2].sum(dtype=np.int64))
    rt.check(rt.lib().rt_tonemap(g.g, rgba, W, H, None))
    # the profiled call (a heartbeat on stderr meanwhile: under the counters a
    # 256-pass call runs for minutes)
    import threading

    done = threading.Event()

    def heartbeat():
        while not done.wait(30.0):
            print("[bench pmc child] profiled call running", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    rt.render(dscene, g, host.camera, 1, rt.options(W, H, args.passes, **kw))
    done.set()
    print(f"[bench pmc child] profiled call of {args.passes} passes done", file=sys.stderr, flush=True)
    rt.check(rt.lib().rt_synchronize())
    rt.check(rt.lib().rt_tonemap(g.g, rgba, W, H, None))
    rt.check(rt.lib().rt_synchronize())
    samples = int(g.download()[2].sum(dtype=np.int64)) - before
    print(json.dumps({"pmc_child": 1, "samples": samples}), flush=True)


def roofline_from_pmc(pmc, samples_per_s):
    """Chip-wide HBM rate of the whole call from the counter passes."""
    f = pmc["passes"]["fetch"]
    w = pmc["passes"]["write"]
    sq = pmc["passes"]["sq"]["counters"]
    fetch_kb, write_kb = f["counters"].get("FETCH_SIZE", 0.0), w["counters"].get("WRITE_SIZE", 0.0)
    raw = (1024.0 * fetch_kb + 1024.0 * write_kb) / f["samples"]
    corr = (2 * 1024.0 * fetch_kb + 1024.0 * write_kb) / f["samples"]
    achieved = corr * samples_per_s / 1e9
    trace = {k: v for k, v in f["kernel_trace"].items()}
    # dominant = the kernel that moves the most bytes (wf_long's slices poll for
    # published paths, so their summed duration says nothing about work)
    dom = max(f["per_kernel"].items(), key=lambda kv: kv[1].get("FETCH_SIZE", 0.0))[0] if f["per_kernel"] else None
    lat = {}
    # latency evidence of the dominant kernel alone (wf_long's slices spend most
    # of their wave-cycles polling, so whole-call SQ ratios mix in idle waves)
    sqk = pmc["passes"]["sq"]["per_kernel"].get(dom, sq) if dom else sq
    lat["scope"] = dom if dom and dom in pmc["passes"]["sq"]["per_kernel"] else "whole call"
    if sqk.get("SQ_WAVE_CYCLES"):
        lat["wait_frac"] = round(sqk["SQ_WAIT_ANY"] / sqk["SQ_WAVE_CYCLES"], 3)
        lat["issue_frac"] = round(sqk["SQ_ACTIVE_INST_ANY"] / sqk["SQ_WAVE_CYCLES"], 3)
    if sqk.get("SQ_ACTIVE_INST_VALU"):
        lat["valu_lane_util"] = round(sqk["SQ_THREAD_CYCLES_VALU"] / (64.0 * sqk["SQ_ACTIVE_INST_VALU"]), 3)
    if sq.get("SQ_WAVE_CYCLES"):
        lat["call_wait_frac"] = round(sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"], 3)
    if dom and dom in trace and trace[dom].get("vgpr"):
        v = trace[dom]["vgpr"]
        alloc = -(-v // 8) * 8
        lat["dominant_vgpr"] = v
        lat["dominant_waves_per_simd_vgpr_limit"] = min(8, 512 // max(alloc, 1))
    pk = {}
    for k, c in f["per_kernel"].items():
        pk[k] = {"fetch_GB": round(2 * 1024.0 * c.get("FETCH_SIZE", 0.0) / 1e9, 3)}
    for k, c in w["per_kernel"].items():
        pk.setdefault(k, {})["write_GB"] = round(1024.0 * c.get("WRITE_SIZE", 0.0) / 1e9, 3)
    for k, t in trace.items():
        pk.setdefault(k, {})["profiled_ms"] = round(t["ns"] / 1e6, 2)
        pk[k]["dispatches"] = t["dispatches"]
    return achieved, {
        "hbm_bytes_per_sample": round(corr, 1),
        "hbm_bytes_per_sample_raw": round(raw, 1),
        "achieved_raw_GBps": round(raw * samples_per_s / 1e9, 1),
        "correction": "FETCH_SIZE (KiB) x2: gfx950 tallies 128-B requests at 64 B (MI355X_MICROARCH.md HBM section; "
                      "calibrated for this kernel's gather widths in profiles/r02/fetch_calibration.json); "
                      "WRITE_SIZE x1; Infinity-Cache hits are counted as fetches, so both are upper bounds on HBM",
        "dominant_kernel": dom,
        "latency": lat,
        "per_kernel": pk,
        "counter_passes": {k: {"wall_s": v["wall_s"], "dispatches": v["dispatches"]} for k, v in pmc["passes"].items()},
    }


# ------------------------------------------------------------------ helpers
def ensure_scene(args, rt):
    scene_dir = os.path.join(args.scene_dir, args.scene)
    scene_file = os.path.join(scene_dir, "scene.txt")
    if not os.path.exists(scene_file):
        os.makedirs(scene_dir, exist_ok=True)
        rt.generate_scene(args.scene, scene_dir)
    return scene_file


def cpu_info():
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return model, os.cpu_count() or 1, usable


def cpu_baseline(scene_path, W, H, cap_seconds, passes=1):
    """The C oracle (OpenMP) on BASELINE.md's CPU budget: the full frame x
    `passes` spp (1 for configs 2-5; the whole job for the Cornell config).
    Threads: the CPU share this job was given (OMP_NUM_THREADS on the GPU box,
    which sets it to the box's share), else every usable core.  If a probe
    predicts more than cap_seconds, a bounded pixel sample is timed instead
    (and the line says so)."""
    import oracle

    model, nproc, usable = cpu_info()
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(usable, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else usable
    sc = oracle.OracleScene(scene_path)
    n = W * H

    def run(pixels, p):
        fb = np.zeros(n * 3, np.float32)
        sq = np.zeros(n, np.float32)
        cnt = np.zeros(n, np.int32)
        rng = oracle.mt19937(n)
        t = time.perf_counter()
        sc.render(sc.camera, fb, sq, cnt, rng, W, H, p, sample_count_arg=0, pixels=pixels, adaptive=False,
                  threads=threads)
        return time.perf_counter() - t

    probe = np.arange(0, n, max(1, n // 4096), dtype=np.int32)
    dt = run(probe, 1)
    predicted = dt * n * passes / len(probe)
    if predicted <= cap_seconds:
        dt = run(None, passes)
        count, what = n * passes, f"the full {W}x{H} frame x {passes} spp"
    else:
        count = int(max(len(probe), len(probe) * cap_seconds / max(dt, 1e-6)))
        count = min(n, count)
        pixels = np.linspace(0, n - 1, count).astype(np.int32)
        dt = run(pixels, 1)
        what = (f"{count} pixels spread over the {W}x{H} frame x 1 spp (the full-frame budget was predicted at "
                f"{predicted:.0f} s > --cpu-seconds {cap_seconds:.0f})")
    value = count / dt / 1e6
    return {"value": round(value, 6), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "per_core": round(value / threads, 6), "cpu_model": model, "nproc": nproc, "usable_cpus": usable,
            "sample": f"{what} ({dt:.1f} s, OpenMP {threads} threads = the job's CPU share, oracle/rt_oracle.c)",
            "reference_single_core": REF_SINGLE_CORE}


# ------------------------------------------------------------------ main
def main(argv=None, binding=None):
    """`binding`: the ctypes binding module (default: isaklm-raytracer_amd/rt.py,
    the HIP library).  Tests pass a CPU stand-in to exercise the multi-rank
    accounting without a GPU (tests/test_bench_ranks.py)."""
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.pmc_child:
        import rt

        return pmc_child(args, rt)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", 1))
    rank = int(os.environ.get("RANK", 0))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2

    dist = None
    if world > 1:
        import datetime

        import torch.distributed as dist

        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=900))
    parallelism = f"spp-sliced x{world} + RCCL reduce" if world > 1 else "single GPU"
    if args.dry_run:
        return dry_run(args, dist, world, rank, local, parallelism)

    # counter passes first: the children must own the GPU alone, and this
    # process must not have initialised it yet
    pmc = None
    if rank == 0 and world == 1 and not args.no_pmc and binding is None:
        import rt as rt_host_only

        ensure_scene(args, rt_host_only)  # host-only scene generation, once, outside the profiled children
        pmc = measure_pmc(args, args.pmc_save)

    if binding is None:
        import rt
    else:
        rt = binding

    ndev = ctypes.c_int(0)
    rt.check(rt.lib().rt_device_count(ctypes.byref(ndev)))
    if local >= ndev.value:
        print(f"bench.py: rank {rank} needs device {local}, {ndev.value} visible", file=sys.stderr)
        return 2
    rt.check(rt.lib().rt_set_device(local))
    comm = None
    if world > 1:
        uid = [rt.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = rt.Comm(world, rank, uid[0])

    if local == 0:
        ensure_scene(args, rt)
    if dist:
        dist.barrier()
    scene_file = ensure_scene(args, rt)
    t = time.perf_counter()
    host = rt.HostScene(scene_file)
    dscene = rt.DeviceScene(host)
    setup_s = time.perf_counter() - t
    info = dscene.info()

    W, H, P = args.width, args.height, args.passes
    n = W * H
    gb = rt.GBuffer(W, H, rank * n)  # spp slice r: mt19937 outputs [r*W*H, (r+1)*W*H) (shard.seed_skip)
    kernel = rt.KERNEL_WAVEFRONT if args.kernel == "wavefront" else rt.KERNEL_MEGA
    wavefront = kernel == rt.KERNEL_WAVEFRONT
    render_kw = dict(adaptive=args.adaptive, min_samples=args.min_samples, max_depth=args.max_depth, kernel=kernel,
                     traversal=traversal_of(args, rt), check_interval=args.check_interval,
                     debug=args.debug)
    bounded = wavefront and args.traversal == "bounded"
    spc = max(1, args.steps_per_call)
    profiles = []
    # chained calls only where the timed region has several calls to chain (a lone call is
    # faster unchained: its finisher takes returned pixels back at once instead of a drain)
    chain = bool(args.overlap) and len(call_plan(args.warmup, args.steps, spc)) > 1

    def steps(first, count):
        """render steps [first, first + count) in calls of up to spc steps (profiled: their kernel
        times are read back after the timed region, rt_profile_history, so that no call waits)"""
        for start, k in call_plan(first, count, spc):
            rt.render(dscene, gb, host.camera, 0 if start == 0 else 1,
                      rt.options(W, H, P * k, profile=wavefront, overlap=chain, **render_kw))

    steps(0, args.warmup)
    rt.check(rt.lib().rt_synchronize())
    cnt_before = int(gb.download()[2].sum(dtype=np.int64))  # accumulated samples (adaptive: actual)
    if dist:
        import torch

        cb = torch.tensor([cnt_before], dtype=torch.int64)
        dist.all_reduce(cb)  # every rank's warm-up samples: rank 0 holds them all after the reduce
        cnt_before = int(cb.item())
    rgba = ctypes.c_void_p()
    rt.check(rt.lib().rt_device_alloc(ctypes.byref(rgba), n * 4))
    rt.check(rt.lib().rt_synchronize())
    rt.deviation_stats(reset=True)  # always-on deviation statistics: the timed region only
    if wavefront:
        rt.profile_history(reset=True)  # (the warm-up calls' profiles dropped)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    steps(args.warmup, args.steps)
    if comm:  # ONE RCCL reduce over xGMI of fb/sq/count into rank 0 (rt_reduce_shards)
        comm.reduce(gb.g, W, H, root=0, stream=None)
    if rank == 0:
        rt.check(rt.lib().rt_tonemap(gb.g, rgba, W, H, None))
    rt.check(rt.lib().rt_synchronize())
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        import torch

        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    if wavefront:
        plan = call_plan(args.warmup, args.steps, spc)
        hist = rt.profile_history(reset=True)
        profiles = [dict(h, passes=P * k) for h, (_, k) in zip(hist, plan)]
    dev = rt.deviation_stats(reset=False)
    if dist:  # every rank's statistics (sums; max of the longest path)
        import torch

        hk = list(getattr(rt, "HANDOFF_FIELDS", ()))
        dv = torch.tensor([dev["watchdog_paths"], dev["cut_paths"], dev["deep_paths"], dev["bounded_checked"],
                           dev["bounded_mismatches"]] + [dev.get(k, 0) for k in hk] + dev["deep_hist"],
                          dtype=torch.int64)
        dist.all_reduce(dv)
        mx = torch.tensor([dev["max_deep_depth"]], dtype=torch.int64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        v = [int(x) for x in dv.tolist()]
        dev = {"watchdog_paths": v[0], "cut_paths": v[1], "deep_paths": v[2], "bounded_checked": v[3],
               "bounded_mismatches": v[4], **dict(zip(hk, v[5:5 + len(hk)])), "deep_hist": v[5 + len(hk):],
               "max_deep_depth": int(mx.item()), "mismatch_ray": dev.get("mismatch_ray")}
    total_samples = world * n * P * args.steps
    value = total_samples / elapsed / 1e6
    acc = gb.download()[2]
    got = int(acc.sum(dtype=np.int64)) if rank == 0 else None
    timed_samples = (int(acc.sum(dtype=np.int64)) - cnt_before) if world == 1 else n * P * args.steps
    # rank 0 after the reduce holds every rank's counts
    actual_samples = got - cnt_before if rank == 0 else None
    expect = world * P * (args.warmup + args.steps)

    # work counters of one extra (untimed) call -> algorithmic bytes and the
    # reference deviations (watchdog, longest path, pushes past the 19-entry
    # stack): the KD traversal, whose counters are the reference's
    counters = rt.DeviceCounters()
    copt = rt.options(W, H, P, counters=counters.p, profile=wavefront, **dict(render_kw, traversal=rt.TRAVERSAL_KD))
    rt.render(dscene, gb, host.camera, 1, copt)
    c = counters.read(finisher=True)
    bytes_per_call = algorithmic_bytes(c)
    if wavefront:
        launches = sum(p["trace_launches"] for p in profiles)
        avg_launch_ms = sum(p["trace_ms"] for p in profiles) / max(launches, 1)
        if bounded:
            # the dominant kernel (the bounded finisher runs the whole call: one
            # launch per call) and its own work: one more call of the timed
            # calls' shape (passes x steps-per-call, the whole-call finisher) with
            # that finisher counting its own work (RT_TRAVERSAL_BOUNDED_COUNTED:
            # its COUNT instantiation, one launch)
            bcnt = rt.DeviceCounters()
            cp = P * call_steps(args)
            rt.render(dscene, gb, host.camera, 1, rt.options(W, H, cp, counters=bcnt.p, profile=True,
                                                             **dict(render_kw, traversal=rt.TRAVERSAL_BOUNDED_COUNTED)))
            bc = bcnt.read(finisher=True)
            cprof = rt.last_profile()
            kname = "wf_finish_bvh<false>"
            launches = sum(p["finish_launches"] for p in profiles)
            # per call: the finishers' busy time (the union of their device spans: chained calls'
            # finishers overlap, and a finisher goes on with the next issued call's pixels) over the
            # timed calls — the time one launch's worth of work (a call's W x H x passes samples) took
            busy, hi = 0.0, None
            for a, b in sorted((p["start_ms"], p["start_ms"] + p["finish_ms"]) for p in profiles):
                if hi is None or a > hi:
                    busy += b - a
                    hi = b
                elif b > hi:
                    busy += b - hi
                    hi = b
            avg_launch_ms = busy / max(launches, 1)
            # per launch: the counted bytes per sample x the samples one timed call ran (the timed
            # region's accumulated samples / its launches: adaptive sampling skips some)
            samples_per_launch = timed_samples / max(launches, 1)
            trace_bytes = bounded_kernel_bytes(bc) / max(bc["sample"], 1) * samples_per_launch
            counted_launches = 1
            work = {"rays": bc["ray"], "bvh_nodes_per_ray": round(bc["b_bvh_node"] / max(bc["ray"], 1), 2),
                    "bvh_tests_per_ray": round(bc["b_bvh_tri"] / max(bc["ray"], 1), 2),
                    "kd_nodes_per_ray": round(bc["node"] / max(bc["ray"], 1), 2),
                    "kd_tests_per_ray": round(bc["tri"] / max(bc["ray"], 1), 2),
                    "bary_per_ray": round(bc["b_bary"] / max(bc["ray"], 1), 2),
                    "rays_per_sample": round(bc["ray"] / max(bc["sample"], 1), 3),
                    "bytes_per_sample": round(bounded_kernel_bytes(bc) / max(bc["sample"], 1), 1),
                    "counted_call_passes": cp,
                    "counted_call_launches": cprof["finish_launches"],
                    "samples_per_timed_launch": round(samples_per_launch),
                    "scope": "the finisher's paths; the deep paths handed to wf_long (depth > 64) are not counted"}
        else:
            cprof = rt.last_profile()
            trace_bytes = 8 * (c["node"] - c["finish_node"]) + 40 * (c["tri"] - c["finish_tri"])
            kname = "wf_trace_coop<false>"
            counted_launches = cprof["trace_launches"]
            work = {}
        bytes_per_launch = trace_bytes / max(counted_launches, 1)
        kernel_detail = {
            "kernel": kname,
            "pipelines": cprof["pipelines"],
            "launches_per_call": launches / max(len(profiles), 1),
            "avg_launch_ms": round(avg_launch_ms, 4),
            "algorithmic_bytes_per_launch": round(bytes_per_launch),
            "algorithmic_GBps_per_launch": (round(bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9, 1)
                                            if avg_launch_ms > 0 else None),
            "trace_union_ms_per_call": round(float(np.mean([p["trace_union_ms"] for p in profiles])), 3),
            "trace_ms_per_call": round(float(np.mean([p["trace_ms"] for p in profiles])), 3),
            "shade_ms_per_call": round(float(np.mean([p["shade_ms"] for p in profiles])), 3),
            "finish_ms_per_call": round(float(np.mean([p["finish_ms"] for p in profiles])), 3),
            "finisher_spans_ms": [[round(p["start_ms"], 1), round(p["start_ms"] + p["finish_ms"], 1)] for p in profiles]
            if bounded else None,
            "call_ms": round(float(np.mean([p["call_ms"] for p in profiles])), 3),
            "iterations_per_call": round(float(np.mean([p["iterations"] for p in profiles])), 1),
            "passes_per_call": round(float(np.mean([p["passes"] for p in profiles])), 1),
        }
        if work:
            kernel_detail["kernel_work"] = work
    else:
        kernel_detail = {"kernel": "rt_path_kernel<false,20>"}

    if comm:
        comm.close()
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return 0
    samples_per_s = total_samples / elapsed
    algorithmic_GBps = bytes_per_call / c["sample"] * samples_per_s / 1e9 if c["sample"] else None
    roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": None, "traffic": None}
    if pmc and "error" not in pmc:
        achieved, detail = roofline_from_pmc(pmc, samples_per_s)
        roof.update(achieved=round(achieved, 1), frac=round(achieved / HBM_PEAK_GBPS, 4),
                    traffic=round(detail["hbm_bytes_per_sample"] * n * P), **detail)
        roof["traffic_unit"] = (f"HBM bytes per step of {P} passes (whole frame, every kernel), from one profiled "
                                f"call of {P * call_steps(args)} passes = the timed calls' shape")
        roof["pmc_call_shape"] = ("one UNCHAINED call of the timed calls' passes: counter collection serialises "
                                  "dispatches, so the chained calls' overlap (a call's deep-path tail beside the "
                                  "next call's finisher) cannot run under it; the finisher kernel and its per-sample "
                                  "work are the same, the bytes per sample are applied to the chained timed rate")
        dk = detail["per_kernel"].get(detail["dominant_kernel"] or "", {})
        if wavefront and dk.get("dispatches") and kernel_detail["kernel"].split("<")[0] in (detail["dominant_kernel"] or ""):
            # the dominant kernel alone: its counter bytes per launch / its live
            # average launch time (HIP events on its pipeline's stream, timed steps)
            per_launch = 1e9 * (dk.get("fetch_GB", 0.0) + dk.get("write_GB", 0.0)) / dk["dispatches"]
            kernel_detail["hbm_bytes_per_launch"] = round(per_launch)
            kernel_detail["hbm_GBps_per_launch"] = round(per_launch / (kernel_detail["avg_launch_ms"] * 1e-3) / 1e9, 1)
            kernel_detail["hbm_frac_per_launch"] = round(kernel_detail["hbm_GBps_per_launch"] / HBM_PEAK_GBPS, 4)
    elif pmc:
        roof["pmc_error"] = pmc["error"]
        if "settle_s" in pmc:
            roof["pmc_settle_s"] = pmc["settle_s"]
    roof.update({
        "definition": "achieved = counter-measured HBM bytes per sample (FETCH_SIZE x2 + WRITE_SIZE over every "
                      "dispatch of one profiled call) x timed samples/s; chip-wide, call-level",
        "algorithmic_GBps": round(algorithmic_GBps, 1) if algorithmic_GBps else None,
        "algorithmic_bytes_per_sample": round(bytes_per_call / max(c["sample"], 1), 1),
        "algorithmic_note": "SURVEY §8d bytes the reference's algorithm (the KD traversal) touches; the product's "
                            "BVH-bounded traversal skips the KD leaves that cannot hold the hit (DESIGN.md §5), so "
                            "this rate is EXPECTED to exceed the HBM peak: it measures work avoided, not bandwidth",
        **kernel_detail,
    })
    work = kernel_detail.get("kernel_work") or {}
    if work.get("bytes_per_sample"):
        # the product's own algorithmic bytes (counted by the kernels in a BOUNDED_COUNTED call of the timed
        # calls' shape) beside the reference algorithm's: the work ratio, and the product bytes' HBM rate / peak
        pb = work["bytes_per_sample"]
        roof["product_bytes_per_sample"] = pb
        roof["work_ratio"] = round(roof["algorithmic_bytes_per_sample"] / pb, 2)
        roof["product_GBps"] = round(pb * samples_per_s / 1e9, 1)
        roof["product_frac"] = round(pb * samples_per_s / 1e9 / HBM_PEAK_GBPS, 4)
        roof["product_note"] = ("product_bytes_per_sample: per ray 112 B per 4-wide BVH node, 16 B per plane test, 56 B per "
                                "barycentric record, 8 B per KD node; per hit 176 B of shading records; per sample "
                                "40 B of pixel state (bench.py bounded_kernel_bytes); frac = the counter-measured "
                                "HBM traffic / peak, product_frac = these bytes at the timed rate / peak")
    line = {
        # BASELINE.json's metric names 1920x1080; another frame size says so
        "metric": METRIC if (W, H) == (1920, 1080) else METRIC.replace("1920×1080", f"{W}×{H}"),
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": (f"BASELINE configs[2]: README-like 2M-triangle synthetic room '{args.scene}', {W}x{H}, "
                         f"{P} spp per step per GPU, adaptive off"
                         if not args.adaptive and args.max_depth == 0 and args.scene == "room2m" else
                         f"scene '{args.scene}', {W}x{H}, {P} spp per step per GPU, adaptive "
                         f"{'on (min ' + str(args.min_samples) + ')' if args.adaptive else 'off'}, "
                         f"max depth {args.max_depth or 'unbounded'}"),
            "adaptive": args.adaptive, "max_depth": args.max_depth,
            "scene": args.scene, "width": W, "height": H, "spp_per_step": P, "steps_per_call": spc, "chained_calls": chain,
            "triangles": info["triangles"], "kd_nodes": info["nodes"], "kd_indices": info["indices"],
            "parallelism": parallelism,
        },
        "roofline": roof,
        "per_sample": {k: round(c[k] / max(c["sample"], 1), 3) for k in ("ray", "node", "tri", "hit", "nee")},
        "deviations": {
            "scope": f"timed region: every path of the {args.steps} timed steps on all ranks "
                     "(always-on statistics of the non-counting bench kernels, rt_deviation_stats)",
            "watchdog_paths": dev["watchdog_paths"], "cut_paths": dev["cut_paths"],
            "max_path_depth": dev["max_deep_depth"] if dev["deep_paths"] else c["maxdepth"],
            "deep_paths": dev["deep_paths"],
            "deep_path_hist": {f"{64 << k}-{(64 << (k + 1)) - 1}": h for k, h in enumerate(dev["deep_hist"]) if h},
            "watchdog_limit": 16777215,
            "deep_pushes": c["deep_push"], "deep_pushes_scope": "one extra counted call of the same options",
            "bounded_checked": dev.get("bounded_checked"), "bounded_mismatches": dev.get("bounded_mismatches"),
            "handoff": {k: dev.get(k) for k in getattr(rt, "HANDOFF_FIELDS", ())},
            "handoff_note": "the deep-path hand-off over the timed region: owed_pixels / owed_passes = pixels that "
                            "chained calls skipped while out in wf_long and the passes run for them later (the "
                            "chained-call protocol firing); long_safety_quits, stranded_pixels, check_dropped = "
                            "failure signals (0 in a working render); linger_expiries = finisher waves that stopped "
                            "waiting for pixels out in wf_long",
            "bounded_check_note": "run-time guard of the BVH-bounded traversal: a deterministic 1-in-"
                                  f"{args.check_interval or 4096} sample of the finisher's rays, re-traced by the "
                                  "plain KD traversal (trace_ray) inside the timed region and compared bit for bit",
            "note": "paths cut by the 2^24-1-bounce watchdog (SURVEY H8; the reference loops unbounded), paths cut "
                    "by max_depth, the longest path in bounces and the histogram of paths that ended at depth >= 64; "
                    "deep_pushes = traversal pushes at stack index >= 19 (past the reference's 19-entry arrays, "
                    "SURVEY H16)"},
        "samples_check": {"accumulated": got, "expected": None if args.adaptive else expect * n},
        "actual_samples": actual_samples,
        "value_actual": round(actual_samples / elapsed / 1e6, 3) if actual_samples is not None else None,
        "setup_s": round(setup_s, 2),
    }
    if world == 1 and not args.no_cpu_baseline:
        # the whole job for the Cornell config, full frame x 1 spp otherwise
        job = P * args.steps if args.scene == "cornell" else 1
        line["cpu_baseline"] = cpu_baseline(scene_file, W, H, args.cpu_seconds, passes=job)
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0


def dry_run(args, dist, world, rank, local, parallelism):
    """No GPU: the ranks meet (barrier, max of their clocks, who is who) and
    rank 0 prints the line the real run would frame."""
    t0 = time.perf_counter()
    ranks = [(rank, local, world)]
    if dist:
        dist.barrier()
        gathered = [None] * world
        dist.all_gather_object(gathered, (rank, local, world))
        ranks = gathered
    elapsed = time.perf_counter() - t0
    if dist:
        import torch

        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Msamples/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "dry_run": True, "ranks": ranks,
                          "config": {"parallelism": parallelism}, "barrier_s": round(elapsed, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
