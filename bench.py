"""Bench: Msamples/s of the render hot path at 1920x1080 (BASELINE.json metric).

Workload (BASELINE.json configs[2]): the README-like 2M-triangle synthetic
room ("room2m": room + 1,997,568-triangle displaced gold mesh + two glass
spheres + emissive quad), 1920x1080, adaptive sampling off.  One step = one
rt_render call of `--passes` passes (spp) over the full frame (default 64:
16 steps are the config's 1024 spp).  With --gpus N
each rank renders its own spp slice (seeds = mt19937 outputs [rank*W*H,
(rank+1)*W*H)) and one RCCL reduce (sum) of fb/sq/count into
rank 0 plus the tonemap closes the timed region.  value = samples of all ranks
/ max-over-ranks wall time.

Also reported: the roofline of the dominant kernel (wavefront: wf_trace_coop,
whose SURVEY §8d traversal bytes 8*node + 40*tri come from the work counters
of one counted call, over its launches' HIP-event time inside the timed
steps, against 8 TB/s HBM) and the CPU oracle's rate on a bounded pixel
sample (rank 0, N=1).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import rt  # noqa: E402
import shard  # noqa: E402

METRIC = "Msamples/sec (W×H×spp/s) at 1920×1080; achieved HBM GB/s vs peak"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def algorithmic_bytes(c):
    """bytes the reference's algorithm reads/writes, layout-independent."""
    return (8 * c["node"] + 40 * c["tri"] + 116 * c["hit"] + 4 * c["texel"] + 40 * c["nee"] + 48 * c["sample"] +
            20 * c["skip"])


class TorchGBuffer:
    """G_Buffer whose four arrays are torch tensors (so RCCL can reduce them)."""

    def __init__(self, torch, n, seed_skip):
        self.fb = torch.zeros(n * 3, dtype=torch.float32, device="cuda")
        self.sq = torch.zeros(n, dtype=torch.float32, device="cuda")
        self.cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
        self.rng = torch.from_numpy(rt.seeds(n, seed_skip).view(np.int32)).cuda()
        self.g = rt.G_Buffer(self.fb.data_ptr(), self.sq.data_ptr(), self.cnt.data_ptr(), self.rng.data_ptr())


def pmc_traffic(kernel_name):
    """HBM bytes per launch of `kernel_name` from the newest committed rocprofv3
    PMC summary (profiles/r*/pmc_traffic_*.json: FETCH_SIZE / WRITE_SIZE passes
    of this bench command, corrected as MI355X_MICROARCH.md prescribes)."""
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic_*.json")), reverse=True):
        d = json.load(open(f))
        if d.get("kernel") == kernel_name:
            return d["traffic_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(scene_path, W, H, seconds, threads):
    import oracle

    sc = oracle.OracleScene(scene_path)
    n = W * H

    def run(pixels):
        fb = np.zeros(n * 3, np.float32)
        sq = np.zeros(n, np.float32)
        cnt = np.zeros(n, np.int32)
        rng = oracle.mt19937(n)
        t = time.perf_counter()
        sc.render(sc.camera, fb, sq, cnt, rng, W, H, 1, sample_count_arg=0, pixels=pixels, adaptive=False,
                  threads=threads)
        return time.perf_counter() - t

    probe = np.arange(0, n, max(1, n // 2048), dtype=np.int32)
    dt = run(probe)
    rate = len(probe) / max(dt, 1e-6)
    count = int(min(n, max(len(probe), rate * seconds)))
    pixels = np.linspace(0, n - 1, count).astype(np.int32)
    dt = run(pixels)
    return {"value": round(count / dt / 1e6, 6), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{count} pixels spread over the {W}x{H} frame x 1 spp ({dt:.1f} s, OpenMP {threads} threads, "
                      f"oracle/rt_oracle.c)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--passes", type=int, default=64, help="spp per step (passes per rt_render call)")
    ap.add_argument("--scene", default="room2m")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel", choices=["mega", "wavefront"], default="wavefront")
    ap.add_argument("--adaptive", action="store_true", help="adaptive sampling (configs[4]); value stays nominal "
                    "W*H*spp/s, value_actual = accumulated samples/s")
    ap.add_argument("--min-samples", type=int, default=100)
    ap.add_argument("--max-depth", type=int, default=0, help="0 = unbounded (reference)")
    ap.add_argument("--shard-mode", choices=["spp", "rows"], default="spp",
                    help="N>1: spp slices (north star, seeds skipped per rank) or row-interleaved shards "
                         "(bit-identical to one GPU)")
    ap.add_argument("--scene-dir", default=os.environ.get("RT_SCENE_DIR", os.path.join(ROOT, "build", "scenes")))
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch

    torch.cuda.set_device(local)
    rt.check(rt.lib().rt_set_device(local))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl")

    scene_dir = os.path.join(args.scene_dir, args.scene)
    scene_file = os.path.join(scene_dir, "scene.txt")
    if local == 0 and not os.path.exists(scene_file):
        rt.generate_scene(args.scene, scene_dir)
    if dist:
        dist.barrier()
    t = time.perf_counter()
    host = rt.HostScene(scene_file)
    dscene = rt.DeviceScene(host)
    setup_s = time.perf_counter() - t
    info = dscene.info()

    W, H, P = args.width, args.height, args.passes
    n = W * H
    rows = args.shard_mode == "rows" and world > 1
    gb = TorchGBuffer(torch, n, 0 if rows else shard.seed_skip(rank, W, H))
    stream = torch.cuda.current_stream()
    kernel = rt.KERNEL_WAVEFRONT if args.kernel == "wavefront" else rt.KERNEL_MEGA
    wavefront = kernel == rt.KERNEL_WAVEFRONT
    shard_kw = dict(shard_id=rank, num_shards=world) if rows else {}
    render_kw = dict(adaptive=args.adaptive, min_samples=args.min_samples, max_depth=args.max_depth, kernel=kernel,
                     **shard_kw)
    opt = rt.options(W, H, P, stream=ctypes.c_void_p(stream.cuda_stream), profile=wavefront, **render_kw)
    profiles = []

    def step(i):
        rt.render(dscene, gb, host.camera, 0 if i == 0 else 1, opt)
        if wavefront:
            profiles.append(rt.last_profile())

    for i in range(args.warmup):
        step(i)
    profiles.clear()
    torch.cuda.synchronize()
    cnt_before = gb.cnt.sum(dtype=torch.int64)  # accumulated samples before the timed steps (adaptive: actual)
    if dist:
        dist.all_reduce(cnt_before)
        dist.barrier()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    rgba = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        starts[k].record(stream)
        step(args.warmup + k)
        ends[k].record(stream)
    if dist:  # one RCCL reduce over xGMI into rank 0's accumulation buffers
        shard.reduce_to_root(dist, gb.fb, gb.sq, gb.cnt, root=0)
    if rank == 0:
        rt.check(rt.lib().rt_tonemap(gb.g, ctypes.c_void_p(rgba.data_ptr()), W, H,
                                     ctypes.c_void_p(stream.cuda_stream)))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    kernel_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))
    total_samples = (1 if rows else world) * n * P * args.steps
    value = total_samples / elapsed / 1e6
    actual_samples = int((gb.cnt.sum(dtype=torch.int64) - cnt_before).item()) if rank == 0 else None

    # samples actually accumulated (every pixel, every pass: adaptive off)
    expect = (1 if rows else world) * P * (args.warmup + args.steps)
    got = int(gb.cnt.sum().item()) if rank == 0 else None

    # work counters on one extra (untimed) step -> algorithmic bytes per call
    counters = rt.DeviceCounters()
    copt = rt.options(W, H, P, counters=counters.p, profile=wavefront, **render_kw)
    rt.render(dscene, gb, host.camera, 1, copt)
    c = counters.read(finisher=True)
    bytes_per_call = algorithmic_bytes(c)
    if wavefront:
        # dominant kernel: wf_trace_coop.  achieved = its SURVEY §8d traversal
        # bytes per launch (the finisher's share taken out, from the counted
        # call) / its average launch duration (HIP events around every launch
        # in the timed steps; rocprof's average must agree).  The concurrent
        # pipelines' launches overlap, so the aggregate rate while any trace
        # launch runs (bytes per call / union of the launch intervals) is
        # reported beside it.
        cprof = rt.last_profile()
        trace_bytes = 8 * (c["node"] - c["finish_node"]) + 40 * (c["tri"] - c["finish_tri"])
        launches = sum(p["trace_launches"] for p in profiles)
        trace_ms_call = float(np.mean([p["trace_ms"] for p in profiles]))
        union_ms_call = float(np.mean([p["trace_union_ms"] for p in profiles]))
        avg_launch_ms = sum(p["trace_ms"] for p in profiles) / max(launches, 1)
        bytes_per_launch = trace_bytes / max(cprof["trace_launches"], 1)
        achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
        roof_kernel = "wf_trace_coop<false>"
        kernel_detail = {
            "pipelines": cprof["pipelines"],
            "trace_launches_per_call": launches / len(profiles),
            "avg_launch_ms": round(avg_launch_ms, 4),
            "trace_union_ms_per_call": round(union_ms_call, 3),
            "aggregate_GBps": round(trace_bytes / (union_ms_call * 1e-3) / 1e9, 1),
            "aggregate_definition": "trace algorithmic bytes per call / wall ms with >= 1 trace launch running "
                                    "(can exceed HBM peak: the caches absorb the reference's re-reads)",
            "trace_ms_per_call": round(trace_ms_call, 3),
            "shade_ms_per_call": round(float(np.mean([p["shade_ms"] for p in profiles])), 3),
            "finish_ms_per_call": round(float(np.mean([p["finish_ms"] for p in profiles])), 3),
            "call_ms": round(float(np.mean([p["call_ms"] for p in profiles])), 3),
            "trace_bytes_per_call": trace_bytes,
            "trace_bytes_per_launch": round(bytes_per_launch),
            "finisher_ray_share": round(c["finish_ray"] / max(c["ray"], 1), 4),
            "call_achieved_GBps": round(bytes_per_call / (kernel_ms * 1e-3) / 1e9, 1),
        }
    else:
        achieved = bytes_per_call / (kernel_ms * 1e-3) / 1e9
        roof_kernel = "rt_path_kernel<false,20>"
        kernel_detail = {"kernel_ms": round(kernel_ms, 3)}

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    traffic, traffic_src = pmc_traffic(roof_kernel)
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if rows else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": (f"BASELINE configs[2]: README-like 2M-triangle synthetic room '{args.scene}', {W}x{H}, "
                         f"{P} spp per step, adaptive off"
                         if not args.adaptive and args.max_depth == 0 and args.scene == "room2m" else
                         f"scene '{args.scene}', {W}x{H}, {P} spp per step, adaptive "
                         f"{'on (min ' + str(args.min_samples) + ')' if args.adaptive else 'off'}, "
                         f"max depth {args.max_depth or 'unbounded'}"),
            "adaptive": args.adaptive, "max_depth": args.max_depth,
            "scene": args.scene, "width": W, "height": H, "spp_per_step": P,
            "triangles": info["triangles"], "kd_nodes": info["nodes"], "kd_indices": info["indices"],
            "parallelism": (f"{'row-interleaved' if rows else 'spp-sliced'} x{world} + RCCL reduce" if world > 1
                            else "single GPU"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": roof_kernel,
            **kernel_detail,
            "call_algorithmic_bytes": bytes_per_call,
            "bytes_per_sample": round(bytes_per_call / max(c["sample"], 1), 1),
        },
        "per_sample": {k: round(c[k] / max(c["sample"], 1), 3) for k in ("ray", "node", "tri", "hit", "nee")},
        "samples_check": {"accumulated": got, "expected": None if args.adaptive else expect * n},
        "actual_samples": actual_samples,
        "value_actual": round(actual_samples / elapsed / 1e6, 3),
        "setup_s": round(setup_s, 2),
    }
    if world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        line["cpu_baseline"] = cpu_baseline(scene_file, W, H, args.cpu_seconds, threads)
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
