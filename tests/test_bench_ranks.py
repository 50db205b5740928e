"""bench.py's N > 1 branch end to end on CPU (no GPU): two ranks over gloo
with a CPU stand-in binding (tests/bench_stub_rt.py: oracle renders, a gloo
reduce for rt_reduce_shards).  Checks the rank-0 JSON line's accounting —
n_gpus, samples of all ranks, accumulated vs expected counts after the
reduce, value = all ranks' samples / the max-over-ranks wall time — and
that each rank rendered its own spp slice (rt/main.cu:114-155 sharded)."""
import json
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_accounting(tmp_path):
    import helpers

    helpers.scene_path("cornell")  # generated once, before the ranks start
    W, H, P, STEPS, WARM = 24, 16, 2, 3, 1
    argv = ["--gpus", "2", "--steps", str(STEPS), "--warmup", str(WARM), "--passes", str(P), "--steps-per-call", "2",
            "--scene", "cornell", "--width", str(W), "--height", str(H), "--no-pmc", "--scene-dir", helpers.SCENE_DIR]
    port = str(_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, STUB_SLOW_RANK="1", STUB_SLOW_S="0.4",
                   OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "bench_rank_child.py")] + argv, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, o + e
    lines = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and not [ln for ln in outs[1][0].splitlines() if ln.startswith("{")]
    line = json.loads(lines[0])
    n = W * H
    assert line["n_gpus"] == 2 and line["steps"] == STEPS and line["warmup"] == WARM
    assert "spp-sliced x2" in line["config"]["parallelism"]
    # rank 0 holds every rank's counts after the reduce
    assert line["samples_check"]["accumulated"] == line["samples_check"]["expected"] == 2 * n * P * (WARM + STEPS)
    assert line["actual_samples"] == 2 * n * P * STEPS
    # value = samples of ALL ranks / the max-over-ranks wall time (rank 1 sleeps 0.4 s per call: 2 timed calls)
    elapsed = line["ms_per_step"] * STEPS / 1e3
    assert elapsed >= 0.8
    assert abs(line["value"] - 2 * n * P * STEPS / elapsed / 1e6) <= 1e-3 * line["value"] + 1e-3
    assert line["cpu_baseline"] is None  # rank 0 at N = 1 only
    assert line["deviations"]["watchdog_paths"] == 0
