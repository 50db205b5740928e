"""The N>1 path on CPU: two gloo ranks each render their spp slice (seeded
with their own mt19937 window), reduce into rank 0, and rank 0 checks the sum
against a single-process emulation of the same shards — bit for bit."""
import os
import socket

import numpy as np
import pytest

import helpers
import shard

W, H, PASSES = 16, 12, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _render_shard(path, rank):
    (fb, sq, cnt, rng), _ = helpers.oracle_render(path, W, H, PASSES, seed_skip=shard.seed_skip(rank, W, H))
    return fb, sq, cnt


def _worker(rank, world, port, path, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fb, sq, cnt = _render_shard(path, rank)
        t_fb, t_sq, t_cnt = torch.from_numpy(fb.copy()), torch.from_numpy(sq.copy()), torch.from_numpy(cnt.copy())
        shard.reduce_to_root(dist, t_fb, t_sq, t_cnt, root=0)
        if rank == 0:
            q.put((t_fb.numpy().copy(), t_sq.numpy().copy(), t_cnt.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_pass_slices_cover_the_job():
    for world in (1, 2, 3, 8):
        spans = [shard.pass_slice(r, world, 5000) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == 5000
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_two_rank_gloo_reduce_matches_emulation():
    import torch.multiprocessing as mp

    path = helpers.scene_path("cornell")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a = _render_shard(path, 0)
    b = _render_shard(path, 1)
    np.testing.assert_array_equal(got[0].view(np.uint32), (a[0] + b[0]).view(np.uint32))
    np.testing.assert_array_equal(got[1].view(np.uint32), (a[1] + b[1]).view(np.uint32))
    np.testing.assert_array_equal(got[2], a[2] + b[2])
    assert np.all(got[2] == 2 * PASSES)
    # rank 0's slice alone is the single-stream reference for its passes
    single, _ = helpers.oracle_render(path, W, H, PASSES)
    np.testing.assert_array_equal(a[0].view(np.uint32), single[0].view(np.uint32))


def _render_rows(path, rank, world):
    """Row-interleaved shard (RtOptions.shard_id/num_shards): the rank's rows with
    the single-stream seeds, adaptive on; other rows stay zero."""
    pix = np.array([i for i in range(W * H) if (i // W) % world == rank], np.int32)
    (fb, sq, cnt, rng), _ = helpers.oracle_render(path, W, H, PASSES, calls=2, adaptive=True, min_samples=2,
                                                  pixels=pix)
    return fb, sq, cnt


def _rows_worker(rank, world, port, path, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fb, sq, cnt = _render_rows(path, rank, world)
        t_fb, t_sq, t_cnt = torch.from_numpy(fb.copy()), torch.from_numpy(sq.copy()), torch.from_numpy(cnt.copy())
        shard.reduce_to_root(dist, t_fb, t_sq, t_cnt, root=0)
        if rank == 0:
            q.put((t_fb.numpy().copy(), t_sq.numpy().copy(), t_cnt.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_row_shards_equal_single_stream():
    """SURVEY §8e's parity-exact option: row shards reduced over gloo are the
    one-process frame bit for bit, adaptive sampling included."""
    import torch.multiprocessing as mp

    path = helpers.scene_path("cornell")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rows_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single, _ = helpers.oracle_render(path, W, H, PASSES, calls=2, adaptive=True, min_samples=2)
    np.testing.assert_array_equal(got[0].view(np.uint32), single[0].view(np.uint32))
    np.testing.assert_array_equal(got[1].view(np.uint32), single[1].view(np.uint32))
    np.testing.assert_array_equal(got[2], single[2])


def test_bench_launcher_starts_n_ranks():
    """`bench.py --gpus 2` (as the driver runs it, no WORLD_SIZE in the env)
    starts its two ranks itself; they meet over gloo and rank 0 frames the
    line with n_gpus 2 (--dry-run: the rank wiring only, no GPU)."""
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(helpers.ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "spp-sliced x2 + RCCL reduce"
    assert sorted(tuple(x) for x in line["ranks"]) == [(0, 0, 2), (1, 1, 2)]
