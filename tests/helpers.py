"""Shared helpers: scene cache, GPU render through the C-ABI, oracle render."""
import os

import numpy as np

import oracle
import rt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENE_DIR = os.environ.get("RT_SCENE_DIR", os.path.join(ROOT, "build", "scenes"))


def scene_path(name):
    d = os.path.join(SCENE_DIR, name)
    p = os.path.join(d, "scene.txt")
    if not os.path.exists(p):
        os.makedirs(d, exist_ok=True)
        rt.generate_scene(name, d)
    return p


def gpu_has_device():
    import ctypes

    n = ctypes.c_int(0)
    return rt.lib().rt_device_count(ctypes.byref(n)) == 0 and n.value > 0


class GpuRun:
    """One scene on the device; renders through rt_render."""

    def __init__(self, name_or_path):
        path = name_or_path if name_or_path.endswith(".txt") else scene_path(name_or_path)
        self.path = path
        self.host = rt.HostScene(path)
        self.dev = rt.DeviceScene(self.host)
        self.camera = self.host.camera

    def render(self, W, H, passes, calls=1, adaptive=False, min_samples=100, tolerance=0.05, max_depth=0,
               seed_skip=0, count=False, kernel=0, wf_tail=0, wf_finish_waves=0, wf_wide=0, shard_id=0,
               num_shards=1, wf_pipelines=0, wf_long_depth=0):
        g = rt.GBuffer(W, H, seed_skip)
        cnt = rt.DeviceCounters() if count else None
        for c in range(calls):
            opt = rt.options(W, H, passes, adaptive, min_samples, tolerance, max_depth,
                             counters=cnt.p if cnt else None, kernel=kernel, wf_tail=wf_tail,
                             wf_finish_waves=wf_finish_waves, wf_wide=wf_wide, shard_id=shard_id,
                             num_shards=num_shards, wf_pipelines=wf_pipelines, wf_long_depth=wf_long_depth)
            rt.render(self.dev, g, self.camera, 0 if c == 0 else 1, opt)
        out = g.download()
        counters = cnt.read() if cnt else None
        return out, counters, g


def oracle_render(path, W, H, passes, calls=1, adaptive=False, min_samples=100, tolerance=0.05, max_depth=0,
                  seed_skip=0, pixels=None, scene=None, camera=None):
    sc = scene or oracle.OracleScene(path)
    n = W * H
    fb = np.zeros(n * 3, np.float32)
    sq = np.zeros(n, np.float32)
    cnt = np.zeros(n, np.int32)
    rng = oracle.mt19937(n, seed_skip)
    cam = sc.camera if camera is None else camera
    total = {}
    for c in range(calls):
        k = sc.render(cam, fb, sq, cnt, rng, W, H, passes, sample_count_arg=0 if c == 0 else 1, pixels=pixels,
                      adaptive=adaptive, min_samples=min_samples, tolerance=tolerance, max_depth=max_depth)
        for key, v in k.items():
            total[key] = max(total.get(key, 0), v) if key == "maxdepth" else total.get(key, 0) + v
    return (fb.reshape(n, 3), sq, cnt, rng), total


def assert_bitwise(gpu, ref, pixels=None, what=""):
    names = ["frame_buffer", "squared_luminance", "sample_count", "random_numbers"]
    for name, a, b in zip(names, gpu, ref):
        if pixels is not None:
            a, b = a[pixels], b[pixels]
        av = a.view(np.uint32) if a.dtype == np.float32 else a
        bv = b.view(np.uint32) if b.dtype == np.float32 else b
        bad = np.nonzero((av != bv).reshape(len(av), -1).any(axis=1))[0]
        assert len(bad) == 0, (f"{what} {name}: {len(bad)} of {len(av)} pixels differ; first {bad[:8]}: "
                               f"gpu {a[bad[:3]]} oracle {b[bad[:3]]}")


def rel_linf(gpu_fb, gpu_cnt, ref_fb, ref_cnt):
    """L-infinity of per-channel relative radiance error (fb/count), north_star's 1e-4 bar."""
    a = gpu_fb / np.maximum(gpu_cnt, 1)[:, None]
    b = ref_fb / np.maximum(ref_cnt, 1)[:, None]
    den = np.maximum(np.abs(b), 1e-30)
    return float(np.max(np.abs(a - b) / den)) if len(a) else 0.0
