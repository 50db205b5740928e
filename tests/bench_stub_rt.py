"""TEST INFRASTRUCTURE ONLY: a CPU stand-in for the ctypes binding
(isaklm-raytracer_amd/rt.py) with the surface bench.py uses, so that
bench.main's multi-rank branch — ranks meeting over gloo, the per-rank spp
slice seeds, the closing reduce into rank 0, the max-over-ranks clock and
the sample accounting — runs end to end on a machine without a GPU
(tests/test_bench_ranks.py).  Renders go through the oracle; the reduce is a
gloo reduce of the host arrays.  Rank 1 is made slower (STUB_SLOW_RANK) so
the test can see the max over ranks.
"""
import ctypes
import os
import time

import numpy as np

import oracle

KERNEL_MEGA = 0
KERNEL_WAVEFRONT = 1
TRAVERSAL_BOUNDED, TRAVERSAL_KD, TRAVERSAL_BOUNDED_COUNTED = 0, 1, 2
SLOW_RANK = int(os.environ.get("STUB_SLOW_RANK", "1"))
SLOW_S = float(os.environ.get("STUB_SLOW_S", "0.25"))
calls = []  # (rank, sample_count, passes) of every render


class RtError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        raise RtError(f"stub rc {rc}")


class _Lib:
    def rt_device_count(self, p):
        ctypes.cast(p, ctypes.POINTER(ctypes.c_int))[0] = 8
        return 0

    def rt_set_device(self, d):
        return 0

    def rt_device_alloc(self, p, n):
        return 0

    def rt_synchronize(self):
        return 0

    def rt_tonemap(self, *a):
        return 0


_LIB = _Lib()


def lib():
    return _LIB


def generate_scene(name, out_dir):
    import rt  # host-only scene generator of the real library (no GPU call)

    return rt.generate_scene(name, out_dir)


class HostScene:
    def __init__(self, path):
        self.path = path
        self.osc = oracle.OracleScene(path)
        self.camera = self.osc.camera


class DeviceScene:
    def __init__(self, host):
        self.host = host

    def info(self):
        o = self.host.osc
        return {"triangles": o.ntris, "nodes": o.nnodes, "indices": o.nindices}


class GBuffer:
    def __init__(self, W, H, seed_skip=0):
        n = W * H
        self.W, self.H = W, H
        self.fb = np.zeros(n * 3, np.float32)
        self.sq = np.zeros(n, np.float32)
        self.cnt = np.zeros(n, np.int32)
        self.rng = oracle.mt19937(n, seed_skip)
        self.g = self

    def download(self):
        return self.fb.reshape(-1, 3).copy(), self.sq.copy(), self.cnt.copy(), self.rng.copy()


class _Opt:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def options(W, H, passes=1, adaptive=True, min_samples=100, max_depth=0, kernel=KERNEL_MEGA, counters=None,
            profile=False, **_):
    return _Opt(W=W, H=H, passes=passes, adaptive=adaptive, min_samples=min_samples, max_depth=max_depth,
                counters=counters)


_last = {}


def render(dscene, gb, camera, sample_count, opt):
    rank = int(os.environ.get("RANK", 0))
    t = time.perf_counter()
    k = dscene.host.osc.render(camera, gb.fb, gb.sq, gb.cnt, gb.rng, opt.W, opt.H, opt.passes,
                               sample_count_arg=sample_count, adaptive=opt.adaptive, min_samples=opt.min_samples,
                               max_depth=opt.max_depth)
    if rank == SLOW_RANK:
        time.sleep(SLOW_S)
    if opt.counters is not None:
        opt.counters.add(k)
    calls.append((rank, sample_count, opt.passes))
    ms = (time.perf_counter() - t) * 1e3
    _last.update(iterations=1, trace_launches=1, shade_launches=1, finish_launches=0, start_ms=0.0, trace_ms=ms,
                 shade_ms=0.0, finish_ms=0.0, call_ms=ms, trace_union_ms=ms, pipelines=1)
    _hist.append(dict(_last))


_hist = []


def last_profile():
    return dict(_last)


def profile_history(reset=False):
    out = [dict(h) for h in _hist]
    if reset:
        _hist.clear()
    return out


class DeviceCounters:
    def __init__(self):
        self.c = {}
        self.p = self

    def add(self, k):
        for key, v in k.items():
            if isinstance(v, (int, np.integer)):
                self.c[key] = max(self.c.get(key, 0), v) if key == "maxdepth" else self.c.get(key, 0) + v

    def read(self, finisher=False):
        out = {k: self.c.get(k, 0) for k in oracle.COUNTER_NAMES}
        out["deep_push"] = self.c.get("deep_push", 0)
        if finisher:
            out.update(finish_node=0, finish_tri=0, finish_ray=0, b_bvh_node=0, b_bvh_tri=0, b_bary=0)
        return out


def deviation_stats(reset=False):
    return {"watchdog_paths": 0, "cut_paths": 0, "max_deep_depth": 0, "deep_paths": 0, "deep_hist": [0] * 18,
            "bounded_checked": 0, "bounded_mismatches": 0, "mismatch_ray": [0.0] * 6}


class Comm:
    @staticmethod
    def unique_id():
        return b"stub" * 32

    def __init__(self, nranks, rank, uid):
        assert len(uid) == 128
        self.nranks, self.rank = nranks, rank

    def reduce(self, gb, W, H, root=0, stream=None):
        """rt_reduce_shards: sum fb / sq / count of every rank into root"""
        import torch
        import torch.distributed as dist

        for a in (gb.fb, gb.sq, gb.cnt):
            t = torch.from_numpy(a)
            dist.reduce(t, dst=root)
            if self.rank == root:
                a[...] = t.numpy()

    def close(self):
        pass
