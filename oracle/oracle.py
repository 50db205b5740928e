"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU restatement
(oracle/rt_oracle.c).  Used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker; never by the product path.

Parity status: "parity unpinned" for radiance (the reference is unbuildable
here; see rt_oracle.h and DESIGN.md §Parity).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
N_COUNTERS = 40
COUNTER_NAMES = ["node", "tri", "hit", "texel", "nee", "sample", "skip", "ray", "watchdog", "maxdepth"]
DEEP_PUSH = 15  # CNT_DEEP_PUSH / RT_CNT_DEEP_PUSH
CUT = 16  # CNT_CUT: paths cut at the depth limit (watchdog or max_depth)
DEEP_HIST = 17  # CNT_DEEP_HIST: 18 bins of paths ending at depth in [64*2^k, 64*2^(k+1))
DEEP_HIST_BINS = 18
# hazard instrumentation: inputs that triggered each quirk
HAZARDS = {"xi_one": 35, "exit_tie": 36, "on_split": 37, "axis_parallel": 38, "degenerate": 39}

_lib = None


class OrOptions(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("passes", ctypes.c_int),
                ("adaptive", ctypes.c_int), ("min_samples", ctypes.c_int), ("tolerance", ctypes.c_float),
                ("max_depth", ctypes.c_int), ("threads", ctypes.c_int)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i = ctypes.c_void_p, ctypes.c_int
        L.or_last_error.restype = ctypes.c_char_p
        L.or_mt19937.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint64]
        L.or_mt19937.restype = None
        L.or_rng_next.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        L.or_rng_next.restype = ctypes.c_float
        L.or_scene_load.argtypes = [ctypes.c_char_p, vp]
        L.or_scene_load.restype = vp
        L.or_scene_from_triangles.argtypes = [vp, i]
        L.or_scene_from_triangles.restype = vp
        L.or_scene_free.argtypes = [vp]
        L.or_scene_free.restype = None
        L.or_scene_counts.argtypes = [vp, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i)]
        L.or_scene_copy.argtypes = [vp, vp, vp, vp, vp, vp]
        L.or_scene_copy.restype = None
        L.or_load_material.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp]
        L.or_register_texture.argtypes = [ctypes.c_char_p, vp, i, i]
        L.or_trace_rays.argtypes = [vp, vp, i, vp]
        L.or_trace_rays.restype = None
        L.or_scatter.argtypes = [vp, vp, i, ctypes.c_uint32, vp, ctypes.POINTER(ctypes.c_uint32),
                                 ctypes.POINTER(i), ctypes.POINTER(i)]
        L.or_scatter.restype = None
        L.or_direct_light.argtypes = [vp, vp, vp, ctypes.POINTER(ctypes.c_uint32), vp]
        L.or_direct_light.restype = None
        L.or_render.argtypes = [vp, vp, vp, vp, vp, vp, vp, i, i, ctypes.POINTER(OrOptions), vp]
        L.or_default_options.argtypes = [ctypes.POINTER(OrOptions)]
        L.or_default_options.restype = None
        L.or_tonemap.argtypes = [vp, vp, i, vp]
        L.or_tonemap.restype = None
        L.or_correct_color.argtypes = [vp, vp]
        L.or_correct_color.restype = None
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def mt19937(count, skip=0):
    out = np.zeros(count, dtype=np.uint32)
    lib().or_mt19937(_p(out), count, skip)
    return out


def rng_sequence(state, n):
    s = ctypes.c_uint32(state)
    vals = []
    for _ in range(n):
        vals.append(lib().or_rng_next(ctypes.byref(s)))
    return np.array(vals, dtype=np.float32), s.value


class OracleScene:
    def __init__(self, scene_path=None, triangles=None, count=None):
        L = lib()
        self.camera = np.zeros(7, dtype=np.float32)
        if scene_path is not None:
            self.h = L.or_scene_load(scene_path.encode(), _p(self.camera))
        else:
            buf = ctypes.create_string_buffer(triangles, len(triangles))
            self.h = L.or_scene_from_triangles(ctypes.cast(buf, ctypes.c_void_p), count)
        if not self.h:
            raise RuntimeError("oracle scene load failed: " + L.or_last_error().decode())
        t, n, i, l = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        L.or_scene_counts(self.h, ctypes.byref(t), ctypes.byref(n), ctypes.byref(i), ctypes.byref(l))
        self.ntris, self.nnodes, self.nindices, self.nlights = t.value, n.value, i.value, l.value

    def arrays(self):
        tris = ctypes.create_string_buffer(self.ntris * 152)
        nodes = ctypes.create_string_buffer(max(self.nnodes, 1) * 20)
        idx = np.zeros(max(self.nindices, 1), dtype=np.int32)
        lights = np.zeros(max(self.nlights, 1), dtype=np.int32)
        bounds = np.zeros(6, dtype=np.float32)
        lib().or_scene_copy(self.h, ctypes.cast(tris, ctypes.c_void_p), ctypes.cast(nodes, ctypes.c_void_p),
                            _p(idx), _p(lights), _p(bounds))
        return (tris.raw, nodes.raw[: self.nnodes * 20], idx[: self.nindices], lights[: self.nlights], bounds)

    def trace_rays(self, rays):
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        out = np.zeros((len(rays), 12), dtype=np.float32)
        lib().or_trace_rays(self.h, _p(rays), len(rays), _p(out))
        return out

    def direct_light(self, pos, normal, rng):
        """sample_direct_light at one point -> (radiance float32[3], rng after)."""
        p = np.ascontiguousarray(pos, dtype=np.float32)
        n = np.ascontiguousarray(normal, dtype=np.float32)
        out = np.zeros(3, dtype=np.float32)
        st = ctypes.c_uint32(int(rng))
        lib().or_direct_light(self.h, _p(p), _p(n), ctypes.byref(st), _p(out))
        return out, st.value

    def render(self, camera, fb, sq, cnt, rng, width, height, passes, sample_count_arg=1, pixels=None,
               adaptive=True, min_samples=100, tolerance=0.05, max_depth=0, threads=0):
        """path_tracing over `passes` passes on G_Buffer-layout arrays (modified in place)."""
        o = OrOptions()
        lib().or_default_options(ctypes.byref(o))
        o.width, o.height, o.passes = width, height, passes
        o.adaptive, o.min_samples, o.tolerance, o.max_depth, o.threads = (int(adaptive), min_samples, tolerance,
                                                                         max_depth, threads)
        cam = np.ascontiguousarray(camera, dtype=np.float32)
        counters = np.zeros(N_COUNTERS, dtype=np.uint64)
        px = None if pixels is None else np.ascontiguousarray(pixels, dtype=np.int32)
        for a, dt in ((fb, np.float32), (sq, np.float32), (cnt, np.int32), (rng, np.uint32)):
            assert a.dtype == dt and a.flags["C_CONTIGUOUS"]
        lib().or_render(self.h, _p(cam), _p(fb), _p(sq), _p(cnt), _p(rng), _p(px),
                        0 if px is None else len(px), sample_count_arg, ctypes.byref(o), _p(counters))
        out = {k: int(counters[i]) for i, k in enumerate(COUNTER_NAMES)}
        out["deep_push"] = int(counters[DEEP_PUSH])
        out["cut"] = int(counters[CUT])
        out["deep_hist"] = [int(v) for v in counters[DEEP_HIST:DEEP_HIST + DEEP_HIST_BINS]]
        out["hazards"] = {k: int(counters[i]) for k, i in HAZARDS.items()}
        return out

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().or_scene_free(self.h)
                self.h = None
        except Exception:
            pass


def tonemap(fb, cnt):
    fb = np.ascontiguousarray(fb, dtype=np.float32)
    cnt = np.ascontiguousarray(cnt, dtype=np.int32)
    out = np.zeros((len(cnt), 4), dtype=np.uint8)
    lib().or_tonemap(_p(fb), _p(cnt), len(cnt), _p(out))
    return out


def correct_color(c):
    a = np.ascontiguousarray(c, dtype=np.float32)
    o = np.zeros(3, dtype=np.float32)
    lib().or_correct_color(_p(a), _p(o))
    return o


def register_texture(path, rgba):
    """texels (H, W, 4) uint8 for `texture <path>` in .mat files (the oracle decodes no images)."""
    a = np.ascontiguousarray(rgba, dtype=np.uint8)
    if lib().or_register_texture(path.encode(), _p(a), a.shape[1], a.shape[0]) != 0:
        raise RuntimeError("or_register_texture failed")


def load_material(path, name):
    out = np.zeros(10, dtype=np.float32)
    rc = lib().or_load_material(path.encode(), name.encode(), _p(out))
    return rc, out
