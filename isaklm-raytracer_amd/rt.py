"""ctypes binding of include/isaklm_rt.h — the host-side mirror of the
reference's render interface (create_scene / G_Buffer / Camera / render /
save_render, rt/main.cu:97-132) used by the tests, smoke() and bench.py.

The product path is the in-tree libisaklm_rt.so (HIP kernels for gfx950);
importing this module fails loudly if it is missing — there is no CPU
fallback.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libisaklm_rt.so")
# tooling only (tools/ab.py A/B of kernel builds): load another build of the same library
LIB_PATH = os.environ.get("ISAKLM_RT_LIB_OVERRIDE", LIB_PATH)


class Vec3D(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float)]


class Bounding_Box(ctypes.Structure):
    _fields_ = [("min", Vec3D), ("max", Vec3D)]


class KD_Tree(ctypes.Structure):
    _fields_ = [("bounding_box", Bounding_Box), ("nodes", ctypes.c_void_p), ("triangle_indicies", ctypes.c_void_p)]


class Scene(ctypes.Structure):  # rt/scene.cuh:114-121
    _fields_ = [("triangles", ctypes.c_void_p), ("triangle_count", ctypes.c_int),
                ("light_indicies", ctypes.c_void_p), ("light_count", ctypes.c_int), ("kd_tree", KD_Tree)]


class G_Buffer(ctypes.Structure):  # rt/screen.cuh:15-21
    _fields_ = [("frame_buffer", ctypes.c_void_p), ("squared_luminance", ctypes.c_void_p),
                ("sample_count", ctypes.c_void_p), ("random_numbers", ctypes.c_void_p)]


class Camera(ctypes.Structure):  # rt/camera.cuh:15-26
    _fields_ = [("position", Vec3D), ("yaw", ctypes.c_float), ("pitch", ctypes.c_float),
                ("FOV", ctypes.c_float), ("aperture_radius", ctypes.c_float)]

    def as_list(self):
        p = self.position
        return [p.x, p.y, p.z, self.yaw, self.pitch, self.FOV, self.aperture_radius]


class RtOptions(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("passes", ctypes.c_int),
                ("adaptive", ctypes.c_int), ("min_samples", ctypes.c_int), ("tolerance", ctypes.c_float),
                ("max_depth", ctypes.c_int), ("kernel", ctypes.c_int), ("stream", ctypes.c_void_p),
                ("counters_device", ctypes.c_void_p), ("wave_times_device", ctypes.c_void_p),
                ("wf_tail", ctypes.c_int), ("wf_finish_waves", ctypes.c_int), ("profile", ctypes.c_int),
                ("wf_descent_cap", ctypes.c_int), ("wf_postpone", ctypes.c_int), ("wf_wide", ctypes.c_int),
                ("shard_id", ctypes.c_int), ("num_shards", ctypes.c_int), ("wf_pipelines", ctypes.c_int),
                ("wf_long_depth", ctypes.c_int), ("traversal", ctypes.c_int), ("overlap", ctypes.c_int),
                ("check_interval", ctypes.c_int), ("debug", ctypes.c_int), ("coalesce_passes", ctypes.c_int)]


class RtProfile(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int), ("trace_launches", ctypes.c_int), ("shade_launches", ctypes.c_int),
                ("finish_launches", ctypes.c_int), ("start_ms", ctypes.c_float), ("trace_ms", ctypes.c_float),
                ("shade_ms", ctypes.c_float), ("finish_ms", ctypes.c_float), ("call_ms", ctypes.c_float),
                ("trace_union_ms", ctypes.c_float), ("pipelines", ctypes.c_int)]


def last_profile():
    """Kernel timing of the last rt_render with options(profile=True) on this device."""
    p = RtProfile()
    check(lib().rt_last_profile(ctypes.byref(p)))
    return {k: getattr(p, k) for k, _ in RtProfile._fields_}


def profile_history(reset=False):
    """RtProfile of every profiled rt_render since the last reset, oldest first
    (rt_profile_history: waits for those calls' kernels, not for the chain)."""
    n = ctypes.c_int(0)
    check(lib().rt_profile_history(None, 0, ctypes.byref(n), 0))
    buf = (RtProfile * max(n.value, 1))()
    check(lib().rt_profile_history(buf, n.value, ctypes.byref(n), int(reset)))
    return [{k: getattr(buf[i], k) for k, _ in RtProfile._fields_} for i in range(n.value)]


DEV_HIST_BINS = 18


class RtDeviations(ctypes.Structure):
    _fields_ = [("watchdog_paths", ctypes.c_ulonglong), ("cut_paths", ctypes.c_ulonglong),
                ("max_deep_depth", ctypes.c_ulonglong), ("deep_paths", ctypes.c_ulonglong),
                ("deep_hist", ctypes.c_ulonglong * DEV_HIST_BINS),
                ("bounded_checked", ctypes.c_ulonglong), ("bounded_mismatches", ctypes.c_ulonglong),
                ("mismatch_ray", ctypes.c_float * 6),
                ("owed_pixels", ctypes.c_ulonglong), ("owed_passes", ctypes.c_ulonglong),
                ("long_safety_quits", ctypes.c_ulonglong), ("stranded_pixels", ctypes.c_ulonglong),
                ("check_dropped", ctypes.c_ulonglong), ("linger_expiries", ctypes.c_ulonglong),
                ("long_closed", ctypes.c_ulonglong)]


HANDOFF_FIELDS = ("owed_pixels", "owed_passes", "long_safety_quits", "stranded_pixels", "check_dropped",
                  "linger_expiries", "long_closed")


def deviation_stats(reset=False):
    """Always-on deviation statistics of every rt_render on this device since
    the last reset (rt_deviation_stats): watchdog / depth-limit cuts, the
    histogram of paths that ended at depth >= 64 (bin k: [64*2^k, 64*2^(k+1))),
    the guard's checks, and the deep-path hand-off's events (owed passes of
    chained calls; safety-net exits, stranded pixels, dropped guard records
    and linger expiries, which a working render keeps at 0)."""
    d = RtDeviations()
    check(lib().rt_deviation_stats(ctypes.byref(d), int(reset)))
    out = {"watchdog_paths": d.watchdog_paths, "cut_paths": d.cut_paths, "max_deep_depth": d.max_deep_depth,
           "deep_paths": d.deep_paths, "deep_hist": [int(v) for v in d.deep_hist],
           "bounded_checked": int(d.bounded_checked), "bounded_mismatches": int(d.bounded_mismatches),
           "mismatch_ray": [float(v) for v in d.mismatch_ray]}
    out.update({k: int(getattr(d, k)) for k in HANDOFF_FIELDS})
    return out


def join(stream=None):
    """rt_join: `stream` (None: the host) waits for every render's device work,
    chained calls' deep-path tails included."""
    check(lib().rt_join(stream))


ABI_VERSION = 8  # RT_ABI_VERSION of include/isaklm_rt.h
E_INCOMPLETE = -7  # RT_E_INCOMPLETE: a join found stranded pixels
DEBUG_CALL_LOG, DEBUG_LONG_LOG, DEBUG_CHECK_FAULT, DEBUG_LONG_QUIT = 1, 2, 4, 8  # RtOptions.debug bits
DEBUG_SERIAL_LONG_FIRST, DEBUG_SERIAL_FIN_FIRST = 16, 32  # (tests: serialised dispatch in either order)
TRIANGLE_BYTES = 152
NODE_BYTES = 20
COUNTER_NAMES = ["node", "tri", "hit", "texel", "nee", "sample", "skip", "ray", "watchdog", "maxdepth"]
FINISH_COUNTER_NAMES = ["finish_node", "finish_tri", "finish_ray", "cand", "plane", "deep_push", "t_descend", "t_leaves",
                        "t_fetch", "rounds", "chunks", "bary", "wide_calls", "wide_rounds", "t_wide", "t_wide_load", "t_wide_leaf", "t_wide_expand",
                       "t_leaf_wait", "t_leaf_setup", "t_leaf_test", "t_leaf_bary", "spill_push", "spill_pop",
                        "pend_lanes", "leaf_tests", "t_desc_wait", "b_bvh_node", "b_bvh_tri", "b_bary"]
N_COUNTERS = 40

_lib = None


class RtError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RtError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.rt_last_error.restype = ctypes.c_char_p
        L.rt_version.restype = ctypes.c_char_p
        L.rt_device_alloc.argtypes = [ctypes.POINTER(vp), sz]
        L.rt_free.argtypes = [vp]
        L.rt_upload.argtypes = [vp, vp, sz]
        L.rt_download.argtypes = [vp, vp, sz]
        L.rt_memset.argtypes = [vp, i, sz]
        L.rt_device_count.argtypes = [ctypes.POINTER(i)]
        L.rt_set_device.argtypes = [i]
        L.rt_host_free.argtypes = [vp]
        L.rt_host_free.restype = None
        L.rt_gbuffer_save.argtypes = [G_Buffer, i, i, i, ctypes.c_char_p]
        L.rt_gbuffer_load.argtypes = [ctypes.c_char_p, G_Buffer, i, i, ctypes.POINTER(i)]
        L.rt_decode_image.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp), ctypes.POINTER(i), ctypes.POINTER(i)]
        L.rt_decode_image_memory.argtypes = [vp, sz, ctypes.POINTER(vp), ctypes.POINTER(i), ctypes.POINTER(i)]
        L.rt_gbuffer_seeds.argtypes = [vp, sz, ctypes.c_uint64]
        L.rt_gbuffer_create.argtypes = [i, i, ctypes.c_uint64, ctypes.POINTER(G_Buffer)]
        L.rt_gbuffer_destroy.argtypes = [ctypes.POINTER(G_Buffer)]
        L.rt_host_scene_create.argtypes = [ctypes.POINTER(vp)]
        L.rt_host_scene_destroy.argtypes = [vp]
        L.rt_host_scene_destroy.restype = None
        L.rt_host_scene_load_mesh.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, vp, vp, i]
        L.rt_host_scene_load_file.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(Camera)]
        L.rt_host_scene_triangles.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(i)]
        L.rt_generate_scene.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, sz]
        L.rt_build_kd_tree.argtypes = [vp, i, ctypes.POINTER(vp), ctypes.POINTER(i), ctypes.POINTER(vp),
                                       ctypes.POINTER(i), ctypes.POINTER(Bounding_Box)]
        L.rt_create_scene.argtypes = [vp, ctypes.POINTER(Scene), ctypes.POINTER(i), ctypes.POINTER(i)]
        L.rt_destroy_scene.argtypes = [ctypes.POINTER(Scene)]
        L.rt_scene_prepare.argtypes = [ctypes.POINTER(Scene), ctypes.POINTER(vp)]
        L.rt_scene_prepare_counts.argtypes = [ctypes.POINTER(Scene), i, i, ctypes.POINTER(vp)]
        L.rt_scene_prepare_host.argtypes = [vp, i, vp, i, vp, i, vp, i, Bounding_Box, ctypes.POINTER(vp)]
        L.rt_scene_release.argtypes = [vp]
        L.rt_scene_info.argtypes = [vp, ctypes.POINTER(sz), ctypes.POINTER(i), ctypes.POINTER(i),
                                    ctypes.POINTER(i), ctypes.POINTER(i)]
        L.rt_default_options.argtypes = [ctypes.POINTER(RtOptions)]
        L.rt_default_options.restype = None
        L.rt_render.argtypes = [vp, G_Buffer, Camera, i, ctypes.POINTER(RtOptions)]
        L.rt_tonemap.argtypes = [G_Buffer, vp, i, i, vp]
        L.rt_save_render.argtypes = [G_Buffer, i, i, ctypes.c_char_p]
        L.rt_deviation_stats.argtypes = [ctypes.POINTER(RtDeviations), i]
        L.rt_join.argtypes = [vp]
        L.rt_profile_history.argtypes = [ctypes.POINTER(RtProfile), i, ctypes.POINTER(i), i]
        L.rt_shutdown.restype = None
        L.rt_abi_version.restype = i
        if L.rt_abi_version() != ABI_VERSION:
            raise RtError(f"{LIB_PATH}: ABI version {L.rt_abi_version()}, this binding expects {ABI_VERSION} "
                          "(rebuild with __graft_entry__.build())")
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise RtError(f"rt error {rc}: {lib().rt_last_error().decode()}")


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def generate_scene(name, out_dir):
    buf = ctypes.create_string_buffer(4096)
    check(lib().rt_generate_scene(name.encode(), out_dir.encode(), buf, 4096))
    return buf.value.decode()


def seeds(count, skip=0):
    out = np.zeros(count, dtype=np.uint32)
    check(lib().rt_gbuffer_seeds(_ptr(out), count, skip))
    return out


class HostScene:
    """Host triangle list (create_models / load_mesh, rt/create_models.cuh:17)."""

    def __init__(self, scene_path=None):
        h = ctypes.c_void_p()
        check(lib().rt_host_scene_create(ctypes.byref(h)))
        self.h = h
        self.camera = Camera()
        if scene_path:
            check(lib().rt_host_scene_load_file(self.h, scene_path.encode(), ctypes.byref(self.camera)))

    def load_mesh(self, obj, mat, offset, matrix, smooth=False):
        off = np.asarray(offset, dtype=np.float32)
        m = np.asarray(matrix, dtype=np.float32).reshape(9)
        check(lib().rt_host_scene_load_mesh(self.h, obj.encode(), mat.encode(), _ptr(off), _ptr(m), int(smooth)))

    def triangles_bytes(self):
        p, n = ctypes.c_void_p(), ctypes.c_int()
        check(lib().rt_host_scene_triangles(self.h, ctypes.byref(p), ctypes.byref(n)))
        return ctypes.string_at(p, n.value * TRIANGLE_BYTES), n.value

    def triangle_ptr(self):
        p, n = ctypes.c_void_p(), ctypes.c_int()
        check(lib().rt_host_scene_triangles(self.h, ctypes.byref(p), ctypes.byref(n)))
        return p, n.value

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().rt_host_scene_destroy(self.h)
                self.h = None
        except Exception:
            pass


def decode_image(path=None, data=None):
    """stbi_load(path, &w, &h, &n, 4) as make_texture calls it (rt/scene.cuh:33):
    RGBA8 (H, W, 4) uint8, rows in file order.  PNG and baseline JPEG."""
    p, w, h = ctypes.c_void_p(), ctypes.c_int(), ctypes.c_int()
    if data is not None:
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        check(lib().rt_decode_image_memory(_ptr(buf), buf.nbytes, ctypes.byref(p), ctypes.byref(w), ctypes.byref(h)))
    else:
        check(lib().rt_decode_image(path.encode(), ctypes.byref(p), ctypes.byref(w), ctypes.byref(h)))
    try:
        n = w.value * h.value * 4
        return np.frombuffer(ctypes.string_at(p, n), dtype=np.uint8).reshape(h.value, w.value, 4).copy()
    finally:
        lib().rt_host_free(p)


def build_kd_tree(tri_ptr, n):
    """create_kd_tree on the host -> (nodes bytes, indices int32 array, bounds[6])."""
    L = lib()
    nodes, idx = ctypes.c_void_p(), ctypes.c_void_p()
    nn, ni = ctypes.c_int(), ctypes.c_int()
    bb = Bounding_Box()
    check(L.rt_build_kd_tree(tri_ptr, n, ctypes.byref(nodes), ctypes.byref(nn), ctypes.byref(idx),
                             ctypes.byref(ni), ctypes.byref(bb)))
    nb = ctypes.string_at(nodes, nn.value * NODE_BYTES)
    ib = np.frombuffer(ctypes.string_at(idx, ni.value * 4), dtype=np.int32).copy()
    L.rt_host_free(nodes)
    L.rt_host_free(idx)
    return nb, ib, [bb.min.x, bb.min.y, bb.min.z, bb.max.x, bb.max.y, bb.max.z]


class DeviceScene:
    """create_scene (rt/create_scene.cuh:18) -> reference-layout device Scene,
    then rt_scene_prepare -> traversal layout.  rt_scene_prepare takes the
    Scene alone (the reference's Scene has no node/index counts); the counts
    rt_create_scene reports are kept only to cross-check what prepare derived."""

    def __init__(self, host_scene):
        self.scene = Scene()
        nn, ni = ctypes.c_int(), ctypes.c_int()
        check(lib().rt_create_scene(host_scene.h, ctypes.byref(self.scene), ctypes.byref(nn), ctypes.byref(ni)))
        self.node_count, self.index_count = nn.value, ni.value
        self.prepared = ctypes.c_void_p()
        check(lib().rt_scene_prepare(ctypes.byref(self.scene), ctypes.byref(self.prepared)))

    def info(self):
        b, t, n, i, d = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().rt_scene_info(self.prepared, ctypes.byref(b), ctypes.byref(t), ctypes.byref(n), ctypes.byref(i),
                                  ctypes.byref(d)))
        return {"device_bytes": b.value, "triangles": t.value, "nodes": n.value, "indices": i.value,
                "max_depth": d.value, "lights": self.scene.light_count}

    def release(self):
        if getattr(self, "prepared", None):
            lib().rt_scene_release(self.prepared)
            self.prepared = None
        if getattr(self, "scene", None) is not None and self.scene.triangles:
            lib().rt_destroy_scene(ctypes.byref(self.scene))

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class GBuffer:
    """G_Buffer (rt/screen.cuh:22-46) on the device; seeds = mt19937 outputs
    [seed_skip, seed_skip + W*H)."""

    def __init__(self, width, height, seed_skip=0):
        self.width, self.height = width, height
        self.g = G_Buffer()
        check(lib().rt_gbuffer_create(width, height, seed_skip, ctypes.byref(self.g)))

    @property
    def n(self):
        return self.width * self.height

    def download(self):
        n = self.n
        fb = np.zeros((n, 3), dtype=np.float32)
        sq = np.zeros(n, dtype=np.float32)
        cnt = np.zeros(n, dtype=np.int32)
        rng = np.zeros(n, dtype=np.uint32)
        L = lib()
        check(L.rt_download(_ptr(fb), self.g.frame_buffer, fb.nbytes))
        check(L.rt_download(_ptr(sq), self.g.squared_luminance, sq.nbytes))
        check(L.rt_download(_ptr(cnt), self.g.sample_count, cnt.nbytes))
        check(L.rt_download(_ptr(rng), self.g.random_numbers, rng.nbytes))
        return fb, sq, cnt, rng

    def upload(self, fb, sq, cnt, rng):
        L = lib()
        fb = np.ascontiguousarray(fb, dtype=np.float32)
        sq = np.ascontiguousarray(sq, dtype=np.float32)
        cnt = np.ascontiguousarray(cnt, dtype=np.int32)
        rng = np.ascontiguousarray(rng, dtype=np.uint32)
        check(L.rt_upload(self.g.frame_buffer, _ptr(fb), fb.nbytes))
        check(L.rt_upload(self.g.squared_luminance, _ptr(sq), sq.nbytes))
        check(L.rt_upload(self.g.sample_count, _ptr(cnt), cnt.nbytes))
        check(L.rt_upload(self.g.random_numbers, _ptr(rng), rng.nbytes))

    def save(self, path, sample_count):
        """checkpoint (rt_gbuffer_save): the whole progressive state + the caller's sample count"""
        check(lib().rt_gbuffer_save(self.g, self.width, self.height, sample_count, str(path).encode()))

    def load(self, path):
        """resume (rt_gbuffer_load); returns the saved sample count"""
        sc = ctypes.c_int()
        check(lib().rt_gbuffer_load(str(path).encode(), self.g, self.width, self.height, ctypes.byref(sc)))
        return sc.value

    def free(self):
        if getattr(self, "g", None) is not None and self.g.frame_buffer:
            lib().rt_gbuffer_destroy(ctypes.byref(self.g))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


KERNEL_MEGA = 0
KERNEL_WAVEFRONT = 1
TRAVERSAL_BOUNDED = 0
TRAVERSAL_KD = 1
TRAVERSAL_BOUNDED_COUNTED = 2  # measurement: the bounded queue trace kernel counts its own work


def options(width, height, passes=1, adaptive=True, min_samples=100, tolerance=0.05, max_depth=0, stream=None,
            counters=None, kernel=KERNEL_MEGA, wf_tail=0, wf_finish_waves=0, profile=False, wf_descent_cap=0,
            wf_postpone=0, wf_wide=0, shard_id=0, num_shards=1, wave_times=None, wf_pipelines=0, wf_long_depth=0,
            traversal=None, overlap=False, check_interval=0, debug=0, coalesce_passes=0):
    """RtOptions; traversal: TRAVERSAL_BOUNDED / TRAVERSAL_KD (None: the
    library default, or RT_TRAVERSAL from the environment); overlap: chained
    calls (RtOptions.overlap: join before reading the frame); check_interval:
    the bounded traversal's run-time guard (0: the library default, 1 ray in
    4096; < 0: off); coalesce_passes: chained calls of fewer passes are
    coalesced up to this many (0: the library default 256; < 0: off)."""
    o = RtOptions()
    lib().rt_default_options(ctypes.byref(o))
    o.width, o.height, o.passes = width, height, passes
    o.adaptive, o.min_samples, o.tolerance, o.max_depth = int(adaptive), min_samples, tolerance, max_depth
    o.kernel = kernel
    o.stream = stream
    o.counters_device = counters
    o.wf_tail, o.wf_finish_waves, o.profile = wf_tail, wf_finish_waves, int(profile)
    o.wf_descent_cap, o.wf_postpone, o.wf_wide = wf_descent_cap, wf_postpone, wf_wide
    o.shard_id, o.num_shards = shard_id, num_shards
    o.wave_times_device = wave_times
    o.wf_pipelines = wf_pipelines
    o.wf_long_depth = wf_long_depth
    o.overlap, o.check_interval, o.debug = int(overlap), check_interval, debug
    o.coalesce_passes = coalesce_passes
    if traversal is None and os.environ.get("RT_TRAVERSAL"):
        traversal = {"bounded": TRAVERSAL_BOUNDED, "kd": TRAVERSAL_KD,
                     "bounded_counted": TRAVERSAL_BOUNDED_COUNTED}[os.environ["RT_TRAVERSAL"]]
    if traversal is not None:
        o.traversal = traversal
    return o


def render(dscene, gbuf, camera, sample_count, opt):
    """render() (rt/render.cuh:62): resets when sample_count == 0, then opt.passes passes."""
    check(lib().rt_render(dscene.prepared, gbuf.g, camera, sample_count, ctypes.byref(opt)))


class DeviceCounters:
    def __init__(self):
        p = ctypes.c_void_p()
        check(lib().rt_device_alloc(ctypes.byref(p), N_COUNTERS * 8))
        self.p = p
        self.zero()

    def zero(self):
        check(lib().rt_memset(self.p, 0, N_COUNTERS * 8))

    def read(self, finisher=False):
        """The reference-comparable counters; finisher=True adds the wavefront
        finisher's share of node/tri/ray (RT_CNT_FIN_*)."""
        a = np.zeros(N_COUNTERS, dtype=np.uint64)
        check(lib().rt_download(_ptr(a), self.p, a.nbytes))
        out = {k: int(a[i]) for i, k in enumerate(COUNTER_NAMES)}
        out["deep_push"] = int(a[15])  # RT_CNT_DEEP_PUSH: reference-comparable (the oracle counts it too)
        if finisher:
            out.update({k: int(a[10 + i]) for i, k in enumerate(FINISH_COUNTER_NAMES) if k})
        return out

    def __del__(self):
        try:
            lib().rt_free(self.p)
        except Exception:
            pass


def tonemap(gbuf):
    """draw_frame colour math -> (H*W, 4) uint8, row 0 = bottom."""
    L = lib()
    n = gbuf.n
    d = ctypes.c_void_p()
    check(L.rt_device_alloc(ctypes.byref(d), n * 4))
    try:
        check(L.rt_tonemap(gbuf.g, d, gbuf.width, gbuf.height, None))
        out = np.zeros((n, 4), dtype=np.uint8)
        check(L.rt_download(_ptr(out), d, out.nbytes))
    finally:
        L.rt_free(d)
    return out


def save_render(gbuf, path):
    check(lib().rt_save_render(gbuf.g, gbuf.width, gbuf.height, path.encode()))


COMM_ID_BYTES = 128


class Comm:
    """RCCL communicator of the C-ABI (rt_comm_*): rt_reduce_shards sums the
    shards' fb / sq / count into `root`."""

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        check(lib().rt_comm_unique_id(buf))
        return buf.raw

    def __init__(self, nranks, rank, uid):
        L = lib()
        L.rt_comm_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
        L.rt_comm_destroy.argtypes = [ctypes.c_void_p]
        L.rt_reduce_shards.argtypes = [ctypes.c_void_p, G_Buffer, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p]
        self.h = ctypes.c_void_p()
        check(L.rt_comm_create(nranks, rank, uid, ctypes.byref(self.h)))

    def reduce(self, gbuf_g, width, height, root=0, stream=None):
        check(lib().rt_reduce_shards(self.h, gbuf_g, width, height, root, stream))

    def close(self):
        if self.h:
            check(lib().rt_comm_destroy(self.h))
            self.h = ctypes.c_void_p()
