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
               num_shards=1, wf_pipelines=0, wf_long_depth=0, traversal=None, overlap=False, check_interval=0,
               debug=0, stream=None, coalesce_passes=0):
        g = rt.GBuffer(W, H, seed_skip)
        cnt = rt.DeviceCounters() if count else None
        per_call = list(passes) if isinstance(passes, (list, tuple)) else [passes] * calls  # passes of each call
        for c, pc in enumerate(per_call):
            opt = rt.options(W, H, pc, adaptive, min_samples, tolerance, max_depth,
                             counters=cnt.p if cnt else None, kernel=kernel, wf_tail=wf_tail,
                             wf_finish_waves=wf_finish_waves, wf_wide=wf_wide, shard_id=shard_id,
                             num_shards=num_shards, wf_pipelines=wf_pipelines, wf_long_depth=wf_long_depth,
                             traversal=traversal, overlap=overlap, check_interval=check_interval, debug=debug,
                             stream=stream, coalesce_passes=coalesce_passes)
            rt.render(self.dev, g, self.camera, 0 if c == 0 else 1, opt)
        rt.join()  # (chained calls: their deep-path tails) — download() uses the null stream
        out = g.download()
        counters = cnt.read() if cnt else None
        return out, counters, g


def oracle_render(path, W, H, passes, calls=1, adaptive=False, min_samples=100, tolerance=0.05, max_depth=0,
                  seed_skip=0, pixels=None, scene=None, camera=None, deviations=None):
    """The oracle over the same calls as GpuRun.render.  Returns the G_Buffer
    arrays and the counters comparable with the GPU's counting build; the
    deviation statistics (depth-limit cuts, deep-path histogram: the GPU's
    always-on rt_deviation_stats) go into the `deviations` dict if given."""
    sc = scene or oracle.OracleScene(path)
    n = W * H
    fb = np.zeros(n * 3, np.float32)
    sq = np.zeros(n, np.float32)
    cnt = np.zeros(n, np.int32)
    rng = oracle.mt19937(n, seed_skip)
    cam = sc.camera if camera is None else camera
    total = {}
    per_call = list(passes) if isinstance(passes, (list, tuple)) else [passes] * calls  # passes of each call
    for c, pc in enumerate(per_call):
        k = sc.render(cam, fb, sq, cnt, rng, W, H, pc, sample_count_arg=0 if c == 0 else 1, pixels=pixels,
                      adaptive=adaptive, min_samples=min_samples, tolerance=tolerance, max_depth=max_depth)
        cut, hist, haz = k.pop("cut"), k.pop("deep_hist"), k.pop("hazards")
        if deviations is not None:
            deviations["cut"] = deviations.get("cut", 0) + cut
            old = deviations.get("deep_hist", [0] * len(hist))
            deviations["deep_hist"] = [a + b for a, b in zip(old, hist)]
            h = deviations.setdefault("hazards", {})
            for key, v in haz.items():
                h[key] = h.get(key, 0) + v
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


# ------------------------------------------------------------ deep-path trap
def make_trap_scene(d, length=60.0):
    """Deep paths on demand: a light guide.  The camera looks
    obliquely into the end face of a long, thin glass rod (glass.mat: n 1.51,
    roughness 0.001).  A camera ray refracted through the end face meets the
    side faces beyond the critical angle, so it is guided down the rod by
    total internal reflection; inside the medium the reference's specular
    weight is exactly 1 (rt/path_tracing.cuh:194-197) and the roulette
    survives with p = max(T) = 1, so the path runs ~100-1,000 bounces to the
    far end.  Rod 0.2 x 0.2 x `length` (the loader re-centres it: z in
    [-length/2, length/2]), a floor and a lamp beside it."""
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "trap.mat"), "w") as f:
        f.write("material glass\nalbedo 0.995 0.995 0.995\nroughness 0.001\nn 1.51\ntransparent\n\n"
                "material floor\nalbedo 0.7 0.7 0.7\nroughness 0.5\nn 1.5\n\n"
                "material lamp\nalbedo 0.8 0.8 0.8\nemittance 6.0 5.5 5.0\nroughness 0.5\nn 1.5\n")
    h, L = 0.1, length
    v = [(-h, -h, 0), (h, -h, 0), (h, h, 0), (-h, h, 0), (-h, -h, L), (h, -h, L), (h, h, L), (-h, h, L)]
    rod = ["# glass rod"] + [f"v {x} {y} {z}" for x, y, z in v]
    rod += ["usemtl glass", "f 1 4 3 2", "f 5 6 7 8", "f 1 2 6 5", "f 4 8 7 3", "f 1 5 8 4", "f 2 3 7 6"]
    with open(os.path.join(d, "rod.obj"), "w") as fh:
        fh.write("\n".join(rod) + "\n")
    room = ["# floor and lamp", "v -4 0 -4", "v 4 0 -4", "v 4 0 4", "v -4 0 4",
            "v -0.5 3 -0.5", "v 0.5 3 -0.5", "v 0.5 3 0.5", "v -0.5 3 0.5",
            "usemtl floor", "f 1 2 3 4", "usemtl lamp", "f 5 8 7 6"]
    with open(os.path.join(d, "room.obj"), "w") as fh:
        fh.write("\n".join(room) + "\n")
    scene = os.path.join(d, "scene.txt")
    with open(scene, "w") as fh:
        # the camera 0.43 in front of the end face (z = -length/2), 35 degrees off its axis
        fh.write("mesh rod.obj trap.mat 0 0 0 0 0 1 0\n"
                 f"mesh room.obj trap.mat 0 0.5 {-L / 2:.1f} 0 0 1 0\n"
                 f"camera -0.25 0.02 {-L / 2 - 0.35:.2f} 0.6202 -0.0465 0.3 0.002\n")
    return scene


# ------------------------------------------------------------ textured scene
TEXTURED_VARIANTS = {"floor": "jpeg_ycc420_odd", "wall": "png_pal8_trns", "lamp": "png_rgba8_adam7",
                     "back": "jpeg_ycc_q100", "grey": "png_grey4_trns"}


def make_textured_scene(d):
    """A closed room whose materials use textures (sample_texture, rt/trace_ray.cuh:31-46):
    UVs far outside [0, 1] (mod wrap), a triangle whose UVs are a tiny negative
    number (mod(uv, 1) == 1.0: the index reaches the padded texel after the
    image), an emissive textured lamp (emittance * texel), a
    material whose texture file is missing (untextured, as in the reference)
    and one untextured material.  Texture files are synthetic variants whose
    stb_image decode is recorded in tests/golden/textures.json.
    Returns (scene_path, {texture path as in the .mat: variant name})."""
    import texture_fixtures

    os.makedirs(os.path.join(d, "textures"), exist_ok=True)
    files = {}
    data = texture_fixtures.variants()
    for mat, var in TEXTURED_VARIANTS.items():
        ext = "jpg" if var.startswith("jpeg") else "png"
        rel = f"textures/{mat}.{ext}"
        with open(os.path.join(d, rel), "wb") as f:
            f.write(data[var])
        files[rel] = var
    mat_txt = ""
    for mat in ("floor", "wall", "back", "grey"):
        rel = [k for k, v in files.items() if v == TEXTURED_VARIANTS[mat]][0]
        mat_txt += f"material {mat}\nalbedo 0.9 0.85 0.8\nroughness 0.4\nn 1.5\ntexture {rel}\n\n"
    lamp = [k for k, v in files.items() if v == TEXTURED_VARIANTS["lamp"]][0]
    mat_txt += f"material lamp\nalbedo 0.7 0.7 0.7\nemittance 12.0 11.0 9.0\nroughness 0.5\nn 1.5\ntexture {lamp}\n\n"
    mat_txt += "material plain\nalbedo 0.5 0.6 0.7\nroughness 0.3\nn 1.4\n\n"
    mat_txt += "material lost\nalbedo 0.8 0.3 0.3\nroughness 0.3\nn 1.4\ntexture textures/does_not_exist.png\n\n"
    mat_txt += "material metal\nalbedo 0.95 0.9 0.8\nroughness 0.05\nn 1.2\nk 3.5\ntexture textures/floor.jpg\n"
    with open(os.path.join(d, "room.mat"), "w") as f:
        f.write(mat_txt)
    v = [(-1, 0, -1), (1, 0, -1), (1, 0, 1), (-1, 0, 1), (-1, 2, -1), (1, 2, -1), (1, 2, 1), (-1, 2, 1),
         (-0.3, 1.99, -0.3), (0.3, 1.99, -0.3), (0.3, 1.99, 0.3), (-0.3, 1.99, 0.3),
         (-0.5, 0.001, 0.2), (0.1, 0.001, 0.2), (-0.2, 0.6, 0.3)]
    vt = [(-1.3, -0.7), (2.7, -0.7), (2.7, 3.1), (-1.3, 3.1), (0, 0), (1, 0), (1, 1), (0, 1),
          (-1e-9, -1e-9), (0.25, 0.75)]
    obj = ["# textured room"] + [f"v {x} {y} {z}" for x, y, z in v] + [f"vt {a} {b}" for a, b in vt]
    obj += ["usemtl floor", "f 1/1 2/2 3/3 4/4",
            "usemtl wall", "f 1/5 4/6 8/7 5/8",
            "usemtl back", "f 4/1 3/2 7/3 8/4",
            "usemtl grey", "f 2/5 6/6 7/7 3/8",
            "usemtl plain", "f 5/5 8/6 7/7 6/8",
            "usemtl lost", "f 1/5 5/6 6/7 2/8",
            "usemtl lamp", "f 9/5 12/8 11/7 10/6",
            "usemtl metal", "f 13/9 14/9 15/9",
            "usemtl grey", "f 13/10 15/10 14/9"]
    with open(os.path.join(d, "room.obj"), "w") as f:
        f.write("\n".join(obj) + "\n")
    scene = os.path.join(d, "scene.txt")
    with open(scene, "w") as f:
        f.write("mesh room.obj room.mat 0 0 0 0 0 1 0\ncamera 0.05 1.0 -0.93 0.07 -0.05 1.3 0.005\n")
    return scene, files
