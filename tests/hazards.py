"""Inputs built to trigger the reference's numerical hazards (SURVEY
Appendix A) — test helpers for tests/test_gpu_hazards.py and
tests/test_hazards_cpu.py.

The per-pixel RNG of the reference (get_random_unilateral,
rt/path_tracing.cuh:34-43) is x' = out(x * 747796405 + 2891336453) with the
PCG RXS-M-XS output permutation out(s) = w ^ (w >> 22),
w = ((s >> ((s >> 28) + 4)) ^ s) * 277803737.  Every step is a bijection
of the 32-bit words, so the G-buffer seed that makes the k-th draw of a pass
return a chosen word can be computed backwards (rng_back).
"""
import os

import numpy as np

M_LCG, C_LCG, M_OUT = 747796405, 2891336453, 277803737
MASK = 0xFFFFFFFF


def rng_step(x):
    """one draw: the new state (= the returned word)"""
    s = (x * M_LCG + C_LCG) & MASK
    w = (((s >> ((s >> 28) + 4)) ^ s) * M_OUT) & MASK
    return (w >> 22) ^ w


def rng_step_inv(r):
    """the state x with rng_step(x) == r"""
    w = r ^ (r >> 22)  # bits 31..22 of w and r agree
    s_xs = (w * pow(M_OUT, -1, 1 << 32)) & MASK
    s = s_xs  # invert s ^ (s >> k): the top 4 bits fix k = (s >> 28) + 4 >= 4
    k = (s_xs >> 28) + 4
    for _ in range(8):
        s = s_xs ^ (s >> k)
    return ((s - C_LCG) * pow(M_LCG, -1, 1 << 32)) & MASK


def rng_back(word, k):
    """the seed whose (k+1)-th draw (index k) returns `word`"""
    x = word
    for _ in range(k + 1):
        x = rng_step_inv(x)
    return x


def unilateral(word):
    """the float the reference returns for a drawn word: float(x) / UINT32_MAX in f32"""
    return np.float32(np.float32(word) / np.float32(4294967295.0))


# words whose draw is exactly 1.0f: float(x) rounds to 2^32
ONE_WORDS = range((1 << 32) - 128, 1 << 32)


def cornell_variant(d, name, yaw_room=0.1, camera=None, extra_obj="", extra_mat=""):
    """The cornell scene's geometry (build/scenes/cornell) with the room
    rotated by `yaw_room` (0: every wall axis-aligned, so KD split planes
    coincide with wall planes) and an optional camera line / extra faces."""
    import helpers

    src = os.path.dirname(helpers.scene_path("cornell"))
    os.makedirs(d, exist_ok=True)
    obj = open(os.path.join(src, "cornell.obj")).read() + extra_obj
    mat = open(os.path.join(src, "cornell.mat")).read() + extra_mat
    with open(os.path.join(d, f"{name}.obj"), "w") as f:
        f.write(obj)
    with open(os.path.join(d, f"{name}.mat"), "w") as f:
        f.write(mat)
    cam = camera or "-0.3458 1.0 -3.5834 0.1 0 0.8 0"
    p = os.path.join(d, "scene.txt")
    with open(p, "w") as f:
        f.write(f"mesh {name}.obj {name}.mat 0 1 0 {yaw_room} 0 1 0\ncamera {cam}\n")
    return p


def root_split(osc):
    """(axis, offset) of the KD root (20-B reference nodes: plane_axis u8 @8, plane_offset f32 @12)"""
    _, nodes, _, _, _ = osc.arrays()
    axis = nodes[8]
    off = np.frombuffer(nodes[12:16], dtype=np.float32)[0]
    return int(axis), np.float32(off)


# ------------------------------------------------------------ input builders
def h4_seeds(osc, W, H, step=5, k=9):
    """mt19937 seeds with every `step`-th pixel replaced by a seed whose draw
    k (the NEE light pick of a pass whose first bounce is diffuse) returns a
    word whose float is exactly 1.0 — kept only where the oracle confirms the
    pick happened (single-pixel oracle runs).  Returns (seeds, planted)."""
    n = W * H
    rng0 = _mt(n)
    planted = 0
    for pix in range(0, n, step):
        for word in ONE_WORDS:
            seed = rng_back(word, k)
            trial = rng0.copy()
            trial[pix] = seed  # (the render advances trial in place)
            fb, sq, ct = np.zeros(n * 3, np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32)
            c = osc.render(osc.camera, fb, sq, ct, trial, W, H, 1, sample_count_arg=0,
                           pixels=np.array([pix], np.int32), adaptive=False)
            if c["hazards"]["xi_one"]:
                rng0[pix] = seed
                planted += 1
                break
    return rng0, planted


def h5_cameras(osc):
    """(camera on the root split plane, camera one ulp off it), aperture 0"""
    axis, split = root_split(osc)
    on = osc.camera.copy()
    on[6] = 0.0
    on[axis] = split
    off = on.copy()
    off[axis] = np.nextafter(split, np.float32(np.inf))
    return on, off


def h7_axis_seeds(W, H):
    """seeds: column x = W/2 - 1 draws 1.0f first (x jitter: direction.x ==
    0 for an axis-aligned camera), row y = H/2 - 1 draws 1.0f second
    (direction.y == 0)"""
    rng0 = _mt(W * H)
    one = (1 << 32) - 1
    for y in range(H):
        rng0[y * W + W // 2 - 1] = rng_back(one, 0)
    for x in range(W):
        rng0[(H // 2 - 1) * W + x] = rng_back(one, 1)
    return rng0


AXIS_CAMERA = "-0.3458 1.0 -3.5834 0 0 0.8 0"  # yaw 0, pitch 0, aperture 0: rotation = identity exactly

# zero-area triangles in the middle of the room: a repeated vertex (cross
# product exactly 0 after any transform: normalize -> NaN), three collinear
# points, and a nearly collinear one
DEGENERATE_OBJ = ("\nusemtl white\nv 0.2 1.2 0.3\nv 0.2 1.2 0.3\nv -0.1 0.9 0.2\nf -3 -2 -1\n"
                  "v -0.5 0.5 0.1\nv 0.0 0.5 0.1\nv 0.5 0.5 0.1\nf -3 -2 -1\n"
                  "v -0.4 0.3 -0.2\nv 0.4 1.3 0.4\nv 0.0 0.8 0.1\nf -3 -2 -1\n"
                  "v 0.1 0.2 -0.3\nv 0.1 1.6 -0.3\nv 0.1 1.6 -0.3\nf -3 -2 -1\n")


# The same two triangles twice, red then green, facing the camera: every hit on
# the quad has two passing tests at exactly the same s (identical records), the
# reference keeps the first listed in its leaf (strict <), and the bounded
# traversal's T* leaf shortcut must step aside (bvh_trace.h leaf_scan_min: a
# tie) — the colour says which copy won.
DUPLICATE_OBJ = ("\nusemtl red\nv -0.45 0.35 0.25\nv 0.45 0.35 0.25\nv 0.45 1.25 0.25\nv -0.45 1.25 0.25\n"
                 "f -4 -3 -2\nf -4 -2 -1\n"
                 "usemtl green\nv -0.45 0.35 0.25\nv 0.45 0.35 0.25\nv 0.45 1.25 0.25\nv -0.45 1.25 0.25\n"
                 "f -4 -3 -2\nf -4 -2 -1\n")

def _mt(n):
    import oracle

    return oracle.mt19937(n)


# ------------------------------------------------------------ adversarial geometry
ADV_MAT = ("material white\nalbedo 0.73 0.73 0.73\nroughness 0.5\nn 1.5\n\n"
           "material red\nalbedo 0.65 0.05 0.05\nroughness 0.5\nn 1.5\n\n"
           "material gold\nalbedo 0.9 0.7 0.3\nroughness 0.15\nn 1.2\nk 3.0\n\n"
           "material glass\nalbedo 0.99 0.99 0.99\nroughness 0.01\nn 1.5\ntransparent\n\n"
           "material light\nalbedo 0.78 0.78 0.78\nemittance 15.0 15.0 15.0\nroughness 0.5\nn 1.5\n")


def _adversarial_obj(seed):
    """A closed room (y in [0, 2]) holding the cases the BVH margins are
    hardest on: slivers (a vertex 1e-7..1e-2 of the edge length off the
    opposite edge), needles (two vertices 1e-7..1e-3 apart), near-degenerate
    fans sharing a vertex, and a dense cluster of tiny triangles — in every
    orientation, some axis-aligned."""
    rng = np.random.default_rng(seed)
    lines = ["# adversarial room"]
    vs = []

    def quad(mat, a, b, c, d):
        base = len(vs) + 1
        vs.extend([a, b, c, d])
        lines.append(f"usemtl {mat}")
        lines.append(f"f {base} {base + 1} {base + 2} {base + 3}")

    def tri(mat, a, b, c):
        base = len(vs) + 1
        vs.extend([a, b, c])
        lines.append(f"usemtl {mat}")
        lines.append(f"f {base} {base + 1} {base + 2}")

    quad("white", (-1, 0, -1), (1, 0, -1), (1, 0, 1), (-1, 0, 1))
    quad("white", (-1, 2, -1), (-1, 2, 1), (1, 2, 1), (1, 2, -1))
    quad("white", (-1, 0, 1), (1, 0, 1), (1, 2, 1), (-1, 2, 1))
    quad("red", (-1, 0, -1), (-1, 0, 1), (-1, 2, 1), (-1, 2, -1))
    quad("white", (1, 0, -1), (1, 2, -1), (1, 2, 1), (1, 0, 1))
    quad("light", (-0.3, 1.98, -0.3), (0.3, 1.98, -0.3), (0.3, 1.98, 0.3), (-0.3, 1.98, 0.3))

    def unit():
        v = rng.normal(size=3)
        return v / np.linalg.norm(v)

    mats = ["white", "gold", "glass", "red"]
    for k in range(300):  # slivers
        c = rng.uniform([-0.8, 0.2, -0.8], [0.8, 1.8, 0.8])
        u, w = unit(), unit()
        if k % 5 == 0:  # axis-aligned edge and offset
            u, w = np.eye(3)[k % 3], np.eye(3)[(k + 1) % 3]
        L = 10 ** rng.uniform(-2.5, -0.5)
        eps = L * 10 ** rng.uniform(-7, -2)
        p1, p2 = c, c + L * u
        p3 = c + L * rng.uniform(0, 1) * u + eps * w
        tri(mats[k % 4], p1, p2, p3)
    for k in range(300):  # needles
        c = rng.uniform([-0.8, 0.2, -0.8], [0.8, 1.8, 0.8])
        u, w = unit(), unit()
        L = 10 ** rng.uniform(-2, -0.3)
        p2 = c + L * u
        tri(mats[(k + 1) % 4], c, p2, p2 + L * 10 ** rng.uniform(-7, -3) * w)
    for k in range(20):  # fans of thin wedges around a shared vertex
        c = rng.uniform([-0.6, 0.4, -0.6], [0.6, 1.6, 0.6])
        u, w = unit(), unit()
        w = w - np.dot(w, u) * u
        w /= np.linalg.norm(w)
        L = 10 ** rng.uniform(-1.5, -0.7)
        angs = np.sort(rng.uniform(0, 2 * np.pi, 24))
        for a0, a1 in zip(angs[:-1], angs[1:]):
            tri(mats[k % 4], c, c + L * (np.cos(a0) * u + np.sin(a0) * w), c + L * (np.cos(a1) * u + np.sin(a1) * w))
    cl = np.array([0.2, 0.9, 0.1])  # a cloud of tiny triangles (1e-4..1e-3 of the room)
    for k in range(400):
        c = cl + rng.normal(scale=0.05, size=3)
        s = 2 * 10 ** rng.uniform(-4, -3)
        tri(mats[k % 3], c, c + s * unit(), c + s * unit())
    out = [lines[0]] + [f"v {x:.9g} {y:.9g} {z:.9g}" for x, y, z in vs] + lines[1:]
    return "\n".join(out) + "\n"


def adversarial_scene(d, variant="far", seed=1):
    """The adversarial room (_adversarial_obj) placed where float rounding is
    coarsest relative to its features:
      far   — translated to x = 1.2e4, z = -8e3 (|x| ~ 10^4, 1 ulp ~ 1e-3 m);
      tiny  — scaled to 2 cm and placed 100 units from the origin, so its
              cloud triangles are sub-millimetre (0.2-2 um .. 20 um) 100 m away;
      near  — at the origin (reference)."""
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "adv.obj"), "w") as f:
        f.write(_adversarial_obj(seed))
    with open(os.path.join(d, "adv.mat"), "w") as f:
        f.write(ADV_MAT)
    ox, oy, oz, sc = {"far": (12000.0, 1.0, -8000.0, 1.0), "tiny": (100.0, 0.01, 0.0, 0.01),
                      "near": (0.0, 1.0, 0.0, 1.0)}[variant]
    cam = (ox - 0.3458 * sc, oy, oz - 3.5834 * sc)
    p = os.path.join(d, "scene.txt")
    with open(p, "w") as f:
        f.write(f"mesh adv.obj adv.mat {ox!r} {oy!r} {oz!r} 0.1 0 {sc!r} 0\n"
                f"camera {cam[0]!r} {cam[1]!r} {cam[2]!r} 0.1 0 0.8 0.0001\n")
    return p
