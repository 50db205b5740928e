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


def _mt(n):
    import oracle

    return oracle.mt19937(n)
