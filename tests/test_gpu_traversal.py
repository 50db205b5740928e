"""The BVH-bounded traversal (RT_TRAVERSAL_BOUNDED, csrc/bvh_trace.h) is the
product path of the wavefront kernel.  It must give the reference's result
for every ray: checked against the oracle on pixel samples, and against the
plain KD traversal (RT_TRAVERSAL_KD, itself pinned to the oracle by the
counting tests) on whole frames at full size, where the oracle would take
hours — every pixel's G-buffer bit for bit after many passes.  Scenes: the
Cornell box, the 50k-triangle blob, the small and 2M-triangle rooms (glass
spheres, textures), the axis-aligned room (hits on split planes) and the
glass light guide (paths of hundreds of bounces).
"""
import numpy as np
import pytest

import hazards
import helpers
import oracle
import rt

pytestmark = pytest.mark.gpu
W_BOUNDED, W_KD = rt.TRAVERSAL_BOUNDED, rt.TRAVERSAL_KD


def _both(run, W, H, passes, **kw):
    a, _, _ = run.render(W, H, passes, kernel=rt.KERNEL_WAVEFRONT, traversal=W_BOUNDED, **kw)
    b, _, _ = run.render(W, H, passes, kernel=rt.KERNEL_WAVEFRONT, traversal=W_KD, **kw)
    return a, b


@pytest.mark.parametrize("name,W,H,P,calls", [("cornell", 256, 256, 8, 2), ("cornell_blob", 640, 360, 8, 2),
                                              ("room_small", 640, 360, 8, 2), ("room2m", 1920, 1080, 16, 1)])
def test_bounded_equals_kd_full_frame(name, W, H, P, calls):
    run = helpers.GpuRun(name)
    a, b = _both(run, W, H, [P] * calls)
    helpers.assert_bitwise(a, b, what=f"{name} bounded vs kd")
    assert int(a[2].sum()) == W * H * P * calls


def test_bounded_equals_kd_adaptive():
    run = helpers.GpuRun("room_small")
    a, b = _both(run, 480, 270, [12, 12], adaptive=True, min_samples=8)
    helpers.assert_bitwise(a, b, what="adaptive bounded vs kd")


@pytest.mark.parametrize("name,W,H,P,stride", [("cornell", 64, 64, 4, 1), ("cornell_blob", 320, 180, 4, 61),
                                               ("room2m", 480, 270, 4, 127)])
def test_bounded_vs_oracle(name, W, H, P, stride):
    run = helpers.GpuRun(name)
    gpu, _, _ = run.render(W, H, P, kernel=rt.KERNEL_WAVEFRONT, traversal=W_BOUNDED)
    pixels = np.arange(0, W * H, stride)
    ref, _ = helpers.oracle_render(run.path, W, H, P, pixels=pixels)
    helpers.assert_bitwise(gpu, ref, pixels=pixels, what=f"{name} bounded vs oracle")


def test_bounded_hazard_scenes(tmp_path):
    """axis-aligned room (hits on leaf exits, origins on splits), the camera on
    the root split, axis-parallel camera rays, zero-area triangles, and the
    glass light guide — every pixel against the oracle"""
    cases = []
    aligned = hazards.cornell_variant(str(tmp_path / "a"), "aligned", yaw_room=0.0)
    cases.append((aligned, None, oracle.mt19937(40 * 32)))
    osc = oracle.OracleScene(helpers.scene_path("cornell"))
    on, _ = hazards.h5_cameras(osc)
    cases.append((helpers.scene_path("cornell"), on, oracle.mt19937(40 * 32)))
    axis = hazards.cornell_variant(str(tmp_path / "x"), "aligned", yaw_room=0.0, camera=hazards.AXIS_CAMERA)
    cases.append((axis, None, hazards.h7_axis_seeds(40, 32)))
    degen = hazards.cornell_variant(str(tmp_path / "d"), "degenerate", yaw_room=0.1, extra_obj=hazards.DEGENERATE_OBJ)
    cases.append((degen, None, oracle.mt19937(40 * 32)))
    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    cases.append((trap, None, oracle.mt19937(40 * 32)))
    W, H, P = 40, 32, 3
    n = W * H
    for path, cam_arr, rng0 in cases:
        run = helpers.GpuRun(path)
        sc = oracle.OracleScene(path)
        cam_arr = sc.camera if cam_arr is None else cam_arr
        cam = rt.Camera()
        cam.position.x, cam.position.y, cam.position.z = (float(v) for v in cam_arr[:3])
        cam.yaw, cam.pitch, cam.FOV, cam.aperture_radius = (float(v) for v in cam_arr[3:7])
        g = rt.GBuffer(W, H)
        g.upload(np.zeros((n, 3), np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32), rng0)
        rt.render(run.dev, g, cam, 0, rt.options(W, H, P, adaptive=False, kernel=rt.KERNEL_WAVEFRONT,
                                                 traversal=W_BOUNDED))
        fb = np.zeros(n * 3, np.float32)
        sq = np.zeros(n, np.float32)
        ct = np.zeros(n, np.int32)
        rng = rng0.copy()
        sc.render(np.asarray(cam_arr, np.float32), fb, sq, ct, rng, W, H, P, sample_count_arg=0, adaptive=False)
        helpers.assert_bitwise(g.download(), (fb.reshape(n, 3), sq, ct, rng), what=path)


@pytest.mark.parametrize("variant", ["far", "tiny", "near"])
def test_bounded_equals_kd_adversarial_full_frame(tmp_path, variant):
    """slivers (a vertex 1e-7..1e-2 of the edge off the
    opposite edge), needles, thin fans and a cloud of tiny triangles in glass,
    gold and diffuse materials — at the origin, translated to |x| ~ 10^4, and
    shrunk to sub-millimetre triangles 100 units from the origin
    (hazards.adversarial_scene).  Whole frames, the bounded traversal (the
    product path, with its run-time guard on every 16th ray) against the KD
    traversal, bit for bit; the guard sees no mismatch; pixel samples
    against the oracle."""
    path = hazards.adversarial_scene(str(tmp_path / variant), variant)
    run = helpers.GpuRun(path)
    W, H = 320, 240
    rt.deviation_stats(reset=True)
    a, _, _ = run.render(W, H, [4, 4], kernel=rt.KERNEL_WAVEFRONT, traversal=W_BOUNDED, check_interval=16)
    dev = rt.deviation_stats(reset=True)
    b, _, _ = run.render(W, H, [4, 4], kernel=rt.KERNEL_WAVEFRONT, traversal=W_KD)
    helpers.assert_bitwise(a, b, what=f"adversarial {variant}: bounded vs kd")
    assert dev["bounded_checked"] > 10_000 and dev["bounded_mismatches"] == 0, dev
    pixels = np.arange(0, W * H, 97)
    ref, _ = helpers.oracle_render(path, W, H, [4, 4], pixels=pixels)
    helpers.assert_bitwise(a, ref, pixels=pixels, what=f"adversarial {variant}: bounded vs oracle")
