"""GPU tests built to trigger each numerical hazard of the reference (SURVEY
Appendix A) and compared bit for bit (fb, sq, count, RNG state) and counter
for counter with the oracle, on both kernels.  The oracle's hazard
instrumentation (oracle.HAZARDS) shows each input really triggers its quirk.

  H4  xi == 1.0 in the NEE light pick reads light_indicies[light_count]
      (rt/path_tracing.cuh:237): both sides read a padded entry (= the last
      light); seeds planted by inverting the RNG (tests/hazards.py)
  H5  ray origin exactly on a split plane (rt/trace_ray.cuh:278-295): the
      camera on the root split, aperture 0
  H6  a hit exactly at a leaf's exit is deferred to the next leaf
      (rt/trace_ray.cuh:121,133,310-313): axis-aligned walls on split planes
  H7  axis-parallel rays (+-inf / NaN split distances, rt/trace_ray.cuh:
      190-242; the plain-division fallback of rt_div_by) and zero-area
      triangles (normalize(0) = NaN, :75)
"""
import numpy as np
import pytest

import hazards
import helpers
import oracle
import rt

pytestmark = pytest.mark.gpu
KERNELS = [pytest.param(rt.KERNEL_MEGA, id="mega"), pytest.param(rt.KERNEL_WAVEFRONT, id="wavefront")]


def _camera(run, arr):
    c = rt.Camera()
    c.position.x, c.position.y, c.position.z = float(arr[0]), float(arr[1]), float(arr[2])
    c.yaw, c.pitch, c.FOV, c.aperture_radius = float(arr[3]), float(arr[4]), float(arr[5]), float(arr[6])
    return c


def _gpu(run, W, H, P, rng0, cam_arr, kernel, calls, cnt, traversal=None):
    n = W * H
    g = rt.GBuffer(W, H)
    g.upload(np.zeros((n, 3), np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32), rng0)
    cam = _camera(run, cam_arr)
    for c in range(calls):
        rt.render(run.dev, g, cam, 0 if c == 0 else 1,
                  rt.options(W, H, P, adaptive=False, counters=cnt.p if cnt else None, kernel=kernel,
                             traversal=traversal))
    return g.download()


def _render_both(run, osc, W, H, P, rng0, cam_arr, kernel, calls=1):
    """GPU render with the G-buffer seeds rng0 and camera cam_arr against the
    oracle on the same inputs, three ways: the counting build (KD traversal,
    counters compared too) and the product build with each traversal
    (RT_TRAVERSAL_BOUNDED: the BVH-bounded one on the wavefront kernel);
    returns the oracle's hazard counts"""
    n = W * H
    cnt = rt.DeviceCounters()
    gpu = _gpu(run, W, H, P, rng0, cam_arr, kernel, calls, cnt)
    products = [(t, _gpu(run, W, H, P, rng0, cam_arr, kernel, calls, None, traversal=t))
                for t in (rt.TRAVERSAL_BOUNDED, rt.TRAVERSAL_KD)]
    fb = np.zeros(n * 3, np.float32)
    sq = np.zeros(n, np.float32)
    ct = np.zeros(n, np.int32)
    rng = rng0.copy()
    total, haz = {}, {}
    for c in range(calls):
        k = osc.render(np.asarray(cam_arr, np.float32), fb, sq, ct, rng, W, H, P, sample_count_arg=0 if c == 0 else 1,
                       adaptive=False)
        for key, v in k.pop("hazards").items():
            haz[key] = haz.get(key, 0) + v
        k.pop("cut"), k.pop("deep_hist")
        for key, v in k.items():
            total[key] = max(total.get(key, 0), v) if key == "maxdepth" else total.get(key, 0) + v
    helpers.assert_bitwise(gpu, (fb.reshape(n, 3), sq, ct, rng))
    assert cnt.read() == total, (cnt.read(), total)
    for t, out in products:
        helpers.assert_bitwise(out, (fb.reshape(n, 3), sq, ct, rng), what=f"traversal {t}")
    return haz


@pytest.mark.parametrize("kernel", KERNELS)
def test_h4_light_pick_xi_one(kernel):
    """Seeds planted so that the NEE light-pick draw (draw 9 of a pass whose
    first bounce is diffuse: 2 jitter + 2 pinhole + 2 microfacet + Fresnel +
    2 diffuse) returns a word >= 2^32 - 128, i.e. xi == 1.0f exactly."""
    run = helpers.GpuRun("cornell")
    osc = oracle.OracleScene(run.path)
    W, H = 16, 16
    rng0, planted = hazards.h4_seeds(osc, W, H)
    assert planted >= 30, planted
    haz = _render_both(run, osc, W, H, 3, rng0, osc.camera, kernel)
    assert haz["xi_one"] >= planted, haz


@pytest.mark.parametrize("kernel", KERNELS)
def test_h5_camera_on_root_split(kernel):
    """Every primary ray starts exactly on the root split plane (camera
    coordinate = split, aperture 0): near = child2 by origin >= split, t = 0
    <= entry sends it to the far child — the reference's missing-wall image
    (SURVEY H5).  The render must differ from a camera one ulp off the plane
    (the quirk is visible) and match the oracle bit for bit."""
    run = helpers.GpuRun("cornell")
    osc = oracle.OracleScene(run.path)
    on, off = hazards.h5_cameras(osc)
    W, H, P = 40, 32, 2
    haz = _render_both(run, osc, W, H, P, oracle.mt19937(W * H), on, kernel)
    assert haz["on_split"] >= W * H * P, haz
    a, _ = helpers.oracle_render(run.path, W, H, P, scene=osc, camera=on)
    b, _ = helpers.oracle_render(run.path, W, H, P, scene=osc, camera=off)
    differ = np.count_nonzero(np.any(a[0] != b[0], axis=1))
    assert differ > W * H // 10, differ


@pytest.mark.parametrize("kernel", KERNELS)
def test_h6_hits_on_leaf_exits(kernel, tmp_path):
    """Axis-aligned room (no 0.1 rad rotation): walls lie on KD split planes,
    so hits at t == the leaf's exit (strict t < smallest_t, smallest_t =
    exit) are deferred to the next leaf — many per frame."""
    path = hazards.cornell_variant(str(tmp_path), "aligned", yaw_room=0.0)
    run = helpers.GpuRun(path)
    osc = oracle.OracleScene(path)
    W, H, P = 40, 32, 3
    haz = _render_both(run, osc, W, H, P, oracle.mt19937(W * H), osc.camera, kernel)
    assert haz["exit_tie"] > 100 and haz["on_split"] > 0, haz


@pytest.mark.parametrize("kernel", KERNELS)
def test_h7_axis_parallel_camera_rays(kernel, tmp_path):
    """Axis-aligned camera (yaw 0, pitch 0, aperture 0) in the axis-aligned
    room; pixel column x = W/2 - 1 gets seeds whose first draw (x jitter) is
    1.0f and row y = H/2 - 1 seeds whose second draw (y jitter) is 1.0f, so
    their camera rays have direction.x (.y) == 0 exactly — +-inf slab and
    split distances, NaN at origin == split, and rt_div_by's plain-division
    fallback."""
    path = hazards.cornell_variant(str(tmp_path), "aligned", yaw_room=0.0, camera=hazards.AXIS_CAMERA)
    run = helpers.GpuRun(path)
    osc = oracle.OracleScene(path)
    W, H, P = 32, 24, 2
    base = _render_both(run, osc, W, H, P, oracle.mt19937(W * H), osc.camera, kernel)
    haz = _render_both(run, osc, W, H, P, hazards.h7_axis_seeds(W, H), osc.camera, kernel)
    assert haz["axis_parallel"] > base["axis_parallel"] + H, (base, haz)


@pytest.mark.parametrize("kernel", KERNELS)
def test_h7_degenerate_triangles(kernel, tmp_path):
    """Zero-area triangles in the middle of the room (hazards.DEGENERATE_OBJ):
    normalize(cross(...)) = NaN, so every test of them fails (NaN
    comparisons), as in the reference — tested thousands of times."""
    path = hazards.cornell_variant(str(tmp_path), "degenerate", yaw_room=0.1, extra_obj=hazards.DEGENERATE_OBJ)
    run = helpers.GpuRun(path)
    osc = oracle.OracleScene(path)
    W, H, P = 40, 32, 3
    haz = _render_both(run, osc, W, H, P, oracle.mt19937(W * H), osc.camera, kernel)
    assert haz["degenerate"] > 1000, haz


@pytest.mark.parametrize("kernel", KERNELS)
def test_duplicate_triangles_tie(kernel, tmp_path):
    """Two identical copies of a quad (hazards.DUPLICATE_OBJ, red then green):
    their tests tie at exactly the same s on every hit, the reference keeps the
    copy listed first in the leaf — the BVH query sees the tie and the KD phase
    scans the leaf in full instead of taking the unique-minimum shortcut."""
    path = hazards.cornell_variant(str(tmp_path), "duplicate", yaw_room=0.1, extra_obj=hazards.DUPLICATE_OBJ)
    run = helpers.GpuRun(path)
    osc = oracle.OracleScene(path)
    W, H, P = 40, 32, 3
    _render_both(run, osc, W, H, P, oracle.mt19937(W * H), osc.camera, kernel)
