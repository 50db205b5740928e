"""CPU checks of the BVH-bounded traversal (csrc/bvh_trace.h; host side
csrc/host/bvh_build.*):

* tests/native/bvh_margin_check.cpp — the conservative margins never cull a
  passing triangle test (adversarial triangles and rays), and triangles left
  out of the BVH never pass;
* tests/native/bvh_trace_check.cpp — a host restatement of the bounded
  traversal over the library's own prepared arrays returns the plain KD
  traversal's (= trace_ray's) result bit for bit on millions of camera and
  bounce rays, including the hazard scenes (walls on split planes, the camera
  on the root split, axis-parallel and grazing rays, zero-area triangles, the
  glass light guide).

The GPU kernel itself is compared with the oracle and the KD traversal in
tests/test_gpu_traversal.py.
"""
import os
import subprocess

import numpy as np
import pytest

import hazards
import helpers
import oracle
import rt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
CSRC = os.path.join(ROOT, "isaklm-raytracer_amd", "csrc")
INC = os.path.join(ROOT, "include")
FLAGS = ["-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-I" + INC, "-I" + CSRC]


def _build(tmp_path_factory, name, link_lib):
    out = str(tmp_path_factory.mktemp("bvh") / name)
    cmd = ["g++"] + FLAGS + [os.path.join(NATIVE, name + ".cpp"), "-o", out]
    if link_lib:
        libdir = os.path.dirname(rt.LIB_PATH)
        cmd += ["-fopenmp", "-L" + libdir, "-lisaklm_rt", "-Wl,-rpath," + libdir, "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


@pytest.fixture(scope="module")
def margin_check(tmp_path_factory):
    return _build(tmp_path_factory, "bvh_margin_check", False)


@pytest.fixture(scope="module")
def trace_check(tmp_path_factory):
    rt.lib()  # the library must exist (and match the header)
    return _build(tmp_path_factory, "bvh_trace_check", True)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_margins_never_cull_a_passing_test(margin_check, seed):
    r = subprocess.run([margin_check, "3", str(seed)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    stats = dict(zip(r.stdout.split()[::2], r.stdout.split()[1::2]))
    assert int(stats["passes"]) > 1_000_000 and int(stats["violations"]) == 0 and int(stats["nan_passes"]) == 0
    # the margins are generous: a hit point never used more than a small part of them
    assert float(stats["max_used"]) < 0.05, stats
    # the written-out bound (bvh_build.h tri_margin_bound): every exact hit point lies within it, and
    # the shipped margins are at least it for every finite-margin triangle and any origin
    assert int(stats["bound_fails"]) == 0 and int(stats["margin_short"]) == 0 and int(stats["bound_inf"]) == 0, stats
    assert float(stats["min_ratio"]) >= 1.0, stats


def _run_trace_check(exe, scene, rays=1_000_000, seed=7, cam=None, env=None):
    args = [exe, scene, str(rays), str(seed)] + ([" ".join(float(v).hex() for v in cam)] if cam is not None else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="4", **(env or {})))
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("name", ["cornell", "cornell_blob", "room_small"])
def test_bounded_equals_kd_host(trace_check, name):
    out = _run_trace_check(trace_check, helpers.scene_path(name))
    assert "mismatches 0" in out, out
    # the unique-minimum shortcut of the KD phase (bvh_trace.h kd_bounded's T* leaf) is taken
    assert int(out.split("T* leaves: ")[1].split()[0]) > 100_000, out
    # every triangle of the scene: shipped margin >= the proven bound
    assert "shipped below the proven bound 0, unproven 0" in out, out


def test_bounded_equals_kd_hazard_scenes(trace_check, tmp_path):
    aligned = hazards.cornell_variant(str(tmp_path / "a"), "aligned", yaw_room=0.0)
    assert "mismatches 0" in _run_trace_check(trace_check, aligned, 500_000)
    degen = hazards.cornell_variant(str(tmp_path / "d"), "degenerate", yaw_room=0.1, extra_obj=hazards.DEGENERATE_OBJ)
    out = _run_trace_check(trace_check, degen, 500_000)
    assert "mismatches 0" in out and "dropped 0" not in out, out  # the zero-area triangles are left out
    # two identical copies of a quad: ties at s_min (the T* shortcut steps aside), identical results
    dup = hazards.cornell_variant(str(tmp_path / "u"), "duplicate", yaw_room=0.1, extra_obj=hazards.DUPLICATE_OBJ)
    out = _run_trace_check(trace_check, dup, 500_000)
    assert "mismatches 0" in out and int(out.split("two tests share: ")[1].split()[0]) > 1000, out
    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    assert "mismatches 0" in _run_trace_check(trace_check, trap, 500_000)
    # camera rays from exactly the root split plane
    path = helpers.scene_path("cornell")
    on, _ = hazards.h5_cameras(oracle.OracleScene(path))
    assert "mismatches 0" in _run_trace_check(trace_check, path, 500_000, cam=on[:3])


def test_origin_cell_entry_host(trace_check, tmp_path):
    """wf_long's deep bounces enter the KD traversal at the grid cell holding
    the ray's origin (coop_trace.h kd_origin_frontier): the replayed root path,
    checked decision by decision, gives the plain traversal's result."""
    for path in (helpers.scene_path("cornell_blob"), helpers.make_trap_scene(str(tmp_path / "t"))):
        out = _run_trace_check(trace_check, path, 300_000, seed=11)
        assert "rays 300000" in out and " mismatches 0\n" in out, out
        line = out.split("origin-cell entry: ")[1]
        assert int(line.split(" resumed")[0]) > 0 and line.split("traversal ")[1].startswith("0"), out


@pytest.mark.parametrize("variant", ["far", "tiny", "near"])
def test_bounded_equals_kd_adversarial_host(trace_check, tmp_path, variant):
    """Slivers, needles, thin fans and a cloud of tiny triangles, at the origin,
    translated to |x| ~ 10^4, and scaled to sub-millimetre triangles 100 units
    away (hazards.adversarial_scene): the bounded traversal equals the KD
    traversal on every ray, and every triangle's margin is at least the proven
    bound."""
    path = hazards.adversarial_scene(str(tmp_path / variant), variant)
    out = _run_trace_check(trace_check, path, 1_000_000, seed=3)
    assert "rays 1000000" in out and " mismatches 0\n" in out, out
    assert "shipped below the proven bound 0, unproven 0" in out, out


# A camera ray of the adversarial "near" scene on which the bounded traversal
# once returned the wrong triangle: always-tested slivers (no usable margin)
# pass the reference's test at s = 0.71 and 1.91, before the ray enters the
# scene box (2.62), and a scene-sized box let the query cull them — s_min then
# was no lower bound, and the T* leaf returned triangle 107 where the
# reference returns 44.  (Found by the run-time guard on the GPU,
# tools/mismatch_ray.py.)
NEAR_RAY = "-0x1.62103ap-2 0x1.000406p+0 -0x1.caacf8p+1 0x1.64d0bp-7 -0x1.01092ap-2 0x1.ef9396p-1"


def test_bounded_equals_kd_real_rays_near_host(trace_check, tmp_path):
    """The oracle's own rays (camera, bounce and shadow rays of a 160x120
    frame, oracle or_log_rays) of the adversarial near scene, and the ray
    above, through the host restatement: bounded == plain KD on every one."""
    import ctypes

    path = hazards.adversarial_scene(str(tmp_path / "near"), "near")
    r = subprocess.run([trace_check, path, "ray", NEAR_RAY], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and " kd 44 bounded 44\n" in r.stdout, r.stdout[-2000:]
    lib = oracle.lib()
    lib.or_log_rays.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] * 2 + [ctypes.c_void_p, ctypes.c_int,
                                                                            ctypes.c_void_p, ctypes.c_int]
    osc = oracle.OracleScene(path)
    W, H = 160, 120
    pix = np.arange(W * H, dtype=np.int32)
    rays = np.zeros((len(pix) * 200, 6), np.float32)
    n = lib.or_log_rays(osc.h, osc.camera.ctypes.data, W, H, pix.ctypes.data, len(pix), rays.ctypes.data,
                        len(rays))
    f = str(tmp_path / "rays.f32")
    rays[:n].tofile(f)
    r = subprocess.run([trace_check, path, "file", f], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert r.returncode == 0 and f"rays {n} mismatches 0;" in r.stdout and n > 30_000, r.stdout
