"""The oracle's whole render path against a second, independent restatement
(tests/independent_path.py: camera/pinhole ray, adaptive test, trace_path
bookkeeping, trace_ray traversal, leaf tests, texel index — numpy float32,
written from the reference source without the oracle): fb, sq, count and
the final RNG state bit for bit on small frames of the Cornell box, a
textured room, an axis-aligned room whose walls lie on KD split planes
 and the camera on the root split (H5), adaptive sampling off and
on.  The GPU path is bit-identical to the oracle (tests/test_gpu_*.py), so a
misreading shared by the oracle and the kernels would have to be made a third
time, the same way, to pass here."""
import ctypes
import os

import numpy as np
import pytest

import hazards
import helpers
import independent_path as ip
import oracle
import rt


def _run_both(path, W, H, P, adaptive=False, min_samples=100, camera=None, textures=None):
    host = rt.HostScene(path)
    tri_bytes, ntri = host.triangles_bytes()
    sc = ip.Scene(tri_bytes, textures=textures(host) if textures else None)
    cam = np.asarray(camera if camera is not None else host.camera.as_list(), np.float32)
    n = W * H
    seeds = ip.reference_seeds(n)
    np.testing.assert_array_equal(seeds, oracle.mt19937(n))  # numpy's MT19937 == the oracle's == std::mt19937
    fb, sq, cnt, rng = np.zeros((n, 3), np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32), seeds.copy()
    ip.render(sc, cam, W, H, P, fb, sq, cnt, rng, adaptive=adaptive, min_samples=min_samples)
    ref, rcnt = helpers.oracle_render(path, W, H, P, adaptive=adaptive, min_samples=min_samples, camera=cam)
    helpers.assert_bitwise((fb, sq, cnt, rng), ref, what="independent restatement")
    return cnt, rcnt


@pytest.mark.parametrize("adaptive", [False, True], ids=["adaptive-off", "adaptive-on"])
def test_cornell_matches_oracle(adaptive):
    cnt, rcnt = _run_both(helpers.scene_path("cornell"), 8, 8, 4, adaptive=adaptive, min_samples=2)
    assert rcnt["hit"] > 0 and rcnt["nee"] > 0
    if adaptive:
        assert rcnt["skip"] > 0  # the adaptive test really skipped pixel-passes


def test_textured_room_matches_oracle(tmp_path):
    """sample_texture's index (H10): wrapping UVs, mod(uv, 1) == 1.0, a
    textured emitter, a missing texture; texels read from the loader's host
    buffers (the oracle gets the same texels through its registry)."""
    scene, files = helpers.make_textured_scene(str(tmp_path))
    for rel in files:
        oracle.register_texture(rel, rt.decode_image(os.path.join(str(tmp_path), rel)))

    def textures(host):
        out = {}
        tb, n = host.triangles_bytes()
        raw = np.frombuffer(tb, np.uint8).reshape(n, 152)
        for i in range(n):
            key = int.from_bytes(raw[i, 136:144].tobytes(), "little")
            w, h = np.frombuffer(raw[i, 144:152].tobytes(), np.int32)
            if key and key not in out:
                out[key] = np.frombuffer(ctypes.string_at(key, int(w) * int(h) * 4), np.uint8).reshape(h, w, 4)
        return out

    _, rcnt = _run_both(scene, 8, 8, 3, textures=textures)
    assert rcnt["texel"] > 0


def test_axis_aligned_room_and_camera_on_split_match_oracle(tmp_path):
    """H6 (hits on a leaf exit, deferred) and H5 (every camera ray starts on
    the root split plane, aperture 0)."""
    path = hazards.cornell_variant(str(tmp_path), "aligned", yaw_room=0.0)
    dev = {}
    _run_both(path, 8, 8, 3)
    helpers.oracle_render(path, 8, 8, 3, deviations=dev)
    assert dev["hazards"]["exit_tie"] > 0
    osc = oracle.OracleScene(helpers.scene_path("cornell"))
    on, _ = hazards.h5_cameras(osc)
    _run_both(helpers.scene_path("cornell"), 8, 8, 2, camera=on)


def test_glass_light_guide_matches_oracle(tmp_path):
    """Transmission (inside_medium toggles), specular reflection inside the
    medium with weight 1 (rt/path_tracing.cuh:194-197) and the
    long total-internal-reflection paths it makes: the light guide of
    helpers.make_trap_scene."""
    path = helpers.make_trap_scene(str(tmp_path), 60.0)
    _, rcnt = _run_both(path, 6, 6, 2)
    assert rcnt["maxdepth"] >= 64
