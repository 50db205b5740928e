"""CPU checks of the hazard inputs (tests/hazards.py) the GPU hazard tests
use: the RNG inversion reproduces the reference's generator, and each built
input triggers its quirk in the oracle."""
import random

import numpy as np

import hazards
import helpers
import oracle


def test_rng_inverse_matches_the_generator():
    """rng_step is get_random_unilateral's state update (rt/path_tracing.cuh:
    34-43, via the oracle), rng_step_inv its inverse, rng_back(word, k) the seed
    whose draw k returns word"""
    r = random.Random(7)
    for _ in range(2000):
        x = r.getrandbits(32)
        assert hazards.rng_step_inv(hazards.rng_step(x)) == x
    seed = 123456789
    vals, _ = oracle.rng_sequence(seed, 12)
    x = seed
    for v in vals:
        x = hazards.rng_step(x)
        assert hazards.unilateral(x) == v
    for k in (0, 1, 9):
        vals, _ = oracle.rng_sequence(hazards.rng_back((1 << 32) - 1, k), k + 1)
        assert vals[k] == np.float32(1.0)
    assert hazards.unilateral((1 << 32) - 128) == np.float32(1.0)
    assert hazards.unilateral((1 << 32) - 129) < np.float32(1.0)


def test_h4_seeds_trigger_xi_one():
    osc = oracle.OracleScene(helpers.scene_path("cornell"))
    rng0, planted = hazards.h4_seeds(osc, 16, 16)
    assert planted >= 30
    dev = {}
    n = 256
    fb, sq, ct = np.zeros(n * 3, np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32)
    k = osc.render(osc.camera, fb, sq, ct, rng0.copy(), 16, 16, 1, sample_count_arg=0, adaptive=False)
    assert k["hazards"]["xi_one"] >= planted
    del dev


def test_h5_camera_on_split_changes_the_image():
    osc = oracle.OracleScene(helpers.scene_path("cornell"))
    on, off = hazards.h5_cameras(osc)
    dev = {}
    a, _ = helpers.oracle_render(None, 40, 32, 2, scene=osc, camera=on, deviations=dev)
    b, _ = helpers.oracle_render(None, 40, 32, 2, scene=osc, camera=off)
    assert dev["hazards"]["on_split"] >= 40 * 32 * 2
    assert np.count_nonzero(np.any(a[0] != b[0], axis=1)) > 40 * 32 // 10


def test_h6_h7_inputs_trigger(tmp_path):
    p = hazards.cornell_variant(str(tmp_path / "a"), "aligned", yaw_room=0.0)
    dev = {}
    helpers.oracle_render(p, 40, 32, 3, deviations=dev)
    assert dev["hazards"]["exit_tie"] > 100
    p = hazards.cornell_variant(str(tmp_path / "b"), "aligned", yaw_room=0.0, camera=hazards.AXIS_CAMERA)
    osc = oracle.OracleScene(p)
    base, mod = {}, {}
    for seeds, dev in ((oracle.mt19937(32 * 24), base), (hazards.h7_axis_seeds(32, 24), mod)):
        n = 32 * 24
        fb, sq, ct = np.zeros(n * 3, np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32)
        dev.update(osc.render(osc.camera, fb, sq, ct, seeds, 32, 24, 2, sample_count_arg=0, adaptive=False))
    assert mod["hazards"]["axis_parallel"] > base["hazards"]["axis_parallel"] + 24
    p = hazards.cornell_variant(str(tmp_path / "c"), "degenerate", yaw_room=0.1, extra_obj=hazards.DEGENERATE_OBJ)
    dev = {}
    helpers.oracle_render(p, 40, 32, 3, deviations=dev)
    assert dev["hazards"]["degenerate"] > 1000


def test_trap_scene_makes_deep_paths(tmp_path):
    """the light guide (helpers.make_trap_scene) gives paths past depth 64 and
    past 512 (SURVEY H8 tail), none cut"""
    p = helpers.make_trap_scene(str(tmp_path), 600.0)
    dev = {}
    _, cnt = helpers.oracle_render(p, 32, 24, 2, deviations=dev)
    assert sum(dev["deep_hist"]) > 100 and sum(dev["deep_hist"][3:]) > 0, dev
    assert dev["cut"] == 0 and cnt["watchdog"] == 0
    assert cnt["maxdepth"] >= 512
