"""The C++ driver (isaklm-raytracer_amd/apps/rt_render_main.cpp): the
reference's main() (rt/main.cu:60-155) without the GLFW window, over the
C-ABI only.  CPU: it is built and rejects bad usage.  GPU: its saved PNG
(save_render: tonemap, vertical flip) equals the oracle's tonemapped frame."""
import os
import subprocess

import numpy as np
import pytest

import helpers
import oracle
import rt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "isaklm-raytracer_amd", "rt_render")


def test_driver_built_and_usage():
    assert os.access(APP, os.X_OK), "run __graft_entry__.build()"
    r = subprocess.run([APP, "--bogus"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage: rt_render" in r.stderr


@pytest.mark.gpu
@pytest.mark.timeout(180)
@pytest.mark.parametrize("kernel", ["wavefront", "mega"])
def test_driver_png_matches_oracle(tmp_path, kernel):
    W, H, SPP, P = 64, 48, 10, 4  # 3 render() calls of 4 + 4 + 2 passes
    scene = helpers.scene_path("cornell")
    out = tmp_path / "render.png"
    r = subprocess.run([APP, "--scene", scene, "--width", str(W), "--height", str(H), "--spp", str(SPP), "--passes",
                        str(P), "--adaptive", "0", "--kernel", kernel, "--out", str(out), "--quiet"],
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout + r.stderr
    png = rt.decode_image(str(out))
    # oracle: the same calls (render() keeps its state across calls), then the tonemap
    osc = oracle.OracleScene(scene)
    n = W * H
    fb, sq, cnt = np.zeros(n * 3, np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32)
    seeds = oracle.mt19937(n)
    done = 0
    while done < SPP:
        k = min(P, SPP - done)
        osc.render(osc.camera, fb, sq, cnt, seeds, W, H, k, sample_count_arg=done, adaptive=False)
        done += k
    rgba = oracle.tonemap(fb, cnt).reshape(H, W, 4)[::-1]  # save_render flips (rt/save_render.cuh:55)
    assert np.all(cnt == SPP)
    np.testing.assert_array_equal(png, rgba)


@pytest.mark.gpu
@pytest.mark.timeout(180)
def test_driver_checkpoint_resume(tmp_path):
    """--checkpoint after 6 of 10 spp, then --resume to 10: the PNG equals a
    straight 10-spp run bit for bit (adaptive sampling on, so the resumed
    count/sq planes matter)."""
    W, H = 64, 48
    scene = helpers.scene_path("cornell")
    base = [APP, "--scene", scene, "--width", str(W), "--height", str(H), "--passes", "3", "--min-samples", "4",
            "--quiet"]
    straight, resumed, ck = tmp_path / "straight.png", tmp_path / "resumed.png", tmp_path / "g.ckpt"
    for args in (["--spp", "10", "--out", str(straight)],
                 ["--spp", "6", "--checkpoint", str(ck), "--out", str(tmp_path / "half.png")],
                 ["--spp", "10", "--resume", str(ck), "--out", str(resumed)]):
        r = subprocess.run(base + args, capture_output=True, text=True, timeout=150)
        assert r.returncode == 0, r.stdout + r.stderr
    assert ck.stat().st_size == 8 + 16 + W * H * 24 and not os.path.exists(str(ck) + ".tmp")
    np.testing.assert_array_equal(rt.decode_image(str(resumed)), rt.decode_image(str(straight)))
    assert not np.array_equal(rt.decode_image(str(tmp_path / "half.png")), rt.decode_image(str(straight)))


@pytest.mark.gpu
@pytest.mark.timeout(180)
def test_reference_shaped_main_renders_like_the_oracle(tmp_path):
    """The reference-main-shaped program (tests/native/ref_main_shape.cpp: the
    caller's own reference types, cudaMalloc/cudaMemcpy -> rt_device_alloc /
    rt_upload, G_Buffer(), create_scene(), rt_scene_prepare on the Scene
    alone, the pass loop over rt_render, save_render) writes the oracle's
    tonemapped frame bit for bit."""
    import test_abi

    exe = test_abi.build_main_shape(tmp_path)
    W, H, SPP, P = 48, 40, 7, 3
    scene = helpers.scene_path("cornell")
    out = tmp_path / "main_shape.png"
    r = subprocess.run([exe, scene, str(W), str(H), str(SPP), str(P), str(out)], capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
    osc = oracle.OracleScene(scene)
    n = W * H
    fb, sq, cnt = np.zeros(n * 3, np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32)
    seeds = oracle.mt19937(n)
    done = 0
    while done < SPP:
        k = min(P, SPP - done)
        osc.render(osc.camera, fb, sq, cnt, seeds, W, H, k, sample_count_arg=done, adaptive=False)
        done += k
    np.testing.assert_array_equal(rt.decode_image(str(out)), oracle.tonemap(fb, cnt).reshape(H, W, 4)[::-1])
