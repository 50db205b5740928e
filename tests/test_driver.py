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
