"""BASELINE.json configs at their stated sizes, and the always-on deviation
statistics (the reference's bounce loop is unbounded,
rt/path_tracing.cuh:279-319).  Every image check is bit-for-bit against the
oracle (fb, sq, count, final RNG state); large frames are checked on sparse
pixel subsets (pixels are independent).
"""
import numpy as np
import pytest

import helpers
import rt

pytestmark = pytest.mark.gpu
KERNELS = [pytest.param(rt.KERNEL_MEGA, id="mega"), pytest.param(rt.KERNEL_WAVEFRONT, id="wavefront")]
BENCH_CALL = 256  # bench.py: steps of 64 passes rendered 4 per rt_render call


def _stats_reset():
    rt.deviation_stats(reset=True)


# ------------------------------------------------------------ deviations (H8)
@pytest.mark.timeout(300)
@pytest.mark.parametrize("kernel", KERNELS)
def test_deviation_stats_deep_paths(kernel, tmp_path):
    """A light guide (helpers.make_trap_scene): thousands of paths run past
    depth 64 and some past 512 (total internal reflection, specular weight 1
    inside glass).  The always-on statistics of the NON-counting kernels (the
    bench's) — the deep-path histogram and the longest path — equal the
    oracle's, and no path is cut.  The wavefront run hands every path deeper
    than 64 bounces to wf_long, so the hand-off carries most of the work."""
    path = helpers.make_trap_scene(str(tmp_path), 600.0)
    run = helpers.GpuRun(path)
    W, H, P = 64, 48, 4
    _stats_reset()
    gpu, _, _ = run.render(W, H, P, calls=2, kernel=kernel)
    st = rt.deviation_stats(reset=True)
    dev = {}
    ref, rcnt = helpers.oracle_render(path, W, H, P, calls=2, deviations=dev)
    helpers.assert_bitwise(gpu, ref, what="trap")
    assert st["deep_hist"] == dev["deep_hist"], (st, dev)
    assert st["max_deep_depth"] == rcnt["maxdepth"] >= 512, (st, rcnt)
    assert st["deep_paths"] > 1000 and st["cut_paths"] == 0 and st["watchdog_paths"] == 0, st


@pytest.mark.parametrize("kernel", KERNELS)
def test_deviation_stats_depth_cut(kernel):
    """RtOptions.max_depth cuts are counted by every kernel (counting or not)
    exactly as the oracle cuts them; they are not watchdog firings."""
    run = helpers.GpuRun("cornell")
    W, H, P = 48, 32, 4
    _stats_reset()
    gpu, _, _ = run.render(W, H, P, max_depth=3, kernel=kernel)
    st = rt.deviation_stats(reset=True)
    dev = {}
    ref, _ = helpers.oracle_render(run.path, W, H, P, max_depth=3, deviations=dev)
    helpers.assert_bitwise(gpu, ref, what="max_depth 3")
    assert st["cut_paths"] == dev["cut"] > 0 and st["watchdog_paths"] == 0, (st, dev)


# ------------------------------------------------------------ BASELINE configs
@pytest.mark.timeout(240)
@pytest.mark.parametrize("kernel", KERNELS)
def test_configs0_cornell_256_full_frame(kernel):
    """configs[0]: Cornell box, 256x256, 64 spp — every pixel bit-identical."""
    run = helpers.GpuRun("cornell")
    W, H, P = 256, 256, 64
    gpu, _, _ = run.render(W, H, P, kernel=kernel)
    ref, rcnt = helpers.oracle_render(run.path, W, H, P)
    helpers.assert_bitwise(gpu, ref, what="configs[0]")
    assert np.all(gpu[2] == P) and rcnt["watchdog"] == 0
    assert helpers.rel_linf(gpu[0], gpu[2], ref[0], ref[2]) < 1e-4


@pytest.mark.timeout(300)
def test_configs1_cornell_blob_720p_256spp():
    """configs[1]: Cornell + 50k-triangle OBJ, 1280x720, 256 spp, with the
    bench's call split (a 64-pass call that resets, then 192 passes) on the
    bench kernel; every 997th pixel re-rendered by the oracle."""
    run = helpers.GpuRun("cornell_blob")
    W, H = 1280, 720
    calls = [64, 192]
    _stats_reset()
    gpu, _, _ = run.render(W, H, calls, kernel=rt.KERNEL_WAVEFRONT)
    st = rt.deviation_stats(reset=True)
    pixels = np.arange(0, W * H, 997, dtype=np.int32)
    ref, rcnt = helpers.oracle_render(run.path, W, H, calls, pixels=pixels)
    helpers.assert_bitwise(gpu, ref, pixels=pixels, what="configs[1]")
    assert np.all(gpu[2] == sum(calls))
    assert st["watchdog_paths"] == 0 and rcnt["watchdog"] == 0, st
    assert helpers.rel_linf(gpu[0][pixels], gpu[2][pixels], ref[0][pixels], ref[2][pixels]) < 1e-4


@pytest.mark.timeout(400)
@pytest.mark.parametrize("shard", [1, 7])
def test_configs3_shard_seed_windows_room2m(shard):
    """configs[3]'s spp slices: GPU g of 8 seeds its G_Buffer with mt19937
    outputs [g*W*H, (g+1)*W*H) (rt/screen.cuh:34-45 continued).  Shards 1 and
    7 of room2m at 1920x1080, a 64-pass then a 256-pass call on the bench
    kernel; every 4099th pixel re-rendered by the oracle with the same seed
    window."""
    run = helpers.GpuRun("room2m")
    W, H = 1920, 1080
    calls = [64, BENCH_CALL]
    skip = shard * W * H
    _stats_reset()
    gpu, _, _ = run.render(W, H, calls, seed_skip=skip, kernel=rt.KERNEL_WAVEFRONT)
    st = rt.deviation_stats(reset=True)
    pixels = np.arange(0, W * H, 4099, dtype=np.int32)
    ref, rcnt = helpers.oracle_render(run.path, W, H, calls, seed_skip=skip, pixels=pixels)
    helpers.assert_bitwise(gpu, ref, pixels=pixels, what=f"configs[3] shard {shard}")
    assert np.all(gpu[2] == sum(calls))
    assert st["watchdog_paths"] == 0 and rcnt["watchdog"] == 0, st


@pytest.mark.timeout(500)
def test_room2m_headline_budget_1024spp():
    """configs[2]'s whole budget: room2m at 1920x1080, 1,024 spp in the
    bench's calls (4 x 256 passes, non-counting bench kernels), every 4099th
    pixel bit-identical to the oracle over the same 1,024 spp, and no path cut
    by the watchdog anywhere in the frame (always-on statistics over all
    2.1 G samples)."""
    run = helpers.GpuRun("room2m")
    W, H = 1920, 1080
    calls = [BENCH_CALL] * 4
    _stats_reset()
    gpu, _, _ = run.render(W, H, calls, kernel=rt.KERNEL_WAVEFRONT)
    st = rt.deviation_stats(reset=True)
    print(f"\nroom2m 1024 spp deviations: {st}")
    pixels = np.arange(0, W * H, 4099, dtype=np.int32)
    ref, rcnt = helpers.oracle_render(run.path, W, H, calls, pixels=pixels)
    helpers.assert_bitwise(gpu, ref, pixels=pixels, what="room2m 1024 spp")
    assert np.all(gpu[2] == 1024)
    assert st["watchdog_paths"] == 0 and st["cut_paths"] == 0, st
    assert st["deep_paths"] > 0 and st["max_deep_depth"] >= rcnt["maxdepth"], (st, rcnt)


# ------------------------------------------------ configs[4]: adaptive at the reference's constants
REF_MIN_SAMPLES, REF_TOLERANCE = 100, 0.05  # rt/macros.h:13,17 (the test of rt/path_tracing.cuh:352-376)


@pytest.mark.timeout(500)
@pytest.mark.parametrize("shard", [0, 7])
def test_configs4_room2m_glass_adaptive_reference_constants(shard):
    """configs[4]: the dielectric stress scene at 1920x1080 with adaptive
    sampling at the reference's own MIN_SAMPLES 100 / MAX_TOLERANCE 0.05 and
    depth 32, on the bench kernel as the bench calls it (a 64-pass call that
    resets, then a chained 192-pass call), so pixels cross 100 samples and the
    test starts stopping them.  Every 3001st pixel bit-identical to the
    oracle; shard 7's seed window is the 8-GPU configuration's (each GPU
    evaluates adaptivity on its own slice's statistics)."""
    run = helpers.GpuRun("room2m_glass")
    W, H = 1920, 1080
    calls = [64, 192]
    skip = shard * W * H
    gpu, _, _ = run.render(W, H, calls, adaptive=True, min_samples=REF_MIN_SAMPLES, tolerance=REF_TOLERANCE,
                           max_depth=32, seed_skip=skip, kernel=rt.KERNEL_WAVEFRONT, overlap=True)
    pixels = np.arange(0, W * H, 3001, dtype=np.int32)
    ref, rcnt = helpers.oracle_render(run.path, W, H, calls, adaptive=True, min_samples=REF_MIN_SAMPLES,
                                      tolerance=REF_TOLERANCE, max_depth=32, seed_skip=skip, pixels=pixels)
    helpers.assert_bitwise(gpu, ref, pixels=pixels, what=f"configs[4] seed window {shard}")
    cnt = gpu[2]
    # the adaptive test stopped pixels after their 100th sample, and only then
    assert rcnt["skip"] > 0 and cnt.min() >= REF_MIN_SAMPLES and (cnt < sum(calls)).sum() > W * H // 100, \
        (rcnt["skip"], int(cnt.min()), int((cnt < sum(calls)).sum()))


@pytest.mark.timeout(400)
def test_configs4_regime_full_frame_cut_paths():
    """The same regime (MIN_SAMPLES 100, tolerance 0.05, depth 32, 64 + 192
    chained passes) on a whole 128x72 frame: every pixel bit-identical, and
    the paths cut at depth 32 counted by the non-counting bench kernels equal
    the oracle's over the same frame."""
    run = helpers.GpuRun("room2m_glass")
    W, H = 128, 72
    calls = [64, 192]
    _stats_reset()
    gpu, _, _ = run.render(W, H, calls, adaptive=True, min_samples=REF_MIN_SAMPLES, tolerance=REF_TOLERANCE,
                           max_depth=32, kernel=rt.KERNEL_WAVEFRONT, overlap=True)
    st = rt.deviation_stats(reset=True)
    dev = {}
    ref, rcnt = helpers.oracle_render(run.path, W, H, calls, adaptive=True, min_samples=REF_MIN_SAMPLES,
                                      tolerance=REF_TOLERANCE, max_depth=32, deviations=dev)
    helpers.assert_bitwise(gpu, ref, what="configs[4] regime 128x72")
    assert rcnt["skip"] > 0, rcnt
    assert st["cut_paths"] == dev["cut"] > 0 and st["watchdog_paths"] == 0, (st, dev)
