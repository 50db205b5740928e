"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the
same seeds, for both kernel variants (megakernel, wavefront).  The bar is
bit-exact accumulators (fb, sq, count, RNG state) and equal work counters;
north_star's 1e-4 relative L-infinity is asserted too.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

import helpers
import oracle
import rt

pytestmark = pytest.mark.gpu
KERNELS = [pytest.param(rt.KERNEL_MEGA, id="mega"), pytest.param(rt.KERNEL_WAVEFRONT, id="wavefront")]


@pytest.fixture(scope="module")
def cornell():
    return helpers.GpuRun("cornell")


@pytest.mark.parametrize("kernel", KERNELS)
def test_cornell_bitwise_adaptive_off(cornell, kernel):
    W, H, P = 64, 64, 8
    gpu, gcnt, _ = cornell.render(W, H, P, count=True, kernel=kernel)
    ref, rcnt = helpers.oracle_render(cornell.path, W, H, P)
    helpers.assert_bitwise(gpu, ref, what="cornell")
    for k in rt.COUNTER_NAMES:
        assert gcnt[k] == rcnt[k], (k, gcnt, rcnt)
    assert helpers.rel_linf(gpu[0], gpu[2], ref[0], ref[2]) < 1e-4


@pytest.mark.parametrize("kernel", KERNELS)
def test_cornell_split_calls_equal_one_call(cornell, kernel):
    """render() called 3x with passes=2 == one call with passes=6 (state carried in the G_Buffer)."""
    W, H = 48, 32
    a, _, _ = cornell.render(W, H, 2, calls=3, kernel=kernel)
    b, _, _ = cornell.render(W, H, 6, calls=1, kernel=kernel)
    helpers.assert_bitwise(a, b, what="split")


@pytest.mark.parametrize("kernel", KERNELS)
def test_cornell_adaptive_on(cornell, kernel):
    """Adaptive sampling (rt/path_tracing.cuh:352-376) with a low min_samples so it engages."""
    W, H, P = 40, 40, 24
    gpu, gcnt, _ = cornell.render(W, H, P, adaptive=True, min_samples=6, count=True, kernel=kernel)
    ref, rcnt = helpers.oracle_render(cornell.path, W, H, P, adaptive=True, min_samples=6)
    helpers.assert_bitwise(gpu, ref, what="adaptive")
    assert gcnt == rcnt
    assert rcnt["skip"] > 0  # the test really skipped pixels


@pytest.mark.parametrize("kernel", KERNELS)
def test_odd_resolution_and_max_depth(cornell, kernel):
    """W, H odd (SCREEN_W/2 integer truncation), max_depth cap applied identically."""
    W, H, P = 37, 23, 5
    gpu, gcnt, _ = cornell.render(W, H, P, max_depth=3, count=True, kernel=kernel)
    ref, rcnt = helpers.oracle_render(cornell.path, W, H, P, max_depth=3)
    helpers.assert_bitwise(gpu, ref, what="odd")
    assert gcnt == rcnt


@pytest.mark.parametrize("variant", [2, 3], ids=["wavefront-static-trace", "wavefront-lane-fetch"])
def test_other_trace_variants(variant):
    run = helpers.GpuRun("room_small")
    W, H, P = 48, 27, 3
    gpu, gcnt, _ = run.render(W, H, P, count=True, kernel=variant)
    ref, rcnt = helpers.oracle_render(run.path, W, H, P)
    helpers.assert_bitwise(gpu, ref, what=f"variant{variant}")
    assert gcnt == rcnt


@pytest.mark.parametrize("scene", ["room_small", "cornell_blob"])
@pytest.mark.parametrize("tail,waves,wide", [(1 << 30, 3, 0), (1 << 30, 3, 3), (1 << 30, 1 << 20, 0),
                                             (1 << 30, 1 << 20, -1), (700, 5, 0), (1, 0, 0)],
                         ids=["finisher-only-refetch", "finisher-only-refetch-wide-3", "finisher-only-wide",
                              "finisher-only-1-per-wave-narrow", "late-handoff-refetch", "queues-only"])
def test_wavefront_finisher_modes(scene, tail, waves, wide):
    """The cooperative finisher (wf_finish_coop) at every hand-off point and
    width: whole call in the finisher with few waves (lanes refetch paths;
    waves with at most 32 — or 3 — live rays trace them one by one with all
    lanes, resuming rays in mid-traversal), one path per wave (every ray
    traced by a whole wave: wide_trace, or not), a late hand-off, and no
    finisher at all."""
    run = helpers.GpuRun(scene)
    W, H, P = 48, 27, 3
    gpu, gcnt, _ = run.render(W, H, P, count=True, kernel=rt.KERNEL_WAVEFRONT, wf_tail=tail, wf_finish_waves=waves,
                              wf_wide=wide)
    ref, rcnt = helpers.oracle_render(run.path, W, H, P)
    helpers.assert_bitwise(gpu, ref, what=f"finisher tail={tail} waves={waves} wide={wide}")
    assert gcnt == rcnt


@pytest.mark.parametrize("scene", ["room_small", "cornell_blob", "room2m"])
def test_bounded_queue_path(scene):
    """The queue path with the bounded traversal (wf_tail = 1: trace / shade
    iterations to the end, no finisher): its trace launches run
    wf_trace_bvh_dyn (per-lane ray refill, capped steps per round), which
    must give trace_bvh's hits bit for bit — every pixel against the oracle."""
    run = helpers.GpuRun(scene)
    W, H, P = (160, 90, 3) if scene == "room2m" else (48, 27, 3)
    gpu, _, _ = run.render(W, H, P, calls=2, kernel=rt.KERNEL_WAVEFRONT, wf_tail=1)
    ref, _ = helpers.oracle_render(run.path, W, H, P, calls=2)
    helpers.assert_bitwise(gpu, ref, what=f"{scene} bounded queue path")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("scene", ["room_small", "cornell_blob"])
@pytest.mark.parametrize("long_depth,pipes", [(1, 3), (3, 1), (-1, 2)],
                         ids=["long-handoff-all", "long-handoff-deep-1-pipe", "no-handoff-2-pipes"])
def test_wavefront_long_paths_and_pipelines(scene, long_depth, pipes):
    """Paths handed to wf_long (every path deeper than 1 or 3 bounces, so the
    cross-kernel hand-off is exercised thousands of times) and the pipeline
    split leave every accumulator and counter bit-identical."""
    run = helpers.GpuRun(scene)
    W, H, P = 48, 27, 3
    gpu, gcnt, _ = run.render(W, H, P, calls=2, count=True, kernel=rt.KERNEL_WAVEFRONT, wf_long_depth=long_depth,
                              wf_pipelines=pipes)
    ref, rcnt = helpers.oracle_render(run.path, W, H, P, calls=2)
    helpers.assert_bitwise(gpu, ref, what=f"long_depth={long_depth} pipes={pipes}")
    assert gcnt == rcnt


@pytest.mark.timeout(180)
def test_long_handoff_with_shared_hw_queues():
    """The wf_long slices run on the caller's stream beside the pipeline
    streams.  With the process's hardware queues taken by other streams first
    (RCCL's, in a multi-GPU bench) the runtime maps several streams onto one
    queue: the slices must not wait on work queued behind them.  Runs in a
    child process (fresh stream-to-queue mapping), bounded by a timeout."""
    import subprocess
    import sys

    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "queue_sharing_child.py")
    r = subprocess.run([sys.executable, child, "8"], capture_output=True, text=True, timeout=150)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.parametrize("kernel", KERNELS)
def test_textured_scene_bitwise(kernel, tmp_path):
    """sample_texture (rt/trace_ray.cuh:31-46) on the GPU: textures decoded by
    the product loader (PNG palette/Adam7/grey, baseline JPEG 4:2:0 and q100;
    digests pinned to stb_image in tests/golden/textures.json), UVs wrapping
    far outside [0, 1], a triangle whose mod(uv, 1) is 1.0 (padded texel), a
    textured emitter and a missing texture file.  The oracle gets the same
    texels through its registry."""
    import hashlib
    import json

    scene, files = helpers.make_textured_scene(str(tmp_path))
    golden = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "textures.json")))
    for rel, var in files.items():
        a = rt.decode_image(os.path.join(str(tmp_path), rel))
        d = hashlib.sha256(a.tobytes()).hexdigest() + f":{a.shape[1]}x{a.shape[0]}"
        assert d == golden["variants"][var], rel
        oracle.register_texture(rel, a)
    run = helpers.GpuRun(scene)
    W, H, P = 48, 32, 6
    gpu, gcnt, _ = run.render(W, H, P, calls=2, count=True, kernel=kernel)
    ref, rcnt = helpers.oracle_render(scene, W, H, P, calls=2)
    helpers.assert_bitwise(gpu, ref, what="textured")
    assert gcnt == rcnt, (gcnt, rcnt)
    assert rcnt["texel"] > 0


@pytest.mark.parametrize("kernel", KERNELS)
def test_checkpoint_resume_bitwise(cornell, kernel, tmp_path):
    """rt_gbuffer_save after 3 passes, rt_gbuffer_load into a fresh G_Buffer
    (other seeds), 4 more passes == 7 passes in one G_Buffer (adaptive on)."""
    W, H = 40, 24
    opt = lambda p: rt.options(W, H, p, adaptive=True, min_samples=4, kernel=kernel)  # noqa: E731
    a = rt.GBuffer(W, H)
    rt.render(cornell.dev, a, cornell.camera, 0, opt(3))
    a.save(tmp_path / "ck.gbuf", 3)
    b = rt.GBuffer(W, H, seed_skip=12345)
    assert b.load(tmp_path / "ck.gbuf") == 3
    rt.render(cornell.dev, b, cornell.camera, 3, opt(4))
    c = rt.GBuffer(W, H)
    rt.render(cornell.dev, c, cornell.camera, 0, opt(7))
    helpers.assert_bitwise(b.download(), c.download(), what="resume")


def test_kernels_agree_multi_call(cornell):
    """Megakernel and wavefront give the same bits across calls with reset."""
    W, H = 33, 31
    a, _, _ = cornell.render(W, H, 3, calls=2, kernel=rt.KERNEL_MEGA)
    b, _, _ = cornell.render(W, H, 3, calls=2, kernel=rt.KERNEL_WAVEFRONT)
    helpers.assert_bitwise(a, b, what="mega-vs-wavefront")


def test_tonemap_matches_oracle(cornell):
    W, H = 32, 32
    gpu, _, g = cornell.render(W, H, 4)
    img = rt.tonemap(g)
    ref = oracle.tonemap(gpu[0], gpu[2])
    assert np.max(np.abs(img.astype(int) - ref.astype(int))) <= 1


@pytest.mark.parametrize("kernel", KERNELS)
def test_seed_shard_offset(cornell, kernel):
    """Shard g of an spp-sliced render seeds from mt19937 outputs [g*W*H, (g+1)*W*H)."""
    W, H, P = 24, 24, 3
    gpu, _, _ = cornell.render(W, H, P, seed_skip=2 * W * H, kernel=kernel)
    ref, _ = helpers.oracle_render(cornell.path, W, H, P, seed_skip=2 * W * H)
    helpers.assert_bitwise(gpu, ref, what="shard")


@pytest.mark.parametrize("kernel", KERNELS)
def test_cornell_blob_bitwise(kernel):
    run = helpers.GpuRun("cornell_blob")
    W, H, P = 64, 36, 4
    gpu, gcnt, _ = run.render(W, H, P, count=True, kernel=kernel)
    ref, rcnt = helpers.oracle_render(run.path, W, H, P)
    helpers.assert_bitwise(gpu, ref, what="cornell_blob")
    assert gcnt == rcnt


@pytest.mark.parametrize("kernel", KERNELS)
def test_room_small_bitwise(kernel):
    run = helpers.GpuRun("room_small")
    W, H, P = 64, 36, 4
    gpu, gcnt, _ = run.render(W, H, P, count=True, kernel=kernel)
    ref, rcnt = helpers.oracle_render(run.path, W, H, P)
    helpers.assert_bitwise(gpu, ref, what="room_small")
    assert gcnt == rcnt


def _golden_cases():
    import json
    import os

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_regression.json")
    return sorted(json.load(open(path))["renders"].items())


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("key,gold", _golden_cases(), ids=[k for k, _ in _golden_cases()])
def test_golden_vectors(key, gold, kernel):
    """The committed fixtures (tests/golden/oracle_regression.json) reproduced on the GPU."""
    import sys
    import os

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden

    name, W, H, P, calls, adaptive, ms, md, skip = gold["case"]
    run = helpers.GpuRun(name)
    (fb, sq, cnt, rng), counters, _ = run.render(W, H, P, calls=calls, adaptive=adaptive, min_samples=ms,
                                                 max_depth=md, seed_skip=skip, count=True, kernel=kernel)
    assert make_golden.accum_digest(fb, sq, cnt, rng) == gold["sha256"]
    assert counters == gold["counters"]


@pytest.mark.parametrize("kernel", KERNELS)
def test_room2m_full_frame_sparse_pixels(kernel):
    """BASELINE config 3 scene at 1920x1080: full-frame GPU render, every
    4099th pixel re-rendered by the oracle (pixels are independent)."""
    run = helpers.GpuRun("room2m")
    W, H, P = 1920, 1080, 2
    gpu, _, _ = run.render(W, H, P, kernel=kernel)
    pixels = np.arange(0, W * H, 4099, dtype=np.int32)
    ref, _ = helpers.oracle_render(run.path, W, H, P, pixels=pixels)
    helpers.assert_bitwise(gpu, ref, pixels=pixels, what="room2m")
    assert np.all(gpu[2] == P)


@pytest.mark.timeout(280)
def test_room2m_every_pixel_bench_options():
    """Every one of the 2,073,600 pixels of the 1920x1080 room2m frame, 2
    passes with the bench's kernel and defaults (pipelines, long-path
    hand-off, wide tails, finisher), bit-identical to the oracle (~25 s of
    oracle time on the GPU box's 16 cores)."""
    run = helpers.GpuRun("room2m")
    W, H, P = 1920, 1080, 2
    gpu, _, _ = run.render(W, H, P, kernel=rt.KERNEL_WAVEFRONT)
    ref, rcnt = helpers.oracle_render(run.path, W, H, P)
    helpers.assert_bitwise(gpu, ref, what="room2m every pixel")
    assert rcnt["sample"] == W * H * P and rcnt["watchdog"] == 0
    assert helpers.rel_linf(gpu[0], gpu[2], ref[0], ref[2]) < 1e-4


@pytest.mark.timeout(240)
def test_room2m_bench_configuration_sparse_pixels():
    """The driver-default bench (`python bench.py`: 1 warm-up + 4 timed steps)
    rendered UNCHAINED: room2m at 1920x1080, a call of 64 passes (sample_count
    0) then one of 4 steps = 256 passes (sample_count 1), the default render
    (bounded traversal, the whole call in one finisher, deep paths handed to
    wf_long at depth 64, the run-time guard), no counters.  Every 1031st pixel
    re-rendered by the oracle over the same 320 spp.  A counted call of the
    same options must not fire the 2^24 - 1-bounce watchdog.  The
    chained shape of `--steps 20 --warmup 5` is pinned by
    test_room2m_bench_chained_shape_sparse_pixels."""
    run = helpers.GpuRun("room2m")
    W, H, P = 1920, 1080, 64
    calls = [P, 4 * P]
    gpu, _, g = run.render(W, H, calls, kernel=rt.KERNEL_WAVEFRONT)
    pixels = np.arange(0, W * H, 1031, dtype=np.int32)
    ref, rcnt = helpers.oracle_render(run.path, W, H, calls, pixels=pixels)
    helpers.assert_bitwise(gpu, ref, pixels=pixels, what="room2m bench configuration")
    assert np.all(gpu[2] == sum(calls))
    assert helpers.rel_linf(gpu[0][pixels], gpu[2][pixels], ref[0][pixels], ref[2][pixels]) < 1e-4
    assert rcnt["watchdog"] == 0
    cnt = rt.DeviceCounters()
    rt.render(run.dev, g, run.camera, 1, rt.options(W, H, P, adaptive=False, counters=cnt.p, kernel=rt.KERNEL_WAVEFRONT))
    c = cnt.read()
    assert c["watchdog"] == 0, c
    assert c["sample"] == W * H * P
    assert c["maxdepth"] > 64  # glass paths run past the long-path hand-off depth


@pytest.mark.timeout(420)
def test_room2m_bench_chained_shape_sparse_pixels():
    """the driver's bench command (`bench.py --steps 20
    --warmup 5`) exactly, through bench.py's own call plan: warm-up calls of
    256 + 64 passes (chained), the bench's rt_synchronize (a join), five
    chained timed calls of 256 passes, and rt_tonemap without a stream as the
    join that ends the timed region.  Every 4099th pixel re-rendered by the
    oracle over the same 1,600 spp, bit for bit.  The owed-passes protocol must
    really have fired (pixels skipped while out in wf_long, their passes run
    later) and the hand-off must report no failure."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    run = helpers.GpuRun("room2m")
    W, H, P, spc, warmup, steps = 1920, 1080, 64, 4, 5, 20
    chain = len(bench.call_plan(warmup, steps, spc)) > 1
    assert chain
    g = rt.GBuffer(W, H)
    passes = []
    rt.deviation_stats(reset=True)

    def calls(first, count):
        for start, k in bench.call_plan(first, count, spc):
            rt.render(run.dev, g, run.camera, 0 if start == 0 else 1,
                      rt.options(W, H, P * k, adaptive=False, kernel=rt.KERNEL_WAVEFRONT, overlap=chain))
            passes.append(P * k)

    calls(0, warmup)
    rt.check(rt.lib().rt_synchronize())
    calls(warmup, steps)
    rgba = ctypes.c_void_p()
    rt.check(rt.lib().rt_device_alloc(ctypes.byref(rgba), W * H * 4))
    rt.check(rt.lib().rt_tonemap(g.g, rgba, W, H, None))
    rt.check(rt.lib().rt_free(rgba))
    dev = rt.deviation_stats(reset=True)
    gpu = g.download()
    assert passes == [256, 64, 256, 256, 256, 256, 256]
    pixels = np.arange(0, W * H, 4099, dtype=np.int32)
    ref, rcnt = helpers.oracle_render(run.path, W, H, passes, pixels=pixels)
    helpers.assert_bitwise(gpu, ref, pixels=pixels, what="room2m, the bench's chained timed shape")
    assert np.all(gpu[2] == sum(passes))
    assert rcnt["watchdog"] == 0
    assert dev["deep_paths"] > 0 and dev["owed_pixels"] > 0 and dev["owed_passes"] >= dev["owed_pixels"], dev
    assert dev["stranded_pixels"] == 0 and dev["long_safety_quits"] == 0 and dev["check_dropped"] == 0, dev
    assert dev["bounded_checked"] > 0 and dev["bounded_mismatches"] == 0, dev


@pytest.mark.timeout(240)
@pytest.mark.parametrize("coalesce", [-1, 0])
def test_room2m_single_pass_chained_calls(coalesce):
    """The reference's call granularity (one render() per pass,
    rt/main.cu:114-122) through chained calls: room2m at 480x270, 16 chained
    calls of 1 pass, then the join; every pixel against the oracle."""
    run = helpers.GpuRun("room2m")
    W, H = 480, 270
    rt.deviation_stats(reset=True)
    gpu, _, _ = run.render(W, H, [1] * 16, kernel=rt.KERNEL_WAVEFRONT, overlap=True, coalesce_passes=coalesce)
    dev = rt.deviation_stats(reset=True)
    ref, _ = helpers.oracle_render(run.path, W, H, [1] * 16)
    helpers.assert_bitwise(gpu, ref, what="room2m, 16 chained 1-pass calls")
    assert dev["stranded_pixels"] == 0 and dev["long_safety_quits"] == 0, dev


@pytest.mark.timeout(240)
def test_room2m_glass_adaptive_full_frame_sparse_pixels():
    """BASELINE configs[4] setting per GPU: the dielectric stress scene
    (2M-triangle glass mesh, smooth normals) at 1920x1080, adaptive sampling
    on (engaging after min_samples), max depth 32, wavefront kernel with its
    default pipelines / long-path hand-off; every 3001st pixel re-rendered by
    the oracle.  Pixels are independent, so the sparse check covers the
    full-frame launch."""
    run = helpers.GpuRun("room2m_glass")
    W, H, P, MS = 1920, 1080, 24, 16
    gpu, _, _ = run.render(W, H, P, adaptive=True, min_samples=MS, max_depth=32, kernel=rt.KERNEL_WAVEFRONT)
    pixels = np.arange(0, W * H, 3001, dtype=np.int32)
    ref, rcnt = helpers.oracle_render(run.path, W, H, P, adaptive=True, min_samples=MS, max_depth=32, pixels=pixels)
    helpers.assert_bitwise(gpu, ref, pixels=pixels, what="room2m_glass adaptive")
    assert rcnt["skip"] > 0  # the adaptive test really skipped pixel-passes
    assert rcnt["watchdog"] == 0  # no path cut by the 65,536-bounce watchdog
    assert helpers.rel_linf(gpu[0][pixels], gpu[2][pixels], ref[0][pixels], ref[2][pixels]) < 1e-4


@pytest.mark.parametrize("long_depth,pipes,traversal", [
    (1, (0, 0), None),
    (-1, (3, 1), None),
    (1, (1, 3), "kd"),
    (-1, (0, 2), "kd"),
])
def test_consecutive_calls_on_different_streams(long_depth, pipes, traversal):
    """rt_render on stream A, then at once on stream B (no host sync between):
    the second call shares the device workspace (path state, long-path
    hand-off) and must wait for the first call's last wf_long slice and
    pipelines.  With wf_long_depth 1 every path deeper than 1 bounce goes
    through wf_long, so the first call's slices are still running when the
    second starts; with -1 (no hand-off) and a different pipeline count on
    the second call, pixels move to other pipelines while the first call's
    finisher may still write their path state."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    streams = [ctypes.c_void_p(), ctypes.c_void_p()]
    for s in streams:
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    try:
        run = helpers.GpuRun("room_small")
        W, H, P = 48, 27, 3
        g = rt.GBuffer(W, H)
        trav = {None: None, "kd": rt.TRAVERSAL_KD}[traversal]
        for c, s in enumerate(streams):
            opt = rt.options(W, H, P, adaptive=False, kernel=rt.KERNEL_WAVEFRONT, wf_long_depth=long_depth, stream=s,
                             wf_pipelines=pipes[c], traversal=trav)
            rt.render(run.dev, g, run.camera, 0 if c == 0 else 1, opt)
        rt.check(rt.lib().rt_synchronize())
        gpu = g.download()
        ref, _ = helpers.oracle_render(run.path, W, H, P, calls=2)
        helpers.assert_bitwise(gpu, ref, what="two streams")
    finally:
        for s in streams:
            hip.hipStreamDestroy(s)
