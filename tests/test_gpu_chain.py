"""Chained calls (RtOptions.overlap) and the bounded traversal's run-time
guard (RtOptions.check_interval), both on the default render (the bounded
traversal, one persistent finisher per call, deep paths in wf_long).

Chained calls let a call's deep-path tail (glass loops of 10^4+ bounces,
SURVEY H8) run on while the next call of the same frame starts; pixels still
out are owed the new call's passes.  A pixel's passes still run in order, so
the frame must be bit-identical to unchained calls and to the oracle — over
back-to-back calls on one stream, with the frame read (joined) in between,
with adaptive sampling, and with calls that change the camera (which must not
chain).  The guard re-traces a deterministic sample of the finisher's rays
with the plain KD traversal (trace_ray, rt/trace_ray.cuh:244-318): its
counters must show checks and no mismatch, and a deliberately corrupted
record must be caught.
"""
import ctypes

import numpy as np
import pytest

import helpers
import rt

pytestmark = pytest.mark.gpu
WF = rt.KERNEL_WAVEFRONT


_HIP = None
_STREAMS = []


def _stream():
    """a raw hipStream_t (kept for the session: the library may still hold events on it)"""
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
    s = ctypes.c_void_p()
    assert _HIP.hipStreamCreate(ctypes.byref(s)) == 0
    _STREAMS.append(s)
    return s


# the chained-call protocol tests launch every call (coalesce_passes < 0): coalescing
# (the default, RtOptions.coalesce_passes) would merge their small calls into one launch;
# tests of coalescing pass coalesce_passes explicitly
NOCO = -1


def _render_calls(run, W, H, passes, stream=None, overlap=True, **kw):
    kw.setdefault("coalesce_passes", NOCO)
    return run.render(W, H, passes, kernel=WF, overlap=overlap, stream=stream, **kw)[0]


@pytest.mark.parametrize("coalesce", [NOCO, 0])
@pytest.mark.parametrize("name,W,H,split", [("room2m", 1920, 1080, [16, 16, 16, 16]),
                                            ("cornell_blob", 640, 360, [1, 2, 5, 8])])
def test_chained_calls_equal_one_call(name, W, H, split, coalesce):
    run = helpers.GpuRun(name)
    one = _render_calls(run, W, H, [sum(split)], overlap=False)
    s = _stream()
    chained = _render_calls(run, W, H, split, stream=s, coalesce_passes=coalesce)
    helpers.assert_bitwise(chained, one, what=f"{name} {len(split)} chained calls vs one call")
    assert int(chained[2].sum()) == W * H * sum(split)


def test_chained_deep_paths_vs_oracle(tmp_path):
    """The glass light guide: hundreds of bounces per path, most pixels' samples
    handed to wf_long; 1-pass chained calls (the reference's granularity,
    rt/main.cu:114-155) must give the oracle's frame."""
    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    run = helpers.GpuRun(trap)
    W, H = 96, 64
    split = [1] * 6 + [3]
    rt.deviation_stats(reset=True)
    gpu = _render_calls(run, W, H, split, wf_long_depth=8)
    dev = rt.deviation_stats(reset=False)
    ref, _ = helpers.oracle_render(trap, W, H, split)
    helpers.assert_bitwise(gpu, ref, what="light guide, chained 1-pass calls")
    assert dev["deep_paths"] > 0, dev  # the hand-off really ran
    # ... and the owed-passes protocol fired: pixels out in wf_long were skipped by later calls
    assert dev["owed_pixels"] > 0 and dev["owed_passes"] >= dev["owed_pixels"], dev
    assert dev["stranded_pixels"] == 0 and dev["long_safety_quits"] == 0, dev


def test_checkpoint_mid_chain(tmp_path):
    """rt_gbuffer_save between chained calls must join the open
    chain first (its owed passes run in the drain), so the checkpoint holds
    exactly the passes of the calls so far; resuming from it in a fresh
    G_Buffer and finishing the passes is bit-identical to the oracle's
    uninterrupted render.  The light guide keeps pixels out in wf_long across
    call boundaries, so the chain really is open with passes owed."""
    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    run = helpers.GpuRun(trap)
    W, H = 96, 64
    rt.deviation_stats(reset=True)
    g = rt.GBuffer(W, H)
    ck = tmp_path / "mid.gbuf"
    for c in range(4):
        rt.render(run.dev, g, run.camera, 0 if c == 0 else 1,
                  rt.options(W, H, 1, adaptive=False, kernel=WF, overlap=True, wf_long_depth=8,
                             coalesce_passes=NOCO))
    g.save(ck, 4)  # mid-chain: joins (drains) first
    dev = rt.deviation_stats(reset=False)
    assert dev["owed_pixels"] > 0, dev  # the chain was open with owed passes at the save
    mid_ref, _ = helpers.oracle_render(trap, W, H, [1, 1, 1, 1])
    g2 = rt.GBuffer(W, H, 12345)  # other seeds: everything must come from the file
    assert g2.load(ck) == 4
    helpers.assert_bitwise(g2.download(), mid_ref, what="checkpoint taken mid-chain")
    for c in range(3):  # resume: chained calls again, on the loaded G_Buffer
        rt.render(run.dev, g2, run.camera, 1, rt.options(W, H, 1, adaptive=False, kernel=WF, overlap=True,
                                                         wf_long_depth=8, coalesce_passes=NOCO))
    ref, _ = helpers.oracle_render(trap, W, H, [1] * 7)
    helpers.assert_bitwise(g2.download(), ref, what="resumed from a mid-chain checkpoint")


@pytest.mark.parametrize("overlap", [False, True])
def test_long_kernel_quit_is_reported(tmp_path, overlap):
    """a failure of the hand-off must not pass silently.
    RT_DEBUG_LONG_QUIT makes wf_long leave at once, as if its safety net had
    fired: every pixel handed to it is stranded.  The join must say so
    (RT_E_INCOMPLETE), RtDeviations must count the exits and the stranded
    pixels, and the workspace must recover: the next render is exact."""
    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    run = helpers.GpuRun(trap)
    W, H = 96, 64
    rt.deviation_stats(reset=True)
    g = rt.GBuffer(W, H)
    for c in range(2):
        rt.render(run.dev, g, run.camera, 0 if c == 0 else 1,
                  rt.options(W, H, 2, adaptive=False, kernel=WF, overlap=overlap, wf_long_depth=8,
                             debug=rt.DEBUG_LONG_QUIT, coalesce_passes=NOCO))
    with pytest.raises(rt.RtError) as ei:
        rt.join()
    assert f"rt error {rt.E_INCOMPLETE}" in str(ei.value) and "stranded" in str(ei.value), str(ei.value)
    dev = rt.deviation_stats(reset=True)
    assert dev["long_safety_quits"] > 0 and dev["stranded_pixels"] > 0, dev
    rt.join()  # reported once: the stranded pixels were released
    gpu = _render_calls(run, W, H, [2, 2], overlap=overlap, wf_long_depth=8)
    ref, _ = helpers.oracle_render(trap, W, H, [2, 2])
    helpers.assert_bitwise(gpu, ref, what="render after a stranded frame")
    dev = rt.deviation_stats(reset=True)
    assert dev["stranded_pixels"] == 0 and dev["long_safety_quits"] == 0, dev


def test_chained_adaptive_and_reads_between(tmp_path):
    """Adaptive sampling over chained calls, the frame read (tonemap: joins) in
    between, and a camera change (must not chain) — equal to plain calls."""
    run = helpers.GpuRun("room_small")
    W, H = 480, 270
    ref = _render_calls(run, W, H, [6, 6, 6, 6], overlap=False, adaptive=True, min_samples=8)
    g = rt.GBuffer(W, H)
    for c in range(4):
        opt = rt.options(W, H, 6, adaptive=True, min_samples=8, kernel=WF, overlap=True)
        rt.render(run.dev, g, run.camera, 0 if c == 0 else 1, opt)
        if c == 1:
            rt.tonemap(g)  # reads the frame: joins the chained tail first
    helpers.assert_bitwise(g.download(), ref, what="adaptive chained with a read between")
    # a call with another camera does not chain onto the previous one
    cam2 = rt.Camera()
    ctypes.memmove(ctypes.byref(cam2), ctypes.byref(run.camera), ctypes.sizeof(rt.Camera))
    cam2.yaw += 0.05
    g1, g2 = rt.GBuffer(W, H), rt.GBuffer(W, H)
    for g_, ov in ((g1, True), (g2, False)):
        rt.render(run.dev, g_, run.camera, 0, rt.options(W, H, 4, adaptive=False, kernel=WF, overlap=ov))
        rt.render(run.dev, g_, cam2, 1, rt.options(W, H, 4, adaptive=False, kernel=WF, overlap=ov))
    helpers.assert_bitwise(g1.download(), g2.download(), what="camera change between chained calls")


def test_guard_counts_checks_and_no_mismatch():
    run = helpers.GpuRun("room2m")
    rt.deviation_stats(reset=True)
    _render_calls(run, 960, 540, [8, 8], check_interval=64)
    dev = rt.deviation_stats(reset=True)
    # ~960*540*16 samples x ~3 rays / 64
    assert dev["bounded_checked"] > 200_000, dev
    assert dev["bounded_mismatches"] == 0, dev


def test_guard_catches_a_corrupted_result():
    """RT_DEBUG_CHECK_FAULT records every checked ray with a wrong result (a
    hit's triangle index flipped, a miss as a hit of triangle 0): the KD
    re-trace must flag every one of them."""
    run = helpers.GpuRun("cornell")
    rt.deviation_stats(reset=True)
    _render_calls(run, 128, 128, [4], check_interval=16, debug=4)
    dev = rt.deviation_stats(reset=True)
    assert dev["bounded_checked"] > 1000, dev
    assert dev["bounded_mismatches"] == dev["bounded_checked"], dev
    assert any(v != 0.0 for v in dev["mismatch_ray"]), dev


def test_megakernel_two_streams_equal_serial():
    """two bounded megakernel calls on different streams share the
    per-device spill area; the library serialises them on it."""
    run = helpers.GpuRun("room_small")
    W, H = 320, 180
    ga, gb = rt.GBuffer(W, H), rt.GBuffer(W, H, W * H)
    s1, s2 = _stream(), _stream()
    for g_, s in ((ga, s1), (gb, s2)):
        rt.render(run.dev, g_, run.camera, 0, rt.options(W, H, 4, adaptive=False, kernel=rt.KERNEL_MEGA,
                                                         stream=s))
    rt.check(rt.lib().rt_synchronize())
    ra, _, _ = run.render(W, H, 4, kernel=rt.KERNEL_MEGA)
    rb, _, _ = run.render(W, H, 4, kernel=rt.KERNEL_MEGA, seed_skip=W * H)
    helpers.assert_bitwise(ga.download(), ra, what="megakernel stream 1")
    helpers.assert_bitwise(gb.download(), rb, what="megakernel stream 2")


def test_small_frame_after_a_large_one(tmp_path):
    """The per-device workspace is sized by the largest frame so far; a later,
    smaller frame must not see that frame's hand-off ring entries (a stale
    sequence tag beyond the small frame's pixel count looks published).  A
    1080p room2m call, then the 600-unit light guide (every path past 64
    bounces goes through the ring, many more entries than pixels) against the
    oracle."""
    big = helpers.GpuRun("room2m")
    big.render(1920, 1080, [2], kernel=WF)
    trap = helpers.make_trap_scene(str(tmp_path / "t"), 600.0)
    run = helpers.GpuRun(trap)
    W, H, P = 64, 48, 4
    gpu, _, _ = run.render(W, H, P, calls=2, kernel=WF)
    ref, _ = helpers.oracle_render(trap, W, H, P, calls=2)
    helpers.assert_bitwise(gpu, ref, what="light guide after a 1080p frame")


@pytest.mark.parametrize("coalesce", [NOCO, 0])
def test_chain_interrupted_by_another_frame(tmp_path, coalesce):
    """A chain left open on one G_Buffer is drained when a call for another
    frame comes (join_all in the fresh call): both frames equal their
    unchained renders.  The light guide keeps pixels out in wf_long across
    call boundaries, so the first chain really has owed passes to drain."""
    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    run = helpers.GpuRun(trap)
    W, H = 96, 64
    ga, gb = rt.GBuffer(W, H), rt.GBuffer(W, H, W * H)
    for c in range(3):
        rt.render(run.dev, ga, run.camera, 0 if c == 0 else 1,
                  rt.options(W, H, 1, adaptive=False, kernel=WF, overlap=True, wf_long_depth=8,
                             coalesce_passes=coalesce))
    for c in range(3):  # another frame: not a continuation, the open chain (or batch) drains first
        rt.render(run.dev, gb, run.camera, 0 if c == 0 else 1,
                  rt.options(W, H, 2, adaptive=False, kernel=WF, overlap=True, wf_long_depth=8,
                             coalesce_passes=coalesce))
    rt.join()
    ra, _ = helpers.oracle_render(trap, W, H, [1, 1, 1])
    rb, _ = helpers.oracle_render(trap, W, H, [2, 2, 2], seed_skip=W * H)
    helpers.assert_bitwise(ga.download(), ra, what="chain A drained by frame B's call")
    helpers.assert_bitwise(gb.download(), rb, what="chain B")


def test_chain_left_open_at_exit(tmp_path):
    """A process that ends with a chain still open (no rt_join): rt_shutdown
    (atexit) drains it before it frees the workspace — the process exits
    cleanly and promptly."""
    import subprocess
    import sys
    import textwrap
    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    code = textwrap.dedent(f"""
        import sys
        sys.path[:0] = {[p for p in sys.path if p.endswith(('isaklm-raytracer_amd', 'tests', 'oracle'))]!r}
        import helpers, rt
        rt.check(rt.lib().rt_set_device(0))
        run = helpers.GpuRun({trap!r})
        g = rt.GBuffer(96, 64)
        for c in range(4):
            rt.render(run.dev, g, run.camera, 0 if c == 0 else 1,
                      rt.options(96, 64, 1, adaptive=False, kernel=rt.KERNEL_WAVEFRONT, overlap=True,
                                 wf_long_depth=8))
        print("enqueued", flush=True)
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "enqueued" in r.stdout, r.stdout + r.stderr


def test_unchained_long_calls_run_each_pass_once():
    """Two unchained 256-pass room2m calls: every pixel ends with exactly 512
    samples.  (Round 5 regression: a finisher's lingering waves kept claiming
    from the exhausted pixel list on every idle trip, wrapped its 32-bit
    cursor during a long linger and ran the call's pixels a second time; the
    1,024-spp budget test caught it as a 1.25x frame.)"""
    run = helpers.GpuRun("room2m")
    W, H = 1920, 1080
    gpu = _render_calls(run, W, H, [256, 256], overlap=False)
    assert int(gpu[2].min()) == 512 and int(gpu[2].max()) == 512


def _stream_nonblocking():
    """a raw non-blocking hipStream_t (hipStreamNonBlocking: not ordered against the null stream)"""
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
    s = ctypes.c_void_p()
    assert _HIP.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1)) == 0
    _STREAMS.append(s)
    return s


@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("order", ["long_first", "fin_first"])
def test_serialised_dispatch_is_exact(tmp_path, order, overlap):
    """under rocprofv3 counter collection the path kernel
    (the finisher) and the long-path kernel (wf_long) dispatch one at a time,
    in either order — the bench's counter pass hung when wf_long went first
    and waited for a finisher that could not start.  The debug bits force each
    order: wf_long first must close its hand-off ring after its bounded wait
    and leave (the finisher then runs its deep paths itself); the finisher
    first must stop lingering for wf_long (bounded by loop trips, not by the
    clock).  Both must be bit-exact, strand nothing, and finish in seconds."""
    import time

    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    run = helpers.GpuRun(trap)
    W, H = 96, 64
    bit = rt.DEBUG_SERIAL_LONG_FIRST if order == "long_first" else rt.DEBUG_SERIAL_FIN_FIRST
    rt.join()
    rt.deviation_stats(reset=True)
    t = time.perf_counter()
    gpu = _render_calls(run, W, H, [2, 3, 1], overlap=overlap, wf_long_depth=8, debug=bit)
    dt = time.perf_counter() - t
    ref, _ = helpers.oracle_render(trap, W, H, [2, 3, 1])
    helpers.assert_bitwise(gpu, ref, what=f"serialised dispatch ({order}, overlap {overlap})")
    dev = rt.deviation_stats(reset=True)
    assert dev["stranded_pixels"] == 0 and dev["long_safety_quits"] == 0, dev
    if order == "long_first":
        assert dev["long_closed"] > 0, dev  # every call's wf_long found its finisher not started
    else:
        assert dev["long_closed"] == 0, dev
    assert dt < 30.0, dt
    # the workspace recovers: the next (unserialised) render hands deep paths off again, exactly
    rt.deviation_stats(reset=True)
    gpu = _render_calls(run, W, H, [2, 2], overlap=overlap, wf_long_depth=8)
    ref, _ = helpers.oracle_render(trap, W, H, [2, 2])
    helpers.assert_bitwise(gpu, ref, what="render after serialised dispatch")
    assert rt.deviation_stats(reset=True)["long_closed"] == 0


def test_serialised_dispatch_room2m_bench_shape():
    """The bench's counter pass, as it hung: an unchained 1080p room2m call
    with wf_long dispatched before the finisher.  Bit-identical to the
    unserialised call of the same passes."""
    run = helpers.GpuRun("room2m")
    W, H = 1920, 1080
    plain = _render_calls(run, W, H, [2, 6], overlap=False)
    rt.deviation_stats(reset=True)
    serial = _render_calls(run, W, H, [2, 6], overlap=False, debug=rt.DEBUG_SERIAL_LONG_FIRST)
    helpers.assert_bitwise(serial, plain, what="room2m 1080p, wf_long dispatched first")
    dev = rt.deviation_stats(reset=True)
    assert dev["long_closed"] > 0 and dev["stranded_pixels"] == 0, dev


def test_incomplete_status_is_sticky(tmp_path):
    """a library join that does not report (rt_deviation_stats)
    must not swallow a stranded frame: the next reporting join still returns
    RT_E_INCOMPLETE, once."""
    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    run = helpers.GpuRun(trap)
    W, H = 96, 64
    rt.join()
    rt.deviation_stats(reset=True)
    g = rt.GBuffer(W, H)
    rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 2, adaptive=False, kernel=WF, wf_long_depth=8,
                                                    debug=rt.DEBUG_LONG_QUIT))
    dev = rt.deviation_stats(reset=False)  # joins, does not report
    assert dev["stranded_pixels"] > 0, dev
    with pytest.raises(rt.RtError) as ei:
        rt.join()
    assert f"rt error {rt.E_INCOMPLETE}" in str(ei.value), str(ei.value)
    rt.join()  # reported once
    rt.deviation_stats(reset=True)


def test_stream_join_then_render_on_another_stream(tmp_path):
    """a stream join enqueues the hand-off check
    (wf_verify, which rewrites every pixel's ownership word) on that stream;
    a render on another, non-blocking stream right after must run after it —
    else the check can free a pixel a new finisher lane holds."""
    trap = helpers.make_trap_scene(str(tmp_path / "t"))
    run = helpers.GpuRun(trap)
    W, H = 96, 64
    a, b = _stream_nonblocking(), _stream_nonblocking()
    g = rt.GBuffer(W, H)
    split = [2, 1, 2, 3]
    for c, p in enumerate(split):
        s = a if c < 2 else b
        rt.render(run.dev, g, run.camera, 0 if c == 0 else 1,
                  rt.options(W, H, p, adaptive=False, kernel=WF, overlap=c < 2, wf_long_depth=8, stream=s,
                             coalesce_passes=NOCO))
        if c == 1:
            rt.join(a)  # drain + wf_verify on a; the host does not wait
    rt.join()
    ref, _ = helpers.oracle_render(trap, W, H, split)
    helpers.assert_bitwise(g.download(), ref, what="render on stream b after a join on stream a")


def test_coalesced_chained_calls():
    """RtOptions.coalesce_passes: chained calls of fewer passes are recorded
    and launched as one chained call once the batch holds that many passes, or
    before anything that must see them.  16 chained 1-pass calls with the
    default threshold (256) run as ONE launch (one profile record); with a
    threshold of 4, as launches of 4, 4, 4 and 4 passes; a read of the frame in
    between (rt_tonemap: joins) launches the batch first; a call of another
    frame launches the batch first.  Every frame equals the oracle's."""
    run = helpers.GpuRun("cornell_blob")
    W, H = 320, 180
    ref, _ = helpers.oracle_render(run.path, W, H, [1] * 16)
    for thr, launches in ((0, 1), (4, 4)):
        rt.join()
        rt.profile_history(reset=True)
        g = rt.GBuffer(W, H)
        rt.render(run.dev, g, run.camera, 0, rt.options(W, H, 1, adaptive=False, kernel=WF))  # (resets: not chained)
        for _ in range(15):
            rt.render(run.dev, g, run.camera, 1, rt.options(W, H, 1, adaptive=False, kernel=WF, overlap=True,
                                                            profile=True, coalesce_passes=thr))
        rt.join()
        hist = rt.profile_history(reset=True)
        helpers.assert_bitwise(g.download(), ref, what=f"16 1-pass calls, coalesce_passes {thr}")
        # the resetting call (not profiled) + 15 chained passes: 1 batch of 15 (thr 256) or 4+4+4+3 (thr 4)
        assert len(hist) == launches, (thr, len(hist))
    # a read between chained calls launches (and joins) the pending batch
    g = rt.GBuffer(W, H)
    ref8, _ = helpers.oracle_render(run.path, W, H, [1] * 8)
    for c in range(8):
        rt.render(run.dev, g, run.camera, 0 if c == 0 else 1, rt.options(W, H, 1, adaptive=False, kernel=WF,
                                                                         overlap=True))
        if c == 4:
            rt.tonemap(g)
            assert int(g.download()[2].min()) == 5  # the 4 pending chained passes ran before the read
    rt.join()
    helpers.assert_bitwise(g.download(), ref8, what="coalesced calls with a read between")
