"""The drop-in boundary with the reference's own Scene (rt/scene.cuh:107-121):
a device Scene assembled the way the reference's create_scene() does it
(rt/create_scene.cuh:18-73: cudaMalloc + cudaMemcpy of the triangle AoS, the
light list and create_kd_tree's nodes / indices, here through rt_device_alloc
/ rt_upload) carries no node or index count; rt_scene_prepare(&scene, &h)
must recover them from the tree and render bit-identically to the oracle.
"""
import ctypes

import numpy as np
import pytest

import helpers
import rt

pytestmark = pytest.mark.gpu


def _upload(data: bytes):
    p = ctypes.c_void_p()
    rt.check(rt.lib().rt_device_alloc(ctypes.byref(p), max(len(data), 4)))
    buf = ctypes.create_string_buffer(data, len(data))
    if data:
        rt.check(rt.lib().rt_upload(p, buf, len(data)))
    return p


def reference_layout_scene(host):
    """create_scene (rt/create_scene.cuh:18-73) with the allocator swapped:
    exact-size device arrays, no side-channel counts."""
    tri_bytes, ntris = host.triangles_bytes()
    tris = np.frombuffer(tri_bytes, dtype=np.uint8).reshape(ntris, rt.TRIANGLE_BYTES)
    emit = tris[:, 96 + 12:96 + 24].copy().view(np.float32).reshape(ntris, 3)
    lights = np.nonzero((emit > 0).any(axis=1))[0].astype(np.int32)  # :40-64 (any emittance component > 0)
    tp, n = host.triangle_ptr()
    nodes, idx, bb = rt.build_kd_tree(tp, n)
    s = rt.Scene()
    s.triangles = _upload(tri_bytes).value
    s.triangle_count = ntris
    s.light_indicies = _upload(lights.tobytes()).value
    s.light_count = len(lights)
    s.kd_tree.nodes = _upload(nodes).value
    s.kd_tree.triangle_indicies = _upload(idx.tobytes()).value
    s.kd_tree.bounding_box = rt.Bounding_Box(rt.Vec3D(*bb[:3]), rt.Vec3D(*bb[3:]))
    return s, len(nodes) // rt.NODE_BYTES, len(idx)


@pytest.mark.parametrize("scene", ["cornell", "cornell_blob"])
def test_prepare_from_reference_scene_without_counts(scene):
    run = helpers.GpuRun(scene)
    s, nn, ni = reference_layout_scene(run.host)
    h = ctypes.c_void_p()
    rt.check(rt.lib().rt_scene_prepare(ctypes.byref(s), ctypes.byref(h)))

    class Prepared:
        prepared = h

    info = {}
    b, t, n, i, d = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rt.check(rt.lib().rt_scene_info(h, ctypes.byref(b), ctypes.byref(t), ctypes.byref(n), ctypes.byref(i),
                                    ctypes.byref(d)))
    info = {"nodes": n.value, "indices": i.value, "triangles": t.value}
    assert info == {"nodes": nn, "indices": ni, "triangles": run.host.triangle_ptr()[1]}
    W, H, P = 48, 32, 4
    g = rt.GBuffer(W, H)
    cnt = rt.DeviceCounters()
    rt.render(Prepared, g, run.camera, 0, rt.options(W, H, P, adaptive=False, counters=cnt.p,
                                                     kernel=rt.KERNEL_WAVEFRONT))
    gpu = g.download()
    ref, rcnt = helpers.oracle_render(run.path, W, H, P)
    helpers.assert_bitwise(gpu, ref, what="reference-layout Scene")
    gc = cnt.read()
    assert all(gc[k] == rcnt[k] for k in rt.COUNTER_NAMES), (gc, rcnt)
    rt.lib().rt_scene_release(h)
    for p in (s.triangles, s.light_indicies, s.kd_tree.nodes, s.kd_tree.triangle_indicies):
        rt.lib().rt_free(p)


def test_prepare_rejects_child_outside_allocation():
    run = helpers.GpuRun("cornell")
    s, nn, ni = reference_layout_scene(run.host)
    nodes = bytearray(nn * rt.NODE_BYTES)
    rt.check(rt.lib().rt_download((ctypes.c_char * len(nodes)).from_buffer(nodes), s.kd_tree.nodes, len(nodes)))
    # root is an inner node: point its second child past the end of the node array
    assert nodes[16] == 0
    nodes[4:8] = np.int32(nn + 5).tobytes()
    buf = ctypes.create_string_buffer(bytes(nodes), len(nodes))
    rt.check(rt.lib().rt_upload(s.kd_tree.nodes, buf, len(nodes)))
    h = ctypes.c_void_p()
    rc = rt.lib().rt_scene_prepare(ctypes.byref(s), ctypes.byref(h))
    assert rc == -1 and b"outside the node allocation" in rt.lib().rt_last_error()
    for p in (s.triangles, s.light_indicies, s.kd_tree.nodes, s.kd_tree.triangle_indicies):
        rt.lib().rt_free(p)
