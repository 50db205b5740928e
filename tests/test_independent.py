"""The oracle's BSDF, NEE and KD builder against second, independent
restatements of the reference (tests/independent.py, numpy float32).  The GPU
path is pinned bit for bit to the oracle elsewhere (test_gpu_parity.py), so an
agreement here carries over to it.  CPU only."""
import ctypes

import numpy as np
import pytest

import helpers
import independent as ind
import oracle
import rt

f32 = np.float32


def _unit(rng, n):
    v = rng.normal(size=(n, 3)).astype(f32)
    return ind.normalize(v)


def _frames(rng, n):
    """normal / tangent / bitangent as trace_leaf_node builds them (rt/trace_ray.cuh:148-150)."""
    nrm = _unit(rng, n)
    edge = _unit(rng, n)
    tan = ind.normalize(ind.cross(edge, nrm))
    bit = ind.normalize(ind.cross(nrm, tan))
    return nrm, tan, bit


def _same(a, b):
    a, b = np.asarray(a, f32), np.asarray(b, f32)
    both_nan = np.isnan(a) & np.isnan(b)
    return (a.view(np.uint32) == b.view(np.uint32)) | both_nan


def test_scatter_matches_independent_restatement():
    """get_scattered_light (rt/path_tracing.cuh:151-219) on 60,000 random
    samples covering every branch: metallic (fresnel_conductor), dielectric
    specular from outside and inside (total internal reflection included),
    transmission (refraction_direction, inside flips) and diffuse
    (diffuse_direction); the FP64 island of microfacet_normal."""
    g = np.random.default_rng(1234)
    N = 60_000
    d = _unit(g, N)
    nrm, tan, bit = _frames(g, N)
    # the reference flips the shading normal against the incoming ray (:153-156)
    flip = ind.dot(d, nrm) > 0
    nrm = np.where(flip[:, None], -nrm, nrm).astype(f32)
    bit = ind.normalize(ind.cross(nrm, tan))
    albedo = g.uniform(0, 1, (N, 3)).astype(f32)
    rough = g.choice(np.array([0.001, 0.05, 0.3, 0.7, 1.0], f32), N) * g.uniform(0.5, 1, N).astype(f32)
    rough = rough.astype(f32)
    ior = g.uniform(1.0, 2.6, N).astype(f32)
    ext = np.where(g.uniform(size=N) < 0.3, g.uniform(0.05, 4, N), 0).astype(f32)
    transparent = g.uniform(size=N) < 0.5
    inside = g.uniform(size=N) < 0.4
    pos = g.uniform(-3, 3, (N, 3)).astype(f32)
    state = g.integers(0, 2 ** 32, N, dtype=np.uint64).astype(np.uint32)

    o_pos, o_dir, o_w, o_type, o_in, o_rng = ind.scatter(d, inside, state, albedo, rough, ior, ext, transparent, pos,
                                                         nrm, tan, bit)
    L = oracle.lib()
    out = np.zeros(12, f32)
    smp = np.zeros(22, f32)
    r_out, in_out, ty_out = ctypes.c_uint32(), ctypes.c_int(), ctypes.c_int()
    got_dir = np.zeros((N, 3), f32)
    got_w = np.zeros((N, 3), f32)
    got_t = np.zeros(N, np.int64)
    got_in = np.zeros(N, bool)
    got_rng = np.zeros(N, np.uint32)
    for k in range(N):
        smp[0:3] = albedo[k]
        smp[6], smp[7], smp[8], smp[9] = rough[k], ior[k], ext[k], float(transparent[k])
        smp[10:13], smp[13:16], smp[16:19], smp[19:22] = pos[k], nrm[k], tan[k], bit[k]
        dk = np.ascontiguousarray(d[k])
        L.or_scatter(dk.ctypes.data, smp.ctypes.data, int(inside[k]), int(state[k]), out.ctypes.data,
                     ctypes.byref(r_out), ctypes.byref(in_out), ctypes.byref(ty_out))
        got_dir[k], got_w[k] = out[3:6], out[6:9]
        got_t[k], got_in[k], got_rng[k] = ty_out.value, bool(in_out.value), r_out.value
    assert np.array_equal(got_t, o_type)
    assert np.array_equal(got_in, o_in)
    assert np.array_equal(got_rng, o_rng)
    bad = ~(_same(got_dir, o_dir).all(axis=1) & _same(got_w, o_w).all(axis=1))
    assert not bad.any(), (np.nonzero(bad)[0][:5], got_dir[bad][:2], o_dir[bad][:2], got_w[bad][:2], o_w[bad][:2])
    # branch coverage
    for t in (ind.METALLIC, ind.SPECULAR, ind.TRANSMISSION, ind.DIFFUSE):
        assert (o_type == t).sum() > 1000, t
    assert ((o_type == ind.SPECULAR) & inside).sum() > 1000  # inside the medium: weight 1
    # total internal reflection: inside the medium, g clamps to 0, Fresnel = 1
    i = -d
    h = ind.microfacet_normal(*[ind.rng_next(s)[0] for s in (state, ind.rng_next(state)[1])], nrm, tan, bit, rough)
    c = np.abs(ind.dot(i, h))
    tir = inside & (ext == 0) & ((f32(1) / (ior * ior)) - f32(1) + c * c <= 0)
    assert tir.sum() > 1000 and np.all(o_type[tir] == ind.SPECULAR)


def test_direct_light_matches_independent_restatement():
    """sample_direct_light + random_point_in_triangle (rt/path_tracing.cuh:
    222-265) at 4,000 surface points of the Cornell box (lit, occluded and
    back-facing cases), the same shadow-ray tracer on both sides."""
    path = helpers.scene_path("cornell")
    osc = oracle.OracleScene(path)
    tris_raw, _, _, lights, bounds = osc.arrays()
    tris = np.frombuffer(tris_raw, np.uint8).reshape(-1, 152)
    g = np.random.default_rng(99)
    N = 4000
    cam = ((bounds[:3] + bounds[3:]) * f32(0.5)).astype(f32)  # inside the box
    rays = np.concatenate([np.repeat(cam[None], N, 0), _unit(g, N)], axis=1).astype(f32)
    hit = osc.trace_rays(rays)
    ok = hit[:, 0] == 1
    pos = hit[ok, 2:5].astype(f32)
    nrm = hit[ok, 5:8].astype(f32)
    n = len(pos)
    assert n > 2000  # the box is open at the front
    state = g.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)

    def trace(rays6):  # the Cornell box is untextured: a hit's emittance is its material's
        o = osc.trace_rays(rays6)
        tri = o[:, 1].astype(np.int64)
        emit = tris[np.maximum(tri, 0), 108:120].copy().view(f32).reshape(-1, 3)
        return o[:, 0] == 1, tri, o[:, 5:8].astype(f32), emit

    mine, mine_rng = ind.direct_light(tris, lights, trace, pos, nrm, state)
    got = np.zeros((n, 3), f32)
    got_rng = np.zeros(n, np.uint32)
    for k in range(n):
        got[k], got_rng[k] = osc.direct_light(pos[k], nrm[k], int(state[k]))
    assert np.array_equal(got_rng, mine_rng)
    assert _same(got, mine).all(), np.nonzero(~_same(got, mine).all(axis=1))[0][:8]
    lit = (mine > 0).any(axis=1).sum()
    assert 0.2 * n < lit < n  # both lit and unlit (occluded / facing away) points


@pytest.mark.parametrize("name", ["features", "cornell", "room_small", "cornell_blob"])
def test_kd_builder_matches_independent_restatement(name):
    """create_kd_tree (rt/create_kd_tree.cuh:18-328): node bytes (20-B
    reference layout), triangle_indicies and the bounding box of an
    independent numpy restatement equal the oracle's and the product's
    (csrc/host/kd_build.cpp)."""
    import os

    path = (os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "features", "scene.txt")
            if name == "features" else helpers.scene_path(name))
    osc = oracle.OracleScene(path)
    tris_raw, onodes, oidx, _, obounds = osc.arrays()
    tris = np.frombuffer(tris_raw, np.uint8).reshape(-1, 152)
    nodes, idx, bounds = ind.create_kd_tree(tris)
    assert len(nodes) == len(onodes)
    assert nodes == onodes
    np.testing.assert_array_equal(idx, oidx)
    np.testing.assert_array_equal(bounds, obounds)
    hs = rt.HostScene(path)
    ptr, cnt = hs.triangle_ptr()
    pnodes, pidx, pbounds = rt.build_kd_tree(ptr, cnt)
    assert pnodes == nodes
    np.testing.assert_array_equal(pidx, idx)
    np.testing.assert_array_equal(np.array(pbounds, f32), bounds)
