"""Second, independent restatements of reference functions (TEST
INFRASTRUCTURE ONLY), written directly from the reference source in numpy
float32 (float64 only where the reference computes in double), without
looking at or calling oracle/rt_oracle.c.  tests/test_independent.py checks
the oracle (and through it the GPU path, which is bit-identical to the oracle)
against these on randomized inputs: a misreading of the reference shared by
the oracle and the kernels would have to be made a third time, the same way,
to go unnoticed.

Covered (reference = INDA23PlusPlus/isaklm-raytracer):
  * get_random_unilateral          rt/path_tracing.cuh:34-43
  * get_scattered_light + helpers  rt/path_tracing.cuh:45-219
    (diffuse_direction, fresnel_dielectric, fresnel_conductor,
     microfacet_normal with its FP64 island, lambda, specular_weight,
     specular_direction, refraction_direction)
  * random_point_in_triangle, sample_direct_light  rt/path_tracing.cuh:222-265
  * create_kd_tree + helpers       rt/create_kd_tree.cuh:18-328
"""
import struct

import numpy as np

f32 = np.float32
PI = f32(3.1415926536)  # rt/math_library.cuh:9
TAU = f32(PI * f32(2))  # :10
DIFFUSE, SPECULAR, METALLIC, TRANSMISSION = 1, 2, 3, 4  # Ray_Type (rt/path_tracing.cuh:18-25)


# ---------------------------------------------------------------- basics
def sinf(x):
    """Correctly rounded sinf (what the reference's sinf is taken to return)."""
    return np.sin(np.asarray(x, np.float64)).astype(f32)


def cosf(x):
    return np.cos(np.asarray(x, np.float64)).astype(f32)


def dot(a, b):
    """((x*x' + y*y') + z*z') on (..., 3) float32 arrays (rt/math_library.cuh:212-215)."""
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def sv(s, v):
    """float * Vec3D, per component."""
    return v * s[..., None]


def normalize(v):
    r = f32(1) / np.sqrt(dot(v, v))
    return sv(r, v)


def cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1], a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], axis=-1)


def rng_next(state):
    """get_random_unilateral on a uint32 array; returns (xi float32, new state)."""
    s = state.astype(np.uint64)
    s = (s * 747796405 + 2891336453) & 0xFFFFFFFF
    word = (((s >> ((s >> 28) + 4)) ^ s) * 277803737) & 0xFFFFFFFF
    r = ((word >> 22) ^ word) & 0xFFFFFFFF
    # float(r) / UINT32_MAX: both operands converted to float (UINT32_MAX -> 2^32)
    return r.astype(np.uint32).astype(f32) / f32(4294967295.0), r.astype(np.uint32)


# ---------------------------------------------------------------- BSDF
def microfacet_normal(xi1, xi2, n, t, b, rough):
    """:103-118.  `double random_unilateral` — the quotient is evaluated in
    double and converted to float by sqrtf's parameter."""
    ru = xi1.astype(np.float64)
    q = (1.0 - ru) / (ru * (rough * rough - f32(1)).astype(np.float64) + 1.0)
    cos_t = np.sqrt(q.astype(f32))
    sin_t = np.sqrt(f32(1) - cos_t * cos_t)
    phi = xi2 * TAU
    cp, sp = cosf(phi), sinf(phi)
    return (sv(cp, sv(sin_t, t)) + sv(cos_t, n)) + sv(sp, sv(sin_t, b))


def fresnel_dielectric(i, h, n1, n2):  # :61-73
    c = np.abs(dot(i, h))
    g = np.sqrt(np.fmax((n2 * n2) / (n1 * n1) - f32(1) + c * c, f32(0)))
    x = (g - c) / (g + c)
    f1 = f32(0.5) * (x * x)
    y = (c * (g + c) - f32(1)) / (c * (g - c) + f32(1))
    return f1 * (f32(1) + y * y)


def fresnel_conductor(i, h, n, k):  # :75-101
    n2, k2 = n * n, k * k
    ct = dot(i, h)
    ct2 = ct * ct
    st2 = f32(1) - ct2
    t0 = n2 - k2 - st2
    ab = np.sqrt(t0 * t0 + f32(4) * n2 * k2)
    a = np.sqrt(f32(0.5) * (ab + t0))
    t1 = ab + ct2
    t2 = f32(2) * a * ct
    rs = (t1 - t2) / (t1 + t2)
    t3 = ct2 * ab * (st2 * st2)
    t4 = t2 * st2
    rp = rs * (t3 - t4) / (t3 + t4)
    return (rs + rp) * f32(0.5)


def lam(d, n, rough):  # :120-127
    dn = dot(d, n)
    dn2 = dn * dn
    with np.errstate(divide="ignore", invalid="ignore"):
        tan2 = (f32(1) - dn2) / dn2
    return (np.sqrt(f32(1) + rough * rough + tan2) - f32(1)) * f32(0.5)


def specular_weight(i, o, h, n, rough):  # :129-136
    g = f32(1) / (f32(1) + lam(i, n, rough) + lam(o, n, rough))
    return np.abs(dot(i, h)) * g / np.abs(dot(n, h) * np.abs(dot(i, n)))


def specular_direction(i, h):  # :138-141
    return sv(f32(2) * dot(i, h), h) - i


def refraction_direction(i, h, n1, n2):  # :143-149
    c = dot(i, h)
    n = n1 / n2
    return sv(n * c - np.sqrt(np.fmax(f32(1) + n * n * (c * c - f32(1)), f32(0))), h) - sv(n, i)


def scatter(ray_dir, inside, rng, albedo, rough, ior, ext, transparent, pos, n, t, b):
    """get_scattered_light (:151-219) on arrays of N samples.  Returns
    (origin, direction, weight, type, inside, rng)."""
    i = -ray_dir
    xi1, rng = rng_next(rng)
    xi2, rng = rng_next(rng)
    h = microfacet_normal(xi1, xi2, n, t, b, rough)
    metal = ext > f32(0)
    # metallic reflection
    Fm = fresnel_conductor(i, h, ior, ext)
    o_spec = specular_direction(i, h)
    w_metal = sv(Fm, albedo * specular_weight(i, o_spec, h, n, rough)[..., None])
    # dielectric
    n1 = np.where(inside, ior, f32(1)).astype(f32)
    n2 = np.where(inside, f32(1), ior).astype(f32)
    Fd = fresnel_dielectric(i, h, n1, n2)
    choose, rng_d = rng_next(rng)
    spec = ~metal & (choose < Fd)
    w_spec = np.where(inside[:, None], f32(1), np.repeat(specular_weight(i, o_spec, h, n, rough)[:, None], 3, 1))
    trans = ~metal & ~spec & transparent
    o_tr = refraction_direction(i, h, n1, n2)
    w_tr = albedo * specular_weight(i, o_tr, h, n, rough)[..., None]
    diff = ~metal & ~spec & ~transparent
    phi, rng_x = rng_next(rng_d)
    ru, rng_y = rng_next(rng_x)
    sq = np.sqrt(ru)
    o_diff = (sv(sq * cosf(phi * TAU), t) + sv(np.sqrt(f32(1) - ru), n)) + sv(sq * sinf(phi * TAU), b)
    # (phi above is the raw draw; the angle is draw * TAU)
    direction = np.select([metal[:, None], spec[:, None], trans[:, None]], [o_spec, o_spec, o_tr], o_diff)
    weight = np.select([metal[:, None], spec[:, None], trans[:, None]], [w_metal, w_spec, w_tr], albedo)
    typ = np.select([metal, spec, trans], [METALLIC, SPECULAR, TRANSMISSION], DIFFUSE)
    inside_out = np.where(trans, ~inside, inside)
    rng_out = np.select([metal, diff], [rng, rng_y], rng_d)
    return pos, direction.astype(f32), weight.astype(f32), typ, inside_out, rng_out


# ---------------------------------------------------------------- NEE
def random_point_in_triangle(p1, p2, p3, rng):  # :222-233
    x, rng = rng_next(rng)
    y, rng = rng_next(rng)
    sx = np.sqrt(x)
    u = f32(1) - sx
    v = y * sx
    w = f32(1) - u - v
    return (sv(u, p1) + sv(v, p2)) + sv(w, p3), rng


def direct_light(tris, lights, trace, pos, normal, rng):
    """sample_direct_light (:235-265) at N points.  `tris` = (n, 152) uint8
    reference-layout triangles, `lights` = light_indicies, `trace(rays6)` a
    trace_ray returning (hit, triangle_index, surface normal, emittance) per
    ray — the emittance of the hit Sample, i.e. texture-modulated
    (sample_texture, rt/trace_ray.cuh:155), which is what the reference
    scales (:259), not the light's material emittance.  The reference reads
    light_indicies[light_count] when the draw is exactly 1.0:
    taken here as the last light."""
    xi, rng = rng_next(rng)
    nl = len(lights)
    if nl == 0:
        _, rng = rng_next(rng)
        _, rng = rng_next(rng)
        return np.zeros((len(pos), 3), f32), rng
    k = (xi * f32(nl)).astype(np.int64)
    li = np.asarray(lights, np.int64)[np.minimum(k, nl - 1)]
    P = tris[li, :36].copy().view(f32).reshape(-1, 3, 3)
    rp, rng = random_point_in_triangle(P[:, 0], P[:, 1], P[:, 2], rng)
    d = normalize(rp - pos)
    hit, tri, snorm, emit = trace(np.concatenate([pos, d], axis=1).astype(f32))
    e1, e2 = P[:, 1] - P[:, 0], P[:, 2] - P[:, 0]
    cr = cross(e1, e2)
    area = (0.5 * np.sqrt(dot(cr, cr)).astype(np.float64)).astype(f32)  # 0.5 is a double
    diff = rp - pos
    d2 = dot(diff, diff)
    c1 = np.fmax(-dot(d, snorm), f32(0))
    c2 = np.fmax(dot(d, normal), f32(0))
    s = area * f32(nl) * c1 * c2 / np.fmax(d2 * PI, f32(0.001))
    out = sv(s, emit)
    ok = hit & (tri == li)
    return np.where(ok[:, None], out, f32(0)).astype(f32), rng


# ---------------------------------------------------------------- KD builder
KD_TREE_DEPTH = 19  # rt/macros.h:11
MIN_TRIANGLE_COUNT = 7  # rt/create_kd_tree.cuh:221


def create_kd_tree(tris):
    """create_kd_tree (rt/create_kd_tree.cuh:269-328) on (n, 152) uint8
    triangles.  Returns (node bytes (20 B each, reference layout, zero
    padding), triangle_indicies int32, bounding box float32[6])."""
    P = tris[:, :36].copy().view(f32).reshape(-1, 3, 3)
    lo = np.fmin(P[:, 0], np.fmin(P[:, 1], P[:, 2]))  # fminf(p1, fminf(p2, p3)) per axis
    hi = np.fmax(P[:, 0], np.fmax(P[:, 1], P[:, 2]))
    mid = (lo + hi) * f32(0.5)
    nodes = [None]  # node 0: the root, filled by its add_child_nodes
    indices = []

    def leaf(tri_list):
        nodes.append((len(indices), len(tri_list), 0, f32(0), True))
        indices.extend(tri_list.tolist())

    def add_child_nodes(slot, tri_list, depth):  # :162-265, iterative over the two children
        axis = depth % 3
        vals = np.sort(mid[tri_list, axis], kind="stable")
        off = vals[len(vals) // 2]  # std::sort + middle element (:158-160)
        behind = tri_list[lo[tri_list, axis] <= off]  # triangle_behind_plane (:58-91)
        afore = tri_list[hi[tri_list, axis] >= off]  # triangle_afore_plane (:93-126)
        kids = []
        for child in (behind, afore):
            idx = len(nodes)
            kids.append(idx)
            if len(child) > MIN_TRIANGLE_COUNT and depth < KD_TREE_DEPTH:
                nodes.append(None)
                add_child_nodes(idx, child, depth + 1)
            else:
                leaf(child)
        nodes[slot] = (kids[0], kids[1], axis, off, False)

    add_child_nodes(0, np.arange(len(tris), dtype=np.int64), 0)
    raw = b"".join(struct.pack("<iiB3xf?3x", a, b, ax, float(o), lf) for a, b, ax, o, lf in nodes)
    eps = f32(0.01)
    bounds = np.concatenate([lo.min(axis=0) - eps, hi.max(axis=0) + eps]).astype(f32)  # get_bounding_box (:18-56)
    return raw, np.asarray(indices, np.int32), bounds
