// bvh_common.h — arithmetic shared by the BVH-bounded traversal
// (bvh_trace.h, device), its builder (host/bvh_build.*) and the margin
// stress test (tests/native/bvh_margin_check.cpp), so that all three run
// exactly the same float operations (-ffp-contract=off everywhere).
#pragma once
#include "rt_device.h"
#include "rt_vecmath.h"

// Per-ray part of the conservative margin (host/bvh_build.h): the origin's
// share of a passing test's plane-distance error, the rounding of o + d*s
// and of the slab test; `scale` = the scene's largest |vertex|_1.
RT_HD float rt_ray_margin(float ox, float oy, float oz, float scale)
{
    return 0x1p-16f * (fabsf(ox) + fabsf(oy) + fabsf(oz) + 2.0f * scale);
}

// whether v is one of the sorted values vals[lo, hi) (float ==: -0 == +0)
RT_HD bool rt_sorted_contains(const float *vals, int lo, int hi, float v)
{
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const float m = vals[mid];
        if (m == v) return true;
        if (m < v) lo = mid + 1;
        else hi = mid;
    }
    return false;
}

// Whether the bound applies to this ray.  The skip rule needs every KD
// split distance t = (split - o) / d to be a number (+-inf allowed): then
// the exits inside a near subtree never exceed its split distance.  Only a
// ray lying IN a split plane (direction component exactly 0, origin
// coordinate == the split value) makes t = 0 / 0 = NaN; the reference then
// pushes with NaN, and later pushes inside that subtree can carry exits
// beyond the split (its leaf order is no longer front to back).  So a ray
// with a zero component is checked against the tree's split values on that
// axis (`splits`: per axis sorted, `off[a]..off[a+1]`); one lying in a split
// plane (and any non-finite ray) takes the plain KD traversal.  About 0.2 % of
// room2m's rays have a zero component; lying in a split plane is rarer still.
// (Also an origin beyond 2^64 in |o|_1 takes the plain traversal: the slab
// test's per-ray products, rt_slab, stay finite below it.)
RT_HD bool rt_bounded_ray(Vec3D o, Vec3D d, const float *splits, const int *off)
{
    if (!(o.x - o.x == 0.0f && o.y - o.y == 0.0f && o.z - o.z == 0.0f && d.x - d.x == 0.0f && d.y - d.y == 0.0f &&
          d.z - d.z == 0.0f))
        return false;
    if (!(fabsf(o.x) + fabsf(o.y) + fabsf(o.z) < 0x1p64f)) return false;
    if (d.x == 0.0f && rt_sorted_contains(splits, off[0], off[1], o.x)) return false;
    if (d.y == 0.0f && rt_sorted_contains(splits, off[1], off[2], o.y)) return false;
    if (d.z == 0.0f && rt_sorted_contains(splits, off[2], off[3], o.z)) return false;
    return true;
}

// The slab test's per-ray constants: inv = 1 / d clamped to [-2^60, 2^60],
// lo = -(om * inv) and hi = -(op * inv) for om = o + margin, op = o - margin,
// so that a face costs one fma (rt_bvh_box).  Finite: |inv| <= 2^60, and
// |om|, |op| < 2^65 (rt_bounded_ray: |o|_1 < 2^64; scene_prepare: scale <
// 2^64).  Its rounding, u|om inv| + u|lx inv - om inv| in t, is the slab
// term 3u(|box|_1 + |o|_1) of the margin's derivation as
// the form (lx - om) * inv's was.  The clamp changes only axes with |d| <
// 2^-60: over the query (t <= the scene box's exit, <= 6 scale) such a ray
// moves < 2^-57 scale along the axis, so a hit point in the box leaves its
// origin inside the grown slab by more than margin / 2, and the clamped
// interval there still spans beyond +-2^42 scale (no cull); an origin
// closer to a grown face has no hit point in that box to lose.
struct RtSlab {
    Vec3D inv, lo, hi;
};
RT_HD RtSlab rt_slab(Vec3D o, Vec3D d, float m)
{
    const float H = 0x1p60f;
    RtSlab r;
    r.inv = rt_v3(fminf(fmaxf(1.0f / d.x, -H), H), fminf(fmaxf(1.0f / d.y, -H), H), fminf(fmaxf(1.0f / d.z, -H), H));
    r.lo = rt_v3(-((o.x + m) * r.inv.x), -((o.y + m) * r.inv.y), -((o.z + m) * r.inv.z));
    r.hi = rt_v3(-((o.x - m) * r.inv.x), -((o.y - m) * r.inv.y), -((o.z - m) * r.inv.z));
    return r;
}

// Slab test of a box grown by the ray's margin (rt_slab).  True when the
// ray's [0, best] may meet the box, with tn its entry distance.
RT_HD bool rt_bvh_box(float lx, float ly, float lz, float hx, float hy, float hz, const RtSlab &r, float best,
                      float &tn)
{
    const float ax = fmaf(lx, r.inv.x, r.lo.x), bx = fmaf(hx, r.inv.x, r.hi.x);
    const float ay = fmaf(ly, r.inv.y, r.lo.y), by = fmaf(hy, r.inv.y, r.hi.y);
    const float az = fmaf(lz, r.inv.z, r.lo.z), bz = fmaf(hz, r.inv.z, r.hi.z);
    tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    return tn <= tf && tf >= 0.0f && tn <= best;
}

// intersect_triangle's plane part (rt/trace_ray.cuh:73-96) on the
// precomputed plane A = {n, dot(n, p1)}: s, and whether the test goes on
// (dn != 0, s >= 1e-5, s < closest)
RT_HD bool rt_tri_plane(RtF4 A, Vec3D o, Vec3D d, float closest, float &s)
{
    const float dn = d.x * A.x + d.y * A.y + d.z * A.z;
    s = (A.w - (o.x * A.x + o.y * A.y + o.z * A.z)) / dn;
    return dn != 0 && s >= 0.00001f && s < closest;
}

// calculate_barycentric_coordinates + the range test (rt/trace_ray.cuh:48-71,
// :97-110) on the precomputed record {p1, d00}, {v0, d01}, {v1, d11}, 1/den
RT_HD bool rt_tri_bary(RtF4 B, RtF4 C, RtF4 D, float rd, Vec3D o, Vec3D d, float s, float &cx, float &cy, float &cz)
{
    const float px = o.x + d.x * s, py = o.y + d.y * s, pz = o.z + d.z * s;
    const float v2x = px - B.x, v2y = py - B.y, v2z = pz - B.z;
    const float d20 = v2x * C.x + v2y * C.y + v2z * C.z;
    const float d21 = v2x * D.x + v2y * D.y + v2z * D.z;
    cy = (D.w * d20 - C.w * d21) * rd;
    cz = (B.w * d21 - C.w * d20) * rd;
    cx = 1.0f - cy - cz;
    return rt_bary_inside(cx, cy, cz);
}
