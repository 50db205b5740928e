// bvh_build.h — the conservative BVH that bounds each ray's first hit
// (host side; the device traversal is bvh_trace.h).
//
// Why a second structure next to the reference's KD tree: trace_ray's
// result (rt/trace_ray.cuh:244-318) is defined by the KD traversal order —
// the first leaf, front to back, holding a triangle whose test passes with
// s < that leaf's exit, and the smallest (s, entry order) inside it.  Every
// triangle test is a pure function of (ray, triangle): it does not depend
// on the leaf.  So if s_min is the smallest s of ANY passing test in the
// scene, every leaf whose exit is <= s_min holds no hit and the reference
// tests it for nothing; the first leaf with exit > s_min is where the
// reference's answer starts.  The BVH finds s_min with the reference's own
// per-triangle arithmetic (bit-identical test), visiting a few dozen nodes
// instead of the KD traversal's ~650 node fetches and ~1,700 tests per ray.
//
// Exactness needs the BVH never to cull a triangle whose test passes with
// s < the current bound.  A passing test's hit point P = o + d*s (the float
// s, exact arithmetic) lies near the triangle, but not on it: the plane
// distance picks up the rounding of num / dn, and the barycentric test
// (rt/trace_ray.cuh:48-71) accepts points whose computed coordinates
// round into [0, 1].  tri_margin() bounds how far P can be from the
// triangle's vertex box for ANY ray through the scene; the leaf boxes are
// grown by it (and by a per-ray term for the origin, added at query time),
// so the culling is conservative.  Triangles whose bound is useless
// (slivers: the barycentric error is amplified by 1 / sin^2 of the angle
// and by the aspect ratio) get the whole scene box: always tested.
// Triangles that can never pass (a zero-area triangle's normal or 1/den is
// NaN / inf: every comparison fails) are left out.  tests/native/
// bvh_margin_check.cpp checks the bound against the reference arithmetic on
// adversarial rays and triangles.
#pragma once
#include <math.h>
#include <stdint.h>

#include <vector>

#include "../bvh_common.h"

namespace rt_host {

constexpr float kUlp = 0x1p-24f;

// margin of triangle (p1, v0 = p2 - p1, v1 = p3 - p1, rd = 1 / den) for
// rays through a scene whose coordinates are at most `scale` in |.|_1 (see
// bvh_build.h's head comment); +inf = the triangle needs the whole scene box;
// NaN = it can never pass a test (leave it out)
inline float tri_margin(Vec3D p1, Vec3D v0, Vec3D v1, float rd, float nx, float ny, float nz)
{
    if (!(fabsf(nx) <= 2.0f && fabsf(ny) <= 2.0f && fabsf(nz) <= 2.0f) || !isfinite(rd)) return NAN;
    const double l0 = sqrt((double)v0.x * v0.x + (double)v0.y * v0.y + (double)v0.z * v0.z);
    const double l1 = sqrt((double)v1.x * v1.x + (double)v1.y * v1.y + (double)v1.z * v1.z);
    const double L = l0 > l1 ? l0 : l1;
    // barycentric error per unit of |v2| scaled to the triangle: generous
    // (about 40x the first-order bound, see the head comment)
    const double E = 16384.0 * kUlp * L * L * L * L * fabs((double)rd) + 128.0 * kUlp;
    if (!(E < 0.125)) return INFINITY;
    const double p1n = fabs((double)p1.x) + fabs((double)p1.y) + fabs((double)p1.z);
    return (float)(8.0 * E * L + 256.0 * kUlp * (p1n + L) + 1e-30);
}

// (the per-ray margin, rt_ray_margin, is in bvh_common.h: the traversal adds it)

struct BvhHost {
    std::vector<RtF4> nodes;       // 4 per node (bvh_trace.h layout)
    std::vector<uint32_t> order;   // BVH leaf slot -> triangle index
    float scale = 0.0f;            // largest |coordinate|_1 of the scene (ray_margin)
    int depth = 0;
    int always = 0;                // triangles with the whole-scene box
    int dropped = 0;               // triangles that can never pass a test
};

// builds the BVH over the triangles' conservative boxes; planes / records
// are gathered into `order` by the caller
int build_bvh(const Triangle *tris, int ntris, const RtF4 *plane, const RtIsectBary *bary, BvhHost &out);

} // namespace rt_host
