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

// A proven bound (DESIGN.md §5 "The margin, derived") on the inf-norm
// distance from the triangle's vertex box of the EXACT point o + s*d of any
// passing test (rt_tri_plane + rt_tri_bary, the reference's arithmetic on
// these precomputed floats) of a ray with |o|_1 <= on1 (any direction), plus
// the slab test's own rounding at a box whose corners have |.|_1 <= box1 (so
// that tri_margin + rt_ray_margin
// >= this value means the culling never drops a passing test).  Standard
// rounding-error analysis (gamma_k = k u / (1 - k u), u = 2^-24, every float
// operation of the test and of the precomputation), evaluated in double and
// inflated by 1e-6 relative; +inf when its conditioning premise fails.  Not
// used by the build: tests/native/bvh_margin_check.cpp and bvh_trace_check.cpp
// check tri_margin + rt_ray_margin against it for every triangle they see.
inline double tri_margin_bound(Vec3D p1, Vec3D v0, Vec3D v1, float rd, double on1, double box1)
{
    const double u = 0x1p-24;
    auto gam = [&](double k) { return k * u / (1.0 - k * u); };
    const double g2 = gam(2), g3 = gam(3);
    const double l0 = sqrt((double)v0.x * v0.x + (double)v0.y * v0.y + (double)v0.z * v0.z);
    const double l1 = sqrt((double)v1.x * v1.x + (double)v1.y * v1.y + (double)v1.z * v1.z);
    const double L = l0 > l1 ? l0 : l1;
    if (!(L > 0.0) || !isfinite(rd)) return INFINITY;
    const double kappa = L * L * L * L * fabs((double)rd); // ~ 1 / sin^2 of the triangle's angles
    // |d_ij - v_i.v_j| <= g3 L^2, product / difference roundings: the Cramer
    // numerators and den = d00 d11 - d01^2 are off by at most a1 R L^3 / a1 L^4
    const double a1 = 2.0 * g3 * (2.0 + g3) + 2.0 * g2 * (1.0 + g3) * (1.0 + g3);
    const double b = u + a1 * kappa * (1.0 + u) * (1.0 + u); // |rd * det G - 1|
    if (!(b < 0.25)) return INFINITY;
    const double bp = b + u * (1.0 + b);
    const double c = (1.0 + u) * a1 * kappa;
    const double D = 1.0 - bp - 2.0 * c;
    if (!(D > 0.5)) return INFINITY;
    // angle of the stored normal n = normalize(cross(v0, v1)) to the exact one
    const double tau = 1.5708 * g2 * sqrt(2.0 * kappa / (1.0 - b)) + 4.0 * u;
    const double p1n = fabs((double)p1.x) + fabs((double)p1.y) + fabs((double)p1.z);
    const double s3 = 1.7320508075688772;
    // R = |v2| (v2 = fl(P - p1)): R <= 2 (1 + delta) L + h', where delta bounds
    // the barycentric error and h' the distance of p1 + v2 from the plane;
    // F below is that bound as a (monotone, contracting) function of R
    double hp = 0, eP = 0, eV = 0, delta = 0;
    auto F = [&](double R) {
        // |X|_1 <= |p1|_1 + sqrt3 |X - p1|, |X - p1| <= R (1 + 3u) + e_P; e_P = |P - X| (P = fl(o + fl(d s)))
        double e = 0.0;
        for (int it = 0; it < 4; ++it) {
            const double xn = p1n + s3 * (R * (1.0 + 3.0 * u) + e);
            const double sdn = xn + on1; // |s| |d|_1 = |X - o|_1
            e = g2 * (sdn + xn) * (1.0 + 1e-9);
        }
        eP = e;
        const double xn = p1n + s3 * (R * (1.0 + 3.0 * u) + eP), sdn = xn + on1;
        eV = u * R * (1.0 + 3.0 * u); // v2 = fl(P - p1)
        // n.(X - p1) for the plane test's s: the roundings of w = n.p1, n.o, d.n, num and num / dn
        const double A0 = g2 * (1.0 + g3) * (1.0 + 4.0 * u) * (p1n + on1) +
                          g3 * (1.0 + 4.0 * u) * (on1 + p1n + sdn);
        hp = A0 + tau * (R * (1.0 + 3.0 * u) + eP) + eP + eV;
        delta = (c * (2.0 + hp / L) + bp) / D;
        return 2.0 * (1.0 + delta) * L + hp;
    };
    double R = 2.0 * L;
    for (int it = 0; it < 200; ++it) R = F(R);
    R = R * (1.0 + 1e-9) + 1e-30;
    if (!(F(R) <= R)) return INFINITY; // (no contraction: the premise fails)
    (void)F(R);
    // Q = p1 + cy v0 + cz v1 lies in the triangle grown by u (cy, cz >= 0,
    // cy + cz <= 1 + u), whose vertex box is within u L of the real one
    const double dist = 2.0 * u * L + eP + eV + hp + 2.0 * delta * L;
    // the slab test's rounding at a box within box1 (|corner|_1) of the origin
    const double slab = 3.0 * u * (box1 + on1);
    return (dist + slab) * (1.0 + 1e-6) + 1e-30;
}

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

// the 4-wide collapse of a binary BVH (nodes as BvhHost::nodes): the same
// boxes and leaves, half the levels — what the device's s_min query walks
// (bvh_trace.h bvh_bound).  8 RtF4 per node (SoA of 4 children: lo.x, lo.y,
// lo.z, hi.x, hi.y, hi.z, references, padding).
void collapse_bvh4(const std::vector<RtF4> &bin, std::vector<RtF4> &out4);

} // namespace rt_host
