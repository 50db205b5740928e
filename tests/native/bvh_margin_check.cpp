// bvh_margin_check.cpp — stress test of the conservative BVH margins
// (csrc/host/bvh_build.h): for adversarial triangles (regular, slivers,
// needles, large axis-aligned walls, far from the origin) and rays aimed at
// and around them (grazing, axis-parallel, from far away), every triangle
// test that passes with the reference arithmetic (rt/trace_ray.cuh:48-113,
// the same float operations as the GPU: bvh_common.h) must NOT be culled by
// the slab test of the triangle's grown box with best = s.  Reports the
// largest fraction of the margin a hit point actually used (the slack), and
// checks that triangles left out (NaN margin) never pass.  Also checks the
// written-out bound (bvh_build.h tri_margin_bound): every exact
// hit point lies within it (the derivation holds on these cases), and the
// shipped margins — tri_margin + rt_ray_margin — are at least that bound for
// every finite-margin triangle and any origin (the culling is proven safe,
// not only sampled); reports the smallest ratio shipped / proven.
//
// Build: g++ -O2 -std=c++17 -ffp-contract=off -fno-fast-math -I include -I csrc ...
// Usage: bvh_margin_check [pairs_millions] [seed]; exit 0 = no violation.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>

#include "host/bvh_build.h"

using rt_host::tri_margin;

namespace {

struct Rec {
    RtF4 A, B, C, D;
    float rd;
};

Rec prepare(Vec3D p1, Vec3D p2, Vec3D p3) // scene_prepare.cpp's per-triangle constants
{
    Rec r;
    Vec3D v0 = p2 - p1, v1 = p3 - p1;
    Vec3D n = rt_normalize(rt_cross(v0, v1));
    float d = rt_dot(n, p1);
    float d00 = rt_dot(v0, v0), d01 = rt_dot(v0, v1), d11 = rt_dot(v1, v1);
    r.rd = 1.0f / (d00 * d11 - d01 * d01);
    r.A = RtF4{n.x, n.y, n.z, d};
    r.B = RtF4{p1.x, p1.y, p1.z, d00};
    r.C = RtF4{v0.x, v0.y, v0.z, d01};
    r.D = RtF4{v1.x, v1.y, v1.z, d11};
    return r;
}

struct Stats {
    long long pairs = 0, passes = 0, violations = 0, nan_tris = 0, nan_passes = 0, inf_tris = 0, tris = 0;
    double max_used = 0.0; // largest (distance of the exact hit point outside the vertex box) / (margin + ray margin)
    long long bound_fails = 0;    // exact hit points outside the proven bound (must be 0)
    long long margin_short = 0;   // triangles whose shipped margin is below the proven bound (must be 0)
    long long bound_inf = 0;      // finite shipped margin but no proven bound (must be 0)
    double min_ratio = INFINITY;  // smallest (tri_margin + rt_ray_margin) / proven bound
    double max_bound_used = 0.0;  // largest (distance outside the vertex box) / proven bound
};

std::mt19937_64 rng;
double U(double a, double b) { return std::uniform_real_distribution<double>(a, b)(rng); }
Vec3D V(double a, double b) { return rt_v3((float)U(a, b), (float)U(a, b), (float)U(a, b)); }
double logU(double lo, double hi) { return exp(U(log(lo), log(hi))); }

Vec3D unit()
{
    while (true) {
        Vec3D v = V(-1, 1);
        double l = (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z;
        if (l > 1e-6 && l <= 1.0) return rt_normalize(v);
    }
}

void check_triangle(Vec3D p1, Vec3D p2, Vec3D p3, int rays, Stats &st)
{
    ++st.tris;
    const Rec r = prepare(p1, p2, p3);
    const float m = tri_margin(p1, p2 - p1, p3 - p1, r.rd, r.A.x, r.A.y, r.A.z);
    if (m != m) ++st.nan_tris;
    if (isinf(m)) {
        ++st.inf_tris;
        return; // the whole-scene box: not culled by construction
    }
    float lo[3] = {fminf(fminf(p1.x, p2.x), p3.x), fminf(fminf(p1.y, p2.y), p3.y), fminf(fminf(p1.z, p2.z), p3.z)};
    float hi[3] = {fmaxf(fmaxf(p1.x, p2.x), p3.x), fmaxf(fmaxf(p1.y, p2.y), p3.y), fmaxf(fmaxf(p1.z, p2.z), p3.z)};
    float glo[3], ghi[3];
    for (int a = 0; a < 3; ++a) {
        glo[a] = nextafterf(lo[a] - m, -INFINITY);
        ghi[a] = nextafterf(hi[a] + m, INFINITY);
    }
    // the scene: at least this triangle; sometimes a larger one around it
    double scale = 0.0;
    for (Vec3D p : {p1, p2, p3}) scale = fmax(scale, fabs((double)p.x) + fabs((double)p.y) + fabs((double)p.z));
    if (U(0, 1) < 0.3) scale *= logU(1.0, 50.0);
    const float fscale = (float)scale;
    const double L = fmax(fmax(fabs((double)hi[0] - lo[0]), fabs((double)hi[1] - lo[1])), fabs((double)hi[2] - lo[2]));
    // the shipped margins against the proven bound, for origins from 0 to far beyond the scene
    // (both sides are affine in |o|_1: the ends and the scene's own range decide)
    if (m == m) {
        for (double on1 : {0.0, (double)fscale, 3.0 * fscale, 1e3 * fscale, 1e6 * fscale + 1.0}) {
            const double pb = rt_host::tri_margin_bound(p1, p2 - p1, p3 - p1, r.rd, on1, 3.0 * fscale);
            if (isinf(pb)) {
                ++st.bound_inf;
                continue;
            }
            // the per-ray margin as the traversal computes it for an origin with |o|_1 = on1
            const float of = (float)(on1 / 3.0);
            const double shipped = (double)m + (double)rt_ray_margin(of, of, of, fscale);
            st.min_ratio = fmin(st.min_ratio, shipped / pb);
            if (shipped < pb) ++st.margin_short;
        }
    }
    for (int k = 0; k < rays; ++k) {
        ++st.pairs;
        // target: a point near the triangle (barycentrics slightly outside [0, 1] too)
        double b1 = U(0, 1), b2 = U(0, 1);
        if (b1 + b2 > 1) {
            b1 = 1 - b1;
            b2 = 1 - b2;
        }
        const int mode = (int)U(0, 6);
        if (mode == 0) { // on an edge or vertex, pushed out a little
            const double e = (U(0, 1) < 0.5 ? -1 : 1) * logU(1e-9, 1e-3);
            if (U(0, 1) < 0.5) b1 = e; else b2 = e;
        }
        const double b0 = 1 - b1 - b2;
        double tx = b0 * p1.x + b1 * p2.x + b2 * p3.x, ty = b0 * p1.y + b1 * p2.y + b2 * p3.y,
               tz = b0 * p1.z + b1 * p2.z + b2 * p3.z;
        // origin: near, far, grazing (close to the plane), inside the scene
        Vec3D o;
        double dist = (mode == 1) ? logU(1e-4, 1e-1) * (L + 1e-3) : logU(1e-3, 4.0) * (scale + 1e-3);
        Vec3D u = unit();
        if (mode == 2) { // grazing: direction almost in the plane
            const Vec3D n = rt_v3(r.A.x, r.A.y, r.A.z);
            const float c = rt_dot(u, n);
            u = rt_normalize(u - c * n + (float)(logU(1e-7, 1e-2) * (U(0, 1) < 0.5 ? -1 : 1)) * n);
        }
        o = rt_v3((float)(tx + dist * u.x), (float)(ty + dist * u.y), (float)(tz + dist * u.z));
        Vec3D d = rt_normalize(rt_v3((float)(tx - o.x), (float)(ty - o.y), (float)(tz - o.z)));
        if (mode == 3) { // axis-parallel component(s)
            const int a = (int)U(0, 3);
            if (a == 0) d.x = 0.0f; else if (a == 1) d.y = 0.0f; else d.z = 0.0f;
            if (U(0, 1) < 0.3) { if (a == 0) d.y = 0.0f; else d.x = 0.0f; }
            d = rt_normalize(d);
            if (d.x != d.x) continue;
        }
        float s;
        if (!rt_tri_plane(r.A, o, d, INFINITY, s)) continue;
        float cx, cy, cz;
        if (!rt_tri_bary(r.B, r.C, r.D, r.rd, o, d, s, cx, cy, cz)) continue;
        ++st.passes;
        if (m != m) {
            ++st.nan_passes;
            continue;
        }
        const float mr = rt_ray_margin(o.x, o.y, o.z, fscale);
        const RtSlab sl = rt_slab(o, d, mr);
        float tn;
        const bool kept = rt_bvh_box(glo[0], glo[1], glo[2], ghi[0], ghi[1], ghi[2], sl, s, tn);
        // the slack: how far outside the vertex box the exact hit point lies
        const double P[3] = {(double)o.x + (double)d.x * s, (double)o.y + (double)d.y * s, (double)o.z + (double)d.z * s};
        double out = 0.0;
        for (int a = 0; a < 3; ++a) out = fmax(out, fmax(lo[a] - P[a], P[a] - hi[a]));
        const double used = out / ((double)m + mr);
        if (used > st.max_used) st.max_used = used;
        const double on1 = fabs((double)o.x) + fabs((double)o.y) + fabs((double)o.z);
        const double pb = rt_host::tri_margin_bound(p1, r.C.x == r.C.x ? rt_v3(r.C.x, r.C.y, r.C.z) : p2 - p1,
                                                    rt_v3(r.D.x, r.D.y, r.D.z), r.rd, on1, 3.0 * fscale);
        if (!isinf(pb)) {
            st.max_bound_used = fmax(st.max_bound_used, out / pb);
            if (out > pb && ++st.bound_fails <= 10)
                fprintf(stderr, "BOUND FAIL: tri (%a %a %a) (%a %a %a) (%a %a %a) o (%a %a %a) d (%a %a %a) out %g bound %g\n",
                        p1.x, p1.y, p1.z, p2.x, p2.y, p2.z, p3.x, p3.y, p3.z, o.x, o.y, o.z, d.x, d.y, d.z, out, pb);
        }
        if (!kept) {
            if (++st.violations <= 10)
                fprintf(stderr,
                        "VIOLATION: tri (%a %a %a) (%a %a %a) (%a %a %a) o (%a %a %a) d (%a %a %a) s %a m %g mr %g "
                        "used %g\n",
                        p1.x, p1.y, p1.z, p2.x, p2.y, p2.z, p3.x, p3.y, p3.z, o.x, o.y, o.z, d.x, d.y, d.z, s, m, mr,
                        used);
        }
    }
}

} // namespace

int main(int argc, char **argv)
{
    const double millions = argc > 1 ? atof(argv[1]) : 2.0;
    rng.seed(argc > 2 ? strtoull(argv[2], nullptr, 10) : 12345);
    Stats st;
    const long long target = (long long)(millions * 1e6);
    const int rays = 64;
    while (st.pairs < target) {
        const int cls = (int)U(0, 5);
        const double L = logU(1e-3, 20.0);
        const Vec3D c = (U(0, 1) < 0.5) ? V(-2, 2) : V(-200, 200);
        Vec3D p1, p2, p3;
        if (cls == 0) { // regular
            p1 = c + (float)L * V(-1, 1);
            p2 = c + (float)L * V(-1, 1);
            p3 = c + (float)L * V(-1, 1);
        } else if (cls == 1) { // sliver: third vertex close to the first edge
            Vec3D u = unit(), w = unit();
            const float eps = (float)(L * logU(1e-7, 1e-1));
            p1 = c;
            p2 = c + (float)L * u;
            p3 = c + (float)(L * U(0, 1)) * u + eps * w;
        } else if (cls == 2) { // needle: two vertices close together
            Vec3D u = unit(), w = unit();
            p1 = c;
            p2 = c + (float)L * u;
            p3 = p2 + (float)(L * logU(1e-7, 1e-1)) * w;
        } else if (cls == 3) { // axis-aligned wall (room-style quads), large
            const int a = (int)U(0, 3);
            const float W = (float)(L * 5);
            Vec3D e1 = rt_v3(a == 0 ? 0.0f : W, a == 0 ? W : 0.0f, 0.0f);
            Vec3D e2 = rt_v3(0.0f, a == 2 ? W : 0.0f, a == 2 ? 0.0f : W);
            p1 = c;
            p2 = c + e1;
            p3 = c + e2;
        } else { // tiny triangle far from the origin
            const Vec3D far = V(-1000, 1000);
            const float l = (float)logU(1e-4, 1e-1);
            p1 = far;
            p2 = far + l * unit();
            p3 = far + l * unit();
        }
        check_triangle(p1, p2, p3, rays, st);
    }
    printf("pairs %lld passes %lld violations %lld tris %lld nan_tris %lld nan_passes %lld inf_tris %lld max_used %.3g "
           "bound_fails %lld margin_short %lld bound_inf %lld min_ratio %.4g max_bound_used %.4g\n",
           st.pairs, st.passes, st.violations, st.tris, st.nan_tris, st.nan_passes, st.inf_tris, st.max_used,
           st.bound_fails, st.margin_short, st.bound_inf, st.min_ratio, st.max_bound_used);
    return st.violations == 0 && st.nan_passes == 0 && st.bound_fails == 0 && st.margin_short == 0 &&
                   st.bound_inf == 0
               ? 0
               : 1;
}
