// deep_ray_work.cpp — work per ray of a deep (total internal reflection)
// path's bounce on the host: rays from random points of the transparent
// triangles into the glass, at TIR-like angles.  Counts, per ray, the plain
// KD traversal's nodes / leaves / tests, the bounded traversal's BVH nodes /
// leaf visits and KD nodes, and the s_min query over an 8-wide collapse of the
// same BVH (node visits, visits that test leaves) — the dependent-load chains
// a lone ray pays.  Experiment tooling, not product code.
//
// usage: deep_ray_work scene.txt [rays] [seed]
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <vector>

#include "host/bvh_build.h"
#include "host/rt_host.h"

namespace {

float bitsf(uint32_t u)
{
    float f;
    memcpy(&f, &u, 4);
    return f;
}

bool test(const RtF4 *A, const RtIsectBary *R, uint32_t e, Vec3D o, Vec3D d, float closest, float &s)
{
    if (!rt_tri_plane(A[e], o, d, closest, s)) return false;
    float b[3];
    return rt_tri_bary(R[e].b, R[e].c, R[e].d, bitsf(R[e].rd), o, d, s, b[0], b[1], b[2]);
}

struct W {
    double kd_nodes = 0, kd_leaves = 0, kd_tests = 0, b_nodes = 0, b_leaves = 0, bk_nodes = 0, bk_leaves = 0,
           w_nodes = 0, w_leafvis = 0, w_tests = 0, n = 0;
};

bool box(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, float &t1, float &t2)
{
    const Bounding_Box &b = h.bounds;
    float a0 = (b.min.x - o.x) / d.x, a1 = (b.max.x - o.x) / d.x, b0 = (b.min.y - o.y) / d.y,
          b1 = (b.max.y - o.y) / d.y, c0 = (b.min.z - o.z) / d.z, c1 = (b.max.z - o.z) / d.z;
    t1 = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fminf(c0, c1));
    t2 = fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fmaxf(c0, c1));
    return t1 <= t2;
}

// KD traversal (rt/trace_ray.cuh:244-318) with the skip bound s_min (-inf: plain)
int kd(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, float entry, float exit_, float s_min, double &nodes,
       double &leaves, double &tests)
{
    struct E { uint32_t n; float e; } stk[64];
    int sp = 0;
    const float root_exit = exit_;
    uint32_t node = 0;
    while (true) {
        uint32_t x = h.nodes[2 * node], y = h.nodes[2 * node + 1];
        ++nodes;
        while ((y & 3u) != RT_LEAF_TAG) {
            const uint32_t a = y & 3u;
            const float split = bitsf(x), oa = a == 0 ? o.x : a == 1 ? o.y : o.z, da = a == 0 ? d.x : a == 1 ? d.y : d.z;
            uint32_t nc = node + 1, fc = y >> 2;
            if (oa >= split) std::swap(nc, fc);
            const float t = (split - oa) / da;
            if (t >= exit_ || t < 0) node = nc;
            else if (t <= entry) node = fc;
            else if (t <= s_min) { node = fc; entry = t; }
            else { stk[sp++] = E{fc, t}; node = nc; exit_ = t; }
            x = h.nodes[2 * node];
            y = h.nodes[2 * node + 1];
            ++nodes;
        }
        const uint32_t cnt = y >> 2;
        if (cnt > 0 && exit_ > s_min) {
            ++leaves;
            float sm = exit_;
            int best = -1;
            for (uint32_t e = x; e < x + cnt; ++e) {
                float s;
                ++tests;
                if (test(h.isect_a.data(), h.isect_bary.data(), e, o, d, sm, s)) { sm = s; best = (int)h.isect_bary[e].tri; }
            }
            if (best >= 0) return best;
        }
        if (sp == 0) return -1;
        --sp;
        node = stk[sp].n;
        entry = stk[sp].e;
        exit_ = sp > 0 ? stk[sp - 1].e : root_exit;
    }
}

// the binary BVH query (bvh_trace.h bvh_bound)
float bvh2(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, float best, double &nodes, double &leaves)
{
    const float m = rt_ray_margin(o.x, o.y, o.z, h.bvh_scale);
    const RtSlab sl = rt_slab(o, d, m);
    struct E { uint32_t r; float tn; } stk[RT_BVH_STACK];
    int sp = 0;
    uint32_t cur = 0;
    while (true) {
        if (!(cur & RT_BVH_LEAF)) {
            ++nodes;
            const RtF4 *nd = &h.bvh_nodes[4 * (size_t)cur];
            uint32_t c0, c1;
            memcpy(&c0, &nd[3].x, 4);
            memcpy(&c1, &nd[3].y, 4);
            float t0, t1;
            const bool h0 = rt_bvh_box(nd[0].x, nd[0].y, nd[0].z, nd[0].w, nd[1].x, nd[1].y, sl, best, t0) && c0 != RT_BVH_EMPTY;
            const bool h1 = rt_bvh_box(nd[1].z, nd[1].w, nd[2].x, nd[2].y, nd[2].z, nd[2].w, sl, best, t1) && c1 != RT_BVH_EMPTY;
            if (h0 && h1) {
                const bool sf = t1 < t0;
                stk[sp++] = E{sf ? c0 : c1, sf ? t0 : t1};
                cur = sf ? c1 : c0;
                continue;
            }
            if (h0 || h1) { cur = h0 ? c0 : c1; continue; }
        } else {
            ++leaves;
            const uint32_t f = (cur & ~RT_BVH_LEAF) >> 3, e1 = f + (cur & 7u) + 1u;
            for (uint32_t e = f; e < e1; ++e) {
                float s;
                if (test(h.bvh_a.data(), h.bvh_bary.data(), e, o, d, best, s)) best = s;
            }
        }
        bool more = false;
        while (sp > 0) {
            --sp;
            if (stk[sp].tn <= best) { cur = stk[sp].r; more = true; break; }
        }
        if (!more) return best;
    }
}

// 8-wide collapse: child refs (binary inner index / leaf ref) with their boxes
struct Node8 {
    int n = 0;
    uint32_t ref[8];
    float lo[8][3], hi[8][3];
};

void child_of(const rt_host::PreparedHost &h, uint32_t node, int c, uint32_t &ref, float *lo, float *hi)
{
    const RtF4 *nd = &h.bvh_nodes[4 * (size_t)node];
    uint32_t r[2];
    memcpy(&r[0], &nd[3].x, 4);
    memcpy(&r[1], &nd[3].y, 4);
    ref = r[c];
    if (c == 0) { lo[0] = nd[0].x; lo[1] = nd[0].y; lo[2] = nd[0].z; hi[0] = nd[0].w; hi[1] = nd[1].x; hi[2] = nd[1].y; }
    else { lo[0] = nd[1].z; lo[1] = nd[1].w; lo[2] = nd[2].x; hi[0] = nd[2].y; hi[1] = nd[2].z; hi[2] = nd[2].w; }
}

Node8 collapse(const rt_host::PreparedHost &h, uint32_t node)
{
    Node8 m;
    for (int c = 0; c < 2; ++c) {
        child_of(h, node, c, m.ref[m.n], m.lo[m.n], m.hi[m.n]);
        if (m.ref[m.n] != RT_BVH_EMPTY) ++m.n;
    }
    while (m.n < 8) {
        int pick = -1;
        float area = -1;
        for (int k = 0; k < m.n; ++k) {
            if (m.ref[k] & RT_BVH_LEAF) continue;
            const float ex = m.hi[k][0] - m.lo[k][0], ey = m.hi[k][1] - m.lo[k][1], ez = m.hi[k][2] - m.lo[k][2];
            const float a = ex * ey + ey * ez + ez * ex;
            if (a > area) { area = a; pick = k; }
        }
        if (pick < 0) break;
        const uint32_t inner = m.ref[pick];
        uint32_t r2[2];
        float l2[2][3], h2[2][3];
        child_of(h, inner, 0, r2[0], l2[0], h2[0]);
        child_of(h, inner, 1, r2[1], l2[1], h2[1]);
        int put = 0;
        for (int c = 0; c < 2; ++c) {
            if (r2[c] == RT_BVH_EMPTY) continue;
            const int k = put == 0 ? pick : m.n++;
            ++put;
            m.ref[k] = r2[c];
            memcpy(m.lo[k], l2[c], 12);
            memcpy(m.hi[k], h2[c], 12);
        }
        if (put == 0) { // (both empty: drop the child)
            m.ref[pick] = m.ref[--m.n];
            memcpy(m.lo[pick], m.lo[m.n], 12);
            memcpy(m.hi[pick], m.hi[m.n], 12);
        }
    }
    return m;
}

// the 8-wide query: per node, all child boxes at once, every hit leaf child's
// triangles at once (one batch), then the hit inner children nearest first
float bvh8(const rt_host::PreparedHost &h, const std::vector<Node8> &N, const std::vector<int> &idx, Vec3D o, Vec3D d,
           float best, double &visits, double &leafvis, double &tests)
{
    const float m = rt_ray_margin(o.x, o.y, o.z, h.bvh_scale);
    const RtSlab sl = rt_slab(o, d, m);
    struct E { uint32_t r; float tn; } stk[512];
    int sp = 0;
    uint32_t cur = 0;
    while (true) {
        ++visits;
        const Node8 &nd = N[(size_t)idx[cur]];
        float tn[8];
        bool hit[8];
        for (int k = 0; k < nd.n; ++k)
            hit[k] = rt_bvh_box(nd.lo[k][0], nd.lo[k][1], nd.lo[k][2], nd.hi[k][0], nd.hi[k][1], nd.hi[k][2], sl,
                                best, tn[k]);
        bool any_leaf = false;
        for (int k = 0; k < nd.n; ++k) {
            if (!hit[k] || !(nd.ref[k] & RT_BVH_LEAF)) continue;
            any_leaf = true;
            const uint32_t f = (nd.ref[k] & ~RT_BVH_LEAF) >> 3, e1 = f + (nd.ref[k] & 7u) + 1u;
            for (uint32_t e = f; e < e1; ++e) {
                float s;
                ++tests;
                if (test(h.bvh_a.data(), h.bvh_bary.data(), e, o, d, best, s)) best = s;
            }
        }
        if (any_leaf) ++leafvis;
        int order[8], no = 0;
        for (int k = 0; k < nd.n; ++k)
            if (hit[k] && !(nd.ref[k] & RT_BVH_LEAF) && tn[k] <= best) order[no++] = k;
        std::sort(order, order + no, [&](int a, int b) { return tn[a] > tn[b]; }); // farthest first
        for (int i = 0; i + 1 < no; ++i) stk[sp++] = E{nd.ref[order[i]], tn[order[i]]};
        if (no > 0) { cur = nd.ref[order[no - 1]]; continue; }
        bool more = false;
        while (sp > 0) {
            --sp;
            if (stk[sp].tn <= best) { cur = stk[sp].r; more = true; break; }
        }
        if (!more) return best;
    }
}

} // namespace

int main(int argc, char **argv)
{
    if (argc < 2) return 2;
    const long long rays = argc > 2 ? atoll(argv[2]) : 20000;
    std::mt19937_64 rng(argc > 3 ? strtoull(argv[3], nullptr, 10) : 5);
    RtHostScene scene;
    Camera cam;
    if (rt_host::load_scene_file(scene, argv[1], &cam) != RT_OK) return 2;
    const int n = (int)scene.tris.size();
    std::vector<KD_Tree_Node> nodes;
    std::vector<int> indices;
    Bounding_Box bounds;
    if (rt_host::build_kd_tree(scene.tris.data(), n, nodes, indices, bounds) != RT_OK) return 2;
    std::vector<int> lights = rt_host::light_list(scene.tris.data(), n);
    rt_host::PreparedHost h;
    if (rt_host::prepare_host(scene.tris.data(), n, nodes.data(), (int)nodes.size(), indices.data(), (int)indices.size(),
                              lights.data(), (int)lights.size(), bounds, h) != RT_OK || h.bvh_depth < 0)
        return 2;
    // the 8-wide collapse of every binary node reachable as a node of it
    std::vector<Node8> N;
    std::vector<int> idx(h.bvh_nodes.size() / 4, -1);
    std::vector<uint32_t> todo{0};
    while (!todo.empty()) {
        const uint32_t b = todo.back();
        todo.pop_back();
        idx[b] = (int)N.size();
        N.push_back(collapse(h, b));
        for (int k = 0; k < N.back().n; ++k)
            if (!(N.back().ref[k] & RT_BVH_LEAF)) todo.push_back(N.back().ref[k]);
    }
    // glass triangles and their spheres' centres (split at the middle of their x range)
    std::vector<int> glass;
    double xmin = 1e30, xmax = -1e30;
    for (int i = 0; i < n; ++i)
        if (scene.tris[i].material.transparent) {
            glass.push_back(i);
            xmin = std::min(xmin, (double)scene.tris[i].p1.x);
            xmax = std::max(xmax, (double)scene.tris[i].p1.x);
        }
    if (glass.empty()) return 2;
    const double xmid = 0.5 * (xmin + xmax);
    double c[2][3] = {}, cn[2] = {};
    for (int i : glass) {
        const Triangle &t = scene.tris[i];
        const int k = t.p1.x < xmid ? 0 : 1;
        c[k][0] += t.p1.x; c[k][1] += t.p1.y; c[k][2] += t.p1.z;
        cn[k] += 1;
    }
    for (int k = 0; k < 2; ++k)
        for (int a = 0; a < 3; ++a) c[k][a] /= cn[k] > 0 ? cn[k] : 1;
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    W w;
    long long mism = 0;
    for (long long r = 0; r < rays; ++r) {
        const Triangle &t = scene.tris[glass[(size_t)(U(rng) * glass.size()) % glass.size()]];
        float b1 = U(rng), b2 = U(rng);
        if (b1 + b2 > 1) { b1 = 1 - b1; b2 = 1 - b2; }
        const Vec3D o = t.p1 + b1 * (t.p2 - t.p1) + b2 * (t.p3 - t.p1);
        const int k = o.x < xmid ? 0 : 1;
        const Vec3D a = rt_normalize(rt_v3((float)c[k][0] - o.x, (float)c[k][1] - o.y, (float)c[k][2] - o.z));
        Vec3D d;
        while (true) { // inward at a TIR-like angle: cos to the inward axis in (0.2, 0.7)
            Vec3D v = rt_v3(2 * U(rng) - 1, 2 * U(rng) - 1, 2 * U(rng) - 1);
            const float l = rt_dot(v, v);
            if (l < 1e-6f || l > 1.0f) continue;
            v = rt_normalize(v);
            const float ca = rt_dot(v, a);
            if (ca > 0.2f && ca < 0.7f) { d = v; break; }
        }
        float t1, t2;
        if (!box(h, o, d, t1, t2)) continue;
        w.n += 1;
        const int plain = kd(h, o, d, t1, t2, -INFINITY, w.kd_nodes, w.kd_leaves, w.kd_tests);
        const float s2 = bvh2(h, o, d, t2, w.b_nodes, w.b_leaves);
        double dummy = 0;
        const float s8 = bvh8(h, N, idx, o, d, t2, w.w_nodes, w.w_leafvis, w.w_tests);
        if (s8 != s2) ++mism;
        const int bounded = s2 < t2 ? kd(h, o, d, t1, t2, s2, w.bk_nodes, w.bk_leaves, dummy) : -1;
        if (bounded != plain) ++mism;
    }
    const double R = w.n > 0 ? w.n : 1;
    printf("rays %.0f mismatches %lld (8-wide nodes %zu)\n", w.n, mism, N.size());
    printf("plain KD per ray: nodes %.1f leaves %.1f tests %.1f\n", w.kd_nodes / R, w.kd_leaves / R, w.kd_tests / R);
    printf("bounded per ray: BVH nodes %.1f leaf visits %.1f; KD nodes %.1f leaves %.2f\n", w.b_nodes / R,
           w.b_leaves / R, w.bk_nodes / R, w.bk_leaves / R);
    printf("8-wide BVH per ray: node visits %.1f visits with leaf tests %.1f tests %.1f\n", w.w_nodes / R,
           w.w_leafvis / R, w.w_tests / R);
    return 0;
}
