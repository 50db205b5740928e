// kd_jump_sim.cpp — host experiment for the bounded trace's KD phase: once
// the BVH query has s_min, the KD phase's descent is stateless (at every split
// it goes to the origin's side iff t < 0 or t > s_min), i.e. it locates the
// leaf whose interval holds s_min.  This replays the root path of the grid
// cell holding P = o + d*s_min (build_kd_starts' rows, independent loads, each
// decision checked, the root on any difference) and descends from there.
// Reports, on a dumped ray mix (tools/dump_rays.py), the per-ray work of the
// BVH query, the KD phase from the root and the KD phase from P's cell, the
// lockstep wave cost of each (64 rays per wave, the slowest lane), and checks
// every result bit for bit against the plain KD traversal.  Experiment
// tooling, not product code.
//
// usage: kd_jump_sim scene.txt rays.f32
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

struct Work {
    long long nodes = 0, tests = 0, bvh_nodes = 0, bvh_tests = 0, rows = 0;
};

struct E { uint32_t node; float entry; };

struct Resume {
    uint32_t node = 0;
    float entry = 0, exit_ = 0;
    int sp = 0;
    E stk[64];
};

struct Hit {
    int tri = -1;
    float b[3] = {0, 0, 0};
};

bool scene_box(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, float &t1, float &t2)
{
    const Bounding_Box &b = h.bounds;
    float tminx = (b.min.x - o.x) / d.x, tminy = (b.min.y - o.y) / d.y, tminz = (b.min.z - o.z) / d.z;
    float tmaxx = (b.max.x - o.x) / d.x, tmaxy = (b.max.y - o.y) / d.y, tmaxz = (b.max.z - o.z) / d.z;
    t1 = fmaxf(fmaxf(fminf(tminx, tmaxx), fminf(tminy, tmaxy)), fminf(tminz, tmaxz));
    t2 = fminf(fminf(fmaxf(tminx, tmaxx), fmaxf(tminy, tmaxy)), fmaxf(tminz, tmaxz));
    return t1 <= t2;
}

bool test(const RtF4 *A, const RtIsectBary *R, uint32_t e, Vec3D o, Vec3D d, float closest, float &s, float *b)
{
    if (!rt_tri_plane(A[e], o, d, closest, s)) return false;
    return rt_tri_bary(R[e].b, R[e].c, R[e].d, bitsf(R[e].rd), o, d, s, b[0], b[1], b[2]);
}

Hit kd_trace(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, float entry, float exit_, float s_min, Work &w,
             const Resume *from = nullptr)
{
    Hit hit;
    E stk[64];
    int sp = 0;
    const float root_exit = exit_;
    uint32_t node = 0;
    if (from) {
        node = from->node;
        entry = from->entry;
        exit_ = from->exit_;
        sp = from->sp;
        memcpy(stk, from->stk, sizeof(E) * (size_t)sp);
    }
    while (true) {
        uint32_t nx = h.nodes[2 * node], ny = h.nodes[2 * node + 1];
        ++w.nodes;
        while ((ny & 3u) != RT_LEAF_TAG) {
            const uint32_t axis = ny & 3u;
            const float split = bitsf(nx);
            const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
            const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
            uint32_t near_c = node + 1, far_c = ny >> 2;
            if (oax >= split) {
                near_c = ny >> 2;
                far_c = node + 1;
            }
            const float t = (split - oax) / dax;
            if (t >= exit_ || t < 0) {
                node = near_c;
            } else if (t <= entry) {
                node = far_c;
            } else if (t <= s_min) {
                node = far_c;
                entry = t;
            } else {
                stk[sp++] = E{far_c, t};
                node = near_c;
                exit_ = t;
            }
            nx = h.nodes[2 * node];
            ny = h.nodes[2 * node + 1];
            ++w.nodes;
        }
        const uint32_t count = ny >> 2;
        if (count > 0 && exit_ > s_min) {
            float smallest = exit_;
            for (uint32_t e = nx; e < nx + count; ++e) {
                float s, b[3];
                ++w.tests;
                if (test(h.isect_a.data(), h.isect_bary.data(), e, o, d, smallest, s, b)) {
                    smallest = s;
                    hit.tri = (int)h.isect_bary[e].tri;
                    memcpy(hit.b, b, sizeof b);
                }
            }
            if (hit.tri >= 0) return hit;
        }
        if (sp == 0) return hit;
        --sp;
        node = stk[sp].node;
        entry = stk[sp].entry;
        exit_ = sp > 0 ? stk[sp - 1].entry : root_exit;
    }
}

float g_margin_scale = 1.0f; // (experiment: the per-ray margin scaled; results still checked)

float bvh4_bound(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, float best, Work &w)
{
    const float m = g_margin_scale * rt_ray_margin(o.x, o.y, o.z, h.bvh_scale);
    const RtSlab sl = rt_slab(o, d, m);
    struct SE { uint32_t ref; float tn; };
    std::vector<SE> stk;
    uint32_t cur = 0;
    auto pop = [&]() -> uint32_t {
        while (!stk.empty()) {
            const SE e = stk.back();
            stk.pop_back();
            if (e.tn <= best) return e.ref;
        }
        return RT_BVH_EMPTY;
    };
    while (true) {
        while (!(cur & RT_BVH_LEAF)) {
            ++w.bvh_nodes;
            const float *f = reinterpret_cast<const float *>(&h.bvh4[8 * (size_t)cur]);
            const uint32_t *rf = reinterpret_cast<const uint32_t *>(f + 24);
            SE c[4];
            for (int k = 0; k < 4; ++k) {
                float tn;
                const bool hit = rt_bvh_box(f[k], f[4 + k], f[8 + k], f[12 + k], f[16 + k], f[20 + k], sl,
                                            best, tn) && rf[k] != RT_BVH_EMPTY;
                c[k] = hit ? SE{rf[k], tn} : SE{RT_BVH_EMPTY, INFINITY};
            }
            std::stable_sort(c, c + 4, [](const SE &a, const SE &b) {
                const bool ea = a.ref == RT_BVH_EMPTY, eb = b.ref == RT_BVH_EMPTY;
                return ea != eb ? eb : a.tn < b.tn;
            });
            for (int k = 3; k >= 1; --k)
                if (c[k].ref != RT_BVH_EMPTY) stk.push_back(c[k]);
            cur = c[0].ref != RT_BVH_EMPTY ? c[0].ref : pop();
        }
        if (cur == RT_BVH_EMPTY) return best;
        const uint32_t first = (cur & ~RT_BVH_LEAF) >> 3, end = first + (cur & 7u) + 1u;
        for (uint32_t e = first; e < end; ++e) {
            float s, b[3];
            ++w.bvh_tests;
            if (test(h.bvh_a.data(), h.bvh_bary.data(), e, o, d, best, s, b)) best = s;
        }
        cur = pop();
        if (cur == RT_BVH_EMPTY) return best;
    }
}

// the bounded descent's decisions along a grid cell's stored root path, each
// checked against the path (false: some decision differs -> the root)
bool kd_resume(const rt_host::PreparedHost &h, uint32_t start, uint32_t packed, Vec3D o, Vec3D d, float entry,
               float exit_, float s_min, Resume &r, Work &w)
{
    if (start == 0xFFFFFFFFu) return false;
    const uint32_t depth = packed & 31u;
    const uint32_t *row = h.kd_rows.data() + 4 * (size_t)(packed >> 5);
    r.sp = 0;
    for (uint32_t k = 0; k < depth; ++k) {
        const uint32_t *rec = row + 4 * k;
        ++w.rows;
        const uint32_t axis = rec[1] & 3u, anc = rec[2];
        const float split = bitsf(rec[0]);
        const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
        const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
        uint32_t near_c = anc + 1, far_c = rec[1] >> 2;
        if (oax >= split) {
            near_c = rec[1] >> 2;
            far_c = anc + 1;
        }
        const uint32_t taken = rec[3] ? rec[1] >> 2 : anc + 1;
        const float t = (split - oax) / dax;
        if (t >= exit_ || t < 0) {
            if (near_c != taken) return false;
        } else if (t <= entry) {
            if (far_c != taken) return false;
        } else if (t <= s_min) {
            if (far_c != taken) return false;
            entry = t;
        } else {
            if (near_c != taken) return false;
            r.stk[r.sp++] = E{far_c, t};
            exit_ = t;
        }
    }
    r.node = start;
    r.entry = entry;
    r.exit_ = exit_;
    return true;
}

bool cell_of(const rt_host::PreparedHost &h, Vec3D p, size_t &k)
{
    if (h.kd_grid <= 0) return false;
    const int G = h.kd_grid;
    const float q[3] = {p.x, p.y, p.z};
    const float bmin[3] = {h.bounds.min.x, h.bounds.min.y, h.bounds.min.z};
    int c[3];
    for (int a = 0; a < 3; ++a) {
        const float f = (q[a] - bmin[a]) * h.kd_grid_scale[a];
        if (!(f == f)) return false;
        c[a] = f >= 0.0f ? (f < (float)(G - 1) ? (int)f : G - 1) : 0;
    }
    k = ((size_t)c[2] * G + c[1]) * G + c[0];
    return true;
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
    const float m = g_margin_scale * rt_ray_margin(o.x, o.y, o.z, h.bvh_scale);
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
                float bb[3];
                if (test(h.bvh_a.data(), h.bvh_bary.data(), e, o, d, best, s, bb)) best = s;
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



// ---- the stateless entry: descend from P's grid cell start node by the rule
// "near iff t < 0 or t > s_min", certify the leaf by its cell faces (the rule
// is monotone in the split value except at a split == the origin coordinate
// with d > 0: those origins are looked up in the axis's split-value set), take
// exit = min(root exit, face t > s_min), test the leaf; fall back to the root
// descent if the leaf does not hit
struct Cells {
    std::vector<float> lo, hi; // per node: its cell (+-inf where no ancestor bounds it)
    std::vector<std::vector<float>> vals; // per axis: sorted distinct split values
};

void build_cells(const rt_host::PreparedHost &h, Cells &C)
{
    const size_t nn = h.nodes.size() / 2;
    C.lo.assign(3 * nn, -INFINITY);
    C.hi.assign(3 * nn, INFINITY);
    C.vals.assign(3, {});
    std::vector<uint32_t> todo{0};
    while (!todo.empty()) {
        const uint32_t n = todo.back();
        todo.pop_back();
        const uint32_t y = h.nodes[2 * n + 1];
        if ((y & 3u) == RT_LEAF_TAG) continue;
        const int a = (int)(y & 3u);
        const float sp = bitsf(h.nodes[2 * n]);
        C.vals[a].push_back(sp == 0.0f ? 0.0f : sp);
        const uint32_t l = n + 1, r = y >> 2;
        for (int k = 0; k < 3; ++k) {
            C.lo[3 * l + k] = C.lo[3 * n + k];
            C.hi[3 * l + k] = C.hi[3 * n + k];
            C.lo[3 * r + k] = C.lo[3 * n + k];
            C.hi[3 * r + k] = C.hi[3 * n + k];
        }
        C.hi[3 * l + a] = std::min(C.hi[3 * l + a], sp); // left child: below the split (the tightest per side)
        C.lo[3 * r + a] = std::max(C.lo[3 * r + a], sp);
        todo.push_back(l);
        todo.push_back(r);
    }
    for (auto &v : C.vals) {
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
    }
}

// the child the bounded descent takes at split v on axis a (0 left, 1 right)
int side(float v, float oa, float da, float s_min)
{
    const int near_c = oa >= v ? 1 : 0;
    const float t = (v - oa) / da;
    return (t < 0 || t > s_min) ? near_c : 1 - near_c;
}

long long g_sj_fail[6] = {0, 0, 0, 0, 0, 0}; // entry, cell, face, origin, miss, ok
long long g_origin_checks = 0, g_below = 0;
int g_fine = 1; // (experiment) subgrid factor under the top grid
// the entry certified at the start node N: N's cell faces by the rule's
// monotonicity (+ the origin lookups), then the exact rule below N with the
// exit tracked (exit = min(exit, t) for every t > s_min)
Hit stateless_trace(const rt_host::PreparedHost &h, const Cells &C, Vec3D o, Vec3D d, float t1, float t2, float s_min,
                    Work &w, double &steps)
{
    auto full = [&]() { return kd_trace(h, o, d, t1, t2, s_min, w); };
    if (!(s_min >= t1)) { ++g_sj_fail[0]; steps += 1; return full(); }
    const Vec3D p = rt_v3(o.x + d.x * s_min, o.y + d.y * s_min, o.z + d.z * s_min);
    size_t k;
    if (!cell_of(h, p, k) || h.kd_cell[2 * k] == 0xFFFFFFFFu) { ++g_sj_fail[1]; steps += 1; return full(); }
    uint32_t node = h.kd_cell[2 * k];
    steps += 2; // the cell word, N's box (independent loads)
    if (g_fine > 1) { // a subgrid of g_fine^3 under P's top cell: the deepest node holding P's subcell
        const float bmin[3] = {h.bounds.min.x, h.bounds.min.y, h.bounds.min.z};
        const float ext[3] = {h.bounds.max.x - h.bounds.min.x, h.bounds.max.y - h.bounds.min.y,
                              h.bounds.max.z - h.bounds.min.z};
        const int G = h.kd_grid * g_fine;
        const float q[3] = {p.x, p.y, p.z};
        float lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            const float f = (q[a] - bmin[a]) * ((float)G / ext[a]);
            const int c = f >= 0 ? (f < G - 1 ? (int)f : G - 1) : 0;
            lo[a] = bmin[a] + ext[a] * (float)c / (float)G;
            hi[a] = bmin[a] + ext[a] * (float)(c + 1) / (float)G;
        }
        uint32_t n = 0;
        while (true) {
            const uint32_t x = h.nodes[2 * n], y = h.nodes[2 * n + 1];
            if ((y & 3u) == RT_LEAF_TAG) break;
            const int a = (int)(y & 3u);
            const float sp = bitsf(x);
            if (hi[a] < sp) n = n + 1;
            else if (lo[a] > sp) n = y >> 2;
            else break;
        }
        if (n != node) { node = n; steps += 1; } // (the subcell record: one more dependent load)
    }
    const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    float ex = t2;
    for (int a = 0; a < 3; ++a) {
        const float lo = C.lo[3 * node + a], hi = C.hi[3 * node + a];
        if (lo > -INFINITY) {
            if (side(lo, oo[a], dd[a], s_min) != 1) { ++g_sj_fail[2]; return full(); }
            const float t = (lo - oo[a]) / dd[a];
            if (t > s_min) ex = std::min(ex, t);
        }
        if (hi < INFINITY) {
            if (side(hi, oo[a], dd[a], s_min) != 0) { ++g_sj_fail[2]; return full(); }
            const float t = (hi - oo[a]) / dd[a];
            if (t > s_min) ex = std::min(ex, t);
        }
        if (dd[a] > 0 && lo > -INFINITY && oo[a] < lo) {
            ++g_origin_checks;
            const float v = oo[a] == 0.0f ? 0.0f : oo[a];
            if (std::binary_search(C.vals[a].begin(), C.vals[a].end(), v)) { ++g_sj_fail[3]; return full(); }
        }
    }
    while (true) {
        const uint32_t x = h.nodes[2 * node], y = h.nodes[2 * node + 1];
        steps += 1;
        if ((y & 3u) == RT_LEAF_TAG) break;
        ++g_below;
        const int a = (int)(y & 3u);
        const float v = bitsf(x);
        const float t = (v - oo[a]) / dd[a];
        if (t > s_min) ex = std::min(ex, t);
        node = side(v, oo[a], dd[a], s_min) ? (y >> 2) : node + 1;
    }
    const uint32_t ny = h.nodes[2 * node + 1], nx = h.nodes[2 * node];
    const uint32_t count = ny >> 2;
    Hit hit;
    if (count > 0 && ex > s_min) {
        float smallest = ex;
        for (uint32_t e = nx; e < nx + count; ++e) {
            float s, b[3];
            ++w.tests;
            if (test(h.isect_a.data(), h.isect_bary.data(), e, o, d, smallest, s, b)) {
                smallest = s;
                hit.tri = (int)h.isect_bary[e].tri;
                memcpy(hit.b, b, sizeof b);
            }
        }
        steps += count / 4.0;
    }
    if (hit.tri >= 0) { ++g_sj_fail[5]; return hit; }
    ++g_sj_fail[4];
    return full();
}

// descent length from the deepest node holding P's cell of a G^3 grid (the start node) to P's leaf
void grid_depth_stats(const rt_host::PreparedHost &h, const std::vector<float> &R, int G)
{
    const float bmin[3] = {h.bounds.min.x, h.bounds.min.y, h.bounds.min.z};
    const float ext[3] = {h.bounds.max.x - h.bounds.min.x, h.bounds.max.y - h.bounds.min.y, h.bounds.max.z - h.bounds.min.z};
    std::vector<int> rem;
    double top = 0;
    for (size_t i = 0; i < R.size() / 6; ++i) {
        const float P[3] = {R[6 * i], R[6 * i + 1], R[6 * i + 2]}; // (the origins: a stand-in for hit points)
        int c[3];
        float lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            const float f = (P[a] - bmin[a]) * ((float)G / ext[a]);
            c[a] = f >= 0 ? (f < G - 1 ? (int)f : G - 1) : 0;
            lo[a] = bmin[a] + ext[a] * (float)c[a] / (float)G;
            hi[a] = bmin[a] + ext[a] * (float)(c[a] + 1) / (float)G;
        }
        uint32_t n = 0;
        int dtop = 0;
        while (true) {
            const uint32_t x = h.nodes[2 * n], y = h.nodes[2 * n + 1];
            if ((y & 3u) == RT_LEAF_TAG) break;
            const int a = (int)(y & 3u);
            const float sp = bitsf(x);
            if (hi[a] < sp) n = n + 1;
            else if (lo[a] > sp) n = y >> 2;
            else break;
            ++dtop;
        }
        int r = 0;
        while (true) {
            const uint32_t x = h.nodes[2 * n], y = h.nodes[2 * n + 1];
            if ((y & 3u) == RT_LEAF_TAG) break;
            const int a = (int)(y & 3u);
            n = P[a] < bitsf(x) ? n + 1 : (y >> 2);
            ++r;
        }
        rem.push_back(r);
        top += dtop;
    }
    std::sort(rem.begin(), rem.end());
    double m = 0;
    for (int v : rem) m += v;
    const size_t k = rem.size();
    printf("grid %d: start depth %.1f, levels below start mean %.2f p50 %d p90 %d p99 %d max %d\n", G, top / k, m / k,
           rem[k / 2], rem[k * 9 / 10], rem[k * 99 / 100], rem[k - 1]);
}
bool same(const Hit &a, const Hit &b) { return a.tri == b.tri && memcmp(a.b, b.b, sizeof a.b) == 0; }

} // namespace

int main(int argc, char **argv)
{
    if (argc < 3) return 2;
    if (getenv("MARGIN_SCALE")) g_margin_scale = (float)atof(getenv("MARGIN_SCALE"));
    if (getenv("FINE")) g_fine = atoi(getenv("FINE"));
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
    std::vector<Node8> N8;
    std::vector<int> idx8(h.bvh_nodes.size() / 4, -1);
    {
        std::vector<uint32_t> todo{0};
        while (!todo.empty()) {
            const uint32_t b = todo.back();
            todo.pop_back();
            idx8[b] = (int)N8.size();
            N8.push_back(collapse(h, b));
            for (int k = 0; k < N8.back().n; ++k)
                if (!(N8.back().ref[k] & RT_BVH_LEAF)) todo.push_back(N8.back().ref[k]);
        }
    }
    Cells C;
    build_cells(h, C);
    FILE *f = fopen(argv[2], "rb");
    if (!f) return 2;
    std::vector<float> R;
    float buf[6];
    while (fread(buf, sizeof buf, 1, f) == 1) R.insert(R.end(), buf, buf + 6);
    fclose(f);
    const size_t nr = R.size() / 6;
    if (getenv("GRID_STATS")) {
        for (int G : {64, 127, 256, 512, 1024, 2048}) grid_depth_stats(h, R, G);
        return 0;
    }
    printf("scene tris %d kd nodes %zu grid %d rows %zu rays %zu\n", n, h.nodes.size() / 2, h.kd_grid,
           h.kd_rows.size() / 4, nr);
    // per ray lane steps: bvh (nodes + tests/4), kd from the root, kd from P's cell (rows/4 + nodes + tests/4)
    std::vector<double> sb(nr, 0), sk(nr, 0), sj(nr, 0), s8(nr, 0), ss(nr, 0);
    long long mism8 = 0;
    long long mism = 0, jumped = 0, fell = 0, bounded = 0, nodes_root = 0, nodes_jump = 0, rows = 0;
    for (size_t i = 0; i < nr; ++i) {
        const Vec3D o = rt_v3(R[6 * i], R[6 * i + 1], R[6 * i + 2]), d = rt_v3(R[6 * i + 3], R[6 * i + 4], R[6 * i + 5]);
        float t1, t2;
        if (!scene_box(h, o, d, t1, t2)) continue;
        Work wp;
        const Hit plain = kd_trace(h, o, d, t1, t2, -INFINITY, wp);
        if (!rt_bounded_ray(o, d, h.split_vals.data(), h.split_off)) {
            sk[i] = sj[i] = wp.nodes + wp.tests / 4.0;
            continue;
        }
        ++bounded;
        Work wb;
        const float s_min = bvh4_bound(h, o, d, t2, wb);
        sb[i] = wb.bvh_nodes + wb.bvh_tests / 4.0;
        {
            double vis = 0, lv = 0, tests = 0;
            const float q8 = bvh8(h, N8, idx8, o, d, t2, vis, lv, tests);
            if (memcmp(&q8, &s_min, 4) != 0) ++mism8;
            s8[i] = vis + tests / 4.0;
        }
        if (!(s_min < t2)) {
            if (plain.tri >= 0) ++mism;
            continue;
        }
        Work wk;
        const Hit hk = kd_trace(h, o, d, t1, t2, s_min, wk);
        if (!same(hk, plain)) ++mism;
        sk[i] = wk.nodes + wk.tests / 4.0;
        nodes_root += wk.nodes;
        // from P's cell
        const Vec3D p = rt_v3(o.x + d.x * s_min, o.y + d.y * s_min, o.z + d.z * s_min);
        size_t k;
        Work wj;
        Resume r;
        Hit hj;
        if (cell_of(h, p, k) && kd_resume(h, h.kd_cell[2 * k], h.kd_cell[2 * k + 1], o, d, t1, t2, s_min, r, wj)) {
            ++jumped;
            hj = kd_trace(h, o, d, t1, t2, s_min, wj, &r);
        } else {
            ++fell;
            hj = kd_trace(h, o, d, t1, t2, s_min, wj);
        }
        if (!same(hj, plain)) ++mism;
        {
            Work ws;
            double st = 0;
            const Hit hs = stateless_trace(h, C, o, d, t1, t2, s_min, ws, st);
            if (!same(hs, plain)) ++mism;
            ss[i] = st + ws.nodes + (ws.tests > 0 && st == 0 ? 0 : 0) + (ws.nodes ? ws.tests / 4.0 : 0);
        }
        sj[i] = wj.rows / 4.0 + wj.nodes + wj.tests / 4.0;
        nodes_jump += wj.nodes;
        rows += wj.rows;
    }
    printf("bounded %lld jumped %lld fell back %lld mismatches %lld\n", bounded, jumped, fell, mism);
    printf("kd nodes per bounded ray: root %.2f jump %.2f (+ rows %.2f)\n", (double)nodes_root / bounded,
           (double)nodes_jump / bounded, (double)rows / bounded);
    // lockstep: 64 random rays per wave query
    std::vector<size_t> perm(nr);
    for (size_t i = 0; i < nr; ++i) perm[i] = i;
    std::mt19937_64 rng(7);
    double lane_8 = 0, wave_8 = 0;
    double lane_b = 0, lane_k = 0, lane_j = 0, wave_b = 0, wave_k = 0, wave_j = 0, waves = 0;
    for (int rep = 0; rep < 8; ++rep) {
        std::shuffle(perm.begin(), perm.end(), rng);
        for (size_t w0 = 0; w0 + 64 <= nr; w0 += 64) {
            double mb = 0, mk = 0, mj = 0, m8 = 0;
            for (size_t j = w0; j < w0 + 64; ++j) {
                const size_t i = perm[j];
                lane_b += sb[i];
                lane_8 += s8[i];
                m8 = std::max(m8, s8[i]);
                lane_k += sk[i];
                lane_j += sj[i];
                mb = std::max(mb, sb[i]);
                mk = std::max(mk, sk[i]);
                mj = std::max(mj, sj[i]);
            }
            wave_b += mb;
            wave_8 += m8;
            wave_k += mk;
            wave_j += mj;
            waves += 1;
        }
    }
    const double rays = waves * 64;
    printf("lane steps per ray: bvh %.2f kd %.2f kd_jump %.2f\n", lane_b / rays, lane_k / rays, lane_j / rays);
    printf("wave steps per query: bvh %.2f kd %.2f kd_jump %.2f\n", wave_b / waves, wave_k / waves, wave_j / waves);
    printf("efficiency: bvh %.3f kd %.3f kd_jump %.3f\n", lane_b / rays / (wave_b / waves),
           lane_k / rays / (wave_k / waves), lane_j / rays / (wave_j / waves));
    auto pct = [&](std::vector<double> v, const char *name) {
        std::sort(v.begin(), v.end());
        const size_t m = v.size();
        printf("%s p50 %.1f p90 %.1f p99 %.1f p99.9 %.1f max %.1f\n", name, v[m / 2], v[m * 9 / 10], v[m * 99 / 100],
               v[m * 999 / 1000], v[m - 1]);
    };
    if (getenv("DUMP_COSTS")) { // per ray: bvh, kd, kd_jump, bvh8 lane steps (float64)
        FILE *o = fopen(getenv("DUMP_COSTS"), "wb");
        for (size_t i = 0; i < nr; ++i) {
            const double v[4] = {sb[i], sk[i], sj[i], s8[i]};
            fwrite(v, sizeof v, 1, o);
        }
        fclose(o);
    }
    pct(sb, "bvh");
    pct(ss, "kd_stateless");
    {
        double l = 0, wv = 0, nw = 0;
        std::mt19937_64 r2(9);
        std::vector<size_t> pm(nr);
        for (size_t i = 0; i < nr; ++i) pm[i] = i;
        for (int rep = 0; rep < 8; ++rep) {
            std::shuffle(pm.begin(), pm.end(), r2);
            for (size_t w0 = 0; w0 + 64 <= nr; w0 += 64) {
                double m = 0;
                for (size_t j = w0; j < w0 + 64; ++j) { l += ss[pm[j]]; m = std::max(m, ss[pm[j]]); }
                wv += m;
                nw += 1;
            }
        }
        printf("kd_stateless: lane %.2f wave %.2f; fail entry %lld cell %lld face %lld origin %lld leafmiss %lld ok %lld"
               " origin checks %lld levels below N %.2f\n",
               l / (nw * 64), wv / nw, g_sj_fail[0], g_sj_fail[1], g_sj_fail[2], g_sj_fail[3], g_sj_fail[4],
               g_sj_fail[5], g_origin_checks, (double)g_below / (g_sj_fail[4] + g_sj_fail[5]));
    }
    pct(s8, "bvh8");
    printf("bvh8: nodes %zu s_min mismatches %lld lane %.2f wave %.2f eff %.3f\n", N8.size(), mism8, lane_8 / rays,
           wave_8 / waves, lane_8 / rays / (wave_8 / waves));
    pct(sk, "kd");
    pct(sj, "kd_jump");
    if (getenv("DUMP_TOP")) {
        std::vector<size_t> ord(nr);
        for (size_t i = 0; i < nr; ++i) ord[i] = i;
        std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return sb[a] > sb[b]; });
        for (int j = 0; j < atoi(getenv("DUMP_TOP")); ++j) {
            const size_t i = ord[(size_t)j * 7];
            printf("ray %zu bvh %.1f kd %.1f o %g %g %g d %g %g %g\n", i, sb[i], sk[i], R[6 * i], R[6 * i + 1],
                   R[6 * i + 2], R[6 * i + 3], R[6 * i + 4], R[6 * i + 5]);
        }
    }
    return mism == 0 ? 0 : 1;
}
