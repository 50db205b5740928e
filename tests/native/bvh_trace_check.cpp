// bvh_trace_check.cpp — host restatement of the BVH-bounded trace_ray
// (csrc/bvh_trace.h) checked against the plain KD traversal (trace_ray,
// rt/trace_ray.cuh:244-318, as csrc/rt_kernels.h trace()) on a real scene:
// camera rays and bounce-like rays (from random points on the triangles, in
// random directions, some grazing), every result compared bit for bit
// (triangle, barycentrics).  Also reports the work per ray of both
// traversals (nodes, triangle tests) — the reason for the bounded one.
//
// Links the library's host code (rt_host::*): the scene loader, the KD
// build and prepare_host, i.e. the very arrays the GPU gets.
//
// Usage: bvh_trace_check scene.txt [rays] [seed] ["x y z" camera position,
// hex floats]; exit 0 = all identical.
#include <math.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <vector>

#include "host/bvh_build.h"
#include "host/rt_host.h"

namespace {

bool g_debug = false;

float bitsf(uint32_t u)
{
    float f;
    memcpy(&f, &u, 4);
    return f;
}

struct Work {
    long long nodes = 0, tests = 0, bvh_nodes = 0, bvh_tests = 0, leaves = 0, rows = 0;
};

struct E { uint32_t node; float entry; };

// the state the descent resumes from (the origin-cell replay): node, interval, stack
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

// the KD traversal with s_min = -inf is trace_ray itself; with the bound it
// is bvh_trace.h's step 3
long long g_fast = 0, g_ties = 0; // T* leaves taken / rays whose s_min two tests share

// tstar >= 0 (bvh_trace.h kd_bounded): a leaf that lists T* tests T*'s entry only
Hit kd_trace(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, float entry, float exit_, float s_min, Work &w,
             const Resume *from = nullptr, int tstar = -1)
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
        if (g_debug) printf("  leaf node %u count %u entry %a exit %a sp %d\n", node, count, entry, exit_, sp);
        if (count > 0 && exit_ > s_min) {
            ++w.leaves;
            float smallest = exit_;
            uint32_t lo = nx, hi = nx + count;
            if (tstar >= 0) {
                for (uint32_t e = nx; e < nx + count; ++e)
                    if (h.isect_tri[e] == (uint32_t)tstar) {
                        lo = e;
                        hi = e + 1;
#pragma omp atomic
                        ++g_fast;
                        break;
                    }
            }
            for (uint32_t e = lo; e < hi; ++e) {
                float s, b[3];
                ++w.tests;
                if (test(h.isect_a.data(), h.isect_bary.data(), e, o, d, smallest, s, b)) {
                    smallest = s;
                    hit.tri = (int)h.isect_bary[e].tri;
                    memcpy(hit.b, b, sizeof b);
                }
            }
            if (hit.tri >= 0) return hit;
            if (hi - lo != count) {
                fprintf(stderr, "T* entry of a leaf did not pass\n");
                exit(3);
            }
        }
        if (sp == 0) return hit;
        --sp;
        node = stk[sp].node;
        entry = stk[sp].entry;
        exit_ = sp > 0 ? stk[sp - 1].entry : root_exit;
    }
}

float bvh_bound(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, float best, Work &w)
{
    const float m = rt_ray_margin(o.x, o.y, o.z, h.bvh_scale);
    const RtSlab sl = rt_slab(o, d, m);
    struct E { uint32_t ref; float tn; };
    E stk[RT_BVH_STACK];
    int sp = 0;
    uint32_t cur = 0;
    while (true) {
        if (!(cur & RT_BVH_LEAF)) {
            ++w.bvh_nodes;
            const RtF4 *nd = &h.bvh_nodes[4 * (size_t)cur];
            uint32_t c0, c1;
            memcpy(&c0, &nd[3].x, 4);
            memcpy(&c1, &nd[3].y, 4);
            float tn0, tn1;
            const bool h0 = rt_bvh_box(nd[0].x, nd[0].y, nd[0].z, nd[0].w, nd[1].x, nd[1].y, sl, best, tn0) &&
                            c0 != RT_BVH_EMPTY;
            const bool h1 = rt_bvh_box(nd[1].z, nd[1].w, nd[2].x, nd[2].y, nd[2].z, nd[2].w, sl, best, tn1) &&
                            c1 != RT_BVH_EMPTY;
            if (h0 && h1) {
                const bool sf = tn1 < tn0;
                stk[sp++] = E{sf ? c0 : c1, sf ? tn0 : tn1};
                cur = sf ? c1 : c0;
                continue;
            }
            if (h0 || h1) {
                cur = h0 ? c0 : c1;
                continue;
            }
        } else {
            const uint32_t first = (cur & ~RT_BVH_LEAF) >> 3, end = first + (cur & 7u) + 1u;
            for (uint32_t e = first; e < end; ++e) {
                float s, b[3];
                ++w.bvh_tests;
                if (test(h.bvh_a.data(), h.bvh_bary.data(), e, o, d, best, s, b)) {
                    best = s;
                }
            }
        }
        bool more = false;
        while (sp > 0) {
            --sp;
            if (stk[sp].tn <= best) {
                cur = stk[sp].ref;
                more = true;
                break;
            }
        }
        if (!more) return best;
    }
}

long long g_origin_mism = 0;
long long g_bvh4_mism = 0;

// the product's s_min query on the 4-wide collapse (bvh_trace.h bvh4_bound):
// nearest-first, the other hit children pushed farthest-first
// tstar: the triangle whose test alone set the smallest s (bvh_trace.h leaf_scan_min), else -1
float bvh4_bound(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, float best, Work &w, int &tstar)
{
    int tk = -1; // the slot of the smallest passing test, -2: two tests share it
    const float m = rt_ray_margin(o.x, o.y, o.z, h.bvh_scale);
    const RtSlab sl = rt_slab(o, d, m);
    struct E { uint32_t ref; float tn; };
    std::vector<E> stk;
    uint32_t cur = 0;
    auto pop = [&]() -> uint32_t {
        while (!stk.empty()) {
            const E e = stk.back();
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
            E c[4];
            for (int k = 0; k < 4; ++k) {
                float tn;
                const bool hit = rt_bvh_box(f[k], f[4 + k], f[8 + k], f[12 + k], f[16 + k], f[20 + k], sl,
                                            best, tn) && rf[k] != RT_BVH_EMPTY;
                c[k] = hit ? E{rf[k], tn} : E{RT_BVH_EMPTY, INFINITY};
            }
            std::stable_sort(c, c + 4, [](const E &a, const E &b) {
                const bool ea = a.ref == RT_BVH_EMPTY, eb = b.ref == RT_BVH_EMPTY;
                return ea != eb ? eb : a.tn < b.tn;
            });
            for (int k = 3; k >= 1; --k)
                if (c[k].ref != RT_BVH_EMPTY) stk.push_back(c[k]);
            cur = c[0].ref != RT_BVH_EMPTY ? c[0].ref : pop();
        }
        if (cur == RT_BVH_EMPTY) break;
        const uint32_t first = (cur & ~RT_BVH_LEAF) >> 3, end = first + (cur & 7u) + 1u;
        for (uint32_t e = first; e < end; ++e) {
            float s, b[3];
            ++w.bvh_tests;
            if (!rt_tri_plane(h.bvh_a[e], o, d, INFINITY, s) || !(s <= best)) continue;
            const bool lt = s < best;
            if (!lt && tk < 0) continue;
            const RtIsectBary &R = h.bvh_bary[e];
            if (!rt_tri_bary(R.b, R.c, R.d, bitsf(R.rd), o, d, s, b[0], b[1], b[2])) continue;
            if (lt) {
                best = s;
                tk = (int)e;
            } else {
                tk = -2;
            }
        }
        cur = pop();
        if (cur == RT_BVH_EMPTY) break;
    }
    if (tk == -2) {
#pragma omp atomic
        ++g_ties;
    }
    tstar = tk >= 0 ? (int)h.bvh_bary[tk].tri : -1;
    return best;
}

// restatement of coop_trace.h kd_origin_frontier's replay: the descent along
// the stored root path of a grid cell's start node, each decision checked
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

Hit bounded_trace(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, Work &w)
{
    float t1, t2;
    if (!scene_box(h, o, d, t1, t2)) return Hit{};
    if (!rt_bounded_ray(o, d, h.split_vals.data(), h.split_off)) return kd_trace(h, o, d, t1, t2, -INFINITY, w);
    Work w2;
    const float s_bin = bvh_bound(h, o, d, t2, w2);
    int tstar = -1;
    const float s_min = bvh4_bound(h, o, d, t2, w, tstar); // the product's query
    if (memcmp(&s_bin, &s_min, 4) != 0) {
#pragma omp atomic
        ++g_bvh4_mism;
    }
    if (!(s_min < t2)) return Hit{};
    return kd_trace(h, o, d, t1, t2, s_min, w, nullptr, tstar);
}

// the plain traversal entered at the KD node of the grid cell holding the
// origin (wavefront.hip wf_long, coop_trace.h kd_origin_frontier): the
// replay with s_min = -inf, then the rest from that state
long long g_origin_resumed = 0;
Hit origin_trace(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, Work &w)
{
    float t1, t2;
    if (!scene_box(h, o, d, t1, t2)) return Hit{};
    if (h.kd_grid > 0) {
        const int G = h.kd_grid;
        const float p[3] = {o.x, o.y, o.z};
        const float bmin[3] = {h.bounds.min.x, h.bounds.min.y, h.bounds.min.z};
        int c[3];
        for (int a = 0; a < 3; ++a) {
            const float f = (p[a] - bmin[a]) * h.kd_grid_scale[a];
            c[a] = f >= 0.0f ? (f < (float)(G - 1) ? (int)f : G - 1) : 0;
        }
        const size_t k = ((size_t)c[2] * G + c[1]) * G + c[0];
        Resume r;
        if (kd_resume(h, h.kd_cell[2 * k], h.kd_cell[2 * k + 1], o, d, t1, t2, -INFINITY, r, w)) {
#pragma omp atomic
            ++g_origin_resumed;
            return kd_trace(h, o, d, t1, t2, -INFINITY, w, &r);
        }
    }
    return kd_trace(h, o, d, t1, t2, -INFINITY, w);
}

Hit plain_trace(const rt_host::PreparedHost &h, Vec3D o, Vec3D d, Work &w)
{
    float t1, t2;
    if (!scene_box(h, o, d, t1, t2)) return Hit{};
    return kd_trace(h, o, d, t1, t2, -INFINITY, w);
}

} // namespace

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s scene.txt [rays] [seed]\n", argv[0]);
        return 2;
    }
    const long long rays = argc > 2 ? atoll(argv[2]) : 200000;
    std::mt19937_64 rng(argc > 3 ? strtoull(argv[3], nullptr, 10) : 7);
    RtHostScene scene;
    Camera cam;
    if (rt_host::load_scene_file(scene, argv[1], &cam) != RT_OK) {
        fprintf(stderr, "scene load failed\n");
        return 2;
    }
    const int n = (int)scene.tris.size();
    std::vector<KD_Tree_Node> nodes;
    std::vector<int> indices;
    Bounding_Box bounds;
    if (rt_host::build_kd_tree(scene.tris.data(), n, nodes, indices, bounds) != RT_OK) return 2;
    std::vector<int> lights = rt_host::light_list(scene.tris.data(), n);
    rt_host::PreparedHost h;
    if (rt_host::prepare_host(scene.tris.data(), n, nodes.data(), (int)nodes.size(), indices.data(),
                              (int)indices.size(), lights.data(), (int)lights.size(), bounds, h) != RT_OK) {
        fprintf(stderr, "prepare failed\n");
        return 2;
    }
    if (argc > 3 && strcmp(argv[2], "file") == 0) { // a ray file: float32 (n, 6) o, d (tools/dump_rays.py)
        FILE *f = fopen(argv[3], "rb");
        if (!f) return 2;
        std::vector<float> v;
        float buf[6];
        while (fread(buf, sizeof buf, 1, f) == 1) v.insert(v.end(), buf, buf + 6);
        fclose(f);
        const long long nr = (long long)(v.size() / 6);
        long long bad = 0;
        Work wb, wp;
        for (long long i = 0; i < nr; ++i) {
            const Vec3D o = rt_v3(v[6 * i], v[6 * i + 1], v[6 * i + 2]), d = rt_v3(v[6 * i + 3], v[6 * i + 4], v[6 * i + 5]);
            const Hit a = plain_trace(h, o, d, wp), b = bounded_trace(h, o, d, wb);
            if (a.tri != b.tri || memcmp(a.b, b.b, sizeof a.b) != 0) {
                if (bad < 5)
                    printf("mismatch ray %a %a %a %a %a %a: kd %d bounded %d\n", o.x, o.y, o.z, d.x, d.y, d.z, a.tri,
                           b.tri);
                ++bad;
            }
        }
        printf("rays %lld mismatches %lld; T* leaves %lld, ties %lld\n", nr, bad, g_fast, g_ties);
        return bad == 0 ? 0 : 1;
    }
    if (argc > 3 && strcmp(argv[2], "ray") == 0) { // debug one ray: "ox oy oz dx dy dz" (hex floats)
        Vec3D o, d;
        if (sscanf(argv[3], "%a %a %a %a %a %a", &o.x, &o.y, &o.z, &d.x, &d.y, &d.z) != 6) return 2;
        Work w;
        float t1, t2;
        const bool in = scene_box(h, o, d, t1, t2);
        const float s_min = in ? bvh_bound(h, o, d, t2, w) : NAN;
        g_debug = true;
        printf("plain:\n");
        const Hit a = plain_trace(h, o, d, w);
        printf("bounded:\n");
        const Hit b = bounded_trace(h, o, d, w);
        g_debug = false;
        printf("box %d [%a, %a] s_min %a kd %d bounded %d\n", in, t1, t2, s_min, a.tri, b.tri);
        if (in) {
            int ts = -1;
            const float s4 = bvh4_bound(h, o, d, t2, w, ts);
            printf("4-wide query: s_min %a, T* %d\n", s4, ts);
        }
        for (int e = 0; e < (int)h.isect_a.size(); ++e) { // every passing test (KD entry order)
            float s, bb[3];
            if (test(h.isect_a.data(), h.isect_bary.data(), (uint32_t)e, o, d, INFINITY, s, bb))
                printf("  pass: entry %d tri %u s %a\n", e, h.isect_bary[e].tri, s);
        }
        for (size_t k = 0; k < h.bvh_a.size(); ++k) {
            float s, bb[3];
            if (test(h.bvh_a.data(), h.bvh_bary.data(), (uint32_t)k, o, d, INFINITY, s, bb))
                printf("  bvh pass: slot %zu tri %u s %a\n", k, h.bvh_bary[k].tri, s);
        }
        return 0;
    }
    if (argc > 4 && sscanf(argv[4], "%a %a %a", &cam.position.x, &cam.position.y, &cam.position.z) != 3) {
        fprintf(stderr, "bad camera position '%s'\n", argv[4]);
        return 2;
    }
    if (h.bvh_depth < 0) {
        fprintf(stderr, "no BVH built\n");
        return 2;
    }
    printf("tris %d kd_nodes %zu bvh_nodes %zu bvh_depth %d always %d dropped %d\n", n, nodes.size(),
           h.bvh_nodes.size() / 4, h.bvh_depth, h.bvh_always, h.bvh_dropped);
    {
        // every triangle's shipped margin (tri_margin + rt_ray_margin, for origins from the scene's
        // centre to far outside it) against the proven bound (bvh_build.h tri_margin_bound)
        const Bounding_Box &b = h.bounds;
        const double box1 = fmax(fabs((double)b.min.x), fabs((double)b.max.x)) +
                            fmax(fabs((double)b.min.y), fabs((double)b.max.y)) +
                            fmax(fabs((double)b.min.z), fabs((double)b.max.z));
        long long shorts = 0, unproven = 0, finite = 0;
        double min_ratio = INFINITY;
#pragma omp parallel for reduction(+ : shorts, unproven, finite) reduction(min : min_ratio)
        for (long long k = 0; k < (long long)h.bvh_bary.size(); ++k) {
            const RtIsectBary &r = h.bvh_bary[(size_t)k];
            const RtF4 &A = h.bvh_a[(size_t)k];
            const Vec3D p1 = rt_v3(r.b.x, r.b.y, r.b.z), v0 = rt_v3(r.c.x, r.c.y, r.c.z), v1 = rt_v3(r.d.x, r.d.y, r.d.z);
            const float rd = bitsf(r.rd);
            const float m = rt_host::tri_margin(p1, v0, v1, rd, A.x, A.y, A.z);
            if (!(m == m) || isinf(m)) continue; // (whole-scene box / left out)
            ++finite;
            for (double on1 : {0.0, box1, 1e3 * box1, 1e6 * box1 + 1.0}) {
                const double pb = rt_host::tri_margin_bound(p1, v0, v1, rd, on1, box1);
                if (isinf(pb)) {
                    ++unproven;
                    continue;
                }
                const float of = (float)(on1 / 3.0);
                const double shipped = (double)m + (double)rt_ray_margin(of, of, of, h.bvh_scale);
                min_ratio = fmin(min_ratio, shipped / pb);
                if (shipped < pb) ++shorts;
            }
        }
        printf("margins: %lld finite, shipped below the proven bound %lld, unproven %lld, min ratio %.4g\n", finite,
               shorts, unproven, min_ratio);
        if (shorts || unproven) return 1;
    }
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    auto unit = [&]() {
        while (true) {
            Vec3D v = rt_v3(2 * U(rng) - 1, 2 * U(rng) - 1, 2 * U(rng) - 1);
            float l = rt_dot(v, v);
            if (l > 1e-6f && l <= 1.0f) return rt_normalize(v);
        }
    };
    Work wp, wb;
    long long mism = 0, hits = 0;
#pragma omp parallel
    {
        Work lp, lb;
        long long lm = 0, lh = 0;
        std::mt19937_64 r2(rng() + 0x9e3779b97f4a7c15ull * (unsigned)omp_get_thread_num());
        std::uniform_real_distribution<float> V(0.0f, 1.0f);
        auto unit2 = [&]() {
            while (true) {
                Vec3D v = rt_v3(2 * V(r2) - 1, 2 * V(r2) - 1, 2 * V(r2) - 1);
                float l = rt_dot(v, v);
                if (l > 1e-6f && l <= 1.0f) return rt_normalize(v);
            }
        };
#pragma omp for schedule(dynamic, 1024)
        for (long long k = 0; k < rays; ++k) {
            Vec3D o, d;
            const int mode = (int)(k % 4);
            if (mode == 0) { // from the camera
                o = cam.position;
                d = unit2();
            } else { // from a point on a random triangle (a bounce), some grazing / axis-parallel
                const Triangle &t = scene.tris[(size_t)(V(r2) * n) % n];
                float b1 = V(r2), b2 = V(r2);
                if (b1 + b2 > 1) {
                    b1 = 1 - b1;
                    b2 = 1 - b2;
                }
                o = t.p1 + b1 * (t.p2 - t.p1) + b2 * (t.p3 - t.p1);
                d = unit2();
                if (mode == 2) {
                    Vec3D nn = rt_normalize(rt_cross(t.p2 - t.p1, t.p3 - t.p1));
                    if (nn.x == nn.x) d = rt_normalize(d - rt_dot(d, nn) * nn + 1e-4f * (V(r2) - 0.5f) * nn);
                } else if (mode == 3 && (k & 4)) {
                    const int a = (int)(k >> 3) % 3;
                    if (a == 0) d.x = 0; else if (a == 1) d.y = 0; else d.z = 0;
                    d = rt_normalize(d);
                }
                if (d.x != d.x) continue;
            }
            const Hit a = plain_trace(h, o, d, lp), b = bounded_trace(h, o, d, lb);
            Work lo;
            const Hit oc = origin_trace(h, o, d, lo);
            if (oc.tri != a.tri || memcmp(oc.b, a.b, sizeof a.b) != 0) {
#pragma omp atomic
                ++g_origin_mism;
            }
            if (a.tri >= 0) ++lh;
            if (a.tri != b.tri || memcmp(a.b, b.b, sizeof a.b) != 0) {
                if (++lm <= 5) {
#pragma omp critical
                    fprintf(stderr, "MISMATCH o (%a %a %a) d (%a %a %a): kd %d, bounded %d\n", o.x, o.y, o.z, d.x,
                            d.y, d.z, a.tri, b.tri);
                }
            }
        }
#pragma omp critical
        {
            mism += lm;
            hits += lh;
            wp.nodes += lp.nodes;
            wp.tests += lp.tests;
            wp.leaves += lp.leaves;
            wb.nodes += lb.nodes;
            wb.tests += lb.tests;
            wb.leaves += lb.leaves;
            wb.bvh_nodes += lb.bvh_nodes;
            wb.bvh_tests += lb.bvh_tests;
        }
    }
    (void)unit;
    const double R = (double)rays;
    printf("rays %lld hits %lld mismatches %lld\n", rays, hits, mism);
    printf("kd-only per ray: nodes %.1f leaves %.1f tests %.1f\n", wp.nodes / R, wp.leaves / R, wp.tests / R);
    printf("bounded per ray: bvh nodes %.1f bvh tests %.1f kd nodes %.1f leaves %.2f tests %.1f\n", wb.bvh_nodes / R,
           wb.bvh_tests / R, wb.nodes / R, wb.leaves / R, wb.tests / R);
    printf("origin-cell entry: %lld resumed, mismatches vs the plain traversal %lld\n", g_origin_resumed, g_origin_mism);
    printf("4-wide s_min query: %zu nodes, deepest stack %d, s_min differing from the binary query %lld\n",
           h.bvh4.size() / 8, h.bvh4_stack, g_bvh4_mism);
    printf("T* leaves: %lld tested by T*'s entry alone; rays whose s_min two tests share: %lld\n", g_fast, g_ties);
    return mism == 0 && g_origin_mism == 0 && g_bvh4_mism == 0 ? 0 : 1;
}
