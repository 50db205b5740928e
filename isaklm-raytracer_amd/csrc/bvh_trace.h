// bvh_trace.h — trace_ray (rt/trace_ray.cuh:244-318) bounded by the
// conservative BVH (host/bvh_build.h): same result, bit for bit, with a
// fraction of the KD traversal's work.
//
//  1. the reference's scene-box test gives [entry, exit] (no box: miss);
//  2. the BVH query computes s_min = the smallest s of any triangle test
//     that passes with s < exit, with the reference's own per-triangle
//     arithmetic (intersect_triangle + barycentrics, rt/trace_ray.cuh:48-113);
//     the BVH's boxes are grown so that no passing test is culled.  None:
//     every leaf test of the reference fails too (a hit needs s < the leaf's
//     exit <= the root's exit) — a miss;
//  3. the reference's KD traversal, unchanged (split distance, near / far
//     order, the implied-exit stack), except that a split crossing at
//     t <= s_min goes straight to the far side with entry = t: every leaf
//     under the near side has exit <= t <= s_min, and a test there can only
//     pass with s >= s_min >= exit — the reference finds nothing in it and
//     continues at the far side with exactly that entry.  Leaves with exit
//     <= s_min are skipped for the same reason; the others get the
//     reference's leaf test (closest starts at the leaf's exit, strict <,
//     first wins).
// Any lower bound of the smallest passing s would do (a smaller one only
// skips less), so the query may cull with any best-so-far it has proven.
#pragma once
#include "bvh_common.h"
#include "rt_kernels.h"

namespace rtk {

// Scene data is read-only for a kernel's lifetime: loaded through the
// constant address space (a wave-uniform address becomes a scalar load
// through the scalar cache; a divergent one stays a vector load).
// (the host pass of the single-source compile sees plain loads: these are
// __device__ functions and never run there)
#if defined(__HIP_DEVICE_COMPILE__)
#define RT_CONST __attribute__((address_space(4)))
#else
#define RT_CONST
#endif
__device__ __forceinline__ RtF4 ldc4(const RtF4 *p)
{
    const RT_CONST RtF4 *q = (const RT_CONST RtF4 *)p;
    return RtF4{q->x, q->y, q->z, q->w};
}
__device__ __forceinline__ uint2 ldc_u2(const void *p)
{
    const RT_CONST uint32_t *q = (const RT_CONST uint32_t *)p;
    return make_uint2(q[0], q[1]);
}
__device__ __forceinline__ float ldc_f(const uint32_t *p) { return __uint_as_float(*(const RT_CONST uint32_t *)p); }
__device__ __forceinline__ uint4 ldc_u4(const uint32_t *p)
{
    const RT_CONST uint4 *q = (const RT_CONST uint4 *)p;
    return *q;
}

// The tests of leaf entries [e0, e1) in order (trace_leaf_node,
// rt/trace_ray.cuh:115-172: intersect_triangle + calculate_barycentric_
// coordinates, :48-113, on precomputed records): an entry passes with
// dn != 0, s >= 1e-5, s < smallest and barycentrics in [0, 1], and then
// becomes the smallest.  The plane records are loaded 4 at a time (a leaf
// costs a few load round trips instead of one per entry), the plane test is
// pre-screened against the smallest at the start of the chunk (a superset)
// and re-checked in entry order against the running smallest — the
// reference's result.  Returns the passing entry that is the smallest (-1: none) and its
// barycentric coordinates.
template <bool COUNT>
__device__ __forceinline__ int leaf_scan(const RtF4 *plane, const RtIsectBary *bary, uint32_t e0, uint32_t e1, Vec3D o,
                                         Vec3D d, float &smallest, float &bx, float &by, float &bz, Cnt &c)
{
    int best = -1;
    for (uint32_t e = e0; e < e1; e += 4) {
        float s[4];
        bool p[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool in = e + k < e1;
            const RtF4 A = ldc4(plane + (in ? e + k : e));
            p[k] = rt_tri_plane(A, o, d, smallest, s[k]) && in;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!p[k] || !(s[k] < smallest)) continue;
            if (COUNT) c.v[RT_CNT_B_BARY]++;
            float cx, cy, cz;
            if (rt_tri_bary(ldc4(&bary[e + k].b), ldc4(&bary[e + k].c), ldc4(&bary[e + k].d),
                            ldc_f(&bary[e + k].rd), o, d, s[k], cx, cy, cz)) {
                smallest = s[k];
                best = (int)(e + k);
                bx = cx;
                by = cy;
                bz = cz;
            }
        }
    }
    return best;
}

// The s_min query's leaf scan (step 2): as leaf_scan, and it also keeps which
// slot's test set the smallest s (tk; -1: none yet).  A second passing test at
// exactly that s — another triangle: a triangle has one BVH slot — makes it
// RT_TK_TIE.  (A test at s == best0, the root's exit, before any pass is no
// pass: the reference's tests need s < the leaf's exit <= the root's.)
#define RT_TK_TIE (-2)
template <bool COUNT>
__device__ __forceinline__ void leaf_scan_min(const RtF4 *plane, const RtIsectBary *bary, uint32_t e0, uint32_t e1,
                                              Vec3D o, Vec3D d, float &smallest, int &tk, Cnt &c)
{
    for (uint32_t e = e0; e < e1; e += 4) {
        float s[4];
        bool p[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool in = e + k < e1;
            const RtF4 A = ldc4(plane + (in ? e + k : e));
            p[k] = rt_tri_plane(A, o, d, INFINITY, s[k]) && s[k] <= smallest && in;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!p[k] || !(s[k] <= smallest)) continue;
            const bool lt = s[k] < smallest;
            if (!lt && tk < 0) continue; // (at best0, or a tie already)
            if (COUNT) c.v[RT_CNT_B_BARY]++;
            float cx, cy, cz;
            if (rt_tri_bary(ldc4(&bary[e + k].b), ldc4(&bary[e + k].c), ldc4(&bary[e + k].d),
                            ldc_f(&bary[e + k].rd), o, d, s[k], cx, cy, cz)) {
                if (lt) {
                    smallest = s[k];
                    tk = (int)(e + k);
                } else {
                    tk = RT_TK_TIE;
                }
            }
        }
    }
}

// s_min of step 2: the smallest s < best of any passing test (best if none)
template <bool COUNT, typename STACK>
__device__ __forceinline__ float bvh_bound(const RtDevScene &sc, Vec3D o, Vec3D d, float best, STACK &stk, Cnt &cn)
{
    const RtSlab sl = rt_slab(o, d, rt_ray_margin(o.x, o.y, o.z, sc.bvh_scale));
    int sp = 0;
    uint32_t cur = 0; // the root (always an inner node)
    // pop the next subtree that may still hold a smaller s (RT_BVH_EMPTY: none)
    auto pop = [&]() -> uint32_t {
        while (sp > 0) {
            --sp;
            uint32_t n;
            float tn;
            stk.get(sp, n, tn);
            if (tn <= best) return n;
        }
        return RT_BVH_EMPTY;
    };
    // "while-while" (SIMT): the lanes descend inner nodes together until each
    // holds a leaf (or is done), then test their leaves together — a lane at a
    // leaf does not drag its wave through every other lane's node steps one
    // iteration at a time
    while (true) {
        while (!(cur & RT_BVH_LEAF)) {
            const RtF4 *nd = sc.bvh_nodes + 4 * (size_t)cur;
            if (COUNT) cn.v[RT_CNT_B_BVH_NODE]++;
            const RtF4 a = ldc4(nd), b = ldc4(nd + 1), c = ldc4(nd + 2);
            const uint2 ch = ldc_u2(nd + 3);
            float tn0, tn1;
            const bool h0 = rt_bvh_box(a.x, a.y, a.z, a.w, b.x, b.y, sl, best, tn0) && ch.x != RT_BVH_EMPTY;
            const bool h1 = rt_bvh_box(b.z, b.w, c.x, c.y, c.z, c.w, sl, best, tn1) && ch.y != RT_BVH_EMPTY;
            if (h0 && h1) {
                const bool second_first = tn1 < tn0;
                stk.put(sp, second_first ? ch.x : ch.y, second_first ? tn0 : tn1);
                ++sp;
                cur = second_first ? ch.y : ch.x;
            } else if (h0 || h1) {
                cur = h0 ? ch.x : ch.y;
            } else {
                cur = pop();
            }
        }
        if (cur == RT_BVH_EMPTY) return best;
        const uint32_t first = (cur & ~RT_BVH_LEAF) >> 3, end = first + (cur & 7u) + 1u;
        if (COUNT) cn.v[RT_CNT_B_BVH_TRI] += end - first;
        float bx, by, bz;
        (void)leaf_scan<COUNT>(sc.bvh_a, sc.bvh_bary, first, end, o, d, best, bx, by, bz, cn);
        cur = pop();
        if (cur == RT_BVH_EMPTY) return best;
    }
}

// s_min of step 2 over the 4-wide collapse of the BVH (host/bvh_build.h
// collapse_bvh4): the same conservative boxes and leaves as bvh_bound's
// binary tree, so the same smallest passing s whatever the visiting order,
// with half the dependent node loads (a node is one 128-B line: the 4 child
// boxes SoA and their references).  The hit children go nearest-first: the
// nearest is descended into, the others pushed farthest-first with their
// entry distance, and popped only while that distance is <= the best s so far.
#ifndef RT_BVH4
#define RT_BVH4 1 // trace_bvh's s_min query on the 4-wide collapse (0: the binary tree)
#endif
//
// The query's state between two node steps is (cur, sp, best) plus the stack
// (LDS / spill area): PARK stops the query before its cap-th node step and
// hands that state back (returns false), and a later call with resume picks
// it up where it stopped — the same visiting order, the same s_min.  The
// whole-call finisher parks a lane's long query so that the rest of its wave
// goes on with shading instead of waiting for that one lane (wf_finish_bvh).
struct BvhPark {
    uint32_t cur;
    int sp;
    float best;
    int tk; // the slot whose test set best (leaf_scan_min)
};

// One node step of the 4-wide query: node `cur`'s children whose grown box
// the ray may meet within [0, best], nearest first — the nearest returned,
// the others pushed farthest-first with their entry distance (RT_BVH_EMPTY:
// none hit).  A missed child sorts last by its entry alone (INFINITY; a hit's
// entry is <= best, finite): a 5-comparator network on (entry, reference).
template <typename STACK>
__device__ __forceinline__ uint32_t bvh4_children(const RtDevScene &sc, uint32_t cur, const RtSlab &sl, float best,
                                                  STACK &stk, int &sp)
{
    const RtF4 *nd = sc.bvh4 + 8 * (size_t)cur;
    const RtF4 lx = ldc4(nd), ly = ldc4(nd + 1), lz = ldc4(nd + 2), hx = ldc4(nd + 3), hy = ldc4(nd + 4),
               hz = ldc4(nd + 5);
    const uint4 rf = ldc_u4(reinterpret_cast<const uint32_t *>(nd + 6));
    float t0, t1, t2, t3;
    uint32_t r0 = rf.x, r1 = rf.y, r2 = rf.z, r3 = rf.w;
    // (an unused slot's box is culled by its own slab test: host/bvh_build.cpp collapse_bvh4)
    if (!rt_bvh_box(lx.x, ly.x, lz.x, hx.x, hy.x, hz.x, sl, best, t0)) t0 = INFINITY;
    if (!rt_bvh_box(lx.y, ly.y, lz.y, hx.y, hy.y, hz.y, sl, best, t1)) t1 = INFINITY;
    if (!rt_bvh_box(lx.z, ly.z, lz.z, hx.z, hy.z, hz.z, sl, best, t2)) t2 = INFINITY;
    if (!rt_bvh_box(lx.w, ly.w, lz.w, hx.w, hy.w, hz.w, sl, best, t3)) t3 = INFINITY;
    auto cswap = [](float &ta, uint32_t &ra, float &tb, uint32_t &rb) {
        const bool sw = tb < ta;
        const float t = sw ? tb : ta, u = sw ? ta : tb;
        const uint32_t r = sw ? rb : ra, q = sw ? ra : rb;
        ta = t;
        tb = u;
        ra = r;
        rb = q;
    };
    cswap(t0, r0, t1, r1);
    cswap(t2, r2, t3, r3);
    cswap(t0, r0, t2, r2);
    cswap(t1, r1, t3, r3);
    cswap(t1, r1, t2, r2);
    if (t3 != INFINITY) {
        stk.put(sp, r3, t3);
        ++sp;
    }
    if (t2 != INFINITY) {
        stk.put(sp, r2, t2);
        ++sp;
    }
    if (t1 != INFINITY) {
        stk.put(sp, r1, t1);
        ++sp;
    }
    return t0 != INFINITY ? r0 : RT_BVH_EMPTY;
}

template <bool COUNT, bool PARK, typename STACK>
__device__ __forceinline__ bool bvh4_query(const RtDevScene &sc, Vec3D o, Vec3D d, float best0, STACK &stk, Cnt &cn,
                                           int cap, bool resume, BvhPark &pk)
{
    const RtSlab sl = rt_slab(o, d, rt_ray_margin(o.x, o.y, o.z, sc.bvh_scale));
    int sp = 0;
    uint32_t cur = 0; // the root (always an inner node)
    float best = best0;
    int tk = -1;
    if (PARK && resume) {
        sp = pk.sp;
        cur = pk.cur;
        best = pk.best;
        tk = pk.tk;
    }
    int steps = 0;
    auto pop = [&]() -> uint32_t {
        while (sp > 0) {
            --sp;
            uint32_t n;
            float tn;
            stk.get(sp, n, tn);
            if (tn <= best) return n;
        }
        return RT_BVH_EMPTY;
    };
    while (true) {
        while (!(cur & RT_BVH_LEAF)) {
            if (PARK) {
                if (steps >= cap) {
                    pk.cur = cur;
                    pk.sp = sp;
                    pk.best = best;
                    pk.tk = tk;
                    return false;
                }
                ++steps;
            }
            if (COUNT) cn.v[RT_CNT_B_BVH_NODE]++;
            const uint32_t next = bvh4_children(sc, cur, sl, best, stk, sp);
            cur = next != RT_BVH_EMPTY ? next : pop();
        }
        if (cur == RT_BVH_EMPTY) break;
        const uint32_t first = (cur & ~RT_BVH_LEAF) >> 3, end = first + (cur & 7u) + 1u;
        if (COUNT) cn.v[RT_CNT_B_BVH_TRI] += end - first;
        leaf_scan_min<COUNT>(sc.bvh_a, sc.bvh_bary, first, end, o, d, best, tk, cn);
        cur = pop();
        if (cur == RT_BVH_EMPTY) break;
    }
    pk.best = best;
    pk.tk = tk;
    return true;
}

// (tstar: the triangle whose test alone set s_min — kd_bounded's fast leaf —, else -1)
template <bool COUNT, typename STACK>
__device__ __forceinline__ float bvh4_bound(const RtDevScene &sc, Vec3D o, Vec3D d, float best, STACK &stk, Cnt &cn,
                                            int &tstar)
{
    BvhPark pk;
    (void)bvh4_query<COUNT, false>(sc, o, d, best, stk, cn, 0, false, pk);
    tstar = pk.tk >= 0 ? (int)sc.bvh_bary[pk.tk].tri : -1;
    return pk.best;
}

// step 3: the reference's KD traversal with the skip bound s_min (-inf: the
// plain traversal), from the scene box's [entry, root_exit]
template <bool COUNT, typename STACK>
__device__ __forceinline__ int kd_bounded(const RtDevScene &sc, const Vec3D o, const Vec3D d, float entry,
                                          const float root_exit, const float s_min, const int tstar, float &hbx,
                                          float &hby, float &hbz, STACK &stk, Cnt &c)
{
    float exit_ = root_exit;
    const float yx = rt_recip_guard(d.x), yy = rt_recip_guard(d.y), yz = rt_recip_guard(d.z);
    int sp = 0;
    uint32_t node = 0;
    while (true) {
        uint2 nd = ldc_u2(sc.nodes + 2 * (size_t)node);
        if (COUNT) c.v[RT_CNT_NODE]++;
        while ((nd.y & 3u) != RT_LEAF_TAG) {
            const uint32_t axis = nd.y & 3u;
            const float split = as_float(nd.x);
            const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
            const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
            const float yax = axis == 0 ? yx : (axis == 1 ? yy : yz);
            uint32_t near_c = node + 1, far_c = nd.y >> 2;
            if (oax >= split) { // ray_behind_plane (:174-188)
                near_c = nd.y >> 2;
                far_c = node + 1;
            }
            const float t = rt_div_by(split - oax, dax, yax); // intersect_plane (:190-210)
            if (t >= exit_ || t < 0) {
                node = near_c;
            } else if (t <= entry) {
                node = far_c;
            } else if (t <= s_min) { // the near side holds no hit: its leaves' exits are <= t
                node = far_c;
                entry = t;
            } else {
                stk.put(sp, far_c, t);
                ++sp;
                node = near_c;
                exit_ = t;
            }
            nd = ldc_u2(sc.nodes + 2 * (size_t)node);
            if (COUNT) c.v[RT_CNT_NODE]++;
        }
        const uint32_t count = nd.y >> 2;
        if (count > 0 && exit_ > s_min) {
            // trace_leaf_node (:115-172): closest starts at the leaf's exit
            float smallest = exit_;
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            int be = -1;
            const uint32_t e0 = nd.x, e1 = nd.x + count;
            if (tstar >= 0) {
                // s_min is the smallest s of every passing test and T*'s test alone has it (tstar,
                // leaf_scan_min): where this leaf lists T*, T*'s test is the leaf's result — it passes
                // (s_min < exit), nothing passes below s_min, nothing else at it — and the reference's
                // scan returns exactly that entry (its first listing; its arithmetic on the same record)
                uint32_t at = e1;
                for (uint32_t e = e0; e < e1 && at == e1; e += 4) {
                    uint32_t id[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) id[k] = *(const RT_CONST uint32_t *)(sc.isect_tri + (e + k < e1 ? e + k : e));
#pragma unroll
                    for (int k = 3; k >= 0; --k)
                        if (e + k < e1 && id[k] == (uint32_t)tstar) at = e + k;
                }
                if (at != e1) { // T*'s entry alone: leaf_scan's test of it, not a 4-wide chunk
                    float st, cx, cy, cz;
                    if (COUNT) c.v[RT_CNT_TRI] += 1;
                    if (rt_tri_plane(ldc4(sc.isect_a + at), o, d, smallest, st) &&
                        rt_tri_bary(ldc4(&sc.isect_bary[at].b), ldc4(&sc.isect_bary[at].c), ldc4(&sc.isect_bary[at].d),
                                    ldc_f(&sc.isect_bary[at].rd), o, d, st, cx, cy, cz)) {
                        smallest = st;
                        be = (int)at;
                        bx = cx;
                        by = cy;
                        bz = cz;
                    }
                }
            }
            if (be < 0) { // the whole leaf (no T*, or a T* entry that did not pass — excluded above)
                if (COUNT) c.v[RT_CNT_TRI] += count;
                be = leaf_scan<COUNT>(sc.isect_a, sc.isect_bary, e0, e1, o, d, smallest, bx, by, bz, c);
            }
            const int best = be >= 0 ? (int)ldc_u2(&sc.isect_bary[be].rd).y : -1;
            if (best >= 0) {
                if (COUNT) c.v[RT_CNT_HIT]++;
                hbx = bx;
                hby = by;
                hbz = bz;
                return best;
            }
        }
        if (sp == 0) return -1;
        --sp;
        node = stk.node_at(sp);
        entry = stk.entry_at(sp);
        exit_ = sp > 0 ? stk.entry_at(sp - 1) : root_exit;
    }
}


// trace_ray with the bound: returns the triangle index or -1 and the hit's
// barycentric coordinates, bit-identical to trace().  COUNT (RT_TRAVERSAL_
// BOUNDED_COUNTED): this traversal's own work — RT_CNT_RAY, RT_CNT_NODE / _TRI
// (KD nodes / plane tests), RT_CNT_B_* (BVH nodes / plane tests, barycentric
// records of both phases)
template <bool COUNT, typename STACK>
__device__ __forceinline__ int trace_bvh(const RtDevScene &sc, const Vec3D o, const Vec3D d, float &hbx, float &hby,
                                         float &hbz, STACK &stk, Cnt &c)
{
    if (COUNT) c.v[RT_CNT_RAY]++;
    float entry, exit_;
    if (!bbox_hit(sc, o, d, entry, exit_)) return -1;
    const float root_exit = exit_;
    float s_min = -INFINITY; // (the plain KD traversal)
    int tstar = -1;
    if (rt_bounded_ray(o, d, sc.split_vals, sc.split_off)) {
        s_min = RT_BVH4 ? bvh4_bound<COUNT>(sc, o, d, exit_, stk, c, tstar) : bvh_bound<COUNT>(sc, o, d, exit_, stk, c);
        if (!(s_min < root_exit)) return -1;
    }
    return kd_bounded<COUNT>(sc, o, d, entry, root_exit, s_min, tstar, hbx, hby, hbz, stk, c);
}

// trace_bvh with the s_min query parked after `cap` node steps (bvh4_query):
// false = parked (pk holds the query's state; call again with resume), true =
// done with the hit in `hit` (-1: miss) — trace_bvh's result, bit for bit
template <bool COUNT, typename STACK>
__device__ __forceinline__ bool trace_bvh_park(const RtDevScene &sc, const Vec3D o, const Vec3D d, int &hit, float &hbx,
                                               float &hby, float &hbz, STACK &stk, Cnt &c, int cap, bool resume,
                                               BvhPark &pk)
{
    if (COUNT && !resume) c.v[RT_CNT_RAY]++;
    hit = -1;
    float entry, exit_;
    if (!bbox_hit(sc, o, d, entry, exit_)) return true;
    const float root_exit = exit_;
    float s_min = -INFINITY; // (the plain KD traversal)
    int tstar = -1;
    if (rt_bounded_ray(o, d, sc.split_vals, sc.split_off)) {
        if (!bvh4_query<COUNT, true>(sc, o, d, exit_, stk, c, cap, resume, pk)) return false;
        s_min = pk.best;
        if (!(s_min < root_exit)) return true;
        if (pk.tk >= 0) tstar = (int)sc.bvh_bary[pk.tk].tri;
    }
    hit = kd_bounded<COUNT>(sc, o, d, entry, root_exit, s_min, tstar, hbx, hby, hbz, stk, c);
    return true;
}

} // namespace rtk
