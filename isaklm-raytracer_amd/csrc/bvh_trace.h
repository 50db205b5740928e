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

#ifdef RT_PHASE_PROF
// phase profile (a -DRT_PHASE_PROF build, tools/phase_profile.py): per wave,
// the s_memtime at which trace_bvh's BVH query ends (the KD phase starts)
__device__ unsigned long long g_phase_mid[16384];
__device__ unsigned long long g_phase_acc[8]; // wf_finish_bvh's per-phase sums (wavefront.hip)
#define RT_PHASE_MID()                                                                                              \
    g_phase_mid[((blockIdx.x * blockDim.x + threadIdx.x) >> 6) & 16383] = __builtin_amdgcn_s_memtime()
#else
#define RT_PHASE_MID()
#endif
#if defined(RT_LOCKSTEP_PROF) && !defined(RT_PHASE_PROF)
// lockstep profile (a -DRT_LOCKSTEP_PROF build, tools/lockstep_profile.py): the counting
// finisher's per-query lane steps against the wave's (wavefront.hip wf_finish_bvh)
__device__ unsigned long long g_phase_acc[8];
#endif

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

// s_min of step 2: the smallest s < best of any passing test (best if none)
template <bool COUNT, typename STACK>
__device__ __forceinline__ float bvh_bound(const RtDevScene &sc, Vec3D o, Vec3D d, float best, STACK &stk, Cnt &cn)
{
    const float m = rt_ray_margin(o.x, o.y, o.z, sc.bvh_scale);
    const Vec3D om = rt_v3(o.x + m, o.y + m, o.z + m), op = rt_v3(o.x - m, o.y - m, o.z - m);
    const Vec3D inv = rt_v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
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
            const bool h0 = rt_bvh_box(a.x, a.y, a.z, a.w, b.x, b.y, om, op, inv, best, tn0) && ch.x != RT_BVH_EMPTY;
            const bool h1 = rt_bvh_box(b.z, b.w, c.x, c.y, c.z, c.w, om, op, inv, best, tn1) && ch.y != RT_BVH_EMPTY;
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
};

template <bool COUNT, bool PARK, typename STACK>
__device__ __forceinline__ bool bvh4_query(const RtDevScene &sc, Vec3D o, Vec3D d, float best0, STACK &stk, Cnt &cn,
                                           int cap, bool resume, BvhPark &pk)
{
    const float m = rt_ray_margin(o.x, o.y, o.z, sc.bvh_scale);
    const Vec3D om = rt_v3(o.x + m, o.y + m, o.z + m), op = rt_v3(o.x - m, o.y - m, o.z - m);
    const Vec3D inv = rt_v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    int sp = 0;
    uint32_t cur = 0; // the root (always an inner node)
    float best = best0;
    if (PARK && resume) {
        sp = pk.sp;
        cur = pk.cur;
        best = pk.best;
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
                    return false;
                }
                ++steps;
            }
            if (COUNT) cn.v[RT_CNT_B_BVH_NODE]++;
            const RtF4 *nd = sc.bvh4 + 8 * (size_t)cur;
            const RtF4 lx = ldc4(nd), ly = ldc4(nd + 1), lz = ldc4(nd + 2), hx = ldc4(nd + 3), hy = ldc4(nd + 4),
                       hz = ldc4(nd + 5);
            const uint4 rf = ldc_u4(reinterpret_cast<const uint32_t *>(nd + 6));
            float t0, t1, t2, t3;
            uint32_t r0 = rf.x, r1 = rf.y, r2 = rf.z, r3 = rf.w;
            if (!(rt_bvh_box(lx.x, ly.x, lz.x, hx.x, hy.x, hz.x, om, op, inv, best, t0) && r0 != RT_BVH_EMPTY)) {
                t0 = INFINITY;
                r0 = RT_BVH_EMPTY;
            }
            if (!(rt_bvh_box(lx.y, ly.y, lz.y, hx.y, hy.y, hz.y, om, op, inv, best, t1) && r1 != RT_BVH_EMPTY)) {
                t1 = INFINITY;
                r1 = RT_BVH_EMPTY;
            }
            if (!(rt_bvh_box(lx.z, ly.z, lz.z, hx.z, hy.z, hz.z, om, op, inv, best, t2) && r2 != RT_BVH_EMPTY)) {
                t2 = INFINITY;
                r2 = RT_BVH_EMPTY;
            }
            if (!(rt_bvh_box(lx.w, ly.w, lz.w, hx.w, hy.w, hz.w, om, op, inv, best, t3) && r3 != RT_BVH_EMPTY)) {
                t3 = INFINITY;
                r3 = RT_BVH_EMPTY;
            }
            // sort the 4 (entry, ref) pairs by entry (misses last): a 5-comparator network
            auto cswap = [](float &ta, uint32_t &ra, float &tb, uint32_t &rb) {
                const bool sw = tb < ta || (ra == RT_BVH_EMPTY && rb != RT_BVH_EMPTY);
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
            if (r3 != RT_BVH_EMPTY) {
                stk.put(sp, r3, t3);
                ++sp;
            }
            if (r2 != RT_BVH_EMPTY) {
                stk.put(sp, r2, t2);
                ++sp;
            }
            if (r1 != RT_BVH_EMPTY) {
                stk.put(sp, r1, t1);
                ++sp;
            }
            cur = r0 != RT_BVH_EMPTY ? r0 : pop();
        }
        if (cur == RT_BVH_EMPTY) break;
        const uint32_t first = (cur & ~RT_BVH_LEAF) >> 3, end = first + (cur & 7u) + 1u;
        if (COUNT) cn.v[RT_CNT_B_BVH_TRI] += end - first;
        float bx, by, bz;
        (void)leaf_scan<COUNT>(sc.bvh_a, sc.bvh_bary, first, end, o, d, best, bx, by, bz, cn);
        cur = pop();
        if (cur == RT_BVH_EMPTY) break;
    }
    pk.best = best;
    return true;
}

template <bool COUNT, typename STACK>
__device__ __forceinline__ float bvh4_bound(const RtDevScene &sc, Vec3D o, Vec3D d, float best, STACK &stk, Cnt &cn)
{
    BvhPark pk;
    (void)bvh4_query<COUNT, false>(sc, o, d, best, stk, cn, 0, false, pk);
    return pk.best;
}

// Step 3's descent, given s_min, is stateless: at every split it goes to the
// origin's side iff t < 0 or t > s_min (with entry <= s_min < exit, which
// holds all the way down when s_min >= the scene-box entry), i.e. it walks to
// the leaf whose interval holds s_min, with exit = min(root exit, every
// split's t > s_min on the way) — no pop happens before that first leaf.  So
// it may start below the root.  Per cell of a grid over the scene box the
// host stores (build_kd_starts) the deepest KD node N whose cell holds the
// grid cell, and N's own cell [lo, hi] (its ancestors' splits; +-inf where
// none bounds it).  For P = o + d s_min's grid cell:
//  * the side the rule takes at a split value v on axis a is monotone in v
//    (t = (v - o_a) / d_a is, and the near child flips only at v = o_a),
//    except at v == o_a with d_a > 0 (t = +0: the far, left child although
//    the ray moves right).  So if the rule takes N's side at N's faces lo_a and
//    hi_a, it takes it at every ancestor of N — unless o_a (d_a > 0, o_a <
//    lo_a) is an ancestor's split value, which the axis's split hash set rules
//    out.  The exit down to N is then min(root exit, face t > s_min) (the
//    tightest ancestor per side is the face, by the same monotonicity);
//  * below N the rule runs exactly as the descent would (exit tracked), to the
//    leaf, whose test (closest = its exit) is the descent's first leaf test;
//  * if a face check or a lookup fails, or that leaf holds no hit (the descent
//    would pop), the descent runs from the root as before.
// So the result is the descent's own, bit for bit; the entry saves the
// dependent node fetches and the push / interval bookkeeping above N and
// below it.  COUNT: the cell record counts as four node fetches (32 B), a
// hash probe as one.
#ifndef RT_KD_ENTER
#define RT_KD_ENTER 0 // (measured slower on room2m: the wave still waits for its deepest lane; A/B only)
#endif
__device__ __forceinline__ bool split_hash_has(const RtDevScene &sc, int a, float v)
{
    const uint32_t bits = rt_split_bits(v), mask = sc.split_hash_mask[a];
    const uint32_t *tbl = sc.split_hash + sc.split_hash_off[a];
    uint32_t i = rt_split_hash(bits) & mask;
    while (true) { // (a free slot always exists: the table is at least twice the set)
        const uint32_t w = *(const RT_CONST uint32_t *)(tbl + i);
        if (w == bits) return true;
        if (w == RT_SPLIT_HASH_EMPTY) return false;
        i = (i + 1) & mask;
    }
}

// the rule's child at split value v on axis a: true = child1 (above the split)
__device__ __forceinline__ bool kd_rule_above(float v, float oa, float da, float ya, float s_min, float &ex)
{
    const float t = rt_div_by(v - oa, da, ya); // intersect_plane (rt/trace_ray.cuh:190-210)
    const bool near_above = oa >= v;           // ray_behind_plane (:174-188)
    const bool go_near = t < 0 || t > s_min;
    if (t > s_min) ex = fminf(ex, t);
    return go_near ? near_above : !near_above;
}

// the leaf the descent reaches first and its exit, if certified (false: run the descent from the root)
template <bool COUNT>
__device__ __forceinline__ bool kd_entry_leaf(const RtDevScene &sc, const Vec3D o, const Vec3D d, const float yx,
                                              const float yy, const float yz, const float s_min,
                                              const float root_exit, uint2 &leaf, float &ex, Cnt &c)
{
    const int G = sc.kd_grid;
    const float px = o.x + d.x * s_min, py = o.y + d.y * s_min, pz = o.z + d.z * s_min;
    const float f0 = (px - sc.bmin[0]) * sc.kd_gscale[0], f1 = (py - sc.bmin[1]) * sc.kd_gscale[1],
                f2 = (pz - sc.bmin[2]) * sc.kd_gscale[2];
    const int c0 = f0 >= 0.0f ? (f0 < (float)(G - 1) ? (int)f0 : G - 1) : 0; // (NaN: 0)
    const int c1 = f1 >= 0.0f ? (f1 < (float)(G - 1) ? (int)f1 : G - 1) : 0;
    const int c2 = f2 >= 0.0f ? (f2 < (float)(G - 1) ? (int)f2 : G - 1) : 0;
    const size_t k = ((size_t)c2 * (size_t)G + (size_t)c1) * (size_t)G + (size_t)c0;
    const RtF4 r0 = ldc4(sc.kd_entry + 2 * k), r1 = ldc4(sc.kd_entry + 2 * k + 1);
    if (COUNT) c.v[RT_CNT_NODE] += 4;
    uint32_t node = __float_as_uint(r0.x);
    if (node == 0xFFFFFFFFu) return false;
    ex = root_exit;
    bool ok = true;
    // N's faces (-inf / +inf: no split bounds that side) and the origin lookups
    const float lo[3] = {r0.y, r0.z, r0.w}, hi[3] = {r1.x, r1.y, r1.z};
    const float oa[3] = {o.x, o.y, o.z}, da[3] = {d.x, d.y, d.z}, ya[3] = {yx, yy, yz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (lo[a] > -INFINITY) ok = ok && kd_rule_above(lo[a], oa[a], da[a], ya[a], s_min, ex);
        if (hi[a] < INFINITY) ok = ok && !kd_rule_above(hi[a], oa[a], da[a], ya[a], s_min, ex);
    }
    if (!ok) return false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (da[a] > 0.0f && lo[a] > -INFINITY && oa[a] < lo[a]) {
            if (COUNT) c.v[RT_CNT_NODE]++;
            if (split_hash_has(sc, a, oa[a])) return false;
        }
    }
    // below N: the rule itself
    uint2 nd = ldc_u2(sc.nodes + 2 * (size_t)node);
    if (COUNT) c.v[RT_CNT_NODE]++;
    while ((nd.y & 3u) != RT_LEAF_TAG) {
        const uint32_t axis = nd.y & 3u;
        const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
        const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
        const float yax = axis == 0 ? yx : (axis == 1 ? yy : yz);
        node = kd_rule_above(as_float(nd.x), oax, dax, yax, s_min, ex) ? nd.y >> 2 : node + 1;
        nd = ldc_u2(sc.nodes + 2 * (size_t)node);
        if (COUNT) c.v[RT_CNT_NODE]++;
    }
    leaf = nd;
    return true;
}

// step 3: the reference's KD traversal with the skip bound s_min (-inf: the
// plain traversal), from the scene box's [entry, root_exit]
template <bool COUNT, typename STACK>
__device__ __forceinline__ int kd_bounded(const RtDevScene &sc, const Vec3D o, const Vec3D d, float entry,
                                          const float root_exit, const float s_min, float &hbx, float &hby, float &hbz,
                                          STACK &stk, Cnt &c)
{
    float exit_ = root_exit;
    const float yx = rt_recip_guard(d.x), yy = rt_recip_guard(d.y), yz = rt_recip_guard(d.z);
    int sp = 0;
    uint32_t node = 0;
    if (RT_KD_ENTER && sc.kd_entry && s_min > -INFINITY && s_min >= entry) {
        uint2 lf;
        float ex;
        if (kd_entry_leaf<COUNT>(sc, o, d, yx, yy, yz, s_min, root_exit, lf, ex, c)) {
            const uint32_t count = lf.y >> 2;
            if (count > 0 && ex > s_min) { // the descent's first leaf test (trace_leaf_node, :115-172)
                float smallest = ex;
                float bx = 0.0f, by = 0.0f, bz = 0.0f;
                if (COUNT) c.v[RT_CNT_TRI] += count;
                const int be = leaf_scan<COUNT>(sc.isect_a, sc.isect_bary, lf.x, lf.x + count, o, d, smallest, bx, by,
                                                bz, c);
                if (be >= 0) {
                    if (COUNT) c.v[RT_CNT_HIT]++;
                    hbx = bx;
                    hby = by;
                    hbz = bz;
                    return (int)ldc_u2(&sc.isect_bary[be].rd).y;
                }
            }
        }
    }
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
            if (COUNT) c.v[RT_CNT_TRI] += count;
            const int be = leaf_scan<COUNT>(sc.isect_a, sc.isect_bary, nd.x, nd.x + count, o, d, smallest, bx, by, bz, c);
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
    if (rt_bounded_ray(o, d, sc.split_vals, sc.split_off)) {
        s_min = RT_BVH4 ? bvh4_bound<COUNT>(sc, o, d, exit_, stk, c) : bvh_bound<COUNT>(sc, o, d, exit_, stk, c);
        RT_PHASE_MID();
        if (!(s_min < root_exit)) return -1;
    }
    return kd_bounded<COUNT>(sc, o, d, entry, root_exit, s_min, hbx, hby, hbz, stk, c);
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
    if (rt_bounded_ray(o, d, sc.split_vals, sc.split_off)) {
        if (!bvh4_query<COUNT, true>(sc, o, d, exit_, stk, c, cap, resume, pk)) return false;
        s_min = pk.best;
        RT_PHASE_MID();
        if (!(s_min < root_exit)) return true;
    }
    hit = kd_bounded<COUNT>(sc, o, d, entry, root_exit, s_min, hbx, hby, hbz, stk, c);
    return true;
}

} // namespace rtk
