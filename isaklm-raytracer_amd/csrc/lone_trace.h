// lone_trace.h — trace_ray (rt/trace_ray.cuh:244-318) for ONE ray with a
// whole wave: the deep total-internal-reflection paths of wf_long, where a
// path's bounces are a serial chain and only the latency of one bounce counts.
//
// Same result as bvh_trace.h's trace_bvh (and so as the reference), bit for
// bit; what changes is how many dependent memory round trips a bounce costs:
//  1. s_min from the 8-wide collapse of the conservative BVH (host/
//     scene_prepare.cpp build_bvh8): per visited node, lanes 0-7 test its
//     eight child boxes at once, every hit leaf child's triangles are tested
//     at once (lane = child * 8 + triangle; the leaf's plane and barycentric
//     records in one round trip), and the hit inner children go on the
//     wave's LDS stack nearest-last.  A box is culled only when the ray's
//     [0, best] misses it, so the smallest passing s is exact whatever the
//     order (bvh_trace.h's argument);
//  2. the KD descent with the skip rule, entered through kd_resume's replay
//     of the stored root path of the s_min leaf's start node (all its records
//     loaded at once, one per lane; each decision checked against the path);
//  3. a leaf's entries tested 64 at a time: the winner is the smallest s,
//     ties to the first entry — trace_leaf_node's strict-< scan
//     (rt/trace_ray.cuh:124-141), since a test does not depend on the others.
// Host model of the work per sphere-chord ray (tools/deep_ray_work.cpp,
// room2m): 20 node visits + 6 leaf batches instead of 61 nodes + 8.5 leaves
// for the binary query.
#pragma once
#include "bvh_trace.h"

namespace rtk {

#define LONE_STACK 96 // per-wave LDS stack entries (BVH8 query, then KD descent)
static_assert(LONE_STACK >= RT_STACK_DEPTH, "the KD descent pushes at most the tree's depth");

typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;
typedef __attribute__((address_space(3))) volatile float lds_vf32;

struct LoneLds {
    uint32_t *node; // LONE_STACK
    float *key;     // LONE_STACK: the BVH entry's tn / the KD entry's entry t
};

__device__ __forceinline__ float wave_fmin(float v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off));
    return v;
}

// step 1 (all 64 lanes, wave-uniform results).  false: the stack would
// overflow (the caller takes the binary query instead)
__device__ __forceinline__ bool lone_bound(const RtDevScene &sc, Vec3D o, Vec3D d, float &best, uint32_t &best_first,
                                           const LoneLds &L)
{
    lds_vu32 *sn = (lds_vu32 *)L.node;
    lds_vf32 *sk = (lds_vf32 *)L.key;
    const int lane = __lane_id();
    const float m = rt_ray_margin(o.x, o.y, o.z, sc.bvh_scale);
    const Vec3D om = rt_v3(o.x + m, o.y + m, o.z + m), op = rt_v3(o.x - m, o.y - m, o.z - m);
    const Vec3D inv = rt_v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    best_first = RT_BVH_EMPTY;
    uint32_t cur = 0;
    int sp = 0;
    while (true) {
        const RtF4 *nd = sc.bvh8 + 16 * (size_t)cur + 2 * (lane & 7);
        const RtF4 a = ldf4(nd), b = ldf4(nd + 1);
        const uint32_t ref = __float_as_uint(b.z);
        float tn = INFINITY;
        const bool hit = lane < 8 && ref != RT_BVH_EMPTY && rt_bvh_box(a.x, a.y, a.z, a.w, b.x, b.y, om, op, inv, best, tn);
        const bool is_leaf = (ref & RT_BVH_LEAF) != 0u;
        const unsigned long long lm = __ballot(hit && is_leaf);
        if (lm) { // every hit leaf child's triangles at once: lane = child * 8 + triangle
            const int c = lane >> 3, j = lane & 7;
            const uint32_t rc = (uint32_t)__shfl((int)ref, c);
            const uint32_t first = (rc & ~RT_BVH_LEAF) >> 3;
            float s = INFINITY;
            if (((lm >> c) & 1ull) && (uint32_t)j <= (rc & 7u)) {
                const uint32_t e = first + (uint32_t)j;
                const RtF4 A = ldf4(sc.bvh_a + e);
                const RtIsectBary *r = sc.bvh_bary + e;
                const RtF4 B = ldf4(&r->b), C = ldf4(&r->c), D = ldf4(&r->d);
                const float rd = __uint_as_float(r->rd);
                float sv, cx, cy, cz;
                if (rt_tri_plane(A, o, d, best, sv) && rt_tri_bary(B, C, D, rd, o, d, sv, cx, cy, cz)) s = sv;
            }
            const float mn = wave_fmin(s);
            if (mn < best) {
                best = mn;
                const unsigned long long w = __ballot(s == mn);
                best_first = (uint32_t)__shfl((int)first, __ffsll((long long)w) - 1);
            }
        }
        // the hit inner children that may still hold a smaller s: nearest next, the others stacked
        const bool in = hit && !is_leaf && tn <= best;
        const unsigned long long im = __ballot(in);
        const int cnt = __popcll(im);
        if (cnt > 0) {
            int rank = 0; // among the stacked children, 0 = nearest (ties: lower lane)
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const float tq = __shfl(tn, q);
                rank += (((im >> q) & 1ull) && (tq < tn || (tq == tn && q < lane))) ? 1 : 0;
            }
            if (sp + cnt - 1 > LONE_STACK) return false;
            if (in && rank > 0) { // the second nearest on top
                sn[sp + cnt - 1 - rank] = ref;
                sk[sp + cnt - 1 - rank] = tn;
            }
            sp += cnt - 1;
            cur = (uint32_t)__shfl((int)ref, __ffsll((long long)__ballot(in && rank == 0)) - 1);
            continue;
        }
        while (true) { // pop the next subtree that may still hold a smaller s
            if (sp == 0) return true;
            --sp;
            const float t = sk[sp];
            if (t <= best) {
                cur = sn[sp];
                break;
            }
        }
    }
}

// trace_ray for the wave-uniform ray (o, d): the triangle index or -1 and the
// hit's barycentric coordinates (wave-uniform).  Needs sc.bvh8; falls back to
// the binary query on a stack overflow.
template <typename STACK>
__device__ __forceinline__ int lone_trace(const RtDevScene &sc, Vec3D o, Vec3D d, float &hbx, float &hby, float &hbz,
                                          const LoneLds &L, STACK &bstk, Cnt &c)
{
    lds_vu32 *sn = (lds_vu32 *)L.node;
    lds_vf32 *sk = (lds_vf32 *)L.key;
    const int lane = __lane_id();
    float entry, exit_;
    if (!bbox_hit(sc, o, d, entry, exit_)) return -1;
    const float root_exit = exit_;
    float s_min = -INFINITY; // (the plain KD traversal)
    uint32_t best_first = RT_BVH_EMPTY;
    if (rt_bounded_ray(o, d, sc.split_vals, sc.split_off)) {
        s_min = exit_;
        if (!lone_bound(sc, o, d, s_min, best_first, L)) s_min = bvh_bound<false>(sc, o, d, exit_, bstk, c, best_first);
        if (!(s_min < root_exit)) return -1;
    }
    const float yx = rt_recip_guard(d.x), yy = rt_recip_guard(d.y), yz = rt_recip_guard(d.z);
    int sp = 0;
    uint32_t node = 0;
    // step 2: replay the start node's root path (kd_resume's rule, records one per lane)
    if (sc.kd_rows && best_first != RT_BVH_EMPTY) {
        const uint2 st = ldc_u2(sc.kd_start + 2 * (size_t)best_first);
        const uint32_t depth = st.y & 31u;
        uint4 mine = make_uint4(0u, 0u, 0u, 0u);
        if (st.x != 0xFFFFFFFFu && (uint32_t)lane < depth)
            mine = *reinterpret_cast<const uint4 *>(sc.kd_rows + 4 * ((size_t)(st.y >> 5) + (size_t)lane));
        bool ok = st.x != 0xFFFFFFFFu;
        float en = entry, ex = exit_;
        int k = 0;
        for (uint32_t i = 0; ok && i < depth; ++i) {
            const uint32_t rx = (uint32_t)__builtin_amdgcn_readlane((int)mine.x, (int)i);
            const uint32_t ry = (uint32_t)__builtin_amdgcn_readlane((int)mine.y, (int)i);
            const uint32_t anc = (uint32_t)__builtin_amdgcn_readlane((int)mine.z, (int)i);
            const uint32_t rw = (uint32_t)__builtin_amdgcn_readlane((int)mine.w, (int)i);
            const uint32_t axis = ry & 3u;
            const float split = as_float(rx);
            const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
            const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
            const float yax = axis == 0 ? yx : (axis == 1 ? yy : yz);
            uint32_t near_c = anc + 1, far_c = ry >> 2;
            if (oax >= split) {
                near_c = ry >> 2;
                far_c = anc + 1;
            }
            const float t = rt_div_by(split - oax, dax, yax);
            const uint32_t taken = rw ? ry >> 2 : anc + 1;
            if (t >= ex || t < 0) {
                ok = near_c == taken;
            } else if (t <= en) {
                ok = far_c == taken;
            } else if (t <= s_min) {
                ok = far_c == taken;
                en = t;
            } else {
                ok = near_c == taken;
                if (ok) {
                    if (k >= LONE_STACK) {
                        ok = false;
                    } else {
                        sn[k] = far_c;
                        sk[k] = t;
                        ++k;
                        ex = t;
                    }
                }
            }
        }
        if (ok) {
            node = st.x;
            entry = en;
            exit_ = ex;
            sp = k;
        }
    }
    // the descent (bvh_trace.h trace_bvh's, wave-uniform), leaves 64 entries at a time
    while (true) {
        uint2 nd = ldc_u2(sc.nodes + 2 * (size_t)node);
        while ((nd.y & 3u) != RT_LEAF_TAG) {
            const uint32_t axis = nd.y & 3u;
            const float split = as_float(nd.x);
            const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
            const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
            const float yax = axis == 0 ? yx : (axis == 1 ? yy : yz);
            uint32_t near_c = node + 1, far_c = nd.y >> 2;
            if (oax >= split) {
                near_c = nd.y >> 2;
                far_c = node + 1;
            }
            const float t = rt_div_by(split - oax, dax, yax);
            if (t >= exit_ || t < 0) {
                node = near_c;
            } else if (t <= entry) {
                node = far_c;
            } else if (t <= s_min) {
                node = far_c;
                entry = t;
            } else {
                sn[sp] = far_c; // (sp < the tree's depth <= RT_STACK_DEPTH <= LONE_STACK)
                sk[sp] = t;
                ++sp;
                node = near_c;
                exit_ = t;
            }
            nd = ldc_u2(sc.nodes + 2 * (size_t)node);
        }
        const uint32_t count = nd.y >> 2;
        if (count > 0 && exit_ > s_min) {
            // trace_leaf_node: closest starts at the leaf's exit; smallest s, ties to the first entry
            float bs = exit_;
            uint32_t be = 0xFFFFFFFFu;
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            for (uint32_t base = 0; base < count; base += 64) {
                float s = INFINITY, cx = 0.0f, cy = 0.0f, cz = 0.0f;
                const uint32_t e = nd.x + base + (uint32_t)lane;
                if (base + (uint32_t)lane < count) {
                    const RtF4 A = ldf4(sc.isect_a + e);
                    const RtIsectBary *r = sc.isect_bary + e;
                    const RtF4 B = ldf4(&r->b), C = ldf4(&r->c), D = ldf4(&r->d);
                    const float rd = __uint_as_float(r->rd);
                    float sv;
                    if (rt_tri_plane(A, o, d, exit_, sv) && rt_tri_bary(B, C, D, rd, o, d, sv, cx, cy, cz)) s = sv;
                }
                const float mn = wave_fmin(s);
                if (mn < bs) { // (an equal s of a later chunk is a later entry: the earlier one stays)
                    const int w = __ffsll((long long)__ballot(s == mn)) - 1;
                    bs = mn;
                    be = (uint32_t)__shfl((int)e, w);
                    bx = __shfl(cx, w);
                    by = __shfl(cy, w);
                    bz = __shfl(cz, w);
                }
            }
            if (be != 0xFFFFFFFFu) {
                hbx = bx;
                hby = by;
                hbz = bz;
                return (int)ldc_u2(&sc.isect_bary[be].rd).y;
            }
        }
        if (sp == 0) return -1;
        --sp;
        node = sn[sp];
        entry = sk[sp];
        exit_ = sp > 0 ? sk[sp - 1] : root_exit;
    }
}

} // namespace rtk
