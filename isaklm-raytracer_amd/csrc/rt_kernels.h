// rt_kernels.h — device functions of the render hot path shared by the
// megakernel (path_kernel.hip) and the wavefront kernels (wavefront.hip).
//
// Restates rt/path_tracing.cuh (RNG :34-43, BSDF :45-219, NEE :222-265) and
// rt/trace_ray.cuh (trace_ray :244-318, trace_leaf_node :115-172,
// intersect_triangle :73-113, sample_texture :31-46) operation for operation
// (-ffp-contract=off; sin/cos from rt_libm.h; IEEE division and sqrt).
#pragma once
#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_vecmath.h"

namespace rtk {

enum { PRIMARY = 0, DIFFUSE = 1, SPECULAR = 2, METALLIC = 3, TRANSMISSION = 4 }; // :18-25

struct Cnt {
    unsigned long long v[RT_CNT_COUNT]; // RT_CNT_* ; v[RT_CNT_MAXDEPTH] is a max
    __device__ void zero()
    {
        for (int k = 0; k < RT_CNT_COUNT; ++k) v[k] = 0;
    }
    __device__ void path_end(int depth)
    {
        if ((unsigned long long)depth > v[RT_CNT_MAXDEPTH]) v[RT_CNT_MAXDEPTH] = (unsigned long long)depth;
    }
};

__device__ __forceinline__ float as_float(uint32_t u) { return __uint_as_float(u); }

// Always-on deviation statistics, counting build or not: a path
// cut at the depth limit (rare: never, at the watchdog's 2^24 - 1) and a path
// that ends at depth >= RT_DEEP_PATH (total internal reflection in glass; ~1
// in 10^4 paths on room2m) each cost one or three device-scope atomics.
__device__ __forceinline__ void dev_record_cut(const RtDevFrame &fr)
{
    atomicAdd(fr.dev_stats + RT_DEV_CUT, 1ull);
    if (fr.max_depth <= 0) atomicAdd(fr.dev_stats + RT_DEV_WATCHDOG, 1ull);
}
__device__ __forceinline__ void dev_record_end(const RtDevFrame &fr, int depth)
{
    if (depth < RT_DEEP_PATH) return;
    atomicMax(fr.dev_stats + RT_DEV_MAXDEPTH, (unsigned long long)depth);
    int k = 31 - __clz(depth / RT_DEEP_PATH); // floor(log2(depth / 64))
    k = k < RT_DEV_HIST_BINS - 1 ? k : RT_DEV_HIST_BINS - 1;
    atomicAdd(fr.dev_stats + RT_DEV_HIST + k, 1ull);
}

// the pixel rows this call renders (RtOptions.num_shards > 1: row-interleaved shards)
__device__ __forceinline__ bool rt_row_owned(const RtDevFrame &fr, int y)
{
    return fr.num_shards <= 1 || y % fr.num_shards == fr.shard_id;
}

// get_random_unilateral (rt/path_tracing.cuh:34-43)
__device__ __forceinline__ float rng_next(uint32_t &st)
{
    uint32_t state = st * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    uint32_t r = (word >> 22u) ^ word;
    st = r;
    return (float)r / (float)UINT32_MAX;
}

__device__ __forceinline__ Vec3D ld3(const RtF4 &f) { return rt_v3(f.x, f.y, f.z); }

__device__ __forceinline__ RtF4 ldf4(const RtF4 *p)
{
    float4 v = *reinterpret_cast<const float4 *>(p);
    return RtF4{v.x, v.y, v.z, v.w};
}

// intersect_bounding_box (rt/trace_ray.cuh:212-242)
// the same with the ray's guarded reciprocals (rt_recip_guard): each slab
// division by rt_div_by, bit-identical to the IEEE one
__device__ __forceinline__ bool bbox_hit_recip(const RtDevScene &sc, Vec3D o, Vec3D d, float yx, float yy, float yz,
                                               float &t1, float &t2)
{
    float tminx = rt_div_by(sc.bmin[0] - o.x, d.x, yx), tminy = rt_div_by(sc.bmin[1] - o.y, d.y, yy),
          tminz = rt_div_by(sc.bmin[2] - o.z, d.z, yz);
    float tmaxx = rt_div_by(sc.bmax[0] - o.x, d.x, yx), tmaxy = rt_div_by(sc.bmax[1] - o.y, d.y, yy),
          tmaxz = rt_div_by(sc.bmax[2] - o.z, d.z, yz);
    float s1x = fminf(tminx, tmaxx), s1y = fminf(tminy, tmaxy), s1z = fminf(tminz, tmaxz);
    float s2x = fmaxf(tminx, tmaxx), s2y = fmaxf(tminy, tmaxy), s2z = fmaxf(tminz, tmaxz);
    t1 = fmaxf(fmaxf(s1x, s1y), s1z);
    t2 = fminf(fminf(s2x, s2y), s2z);
    return t1 <= t2;
}

__device__ __forceinline__ bool bbox_hit(const RtDevScene &sc, Vec3D o, Vec3D d, float &t1, float &t2)
{
    float tminx = (sc.bmin[0] - o.x) / d.x, tminy = (sc.bmin[1] - o.y) / d.y, tminz = (sc.bmin[2] - o.z) / d.z;
    float tmaxx = (sc.bmax[0] - o.x) / d.x, tmaxy = (sc.bmax[1] - o.y) / d.y, tmaxz = (sc.bmax[2] - o.z) / d.z;
    float s1x = fminf(tminx, tmaxx), s1y = fminf(tminy, tmaxy), s1z = fminf(tminz, tmaxz);
    float s2x = fmaxf(tminx, tmaxx), s2y = fmaxf(tminy, tmaxy), s2z = fmaxf(tminz, tmaxz);
    t1 = fmaxf(fmaxf(s1x, s1y), s1z);
    t2 = fminf(fminf(s2x, s2y), s2z);
    return t1 <= t2;
}

// The same stack addressed from a wave-uniform base plus the lane id (v_mbcnt,
// recomputed where it is used): no per-lane base address has to stay live —
// or be spilled — across a long loop around the traversal.
// the lane id, computed where it is used (volatile: not hoisted into a register that lives across the loop)
__device__ __forceinline__ int lane_id_here()
{
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

template <int LDS_DEPTH>
struct LaneStack {
    uint32_t *lds_node; // wave-uniform: this wave's column 0
    float *lds_entry;
    int stride;
    uint2 *spill; // wave-uniform
    int spill_stride;
    __device__ __forceinline__ void put(int k, uint32_t node, float t)
    {
        const int l = lane_id_here();
        if (k < LDS_DEPTH) {
            lds_node[k * stride + l] = node;
            lds_entry[k * stride + l] = t;
        } else {
            spill[(size_t)(k - LDS_DEPTH) * spill_stride + l] = make_uint2(node, __float_as_uint(t));
        }
    }
    __device__ __forceinline__ void get(int k, uint32_t &node, float &entry) const
    {
        const int l = lane_id_here();
        if (k < LDS_DEPTH) {
            node = lds_node[k * stride + l];
            entry = lds_entry[k * stride + l];
        } else {
            unsigned long long *p =
                reinterpret_cast<unsigned long long *>(spill + (size_t)(k - LDS_DEPTH) * spill_stride + l);
            const unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            node = (uint32_t)v;
            entry = __uint_as_float((uint32_t)(v >> 32));
        }
    }
    __device__ __forceinline__ uint32_t node_at(int k) const
    {
        uint32_t n;
        float e;
        get(k, n, e);
        return n;
    }
    __device__ __forceinline__ float entry_at(int k) const
    {
        uint32_t n;
        float e;
        get(k, n, e);
        return e;
    }
};

// Traversal stack of (node, entry t).  Entries [0, LDS_DEPTH) live in LDS at
// lds[k * stride]; deeper ones (rare) in a per-thread global spill area at
// spill[(k - LDS_DEPTH) * spill_stride].  The exit t of an entry equals the
// entry t of the one below it (or the root's exit): not stored.
template <int LDS_DEPTH>
struct Stack {
    uint32_t *lds_node;
    float *lds_entry;
    int stride;
    uint2 *spill;
    int spill_stride;
    __device__ __forceinline__ void put(int k, uint32_t node, float t)
    {
        if (k < LDS_DEPTH) {
            lds_node[k * stride] = node;
            lds_entry[k * stride] = t;
        } else {
            spill[(size_t)(k - LDS_DEPTH) * spill_stride] = make_uint2(node, __float_as_uint(t));
        }
    }
    // (The spill read is a relaxed atomic load: otherwise the compiler merges
    // the two branches into one generic `flat` load through a selected
    // pointer, which makes every LDS pop pay the flat path.)
    __device__ __forceinline__ void get(int k, uint32_t &node, float &entry) const
    {
        if (k < LDS_DEPTH) {
            node = lds_node[k * stride];
            entry = lds_entry[k * stride];
        } else {
            unsigned long long *p = reinterpret_cast<unsigned long long *>(spill + (size_t)(k - LDS_DEPTH) * spill_stride);
            const unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            node = (uint32_t)v;
            entry = __uint_as_float((uint32_t)(v >> 32));
        }
    }
    __device__ __forceinline__ uint32_t node_at(int k) const
    {
        uint32_t n;
        float e;
        get(k, n, e);
        return n;
    }
    __device__ __forceinline__ float entry_at(int k) const
    {
        uint32_t n;
        float e;
        get(k, n, e);
        return e;
    }
};

// trace_ray (rt/trace_ray.cuh:244-318): closest hit inside the first leaf
// (front to back) that has one.  Returns the triangle index or -1 and the
// barycentric coordinates of the hit.
template <bool COUNT, typename STACK>
__device__ __forceinline__ int trace(const RtDevScene &sc, const Vec3D o, const Vec3D d, float &hbx, float &hby,
                                     float &hbz, STACK &stk, Cnt &c)
{
    if (COUNT) c.v[RT_CNT_RAY]++;
    float entry, exit_;
    if (!bbox_hit(sc, o, d, entry, exit_)) return -1;
    const float root_exit = exit_;
    int sp = 0;
    uint32_t node = 0;
    while (true) {
        uint2 nd = *reinterpret_cast<const uint2 *>(sc.nodes + 2 * (size_t)node);
        if (COUNT) c.v[RT_CNT_NODE]++;
        while ((nd.y & 3u) != RT_LEAF_TAG) {
            const uint32_t axis = nd.y & 3u;
            const float split = as_float(nd.x);
            const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
            const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
            uint32_t near_c = node + 1, far_c = nd.y >> 2;
            if (oax >= split) { // ray_behind_plane (:174-188)
                near_c = nd.y >> 2;
                far_c = node + 1;
            }
            const float t = (split - oax) / dax; // intersect_plane (:190-210)
            if (t >= exit_ || t < 0) {
                node = near_c;
            } else if (t <= entry) {
                node = far_c;
            } else {
                if (COUNT && sp >= RT_REF_STACK) c.v[RT_CNT_DEEP_PUSH]++;
                stk.put(sp, far_c, t);
                ++sp;
                node = near_c;
                exit_ = t;
            }
            nd = *reinterpret_cast<const uint2 *>(sc.nodes + 2 * (size_t)node);
            if (COUNT) c.v[RT_CNT_NODE]++;
        }
        const int count = (int)(nd.y >> 2);
        if (count > 0) {
            // trace_leaf_node (:115-172) + intersect_triangle (:73-113), two
            // entries per step so both plane loads (and both Cramer loads) are
            // in flight together.  A hit needs dn != 0, s >= 1e-5, s < closest
            // and barycentrics in [0,1]; the plane part is pre-screened against
            // the closest t at the start of the step (a superset) and
            // re-checked in entry order, so the winner is the reference's.
            const uint32_t e0 = nd.x, e1 = nd.x + (uint32_t)count;
            float smallest = exit_;
            int best = -1;
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            for (uint32_t e = e0; e < e1; e += 2) {
                const bool two = e + 1 < e1;
                if (COUNT) c.v[RT_CNT_TRI] += two ? 2 : 1;
                const RtF4 A0 = ldf4(sc.isect_a + e); // n, d
                const RtF4 A1 = ldf4(sc.isect_a + (two ? e + 1 : e));
                const float dn0 = d.x * A0.x + d.y * A0.y + d.z * A0.z;
                const float dn1 = d.x * A1.x + d.y * A1.y + d.z * A1.z;
                const float s0 = (A0.w - (o.x * A0.x + o.y * A0.y + o.z * A0.z)) / dn0;
                const float s1 = (A1.w - (o.x * A1.x + o.y * A1.y + o.z * A1.z)) / dn1;
                const bool p0 = dn0 != 0 && s0 >= 0.00001f && s0 < smallest;
                const bool p1 = two && dn1 != 0 && s1 >= 0.00001f && s1 < smallest;
                RtF4 B0, C0, D0, B1, C1, D1;
                uint2 R0, R1;
                if (p0) {
                    B0 = ldf4(&sc.isect_bary[e].b); // p1, d00
                    C0 = ldf4(&sc.isect_bary[e].c); // v0, d01
                    D0 = ldf4(&sc.isect_bary[e].d); // v1, d11
                    R0 = *reinterpret_cast<const uint2 *>(&sc.isect_bary[e].rd);
                }
                if (p1) {
                    B1 = ldf4(&sc.isect_bary[e + 1].b);
                    C1 = ldf4(&sc.isect_bary[e + 1].c);
                    D1 = ldf4(&sc.isect_bary[e + 1].d);
                    R1 = *reinterpret_cast<const uint2 *>(&sc.isect_bary[e + 1].rd);
                }
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const bool p = k == 0 ? p0 : p1;
                    const float s = k == 0 ? s0 : s1;
                    if (!p || !(s < smallest)) continue;
                    const RtF4 B = k == 0 ? B0 : B1, C = k == 0 ? C0 : C1, D = k == 0 ? D0 : D1;
                    const uint2 R = k == 0 ? R0 : R1;
                    const float rd = as_float(R.x);
                    const float px = o.x + d.x * s, py = o.y + d.y * s, pz = o.z + d.z * s;
                    const float v2x = px - B.x, v2y = py - B.y, v2z = pz - B.z;
                    const float d20 = v2x * C.x + v2y * C.y + v2z * C.z;
                    const float d21 = v2x * D.x + v2y * D.y + v2z * D.z;
                    const float cy = (D.w * d20 - C.w * d21) * rd;
                    const float cz = (B.w * d21 - C.w * d20) * rd;
                    const float cx = 1.0f - cy - cz;
                    if (rt_bary_inside(cx, cy, cz)) {
                        smallest = s;
                        best = (int)R.y;
                        bx = cx;
                        by = cy;
                        bz = cz;
                    }
                }
            }
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

// sample_texture (rt/trace_ray.cuh:31-46)
__device__ __forceinline__ Vec3D sample_texture(const RtDevMaterial &m, Vec3D blend, Vec2D uv)
{
    if (m.tex == nullptr) return blend;
    float u = rt_mod(uv.x, 1.0f);
    float v = rt_mod(uv.y, 1.0f);
    int pn = (int)((float)((int)(v * (float)m.tex_height) * m.tex_width) + (u * (float)m.tex_width));
    // one 4-B global load (the texel array is device memory; a generic uchar4
    // read becomes 2 flat loads)
    typedef __attribute__((address_space(1))) const uint32_t gu32;
    const uint32_t c = *((gu32 *)(m.tex) + pn);
    return rt_v3((float)(c & 0xffu) / (float)RT_MAX_COLOR_CHANNEL, (float)((c >> 8) & 0xffu) / (float)RT_MAX_COLOR_CHANNEL,
                 (float)((c >> 16) & 0xffu) / (float)RT_MAX_COLOR_CHANNEL) *
           blend;
}

__device__ __forceinline__ const RtDevMaterial &material_of(const RtDevScene &sc, int tri)
{
    return sc.materials[__float_as_uint(sc.shade[7 * (size_t)tri].w)];
}

struct Surface { // Sample (rt/trace_ray.cuh:17-29), hit part of trace_leaf_node (:144-169)
    Vec3D albedo, emittance;
    float roughness, refractive_index, extinction;
    bool transparent;
    Vec3D position, normal, tangent, bitangent;
};

template <bool COUNT>
__device__ __forceinline__ void shade(const RtDevScene &sc, int tri, float bx, float by, float bz, Vec3D dir,
                                      Surface &s, Cnt &c)
{
    const RtF4 *r = sc.shade + 7 * (size_t)tri;
    const RtF4 s0 = ldf4(r), s1 = ldf4(r + 1), s2 = ldf4(r + 2), s3 = ldf4(r + 3), s4 = ldf4(r + 4),
               s5 = ldf4(r + 5), s6 = ldf4(r + 6);
    const RtDevMaterial &m = sc.materials[__float_as_uint(s0.w)];
    Vec2D uv = rt_v2(s1.w, s2.w) * bx + rt_v2(s3.w, s4.w) * by + rt_v2(s5.w, s6.x) * bz;
    s.albedo = sample_texture(m, rt_v3(m.albedo[0], m.albedo[1], m.albedo[2]), uv);
    s.emittance = sample_texture(m, rt_v3(m.emittance[0], m.emittance[1], m.emittance[2]), uv);
    if (COUNT && m.tex) c.v[RT_CNT_TEXEL] += 2;
    s.roughness = m.roughness;
    s.refractive_index = m.refractive_index;
    s.extinction = m.extinction;
    s.transparent = m.transparent != 0;
    const Vec3D p1 = ld3(s0), p2 = ld3(s1), p3 = ld3(s2);
    s.position = bx * p1 + by * p2 + bz * p3;
    s.normal = rt_normalize(bx * ld3(s3) + by * ld3(s4) + bz * ld3(s5));
    s.tangent = rt_normalize(rt_cross(p2 - p1, s.normal));
    s.bitangent = rt_normalize(rt_cross(s.normal, s.tangent));
    if (rt_dot(dir, s.normal) > 0) s.normal = -s.normal;
}

// the part of the hit Sample sample_direct_light uses (normal, emittance), and the
// light's area (precomputed in the record, host/scene_prepare.cpp)
__device__ __forceinline__ void shade_light(const RtDevScene &sc, int tri, float bx, float by, float bz, Vec3D dir,
                                            Vec3D &normal, Vec3D &emittance, float &area)
{
    const RtF4 *r = sc.shade + 7 * (size_t)tri;
    const RtF4 s0 = ldf4(r), s1 = ldf4(r + 1), s2 = ldf4(r + 2), s3 = ldf4(r + 3), s4 = ldf4(r + 4),
               s5 = ldf4(r + 5), s6 = ldf4(r + 6);
    const RtDevMaterial &m = sc.materials[__float_as_uint(s0.w)];
    Vec2D uv = rt_v2(s1.w, s2.w) * bx + rt_v2(s3.w, s4.w) * by + rt_v2(s5.w, s6.x) * bz;
    emittance = sample_texture(m, rt_v3(m.emittance[0], m.emittance[1], m.emittance[2]), uv);
    normal = rt_normalize(bx * ld3(s3) + by * ld3(s4) + bz * ld3(s5));
    if (rt_dot(dir, normal) > 0) normal = -normal;
    area = s6.y;
}

// ---- BSDF (rt/path_tracing.cuh:45-219) ----
__device__ __forceinline__ float fresnel_dielectric(Vec3D i, Vec3D h, float n1, float n2) // :61-74
{
    float c = fabsf(rt_dot(i, h));
    float g = sqrtf(fmaxf(rt_square(n2) / rt_square(n1) - 1.0f + rt_square(c), 0.0f));
    float f1 = 0.5f * rt_square((g - c) / (g + c));
    float f2 = 1.0f + rt_square((c * (g + c) - 1.0f) / (c * (g - c) + 1.0f));
    return f1 * f2;
}
__device__ __forceinline__ float fresnel_conductor(Vec3D i, Vec3D h, float n, float k) // :76-101
{
    float n2 = n * n, k2 = k * k;
    float cs = rt_dot(i, h);
    float cs2 = rt_square(cs);
    float sn2 = 1.0f - cs2;
    float t0 = n2 - k2 - sn2;
    float a2b2 = sqrtf(rt_square(t0) + 4.0f * n2 * k2);
    float a = sqrtf(0.5f * (a2b2 + t0));
    float t1 = a2b2 + cs2;
    float t2 = 2.0f * a * cs;
    float rs = (t1 - t2) / (t1 + t2);
    float t3 = cs2 * a2b2 * rt_square(sn2);
    float t4 = t2 * sn2;
    float rp = rs * (t3 - t4) / (t3 + t4);
    return (rs + rp) * 0.5f;
}
__device__ __forceinline__ float lambda_(Vec3D d, Vec3D n, float rough) // :120-127
{
    float dn = rt_dot(d, n);
    float dn2 = rt_square(dn);
    float tan2 = (1 - dn2) / dn2;
    return (sqrtf(1.0f + rt_square(rough) + tan2) - 1.0f) * 0.5f;
}
__device__ __forceinline__ Vec3D specular_weight(Vec3D i, Vec3D o, Vec3D h, Vec3D n, float rough) // :129-136
{
    float g = 1.0f / (1.0f + lambda_(i, n, rough) + lambda_(o, n, rough));
    float w = fabsf(rt_dot(i, h)) * g / (fabsf(rt_dot(n, h) * fabsf(rt_dot(i, n))));
    return rt_v3(w, w, w);
}
__device__ __forceinline__ Vec3D specular_direction(Vec3D i, Vec3D h) { return 2.0f * rt_dot(i, h) * h - i; } // :138-141
__device__ __forceinline__ Vec3D refraction_direction(Vec3D i, Vec3D h, float n1, float n2)           // :143-149
{
    float c = rt_dot(i, h);
    float n = n1 / n2;
    return (n * c - sqrtf(fmaxf(1.0f + n * n * (c * c - 1.0f), 0.0f))) * h - n * i;
}

// get_scattered_light (:151-219): returns the event type, new direction and weight
__device__ __forceinline__ int scatter(Vec3D dir, bool &inside, uint32_t &rng, const Surface &s, Vec3D &out_dir,
                                       Vec3D &weight)
{
    dir = -dir;
    // microfacet_normal (:103-118), FP64 island
    double ru = rng_next(rng);
    float cos_theta = sqrtf((float)((1.0f - ru) / (ru * (double)(s.roughness * s.roughness - 1.0f) + 1.0f)));
    float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
    float phi = rng_next(rng) * RT_TAU;
    float cos_phi, sin_phi;
    rt_sincosf(phi, &sin_phi, &cos_phi);
    Vec3D h = s.tangent * sin_theta * cos_phi + s.normal * cos_theta + s.bitangent * sin_theta * sin_phi;
    if (s.extinction > 0.0f) {
        float F = fresnel_conductor(dir, h, s.refractive_index, s.extinction);
        out_dir = specular_direction(dir, h);
        weight = s.albedo * specular_weight(dir, out_dir, h, s.normal, s.roughness) * F;
        return METALLIC;
    }
    float n1 = 1.0f, n2 = s.refractive_index;
    if (inside) {
        n1 = n2;
        n2 = 1.0f;
    }
    float F = fresnel_dielectric(dir, h, n1, n2);
    float choose = rng_next(rng);
    if (choose < F) {
        out_dir = specular_direction(dir, h);
        weight = rt_v3(1.0f, 1.0f, 1.0f);
        if (!inside) weight = specular_weight(dir, out_dir, h, s.normal, s.roughness);
        return SPECULAR;
    }
    if (s.transparent) {
        inside = !inside;
        out_dir = refraction_direction(dir, h, n1, n2);
        weight = specular_weight(dir, out_dir, h, s.normal, s.roughness) * s.albedo;
        return TRANSMISSION;
    }
    // diffuse_direction (:45-59)
    float dphi = rng_next(rng) * RT_TAU;
    float ds, dc;
    rt_sincosf(dphi, &ds, &dc);
    float ru2 = rng_next(rng);
    float sq = sqrtf(ru2);
    out_dir = sq * dc * s.tangent + sqrtf(1.0f - ru2) * s.normal + sq * ds * s.bitangent;
    weight = s.albedo;
    return DIFFUSE;
}

__device__ __forceinline__ Vec3D mat_mul(const float *R, Vec3D v)
{
    RtM3 m = {rt_v3(R[0], R[1], R[2]), rt_v3(R[3], R[4], R[5]), rt_v3(R[6], R[7], R[8])};
    return m * v;
}

// adaptive test (rt/path_tracing.cuh:352-376): true = run a sample this pass
__device__ __forceinline__ bool adaptive_run(const RtDevFrame &fr, Vec3D fb, float sq, int count)
{
    if (!fr.adaptive || count < fr.min_samples) return true;
    float tl = rt_luminance(fb);
    float mean = tl / (float)count;
    float var = (sq - rt_square(tl) / (float)count) / (float)(count - 1);
    float iw = fr.z_const * sqrtf(var / (float)count);
    return iw > mean * fr.tolerance;
}

// camera ray (:381-391) and random_point_in_pinhole (:327-336)
__device__ __forceinline__ void camera_ray(const RtDevFrame &fr, const RtDevCamera &cam, int x, int y, uint32_t &rng,
                                           Vec3D &ro, Vec3D &rd)
{
    float rx = rng_next(rng);
    float ry = rng_next(rng);
    Vec3D dir = rt_normalize(rt_v3(cam.tan_half_fov * ((float)x + rx - (float)fr.half_w) / (float)fr.half_w,
                                   cam.tan_half_fov * ((float)y + ry - (float)fr.half_h) / (float)fr.half_w, 1.0f));
    rd = mat_mul(cam.R, dir);
    float theta = rng_next(rng) * RT_TAU;
    float r = sqrtf(rng_next(rng)) * cam.aperture;
    float st, ct;
    rt_sincosf(theta, &st, &ct);
    float ox = r * ct;
    float oy = r * st;
    ro = rt_v3(cam.pos[0], cam.pos[1], cam.pos[2]) + mat_mul(cam.R, rt_v3(ox, 0.0f, 0.0f)) +
         mat_mul(cam.R, rt_v3(0.0f, oy, 0.0f));
}

// random_point_in_triangle (:222-233) on light `light`
__device__ __forceinline__ Vec3D light_point(const RtDevScene &sc, int light, uint32_t &rng)
{
    const RtF4 *lr = sc.shade + 7 * (size_t)light;
    const Vec3D lp1 = ld3(ldf4(lr)), lp2 = ld3(ldf4(lr + 1)), lp3 = ld3(ldf4(lr + 2));
    float px = rng_next(rng);
    float py = rng_next(rng);
    float sx = sqrtf(px);
    float u = 1.0f - sx;
    float v = py * sx;
    float w = 1.0f - u - v;
    return u * lp1 + v * lp2 + w * lp3;
}

// contribution of a shadow ray that hit the chosen light (:251-261)
__device__ __forceinline__ Vec3D light_contribution(const RtDevScene &sc, int light, float bx, float by, float bz,
                                                   Vec3D ro, Vec3D rd, Vec3D rp, Vec3D surface_normal)
{
    Vec3D ln, le;
    float area; // (float)(0.5 * (double)|cross(p2 - p1, p3 - p1)|), precomputed
    shade_light(sc, light, bx, by, bz, rd, ln, le, area);
    float d2 = rt_magnitude_squared(rp - ro);
    float c1 = fmaxf(-rt_dot(rd, ln), 0.0f);
    float c2 = fmaxf(rt_dot(rd, surface_normal), 0.0f);
    return le * (area * (float)sc.light_count * c1 * c2 / fmaxf(d2 * RT_PI, 0.001f));
}

// counters: wave-reduce and add once per wave
__device__ __forceinline__ void flush_counters(Cnt &c, unsigned long long *out)
{
    for (int k = 0; k < RT_CNT_COUNT; ++k) {
        unsigned long long v = c.v[k];
        for (int off = 32; off > 0; off >>= 1) {
            unsigned long long o = __shfl_xor(v, off);
            v = k == RT_CNT_MAXDEPTH ? (o > v ? o : v) : v + o;
        }
        c.v[k] = v;
    }
    if ((threadIdx.x & 63) == 0) {
        for (int k = 0; k < RT_CNT_COUNT; ++k)
            if (k != RT_CNT_MAXDEPTH && c.v[k]) atomicAdd(out + k, c.v[k]);
        atomicMax(out + RT_CNT_MAXDEPTH, c.v[RT_CNT_MAXDEPTH]);
    }
}

// after flush_counters: the finisher's share of node / tri / ray
__device__ __forceinline__ void flush_finish_counters(const Cnt &c, unsigned long long *out)
{
    if ((threadIdx.x & 63) == 0) {
        if (c.v[RT_CNT_NODE]) atomicAdd(out + RT_CNT_FIN_NODE, c.v[RT_CNT_NODE]);
        if (c.v[RT_CNT_TRI]) atomicAdd(out + RT_CNT_FIN_TRI, c.v[RT_CNT_TRI]);
        if (c.v[RT_CNT_RAY]) atomicAdd(out + RT_CNT_FIN_RAY, c.v[RT_CNT_RAY]);
    }
}

// per-wave [start, end] s_memrealtime stamps (100 MHz) into a debug buffer
__device__ __forceinline__ unsigned long long realtime() { return __builtin_amdgcn_s_memrealtime(); }

// Wave64 inclusive scans on DPP (CDNA row_shr 1/2/4/8 inside 16-lane rows,
// then row_bcast:15 into rows 1,3 and row_bcast:31 into rows 2,3): six
// dependent VALU ops instead of a chain of six ds_bpermute round trips.
// Lanes whose DPP source is outside the row (or whose row is masked off)
// read the identity through `old`.
__device__ __forceinline__ int wave_incl_add(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false); // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false); // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false); // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false); // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false); // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return v;
}
__device__ __forceinline__ int wave_incl_max(int v) // identity -1
{
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xc, 0xf, false));
    return v;
}
// inclusive max-scan of non-negative values: identity 0, so each step is one
// v_max_u32 with a DPP operand (no separate v_mov of an identity)
__device__ __forceinline__ uint32_t wave_incl_umax(uint32_t v)
{
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}
// a constant materialised where it is used: the compiler otherwise hoists
// constant register tuples (the miss record, the ~0 key) out of the traversal
// loop and, short of registers, spills and reloads them from scratch there
__device__ __forceinline__ int vconst(int c)
{
    int r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "i"(c));
    return r;
}
__device__ __forceinline__ float4 miss_record() // hits[]: tri = -1, no barycentrics
{
    return make_float4(__int_as_float(vconst(-1)), __int_as_float(vconst(0)), __int_as_float(vconst(0)),
                       __int_as_float(vconst(0)));
}
__device__ __forceinline__ int lane63(int v) { return __builtin_amdgcn_readlane(v, 63); }

// Owner lane of every position of a 64-wide chunk [base, base + 64) of a
// segmented range (lane j owns [start_j, start_j + count_j)): lanes whose
// segment starts inside the chunk mark their start in `mark` (64 ints of
// LDS per wave), a max-scan spreads the marks, and `carry` (the owner of
// position base - 1) covers segments that began in an earlier chunk.
// Cross-lane LDS traffic must not be optimised as single-thread code (the
// compiler would forward a lane's own `mark[lane] = -1` to its reload on the
// path where that lane wrote no mark, missing the other lanes' marks), so it
// goes through volatile pointers — in the LDS address space, since a volatile
// generic pointer becomes a system-coherent `flat` access.
typedef __attribute__((address_space(3))) volatile int lds_vint;
typedef __attribute__((address_space(3))) volatile float lds_vfloat;
typedef __attribute__((address_space(3))) volatile unsigned long long lds_vu64;
__device__ __forceinline__ int chunk_owner(int *mark_, int start, int count, int base, int carry)
{
    lds_vint *mark = (lds_vint *)mark_;
    const int lane = __lane_id();
#ifdef RT_OWNER_SMAX
    mark[lane] = -1;
    if (count > 0 && start >= base && start < base + 64) mark[start - base] = lane;
    const int m = wave_incl_max(mark[lane]);
    return max(m, carry);
#else
    // marks are lane + 1 (0 = none): the scan's identity is 0.  Addressed
    // relative to the lane's own slot (no second base-address register).
    lds_vint *mine = mark + lane;
    mine[0] = 0;
    // every lane stores: a lane whose segment does not start in this chunk
    // writes 0 to its own junk slot 64 + lane (the mark array has 128 slots)
    const bool marks = count > 0 && start >= base && start < base + 64;
    int rel = marks ? start - base - lane : 64;
    asm volatile("" : "+v"(rel)); // keep `mine + rel` (the compiler would re-derive the base)
    mine[rel] = marks ? lane + 1 : 0;
    const int m = (int)wave_incl_umax((uint32_t)mine[0]) - 1;
    return max(m, carry);
#endif
}

// block -> 16x16 tile, remapped so each XCD (blocks b, b+8, ...) owns one
// contiguous band of tiles; bijective for any block count
__device__ __forceinline__ int xcd_tile(int b, int nb)
{
    const int q = nb / 8, r = nb % 8, xcd = b % 8, k = b / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

} // namespace rtk
