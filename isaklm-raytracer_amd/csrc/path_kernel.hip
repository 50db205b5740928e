// path_kernel.hip — gfx950 kernels of the render hot path.
//
// Replaces rt/path_tracing.cuh (kernel path_tracing :338-395, trace_path
// :268-325, BSDF :45-219, NEE :222-265), rt/trace_ray.cuh (trace_ray
// :244-318, trace_leaf_node :115-172, intersect_triangle :73-113) and the
// reset_frame / draw_frame kernels of rt/render.cuh:18-59.
//
// Design (MI355X-first, not a translation):
//  * one lane owns one pixel for all `passes` of a launch: RNG state,
//    fb/sq/count live in VGPRs and hit HBM once per launch (the reference
//    does a global read-modify-write per RNG draw and one launch per pass);
//  * a lane whose path ends starts its pixel's next pass immediately (path
//    regeneration), so a wave is not held by its longest path each pass;
//  * every loop iteration issues exactly one ray query from one call site:
//    extension rays and NEE shadow rays (rt/path_tracing.cuh:235-265) are two
//    states of the same loop, so lanes in either state traverse together;
//  * waves are 8x8 pixel tiles and blocks 16x16 tiles, remapped so that each
//    XCD (private L2) renders one contiguous band of the image;
//  * KD stack (node, entry t) in LDS, [depth][lane] => conflict-free; the
//    exit t of a popped entry equals the entry t of the one below it (or the
//    root's exit), so it is not stored;
//  * triangle constants precomputed (rt_device.h); a plane-rejected test
//    reads 16 bytes.
// Arithmetic is the reference's, operation for operation, compiled with
// -ffp-contract=off; sin/cos come from rt_libm.h; division and sqrt are
// IEEE-rounded (hipcc default).  Results are bit-identical to the CPU oracle.
#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_vecmath.h"

#define RT_BLOCK 256

namespace {

enum { PRIMARY = 0, DIFFUSE = 1, SPECULAR = 2, METALLIC = 3, TRANSMISSION = 4 }; // :18-25

struct Cnt {
    unsigned long long v[9];
};

__device__ __forceinline__ float as_float(uint32_t u) { return __uint_as_float(u); }

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

// trace_ray (rt/trace_ray.cuh:244-318): closest hit inside the first leaf
// (front to back) that has one.  Returns the triangle index or -1 and the
// barycentric coordinates of the hit.
template <bool COUNT, int STACK>
__device__ __forceinline__ int trace(const RtDevScene &sc, const Vec3D o, const Vec3D d, float &hbx, float &hby,
                                     float &hbz, uint32_t *s_node, float *s_entry, Cnt &c)
{
    if (COUNT) c.v[RT_CNT_RAY]++;
    float entry, exit_;
    if (!bbox_hit(sc, o, d, entry, exit_)) return -1;
    const float root_exit = exit_;
    const float oa[3] = {o.x, o.y, o.z};
    const float da[3] = {d.x, d.y, d.z};
    int sp = 0;
    uint32_t node = 0;
    while (true) {
        uint2 nd = *reinterpret_cast<const uint2 *>(sc.nodes + 2 * (size_t)node);
        if (COUNT) c.v[RT_CNT_NODE]++;
        while ((nd.y & 3u) != RT_LEAF_TAG) {
            const uint32_t axis = nd.y & 3u;
            const float split = as_float(nd.x);
            const float oax = axis == 0 ? oa[0] : (axis == 1 ? oa[1] : oa[2]);
            const float dax = axis == 0 ? da[0] : (axis == 1 ? da[1] : da[2]);
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
                s_node[sp * RT_BLOCK] = far_c;
                s_entry[sp * RT_BLOCK] = t;
                ++sp;
                node = near_c;
                exit_ = t;
            }
            nd = *reinterpret_cast<const uint2 *>(sc.nodes + 2 * (size_t)node);
            if (COUNT) c.v[RT_CNT_NODE]++;
        }
        const int count = (int)(nd.y >> 2);
        if (count > 0) {
            // trace_leaf_node (:115-172) + intersect_triangle (:73-113)
            const int *idx = sc.leaf_tris + nd.x;
            float smallest = exit_;
            int best = -1;
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            for (int i = 0; i < count; ++i) {
                const int tri = idx[i];
                if (COUNT) c.v[RT_CNT_TRI]++;
                const RtF4 A = ldf4(sc.isect_a + tri); // n, d
                const float dn = d.x * A.x + d.y * A.y + d.z * A.z;
                if (dn == 0) continue;
                const float s = (A.w - (o.x * A.x + o.y * A.y + o.z * A.z)) / dn;
                if (s < 0.00001f || !(s < smallest)) continue;
                const RtF4 B = ldf4(sc.isect_b + tri); // p1, d00
                const RtF4 C = ldf4(sc.isect_c + tri); // v0, d01
                const RtF4 D = ldf4(sc.isect_d + tri); // v1, d11
                const float rd = sc.isect_r[tri];
                const float px = o.x + d.x * s, py = o.y + d.y * s, pz = o.z + d.z * s;
                const float v2x = px - B.x, v2y = py - B.y, v2z = pz - B.z;
                const float d20 = v2x * C.x + v2y * C.y + v2z * C.z;
                const float d21 = v2x * D.x + v2y * D.y + v2z * D.z;
                const float cy = (D.w * d20 - C.w * d21) * rd;
                const float cz = (B.w * d21 - C.w * d20) * rd;
                const float cx = 1.0f - cy - cz;
                if (cx >= 0.0f && cx <= 1.0f && cy >= 0.0f && cy <= 1.0f && cz >= 0.0f && cz <= 1.0f) {
                    smallest = s;
                    best = tri;
                    bx = cx;
                    by = cy;
                    bz = cz;
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
        node = s_node[sp * RT_BLOCK];
        entry = s_entry[sp * RT_BLOCK];
        exit_ = sp > 0 ? s_entry[(sp - 1) * RT_BLOCK] : root_exit;
    }
}

// sample_texture (rt/trace_ray.cuh:31-46)
__device__ __forceinline__ Vec3D sample_texture(const RtDevMaterial &m, Vec3D blend, Vec2D uv)
{
    if (m.tex == nullptr) return blend;
    float u = rt_mod(uv.x, 1.0f);
    float v = rt_mod(uv.y, 1.0f);
    int pn = (int)((float)((int)(v * (float)m.tex_height) * m.tex_width) + (u * (float)m.tex_width));
    RtUChar4 c = m.tex[pn];
    return rt_v3(c.x / (float)RT_MAX_COLOR_CHANNEL, c.y / (float)RT_MAX_COLOR_CHANNEL,
                 c.z / (float)RT_MAX_COLOR_CHANNEL) *
           blend;
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

// the part of the hit Sample sample_direct_light uses (normal, emittance)
template <bool COUNT>
__device__ __forceinline__ void shade_light(const RtDevScene &sc, int tri, float bx, float by, float bz, Vec3D dir,
                                            Vec3D &normal, Vec3D &emittance, Cnt &c)
{
    const RtF4 *r = sc.shade + 7 * (size_t)tri;
    const RtF4 s0 = ldf4(r), s1 = ldf4(r + 1), s2 = ldf4(r + 2), s3 = ldf4(r + 3), s4 = ldf4(r + 4),
               s5 = ldf4(r + 5), s6 = ldf4(r + 6);
    const RtDevMaterial &m = sc.materials[__float_as_uint(s0.w)];
    Vec2D uv = rt_v2(s1.w, s2.w) * bx + rt_v2(s3.w, s4.w) * by + rt_v2(s5.w, s6.x) * bz;
    emittance = sample_texture(m, rt_v3(m.emittance[0], m.emittance[1], m.emittance[2]), uv);
    normal = rt_normalize(bx * ld3(s3) + by * ld3(s4) + bz * ld3(s5));
    if (rt_dot(dir, normal) > 0) normal = -normal;
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

// get_scattered_light (:151-219): returns the new direction, weight and type
__device__ __forceinline__ int scatter(Vec3D dir, bool &inside, uint32_t &rng, const Surface &s, Vec3D &out_dir,
                                       Vec3D &weight)
{
    dir = -dir;
    // microfacet_normal (:103-118), FP64 island
    double ru = rng_next(rng);
    float cos_theta = sqrtf((float)((1.0f - ru) / (ru * (double)(s.roughness * s.roughness - 1.0f) + 1.0f)));
    float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
    float phi = rng_next(rng) * RT_TAU;
    float cos_phi = rt_cosf(phi);
    float sin_phi = rt_sinf(phi);
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
    float ds = rt_sinf(dphi);
    float dc = rt_cosf(dphi);
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

// block -> 16x16 tile, remapped so each XCD (blocks b, b+8, ...) owns one
// contiguous band of tiles; bijective for any block count
__device__ __forceinline__ int xcd_tile(int b, int nb)
{
    const int q = nb / 8, r = nb % 8, xcd = b % 8, k = b / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

} // namespace

// path_tracing (rt/path_tracing.cuh:338-395) for `passes` passes, with
// reset_frame (rt/render.cuh:18-34) fused in when fr.reset is set.
template <bool COUNT, int STACK>
__global__ void __launch_bounds__(RT_BLOCK) rt_path_kernel(RtDevScene sc, RtDevFrame fr, RtDevCamera cam)
{
    __shared__ uint32_t s_node[STACK * RT_BLOCK];
    __shared__ float s_entry[STACK * RT_BLOCK];
    const int tid = threadIdx.x;
    const int tiles_x = (fr.width + 15) / 16;
    const int tile = xcd_tile(blockIdx.x, gridDim.x);
    const int wave = tid >> 6, lane = tid & 63;
    const int x = (tile % tiles_x) * 16 + (wave & 1) * 8 + (lane & 7);
    const int y = (tile / tiles_x) * 16 + (wave >> 1) * 8 + (lane >> 3);
    if (x >= fr.width || y >= fr.height) return;
    const int pi = y * fr.width + x;
    uint32_t *sn = s_node + tid;
    float *se = s_entry + tid;

    Cnt c;
    if (COUNT)
        for (int k = 0; k < 9; ++k) c.v[k] = 0;

    uint32_t rng = fr.rng[pi];
    Vec3D fb;
    float sq;
    int count;
    if (fr.reset) {
        fb = rt_v3(0.0f, 0.0f, 0.0f);
        sq = 0.0f;
        count = 0;
    } else {
        fb = fr.fb[pi];
        sq = fr.sq[pi];
        count = fr.count[pi];
    }

    int passes_left = fr.passes;
    bool have_path = false;
    bool shadow = false;  // current query is an NEE shadow ray
    bool inside = false;  // inside_medium
    int prev_type = PRIMARY;
    int depth = 0;
    int light = 0;
    const int limit = fr.max_depth > 0 ? fr.max_depth : RT_WATCHDOG_BOUNCES;
    Vec3D ro = rt_v3(0, 0, 0), rd = rt_v3(0, 0, 0); // ray being traced
    Vec3D cont = rt_v3(0, 0, 0);                     // scattered direction waiting behind a shadow ray
    Vec3D sn_normal = rt_v3(0, 0, 0), rp = rt_v3(0, 0, 0);
    Vec3D T = rt_v3(1, 1, 1), L = rt_v3(0, 0, 0);

    while (true) {
        if (!have_path) {
            while (passes_left > 0) {
                --passes_left;
                bool run = true;
                if (fr.adaptive && count >= fr.min_samples) { // :352-376
                    float tl = rt_luminance(fb);
                    float mean = tl / (float)count;
                    float var = (sq - rt_square(tl) / (float)count) / (float)(count - 1);
                    float iw = fr.z_const * sqrtf(var / (float)count);
                    run = iw > mean * fr.tolerance;
                }
                if (!run) {
                    if (COUNT) c.v[RT_CNT_SKIP]++;
                    continue;
                }
                // camera ray (:381-391) and random_point_in_pinhole (:327-336)
                float rx = rng_next(rng);
                float ry = rng_next(rng);
                Vec3D dir = rt_normalize(
                    rt_v3(cam.tan_half_fov * ((float)x + rx - (float)fr.half_w) / (float)fr.half_w,
                          cam.tan_half_fov * ((float)y + ry - (float)fr.half_h) / (float)fr.half_w, 1.0f));
                rd = mat_mul(cam.R, dir);
                float theta = rng_next(rng) * RT_TAU;
                float r = sqrtf(rng_next(rng)) * cam.aperture;
                float ox = r * rt_cosf(theta);
                float oy = r * rt_sinf(theta);
                ro = rt_v3(cam.pos[0], cam.pos[1], cam.pos[2]) + mat_mul(cam.R, rt_v3(ox, 0.0f, 0.0f)) +
                     mat_mul(cam.R, rt_v3(0.0f, oy, 0.0f));
                T = rt_v3(1.0f, 1.0f, 1.0f);
                L = rt_v3(0.0f, 0.0f, 0.0f);
                inside = false;
                prev_type = PRIMARY;
                depth = 0;
                shadow = false;
                have_path = true;
                if (COUNT) c.v[RT_CNT_SAMPLE]++;
                break;
            }
            if (!have_path) break;
        }

        bool finish = false;
        if (!shadow && depth == limit) { // max_depth / watchdog
            if (COUNT && fr.max_depth <= 0) c.v[RT_CNT_WATCHDOG]++;
            finish = true;
        } else {
            if (!shadow) ++depth;
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            const int hit = trace<COUNT, STACK>(sc, ro, rd, bx, by, bz, sn, se, c);
            bool roulette = true;
            if (!shadow) {
                if (hit < 0) {
                    finish = true; // miss: break without roulette (:303-306)
                    roulette = false;
                } else {
                    Surface s;
                    shade<COUNT>(sc, hit, bx, by, bz, rd, s, c);
                    if (prev_type != DIFFUSE) L = L + s.emittance * T; // :285-288
                    Vec3D nd, w;
                    prev_type = scatter(rd, inside, rng, s, nd, w);
                    T = T * w;
                    ro = s.position;
                    rd = nd;
                    if (prev_type == DIFFUSE) { // sample_direct_light (:235-265)
                        if (COUNT) c.v[RT_CNT_NEE]++;
                        float xi = rng_next(rng);
                        if (sc.light_count == 0) {
                            rng_next(rng);
                            rng_next(rng);
                            L = L + rt_v3(0.0f, 0.0f, 0.0f) * T;
                        } else {
                            light = sc.lights[(int)(xi * (float)sc.light_count)];
                            const RtF4 *lr = sc.shade + 7 * (size_t)light;
                            const Vec3D lp1 = ld3(ldf4(lr)), lp2 = ld3(ldf4(lr + 1)), lp3 = ld3(ldf4(lr + 2));
                            // random_point_in_triangle (:222-233)
                            float px = rng_next(rng);
                            float py = rng_next(rng);
                            float sx = sqrtf(px);
                            float u = 1.0f - sx;
                            float v = py * sx;
                            float wgt = 1.0f - u - v;
                            rp = u * lp1 + v * lp2 + wgt * lp3;
                            cont = rd;
                            sn_normal = s.normal;
                            rd = rt_normalize(rp - ro);
                            shadow = true;
                            roulette = false; // roulette after the shadow ray
                        }
                    }
                }
            } else {
                Vec3D direct = rt_v3(0.0f, 0.0f, 0.0f);
                if (hit >= 0 && hit == light) {
                    Vec3D ln, le;
                    shade_light<COUNT>(sc, hit, bx, by, bz, rd, ln, le, c);
                    const RtF4 *lr = sc.shade + 7 * (size_t)light;
                    const Vec3D lp1 = ld3(ldf4(lr)), lp2 = ld3(ldf4(lr + 1)), lp3 = ld3(ldf4(lr + 2));
                    float area = (float)(0.5 * (double)rt_magnitude(rt_cross(lp2 - lp1, lp3 - lp1)));
                    float d2 = rt_magnitude_squared(rp - ro);
                    float c1 = fmaxf(-rt_dot(rd, ln), 0.0f);
                    float c2 = fmaxf(rt_dot(rd, sn_normal), 0.0f);
                    direct = le * (area * (float)sc.light_count * c1 * c2 / fmaxf(d2 * RT_PI, 0.001f));
                }
                if (COUNT && hit >= 0) { // the reference shades every hit (2 texel reads if textured)
                    const RtDevMaterial &m = sc.materials[__float_as_uint(sc.shade[7 * (size_t)hit].w)];
                    if (m.tex) c.v[RT_CNT_TEXEL] += 2;
                }
                L = L + direct * T;
                rd = cont;
                shadow = false;
            }
            if (roulette) { // Russian roulette (:309-318)
                float p = fmaxf(T.x, fmaxf(T.y, T.z));
                float r = rng_next(rng);
                if (r > p) finish = true;
                else T = T * (1.0f / p);
            }
        }
        if (finish) { // accumulation (:322-324)
            fb = fb + L;
            sq = sq + rt_square(rt_luminance(L));
            ++count;
            have_path = false;
        }
    }

    fr.fb[pi] = fb;
    fr.sq[pi] = sq;
    fr.count[pi] = count;
    fr.rng[pi] = rng;

    if (COUNT) {
        for (int k = 0; k < 9; ++k) {
            unsigned long long v = c.v[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            c.v[k] = v;
        }
        if (lane == 0)
            for (int k = 0; k < 9; ++k) atomicAdd(fr.counters + k, c.v[k]);
    }
}

// draw_frame colour math (rt/render.cuh:44-53) into an RGBA8 HBM buffer
__global__ void __launch_bounds__(256) rt_tonemap_kernel(const Vec3D *fb, const int *count, RtUChar4 *out, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    Vec3D c = fb[i] * (1.0f / (float)count[i]);
    c = rt_correct_color(c);
    RtUChar4 o;
    o.x = (uint8_t)(c.x * RT_MAX_COLOR_CHANNEL);
    o.y = (uint8_t)(c.y * RT_MAX_COLOR_CHANNEL);
    o.z = (uint8_t)(c.z * RT_MAX_COLOR_CHANNEL);
    o.w = RT_MAX_COLOR_CHANNEL;
    out[i] = o;
}

// ---- host launchers (called by abi.hip) ----
int rt_launch_path(const RtDevScene &sc, const RtDevFrame &fr, const RtDevCamera &cam, int stack_depth,
                   hipStream_t stream)
{
    const int tiles = ((fr.width + 15) / 16) * ((fr.height + 15) / 16);
    dim3 grid(tiles), block(RT_BLOCK);
    const bool count = fr.counters != nullptr;
    if (stack_depth <= 19) {
        if (count) hipLaunchKernelGGL((rt_path_kernel<true, 19>), grid, block, 0, stream, sc, fr, cam);
        else hipLaunchKernelGGL((rt_path_kernel<false, 19>), grid, block, 0, stream, sc, fr, cam);
    } else {
        if (count) hipLaunchKernelGGL((rt_path_kernel<true, RT_STACK_DEPTH>), grid, block, 0, stream, sc, fr, cam);
        else hipLaunchKernelGGL((rt_path_kernel<false, RT_STACK_DEPTH>), grid, block, 0, stream, sc, fr, cam);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int rt_launch_tonemap(const Vec3D *fb, const int *count, RtUChar4 *out, int n, hipStream_t stream)
{
    hipLaunchKernelGGL(rt_tonemap_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, fb, count, out, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
