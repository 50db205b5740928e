/*
 * rt_oracle.c — TEST INFRASTRUCTURE ONLY (see rt_oracle.h for the parity
 * status: "parity unpinned" for radiance, the reference being unbuildable
 * here).
 *
 * Plain-C restatement of INDA23PlusPlus/isaklm-raytracer's render path.
 * Every function cites the reference lines it restates (rt/ =
 * /root/reference/isaklm-raytracer/).  Expressions keep the reference's
 * evaluation order and implicit conversions (float*int, the double island in
 * microfacet_normal, ...).  Compiled with -O2 -ffp-contract=off -fno-fast-math
 * (oracle/Makefile) so no FMA contraction changes a rounding.
 *
 * Transcendentals come from the shared rt_libm.h (sinf/cosf/tanf/powf
 * stand-ins for CUDA libdevice, SURVEY §8c "one shared implementation").
 */
#define _POSIX_C_SOURCE 200809L
#include "rt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../isaklm-raytracer_amd/csrc/rt_libm.h"

/* ---------------------------------------------------------------- errors */
static char g_err[512];
static void set_err(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}
const char *or_last_error(void) { return g_err; }

/* ------------------------------------------- constants (rt/macros.h, math) */
#define KD_TREE_DEPTH 19                 /* rt/macros.h:11 */
#define MAX_COLOR_CHANNEL 255            /* rt/macros.h:9 */
#define PIF 3.1415926536f                /* rt/math_library.cuh:9 */
#define TAUF (PIF * 2)                   /* rt/math_library.cuh:10 */
#define WATCHDOG_BOUNCES ((1 << 24) - 1) /* as the product (rt_device.h); never fires in parity configs */
#define DEEP_PATH 64                     /* deviation histogram: paths ending at depth >= 64 */
#define DEEP_HIST_BINS 18

enum { CNT_NODE = 0, CNT_TRI, CNT_HIT, CNT_TEXEL, CNT_NEE, CNT_SAMPLE, CNT_SKIP, CNT_RAY, CNT_WATCHDOG, CNT_MAXDEPTH,
       CNT_DEEP_PUSH = 15 /* pushes at stack index >= KD_TREE_DEPTH: past the reference's arrays */,
       CNT_CUT = 16       /* paths cut at the depth limit (watchdog or max_depth) */,
       CNT_DEEP_HIST = 17 /* + k: paths ending at depth in [64 * 2^k, 64 * 2^(k+1)), k < DEEP_HIST_BINS
                             (the product's always-on RtDeviations, rt_deviation_stats) */,
       /* hazard instrumentation: how often an input
        * triggered each quirk the build reproduces, so a test can show it
        * was exercised */
       CNT_XI_ONE = 35,        /* H4: NEE light pick with xi == 1.0 (reads the padded entry) */
       CNT_EXIT_TIE = 36,      /* H6: an inside hit with t == the leaf's exit (deferred to a later leaf) */
       CNT_ON_SPLIT = 37,      /* H5: inner node visited with the ray origin exactly on its split */
       CNT_AXIS_PARALLEL = 38, /* H7: inner node visited with direction[axis] == 0 (t = +-inf / NaN) */
       CNT_DEGENERATE = 39     /* H7: triangle test with a NaN plane normal (zero-area triangle) */ };

/* ------------------------------------------------ types (rt/scene.cuh etc.) */
typedef struct { float x, y; } V2;                     /* rt/math_library.cuh:55-66 */
typedef struct { float x, y, z; } V3;                  /* rt/math_library.cuh:99-115 */
typedef struct { V3 i, j, k; } M3;                     /* rt/math_library.cuh:319-335 */
typedef struct { V3 position, direction; } Ray;        /* rt/math_library.cuh:312-316 */
typedef struct { uint8_t x, y, z, w; } UC4;

typedef struct { UC4 *buffer; int width, height; } Texture;                 /* rt/scene.cuh:16-21 */
typedef struct {                                                             /* rt/scene.cuh:65-74 */
    V3 albedo, emittance;
    float roughness, refractive_index, extinction;
    bool transparent;
    Texture texture;
} Material;
typedef struct {                                                             /* rt/scene.cuh:76-82 */
    V3 p1, p2, p3, n1, n2, n3;
    V2 uv1, uv2, uv3;
    Material material;
} Triangle;
typedef struct {                                                             /* rt/scene.cuh:84-100 */
    int a;            /* index_offset / child_index1 */
    int b;            /* triangle_count / child_index2 */
    uint8_t plane_axis;
    float plane_offset;
    bool is_leaf_node;
} Node;
typedef struct { V3 min, max; } BBox;                                        /* rt/scene.cuh:102-105 */

_Static_assert(sizeof(Triangle) == 152, "Triangle layout");
_Static_assert(sizeof(Node) == 20, "Node layout");
_Static_assert(sizeof(Material) == 56, "Material layout");

struct OrScene {
    Triangle *tris;
    int ntris;
    int *lights;       /* light_count + 1 entries, see SURVEY H4 */
    int nlights;
    Node *nodes;
    int nnodes, nodecap;
    int *indices;
    int nindices, indexcap;
    BBox bounds;
    unsigned char *degenerate; /* per triangle: NaN plane normal (test instrumentation, CNT_DEGENERATE) */
};

/* -------------------------------------------- math (rt/math_library.cuh) */
static inline float square(float x) { return x * x; }                        /* :17-20 */
static inline float clampf_(float x, float lo, float hi) { return fmaxf(lo, fminf(hi, x)); } /* :22-25 */
static inline float modf_(float x, float m) { return x - m * floorf(x / m); } /* :32-35 */
static inline V3 v3(float x, float y, float z) { V3 r = {x, y, z}; return r; }
static inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }  /* :117-120 */
static inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }  /* :122-125 */
static inline V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }                       /* :127-130 */
static inline V3 mulvs(V3 v, float s) { return v3(v.x * s, v.y * s, v.z * s); }   /* :132-140 */
static inline V3 mulvv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); } /* :142-145 */
static inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* :212-215 */
static inline V3 cross(V3 a, V3 b)                                                /* :217-220 */
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float magnitude(V3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); } /* :222-225 */
static inline float magnitude_squared(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; } /* :227-230 */
static inline V3 normalize(V3 v)                                                   /* :232-237 */
{
    float r = 1.0f / sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return v3(v.x * r, v.y * r, v.z * r);
}
static inline float luminance(V3 c) { return dot(c, v3(0.2126f, 0.7152f, 0.0722f)); } /* :263-266 */
static inline V2 mul2(V2 v, float s) { V2 r = {v.x * s, v.y * s}; return r; }   /* :78-86 */
static inline V2 add2(V2 a, V2 b) { V2 r = {a.x + b.x, a.y + b.y}; return r; }   /* :68-71 */

/* m * v = v.x*i + v.y*j + v.z*k  (:347-350) */
static inline V3 mmul(M3 m, V3 v) { return add(add(mulvs(m.i, v.x), mulvs(m.j, v.y)), mulvs(m.k, v.z)); }
/* m2 * m1 (:352-355) */
static inline M3 mmm(M3 m2, M3 m1) { M3 r = {mmul(m2, m1.i), mmul(m2, m1.j), mmul(m2, m1.k)}; return r; }
/* m * s = {s*i, s*j, s*k} (:337-340) */
static inline M3 mscale(M3 m, float s) { M3 r = {mulvs(m.i, s), mulvs(m.j, s), mulvs(m.k, s)}; return r; }

/* rotation_matrix(yaw, pitch, roll = 0)  (:384-408) */
static M3 rotation_matrix(float yaw, float pitch)
{
    float roll = 0.0f;
    M3 y = {{rt_cosf(yaw), 0.0f, -rt_sinf(yaw)}, {0.0f, 1.0f, 0.0f}, {rt_sinf(yaw), 0.0f, rt_cosf(yaw)}};
    M3 x = {{1.0f, 0.0f, 0.0f}, {0.0f, rt_cosf(pitch), rt_sinf(pitch)}, {0.0f, -rt_sinf(pitch), rt_cosf(pitch)}};
    M3 z = {{rt_cosf(roll), rt_sinf(roll), 0.0f}, {-rt_sinf(roll), rt_cosf(roll), 0.0f}, {0.0f, 0.0f, 1.0f}};
    return mmm(mmm(z, y), x);
}

/* gamma_correction (:37-47): double constants, powf with the exponent
 * 1.0/2.4 converted to float */
static float gamma_correction(float x)
{
    float output = (float)(12.92 * (double)x);
    if ((double)x > 0.0031308) output = (float)(1.055 * (double)rt_powf(x, (float)(1.0 / 2.4)) - 0.055);
    return output;
}
static float aces_curve(float x) /* :49-52 */
{
    return (x * (x + 0.0245786f) - 0.000090537f) / (x * (0.983729f * x + 0.4329510f) + 0.238081f);
}
static V3 aces_tone_mapping(V3 c) /* :422-443 */
{
    M3 in = {{0.59719f, 0.07600f, 0.02840f}, {0.35458f, 0.90834f, 0.13383f}, {0.04823f, 0.01566f, 0.83777f}};
    M3 out = {{1.60475f, -0.10208f, -0.00327f}, {-0.53108f, 1.10813f, -0.07276f}, {-0.07367f, -0.00605f, 1.07602f}};
    c = mmul(in, c);
    c = v3(aces_curve(c.x), aces_curve(c.y), aces_curve(c.z));
    return mmul(out, c);
}
static V3 correct_color(V3 c) /* :445-460 */
{
    c.x = fmaxf(c.x, 0.0f);
    c.y = fmaxf(c.y, 0.0f);
    c.z = fmaxf(c.z, 0.0f);
    c = aces_tone_mapping(c);
    c = v3(gamma_correction(c.x), gamma_correction(c.y), gamma_correction(c.z));
    c.x = clampf_(c.x, 0.0f, 1.0f);
    c.y = clampf_(c.y, 0.0f, 1.0f);
    c.z = clampf_(c.z, 0.0f, 1.0f);
    return c;
}
void or_correct_color(const float in[3], float out[3])
{
    V3 c = correct_color(v3(in[0], in[1], in[2]));
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}

/* ---------------------------------------------------------- mt19937 seeds */
/* std::mt19937 default-constructed (seed 5489) + uniform_int_distribution<
 * uint32_t>(0, UINT32_MAX) = raw 32-bit engine outputs (rt/screen.cuh:34-45). */
void or_mt19937(uint32_t *out, size_t count, uint64_t skip)
{
    uint32_t mt[624];
    mt[0] = 5489u;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    int idx = 624;
    uint64_t total = skip + count;
    for (uint64_t n = 0; n < total; ++n) {
        if (idx >= 624) {
            for (int i = 0; i < 624; ++i) {
                uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            idx = 0;
        }
        uint32_t y = mt[idx++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        if (n >= skip) out[n - skip] = y;
    }
}

/* ---------------------------------------- RNG (rt/path_tracing.cuh:34-43) */
static inline float rng_next(uint32_t *st)
{
    uint32_t state = *st * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    uint32_t r = (word >> 22u) ^ word;
    *st = r;
    return (float)r / (float)UINT32_MAX; /* float(x) / UINT32_MAX -> / 4294967296.0f */
}
float or_rng_next(uint32_t *state) { return rng_next(state); }

/* ----------------------------------------------- ray query (trace_ray.cuh) */
typedef struct {              /* rt/trace_ray.cuh:17-29 */
    V3 albedo, emittance;
    float roughness, refractive_index, extinction;
    bool transparent;
    int triangle_index;
    V3 position, normal, tangent, bitangent;
} Sample;

/* sample_texture (rt/trace_ray.cuh:31-46) */
static V3 sample_texture(Texture t, V3 blend, V2 uv, unsigned long long *cnt)
{
    if (t.buffer == NULL) return blend;
    uv.x = modf_(uv.x, 1.0f);
    uv.y = modf_(uv.y, 1.0f);
    /* int * int + float -> float -> int */
    int pixel_number = (int)((float)((int)(uv.y * (float)t.height) * t.width) + (uv.x * (float)t.width));
    UC4 c = t.buffer[pixel_number];
    cnt[CNT_TEXEL] += 1;
    return mulvv(v3(c.x / (float)MAX_COLOR_CHANNEL, c.y / (float)MAX_COLOR_CHANNEL, c.z / (float)MAX_COLOR_CHANNEL),
                 blend);
}

/* calculate_barycentric_coordinates (rt/trace_ray.cuh:48-71) */
static V3 barycentric(V3 p, const Triangle *t)
{
    V3 v0 = sub(t->p2, t->p1), v1 = sub(t->p3, t->p1), v2 = sub(p, t->p1);
    float d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1), d20 = dot(v2, v0), d21 = dot(v2, v1);
    float rd = 1.0f / (d00 * d11 - d01 * d01);
    V3 b = {0.0f, 0.0f, 0.0f};
    b.y = (d11 * d20 - d01 * d21) * rd;
    b.z = (d00 * d21 - d01 * d20) * rd;
    b.x = 1.0f - b.y - b.z;
    return b;
}

/* intersect_triangle (rt/trace_ray.cuh:73-113) */
static bool intersect_triangle(Ray ray, const Triangle *t, V3 *bary, float *tt)
{
    V3 n = normalize(cross(sub(t->p2, t->p1), sub(t->p3, t->p1)));
    float dn = dot(ray.direction, n);
    if (dn == 0) return false;
    float d = dot(n, t->p1);
    float s = (d - dot(ray.position, n)) / dn;
    if (s < 0.00001f) return false;
    *tt = s;
    V3 p = add(ray.position, mulvs(ray.direction, s));
    V3 b = barycentric(p, t);
    if (b.x >= 0.0f && b.x <= 1.0f && b.y >= 0.0f && b.y <= 1.0f && b.z >= 0.0f && b.z <= 1.0f) {
        *bary = b;
        return true;
    }
    return false;
}

/* trace_leaf_node (rt/trace_ray.cuh:115-172) */
static bool trace_leaf(const OrScene *sc, Ray ray, float max_t, int off, int count, Sample *sm,
                       unsigned long long *cnt)
{
    bool hit = false;
    int ti = -1;
    V3 bc = {0.0f, 0.0f, 0.0f};
    float smallest = max_t;
    for (int i = 0; i < count; ++i) {
        int index = sc->indices[off + i];
        const Triangle *t = &sc->tris[index];
        V3 b = {0.0f, 0.0f, 0.0f};
        float tt = FLT_MAX;
        cnt[CNT_TRI] += 1;
        const bool inside = intersect_triangle(ray, t, &b, &tt);
        if (inside && tt == max_t) cnt[CNT_EXIT_TIE] += 1;
        if (sc->degenerate[index]) cnt[CNT_DEGENERATE] += 1;
        if (inside && (tt < smallest)) {
            hit = true;
            smallest = tt;
            ti = index;
            bc = b;
        }
    }
    if (hit) {
        const Triangle *t = &sc->tris[ti];
        cnt[CNT_HIT] += 1;
        V2 uv = add2(add2(mul2(t->uv1, bc.x), mul2(t->uv2, bc.y)), mul2(t->uv3, bc.z));
        sm->albedo = sample_texture(t->material.texture, t->material.albedo, uv, cnt);
        sm->emittance = sample_texture(t->material.texture, t->material.emittance, uv, cnt);
        sm->roughness = t->material.roughness;
        sm->refractive_index = t->material.refractive_index;
        sm->extinction = t->material.extinction;
        sm->transparent = t->material.transparent;
        sm->triangle_index = ti;
        sm->position = add(add(mulvs(t->p1, bc.x), mulvs(t->p2, bc.y)), mulvs(t->p3, bc.z));
        sm->normal = normalize(add(add(mulvs(t->n1, bc.x), mulvs(t->n2, bc.y)), mulvs(t->n3, bc.z)));
        sm->tangent = normalize(cross(sub(t->p2, t->p1), sm->normal));
        sm->bitangent = normalize(cross(sm->normal, sm->tangent));
        if (dot(ray.direction, sm->normal) > 0) sm->normal = neg(sm->normal);
    }
    return hit;
}

static inline float axis_of(V3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

/* intersect_bounding_box (rt/trace_ray.cuh:212-242) */
static bool intersect_bbox(Ray r, BBox b, float *t1, float *t2)
{
    V3 tmin, tmax;
    tmin.x = (b.min.x - r.position.x) / r.direction.x;
    tmin.y = (b.min.y - r.position.y) / r.direction.y;
    tmin.z = (b.min.z - r.position.z) / r.direction.z;
    tmax.x = (b.max.x - r.position.x) / r.direction.x;
    tmax.y = (b.max.y - r.position.y) / r.direction.y;
    tmax.z = (b.max.z - r.position.z) / r.direction.z;
    V3 s1 = {fminf(tmin.x, tmax.x), fminf(tmin.y, tmax.y), fminf(tmin.z, tmax.z)};
    V3 s2 = {fmaxf(tmin.x, tmax.x), fmaxf(tmin.y, tmax.y), fmaxf(tmin.z, tmax.z)};
    float tn = fmaxf(fmaxf(s1.x, s1.y), s1.z);
    float tf = fminf(fminf(s2.x, s2.y), s2.z);
    *t1 = tn;
    *t2 = tf;
    return tn <= tf;
}

/* analysis aids (single-threaded use only): a log of traced rays, and of the
 * (descent steps, leaf size) sequence of each traversal */
static float *g_raylog = NULL;
static int g_raylog_n = 0, g_raylog_cap = 0;
static int *g_visits = NULL;
static int g_visits_n = 0, g_visits_cap = 0;

/* trace_ray (rt/trace_ray.cuh:244-318) with ray_behind_plane (:174-188) and
 * intersect_plane (:190-210) inlined */
static bool trace_ray(const OrScene *sc, Ray ray, Sample *sm, unsigned long long *cnt)
{
    int node_idx[KD_TREE_DEPTH + 8];
    float entry_d[KD_TREE_DEPTH + 8], exit_d[KD_TREE_DEPTH + 8];
    float t1, t2;
    cnt[CNT_RAY] += 1;
    if (g_raylog && g_raylog_n < g_raylog_cap) {
        float *r = g_raylog + 6 * g_raylog_n++;
        r[0] = ray.position.x; r[1] = ray.position.y; r[2] = ray.position.z;
        r[3] = ray.direction.x; r[4] = ray.direction.y; r[5] = ray.direction.z;
    }
    unsigned long long nodes_before = cnt[CNT_NODE];
    if (!intersect_bbox(ray, sc->bounds, &t1, &t2)) return false;
    node_idx[0] = 0;
    entry_d[0] = t1;
    exit_d[0] = t2;
    int sp = 1;
    while (sp > 0) {
        --sp;
        Node node = sc->nodes[node_idx[sp]];
        cnt[CNT_NODE] += 1;
        float entry = entry_d[sp];
        float exit_ = exit_d[sp];
        while (!node.is_leaf_node) {
            int near_i = node.a, far_i = node.b;
            if (axis_of(ray.position, node.plane_axis) == node.plane_offset) cnt[CNT_ON_SPLIT] += 1;
            if (axis_of(ray.direction, node.plane_axis) == 0.0f) cnt[CNT_AXIS_PARALLEL] += 1;
            if (axis_of(ray.position, node.plane_axis) >= node.plane_offset) {
                near_i = node.b;
                far_i = node.a;
            }
            float t = (node.plane_offset - axis_of(ray.position, node.plane_axis)) /
                      axis_of(ray.direction, node.plane_axis);
            if (t >= exit_ || t < 0) {
                node = sc->nodes[near_i];
            } else if (t <= entry) {
                node = sc->nodes[far_i];
            } else {
                if (sp >= KD_TREE_DEPTH + 8) abort(); /* reference: stack overflow is UB */
                if (sp >= KD_TREE_DEPTH) cnt[CNT_DEEP_PUSH] += 1; /* rt/trace_ray.cuh:246-248 hold 19 */
                node_idx[sp] = far_i;
                entry_d[sp] = t;
                exit_d[sp] = exit_;
                ++sp;
                node = sc->nodes[near_i];
                exit_ = t;
            }
            cnt[CNT_NODE] += 1;
        }
        if (g_visits && g_visits_n + 2 <= g_visits_cap) {
            g_visits[g_visits_n++] = (int)(cnt[CNT_NODE] - nodes_before);
            g_visits[g_visits_n++] = node.b;
            nodes_before = cnt[CNT_NODE];
        }
        if (node.b > 0) {
            if (trace_leaf(sc, ray, exit_, node.a, node.b, sm, cnt)) return true;
        }
    }
    return false;
}

/* analysis: path-trace `pixels` (1 pass each, single thread) logging every traced ray */
int or_log_rays(const OrScene *s, const float cam[7], int width, int height, const int *pixels, int npix,
                float *rays_out, int max_rays)
{
    OrOptions o;
    or_default_options(&o);
    o.width = width;
    o.height = height;
    o.adaptive = 0;
    o.threads = 1;
    int n = width * height;
    float *fb = (float *)calloc((size_t)n * 3, sizeof(float));
    float *sq = (float *)calloc((size_t)n, sizeof(float));
    int *count = (int *)calloc((size_t)n, sizeof(int));
    uint32_t *rng = (uint32_t *)malloc((size_t)n * sizeof(uint32_t));
    or_mt19937(rng, (size_t)n, 0);
    g_raylog = rays_out;
    g_raylog_n = 0;
    g_raylog_cap = max_rays;
    or_render(s, cam, fb, sq, count, rng, pixels, npix, 0, &o, NULL);
    int got = g_raylog_n;
    g_raylog = NULL;
    free(fb); free(sq); free(count); free(rng);
    return got;
}

/* analysis: per ray, the sequence of (descent node fetches, leaf size) pairs.
 * offsets[i]..offsets[i+1] index pairs in visits_out (2 ints each). */
int or_trace_visits(const OrScene *s, const float *rays6, int n, int *offsets, int *visits_out, int cap_ints)
{
    unsigned long long cnt[OR_CNT_COUNT] = {0};
    g_visits = visits_out;
    g_visits_n = 0;
    g_visits_cap = cap_ints;
    for (int i = 0; i < n; ++i) {
        offsets[i] = g_visits_n / 2;
        Ray r = {v3(rays6[6 * i], rays6[6 * i + 1], rays6[6 * i + 2]),
                 v3(rays6[6 * i + 3], rays6[6 * i + 4], rays6[6 * i + 5])};
        Sample sm;
        trace_ray(s, r, &sm, cnt);
    }
    offsets[n] = g_visits_n / 2;
    g_visits = NULL;
    return offsets[n];
}

void or_trace_rays(const OrScene *s, const float *rays6, int n, float *out12)
{
    unsigned long long cnt[OR_CNT_COUNT] = {0};
    for (int i = 0; i < n; ++i) {
        Ray r = {v3(rays6[6 * i], rays6[6 * i + 1], rays6[6 * i + 2]),
                 v3(rays6[6 * i + 3], rays6[6 * i + 4], rays6[6 * i + 5])};
        Sample sm;
        memset(&sm, 0, sizeof sm);
        bool h = trace_ray(s, r, &sm, cnt);
        float *o = out12 + 12 * i;
        o[0] = h ? 1.0f : 0.0f;
        o[1] = h ? (float)sm.triangle_index : -1.0f;
        o[2] = sm.position.x; o[3] = sm.position.y; o[4] = sm.position.z;
        o[5] = sm.normal.x; o[6] = sm.normal.y; o[7] = sm.normal.z;
        o[8] = sm.tangent.x; o[9] = sm.tangent.y; o[10] = sm.tangent.z;
        o[11] = 0.0f;
    }
}

/* the shared transcendentals (rt_libm.h) for tests: kind 0 sinf, 1 cosf, 2 tanf, 3 powf(x, 1/2.4) */
void or_libm(int kind, const float *in, float *out, int n)
{
    for (int i = 0; i < n; ++i) {
        switch (kind) {
        case 0: out[i] = rt_sinf(in[i]); break;
        case 1: out[i] = rt_cosf(in[i]); break;
        case 2: out[i] = rt_tanf(in[i]); break;
        default: out[i] = rt_powf(in[i], (float)(1.0 / 2.4)); break;
        }
    }
}

/* per-ray work statistics (analysis aid): out per ray = [nodes, tris, hit] */
void or_trace_stats(const OrScene *s, const float *rays6, int n, unsigned long long *out3)
{
#pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < n; ++i) {
        unsigned long long cnt[OR_CNT_COUNT] = {0};
        Ray r = {v3(rays6[6 * i], rays6[6 * i + 1], rays6[6 * i + 2]),
                 v3(rays6[6 * i + 3], rays6[6 * i + 4], rays6[6 * i + 5])};
        Sample sm;
        bool h = trace_ray(s, r, &sm, cnt);
        out3[3 * i] = cnt[CNT_NODE];
        out3[3 * i + 1] = cnt[CNT_TRI];
        out3[3 * i + 2] = h ? 1 : 0;
    }
}

/* ------------------------------------------- BSDF (rt/path_tracing.cuh) */
enum { PRIMARY, DIFFUSE, SPECULAR, METALLIC, TRANSMISSION }; /* :18-25 */
typedef struct { Ray ray; V3 weight; int type; } Event;     /* :27-32 */

static V3 diffuse_direction(uint32_t *rng, V3 n, V3 t, V3 b) /* :45-59 */
{
    float phi = rng_next(rng) * TAUF;
    float sin_phi = rt_sinf(phi);
    float cos_phi = rt_cosf(phi);
    float ru = rng_next(rng);
    float sq = sqrtf(ru);
    return add(add(mulvs(t, sq * cos_phi), mulvs(n, sqrtf(1.0f - ru))), mulvs(b, sq * sin_phi));
}
static float fresnel_dielectric(V3 i, V3 h, float n1, float n2) /* :61-74 */
{
    float c = fabsf(dot(i, h));
    float g = sqrtf(fmaxf(square(n2) / square(n1) - 1.0f + square(c), 0.0f));
    float f1 = 0.5f * square((g - c) / (g + c));
    float f2 = 1.0f + square((c * (g + c) - 1.0f) / (c * (g - c) + 1.0f));
    return f1 * f2;
}
static float fresnel_conductor(V3 i, V3 h, float n, float k) /* :76-101 */
{
    float n2 = n * n, k2 = k * k;
    float cs = dot(i, h);
    float cs2 = square(cs);
    float sn2 = 1.0f - cs2;
    float t0 = n2 - k2 - sn2;
    float a2b2 = sqrtf(square(t0) + 4.0f * n2 * k2);
    float a = sqrtf(0.5f * (a2b2 + t0));
    float t1 = a2b2 + cs2;
    float t2 = 2.0f * a * cs;
    float rs = (t1 - t2) / (t1 + t2);
    float t3 = cs2 * a2b2 * square(sn2);
    float t4 = t2 * sn2;
    float rp = rs * (t3 - t4) / (t3 + t4);
    return (rs + rp) * 0.5f;
}
static V3 microfacet_normal(uint32_t *rng, V3 n, V3 t, V3 b, float rough) /* :103-118 */
{
    double ru = rng_next(rng); /* the FP64 island */
    float cos_theta = sqrtf((float)((1.0f - ru) / (ru * (double)(rough * rough - 1.0f) + 1.0f)));
    float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
    float phi = rng_next(rng) * TAUF;
    float cos_phi = rt_cosf(phi);
    float sin_phi = rt_sinf(phi);
    return add(add(mulvs(mulvs(t, sin_theta), cos_phi), mulvs(n, cos_theta)), mulvs(mulvs(b, sin_theta), sin_phi));
}
static float lambda_(V3 d, V3 n, float rough) /* :120-127 */
{
    float dn = dot(d, n);
    float dn2 = square(dn);
    float tan2 = (1 - dn2) / dn2;
    return (sqrtf(1.0f + square(rough) + tan2) - 1.0f) * 0.5f;
}
static V3 specular_weight(V3 i, V3 o, V3 h, V3 n, float rough) /* :129-136 */
{
    float g = 1.0f / (1.0f + lambda_(i, n, rough) + lambda_(o, n, rough));
    float w = fabsf(dot(i, h)) * g / (fabsf(dot(n, h) * fabsf(dot(i, n))));
    return v3(w, w, w);
}
static V3 specular_direction(V3 i, V3 h) { return sub(mulvs(h, 2.0f * dot(i, h)), i); } /* :138-141 */
static V3 refraction_direction(V3 i, V3 h, float n1, float n2)                           /* :143-149 */
{
    float c = dot(i, h);
    float n = n1 / n2;
    return sub(mulvs(h, n * c - sqrtf(fmaxf(1.0f + n * n * (c * c - 1.0f), 0.0f))), mulvs(i, n));
}

/* get_scattered_light (:151-219) */
static Event scatter(V3 dir, bool *inside, uint32_t *rng, const Sample *s)
{
    dir = neg(dir);
    V3 h = microfacet_normal(rng, s->normal, s->tangent, s->bitangent, s->roughness);
    Event e;
    if (s->extinction > 0.0f) {
        float F = fresnel_conductor(dir, h, s->refractive_index, s->extinction);
        V3 o = specular_direction(dir, h);
        e.ray.position = s->position;
        e.ray.direction = o;
        e.weight = mulvs(mulvv(s->albedo, specular_weight(dir, o, h, s->normal, s->roughness)), F);
        e.type = METALLIC;
        return e;
    }
    float n1 = 1.0f, n2 = s->refractive_index;
    if (*inside) {
        n1 = n2;
        n2 = 1.0f;
    }
    float F = fresnel_dielectric(dir, h, n1, n2);
    float choose = rng_next(rng);
    e.ray.position = s->position;
    if (choose < F) {
        V3 o = specular_direction(dir, h);
        V3 w = v3(1.0f, 1.0f, 1.0f);
        if (!*inside) w = specular_weight(dir, o, h, s->normal, s->roughness);
        e.ray.direction = o;
        e.weight = w;
        e.type = SPECULAR;
    } else if (s->transparent) {
        *inside = !*inside;
        V3 o = refraction_direction(dir, h, n1, n2);
        e.ray.direction = o;
        e.weight = mulvv(specular_weight(dir, o, h, s->normal, s->roughness), s->albedo);
        e.type = TRANSMISSION;
    } else {
        e.ray.direction = diffuse_direction(rng, s->normal, s->tangent, s->bitangent);
        e.weight = s->albedo;
        e.type = DIFFUSE;
    }
    return e;
}

void or_scatter(const float d[3], const float s[22], int inside, uint32_t rng, float out[12],
                uint32_t *rng_out, int *inside_out, int *type_out)
{
    Sample sm;
    memset(&sm, 0, sizeof sm);
    sm.albedo = v3(s[0], s[1], s[2]);
    sm.emittance = v3(s[3], s[4], s[5]);
    sm.roughness = s[6];
    sm.refractive_index = s[7];
    sm.extinction = s[8];
    sm.transparent = s[9] != 0.0f;
    sm.position = v3(s[10], s[11], s[12]);
    sm.normal = v3(s[13], s[14], s[15]);
    sm.tangent = v3(s[16], s[17], s[18]);
    sm.bitangent = v3(s[19], s[20], s[21]);
    bool in = inside != 0;
    Event e = scatter(v3(d[0], d[1], d[2]), &in, &rng, &sm);
    out[0] = e.ray.position.x; out[1] = e.ray.position.y; out[2] = e.ray.position.z;
    out[3] = e.ray.direction.x; out[4] = e.ray.direction.y; out[5] = e.ray.direction.z;
    out[6] = e.weight.x; out[7] = e.weight.y; out[8] = e.weight.z;
    out[9] = out[10] = out[11] = 0.0f;
    *rng_out = rng;
    *inside_out = in;
    *type_out = e.type;
}

/* random_point_in_triangle (:222-233) */
static V3 random_point_in_triangle(const Triangle *t, uint32_t *rng)
{
    float x = rng_next(rng);
    float y = rng_next(rng);
    float sx = sqrtf(x);
    float u = 1.0f - sx;
    float v = y * sx;
    float w = 1.0f - u - v;
    return add(add(mulvs(t->p1, u), mulvs(t->p2, v)), mulvs(t->p3, w));
}

/* sample_direct_light (:235-265).  light_indicies carries one padding entry
 * (= the last light) so the xi == 1.0 read of index light_count is defined
 * (SURVEY H4); with no lights the three draws are made and nothing is traced. */
static V3 sample_direct_light(const OrScene *sc, V3 pos, V3 normal, uint32_t *rng, unsigned long long *cnt)
{
    cnt[CNT_NEE] += 1;
    float xi = rng_next(rng);
    if (sc->nlights == 0) {
        rng_next(rng);
        rng_next(rng);
        return v3(0.0f, 0.0f, 0.0f);
    }
    if (xi == 1.0f) cnt[CNT_XI_ONE] += 1;
    int li = sc->lights[(int)(xi * (float)sc->nlights)];
    const Triangle *light = &sc->tris[li];
    V3 rp = random_point_in_triangle(light, rng);
    Ray shadow = {pos, normalize(sub(rp, pos))};
    Sample sm;
    if (trace_ray(sc, shadow, &sm, cnt)) {
        if (sm.triangle_index == li) {
            float area = (float)(0.5 * (double)magnitude(cross(sub(light->p2, light->p1), sub(light->p3, light->p1))));
            float d2 = magnitude_squared(sub(rp, pos));
            float c1 = fmaxf(-dot(shadow.direction, sm.normal), 0.0f);
            float c2 = fmaxf(dot(shadow.direction, normal), 0.0f);
            return mulvs(sm.emittance, area * (float)sc->nlights * c1 * c2 / fmaxf(d2 * PIF, 0.001f));
        }
    }
    return v3(0.0f, 0.0f, 0.0f);
}

/* sample_direct_light for one shading point (tests' independent NEE restatement) */
void or_direct_light(const OrScene *s, const float pos[3], const float normal[3], uint32_t *rng, float out[3])
{
    unsigned long long cnt[OR_CNT_COUNT] = {0};
    V3 r = sample_direct_light(s, v3(pos[0], pos[1], pos[2]), v3(normal[0], normal[1], normal[2]), rng, cnt);
    out[0] = r.x;
    out[1] = r.y;
    out[2] = r.z;
}

/* trace_path (:268-325); returns the sample's radiance */
static V3 trace_path(const OrScene *sc, Ray primary, uint32_t *rng, int max_depth, unsigned long long *cnt)
{
    V3 L = {0.0f, 0.0f, 0.0f};
    V3 T = {1.0f, 1.0f, 1.0f};
    bool inside = false;
    Event ev = {primary, {0.0f, 0.0f, 0.0f}, PRIMARY};
    int limit = (max_depth > 0) ? max_depth : WATCHDOG_BOUNCES;
    int depth = 0;
    cnt[CNT_SAMPLE] += 1;
    while (1) {
        if (depth == limit) {
            if (max_depth <= 0) cnt[CNT_WATCHDOG] += 1;
            cnt[CNT_CUT] += 1;
            break;
        }
        ++depth;
        Sample sm;
        if (trace_ray(sc, ev.ray, &sm, cnt)) {
            if (ev.type != DIFFUSE) L = add(L, mulvv(sm.emittance, T));
            ev = scatter(ev.ray.direction, &inside, rng, &sm);
            T = mulvv(T, ev.weight);
            if (ev.type == DIFFUSE) {
                V3 direct = sample_direct_light(sc, ev.ray.position, sm.normal, rng, cnt);
                L = add(L, mulvv(direct, T));
            }
        } else {
            break;
        }
        float p = fmaxf(T.x, fmaxf(T.y, T.z));
        float r = rng_next(rng);
        if (r > p) break;
        T = mulvs(T, 1.0f / p);
    }
    if ((unsigned long long)depth > cnt[CNT_MAXDEPTH]) cnt[CNT_MAXDEPTH] = (unsigned long long)depth;
    if (depth >= DEEP_PATH) {
        int k = 0;
        while (k < DEEP_HIST_BINS - 1 && depth >= (DEEP_PATH << (k + 1))) ++k;
        cnt[CNT_DEEP_HIST + k] += 1;
    }
    return L;
}

/* one pixel-pass of path_tracing (:338-395) */
static void pixel_pass(const OrScene *sc, const float cam[7], const M3 *R, float tan_half_fov, int x, int y,
                       int pi, float *fb, float *sq, int *count, uint32_t *rngs, const OrOptions *o,
                       float z_const, unsigned long long *cnt)
{
    bool run = false;
    int n = count[pi];
    if (!o->adaptive || n < o->min_samples) {
        run = true;
    } else {
        float tl = luminance(v3(fb[3 * pi], fb[3 * pi + 1], fb[3 * pi + 2]));
        float tsq = sq[pi];
        float mean = tl / (float)n;
        float var = (tsq - square(tl) / (float)n) / (float)(n - 1);
        float i = z_const * sqrtf(var / (float)n);
        if (i > mean * o->tolerance) run = true;
    }
    if (!run) {
        cnt[CNT_SKIP] += 1;
        return;
    }
    uint32_t rng = rngs[pi];
    int half_w = o->width / 2, half_h = o->height / 2; /* SCREEN_W / 2 (int) */
    float rx = rng_next(&rng);
    float ry = rng_next(&rng);
    V3 dir = normalize(v3(tan_half_fov * ((float)x + rx - (float)half_w) / (float)half_w,
                          tan_half_fov * ((float)y + ry - (float)half_h) / (float)half_w, 1.0f));
    dir = mmul(*R, dir);
    /* random_point_in_pinhole (:327-336) */
    float theta = rng_next(&rng) * TAUF;
    float r = sqrtf(rng_next(&rng)) * cam[6];
    float ox = r * rt_cosf(theta);
    float oy = r * rt_sinf(theta);
    V3 pos = add(add(v3(cam[0], cam[1], cam[2]), mmul(*R, v3(ox, 0.0f, 0.0f))), mmul(*R, v3(0.0f, oy, 0.0f)));
    Ray primary = {pos, dir};
    V3 L = trace_path(sc, primary, &rng, o->max_depth, cnt);
    /* accumulation (:322-324) */
    fb[3 * pi] += L.x;
    fb[3 * pi + 1] += L.y;
    fb[3 * pi + 2] += L.z;
    sq[pi] += square(luminance(L));
    count[pi] += 1;
    rngs[pi] = rng;
}

void or_default_options(OrOptions *o)
{
    o->width = 1920;
    o->height = 1080;
    o->passes = 1;
    o->adaptive = 1;
    o->min_samples = 100;
    o->tolerance = 0.05f;
    o->max_depth = 0;
    o->threads = 0;
}

int or_render(const OrScene *sc, const float cam[7], float *fb, float *sq, int *count, uint32_t *rngs,
              const int *pixels, int pixel_count, int sample_count_arg, const OrOptions *o,
              unsigned long long *counters)
{
    int total = o->width * o->height;
    int n = pixels ? pixel_count : total;
    M3 R = rotation_matrix(cam[3], cam[4]);                     /* Camera::rotation (rt/camera.cuh:22-25) */
    float tan_half = rt_tanf(cam[5] / 2);                      /* :381 */
    float z_const = rt_adaptive_z(o->tolerance);              /* sqrtf(2)*erfinvf(1-tol) (:370) */
    if (sample_count_arg == 0) {                               /* reset_frame (rt/render.cuh:18-34) */
        for (int k = 0; k < n; ++k) {
            int pi = pixels ? pixels[k] : k;
            fb[3 * pi] = fb[3 * pi + 1] = fb[3 * pi + 2] = 0.0f;
            sq[pi] = 0.0f;
            count[pi] = 0;
        }
    }
#ifdef _OPENMP
    if (o->threads > 0) omp_set_num_threads(o->threads);
#endif
#pragma omp parallel
    {
        unsigned long long cnt[OR_CNT_COUNT] = {0};
#pragma omp for schedule(dynamic, 16)
        for (int k = 0; k < n; ++k) {
            int pi = pixels ? pixels[k] : k;
            if (pi < 0 || pi >= total) continue;
            int x = pi % o->width, y = pi / o->width;
            for (int p = 0; p < o->passes; ++p)
                pixel_pass(sc, cam, &R, tan_half, x, y, pi, fb, sq, count, rngs, o, z_const, cnt);
        }
        if (counters) {
#pragma omp critical
            for (int c = 0; c < OR_CNT_COUNT; ++c) {
                if (c == CNT_MAXDEPTH) counters[c] = counters[c] > cnt[c] ? counters[c] : cnt[c];
                else counters[c] += cnt[c];
            }
        }
    }
    return 0;
}

/* draw_frame colour (rt/render.cuh:44-53 / rt/save_render.cuh:47-52) */
void or_tonemap(const float *fb, const int *count, int n, uint8_t *rgba)
{
    for (int i = 0; i < n; ++i) {
        V3 c = mulvs(v3(fb[3 * i], fb[3 * i + 1], fb[3 * i + 2]), 1.0f / (float)count[i]);
        c = correct_color(c);
        rgba[4 * i + 0] = (uint8_t)(c.x * MAX_COLOR_CHANNEL);
        rgba[4 * i + 1] = (uint8_t)(c.y * MAX_COLOR_CHANNEL);
        rgba[4 * i + 2] = (uint8_t)(c.z * MAX_COLOR_CHANNEL);
        rgba[4 * i + 3] = MAX_COLOR_CHANNEL;
    }
}

/* ---------------------------------- KD builder (rt/create_kd_tree.cuh) */
typedef struct { int *v; int n; } IVec;

static void node_push(OrScene *sc, Node nd)
{
    if (sc->nnodes == sc->nodecap) {
        sc->nodecap = sc->nodecap ? sc->nodecap * 2 : 1024;
        sc->nodes = (Node *)realloc(sc->nodes, (size_t)sc->nodecap * sizeof(Node));
    }
    sc->nodes[sc->nnodes++] = nd;
}
static void index_push(OrScene *sc, int v)
{
    if (sc->nindices == sc->indexcap) {
        sc->indexcap = sc->indexcap ? sc->indexcap * 2 : 4096;
        sc->indices = (int *)realloc(sc->indices, (size_t)sc->indexcap * sizeof(int));
    }
    sc->indices[sc->nindices++] = v;
}
static inline float tri_min(const Triangle *t, int a)
{
    return fminf(axis_of(t->p1, a), fminf(axis_of(t->p2, a), axis_of(t->p3, a)));
}
static inline float tri_max(const Triangle *t, int a)
{
    return fmaxf(axis_of(t->p1, a), fmaxf(axis_of(t->p2, a), axis_of(t->p3, a)));
}
static int cmp_float(const void *a, const void *b)
{
    float x = *(const float *)a, y = *(const float *)b;
    return (x < y) ? -1 : (x > y ? 1 : 0);
}
/* get_plane_offset (:125-160): median of AABB centres, sorted[size/2] */
static float plane_offset(const OrScene *sc, const IVec *ids, int axis)
{
    float *vals = (float *)malloc((size_t)(ids->n > 0 ? ids->n : 1) * sizeof(float));
    for (int i = 0; i < ids->n; ++i) {
        const Triangle *t = &sc->tris[ids->v[i]];
        vals[i] = (tri_min(t, axis) + tri_max(t, axis)) * 0.5f;
    }
    qsort(vals, (size_t)ids->n, sizeof(float), cmp_float);
    float r = ids->n > 0 ? vals[ids->n / 2] : 0.0f;
    free(vals);
    return r;
}
/* add_child_nodes (:162-265).  Nodes are addressed by index because the
 * array may be reallocated during recursion (the reference uses a std::list). */
static void add_child_nodes(OrScene *sc, int parent, IVec *ids, int depth)
{
    int axis = depth % 3;
    float split = plane_offset(sc, ids, axis);
    sc->nodes[parent].plane_axis = (uint8_t)axis;
    sc->nodes[parent].plane_offset = split;
    IVec c1 = {(int *)malloc((size_t)(ids->n + 1) * sizeof(int)), 0};
    IVec c2 = {(int *)malloc((size_t)(ids->n + 1) * sizeof(int)), 0};
    for (int i = 0; i < ids->n; ++i) {
        const Triangle *t = &sc->tris[ids->v[i]];
        if (tri_min(t, axis) <= split) c1.v[c1.n++] = ids->v[i];   /* triangle_behind_plane :59-90 */
        if (tri_max(t, axis) >= split) c2.v[c2.n++] = ids->v[i];   /* triangle_afore_plane :92-123 */
    }
    const int min_count = 7;
    Node inner = {0, 0, 0, 0.0f, false};
    for (int side = 0; side < 2; ++side) {
        IVec *c = side == 0 ? &c1 : &c2;
        int child = sc->nnodes;
        if (side == 0) sc->nodes[parent].a = child; else sc->nodes[parent].b = child;
        if (c->n > min_count && depth < KD_TREE_DEPTH) {
            node_push(sc, inner);
            add_child_nodes(sc, child, c, depth + 1);
        } else {
            Node leaf = {sc->nindices, c->n, 0, 0.0f, true};
            node_push(sc, leaf);
            for (int i = 0; i < c->n; ++i) index_push(sc, c->v[i]);
        }
    }
    free(c1.v);
    free(c2.v);
}
/* get_bounding_box (:18-57) */
static BBox scene_bounds(const OrScene *sc)
{
    const float eps = 0.01f;
    BBox b = {{FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX}};
    for (int i = 0; i < sc->ntris; ++i) {
        const Triangle *t = &sc->tris[i];
        b.min.x = fminf(tri_min(t, 0), b.min.x);
        b.min.y = fminf(tri_min(t, 1), b.min.y);
        b.min.z = fminf(tri_min(t, 2), b.min.z);
        b.max.x = fmaxf(tri_max(t, 0), b.max.x);
        b.max.y = fmaxf(tri_max(t, 1), b.max.y);
        b.max.z = fmaxf(tri_max(t, 2), b.max.z);
    }
    b.min = sub(b.min, v3(eps, eps, eps));
    b.max = add(b.max, v3(eps, eps, eps));
    return b;
}
/* create_kd_tree (:267-328) + light list of create_scene (rt/create_scene.cuh:40-64) */
static void finish_scene(OrScene *sc)
{
    Node root = {0, 0, 0, 0.0f, false};
    node_push(sc, root);
    IVec all = {(int *)malloc((size_t)(sc->ntris + 1) * sizeof(int)), sc->ntris};
    for (int i = 0; i < sc->ntris; ++i) all.v[i] = i;
    add_child_nodes(sc, 0, &all, 0);
    free(all.v);
    sc->bounds = scene_bounds(sc);
    sc->lights = (int *)malloc((size_t)(sc->ntris + 1) * sizeof(int));
    sc->nlights = 0;
    for (int i = 0; i < sc->ntris; ++i) {
        V3 e = sc->tris[i].material.emittance;
        if (e.x > 0 || e.y > 0 || e.z > 0) sc->lights[sc->nlights++] = i;
    }
    sc->lights[sc->nlights] = sc->nlights > 0 ? sc->lights[sc->nlights - 1] : 0; /* H4 padding */
    sc->degenerate = (unsigned char *)calloc((size_t)sc->ntris + 1, 1);
    for (int i = 0; i < sc->ntris; ++i) {
        const Triangle *t = &sc->tris[i];
        V3 n = normalize(cross(sub(t->p2, t->p1), sub(t->p3, t->p1)));
        sc->degenerate[i] = n.x != n.x || n.y != n.y || n.z != n.z;
    }
}

/* ------------------------------------------ loader (rt/mesh_loading.cuh) */
typedef struct { char **s; int n, cap; } SVec;
static void sv_push(SVec *v, const char *b, size_t len)
{
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 8;
        v->s = (char **)realloc(v->s, (size_t)v->cap * sizeof(char *));
    }
    char *c = (char *)malloc(len + 1);
    memcpy(c, b, len);
    c[len] = 0;
    v->s[v->n++] = c;
}
static void sv_free(SVec *v)
{
    for (int i = 0; i < v->n; ++i) free(v->s[i]);
    free(v->s);
    v->s = NULL;
    v->n = v->cap = 0;
}
/* split_string (:73-103) */
static SVec split(const char *s, char delim, bool include_empty)
{
    SVec out = {0};
    size_t start = 0, len = strlen(s), cur = 0;
    for (size_t i = 0; i < len; ++i) {
        if (s[i] == delim) {
            if (cur > 0 || include_empty) sv_push(&out, s + start, cur);
            start = i + 1;
            cur = 0;
        } else {
            if (cur == 0) start = i;
            ++cur;
        }
    }
    if (cur > 0) sv_push(&out, s + start, cur);
    return out;
}
static float stof_(const char *s, bool *ok)
{
    char *end;
    float v = strtof(s, &end);
    if (end == s) *ok = false;
    return v;
}
static int stoi_(const char *s, bool *ok)
{
    char *end;
    long v = strtol(s, &end, 10);
    if (end == s) *ok = false;
    return (int)v;
}
static char *read_line(FILE *f, char **buf, size_t *cap)
{
    ssize_t n = getline(buf, cap, f);
    if (n < 0) return NULL;
    if (n > 0 && (*buf)[n - 1] == '\n') (*buf)[n - 1] = 0;
    return *buf;
}

/* Textures (make_texture, rt/scene.cuh:25-63).  The oracle does not decode
 * images: the test registers the RGBA8 texels of each `texture` path (the
 * string as written in the .mat file) beforehand; a path with no registered
 * texels stays NO_TEXTURE, like a file stbi_load cannot open.  Each texture is
 * stored with width + 1 zero texels after the image (mod() can return 1.0,
 * SURVEY H10), as the product pads its device copy. */
typedef struct { char *path; UC4 *texels; int width, height; } OrTex;
static OrTex *g_tex = NULL;
static int g_ntex = 0;

int or_register_texture(const char *path, const uint8_t *rgba, int width, int height)
{
    if (!path || !rgba || width <= 0 || height <= 0) return -1;
    OrTex *t = realloc(g_tex, sizeof(OrTex) * (size_t)(g_ntex + 1));
    if (!t) return -1;
    g_tex = t;
    const size_t n = (size_t)width * height;
    UC4 *tx = calloc(n + (size_t)width + 1, sizeof(UC4));
    if (!tx) return -1;
    memcpy(tx, rgba, n * 4);
    g_tex[g_ntex].path = strdup(path);
    g_tex[g_ntex].texels = tx;
    g_tex[g_ntex].width = width;
    g_tex[g_ntex].height = height;
    ++g_ntex;
    return 0;
}

static Texture find_texture(const char *path)
{
    Texture t = {NULL, 0, 0};
    for (int i = g_ntex - 1; i >= 0; --i)
        if (!strcmp(g_tex[i].path, path)) {
            t.buffer = g_tex[i].texels;
            t.width = g_tex[i].width;
            t.height = g_tex[i].height;
            break;
        }
    return t;
}

/* load_material (:152-219) */
static bool load_material(const char *path, const char *name, Material *m, bool *ok)
{
    memset(m, 0, sizeof *m);
    FILE *f = fopen(path, "r");
    bool found = false;
    if (!f) return false;
    char *buf = NULL;
    size_t cap = 0;
    char header[1024];
    snprintf(header, sizeof header, "material %s", name);
    char *line;
    while ((line = read_line(f, &buf, &cap))) {
        if (strcmp(line, header) == 0) {
            found = true;
        } else if (found) {
            if (line[0] == 0) break;
            SVec s = split(line, ' ', false);
            if (s.n == 0) { sv_free(&s); *ok = false; break; }
            if (!strcmp(s.s[0], "albedo") && s.n >= 4) {
                m->albedo = v3(stof_(s.s[1], ok), stof_(s.s[2], ok), stof_(s.s[3], ok));
            } else if (!strcmp(s.s[0], "emittance") && s.n >= 4) {
                m->emittance = v3(stof_(s.s[1], ok), stof_(s.s[2], ok), stof_(s.s[3], ok));
            } else if (!strcmp(s.s[0], "roughness") && s.n >= 2) {
                m->roughness = stof_(s.s[1], ok);
            } else if (!strcmp(s.s[0], "n") && s.n >= 2) {
                m->refractive_index = stof_(s.s[1], ok);
            } else if (!strcmp(s.s[0], "k") && s.n >= 2) {
                m->extinction = stof_(s.s[1], ok);
            } else if (!strcmp(s.s[0], "transparent")) {
                m->transparent = true;
            } else if (!strcmp(s.s[0], "texture") && s.n >= 2) {
                m->texture = find_texture(s.s[1]);
            }
            sv_free(&s);
        }
    }
    free(buf);
    fclose(f);
    return found;
}

int or_load_material(const char *path, const char *name, float out[10])
{
    Material m;
    bool ok = true;
    int found = load_material(path, name, &m, &ok) ? 1 : 0;
    out[0] = m.albedo.x; out[1] = m.albedo.y; out[2] = m.albedo.z;
    out[3] = m.emittance.x; out[4] = m.emittance.y; out[5] = m.emittance.z;
    out[6] = m.roughness; out[7] = m.refractive_index; out[8] = m.extinction;
    out[9] = m.transparent ? 1.0f : 0.0f;
    return ok ? found : -1;
}

typedef struct { int p, t, n; } OVert;                 /* OBJ::Vertex (:27-32) */
typedef struct { OVert v1, v2, v3; int mat; } OTri;    /* OBJ::Triangle (:34-39), material by id */

/* create_vertex (:105-150) */
static OVert create_vertex(const char *tok, int npos, int ntex, int nnor, bool *ok)
{
    OVert v = {-1, -1, -1};
    SVec d = split(tok, '/', true);
    if (d.n > 0) {
        int i = stoi_(d.s[0], ok);
        v.p = i > 0 ? i - 1 : npos + i;
    }
    if (d.n > 1 && d.s[1][0] != 0) {
        int i = stoi_(d.s[1], ok);
        v.t = i > 0 ? i - 1 : ntex + i;
    }
    if (d.n > 2) {
        int i = stoi_(d.s[2], ok);
        v.n = i > 0 ? i - 1 : nnor + i;
    }
    sv_free(&d);
    return v;
}

#define GROW(ptr, n, cap, T)                                                   \
    do {                                                                       \
        if ((n) == (cap)) {                                                    \
            (cap) = (cap) ? (cap) * 2 : 1024;                                  \
            (ptr) = (T *)realloc((ptr), (size_t)(cap) * sizeof(T));            \
        }                                                                      \
    } while (0)

/* load_mesh (:221-440) */
static int load_mesh(OrScene *sc, const char *obj, const char *mat, V3 offset, M3 matrix, bool smooth)
{
    FILE *f = fopen(obj, "r");
    if (!f) { set_err("cannot open %s", obj); return -1; }
    V3 *pos = NULL, *nor = NULL; V2 *tex = NULL; OTri *mesh = NULL;
    int npos = 0, cpos = 0, nnor = 0, cnor = 0, ntex = 0, ctex = 0, nmesh = 0, cmesh = 0;
    bool *false_normal = NULL; int cfalse = 0;
    /* materials: std::map<std::string, Material> keyed by name */
    char **mnames = NULL; Material *mats = NULL; int nmats = 0, cmats = 0;
    int cur_mat = -1; /* "" until usemtl */
    bool ok = true;
    char *buf = NULL; size_t cap = 0; char *line;
    while ((line = read_line(f, &buf, &cap))) {
        SVec s = split(line, ' ', false);
        if (s.n > 0) {
            if (!strcmp(s.s[0], "v") && s.n >= 4) {
                GROW(pos, npos, cpos, V3);
                pos[npos++] = v3(stof_(s.s[1], &ok), stof_(s.s[2], &ok), stof_(s.s[3], &ok));
            } else if (!strcmp(s.s[0], "vn") && s.n >= 4) {
                V3 nn = v3(stof_(s.s[1], &ok), stof_(s.s[2], &ok), stof_(s.s[3], &ok));
                if (nnor >= cfalse) {
                    int old = cfalse;
                    cfalse = cfalse ? cfalse * 2 : 1024;
                    false_normal = (bool *)realloc(false_normal, (size_t)cfalse);
                    memset(false_normal + old, 0, (size_t)(cfalse - old));
                }
                false_normal[nnor] = (nn.x == 0 && nn.y == 0 && nn.z == 0);
                GROW(nor, nnor, cnor, V3);
                nor[nnor++] = nn;
            } else if (!strcmp(s.s[0], "vt") && s.n >= 3) {
                V2 t = {1.0f, 1.0f}; /* ZERO_VEC2D */
                t.x = stof_(s.s[1], &ok);
                t.y = 1.0f - stof_(s.s[2], &ok);
                GROW(tex, ntex, ctex, V2);
                tex[ntex++] = t;
            } else if (!strcmp(s.s[0], "usemtl") && s.n >= 2) {
                int found = -1;
                for (int i = 0; i < nmats; ++i)
                    if (!strcmp(mnames[i], s.s[1])) found = i;
                if (found < 0) {
                    GROW(mnames, nmats, cmats, char *);
                    mats = (Material *)realloc(mats, (size_t)cmats * sizeof(Material));
                    mnames[nmats] = strdup(s.s[1]);
                    load_material(mat, s.s[1], &mats[nmats], &ok);
                    found = nmats++;
                }
                cur_mat = found;
            } else if (!strcmp(s.s[0], "f") && s.n >= 2) {
                OVert a = create_vertex(s.s[1], npos, ntex, nnor, &ok);
                bool is_false = (a.n >= 0 && a.n < nnor) ? false_normal[a.n] : false;
                if (!is_false) {
                    for (int i = 3; i < s.n; ++i) {
                        OVert b = create_vertex(s.s[i - 1], npos, ntex, nnor, &ok);
                        OVert c = create_vertex(s.s[i], npos, ntex, nnor, &ok);
                        GROW(mesh, nmesh, cmesh, OTri);
                        OTri t = {a, b, c, cur_mat};
                        mesh[nmesh++] = t;
                    }
                }
            }
        }
        sv_free(&s);
    }
    free(buf);
    fclose(f);
    if (!ok) { set_err("parse error in %s", obj); return -1; }
    for (int i = 0; i < nmesh; ++i) {
        OVert *vs[3] = {&mesh[i].v1, &mesh[i].v2, &mesh[i].v3};
        for (int k = 0; k < 3; ++k) {
            if (vs[k]->p < 0 || vs[k]->p >= npos || vs[k]->t >= ntex || vs[k]->n >= nnor || vs[k]->t < -1 ||
                vs[k]->n < -1) {
                set_err("index out of range in %s", obj);
                return -1;
            }
        }
    }
    /* computed_normals (:328-342) */
    V3 *cn = (V3 *)calloc((size_t)(npos > 0 ? npos : 1), sizeof(V3));
    for (int i = 0; i < nmesh; ++i) {
        V3 p1 = pos[mesh[i].v1.p], p2 = pos[mesh[i].v2.p], p3 = pos[mesh[i].v3.p];
        V3 nn = normalize(cross(sub(p2, p1), sub(p3, p1)));
        cn[mesh[i].v1.p] = add(cn[mesh[i].v1.p], nn);
        cn[mesh[i].v2.p] = add(cn[mesh[i].v2.p], nn);
        cn[mesh[i].v3.p] = add(cn[mesh[i].v3.p], nn);
    }
    int prior = sc->ntris;
    sc->tris = (Triangle *)realloc(sc->tris, (size_t)(prior + nmesh + 1) * sizeof(Triangle));
    sc->ntris = prior + nmesh;
    Material empty;
    memset(&empty, 0, sizeof empty);
    for (int i = 0; i < nmesh; ++i) { /* :349-415 */
        OTri *o = &mesh[i];
        Triangle t;
        memset(&t, 0, sizeof t);
        t.p1 = pos[o->v1.p]; t.p2 = pos[o->v2.p]; t.p3 = pos[o->v3.p];
        V3 nn = normalize(cross(sub(t.p2, t.p1), sub(t.p3, t.p1)));
        t.n1 = nn; t.n2 = nn; t.n3 = nn;
        if (o->v1.n != -1) t.n1 = nor[o->v1.n]; else if (smooth) t.n1 = cn[o->v1.p];
        if (o->v2.n != -1) t.n2 = nor[o->v2.n]; else if (smooth) t.n2 = cn[o->v2.p];
        if (o->v3.n != -1) t.n3 = nor[o->v3.n]; else if (smooth) t.n3 = cn[o->v3.p];
        V2 z2 = {1.0f, 1.0f};
        t.uv1 = z2; t.uv2 = z2; t.uv3 = z2;
        if (o->v1.t != -1) t.uv1 = tex[o->v1.t];
        if (o->v2.t != -1) t.uv2 = tex[o->v2.t];
        if (o->v3.t != -1) t.uv3 = tex[o->v3.t];
        t.material = o->mat >= 0 ? mats[o->mat] : empty; /* materials[""] value-initialised */
        sc->tris[prior + i] = t;
    }
    /* transform (:418-439): bbox (no epsilon), centre, M*p + offset, normalize(M*n) */
    BBox b = {{FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX}};
    for (int i = prior; i < sc->ntris; ++i) {
        const Triangle *t = &sc->tris[i];
        b.min.x = fminf(tri_min(t, 0), b.min.x);
        b.min.y = fminf(tri_min(t, 1), b.min.y);
        b.min.z = fminf(tri_min(t, 2), b.min.z);
        b.max.x = fmaxf(tri_max(t, 0), b.max.x);
        b.max.y = fmaxf(tri_max(t, 1), b.max.y);
        b.max.z = fmaxf(tri_max(t, 2), b.max.z);
    }
    V3 center = v3((b.min.x + b.max.x) * 0.5f, (b.min.y + b.max.y) * 0.5f, (b.min.z + b.max.z) * 0.5f);
    for (int i = prior; i < sc->ntris; ++i) {
        Triangle *t = &sc->tris[i];
        t->p1 = sub(t->p1, center);
        t->p2 = sub(t->p2, center);
        t->p3 = sub(t->p3, center);
        t->p1 = add(mmul(matrix, t->p1), offset);
        t->p2 = add(mmul(matrix, t->p2), offset);
        t->p3 = add(mmul(matrix, t->p3), offset);
        t->n1 = normalize(mmul(matrix, t->n1));
        t->n2 = normalize(mmul(matrix, t->n2));
        t->n3 = normalize(mmul(matrix, t->n3));
    }
    free(cn); free(pos); free(nor); free(tex); free(mesh); free(false_normal);
    for (int i = 0; i < nmats; ++i) free(mnames[i]);
    free(mnames); free(mats);
    return 0;
}

static void dir_of(const char *path, char *out, size_t n)
{
    snprintf(out, n, "%s", path);
    char *slash = strrchr(out, '/');
    if (slash) slash[1] = 0; else out[0] = 0;
}
static void resolve(const char *dir, const char *p, char *out, size_t n)
{
    if (p[0] == '/') snprintf(out, n, "%s", p); else snprintf(out, n, "%s%s", dir, p);
}

/* scene file = create_models (rt/create_models.cuh:17-43) as data + the
 * camera of rt/main.cu:101-104 */
OrScene *or_scene_load(const char *path, float cam[7])
{
    FILE *f = fopen(path, "r");
    if (!f) { set_err("cannot open %s", path); return NULL; }
    char dir[1024];
    dir_of(path, dir, sizeof dir);
    OrScene *sc = (OrScene *)calloc(1, sizeof(OrScene));
    char *buf = NULL; size_t cap = 0; char *line;
    bool ok = true;
    while ((line = read_line(f, &buf, &cap))) {
        SVec s = split(line, ' ', false);
        if (s.n > 0 && s.s[0][0] != '#') {
            if (!strcmp(s.s[0], "mesh") && s.n == 10) {
                char obj[2048], mat[2048];
                resolve(dir, s.s[1], obj, sizeof obj);
                resolve(dir, s.s[2], mat, sizeof mat);
                V3 off = v3(stof_(s.s[3], &ok), stof_(s.s[4], &ok), stof_(s.s[5], &ok));
                float yaw = stof_(s.s[6], &ok), pitch = stof_(s.s[7], &ok), scale = stof_(s.s[8], &ok);
                int smooth = stoi_(s.s[9], &ok);
                M3 m = mscale(rotation_matrix(yaw, pitch), scale);
                if (load_mesh(sc, obj, mat, off, m, smooth != 0) != 0) ok = false;
            } else if (!strcmp(s.s[0], "camera") && s.n == 8) {
                for (int k = 0; k < 7; ++k) cam[k] = stof_(s.s[k + 1], &ok);
            } else {
                set_err("bad scene line: %s", line);
                ok = false;
            }
        }
        sv_free(&s);
        if (!ok) break;
    }
    free(buf);
    fclose(f);
    if (!ok || sc->ntris == 0) {
        if (ok) set_err("empty scene %s", path);
        or_scene_free(sc);
        return NULL;
    }
    finish_scene(sc);
    return sc;
}

OrScene *or_scene_from_triangles(const void *tris, int count)
{
    if (count <= 0) { set_err("empty scene"); return NULL; }
    OrScene *sc = (OrScene *)calloc(1, sizeof(OrScene));
    sc->tris = (Triangle *)malloc((size_t)count * sizeof(Triangle));
    memcpy(sc->tris, tris, (size_t)count * sizeof(Triangle));
    for (int i = 0; i < count; ++i) memset(&sc->tris[i].material.texture, 0, sizeof(Texture));
    sc->ntris = count;
    finish_scene(sc);
    return sc;
}

void or_scene_free(OrScene *s)
{
    if (!s) return;
    free(s->tris); free(s->lights); free(s->nodes); free(s->indices); free(s->degenerate);
    free(s);
}

int or_scene_counts(const OrScene *s, int *t, int *n, int *i, int *l)
{
    *t = s->ntris; *n = s->nnodes; *i = s->nindices; *l = s->nlights;
    return 0;
}

void or_scene_copy(const OrScene *s, void *tris, void *nodes, int *indices, int *lights, float bounds[6])
{
    if (tris) memcpy(tris, s->tris, (size_t)s->ntris * sizeof(Triangle));
    if (nodes) {
        /* normalise padding bytes so comparisons are byte-exact */
        unsigned char *o = (unsigned char *)nodes;
        for (int i = 0; i < s->nnodes; ++i) {
            Node nd;
            memset(&nd, 0, sizeof nd);
            nd.a = s->nodes[i].a; nd.b = s->nodes[i].b; nd.plane_axis = s->nodes[i].plane_axis;
            nd.plane_offset = s->nodes[i].plane_offset; nd.is_leaf_node = s->nodes[i].is_leaf_node;
            memcpy(o + 20 * (size_t)i, &nd, 20);
        }
    }
    if (indices) memcpy(indices, s->indices, (size_t)s->nindices * sizeof(int));
    if (lights) memcpy(lights, s->lights, (size_t)s->nlights * sizeof(int));
    if (bounds) {
        bounds[0] = s->bounds.min.x; bounds[1] = s->bounds.min.y; bounds[2] = s->bounds.min.z;
        bounds[3] = s->bounds.max.x; bounds[4] = s->bounds.max.y; bounds[5] = s->bounds.max.z;
    }
}
