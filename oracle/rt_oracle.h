/*
 * rt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C11 + OpenMP) of INDA23PlusPlus/isaklm-raytracer's
 * render hot path, used as the parity checker by tests/, by
 * __graft_entry__.smoke() and as bench.py's cpu_baseline ("kind": "port").
 * Nothing in the product (isaklm-raytracer_amd/) links, loads or calls it.
 *
 * Parity status: the reference itself cannot be built in this image (its path
 * includes <cuda_runtime.h>, <device_launch_parameters.h>,
 * <cuda_gl_interop.h>, <surface_functions.h> and GLFW/GL; no CUDA toolkit is
 * installed and stand-in headers are not allowed), and the reference ships no
 * tests or fixtures for this path.  The restatement is therefore
 * "parity unpinned" for radiance; it is pinned where public known answers
 * exist (mt19937: C++ standard [rand.predef] 10000th output and the
 * reference-run seeds recorded in SURVEY §8c; .mat parsing against the
 * reference's own material files).  See DESIGN.md §Parity.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OrScene OrScene;

/* counters.  Only indices 0..9 (RT_CNT_NODE .. RT_CNT_MAXDEPTH) and 15
 * (RT_CNT_DEEP_PUSH) have the meaning of the product's RT_CNT_* in
 * include/isaklm_rt.h; the rest are the oracle's own and must not be
 * compared element-wise with the product's array: [16] depth-limit cuts,
 * [17..34] deep-path histogram (the product reports these through
 * rt_deviation_stats), [35..39] hazard triggers (oracle.py HAZARDS; the
 * product's 35..39 are timing / bounded-traversal counters). */
#define OR_CNT_COUNT 40

typedef struct OrOptions {
    int width, height;
    int passes;
    int adaptive;
    int min_samples;
    float tolerance;
    int max_depth; /* 0 = unbounded */
    int threads;   /* OpenMP threads, 0 = default */
} OrOptions;

void or_default_options(OrOptions *o);

/* mt19937 (default seed 5489) outputs [skip, skip+count) */
void or_mt19937(uint32_t *out, size_t count, uint64_t skip);
/* one step of get_random_unilateral (rt/path_tracing.cuh:34-43) */
float or_rng_next(uint32_t *state);

/* scene text file -> triangles (load_mesh restatement), KD tree, light list.
 * camera_out[7] = position xyz, yaw, pitch, FOV, aperture.  NULL on error. */
OrScene *or_scene_load(const char *scene_path, float camera_out[7]);
/* build from a caller-supplied reference-layout triangle array (152 B each) */
OrScene *or_scene_from_triangles(const void *triangles152, int count);
void or_scene_free(OrScene *s);
const char *or_last_error(void);
int or_scene_counts(const OrScene *s, int *triangles, int *nodes, int *indices, int *lights);
/* copies reference-layout bytes: 152 B triangles, 20 B nodes, int indices, int lights,
 * bounds[6] */
void or_scene_copy(const OrScene *s, void *triangles152, void *nodes20, int *indices, int *lights,
                   float bounds[6]);
/* load_material (rt/mesh_loading.cuh:152-219): out[10] = albedo3, emittance3,
 * roughness, n, k, transparent(0/1); returns 1 if found, 0 if not */
int or_load_material(const char *mat_path, const char *name, float out[10]);

/* registers the RGBA8 texels load_material uses for `texture <path>` (the
 * string as written in the .mat file); the oracle decodes no images */
int or_register_texture(const char *path, const uint8_t *rgba, int width, int height);

/* trace_ray (rt/trace_ray.cuh:244-318) for n rays (o.xyz, d.xyz);
 * out per ray: [hit, triangle_index, position.xyz, normal.xyz, tangent.xyz] as float[12] */
void or_trace_rays(const OrScene *s, const float *rays6, int n, float *out12);

/* get_scattered_light (rt/path_tracing.cuh:151-219) for one Sample:
 * in: ray_dir[3], sample[20] = albedo3 emittance3 roughness n k transparent
 *     position3 normal3 tangent3 bitangent3 (as floats), inside, rng state
 * out: ray(pos3,dir3) weight3 type inside rng → float[12] (type, inside, rng bits as floats) */
void or_scatter(const float ray_dir[3], const float sample[22], int inside, uint32_t rng, float out[12],
                uint32_t *rng_out, int *inside_out, int *type_out);

/* sample_direct_light (rt/path_tracing.cuh:235-265) at one shading point:
 * radiance out[3], *rng advanced by the draws the reference makes */
void or_direct_light(const OrScene *s, const float pos[3], const float normal[3], uint32_t *rng, float out[3]);

/* path_tracing (rt/path_tracing.cuh:338-395) over `passes` passes, for the
 * pixels in `pixels` (NULL = all W*H), on G_Buffer-layout host arrays.
 * sample_count_arg == 0 resets fb/sq/count of the listed pixels first
 * (reset_frame, rt/render.cuh:18-34).  counters: u64[OR_CNT_COUNT] (adds). */
int or_render(const OrScene *s, const float camera[7], float *frame_buffer, float *squared_luminance,
              int *sample_count, uint32_t *random_numbers, const int *pixels, int pixel_count,
              int sample_count_arg, const OrOptions *o, unsigned long long *counters);

/* draw_frame / save_render colour math (rt/render.cuh:44-53) -> RGBA8 (row 0 = bottom) */
void or_tonemap(const float *frame_buffer, const int *sample_count, int n, uint8_t *rgba);
/* correct_color (rt/math_library.cuh:445-460) on one colour */
void or_correct_color(const float in[3], float out[3]);

#ifdef __cplusplus
}
#endif
#endif
