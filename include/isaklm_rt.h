/*
 * isaklm_rt.h — C-ABI of the MI355X-native path-tracing hot path.
 *
 * Drop-in boundary for INDA23PlusPlus/isaklm-raytracer's render path
 * (SURVEY §8b).  Paths below are relative to /root/reference/isaklm-raytracer
 * and abbreviated "rt/".
 *
 *   reference                                   this ABI
 *   -------------------------------------------------------------------------
 *   cudaMalloc / cudaMemcpy on the host path     rt_device_alloc / rt_upload /
 *     (rt/create_scene.cuh:33-34,62-63,            rt_download / rt_free
 *      rt/create_kd_tree.cuh:319-324,
 *      rt/scene.cuh:58-59, rt/screen.cuh:24-45)
 *   G_Buffer::G_Buffer()  rt/screen.cuh:22-46     rt_gbuffer_create / rt_gbuffer_seeds
 *   load_mesh()           rt/mesh_loading.cuh:221 rt_host_scene_load_mesh
 *   create_models()       rt/create_models.cuh:17 rt_host_scene_load_file (scene text file)
 *   create_kd_tree()      rt/create_kd_tree.cuh:267  rt_build_kd_tree
 *   create_scene()        rt/create_scene.cuh:18  rt_create_scene
 *   (new) device re-layout                        rt_scene_prepare
 *   render()              rt/render.cuh:62        rt_render
 *   reset_frame<<<>>>     rt/render.cuh:18        (inside rt_render, sample_count==0)
 *   draw_frame<<<>>>      rt/render.cuh:37        rt_tonemap (into an HBM RGBA8 buffer)
 *   save_render()         rt/save_render.cuh:25   rt_save_render (PNG, same flip)
 *
 * Conventions: every function returns 0 on success and a negative RT_E_*
 * code otherwise (rt_last_error() describes the last failure of the calling
 * thread).  Pointers named *_device are HIP device pointers.  The caller owns
 * every allocation and frees it explicitly (the reference leaks; see
 * rt/screen.cuh:24-31); rt_shutdown releases the library's own per-device
 * workspaces (it is also registered to run at exit).  Calls are synchronous
 * unless an RtOptions.stream is given, in which case the default render (the
 * bounded traversal, one persistent finisher per call) and the megakernel
 * only enqueue; the queue variants (RT_TRAVERSAL_KD, counting calls) block the
 * calling thread until their queue iterations are done (their host threads
 * read each iteration's live path count).  Consecutive calls may use
 * different streams: a call waits for the previous calls' device work first
 * (they share the per-device workspace) — except a chained call
 * (RtOptions.overlap), see there.
 */
#ifndef ISAKLM_RT_H
#define ISAKLM_RT_H

#include <stddef.h>
#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version: 3 = rt_scene_prepare(const Scene *, rt_scene_t *) without
 * counts (the counted form is rt_scene_prepare_counts), RtDeviations and
 * rt_deviation_stats, rt_abi_version; 4 = RT_CNT_COUNT 40 (the optional
 * counters buffer grew); 5 = RtOptions.traversal; 6 = RtOptions.overlap /
 * check_interval / debug, RtDeviations' bounded-traversal guard fields,
 * rt_join, rt_shutdown; 7 = RtDeviations' hand-off fields (owed passes,
 * safety-net exits, stranded pixels, dropped guard records, linger
 * expiries), RT_E_INCOMPLETE from the joins, rt_profile_history; 8 =
 * RtDeviations.long_closed, RtOptions.coalesce_passes (both structs grew).
 * An integrator checks
 * rt_abi_version() == RT_ABI_VERSION at start-up: a binary built against an
 * older header would otherwise link (C linkage) and mis-pass arguments. */
#define RT_ABI_VERSION 8

/* CUDA uchar4, used for texels (rt/scene.cuh:18) */
typedef struct RtUChar4 { uint8_t x, y, z, w; } RtUChar4;

/* ---------------- reference-layout types (byte-identical) ----------------
 * A C++ caller that brings the reference's own types — the reference is one
 * translation unit (rt/main.cu:8-14) whose headers define Vec2D, Vec3D
 * (rt/math_library.cuh:55,99), Texture, Material, Triangle, KD_Tree_Node,
 * Bounding_Box, KD_Tree, Scene (rt/scene.cuh:16-121), G_Buffer
 * (rt/screen.cuh:15) and Camera (rt/camera.cuh:15) — defines
 * ISAKLM_RT_CALLER_TYPES before including this header.  The definitions
 * below are then replaced by forward declarations, so the header can come
 * BEFORE those types (G_Buffer's constructor, rt/screen.cuh:22-46, already
 * calls the allocation functions) or after them; the functions take the
 * caller's types (C linkage: type names do not enter the symbols).  Once all
 * of them are defined, the caller writes ISAKLM_RT_CHECK_LAYOUT(); at
 * namespace scope: the static_asserts of the byte layout this library
 * assumes.  See INTEGRATION.md and tests/native/ref_main_shape.cpp. */
#ifdef ISAKLM_RT_CALLER_TYPES
#ifndef __cplusplus
#error "ISAKLM_RT_CALLER_TYPES: the reference's types are C++ (anonymous unions, constructors)"
#endif
struct Vec2D;
struct Vec3D;
struct Texture;
struct Material;
struct Triangle;
struct KD_Tree_Node;
struct Bounding_Box;
struct KD_Tree;
struct Scene;
struct G_Buffer;
struct Camera;
#else

/* rt/math_library.cuh:71-82 (union {x,u},{y,v}) */
typedef struct Vec2D { float x, y; } Vec2D;
/* rt/math_library.cuh:115-131 (union {x,r},{y,g},{z,b}) */
typedef struct Vec3D { float x, y, z; } Vec3D;

/* rt/scene.cuh:16-21 */
typedef struct Texture {
    RtUChar4 *buffer; /* device RGBA8 texels, NULL = no texture */
    int width;
    int height;
} Texture;

/* rt/scene.cuh:65-74 */
typedef struct Material {
    Vec3D albedo;
    Vec3D emittance;
    float roughness;
    float refractive_index;
    float extinction;
    bool transparent;
    Texture texture;
} Material;

/* rt/scene.cuh:76-82 */
typedef struct Triangle {
    Vec3D p1, p2, p3;
    Vec3D n1, n2, n3;
    Vec2D uv1, uv2, uv3;
    Material material;
} Triangle;

/* rt/scene.cuh:84-100 */
typedef struct KD_Tree_Node {
    union { int index_offset; int child_index1; };
    union { int triangle_count; int child_index2; };
    uint8_t plane_axis;
    float plane_offset;
    bool is_leaf_node;
} KD_Tree_Node;

/* rt/scene.cuh:102-105 */
typedef struct Bounding_Box { Vec3D min, max; } Bounding_Box;

/* rt/scene.cuh:107-112 */
typedef struct KD_Tree {
    Bounding_Box bounding_box;
    KD_Tree_Node *nodes;       /* device, pre-order (rt/create_kd_tree.cuh:286-298) */
    int *triangle_indicies;    /* device (rt/create_kd_tree.cuh:300-312) */
} KD_Tree;

/* rt/scene.cuh:114-121 */
typedef struct Scene {
    Triangle *triangles;       /* device AoS */
    int triangle_count;
    int *light_indicies;       /* device */
    int light_count;
    KD_Tree kd_tree;
} Scene;

/* rt/screen.cuh:15-21 (per-pixel SoA device arrays, row-major, row 0 = bottom) */
typedef struct G_Buffer {
    Vec3D *frame_buffer;
    float *squared_luminance;
    int *sample_count;
    uint32_t *random_numbers;
} G_Buffer;

/* rt/camera.cuh:15-26 */
typedef struct Camera {
    Vec3D position;
    float yaw, pitch;
    float FOV;
    float aperture_radius;
} Camera;

#endif /* ISAKLM_RT_CALLER_TYPES */

#ifdef __cplusplus
/* the reference's byte layout */
#define ISAKLM_RT_CHECK_LAYOUT()                                                                              \
static_assert(sizeof(Vec2D) == 8, "Vec2D"); \
static_assert(sizeof(Vec3D) == 12, "Vec3D"); \
static_assert(sizeof(Texture) == 16, "Texture"); \
static_assert(sizeof(Material) == 56 && offsetof(Material, roughness) == 24 && \
              offsetof(Material, transparent) == 36 && offsetof(Material, texture) == 40, "Material"); \
static_assert(sizeof(Triangle) == 152 && offsetof(Triangle, n1) == 36 && offsetof(Triangle, uv1) == 72 && \
              offsetof(Triangle, material) == 96, "Triangle"); \
static_assert(sizeof(KD_Tree_Node) == 20 && offsetof(KD_Tree_Node, plane_axis) == 8 && \
              offsetof(KD_Tree_Node, plane_offset) == 12 && offsetof(KD_Tree_Node, is_leaf_node) == 16, \
              "KD_Tree_Node"); \
static_assert(sizeof(Bounding_Box) == 24, "Bounding_Box"); \
static_assert(sizeof(KD_Tree) == 40, "KD_Tree"); \
static_assert(sizeof(Scene) == 72 && offsetof(Scene, light_indicies) == 16 && offsetof(Scene, kd_tree) == 32, \
              "Scene"); \
static_assert(sizeof(G_Buffer) == 32, "G_Buffer"); \
static_assert(sizeof(Camera) == 28 && offsetof(Camera, FOV) == 20, "Camera");
#ifndef ISAKLM_RT_CALLER_TYPES
ISAKLM_RT_CHECK_LAYOUT()
#endif
#endif

/* ---------------- status codes ---------------- */
#define RT_OK 0
#define RT_E_INVALID (-1)   /* bad argument / shape */
#define RT_E_HIP (-2)       /* HIP runtime failure */
#define RT_E_IO (-3)        /* file could not be read / written */
#define RT_E_PARSE (-4)     /* malformed OBJ / .mat / scene file */
#define RT_E_UNSUPPORTED (-5) /* e.g. KD tree deeper than the traversal stack */
#define RT_E_NOMEM (-6)
#define RT_E_INCOMPLETE (-7) /* a join found pixels whose deep-path samples never came back
                              * (RtDeviations.stranded_pixels): the frame misses passes */

const char *rt_last_error(void);
const char *rt_version(void);
int rt_abi_version(void); /* RT_ABI_VERSION of the built library */

/* ---------------- texture decoding ----------------
 * stbi_load(path, &w, &h, &n, 4) as make_texture (rt/scene.cuh:25-63) calls
 * it: RGBA8 rows in file order (no flip).  PNG (all colour types / depths,
 * Adam7, tRNS) and baseline / extended-sequential / progressive JPEG,
 * bit-identical to stb_image v2.28; other formats -> RT_E_UNSUPPORTED.
 * The pixels are a host array (rt_host_free).  rt_host_scene_load_mesh decodes
 * a material's `texture` with it, and rt_create_scene uploads each texture
 * with width + 1 zero texels after the image: mod(uv, 1) can return 1.0, so
 * sample_texture's index reaches width*height + width.  Callers
 * of rt_scene_prepare_host that supply their own device texels should pad
 * them the same way. */
int rt_decode_image(const char *path, uint8_t **rgba_out, int *width, int *height);
int rt_decode_image_memory(const void *data, size_t size, uint8_t **rgba_out, int *width, int *height);

/* ---------------- device memory (hipMalloc/hipMemcpy stand-ins) ---------------- */
int rt_device_alloc(void **ptr_device, size_t bytes);
int rt_free(void *ptr_device);
int rt_upload(void *dst_device, const void *src_host, size_t bytes);
int rt_download(void *dst_host, const void *src_device, size_t bytes);
int rt_memset(void *dst_device, int value, size_t bytes);
int rt_device_count(int *count);
/* selects the device for the calling thread and creates the wavefront
 * pipelines' streams there (call it before other GPU users of the process,
 * e.g. RCCL, take the hardware queues) */
int rt_set_device(int device);
/* hipDeviceSynchronize after rt_join(NULL): chained renders are complete */
int rt_synchronize(void);
/* `stream` (NULL: the calling thread) waits for every rt_render's device work
 * on the current device, including the deep-path tails that chained calls
 * (RtOptions.overlap) leave running past their stream point (an open chain is
 * drained first: one more finisher launch for the pixels still owed passes).
 * After the drain every pixel handed to the long-path kernel must be back; a
 * check kernel verifies it (and releases any that are not).  Host joins
 * (NULL, and rt_synchronize, rt_download, rt_tonemap / rt_save_render without
 * a stream, rt_gbuffer_save) return RT_E_INCOMPLETE if that check — theirs or
 * an earlier stream join's — found stranded pixels; RtDeviations counts them. */
int rt_join(void *stream);
/* releases the library's per-device workspaces (streams, events, device
 * buffers) after their device work is done; registered with atexit by
 * rt_set_device / the first render.  Renders after it create them again. */
void rt_shutdown(void);
void rt_host_free(void *ptr_host);  /* frees host arrays returned by this library */

/* ---------------- G_Buffer (rt/screen.cuh:22-46) ---------------- */
/* outputs [skip, skip+count) of std::mt19937 (default seed 5489) through
 * uniform_int_distribution<uint32_t>(0, UINT32_MAX), i.e. the raw engine words
 * (rt/screen.cuh:34-45).  Shard g of an spp-sliced render uses skip = g*W*H. */
int rt_gbuffer_seeds(uint32_t *host_out, size_t count, uint64_t skip);
/* allocates the four arrays for width*height pixels, zeroes fb/sq/count
 * (the reference leaves them uninitialised until reset_frame) and uploads the
 * seeds */
int rt_gbuffer_create(int width, int height, uint64_t seed_skip, G_Buffer *out);
int rt_gbuffer_destroy(G_Buffer *g);
/* checkpoint / resume: the G_Buffer is a frame's whole
 * progressive state (the reference keeps it in device memory only).  Save it
 * with the caller's sample count; loading it into a G_Buffer of the same size
 * and calling rt_render with that sample count continues the render bit for
 * bit.  Errors: RT_E_IO (file), RT_E_PARSE (not a checkpoint / truncated),
 * RT_E_INVALID (size mismatch). */
int rt_gbuffer_save(G_Buffer g_buffer, int width, int height, int sample_count, const char *path);
int rt_gbuffer_load(const char *path, G_Buffer g_buffer, int width, int height, int *sample_count_out);

/* ---------------- host scene path ---------------- */
typedef struct RtHostScene RtHostScene;
int rt_host_scene_create(RtHostScene **out);
void rt_host_scene_destroy(RtHostScene *scene);
/* load_mesh (rt/mesh_loading.cuh:221-440): appends the OBJ's triangles,
 * materials from the .mat file, re-centred on the mesh AABB and transformed by
 * `matrix` (column vectors i,j,k = matrix[0..2],[3..5],[6..8]) + `offset`. */
int rt_host_scene_load_mesh(RtHostScene *scene, const char *obj_path, const char *mat_path,
                            const float offset[3], const float matrix[9], int smooth_normals);
/* scene text file: "mesh <obj> <mat> ox oy oz yaw pitch scale smooth" lines
 * (create_models' rotation_matrix(yaw,pitch)*scale transforms,
 * rt/create_models.cuh:21-39) and one "camera px py pz yaw pitch fov aperture"
 * line (rt/main.cu:101-104).  Relative paths resolve against the file's dir. */
int rt_host_scene_load_file(RtHostScene *scene, const char *scene_path, Camera *camera_out);
int rt_host_scene_triangles(const RtHostScene *scene, const Triangle **triangles, int *count);
/* Synthetic scenes for BASELINE.json's configs (the reference's OBJ models
 * are unpublished): writes OBJ + .mat + scene.txt into out_dir and
 * returns the scene.txt path.  Names: cornell (cfg 1), cornell_blob (cfg 2),
 * room2m (cfg 3/4), room2m_glass (cfg 5), room_small (tests). */
int rt_generate_scene(const char *name, const char *out_dir, char *scene_path_out, size_t cap);

/* create_kd_tree (rt/create_kd_tree.cuh:267-328) on the host: identical tree,
 * node numbering and index order.  Outputs are host arrays (rt_host_free). */
int rt_build_kd_tree(const Triangle *host_triangles, int triangle_count, KD_Tree_Node **nodes_out,
                     int *node_count, int **indices_out, int *index_count, Bounding_Box *bounds_out);

/* create_scene (rt/create_scene.cuh:18-73): uploads triangles, the light list
 * and the KD tree into a reference-layout device Scene. */
int rt_create_scene(const RtHostScene *scene, Scene *out, int *node_count, int *index_count);
int rt_destroy_scene(Scene *scene);

/* ---------------- prepared (MI355X-layout) scene ---------------- */
typedef struct RtPreparedScene *rt_scene_t;
/* Re-lays a reference-layout device Scene into the traversal layout (SoA
 * nodes, precomputed triangle planes).  Bit-preserving: every precomputed
 * value is the reference's own expression evaluated once.  Takes the Scene
 * exactly as the reference's `Scene create_scene()` (rt/create_scene.cuh:
 * 18-73) returns it: the KD node and index counts, which Scene does not carry
 * (rt/scene.cuh:107-121), are recovered by walking the device tree
 * pre-order from node 0 within its device allocation.  The arrays must be
 * device allocations of this process (rt_device_alloc / hipMalloc). */
int rt_scene_prepare(const Scene *device_scene, rt_scene_t *out);
/* the same with the counts given (e.g. memory from a sub-allocator that
 * hipMemGetAddressRange cannot bound) */
int rt_scene_prepare_counts(const Scene *device_scene, int node_count, int index_count, rt_scene_t *out);
/* same from host arrays (skips a device round trip) */
int rt_scene_prepare_host(const Triangle *triangles, int triangle_count, const KD_Tree_Node *nodes,
                          int node_count, const int *indices, int index_count, const int *lights,
                          int light_count, Bounding_Box bounds, rt_scene_t *out);
int rt_scene_release(rt_scene_t scene);
/* device bytes held by the prepared scene */
int rt_scene_info(rt_scene_t scene, size_t *device_bytes, int *triangle_count, int *node_count,
                  int *index_count, int *max_depth);

/* ---------------- render (rt/render.cuh:62-76) ---------------- */
/* work counters (SURVEY §8d algorithmic bytes) */
enum {
    RT_CNT_NODE = 0,   /* KD node fetches */
    RT_CNT_TRI = 1,    /* triangle tests */
    RT_CNT_HIT = 2,    /* closest-hit shadings */
    RT_CNT_TEXEL = 3,  /* texel reads */
    RT_CNT_NEE = 4,    /* next-event estimations */
    RT_CNT_SAMPLE = 5, /* samples traced */
    RT_CNT_SKIP = 6,   /* pixel-passes skipped by the adaptive test */
    RT_CNT_RAY = 7,    /* trace_ray calls */
    RT_CNT_WATCHDOG = 8, /* paths cut by the bounce watchdog */
    RT_CNT_MAXDEPTH = 9, /* longest path (extension rays) seen: atomic max, not a sum */
    /* the part of NODE / TRI / RAY done by the wavefront finisher launch
     * (already included in the totals above) */
    RT_CNT_FIN_NODE = 10,
    RT_CNT_FIN_TRI = 11,
    RT_CNT_FIN_RAY = 12,
    /* cooperative traversal diagnostics: plane-test prescreen survivors and
     * exact plane-test passes (barycentric tests) */
    RT_CNT_CAND = 13,
    RT_CNT_PLANE = 14,
    /* traversal pushes at stack index >= 19: each would write past the
     * reference's 19-entry stack arrays (rt/trace_ray.cuh:246-248);
     * reference-comparable, the oracle counts the same */
    RT_CNT_DEEP_PUSH = 15,
    /* cooperative trace, counting build only: wave-time (shader clocks,
     * summed over waves) in descent / leaf tests / ray fetch, and the number
     * of rounds, 64-entry plane chunks and barycentric batches */
    RT_CNT_T_DESCEND = 16,
    RT_CNT_T_LEAVES = 17,
    RT_CNT_T_FETCH = 18,
    RT_CNT_ROUNDS = 19,
    RT_CNT_CHUNKS = 20,
    RT_CNT_BARY = 21,
    /* finisher, counting build only: wide_trace calls / rounds / wave-time */
    RT_CNT_WIDE_CALLS = 22,
    RT_CNT_WIDE_ROUNDS = 23,
    RT_CNT_T_WIDE = 24,
    RT_CNT_T_WIDE_LOAD = 25,   /* wide_trace phases: frontier + node load, */
    RT_CNT_T_WIDE_LEAF = 26,   /* leaf batch, */
    RT_CNT_T_WIDE_EXPAND = 27, /* expansion */
    /* cooperative leaf test, counting build only: wave-time in the chunk
     * loop's plane-load wait, chunk set-up (owner scan, next load issue),
     * plane test + candidate append, and the barycentric stages */
    RT_CNT_T_LEAF_WAIT = 28,
    RT_CNT_T_LEAF_SETUP = 29,
    RT_CNT_T_LEAF_TEST = 30,
    RT_CNT_T_LEAF_BARY = 31,
    /* cooperative trace, counting build only: traversal-stack pushes and
     * pops beyond the LDS part of the stack (HBM spill), pending lanes summed
     * over the wave's leaf tests and the number of those tests, and the
     * descent's wave-time waiting for node loads */
    RT_CNT_SPILL_PUSH = 32,
    RT_CNT_SPILL_POP = 33,
    RT_CNT_PEND_LANES = 34,
    RT_CNT_LEAF_TESTS = 35,
    RT_CNT_T_DESC_WAIT = 36,
    /* RtOptions.traversal = RT_TRAVERSAL_BOUNDED_COUNTED only: the bounded
     * queue trace kernel's own work (RT_CNT_NODE / _TRI then count its KD
     * nodes / plane tests): BVH nodes, BVH plane tests, and the barycentric
     * records read by both phases */
    RT_CNT_B_BVH_NODE = 37,
    RT_CNT_B_BVH_TRI = 38,
    RT_CNT_B_BARY = 39,
    RT_CNT_COUNT = 40
};

#define RT_KERNEL_MEGA 0
#define RT_KERNEL_WAVEFRONT 1

typedef struct RtOptions {
    int width, height;   /* frame (rt/macros.h:3-4: 1920x1080) */
    int passes;          /* passes per call; the reference runs 1 per render() */
    int adaptive;        /* 1: rt/path_tracing.cuh:352-376 test; 0: always sample */
    int min_samples;     /* MIN_SAMPLES (rt/macros.h:13) */
    float tolerance;     /* MAX_TOLERANCE (rt/macros.h:17) */
    int max_depth;       /* 0 = unbounded (reference); else max extension rays per path */
    int kernel;          /* RT_KERNEL_MEGA (one launch) or RT_KERNEL_WAVEFRONT (trace/shade queues) */
    void *stream;        /* hipStream_t; NULL = synchronous on the null stream */
    unsigned long long *counters_device; /* optional RT_CNT_COUNT u64 counters (adds) */
    unsigned long long *wave_times_device; /* optional debug: megakernel (with counters): 2 u64 per wave;
                          * wavefront: 3 u64 per trace launch (first start, first queue
                          * exhaustion, ~last end; s_memrealtime, 100 MHz), pre-set to ~0 */
    /* wavefront tuning (0 = default): below wf_tail (default 65536) live
     * paths the rest of the call runs in one cooperative finisher launch on at
     * most wf_finish_waves waves (default 2048; 512 for trees with fewer than
     * 2^18 leaf entries, whose short rays keep fuller waves busy);
     * wf_tail > width*height runs the whole call in the finisher (persistent
     * per-wave path fetch, no queue iterations) */
    int wf_tail;
    int wf_finish_waves;
    int profile;         /* 1: time the wavefront kernels with HIP events (rt_last_profile) */
    /* cooperative traversal tuning (0 = default): node fetches per descent
     * round, and pending lanes (of 64) before a wave's leaf test runs */
    int wf_descent_cap;
    int wf_postpone;
    int wf_wide;         /* wide single-ray traversal (all 64 lanes on one ray, one ray after the other):
                          * < 0 off; else for the rays of a finisher wave with at most wf_wide live rays
                          * and, once a trace launch's queue is empty, of a trace wave with at most
                          * wf_wide rays left (0 = default 32) */
    /* row-interleaved sharding (the parity-exact option): with
     * num_shards > 1 only rows y % num_shards == shard_id are rendered (the
     * others are left untouched); every shard uses the single-stream seeds,
     * so each owned pixel is bit-identical to the one-GPU render, adaptive
     * sampling included, and a sum of the shards' zero-initialised buffers
     * (rt_reduce_shards) is the one-GPU frame.  The spp-slice sharding of the
     * north star needs no option: seed shard g's G_Buffer from mt19937 outputs
     * [g*W*H, (g+1)*W*H) (rt_gbuffer_seeds skip). */
    int shard_id;
    int num_shards;
    /* wavefront: concurrent pipelines over disjoint pixel tiles, each with
     * its own queues and stream, so one pipeline's latency-bound launch
     * tails and finisher overlap the others' bulk work (0 = default 3, max 3:
     * with the caller's stream that is the 4 hardware queues of a process) */
    int wf_pipelines;
    /* wavefront: a path deeper than this many bounces (total internal
     * reflection loops in glass reach 10^4 and more) is handed to a kernel
     * running beside the pipelines, which finishes it one ray per wave with
     * all 64 lanes (0 = default 64, < 0 = off; values below 16 are raised to
     * 16: the long-path kernel is sized for rare deep paths, and at 8 it took
     * a third of all paths and ran 7x slower) */
    int wf_long_depth;
    /* ray queries (identical results either way): RT_TRAVERSAL_BOUNDED
     * (default) first finds a lower bound of the ray's first hit distance in
     * a conservative BVH built by rt_scene_prepare and skips the KD subtrees
     * the reference would test for nothing; RT_TRAVERSAL_KD runs the KD
     * traversal alone.  Calls with counters_device run the KD traversal (its
     * counters are the reference's) unless traversal is
     * RT_TRAVERSAL_BOUNDED_COUNTED: the wavefront queue trace launches then
     * run the bounded traversal and count its own work (RT_CNT_RAY, _NODE,
     * _TRI, _HIT, RT_CNT_B_*; measurement: the finisher and the long-path
     * kernel are not counted; the megakernel then runs its counting KD build). */
    int traversal;
    /* chained calls (default render only: bounded traversal, not counting).
     * 0: the call is complete at its stream point.  1: the call is only
     * enqueued — the caller's stream does not wait for it — and the NEXT call
     * of the same frame — same scene, G_Buffer, camera and frame options,
     * sample_count != 0, overlap 1 — is enqueued right behind it: its path
     * kernel starts when the previous one ends, without waiting for the
     * long-path kernel, whose deep glass paths (10^4+ bounces) run on beside
     * it; the pixels those paths still hold are owed the new call's passes and
     * run them before they are let go.  Every pixel's passes
     * run in the reference's order, so the frame is bit-identical to
     * unchained calls.  A call with sample_count 0 (reset_frame) is never
     * chained: it completes before the next call starts.  Whatever reads the frame in
     * between must join first: rt_join(stream), rt_synchronize, or the
     * library's own readers (rt_tonemap, rt_save_render, rt_gbuffer_save,
     * rt_reduce_shards, rt_deviation_stats), which join by themselves.  A
     * join of an open chain first enqueues its drain (the pixels still owed
     * passes run to the end); so do a call that does not continue the chain
     * and rt_shutdown.  The
     * reference's render() (rt/render.cuh:62-76) has no such tail: a call is
     * complete when its launches are (rt/main.cu:114-155). */
    int overlap;
    /* run-time exactness guard of the bounded traversal (default render):
     * 1 ray in check_interval (rounded up to a power of two; 0 = 4096) of
     * those the finisher traces is recorded with its result and traced again
     * by the plain KD traversal after the call; disagreements are counted in
     * RtDeviations.bounded_mismatches.  < 0: off. */
    int check_interval;
    int debug;           /* RT_DEBUG_* bits: stderr diagnostics of the wavefront calls */
    /* chained calls (overlap 1) of fewer passes than this are coalesced on
     * the host (ABI 8): such a call is recorded and returns; the pending
     * calls of the same frame, options and stream are launched as ONE chained
     * call once they hold this many passes, or before anything that must see
     * them — another call, rt_join and the library's readers of the frame,
     * rt_last_profile / rt_profile_history (one record per launched batch),
     * rt_shutdown.  k calls of p passes run each pixel's passes in the same
     * order as one call of k*p: bit-identical.  0 = default 256; < 0 = off
     * (every call launches). */
    int coalesce_passes;
} RtOptions;

#define RT_TRAVERSAL_BOUNDED 0
#define RT_TRAVERSAL_KD 1
#define RT_TRAVERSAL_BOUNDED_COUNTED 2
#define RT_DEBUG_CALL_LOG 1  /* per call / queue iteration: counters and host times */
#define RT_DEBUG_LONG_LOG 2  /* every deep sample's claim / end time and bounces (unchained calls) */
#define RT_DEBUG_CHECK_FAULT 4 /* tests of the guard: every checked ray is recorded with a wrong result */
#define RT_DEBUG_LONG_QUIT 8   /* tests of the failure path: the long-path kernel leaves at once, as if its
                                * safety net fired, stranding every pixel handed to it */
#define RT_DEBUG_SERIAL_LONG_FIRST 16 /* tests of serialised dispatch (a profiler's counter collection): the
                                       * long-path kernel runs to its end before the path kernel starts */
#define RT_DEBUG_SERIAL_FIN_FIRST 32  /* ... the path kernel runs to its end before the long-path kernel starts */
/* (calls with RT_DEBUG_CALL_LOG, _LONG_LOG or _SERIAL_* are never coalesced) */

/* Per-call kernel timing of the last rt_render on this device with
 * RtOptions.profile = 1 (wavefront kernels: HIP events on the pipelines'
 * streams for the queue variants, the finisher's device span for the default
 * render; reading it waits for that call's kernels). */
typedef struct RtProfile {
    int iterations;      /* trace/shade queue iterations */
    int trace_launches, shade_launches, finish_launches;
    float start_ms;      /* wf_start */
    float trace_ms;      /* sum over the call's trace launches */
    float shade_ms;      /* sum over the call's shade launches */
    float finish_ms;     /* the finisher launches (0 or 1 per pipeline) */
    float call_ms;       /* first to last event of the call */
    float trace_union_ms; /* wall time with at least one trace launch running (launches of
                          * concurrent pipelines overlap: trace_ms sums their durations) */
    int pipelines;
} RtProfile;
int rt_last_profile(RtProfile *out);
/* every profiled rt_render's RtProfile on this device since the last reset,
 * oldest first: up to `cap` into out, the number recorded into *count.  For
 * the default render (one finisher launch per call) finish_ms and call_ms are
 * the finisher's span on the device, from its first wave's start to its last
 * wave's end (chained calls' finishers overlap: their spans do too), and
 * start_ms its start relative to the earliest start among the calls resolved
 * together (by this call or rt_last_profile).  Waits for those calls'
 * finishers. */
int rt_profile_history(RtProfile *out, int cap, int *count, int reset);

/* Always-on deviation statistics of every rt_render on the current device
 * since the last reset (recorded by every kernel, counting or not, at one
 * device-scope atomic per rare event).  The reference's bounce loop is
 * unbounded (rt/path_tracing.cuh:279-319); the build stops a path only at a
 * watchdog of 2^24 - 1 extension rays or at RtOptions.max_depth.
 * deep_hist[k] counts paths that ended at depth d (extension rays, as
 * RT_CNT_MAXDEPTH) with 64 * 2^k <= d < 64 * 2^(k+1); max_deep_depth is the
 * longest of them (0 if no path reached depth 64).  reset != 0 zeroes the
 * statistics after reading them.  Synchronises the device. */
#define RT_DEV_HIST_BINS 18
typedef struct RtDeviations {
    unsigned long long watchdog_paths; /* cut by the watchdog (max_depth 0): a deviation from the reference */
    unsigned long long cut_paths;      /* cut at the depth limit (watchdog or max_depth) */
    unsigned long long max_deep_depth; /* longest path that reached depth 64 */
    unsigned long long deep_paths;     /* paths that reached depth 64 (sum of deep_hist) */
    unsigned long long deep_hist[RT_DEV_HIST_BINS];
    /* the bounded traversal's run-time guard (RtOptions.check_interval): rays
     * re-traced by the plain KD traversal, results that differed (a deviation
     * from the reference; 0 expected), and the first such ray (o, d) */
    unsigned long long bounded_checked;
    unsigned long long bounded_mismatches;
    float mismatch_ray[6];
    /* the deep-path hand-off of the default render (ABI 7):
     * owed_pixels / owed_passes: pixels taken back from the long-path kernel
     * that chained calls (RtOptions.overlap) had skipped, and the passes they
     * owed (run by the taker, in the pixel's order; > 0 shows the chained-call
     * protocol fired).  Failure signals, 0 in a working render:
     * long_safety_quits: long-path waves that left by a safety net while
     * handed-over paths were still unclaimed; stranded_pixels: pixels still
     * handed over after a join's drain (the frame is incomplete: the join
     * returns RT_E_INCOMPLETE, and the pixels are released so later renders
     * run); check_dropped: rays the guard sampled past its per-call record
     * capacity (not re-traced).  linger_expiries: finisher waves that stopped
     * waiting (1 s) for pixels out in the long-path kernel, which then
     * finishes those pixels itself (a slow tail, not an error).
     * long_closed (ABI 8): long-path kernels that found their call's path
     * kernel not started within their bound (a profiler serialising
     * dispatches, a shared chip) and closed the hand-off until the next
     * unchained call: the path kernel then runs its deep paths itself
     * (identical results, a slower tail). */
    unsigned long long owed_pixels;
    unsigned long long owed_passes;
    unsigned long long long_safety_quits;
    unsigned long long stranded_pixels;
    unsigned long long check_dropped;
    unsigned long long linger_expiries;
    unsigned long long long_closed;
} RtDeviations;
int rt_deviation_stats(RtDeviations *out, int reset);

void rt_default_options(RtOptions *opt);
/* render(): if sample_count == 0 the frame's fb/sq/count are reset first
 * (reset_frame; RNG state is kept), then opt->passes passes run, each one
 * sample for every pixel that passes the adaptive test. */
int rt_render(rt_scene_t scene, G_Buffer g_buffer, Camera camera, int sample_count, const RtOptions *opt);

/* draw_frame's colour math (rt/render.cuh:37-59): correct_color(fb/count) ->
 * RGBA8 into a device buffer of width*height*4 bytes, row 0 = bottom. */
int rt_tonemap(G_Buffer g_buffer, uint8_t *rgba_device, int width, int height, void *stream);
/* save_render (rt/save_render.cuh:25-67): tonemap, flip vertically, write PNG */
int rt_save_render(G_Buffer g_buffer, int width, int height, const char *png_path);
/* the PNG encoder rt_save_render uses (replaces lodepng::encode,
 * rt/save_render.cuh:18-23): host RGBA8 rows top to bottom */
int rt_write_png(const char *png_path, const uint8_t *rgba_host, int width, int height);

/* ---------------- multi-GPU shards ----------------
 * One process per GPU.  Rank 0 makes an id (rt_comm_unique_id), ships its
 * RT_COMM_ID_BYTES to the other ranks out of band, every rank calls
 * rt_comm_create, renders its shard (spp slice: seeds skipped by g*W*H; or
 * rows: RtOptions.shard_id / num_shards), then rt_reduce_shards sums fb, sq
 * and count of every rank into `root` (one RCCL reduce per array, grouped;
 * stream NULL = synchronous). */
#define RT_COMM_ID_BYTES 128
typedef struct RtComm *rt_comm_t;
int rt_comm_unique_id(void *id_out);
int rt_comm_create(int nranks, int rank, const void *id, rt_comm_t *out);
int rt_comm_destroy(rt_comm_t comm);
int rt_reduce_shards(rt_comm_t comm, G_Buffer g_buffer, int width, int height, int root, void *stream);

/* self-test of the traversal's reciprocal-based division against IEEE '/'
 * on n random operand pairs (host); returns the number of mismatches */
unsigned long long rt_selftest_division(unsigned long long n, unsigned long long seed, unsigned long long *tested);

#ifdef __cplusplus
}
#endif
#endif /* ISAKLM_RT_H */
