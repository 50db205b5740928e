// rt_device.h — the MI355X traversal layout of a prepared scene.
//
// The reference keeps 152-B AoS triangles with an embedded material and 20-B
// AoS KD nodes (rt/scene.cuh:65-100).  A ray query there reads 36 of the 152
// bytes per triangle test and recomputes the plane, cross product, normalize
// and Cramer denominators each time (rt/trace_ray.cuh:73-113).  Here:
//
//  * nodes: 8 B each, pre-order, child1 == node+1 implicit
//      inner:  x = plane_offset bits, y = (child2 << 2) | axis      (axis 0..2)
//      leaf:   x = index_offset,      y = (triangle_count << 2) | 3
//  * intersection constants in LEAF-ENTRY order (entry e = position in the
//    KD triangle_indicies array, so a leaf's tests read consecutive memory
//    and need no index load first), each value the reference's own
//    expression evaluated once:
//      isect_a[e]    = {n.x, n.y, n.z, d}   n = normalize(cross(p2-p1, p3-p1)), d = dot(n, p1)
//                      (16-B stream: every test reads it)
//      isect_bary[e] = one 64-B record (one cache line per candidate):
//                      {p1, d00}, {v0 = p2-p1, d01}, {v1 = p3-p1, d11},
//                      {bits(1/(d00*d11 - d01*d01)), triangle index, -, -}
//    A test that is rejected by the plane (dn == 0, s < 1e-5, s >= closest)
//    reads only isect_a (16 B); about 1 in 5 goes on to the record.
//  * shading record (hit only), 7 float4 per triangle: p1..p3, n1..n3,
//    uv1..uv3 and the material id; materials deduplicated into a table.
#pragma once
#include <stdint.h>

#include "../../include/isaklm_rt.h"

// Traversal stack entries.  The reference declares KD_TREE_DEPTH = 19 entries
// (rt/trace_ray.cuh:246-248) but its builder makes inner nodes at depths
// 0..19 (rt/create_kd_tree.cuh:225,246: split while depth < 19), i.e. up to
// 20 nested pushes: a latent overflow in the reference.  The kernel is built
// for 20 (every create_kd_tree tree) and 32 (other trees).
#define RT_STACK_SMALL 20
#define RT_STACK_DEPTH 32
#define RT_REF_STACK 19 // KD_TREE_DEPTH (rt/macros.h): the reference's stack arrays' length
#define RT_LEAF_TAG 3u
// the reference's bounce loop is unbounded (rt/path_tracing.cuh:
// 279-319).  The watchdog cuts a path only at 2^24 - 1 extension rays (the
// largest depth the wavefront path flags hold, flags >> 8): far above the
// longest path measured on any test or bench scene (RtDeviations, bench line).
#define RT_WATCHDOG_BOUNCES ((1 << 24) - 1)
// always-on deviation statistics (rt_deviation_stats): a path that ends at
// this depth or deeper is recorded (max depth, log2 histogram) with one
// device-scope atomic — rare (total internal reflection in glass)
#define RT_DEEP_PATH 64
#define RT_DEV_WATCHDOG 0   // paths cut by the watchdog (max_depth == 0)
#define RT_DEV_MAXDEPTH 1   // longest path that ended at depth >= RT_DEEP_PATH (atomic max)
#define RT_DEV_CUT 2        // paths cut at the depth limit (watchdog or RtOptions.max_depth)
#define RT_DEV_HIST 3       // + k: paths ending at depth in [64 * 2^k, 64 * 2^(k+1)), k < RT_DEV_HIST_BINS
                            // (isaklm_rt.h: 18 bins, 64 * 2^18 = 2^24 > RT_WATCHDOG_BOUNCES)
#define RT_DEV_CHECKED 21   // rays of the bounded traversal re-traced by the KD traversal (wf_check)
#define RT_DEV_MISMATCH 22  // ... whose results differed
#define RT_DEV_MISRAY 23    // 4 words: set flag, then the first mismatching ray's o, d as packed float bits
// the chained-call hand-off protocol (wavefront.hip), one atomic per rare event:
#define RT_DEV_OWED_PIXELS 27 // pixels taken back from wf_long owing passes of later chained calls
#define RT_DEV_OWED_PASSES 28 // ... the passes they owed (run by the taker, in order)
#define RT_DEV_LONG_QUIT 29   // wf_long waves that left by a safety net with hand-off entries unclaimed
#define RT_DEV_LINGER_EXP 30  // finisher waves whose linger expired with pixels still out in wf_long
#define RT_DEV_CHK_DROP 31    // guard records dropped past WF_CHECK_CAP (rays not re-traced)
#define RT_DEV_STRANDED 32    // pixels found still OUT after a join's drain (wf_verify): an incomplete frame
#define RT_DEV_LONG_CLOSED 33 // wf_long closed the hand-off ring: its call's finisher had not started (serialised
                              // dispatch); the finisher's lanes ran their deep paths themselves
#define RT_DEV_WORDS 48
// rt_wavefront_join's return when its hand-off check found stranded pixels (-1: a HIP failure)
#define RT_WAVEFRONT_INCOMPLETE (-2)
static_assert(RT_DEV_HIST + RT_DEV_HIST_BINS <= RT_DEV_CHECKED && RT_DEV_MISRAY + 4 <= RT_DEV_OWED_PIXELS &&
                  RT_DEV_LONG_CLOSED < RT_DEV_WORDS,
              "deviation block");

struct RtDevMaterial {          // 64 B
    float albedo[3];
    float roughness;
    float emittance[3];
    float refractive_index;
    float extinction;
    int transparent;
    int tex_width, tex_height;
    const RtUChar4 *tex;        // device texels or nullptr
    int pad[2];
};
static_assert(sizeof(RtDevMaterial) == 64, "RtDevMaterial");

struct RtF4 { float x, y, z, w; };

struct RtIsectBary {            // 64 B, one per leaf entry
    RtF4 b;                     // p1, d00
    RtF4 c;                     // v0, d01
    RtF4 d;                     // v1, d11
    uint32_t rd;                // bits(1 / (d00*d11 - d01*d01))
    uint32_t tri;               // triangle index
    uint32_t pad[2];
};
static_assert(sizeof(RtIsectBary) == 64, "RtIsectBary");

struct RtDevScene {
    const uint32_t *nodes;      // 2 words per node
    const RtF4 *isect_a;        // per leaf entry: plane
    const RtIsectBary *isect_bary; // per leaf entry: barycentric-test record
    const uint32_t *isect_tri;  // per leaf entry: its triangle (isect_bary[e].tri, 16 to a line: bvh_trace.h's T* scan)
    const RtF4 *shade;          // 7 per triangle
    const RtDevMaterial *materials;
    const int *lights;          // light_count + 1 entries (SURVEY H4 padding)
    int light_count;
    int triangle_count;
    int index_count;            // KD leaf entries
    float bmin[3], bmax[3];
    // conservative BVH bounding each ray's first hit (host/bvh_build.h,
    // bvh_trace.h); bvh_nodes == nullptr: none (KD-only traversal)
    const RtF4 *bvh_nodes;      // 4 per node: child boxes {lo0, hi0.x}, {hi0.yz, lo1.xy}, {lo1.z, hi1}, {ref0, ref1, -, -}
    const RtF4 *bvh4;           // its 4-wide collapse, 8 per node: lo.x, lo.y, lo.z, hi.x, hi.y, hi.z of 4 children, refs, -
    const RtF4 *bvh_a;          // per BVH leaf slot: plane (as isect_a)
    const RtIsectBary *bvh_bary; // per BVH leaf slot: barycentric-test record (as isect_bary)
    float bvh_scale;            // largest |vertex|_1 (rt_ray_margin)
    const float *split_vals;    // the KD tree's split values, per axis sorted (rt_bounded_ray)
    int split_off[4];           // axis a: split_vals[split_off[a], split_off[a + 1])
    // wf_long's origin-cell entry (host/scene_prepare.cpp build_kd_starts,
    // coop_trace.h kd_origin_frontier); nullptr / 0: none
    const uint32_t *kd_rows;    // 4 words per ancestor: split bits, y word, ancestor index, child taken
    const uint32_t *kd_cell;    // per cell of a kd_grid^3 grid over the scene box: {start node, row offset << 5 | depth}
    int kd_grid;                // cell of p: ((p - bmin) * kd_gscale), clamped to [0, kd_grid - 1]
    float kd_gscale[3];
};

// BVH child reference: an inner node's index, or RT_BVH_LEAF | first << 3 |
// (count - 1) for the leaf of slots [first, first + count), or RT_BVH_EMPTY
#define RT_BVH_LEAF 0x80000000u
#define RT_BVH_EMPTY 0xFFFFFFFFu
#define RT_BVH_LEAF_MAX 8
#define RT_BVH_STACK 64 // traversal stack entries: trees deeper than this are not used

struct RtDevCamera {            // Camera precomputed once per call (same ops as the reference)
    float R[9];                 // rotation_matrix(yaw, pitch): i, j, k
    float pos[3];
    float tan_half_fov;         // tanf(FOV / 2)
    float aperture;
};

struct RtDevFrame {
    Vec3D *fb;
    float *sq;
    int *count;
    uint32_t *rng;
    int width, height, half_w, half_h;
    int passes;
    int adaptive;
    int min_samples;
    float tolerance;
    float z_const;              // sqrtf(2) * erfinvf(1 - tolerance)
    int max_depth;              // 0 = unbounded (watchdog)
    int reset;                  // sample_count == 0
    unsigned long long *counters;
    unsigned long long *wave_times; // debug: per-wave s_memrealtime [start, end] (counting variant)
    int shard_id, num_shards;   // row-interleaved sharding: render rows y % num_shards == shard_id
    unsigned long long *dev_stats; // RT_DEV_WORDS always-on deviation statistics (every kernel, counting or not)
};
