// rt_host.h — host-side (CPU) pieces of the render path's boundary:
// scene loading, exact KD build, seeds, scene preparation, image output.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "../rt_device.h"
#include "../rt_vecmath.h"

void rt_set_error(const char *fmt, ...);

// A decoded texture owned by a host scene.  Host triangles' material.texture
// points at `texels` (host memory); rt_create_scene uploads every texture once
// and points the device triangles at the device copy (make_texture,
// rt/scene.cuh:25-63, cudaMallocs at load time instead).
struct RtHostTexture {
    std::string path; // as written in the .mat file
    int width = 0, height = 0;
    std::vector<RtUChar4> texels; // width * height + RT_TEXTURE_PAD
};

struct RtHostScene {
    std::vector<Triangle> tris;
    std::vector<std::unique_ptr<RtHostTexture>> textures;
};

namespace rt_host {

// load_mesh (rt/mesh_loading.cuh:221-440)
int load_mesh(RtHostScene &scene, const std::string &obj_path, const std::string &mat_path, Vec3D offset,
              RtM3 matrix, bool smooth_normals);
// create_models as data (rt/create_models.cuh:17-43) + camera (rt/main.cu:101-104)
int load_scene_file(RtHostScene &scene, const std::string &path, Camera *camera_out);

// create_kd_tree (rt/create_kd_tree.cuh:267-328), identical output
int build_kd_tree(const Triangle *tris, int n, std::vector<KD_Tree_Node> &nodes, std::vector<int> &indices,
                  Bounding_Box &bounds);
// light list of create_scene (rt/create_scene.cuh:40-49)
std::vector<int> light_list(const Triangle *tris, int n);

// std::mt19937 seeds (rt/screen.cuh:34-45)
void mt19937_seeds(uint32_t *out, size_t count, uint64_t skip);

// host image of the device layout (rt_device.h) before upload
struct PreparedHost {
    std::vector<uint32_t> nodes;
    std::vector<RtF4> isect_a;          // leaf-entry order
    std::vector<RtIsectBary> isect_bary; // leaf-entry order
    std::vector<uint32_t> isect_tri;      // leaf-entry order: the entry's triangle (= isect_bary[e].tri)
    std::vector<RtF4> shade;
    std::vector<RtDevMaterial> materials;
    std::vector<int> lights; // light_count + 1
    int light_count = 0;
    int max_depth = 0;
    Bounding_Box bounds;
    // the conservative BVH that bounds each ray's first hit (bvh_build.h);
    // bvh_depth < 0: not built (the KD-only traversal runs)
    std::vector<RtF4> bvh_nodes;          // 4 per node
    std::vector<RtF4> bvh4;               // the 4-wide collapse (bvh_build.h collapse_bvh4), 8 per node
    int bvh4_stack = 0;                   // the deepest stack its query can build (must be < RT_BVH_STACK)
    std::vector<RtF4> bvh_a;              // BVH leaf-slot order
    std::vector<RtIsectBary> bvh_bary;    // BVH leaf-slot order
    float bvh_scale = 0.0f;
    std::vector<float> split_vals;        // per axis sorted, unique (rt_bounded_ray)
    int split_off[4] = {0, 0, 0, 0};
    int bvh_depth = -1, bvh_always = 0, bvh_dropped = 0;
    // wf_long's origin-cell entry (coop_trace.h kd_origin_frontier): per cell
    // of a kd_grid^3 grid over the scene box, {KD start node, row offset << 5
    // | depth} (0xFFFFFFFF: none; cell of a point: (p - bounds.min) *
    // kd_grid_scale), and per start node the root-to-start path, one record
    // per ancestor {split bits, y word, ancestor index, 0 = child0 / 1 = child1}
    std::vector<uint32_t> kd_rows;
    std::vector<uint32_t> kd_cell;
    // the bounded KD phase's entry (bvh_trace.h kd_bounded): per grid cell
    // {start node bits, its cell's lo.xyz}, {hi.xyz, 0} (+-inf where no split
    // bounds it); and the split values per axis as open-addressing hash sets
    int kd_grid = 0;
    float kd_grid_scale[3] = {0, 0, 0};
};
// fills the origin-cell tables from the prepared KD nodes (scene_prepare.cpp)
void build_kd_starts(PreparedHost &out, const Bounding_Box &bounds);
int prepare_host(const Triangle *tris, int ntris, const KD_Tree_Node *nodes, int nnodes, const int *indices,
                 int nindices, const int *lights, int nlights, Bounding_Box bounds, PreparedHost &out);

int write_png(const char *path, const uint8_t *rgba, int width, int height);

// stbi_load(path, &w, &h, &n, 4) for PNG and baseline JPEG (image_decode.cpp)
int decode_image_memory(const uint8_t *data, size_t size, std::vector<uint8_t> &rgba, int &width, int &height,
                        std::string &err);
int decode_image_file(const std::string &path, std::vector<uint8_t> &rgba, int &width, int &height,
                      std::string &err);

} // namespace rt_host
