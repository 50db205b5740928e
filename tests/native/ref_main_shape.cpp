// ref_main_shape.cpp — TEST FIXTURE: a translation unit shaped like the
// reference's rt/main.cu (rt/main.cu:8-14 includes every header, so its own
// types are in scope when the render path is called) switched to the MI355X
// library exactly as INTEGRATION.md describes:
//
//   1. the caller's own types — written here with the reference's
//      names, anonymous-union members and byte layout (rt/math_library.cuh:
//      55,99; rt/scene.cuh:16-121; rt/screen.cuh:15; rt/camera.cuh:15), a
//      G_Buffer with a constructor and a Camera with a member function, as
//      there;
//   2. INTEGRATION.md's compat header comes first, as in front of the
//      reference's headers: isaklm_rt.h with ISAKLM_RT_CALLER_TYPES (its
//      functions over the caller's types, forward-declared) and the macros
//      that send the host path's cudaMalloc / cudaMemcpy to the library;
//   3. once every type is defined, ISAKLM_RT_CHECK_LAYOUT() static_asserts
//      the byte layout the library assumes;
//   4. main() follows rt/main.cu:97-132: G_Buffer(), create_scene(), the
//      camera, the pass loop (rt_render replaces render()), save_render.
//
// create_scene() follows rt/create_scene.cuh:18-73 (triangles -> device,
// light list -> device, KD tree -> device) with the library's host loader
// and builder standing in for create_models() / create_kd_tree(), whose OBJ
// inputs the reference never published.
//
// usage: ref_main_shape SCENE.txt WIDTH HEIGHT SPP PASSES OUT.png
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

// ---- 2. INTEGRATION.md's compat header, in front of the reference's headers:
// the library over the caller's types (declared here, defined below), and
// the CUDA runtime calls of the host path mapped onto it
#define ISAKLM_RT_CALLER_TYPES
#include "isaklm_rt.h"
enum { cudaMemcpyHostToDevice = 1, cudaMemcpyDeviceToHost = 2 };
#define cudaMalloc(pp, bytes) rt_device_alloc((void **)(pp), (bytes))
#define cudaMemcpy(dst, src, bytes, kind) \
    ((kind) == cudaMemcpyHostToDevice ? rt_upload((dst), (src), (bytes)) : rt_download((dst), (src), (bytes)))

// ---- 1. the caller's types (reference layout) --------------------------
struct Vec2D {
    union { float x, u; };
    union { float y, v; };
};
struct Vec3D {
    union { float x, r; };
    union { float y, g; };
    union { float z, b; };
};
struct uchar4 { unsigned char x, y, z, w; };
struct Matrix3X3 { Vec3D i_hat, j_hat, k_hat; };
struct Texture {
    uchar4 *buffer;
    int width = 0;
    int height = 0;
};
struct Material {
    Vec3D albedo, emittance;
    float roughness, refractive_index, extinction;
    bool transparent;
    Texture texture;
};
struct Triangle {
    Vec3D p1, p2, p3;
    Vec3D n1, n2, n3;
    Vec2D uv1, uv2, uv3;
    Material material;
};
struct KD_Tree_Node {
    union { int index_offset, child_index1; };
    union { int triangle_count, child_index2; };
    uint8_t plane_axis;
    float plane_offset;
    bool is_leaf_node;
};
struct Bounding_Box { Vec3D min, max; };
struct KD_Tree {
    Bounding_Box bounding_box;
    KD_Tree_Node *nodes;
    int *triangle_indicies;
};
struct Scene {
    Triangle *triangles;
    int triangle_count;
    int *light_indicies;
    int light_count;
    KD_Tree kd_tree;
};
struct Camera {
    Vec3D position;
    float yaw, pitch;
    float FOV;
    float aperture_radius;
    Matrix3X3 rotation() const { return Matrix3X3{}; } // (the reference's, rt/camera.cuh:22-25; unused here)
};

static int g_w = 1920, g_h = 1080; // SCREEN_W / SCREEN_H (rt/macros.h:3-4)

// G_Buffer() as rt/screen.cuh:22-46 writes it (one allocation per array; the
// reference's doubled cudaMalloc leak is not reproduced) + the zeroing its
// reset_frame would do before the first pass
struct G_Buffer {
    Vec3D *frame_buffer;
    float *squared_luminance;
    int *sample_count;
    uint32_t *random_numbers;
    G_Buffer()
    {
        const size_t n = (size_t)g_w * g_h;
        cudaMalloc(&frame_buffer, n * sizeof(Vec3D));
        cudaMalloc(&squared_luminance, n * sizeof(float));
        cudaMalloc(&sample_count, n * sizeof(int));
        std::vector<uint32_t> seeds(n);
        std::mt19937 generator;
        std::uniform_int_distribution<uint32_t> distribution(0, UINT32_MAX);
        for (size_t i = 0; i < n; ++i) seeds[i] = distribution(generator);
        cudaMalloc(&random_numbers, n * sizeof(uint32_t));
        cudaMemcpy(random_numbers, seeds.data(), n * sizeof(uint32_t), cudaMemcpyHostToDevice);
        rt_memset(frame_buffer, 0, n * sizeof(Vec3D));
        rt_memset(squared_luminance, 0, n * sizeof(float));
        rt_memset(sample_count, 0, n * sizeof(int));
    }
};

// ---- 3. every caller type defined: the layout the library assumes
ISAKLM_RT_CHECK_LAYOUT();

static const char *g_scene_file = nullptr;
static Camera g_camera;

// create_scene (rt/create_scene.cuh:18-73)
static Scene create_scene()
{
    Scene scene{};
    RtHostScene *host = nullptr;
    if (rt_host_scene_create(&host) != RT_OK || rt_host_scene_load_file(host, g_scene_file, &g_camera) != RT_OK) {
        fprintf(stderr, "create_scene: %s\n", rt_last_error());
        exit(1);
    }
    const Triangle *tris = nullptr;
    int count = 0;
    rt_host_scene_triangles(host, &tris, &count); // create_models()
    cudaMalloc(&scene.triangles, count * sizeof(Triangle));
    cudaMemcpy(scene.triangles, tris, count * sizeof(Triangle), cudaMemcpyHostToDevice);
    scene.triangle_count = count;
    std::vector<int> lights; // emissive triangles (:40-64)
    for (int i = 0; i < count; ++i)
        if (tris[i].material.emittance.r > 0 || tris[i].material.emittance.g > 0 || tris[i].material.emittance.b > 0)
            lights.push_back(i);
    cudaMalloc(&scene.light_indicies, lights.size() * sizeof(int));
    cudaMemcpy(scene.light_indicies, lights.data(), lights.size() * sizeof(int), cudaMemcpyHostToDevice);
    scene.light_count = (int)lights.size();
    KD_Tree_Node *nodes = nullptr; // create_kd_tree (rt/create_kd_tree.cuh:267-328)
    int *indices = nullptr, nnodes = 0, nindices = 0;
    Bounding_Box bb;
    if (rt_build_kd_tree(tris, count, &nodes, &nnodes, &indices, &nindices, &bb) != RT_OK) {
        fprintf(stderr, "create_kd_tree: %s\n", rt_last_error());
        exit(1);
    }
    cudaMalloc(&scene.kd_tree.nodes, nnodes * sizeof(KD_Tree_Node));
    cudaMemcpy(scene.kd_tree.nodes, nodes, nnodes * sizeof(KD_Tree_Node), cudaMemcpyHostToDevice);
    cudaMalloc(&scene.kd_tree.triangle_indicies, nindices * sizeof(int));
    cudaMemcpy(scene.kd_tree.triangle_indicies, indices, nindices * sizeof(int), cudaMemcpyHostToDevice);
    scene.kd_tree.bounding_box = bb;
    rt_host_free(nodes);
    rt_host_free(indices);
    // (the host scene owns textures' host texels; the test scenes have none)
    return scene;
}

int main(int argc, char **argv)
{
    if (argc != 7) {
        fprintf(stderr, "usage: ref_main_shape SCENE.txt WIDTH HEIGHT SPP PASSES OUT.png\n");
        return 2;
    }
    if (rt_abi_version() != RT_ABI_VERSION) {
        fprintf(stderr, "library ABI %d, header %d\n", rt_abi_version(), RT_ABI_VERSION);
        return 3;
    }
    g_scene_file = argv[1];
    g_w = atoi(argv[2]);
    g_h = atoi(argv[3]);
    const int max_samples = atoi(argv[4]), passes = atoi(argv[5]);
    if (rt_set_device(0) != RT_OK) {
        fprintf(stderr, "%s\n", rt_last_error());
        return 1;
    }

    G_Buffer g_buffer = G_Buffer();   // rt/main.cu:97
    Scene scene = create_scene();     // rt/main.cu:99
    rt_scene_t prepared;
    if (rt_scene_prepare(&scene, &prepared) != RT_OK) {
        fprintf(stderr, "rt_scene_prepare: %s\n", rt_last_error());
        return 1;
    }
    Camera camera = g_camera;         // rt/main.cu:101-104 (the scene file's camera line)

    RtOptions opt;
    rt_default_options(&opt);
    opt.width = g_w;
    opt.height = g_h;
    opt.adaptive = 0;
    for (int sample_count = 0; sample_count < max_samples; sample_count += opt.passes) { // rt/main.cu:114-132
        opt.passes = max_samples - sample_count < passes ? max_samples - sample_count : passes;
        if (rt_render(prepared, g_buffer, camera, sample_count, &opt) != RT_OK) {
            fprintf(stderr, "rt_render: %s\n", rt_last_error());
            return 1;
        }
    }
    if (rt_save_render(g_buffer, g_w, g_h, argv[6]) != RT_OK) { // save_render (rt/main.cu:126)
        fprintf(stderr, "rt_save_render: %s\n", rt_last_error());
        return 1;
    }
    rt_scene_release(prepared);
    printf("ok\n");
    return 0;
}
