// rt_render — the reference's main() (rt/main.cu:60-155) without the GLFW
// window: C++ host code over the C-ABI of include/isaklm_rt.h.
//
//   G_Buffer g_buffer = G_Buffer();            -> rt_gbuffer_create
//   Scene scene = create_scene();              -> rt_host_scene_load_file (create_models as data)
//                                                 + rt_create_scene + rt_scene_prepare
//   Camera camera = {...}                      -> the scene file's camera line (or the reference's)
//   call_render(...); ++sample_count;          -> rt_render with `passes` passes per call
//   if (sample_count >= MAX_SAMPLES) save_render(g_buffer)  -> rt_save_render
//
// usage: rt_render [--scene FILE | --generate NAME DIR] [--width W] [--height H]
//                  [--spp N] [--passes P] [--adaptive 0|1] [--min-samples N]
//                  [--tolerance T] [--max-depth D] [--kernel mega|wavefront]
//                  [--shard G N] [--device D] [--out PNG] [--quiet]
//                  [--checkpoint FILE] [--resume FILE]
// --checkpoint writes the G_Buffer + sample count after every rt_render call
// (rt_gbuffer_save); --resume continues from such a file (rt_gbuffer_load),
// bit-identical to a render that never stopped.
// Defaults are the reference's macros (rt/macros.h): 1920x1080, MAX_SAMPLES
// 5000, MIN_SAMPLES 100, MAX_TOLERANCE 0.05, adaptive sampling on.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>

#include "isaklm_rt.h"

namespace {

int fail(const char *what)
{
    fprintf(stderr, "rt_render: %s: %s\n", what, rt_last_error());
    return 1;
}

void usage()
{
    fprintf(stderr,
            "usage: rt_render [--scene FILE | --generate NAME DIR] [--width W] [--height H] [--spp N]\n"
            "                 [--passes P] [--adaptive 0|1] [--min-samples N] [--tolerance T] [--max-depth D]\n"
            "                 [--kernel mega|wavefront] [--shard G N] [--device D] [--out PNG] [--quiet]\n"
            "                 [--checkpoint FILE] [--resume FILE]\n");
}

} // namespace

int main(int argc, char **argv)
{
    std::string scene_path, gen_name, gen_dir, out = "render.png", checkpoint, resume;
    int width = 1920, height = 1080, spp = 5000, passes = 64, adaptive = 1, min_samples = 100, max_depth = 0;
    int device = 0, shard_id = 0, num_shards = 1, kernel = RT_KERNEL_WAVEFRONT;
    float tolerance = 0.05f;
    bool quiet = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&](void) -> const char * {
            if (i + 1 >= argc) {
                usage();
                exit(2);
            }
            return argv[++i];
        };
        if (a == "--scene") scene_path = next();
        else if (a == "--generate") { gen_name = next(); gen_dir = next(); }
        else if (a == "--width") width = atoi(next());
        else if (a == "--height") height = atoi(next());
        else if (a == "--spp") spp = atoi(next());
        else if (a == "--passes") passes = atoi(next());
        else if (a == "--adaptive") adaptive = atoi(next());
        else if (a == "--min-samples") min_samples = atoi(next());
        else if (a == "--tolerance") tolerance = (float)atof(next());
        else if (a == "--max-depth") max_depth = atoi(next());
        else if (a == "--kernel") kernel = std::string(next()) == "mega" ? RT_KERNEL_MEGA : RT_KERNEL_WAVEFRONT;
        else if (a == "--shard") { shard_id = atoi(next()); num_shards = atoi(next()); }
        else if (a == "--device") device = atoi(next());
        else if (a == "--out") out = next();
        else if (a == "--quiet") quiet = true;
        else if (a == "--checkpoint") checkpoint = next();
        else if (a == "--resume") resume = next();
        else {
            usage();
            return 2;
        }
    }
    if (scene_path.empty() == gen_name.empty() || width <= 0 || height <= 0 || spp <= 0 || passes <= 0) {
        usage();
        return 2;
    }
    if (!gen_name.empty()) {
        char buf[4096];
        if (rt_generate_scene(gen_name.c_str(), gen_dir.c_str(), buf, sizeof buf) != RT_OK) return fail("generate");
        scene_path = buf;
    }
    if (rt_set_device(device) != RT_OK) return fail("set_device");

    // G_Buffer() (rt/screen.cuh:22-46); a row shard keeps the single-stream seeds
    G_Buffer g_buffer;
    if (rt_gbuffer_create(width, height, 0, &g_buffer) != RT_OK) return fail("G_Buffer");

    // create_scene() (rt/create_scene.cuh:18): create_models, create_kd_tree, upload
    const auto t0 = std::chrono::steady_clock::now();
    RtHostScene *host = nullptr;
    if (rt_host_scene_create(&host) != RT_OK) return fail("host scene");
    Camera camera = {{-2.1f, 1.7f, -1.2f}, 0.975f, 0.3f, 1.57079632679f, 0.002f}; // rt/main.cu:101-104
    if (rt_host_scene_load_file(host, scene_path.c_str(), &camera) != RT_OK) return fail("create_models");
    Scene scene;
    if (rt_create_scene(host, &scene, nullptr, nullptr) != RT_OK) return fail("create_scene");
    rt_scene_t prepared = nullptr;
    if (rt_scene_prepare(&scene, &prepared) != RT_OK) return fail("prepare"); // counts derived from the tree
    rt_host_scene_destroy(host);
    const double setup_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    RtOptions opt;
    rt_default_options(&opt);
    opt.width = width;
    opt.height = height;
    opt.adaptive = adaptive;
    opt.min_samples = min_samples;
    opt.tolerance = tolerance;
    opt.max_depth = max_depth;
    opt.kernel = kernel;
    opt.shard_id = shard_id;
    opt.num_shards = num_shards;

    // the frame loop (rt/main.cu:114-155): call_render, ++sample_count, save at MAX_SAMPLES
    const auto t1 = std::chrono::steady_clock::now();
    int sample_count = 0;
    if (!resume.empty()) {
        if (rt_gbuffer_load(resume.c_str(), g_buffer, width, height, &sample_count) != RT_OK) return fail("resume");
        if (!quiet) printf("resumed at %d samples per pixel\n", sample_count);
    }
    while (sample_count < spp) {
        opt.passes = passes < spp - sample_count ? passes : spp - sample_count;
        if (rt_render(prepared, g_buffer, camera, sample_count, &opt) != RT_OK) return fail("render");
        sample_count += opt.passes;
        if (!checkpoint.empty() && rt_gbuffer_save(g_buffer, width, height, sample_count, checkpoint.c_str()) != RT_OK)
            return fail("checkpoint");
        if (!quiet) printf("samples per pixel: %d\n", sample_count);
    }
    if (rt_synchronize() != RT_OK) return fail("synchronize");
    const double render_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    if (rt_save_render(g_buffer, width, height, out.c_str()) != RT_OK) return fail("save_render");
    printf("rendered %dx%d x %d spp in %.3f s (%.2f Msamples/s nominal; scene setup %.2f s) -> %s\n", width, height,
           spp, render_s, (double)width * height * spp / render_s / 1e6, setup_s, out.c_str());

    rt_scene_release(prepared);
    rt_destroy_scene(&scene);
    rt_gbuffer_destroy(&g_buffer);
    return 0;
}
