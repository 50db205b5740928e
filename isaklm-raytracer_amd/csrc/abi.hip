// abi.hip — implementation of include/isaklm_rt.h (the drop-in boundary).
//
// Thin by design: host scene code lives in host/*.cpp, kernels in
// path_kernel.hip.  Every entry point checks its arguments and every HIP
// call, returning RT_E_* instead of the reference's silent failures
// (SURVEY §5 "Failure detection").
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "host/rt_host.h"

int rt_launch_path(const RtDevScene &sc, const RtDevFrame &fr, const RtDevCamera &cam, int stack_depth,
                   hipStream_t stream, int traversal);
int rt_launch_tonemap(const Vec3D *fb, const int *count, RtUChar4 *out, int n, hipStream_t stream);
int rt_launch_wavefront(const RtDevScene &sc, const RtDevFrame &fr, const RtDevCamera &cam, hipStream_t stream,
                        int variant, int tail, int finish_waves, int profile, int cap, int postpone, int wide,
                        int pipes, int long_depth, int traversal, int overlap, int check_interval, int debug,
                        int coalesce);

int rt_wavefront_device_init();
int rt_wavefront_join(void *stream, int consume);
void rt_wavefront_shutdown();
void rt_path_shutdown();

static thread_local std::string g_error;

void rt_set_error(const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_error = buf;
}

#define HIPCHK(expr)                                                                                 \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) {                                                                      \
            rt_set_error("%s failed: %s", #expr, hipGetErrorString(e_));                             \
            return RT_E_HIP;                                                                         \
        }                                                                                            \
    } while (0)

const char *rt_wavefront_incomplete_msg();

// rt_wavefront_join with the ABI's status: RT_E_INCOMPLETE when the join's
// hand-off check found stranded pixels (a chained render's frame misses
// passes), RT_E_HIP on a HIP failure; `who` names the entry point
// (consume = 0: a stranded-pixel result is left for the next reporting join)
static int join_status(void *stream, const char *who, int consume = 1)
{
    const int rc = rt_wavefront_join(stream, consume);
    if (rc == 0) return RT_OK;
    if (rc == RT_WAVEFRONT_INCOMPLETE) {
        rt_set_error("%s: %s", who, rt_wavefront_incomplete_msg());
        return RT_E_INCOMPLETE;
    }
    rt_set_error("%s: join: %s", who, hipGetErrorString(hipGetLastError()));
    return RT_E_HIP;
}

struct RtPreparedScene {
    RtDevScene dev;
    std::vector<void *> allocs;
    size_t bytes = 0;
    int ntris = 0, nnodes = 0, nindices = 0, max_depth = 0;
};

namespace {

template <typename T>
int upload_vec(RtPreparedScene &s, const std::vector<T> &v, const T **out)
{
    void *p = nullptr;
    size_t n = v.size() * sizeof(T);
    // 64 zero bytes of slack after every array: the traversal's 16-B node-pair
    // loads read one node past the last (never used: the last node in
    // pre-order is a leaf)
    HIPCHK(hipMalloc(&p, n + 64));
    s.allocs.push_back(p);
    s.bytes += n;
    HIPCHK(hipMemset(p, 0, n + 64));
    if (n) HIPCHK(hipMemcpy(p, v.data(), n, hipMemcpyHostToDevice));
    *out = (const T *)p;
    return RT_OK;
}

void release(RtPreparedScene *s)
{
    if (!s) return;
    for (void *p : s->allocs) (void)hipFree(p);
    delete s;
}

int upload_prepared(const rt_host::PreparedHost &h, int ntris, int nindices, rt_scene_t *out)
{
    RtPreparedScene *s = new RtPreparedScene();
    int rc = RT_OK;
    const uint32_t *nodes = nullptr;
    const int *lights = nullptr;
    const RtF4 *a = nullptr, *sh = nullptr;
    const RtIsectBary *bary = nullptr;
    const uint32_t *itri = nullptr;
    const RtDevMaterial *mats = nullptr;
    if ((rc = upload_vec(*s, h.nodes, &nodes)) || (rc = upload_vec(*s, h.isect_a, &a)) ||
        (rc = upload_vec(*s, h.isect_bary, &bary)) || (rc = upload_vec(*s, h.isect_tri, &itri)) ||
        (rc = upload_vec(*s, h.shade, &sh)) ||
        (rc = upload_vec(*s, h.materials, &mats)) || (rc = upload_vec(*s, h.lights, &lights))) {
        release(s);
        return rc;
    }
    RtDevScene &dv = s->dev;
    dv.bvh_nodes = nullptr;
    dv.bvh4 = nullptr;
    dv.bvh_a = nullptr;
    dv.bvh_bary = nullptr;
    dv.bvh_scale = h.bvh_scale;
    dv.split_vals = nullptr;
    dv.kd_rows = nullptr;
    dv.kd_cell = nullptr;
    dv.kd_grid = 0;
    for (int a = 0; a < 3; ++a) dv.kd_gscale[a] = h.kd_grid_scale[a];
    for (int a = 0; a < 4; ++a) dv.split_off[a] = h.split_off[a];
    if (h.bvh_depth >= 0 && ((rc = upload_vec(*s, h.bvh_nodes, &dv.bvh_nodes)) ||
                             (rc = upload_vec(*s, h.bvh4, &dv.bvh4)) ||
                             (rc = upload_vec(*s, h.bvh_a, &dv.bvh_a)) ||
                             (rc = upload_vec(*s, h.bvh_bary, &dv.bvh_bary)) ||
                             (rc = upload_vec(*s, h.split_vals, &dv.split_vals)))) {
        release(s);
        return rc;
    }
    // the root-path records and the grid (wf_long's deep bounces enter at the origin's cell)
    if (!h.kd_rows.empty() && ((rc = upload_vec(*s, h.kd_rows, &dv.kd_rows)) ||
                               (h.kd_grid > 0 && (rc = upload_vec(*s, h.kd_cell, &dv.kd_cell))))) {
        release(s);
        return rc;
    }
    if (dv.kd_cell) dv.kd_grid = h.kd_grid;
    dv.nodes = nodes;
    dv.isect_a = a;
    dv.isect_bary = bary;
    dv.isect_tri = itri;
    dv.shade = sh;
    dv.materials = mats;
    dv.lights = lights;
    dv.light_count = h.light_count;
    dv.triangle_count = ntris;
    dv.index_count = nindices;
    dv.bmin[0] = h.bounds.min.x; dv.bmin[1] = h.bounds.min.y; dv.bmin[2] = h.bounds.min.z;
    dv.bmax[0] = h.bounds.max.x; dv.bmax[1] = h.bounds.max.y; dv.bmax[2] = h.bounds.max.z;
    s->ntris = ntris;
    s->nnodes = (int)(h.nodes.size() / 2);
    s->nindices = nindices;
    s->max_depth = h.max_depth;
    *out = s;
    return RT_OK;
}

// always-on deviation statistics (RT_DEV_*), one zeroed block per device
std::mutex g_dev_mu;
std::map<int, unsigned long long *> g_dev_stats;

unsigned long long *dev_stats_block()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(g_dev_mu);
    auto it = g_dev_stats.find(dev);
    if (it != g_dev_stats.end()) return it->second;
    void *p = nullptr;
    if (hipMalloc(&p, RT_DEV_WORDS * 8) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, RT_DEV_WORDS * 8) != hipSuccess) {
        (void)hipFree(p);
        return nullptr;
    }
    g_dev_stats[dev] = (unsigned long long *)p;
    return (unsigned long long *)p;
}

} // namespace

// rt_shutdown at exit, registered once by rt_set_device / the first render:
// atexit handlers run in reverse registration order, so this one (registered
// after the HIP runtime initialised) runs before the runtime's own finalisers
// and the library's streams, events and blobs are gone before they run
void rt_register_shutdown()
{
    static std::once_flag once;
    std::call_once(once, [] { atexit(rt_shutdown); });
}

extern "C" {

const char *rt_last_error(void) { return g_error.c_str(); }
const char *rt_version(void) { return "isaklm-raytracer_amd 0.3 (gfx950)"; }
int rt_abi_version(void) { return RT_ABI_VERSION; }

void rt_shutdown(void)
{
    rt_wavefront_shutdown();
    rt_path_shutdown();
    std::lock_guard<std::mutex> g(g_dev_mu);
    for (auto &kv : g_dev_stats) {
        if (hipSetDevice(kv.first) == hipSuccess) (void)hipFree(kv.second);
    }
    g_dev_stats.clear();
}

int rt_join(void *stream) { return join_status(stream, "rt_join"); }

int rt_deviation_stats(RtDeviations *out, int reset)
{
    if (!out) { rt_set_error("rt_deviation_stats: null out"); return RT_E_INVALID; }
    unsigned long long *d = dev_stats_block();
    if (!d) { rt_set_error("rt_deviation_stats: no device block"); return RT_E_HIP; }
    unsigned long long w[RT_DEV_WORDS];
    // (chained renders joined first, so their statistics are complete; stranded
    // pixels are not an error here — stranded_pixels reports them — and stay the
    // next reporting join's RT_E_INCOMPLETE: rt_join, rt_download, rt_synchronize ...)
    const int jr = join_status(nullptr, "rt_deviation_stats", 0);
    if (jr != RT_OK && jr != RT_E_INCOMPLETE) return jr;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(w, d, sizeof w, hipMemcpyDeviceToHost));
    memset(out, 0, sizeof *out);
    out->watchdog_paths = w[RT_DEV_WATCHDOG];
    out->cut_paths = w[RT_DEV_CUT];
    out->max_deep_depth = w[RT_DEV_MAXDEPTH];
    for (int k = 0; k < RT_DEV_HIST_BINS; ++k) {
        out->deep_hist[k] = w[RT_DEV_HIST + k];
        out->deep_paths += w[RT_DEV_HIST + k];
    }
    out->bounded_checked = w[RT_DEV_CHECKED];
    out->bounded_mismatches = w[RT_DEV_MISMATCH];
    for (int k = 0; k < 3; ++k) {
        const uint32_t hi = (uint32_t)(w[RT_DEV_MISRAY + 1 + k] >> 32), lo = (uint32_t)w[RT_DEV_MISRAY + 1 + k];
        memcpy(&out->mismatch_ray[2 * k], &hi, 4);
        memcpy(&out->mismatch_ray[2 * k + 1], &lo, 4);
    }
    out->owed_pixels = w[RT_DEV_OWED_PIXELS];
    out->owed_passes = w[RT_DEV_OWED_PASSES];
    out->long_safety_quits = w[RT_DEV_LONG_QUIT];
    out->stranded_pixels = w[RT_DEV_STRANDED];
    out->check_dropped = w[RT_DEV_CHK_DROP];
    out->linger_expiries = w[RT_DEV_LINGER_EXP];
    out->long_closed = w[RT_DEV_LONG_CLOSED];
    if (reset) HIPCHK(hipMemset(d, 0, RT_DEV_WORDS * 8));
    return RT_OK;
}

// ---------------- device memory ----------------
int rt_device_alloc(void **ptr, size_t bytes)
{
    if (!ptr) { rt_set_error("rt_device_alloc: null out"); return RT_E_INVALID; }
    HIPCHK(hipMalloc(ptr, bytes ? bytes : 16));
    return RT_OK;
}
int rt_free(void *ptr)
{
    if (ptr) HIPCHK(hipFree(ptr));
    return RT_OK;
}
int rt_upload(void *dst, const void *src, size_t bytes)
{
    if (bytes == 0) return RT_OK;
    if (!dst || !src) { rt_set_error("rt_upload: null pointer"); return RT_E_INVALID; }
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return RT_OK;
}
int rt_download(void *dst, const void *src, size_t bytes)
{
    if (bytes == 0) return RT_OK;
    if (!dst || !src) { rt_set_error("rt_download: null pointer"); return RT_E_INVALID; }
    // (cudaMemcpy after a render waits for it; so does this, chained renders' tails included)
    const int jr = join_status(nullptr, "rt_download");
    if (jr != RT_OK) return jr;
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return RT_OK;
}
int rt_memset(void *dst, int value, size_t bytes)
{
    if (bytes == 0) return RT_OK;
    HIPCHK(hipMemset(dst, value, bytes));
    return RT_OK;
}
int rt_device_count(int *count)
{
    if (!count) return RT_E_INVALID;
    HIPCHK(hipGetDeviceCount(count));
    return RT_OK;
}
int rt_set_device(int device)
{
    HIPCHK(hipSetDevice(device));
    rt_register_shutdown();
    if (rt_wavefront_device_init() != 0) { // the pipelines' streams take their hardware queues first
        rt_set_error("rt_set_device: wavefront streams: %s", hipGetErrorString(hipGetLastError()));
        return RT_E_HIP;
    }
    return RT_OK;
}
int rt_synchronize(void)
{
    // (chained renders' open chain drained first: hipDeviceSynchronize alone never
    // enqueues the drain, and their owed passes would never run)
    const int jr = join_status(nullptr, "rt_synchronize");
    if (jr != RT_OK) return jr;
    HIPCHK(hipDeviceSynchronize());
    return RT_OK;
}
void rt_host_free(void *p) { free(p); }

// ---------------- texture decoding (make_texture's stbi_load, rt/scene.cuh:33) ----------------
static int decode_out(int rc, const std::vector<uint8_t> &rgba, const std::string &err, int w, int h,
                      uint8_t **rgba_out, int *width, int *height)
{
    if (rc != RT_OK) {
        rt_set_error("rt_decode_image: %s", err.c_str());
        return rc;
    }
    uint8_t *p = (uint8_t *)malloc(rgba.size() ? rgba.size() : 1);
    if (!p) { rt_set_error("rt_decode_image: out of host memory"); return RT_E_NOMEM; }
    memcpy(p, rgba.data(), rgba.size());
    *rgba_out = p;
    *width = w;
    *height = h;
    return RT_OK;
}

int rt_decode_image(const char *path, uint8_t **rgba_out, int *width, int *height)
{
    if (!path || !rgba_out || !width || !height) { rt_set_error("rt_decode_image: null argument"); return RT_E_INVALID; }
    std::vector<uint8_t> rgba;
    std::string err;
    int w = 0, h = 0;
    const int rc = rt_host::decode_image_file(path, rgba, w, h, err);
    return decode_out(rc, rgba, err, w, h, rgba_out, width, height);
}

int rt_decode_image_memory(const void *data, size_t size, uint8_t **rgba_out, int *width, int *height)
{
    if (!data || !rgba_out || !width || !height) {
        rt_set_error("rt_decode_image_memory: null argument");
        return RT_E_INVALID;
    }
    std::vector<uint8_t> rgba;
    std::string err;
    int w = 0, h = 0;
    const int rc = rt_host::decode_image_memory((const uint8_t *)data, size, rgba, w, h, err);
    return decode_out(rc, rgba, err, w, h, rgba_out, width, height);
}

// ---------------- G_Buffer ----------------
int rt_gbuffer_seeds(uint32_t *out, size_t count, uint64_t skip)
{
    if (!out && count) { rt_set_error("rt_gbuffer_seeds: null out"); return RT_E_INVALID; }
    rt_host::mt19937_seeds(out, count, skip);
    return RT_OK;
}

int rt_gbuffer_create(int w, int h, uint64_t skip, G_Buffer *g)
{
    if (!g || w <= 0 || h <= 0) { rt_set_error("rt_gbuffer_create: bad arguments"); return RT_E_INVALID; }
    const size_t n = (size_t)w * (size_t)h;
    memset(g, 0, sizeof *g);
    std::vector<uint32_t> seeds(n);
    rt_host::mt19937_seeds(seeds.data(), n, skip);
    HIPCHK(hipMalloc((void **)&g->frame_buffer, n * sizeof(Vec3D)));
    HIPCHK(hipMalloc((void **)&g->squared_luminance, n * sizeof(float)));
    HIPCHK(hipMalloc((void **)&g->sample_count, n * sizeof(int)));
    HIPCHK(hipMalloc((void **)&g->random_numbers, n * sizeof(uint32_t)));
    HIPCHK(hipMemset(g->frame_buffer, 0, n * sizeof(Vec3D)));
    HIPCHK(hipMemset(g->squared_luminance, 0, n * sizeof(float)));
    HIPCHK(hipMemset(g->sample_count, 0, n * sizeof(int)));
    HIPCHK(hipMemcpy(g->random_numbers, seeds.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice));
    return RT_OK;
}

int rt_gbuffer_destroy(G_Buffer *g)
{
    if (!g) return RT_E_INVALID;
    (void)rt_wavefront_join(nullptr, 0); // (a chained render's tail may still write it)
    (void)hipFree(g->frame_buffer);
    (void)hipFree(g->squared_luminance);
    (void)hipFree(g->sample_count);
    (void)hipFree(g->random_numbers);
    memset(g, 0, sizeof *g);
    return RT_OK;
}

// ---------------- checkpoint / resume ----------------
// file: "RTGBUF01", int32 width, height, sample_count, 0; then fb (12 B/px),
// sq, count, rng (4 B/px each), host byte order
static const char kGbufMagic[8] = {'R', 'T', 'G', 'B', 'U', 'F', '0', '1'};

int rt_gbuffer_save(G_Buffer g, int width, int height, int sample_count, const char *path)
{
    if (!path || width <= 0 || height <= 0 || !g.frame_buffer || !g.squared_luminance || !g.sample_count ||
        !g.random_numbers) {
        rt_set_error("rt_gbuffer_save: bad arguments");
        return RT_E_INVALID;
    }
    const size_t n = (size_t)width * height;
    std::vector<uint8_t> buf(n * 24);
    // rt_render's pipelines run on their own non-blocking streams, and a chained render's
    // owed passes run only in the open chain's drain: join (drain) first, then synchronise
    const int jr = join_status(nullptr, "rt_gbuffer_save");
    if (jr != RT_OK) return jr;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(buf.data(), g.frame_buffer, n * 12, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(buf.data() + n * 12, g.squared_luminance, n * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(buf.data() + n * 16, g.sample_count, n * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(buf.data() + n * 20, g.random_numbers, n * 4, hipMemcpyDeviceToHost));
    // write beside the target and rename over it: an interrupted save never
    // leaves a torn checkpoint in place of the previous one
    const std::string tmp = std::string(path) + ".tmp";
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) {
        rt_set_error("rt_gbuffer_save: cannot write %s", tmp.c_str());
        return RT_E_IO;
    }
    const int32_t hdr[4] = {width, height, sample_count, 0};
    const bool ok = fwrite(kGbufMagic, 1, 8, f) == 8 && fwrite(hdr, 4, 4, f) == 4 &&
                    fwrite(buf.data(), 1, buf.size(), f) == buf.size();
    if (fclose(f) != 0 || !ok || rename(tmp.c_str(), path) != 0) {
        remove(tmp.c_str());
        rt_set_error("rt_gbuffer_save: write error on %s", path);
        return RT_E_IO;
    }
    return RT_OK;
}

int rt_gbuffer_load(const char *path, G_Buffer g, int width, int height, int *sample_count_out)
{
    if (!path) {
        rt_set_error("rt_gbuffer_load: null path");
        return RT_E_INVALID;
    }
    FILE *f = fopen(path, "rb");
    if (!f) {
        rt_set_error("rt_gbuffer_load: cannot read %s", path);
        return RT_E_IO;
    }
    char magic[8];
    int32_t hdr[4];
    if (fread(magic, 1, 8, f) != 8 || memcmp(magic, kGbufMagic, 8) != 0 || fread(hdr, 4, 4, f) != 4) {
        fclose(f);
        rt_set_error("rt_gbuffer_load: %s is not a G_Buffer checkpoint", path);
        return RT_E_PARSE;
    }
    if (hdr[0] != width || hdr[1] != height || !g.frame_buffer || !g.squared_luminance || !g.sample_count ||
        !g.random_numbers) {
        fclose(f);
        rt_set_error("rt_gbuffer_load: checkpoint is %dx%d, G_Buffer %dx%d", hdr[0], hdr[1], width, height);
        return RT_E_INVALID;
    }
    const size_t n = (size_t)width * height;
    std::vector<uint8_t> buf(n * 24);
    const bool ok = fread(buf.data(), 1, buf.size(), f) == buf.size();
    fclose(f);
    if (!ok) {
        rt_set_error("rt_gbuffer_load: %s is truncated", path);
        return RT_E_PARSE;
    }
    // no render may still be writing this G_Buffer (a chained render's tail drained and
    // joined first; the chain is closed, so the next call does not continue it)
    const int jr = join_status(nullptr, "rt_gbuffer_load", 0); // (a stranded result stays the next join's)
    if (jr != RT_OK && jr != RT_E_INCOMPLETE) return jr;
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(g.frame_buffer, buf.data(), n * 12, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(g.squared_luminance, buf.data() + n * 12, n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(g.sample_count, buf.data() + n * 16, n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(g.random_numbers, buf.data() + n * 20, n * 4, hipMemcpyHostToDevice));
    if (sample_count_out) *sample_count_out = hdr[2];
    return RT_OK;
}

// ---------------- host scene ----------------
int rt_host_scene_create(RtHostScene **out)
{
    if (!out) return RT_E_INVALID;
    *out = new RtHostScene();
    return RT_OK;
}
void rt_host_scene_destroy(RtHostScene *s) { delete s; }

int rt_host_scene_load_mesh(RtHostScene *s, const char *obj, const char *mat, const float offset[3],
                            const float m[9], int smooth)
{
    if (!s || !obj || !mat || !offset || !m) { rt_set_error("rt_host_scene_load_mesh: null argument"); return RT_E_INVALID; }
    RtM3 M = {rt_v3(m[0], m[1], m[2]), rt_v3(m[3], m[4], m[5]), rt_v3(m[6], m[7], m[8])};
    return rt_host::load_mesh(*s, obj, mat, rt_v3(offset[0], offset[1], offset[2]), M, smooth != 0);
}

int rt_host_scene_load_file(RtHostScene *s, const char *path, Camera *cam)
{
    if (!s || !path) { rt_set_error("rt_host_scene_load_file: null argument"); return RT_E_INVALID; }
    return rt_host::load_scene_file(*s, path, cam);
}

int rt_host_scene_triangles(const RtHostScene *s, const Triangle **tris, int *count)
{
    if (!s || !tris || !count) return RT_E_INVALID;
    *tris = s->tris.data();
    *count = (int)s->tris.size();
    return RT_OK;
}

int rt_build_kd_tree(const Triangle *tris, int n, KD_Tree_Node **nodes_out, int *node_count, int **idx_out,
                     int *index_count, Bounding_Box *bounds)
{
    if (!tris || n <= 0 || !nodes_out || !node_count || !idx_out || !index_count || !bounds) {
        rt_set_error("rt_build_kd_tree: bad arguments");
        return RT_E_INVALID;
    }
    std::vector<KD_Tree_Node> nodes;
    std::vector<int> idx;
    int rc = rt_host::build_kd_tree(tris, n, nodes, idx, *bounds);
    if (rc) return rc;
    *nodes_out = (KD_Tree_Node *)malloc(nodes.size() * sizeof(KD_Tree_Node));
    *idx_out = (int *)malloc((idx.size() ? idx.size() : 1) * sizeof(int));
    if (!*nodes_out || !*idx_out) { rt_set_error("out of host memory"); return RT_E_NOMEM; }
    memcpy(*nodes_out, nodes.data(), nodes.size() * sizeof(KD_Tree_Node));
    memcpy(*idx_out, idx.data(), idx.size() * sizeof(int));
    *node_count = (int)nodes.size();
    *index_count = (int)idx.size();
    return RT_OK;
}

// create_scene (rt/create_scene.cuh:18-73)
// device textures uploaded by rt_create_scene, per device triangle array (freed by rt_destroy_scene)
static std::mutex g_tex_mu;
static std::map<const void *, std::vector<void *>> g_scene_textures;

int rt_create_scene(const RtHostScene *s, Scene *out, int *node_count, int *index_count)
{
    if (!s || !out || s->tris.empty()) { rt_set_error("rt_create_scene: bad arguments"); return RT_E_INVALID; }
    memset(out, 0, sizeof *out);
    const int n = (int)s->tris.size();
    std::vector<KD_Tree_Node> nodes;
    std::vector<int> idx;
    Bounding_Box bb;
    int rc = rt_host::build_kd_tree(s->tris.data(), n, nodes, idx, bb);
    if (rc) return rc;
    std::vector<int> lights = rt_host::light_list(s->tris.data(), n);
    HIPCHK(hipMalloc((void **)&out->triangles, (size_t)n * sizeof(Triangle)));
    if (s->textures.empty()) {
        HIPCHK(hipMemcpy(out->triangles, s->tris.data(), (size_t)n * sizeof(Triangle), hipMemcpyHostToDevice));
    } else {
        // make_texture's cudaMalloc/cudaMemcpy (rt/scene.cuh:58-59): one device
        // copy per decoded texture (with its zero pad), triangles re-pointed to it
        std::map<const void *, RtUChar4 *> dev;
        std::vector<void *> owned;
        for (const auto &t : s->textures) {
            RtUChar4 *d = nullptr;
            const size_t bytes = t->texels.size() * sizeof(RtUChar4);
            HIPCHK(hipMalloc((void **)&d, bytes));
            owned.push_back(d);
            HIPCHK(hipMemcpy(d, t->texels.data(), bytes, hipMemcpyHostToDevice));
            dev[t->texels.data()] = d;
        }
        std::vector<Triangle> tris(s->tris);
        for (Triangle &t : tris)
            if (t.material.texture.buffer) {
                auto it = dev.find(t.material.texture.buffer);
                if (it == dev.end()) {
                    rt_set_error("rt_create_scene: triangle texture not owned by the host scene");
                    for (void *d : owned) (void)hipFree(d);
                    return RT_E_INVALID;
                }
                t.material.texture.buffer = it->second;
            }
        HIPCHK(hipMemcpy(out->triangles, tris.data(), (size_t)n * sizeof(Triangle), hipMemcpyHostToDevice));
        std::lock_guard<std::mutex> g(g_tex_mu);
        g_scene_textures[out->triangles] = owned;
    }
    out->triangle_count = n;
    HIPCHK(hipMalloc((void **)&out->light_indicies, (lights.size() + 1) * sizeof(int)));
    if (!lights.empty())
        HIPCHK(hipMemcpy(out->light_indicies, lights.data(), lights.size() * sizeof(int), hipMemcpyHostToDevice));
    out->light_count = (int)lights.size();
    HIPCHK(hipMalloc((void **)&out->kd_tree.nodes, nodes.size() * sizeof(KD_Tree_Node)));
    HIPCHK(hipMemcpy(out->kd_tree.nodes, nodes.data(), nodes.size() * sizeof(KD_Tree_Node), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc((void **)&out->kd_tree.triangle_indicies, (idx.size() + 1) * sizeof(int)));
    if (!idx.empty())
        HIPCHK(hipMemcpy(out->kd_tree.triangle_indicies, idx.data(), idx.size() * sizeof(int), hipMemcpyHostToDevice));
    out->kd_tree.bounding_box = bb;
    if (node_count) *node_count = (int)nodes.size();
    if (index_count) *index_count = (int)idx.size();
    return RT_OK;
}

int rt_destroy_scene(Scene *s)
{
    if (!s) return RT_E_INVALID;
    {
        std::lock_guard<std::mutex> g(g_tex_mu);
        auto it = g_scene_textures.find(s->triangles);
        if (it != g_scene_textures.end()) {
            for (void *d : it->second) (void)hipFree(d);
            g_scene_textures.erase(it);
        }
    }
    (void)hipFree(s->triangles);
    (void)hipFree(s->light_indicies);
    (void)hipFree(s->kd_tree.nodes);
    (void)hipFree(s->kd_tree.triangle_indicies);
    memset(s, 0, sizeof *s);
    return RT_OK;
}

// ---------------- prepared scene ----------------
int rt_scene_prepare_host(const Triangle *tris, int ntris, const KD_Tree_Node *nodes, int nnodes, const int *idx,
                          int nidx, const int *lights, int nlights, Bounding_Box bounds, rt_scene_t *out)
{
    if (!out) return RT_E_INVALID;
    rt_host::PreparedHost h;
    int rc = rt_host::prepare_host(tris, ntris, nodes, nnodes, idx, nidx, lights, nlights, bounds, h);
    if (rc) return rc;
    return upload_prepared(h, ntris, nidx, out);
}

// bytes from p to the end of the device allocation that holds it
static int bytes_to_alloc_end(const void *p, size_t *bytes)
{
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (!p || hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) != hipSuccess || !base) {
        (void)hipGetLastError();
        return -1;
    }
    *bytes = (size_t)((const char *)base + size - (const char *)p);
    return 0;
}

// The reference's Scene (rt/scene.cuh:107-121) carries no node or index
// count (they are locals of create_kd_tree, rt/create_kd_tree.cuh:286,300),
// so they are recovered from the device tree itself: the tree is walked
// pre-order from node 0 over a copy of its allocation (hipMemGetAddressRange
// bounds the copy); node_count = highest reachable node + 1, index_count =
// the largest offset + count of a non-empty leaf.  A child index outside the
// allocation, a cycle or a shared subtree is an error.
int rt_scene_prepare(const Scene *ds, rt_scene_t *out)
{
    if (!ds || !out || ds->triangle_count <= 0 || ds->light_count < 0 || !ds->kd_tree.nodes || !ds->triangles) {
        rt_set_error("rt_scene_prepare: bad arguments");
        return RT_E_INVALID;
    }
    size_t node_bytes = 0, index_bytes = 0;
    if (bytes_to_alloc_end(ds->kd_tree.nodes, &node_bytes) != 0) {
        rt_set_error("rt_scene_prepare: kd_tree.nodes is not a device allocation of this process");
        return RT_E_INVALID;
    }
    const size_t max_nodes = node_bytes / sizeof(KD_Tree_Node);
    if (max_nodes == 0 || max_nodes >= (1u << 30)) {
        rt_set_error("rt_scene_prepare: node allocation of %zu bytes", node_bytes);
        return RT_E_INVALID;
    }
    std::vector<KD_Tree_Node> nodes(max_nodes);
    HIPCHK(hipMemcpy(nodes.data(), ds->kd_tree.nodes, max_nodes * sizeof(KD_Tree_Node), hipMemcpyDeviceToHost));
    std::vector<uint8_t> seen(max_nodes, 0);
    std::vector<int> stack{0};
    long long max_node = 0, index_count = 0;
    while (!stack.empty()) {
        const int i = stack.back();
        stack.pop_back();
        if (i < 0 || (size_t)i >= max_nodes || seen[(size_t)i]) {
            rt_set_error("rt_scene_prepare: KD node index %d outside the node allocation, or reached twice", i);
            return RT_E_INVALID;
        }
        seen[(size_t)i] = 1;
        max_node = i > max_node ? i : max_node;
        const KD_Tree_Node &n = nodes[(size_t)i];
        if (n.is_leaf_node) {
            if (n.triangle_count > 0) {
                const long long end = (long long)n.index_offset + n.triangle_count;
                index_count = end > index_count ? end : index_count;
            }
        } else {
            stack.push_back(n.child_index2);
            stack.push_back(n.child_index1);
        }
    }
    if (index_count > 0 && (bytes_to_alloc_end(ds->kd_tree.triangle_indicies, &index_bytes) != 0 ||
                            (size_t)index_count > index_bytes / sizeof(int))) {
        rt_set_error("rt_scene_prepare: leaves address %lld triangle indices beyond the index allocation",
                     index_count);
        return RT_E_INVALID;
    }
    return rt_scene_prepare_counts(ds, (int)(max_node + 1), (int)index_count, out);
}

int rt_scene_prepare_counts(const Scene *ds, int node_count, int index_count, rt_scene_t *out)
{
    if (!ds || !out || ds->triangle_count <= 0 || node_count <= 0 || index_count < 0 || ds->light_count < 0) {
        rt_set_error("rt_scene_prepare: bad arguments");
        return RT_E_INVALID;
    }
    std::vector<Triangle> tris((size_t)ds->triangle_count);
    std::vector<KD_Tree_Node> nodes((size_t)node_count);
    std::vector<int> idx((size_t)index_count), lights((size_t)ds->light_count);
    HIPCHK(hipMemcpy(tris.data(), ds->triangles, tris.size() * sizeof(Triangle), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(nodes.data(), ds->kd_tree.nodes, nodes.size() * sizeof(KD_Tree_Node), hipMemcpyDeviceToHost));
    if (index_count)
        HIPCHK(hipMemcpy(idx.data(), ds->kd_tree.triangle_indicies, idx.size() * sizeof(int), hipMemcpyDeviceToHost));
    if (ds->light_count)
        HIPCHK(hipMemcpy(lights.data(), ds->light_indicies, lights.size() * sizeof(int), hipMemcpyDeviceToHost));
    return rt_scene_prepare_host(tris.data(), ds->triangle_count, nodes.data(), node_count, idx.data(), index_count,
                                 lights.data(), ds->light_count, ds->kd_tree.bounding_box, out);
}

int rt_scene_release(rt_scene_t s)
{
    (void)rt_wavefront_join(nullptr, 0); // (a chained render's tail may still read it)
    release(s);
    return RT_OK;
}

int rt_scene_info(rt_scene_t s, size_t *bytes, int *ntris, int *nnodes, int *nidx, int *max_depth)
{
    if (!s) return RT_E_INVALID;
    if (bytes) *bytes = s->bytes;
    if (ntris) *ntris = s->ntris;
    if (nnodes) *nnodes = s->nnodes;
    if (nidx) *nidx = s->nindices;
    if (max_depth) *max_depth = s->max_depth;
    return RT_OK;
}

// ---------------- render ----------------
void rt_default_options(RtOptions *o)
{
    if (!o) return;
    memset(o, 0, sizeof *o);
    o->width = 1920;       // rt/macros.h:3
    o->height = 1080;      // rt/macros.h:4
    o->passes = 1;
    o->adaptive = 1;
    o->min_samples = 100;  // rt/macros.h:13
    o->tolerance = 0.05f;  // rt/macros.h:17
    o->max_depth = 0;
}

// render (rt/render.cuh:62-76)
int rt_render(rt_scene_t scene, G_Buffer g, Camera cam, int sample_count, const RtOptions *opt)
{
    RtOptions o;
    if (opt) o = *opt; else rt_default_options(&o);
    if (!scene || !g.frame_buffer || !g.squared_luminance || !g.sample_count || !g.random_numbers) {
        rt_set_error("rt_render: null scene or G_Buffer array");
        return RT_E_INVALID;
    }
    if (o.width <= 0 || o.height <= 0 || o.width < 2 || o.passes < 0 || o.min_samples < 0 ||
        (long long)o.width * o.height > (1LL << 31) - 1) {
        rt_set_error("rt_render: bad frame size / passes");
        return RT_E_INVALID;
    }
    if (o.num_shards > 1 && (o.shard_id < 0 || o.shard_id >= o.num_shards)) {
        rt_set_error("rt_render: shard_id %d out of [0, %d)", o.shard_id, o.num_shards);
        return RT_E_INVALID;
    }
    RtDevFrame fr;
    fr.fb = g.frame_buffer;
    fr.sq = g.squared_luminance;
    fr.count = g.sample_count;
    fr.rng = g.random_numbers;
    fr.width = o.width;
    fr.height = o.height;
    fr.half_w = o.width / 2;   // SCREEN_W / 2 (integer division)
    fr.half_h = o.height / 2;
    fr.passes = o.passes;
    fr.adaptive = o.adaptive;
    fr.min_samples = o.min_samples;
    fr.tolerance = o.tolerance;
    fr.z_const = rt_adaptive_z(o.tolerance);
    fr.max_depth = o.max_depth;
    fr.reset = sample_count == 0;
    fr.shard_id = o.num_shards > 1 ? o.shard_id : 0;
    fr.num_shards = o.num_shards > 1 ? o.num_shards : 1;
    fr.counters = o.counters_device;
    fr.wave_times = o.wave_times_device;
    fr.dev_stats = dev_stats_block();
    if (!fr.dev_stats) {
        rt_set_error("rt_render: deviation statistics block: %s", hipGetErrorString(hipGetLastError()));
        return RT_E_HIP;
    }

    // Camera::rotation() and tanf(FOV / 2) are frame constants (rt/camera.cuh:22-25, :381)
    RtDevCamera dc;
    RtM3 R = rt_rotation_matrix(cam.yaw, cam.pitch);
    dc.R[0] = R.i.x; dc.R[1] = R.i.y; dc.R[2] = R.i.z;
    dc.R[3] = R.j.x; dc.R[4] = R.j.y; dc.R[5] = R.j.z;
    dc.R[6] = R.k.x; dc.R[7] = R.k.y; dc.R[8] = R.k.z;
    dc.pos[0] = cam.position.x; dc.pos[1] = cam.position.y; dc.pos[2] = cam.position.z;
    dc.tan_half_fov = rt_tanf(cam.FOV / 2);
    dc.aperture = cam.aperture_radius;

    hipStream_t stream = (hipStream_t)o.stream;
    if (o.kernel >= RT_KERNEL_WAVEFRONT && o.kernel <= 3) {
        if (scene->max_depth > RT_STACK_DEPTH ||
            rt_launch_wavefront(scene->dev, fr, dc, stream, o.kernel, o.wf_tail, o.wf_finish_waves, o.profile,
                                o.wf_descent_cap, o.wf_postpone, o.wf_wide, o.wf_pipelines, o.wf_long_depth,
                                o.traversal, o.overlap, o.check_interval, o.debug, o.coalesce_passes) != 0) {
            rt_set_error("rt_render: wavefront launch failed: %s", hipGetErrorString(hipGetLastError()));
            return RT_E_HIP;
        }
    } else {
        const int jr = join_status(stream, "rt_render"); // (chained wavefront calls' tails first: same frame state)
        if (jr != RT_OK) return jr;
        if (rt_launch_path(scene->dev, fr, dc, scene->max_depth, stream, o.traversal) != 0) {
            rt_set_error("rt_render: kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
            return RT_E_HIP;
        }
    }
    if (!o.stream) HIPCHK(hipStreamSynchronize(nullptr));
    return RT_OK;
}

int rt_tonemap(G_Buffer g, uint8_t *rgba, int w, int h, void *stream)
{
    if (!rgba || !g.frame_buffer || !g.sample_count || w <= 0 || h <= 0) {
        rt_set_error("rt_tonemap: bad arguments");
        return RT_E_INVALID;
    }
    const int jr = join_status(stream, "rt_tonemap"); // chained renders' deep-path tails first
    if (jr != RT_OK) return jr;
    if (rt_launch_tonemap(g.frame_buffer, g.sample_count, (RtUChar4 *)rgba, w * h, (hipStream_t)stream) != 0) {
        rt_set_error("rt_tonemap: launch failed");
        return RT_E_HIP;
    }
    if (!stream) HIPCHK(hipStreamSynchronize(nullptr));
    return RT_OK;
}

// save_render (rt/save_render.cuh:25-67): tonemap on the GPU, flip rows, PNG
int rt_save_render(G_Buffer g, int w, int h, const char *path)
{
    if (!path || w <= 0 || h <= 0) { rt_set_error("rt_save_render: bad arguments"); return RT_E_INVALID; }
    const size_t n = (size_t)w * h;
    uint8_t *d = nullptr;
    HIPCHK(hipMalloc((void **)&d, n * 4));
    int rc = rt_tonemap(g, d, w, h, nullptr);
    std::vector<uint8_t> img(n * 4), flipped(n * 4);
    if (rc == RT_OK && hipMemcpy(img.data(), d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        rt_set_error("rt_save_render: download failed");
        rc = RT_E_HIP;
    }
    (void)hipFree(d);
    if (rc) return rc;
    for (int y = 0; y < h; ++y) // flipped_pixel_index = (H - y - 1) * W + x  (:55)
        memcpy(&flipped[(size_t)(h - y - 1) * w * 4], &img[(size_t)y * w * 4], (size_t)w * 4);
    return rt_host::write_png(path, flipped.data(), w, h);
}

int rt_write_png(const char *path, const uint8_t *rgba, int w, int h)
{
    if (!path || !rgba || w <= 0 || h <= 0) { rt_set_error("rt_write_png: bad arguments"); return RT_E_INVALID; }
    return rt_host::write_png(path, rgba, w, h);
}

} // extern "C"
