// path_kernel.hip — the megakernel variant of the render hot path (kernel 0)
// and the tonemap kernel.
//
// Replaces rt/path_tracing.cuh (kernel path_tracing :338-395, trace_path
// :268-325) and the reset_frame / draw_frame kernels of rt/render.cuh:18-59;
// the device arithmetic lives in rt_kernels.h.
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
//  * KD stack (node, entry t) in LDS, [depth][lane] => conflict-free.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include "bvh_trace.h"
#include "rt_kernels.h"

#define RT_BLOCK 256
#ifndef RT_MEGA_BVH_LDS
#define RT_MEGA_BVH_LDS 12 // bounded megakernel: stack entries in LDS; deeper ones spill to HBM
#endif
#ifndef RT_MEGA_BVH_WAVES
#define RT_MEGA_BVH_WAVES 6
#endif

using namespace rtk;

// path_tracing (rt/path_tracing.cuh:338-395) for `passes` passes, with
// reset_frame (rt/render.cuh:18-34) fused in when fr.reset is set.
// BOUNDED: the BVH-bounded traversal (bvh_trace.h), stack entries past STACK
// in `spill` (spill_threads entries apart, indexed by the global thread id)
template <bool COUNT, int STACK, bool BOUNDED>
__global__ void __launch_bounds__(RT_BLOCK, BOUNDED ? RT_MEGA_BVH_WAVES : (STACK <= RT_STACK_SMALL ? 4 : 2))
    rt_path_kernel(RtDevScene sc, RtDevFrame fr, RtDevCamera cam, uint2 *spill, int spill_threads)
{
    __shared__ uint32_t s_node[STACK * RT_BLOCK];
    __shared__ float s_entry[STACK * RT_BLOCK];
    const int tid = threadIdx.x;
    const int tiles_x = (fr.width + 15) / 16;
    const int tile = xcd_tile(blockIdx.x, gridDim.x);
    const int wave = tid >> 6, lane = tid & 63;
    const int x = (tile % tiles_x) * 16 + (wave & 1) * 8 + (lane & 7);
    const int y = (tile / tiles_x) * 16 + (wave >> 1) * 8 + (lane >> 3);
    const bool valid = x < fr.width && y < fr.height && rt_row_owned(fr, y);
    const int pi = valid ? y * fr.width + x : 0;
    Stack<STACK> stk{s_node + tid, s_entry + tid, RT_BLOCK,
                     BOUNDED ? spill + (size_t)blockIdx.x * RT_BLOCK + tid : nullptr, spill_threads};

    Cnt c;
    unsigned long long t_start = 0;
    if (COUNT) {
        c.zero();
        t_start = realtime();
    }

    uint32_t rng = 0;
    Vec3D fb = rt_v3(0.0f, 0.0f, 0.0f);
    float sq = 0.0f;
    int count = 0;
    if (valid) {
        rng = fr.rng[pi];
        if (!fr.reset) {
            fb = fr.fb[pi];
            sq = fr.sq[pi];
            count = fr.count[pi];
        }
    }

    int passes_left = valid ? fr.passes : 0;
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
                if (!adaptive_run(fr, fb, sq, count)) {
                    if (COUNT) c.v[RT_CNT_SKIP]++;
                    continue;
                }
                camera_ray(fr, cam, x, y, rng, ro, rd);
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
            dev_record_cut(fr);
            finish = true;
        } else {
            if (!shadow) ++depth;
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            const int hit = BOUNDED ? trace_bvh<false>(sc, ro, rd, bx, by, bz, stk, c)
                                    : trace<COUNT>(sc, ro, rd, bx, by, bz, stk, c);
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
                            rp = light_point(sc, light, rng);
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
                if (hit >= 0 && hit == light) direct = light_contribution(sc, light, bx, by, bz, ro, rd, rp, sn_normal);
                if (COUNT && hit >= 0 && material_of(sc, hit).tex) c.v[RT_CNT_TEXEL] += 2; // every hit is shaded
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
            if (COUNT) c.path_end(depth);
            dev_record_end(fr, depth);
            fb = fb + L;
            sq = sq + rt_square(rt_luminance(L));
            ++count;
            have_path = false;
        }
    }

    if (valid) {
        fr.fb[pi] = fb;
        fr.sq[pi] = sq;
        fr.count[pi] = count;
        fr.rng[pi] = rng;
    }
    if (COUNT) {
        flush_counters(c, fr.counters);
        if (fr.wave_times && lane == 0) {
            const size_t w = (size_t)blockIdx.x * (RT_BLOCK / 64) + wave;
            fr.wave_times[2 * w] = t_start;
            fr.wave_times[2 * w + 1] = realtime();
        }
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
namespace {
// Per-device spill area of the bounded megakernel (grown on demand), indexed
// by global thread id: one launch at a time may use it.  Launches are
// serialised on it — each waits (on its stream) for the previous launch's
// event, whatever stream that was on — and the buffer is replaced only after
// that launch is done, all under the mutex until the launch is enqueued.
struct MegaSpill {
    uint2 *buf = nullptr;
    size_t entries = 0;
    hipEvent_t last = nullptr; // after the last launch that used buf
    bool recorded = false;
};
std::mutex g_spill_mu;
std::map<int, MegaSpill> g_spill;
} // namespace

void rt_path_shutdown()
{
    std::lock_guard<std::mutex> g(g_spill_mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto &kv : g_spill) {
        if (hipSetDevice(kv.first) != hipSuccess) continue;
        if (kv.second.recorded) (void)hipEventSynchronize(kv.second.last);
        if (kv.second.buf) (void)hipFree(kv.second.buf);
        if (kv.second.last) (void)hipEventDestroy(kv.second.last);
    }
    g_spill.clear();
    (void)hipSetDevice(cur);
}

int rt_launch_path(const RtDevScene &sc, const RtDevFrame &fr, const RtDevCamera &cam, int stack_depth,
                   hipStream_t stream, int traversal)
{
    const int tiles = ((fr.width + 15) / 16) * ((fr.height + 15) / 16);
    dim3 grid(tiles), block(RT_BLOCK);
    const bool count = fr.counters != nullptr;
    if (!count && traversal == RT_TRAVERSAL_BOUNDED && sc.bvh_nodes != nullptr) {
        // the bounded traversal: the KD part needs <= RT_STACK_DEPTH entries, the BVH part <= RT_BVH_STACK
        const size_t threads = (size_t)tiles * RT_BLOCK;
        const int deeper = (RT_BVH_STACK > RT_STACK_DEPTH ? RT_BVH_STACK : RT_STACK_DEPTH) - RT_MEGA_BVH_LDS;
        const size_t entries = threads * (size_t)deeper;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return -1;
        std::lock_guard<std::mutex> g(g_spill_mu);
        MegaSpill &m = g_spill[dev];
        if (!m.last && hipEventCreateWithFlags(&m.last, hipEventDisableTiming) != hipSuccess) return -1;
        if (m.entries < entries) {
            if (m.recorded && hipEventSynchronize(m.last) != hipSuccess) return -1; // the old buffer's last user
            if (m.buf) (void)hipFree(m.buf);
            m.buf = nullptr;
            m.entries = 0;
            void *p = nullptr;
            if (hipMalloc(&p, entries * sizeof(uint2)) != hipSuccess) return -1;
            m.buf = (uint2 *)p;
            m.entries = entries;
        } else if (m.recorded && hipStreamWaitEvent(stream, m.last, 0) != hipSuccess) {
            return -1; // the previous launch (maybe on another stream) leaves the spill slots first
        }
        hipLaunchKernelGGL((rt_path_kernel<false, RT_MEGA_BVH_LDS, true>), grid, block, 0, stream, sc, fr, cam, m.buf,
                           (int)threads);
        if (hipGetLastError() != hipSuccess || hipEventRecord(m.last, stream) != hipSuccess) return -1;
        m.recorded = true;
        return 0;
    }
    if (stack_depth <= RT_STACK_SMALL) {
        if (count)
            hipLaunchKernelGGL((rt_path_kernel<true, RT_STACK_SMALL, false>), grid, block, 0, stream, sc, fr, cam,
                               nullptr, 0);
        else
            hipLaunchKernelGGL((rt_path_kernel<false, RT_STACK_SMALL, false>), grid, block, 0, stream, sc, fr, cam,
                               nullptr, 0);
    } else {
        if (count)
            hipLaunchKernelGGL((rt_path_kernel<true, RT_STACK_DEPTH, false>), grid, block, 0, stream, sc, fr, cam,
                               nullptr, 0);
        else
            hipLaunchKernelGGL((rt_path_kernel<false, RT_STACK_DEPTH, false>), grid, block, 0, stream, sc, fr, cam,
                               nullptr, 0);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int rt_launch_tonemap(const Vec3D *fb, const int *count, RtUChar4 *out, int n, hipStream_t stream)
{
    hipLaunchKernelGGL(rt_tonemap_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, fb, count, out, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
