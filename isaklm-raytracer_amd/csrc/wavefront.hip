// wavefront.hip — the wavefront variant of the render hot path (kernel 1).
//
// The per-pixel loop of rt/path_tracing.cuh:268-325 is cut at its ray
// queries.  Each iteration runs two kernels over a compacted queue of rays:
//   wf_trace  — trace_ray (rt/trace_ray.cuh:244-318) for every queued ray;
//               nothing else, so it is small (VGPRs) and keeps more waves in
//               flight to hide the dependent node/triangle loads
//   wf_shade  — consumes each hit: emission, BSDF sample, NEE shadow-ray set
//               up, roulette, accumulation, and starts the pixel's next pass
//               (adaptive test + camera ray) when its path ends; appends the
//               next ray of every live path to the other queue
// Path state lives in HBM between kernels (SoA, ~72 B per pixel).  Queue
// order is arbitrary (wave-aggregated atomics) but every pixel's sequence of
// events is the reference's, so results are bit-identical to the megakernel
// and the CPU oracle.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "bvh_trace.h"
#include "rt_kernels.h"

using namespace rtk;

#define WF_BLOCK 256
#ifndef WF_TBLOCK
#define WF_TBLOCK 256 // threads per block of the queue kernels (wf_trace_coop, wf_shade)
#endif
// tgrid * WF_TBLOCK == grid * WF_BLOCK threads: the spill area (sized for
// grid * WF_BLOCK threads, indexed by the global thread id) must cover them
static_assert(WF_BLOCK % WF_TBLOCK == 0 && WF_TBLOCK % 64 == 0, "WF_TBLOCK must divide WF_BLOCK in whole waves");
// wave priorities beside the other pipelines' trace waves (A/B, 4 rounds:
// -1 % call time together): a pipeline's shade launch and the tail of its
// trace launch are on its critical path, the other launches' bulk is not
#ifndef WF_SHADE_PRIO
#define WF_SHADE_PRIO 3
#endif
// wf_shade runs in the slots its pipeline's trace launch just left, beside
// the other pipelines' trace waves (80 VGPRs each): at the same footprint
// (6 waves/SIMD, the rest of its ~126 VGPRs spilled) its waves fit those
// holes.  Measured (room2m 1080p, 256 passes/call, 3 rounds, s per call):
// 13.83 at 126 VGPRs, 13.58 at 96, 13.21 at 80, 13.21 at 72, 13.31 at 64
// (and 13.60 for the earlier 102-VGPR build that kept its path state in scratch)
#ifndef WF_SHADE_WAVES
#define WF_SHADE_WAVES 6
#endif
// wf_long, too, runs beside the pipelines' trace waves: at their footprint
// (80 VGPRs, ~85 spilled) its waves fit the slots a trace block leaves.
// Measured (as WF_SHADE_WAVES): 13.16 s at 126 VGPRs, 13.16 at 128 (4
// waves), 12.87 at 80, 12.86 at 72, 12.92 at 64
#ifndef WF_LONG_WAVES
#define WF_LONG_WAVES 5
#endif
#ifndef WF_LONG_PRIO
// wf_long wave priority: a deep path's bounce chain is the call's critical
// path, and in the whole-call mode its wave shares a CU with ~24 finisher
// waves; s_setprio 3 wins it the issue arbitration.  Per 256-pass room2m call
// (5 calls x 2 rounds, tools/gpu_ab_libs5.sh): 6.93 / 6.96 s vs 7.34 / 7.80 s
// for 5 calls at priority 0 (-5.6 % / -11 %)
#define WF_LONG_PRIO 3
#endif
#ifndef WF_FIN_LINGER
#define WF_FIN_LINGER 100000000ull // s_memrealtime ticks (100 MHz): 1 s
#endif
#ifndef WF_FIN_LINGER_WAVES
#define WF_FIN_LINGER_WAVES 256u // finisher waves that linger for returned pixels
#endif
#ifndef WF_HEAVY_FIRST
#define WF_HEAVY_FIRST 1 // whole-call finisher: pixels whose paths went to wf_long before start the call
#endif
#define WF_HEAVY_BLOCKS 256
#ifndef WF_HEAVY_SPLIT
#define WF_HEAVY_SPLIT 4 // hand-offs that put a pixel in the first class (1: one class)
#endif
#ifndef WF_FIN_QUIET_TRIPS
#define WF_FIN_QUIET_TRIPS 4096u // ... while wf_long ran a path within this many of their idle loop trips
#endif
#define WF_FIN_LINGER_TRIPS 1000000u // ... and for at most this many idle loop trips in all (a bound that holds
                                     // where s_memrealtime stands still: rocprofv3 counter collection)
#ifndef WF_FIN_OCC
#define WF_FIN_OCC 1 // wf_finish_coop occupancy floor (1: the compiler's choice, 2 waves/SIMD; 3: no change)
#endif
#ifndef WF_TAIL_PRIO
#define WF_TAIL_PRIO 2
#endif
#ifndef WF_LDS_STACK
#define WF_LDS_STACK 8  // stack entries in LDS; deeper ones spill to HBM (rare)
#endif
#ifndef WF_TRACE_WAVES
#define WF_TRACE_WAVES 6 // wf_trace_coop occupancy target (blocks of 4 waves per CU = waves per SIMD)
#endif
#ifndef WF_BVH_LDS
#define WF_BVH_LDS 10   // wf_finish_bvh / wf_trace_bvh: stack entries in LDS (BVH query and KD descent share the
                        // stack; deeper entries go to the HBM spill area).  10 (34.8 KB per block: 4 finisher blocks
                        // and a wf_long block fit a CU's 160 KB) vs 8 / 9: 745-748 vs 735-738 / 735-742 Msamples/s
                        // (round 6, profiles/r06/ab/ ab19); 12 left no room for the wf_long block (-9 %)
#endif
#ifndef WF_BVH_WAVES
#define WF_BVH_WAVES 6  // wf_trace_bvh occupancy target
#endif
#ifndef WF_CHECK_BLOCKS
#define WF_CHECK_BLOCKS 256 // wf_check's grid (it runs beside the next call's finisher)
#endif
#ifndef WF_BVH_PARK
#define WF_BVH_PARK 6 // wf_finish_bvh: BVH node steps per loop trip before a lane's query parks (0: never; re-swept
                      // after round 6's VALU cuts: 4 / 5 / 6 / 7 / 8 / 12 / 16 = 723-727 / 733 / 738-742 / 739-741 /
                      // 712-731 / 715 / 699-700 Msamples/s, profiles/r06/ab/ ab16-ab17)
#endif
#ifndef WF_FIN_BVH_WAVES
#define WF_FIN_BVH_WAVES 4 // wf_finish_bvh occupancy target: 4 waves/SIMD (128 VGPRs, 29 spilled) run the bench at
                           // 5's rate (566.8-572.2 vs 562.8-573.1 Msamples/s, round 6) with a third of its HBM traffic
                           // for spills: 107 vs 324 GB written and 908 vs 1,350 GB fetched per 256-pass call
                           // (profiles/r06/bench_w4_pmc.json); 6: -9 %.  (Round 5 kept 5 because 4's counter passes
                           // hung: that was wf_long's start race, fixed in round 6, not the occupancy)
#endif
// (chained calls' finishers run one after the other on pipeline 0: a kernel boundary between calls,
// which a pixel's state crosses for free.  The round-5 variants — a finisher going on with the next
// issued call, finishers alternating between two streams — measured slower, one of them inexact,
// and are gone: DESIGN.md §6 keeps their A/B records)
#ifndef WF_NEE_LDS
#define WF_NEE_LDS 1 // wf_finish_bvh keeps a NEE set-up's state in LDS (PathRegsL), not in registers: at 4 waves/SIMD
                     // 8 VGPRs spilled instead of 30, 64 instead of 107 GB written per 256-pass call, the bench
                     // unchanged (569.5 vs 569.3; profiles/r06/bench_nee_lds_pmc.json)
#endif
#ifndef WF_FIN_SMALL_WAVES
#define WF_FIN_SMALL_WAVES 3 // frames of at most this many finisher waves per SIMD take the unspilled build (151 VGPRs: 3 waves)
#endif
// per-thread spill entries: the deeper of the KD stack (past WF_LDS_STACK) and the BVH stack (past WF_BVH_LDS)
#define WF_SPILL_ENTRIES \
    ((RT_STACK_DEPTH - WF_LDS_STACK) > (RT_BVH_STACK - WF_BVH_LDS) ? (RT_STACK_DEPTH - WF_LDS_STACK) \
                                                                    : (RT_BVH_STACK - WF_BVH_LDS))
#define WF_TAIL_DEFAULT 65536u       // RtOptions.wf_tail
#define WF_FINISH_WAVES_DEFAULT 2048u // RtOptions.wf_finish_waves
#define WF_FINISH_WAVES_SMALL 512u    // ... for trees below WF_FIN_WIDE_MIN_ENTRIES leaf entries
#define WF_DESCENT_CAP_DEFAULT 5      // RtOptions.wf_descent_cap
#define WF_POSTPONE_DEFAULT 20        // RtOptions.wf_postpone
#define WF_TIMELINE_LAUNCHES 4096     // debug timeline: 3 u64 per trace launch in RtOptions.wave_times_device
#define WF_WIDE_TAIL_LANES 32         // RtOptions.wf_wide > 0
#define WF_FIN_WIDE_MIN_ENTRIES (1 << 18) // finisher: multi-ray wide tracing only for trees with this many leaf entries
#define WF_MAX_PIPES 6                // concurrent pipelines (RtOptions.wf_pipelines); more than 3 need GPU_MAX_HW_QUEUES > 4
#define WF_PIPES_DEFAULT 3
#ifndef WF_LONG_DEPTH_DEFAULT
#define WF_LONG_DEPTH_DEFAULT 64      // RtOptions.wf_long_depth: paths deeper than this go to wf_long
#endif
#define WF_LONG_DEPTH_MIN 16          // ... smaller values are raised to this (profiles/r05/small_calls/long_depth_sweep)
#define WF_COALESCE_DEFAULT 256       // RtOptions.coalesce_passes: chained calls are coalesced up to this many passes
#ifndef WF_LONG_BLOCKS
#define WF_LONG_BLOCKS 64 // wf_long grid (4 waves each, one path per wave at a time)
#endif
// Cross-kernel waits (finisher <-> wf_long).  No kernel may wait for work of
// a kernel that is not resident: under rocprofv3 counter collection the
// dispatches are serialised (either kernel may run first, alone), and a shared
// chip may delay either one.  So every such wait is bounded by a count of the
// waiting loop's trips — s_memrealtime stands still under counter collection
// (ae07d5e), so the clock bounds below are a second, faster exit, never the
// only one — and a bound that expires leaves the protocol in a state the
// other side completes on its own:
//  * wf_long waits for its call's finisher only once a finisher wave has
//    started (WF_FIN_STARTED).  Before that it waits at most
//    WF_LONG_START_TRIPS idle trips, then CLOSES the hand-off ring
//    (WF_LONG_CLOSED in the reserved counter, set only while every reserved
//    entry is claimed) and leaves: the finisher's hand-offs then fail and its
//    lanes run their deep paths to the end themselves (the same shade_step
//    sequence: bit-identical).  The ring stays closed until the next call
//    that does not continue a chain resets it (RT_DEV_LONG_CLOSED counts it);
//  * a finisher lingers for pixels out in wf_long at most WF_FIN_QUIET_TRIPS
//    trips while no wf_long wave runs a path, and at most st.linger ticks;
//  * a finisher claims a return wf_long reserved only while wf_long is
//    resident (it reserves while running); its wait for the entry's
//    publication is bounded by WF_SPIN_TRIPS (expired: the pixel is left out,
//    found by wf_verify, RT_E_INCOMPLETE);
//  * the safety nets of wf_long's claim loop, never reached by a working
//    protocol: an entry reserved but never published (WF_LONG_PUBLISH_TRIPS /
//    _WAIT) and nothing left that could bring work (WF_LONG_IDLE_TRIPS /
//    WF_LONG_IDLE).  A net exit with entries unclaimed strands pixels instead
//    of hanging the GPU — counted (RT_DEV_LONG_QUIT), found by the join's
//    wf_verify and reported.
// (A trip of these loops is an s_sleep plus 2-4 L2 atomics: ~1-2 us.)
#define WF_FIN_STARTED 0x80000000u        // fin_live: a finisher wave of the call has started
#define WF_LONG_CLOSED 0x80000000u        // long_ctr[0]: the ring takes no more hand-offs
#define WF_LONG_START_TRIPS 20000u        // idle trips before wf_long closes the ring on an unstarted finisher
#define WF_LONG_IDLE 200000000ull         // 2 s idle with nothing that could still bring work
#define WF_LONG_IDLE_TRIPS 2000000u       // ... or this many trips
#define WF_LONG_PUBLISH_WAIT 100000000ull // 1 s on one reserved, unpublished entry (publication is ~1 us)
#define WF_LONG_PUBLISH_TRIPS 1000000u    // ... or this many trips
#define WF_SPIN_TRIPS (1u << 24)          // a finisher lane's wait for a reserved return's publication
// an idle persistent wf_long wave of an open chain stays until no entry has
// been reserved (for any wave) for this long (50 ms, or WF_LONG_CHAIN_TRIPS
// trips) AND no wave runs a path: the next calls' deep paths
// (WfState.chain_flag).  The grid leaves as a whole — one whose idle waves
// left while a few ran 10^4-bounce samples on (a call's tail can go 50 ms
// without a hand-off) served the next calls with those few waves, its
// stream-queued successor blocked behind them.
#define WF_LONG_CHAIN_IDLE 5000000ull
#define WF_LONG_CHAIN_TRIPS 50000u
// RtOptions.check_interval: 1 ray in this many re-traced by the KD traversal
// (a KD re-trace costs ~50 bounded queries: 1024 took 4 % of a 256-pass
// room2m call, 4096 ~1 %, and still checks ~2M rays in the 20-step bench)
#define WF_CHECK_INTERVAL_DEFAULT 4096u
#define WF_CHECK_CAP (1u << 22)         // cross-check records per launch (more are dropped: RT_DEV_CHK_DROP;
                                        // a chained launch may run several calls' pixels)
// per-pixel ownership word (WfState.pxo) of the whole-call render: a pixel is
// BUSY while a finisher lane runs its passes and OUT while wf_long holds it
// (handed over, or in the return ring), until a finisher lane takes it back or
// wf_long finishes it.  A call that finds its pixel held adds its passes to
// the low bits (owed) and moves on; the holder runs them, in the pixel's order,
// before it lets go.  Free: 0, or REL when the last holder may run concurrently
// with the next one (a chained finisher, wf_long): its stores were released
// before the word said so, and the next claimer acquires first.
#define RT_PX_OUT 0x80000000u
#define RT_PX_REL 0x40000000u
#define RT_PX_LONGDONE RT_PX_REL
#define RT_PX_BUSY 0x20000000u
#define RT_PX_PASSES 0x1FFFFFFFu

struct WfState {
    int *passes_left;
    uint32_t *flags;   // bit0 shadow, bit1 inside, bits 2..4 prev_type, bit5 dual, bit6 ext_live, bits 8.. depth
    Vec3D *T, *L, *cont, *snorm, *rp;
    Vec3D *ro;         // origin of the path's pending ray(s); cont = the pending extension direction
    uint32_t *e_sh, *e_ext; // queue entries of the path's pending shadow / extension ray
    int *light;
    uint32_t *q_slot[2]; // path lists: the pixels (slots) with rays in ray queue q
    RtF4 *q_ray[2];    // ray queues, 2 RtF4 per entry: {o.xyz, -}, {d.xyz, -}
    RtF4 *hits;        // per ray-queue entry: {tri bits, bx, by, bz}
    uint32_t *counts;  // [0], [1]: ray queue sizes; [2], [3]: fetch cursors; [4] finisher fetch; [6], [7]: path list sizes
    uint2 *spill;      // traversal stack spill
    int spill_threads;
    // long-path hand-off (wf_long): a path deeper than long_depth leaves its
    // pipeline for the concurrently running wf_long kernel through a ring of
    // long_cap entries: entry e (counted from the last reset) lives at e %
    // long_cap, published as long_ent = (e + 1) << 32 | slot after its ray
    uint32_t *long_ctr;   // [0] entries reserved (| WF_LONG_CLOSED), [1] entries claimed, [3] paths running in wf_long
    unsigned long long *long_ent;
    RtF4 *long_ray;       // 2 per ring slot
    int long_depth;       // 0 = off
    uint32_t long_cap;    // ring slots (the pixels)
    // whole-call finisher (bounded traversal): wf_long runs a handed-over path
    // only to the end of its SAMPLE and returns the pixel through this ring to
    // the finishers, whose lanes run its remaining passes
    int long_return;
    unsigned long long *ret_ring; // entry e at e % long_cap: (e + 1) << 32 | slot once published
    unsigned long long *long_log; // debug (RT_DEBUG_LONG_LOG): [0] call start, then per claim {claim, end, bounces, slot}
    // ret_ctr: u64 [0] = finisher waves alive << 32 | returns reserved (wf_long
    // reserves only while a finisher wave is alive; a wave leaves only when
    // every reserved return is claimed: no pixel is stranded.  The finisher
    // never waits for a wf_long that is not resident: returns are reserved by
    // a running wf_long wave, and lingering is bounded — see the cross-kernel
    // waits above);
    // u32 [2] = returns claimed, u32 [3] = pixels out (handed to wf_long, not
    // yet returned or done): an idle finisher wave lingers (s_sleep) while
    // pixels are out — for at most `linger` ticks (0 for chained calls, whose
    // successor takes the returns), so that it never depends on wf_long
    uint32_t *ret_ctr;
    unsigned long long linger;
    // per pixel: RT_PX_OUT / RT_PX_BUSY | passes owed by later chained calls, RT_PX_REL, or 0
    uint32_t *pxo;
    // heavy pixels first (whole-call finisher): a pixel whose path went to wf_long is marked
    // (heavy); before each call wf_heavy_list lists the marked pixels (heavy_list, count
    // heavy_n) and tags them with the call (listed): the finisher's first entries are those
    // pixels, and its tile entries skip a pixel listed for this call.  heavy_list == nullptr:
    // no list (the tiles only)
    uint8_t *heavy;
    uint32_t *listed, *heavy_list, *heavy_n;
    // the whole-call finisher takes this call's pixels itself (no wf_start, no path list): fresh = 1
    int fresh;
    uint32_t fresh_n; // (fresh) entries: 256 per 16x16-pixel tile (fresh_pixel); 0 for a chain's drain
    unsigned long long *span; // RtOptions.profile: {first wave start, last wave end} (s_memrealtime)
    uint32_t call_id; // this launch's call (heavy-pixel list tags)
    // the persistent wf_long's producers: the host sets the word to the finisher's wave count;
    // each finisher wave sets WF_FIN_STARTED when it starts and subtracts 1 once past its last
    // hand-off (nullptr: wf_long runs in host-kicked slices).  wf_long waits for producers only
    // once one has started: a finisher not yet dispatched (counter collection serialises
    // dispatches) is never waited for
    uint32_t *fin_live;
    // 1 while a chain of calls is open (set by chained calls, cleared by its
    // drain): an idle persistent wf_long wave then stays up to WF_LONG_CHAIN_IDLE
    // for the later calls' deep paths instead of leaving at its first idle
    // moment (which left the next calls' entries to the few waves still busy,
    // the stream-queued successor blocked behind them).  Bounded: the drain's
    // clear may sit behind this very wf_long when streams share a hardware queue.
    uint32_t *chain_flag;
    // run-time exactness guard of the bounded traversal: the finisher records
    // every ray whose hash of (pixel, pass, depth, kind) hits chk_mask (3 RtF4:
    // {o, hit bits}, {d, bx}, {by, bz, -, -}); wf_check re-traces them with the
    // plain KD traversal (nullptr: off)
    RtF4 *chk;
    uint32_t *chk_ctr;
    uint32_t chk_mask;
    uint32_t chk_cap; // records per parity (more are dropped: RT_DEV_CHK_DROP)
    int chk_fault; // (RT_DEBUG_CHECK_FAULT, tests: record a wrong result for every checked ray)
    int debug_quit; // (RT_DEBUG_LONG_QUIT, tests: wf_long leaves at once, as by its safety net)
};

namespace {

__device__ __forceinline__ uint32_t lanemask_lt() { return (uint32_t)__lane_id(); }

// wave-aggregated append of `want` lanes to the list counted by *ctr: returns
// each wanting lane's index
__device__ __forceinline__ uint32_t wave_append(uint32_t *ctr, bool want)
{
    const unsigned long long mask = __ballot(want);
    if (mask == 0) return 0;
    const int lane = __lane_id();
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(mask));
    base = __shfl(base, leader);
    return base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
}

// append `want` lanes' rays to ray queue q; returns the entry
__device__ __forceinline__ uint32_t enqueue_ray(const WfState &st, int q, bool want, Vec3D o, Vec3D d)
{
    const uint32_t e = wave_append(st.counts + q, want);
    if (want) {
        st.q_ray[q][2 * (size_t)e] = RtF4{o.x, o.y, o.z, 0.0f};
        st.q_ray[q][2 * (size_t)e + 1] = RtF4{d.x, d.y, d.z, 0.0f};
    }
    return e;
}

// append `want` lanes' paths to path list q
__device__ __forceinline__ void enqueue_path(const WfState &st, int q, bool want, uint32_t slot)
{
    const uint32_t i = wave_append(st.counts + 6 + q, want);
    if (want) st.q_slot[q][i] = slot;
}

// publish ring entry e of the long-path hand-off: the ray, then (after this
// wave's stores are drained and released: the XCD's L2 written back,
// MI355X_MICROARCH.md hand-off rules) the tag wf_long's claims check
__device__ __forceinline__ void long_publish(const WfState &st, bool to_long, uint32_t e, uint32_t slot, Vec3D o,
                                             Vec3D d)
{
    const uint32_t k = e % st.long_cap;
    if (to_long) {
        st.long_ray[2 * (size_t)k] = RtF4{o.x, o.y, o.z, 0.0f};
        st.long_ray[2 * (size_t)k + 1] = RtF4{d.x, d.y, d.z, 0.0f};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (to_long) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(st.long_ent + k, ((unsigned long long)(e + 1u) << 32) | slot, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
}

// hand `to_long` lanes' paths (state already stored) to wf_long (queue
// kernels: a pixel is handed over at most once per call, and the ring is
// reset per call, so its long_cap = pixels entries never wrap)
__device__ __forceinline__ void publish_long(const WfState &st, bool to_long, uint32_t slot, Vec3D o, Vec3D d)
{
    uint32_t e = 0;
    if (to_long) e = __hip_atomic_fetch_add(st.long_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long_publish(st, to_long, e, slot, o, d);
}

// the finisher's hand-off: as publish_long, but the wave reserves its entries
// with one compare-and-swap that never laps an unclaimed entry (a pixel can be
// handed over several times per call when wf_long returns it after each deep
// sample, and chained calls keep the ring running).  Returns false
// (wave-uniform) when the entries would not fit or the ring is closed: the
// lanes then keep their paths.  The path state is stored by the caller first; the pixel is OUT
// (pxo) from here until a finisher takes it back or wf_long finishes it.
__device__ __forceinline__ bool publish_long_capped(const WfState &st, bool to_long, uint32_t slot, Vec3D o, Vec3D d)
{
    const unsigned long long m = __ballot(to_long);
    const int lane = __lane_id();
    const int leader = __ffsll((long long)m) - 1;
    const uint32_t k = (uint32_t)__popcll(m);
    uint32_t base = 0xffffffffu;
    if (lane == leader) {
        uint32_t r = __hip_atomic_load(st.long_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (true) {
            const uint32_t c = __hip_atomic_load(st.long_ctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // closed (wf_long left: see WF_LONG_CLOSED), the count's 31 bits used up, or a lap of an
            // unclaimed entry (c may be stale-low: conservative): the lanes keep their paths
            if ((r & WF_LONG_CLOSED) || r + k >= WF_LONG_CLOSED || r + k - c > st.long_cap) break;
            if (__hip_atomic_compare_exchange_strong(st.long_ctr, &r, r + k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                base = r;
                break;
            }
        }
        if (base != 0xffffffffu && st.long_return) // out before the entries can be seen
            __hip_atomic_fetch_add(st.ret_ctr + 3, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    base = (uint32_t)__shfl((int)base, leader);
    if (base == 0xffffffffu) return false;
    const uint32_t e = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    // (BUSY -> OUT, owed passes kept: one atomic)
    if (to_long && st.long_return)
        __hip_atomic_fetch_xor(st.pxo + slot, RT_PX_OUT ^ RT_PX_BUSY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long_publish(st, to_long, e, slot, o, d);
    return true;
}

// start the pixel's next pass(es): adaptive test, camera ray.  Returns true
// (and the ray) when a sample starts.
template <bool COUNT>
__device__ __forceinline__ bool start_sample(const RtDevFrame &fr, const RtDevCamera &cam, int slot, int &passes_left,
                                             uint32_t &rng, Vec3D fb, float sq, int count, Vec3D &ro, Vec3D &rd,
                                             Cnt &c)
{
    while (passes_left > 0) {
        --passes_left;
        if (!adaptive_run(fr, fb, sq, count)) {
            if (COUNT) c.v[RT_CNT_SKIP]++;
            continue;
        }
        camera_ray(fr, cam, slot % fr.width, slot / fr.width, rng, ro, rd);
        if (COUNT) c.v[RT_CNT_SAMPLE]++;
        return true;
    }
    return false;
}

} // namespace

template <bool COUNT>
__global__ void __launch_bounds__(WF_BLOCK) wf_start(RtDevFrame fr, RtDevCamera cam, WfState st, int pipe,
                                                     int npipes)
{
    Cnt c;
    if (COUNT) c.zero();
    const int n = fr.width * fr.height;
    const int tile = xcd_tile(blockIdx.x, gridDim.x);
    if (tile % npipes != pipe) return; // another pipeline's 16x16 tile (block-uniform)
    const int tiles_x = (fr.width + 15) / 16;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int x = (tile % tiles_x) * 16 + (wave & 1) * 8 + (lane & 7);
    const int y = (tile / tiles_x) * 16 + (wave >> 1) * 8 + (lane >> 3);
    const bool valid = x < fr.width && y < fr.height && rt_row_owned(fr, y);
    const int slot = valid ? y * fr.width + x : 0;
    bool want = false;
    Vec3D ro = rt_v3(0, 0, 0), rd = rt_v3(0, 0, 0);
    if (valid && slot < n) {
        Vec3D fb = rt_v3(0.0f, 0.0f, 0.0f);
        float sq = 0.0f;
        int count = 0;
        if (fr.reset) {
            fr.fb[slot] = fb;
            fr.sq[slot] = sq;
            fr.count[slot] = count;
        } else {
            fb = fr.fb[slot];
            sq = fr.sq[slot];
            count = fr.count[slot];
        }
        int passes_left = fr.passes;
        uint32_t rng = fr.rng[slot];
        want = start_sample<COUNT>(fr, cam, slot, passes_left, rng, fb, sq, count, ro, rd, c);
        fr.rng[slot] = rng;
        st.passes_left[slot] = passes_left;
        st.flags[slot] = 1u << 8; // depth 1 (first extension ray), prev PRIMARY
        st.T[slot] = rt_v3(1.0f, 1.0f, 1.0f);
        st.L[slot] = rt_v3(0.0f, 0.0f, 0.0f);
        st.ro[slot] = ro;
        st.cont[slot] = rd;
    }
    const uint32_t e = enqueue_ray(st, 0, want, ro, rd);
    if (want) st.e_ext[slot] = e;
    enqueue_path(st, 0, want, (uint32_t)slot);
    if (COUNT) flush_counters(c, fr.counters);
}

template <bool COUNT>
__global__ void __launch_bounds__(WF_BLOCK) wf_trace(RtDevScene sc, WfState st, int q, unsigned long long *counters)
{
    __shared__ uint32_t s_node[WF_LDS_STACK * WF_BLOCK];
    __shared__ float s_entry[WF_LDS_STACK * WF_BLOCK];
    const int tid = threadIdx.x;
    const int gtid = blockIdx.x * WF_BLOCK + tid;
    Stack<WF_LDS_STACK> stk{s_node + tid, s_entry + tid, WF_BLOCK, st.spill + gtid, st.spill_threads};
    Cnt c;
    if (COUNT) c.zero();
    const uint32_t n = st.counts[q];
    const RtF4 *rays = st.q_ray[q];
    for (uint32_t base = blockIdx.x * WF_BLOCK; base < n; base += gridDim.x * WF_BLOCK) {
        const uint32_t e = base + tid;
        if (e < n) {
            const RtF4 o4 = ldf4(rays + 2 * (size_t)e), d4 = ldf4(rays + 2 * (size_t)e + 1);
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            const int hit = trace<COUNT>(sc, ld3(o4), ld3(d4), bx, by, bz, stk, c);
            *reinterpret_cast<float4 *>(st.hits + e) = make_float4(__int_as_float(hit), bx, by, bz);
        }
    }
    if (COUNT) flush_counters(c, counters);
}

// trace_ray bounded by the conservative BVH (bvh_trace.h): one ray per lane,
// lanes refill from the queue (one wave-aggregated atomic per refill round)
// so a wave is not held by its slowest ray's successors
template <bool COUNT>
__global__ void __launch_bounds__(WF_BLOCK, WF_BVH_WAVES) wf_trace_bvh(RtDevScene sc, WfState st, int q,
                                                                      unsigned long long *counters)
{
    Cnt c;
    if (COUNT) c.zero();
    __shared__ uint32_t s_node[WF_BVH_LDS * WF_BLOCK];
    __shared__ float s_entry[WF_BVH_LDS * WF_BLOCK];
    const int tid = threadIdx.x;
    const int gtid = blockIdx.x * WF_BLOCK + tid;
    Stack<WF_BVH_LDS> stk{s_node + tid, s_entry + tid, WF_BLOCK, st.spill + gtid, st.spill_threads};
    const uint32_t n = st.counts[q];
    const RtF4 *rays = st.q_ray[q];
    uint32_t *fetch = st.counts + 2 + q;
    const int lane = __lane_id();
    while (true) {
        const unsigned long long m = __ballot(true);
        const int leader = __ffsll((long long)m) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(fetch, (uint32_t)__popcll(m));
        base = __shfl(base, leader);
        const uint32_t e = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (e >= n) break;
        const RtF4 o4 = ldf4(rays + 2 * (size_t)e), d4 = ldf4(rays + 2 * (size_t)e + 1);
        float bx = 0.0f, by = 0.0f, bz = 0.0f;
        const int hit = trace_bvh<COUNT>(sc, ld3(o4), ld3(d4), bx, by, bz, stk, c);
        *reinterpret_cast<float4 *>(st.hits + e) = make_float4(__int_as_float(hit), bx, by, bz);
    }
    if (COUNT) flush_counters(c, counters);
}

// trace_bvh (bvh_trace.h) with dynamic ray fetch: every lane runs its own ray
// through the same steps — the s_min query over the 4-wide BVH, then the
// bounded KD phase — but a round advances each lane by at most `cap` node
// steps of its current phase and one leaf, and a lane whose ray is done takes
// the next queued ray at the start of the next round (Aila & Laine's
// persistent while-while with per-lane refill), so a wave is not held for its
// slowest ray.  Same per-ray arithmetic and visiting order as trace_bvh: the
// same hits, bit for bit.  (Rays that lie in a KD split plane — zero direction
// components — take the plain KD traversal, as in trace_bvh: s_min = -inf.)
#ifndef WF_DYN_WAVES
#define WF_DYN_WAVES 6
#endif
#ifndef WF_BVH_DYN
#define WF_BVH_DYN 1 // the queue path's bounded trace launches: per-lane refill (0: wf_trace_bvh, lockstep rays)
#endif
#ifndef WF_BVH_DYN_CAP
#define WF_BVH_DYN_CAP 8 // node steps per phase per round
#endif
template <bool COUNT>
__global__ void __launch_bounds__(WF_BLOCK, WF_DYN_WAVES) wf_trace_bvh_dyn(RtDevScene sc, WfState st, int q,
                                                                          unsigned long long *counters, int cap)
{
    Cnt c;
    if (COUNT) c.zero();
    __shared__ uint32_t s_node[WF_BVH_LDS * WF_BLOCK];
    __shared__ float s_entry[WF_BVH_LDS * WF_BLOCK];
    const int tid = threadIdx.x;
    const int gtid = blockIdx.x * WF_BLOCK + tid;
    Stack<WF_BVH_LDS> stk{s_node + tid, s_entry + tid, WF_BLOCK, st.spill + gtid, st.spill_threads};
    const uint32_t n = st.counts[q];
    const RtF4 *rays = st.q_ray[q];
    uint32_t *fetch = st.counts + 2 + q;
    const int lane = __lane_id();
    // per lane: 0 no ray, 1 s_min query (cur: BVH4 reference), 2 KD phase (node, nd: its words once loaded)
    int phase = 0;
    bool exhausted = false;
    uint32_t e = 0, cur = 0, node = 0;
    uint2 nd = make_uint2(0u, 0u);
    bool nd_ok = false; // nd holds node's words
    int sp = 0;
    Vec3D o = rt_v3(0, 0, 0), d = rt_v3(0, 0, 0);
    RtSlab sl{rt_v3(0, 0, 0), rt_v3(0, 0, 0), rt_v3(0, 0, 0)};
    float best = 0.0f, entry = 0.0f, exit_ = 0.0f, root_exit = 0.0f, s_min = 0.0f;
    while (true) {
        // ---- refill: lanes without a ray take the next queued one
        const bool need = phase == 0 && !exhausted;
        const unsigned long long mm = __ballot(need);
        if (mm) {
            const int leader = __ffsll((long long)mm) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(fetch, (uint32_t)__popcll(mm));
            base = __shfl(base, leader);
            if (need) {
                e = base + (uint32_t)__popcll(mm & ((1ull << lane) - 1ull));
                if (e >= n) {
                    exhausted = true;
                } else {
                    o = ld3(ldf4(rays + 2 * (size_t)e));
                    d = ld3(ldf4(rays + 2 * (size_t)e + 1));
                    if (COUNT) c.v[RT_CNT_RAY]++;
                    if (!bbox_hit(sc, o, d, entry, exit_)) {
                        *reinterpret_cast<float4 *>(st.hits + e) = miss_record();
                    } else {
                        root_exit = exit_;
                        sp = 0;
                        if (rt_bounded_ray(o, d, sc.split_vals, sc.split_off)) {
                            phase = 1;
                            sl = rt_slab(o, d, rt_ray_margin(o.x, o.y, o.z, sc.bvh_scale));
                            best = exit_;
                            cur = 0;
                        } else {
                            phase = 2; // the plain KD traversal
                            s_min = -INFINITY;
                            node = 0;
                            nd_ok = false;
                        }
                    }
                }
            }
        }
        if (!__any(phase != 0)) {
            if (__all(exhausted)) break;
            continue;
        }
        // ---- s_min query: up to `cap` inner nodes, then a leaf (bvh4_bound)
        for (int i = 0; i < cap; ++i) {
            const bool step = phase == 1 && !(cur & RT_BVH_LEAF);
            if (!__any(step)) break;
            if (step) {
                if (COUNT) c.v[RT_CNT_B_BVH_NODE]++;
                const uint32_t next = bvh4_children(sc, cur, sl, best, stk, sp);
                if (next != RT_BVH_EMPTY) {
                    cur = next;
                } else { // pop the next subtree that may still hold a smaller s
                    cur = RT_BVH_EMPTY;
                    while (sp > 0) {
                        uint32_t nn;
                        float tn;
                        stk.get(--sp, nn, tn);
                        if (tn <= best) {
                            cur = nn;
                            break;
                        }
                    }
                }
            }
        }
        // (cur == RT_BVH_EMPTY carries the leaf bit: such a lane is done with the query)
        const bool bleaf = phase == 1 && (cur & RT_BVH_LEAF) && cur != RT_BVH_EMPTY;
        if (__any(bleaf) && bleaf) {
            const uint32_t first = (cur & ~RT_BVH_LEAF) >> 3, end = first + (cur & 7u) + 1u;
            if (COUNT) c.v[RT_CNT_B_BVH_TRI] += end - first;
            float bx, by, bz;
            (void)leaf_scan<COUNT>(sc.bvh_a, sc.bvh_bary, first, end, o, d, best, bx, by, bz, c);
            cur = RT_BVH_EMPTY;
            while (sp > 0) {
                uint32_t nn;
                float tn;
                stk.get(--sp, nn, tn);
                if (tn <= best) {
                    cur = nn;
                    break;
                }
            }
        }
        if (phase == 1 && cur == RT_BVH_EMPTY) { // the query is over: s_min, then the KD phase (or a miss)
            s_min = best;
            if (!(s_min < root_exit)) {
                *reinterpret_cast<float4 *>(st.hits + e) = miss_record();
                phase = 0;
            } else {
                phase = 2;
                node = 0;
                nd_ok = false;
                sp = 0;
                exit_ = root_exit; // (entry: the scene box's, unchanged since the refill)
            }
        }
        // ---- KD phase (trace_bvh's): up to `cap` node fetches, then the leaf
        for (int i = 0; i < cap; ++i) {
            const bool step = phase == 2 && !(nd_ok && (nd.y & 3u) == RT_LEAF_TAG);
            if (!__any(step)) break;
            if (step) {
                if (nd_ok) { // an inner node: the reference's split step
                    const uint32_t axis = nd.y & 3u;
                    const float split = as_float(nd.x);
                    const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
                    const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
                    const float yax = rt_recip_guard(dax);
                    uint32_t near_c = node + 1, far_c = nd.y >> 2;
                    if (oax >= split) { // ray_behind_plane (rt/trace_ray.cuh:174-188)
                        near_c = nd.y >> 2;
                        far_c = node + 1;
                    }
                    const float t = rt_div_by(split - oax, dax, yax); // intersect_plane (:190-210)
                    if (t >= exit_ || t < 0) {
                        node = near_c;
                    } else if (t <= entry) {
                        node = far_c;
                    } else if (t <= s_min) { // the near side holds no hit: its leaves' exits are <= t
                        node = far_c;
                        entry = t;
                    } else {
                        stk.put(sp++, far_c, t);
                        node = near_c;
                        exit_ = t;
                    }
                }
                nd = ldc_u2(sc.nodes + 2 * (size_t)node);
                nd_ok = true;
                if (COUNT) c.v[RT_CNT_NODE]++;
            }
        }
        const bool kleaf = phase == 2 && nd_ok && (nd.y & 3u) == RT_LEAF_TAG;
        if (__any(kleaf) && kleaf) {
            const uint32_t count = nd.y >> 2;
            int best_tri = -1;
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            if (count > 0 && exit_ > s_min) { // trace_leaf_node (:115-172): closest starts at the leaf's exit
                float smallest = exit_;
                if (COUNT) c.v[RT_CNT_TRI] += count;
                const int be = leaf_scan<COUNT>(sc.isect_a, sc.isect_bary, nd.x, nd.x + count, o, d, smallest, bx, by,
                                                bz, c);
                best_tri = be >= 0 ? (int)ldc_u2(&sc.isect_bary[be].rd).y : -1;
            }
            if (best_tri >= 0) {
                if (COUNT) c.v[RT_CNT_HIT]++;
                *reinterpret_cast<float4 *>(st.hits + e) = make_float4(__int_as_float(best_tri), bx, by, bz);
                phase = 0;
            } else if (sp == 0) {
                *reinterpret_cast<float4 *>(st.hits + e) = miss_record();
                phase = 0;
            } else {
                --sp;
                node = stk.node_at(sp);
                entry = stk.entry_at(sp);
                exit_ = sp > 0 ? stk.entry_at(sp - 1) : root_exit;
                nd_ok = false;
            }
        }
    }
    if (COUNT) flush_counters(c, counters);
}

// Persistent trace with dynamic ray fetch: every lane runs rays one leaf at a
// time; a lane whose ray is done writes its hit and takes the next queued ray
// at the next leaf boundary (one wave-aggregated atomic), so a wave is never
// held by its slowest ray.  Same per-ray arithmetic as trace().
template <bool COUNT>
__global__ void __launch_bounds__(WF_BLOCK) wf_trace_dyn(RtDevScene sc, WfState st, int q,
                                                         unsigned long long *counters)
{
    __shared__ uint32_t s_node[WF_LDS_STACK * WF_BLOCK];
    __shared__ float s_entry[WF_LDS_STACK * WF_BLOCK];
    const int tid = threadIdx.x;
    const int gtid = blockIdx.x * WF_BLOCK + tid;
    Stack<WF_LDS_STACK> stk{s_node + tid, s_entry + tid, WF_BLOCK, st.spill + gtid, st.spill_threads};
    Cnt c;
    if (COUNT) c.zero();
    const uint32_t n = st.counts[q];
    const RtF4 *rays = st.q_ray[q];
    uint32_t *fetch = st.counts + 2 + q;
    const int lane = __lane_id();

    bool live = false, exhausted = false;
    uint32_t e = 0, node = 0;
    int sp = 0;
    Vec3D o = rt_v3(0, 0, 0), d = rt_v3(0, 0, 0);
    float entry = 0.0f, exit_ = 0.0f, root_exit = 0.0f;
    while (true) {
        // ---- refill idle lanes
        const bool need = !live && !exhausted;
        const unsigned long long m = __ballot(need);
        if (m) {
            const int leader = __ffsll((long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(fetch, (uint32_t)__popcll(m));
            base = __shfl(base, leader);
            if (need) {
                e = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (e >= n) {
                    exhausted = true;
                } else {
                    o = ld3(ldf4(rays + 2 * (size_t)e));
                    d = ld3(ldf4(rays + 2 * (size_t)e + 1));
                    if (COUNT) c.v[RT_CNT_RAY]++;
                    if (bbox_hit(sc, o, d, entry, exit_)) {
                        root_exit = exit_;
                        node = 0;
                        sp = 0;
                        live = true;
                    } else {
                        *reinterpret_cast<float4 *>(st.hits + e) = miss_record();
                    }
                }
            }
        }
        if (!__any(live)) {
            if (__all(exhausted)) break;
            continue;
        }
        if (!live) continue;
        // ---- descend to a leaf (rt/trace_ray.cuh:273-306)
        uint2 nd = *reinterpret_cast<const uint2 *>(sc.nodes + 2 * (size_t)node);
        if (COUNT) c.v[RT_CNT_NODE]++;
        while ((nd.y & 3u) != RT_LEAF_TAG) {
            const uint32_t axis = nd.y & 3u;
            const float split = as_float(nd.x);
            const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
            const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
            uint32_t near_c = node + 1, far_c = nd.y >> 2;
            if (oax >= split) {
                near_c = nd.y >> 2;
                far_c = node + 1;
            }
            const float t = (split - oax) / dax;
            if (t >= exit_ || t < 0) {
                node = near_c;
            } else if (t <= entry) {
                node = far_c;
            } else {
                if (COUNT && sp >= RT_REF_STACK) c.v[RT_CNT_DEEP_PUSH]++;
                stk.put(sp, far_c, t);
                ++sp;
                node = near_c;
                exit_ = t;
            }
            nd = *reinterpret_cast<const uint2 *>(sc.nodes + 2 * (size_t)node);
            if (COUNT) c.v[RT_CNT_NODE]++;
        }
        // ---- leaf (rt/trace_ray.cuh:115-172)
        const int count = (int)(nd.y >> 2);
        int best = -1;
        float bx = 0.0f, by = 0.0f, bz = 0.0f;
        if (count > 0) {
            const uint32_t e0 = nd.x, e1 = nd.x + (uint32_t)count;
            float smallest = exit_;
            for (uint32_t k = e0; k < e1; k += 2) {
                const bool two = k + 1 < e1;
                if (COUNT) c.v[RT_CNT_TRI] += two ? 2 : 1;
                const RtF4 A0 = ldf4(sc.isect_a + k);
                const RtF4 A1 = ldf4(sc.isect_a + (two ? k + 1 : k));
                const float dn0 = d.x * A0.x + d.y * A0.y + d.z * A0.z;
                const float dn1 = d.x * A1.x + d.y * A1.y + d.z * A1.z;
                const float s0 = (A0.w - (o.x * A0.x + o.y * A0.y + o.z * A0.z)) / dn0;
                const float s1 = (A1.w - (o.x * A1.x + o.y * A1.y + o.z * A1.z)) / dn1;
                const bool p0 = dn0 != 0 && s0 >= 0.00001f && s0 < smallest;
                const bool p1 = two && dn1 != 0 && s1 >= 0.00001f && s1 < smallest;
                RtF4 B0, C0, D0, B1, C1, D1;
                uint2 R0, R1;
                if (p0) {
                    B0 = ldf4(&sc.isect_bary[k].b);
                    C0 = ldf4(&sc.isect_bary[k].c);
                    D0 = ldf4(&sc.isect_bary[k].d);
                    R0 = *reinterpret_cast<const uint2 *>(&sc.isect_bary[k].rd);
                }
                if (p1) {
                    B1 = ldf4(&sc.isect_bary[k + 1].b);
                    C1 = ldf4(&sc.isect_bary[k + 1].c);
                    D1 = ldf4(&sc.isect_bary[k + 1].d);
                    R1 = *reinterpret_cast<const uint2 *>(&sc.isect_bary[k + 1].rd);
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const bool p = j == 0 ? p0 : p1;
                    const float s = j == 0 ? s0 : s1;
                    if (!p || !(s < smallest)) continue;
                    const RtF4 B = j == 0 ? B0 : B1, C = j == 0 ? C0 : C1, D = j == 0 ? D0 : D1;
                    const uint2 R = j == 0 ? R0 : R1;
                    const float rd = as_float(R.x);
                    const float px = o.x + d.x * s, py = o.y + d.y * s, pz = o.z + d.z * s;
                    const float v2x = px - B.x, v2y = py - B.y, v2z = pz - B.z;
                    const float d20 = v2x * C.x + v2y * C.y + v2z * C.z;
                    const float d21 = v2x * D.x + v2y * D.y + v2z * D.z;
                    const float cy = (D.w * d20 - C.w * d21) * rd;
                    const float cz = (B.w * d21 - C.w * d20) * rd;
                    const float cx = 1.0f - cy - cz;
                    if (rt_bary_inside(cx, cy, cz)) {
                        smallest = s;
                        best = (int)R.y;
                        bx = cx;
                        by = cy;
                        bz = cz;
                    }
                }
            }
        }
        if (best >= 0) {
            if (COUNT) c.v[RT_CNT_HIT]++;
            *reinterpret_cast<float4 *>(st.hits + e) = make_float4(__int_as_float(best), bx, by, bz);
            live = false;
        } else if (sp == 0) {
            *reinterpret_cast<float4 *>(st.hits + e) = miss_record();
            live = false;
        } else {
            --sp;
            node = stk.node_at(sp);
            entry = stk.entry_at(sp);
            exit_ = sp > 0 ? stk.entry_at(sp - 1) : root_exit;
        }
    }
    if (COUNT) flush_counters(c, counters);
}

#include "coop_trace.h"

// Wave-cooperative trace with dynamic ray fetch (coop_trace.h): lanes whose
// ray finished take the next queued ray at the next round; descents are
// capped at `cap` node fetches per round and the leaf test waits for
// `postpone` pending lanes.
template <bool COUNT>
__global__ void __launch_bounds__(WF_TBLOCK, WF_TRACE_WAVES) wf_trace_coop(RtDevScene sc, WfState st, int q,
                                                          unsigned long long *counters, int cap, int postpone,
                                                          int wide_lanes, unsigned long long *timeline)
{
    // debug timeline (RtOptions.wave_times_device): s_memrealtime of the
    // launch's first wave start, first queue exhaustion, last wave end
    // (stored as ~t so that all three are atomicMin)
    if (timeline && __lane_id() == 0) atomicMin(timeline, __builtin_amdgcn_s_memrealtime());
    __shared__ uint32_t s_node[WF_LDS_STACK * WF_TBLOCK];
    __shared__ float s_entry[WF_LDS_STACK * WF_TBLOCK];
    __shared__ unsigned long long s_key[WF_TBLOCK];
    __shared__ CoopCand s_list[(WF_TBLOCK / 64) * WF_COOP_LIST];
    __shared__ int s_mark[2 * WF_TBLOCK]; // 128 per wave: chunk_owner marks + junk slots
    const int tid = threadIdx.x;
    const int gtid = blockIdx.x * WF_TBLOCK + tid;
    const int lane = __lane_id();
    const int wave = tid >> 6;
    Stack<WF_LDS_STACK> stk{s_node + tid, s_entry + tid, WF_TBLOCK, st.spill + gtid, st.spill_threads};
    unsigned long long *wkey = s_key + wave * 64;
    CoopCand *list = s_list + wave * WF_COOP_LIST;
    const CoopLds w{wkey, list, s_mark + wave * 128};
    Cnt c;
    if (COUNT) c.zero();
    const uint32_t n = st.counts[q];
    const RtF4 *rays = st.q_ray[q];
    uint32_t *fetch = st.counts + 2 + q;

    CoopRay r;
    coop_idle(r);
    bool exhausted = false;
    uint32_t e = 0;
    while (true) {
        const unsigned long long tf = COUNT ? __builtin_amdgcn_s_memtime() : 0ull;
        // ---- refill idle lanes (dynamic ray fetch)
        const bool need = !r.live && !exhausted;
        const unsigned long long m = __ballot(need);
        if (m) {
            const int leader = __ffsll((long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(fetch, (uint32_t)__popcll(m));
            base = __shfl(base, leader);
            if (need) {
                e = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (e >= n) {
                    exhausted = true;
                    if (timeline && e == n) atomicMin(timeline + 1, __builtin_amdgcn_s_memrealtime());
                } else {
                    if (COUNT) c.v[RT_CNT_RAY]++;
                    if (!coop_begin(sc, r, ld3(ldf4(rays + 2 * (size_t)e)), ld3(ldf4(rays + 2 * (size_t)e + 1))))
                        *reinterpret_cast<float4 *>(st.hits + e) = miss_record();
                }
            }
        }
        if (COUNT && lane == 0) c.v[RT_CNT_T_FETCH] += __builtin_amdgcn_s_memtime() - tf;
        if (WF_TAIL_PRIO > 0 && __any(exhausted)) __builtin_amdgcn_s_setprio(WF_TAIL_PRIO); // the launch's tail
        if (!__any(r.live)) {
            if (__all(exhausted)) break;
            continue;
        }
        int tri = -1;
        float bx = 0.0f, by = 0.0f, bz = 0.0f;
        // the launch's tail: the queue is empty and few rays are left in this
        // wave — leave the loop and finish them wide (below)
        if (wide_lanes > 0 && __any(exhausted) && __popcll(__ballot(r.live)) <= wide_lanes) break;
        if (coop_round<COUNT>(sc, r, stk, w, cap, postpone, tri, bx, by, bz, c))
            *reinterpret_cast<float4 *>(st.hits + e) = make_float4(__int_as_float(tri), bx, by, bz);
    }
    // finish the wave's remaining rays one at a time with all 64 lanes
    // (wide_resume) instead of letting the longest run alone at one lane's pace
    const unsigned long long lm = __ballot(r.live);
    if (lm) {
        const WideLds W{reinterpret_cast<WideItem *>(list),
                        WF_COOP_LIST * (int)sizeof(CoopCand) / (int)sizeof(WideItem), wkey,
                        reinterpret_cast<float *>(wkey + 1), w.mark};
        for (unsigned long long mm = lm; mm; mm &= mm - 1) {
            const int owner = __ffsll((long long)mm) - 1;
            const int ot = wave * 64 + owner;
            const Stack<WF_LDS_STACK> so{s_node + ot, s_entry + ot, WF_TBLOCK, st.spill + blockIdx.x * WF_TBLOCK + ot,
                                         st.spill_threads};
            int tri = -1;
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            wide_resume<COUNT>(sc, r, owner, so, W, tri, bx, by, bz, c);
            if (lane == owner) *reinterpret_cast<float4 *>(st.hits + e) = make_float4(__int_as_float(tri), bx, by, bz);
        }
    }
    if (timeline && lane == 0) atomicMin(timeline + 2, ~__builtin_amdgcn_s_memrealtime());
    if (COUNT) flush_counters(c, counters);
}

namespace {

// a ? x : y of two Vec3D values (a conditional of two lvalues selects their
// ADDRESSES, which keeps the path state in scratch memory)
__device__ __forceinline__ Vec3D pick(bool a, Vec3D x, Vec3D y)
{
    return rt_v3(a ? x.x : y.x, a ? x.y : y.y, a ? x.z : y.z);
}

// the state of one pixel's path between two ray queries
struct PathRegs {
    uint32_t slot;
    bool shadow, inside;
    bool dual;     // the roulette after this path's pending shadow ray was drawn when it was set up
    bool ext_live; // ... and let the path continue: its extension ray (ro, cont) is pending too
    int prev_type, depth, passes_left, light;
    uint32_t rng;
    Vec3D T, L, rp, cont, snorm, ro, rd;
};

// (wf_finish_bvh) a NEE set-up's state — light point, continuation, shading normal, light — in LDS
// between the set-up and its shadow ray's shading: written once and read once per diffuse bounce, it
// holds no registers through the traversal.  Addressed from a wave-uniform base plus the lane id
// recomputed at use (lane_id_here), so no per-lane address stays live either.
struct LdsV3 {
    float *w; // wave-uniform: this wave's column 0 of three WF_BLOCK-strided rows
    __device__ __forceinline__ operator Vec3D() const
    {
        const int l = lane_id_here();
        return rt_v3(w[l], w[WF_BLOCK + l], w[2 * WF_BLOCK + l]);
    }
    __device__ __forceinline__ LdsV3 &operator=(Vec3D v)
    {
        const int l = lane_id_here();
        w[l] = v.x;
        w[WF_BLOCK + l] = v.y;
        w[2 * WF_BLOCK + l] = v.z;
        return *this;
    }
    __device__ __forceinline__ LdsV3 &operator=(const LdsV3 &o) { return *this = (Vec3D)o; }
};
struct LdsInt {
    int *w;
    __device__ __forceinline__ operator int() const { return w[lane_id_here()]; }
    __device__ __forceinline__ LdsInt &operator=(int v)
    {
        w[lane_id_here()] = v;
        return *this;
    }
    __device__ __forceinline__ LdsInt &operator=(const LdsInt &o) { return *this = (int)o; }
};
// PathRegs with the NEE state in LDS (the same fields: shade_step and the load / store helpers take either)
struct PathRegsL {
    uint32_t slot;
    bool shadow, inside, dual, ext_live;
    int prev_type, depth, passes_left;
    LdsInt light;
    uint32_t rng;
    Vec3D T, L;
    LdsV3 rp, cont, snorm;
    Vec3D ro, rd;
};

template <typename P>
__device__ __forceinline__ void load_regs(const WfState &st, const RtDevFrame &fr, uint32_t slot, P &p)
{
    p.slot = slot;
    const uint32_t flags = st.flags[slot];
    p.shadow = flags & 1u;
    p.inside = (flags >> 1) & 1u;
    p.prev_type = (int)((flags >> 2) & 7u);
    p.dual = (flags >> 5) & 1u;
    p.ext_live = (flags >> 6) & 1u;
    p.depth = (int)(flags >> 8);
    p.rng = fr.rng[slot];
    p.T = st.T[slot];
    p.L = st.L[slot];
    p.passes_left = st.passes_left[slot];
    if (p.shadow) {
        p.light = st.light[slot];
        p.rp = st.rp[slot];
        p.cont = st.cont[slot];
        p.snorm = st.snorm[slot];
    }
}

template <typename P>
__device__ __forceinline__ void store_regs(const WfState &st, const RtDevFrame &fr, const P &p)
{
    const uint32_t slot = p.slot;
    fr.rng[slot] = p.rng;
    st.T[slot] = p.T;
    st.L[slot] = p.L;
    st.passes_left[slot] = p.passes_left;
    st.flags[slot] = (p.shadow ? 1u : 0u) | (p.inside ? 2u : 0u) | ((uint32_t)p.prev_type << 2) |
                     (p.dual ? 0x20u : 0u) | (p.ext_live ? 0x40u : 0u) | ((uint32_t)p.depth << 8);
    if (p.shadow) {
        st.light[slot] = p.light;
        st.rp[slot] = p.rp;
        st.cont[slot] = p.cont;
        st.snorm[slot] = p.snorm;
    }
}

// a path of a path list with its first pending ray in p.ro / p.rd (the
// shadow ray if one is pending: its direction recomputed as it was set up)
template <typename P>
__device__ __forceinline__ void first_ray(const WfState &st, const RtDevFrame &fr, uint32_t slot, P &p)
{
    load_regs(st, fr, slot, p);
    p.ro = st.ro[slot];
    p.rd = p.shadow ? rt_normalize(p.rp - p.ro) : st.cont[slot];
}

// One event of trace_path (rt/path_tracing.cuh:268-325) for the hit of the
// ray p.ro/p.rd: emission, BSDF, NEE set-up, roulette, accumulation and the
// pixel's next pass.  Returns true with the next ray in p.ro/p.rd.
//
// DUAL (the queue kernels): when NEE sets up a shadow ray, the Russian
// roulette that the reference draws after the shadow ray (:309-318) is drawn
// right away — nothing between consumes random numbers or changes the
// throughput — so the extension ray (p.ro, p.cont) can be traced in the SAME
// queue iteration as the shadow ray (p.dual, p.ext_live).  The shadow result
// is still applied first (L += direct * T, then T /= p), in the reference's
// order.  Any shade_step (DUAL or not) resumes such a path correctly.
template <bool COUNT, bool DUAL = false, typename P>
__device__ __forceinline__ bool shade_step(const RtDevScene &sc, const RtDevFrame &fr, const RtDevCamera &cam,
                                           P &p, int hit, float bx, float by, float bz, int limit, Cnt &c)
{
    bool finish = false, roulette = true, want = false;
    if (!p.shadow) {
        if (hit < 0) {
            finish = true; // miss: break without roulette (:303-306)
            roulette = false;
        } else {
            Surface s;
            shade<COUNT>(sc, hit, bx, by, bz, p.rd, s, c);
            if (p.prev_type != DIFFUSE) p.L = p.L + s.emittance * p.T; // :285-288
            Vec3D nd, w;
            p.prev_type = scatter(p.rd, p.inside, p.rng, s, nd, w);
            p.T = p.T * w;
            p.ro = s.position;
            p.rd = nd;
            if (p.prev_type == DIFFUSE) { // sample_direct_light (:235-265)
                if (COUNT) c.v[RT_CNT_NEE]++;
                float xi = rng_next(p.rng);
                if (sc.light_count == 0) {
                    rng_next(p.rng);
                    rng_next(p.rng);
                    p.L = p.L + rt_v3(0.0f, 0.0f, 0.0f) * p.T;
                } else {
                    p.light = sc.lights[(int)(xi * (float)sc.light_count)];
                    p.rp = light_point(sc, p.light, p.rng);
                    p.cont = p.rd;
                    p.snorm = s.normal;
                    p.rd = rt_normalize(p.rp - p.ro);
                    p.shadow = true;
                    roulette = false; // roulette after the shadow ray
                    want = true;
                    if (DUAL) { // the roulette now (the same draw as after the shadow ray)
                        const float pr = fmaxf(p.T.x, fmaxf(p.T.y, p.T.z));
                        const float r = rng_next(p.rng);
                        p.dual = true;
                        p.ext_live = false;
                        if (!(r > pr)) {
                            if (p.depth == limit) { // max_depth / watchdog before the next extension ray
                                if (COUNT && fr.max_depth <= 0) c.v[RT_CNT_WATCHDOG]++;
                                dev_record_cut(fr);
                            } else {
                                ++p.depth;
                                p.ext_live = true;
                            }
                        }
                    }
                }
            }
        }
    } else {
        Vec3D direct = rt_v3(0.0f, 0.0f, 0.0f);
        if (hit >= 0 && hit == p.light)
            direct = light_contribution(sc, p.light, bx, by, bz, p.ro, p.rd, p.rp, p.snorm);
        if (COUNT && hit >= 0 && material_of(sc, hit).tex) c.v[RT_CNT_TEXEL] += 2; // every hit is shaded
        p.L = p.L + direct * p.T;
        p.rd = p.cont;
        p.shadow = false;
        if (p.dual) { // the roulette was drawn at the set-up
            p.dual = false;
            roulette = false;
            if (p.ext_live) {
                p.T = p.T * (1.0f / fmaxf(p.T.x, fmaxf(p.T.y, p.T.z)));
                want = true; // depth was advanced at the set-up
            } else {
                finish = true;
            }
            p.ext_live = false;
        }
    }
    if (roulette) { // Russian roulette (:309-318)
        float pr = fmaxf(p.T.x, fmaxf(p.T.y, p.T.z));
        float r = rng_next(p.rng);
        if (r > pr) {
            finish = true;
        } else {
            p.T = p.T * (1.0f / pr);
            if (p.depth == limit) { // max_depth / watchdog before the next extension ray
                if (COUNT && fr.max_depth <= 0) c.v[RT_CNT_WATCHDOG]++;
                dev_record_cut(fr);
                finish = true;
            } else {
                ++p.depth;
                want = true;
            }
        }
    }
    if (finish) { // accumulation (:322-324), then the pixel's next pass
        if (COUNT) c.path_end(p.depth);
        dev_record_end(fr, p.depth);
        const uint32_t slot = p.slot;
        Vec3D fb = fr.fb[slot] + p.L;
        float sq = fr.sq[slot] + rt_square(rt_luminance(p.L));
        int count = fr.count[slot] + 1;
        fr.fb[slot] = fb;
        fr.sq[slot] = sq;
        fr.count[slot] = count;
        if (p.passes_left > 0) {
            want = start_sample<COUNT>(fr, cam, (int)slot, p.passes_left, p.rng, fb, sq, count, p.ro, p.rd, c);
            if (want) {
                p.T = rt_v3(1.0f, 1.0f, 1.0f);
                p.L = rt_v3(0.0f, 0.0f, 0.0f);
                p.inside = false;
                p.prev_type = PRIMARY;
                p.depth = 1;
                p.shadow = false;
            }
        }
    }
    return want;
}

} // namespace

template <bool COUNT>
__global__ void __launch_bounds__(WF_TBLOCK, WF_SHADE_WAVES) wf_shade(RtDevScene sc, RtDevFrame fr, RtDevCamera cam, WfState st, int q)
{
    if (WF_SHADE_PRIO > 0) __builtin_amdgcn_s_setprio(WF_SHADE_PRIO); // ahead of co-resident trace waves
    Cnt c;
    if (COUNT) c.zero();
    const uint32_t n = st.counts[6 + q]; // paths with rays in ray queue q
    const int qn = q ^ 1;
    const int limit = fr.max_depth > 0 ? fr.max_depth : RT_WATCHDOG_BOUNCES;
    for (uint32_t base = blockIdx.x * WF_TBLOCK; base < n; base += gridDim.x * WF_TBLOCK) {
        const uint32_t i = base + threadIdx.x;
        bool want = false;
        PathRegs p;
        p.slot = 0;
        p.shadow = p.ext_live = false;
        p.ro = p.rd = p.cont = rt_v3(0, 0, 0);
        if (i < n) {
            const uint32_t slot = st.q_slot[q][i];
            load_regs(st, fr, slot, p);
            p.ro = st.ro[slot];
            if (p.shadow) {
                // the shadow ray (set up DUAL: its roulette is drawn) and, if the
                // path went on, its extension ray were traced in this iteration
                const bool both = p.ext_live;
                p.rd = rt_normalize(p.rp - p.ro); // the shadow ray's direction, as set up
                const RtF4 h = ldf4(st.hits + st.e_sh[slot]);
                want = shade_step<COUNT, true>(sc, fr, cam, p, __float_as_int(h.x), h.y, h.z, h.w, limit, c);
                if (both) { // p.ro / p.rd = the extension ray: its hit is in too
                    const RtF4 g = ldf4(st.hits + st.e_ext[slot]);
                    want = shade_step<COUNT, true>(sc, fr, cam, p, __float_as_int(g.x), g.y, g.z, g.w, limit, c);
                }
            } else {
                p.rd = st.cont[slot];
                const RtF4 h = ldf4(st.hits + st.e_ext[slot]);
                want = shade_step<COUNT, true>(sc, fr, cam, p, __float_as_int(h.x), h.y, h.z, h.w, limit, c);
            }
            store_regs(st, fr, p);
            if (want) { // the pending ray(s): extension = (ro, cont)
                st.ro[slot] = p.ro;
                st.cont[slot] = pick(p.shadow, p.cont, p.rd);
            }
        }
        const bool to_long = want && st.long_depth > 0 && p.depth > st.long_depth;
        const bool go = want && !to_long;
        const bool sh = go && p.shadow, ex = go && (!p.shadow || p.ext_live);
        const uint32_t es = enqueue_ray(st, qn, sh, p.ro, p.rd);
        const uint32_t ee = enqueue_ray(st, qn, ex, p.ro, pick(p.shadow, p.cont, p.rd));
        if (sh) st.e_sh[p.slot] = es;
        if (ex) st.e_ext[p.slot] = ee;
        enqueue_path(st, qn, go, p.slot);
        // wf_long takes the path with its first pending ray (the shadow ray if any)
        if (__any(to_long)) publish_long(st, to_long, p.slot, p.ro, p.rd);
    }
    if (COUNT) flush_counters(c, fr.counters);
}

// Tail finisher: once few paths remain, each remaining pixel is run to the end
// of its passes by one lane (trace + shade in registers, megakernel style), so
// the long total-internal-reflection paths cost one launch instead of one
// trace/shade iteration per bounce.
template <bool COUNT>
__global__ void __launch_bounds__(WF_BLOCK) wf_finish(RtDevScene sc, RtDevFrame fr, RtDevCamera cam, WfState st, int q)
{
    __shared__ uint32_t s_node[WF_LDS_STACK * WF_BLOCK];
    __shared__ float s_entry[WF_LDS_STACK * WF_BLOCK];
    const int tid = threadIdx.x;
    const int gtid = blockIdx.x * WF_BLOCK + tid;
    Stack<WF_LDS_STACK> stk{s_node + tid, s_entry + tid, WF_BLOCK, st.spill + gtid, st.spill_threads};
    Cnt c;
    if (COUNT) c.zero();
    const uint32_t n = st.counts[6 + q]; // paths of path list q
    const int limit = fr.max_depth > 0 ? fr.max_depth : RT_WATCHDOG_BOUNCES;
    for (uint32_t base = blockIdx.x * WF_BLOCK; base < n; base += gridDim.x * WF_BLOCK) {
        const uint32_t e = base + tid;
        if (e < n) {
            PathRegs p;
            first_ray(st, fr, st.q_slot[q][e], p);
            while (true) {
                float bx = 0.0f, by = 0.0f, bz = 0.0f;
                const int hit = trace<COUNT>(sc, p.ro, p.rd, bx, by, bz, stk, c);
                if (!shade_step<COUNT>(sc, fr, cam, p, hit, bx, by, bz, limit, c)) break;
            }
            store_regs(st, fr, p);
        }
    }
    if (COUNT) {
        flush_counters(c, fr.counters);
        flush_finish_counters(c, fr.counters);
    }
}

namespace {

// a 4-byte load past the CU's L1 (global_load sc1: L2-served), for data another CU released
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p)
{
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a 4-byte write-through store (global_store sc1), for data another CU will read
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// fresh entry e of the whole-call finisher's pixel list -> its pixel: 256
// entries per 16x16-pixel tile, 64 per 8x8-pixel wave tile (wf_start's
// layout); false for a pixel outside the frame or in a row another shard owns
__device__ __forceinline__ bool fresh_pixel(const RtDevFrame &fr, uint32_t e, int &slot)
{
    const uint32_t tiles_x = (uint32_t)(fr.width + 15) / 16u;
    const uint32_t t = e >> 8, w = (e >> 6) & 3u, l = e & 63u;
    const int x = (int)((t % tiles_x) * 16u + (w & 1u) * 8u + (l & 7u));
    const int y = (int)((t / tiles_x) * 16u + (w >> 1) * 8u + (l >> 3));
    if (x >= fr.width || y >= fr.height || !rt_row_owned(fr, y)) return false;
    slot = y * fr.width + x;
    return true;
}

// a sample's path state at its camera ray (trace_path's start, rt/path_tracing.cuh:270-277)
template <typename P>
__device__ __forceinline__ void begin_path(P &p)
{
    p.T = rt_v3(1.0f, 1.0f, 1.0f);
    p.L = rt_v3(0.0f, 0.0f, 0.0f);
    p.inside = false;
    p.prev_type = PRIMARY;
    p.depth = 1;
    p.shadow = false;
    p.dual = false;
    p.ext_live = false;
}

} // namespace

// Finisher with the BVH-bounded traversal (bvh_trace.h): every lane runs one
// path to the end of its pixel's passes (trace + shade in registers,
// megakernel style) and then takes the next queued path (wave-aggregated
// atomic on counts[4]); a path deeper than long_depth goes on in wf_long.
// With the bounded traversal this runs the WHOLE call (wf_start's path list:
// no queue iterations), see rt_launch_wavefront.  COUNT: the traversal's own
// work (trace_bvh) and the reference's shading counters.
// WAVES: the occupancy it is built for — WF_FIN_BVH_WAVES (96 VGPRs, the rest
// spilled) when the chip is full of its waves; 1 (no register cap, no spills)
// for a frame whose pixels fill at most WF_FIN_SMALL_WAVES waves per SIMD, where
// the occupancy is the pixel count's anyway and every spill's latency shows
template <bool COUNT, int WAVES = WF_FIN_BVH_WAVES>
__global__ void __launch_bounds__(WF_BLOCK, WAVES) wf_finish_bvh(RtDevScene sc, RtDevFrame fr, RtDevCamera cam,
                                                                 WfState st, int q)
{
    __shared__ uint32_t s_node[WF_BVH_LDS * WF_BLOCK];
    __shared__ float s_entry[WF_BVH_LDS * WF_BLOCK];
    const int tid = threadIdx.x;
    const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63); // (wave-uniform)
    LaneStack<WF_BVH_LDS> stk{s_node + wbase, s_entry + wbase, WF_BLOCK, st.spill + (blockIdx.x * WF_BLOCK + wbase),
                              st.spill_threads};
    Cnt c;
    if (COUNT) c.zero();
    // fresh: this call's pixels, 256 entries per 16x16-pixel tile (fresh_pixel); else the paths of path list q
    // (fresh: the listed heavy pixels first, then the tiles)
    const uint32_t n_heavy = st.fresh && st.heavy_list ? *st.heavy_n : 0u;
    const uint32_t n = st.fresh ? n_heavy + st.fresh_n : st.counts[6 + q];
    uint32_t *fetch = st.counts + 4;
    const int limit = fr.max_depth > 0 ? fr.max_depth : RT_WATCHDOG_BOUNCES;
    const int lane = __lane_id();
    unsigned long long *const ret_word = reinterpret_cast<unsigned long long *>(st.ret_ctr);
    uint32_t *const ret_claimed = st.ret_ctr + 2;
    if (lane == 0) {
        // the call's finisher has started: from here wf_long waits for its producers (WF_FIN_STARTED)
        if (st.fin_live && !(__hip_atomic_load(st.fin_live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & WF_FIN_STARTED))
            __hip_atomic_fetch_or(st.fin_live, WF_FIN_STARTED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (st.long_return) // this wave is alive: wf_long may return pixels to it
            __hip_atomic_fetch_add(ret_word, 1ull << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (st.span) atomicMin(st.span, __builtin_amdgcn_s_memrealtime());
        if (st.long_log && blockIdx.x == 0 && threadIdx.x == 0) st.long_log[0] = __builtin_amdgcn_s_memrealtime();
    }
#if WF_NEE_LDS
    __shared__ float s_nee[10 * WF_BLOCK];
    PathRegsL p;
    p.rp.w = s_nee + wbase;
    p.cont.w = s_nee + 3 * WF_BLOCK + wbase;
    p.snorm.w = s_nee + 6 * WF_BLOCK + wbase;
    p.light.w = reinterpret_cast<int *>(s_nee + 9 * WF_BLOCK) + wbase;
#else
    PathRegs p;
#endif
    p.slot = 0;
    p.ro = p.rd = rt_v3(0, 0, 0);
    bool active = false, exhausted = false; // exhausted: this lane found the path list empty
    bool rel = false;                       // (fresh) the lane's pixel has no passes left: let it go
    unsigned long long idle_since = 0;      // (lane 0) when the wave first had nothing to do
    uint32_t quiet_trips = 0;               // (lane 0) idle loop trips in a row with no wf_long path running
    uint32_t idle_trips = 0;                // (lane 0) idle loop trips in a row
    bool seated = false;                    // (lane 0) holds a linger seat
#if WF_BVH_PARK
    // a lane whose s_min query ran WF_BVH_PARK node steps parks it (its state in LDS, the stack in
    // place) and resumes it in the wave's next loop trip: the rest of the wave shades meanwhile
    __shared__ uint32_t s_pk_cur[WF_BLOCK];
    __shared__ int s_pk_sp[WF_BLOCK];
    __shared__ float s_pk_best[WF_BLOCK];
    __shared__ int s_pk_tk[WF_BLOCK];
    bool parked = false;
#endif
    while (true) {
        // (fresh) pixels whose passes are done are let go — unless a later chained call queued
        // passes for them meanwhile: those run next, in the pixel's order (its state is this lane's).
        // (The next claimer is a later launch — chained finishers run one after the other — whose
        // kernel boundary orders this lane's stores before its loads.)
        while (st.fresh && __any(rel)) {
            if (rel) {
                uint32_t x = RT_PX_BUSY;
                if (__hip_atomic_compare_exchange_strong(st.pxo + p.slot, &x, 0u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)) {
                    rel = false;
                } else {
                    x = __hip_atomic_exchange(st.pxo + p.slot, RT_PX_BUSY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t owed = x & RT_PX_PASSES;
                    __hip_atomic_fetch_max(st.ret_ctr + 5, owed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_add(st.ret_ctr + 6, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    atomicAdd(fr.dev_stats + RT_DEV_OWED_PIXELS, 1ull);
                    atomicAdd(fr.dev_stats + RT_DEV_OWED_PASSES, (unsigned long long)owed);
                    p.passes_left = (int)owed;
                    const Vec3D fb = fr.fb[p.slot];
                    const float sq = fr.sq[p.slot];
                    const int count = fr.count[p.slot];
                    if (start_sample<COUNT>(fr, cam, (int)p.slot, p.passes_left, p.rng, fb, sq, count, p.ro, p.rd,
                                            c)) {
                        begin_path(p);
                        rel = false;
                        active = true;
                    }
                }
            }
        }
        if (st.long_return) {
            // free lanes take pixels wf_long returned BEFORE fresh ones (one
            // compare-and-swap per wave): a returned pixel is mid-chain — it may
            // carry the passes of chained calls that skipped it (pxo) — and
            // started only at the end of the path list it would end the call late.
            // Chained calls (no linger): only while the path list lasts — the call's
            // tail leaves later returns to the next call's (or the drain's) finisher
            const bool chained = st.linger == 0ull;
            const bool idle = !active && !(chained && exhausted);
            const unsigned long long im = __ballot(idle);
            if (im) {
                const int leader = __ffsll((long long)im) - 1;
                uint32_t base = 0, got = 0;
                if (lane == leader) {
                    uint32_t c0 = __hip_atomic_load(ret_claimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t r =
                        (uint32_t)__hip_atomic_load(ret_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t want_n = (uint32_t)__popcll(im);
                    uint32_t take = r > c0 ? (r - c0 < want_n ? r - c0 : want_n) : 0u;
                    if (take && chained && __hip_atomic_load(fetch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n)
                        take = 0u;
                    if (take && __hip_atomic_compare_exchange_strong(ret_claimed, &c0, c0 + take, __ATOMIC_RELAXED,
                                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        base = c0;
                        got = take;
                    }
                }
                base = (uint32_t)__shfl((int)base, leader);
                got = (uint32_t)__shfl((int)got, leader);
                const uint32_t rank = (uint32_t)__popcll(im & ((1ull << lane) - 1ull));
                if (idle && rank < got) {
                    // reserved by a running wf_long wave, which publishes it right after (store
                    // in flight): a bounded wait — expired, the pixel stays out (wf_verify
                    // reports it stranded) rather than the wave spinning on
                    const uint32_t e = base + rank;
                    unsigned long long v = 0;
                    bool pub = false;
                    for (uint32_t spin = 0; spin < WF_SPIN_TRIPS; ++spin) {
                        v = __hip_atomic_load(st.ret_ring + e % st.long_cap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        pub = (uint32_t)(v >> 32) == e + 1u;
                        if (pub) break;
                        __builtin_amdgcn_s_sleep(1);
                    }
                    if (!pub) {
                        atomicAdd(fr.dev_stats + RT_DEV_LONG_QUIT, 1ull);
                    } else {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        __hip_atomic_fetch_sub(st.ret_ctr + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        active = true;
                        first_ray(st, fr, (uint32_t)v, p);
                        // back from wf_long: no longer OUT but BUSY (this lane's); plus the passes chained
                        // calls queued meanwhile
                        const uint32_t owed = __hip_atomic_exchange(st.pxo + (uint32_t)v, RT_PX_BUSY, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT);
                        p.passes_left += (int)(owed & RT_PX_PASSES);
                        if (owed & RT_PX_PASSES) { // (RT_DEBUG_CALL_LOG: most passes owed, pixels owed; RtDeviations)
                            __hip_atomic_fetch_max(st.ret_ctr + 5, owed & RT_PX_PASSES, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_fetch_add(st.ret_ctr + 6, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            atomicAdd(fr.dev_stats + RT_DEV_OWED_PIXELS, 1ull);
                            atomicAdd(fr.dev_stats + RT_DEV_OWED_PASSES, (unsigned long long)(owed & RT_PX_PASSES));
                        }
                    }
                }
            }
        }
        if (st.fresh) {
            // this call's pixels (wf_start's work, in its 8x8-pixel wave tiles): a lane claims its
            // pixel (BUSY) unless another holder still has it — a previous chained call's finisher
            // lane or wf_long —, which then owes it this call's passes and runs them next
            // (a lane that found the list run out stays out: idle trips must not keep adding to
            // the cursor — a lingering wave's trips wrapped it past 2^32 and re-ran the call's
            // pixels)
            bool claim = !active && !rel && !exhausted, started = false, acq = false;
            while (__any(claim)) {
                const unsigned long long m = __ballot(claim);
                const int leader = __ffsll((long long)m) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(fetch, (uint32_t)__popcll(m));
                base = __shfl(base, leader);
                if (claim) {
                    const uint32_t e = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                    int slot = 0;
                    if (e >= n) {
                        claim = false;
                        exhausted = true;
                    } else if (e < n_heavy ? (slot = (int)st.heavy_list[e], true)
                                           : fresh_pixel(fr, e - n_heavy, slot) &&
                                                 !(st.heavy_list && st.listed[slot] == st.call_id)) {
                        uint32_t x = __hip_atomic_load(st.pxo + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        while (true) {
                            if (x & (RT_PX_OUT | RT_PX_BUSY)) { // held: owed this call's passes
                                if (__hip_atomic_compare_exchange_strong(st.pxo + slot, &x, x + (uint32_t)fr.passes,
                                                                         __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT))
                                    break;
                            } else if (__hip_atomic_compare_exchange_strong(st.pxo + slot, &x, RT_PX_BUSY,
                                                                            __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_AGENT)) {
                                claim = false;
                                started = true;
                                acq = (x & RT_PX_REL) != 0u; // (released by wf_long, which runs beside this)
                                p.slot = (uint32_t)slot;
                                break;
                            }
                        }
                    }
                }
            }
            // (a pixel whose last holder was wf_long, running beside this finisher, was released with
            // plain stores + an agent release before the word said free (LONGDONE): read it after an
            // agent acquire.  sc1 loads alone are no acquire for plain-stored bytes
            // (MI355X_MICROARCH.md, Valid forms): this XCD's L2 may hold the line from a neighbouring
            // pixel read earlier.  A pixel last held by an earlier launch needs none: the launch
            // boundary is the release / acquire.)
            if (__any(acq)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (started) { // the pixel's state and its first pass (wf_start's)
                const uint32_t slot = p.slot;
                p.rng = ld_sc1(fr.rng + slot);
                Vec3D fb = rt_v3(0.0f, 0.0f, 0.0f);
                float sq = 0.0f;
                int count = 0;
                if (fr.reset) { // reset_frame (rt/render.cuh:18-34)
                    fr.fb[slot] = fb;
                    fr.sq[slot] = sq;
                    fr.count[slot] = count;
                } else {
                    const uint32_t *f3 = reinterpret_cast<const uint32_t *>(fr.fb + slot);
                    fb = rt_v3(__uint_as_float(ld_sc1(f3)), __uint_as_float(ld_sc1(f3 + 1)), __uint_as_float(ld_sc1(f3 + 2)));
                    sq = __uint_as_float(ld_sc1(reinterpret_cast<const uint32_t *>(fr.sq + slot)));
                    count = (int)ld_sc1(reinterpret_cast<const uint32_t *>(fr.count + slot));
                }
                p.passes_left = fr.passes;
                if (start_sample<COUNT>(fr, cam, (int)slot, p.passes_left, p.rng, fb, sq, count, p.ro, p.rd, c)) {
                    begin_path(p);
                    active = true;
                } else {
                    rel = true; // no sample this call (adaptive test): let it go
                }
            }
        } else {
            const bool need = !active && !exhausted;
            const unsigned long long m = __ballot(need);
            if (m) {
                const int leader = __ffsll((long long)m) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(fetch, (uint32_t)__popcll(m));
                base = __shfl(base, leader);
                if (need) {
                    const uint32_t e = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                    if (e >= n) {
                        exhausted = true;
                    } else {
                        active = true;
                        first_ray(st, fr, st.q_slot[q][e], p);
                    }
                }
            }
        }
        if (!__any(active || rel)) {
            if (!st.long_return) break; // every lane exhausted
            if (st.linger == 0ull) { // chained: returns left are the next call's (or the drain's)
                if (lane == 0) __hip_atomic_fetch_sub(ret_word, 1ull << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            // leave only while every reserved return is claimed (else: claim them next round), and
            // while pixels are out in wf_long linger for them — bounded: st.linger ticks, and
            // WF_FIN_QUIET_TRIPS trips with no wf_long path running (where wf_long cannot run
            // beside the finisher — counter collection serialises the two launches — lingering
            // would only hold the finisher's end, and the next launch, up), WF_FIN_LINGER_TRIPS in all
            int leave = 0;
            if (lane == 0) {
                if (idle_since == 0) idle_since = __builtin_amdgcn_s_memrealtime();
                if (__hip_atomic_load(st.long_ctr + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
                    ++quiet_trips;
                else
                    quiet_trips = 0;
                ++idle_trips;
                bool out = quiet_trips < WF_FIN_QUIET_TRIPS && idle_trips < WF_FIN_LINGER_TRIPS &&
                           __hip_atomic_load(st.ret_ctr + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
                // only WF_FIN_LINGER_WAVES waves linger (a seat each, kept until they leave): the
                // others leave their slots to wf_long, which the deep paths are waiting for
                if (out && !seated) {
                    if (__hip_atomic_fetch_add(st.ret_ctr + 4, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                        WF_FIN_LINGER_WAVES)
                        seated = true;
                    else
                        out = false;
                }
                unsigned long long w = __hip_atomic_load(ret_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t cl = __hip_atomic_load(ret_claimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)w == cl &&
                    (!out || __builtin_amdgcn_s_memrealtime() - idle_since > st.linger) &&
                    __hip_atomic_compare_exchange_strong(ret_word, &w, w - (1ull << 32), __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    leave = 1;
                    // (pixels still out: wf_long, finding no finisher alive, finishes them itself)
                    if (out) atomicAdd(fr.dev_stats + RT_DEV_LINGER_EXP, 1ull);
                }
            }
            if (__shfl(leave, 0)) break;
            __builtin_amdgcn_s_sleep(8);
            continue;
        }
        idle_since = 0;
        quiet_trips = 0;
        idle_trips = 0;
        bool to_long = false;
        if (active) {
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
#if WF_BVH_PARK
            int hit;
            BvhPark pk{0u, 0, 0.0f, -1};
            if (parked) pk = BvhPark{s_pk_cur[tid], s_pk_sp[tid], s_pk_best[tid], s_pk_tk[tid]};
            const bool done = trace_bvh_park<COUNT>(sc, p.ro, p.rd, hit, bx, by, bz, stk, c, WF_BVH_PARK, parked, pk);
            parked = !done;
            if (parked) {
                s_pk_cur[tid] = pk.cur;
                s_pk_sp[tid] = pk.sp;
                s_pk_best[tid] = pk.best;
                s_pk_tk[tid] = pk.tk;
            }
#else
            const int hit = trace_bvh<COUNT>(sc, p.ro, p.rd, bx, by, bz, stk, c);
            const bool done = true;
#endif
            // run-time exactness guard: a deterministic sample of the rays, with the
            // bounded result, is queued for wf_check's plain KD re-trace
            if (!COUNT && st.chk && done) {
                uint32_t h = p.slot * 0x9E3779B1u ^ (uint32_t)p.passes_left * 0x85EBCA77u ^
                             (uint32_t)p.depth * 0xC2B2AE3Du ^ (p.shadow ? 0x27D4EB2Fu : 0u);
                h ^= h >> 15;
                h *= 0x2C1B3C6Du;
                h ^= h >> 12;
                const bool rec = (h & st.chk_mask) == 0u;
                if (__any(rec)) {
                    const uint32_t i = wave_append(st.chk_ctr, rec);
                    if (rec && i < st.chk_cap) {
                        st.chk[3 * (size_t)i] =
                            RtF4{p.ro.x, p.ro.y, p.ro.z, __int_as_float(st.chk_fault ? (hit >= 0 ? hit ^ 1 : 0) : hit)};
                        st.chk[3 * (size_t)i + 1] = RtF4{p.rd.x, p.rd.y, p.rd.z, bx};
                        st.chk[3 * (size_t)i + 2] = RtF4{by, bz, 0.0f, 0.0f};
                    }
                }
            }
            if (done) {
                const bool want = shade_step<COUNT>(sc, fr, cam, p, hit, bx, by, bz, limit, c);
                // a path deeper than long_depth goes on in wf_long (64 lanes per ray)
                to_long = want && st.long_depth > 0 && p.depth > st.long_depth;
                if (!want || to_long) store_regs(st, fr, p);
                if (!want) {
                    active = false;
                    rel = st.fresh != 0; // (the pixel's passes are done: let go at the top of the loop)
                }
            }
        }
        if (__any(to_long) && publish_long_capped(st, to_long, p.slot, p.ro, p.rd) && to_long) {
            active = false;
            if (st.heavy) { // (first in the next call's list: the more hand-offs, the earlier)
                const uint8_t h = st.heavy[p.slot];
                if (h < 255) st.heavy[p.slot] = (uint8_t)(h + 1);
            }
        }
    }
    if (COUNT) flush_counters(c, fr.counters);
    if (st.span && lane == 0) atomicMax(st.span + 1, __builtin_amdgcn_s_memrealtime());
    if (st.fin_live) { // this wave's hand-offs are published: the persistent wf_long may stop once all are past here
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (lane == 0) __hip_atomic_fetch_sub(st.fin_live, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The run-time exactness guard's second half: every ray wf_finish_bvh
// recorded is traced again with the plain KD traversal (trace(), i.e.
// trace_ray, rt/trace_ray.cuh:244-318) and compared bit for bit with the
// bounded result (triangle, barycentrics).  Counts checks and mismatches in
// the deviation statistics and keeps the first mismatching ray.  One ray per
// lane, grid-stride within the spill area (grid blocks).
__global__ void __launch_bounds__(WF_BLOCK) wf_check(RtDevScene sc, WfState st, unsigned long long *dev)
{
    __shared__ uint32_t s_node[WF_LDS_STACK * WF_BLOCK];
    __shared__ float s_entry[WF_LDS_STACK * WF_BLOCK];
    const int tid = threadIdx.x;
    const int gtid = blockIdx.x * WF_BLOCK + tid;
    Stack<WF_LDS_STACK> stk{s_node + tid, s_entry + tid, WF_BLOCK, st.spill + gtid, st.spill_threads};
    Cnt c;
    uint32_t n = *st.chk_ctr;
    if (n > st.chk_cap && gtid == 0) atomicAdd(dev + RT_DEV_CHK_DROP, (unsigned long long)(n - st.chk_cap));
    n = n < st.chk_cap ? n : st.chk_cap;
    unsigned long long checked = 0, bad = 0;
    // records over the waves first (record e on wave e % waves, lane e / waves): a small call's
    // few records run one or two per wave, each re-trace's node fetches alone in its wave, not
    // 64 in lockstep in the first waves (the slowest re-trace bounds the kernel, and the chained
    // call two later waits for it: its records reuse this parity)
    const uint32_t waves = gridDim.x * (WF_BLOCK / 64);
    const uint32_t first = (uint32_t)(tid & 63) * waves + blockIdx.x * (WF_BLOCK / 64) + (uint32_t)(tid >> 6);
    for (uint32_t e = first; e < n; e += gridDim.x * WF_BLOCK) {
        const RtF4 a = st.chk[3 * (size_t)e], b = st.chk[3 * (size_t)e + 1], q = st.chk[3 * (size_t)e + 2];
        const Vec3D o = rt_v3(a.x, a.y, a.z), d = rt_v3(b.x, b.y, b.z);
        float bx = 0.0f, by = 0.0f, bz = 0.0f;
        const int hit = trace<false>(sc, o, d, bx, by, bz, stk, c);
        ++checked;
        const bool same = hit == __float_as_int(a.w) &&
                          (hit < 0 || (__float_as_uint(bx) == __float_as_uint(b.w) &&
                                       __float_as_uint(by) == __float_as_uint(q.x) &&
                                       __float_as_uint(bz) == __float_as_uint(q.y)));
        if (!same) {
            ++bad;
            if (atomicCAS(dev + RT_DEV_MISRAY, 0ull, 1ull) == 0ull) { // the first mismatch: its ray
                dev[RT_DEV_MISRAY + 1] = (unsigned long long)__float_as_uint(o.x) << 32 | __float_as_uint(o.y);
                dev[RT_DEV_MISRAY + 2] = (unsigned long long)__float_as_uint(o.z) << 32 | __float_as_uint(d.x);
                dev[RT_DEV_MISRAY + 3] = (unsigned long long)__float_as_uint(d.y) << 32 | __float_as_uint(d.z);
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        checked += __shfl_xor(checked, off);
        bad += __shfl_xor(bad, off);
    }
    if ((tid & 63) == 0) {
        if (checked) atomicAdd(dev + RT_DEV_CHECKED, checked);
        if (bad) atomicAdd(dev + RT_DEV_MISMATCH, bad);
    }
}

// The join's check of the hand-off protocol (after every finisher, wf_long and
// drain of the workspace is done): a pixel still OUT was handed to wf_long and
// never came back, one still BUSY was never let go by a finisher lane — its
// frame misses passes.  Counts such pixels (and releases
// them, so later calls run them again) and the protocol's counters that must
// be balanced by now: pixels out, returns reserved but unclaimed, hand-off
// entries reserved but unclaimed, finisher waves still registered alive.
// res: [0] stranded pixels, [1..4] those counters (accumulated until the host reads them).
// Heavy pixels first: the pixels marked heavy (a path of theirs went to wf_long
// in an earlier call) that this call renders, listed (wave-aggregated atomic:
// any order — a pixel's passes run in its own order whoever takes it first)
// and tagged with the call so the finisher's tile entries skip them.  The
// deep-path-prone pixels then start their chains at the call's start instead
// of wherever their tile falls: their deep samples end inside the call rather
// than in the chain's drain.
__global__ void __launch_bounds__(WF_BLOCK) wf_heavy_list(RtDevFrame fr, WfState st, uint32_t call_id,
                                                           uint32_t lo, uint32_t hi)
{
    const uint32_t n = (uint32_t)fr.width * (uint32_t)fr.height;
    const int lane = __lane_id();
    // (wave-uniform loop: every lane of the wave reaches the ballot)
    for (uint32_t w0 = blockIdx.x * WF_BLOCK + (threadIdx.x & ~63u); w0 < n; w0 += WF_BLOCK * gridDim.x) {
        const uint32_t i = w0 + (uint32_t)lane;
        // (pixels handed over lo..hi-1 times so far: the heaviest are listed by the first launch)
        const uint32_t h = i < n ? (uint32_t)st.heavy[i] : 0u;
        const bool take = h >= lo && h < hi && rt_row_owned(fr, (int)(i / (uint32_t)fr.width));
        const unsigned long long m = __ballot(take);
        if (!m) continue;
        const int leader = __ffsll((long long)m) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(st.heavy_n, (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, leader);
        if (take) {
            st.heavy_list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
            st.listed[i] = call_id;
        }
    }
}

__global__ void __launch_bounds__(WF_BLOCK) wf_verify(WfState st, uint32_t n, uint32_t *res, unsigned long long *dev)
{
    uint32_t out = 0;
    for (uint32_t i = blockIdx.x * WF_BLOCK + threadIdx.x; i < n; i += gridDim.x * WF_BLOCK) {
        const uint32_t x = st.pxo[i];
        if (x) { // (free-after-a-concurrent-holder words become plain free: the join ordered everything)
            out += (x & (RT_PX_OUT | RT_PX_BUSY)) ? 1u : 0u;
            st.pxo[i] = 0u;
        }
    }
    for (int off = 32; off > 0; off >>= 1) out += __shfl_xor(out, off);
    if ((threadIdx.x & 63) == 0 && out) {
        atomicAdd(res, out);
        atomicAdd(dev + RT_DEV_STRANDED, (unsigned long long)out);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long rw = *reinterpret_cast<const unsigned long long *>(st.ret_ctr);
        res[1] += st.ret_ctr[3];
        res[2] += (uint32_t)rw - st.ret_ctr[2];
        res[3] += (st.long_ctr[0] & ~WF_LONG_CLOSED) - st.long_ctr[1];
        res[4] += (uint32_t)(rw >> 32);
    }
}

// Cooperative finisher: runs queued paths to the end of their passes in
// registers (shade_step right after each ray query), megakernel style, while
// the whole wave tests leaf entries for its live rays together (coop_round).
// Each wave keeps up to `ppw` (1..64) paths in flight, one per lane; a lane
// whose path is done takes the next queue entry (wave-aggregated atomic on
// counts[4]).  With ppw = 1 a lone long glass path gets its leaves tested 64
// entries at a time instead of one.
template <bool COUNT>
__global__ void __launch_bounds__(WF_BLOCK, WF_FIN_OCC) wf_finish_coop(RtDevScene sc, RtDevFrame fr, RtDevCamera cam, WfState st,
                                                           int q, int ppw, int cap, int postpone, int wide)
{
    __shared__ uint32_t s_node[WF_LDS_STACK * WF_BLOCK];
    __shared__ float s_entry[WF_LDS_STACK * WF_BLOCK];
    __shared__ unsigned long long s_key[WF_BLOCK];
    __shared__ CoopCand s_list[(WF_BLOCK / 64) * WF_COOP_LIST];
    __shared__ int s_mark[2 * WF_BLOCK]; // 128 per wave: chunk_owner marks + junk slots
    __shared__ WideItem s_wide[(WF_BLOCK / 64) * WIDE_CAP];
    const int tid = threadIdx.x;
    const int gtid = blockIdx.x * WF_BLOCK + tid;
    const int lane = __lane_id();
    const int wave = tid >> 6;
    Stack<WF_LDS_STACK> stk{s_node + tid, s_entry + tid, WF_BLOCK, st.spill + gtid, st.spill_threads};
    unsigned long long *wkey = s_key + wave * 64;
    CoopCand *list = s_list + wave * WF_COOP_LIST;
    const CoopLds w{wkey, list, s_mark + wave * 128};
    Cnt c;
    if (COUNT) c.zero();
    const uint32_t n = st.counts[6 + q]; // paths of path list q
    uint32_t *fetch = st.counts + 4;
    const int limit = fr.max_depth > 0 ? fr.max_depth : RT_WATCHDOG_BOUNCES;

    PathRegs p;
    p.slot = 0;
    p.ro = p.rd = rt_v3(0, 0, 0);
    CoopRay r;
    coop_idle(r);
    int hit = -1;
    float bx = 0.0f, by = 0.0f, bz = 0.0f;
    bool active = false;              // the lane holds a path
    bool exhausted = lane >= ppw;     // no more queue entries for this lane
    bool pending = false;             // a finished ray query waiting for shade_step
    while (true) {
        // ---- idle lanes take the next queued paths
        const bool need = !active && !exhausted;
        const unsigned long long m = __ballot(need);
        if (m) {
            const int leader = __ffsll((long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(fetch, (uint32_t)__popcll(m));
            base = __shfl(base, leader);
            if (need) {
                const uint32_t e = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (e >= n) {
                    exhausted = true;
                } else {
                    active = true;
                    first_ray(st, fr, st.q_slot[q][e], p);
                    if (COUNT) c.v[RT_CNT_RAY]++;
                    if (!coop_begin(sc, r, p.ro, p.rd)) {
                        pending = true;
                        hit = -1;
                    }
                }
            }
        }
        while (pending) { // shade, and start the path's next ray (a scene-box miss is shaded at once)
            pending = false;
            if (shade_step<COUNT>(sc, fr, cam, p, hit, bx, by, bz, limit, c)) {
                if (COUNT) c.v[RT_CNT_RAY]++;
                if (!coop_begin(sc, r, p.ro, p.rd)) {
                    pending = true;
                    hit = -1;
                }
            } else {
                store_regs(st, fr, p);
                active = false;
            }
        }
        // here every active lane has a live ray
        const unsigned long long lm = __ballot(r.live);
        if (!lm) {
            if (__all(exhausted)) break;
            continue;
        }
        if (__popcll(lm) <= wide) {
            // few rays left in the wave: each is traced by all 64 lanes, one
            // after the other (wide_resume picks up a ray mid-traversal from
            // its lane's stack) — a cooperative round would advance them
            // together, but at ~5 node fetches per round instead of a level
            // of the whole frontier
            const WideLds W{s_wide + wave * WIDE_CAP, WIDE_CAP, wkey, reinterpret_cast<float *>(wkey + 1), w.mark};
            for (unsigned long long mm = lm; mm; mm &= mm - 1) {
                const int owner = __ffsll((long long)mm) - 1;
                const int ot = wave * 64 + owner;
                const Stack<WF_LDS_STACK> so{s_node + ot, s_entry + ot, WF_BLOCK,
                                             st.spill + blockIdx.x * WF_BLOCK + ot, st.spill_threads};
                int t;
                float x, y, z;
                wide_resume<COUNT>(sc, r, owner, so, W, t, x, y, z, c);
                if (lane == owner) {
                    hit = t;
                    bx = x;
                    by = y;
                    bz = z;
                    r.live = false;
                    pending = true;
                }
            }
            continue;
        }
        if (coop_round<COUNT>(sc, r, stk, w, cap, postpone, hit, bx, by, bz, c)) pending = true;
    }
    if (COUNT) {
        flush_counters(c, fr.counters);
        flush_finish_counters(c, fr.counters);
    }
}

// Long paths (total internal reflection in glass runs to 10^4 bounces and
// more) would otherwise hold up the end of the call one bounce per queue
// iteration or one lane at a time.  Paths deeper than st.long_depth are handed
// to this kernel through the hand-off ring; each wave claims the next
// PUBLISHED entry in order (compare-and-swap on the claim counter, never an
// entry whose publication is still in flight) and runs that path with every
// ray traced by all 64 lanes (wide_trace), lane 0 shading.
//
// Two launch forms:
//  * whole-call mode (st.fin_live != nullptr): ONE persistent launch per call
//    on its own stream, beside the finisher; a wave leaves once every finisher
//    wave of its call is past its last hand-off (fin_live == 0) and every
//    reserved entry is claimed.  It runs a path only to the end of its deep
//    SAMPLE, then returns the pixel to a live finisher (return ring) or, with
//    none alive, runs the pixel's remaining passes itself — including passes
//    that later chained calls owe it (pxo) — and releases it (LONGDONE).
//  * queue mode (fin_live == nullptr): slices on the caller's stream, kicked
//    by the pipelines' host threads; a wave with nothing to claim waits only
//    while another path is running, the final slice drains the rest; a path
//    runs to the end of its pixel's passes.
// Neither form waits for a kernel that is not resident (see the cross-kernel
// waits at WF_FIN_STARTED): a persistent wave waits for its finisher only once
// a finisher wave has started, and closes the ring and leaves when none has
// within WF_LONG_START_TRIPS — so neither can deadlock when the runtime maps
// these streams onto one hardware queue or a profiler serialises dispatches.
template <bool COUNT>
__global__ void __launch_bounds__(WF_BLOCK, WF_LONG_WAVES) wf_long(RtDevScene sc, RtDevFrame fr, RtDevCamera cam, WfState st,
                                                    int final_slice)
{
    __shared__ WideItem s_wide[(WF_BLOCK / 64) * WIDE_CAP];
    __shared__ unsigned long long s_key[(WF_BLOCK / 64) * 4];
    __shared__ int s_mark[2 * WF_BLOCK]; // 128 per wave: chunk_owner marks + junk slots
    if (WF_LONG_PRIO > 0) __builtin_amdgcn_s_setprio(WF_LONG_PRIO);
    const int lane = __lane_id();
    const int wave = threadIdx.x >> 6;
    const WideLds W{s_wide + wave * WIDE_CAP, WIDE_CAP, s_key + wave * 4,
                    reinterpret_cast<float *>(s_key + wave * 4 + 1), s_mark + wave * 128};
    Cnt c;
    if (COUNT) c.zero();
    const int limit = fr.max_depth > 0 ? fr.max_depth : RT_WATCHDOG_BOUNCES;
    uint32_t *const reserved = st.long_ctr, *const claimed = st.long_ctr + 1, *const running = st.long_ctr + 3;
    const bool persist = st.fin_live != nullptr;
    unsigned long long t_idle = __builtin_amdgcn_s_memrealtime(); // (chain window: since entries last flowed)
    unsigned long long t_net = t_idle; // safety net: since anything that could still bring work last held
    unsigned long long t_pub = 0;      // since entry e_pub was first seen reserved but unpublished
    // (the same bounds in loop trips: s_memrealtime stands still under counter collection)
    uint32_t n_idle = 0, n_net = 0, n_pub = 0, n_start = 0;
    uint32_t r_seen = 0, e_pub = 0xffffffffu;
    while (true) {
        // ---- claim the next published entry (lane 0): its tag and ray are read
        // before the claim (a claimed ring slot may be reused at once)
        uint32_t e = 0, slot = 0;
        RtF4 ro4{0, 0, 0, 0}, rd4{0, 0, 0, 0};
        int quit = 0;
        if (lane == 0) {
            while (true) {
                const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                ++n_idle;
                ++n_net;
                // (producers first: once they are all past their last hand-off,
                // `reserved` read after this acquire holds every entry.)  A finisher
                // that has not started is not waited for (WF_LONG_START_TRIPS below)
                const uint32_t fl = persist ? __hip_atomic_load(st.fin_live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                const bool unstarted = persist && !(fl & WF_FIN_STARTED);
                const bool producing = persist && !unstarted && (fl & ~WF_FIN_STARTED) != 0u;
                const bool others = __hip_atomic_load(running, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
                const bool chain_open =
                    persist && __hip_atomic_load(st.chain_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
                if (persist && !producing && !unstarted) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                e = __hip_atomic_load(claimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t rw = __hip_atomic_load(reserved, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool closed = (rw & WF_LONG_CLOSED) != 0u;
                const uint32_t r = rw & ~WF_LONG_CLOSED;
                const bool flowing = r != r_seen;
                if (flowing) { // entries still flowing (to any wave): not idle
                    r_seen = r;
                    t_idle = now;
                    n_idle = 0;
                }
                if (flowing || producing || others) { // work may still come: a bounded wait
                    t_net = now;
                    n_net = 0;
                }
                // done once nothing can bring entries: the ring closed, or the call's finisher
                // past its last hand-off and no chain open (or its window over)
                const bool window_over = (now - t_idle > WF_LONG_CHAIN_IDLE || n_idle > WF_LONG_CHAIN_TRIPS) && !others;
                const bool done = persist && (closed || (!producing && !unstarted && (!chain_open || window_over)));
                if (st.debug_quit) { // (tests: as if the net fired at once)
                    quit = 2;
                    break;
                }
                if (e < r) {
                    const uint32_t k = e % st.long_cap;
                    const unsigned long long v =
                        __hip_atomic_load(st.long_ent + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((uint32_t)(v >> 32) == e + 1u) { // published: acquire, read, then claim
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        ro4 = ldf4(st.long_ray + 2 * (size_t)k);
                        rd4 = ldf4(st.long_ray + 2 * (size_t)k + 1);
                        slot = (uint32_t)v;
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        uint32_t expect = e;
                        if (__hip_atomic_compare_exchange_strong(claimed, &expect, e + 1u, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                            __hip_atomic_fetch_add(running, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                        continue; // another wave took it: try the next one
                    }
                    // reserved, its publication still in flight: wait for it (safety net: 1 s)
                    if (e != e_pub) {
                        e_pub = e;
                        t_pub = now;
                        n_pub = 0;
                    } else if (now - t_pub > WF_LONG_PUBLISH_WAIT || ++n_pub > WF_LONG_PUBLISH_TRIPS) {
                        quit = 2;
                        break;
                    }
                } else {
                    // nothing claimable.  Persistent: done once nothing can bring entries; slices: the
                    // final one once every entry is claimed, the others unless a path still runs.
                    if (persist ? done : (final_slice || !others)) {
                        quit = 1;
                        break;
                    }
                    // the call's finisher has not started: it may be dispatched only after this kernel
                    // ends (serialised dispatch).  After WF_LONG_START_TRIPS such trips close the ring —
                    // atomically with the reservations, so only while every entry is claimed — and
                    // leave: the finisher then keeps its deep paths
                    if (unstarted && !closed && ++n_start > WF_LONG_START_TRIPS) {
                        uint32_t x = r;
                        if (__hip_atomic_compare_exchange_strong(reserved, &x, r | WF_LONG_CLOSED, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                            atomicAdd(fr.dev_stats + RT_DEV_LONG_CLOSED, 1ull);
                            quit = 1;
                            break;
                        }
                        continue; // a reservation came in: serve it
                    }
                }
                if (now - t_net > WF_LONG_IDLE || n_net > WF_LONG_IDLE_TRIPS) { // safety net (see WF_LONG_IDLE)
                    quit = e < r ? 2 : 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(16);
            }
            if (!quit) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (quit == 2) atomicAdd(fr.dev_stats + RT_DEV_LONG_QUIT, 1ull); // entries left unclaimed: stranded
        }
        // (lane 0's values, wave-uniform: readfirstlane — every lane is active here)
        if (__builtin_amdgcn_readfirstlane(quit)) break;
        e = (uint32_t)__builtin_amdgcn_readfirstlane((int)e);
        // ---- run the path (state in lane 0)
        PathRegs p;
        p.slot = 0;
        p.ro = p.rd = rt_v3(0, 0, 0);
        if (lane == 0) {
            load_regs(st, fr, slot, p);
            p.ro = ld3(ro4);
            p.rd = ld3(rd4);
        }
        int want = 0; // after the loop: 0 the pixel's passes are done, 2 returned to the finishers
        uint32_t ret_e = 0;
        const unsigned long long t_claim = __builtin_amdgcn_s_memrealtime();
        uint32_t bounces = 0;
        while (true) {
            ++bounces;
            int hit = -1;
            float bx = 0.0f, by = 0.0f, bz = 0.0f;
            CoopRay r;
            coop_idle(r);
            if (lane == 0) {
                if (COUNT) c.v[RT_CNT_RAY]++;
                coop_begin(sc, r, p.ro, p.rd);
            }
            if (__shfl((int)r.live, 0)) {
                const Vec3D o = rt_v3(__shfl(r.o.x, 0), __shfl(r.o.y, 0), __shfl(r.o.z, 0));
                const Vec3D d = rt_v3(__shfl(r.d.x, 0), __shfl(r.d.y, 0), __shfl(r.d.z, 0));
                const float en = __shfl(r.entry, 0), ex = __shfl(r.exit_, 0);
                // entered at the origin's grid cell (kd_origin_frontier), else from the root
                const int nf = !COUNT && sc.kd_grid > 0 ? kd_origin_frontier(sc, o, d, en, ex, W) : 0;
                if (nf > 0) wide_trace_from<COUNT>(sc, o, d, nf, W, lane == 0, hit, bx, by, bz, c);
                else wide_trace<COUNT>(sc, o, d, en, ex, W, lane == 0, hit, bx, by, bz, c);
            }
            want = 0;
            if (lane == 0) {
                want = shade_step<COUNT>(sc, fr, cam, p, hit, bx, by, bz, limit, c) ? 1 : 0;
                if (!want && st.long_return) {
                    // the pixel's passes are done: run the passes chained calls owe it, or
                    // release it — its state stored and released before the word says so
                    while (true) {
                        store_regs(st, fr, p);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                        uint32_t x = RT_PX_OUT;
                        if (__hip_atomic_compare_exchange_strong(st.pxo + p.slot, &x, RT_PX_LONGDONE, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                            break;
                        x = __hip_atomic_exchange(st.pxo + p.slot, RT_PX_OUT, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
                        p.passes_left = (int)(x & RT_PX_PASSES);
                        if (x & RT_PX_PASSES) { // (RtDeviations: owed passes, run here in the pixel's order)
                            atomicAdd(fr.dev_stats + RT_DEV_OWED_PIXELS, 1ull);
                            atomicAdd(fr.dev_stats + RT_DEV_OWED_PASSES, (unsigned long long)(x & RT_PX_PASSES));
                        }
                        const Vec3D fb = fr.fb[p.slot];
                        const float sq = fr.sq[p.slot];
                        const int count = fr.count[p.slot];
                        if (start_sample<COUNT>(fr, cam, (int)p.slot, p.passes_left, p.rng, fb, sq, count, p.ro, p.rd,
                                                c)) { // as shade_step's next pass
                            p.T = rt_v3(1.0f, 1.0f, 1.0f);
                            p.L = rt_v3(0.0f, 0.0f, 0.0f);
                            p.inside = false;
                            p.prev_type = PRIMARY;
                            p.depth = 1;
                            p.shadow = false;
                            want = 1;
                            break;
                        }
                    }
                }
                // return mode: the deep sample is over once the pixel's next one starts (depth 1);
                // the pixel goes back to the finishers if one is still alive to take it.  While a
                // chain is open: always — this call's, the next call's or the chain's drain
                // finisher takes it (a finisher in its tail takes none: a returned pixel's whole
                // remaining chain would hold up the call's end and the next call's start).  The
                // drain finisher lingers (WF_FIN_LINGER) while a pixel is out, so a return
                // reserved just as its clear of the flag lands is still taken.
                if (want && st.long_return && p.depth == 1 && !p.shadow) {
                    unsigned long long *const ret_word = reinterpret_cast<unsigned long long *>(st.ret_ctr);
                    if (st.linger == 0ull &&
                        __hip_atomic_load(st.chain_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
                        want = 2;
                        ret_e = (uint32_t)__hip_atomic_fetch_add(ret_word, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    unsigned long long w = __hip_atomic_load(ret_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    while (want != 2 && (w >> 32) != 0ull) {
                        if (__hip_atomic_compare_exchange_strong(ret_word, &w, w + 1ull, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                            want = 2;
                            ret_e = (uint32_t)w;
                            break;
                        }
                    }
                }
            }
            want = __builtin_amdgcn_readfirstlane(want);
            if (want != 1) break;
        }
        if (lane == 0) {
            if (st.long_log && e < 65535u) {
                unsigned long long *L = st.long_log + 4 + 4 * (size_t)e;
                L[0] = t_claim;
                L[1] = __builtin_amdgcn_s_memrealtime();
                L[2] = bounces;
                L[3] = p.slot;
            }
            if (want == 2) { // back to the finishers: its state and next ray, then its ring entry
                store_regs(st, fr, p);
                st.ro[p.slot] = p.ro;
                st.cont[p.slot] = p.rd;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(st.ret_ring + ret_e % st.long_cap, ((unsigned long long)(ret_e + 1u) << 32) | p.slot,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (st.long_return) { // done and released above (its state may already be another's)
                __hip_atomic_fetch_sub(st.ret_ctr + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                store_regs(st, fr, p);
            }
            __hip_atomic_fetch_sub(running, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        t_idle = __builtin_amdgcn_s_memrealtime();
        n_idle = 0;
    }
    if (COUNT) flush_counters(c, fr.counters);
}

// ---------------------------------------------------------------- launcher
void rt_register_shutdown(); // abi.hip: rt_shutdown at exit, before the HIP runtime's finalisers

namespace {

// One pipeline = its own ray queues, hits, counters, stack spill area and
// HIP stream over a disjoint set of 16x16 pixel tiles (tile % npipes).  The
// pipelines run concurrently (one host thread each), so the latency-bound
// tail of one pipeline's trace launches and its finisher overlap the other
// pipelines' bulk work.  Per-pixel path state is shared (pixels are disjoint).
// The whole-call mode uses pipeline 0 and runs its persistent wf_long on
// pipeline 1's or 2's stream (alternating per call: a chained call's wf_long
// may start while the previous one still runs deep paths).
struct Pipe {
    std::vector<std::pair<float, float>> trace_iv; // profiled trace launches: [start, end] ms after the call's start
    WfState st{};
    hipStream_t stream = nullptr;
    uint32_t *host_count = nullptr;
    hipEvent_t ev[6] = {};   // RtOptions.profile
    hipEvent_t join = nullptr;
    hipEvent_t fin_done = nullptr; // after the finisher (the host polls it while kicking wf_long slices)
    hipEvent_t long_done = nullptr; // whole-call mode: after a persistent wf_long on this stream
    bool joined = false; // join recorded by a previous call
    bool long_rec = false; // long_done recorded by a previous call
    RtProfile prof{};
};

// the frame a chained call continues (RtOptions.overlap): everything a pixel's
// passes depend on besides its own G_Buffer state
struct ChainKey {
    const void *nodes, *bvh, *fb, *sq, *count, *rng;
    int width, height, adaptive, min_samples, max_depth, shard_id, num_shards, long_depth;
    float tolerance;
    RtDevCamera cam;
};

ChainKey chain_key(const RtDevScene &sc, const RtDevFrame &fr, const RtDevCamera &cam, int long_depth)
{
    ChainKey key;
    memset(&key, 0, sizeof key);
    key.nodes = sc.nodes;
    key.bvh = sc.bvh_nodes;
    key.fb = fr.fb;
    key.sq = fr.sq;
    key.count = fr.count;
    key.rng = fr.rng;
    key.width = fr.width;
    key.height = fr.height;
    key.adaptive = fr.adaptive;
    key.min_samples = fr.min_samples;
    key.max_depth = fr.max_depth;
    key.shard_id = fr.shard_id;
    key.num_shards = fr.num_shards;
    key.long_depth = long_depth;
    key.tolerance = fr.tolerance;
    key.cam = cam;
    return key;
}

// Chained calls of fewer passes than RtOptions.coalesce_passes are coalesced
// on the host: such a call is recorded (its passes added to the pending batch
// of the same frame, options and stream) and the batch is launched as ONE
// chained call once it holds that many passes, or before anything that must
// see it (any other call, a join — rt_join and the library's readers —, the
// profile readers, rt_shutdown).  k chained calls of p passes are the same
// per-pixel pass sequence as one call of k*p passes: bit-identical.
struct Pending {
    bool on = false;
    int dev = 0;
    RtDevScene sc{};
    RtDevFrame fr{};
    RtDevCamera cam{};
    hipStream_t stream = nullptr;
    int long_depth = 0, debug = 0, calls = 0;
    bool prof = false;
    uint32_t check_mask = 0;
    ChainKey key{};
};

struct Workspace {
    Pending pend; // coalesced chained calls not yet launched
    size_t slots = 0;
    int grid = 0;
    int spill_pipes = 0;
    void *blob = nullptr;
    Pipe pipe[WF_MAX_PIPES];
    bool streams_ok = false;
    hipEvent_t fork = nullptr, ev0 = nullptr, ev1 = nullptr, fin_ready = nullptr;
    hipEvent_t long_ev = nullptr; // after the last wf_long slice on the caller's stream (queue mode)
    bool recorded = false;   // long_ev recorded by a previous call
    uint32_t *fin_live = nullptr; // 8 producer words (whole-call mode, one per call in flight: call % 8)
    uint32_t *heavy_list = nullptr; // (WfState.heavy_list: every pixel at most once)
    RtF4 *chk = nullptr;          // the exactness guard's records (2 x chk_cap x 3 RtF4; allocated on the
                                  // first call with the guard on, regrown for a larger frame) and their counter
    uint32_t chk_cap = 0;
    uint32_t *chk_ctr = nullptr;
    // the join's hand-off check (wf_verify): its result words (own allocation: they outlive a
    // blob reallocation), a whole call with the hand-off ran since the last check, a check's
    // result not yet read by a host join
    uint32_t *verify_res = nullptr;
    bool verify_pending = false;
    bool verify_unread = false;
    // after the last wf_verify (on whatever stream joined): every later launch on the workspace,
    // and the host's read of verify_res, wait for it — it rewrites every pixel's ownership word
    hipEvent_t verify_ev = nullptr;
    bool verify_rec = false;
    int cus = 0;                                // compute units of the device (the finisher's grid)
    unsigned long long *long_log_buf = nullptr; // RT_DEBUG_LONG_LOG records
    // the guard's wf_check per record parity on pipeline 2: the event after it (the call two
    // later, whose finisher writes the same records, waits for it)
    hipEvent_t chk_done[2] = {};
    bool chk_rec[2] = {false, false};
    // RtOptions.profile of whole calls: per profiled call its finisher's span on the device
    // ({first wave start, last wave end}, s_memrealtime) in a ring of WF_PROF_SLOTS, resolved
    // into RtProfile records by rt_last_profile / rt_profile_history (they join first)
    unsigned long long *spans = nullptr;
    unsigned long long prof_seq = 0;
    struct PendingProf {
        unsigned long long seq;
        int passes;
    };
    std::vector<PendingProf> prof_pending;
    std::vector<RtProfile> prof_hist; // resolved, since the last rt_profile_history reset (the newest
                                      // WF_PROF_HISTORY: a profiling caller that never reads it stays bounded)
    unsigned long long call_seq = 0;
    bool chain_open = false; // the last call was a whole-call call with RtOptions.overlap
    ChainKey key{};
    // the open chain's last call (its drain runs with them)
    RtDevScene last_sc{};
    RtDevFrame last_fr{};
    RtDevCamera last_cam{};
    int last_long_depth = 0;
    int last_debug = 0;
    RtProfile prof{};        // last profiled call
};

std::mutex g_ws_mu;
std::map<int, Workspace *> g_ws; // per device (owned; released by rt_shutdown)

Workspace &workspace(int dev)
{
    std::lock_guard<std::mutex> g(g_ws_mu);
    Workspace *&w = g_ws[dev];
    if (!w) w = new Workspace();
    return *w;
}

__global__ void wf_bind_stream() {}

// the pipelines' streams (created on first use, each bound to its hardware
// queue by an empty launch: the runtime maps a stream to a queue when it is
// first used, and streams created later share queues once the process has
// used its GPU_MAX_HW_QUEUES)
int ensure_streams(Workspace &w, int npipes)
{
    if (!w.streams_ok) {
        if (hipEventCreateWithFlags(&w.fork, hipEventDisableTiming) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&w.fin_ready, hipEventDisableTiming) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&w.long_ev, hipEventDisableTiming) != hipSuccess) return -1;
        if (hipEventCreate(&w.ev0) != hipSuccess || hipEventCreate(&w.ev1) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&w.verify_ev, hipEventDisableTiming) != hipSuccess) return -1;
        if (hipMalloc((void **)&w.verify_res, 64) != hipSuccess || hipMemset(w.verify_res, 0, 64) != hipSuccess)
            return -1;
        for (auto &e : w.chk_done)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return -1;
        w.streams_ok = true;
    }
    for (int i = 0; i < npipes && i < WF_MAX_PIPES; ++i) {
        Pipe &p = w.pipe[i];
        if (p.stream) continue;
        if (hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking) != hipSuccess) return -1;
        if (hipHostMalloc((void **)&p.host_count, 64) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&p.join, hipEventDisableTiming) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&p.fin_done, hipEventDisableTiming) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&p.long_done, hipEventDisableTiming) != hipSuccess) return -1;
        for (auto &e : p.ev)
            if (hipEventCreate(&e) != hipSuccess) return -1;
        hipLaunchKernelGGL(wf_bind_stream, dim3(1), dim3(64), 0, p.stream);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(p.stream) != hipSuccess) return -1;
    }
    return 0;
}

int launch_drain(Workspace &w);
int flush_pending(Workspace &w);

#define WF_PROF_SLOTS 256 // profiled whole calls in flight before their spans are read back

// RtOptions.profile of a whole call: a span slot ({~0, 0}: the finisher's waves atomicMin their
// start and atomicMax their end into it), reset on the finisher's stream
int resolve_profiles(Workspace &w);
int prof_slot(Workspace &w, hipStream_t s, unsigned long long **span, int passes)
{
    if (!w.spans && hipMalloc((void **)&w.spans, 2 * sizeof(unsigned long long) * WF_PROF_SLOTS) != hipSuccess) {
        w.spans = nullptr;
        return -1;
    }
    if (w.prof_pending.size() >= WF_PROF_SLOTS && resolve_profiles(w) != 0) return -1;
    unsigned long long *p = w.spans + 2 * (size_t)(w.prof_seq % WF_PROF_SLOTS);
    if (hipMemsetD32Async((hipDeviceptr_t)p, (int)0xFFFFFFFF, 2, s) != hipSuccess ||
        hipMemsetAsync(p + 1, 0, 8, s) != hipSuccess)
        return -1;
    w.prof_pending.push_back({w.prof_seq, passes});
    ++w.prof_seq;
    *span = p;
    return 0;
}

#define WF_PROF_HISTORY 65536
void push_history(Workspace &w, const RtProfile &P)
{
    if (w.prof_hist.size() >= WF_PROF_HISTORY) // (drop the oldest half: amortised O(1))
        w.prof_hist.erase(w.prof_hist.begin(), w.prof_hist.begin() + WF_PROF_HISTORY / 2);
    w.prof_hist.push_back(P);
}

// the pending profiled whole calls' spans -> RtProfile records (waits for their finishers)
int resolve_profiles(Workspace &w)
{
    if (w.prof_pending.empty()) return 0;
    for (int pi : {0, 2})
        if (w.pipe[pi].stream && hipStreamSynchronize(w.pipe[pi].stream) != hipSuccess) return -1;
    std::vector<unsigned long long> sp(2 * WF_PROF_SLOTS);
    if (hipMemcpy(sp.data(), w.spans, sp.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    unsigned long long base = ~0ull; // (start_ms: relative to the earliest finisher start of the batch)
    for (const auto &q : w.prof_pending) base = std::min(base, sp[2 * (q.seq % WF_PROF_SLOTS)]);
    for (const auto &q : w.prof_pending) {
        const unsigned long long a = sp[2 * (q.seq % WF_PROF_SLOTS)], b = sp[2 * (q.seq % WF_PROF_SLOTS) + 1];
        RtProfile P{};
        P.start_ms = b > a ? (float)((double)(a - base) * 1e-5) : 0.0f;
        P.finish_launches = 1;
        P.pipelines = 1;
        P.finish_ms = b > a ? (float)((double)(b - a) * 1e-5) : 0.0f; // (s_memrealtime: 100 MHz)
        P.call_ms = P.finish_ms;
        push_history(w, P);
        w.prof = P;
    }
    w.prof_pending.clear();
    return 0;
}

int ensure(Workspace &w, size_t slots, int grid, int npipes)
{
    if (ensure_streams(w, npipes > WF_PIPES_DEFAULT ? npipes : WF_PIPES_DEFAULT) != 0) return -1;
    if (w.slots >= slots && w.grid >= grid && w.spill_pipes >= npipes) return 0;
    // traversal stack spill for the pipelines in use (at least the default 3)
    const int spill_pipes = npipes > WF_PIPES_DEFAULT ? npipes : WF_PIPES_DEFAULT;
    if (w.blob) {
        // (an open chain drained first: its wf_longs use the old blob until then)
        if (launch_drain(w) != 0) return -1;
        (void)hipDeviceSynchronize();
        (void)hipFree(w.blob);
    }
    w.blob = nullptr;
    const size_t spill_threads = (size_t)grid * WF_BLOCK;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    // per pixel
    const size_t o_pl = take(slots * 4), o_fl = take(slots * 4), o_T = take(slots * 12), o_L = take(slots * 12),
                 o_c = take(slots * 12), o_n = take(slots * 12), o_rp = take(slots * 12), o_li = take(slots * 4),
                 o_ro = take(slots * 12), o_es = take(slots * 4), o_ee = take(slots * 4), o_px = take(slots * 4),
                 o_hv = take(slots), o_ls = take(slots * 4), o_hl = take(slots * 4), o_hn = take(256);
    // long-path hand-off (shared by the pipelines), wf_long's stack-free wide traversal needs no spill
    const size_t o_le = take(slots * 8), o_lr = take(slots * 32), o_lc = take(256), o_rr = take(slots * 8),
                 o_rc = take(256), o_ctl = take(256);
    // per pipeline (path lists sized for every pixel: a pipeline never holds
    // more; ray queues for two rays per path: a shadow and an extension ray)
    size_t o_qs0[WF_MAX_PIPES], o_qs1[WF_MAX_PIPES], o_qr0[WF_MAX_PIPES], o_qr1[WF_MAX_PIPES], o_h[WF_MAX_PIPES],
        o_cnt[WF_MAX_PIPES], o_sp[WF_MAX_PIPES];
    for (int i = 0; i < WF_MAX_PIPES; ++i) {
        o_qs0[i] = take(slots * 4);
        o_qs1[i] = take(slots * 4);
        o_qr0[i] = take(2 * slots * 32);
        o_qr1[i] = take(2 * slots * 32);
        o_h[i] = take(2 * slots * 16);
        o_cnt[i] = take(256);
        o_sp[i] = i < spill_pipes ? take(spill_threads * 8 * WF_SPILL_ENTRIES) : 0;
    }
    if (hipMalloc(&w.blob, off) != hipSuccess) {
        w.blob = nullptr;
        return -1;
    }
    char *b = (char *)w.blob;
    if (hipMemset(b + o_px, 0, slots * 4) != hipSuccess) return -1; // no pixel out
    if (hipMemset(b + o_hv, 0, slots) != hipSuccess || hipMemset(b + o_ls, 0, slots * 4) != hipSuccess ||
        hipMemset(b + o_hn, 0, 256) != hipSuccess)
        return -1; // no pixel heavy or listed yet
    if (hipMemset(b + o_ctl, 0, 256) != hipSuccess) return -1;
    w.fin_live = (uint32_t *)(b + o_ctl);
    w.chk_ctr = (uint32_t *)(b + o_ctl + 64);
    w.chain_open = false;
    for (int i = 0; i < WF_MAX_PIPES; ++i) {
        WfState &st = w.pipe[i].st;
        st.passes_left = (int *)(b + o_pl);
        st.flags = (uint32_t *)(b + o_fl);
        st.T = (Vec3D *)(b + o_T);
        st.L = (Vec3D *)(b + o_L);
        st.cont = (Vec3D *)(b + o_c);
        st.snorm = (Vec3D *)(b + o_n);
        st.rp = (Vec3D *)(b + o_rp);
        st.light = (int *)(b + o_li);
        st.ro = (Vec3D *)(b + o_ro);
        st.e_sh = (uint32_t *)(b + o_es);
        st.e_ext = (uint32_t *)(b + o_ee);
        st.q_slot[0] = (uint32_t *)(b + o_qs0[i]);
        st.q_slot[1] = (uint32_t *)(b + o_qs1[i]);
        st.q_ray[0] = (RtF4 *)(b + o_qr0[i]);
        st.q_ray[1] = (RtF4 *)(b + o_qr1[i]);
        st.hits = (RtF4 *)(b + o_h[i]);
        st.counts = (uint32_t *)(b + o_cnt[i]);
        st.spill = i < spill_pipes ? (uint2 *)(b + o_sp[i]) : nullptr;
        st.spill_threads = (int)spill_threads;
        st.long_ctr = (uint32_t *)(b + o_lc);
        st.long_ent = (unsigned long long *)(b + o_le);
        st.long_ray = (RtF4 *)(b + o_lr);
        st.long_depth = 0;
        st.long_cap = (uint32_t)slots;
        st.long_return = 0;
        st.ret_ring = (unsigned long long *)(b + o_rr);
        st.ret_ctr = (uint32_t *)(b + o_rc);
        st.linger = WF_FIN_LINGER;
        st.pxo = (uint32_t *)(b + o_px);
        st.heavy = (uint8_t *)(b + o_hv);
        st.listed = (uint32_t *)(b + o_ls);
        st.heavy_list = nullptr; // (set per call by launch_whole)
        w.heavy_list = (uint32_t *)(b + o_hl);
        st.heavy_n = (uint32_t *)(b + o_hn);
        st.fin_live = nullptr;
        st.chain_flag = (uint32_t *)(b + o_ctl + 128);
        st.fresh = 0;
        st.fresh_n = 0;
        st.span = nullptr;
        st.call_id = 0;
        st.chk = nullptr; // (whole-call mode only: launch_whole)
        st.chk_ctr = nullptr;
        st.chk_mask = 0;
        st.chk_cap = 0;
        st.chk_fault = 0;
        st.debug_quit = 0;
    }
    w.slots = slots;
    w.grid = grid;
    w.spill_pipes = spill_pipes;
    return 0;
}

float elapsed_ms(hipEvent_t a, hipEvent_t b)
{
    float ms = 0.0f;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.0f;
}

// the hand-off check (wf_verify) on `stream`, which has waited for all the workspace's work
int launch_verify(Workspace &w, hipStream_t stream)
{
    if (!w.verify_pending || !w.blob) return 0;
    w.verify_pending = false;
    const int blocks = (int)std::min<size_t>((w.slots + WF_BLOCK - 1) / WF_BLOCK, 1024);
    hipLaunchKernelGGL(wf_verify, dim3(blocks), dim3(WF_BLOCK), 0, stream, w.pipe[0].st, (uint32_t)w.slots,
                       w.verify_res, w.last_fr.dev_stats);
    if (hipGetLastError() != hipSuccess) return -1;
    // (every later launch on the workspace waits for it: join_all; and so does the host's read of its result)
    if (hipEventRecord(w.verify_ev, stream) != hipSuccess) return -1;
    w.verify_rec = true;
    w.verify_unread = true;
    return 0;
}

// `stream` waits for every call's device work on this workspace (the
// pipelines' last launches and every wf_long), an open chain drained first,
// and for the last hand-off check (which another stream may have run: it
// rewrites every ownership word); then the hand-off check runs on it
int join_all(Workspace &w, hipStream_t stream)
{
    if (launch_drain(w) != 0) return -1;
    if (w.verify_rec && hipStreamWaitEvent(stream, w.verify_ev, 0) != hipSuccess) return -1;
    for (int pi = 0; pi < WF_MAX_PIPES; ++pi) {
        Pipe &p = w.pipe[pi];
        if (p.joined && hipStreamWaitEvent(stream, p.join, 0) != hipSuccess) return -1;
        if (p.long_rec && hipStreamWaitEvent(stream, p.long_done, 0) != hipSuccess) return -1;
    }
    if (w.recorded && hipStreamWaitEvent(stream, w.long_ev, 0) != hipSuccess) return -1;
    return launch_verify(w, stream);
}

int debug_long_log(Workspace &w, unsigned long long *buf);

// The whole call in one persistent finisher (bounded traversal, the default):
// wf_finish_bvh takes the call's pixels itself (a lane claims a pixel, runs
// its passes to the end, one path at a time, and takes the next pixel), deep
// paths go to ONE persistent wf_long beside it, and wf_check re-traces the
// guard's sample after it.  Nothing here waits on the host: the call is
// enqueued and returns.
//
// RtOptions.overlap (chained calls): a call of the same frame as the previous
// overlapping call does not wait for that call at all.  Its finisher runs on
// the other of two finisher streams (pipelines 0 and 2), so it starts in the
// slots the previous finisher's tail frees, and a pixel still held there —
// by a previous finisher lane (BUSY) or by wf_long (OUT) — is owed this
// call's passes, which its holder runs before it lets go.  The caller's stream
// does not wait for the call either: rt_join and the library's readers of the
// frame do.  Results are bit-identical to unchained calls: a pixel's passes run
// in order whoever runs them.
int launch_whole_now(Workspace &w, int dev, const RtDevScene &sc, const RtDevFrame &fr, const RtDevCamera &cam,
                     hipStream_t stream, int long_depth, bool prof, bool overlap, uint32_t check_mask, int debug,
                     bool count)
{
    const size_t slots = (size_t)fr.width * fr.height;
    // a resetting call (sample_count 0) neither continues nor opens a chain: its reset of a pixel
    // must come before any later pass, and a chained lane may reach a pixel before it does
    overlap = overlap && !fr.reset;
    // every wave slot at the finisher's occupancy (MI355X: 256 CUs x 4 SIMDs x 4 waves / 4 waves per
    // block = 1,024 blocks), the last WF_LONG_BLOCKS of them left to wf_long
    if (!w.cus) {
        hipDeviceProp_t prop;
        w.cus = hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0
                    ? prop.multiProcessorCount
                    : 256;
    }
    const int grid = w.cus * 4 * WF_FIN_BVH_WAVES / (WF_BLOCK / 64);
    const ChainKey key = chain_key(sc, fr, cam, long_depth);
    const bool chained = overlap && w.chain_open && !fr.reset && memcmp(&key, &w.key, sizeof key) == 0;
    // a fresh call: an open chain drained and every earlier call's work on the
    // workspace first (before a larger frame's workspace replaces the old one)
    if (!chained && join_all(w, stream) != 0) return -1;
    if (ensure(w, slots, grid, 1) != 0) return -1;
    // the finisher's stream (chained calls' finishers one after the other on it); its counters,
    // its stack spill area and its guard records go with it
    Pipe &pp = w.pipe[0];
    WfState st = pp.st;
    const int long_return = long_depth > 0 ? 1 : 0;
    st.long_depth = long_depth;
    st.long_return = long_return;
    st.fresh = 1;
    st.fresh_n = (uint32_t)(((fr.width + 15) / 16) * ((fr.height + 15) / 16)) * 256u;
    st.linger = overlap ? 0ull : WF_FIN_LINGER;
    st.chk_mask = check_mask;
    // the guard's records per call parity (the call two later reuses them after this call's wf_check),
    // sized from the call's rays: <= 8 rays per sample (deep paths go to wf_long; owed passes are few)
    // / the sampling interval, so a small frame does not hold the 2 x 4M-record maximum
    const int par = (int)(w.call_seq & 1);
    if (check_mask != 0xFFFFFFFFu) {
        const unsigned long long want = (unsigned long long)slots * (unsigned long long)fr.passes * 8ull /
                                        ((unsigned long long)check_mask + 1ull);
        uint32_t cap = 1u << 16;
        while (cap < want && cap < WF_CHECK_CAP) cap <<= 1;
        if (cap > w.chk_cap) { // (grown: after every wf_check that reads the old records)
            if (w.chk) {
                if (hipDeviceSynchronize() != hipSuccess) return -1;
                (void)hipFree(w.chk);
                w.chk = nullptr;
                w.chk_cap = 0;
            }
            if (hipMalloc((void **)&w.chk, 2 * (size_t)cap * 3 * sizeof(RtF4)) != hipSuccess) {
                w.chk = nullptr;
                return -1;
            }
            w.chk_cap = cap;
        }
    }
    st.chk = check_mask == 0xFFFFFFFFu ? nullptr : w.chk + 3 * (size_t)w.chk_cap * (size_t)par;
    st.chk_cap = w.chk_cap;
    st.chk_ctr = w.chk_ctr + par;
    st.chk_fault = (debug & RT_DEBUG_CHECK_FAULT) ? 1 : 0;
    st.debug_quit = (debug & RT_DEBUG_LONG_QUIT) ? 1 : 0;
    // debug (RT_DEBUG_LONG_LOG): every deep sample's claim / end time and bounces
    if ((debug & RT_DEBUG_LONG_LOG) && !w.long_log_buf &&
        hipMalloc((void **)&w.long_log_buf, 8 * 4 * 65536) != hipSuccess) {
        w.long_log_buf = nullptr;
        return -1;
    }
    unsigned long long *const long_log_buf = w.long_log_buf;
    st.long_log = (debug & RT_DEBUG_LONG_LOG) ? long_log_buf : nullptr;
    // the finisher: every wave slot but wf_long's blocks, at most one lane per pixel
    int fgrid = (int)((slots + WF_BLOCK - 1) / WF_BLOCK);
    const int fmax = long_return ? grid - WF_LONG_BLOCKS : grid;
    fgrid = fgrid > fmax ? fmax : fgrid;
    const uint32_t k = (uint32_t)(w.call_seq % 8);
    st.fin_live = long_return ? w.fin_live + k : nullptr;
    st.call_id = (uint32_t)w.call_seq + 1u;
    if (!chained) {
        // the hand-off state from zero (nothing of it is in flight now; a ring a wf_long closed reopens)
        if (long_return) {
            // (the rings' whole capacity: the workspace may be sized for an earlier, larger frame, and a
            // stale tag beyond this frame's pixel count would look published to wf_long / the finishers)
            if (hipMemsetAsync(st.long_ctr, 0, 256, stream) != hipSuccess) return -1;
            if (hipMemsetAsync(st.long_ent, 0, (size_t)st.long_cap * 8, stream) != hipSuccess) return -1;
            if (hipMemsetAsync(st.ret_ring, 0, (size_t)st.long_cap * 8, stream) != hipSuccess) return -1;
            if (hipMemsetAsync(st.ret_ctr, 0, 256, stream) != hipSuccess) return -1;
        }
        if (st.long_log && hipMemsetAsync(long_log_buf, 0, 8 * 4 * 65536, stream) != hipSuccess) return -1;
    }
    ++w.call_seq;
    // fork: the finisher's stream starts after the caller's stream
    const hipStream_t s = pp.stream;
    if (hipEventRecord(w.fork, stream) != hipSuccess || hipStreamWaitEvent(s, w.fork, 0) != hipSuccess) return -1;
    if (hipMemsetAsync(st.counts, 0, 256, s) != hipSuccess) return -1;
    // (the producers' word: the finisher's wave count, no wave started yet)
    if (st.fin_live && hipMemsetD32Async((hipDeviceptr_t)st.fin_live, (int)(fgrid * (WF_BLOCK / 64)), 1, s) != hipSuccess)
        return -1;
    if (st.chk) { // (this parity's records: after the wf_check that last read them)
        if (w.chk_rec[par] && hipStreamWaitEvent(s, w.chk_done[par], 0) != hipSuccess) return -1;
        if (hipMemsetAsync(st.chk_ctr, 0, 4, s) != hipSuccess) return -1;
    }
    if (long_return && hipMemsetD32Async((hipDeviceptr_t)st.chain_flag, overlap ? 1 : 0, 1, s) != hipSuccess) return -1;
    // RtOptions.profile: the finisher's span on the device (first wave start, last wave end)
    st.span = nullptr;
    if (prof) {
        if (prof_slot(w, s, &st.span, fr.passes) != 0) return -1;
    }
    // heavy pixels first (wf_heavy_list): listed and tagged with this call before the finisher
    st.heavy_list = nullptr;
    if (long_return && w.heavy_list && WF_HEAVY_FIRST) {
        st.heavy_list = w.heavy_list;
        if (hipMemsetAsync(st.heavy_n, 0, 4, s) != hipSuccess) return -1;
        // two classes: pixels handed over WF_HEAVY_SPLIT+ times so far, then the others
        hipLaunchKernelGGL(wf_heavy_list, dim3(WF_HEAVY_BLOCKS), dim3(WF_BLOCK), 0, s, fr, st, st.call_id,
                           (uint32_t)WF_HEAVY_SPLIT, 256u);
        hipLaunchKernelGGL(wf_heavy_list, dim3(WF_HEAVY_BLOCKS), dim3(WF_BLOCK), 0, s, fr, st, st.call_id, 1u,
                           (uint32_t)WF_HEAVY_SPLIT);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (hipEventRecord(w.fin_ready, s) != hipSuccess) return -1;
    Pipe *lp = long_return ? &w.pipe[1] : nullptr;
    // wf_long on pipeline 1's stream, after the finisher's set-up.  Normally it starts beside the
    // finisher; nothing relies on that (serialised dispatch runs either alone, in either order:
    // see the cross-kernel waits at WF_FIN_STARTED).  Debug: force one order —
    // RT_DEBUG_SERIAL_LONG_FIRST runs wf_long to its end before the finisher starts,
    // RT_DEBUG_SERIAL_FIN_FIRST the finisher to its end before wf_long starts
    const bool long_first = lp && (debug & RT_DEBUG_SERIAL_LONG_FIRST);
    const bool fin_first = lp && !long_first && (debug & RT_DEBUG_SERIAL_FIN_FIRST);
    auto launch_long = [&]() -> int {
        if (hipStreamWaitEvent(lp->stream, fin_first ? pp.fin_done : w.fin_ready, 0) != hipSuccess) return -1;
        hipLaunchKernelGGL(wf_long<false>, dim3(WF_LONG_BLOCKS), dim3(WF_BLOCK), 0, lp->stream, sc, fr, cam, st, 1);
        if (hipGetLastError() != hipSuccess) return -1;
        if (hipEventRecord(lp->long_done, lp->stream) != hipSuccess) return -1;
        lp->long_rec = true;
        return 0;
    };
    if (long_first && (launch_long() != 0 || hipStreamWaitEvent(s, lp->long_done, 0) != hipSuccess)) return -1;
    // Counting: the finisher's own work; wf_long's deep paths are not counted
    if (count) hipLaunchKernelGGL(wf_finish_bvh<true>, dim3(fgrid), dim3(WF_BLOCK), 0, s, sc, fr, cam, st, 0);
    else if (fgrid <= w.cus * WF_FIN_SMALL_WAVES)
        hipLaunchKernelGGL((wf_finish_bvh<false, 1>), dim3(fgrid), dim3(WF_BLOCK), 0, s, sc, fr, cam, st, 0);
    else hipLaunchKernelGGL(wf_finish_bvh<false>, dim3(fgrid), dim3(WF_BLOCK), 0, s, sc, fr, cam, st, 0);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipEventRecord(pp.fin_done, s) != hipSuccess) return -1;
    if (lp && !long_first && launch_long() != 0) return -1;
    if (st.chk) {
        // the guard's re-traces on pipeline 2's stream after the finisher, beside whatever follows it on
        // pipeline 0 (the next call's finisher, a chain's drain); its KD stacks in pipeline 2's spill area
        Pipe &cp = w.pipe[2];
        WfState cs = st;
        cs.spill = cp.st.spill;
        if (!cs.spill) return -1;
        if (hipStreamWaitEvent(cp.stream, pp.fin_done, 0) != hipSuccess) return -1;
        hipLaunchKernelGGL(wf_check, dim3(WF_CHECK_BLOCKS), dim3(WF_BLOCK), 0, cp.stream, sc, cs, fr.dev_stats);
        if (hipGetLastError() != hipSuccess) return -1;
        if (hipEventRecord(w.chk_done[par], cp.stream) != hipSuccess || hipEventRecord(cp.join, cp.stream) != hipSuccess)
            return -1;
        w.chk_rec[par] = true;
        cp.joined = true;
    }
    if (hipEventRecord(pp.join, s) != hipSuccess) return -1;
    pp.joined = true;
    // join: unless the call overlaps the next one, the caller's stream continues after the
    // finisher and after its wf_long (the guard's wf_check touches no frame data: its statistics
    // are read by rt_deviation_stats, which joins it)
    if (!overlap) {
        if (hipStreamWaitEvent(stream, pp.join, 0) != hipSuccess) return -1;
        if (lp && hipStreamWaitEvent(stream, lp->long_done, 0) != hipSuccess) return -1;
    }
    w.chain_open = overlap && long_return;
    w.verify_pending = w.verify_pending || long_return;
    w.key = key;
    w.last_sc = sc;
    w.last_fr = fr;
    w.last_fr.reset = 0;
    w.last_cam = cam;
    w.last_long_depth = long_depth;
    w.last_debug = debug;
    if (debug & RT_DEBUG_CALL_LOG) {
        (void)hipStreamSynchronize(s);
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        uint32_t lc[4] = {}, rc4[7] = {};
        (void)hipMemcpy(lc, st.long_ctr, sizeof lc, hipMemcpyDeviceToHost);
        (void)hipMemcpy(rc4, st.ret_ctr, sizeof rc4, hipMemcpyDeviceToHost);
        fprintf(stderr,
                "[wf] call %llu%s finisher done t %.4f; long entries %u claimed %u running %u; returns reserved %u "
                "claimed %u, finisher waves alive %u, pixels out %u; owed passes: most %u, pixels %u\n",
                w.call_seq, chained ? " (chained)" : "", ts.tv_sec + ts.tv_nsec * 1e-9, lc[0], lc[1], lc[3], rc4[0],
                rc4[2], rc4[1], rc4[3], rc4[5], rc4[6]);
    }
    if (st.long_log && !overlap) return debug_long_log(w, long_log_buf);
    return 0;
}

// the pending batch of coalesced chained calls, launched as one chained call
int flush_pending(Workspace &w)
{
    if (!w.pend.on) return 0;
    Pending b = w.pend;
    w.pend.on = false;
    return launch_whole_now(w, b.dev, b.sc, b.fr, b.cam, b.stream, b.long_depth, b.prof, true, b.check_mask, b.debug,
                            false);
}

// rt_render's whole call (see launch_whole_now), with small chained calls
// coalesced (Pending; coalesce <= 0: off)
int launch_whole(Workspace &w, int dev, const RtDevScene &sc, const RtDevFrame &fr, const RtDevCamera &cam,
                 hipStream_t stream, int long_depth, bool prof, bool overlap, uint32_t check_mask, int debug,
                 bool count, int coalesce)
{
    // (debug diagnostics per call and forced dispatch orders are per launch: never coalesced)
    const bool can = overlap && !fr.reset && !count && coalesce > 0 && !fr.wave_times &&
                     !(debug & (RT_DEBUG_CALL_LOG | RT_DEBUG_LONG_LOG | RT_DEBUG_SERIAL_LONG_FIRST |
                                RT_DEBUG_SERIAL_FIN_FIRST));
    if (w.pend.on) {
        const ChainKey key = chain_key(sc, fr, cam, long_depth);
        if (can && w.pend.dev == dev && w.pend.stream == stream && w.pend.prof == prof &&
            w.pend.check_mask == check_mask && w.pend.debug == debug && w.pend.sc.nodes == sc.nodes &&
            memcmp(&key, &w.pend.key, sizeof key) == 0 && (long long)w.pend.fr.passes + fr.passes < (1LL << 28)) {
            w.pend.fr.passes += fr.passes;
            ++w.pend.calls;
            return w.pend.fr.passes < coalesce ? 0 : flush_pending(w);
        }
        if (flush_pending(w) != 0) return -1;
    }
    if (can && fr.passes < coalesce) {
        Pending &b = w.pend;
        b.on = true;
        b.dev = dev;
        b.sc = sc;
        b.fr = fr;
        b.cam = cam;
        b.stream = stream;
        b.long_depth = long_depth;
        b.debug = debug;
        b.calls = 1;
        b.prof = prof;
        b.check_mask = check_mask;
        b.key = chain_key(sc, fr, cam, long_depth);
        return 0;
    }
    return launch_whole_now(w, dev, sc, fr, cam, stream, long_depth, prof, overlap, check_mask, debug, count);
}

// The drain of an open chain (join_all, i.e. rt_join and every reader of the
// frame, or the next call that does not continue it): a chained call's
// finisher leaves pixels wf_long hands back after its pixel list ran out to
// the next call; here one more finisher with no pixels of its own takes them,
// runs their remaining passes (handing deep samples to its own wf_long again)
// and lingers while any pixel is still out.  Enqueued on pipeline 0 after the
// chain's last finishers on both finisher streams; join_all then waits for it
// and every wf_long.
int launch_drain(Workspace &w)
{
    if (flush_pending(w) != 0) return -1; // (coalesced chained calls: launched, then drained)
    if (!w.chain_open) return 0;
    w.chain_open = false;
    const RtDevFrame &fr = w.last_fr;
    const size_t slots = (size_t)fr.width * fr.height;
    Pipe &pp = w.pipe[0];
    WfState st = pp.st;
    st.long_depth = w.last_long_depth;
    st.long_return = 1;
    st.fresh = 1;
    st.fresh_n = 0; // (no pixels of its own)
    st.span = nullptr;
    st.linger = WF_FIN_LINGER; // (a pixel still out after it: wf_long runs it to the end)
    st.chk = nullptr;
    st.chk_mask = 0;
    st.chk_ctr = w.chk_ctr;
    st.chk_fault = 0;
    st.debug_quit = (w.last_debug & RT_DEBUG_LONG_QUIT) ? 1 : 0;
    st.long_log = nullptr;
    int fgrid = (int)((slots + WF_BLOCK - 1) / WF_BLOCK);
    fgrid = fgrid > w.grid - WF_LONG_BLOCKS ? w.grid - WF_LONG_BLOCKS : fgrid;
    st.fin_live = w.fin_live + (uint32_t)(w.call_seq % 8);
    ++w.call_seq;
    const hipStream_t s = pp.stream;
    // no pixels (counts[4] = 0 of fresh_n 0), no linger seat taken yet
    if (hipMemsetAsync(st.counts, 0, 256, s) != hipSuccess) return -1;
    if (hipMemsetAsync(st.ret_ctr + 4, 0, 4, s) != hipSuccess) return -1;
    if (hipMemsetAsync(st.chain_flag, 0, 4, s) != hipSuccess) return -1; // the chain's wf_longs may leave once idle
    if (hipMemsetD32Async((hipDeviceptr_t)st.fin_live, (int)(fgrid * (WF_BLOCK / 64)), 1, s) != hipSuccess) return -1;
    if (hipEventRecord(w.fin_ready, s) != hipSuccess) return -1;
    if (fgrid <= w.cus * WF_FIN_SMALL_WAVES)
        hipLaunchKernelGGL((wf_finish_bvh<false, 1>), dim3(fgrid), dim3(WF_BLOCK), 0, s, w.last_sc, fr, w.last_cam, st, 0);
    else hipLaunchKernelGGL(wf_finish_bvh<false>, dim3(fgrid), dim3(WF_BLOCK), 0, s, w.last_sc, fr, w.last_cam, st, 0);
    if (hipGetLastError() != hipSuccess) return -1;
    Pipe &lp = w.pipe[1];
    if (hipStreamWaitEvent(lp.stream, w.fin_ready, 0) != hipSuccess) return -1;
    hipLaunchKernelGGL(wf_long<false>, dim3(WF_LONG_BLOCKS), dim3(WF_BLOCK), 0, lp.stream, w.last_sc, fr, w.last_cam, st, 1);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipEventRecord(lp.long_done, lp.stream) != hipSuccess) return -1;
    lp.long_rec = true;
    if (hipEventRecord(pp.join, s) != hipSuccess) return -1;
    pp.joined = true;
    w.verify_pending = true;
    if (w.last_debug & RT_DEBUG_CALL_LOG) {
        (void)hipStreamSynchronize(s);
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        uint32_t rc[7] = {};
        (void)hipMemcpy(rc, st.ret_ctr, sizeof rc, hipMemcpyDeviceToHost);
        fprintf(stderr, "[wf] drain done t %.4f; returns reserved %u claimed %u, pixels out %u; owed passes: most %u, pixels %u\n",
                ts.tv_sec + ts.tv_nsec * 1e-9, rc[0], rc[2], rc[3], rc[5], rc[6]);
    }
    return 0;
}

int debug_long_log(Workspace &w, unsigned long long *buf)
{
    (void)w;
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> L(4 * 65536);
    (void)hipMemcpy(L.data(), buf, 8 * L.size(), hipMemcpyDeviceToHost);
    struct Rec { double start, end; unsigned long long bounces, slot; };
    std::vector<Rec> v;
    double last = 0;
    for (size_t e = 1; e < 65536; ++e)
        if (L[4 * e + 1]) {
            v.push_back({(L[4 * e] - L[0]) * 1e-5, (L[4 * e + 1] - L[0]) * 1e-5, L[4 * e + 2], L[4 * e + 3]});
            last = std::max(last, v.back().end);
        }
    std::sort(v.begin(), v.end(), [](const Rec &a, const Rec &b) { return a.end > b.end; });
    fprintf(stderr, "[wf long log] %zu deep samples, last end %.1f ms; latest 12 (start ms, end ms, bounces, us/bounce, slot):\n",
            v.size(), last);
    for (size_t i = 0; i < v.size() && i < 12; ++i)
        fprintf(stderr, "  %.1f %.1f %llu %.2f %llu\n", v[i].start, v[i].end, v[i].bounces,
                (v[i].end - v[i].start) * 1e3 / (double)(v[i].bounces ? v[i].bounces : 1), v[i].slot);
    std::sort(v.begin(), v.end(), [](const Rec &a, const Rec &b) { return a.bounces > b.bounces; });
    fprintf(stderr, "[wf long log] longest 8:\n");
    for (size_t i = 0; i < v.size() && i < 8; ++i)
        fprintf(stderr, "  %.1f %.1f %llu %.2f %llu\n", v[i].start, v[i].end, v[i].bounces,
                (v[i].end - v[i].start) * 1e3 / (double)(v[i].bounces ? v[i].bounces : 1), v[i].slot);
    // per pixel: deep samples, their summed time in wf_long, first claim and last end
    std::map<unsigned long long, Rec> px;
    std::map<unsigned long long, int> nd;
    for (const Rec &r : v) {
        auto it = px.find(r.slot);
        if (it == px.end()) {
            px[r.slot] = Rec{r.start, r.end, 0, (unsigned long long)0};
            it = px.find(r.slot);
        }
        it->second.start = std::min(it->second.start, r.start);
        it->second.end = std::max(it->second.end, r.end);
        it->second.slot += (unsigned long long)((r.end - r.start) * 1e3); // (us in wf_long)
        it->second.bounces += r.bounces;
        ++nd[r.slot];
    }
    std::vector<std::pair<unsigned long long, Rec>> pv(px.begin(), px.end());
    std::sort(pv.begin(), pv.end(), [](const auto &a, const auto &b) { return a.second.end > b.second.end; });
    fprintf(stderr, "[wf long log] %zu pixels; latest-ending 10 (slot, deep samples, bounces, ms in wf_long, first claim, last end):\n",
            pv.size());
    for (size_t i = 0; i < pv.size() && i < 10; ++i)
        fprintf(stderr, "  %llu %d %llu %.1f %.1f %.1f\n", pv[i].first, nd[pv[i].first], pv[i].second.bounces,
                pv[i].second.slot * 1e-3, pv[i].second.start, pv[i].second.end);
    return 0;
}

} // namespace

// rt_set_device: the default pipelines' streams take their hardware queues
// before anything else in the process (RCCL's streams in a multi-GPU run)
int rt_wavefront_device_init()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    rt_register_shutdown();
    return ensure_streams(workspace(dev), WF_PIPES_DEFAULT);
}

static thread_local char g_incomplete[256];

// the last RT_WAVEFRONT_INCOMPLETE's description (abi.hip: rt_last_error)
const char *rt_wavefront_incomplete_msg() { return g_incomplete; }

// rt_join: `stream` (NULL: the host) waits for every rt_render's device work
// on the current device, chained calls' deep-path tails included, and for the
// hand-off check after them.  A host join returns RT_WAVEFRONT_INCOMPLETE if
// that check, or one enqueued by an earlier stream join, found pixels that
// never came back from wf_long.  consume = 0 (the library's joins that do
// not report: rt_deviation_stats, buffer and scene teardown) leaves such a
// result for the next reporting join: the incomplete status is sticky.
int rt_wavefront_join(void *stream, int consume)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    Workspace *w = nullptr;
    {
        std::lock_guard<std::mutex> g(g_ws_mu);
        auto it = g_ws.find(dev);
        if (it == g_ws.end() || !it->second) return 0;
        w = it->second;
    }
    if (stream) return join_all(*w, (hipStream_t)stream);
    if (launch_drain(*w) != 0) return -1;
    for (int pi = 0; pi < WF_MAX_PIPES; ++pi) {
        Pipe &p = w->pipe[pi];
        if (p.joined && hipEventSynchronize(p.join) != hipSuccess) return -1;
        if (p.long_rec && hipEventSynchronize(p.long_done) != hipSuccess) return -1;
    }
    if (w->recorded && hipEventSynchronize(w->long_ev) != hipSuccess) return -1;
    if (w->verify_pending) {
        const hipStream_t s = w->pipe[0].stream; // (idle: everything above is done)
        if (launch_verify(*w, s) != 0) return -1;
    }
    // (the last check may run on a caller's stream: its result is read after it)
    if (w->verify_rec && hipEventSynchronize(w->verify_ev) != hipSuccess) return -1;
    if (!w->verify_unread) return 0;
    uint32_t r[5] = {};
    if (hipMemcpy(r, w->verify_res, sizeof r, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (!consume) return 0;
    w->verify_unread = false;
    if (hipMemset(w->verify_res, 0, sizeof r) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return -1;
    if (r[0] | r[1] | r[2] | r[3] | r[4]) {
        snprintf(g_incomplete, sizeof g_incomplete,
                 "%u pixels stranded in the deep-path hand-off (pixels out %u, returns unclaimed %u, hand-offs "
                 "unclaimed %u, finisher waves registered %u): the frame misses passes; RtDeviations counts it",
                 r[0], r[1], r[2], r[3], r[4]);
        return RT_WAVEFRONT_INCOMPLETE;
    }
    return 0;
}

// rt_shutdown: every stream, event and device blob of every device's
// workspace, in reverse creation order, after the device work is done
void rt_wavefront_shutdown()
{
    std::lock_guard<std::mutex> g(g_ws_mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto &kv : g_ws) {
        Workspace *w = kv.second;
        if (!w) continue;
        if (hipSetDevice(kv.first) != hipSuccess) continue;
        if (w->blob) (void)launch_drain(*w); // (an open chain's wf_longs leave only after its drain)
        (void)hipDeviceSynchronize();
        if (w->blob) (void)hipFree(w->blob);
        for (void *p : {(void *)w->chk, (void *)w->verify_res, (void *)w->long_log_buf, (void *)w->spans})
            if (p) (void)hipFree(p);
        for (int i = WF_MAX_PIPES - 1; i >= 0; --i) {
            Pipe &p = w->pipe[i];
            for (auto &e : p.ev)
                if (e) (void)hipEventDestroy(e);
            if (p.long_done) (void)hipEventDestroy(p.long_done);
            if (p.fin_done) (void)hipEventDestroy(p.fin_done);
            if (p.join) (void)hipEventDestroy(p.join);
            if (p.host_count) (void)hipHostFree(p.host_count);
            if (p.stream) (void)hipStreamDestroy(p.stream);
        }
        for (hipEvent_t e : {w->verify_ev, w->chk_done[1], w->chk_done[0], w->ev1, w->ev0, w->long_ev, w->fin_ready,
                             w->fork})
            if (e) (void)hipEventDestroy(e);
        delete w;
        kv.second = nullptr;
    }
    g_ws.clear();
    (void)hipSetDevice(cur);
}

extern "C" int rt_last_profile(RtProfile *out)
{
    if (!out) return RT_E_INVALID;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return RT_E_HIP;
    std::lock_guard<std::mutex> g(g_ws_mu);
    auto it = g_ws.find(dev);
    if (it == g_ws.end() || !it->second) {
        *out = RtProfile{};
        return RT_OK;
    }
    if (flush_pending(*it->second) != 0 || resolve_profiles(*it->second) != 0) return RT_E_HIP;
    *out = it->second->prof;
    return RT_OK;
}

extern "C" int rt_profile_history(RtProfile *out, int cap, int *count, int reset)
{
    if ((!out && cap > 0) || cap < 0 || !count) return RT_E_INVALID;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return RT_E_HIP;
    std::lock_guard<std::mutex> g(g_ws_mu);
    auto it = g_ws.find(dev);
    *count = 0;
    if (it == g_ws.end() || !it->second) return RT_OK;
    Workspace &w = *it->second;
    if (flush_pending(w) != 0 || resolve_profiles(w) != 0) return RT_E_HIP;
    *count = (int)w.prof_hist.size();
    for (int i = 0; i < cap && i < *count; ++i) out[i] = w.prof_hist[i];
    if (reset) w.prof_hist.clear();
    return RT_OK;
}

int rt_launch_wavefront(const RtDevScene &sc, const RtDevFrame &fr, const RtDevCamera &cam, hipStream_t stream,
                        int variant, int tail_opt, int finish_waves_opt, int profile, int cap_opt, int postpone_opt,
                        int wide_opt, int pipes_opt, int long_opt, int traversal, int overlap, int check_interval,
                        int debug, int coalesce_opt)
{
    // 1: wave-cooperative leaves (entries packed as k << 6 | lane: needs < 2^26 entries), 2: static, 3: per-lane fetch
    int trace_kind = variant;
    if (trace_kind == 1 && sc.index_count >= (1 << 26)) trace_kind = 3;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    Workspace &w = workspace(dev);
    rt_register_shutdown();
    const size_t slots = (size_t)fr.width * fr.height;
    const bool count = fr.counters != nullptr;
    // the queue trace launches run the BVH-bounded traversal (counting calls: the KD one, whose counters are the reference's)
    const bool bounded = sc.bvh_nodes != nullptr && ((traversal == RT_TRAVERSAL_BOUNDED && !count) ||
                                                     traversal == RT_TRAVERSAL_BOUNDED_COUNTED);
    // paths deeper than this leave their pipeline for wf_long (cooperative trace only)
    // (at least WF_LONG_DEPTH_MIN: wf_long is sized for the rare deep paths — one path per wave on its 64
    // blocks —, and at depth 8 the hand-off took a third of all paths and ran 7x slower)
    const int long_depth = trace_kind == 1 && long_opt >= 0
                               ? (long_opt > 0 ? (long_opt > WF_LONG_DEPTH_MIN ? long_opt : WF_LONG_DEPTH_MIN)
                                               : WF_LONG_DEPTH_DEFAULT)
                               : 0;
    // bounded traversal, not counting: the whole call in the finisher by default
    // — one path per lane to the end of its passes beats queue iterations once
    // a ray query is ~30 dependent loads: 1.22 vs 1.61 s per 256-pass room2m
    // call with deep paths cut (profiles/r03).  It runs as ONE pipeline whose
    // finisher spans the chip: three pipelines' fixed pixel sets finished up
    // to 0.7 s apart, each leaving its third of the chip idle.
    // (RT_TRAVERSAL_BOUNDED_COUNTED: the same whole call, its finisher counting its own work — the
    // bench's per-launch algorithmic bytes then describe the timed launch's own shape)
    const bool whole = bounded && (!count || traversal == RT_TRAVERSAL_BOUNDED_COUNTED) && trace_kind == 1 &&
                       (tail_opt <= 0 || (size_t)tail_opt > slots);
    if (whole) {
        // the run-time exactness guard: 1 ray in check_interval (a power of two) re-traced by the KD traversal
        uint32_t mask = 0xFFFFFFFFu;
        if (check_interval >= 0 && !count) {
            uint32_t iv = check_interval > 0 ? (uint32_t)check_interval : WF_CHECK_INTERVAL_DEFAULT;
            uint32_t p2 = 1;
            while (p2 < iv && p2 < (1u << 30)) p2 <<= 1;
            mask = p2 - 1;
        }
        return launch_whole(w, dev, sc, fr, cam, stream, long_depth, profile != 0, overlap != 0 && !count, mask,
                            debug, count, coalesce_opt < 0 ? 0 : (coalesce_opt > 0 ? coalesce_opt : WF_COALESCE_DEFAULT));
    }
    // persistent-ish grid for trace/shade (grid-stride over the queue).  512
    // blocks = 2,048 waves = a third of the chip's 6,144 wave slots at the
    // trace kernel's 6 waves/SIMD: the 3 pipelines' launches share the chip,
    // and a launch's ~465k rays are ~3.5 per lane, so the lanes stay busy past
    // the launch's first round of rays (1,536 blocks: ~1.2 rays per lane, most
    // of the launch was its tail).  Measured 512 / 704 / 1,536: 37.5 / 37.6 /
    // 33.1 Msamples/s on room2m 1080p (tools/gpu_sweep.sh, profiles/r02).
    const int grid = 512;
    const int tgrid = grid * (WF_BLOCK / WF_TBLOCK); // the same waves in WF_TBLOCK-thread blocks
    // wf_shade: half the trace grid (~2 paths per lane per launch).  Measured
    // per 256-pass room2m call (2 rounds each): 64 / 128 / 256 / 384 / 512 /
    // 1,024 / 2,048 blocks: 13.27 / 12.82 / 12.78 / 12.78 / 12.87 / 13.01 /
    // 13.21 s
    const int sgrid = tgrid / 2 > 16 ? tgrid / 2 : 16;
    const bool prof = profile != 0;
    const int tiles = ((fr.width + 15) / 16) * ((fr.height + 15) / 16);
    int npipes = pipes_opt > 0 ? pipes_opt : WF_PIPES_DEFAULT;
    npipes = npipes > WF_MAX_PIPES ? WF_MAX_PIPES : npipes;
    npipes = npipes > tiles ? tiles : npipes;
    if (ensure(w, slots, grid, npipes) != 0) return -1;
    // below this many live paths the rest of the call runs in one finisher launch
    const uint32_t tail = tail_opt > 0 ? (uint32_t)tail_opt : WF_TAIL_DEFAULT;
    // the cooperative finisher runs on at most this many waves (up to 64 paths in flight each)
    // (small trees: rays are short, so more paths per finisher wave keep its
    // cooperative rounds full — the 36-triangle Cornell box at 256x256 runs
    // 124 vs 91 Msamples/s with 512 waves; room2m is flat from 1024 to 6144)
    const uint32_t finish_waves = finish_waves_opt > 0 ? (uint32_t)finish_waves_opt
                                  : sc.index_count >= WF_FIN_WIDE_MIN_ENTRIES ? WF_FINISH_WAVES_DEFAULT
                                                                              : WF_FINISH_WAVES_SMALL;
    // cooperative traversal: node fetches per descent round, pending lanes before a leaf test
    const int cap = cap_opt > 0 ? cap_opt : WF_DESCENT_CAP_DEFAULT;
    const int postpone = postpone_opt > 0 ? (postpone_opt > 64 ? 64 : postpone_opt) : WF_POSTPONE_DEFAULT;
    // trace launches: once the queue is empty, a wave with at most this many rays left finishes them wide;
    // finisher: a wave with at most this many live rays traces them one by one with all lanes
    const int wide_lanes = wide_opt < 0 ? 0 : (wide_opt > 0 ? (wide_opt > 64 ? 64 : wide_opt) : WF_WIDE_TAIL_LANES);
    // (finisher: tracing several rays one after the other with all lanes pays off
    // when a ray visits hundreds of nodes — large trees; on a small tree, e.g.
    // the 36-triangle Cornell box, a cooperative round of a few lanes is
    // cheaper, and only a lone ray goes wide.  Measured: room2m / cornell_blob
    // finisher time -18 % / -30 % at 32, the Cornell box 2x slower)
    const int wide = sc.index_count >= WF_FIN_WIDE_MIN_ENTRIES ? wide_lanes : (wide_lanes > 0 ? 1 : 0);
    const bool trace_iters = (debug & RT_DEBUG_CALL_LOG) != 0; // per-iteration queue sizes
    for (int pi = 0; pi < WF_MAX_PIPES; ++pi) {
        WfState &st = w.pipe[pi].st;
        st.long_depth = long_depth;
        st.long_return = 0;
        st.fin_live = nullptr;
        st.long_log = nullptr;
    }
    const WfState lst = w.pipe[0].st;

    // the workspace (per-pixel path state, long-path hand-off) is shared by every
    // call on this device: a call must not start before every earlier call's
    // pipelines and wf_long work are done (pixels may move to another pipeline
    // while the previous call's finisher still writes their path state)
    if (join_all(w, stream) != 0) return -1;
    w.chain_open = false;
    if (long_depth > 0) {
        // (the ring from zero — its whole capacity, see launch_whole; a pixel is handed over at most once
        // per call here)
        if (hipMemsetAsync(lst.long_ent, 0, (size_t)lst.long_cap * 8, stream) != hipSuccess) return -1;
        if (hipMemsetAsync(lst.long_ctr, 0, 256, stream) != hipSuccess) return -1;
    }
    // fork: every pipeline stream starts after the caller's stream
    if (hipEventRecord(w.fork, stream) != hipSuccess) return -1;
    if (prof && hipEventRecord(w.ev0, stream) != hipSuccess) return -1;
    std::mutex long_mu;
    bool long_final = false;
    int n_slices = 0; // (debug output)
    // launches a wf_long slice on the caller's stream unless the previous one
    // is still running; the final slice (every producer done) is queued after it
    auto kick_long = [&](bool final) -> int {
        if (long_depth <= 0) return 0;
        std::lock_guard<std::mutex> g(long_mu);
        if (long_final) return 0;
        if (!final) {
            const hipError_t q = hipEventQuery(w.long_ev);
            if (q == hipErrorNotReady) return 0;
            if (q != hipSuccess) return -1;
        }
        const int fin = final ? 1 : 0;
        if (count)
            hipLaunchKernelGGL(wf_long<true>, dim3(WF_LONG_BLOCKS), dim3(WF_BLOCK), 0, stream, sc, fr, cam, lst, fin);
        else
            hipLaunchKernelGGL(wf_long<false>, dim3(WF_LONG_BLOCKS), dim3(WF_BLOCK), 0, stream, sc, fr, cam, lst, fin);
        if (hipGetLastError() != hipSuccess) return -1;
        long_final = final;
        ++n_slices;
        if (hipEventRecord(w.long_ev, stream) != hipSuccess) return -1;
        w.recorded = true;
        return 0;
    };
    std::atomic<int> producing(npipes);
    bool produced_done[WF_MAX_PIPES] = {};
    // a pipeline's queue iterations are over (every shade launch that could
    // publish has completed: the host read its queue size): the last one
    // queues the final wf_long slice
    auto producer_done = [&](int pi) -> int {
        if (produced_done[pi]) return 0;
        produced_done[pi] = true;
        if (producing.fetch_sub(1) != 1) return 0;
        return kick_long(true);
    };

    auto run_pipe = [&](int pi) -> int {
        if (hipSetDevice(dev) != hipSuccess) return -1;
        Pipe &pp = w.pipe[pi];
        pp.trace_iv.clear();
        WfState &st = pp.st;
        hipStream_t s = pp.stream;
        if (hipStreamWaitEvent(s, w.fork, 0) != hipSuccess) return -1;
        RtProfile P{};
        auto mark = [&](int i) { return !prof || hipEventRecord(pp.ev[i], s) == hipSuccess; };
        if (!mark(0)) return -1;
        if (hipMemsetAsync(st.counts, 0, 256, s) != hipSuccess) return -1;
        if (count) hipLaunchKernelGGL(wf_start<true>, dim3(tiles), dim3(WF_BLOCK), 0, s, fr, cam, st, pi, npipes);
        else hipLaunchKernelGGL(wf_start<false>, dim3(tiles), dim3(WF_BLOCK), 0, s, fr, cam, st, pi, npipes);
        if (!mark(1)) return -1;
        // run the `live` paths of queue qq to the end of the call in the finisher
        auto finish = [&](int qq, uint32_t live) -> int {
            if (!mark(2)) return -1;
            if (bounded) {
                // one path per lane (lanes refill from the list), within the spill area (grid blocks)
                int fgrid = (int)((live + WF_BLOCK - 1) / WF_BLOCK);
                fgrid = fgrid > grid ? grid : fgrid;
                if (hipMemsetAsync(st.counts + 4, 0, 4, s) != hipSuccess) return -1;
                if (count) hipLaunchKernelGGL(wf_finish_bvh<true>, dim3(fgrid), dim3(WF_BLOCK), 0, s, sc, fr, cam, st, qq);
                else hipLaunchKernelGGL(wf_finish_bvh<false>, dim3(fgrid), dim3(WF_BLOCK), 0, s, sc, fr, cam, st, qq);
            } else if (trace_kind == 1) {
                // paths per wave: spread over up to finish_waves waves, within the spill area (grid * WF_BLOCK threads)
                const uint32_t max_waves = (uint32_t)grid * (WF_BLOCK / 64);
                uint32_t ppw = (live + finish_waves - 1) / finish_waves;
                ppw = ppw < 1 ? 1 : (ppw > 64 ? 64 : ppw);
                uint32_t waves = (live + ppw - 1) / ppw;
                if (waves > finish_waves) waves = finish_waves;
                if (waves > max_waves) waves = max_waves; // persistent: lanes fetch paths until the queue is empty
                if (hipMemsetAsync(st.counts + 4, 0, 4, s) != hipSuccess) return -1;
                const int fgrid = (int)((waves + WF_BLOCK / 64 - 1) / (WF_BLOCK / 64));
                if (count)
                    hipLaunchKernelGGL(wf_finish_coop<true>, dim3(fgrid), dim3(WF_BLOCK), 0, s, sc, fr, cam, st, qq,
                                       (int)ppw, cap, postpone, wide);
                else
                    hipLaunchKernelGGL(wf_finish_coop<false>, dim3(fgrid), dim3(WF_BLOCK), 0, s, sc, fr, cam, st, qq,
                                       (int)ppw, cap, postpone, wide);
            } else {
                // grid-stride loop: at most `grid` blocks, so gtid stays inside the spill area
                // (sized for grid * WF_BLOCK threads)
                int fgrid = (int)((live + WF_BLOCK - 1) / WF_BLOCK);
                fgrid = fgrid > grid ? grid : fgrid;
                if (count) hipLaunchKernelGGL(wf_finish<true>, dim3(fgrid), dim3(WF_BLOCK), 0, s, sc, fr, cam, st, qq);
                else hipLaunchKernelGGL(wf_finish<false>, dim3(fgrid), dim3(WF_BLOCK), 0, s, sc, fr, cam, st, qq);
            }
            if (hipGetLastError() != hipSuccess || !mark(3)) return -1;
            P.finish_launches = 1;
            return 0;
        };
        int rc = 0;
        // the bounded finisher publishes deep paths to wf_long too: its pipeline
        // is a producer until the finisher is done (meanwhile wf_long slices are
        // kicked as they end; the last producer queues the final slice)
        auto finish_and_release = [&](int qq, uint32_t live) -> int {
            const bool publishes = bounded && long_depth > 0;
            if (!publishes && producer_done(pi) != 0) return -1;
            if (finish(qq, live) != 0) return -1;
            if (!publishes) return 0;
            if (hipEventRecord(pp.fin_done, s) != hipSuccess) return -1;
            while (true) {
                const hipError_t e = hipEventQuery(pp.fin_done);
                if (e == hipSuccess) break;
                if (e != hipErrorNotReady) return -1;
                if (kick_long(false) != 0) return -1;
                std::this_thread::sleep_for(std::chrono::microseconds(200));
            }
            return producer_done(pi);
        };
        for (int it = 0;; ++it) {
            const int q = it & 1;
            if (hipMemsetAsync(st.counts + (q ^ 1), 0, 4, s) != hipSuccess) return -1;     // next ray queue
            if (hipMemsetAsync(st.counts + 6 + (q ^ 1), 0, 4, s) != hipSuccess) return -1; // next path list
            if (hipMemsetAsync(st.counts + 2 + q, 0, 4, s) != hipSuccess) return -1; // fetch cursor
            if (!mark(4)) return -1;
            if (bounded && WF_BVH_DYN) {
                if (count)
                    hipLaunchKernelGGL(wf_trace_bvh_dyn<true>, dim3(grid), dim3(WF_BLOCK), 0, s, sc, st, q, fr.counters,
                                       WF_BVH_DYN_CAP);
                else
                    hipLaunchKernelGGL(wf_trace_bvh_dyn<false>, dim3(grid), dim3(WF_BLOCK), 0, s, sc, st, q, nullptr,
                                       WF_BVH_DYN_CAP);
            } else if (bounded) {
                if (count)
                    hipLaunchKernelGGL(wf_trace_bvh<true>, dim3(grid), dim3(WF_BLOCK), 0, s, sc, st, q, fr.counters);
                else
                    hipLaunchKernelGGL(wf_trace_bvh<false>, dim3(grid), dim3(WF_BLOCK), 0, s, sc, st, q, nullptr);
            } else if (trace_kind == 1) {
                const int li = it * npipes + pi;
                unsigned long long *tl = fr.wave_times && li < WF_TIMELINE_LAUNCHES ? fr.wave_times + 3 * li : nullptr;
                if (count)
                    hipLaunchKernelGGL(wf_trace_coop<true>, dim3(tgrid), dim3(WF_TBLOCK), 0, s, sc, st, q,
                                       fr.counters, cap, postpone, wide_lanes, tl);
                else
                    hipLaunchKernelGGL(wf_trace_coop<false>, dim3(tgrid), dim3(WF_TBLOCK), 0, s, sc, st, q,
                                       fr.counters, cap, postpone, wide_lanes, tl);
            } else if (trace_kind == 3) {
                if (count) hipLaunchKernelGGL(wf_trace_dyn<true>, dim3(grid), dim3(WF_BLOCK), 0, s, sc, st, q, fr.counters);
                else hipLaunchKernelGGL(wf_trace_dyn<false>, dim3(grid), dim3(WF_BLOCK), 0, s, sc, st, q, fr.counters);
            } else {
                if (count) hipLaunchKernelGGL(wf_trace<true>, dim3(grid), dim3(WF_BLOCK), 0, s, sc, st, q, fr.counters);
                else hipLaunchKernelGGL(wf_trace<false>, dim3(grid), dim3(WF_BLOCK), 0, s, sc, st, q, fr.counters);
            }
            if (!mark(5)) return -1;
            if (count) hipLaunchKernelGGL(wf_shade<true>, dim3(sgrid), dim3(WF_TBLOCK), 0, s, sc, fr, cam, st, q);
            else hipLaunchKernelGGL(wf_shade<false>, dim3(sgrid), dim3(WF_TBLOCK), 0, s, sc, fr, cam, st, q);
            if (hipGetLastError() != hipSuccess) return -1;
            if (!mark(2)) return -1;
            if (hipMemcpyAsync(pp.host_count, st.counts, 32, hipMemcpyDeviceToHost, s) != hipSuccess)
                return -1;
            if (hipStreamSynchronize(s) != hipSuccess) return -1;
            const uint32_t live = pp.host_count[6 + (q ^ 1)]; // paths with rays in the next queue
            P.iterations = it + 1;
            if (prof) {
                P.trace_ms += elapsed_ms(pp.ev[4], pp.ev[5]);
                P.shade_ms += elapsed_ms(pp.ev[5], pp.ev[2]);
                pp.trace_iv.emplace_back(elapsed_ms(w.ev0, pp.ev[4]), elapsed_ms(w.ev0, pp.ev[5]));
            }
            if (trace_iters) {
                timespec ts;
                clock_gettime(CLOCK_MONOTONIC, &ts);
                fprintf(stderr, "[wf] pipe %d it %d live %u t %.4f\n", pi, it, live, ts.tv_sec + ts.tv_nsec * 1e-9);
            }
            if (kick_long(false) != 0) return -1; // paths published by this shade launch
            if (live == 0 || live < tail) {
                if (live != 0) rc = finish_and_release(q ^ 1, live);
                else if (producer_done(pi) != 0) return -1;
                break;
            }
        }
        if (rc != 0) return rc;
        if (hipEventRecord(pp.join, s) != hipSuccess) return -1;
        pp.joined = true;
        if (prof) {
            if (!mark(4) || hipEventSynchronize(pp.ev[4]) != hipSuccess) return -1;
            P.trace_launches = P.shade_launches = P.iterations;
            P.start_ms = elapsed_ms(pp.ev[0], pp.ev[1]);
            if (P.finish_launches) P.finish_ms = elapsed_ms(pp.ev[2], pp.ev[3]);
            P.call_ms = elapsed_ms(pp.ev[0], pp.ev[4]);
        }
        pp.prof = P;
        return 0;
    };

    int rcs[WF_MAX_PIPES] = {};
    std::thread threads[WF_MAX_PIPES];
    for (int pi = 1; pi < npipes; ++pi) threads[pi] = std::thread([&, pi] { rcs[pi] = run_pipe(pi); });
    rcs[0] = run_pipe(0);
    for (int pi = 1; pi < npipes; ++pi) threads[pi].join();
    if (!long_final) (void)kick_long(true); // a pipeline failed early: drain the published paths anyway
    if (trace_iters) {
        (void)hipStreamSynchronize(stream);
        uint32_t lc[4] = {};
        (void)hipMemcpy(lc, lst.long_ctr, sizeof lc, hipMemcpyDeviceToHost);
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        fprintf(stderr, "[wf] long paths %u claimed %u running %u; slices %d; caller stream done t %.4f\n", lc[0],
                lc[1], lc[3], n_slices, ts.tv_sec + ts.tv_nsec * 1e-9);
    }
    for (int pi = 0; pi < npipes; ++pi)
        if (rcs[pi] != 0) return rcs[pi];
    // join: the caller's stream continues after every pipeline
    for (int pi = 0; pi < npipes; ++pi)
        if (hipStreamWaitEvent(stream, w.pipe[pi].join, 0) != hipSuccess) return -1;
    if (prof) {
        RtProfile P{};
        for (int pi = 0; pi < npipes; ++pi) { // kernel times summed over the (concurrent) pipelines
            const RtProfile &q = w.pipe[pi].prof;
            P.iterations += q.iterations;
            P.trace_launches += q.trace_launches;
            P.shade_launches += q.shade_launches;
            P.finish_launches += q.finish_launches;
            P.start_ms += q.start_ms;
            P.trace_ms += q.trace_ms;
            P.shade_ms += q.shade_ms;
            P.finish_ms += q.finish_ms;
        }
        if (hipEventRecord(w.ev1, stream) != hipSuccess || hipEventSynchronize(w.ev1) != hipSuccess) return -1;
        P.call_ms = elapsed_ms(w.ev0, w.ev1); // wall time of the call
        std::vector<std::pair<float, float>> iv; // union of the pipelines' trace launch intervals
        for (int pi = 0; pi < npipes; ++pi) iv.insert(iv.end(), w.pipe[pi].trace_iv.begin(), w.pipe[pi].trace_iv.end());
        std::sort(iv.begin(), iv.end());
        float lo = 0.0f, hi = -1.0f;
        for (const auto &x : iv) {
            if (x.first > hi) {
                if (hi > lo) P.trace_union_ms += hi - lo;
                lo = x.first;
                hi = x.second;
            } else if (x.second > hi) {
                hi = x.second;
            }
        }
        if (hi > lo) P.trace_union_ms += hi - lo;
        P.pipelines = npipes;
        w.prof = P;
        push_history(w, P);
    }
    return 0;
}
