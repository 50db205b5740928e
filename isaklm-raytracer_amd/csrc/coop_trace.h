// coop_trace.h — wave-cooperative ray traversal (included by wavefront.hip).
//
// trace_ray (rt/trace_ray.cuh:244-318) for up to 64 rays per wave.  Each
// step, every live lane descends its own ray to the next leaf (per-lane,
// front to back, LDS/HBM stack as in rt_kernels.h); then the whole wave tests
// the UNION of its lanes' leaf entries, 64 (ray, entry) pairs per round, so a
// lane with a 40-entry leaf no longer idles the 63 others — and a single ray
// (the tail finisher) gets its leaf tested 64 entries at a time.  Pair p
// belongs to the lane j with start_j <= p < start_j + count_j (wave prefix sum
// of leaf sizes, found by a 6-step shuffle binary search); the owner's ray
// comes by __shfl.  Plane-test survivors (dn != 0, 1e-5 <= s < leaf exit) are
// compacted into an LDS list and run through the barycentric test 64 at a
// time.  A hit posts (bits(s) << 32 | entry) to the owner's 64-bit LDS key
// with atomicMin: s > 0, so key order is (s, entry order) — exactly the
// first-wins strict-< scan of trace_leaf_node (rt/trace_ray.cuh:124-141).
// The owner then recomputes the winner's barycentrics with the same
// arithmetic.  Results are bit-identical to the sequential scan.
#pragma once

#define WF_COOP_LIST 128 // per-wave LDS list of plane-test candidates
#ifndef WF_NODE_PAIRS
#define WF_NODE_PAIRS 0 // descent: 16-B node-pair loads (child1 arrives with its parent)
#endif
#ifndef WF_CHUNK_UNROLL
#define WF_CHUNK_UNROLL 1 // leaf chunk loop unrolled over two register sets
#endif

namespace rtk {

// barycentric part of intersect_triangle (rt/trace_ray.cuh:48-71,100-110) for
// leaf entry k at the exact plane parameter s
__device__ __forceinline__ bool coop_bary(const RtDevScene &sc, uint32_t k, Vec3D o, Vec3D d, float s, float &cx,
                                          float &cy, float &cz, int &tri)
{
    const RtIsectBary *rec = sc.isect_bary + k;
    const RtF4 B = ldf4(&rec->b), C = ldf4(&rec->c), D = ldf4(&rec->d);
    const uint2 R = *reinterpret_cast<const uint2 *>(&rec->rd);
    const float rd = __uint_as_float(R.x);
    const float px = o.x + d.x * s, py = o.y + d.y * s, pz = o.z + d.z * s;
    const float v2x = px - B.x, v2y = py - B.y, v2z = pz - B.z;
    const float d20 = v2x * C.x + v2y * C.y + v2z * C.z;
    const float d21 = v2x * D.x + v2y * D.y + v2z * D.z;
    cy = (D.w * d20 - C.w * d21) * rd;
    cz = (B.w * d21 - C.w * d20) * rd;
    cx = 1.0f - cy - cz;
    tri = (int)R.y;
    return rt_bary_inside(cx, cy, cz);
}

// A plane-test candidate in the per-wave LDS list: (entry << 6 | owner lane),
// and the numerator / denominator of s = num / dn.
struct CoopCand {
    uint32_t key;
    uint32_t num, dn;
};

// Conservative prescreen of the plane test of intersect_triangle
// (rt/trace_ray.cuh:86-98: reject if d.n == 0 or s < 1e-5, and trace_leaf_node
// keeps only s < max_t = leaf exit).  s' = num * rcp(dn) is within 2^-21
// (relative) of the exact s = RN(num / dn) for |dn| >= 2^-100, so a triangle
// is dropped here only when the exact test would drop it too: s' < 0.99999e-5
// means s < 1e-5, s' >= 1.00001 * exit means s >= exit.  Everything else
// (including NaN / inf / tiny dn) goes on to the exact division and test.
__device__ __forceinline__ bool plane_maybe(float num, float dn, float ex)
{
    if (dn == 0.0f) return false;
    if (!(fabsf(dn) >= 0x1p-100f)) return true;
    const float sa = num * __builtin_amdgcn_rcpf(dn);
    return !(sa < 0.0000099999f) && !(sa >= ex * 1.00001f);
}

// plane_maybe as one expression of compares and selects (same result)
__device__ __forceinline__ bool plane_maybe_sel(float num, float dn, float ex)
{
    const float sa = num * __builtin_amdgcn_rcpf(dn);
    const bool tiny = !(fabsf(dn) >= 0x1p-100f);
    const bool keep = !(sa < 0.0000099999f) & !(sa >= ex * 1.00001f);
    return (dn != 0.0f) & (tiny | keep);
}

// per-wave LDS scratch of the cooperative leaf test
struct CoopLds {
    unsigned long long *key; // 64: per-lane winner key (atomicMin)
    CoopCand *list;          // WF_COOP_LIST plane-test candidates
    int *mark;               // 128: chunk_owner marks (64) + junk slots (64)
};

// per-lane traversal state
struct CoopRay {
    bool live;                  // the lane holds an unfinished ray
    bool pend;                  // ... which has reached a non-empty leaf, waiting for the wave's leaf test
    Vec3D o, d;
    float yx, yy, yz;           // rt_recip_guard(d): the split distance division by reciprocal
    float entry, exit_, root_exit;
    uint32_t node;
    int sp;
    uint32_t leaf_begin;
    int leaf_count;
};

__device__ __forceinline__ void coop_idle(CoopRay &r)
{
    r.live = r.pend = false;
    r.o = r.d = rt_v3(0, 0, 0);
    r.yx = r.yy = r.yz = 0.0f;
    r.entry = r.exit_ = r.root_exit = 0.0f;
    r.node = 0;
    r.sp = 0;
    r.leaf_begin = 0;
    r.leaf_count = 0;
}

// start a ray: slab test on the scene box; false = miss
__device__ __forceinline__ bool coop_begin(const RtDevScene &sc, CoopRay &r, Vec3D o, Vec3D d)
{
    r.o = o;
    r.d = d;
    r.yx = rt_recip_guard(d.x);
    r.yy = rt_recip_guard(d.y);
    r.yz = rt_recip_guard(d.z);
    r.node = 0;
    r.sp = 0;
    r.pend = false;
    r.live = bbox_hit_recip(sc, o, d, r.yx, r.yy, r.yz, r.entry, r.exit_);
    r.root_exit = r.exit_;
    return r.live;
}

// pop the next subtree (rt/trace_ray.cuh:308-316); exit t = entry of the entry below
template <typename STK>
__device__ __forceinline__ void coop_pop(CoopRay &r, STK &stk)
{
    --r.sp;
    stk.get(r.sp, r.node, r.entry);
    r.exit_ = r.sp > 0 ? stk.entry_at(r.sp - 1) : r.root_exit;
}

// Descent (rt/trace_ray.cuh:273-306) of a live, non-pending lane for at most
// `cap` node fetches, stopping at the first non-empty leaf (r.pend).  Empty
// leaves are popped on the spot.  Returns true when the ray ended (a miss:
// an empty leaf with an empty stack).  Capping the descent lets lanes that
// reach a leaf early be tested with the next batch instead of idling until
// the wave's deepest descent is done (postponed leaf testing).
template <bool COUNT, typename STK>
__device__ __forceinline__ bool coop_descend(const RtDevScene &sc, CoopRay &r, STK &stk, int cap, Cnt &c)
{
    // scalar copies: a select between struct members would become a
    // dynamically indexed (scratch) load
    const float ox = r.o.x, oy = r.o.y, oz = r.o.z, dx = r.d.x, dy = r.d.y, dz = r.d.z;
    const float yx = r.yx, yy = r.yy, yz = r.yz;
    // one flag per lane instead of early returns: the loop has a single
    // (wave-uniform) exit, which keeps the exec-mask bookkeeping small
    bool act = r.live && !r.pend, ended = false;
#if WF_NODE_PAIRS
    // Node pairs: child1 is always node + 1 (pre-order), so one 16-B load at
    // node i brings node i + 1 along; a step into child1 right after a load
    // needs no load of its own (one dependent memory round trip fewer).  The
    // node array carries one padding node (upload_vec's slack).
    bool have = false;    // nx = the nodes word pair of r.node, already loaded
    uint2 nx = make_uint2(0u, 0u);
#endif
    for (int k = 0; k < cap && __any(act); ++k) {
        if (!act) continue;
#if WF_NODE_PAIRS
        uint2 nd, n1 = make_uint2(0u, 0u);
        const bool loaded = !have;
        if (have) {
            nd = nx;
        } else {
            const uint2 *np = reinterpret_cast<const uint2 *>(sc.nodes + 2 * (size_t)r.node);
            nd = np[0];
            n1 = np[1];
        }
        have = false;
        const uint32_t at = r.node;
#else
        const uint2 nd = *reinterpret_cast<const uint2 *>(sc.nodes + 2 * (size_t)r.node);
#endif
        if (COUNT) {
            // counting build: the wave-time spent waiting for this node load
            const unsigned long long tq = __builtin_amdgcn_s_memtime();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (__lane_id() == (__ffsll((long long)__ballot(1)) - 1))
                c.v[RT_CNT_T_DESC_WAIT] += __builtin_amdgcn_s_memtime() - tq;
        }
        if (COUNT) c.v[RT_CNT_NODE]++;
        if ((nd.y & 3u) == RT_LEAF_TAG) {
            const int cnt = (int)(nd.y >> 2);
            if (cnt > 0) {
                r.pend = true;
                r.leaf_begin = nd.x;
                r.leaf_count = cnt;
                if (COUNT) c.v[RT_CNT_TRI] += (unsigned long long)cnt;
                act = false;
            } else if (r.sp == 0) {
                r.live = false;
                ended = true;
                act = false;
            } else {
                if (COUNT && r.sp - 1 >= WF_LDS_STACK) c.v[RT_CNT_SPILL_POP]++;
                coop_pop(r, stk);
            }
            continue;
        }
        const uint32_t axis = nd.y & 3u;
        const float split = as_float(nd.x);
        const float oax = axis == 0 ? ox : (axis == 1 ? oy : oz);
        const float dax = axis == 0 ? dx : (axis == 1 ? dy : dz);
        const float yax = axis == 0 ? yx : (axis == 1 ? yy : yz);
        uint32_t near_c = r.node + 1, far_c = nd.y >> 2;
        if (oax >= split) { // ray_behind_plane (:174-188)
            near_c = nd.y >> 2;
            far_c = r.node + 1;
        }
        const float t = rt_div_by(split - oax, dax, yax); // intersect_plane (:190-210): (split - o) / d
        if (t >= r.exit_ || t < 0) {
            r.node = near_c;
        } else if (t <= r.entry) {
            r.node = far_c;
        } else {
            if (COUNT && r.sp >= RT_REF_STACK) c.v[RT_CNT_DEEP_PUSH]++;
            if (COUNT && r.sp >= WF_LDS_STACK) c.v[RT_CNT_SPILL_PUSH]++;
            stk.put(r.sp, far_c, t);
            ++r.sp;
            r.node = near_c;
            r.exit_ = t;
        }
#if WF_NODE_PAIRS
        if (loaded && r.node == at + 1) {
            have = true;
            nx = n1;
        }
#endif
    }
    return ended;
}

// The wave-cooperative test of every pending lane's leaf (call with all 64
// lanes active).  Returns true for a lane whose ray finished here, with
// tri >= 0 and the barycentrics of the hit, or tri = -1 for a miss; other
// pending lanes pop and go back to descending.
template <bool COUNT, typename STK>
__device__ __forceinline__ bool coop_leaves(const RtDevScene &sc, CoopRay &r, STK &stk, const CoopLds &w, int &tri,
                                            float &hbx, float &hby, float &hbz, Cnt &c)
{
    const int lane = __lane_id();
    unsigned long long *wkey = w.key;
    CoopCand *list = w.list;
    const int leaf_count = r.pend ? r.leaf_count : 0;
    const int incl = wave_incl_add(leaf_count);
    const int total = lane63(incl);
    const int start = incl - leaf_count; // exclusive prefix: lane j's pairs are [start, start + leaf_count)
    const uint32_t kbase = r.leaf_begin - (uint32_t)start; // entry of pair p = kbase_j + p
    lds_vu64 *vkey = (lds_vu64 *)wkey; // set and read per lane, lowered by other lanes: see chunk_owner
    vkey[lane] = (unsigned long long)(uint32_t)vconst(-1) << 32 | (uint32_t)vconst(-1);
    int list_n = 0, carry = -1;
    // exact plane + barycentric stage over the first min(list_n, 64) listed
    // candidates; the rest (< 64) moves to the front of the list
    auto bary_stage = [&]() {
        if (COUNT && lane == 0) c.v[RT_CNT_BARY]++;
        const int take = list_n < 64 ? list_n : 64;
        const CoopCand it = list[lane < take ? lane : 0];
        const int j = (int)(it.key & 63u);
        const Vec3D oo = rt_v3(__shfl(r.o.x, j), __shfl(r.o.y, j), __shfl(r.o.z, j));
        const Vec3D dd = rt_v3(__shfl(r.d.x, j), __shfl(r.d.y, j), __shfl(r.d.z, j));
        const float ex = __shfl(r.exit_, j);
        if (lane < take) {
            const float dn = __uint_as_float(it.dn);
            const float s = __uint_as_float(it.num) / dn; // intersect_triangle (:95-98)
            float cx, cy, cz;
            int t;
            const bool plane = dn != 0 && s >= 0.00001f && s < ex;
            if (COUNT && plane) c.v[RT_CNT_PLANE]++;
            if (plane && coop_bary(sc, it.key >> 6, oo, dd, s, cx, cy, cz, t))
                atomicMin(wkey + j, ((unsigned long long)__float_as_uint(s) << 32) | (it.key >> 6));
        }
        const int rest = list_n - take;
        CoopCand mv = CoopCand{0u, 0u, 0u};
        if (lane < rest) mv = list[take + lane];
        if (lane < rest) list[lane] = mv;
        list_n = rest;
    };
    // counting build: wave-time split of the chunk loop (lane 0's clock; the
    // explicit waits make the split observable and perturb it a little)
    unsigned long long tw = 0;
    auto tick = [&](int slot) {
        if (COUNT) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (lane == 0 && slot >= 0) c.v[slot] += t - tw;
            tw = t;
        }
    };
    // one 64-pair chunk: its owner lanes, leaf entries and plane records
    struct Chunk {
        int j;
        uint32_t k;
        RtF4 A;
    };
    auto setup = [&](int b, Chunk &ch) {
        const int p = b + lane;
        ch.j = chunk_owner(w.mark, start, leaf_count, b, carry);
        carry = lane63(ch.j);
        // the shuffle runs on every lane: behind a `p < total` branch it would
        // read 0 from owners whose own position is past the end of the chunk
        const uint32_t k = (uint32_t)__shfl((int)kbase, ch.j) + (uint32_t)p;
        ch.k = p < total ? k : 0u; // past the last pair: entry 0, a valid address
        ch.A = ldf4(sc.isect_a + ch.k);
    };
    // plane test of a chunk and append of its candidates
    auto test = [&](int base, const Chunk &ch) {
        if (COUNT && lane == 0) c.v[RT_CNT_CHUNKS]++;
        const int j = ch.j;
        const RtF4 A = ch.A;
        const bool valid = base + lane < total;
        const Vec3D oo = rt_v3(__shfl(r.o.x, j), __shfl(r.o.y, j), __shfl(r.o.z, j));
        const Vec3D dd = rt_v3(__shfl(r.d.x, j), __shfl(r.d.y, j), __shfl(r.d.z, j));
        const float ex = __shfl(r.exit_, j);
        const float dn = dd.x * A.x + dd.y * A.y + dd.z * A.z;
        const float num = A.w - (oo.x * A.x + oo.y * A.y + oo.z * A.z);
        const bool cand = valid & plane_maybe_sel(num, dn, ex);
        // append without an exec-mask branch: candidates take the next slots
        // in lane order, the other lanes write junk after them (slots below
        // list_n + 64 <= 127, overwritten before they are read)
        const unsigned long long pm = __ballot(cand);
        const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
        const int npm = __popcll(pm);
        const int slot = list_n + (cand ? below : npm + lane - below);
        list[slot] = CoopCand{(ch.k << 6) | (uint32_t)j, __float_as_uint(num), __float_as_uint(dn)};
        if (COUNT && cand) c.v[RT_CNT_CAND]++;
        list_n += npm;
        tick(RT_CNT_T_LEAF_TEST);
        if (list_n >= 64) {
            bary_stage();
            tick(RT_CNT_T_LEAF_BARY);
        }
    };
    // Software pipeline, unrolled twice over two chunk register sets: chunk
    // c + 1's owner scan, entry and plane load are issued before chunk c's
    // test, and each set is reloaded only after its test, so the loaded
    // planes never have to be moved between registers (a loop-carried copy
    // would wait for the load at the end of every iteration and undo the
    // pipelining).
    // The set-ups run unconditionally (a chunk past the end owns entry 0 of
    // lane `carry`: a valid address, never tested): a conditional set-up
    // would merge its registers with the old ones at the join, i.e. copy
    // them, and wait for the load right there.
    tick(-1);
#if !WF_CHUNK_UNROLL
    // (A/B reference: one register set, the loaded planes copied into the
    // next iteration's set at the loop's end)
    if (total > 0) {
        Chunk cur, nxt;
        setup(0, nxt);
        for (int base = 0; base < total; base += 64) {
            cur = nxt;
            if (base + 64 < total) setup(base + 64, nxt);
            test(base, cur);
        }
    }
#else
    if (total > 0) {
        Chunk c0, c1;
        setup(0, c0);
        tick(RT_CNT_T_LEAF_SETUP);
        for (int base = 0;; base += 128) {
            setup(base + 64, c1);
            tick(RT_CNT_T_LEAF_SETUP);
            test(base, c0);
            if (base + 64 >= total) break;
            setup(base + 128, c0);
            tick(RT_CNT_T_LEAF_SETUP);
            test(base + 64, c1);
            if (base + 128 >= total) break;
        }
    }
#endif
    if (list_n > 0) bary_stage();
    tick(RT_CNT_T_LEAF_BARY);
    // ---- per-lane result: winner, or pop, or miss
    const unsigned long long key = vkey[lane];
    bool done = false;
    if (r.pend) {
        r.pend = false;
        if (key != ~0ull) {
            const uint32_t k = (uint32_t)key;
            coop_bary(sc, k, r.o, r.d, __uint_as_float((uint32_t)(key >> 32)), hbx, hby, hbz, tri);
            if (COUNT) c.v[RT_CNT_HIT]++;
            r.live = false;
            done = true;
        } else if (r.sp == 0) {
            tri = -1;
            r.live = false;
            done = true;
        } else {
            if (COUNT && r.sp - 1 >= WF_LDS_STACK) c.v[RT_CNT_SPILL_POP]++;
            coop_pop(r, stk);
        }
    }
    return done;
}

// One round for the wave: capped descent for descending lanes, then the
// cooperative leaf test once at least `postpone` lanes are pending (or no
// lane is still descending).  Call with all 64 lanes active; returns true for
// a lane whose ray finished in this round (tri / barycentrics as above).
template <bool COUNT, typename STK>
__device__ __forceinline__ bool coop_round(const RtDevScene &sc, CoopRay &r, STK &stk, const CoopLds &w, int cap,
                                           int postpone, int &tri, float &hbx, float &hby, float &hbz, Cnt &c)
{
    bool done = false;
    tri = -1;
    const unsigned long long t0 = COUNT ? __builtin_amdgcn_s_memtime() : 0ull;
    if (r.live && !r.pend) done = coop_descend<COUNT>(sc, r, stk, cap, c);
    const unsigned long long pm = __ballot(r.pend), lm = __ballot(r.live);
    const unsigned long long t1 = COUNT ? __builtin_amdgcn_s_memtime() : 0ull;
    if (pm && (__popcll(pm) >= postpone || pm == lm)) {
        if (COUNT && __lane_id() == 0) {
            c.v[RT_CNT_PEND_LANES] += (unsigned long long)__popcll(pm);
            c.v[RT_CNT_LEAF_TESTS]++;
        }
        if (coop_leaves<COUNT>(sc, r, stk, w, tri, hbx, hby, hbz, c)) done = true;
    }
    if (COUNT && __lane_id() == 0) {
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
        c.v[RT_CNT_T_DESCEND] += t1 - t0;
        c.v[RT_CNT_T_LEAVES] += t2 - t1;
        c.v[RT_CNT_ROUNDS]++;
    }
    return done;
}

// ---------------------------------------------------------------------------
// Wide single-ray traversal: the whole wave works on ONE ray (the tail
// finisher's lone long glass paths, where the sequential trace is a chain of
// ~250 dependent node fetches and ~50 leaf tests per bounce).
//
// The traversal's pending work is kept as an ordered frontier F in LDS (a
// stack whose top is the next item in the sequential front-to-back order).
// Each round the top k <= 64 items are loaded in parallel, one per lane.  The
// leading run of leaves is the next stretch of the sequential leaf order: it
// is tested in one cooperative batch (every entry of every leaf, 64 at a
// time) with the key (leaf rank << 58 | bits(s) << 26 | entry), so the winner
// is the first leaf in order that has a hit and, inside it, the smallest
// (s, entry) — exactly trace_ray's first-leaf-wins + strict-< scan
// (rt/trace_ray.cuh:124-141,310-313).  The inner items behind the run are
// expanded in the same round by the sequential rule (near/far by
// ray_behind_plane, t = (split - o)/d, t >= exit or t < 0 -> near only,
// t <= entry -> far only, else near [entry, t] then far [t, exit]), so every
// item carries the same interval the sequential stack would give it.  Items
// beyond the first hit are speculative and dropped.
//
// Work counters stay the reference's: a fetch of an expanded inner node is
// charged to its first child (acc) and committed only when a leaf at or
// before the winning leaf is consumed — the nodes the sequential traversal
// visits are exactly those at or before the winning leaf in order.
#define WIDE_CAP 256        // frontier items per wave
#define WIDE_RESERVE 24     // head-only growth room (tree depth <= 20)
#define WIDE_LEAF_BUDGET 256 // entries tested per batch (at least one whole leaf)

struct WideItem {
    uint32_t node;
    float entry, exit_;
    uint32_t acc; // counting build: counters charged to this item — node fetches
                  // (bits 0..15), deep pushes (bits 16..23, RT_CNT_DEEP_PUSH) —, the
                  // sequential stack size when the item becomes the current node
                  // (bits 24..28) and WIDE_COUNTED (bit 31)
};

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// per-wave LDS scratch of wide_trace
struct WideLds {
    WideItem *F;             // frontier, `cap` items
    int cap;
    unsigned long long *key; // 1: winner key
    float *best;             // 4: winner barycentrics + triangle bits
    int *mark;               // 128: chunk_owner marks (64) + junk slots (64)
};

// an item whose node fetch (and, for a leaf, its triangle tests) the
// sequential traversal already counted (a resumed ray's pending leaf)
#define WIDE_COUNTED 0x80000000u
#define WIDE_SP_SHIFT 24 // acc bits 24..28: the item's sequential stack size

// Trace the wave-uniform ray (o, d) from a frontier of n items already in
// W.F (F[n-1] is the next item in traversal order) with all 64 lanes.
// Returns the hit (tri >= 0, barycentrics) or tri = -1.  Counters are added
// by `counter_lane` only.
template <bool COUNT>
__device__ __forceinline__ void wide_trace_from(const RtDevScene &sc, Vec3D o, Vec3D d, int n, const WideLds &W,
                                                bool counter_lane, int &tri, float &hbx, float &hby, float &hbz,
                                                Cnt &c)
{
    WideItem *F = W.F;
    unsigned long long *wkey = W.key;
    const int lane = __lane_id();
    const float ox = o.x, oy = o.y, oz = o.z, dx = d.x, dy = d.y, dz = d.z;
    const float yx = rt_recip_guard(dx), yy = rt_recip_guard(dy), yz = rt_recip_guard(dz);
    tri = -1;
    const unsigned long long t0 = COUNT ? __builtin_amdgcn_s_memtime() : 0ull;
    if (COUNT && counter_lane) c.v[RT_CNT_WIDE_CALLS]++;
    while (n > 0) {
        if (COUNT && counter_lane) c.v[RT_CNT_WIDE_ROUNDS]++;
        const unsigned long long tr0 = COUNT ? __builtin_amdgcn_s_memtime() : 0ull;
        int k = W.cap - WIDE_RESERVE - n; // expansions add at most one item each
        k = k < 1 ? 1 : (k > 64 ? 64 : k);
        k = k < n ? k : n;
        WideItem it = WideItem{0u, 0.0f, 0.0f, 0u};
        uint2 nd = make_uint2(0u, 0u);
        const bool have = lane < k;
        if (have) {
            it = F[n - 1 - lane];
            nd = *reinterpret_cast<const uint2 *>(sc.nodes + 2 * (size_t)it.node);
        }
        const bool leaf = have && (nd.y & 3u) == RT_LEAF_TAG;
        const unsigned long long lmask = __ballot(leaf);
        unsigned long long tph = 0;
        if (COUNT) {
            __builtin_amdgcn_s_waitcnt(0);
            tph = __builtin_amdgcn_s_memtime();
            if (counter_lane) c.v[RT_CNT_T_WIDE_LOAD] += tph - tr0;
        }
        const int L = ~lmask ? __ffsll((long long)~lmask) - 1 : 64; // leading run of leaves
        // consume leaves 0..Le-1: whole leaves within the entry budget (at least one)
        const int cnt_all = (lane < L) ? (int)(nd.y >> 2) : 0;
        const int incl = wave_incl_add(cnt_all);
        const int Le = __popcll(__ballot(lane < L && (lane == 0 || incl <= WIDE_LEAF_BUDGET)));
        if (Le > 0) {
            const int cnt = lane < Le ? cnt_all : 0;
            const int start = incl - cnt_all; // exclusive prefix (lanes < Le)
            const int total = __builtin_amdgcn_readlane(incl, Le - 1);
            const uint32_t kbase = nd.x - (uint32_t)start; // leaf_begin - start: entry of pair p = kbase_j + p
            if (lane == 0) wkey[0] = ~0ull;
            // one ray: bandwidth is free, latency is not — each pair loads its
            // plane and its barycentric record together (one memory round trip
            // per 64 pairs), and the current winner parks its barycentrics in
            // LDS so the result needs no reload
            lds_vfloat *best = (lds_vfloat *)W.best;    // {bx, by, bz, tri bits}: cross-lane, see chunk_owner
            lds_vu64 *vkey = (lds_vu64 *)wkey;
            int carry = -1;
            for (int base = 0; base < total; base += 64) {
                const int p = base + lane;
                const int j = chunk_owner(W.mark, start, cnt, base, carry); // owner leaf lane of pair p
                carry = lane63(j);
                const uint32_t e = (uint32_t)__shfl((int)kbase, j) + (uint32_t)p;
                const float ex = __shfl(it.exit_, j);
                unsigned long long mine = ~0ull;
                float cx = 0.0f, cy = 0.0f, cz = 0.0f;
                int t = -1;
                if (p < total) {
                    const RtF4 A = ldf4(sc.isect_a + e);
                    const RtIsectBary *rec = sc.isect_bary + e;
                    const RtF4 B = ldf4(&rec->b), C = ldf4(&rec->c), D = ldf4(&rec->d);
                    const uint2 R = *reinterpret_cast<const uint2 *>(&rec->rd);
                    const float dn = dx * A.x + dy * A.y + dz * A.z;
                    const float s = (A.w - (ox * A.x + oy * A.y + oz * A.z)) / dn; // intersect_triangle (:95-98)
                    if (dn != 0 && s >= 0.00001f && s < ex) {
                        const float px = ox + dx * s, py = oy + dy * s, pz = oz + dz * s; // = coop_bary
                        const float v2x = px - B.x, v2y = py - B.y, v2z = pz - B.z;
                        const float d20 = v2x * C.x + v2y * C.y + v2z * C.z;
                        const float d21 = v2x * D.x + v2y * D.y + v2z * D.z;
                        const float rd = __uint_as_float(R.x);
                        cy = (D.w * d20 - C.w * d21) * rd;
                        cz = (B.w * d21 - C.w * d20) * rd;
                        cx = 1.0f - cy - cz;
                        t = (int)R.y;
                        if (rt_bary_inside(cx, cy, cz)) {
                            mine = ((unsigned long long)j << 58) | ((unsigned long long)__float_as_uint(s) << 26) |
                                   (unsigned long long)e;
                            atomicMin(wkey, mine);
                        }
                    }
                }
                if (mine != ~0ull && vkey[0] == mine) {
                    best[0] = cx; // keys are unique: one writer, and a later smaller key overwrites
                    best[1] = cy;
                    best[2] = cz;
                    best[3] = __int_as_float(t);
                }
            }
            const unsigned long long key = vkey[0];
            const int jstar = key != ~0ull ? (int)(key >> 58) : Le - 1;
            if (COUNT) { // leaves 0..jstar are the sequential traversal's next visits
                const bool counted = (it.acc & WIDE_COUNTED) != 0;
                const bool commit = lane <= jstar && !counted;
                const unsigned long long nv = wave_sum(commit ? (it.acc & 0xFFFFu) + 1ull : 0ull);
                const unsigned long long tv = wave_sum(commit ? (unsigned long long)cnt : 0ull);
                const unsigned long long dv = wave_sum(commit ? (unsigned long long)((it.acc >> 16) & 0xFFu) : 0ull);
                if (counter_lane) {
                    c.v[RT_CNT_NODE] += nv;
                    c.v[RT_CNT_TRI] += tv;
                    c.v[RT_CNT_DEEP_PUSH] += dv;
                }
            }
            if (key != ~0ull) {
                hbx = best[0];
                hby = best[1];
                hbz = best[2];
                tri = __float_as_int(best[3]);
                if (COUNT && counter_lane) {
                    c.v[RT_CNT_HIT]++;
                    c.v[RT_CNT_T_WIDE] += __builtin_amdgcn_s_memtime() - t0;
                }
                return;
            }
        }
        unsigned long long tex = 0;
        if (COUNT) {
            tex = __builtin_amdgcn_s_memtime();
            if (counter_lane) c.v[RT_CNT_T_WIDE_LEAF] += tex - tph;
        }
        // expand the rest of the k items (leaves behind an inner item stay as they are)
        int c_out = 0;
        WideItem a = it, b = it;
        if (have && lane >= Le) {
            c_out = 1;
            if (!leaf) {
                // counting build: this node's fetch is charged to its first child
                // (nothing if it was counted already); a child becomes current
                // with the parent's stack size, +1 for the near child of a push
                const uint32_t sp_it = COUNT ? (it.acc >> WIDE_SP_SHIFT) & 31u : 0u;
                const uint32_t acc1 = COUNT ? ((it.acc & WIDE_COUNTED) ? 0u : (it.acc & 0xFFFFFFu) + 1u) : 0u;
                const uint32_t axis = nd.y & 3u;
                const float split = as_float(nd.x);
                const float oax = axis == 0 ? ox : (axis == 1 ? oy : oz);
                const float dax = axis == 0 ? dx : (axis == 1 ? dy : dz);
                const float yax = axis == 0 ? yx : (axis == 1 ? yy : yz);
                uint32_t near_c = it.node + 1, far_c = nd.y >> 2;
                if (oax >= split) { // ray_behind_plane (:174-188)
                    near_c = nd.y >> 2;
                    far_c = it.node + 1;
                }
                const float t = rt_div_by(split - oax, dax, yax); // intersect_plane (:190-210)
                if (t >= it.exit_ || t < 0) {
                    a = WideItem{near_c, it.entry, it.exit_, acc1 | sp_it << WIDE_SP_SHIFT};
                } else if (t <= it.entry) {
                    a = WideItem{far_c, it.entry, it.exit_, acc1 | sp_it << WIDE_SP_SHIFT};
                } else {
                    // the sequential traversal pushes the far child at stack
                    // index sp_it (SURVEY H16 counter).  (Not the item's frontier
                    // position: items below it may already be expanded.)
                    const uint32_t deep = COUNT && sp_it >= RT_REF_STACK ? 1u << 16 : 0u;
                    a = WideItem{near_c, it.entry, t, (acc1 + deep) | (sp_it + 1u) << WIDE_SP_SHIFT};
                    b = WideItem{far_c, t, it.exit_, sp_it << WIDE_SP_SHIFT};
                    c_out = 2;
                }
            }
        }
        int pos = wave_incl_add(c_out);
        const int M = lane63(pos);
        pos -= c_out;
        const int base = n - k;
        if (c_out >= 1) F[base + M - 1 - pos] = a;
        if (c_out == 2) F[base + M - 2 - pos] = b;
        n = base + M;
        if (COUNT && counter_lane) c.v[RT_CNT_T_WIDE_EXPAND] += __builtin_amdgcn_s_memtime() - tex;
    }
    if (COUNT && counter_lane) c.v[RT_CNT_T_WIDE] += __builtin_amdgcn_s_memtime() - t0;
}

// a fresh ray (scene-box interval [entry, exit_]): the frontier is the root
template <bool COUNT>
__device__ __forceinline__ void wide_trace(const RtDevScene &sc, Vec3D o, Vec3D d, float entry, float exit_,
                                           const WideLds &W, bool counter_lane, int &tri, float &hbx, float &hby,
                                           float &hbz, Cnt &c)
{
    if (__lane_id() == 0) W.F[0] = WideItem{0u, entry, exit_, 0u};
    wide_trace_from<COUNT>(sc, o, d, 1, W, counter_lane, tri, hbx, hby, hbz, c);
}

// The wide traversal of a fresh ray entered at the KD node of the grid cell
// holding its origin (host/scene_prepare.cpp build_kd_starts): trace_ray goes
// front to back from the origin, so it descends from the root toward the
// origin's side of every split it crosses — the near child — until it
// reaches that node, pushing the far child wherever the split lies inside
// its interval.  The stored root path lets the wave replay those decisions
// from records loaded at once (one per lane) instead of spending a frontier
// round per level: each decision must be the path's child (near only: t >=
// exit or t < 0; near with the far child pushed: entry < t < exit), anything
// else (a far-only step, a NaN split distance, an origin off the cell) and
// the frontier is the root as usual.  On success W.F holds the same ordered
// frontier wide_resume builds from a sequential stack — pushed far children
// under the start node — and its size is returned (0: not entered).
// (Only for non-counting launches: the skipped levels' node fetches are not
// charged to the reference's counters.)
__device__ __forceinline__ int kd_origin_frontier(const RtDevScene &sc, Vec3D o, Vec3D d, float entry, float exit_,
                                                  const WideLds &W)
{
    const int lane = __lane_id();
    const int G = sc.kd_grid;
    const float f[3] = {(o.x - sc.bmin[0]) * sc.kd_gscale[0], (o.y - sc.bmin[1]) * sc.kd_gscale[1],
                        (o.z - sc.bmin[2]) * sc.kd_gscale[2]};
    int cc[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) cc[a] = f[a] >= 0.0f ? (f[a] < (float)(G - 1) ? (int)f[a] : G - 1) : 0; // (NaN: 0)
    const size_t k = ((size_t)cc[2] * (size_t)G + (size_t)cc[1]) * (size_t)G + (size_t)cc[0];
    const uint2 st = *reinterpret_cast<const uint2 *>(sc.kd_cell + 2 * k);
    if (st.x == 0xFFFFFFFFu) return 0;
    const uint32_t depth = st.y & 31u;
    uint4 mine = make_uint4(0u, 0u, 0u, 0u);
    if ((uint32_t)lane < depth)
        mine = *reinterpret_cast<const uint4 *>(sc.kd_rows + 4 * ((size_t)(st.y >> 5) + (size_t)lane));
    const float yx = rt_recip_guard(d.x), yy = rt_recip_guard(d.y), yz = rt_recip_guard(d.z);
    float ex = exit_; // the current interval's exit: the root's, then the last push's t
    int sp = 0;
    for (uint32_t i = 0; i < depth; ++i) {
        const uint32_t rx = (uint32_t)__builtin_amdgcn_readlane((int)mine.x, (int)i);
        const uint32_t ry = (uint32_t)__builtin_amdgcn_readlane((int)mine.y, (int)i);
        const uint32_t anc = (uint32_t)__builtin_amdgcn_readlane((int)mine.z, (int)i);
        const uint32_t rw = (uint32_t)__builtin_amdgcn_readlane((int)mine.w, (int)i);
        const uint32_t axis = ry & 3u;
        const float split = as_float(rx);
        const float oax = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
        const float dax = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
        const float yax = axis == 0 ? yx : (axis == 1 ? yy : yz);
        uint32_t near_c = anc + 1, far_c = ry >> 2;
        if (oax >= split) { // ray_behind_plane (rt/trace_ray.cuh:174-188)
            near_c = ry >> 2;
            far_c = anc + 1;
        }
        const uint32_t taken = rw ? ry >> 2 : anc + 1;
        if (near_c != taken) return 0;
        const float t = rt_div_by(split - oax, dax, yax); // intersect_plane (:190-210)
        if (t >= ex || t < 0) continue; // near only
        if (!(t > entry)) return 0;     // far only (or NaN): not the origin's way
        if (lane == 0) W.F[sp] = WideItem{far_c, t, ex, (uint32_t)sp << WIDE_SP_SHIFT}; // exit: the entry below
        ++sp;
        ex = t;
    }
    if (lane == 0) W.F[sp] = WideItem{st.x, entry, ex, (uint32_t)sp << WIDE_SP_SHIFT};
    return sp + 1;
}

// Finish lane `owner`'s ray, which is in the middle of its cooperative
// traversal, with all 64 lanes: its sequential state is already an ordered
// frontier — stack entries 0..sp-1 (bottom = last in traversal order, each
// with exit = the entry below it, or the root exit) under the current node
// [entry, exit].  A pending leaf was counted when reached, so it is marked
// WIDE_COUNTED.  `stk_owner` addresses the owner lane's stack.  Call with
// all lanes active; results are wave-uniform.
template <bool COUNT, int LDS_DEPTH>
__device__ __forceinline__ void wide_resume(const RtDevScene &sc, const CoopRay &r, int owner,
                                            const Stack<LDS_DEPTH> &stk_owner, const WideLds &W, int &tri,
                                            float &hbx, float &hby, float &hbz, Cnt &c)
{
    const int lane = __lane_id();
    const int sp = __shfl(r.sp, owner);
    const Vec3D o = rt_v3(__shfl(r.o.x, owner), __shfl(r.o.y, owner), __shfl(r.o.z, owner));
    const Vec3D d = rt_v3(__shfl(r.d.x, owner), __shfl(r.d.y, owner), __shfl(r.d.z, owner));
    uint32_t node = 0;
    float entry = 0.0f;
    if (lane < sp) stk_owner.get(lane, node, entry);
    const float below = __shfl_up(entry, 1); // entry of the stack entry below = this one's exit
    const float root_exit = __shfl(r.root_exit, owner);
    if (lane < sp) W.F[lane] = WideItem{node, entry, lane > 0 ? below : root_exit, (uint32_t)lane << WIDE_SP_SHIFT};
    if (lane == owner)
        W.F[sp] = WideItem{r.node, r.entry, r.exit_, (r.pend ? WIDE_COUNTED : 0u) | (uint32_t)sp << WIDE_SP_SHIFT};
    wide_trace_from<COUNT>(sc, o, d, sp + 1, W, lane == owner, tri, hbx, hby, hbz, c);
}

} // namespace rtk
