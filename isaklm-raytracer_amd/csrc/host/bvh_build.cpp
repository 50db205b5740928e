// bvh_build.cpp — binned-SAH BVH over the triangles' conservative boxes
// (bvh_build.h explains what it is for and why the boxes are grown).
//
// Top-down, 32 bins on the widest centroid axis, surface-area heuristic with
// leaves of at most 8 triangles; the binning of large nodes runs on all
// cores.  Output: binary nodes holding both children's boxes (4 float4,
// one cache line; bvh_trace.h reads them), pre-order, children referenced
// by index or as a leaf (triangle range in `order`).
#include <cmath>
#include <float.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "bvh_build.h"
#include "rt_host.h"

namespace rt_host {

namespace {

struct Box {
    float lo[3], hi[3];
    void empty()
    {
        for (int a = 0; a < 3; ++a) {
            lo[a] = FLT_MAX;
            hi[a] = -FLT_MAX;
        }
    }
    void grow(const Box &b)
    {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b.lo[a]);
            hi[a] = std::max(hi[a], b.hi[a]);
        }
    }
    void grow(const float *p)
    {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], p[a]);
            hi[a] = std::max(hi[a], p[a]);
        }
    }
    double area() const
    {
        if (hi[0] < lo[0]) return 0.0;
        const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
        return 2.0 * (x * y + y * z + z * x);
    }
};

constexpr int kBins = 32;
constexpr int kLeafMax = RT_BVH_LEAF_MAX;
constexpr uint32_t kLeafBit = RT_BVH_LEAF;

struct TNode {
    Box box;
    int left = -1, right = -1; // temporary children (inner)
    int first = 0, count = 0;  // leaf range
};

struct Builder {
    std::vector<Box> pbox;
    std::vector<float> cen; // 3 per primitive
    std::vector<uint32_t> prim;
    std::vector<TNode> nodes;
    int max_depth = 0;

    Box bounds(int b, int e, Box &cb) const
    {
        Box bb;
        bb.empty();
        cb.empty();
        const int n = e - b;
        if (n > 65536) {
#pragma omp parallel
            {
                Box lb, lc;
                lb.empty();
                lc.empty();
#pragma omp for schedule(static) nowait
                for (int i = b; i < e; ++i) {
                    lb.grow(pbox[prim[i]]);
                    lc.grow(&cen[3 * (size_t)prim[i]]);
                }
#pragma omp critical
                {
                    bb.grow(lb);
                    cb.grow(lc);
                }
            }
        } else {
            for (int i = b; i < e; ++i) {
                bb.grow(pbox[prim[i]]);
                cb.grow(&cen[3 * (size_t)prim[i]]);
            }
        }
        return bb;
    }

    // returns the node index
    int build(int b, int e, int depth)
    {
        max_depth = std::max(max_depth, depth);
        Box cb;
        const Box bb = bounds(b, e, cb);
        const int id = (int)nodes.size();
        nodes.push_back(TNode{});
        nodes[id].box = bb;
        const int n = e - b;
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if (cb.hi[a] - cb.lo[a] > cb.hi[axis] - cb.lo[axis]) axis = a;
        const float ext = cb.hi[axis] - cb.lo[axis];
        int mid = -1;
        if (n > kLeafMax || (n > 2 && ext > 0.0f)) {
            // (SAH down to depth 40, then object medians: the depth stays below
            // RT_BVH_STACK for any triangle count below 2^24)
            if (ext > 0.0f && depth < 40) {
                // binned SAH
                Box binb[kBins];
                int binc[kBins] = {};
                for (auto &x : binb) x.empty();
                const float k = (float)kBins * (1.0f - 1e-6f) / ext;
                auto bin_of = [&](uint32_t p) {
                    int i = (int)((cen[3 * (size_t)p + axis] - cb.lo[axis]) * k);
                    return i < 0 ? 0 : (i >= kBins ? kBins - 1 : i);
                };
                if (n > 65536) {
#pragma omp parallel
                    {
                        Box lb[kBins];
                        int lc[kBins] = {};
                        for (auto &x : lb) x.empty();
#pragma omp for schedule(static) nowait
                        for (int i = b; i < e; ++i) {
                            const int j = bin_of(prim[i]);
                            lb[j].grow(pbox[prim[i]]);
                            ++lc[j];
                        }
#pragma omp critical
                        for (int j = 0; j < kBins; ++j) {
                            binb[j].grow(lb[j]);
                            binc[j] += lc[j];
                        }
                    }
                } else {
                    for (int i = b; i < e; ++i) {
                        const int j = bin_of(prim[i]);
                        binb[j].grow(pbox[prim[i]]);
                        ++binc[j];
                    }
                }
                double ra[kBins];
                int rc[kBins];
                Box acc;
                acc.empty();
                int cnt = 0;
                for (int j = kBins - 1; j > 0; --j) {
                    acc.grow(binb[j]);
                    cnt += binc[j];
                    ra[j] = acc.area();
                    rc[j] = cnt;
                }
                acc.empty();
                cnt = 0;
                double best = 1e300;
                int best_j = -1;
                for (int j = 1; j < kBins; ++j) {
                    acc.grow(binb[j - 1]);
                    cnt += binc[j - 1];
                    if (cnt == 0 || rc[j] == 0) continue;
                    const double c = acc.area() * cnt + ra[j] * rc[j];
                    if (c < best) {
                        best = c;
                        best_j = j;
                    }
                }
                const double leaf_cost = bb.area() * n;
                const bool split = best_j > 0 && (n > kLeafMax || best < leaf_cost * 0.9);
                if (split) {
                    auto it = std::partition(prim.begin() + b, prim.begin() + e,
                                             [&](uint32_t p) { return bin_of(p) < best_j; });
                    mid = (int)(it - prim.begin());
                    if (mid == b || mid == e) mid = -1;
                }
            }
            if (mid < 0 && n > kLeafMax) { // no useful SAH split (coincident centroids): object median
                mid = b + n / 2;
                std::nth_element(prim.begin() + b, prim.begin() + mid, prim.begin() + e, [&](uint32_t x, uint32_t y) {
                    return cen[3 * (size_t)x + axis] < cen[3 * (size_t)y + axis];
                });
            }
        }
        if (mid < 0) {
            nodes[id].first = b;
            nodes[id].count = n;
            return id;
        }
        const int l = build(b, mid, depth + 1);
        const int r = build(mid, e, depth + 1);
        nodes[id].left = l;
        nodes[id].right = r;
        return id;
    }
};

inline float f_of(uint32_t u)
{
    float f;
    memcpy(&f, &u, 4);
    return f;
}

} // namespace

int build_bvh(const Triangle *tris, int ntris, const RtF4 *plane, const RtIsectBary *bary, BvhHost &out)
{
    out = BvhHost{};
    Builder B;
    B.pbox.resize((size_t)ntris);
    B.cen.resize(3 * (size_t)ntris);
    std::vector<float> margin((size_t)ntris);
    double scale = 0.0;
    Box scene;
    scene.empty();
    for (int i = 0; i < ntris; ++i) {
        const Triangle &t = tris[i];
        const Vec3D ps[3] = {t.p1, t.p2, t.p3};
        for (const Vec3D &p : ps) {
            const float q[3] = {p.x, p.y, p.z};
            if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
                scene.grow(q);
                scale = std::max(scale, (double)fabsf(p.x) + fabsf(p.y) + fabsf(p.z));
            }
        }
    }
    if (!(scene.hi[0] >= scene.lo[0])) { // no finite vertex at all
        scene.lo[0] = scene.lo[1] = scene.lo[2] = 0.0f;
        scene.hi[0] = scene.hi[1] = scene.hi[2] = 0.0f;
    }
    out.scale = (float)scale;
    // the whole-scene box (for triangles whose margin bound is useless), grown
    const float grow = 0x1p-10f * (float)(scale + 1.0);
    Box all = scene;
    for (int a = 0; a < 3; ++a) {
        all.lo[a] -= grow;
        all.hi[a] += grow;
    }
    std::vector<uint32_t> keep;
    keep.reserve((size_t)ntris);
    std::vector<char> always_tri((size_t)ntris, 0);
    for (int i = 0; i < ntris; ++i) {
        const RtIsectBary &r = bary[i];
        const Vec3D p1 = rt_v3(r.b.x, r.b.y, r.b.z), v0 = rt_v3(r.c.x, r.c.y, r.c.z), v1 = rt_v3(r.d.x, r.d.y, r.d.z);
        const float m = tri_margin(p1, v0, v1, f_of(r.rd), plane[i].x, plane[i].y, plane[i].z);
        if (m != m) {
            ++out.dropped;
            continue;
        }
        const Triangle &t = tris[i];
        Box b;
        if (isinf(m) || !isfinite(t.p1.x + t.p1.y + t.p1.z + t.p2.x + t.p2.y + t.p2.z + t.p3.x + t.p3.y + t.p3.z)) {
            b = all;
            always_tri[(size_t)i] = 1;
            ++out.always;
        } else {
            b.empty();
            const float q1[3] = {t.p1.x, t.p1.y, t.p1.z}, q2[3] = {t.p2.x, t.p2.y, t.p2.z},
                        q3[3] = {t.p3.x, t.p3.y, t.p3.z};
            b.grow(q1);
            b.grow(q2);
            b.grow(q3);
            for (int a = 0; a < 3; ++a) {
                // grown by the margin, then rounded outward
                b.lo[a] = nextafterf(b.lo[a] - m, -INFINITY);
                b.hi[a] = nextafterf(b.hi[a] + m, INFINITY);
            }
        }
        B.pbox[(size_t)i] = b;
        for (int a = 0; a < 3; ++a) B.cen[3 * (size_t)i + a] = 0.5f * (b.lo[a] + b.hi[a]);
        keep.push_back((uint32_t)i);
    }
    auto put = [&](size_t k, const Box &b0, const Box &b1, uint32_t c0, uint32_t c1) {
        out.nodes[4 * k + 0] = RtF4{b0.lo[0], b0.lo[1], b0.lo[2], b0.hi[0]};
        out.nodes[4 * k + 1] = RtF4{b0.hi[1], b0.hi[2], b1.lo[0], b1.lo[1]};
        out.nodes[4 * k + 2] = RtF4{b1.lo[2], b1.hi[0], b1.hi[1], b1.hi[2]};
        out.nodes[4 * k + 3] = RtF4{f_of(c0), f_of(c1), 0.0f, 0.0f};
    };
    Box none;
    none.empty();
    if (keep.empty()) { // nothing can ever be hit: a root with two empty children
        out.nodes.assign(4, RtF4{0, 0, 0, 0});
        put(0, none, none, RT_BVH_EMPTY, RT_BVH_EMPTY);
        return RT_OK;
    }
    if (keep.size() >= (1u << 28)) {
        rt_set_error("bvh: too many triangles");
        return RT_E_UNSUPPORTED;
    }
    B.prim = keep;
    B.nodes.reserve(2 * keep.size() / 3 + 16);
    B.build(0, (int)keep.size(), 0);
    out.depth = B.max_depth;
    out.order = B.prim;
    // An always-tested triangle (no usable margin) may pass a test with its hit point anywhere on
    // the ray — even before the ray enters the scene box (the adversarial scene's slivers: a pass
    // at s = 1.91 for a box entry of 2.62) —, so the boxes of its leaf and of every ancestor are
    // unbounded (tn = -inf for every ray): visited whatever the query's best, they keep s_min a
    // lower bound of every passing test.  (The splits were chosen on the finite scene box above.)
    if (out.always > 0) {
        std::vector<char> inf(B.nodes.size(), 0);
        for (size_t id = B.nodes.size(); id-- > 0;) { // children are created after their parent
            const TNode &t = B.nodes[id];
            if (t.left < 0) {
                for (int k = t.first; k < t.first + t.count; ++k) inf[id] |= always_tri[(size_t)B.prim[(size_t)k]];
            } else {
                inf[id] = inf[(size_t)t.left] | inf[(size_t)t.right];
            }
            if (inf[id]) {
                for (int a = 0; a < 3; ++a) {
                    B.nodes[id].box.lo[a] = -INFINITY;
                    B.nodes[id].box.hi[a] = INFINITY;
                }
            }
        }
    }

    // flatten: every temporary inner node becomes one dual-box node (pre-order)
    std::vector<int> flat((size_t)B.nodes.size(), -1);
    std::vector<int> inner_order;
    {
        std::vector<int> st{0};
        while (!st.empty()) {
            const int id = st.back();
            st.pop_back();
            const TNode &t = B.nodes[(size_t)id];
            if (t.left < 0) continue;
            flat[(size_t)id] = (int)inner_order.size();
            inner_order.push_back(id);
            st.push_back(t.right);
            st.push_back(t.left);
        }
    }
    auto ref = [&](int id) -> uint32_t {
        const TNode &t = B.nodes[(size_t)id];
        if (t.left >= 0) return (uint32_t)flat[(size_t)id];
        return kLeafBit | ((uint32_t)t.first << 3) | (uint32_t)(t.count - 1);
    };
    if (inner_order.empty()) { // the root is a leaf: a root node with the leaf and an empty child
        out.nodes.assign(4, RtF4{0, 0, 0, 0});
        put(0, B.nodes[0].box, none, ref(0), RT_BVH_EMPTY);
        return RT_OK;
    }
    out.nodes.assign(4 * inner_order.size(), RtF4{0, 0, 0, 0});
    for (size_t k = 0; k < inner_order.size(); ++k) {
        const TNode &t = B.nodes[(size_t)inner_order[k]];
        put(k, B.nodes[(size_t)t.left].box, B.nodes[(size_t)t.right].box, ref(t.left), ref(t.right));
    }
    return RT_OK;
}

// The 4-wide collapse (bvh_build.h): starting from a binary node's two
// children, the inner child with the largest box surface is replaced by its
// two children until there are 4 (or only leaves).  Child boxes and leaf
// references are the binary tree's own; an inner child refers to its 4-wide
// node.  Layout per node (8 RtF4, 128 B): lo.x, lo.y, lo.z, hi.x, hi.y, hi.z
// of children 0..3 (one RtF4 each), then the 4 references, then padding;
// unused slots hold RT_BVH_EMPTY.
void collapse_bvh4(const std::vector<RtF4> &bin, std::vector<RtF4> &out4)
{
    out4.clear();
    const size_t nb = bin.size() / 4;
    if (nb == 0) return;
    struct Child {
        uint32_t ref;
        float lo[3], hi[3];
    };
    auto child_of = [&](uint32_t node, int c) {
        const RtF4 *nd = &bin[4 * (size_t)node];
        Child ch;
        memcpy(&ch.ref, c == 0 ? &nd[3].x : &nd[3].y, 4);
        if (c == 0) {
            ch.lo[0] = nd[0].x; ch.lo[1] = nd[0].y; ch.lo[2] = nd[0].z;
            ch.hi[0] = nd[0].w; ch.hi[1] = nd[1].x; ch.hi[2] = nd[1].y;
        } else {
            ch.lo[0] = nd[1].z; ch.lo[1] = nd[1].w; ch.lo[2] = nd[2].x;
            ch.hi[0] = nd[2].y; ch.hi[1] = nd[2].z; ch.hi[2] = nd[2].w;
        }
        return ch;
    };
    std::vector<int> idx(nb, -1);
    std::vector<std::vector<Child>> wide; // per 4-wide node, its children (binary refs)
    std::vector<uint32_t> order{0};
    idx[0] = 0;
    for (size_t q = 0; q < order.size(); ++q) {
        const uint32_t b = order[q];
        std::vector<Child> ch;
        for (int c = 0; c < 2; ++c) {
            const Child x = child_of(b, c);
            if (x.ref != RT_BVH_EMPTY) ch.push_back(x);
        }
        while (ch.size() < 4) {
            int pick = -1;
            float area = -1.0f;
            for (size_t k = 0; k < ch.size(); ++k) {
                if (ch[k].ref & RT_BVH_LEAF) continue;
                const float ex = ch[k].hi[0] - ch[k].lo[0], ey = ch[k].hi[1] - ch[k].lo[1], ez = ch[k].hi[2] - ch[k].lo[2];
                const float a = ex * ey + ey * ez + ez * ex;
                if (!(a <= area)) { // (NaN or larger: take it)
                    area = a;
                    pick = (int)k;
                }
            }
            if (pick < 0) break;
            const uint32_t inner = ch[(size_t)pick].ref;
            ch.erase(ch.begin() + pick);
            for (int c = 0; c < 2; ++c) {
                const Child x = child_of(inner, c);
                if (x.ref != RT_BVH_EMPTY) ch.push_back(x);
            }
        }
        for (const Child &x : ch)
            if (!(x.ref & RT_BVH_LEAF) && idx[x.ref] < 0) {
                idx[x.ref] = (int)order.size();
                order.push_back(x.ref);
            }
        wide.push_back(std::move(ch));
    }
    out4.assign(8 * wide.size(), RtF4{0, 0, 0, 0});
    for (size_t i = 0; i < wide.size(); ++i) {
        float *f = reinterpret_cast<float *>(&out4[8 * i]);
        for (int k = 0; k < 4; ++k) {
            uint32_t ref = RT_BVH_EMPTY;
            // an unused slot's box lies at +FLT_MAX on every axis: every ray's slab test culls it (entry
            // +inf or huge where an axis's 1/d > 0, exit -inf where every 1/d < 0; |1/d| >= 1 for a unit
            // direction), so the query needs no reference check (bvh_trace.h bvh4_children)
            for (int a = 0; a < 6; ++a) f[4 * a + k] = FLT_MAX;
            if ((size_t)k < wide[i].size()) {
                const Child &x = wide[i][(size_t)k];
                ref = (x.ref & RT_BVH_LEAF) ? x.ref : (uint32_t)idx[x.ref];
                for (int a = 0; a < 3; ++a) {
                    f[4 * a + k] = x.lo[a];
                    f[4 * (3 + a) + k] = x.hi[a];
                }
            }
            memcpy(&f[4 * 6 + k], &ref, 4);
        }
    }
}

} // namespace rt_host
