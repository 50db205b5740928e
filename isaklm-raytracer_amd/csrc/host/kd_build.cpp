// kd_build.cpp — create_kd_tree (rt/create_kd_tree.cuh:18-328), same tree.
//
// The traversal result depends on the exact tree, so this
// builder reproduces the reference's choices bit for bit:
//   * axis = depth % 3 (:164)
//   * split = the (n/2)-th smallest AABB centre (min+max)*0.5f (:125-160);
//     std::nth_element finds the same value std::sort()[n/2] does
//   * a triangle goes left iff min <= split, right iff max >= split (:59-123),
//     both when it straddles; order inside a child = parent order (:192-219)
//   * a child is split iff count > 7 and depth < KD_TREE_DEPTH (:222-246)
//   * pre-order numbering: child1's subtree, then child2 (:225-264); leaves
//     append their indices in that order; root AABB padded by 0.01f (:18-57)
// What differs is only the schedule: the top levels build child subtrees in
// parallel (OpenMP tasks) into private arrays that are then spliced in
// pre-order, so the 2M-triangle build takes a fraction of the reference's
// 6.8 s.
#include <string.h>

#include <algorithm>
#include <cfloat>
#include <vector>

#include "rt_host.h"

namespace rt_host {
namespace {

struct Bounds6 { float mn[3], mx[3]; };

struct Sub {
    std::vector<KD_Tree_Node> nodes;
    std::vector<int> idx;
};

const int kMinTriangleCount = 7; // :222
const int kParallelDepth = 7;    // subtrees above this depth are built as tasks

KD_Tree_Node make_node(int a, int b, bool leaf)
{
    KD_Tree_Node n;
    memset(&n, 0, sizeof n);
    n.index_offset = a;
    n.triangle_count = b;
    n.plane_axis = 0;
    n.plane_offset = 0.0f;
    n.is_leaf_node = leaf;
    return n;
}

// splice `s` (local numbering) into `out`; returns the spliced root index
int splice(Sub &out, const Sub &s)
{
    const int node_base = (int)out.nodes.size();
    const int idx_base = (int)out.idx.size();
    for (KD_Tree_Node n : s.nodes) {
        if (n.is_leaf_node) {
            n.index_offset += idx_base;
        } else {
            n.child_index1 += node_base;
            n.child_index2 += node_base;
        }
        out.nodes.push_back(n);
    }
    out.idx.insert(out.idx.end(), s.idx.begin(), s.idx.end());
    return node_base;
}

struct Builder {
    const Bounds6 *tb;

    float plane_offset(const std::vector<int> &ids, int axis) const // :125-160
    {
        std::vector<float> v(ids.size());
        for (size_t i = 0; i < ids.size(); ++i) v[i] = (tb[ids[i]].mn[axis] + tb[ids[i]].mx[axis]) * 0.5f;
        const size_t mid = v.size() / 2;
        std::nth_element(v.begin(), v.begin() + (ptrdiff_t)mid, v.end());
        return v[mid];
    }

    // add_child_nodes (:162-265) for node `parent` of `out`
    void add_child_nodes(Sub &out, int parent, const std::vector<int> &ids, int depth) const
    {
        const int axis = depth % 3;
        const float split = plane_offset(ids, axis);
        out.nodes[parent].plane_axis = (uint8_t)axis;
        out.nodes[parent].plane_offset = split;
        std::vector<int> c1, c2;
        c1.reserve(ids.size());
        c2.reserve(ids.size());
        for (int id : ids) {
            if (tb[id].mn[axis] <= split) c1.push_back(id); // triangle_behind_plane
            if (tb[id].mx[axis] >= split) c2.push_back(id); // triangle_afore_plane
        }
        const bool split1 = (int)c1.size() > kMinTriangleCount && depth < RT_KD_TREE_DEPTH;
        const bool split2 = (int)c2.size() > kMinTriangleCount && depth < RT_KD_TREE_DEPTH;

        if (split1 && split2 && depth < kParallelDepth) {
            Sub s1, s2;
#pragma omp task shared(s1, c1)
            build_subtree(s1, c1, depth + 1);
#pragma omp task shared(s2, c2)
            build_subtree(s2, c2, depth + 1);
#pragma omp taskwait
            out.nodes[parent].child_index1 = splice(out, s1);
            out.nodes[parent].child_index2 = splice(out, s2);
            return;
        }
        for (int side = 0; side < 2; ++side) {
            const std::vector<int> &c = side == 0 ? c1 : c2;
            const bool rec = side == 0 ? split1 : split2;
            const int child = (int)out.nodes.size();
            if (side == 0) out.nodes[parent].child_index1 = child;
            else out.nodes[parent].child_index2 = child;
            if (rec) {
                out.nodes.push_back(make_node(0, 0, false));
                add_child_nodes(out, child, c, depth + 1);
            } else {
                out.nodes.push_back(make_node((int)out.idx.size(), (int)c.size(), true));
                out.idx.insert(out.idx.end(), c.begin(), c.end());
            }
        }
    }

    void build_subtree(Sub &s, const std::vector<int> &ids, int depth) const
    {
        s.nodes.push_back(make_node(0, 0, false));
        add_child_nodes(s, 0, ids, depth);
    }
};

} // namespace

int build_kd_tree(const Triangle *tris, int n, std::vector<KD_Tree_Node> &nodes, std::vector<int> &indices,
                  Bounding_Box &bounds)
{
    if (n <= 0) {
        rt_set_error("build_kd_tree: empty triangle list");
        return RT_E_INVALID;
    }
    std::vector<Bounds6> tb((size_t)n);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        const float *p1 = &tris[i].p1.x, *p2 = &tris[i].p2.x, *p3 = &tris[i].p3.x;
        for (int a = 0; a < 3; ++a) {
            tb[i].mn[a] = fminf(p1[a], fminf(p2[a], p3[a]));
            tb[i].mx[a] = fmaxf(p1[a], fmaxf(p2[a], p3[a]));
        }
    }
    std::vector<int> root(n);
    for (int i = 0; i < n; ++i) root[i] = i;
    Builder b{tb.data()};
    Sub s;
#pragma omp parallel
#pragma omp single
    b.build_subtree(s, root, 0);
    nodes.swap(s.nodes);
    indices.swap(s.idx);

    // get_bounding_box (:18-57)
    const float eps = 0.01f;
    bounds.min = rt_v3(FLT_MAX, FLT_MAX, FLT_MAX);
    bounds.max = -rt_v3(FLT_MAX, FLT_MAX, FLT_MAX);
    for (int i = 0; i < n; ++i) {
        bounds.min.x = fminf(tb[i].mn[0], bounds.min.x);
        bounds.min.y = fminf(tb[i].mn[1], bounds.min.y);
        bounds.min.z = fminf(tb[i].mn[2], bounds.min.z);
        bounds.max.x = fmaxf(tb[i].mx[0], bounds.max.x);
        bounds.max.y = fmaxf(tb[i].mx[1], bounds.max.y);
        bounds.max.z = fmaxf(tb[i].mx[2], bounds.max.z);
    }
    bounds.min = bounds.min - rt_v3(eps, eps, eps);
    bounds.max = bounds.max + rt_v3(eps, eps, eps);
    return RT_OK;
}

} // namespace rt_host
