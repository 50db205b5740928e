// scene_prepare.cpp — reference-layout Scene -> traversal layout (rt_device.h).
//
// Bit-preserving: the per-triangle constants are exactly the sub-expressions
// intersect_triangle / calculate_barycentric_coordinates compute per test
// (rt/trace_ray.cuh:48-113), evaluated once here with the same operations
// (-ffp-contract=off), so a test on the GPU sees the same floats.  Nodes are
// renumbered into pre-order with child1 == node + 1, which is the identity
// for trees from create_kd_tree (rt/create_kd_tree.cuh:225-258) and keeps
// traversal order for any other tree.
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "bvh_build.h"
#include "rt_host.h"

namespace rt_host {

static inline uint32_t fbits(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
static inline float bitsf(uint32_t u)
{
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static inline RtF4 f4(float x, float y, float z, float w) { return RtF4{x, y, z, w}; }

// The origin-cell entry of wf_long's deep bounces (coop_trace.h
// kd_origin_frontier): trace_ray descends, at every split, to the side
// holding the ray's origin until the split separates the origin from the
// ray's interval.  For each cell of a uniform grid over the scene box, the
// deepest KD node whose cell holds the grid cell is where that descent passes
// for an origin in it; its root path, stored as one record per ancestor, lets
// the wide traversal replay those decisions from independent loads — and
// check each against the path, falling back to the root on any difference,
// so the entry never changes a result.
void build_kd_starts(PreparedHost &out, const Bounding_Box &bounds)
{
    out.kd_rows.clear();
    out.kd_cell.clear();
    out.kd_grid = 0;
    if (out.nodes.empty()) return;
    std::unordered_map<uint32_t, uint32_t> row_of; // start node -> row offset
    std::vector<uint32_t> path;
    // {start node, row offset << 5 | depth} of the deepest node holding [lo, hi] (depth <= 31)
    // (cb: the start node's own cell, from its ancestors' splits; +-inf where none bounds it)
    auto start_for = [&](const float *lo, const float *hi, uint32_t &start, uint32_t &packed, float *cb) {
        path.clear();
        uint32_t n = 0;
        for (int a = 0; a < 3; ++a) {
            cb[a] = -INFINITY;
            cb[3 + a] = INFINITY;
        }
        while (path.size() < 31) {
            const uint32_t x = out.nodes[2 * (size_t)n], y = out.nodes[2 * (size_t)n + 1];
            if ((y & 3u) == RT_LEAF_TAG) break;
            float split;
            memcpy(&split, &x, 4);
            const int a = (int)(y & 3u);
            uint32_t next;
            // (the tightest split per side: a split need not lie inside its node's cell)
            if (hi[a] < split) {        // below the split: child0 (node + 1)
                next = n + 1;
                cb[3 + a] = std::min(cb[3 + a], split);
            } else if (lo[a] > split) { // above: child1
                next = y >> 2;
                cb[a] = std::max(cb[a], split);
            } else {
                break;                  // the box straddles the split
            }
            path.push_back(n);
            n = next;
        }
        auto it = row_of.find(n);
        uint32_t off;
        if (it != row_of.end()) {
            off = it->second;
        } else {
            off = (uint32_t)(out.kd_rows.size() / 4);
            if (off >= (1u << 27)) return false; // (row offsets are 27 bits)
            for (size_t k = 0; k < path.size(); ++k) {
                const uint32_t anc = path[k], nxt = k + 1 < path.size() ? path[k + 1] : n;
                out.kd_rows.push_back(out.nodes[2 * (size_t)anc]);
                out.kd_rows.push_back(out.nodes[2 * (size_t)anc + 1]);
                out.kd_rows.push_back(anc);
                out.kd_rows.push_back(nxt == anc + 1 ? 0u : 1u);
            }
            row_of.emplace(n, off);
        }
        start = n;
        packed = off << 5 | (uint32_t)path.size();
        return true;
    };
    // the grid: G^3 cells over the scene box (G ~ the tree's node count^(1/3), 4..128)
    const float ext[3] = {bounds.max.x - bounds.min.x, bounds.max.y - bounds.min.y, bounds.max.z - bounds.min.z};
    if (!(ext[0] > 0 && ext[1] > 0 && ext[2] > 0 && std::isfinite(ext[0] + ext[1] + ext[2]))) return;
    int G = (int)std::cbrt((double)(out.nodes.size() / 2));
    G = G < 4 ? 4 : (G > 128 ? 128 : G);
    const float bmin[3] = {bounds.min.x, bounds.min.y, bounds.min.z};
    out.kd_cell.assign(2 * (size_t)G * G * G, 0xFFFFFFFFu);
    for (int z = 0; z < G; ++z)
        for (int y = 0; y < G; ++y)
            for (int x = 0; x < G; ++x) {
                const int c[3] = {x, y, z};
                float lo[3], hi[3];
                for (int a = 0; a < 3; ++a) {
                    lo[a] = bmin[a] + ext[a] * (float)c[a] / (float)G;
                    hi[a] = bmin[a] + ext[a] * (float)(c[a] + 1) / (float)G;
                }
                const size_t k = ((size_t)z * G + y) * G + x;
                float cb[6];
                if (!start_for(lo, hi, out.kd_cell[2 * k], out.kd_cell[2 * k + 1], cb))
                    out.kd_cell[2 * k] = out.kd_cell[2 * k + 1] = 0xFFFFFFFFu;
            }
    out.kd_grid = G;
    for (int a = 0; a < 3; ++a) out.kd_grid_scale[a] = (float)G / ext[a];
}

int prepare_host(const Triangle *tris, int ntris, const KD_Tree_Node *nodes, int nnodes, const int *indices,
                 int nindices, const int *lights, int nlights, Bounding_Box bounds, PreparedHost &out)
{
    if (ntris <= 0 || nnodes <= 0 || !tris || !nodes || (nindices > 0 && !indices) || nlights < 0 ||
        (nlights > 0 && !lights)) {
        rt_set_error("prepare: invalid scene arrays");
        return RT_E_INVALID;
    }
    if (ntris >= (1 << 30) || nnodes >= (1 << 30) || nindices >= (1 << 30)) {
        rt_set_error("prepare: scene too large for 30-bit node/leaf fields");
        return RT_E_UNSUPPORTED;
    }
    // --- nodes: pre-order renumbering + validation -----------------------
    std::vector<int> new_id((size_t)nnodes, -1);
    std::vector<int> order;
    order.reserve((size_t)nnodes);
    struct Item { int node, depth; };
    std::vector<Item> st;
    st.push_back({0, 0});
    int max_depth = 0;
    while (!st.empty()) {
        Item it = st.back();
        st.pop_back();
        if (it.node < 0 || it.node >= nnodes || new_id[it.node] != -1) {
            rt_set_error("prepare: KD node %d out of range or shared", it.node);
            return RT_E_INVALID;
        }
        new_id[it.node] = (int)order.size();
        order.push_back(it.node);
        const KD_Tree_Node &n = nodes[it.node];
        if (!n.is_leaf_node) {
            if (n.plane_axis > 2) {
                rt_set_error("prepare: node %d has plane axis %d", it.node, (int)n.plane_axis);
                return RT_E_INVALID;
            }
            max_depth = it.depth + 1 > max_depth ? it.depth + 1 : max_depth;
            st.push_back({n.child_index2, it.depth + 1}); // popped after child1's subtree
            st.push_back({n.child_index1, it.depth + 1});
        } else if (n.triangle_count < 0 || n.index_offset < 0 ||
                   (n.triangle_count > 0 && (long long)n.index_offset + n.triangle_count > nindices)) {
            rt_set_error("prepare: leaf %d addresses indices out of range", it.node);
            return RT_E_INVALID;
        }
    }
    if (max_depth > RT_STACK_DEPTH) {
        rt_set_error("prepare: KD tree depth %d exceeds the traversal stack (%d)", max_depth, RT_STACK_DEPTH);
        return RT_E_UNSUPPORTED;
    }
    out.max_depth = max_depth;
    out.nodes.assign(2 * order.size(), 0u);
    for (size_t k = 0; k < order.size(); ++k) {
        const KD_Tree_Node &n = nodes[order[k]];
        if (n.is_leaf_node) {
            out.nodes[2 * k] = (uint32_t)n.index_offset;
            out.nodes[2 * k + 1] = ((uint32_t)n.triangle_count << 2) | RT_LEAF_TAG;
        } else {
            if (new_id[n.child_index1] != (int)k + 1) {
                rt_set_error("prepare: internal renumbering error");
                return RT_E_INVALID;
            }
            out.nodes[2 * k] = fbits(n.plane_offset);
            out.nodes[2 * k + 1] = ((uint32_t)new_id[n.child_index2] << 2) | (uint32_t)n.plane_axis;
        }
    }
    for (int i = 0; i < nindices; ++i)
        if (indices[i] < 0 || indices[i] >= ntris) {
            rt_set_error("prepare: triangle index %d out of range", indices[i]);
            return RT_E_INVALID;
        }

    // --- materials (deduplicated by value) --------------------------------
    std::map<std::string, int> mat_ids;
    std::vector<int> tri_mat((size_t)ntris);
    out.materials.clear();
    for (int i = 0; i < ntris; ++i) {
        const Material &m = tris[i].material;
        RtDevMaterial d;
        memset(&d, 0, sizeof d);
        d.albedo[0] = m.albedo.x; d.albedo[1] = m.albedo.y; d.albedo[2] = m.albedo.z;
        d.roughness = m.roughness;
        d.emittance[0] = m.emittance.x; d.emittance[1] = m.emittance.y; d.emittance[2] = m.emittance.z;
        d.refractive_index = m.refractive_index;
        d.extinction = m.extinction;
        d.transparent = m.transparent ? 1 : 0;
        d.tex = m.texture.buffer;
        d.tex_width = m.texture.buffer ? m.texture.width : 0;
        d.tex_height = m.texture.buffer ? m.texture.height : 0;
        std::string key((const char *)&d, sizeof d);
        auto it = mat_ids.find(key);
        if (it == mat_ids.end()) {
            it = mat_ids.emplace(key, (int)out.materials.size()).first;
            out.materials.push_back(d);
        }
        tri_mat[i] = it->second;
    }

    // --- intersection constants (rt/trace_ray.cuh:48-113), per triangle ---
    std::vector<RtF4> ta((size_t)ntris);
    std::vector<RtIsectBary> tbary((size_t)ntris);
    out.shade.resize(7 * (size_t)ntris);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < ntris; ++i) {
        const Triangle &t = tris[i];
        Vec3D v0 = t.p2 - t.p1;
        Vec3D v1 = t.p3 - t.p1;
        Vec3D n = rt_normalize(rt_cross(v0, v1)); // cross(p2 - p1, p3 - p1)
        float d = rt_dot(n, t.p1);
        float d00 = rt_dot(v0, v0), d01 = rt_dot(v0, v1), d11 = rt_dot(v1, v1);
        float rd = 1.0f / (d00 * d11 - d01 * d01);
        ta[i] = f4(n.x, n.y, n.z, d);
        RtIsectBary &r = tbary[i];
        r.b = f4(t.p1.x, t.p1.y, t.p1.z, d00);
        r.c = f4(v0.x, v0.y, v0.z, d01);
        r.d = f4(v1.x, v1.y, v1.z, d11);
        r.rd = fbits(rd);
        r.tri = (uint32_t)i;
        r.pad[0] = r.pad[1] = 0;
        RtF4 *s = &out.shade[7 * (size_t)i];
        s[0] = f4(t.p1.x, t.p1.y, t.p1.z, bitsf((uint32_t)tri_mat[i]));
        s[1] = f4(t.p2.x, t.p2.y, t.p2.z, t.uv1.x);
        s[2] = f4(t.p3.x, t.p3.y, t.p3.z, t.uv1.y);
        s[3] = f4(t.n1.x, t.n1.y, t.n1.z, t.uv2.x);
        s[4] = f4(t.n2.x, t.n2.y, t.n2.z, t.uv2.y);
        s[5] = f4(t.n3.x, t.n3.y, t.n3.z, t.uv3.x);
        // .y: the triangle's area as sample_direct_light computes it for a light (rt/path_tracing.cuh:251-261:
        // 0.5 * |cross(p2 - p1, p3 - p1)| in double, the magnitude a float sqrtf) — the same operations as
        // the device's, once per triangle instead of per shadow hit (rt_kernels.h light_contribution)
        const float area = (float)(0.5 * (double)rt_magnitude(rt_cross(t.p2 - t.p1, t.p3 - t.p1)));
        s[6] = f4(t.uv3.y, area, 0.0f, 0.0f);
    }
    // ... gathered into leaf-entry order (a leaf's tests read consecutive memory)
    const size_t ne = (size_t)(nindices > 0 ? nindices : 0);
    out.isect_a.resize(ne);
    out.isect_bary.resize(ne);
    out.isect_tri.resize(ne);
#pragma omp parallel for schedule(static)
    for (long long e = 0; e < (long long)ne; ++e) {
        const int t = indices[e];
        out.isect_a[e] = ta[t];
        out.isect_bary[e] = tbary[t];
        out.isect_tri[e] = tbary[t].tri;
    }

    // --- the conservative BVH (bvh_build.h), records in its leaf order ----
    BvhHost bvh;
    out.bvh_depth = -1;
    const int brc = build_bvh(tris, ntris, ta.data(), tbary.data(), bvh);
    if (brc == RT_OK && bvh.depth < RT_BVH_STACK) {
        out.bvh_nodes = std::move(bvh.nodes);
        collapse_bvh4(out.bvh_nodes, out.bvh4);
        // the 4-wide query pushes up to 3 entries per level: the deepest stack any root-to-leaf
        // path can build must fit the traversal stack (RT_BVH_STACK), else no bounded traversal
        {
            int worst = 0;
            std::vector<std::pair<uint32_t, int>> st{{0u, 0}};
            while (!st.empty()) {
                const auto [node, depth] = st.back();
                st.pop_back();
                const uint32_t *ref = reinterpret_cast<const uint32_t *>(&out.bvh4[8 * (size_t)node + 6]);
                int kids = 0;
                for (int k = 0; k < 4; ++k) kids += ref[k] != RT_BVH_EMPTY;
                const int below = depth + (kids > 0 ? kids - 1 : 0);
                worst = below > worst ? below : worst;
                for (int k = 0; k < 4; ++k)
                    if (ref[k] != RT_BVH_EMPTY && !(ref[k] & RT_BVH_LEAF)) st.push_back({ref[k], below});
            }
            out.bvh4_stack = worst;
        }
        out.bvh_a.resize(bvh.order.size());
        out.bvh_bary.resize(bvh.order.size());
#pragma omp parallel for schedule(static)
        for (long long k = 0; k < (long long)bvh.order.size(); ++k) {
            out.bvh_a[k] = ta[bvh.order[k]];
            out.bvh_bary[k] = tbary[bvh.order[k]];
        }
        out.bvh_scale = bvh.scale;
        // (too deep, or a scene beyond 2^64 in |vertex|_1 — the slab test's per-ray products, bvh_common.h
        // rt_slab, need it below —: the KD traversal alone)
        out.bvh_depth = out.bvh4_stack < RT_BVH_STACK && bvh.scale < 0x1p64f ? bvh.depth : -1;
        // the grid cells' start nodes: wf_long enters each deep bounce's KD traversal at the cell
        // of the ray's origin (coop_trace.h kd_origin_frontier)
        build_kd_starts(out, bounds);
        out.bvh_always = bvh.always;
        out.bvh_dropped = bvh.dropped;
    } else if (brc != RT_OK && brc != RT_E_UNSUPPORTED) {
        return brc;
    }
    // the KD split values per axis, sorted (bvh_common.h rt_bounded_ray); a
    // NaN split makes t NaN for every ray that reaches it: no bound then
    {
        std::vector<float> ax[3];
        bool nan_split = false;
        for (int k = 0; k < nnodes; ++k)
            if (!nodes[k].is_leaf_node) {
                const float v = nodes[k].plane_offset;
                if (v != v) nan_split = true;
                else ax[nodes[k].plane_axis].push_back(v);
            }
        out.split_vals.clear();
        for (int a = 0; a < 3; ++a) {
            std::sort(ax[a].begin(), ax[a].end());
            ax[a].erase(std::unique(ax[a].begin(), ax[a].end()), ax[a].end());
            out.split_off[a] = (int)out.split_vals.size();
            out.split_vals.insert(out.split_vals.end(), ax[a].begin(), ax[a].end());
        }
        out.split_off[3] = (int)out.split_vals.size();
        if (nan_split) out.bvh_depth = -1;
    }

    // --- lights: one padding entry for the xi == 1.0 draw -----
    out.lights.assign(lights, lights + nlights);
    for (int l : out.lights)
        if (l < 0 || l >= ntris) {
            rt_set_error("prepare: light index %d out of range", l);
            return RT_E_INVALID;
        }
    out.lights.push_back(nlights > 0 ? lights[nlights - 1] : 0);
    out.light_count = nlights;
    out.bounds = bounds;
    return RT_OK;
}

} // namespace rt_host
