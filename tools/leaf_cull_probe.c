/* leaf_cull_probe.c — how much leaf-test work a per-leaf bounding box of the
 * leaf's triangles could skip (analysis tool, CPU).
 *
 * Reads the reference-layout KD tree (20-B nodes), triangle_indicies,
 * triangles (152 B) and a ray list (o, d as 6 floats) dumped by
 * tools/leaf_cull_probe.py, traverses every ray exactly like trace_ray
 * (rt/trace_ray.cuh:244-318) and, at every non-empty leaf it tests, checks
 * whether the ray segment [0, leaf exit] meets the union AABB of the leaf's
 * triangles (grown by a relative margin).  Prints the share of leaf tests and
 * of triangle tests in leaves whose box the segment misses, and the share of
 * triangle tests that repeat a triangle the same ray already tested in an
 * earlier leaf (the KD builder duplicates straddling triangles into both
 * children: a per-ray mailbox could skip those whose first test failed for a
 * leaf-independent reason).
 * Build: gcc -O2 -fopenmp tools/leaf_cull_probe.c -o /tmp/leaf_cull_probe -lm */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int a, b; uint8_t axis; float off; uint8_t leaf; } Node;

static void *slurp(const char *path, size_t *n)
{
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    *n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    void *p = malloc(*n);
    if (fread(p, 1, *n, f) != *n) exit(1);
    fclose(f);
    return p;
}

int main(int argc, char **argv)
{
    if (argc < 6) { fprintf(stderr, "usage: %s nodes idx tris rays margin\n", argv[0]); return 1; }
    size_t nb, ib, tb, rb;
    uint8_t *nraw = slurp(argv[1], &nb);
    int *idx = slurp(argv[2], &ib);
    uint8_t *traw = slurp(argv[3], &tb);
    float *rays = slurp(argv[4], &rb);
    const float margin = (float)atof(argv[5]);
    const int nn = (int)(nb / 20), nr = (int)(rb / 24), nt = (int)(tb / 152);
    Node *nodes = malloc(sizeof(Node) * nn);
    for (int i = 0; i < nn; ++i) {
        memcpy(&nodes[i].a, nraw + 20 * i, 4);
        memcpy(&nodes[i].b, nraw + 20 * i + 4, 4);
        nodes[i].axis = nraw[20 * i + 8];
        memcpy(&nodes[i].off, nraw + 20 * i + 12, 4);
        nodes[i].leaf = nraw[20 * i + 16];
    }
    float (*tbox)[6] = malloc(sizeof(float[6]) * nt);
    for (int t = 0; t < nt; ++t) {
        float p[9];
        memcpy(p, traw + 152 * (size_t)t, 36);
        for (int k = 0; k < 3; ++k) {
            tbox[t][k] = fminf(p[k], fminf(p[3 + k], p[6 + k]));
            tbox[t][3 + k] = fmaxf(p[k], fmaxf(p[3 + k], p[6 + k]));
        }
    }
    /* leaf boxes (union of the leaf's triangle boxes, grown by margin * extent + 1e-4) */
    float (*lbox)[6] = calloc(nn, sizeof(float[6]));
    for (int i = 0; i < nn; ++i) {
        if (!nodes[i].leaf || nodes[i].b == 0) continue;
        float b[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int k = 0; k < nodes[i].b; ++k) {
            const int t = idx[nodes[i].a + k];
            for (int c = 0; c < 3; ++c) {
                b[c] = fminf(b[c], tbox[t][c]);
                b[3 + c] = fmaxf(b[3 + c], tbox[t][3 + c]);
            }
        }
        float m = 1.0f;
        for (int c = 0; c < 6; ++c) m = fmaxf(m, fabsf(b[c]));
        for (int c = 0; c < 3; ++c) {
            /* margin < 0: the product's growth (scene_prepare.cpp), 1e-4 of the largest coordinate magnitude */
            const float g = margin < 0 ? 1e-4f * m : margin * (b[3 + c] - b[c]) + 1e-4f;
            lbox[i][c] = b[c] - g;
            lbox[i][3 + c] = b[3 + c] + g;
        }
    }
    unsigned long long leaves = 0, culled = 0, tris = 0, tris_culled = 0, win_culled = 0, repeats = 0, cands = 0,
                       cand_repeats = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : leaves, culled, tris, tris_culled, win_culled, repeats, cands, cand_repeats)
    for (int r = 0; r < nr; ++r) {
        int seen_ids[4096], bary_failed[4096];
        int nseen = 0, nbf = 0;
        const float *o = rays + 6 * r, *d = rays + 6 * r + 3;
        /* scene box: the root box is not needed for the statistics, start at [0, inf) */
        int ni[64];
        float en[64], ex[64];
        int sp = 0;
        ni[sp] = 0;
        en[sp] = 0.0f;
        ex[sp] = FLT_MAX;
        ++sp;
        while (sp > 0) {
            --sp;
            int node = ni[sp];
            float entry = en[sp], exit_ = ex[sp];
            while (!nodes[node].leaf) {
                const Node *n = &nodes[node];
                int nearc = n->a, farc = n->b;
                if (o[n->axis] >= n->off) { nearc = n->b; farc = n->a; }
                const float t = (n->off - o[n->axis]) / d[n->axis];
                if (t >= exit_ || t < 0) node = nearc;
                else if (t <= entry) node = farc;
                else { ni[sp] = farc; en[sp] = t; ex[sp] = exit_; ++sp; node = nearc; exit_ = t; }
            }
            const Node *L = &nodes[node];
            if (L->b == 0) continue;
            /* segment [0, exit] vs the leaf box (slab test in double) */
            double t0 = getenv("PROBE_ENTRY") ? (double)entry - fabs((double)entry) * 1e-4 : 0.0;
            double t1 = exit_ == FLT_MAX ? 1e30 : (double)exit_ * 1.0001;
            for (int c = 0; c < 3 && t0 <= t1; ++c) {
                const double inv = 1.0 / (double)d[c];
                double a = ((double)lbox[node][c] - o[c]) * inv, b = ((double)lbox[node][3 + c] - o[c]) * inv;
                if (a > b) { double x = a; a = b; b = x; }
                if (d[c] == 0.0f) { a = (o[c] >= lbox[node][c] && o[c] <= lbox[node][3 + c]) ? -1e30 : 1e30; b = -a; }
                if (a > t0) t0 = a;
                if (b < t1) t1 = b;
            }
            int miss = t0 > t1;
            if (margin < 0) { /* the product's test (coop_trace.h leaf_box_maybe), in float */
                const float y[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
                int guarded = 0;
                for (int c = 0; c < 3; ++c) guarded |= !(fabsf(d[c]) >= 0x1p-60f && fabsf(d[c]) <= 0x1p40f);
                float lo = 0.0f, hi = exit_;
                for (int c = 0; c < 3; ++c) {
                    const float a = (lbox[node][c] - o[c]) * y[c], b = (lbox[node][3 + c] - o[c]) * y[c];
                    lo = fmaxf(lo, fminf(a, b));
                    hi = fminf(hi, fmaxf(a, b));
                }
                miss = !guarded && lo > hi + 0x1p-16f * (fabsf(lo) + fabsf(hi));
            }
            /* mailbox probe: triangles of this leaf already tested earlier along this ray */
            for (int k = 0; k < L->b; ++k) {
                const int tt = idx[L->a + k];
                int seen = 0;
                for (int m = 0; m < nseen && !seen; ++m) seen = seen_ids[m] == tt;
                if (seen) ++repeats;
                else if (nseen < 4096) seen_ids[nseen++] = tt;
            }
            ++leaves;
            tris += (unsigned long long)L->b;
            /* the reference's leaf test: hit = any triangle with 1e-5 <= s < exit inside */
            int hit = 0;
            for (int k = 0; k < L->b; ++k) {
                const uint8_t *T = traw + 152 * (size_t)idx[L->a + k];
                float p[9];
                memcpy(p, T, 36);
                float e1[3] = {p[3] - p[0], p[4] - p[1], p[5] - p[2]}, e2[3] = {p[6] - p[0], p[7] - p[1], p[8] - p[2]};
                float nx = e1[1] * e2[2] - e1[2] * e2[1], ny = e1[2] * e2[0] - e1[0] * e2[2], nz = e1[0] * e2[1] - e1[1] * e2[0];
                float rl = 1.0f / sqrtf(nx * nx + ny * ny + nz * nz);
                nx *= rl; ny *= rl; nz *= rl;
                float dn = d[0] * nx + d[1] * ny + d[2] * nz;
                if (dn == 0) continue;
                float s = ((nx * p[0] + ny * p[1] + nz * p[2]) - (o[0] * nx + o[1] * ny + o[2] * nz)) / dn;
                if (s < 0.00001f || !(s < exit_)) continue;
                float q[3] = {o[0] + s * d[0] - p[0], o[1] + s * d[1] - p[1], o[2] + s * d[2] - p[2]};
                float d00 = e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2], d01 = e1[0] * e2[0] + e1[1] * e2[1] + e1[2] * e2[2];
                float d11 = e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2];
                float d20 = q[0] * e1[0] + q[1] * e1[1] + q[2] * e1[2], d21 = q[0] * e2[0] + q[1] * e2[1] + q[2] * e2[2];
                float rd = 1.0f / (d00 * d11 - d01 * d01);
                float v = (d11 * d20 - d01 * d21) * rd, w = (d00 * d21 - d01 * d20) * rd, u = 1.0f - v - w;
                ++cands;
                const int tt = idx[L->a + k];
                int seen = 0;
                for (int m = 0; m < nbf && !seen; ++m) seen = bary_failed[m] == tt;
                if (seen) ++cand_repeats;
                if (u >= 0 && u <= 1 && v >= 0 && v <= 1 && w >= 0 && w <= 1) hit = 1;
                else if (!seen && nbf < 4096) bary_failed[nbf++] = tt;
            }
            if (miss) {
                ++culled;
                tris_culled += (unsigned long long)L->b;
                if (hit) ++win_culled;
            }
            if (hit) break;
        }
    }
    printf("{\"rays\": %d, \"leaf_tests\": %llu, \"leaf_tests_box_missed\": %llu, \"tri_tests\": %llu, "
           "\"tri_tests_box_missed\": %llu, \"frac_leaves\": %.4f, \"frac_tris\": %.4f, \"hits_in_missed_boxes\": %llu, "
           "\"repeat_tests\": %llu, \"frac_repeat\": %.4f, \"bary_tests\": %llu, "
           "\"bary_repeats_of_failed\": %llu, \"frac_bary_repeat\": %.4f}\n",
           nr, leaves, culled, tris, tris_culled, (double)culled / leaves, (double)tris_culled / tris, win_culled,
           repeats, (double)repeats / tris, cands, cand_repeats, (double)cand_repeats / cands);
    return 0;
}
