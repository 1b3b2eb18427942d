/* occl_sim.c -- CPU estimate of exact occlusion culling for the per-ray traversal (experiment, not product).
 *
 * The kernel's traversal order is pre-order (a node's own sphere is tested when it is entered, ties resolved
 * by the ancestor rule), so when child c of a node is entered the lane's minT already holds its ancestors'
 * spheres and everything before c in the DFS. Every sphere of c's subtree lies in c's bounding sphere
 * (radius 2r around c). If the entry of that ball -- fattened by a margin covering every float rounding of
 * the descendants' tests -- lies strictly beyond minT, no sphere of the subtree can be accepted: the lane
 * may skip the subtree. The max-depth statistic is kept exact by culling only where no node of the subtree
 * could expand deeper than the depth already reached (T_{maxd+1} <= lb).
 *
 * This program runs the plain per-ray traversal and the culling one over a frame, checks that minT, the
 * hit index and the max depth agree on every pixel, and counts bounding tests and expansions of both.
 * Built against oracle/sf_oracle.c (included) by scripts/experiments/occl_sim.py.
 */
#include <stdlib.h>
#include "../../oracle/sf_oracle.c"

typedef struct {
    const float* child;
    const uint32_t* lut;
    int max_depth;
    long long tests, interior, culled, ties, fast_bad, band, hits;
    float margin;     /* relative margin (x |c|) */
    int mode;         /* 1: lb = tca - rho, 2: lb = tca - sqrt(rho^2 - d2); +4: children front to back */
    float axis[3];    /* mode & 8: children ordered along this direction (the tile's centre ray) for every lane */
    float seed;       /* mode & 32: cull bound min(minT, seed) */
    float sinT, cosT; /* the tile's cone (mode & 64: per-depth cone statistics of the unique expansions) */
    long long cone_n[16], cone_cull[16], cone_wide[16], cone_wide_cull[16];
    uint32_t* cnt;    /* per set slot: lanes that expanded the node; wide flag in bit 31 */
    uint64_t* set;    /* per-tile set of expanded heap indices (open addressing, 0 = empty: stores idx + 1) */
    uint32_t set_mask;
    long long uniq;
} ctrav_t;

static int set_add(ctrav_t* tv, uint64_t idx, int wide)
{
    if (!tv->set) return 0;
    uint64_t k = idx + 1, hsh = (k * 0x9E3779B97F4A7C15ull) >> 20;
    for (;;) {
        uint64_t* e = &tv->set[hsh & tv->set_mask];
        if (*e == k) { tv->cnt[hsh & tv->set_mask]++; return 0; }
        if (*e == 0) { *e = k; tv->uniq++; tv->cnt[hsh & tv->set_mask] = 1u | ((uint32_t)wide << 31); return 1; }
        ++hsh;
    }
}

static int is_ancestor(uint64_t a, uint64_t n)
{
    while (n > a) n = (n - 1) / 9;
    return n == a;
}

static float lod_T(float r) { return g_lod_constant * g_lod_constant * r; } /* t < T (approximately: sim only) */

static void intersect_cull(ctrav_t* tv, const float D[3], const float* node_m, hit_t* h, float r, int depth,
                           uint64_t node)
{
    /* node_m: this node's world transform; called for a node that passed bounding + LOD (expanded) */
    if (depth > tv->max_depth) tv->max_depth = depth;
    tv->interior++;
    int wide0 = 0;
    if (tv->set) {
        const float* C0 = node_m + 12;
        const float cc0 = (C0[0] * C0[0] + C0[1] * C0[1]) + C0[2] * C0[2];
        wide0 = cc0 * tv->sinT * tv->sinT >= (2.0f * r) * (2.0f * r);   /* |c| sinT >= R: the cone culls ~nothing */
    }
    const int fresh = set_add(tv, node, wide0);
    const float* C = node_m + 12;
    float scale = (4.0f / 3.0f) * r;
    float rc = r / 3.0f;              /* children's radius */
    float R2b = (rc * 2.0f) * (rc * 2.0f);
    float R2s = rc * rc;
    float Wall[9][16];
    int order[9];
    for (int i = 0; i < 9; ++i) {
        float T[16];
        memcpy(T, tv->child + 16 * i, sizeof T);
        T[12] *= scale; T[13] *= scale; T[14] *= scale;
        matmul(node_m, T, Wall[i]);
        order[i] = i;
    }
    if ((tv->mode & 64) && fresh && depth < 16) {
        const float* A = tv->axis;
        const float R2b = (2.0f * rc) * (2.0f * rc);
        const float cc0 = (C[0] * C[0] + C[1] * C[1]) + C[2] * C[2];
        /* bucket by log2(|c| sinT / r) + 8, clamped to 0..15 */
        int wide = (int)floorf(log2f(sqrtf(cc0) * tv->sinT / r)) + 8;
        if (wide < 0) wide = 0;
        if (wide > 15) wide = 15;
        for (int i = 0; i < 9; ++i) {
            const float* Cc = Wall[i] + 12;
            const float w = (Cc[0] * Cc[0] + Cc[1] * Cc[1]) + Cc[2] * Cc[2];
            const float ca = (Cc[0] * A[0] + Cc[1] * A[1]) + Cc[2] * A[2];
            float q2 = w - ca * ca; if (q2 < 0.0f) q2 = 0.0f;
            const float X = sqrtf(q2) * tv->cosT - ca * tv->sinT;
            const float Y = X * X - (R2b + w * (0x1p-18f + 0x1p-19f));
            const int cull = ca > 0.0f && w - 2.0f * (R2b + w * 0x1p-18f) > 0.0f && X > 0.0f && Y > 0.0f;
            tv->cone_n[depth]++; tv->cone_cull[depth] += cull;
            tv->cone_wide[wide]++; tv->cone_wide_cull[wide] += cull;
        }
    }
    if (tv->mode & 16) {   /* two buckets: children with key below the parent's centre first, index order in each */
        const float* A = tv->axis;
        const float kp = (C[0] * A[0] + C[1] * A[1]) + C[2] * A[2];
        int n = 0;
        for (int i = 0; i < 9; ++i)
            if ((Wall[i][12] * A[0] + Wall[i][13] * A[1]) + Wall[i][14] * A[2] < kp) order[n++] = i;
        for (int i = 0; i < 9; ++i)
            if (!((Wall[i][12] * A[0] + Wall[i][13] * A[1]) + Wall[i][14] * A[2] < kp)) order[n++] = i;
    } else if (tv->mode & 12) {   /* insertion sort by tca (sim only: ties not resolved in reference order) */
        float key[9];
        const float* A = (tv->mode & 8) ? tv->axis : D;
        for (int i = 0; i < 9; ++i) key[i] = (Wall[i][12] * A[0] + Wall[i][13] * A[1]) + Wall[i][14] * A[2];
        for (int i = 1; i < 9; ++i)
            for (int j = i; j > 0 && key[order[j]] < key[order[j - 1]]; --j) { int t_ = order[j]; order[j] = order[j - 1]; order[j - 1] = t_; }
    }
    for (int oi = 0; oi < 9; ++oi) {
        const int i = order[oi];
        float* Wm = Wall[i];
        const float* Cc = Wm + 12;
        tv->tests++;
        float tb;
        if (!ray_sphere(D, Cc, R2b, &tb)) continue;
        {   /* fast LOD decisions of the kernel (tca < T expands; tca (1 - 2^-8) >= Tfar does not): check */
            const float Tt = lod_T(rc);
            const float Tfar = nextafterf((float)((double)Tt + sqrt((double)R2b) * (1.0 + 0x1p-18)), FLT_MAX);
            const float tca = (Cc[0] * D[0] + Cc[1] * D[1]) + Cc[2] * D[2];
            if (tca < Tt && !(tb < Tt)) tv->fast_bad++;
            if (tca * (1.0f - 0x1p-8f) >= Tfar && tb < Tt) tv->fast_bad++;
            if (!(tca < Tt) && !(tca * (1.0f - 0x1p-8f) >= Tfar)) tv->band++;
            tv->hits++;
        }
        int expands = sqrtf(tb / rc) < g_lod_constant || tb < 0.0f;
        /* child's own sphere is tested by the reference even when it does not expand? No: the reference
           returns before the children and the self test when LOD fails (Sphereflake.h:146-153). */
        if (!expands) continue;
        if (depth + 1 > tv->max_depth) tv->max_depth = depth + 1;
        /* cull check at entry */
        if (tv->margin >= 0.0f) {
            float tca = (Cc[0] * D[0] + Cc[1] * D[1]) + Cc[2] * D[2];
            float cc = (Cc[0] * Cc[0] + Cc[1] * Cc[1]) + Cc[2] * Cc[2];
            float R = 2.0f * rc;
            float M = tv->margin * (sqrtf(cc) + R);
            float rho = R + M, lb;
            if ((tv->mode & 3) == 1) lb = tca - rho;
            else {
                float d2 = cc - tca * tca;
                float a = rho * rho - d2;
                lb = tca - sqrtf(a > 0.0f ? a : 0.0f) - M;
            }
            float Tn = lod_T(1.0f / powf(3.0f, (float)(tv->max_depth + 1)));
            float mb = h->minT; if ((tv->mode & 32) && tv->seed < mb) mb = tv->seed;
            if (lb > mb && lb >= Tn && lb >= 0.0f) {
                tv->culled++;
                continue;
            }
        }
        /* own sphere, pre-order with the ancestor tie rule */
        float ts;
        uint64_t idx = 9 * node + 1 + (uint64_t)i;
        if (ray_sphere(D, Cc, R2s, &ts)) {
            if (ts == h->minT && h->depth >= 0 && !is_ancestor(h->index, idx)) tv->ties++;
            if (ts < h->minT || (ts == h->minT && h->depth >= 0 && is_ancestor(h->index, idx))) {
                h->minT = ts;
                h->index = idx;
                h->depth = depth + 1;
            }
        }
        intersect_cull(tv, D, Wm, h, rc, depth + 1, idx);
    }
}

/* plain / culling traversal over rows [y0, y1): minT, index out; stats[0] max depth, [1] tests, [2] interior,
   [3] culled */
int sim_rows(uint32_t W, uint32_t H, const float o[3], const float tl[3], const float tr[3], const float bl[3],
             const float root[16], const float child[9 * 16], const uint32_t* lut, uint32_t y0, uint32_t y1,
             float margin, int mode, float* minT, uint32_t* index, long long* stats)
{
    ctrav_t tv = { child, lut, 0, 0, 0, 0, 0, 0, 0, 0, margin, mode, {0, 0, 0}, 0.0f, 0.0f, 0.0f, {0}, {0}, {0}, {0}, NULL, NULL, 0, 0 };
    float fw = (float)W, fh = (float)H;
    float dx_ = tr[0] - tl[0], dy_ = tr[1] - tl[1], dz_ = tr[2] - tl[2];
    float ex_ = bl[0] - tl[0], ey_ = bl[1] - tl[1], ez_ = bl[2] - tl[2];
    for (uint32_t y = y0; y < y1; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            float u = (float)x / fw, v = (float)y / fh, D[3];
            D[0] = ((tl[0] + dx_ * u) + ex_ * v) - o[0];
            D[1] = ((tl[1] + dy_ * u) + ey_ * v) - o[1];
            D[2] = ((tl[2] + dz_ * u) + ez_ * v) - o[2];
            normalize3(D, lut);
            hit_t h;
            h.minT = FLT_MAX;
            h.index = 0xffffffffu;
            h.depth = -1;
            /* root: bounding + LOD, then its own sphere, then children */
            const float* C = root + 12;
            float tb;
            tv.tests++;
            if (ray_sphere(D, C, 4.0f, &tb) && (sqrtf(tb / 1.0f) < g_lod_constant || tb < 0.0f)) {
                float ts;
                if (ray_sphere(D, C, 1.0f, &ts) && ts < h.minT) { h.minT = ts; h.index = 0; h.depth = 0; }
                intersect_cull(&tv, D, root, &h, 1.0f, 0, 0);
            }
            size_t p = (size_t)(y - y0) * W + x;
            minT[p] = h.minT;
            index[p] = (uint32_t)h.index;
        }
    stats[0] = tv.max_depth; stats[1] = tv.fast_bad; stats[2] = tv.band; stats[3] = tv.hits;
    return 0;
}

/* tile-level: 8x8 tiles of rows [ty*8, ty*8+8), unique expanded nodes per tile summed (a wave visits a node iff
   some lane does) */
int sim_tile_row(uint32_t W, uint32_t H, const float o[3], const float tl[3], const float tr[3], const float bl[3],
                 const float root[16], const float child[9 * 16], const uint32_t* lut, uint32_t ty,
                 float margin, int mode, long long* stats)
{
    const uint32_t cap = 1u << 18;
    uint64_t* set = (uint64_t*)calloc(cap, 8);
    uint32_t* cnt = (uint32_t*)calloc(cap, 4);
    float fw = (float)W, fh = (float)H;
    float dx_ = tr[0] - tl[0], dy_ = tr[1] - tl[1], dz_ = tr[2] - tl[2];
    float ex_ = bl[0] - tl[0], ey_ = bl[1] - tl[1], ez_ = bl[2] - tl[2];
    long long uniq = 0, tests = 0, interior = 0, ties_all = 0;
    for (uint32_t tx = 0; tx < (W + 7) / 8; ++tx) {
        memset(set, 0, (size_t)cap * 8);
        memset(cnt, 0, (size_t)cap * 4);
        ctrav_t tv = { child, lut, 0, 0, 0, 0, 0, 0, 0, 0, margin, mode, {0, 0, 0}, 0.0f, 0.0f, 0.0f, {0}, {0}, {0}, {0}, cnt, set, cap - 1, 0 };
        {
            float u = (float)(tx * 8 + 4) / fw, v = (float)(ty * 8 + 4) / fh;
            tv.axis[0] = ((tl[0] + dx_ * u) + ex_ * v) - o[0];
            tv.axis[1] = ((tl[1] + dy_ * u) + ey_ * v) - o[1];
            tv.axis[2] = ((tl[2] + dz_ * u) + ez_ * v) - o[2];
            normalize3(tv.axis, lut);
            float smax = 0.0f;
            for (uint32_t y = ty * 8; y < ty * 8 + 8 && y < H; ++y)
                for (uint32_t x = tx * 8; x < tx * 8 + 8 && x < W; ++x) {
                    float u = (float)x / fw, v = (float)y / fh, D[3];
                    D[0] = ((tl[0] + dx_ * u) + ex_ * v) - o[0];
                    D[1] = ((tl[1] + dy_ * u) + ey_ * v) - o[1];
                    D[2] = ((tl[2] + dz_ * u) + ez_ * v) - o[2];
                    normalize3(D, lut);
                    const float* a = tv.axis;
                    float c0 = D[1] * a[2] - D[2] * a[1], c1 = D[2] * a[0] - D[0] * a[2], c2 = D[0] * a[1] - D[1] * a[0];
                    float s2 = (c0 * c0 + c1 * c1) + c2 * c2;
                    if (s2 > smax) smax = s2;
                }
            float sm = sqrtf(smax) * (1.0f + 0x1p-16f) + 0x1p-16f;
            tv.sinT = 1.0f; tv.cosT = 0.0f;
            if (sm < 0.5f) { tv.sinT = sm; tv.cosT = sqrtf(1.0f - sm * sm) * (1.0f - 0x1p-16f); }
        }
        for (uint32_t y = ty * 8; y < ty * 8 + 8 && y < H; ++y)
            for (uint32_t x = tx * 8; x < tx * 8 + 8 && x < W; ++x) {
                float u = (float)x / fw, v = (float)y / fh, D[3];
                D[0] = ((tl[0] + dx_ * u) + ex_ * v) - o[0];
                D[1] = ((tl[1] + dy_ * u) + ey_ * v) - o[1];
                D[2] = ((tl[2] + dz_ * u) + ez_ * v) - o[2];
                normalize3(D, lut);
                hit_t h;
                h.minT = FLT_MAX; h.index = 0xffffffffu; h.depth = -1;
                const float* C = root + 12;
                float tb;
                if (mode & 32) {
                    ctrav_t t2 = { child, lut, 0, 0, 0, 0, 0, 0, 0, 0, -1.0f, 0, {0, 0, 0}, 0.0f, 0.0f, 0.0f, {0}, {0}, {0}, {0}, NULL, NULL, 0, 0 };
                    hit_t h2; h2.minT = FLT_MAX; h2.index = 0xffffffffu; h2.depth = -1;
                    if (ray_sphere(D, C, 4.0f, &tb) && (sqrtf(tb) < g_lod_constant || tb < 0.0f)) {
                        float ts;
                        if (ray_sphere(D, C, 1.0f, &ts) && ts < h2.minT) { h2.minT = ts; h2.index = 0; h2.depth = 0; }
                        intersect_cull(&t2, D, root, &h2, 1.0f, 0, 0);
                    }
                    tv.seed = h2.minT;
                }
                if (ray_sphere(D, C, 4.0f, &tb) && (sqrtf(tb) < g_lod_constant || tb < 0.0f)) {
                    float ts;
                    if (ray_sphere(D, C, 1.0f, &ts) && ts < h.minT) { h.minT = ts; h.index = 0; h.depth = 0; }
                    intersect_cull(&tv, D, root, &h, 1.0f, 0, 0);
                }
            }
        uniq += tv.uniq; tests += tv.tests; interior += tv.interior; ties_all += tv.ties;
        for (uint32_t q = 0; q < cap; ++q) {
            if (!set[q]) continue;
            const uint32_t na = cnt[q] & 0x7fffffffu, w = cnt[q] >> 31;
            int b = na <= 2 ? 0 : na <= 4 ? 1 : na <= 8 ? 2 : na <= 16 ? 3 : na <= 32 ? 4 : 5;
            stats[67 + 2 * b + w] += 1;
        }
        for (int k = 0; k < 16; ++k) { stats[3 + k] += tv.cone_n[k]; stats[19 + k] += tv.cone_cull[k];
                                       stats[35 + k] += tv.cone_wide[k]; stats[51 + k] += tv.cone_wide_cull[k]; }
    }
    free(set);
    free(cnt);
    stats[0] += uniq; stats[1] += interior; stats[2] += ties_all;
    return 0;
}
