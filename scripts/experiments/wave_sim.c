/* wave_sim.c -- CPU model of the product kernel's wave-coherent traversal (traverse_ray in
 * sphereflake-raytracer_amd/csrc/sf_kernels.hip), for counting its work per 8x8 tile (experiment, not product).
 *
 * One 8x8 tile = one wave of 64 lanes. The DFS visits a node iff some lane visits it; per lane the reference's
 * per-ray semantics (Sphereflake.h:86-226) are kept through lane masks, exactly as the kernel does:
 *   root bounding + LOD, root self test, expand (child frames, tile-cone cull, inline-leaf bits, front bits),
 *   then the children in entry order (front children first): bounding test of the visiting lanes, LOD,
 *   max-depth update, occlusion cull, self test (pre-order, ancestor tie rule), and a push for non-leaves.
 * It counts what the kernel pays for: expansions, child-loop iterations (and those no lane passes), entries,
 * inline leaves, active lanes per iteration -- per depth -- and checks minT / hit index against the oracle.
 *
 * Variants (mode bits) model candidate kernel changes so they can be priced before they are written:
 *   1: per-node cone -- the cone cull of a node's children uses the half-angle of the lanes visiting the node
 *      (around the tile axis) instead of the whole tile's.
 * Built by scripts/experiments/wave_sim.py against oracle/sf_oracle.c (included).
 */
#include <stdlib.h>
#include <stdio.h>
#include <float.h>
#include "../../oracle/sf_oracle.c"

#define NST 32
#define SF_OCCL_MARGIN_SIM 0x1.8p-9f

/* the kernel's per-depth constants (sf_capi.hip upload_consts, sf_setup.cpp depth_tables / leaf_threshold) */
static float lod_thr(float r, float C)
{
    uint32_t lo = 0, hi = 0x7f800000u;
    while (hi - lo > 1) {
        uint32_t mid = lo + (hi - lo) / 2;
        float t; memcpy(&t, &mid, 4);
        if (sqrtf(t / r) < C || t < 0.0f) lo = mid; else hi = mid;
    }
    float t; memcpy(&t, &hi, 4);
    return t;
}
void wsim_depth8(float lod_constant, float* out /* NST x 8 */)
{
    float r2b[NST + 1], r2s[NST + 1], sc[NST + 1], T[NST + 1];
    float p = 3.0f;
    for (int d = 0; d <= NST; ++d) {
        float r = p / 3.0f; p = r;
        float dr = r * 2.0f;
        r2b[d] = dr * dr; r2s[d] = r * r; sc[d] = (4.0f / 3.0f) * r; T[d] = lod_thr(r, lod_constant);
    }
    for (int d = 0; d < NST; ++d) {
        float* e = out + 8 * d;
        e[0] = r2b[d]; e[1] = r2s[d]; e[2] = sc[d]; e[3] = T[d];
        double Tn = T[d + 1], R = sqrt((double)r2b[d + 1]), s = sc[d];
        double th = (Tn * (1.0 + 0x1p-12) + 2.0 * R + s * (1.0 + 0x1p-8)) / (1.0 - 0x1p-7);
        e[4] = (float)(th * th * (1.0 + 0x1p-10));
        e[5] = nextafterf((float)(sqrt((double)e[0]) * (1.0 + 2.0 * (double)SF_OCCL_MARGIN_SIM)), FLT_MAX);
        e[6] = nextafterf((float)((double)e[3] + sqrt((double)e[0]) * (1.0 + 0x1p-18)), FLT_MAX);
        e[7] = 0.0f;
    }
}
typedef struct {
    long long exp[NST], iter[NST], miss[NST], lodnone[NST], occlnone[NST], entered[NST], leaf[NST], push[NST];
    long long act[NST], hitl[NST];   /* active lanes summed over iterations; bounding-hit lanes summed */
    long long tiles, mismatch, ties, maxd;
    long long cone_tested[NST], cone_culled[NST];
    long long skip_exp[NST], skip_lost[NST];   /* expansions the useless-cone predicate skips; culls lost by it */
    long long cache_hit[NST];                  /* expansions whose level table already holds their children */
} sim_stats_t;

typedef struct {
    const float* child;
    const uint32_t* lut;
    float r2b[NST], r2s[NST], scale[NST], T[NST], leaf[NST], cull[NST], far_[NST];
    int mode;
    float skip_k, skip_f;
    /* tile */
    float D[64][3];
    float ax[3], cosT, sinT;
    float s2[64];            /* per lane |d x a|^2 (mode 1) */
    float minT[64];
    uint64_t idx[64];
    int hdepth[64];
    int maxd;
    float cull_t;
    sim_stats_t* st;
    uint64_t owner[NST];     /* level-table cache: node whose children the wave's table(d) holds (mode 4 reuses it) */
    int split_k, split_p;    /* subtree split model: depth-k nodes n to part n % P */
    int part;                /* pixel part of the tile traced (kernel's SF_PART_*; 0 whole) */
    int cur_part;            /* part owning the current subtree (-1 above depth k) */
    double part_work[8];     /* this tile's work per part (child iterations + 6 per expansion) */
    double shared_work;      /* work above depth k (every part repeats it) */
    int solo;                /* >= 0: trace only part `solo` of the subtree split (its own wave: no other part's hits) */
    double slack;
    float cone_k;
    double pl[4][3];
    float fn[4][3], fbeta, fs, fbh, fbc;
    int npairs, pairs[4][2];   /* mode 128: the kernel's fp32 frustum (normals, beta, slack) */
    long long fr_culled;         /* mode 32: the tile pyramid's side planes (inward unit normals, through the origin) */
} wsim_t;

static int is_anc(uint64_t a, uint64_t n)
{
    while (n > a) n = (n - 1) / 9;
    return n == a;
}

static float near_root_f(float tca, float d2, float R2)
{
    float thc = sqrtf(R2 - d2);
    float t0 = tca + thc, t1 = tca - thc;
    return (t0 <= t1) ? t0 : t1;
}

/* self test of sphere (centre C, cc) at depth dd, heap index id, for the lanes of m */
static void self_test(wsim_t* S, const float C[3], float cc, int dd, uint64_t id, uint64_t m)
{
    for (int l = 0; l < 64; ++l) {
        if (!((m >> l) & 1)) continue;
        const float* D = S->D[l];
        float tca = (C[0] * D[0] + C[1] * D[1]) + C[2] * D[2];
        float d2 = cc - tca * tca;
        float R2 = S->r2s[dd];
        if (!(tca >= 0.0f && d2 <= R2)) continue;
        float ts = near_root_f(tca, d2, R2);
        if (ts < S->minT[l]) {
            S->minT[l] = ts; S->idx[l] = id; S->hdepth[l] = dd;
        } else if (ts == S->minT[l]) {
            if (S->hdepth[l] >= 0 && is_anc(S->idx[l], id)) { S->minT[l] = ts; S->idx[l] = id; S->hdepth[l] = dd; }
            else S->st->ties++;
        }
    }
}

/* the node at depth d with frame M (16 floats) is entered by the lanes of A (already self-tested) and expands */
static void expand_node(wsim_t* S, const float* M, int d, uint64_t node, uint64_t A)
{
    sim_stats_t* st = S->st;
    st->exp[d]++;
    if (S->owner[d] == node) st->cache_hit[d]++;
    S->owner[d] = node;
    const int saved_part = S->cur_part;
    if (S->split_p > 0 && d == S->split_k) S->cur_part = (int)(node % (uint64_t)S->split_p);
#define SIM_WORK(w) do { if (S->cur_part < 0) S->shared_work += (w); else S->part_work[S->cur_part] += (w); } while (0)
    SIM_WORK(6.0);
    const int dc = d + 1;
    float W[9][16];
    float cc[9];
    int front[9], culled[9], leaf[9];
    const float* P = M + 12;
    const float* ax = S->ax;
    const float kp = (P[0] * ax[0] + P[1] * ax[1]) + P[2] * ax[2];
    float sinT = S->sinT, cosT = S->cosT;
    if (S->mode & 1) {   /* per-node cone: max over the visiting lanes */
        float smax = 0.0f;
        for (int l = 0; l < 64; ++l)
            if ((A >> l) & 1) smax = S->s2[l] > smax ? S->s2[l] : smax;
        float sm = sqrtf(smax) * (1.0f + 0x1p-16f) + 0x1p-16f;
        sinT = 1.0f; cosT = 0.0f;
        if (sm < 0.5f) { sinT = sm; cosT = sqrtf(1.0f - sm * sm) * (1.0f - 0x1p-16f); }
    }
    /* predicate: the cone (plus the float tests' slack) is as wide as the node's bounding ball seen from the camera */
    const float pw = (P[0] * P[0] + P[1] * P[1]) + P[2] * P[2];
    const float sk = sinT + S->skip_k;
    const int skip = pw * sk * sk >= S->skip_f * S->r2b[d];
    if (skip) st->skip_exp[d]++;
    for (int i = 0; i < 9; ++i) {
        float T[16];
        memcpy(T, S->child + 16 * i, sizeof T);
        float s = S->scale[d];
        T[12] = T[12] * s; T[13] = T[13] * s; T[14] = T[14] * s;
        matmul(M, T, W[i]);
        const float* C = W[i] + 12;
        float w = (C[0] * C[0] + C[1] * C[1]) + C[2] * C[2];
        cc[i] = w;
        const float R2b = S->r2b[dc];
        float dl = w * 0x1p-18f;
        float ca = (C[0] * ax[0] + C[1] * ax[1]) + C[2] * ax[2];
        float q = w - ca * ca; if (q < 0.0f) q = 0.0f;
        float sq = sqrtf(q);
        float X = sq * cosT - ca * sinT;
        float Y = X * X - (R2b + w * S->cone_k);
        float a1 = ca < w - 2.0f * (R2b + dl) ? ca : w - 2.0f * (R2b + dl);
        float a2 = X < Y ? X : Y;
        float mk = a1 < a2 ? a1 : a2;
        culled[i] = mk > 0.0f;
        if (S->mode & 4096) culled[i] = 0;   /* no cone (mode 128 alone: the frustum replaces it) */
        if ((S->mode & 128) && !culled[i]) {   /* the planned kernel test, in fp32 */
            /* the kernel's arithmetic (traverse_ray expand): R2bq = depth word 7, beta_h = plane.w */
            const float R2bq = nextafterf((float)((double)R2b * (1.0 + 0x1p-16)), FLT_MAX);
            const float Pq = sqrtf(fmaf(0x1.0001p-19f, w, R2bq));
            const float bh = S->fbeta;
            float dk[4];
            for (int k = 0; k < 4; ++k)
                dk[k] = fmaf(S->fn[k][2], C[2], fmaf(S->fn[k][1], C[1], fmaf(S->fn[k][0], C[0], bh)));
            const float vA = fminf(dk[0], dk[1]) + fmaf(bh, w, Pq);
            const float vB = fminf(dk[2], dk[3]) + fmaf(bh, w, Pq);
            if (vA < 0.0f || vB < 0.0f) { culled[i] = 1; st->skip_lost[d]++; }
            else if (getenv("DBGC") && mk > 0.0f) {
                static int nprint = 0;
                if (nprint++ < 12) fprintf(stderr, "cone-only d %d w %g R2b %g dk %g %g %g %g bh %g Pq %g ca %g X %g Y %g\n", d, w, R2b,
                    dk[0], dk[1], dk[2], dk[3], bh, Pq, ca, X, Y);
            }
        }
        if ((S->mode & 8192) && !culled[i]) {   /* plane pairs with the corner bound (kernel arithmetic, fp32) */
            const float R2bq = nextafterf((float)((double)R2b * (1.0 + 0x1p-16)), FLT_MAX);
            const float P2 = fmaf(0x1.0001p-19f, w, R2bq);
            float dk[4], ak[4];
            for (int k = 0; k < 4; ++k) {
                dk[k] = fmaf(S->fn[k][2], C[2], fmaf(S->fn[k][1], C[1], fmaf(S->fn[k][0], C[0], S->fbc)));
                dk[k] = fmaf(S->fbh, w, dk[k]);
                ak[k] = -dk[k] > 0.0f ? -dk[k] : 0.0f;
            }
            int cull = 0;
            for (int pi = 0; pi < S->npairs; ++pi) {
                const int A = S->pairs[pi][0], B = S->pairs[pi][1];
                const float q = fmaf(ak[A], ak[A], ak[B] * ak[B]);
                if (q > P2) cull = 1;
            }
            if (cull) { culled[i] = 1; st->skip_lost[d]++; }
        }
        if ((S->mode & 64) && !culled[i]) {   /* the ideal cone cull: exact arithmetic, no slack */
            double cx = C[0], cy = C[1], cz = C[2];
            double cad = cx * ax[0] + cy * ax[1] + cz * ax[2];
            double px = cy * ax[2] - cz * ax[1], py = cz * ax[0] - cx * ax[2], pz = cx * ax[1] - cy * ax[0];
            double perp = sqrt(px * px + py * py + pz * pz);
            double sT = sinT, cT = sqrt(1.0 - (double)sinT * sinT);
            if (sinT < 1.0f) {
                double X = perp * cT - cad * sT;   /* distance of the centre from the cone surface */
                double R = sqrt((double)R2b + (double)w * S->slack) * (1.0 + 0x1p-12) + sqrt((double)w) * 0x1p-20;
                if (X > R && cad > 0) { culled[i] = 1; st->skip_lost[d]++; }
            }
        }
        if ((S->mode & 32) && !culled[i]) {   /* frustum: outside some side plane by more than R (1 + 2^-12) */
            const double R = sqrt((double)R2b + (double)w * S->slack) * (1.0 + 0x1p-12) + sqrt((double)w) * 0x1p-20;
            for (int k = 0; k < 4; ++k) {
                double dd = S->pl[k][0] * C[0] + S->pl[k][1] * C[1] + S->pl[k][2] * C[2];
                if (dd < -R) {
                    culled[i] = 1; st->skip_lost[d]++;
                    if (getenv("DBG")) for (int l = 0; l < 64; ++l) {
                        const float* D = S->D[l];
                        float tca = (C[0] * D[0] + C[1] * D[1]) + C[2] * D[2];
                        float d2 = w - tca * tca;
                        if (tca >= 0.0f && d2 <= R2b && ((A >> l) & 1))
                            fprintf(stderr, "lane %d plane %d dd %g R %g d %d w %g d2 %g R2b %g pn %g\n", l, k, dd, R, d, w, d2, R2b,
                                    S->pl[k][0] * D[0] + S->pl[k][1] * D[1] + S->pl[k][2] * D[2]);
                    }
                    break;
                }
            }
        }
        leaf[i] = w > S->leaf[dc];
        front[i] = ca < kp;
        st->cone_tested[d]++;
        st->cone_culled[d] += culled[i];
        if (skip && culled[i]) st->skip_lost[d]++;
        if (skip && (S->mode & 2)) culled[i] = 0;
    }
    int order[18], n = 0;
    for (int i = 0; i < 9; ++i) if (!culled[i] && front[i]) order[n++] = i;
    for (int i = 0; i < 9; ++i) if (!culled[i] && !front[i]) order[n++] = i;
    for (int k = 0; k < n; ++k) {
        const int c = order[k];
        const float* C = W[c] + 12;
        if (S->solo >= 0 && S->split_p > 0 && dc == S->split_k &&
            (int)((9 * node + 1 + (uint64_t)c) % (uint64_t)S->split_p) != S->solo) continue;
        st->iter[d]++;
        SIM_WORK(1.0);
        st->act[d] += __builtin_popcountll(A);
        uint64_t hb = 0, ex = 0;
        for (int l = 0; l < 64; ++l) {
            if (!((A >> l) & 1)) continue;
            const float* D = S->D[l];
            float tca = (C[0] * D[0] + C[1] * D[1]) + C[2] * D[2];
            float d2 = cc[c] - tca * tca;
            if (!(tca >= 0.0f && d2 <= S->r2b[dc])) continue;
            hb |= 1ull << l;
            float t = near_root_f(tca, d2, S->r2b[dc]);
            if (t < S->T[dc]) ex |= 1ull << l;
        }
        st->hitl[d] += __builtin_popcountll(hb);
        if (!hb) { st->miss[d]++; continue; }
        if (!ex) { st->lodnone[d]++; continue; }
        if (dc > S->maxd) { S->maxd = dc; S->cull_t = S->T[dc + 1]; }
        uint64_t am = ex;
        for (int l = 0; l < 64; ++l) {
            if (!((ex >> l) & 1)) continue;
            const float* D = S->D[l];
            float tca = (C[0] * D[0] + C[1] * D[1]) + C[2] * D[2];
            float v1 = tca - S->minT[l], v2 = tca - S->cull_t;
            float v = v1 < v2 ? v1 : v2;
            if (v - SF_OCCL_MARGIN_SIM * tca > S->cull[dc]) am &= ~(1ull << l);
        }
        if (!am) { st->occlnone[d]++; continue; }
        st->entered[d]++;
        const uint64_t id = 9 * node + 1 + (uint64_t)c;
        self_test(S, C, cc[c], dc, id, am);
        if (leaf[c]) { st->leaf[d]++; continue; }
        st->push[d]++;
        expand_node(S, W[c], dc, id, am);
    }
    S->cur_part = saved_part;
}

int wsim_tiles(uint32_t W, uint32_t H, const float o[3], const float tl[3], const float tr[3], const float bl[3],
               const float root[16], const float child[9 * 16], const uint32_t* lut, const float* depth8,
               uint32_t t0, uint32_t t1, int mode, const float* ref_minT, const uint32_t* ref_idx, sim_stats_t* st,
               int split_k, int split_p, double* tile_work /* per tile: total, shared, max part (NULL: none) */)
{
    wsim_t S;
    memset(&S, 0, sizeof S);
    S.child = child; S.lut = lut; S.mode = mode; S.st = st;
    S.skip_k = 0x1p-9f; S.skip_f = 4.0f;
    S.part = (mode >> 8) & 7;
    S.cone_k = getenv("CONE_K") ? strtof(getenv("CONE_K"), NULL) : (0x1p-18f + 0x1p-19f);
    S.slack = getenv("SLACK") ? strtod(getenv("SLACK"), NULL) : 0x1p-20;
    S.solo = getenv("SOLO") ? atoi(getenv("SOLO")) : -1;
    if (getenv("SKIP_K")) S.skip_k = strtof(getenv("SKIP_K"), NULL);
    if (getenv("SKIP_F")) S.skip_f = strtof(getenv("SKIP_F"), NULL);
    for (int d = 0; d < NST; ++d) {
        S.r2b[d] = depth8[8 * d + 0]; S.r2s[d] = depth8[8 * d + 1]; S.scale[d] = depth8[8 * d + 2];
        S.T[d] = depth8[8 * d + 3]; S.leaf[d] = depth8[8 * d + 4]; S.cull[d] = depth8[8 * d + 5];
        S.far_[d] = depth8[8 * d + 6];
    }
    const float fw = (float)W, fh = (float)H;
    const float dh[3] = { tr[0] - tl[0], tr[1] - tl[1], tr[2] - tl[2] };
    const float dv[3] = { bl[0] - tl[0], bl[1] - tl[1], bl[2] - tl[2] };
    const uint32_t tw = (W + 7) / 8;
    for (int k = 0; k < NST; ++k) S.owner[k] = ~0ull;
    const uint32_t run = (mode & 8) ? 4u : (mode & 16) ? 2u : 1u;   /* tiles per wave run (cache kept within a run) */
    for (uint32_t t = t0; t < t1; ++t) {
        const uint32_t tx = t % tw, ty = t / tw;
        if ((t - t0) % run == 0) for (int k = 0; k < NST; ++k) S.owner[k] = ~0ull;
        uint64_t valid = 0;
        for (int l = 0; l < 64; ++l) {
            uint32_t x = tx * 8 + (l & 7), y = ty * 8 + (l >> 3);
            float u = (float)x / fw, v = (float)y / fh;
            float* D = S.D[l];
            D[0] = ((tl[0] + dh[0] * u) + dv[0] * v) - o[0];
            D[1] = ((tl[1] + dh[1] * u) + dv[1] * v) - o[1];
            D[2] = ((tl[2] + dh[2] * u) + dv[2] * v) - o[2];
            normalize3(D, lut);
            int in = 1;   /* part units (the kernel's tile_of): 1/2 rows 0-3 / 4-7, 3..6 the 4x4 quarters */
            if (S.part >= 1 && S.part <= 2) in = (l >> 5) + 1 == S.part;
            if (S.part >= 3) { int q = S.part - 3; in = (l >> 5) == (q >> 1) && ((l >> 2) & 1) == (q & 1); }
            if (x < W && y < H && in) valid |= 1ull << l;
            S.minT[l] = FLT_MAX; S.idx[l] = 0xffffffffu; S.hdepth[l] = -1;
        }
        /* tile cone around lane 36's ray */
        memcpy(S.ax, S.D[36], sizeof S.ax);
        float smax = 0.0f;
        for (int l = 0; l < 64; ++l) {
            const float* D = S.D[l];
            const float* a = S.ax;
            float c0 = D[1] * a[2] - D[2] * a[1], c1 = D[2] * a[0] - D[0] * a[2], c2 = D[0] * a[1] - D[1] * a[0];
            float s2 = (c0 * c0 + c1 * c1) + c2 * c2;
            int fwd = (D[0] * a[0] + D[1] * a[1]) + D[2] * a[2] > 0.0f;
            float s2m = fwd ? s2 : 1.0f;
            S.s2[l] = s2m;
            if (s2m > smax) smax = s2m;
        }
        float sm = sqrtf(smax) * (1.0f + 0x1p-16f) + 0x1p-16f;
        S.sinT = 1.0f; S.cosT = 0.0f;
        if (sm < 0.5f) { S.sinT = sm; S.cosT = sqrtf(1.0f - sm * sm) * (1.0f - 0x1p-16f); }
        {   /* mode 32: pyramid of the valid lanes' extreme rays: corners of the tile's valid pixel rectangle */
            int xs = 7, ys = 7;
            while (xs > 0 && tx * 8 + xs >= W) xs--;
            while (ys > 0 && ty * 8 + ys >= H) ys--;
            const float* Cn[4] = { S.D[0], S.D[xs], S.D[ys * 8 + xs], S.D[ys * 8] };
            for (int k = 0; k < 4; ++k) {
                const float* a = Cn[k]; const float* b = Cn[(k + 1) & 3];
                double n0 = (double)a[1] * b[2] - (double)a[2] * b[1], n1 = (double)a[2] * b[0] - (double)a[0] * b[2],
                       n2 = (double)a[0] * b[1] - (double)a[1] * b[0];
                double nn = sqrt(n0 * n0 + n1 * n1 + n2 * n2);
                /* orient inward: the tile centre ray on the positive side */
                const float* c = S.D[36];
                double sg = n0 * c[0] + n1 * c[1] + n2 * c[2];
                if (sg < 0) nn = -nn;
                S.pl[k][0] = n0 / nn; S.pl[k][1] = n1 / nn; S.pl[k][2] = n2 / nn;
            }
        }
        if (mode & (128 | 8192)) {   /* the planned kernel's per-tile frustum, fp32 */
            const int cidx[4] = { 0, 7, 63, 56 };
            float mneg = 0.0f, dmax = 0.0f;
            for (int k = 0; k < 4; ++k) {
                const float* a = S.D[cidx[k]]; const float* b = S.D[cidx[(k + 1) & 3]];
                float n0 = a[1] * b[2] - a[2] * b[1], n1 = a[2] * b[0] - a[0] * b[2], n2 = a[0] * b[1] - a[1] * b[0];
                const float* c = S.D[36];
                float sg = (n0 * c[0] + n1 * c[1]) + n2 * c[2];
                float nn = (n0 * n0 + n1 * n1) + n2 * n2;
                float r = 1.0f / sqrtf(nn);
                if (sg < 0.0f) r = -r;
                S.fn[k][0] = n0 * r; S.fn[k][1] = n1 * r; S.fn[k][2] = n2 * r;
                for (int l = 0; l < 64; ++l) {
                    const float* D = S.D[l];
                    float v = (S.fn[k][0] * D[0] + S.fn[k][1] * D[1]) + S.fn[k][2] * D[2];
                    if (-v > mneg) mneg = -v;
                }
            }
            for (int l = 0; l < 64; ++l) {
                const float* D = S.D[l];
                float e = fmaf(D[2], D[2], fmaf(D[1], D[1], fmaf(D[0], D[0], -1.0f)));
                if (e > dmax) dmax = e;
            }
            S.fbeta = (mneg + 0x1p-19f) * 0x1.00002p-1f;   /* beta_h */
            {   /* pair mode: beta' = mneg + 2^-19; t <= (1 + 2^-9)(w + 1)/2 + 2 */
                const float bp = mneg + 0x1p-19f;
                S.fbh = bp * 0x1.01p-1f;
                S.fbc = S.fbh + 2.0f * bp;
                const char* pe = getenv("PAIRS") ? getenv("PAIRS") : "01,23";
                S.npairs = 0;
                for (const char* q = pe; *q && S.npairs < 4; ) {
                    S.pairs[S.npairs][0] = q[0] - '0'; S.pairs[S.npairs][1] = q[1] - '0'; S.npairs++;
                    q += 2; if (*q == ',') q++;
                }
                float kap = 0.0f;
                for (int pi = 0; pi < S.npairs; ++pi) {
                    const float* u = S.fn[S.pairs[pi][0]]; const float* v = S.fn[S.pairs[pi][1]];
                    float cdot = fabsf((u[0] * v[0] + u[1] * v[1]) + u[2] * v[2]);
                    if (cdot > kap) kap = cdot;
                }
                const float sig = (1.0f - (kap + 0x1p-20f)) * (1.0f - 0x1p-20f);
                if (getenv("DBGK") && t == t0) fprintf(stderr, "kappa %g\n", kap);
                for (int k = 0; k < 4; ++k) { S.fn[k][0] *= sig; S.fn[k][1] *= sig; S.fn[k][2] *= sig; }
                S.fbh *= sig; S.fbc *= sig;
            }
            S.fs = (0x1p-20f + 0x1p-22f + dmax) * (1.0f + 0x1p-16f);
            if (getenv("DBGF")) fprintf(stderr, "tile %u mneg %g dmax %g (u %g)\n", t, mneg, dmax, 0x1p-24);
        }
        /* root */
        S.split_k = split_k; S.split_p = split_p; S.cur_part = -1; S.shared_work = 0.0;
        for (int q = 0; q < 8; ++q) S.part_work[q] = 0.0;
        const float* C = root + 12;
        const float rcc = (C[0] * C[0] + C[1] * C[1]) + C[2] * C[2];
        uint64_t ex0 = 0;
        for (int l = 0; l < 64; ++l) {
            if (!((valid >> l) & 1)) continue;
            const float* D = S.D[l];
            float tca = (C[0] * D[0] + C[1] * D[1]) + C[2] * D[2];
            float d2 = rcc - tca * tca;
            if (tca >= 0.0f && d2 <= S.r2b[0] && near_root_f(tca, d2, S.r2b[0]) < S.T[0]) ex0 |= 1ull << l;
        }
        st->tiles++;
        if (ex0) {
            S.maxd = 0;
            S.cull_t = S.T[1];
            self_test(&S, C, rcc, 0, 0, ex0);
            if (!(rcc > S.leaf[0])) expand_node(&S, root, 0, 0, ex0);
            if (S.maxd > st->maxd) st->maxd = S.maxd;
        }
        if (tile_work) {
            double tot = S.shared_work, mx = 0.0;
            for (int q = 0; q < 8; ++q) { tot += S.part_work[q]; if (S.part_work[q] > mx) mx = S.part_work[q]; }
            tile_work[3 * (t - t0) + 0] = tot;
            tile_work[3 * (t - t0) + 1] = S.shared_work;
            tile_work[3 * (t - t0) + 2] = mx;
        }
        if (ref_minT) {
            for (int l = 0; l < 64; ++l) {
                uint32_t x = tx * 8 + (l & 7), y = ty * 8 + (l >> 3);
                if (x >= W || y >= H) continue;
                size_t p = (size_t)y * W + x;
                uint32_t a, b;
                memcpy(&a, &S.minT[l], 4); memcpy(&b, &ref_minT[p], 4);
                if (a != b || (uint32_t)S.idx[l] != ref_idx[p]) st->mismatch++;
            }
        }
    }
    return 0;
}
