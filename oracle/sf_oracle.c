/*
 * sf_oracle.c -- TEST INFRASTRUCTURE ONLY. CPU restatement of the reference
 * Sphereflake hot path, used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the CHECKER. Nothing in the product links or calls it.
 *
 * Parity status: PINNED. tests/test_oracle.py checks this restatement bit-for-bit
 * against golden frames produced by the reference itself (oracle/ref_harness.cpp,
 * compiled from /root/reference with -O2 -mavx) for every BASELINE config.
 *
 * Semantics are per ray: one ray broadcast to every AVX lane, so the packet-wide
 * early-outs act per ray. Arithmetic is IEEE binary32 with the
 * reference's exact operation order; build with -ffp-contract=off. The x86
 * `rsqrtps` approximation is emulated from a table measured on the instruction
 * (oracle/gen_rsqrtps_lut.c, tests/golden/rsqrtps_lut.bin).
 *
 * Reference citations (paths relative to /root/reference):
 *   ray generation            sphereflake/Sphereflake.cpp:149-150,162-167
 *   Normalize / Dot           sphereflake/SIMD_AVX.h:163-180
 *   4x4 product               sphereflake/SIMD_AVX.h:59-81
 *   RaySphereIntersection     sphereflake/SIMD_AVX.h:236-270
 *   IntersectSphereflake      sphereflake/Sphereflake.h:86-226
 *   G-buffer scatter          sphereflake/Sphereflake.cpp:186-201
 *   Sobol::Sample             sphereflake/Sobol.cpp:41-55
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <float.h>

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* x86 rsqrtps, emulated from the measured table (layout: gen_rsqrtps_lut.c). */
float sfo_rsqrtps(float x, const uint32_t* lut)
{
    uint32_t b = f2u(x);
    uint32_t E = (b >> 23) & 0xffu;
    if ((b & 0x7fffffffu) > 0x7f800000u) return u2f(b | 0x00400000u);      /* NaN -> quiet NaN */
    if (E == 0) return u2f((b & 0x80000000u) | 0x7f800000u);               /* +-0, denormal -> +-inf */
    if (b & 0x80000000u) return u2f(0xffc00000u);                           /* negative -> default NaN */
    if (E == 0xffu) return 0.0f;                                            /* +inf -> +0 */
    uint32_t key = ((E & 1u) << 10) | ((b & 0x7fffffu) >> 13);
    int32_t E0 = (E & 1u) ? 127 : 128;
    int32_t k = ((int32_t)E - E0) / 2;
    return u2f((uint32_t)((int32_t)lut[key] - k * (1 << 23)));
}

/* SIMD::Normalize, SIMD_AVX.h:170-180 */
static void normalize3(float v[3], const uint32_t* lut)
{
    float len = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
    float nr = sfo_rsqrtps(len, lut);
    float muls = (len * nr) * nr;
    float s = (0.5f * nr) * (3.0f - muls);
    v[0] = v[0] * s;
    v[1] = v[1] * s;
    v[2] = v[2] * s;
}

void sfo_normalize(float v[3], const uint32_t* lut) { normalize3(v, lut); }

/* SIMD::operator*(Matrix4, Matrix4), SIMD_AVX.h:59-81. Storage = glm column-major,
 * m[4*c + r]. Result column c = ((a0*b[c][0] + a1*b[c][1]) + a2*b[c][2]) + a3*b[c][3]. */
static void matmul(const float* a, const float* b, float* out)
{
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) {
            float acc = a[r] * b[4 * c + 0];
            acc = a[4 + r] * b[4 * c + 1] + acc;
            acc = a[8 + r] * b[4 * c + 2] + acc;
            acc = a[12 + r] * b[4 * c + 3] + acc;
            out[4 * c + r] = acc;
        }
}

/* SIMD::RaySphereIntersection, SIMD_AVX.h:236-270, one lane. Ray origin is 0. */
static int ray_sphere(const float D[3], const float C[3], float R2, float* t)
{
    float tca = (C[0] * D[0] + C[1] * D[1]) + C[2] * D[2];
    if (!(tca >= 0.0f)) return 0;
    float d2 = ((C[0] * C[0] + C[1] * C[1]) + C[2] * C[2]) - tca * tca;
    if (!(d2 <= R2)) return 0;
    float thc = sqrtf(R2 - d2);
    float t0 = tca + thc;
    float t1 = tca - thc;
    *t = (t0 <= t1) ? t0 : t1;
    return 1;
}

typedef struct {
    const float* child;     /* 9 x 16 */
    const uint32_t* lut;
    int max_depth;
    long long nodes, interior;
} trav_t;

typedef struct {
    float minT;
    float pos[3], nrm[3];
    uint64_t index;
    int depth;
} hit_t;

/* LOD constant of the predicate sqrtf(t / r) < C: 70 in the AVX path (SIMD_AVX.h:25, Sphereflake.h:146),
   60 in the SSE path (SIMD_SSE.h:21, Sphereflake.h:129). Set before rendering (sfo_set_lod_constant). */
static float g_lod_constant = 70.0f;
void sfo_set_lod_constant(float c) { g_lod_constant = c; }

/* Sphereflake::IntersectSphereflake, Sphereflake.h:86-226 (per ray). */
static void intersect(trav_t* tv, const float D[3], const float* parent, hit_t* h,
                      float parentRadius, int depth, uint64_t node)
{
    float r = parentRadius / 3.0f;
    float dr = r * 2.0f;
    float R2b = dr * dr;
    const float* C = parent + 12;
    float t;
    tv->nodes++;
    if (!ray_sphere(D, C, R2b, &t)) return;                       /* :119, :140-144 */
    if (!(sqrtf(t / r) < g_lod_constant || t < 0.0f)) return;    /* :146-153 (SSE :129-136) */
    if (depth > tv->max_depth) tv->max_depth = depth;             /* :157-160 */
    tv->interior++;
    float scale = (4.0f / 3.0f) * r;                              /* :162 */
    for (int i = 0; i < 9; ++i) {                                 /* :165-172 */
        float T[16], Wm[16];
        memcpy(T, tv->child + 16 * i, sizeof T);
        T[12] = T[12] * scale;
        T[13] = T[13] * scale;
        T[14] = T[14] * scale;
        T[15] = T[15] * 1.0f;
        matmul(parent, T, Wm);
        intersect(tv, D, Wm, h, r, depth + 1, 9 * node + 1 + (uint64_t)i);
    }
    float R2s = r * r;                                            /* :180 */
    float ts;
    if (!ray_sphere(D, C, R2s, &ts)) return;                      /* :185 */
    if (!(ts < h->minT)) return;                                  /* :204-211 */
    h->minT = ts;                                                 /* :213 */
    float p[3] = { D[0] * ts, D[1] * ts, D[2] * ts };             /* :218 */
    float n[3] = { p[0] - C[0], p[1] - C[1], p[2] - C[2] };       /* :219-220 */
    normalize3(n, tv->lut);
    memcpy(h->pos, p, sizeof p);
    memcpy(h->nrm, n, sizeof n);
    h->index = node;
    h->depth = depth;
}

/*
 * Render rows [y0, y1) of a W x H frame, per ray. Outputs are row-major for the
 * rendered rows only: pos4/nrm4 as float4 (xyz, 1) exactly like the reference
 * G-buffer scatter (Sphereflake.cpp:186-196, a miss writes (0,0,0,1)); minT
 * (FLT_MAX on a miss); index = heap index 9n+1+i of the hit sphere (low 32 bits,
 * 0xffffffff on a miss); hit_depth (-1 on a miss).
 * stats_out[0] = max depth reached, [1] = hits, [2] = nodes visited, [3] = interior expansions.
 * closest_out = min minT over the rows.
 */
int sfo_render_rows(uint32_t W, uint32_t H,
                    const float o[3], const float tl[3], const float tr[3], const float bl[3],
                    const float root[16], const float child[9 * 16], const uint32_t* lut,
                    uint32_t y0, uint32_t y1,
                    float* pos4, float* nrm4, float* minT, uint32_t* index, int8_t* hit_depth,
                    long long* stats_out, float* closest_out)
{
    trav_t tv = { child, lut, 0, 0, 0 };
    long long hits = 0;
    float closest = FLT_MAX;
    float fw = (float)W, fh = (float)H;
    float dx_ = tr[0] - tl[0], dy_ = tr[1] - tl[1], dz_ = tr[2] - tl[2];
    float ex_ = bl[0] - tl[0], ey_ = bl[1] - tl[1], ez_ = bl[2] - tl[2];
    if (y1 > H || y0 > y1) return -1;
    for (uint32_t y = y0; y < y1; ++y) {
        for (uint32_t x = 0; x < W; ++x) {
            float u = (float)x / fw;                               /* :149-150 (pixel corner) */
            float v = (float)y / fh;
            float D[3];
            D[0] = ((tl[0] + dx_ * u) + ex_ * v) - o[0];           /* :162-166 */
            D[1] = ((tl[1] + dy_ * u) + ey_ * v) - o[1];
            D[2] = ((tl[2] + dz_ * u) + ez_ * v) - o[2];
            normalize3(D, lut);                                    /* :167 */
            hit_t h;
            h.minT = FLT_MAX;
            h.pos[0] = h.pos[1] = h.pos[2] = 0.0f;
            h.nrm[0] = h.nrm[1] = h.nrm[2] = 0.0f;
            h.index = 0xffffffffu;
            h.depth = -1;
            intersect(&tv, D, root, &h, 3.0f, 0, 0);               /* :172-173 */
            size_t p = (size_t)(y - y0) * W + x;
            if (pos4) { pos4[4 * p] = h.pos[0]; pos4[4 * p + 1] = h.pos[1]; pos4[4 * p + 2] = h.pos[2]; pos4[4 * p + 3] = 1.0f; }
            if (nrm4) { nrm4[4 * p] = h.nrm[0]; nrm4[4 * p + 1] = h.nrm[1]; nrm4[4 * p + 2] = h.nrm[2]; nrm4[4 * p + 3] = 1.0f; }
            if (minT) minT[p] = h.minT;
            if (index) index[p] = (uint32_t)h.index;
            if (hit_depth) hit_depth[p] = (int8_t)h.depth;
            if (h.depth >= 0) hits++;
            if (h.minT < closest) closest = h.minT;                /* :197-200 */
        }
    }
    if (stats_out) { stats_out[0] = tv.max_depth; stats_out[1] = hits; stats_out[2] = tv.nodes; stats_out[3] = tv.interior; }
    if (closest_out) *closest_out = closest;
    return 0;
}

/* Sobol::Sample, Sobol.cpp:41-55, for a caller-supplied direction-number table
 * (dims x 52 entries). */
float sfo_sobol_sample(unsigned long long index, unsigned dimension, unsigned scramble, const uint32_t* matrices)
{
    unsigned result = scramble;
    for (unsigned i = dimension * 52u; index; index >>= 1, ++i)
        if (index & 1) result ^= matrices[i];
    return (float)result * (1.f / (float)(1ULL << 32));
}
