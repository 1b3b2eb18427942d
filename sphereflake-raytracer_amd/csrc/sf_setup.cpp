// sf_setup.cpp -- host-side setup math of the renderer (per view / per process, not per ray).
//
// Restates, in plain C++ with IEEE binary32 and the reference's operation order, the glm
// 0.9.5.4 arithmetic the reference runs on the host:
//   - ComputeChildTransformations      Sphereflake.cpp:216-249, Util.h:7-18
//   - SetView root transform           Sphereflake.cpp:83
//   - Camera corners                   camera.h:37-53, 65-68, 111-114
// plus the per-depth constants of IntersectSphereflake (Sphereflake.h:97-111, 146, 162, 180)
// and the x86 rsqrtps table lookup (SIMD_AVX.h:173).
//
// Compiled with g++ -O2 -ffp-contract=off (no FMA on the host) so the results equal the
// reference's host arithmetic bit for bit; tests/test_host.py pins every value against the
// hex dumps of the reference (tests/golden/setup_*.json).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>

#include "sf_internal.h"

namespace sfhost {

namespace {

struct v3 { float x, y, z; };
struct v4 { float x, y, z, w; };
struct m4 { v4 c[4]; };   // glm column-major: c[col]

inline v4 mul(const v4& a, float s) { return { a.x * s, a.y * s, a.z * s, a.w * s }; }
inline v4 add(const v4& a, const v4& b) { return { a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w }; }

m4 identity()
{
    m4 m;
    m.c[0] = { 1, 0, 0, 0 };
    m.c[1] = { 0, 1, 0, 0 };
    m.c[2] = { 0, 0, 1, 0 };
    m.c[3] = { 0, 0, 0, 1 };
    return m;
}

// glm::radians (func_trigonometric.inl): degrees * genType(0.0174532925...)
inline float radians(float deg) { return deg * float(0.01745329251994329576923690768489); }

// glm::normalize(vec3) (func_geometric.inl): x * inversesqrt(dot), inversesqrt = 1 / sqrt
v3 normalize(const v3& v)
{
    float sqr = v.x * v.x + v.y * v.y + v.z * v.z;
    float inv = 1.0f / std::sqrt(sqr);
    return { v.x * inv, v.y * inv, v.z * inv };
}

// glm::rotate(m, angle, axis) (gtc/matrix_transform.inl), m = identity in every use here.
m4 rotate(const m4& m, float a, const v3& v)
{
    float c = std::cos(a);
    float s = std::sin(a);
    v3 axis = normalize(v);
    v3 temp = { (1.0f - c) * axis.x, (1.0f - c) * axis.y, (1.0f - c) * axis.z };
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = 0.0f + temp.x * axis.y + s * axis.z;
    R[0][2] = 0.0f + temp.x * axis.z - s * axis.y;
    R[1][0] = 0.0f + temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = 0.0f + temp.y * axis.z + s * axis.x;
    R[2][0] = 0.0f + temp.z * axis.x + s * axis.y;
    R[2][1] = 0.0f + temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    m4 out;
    for (int j = 0; j < 3; ++j)
        out.c[j] = add(add(mul(m.c[0], R[j][0]), mul(m.c[1], R[j][1])), mul(m.c[2], R[j][2]));
    out.c[3] = m.c[3];
    return out;
}

// glm mat4 * mat4 (detail/type_mat4x4.inl): Result[c] = A0*B[c][0] + A1*B[c][1] + A2*B[c][2] + A3*B[c][3]
m4 matmul(const m4& A, const m4& B)
{
    m4 out;
    for (int c = 0; c < 4; ++c) {
        const v4& b = B.c[c];
        out.c[c] = add(add(add(mul(A.c[0], b.x), mul(A.c[1], b.y)), mul(A.c[2], b.z)), mul(A.c[3], b.w));
    }
    return out;
}

// CreateRotationMatrix (Util.h:13-18)
m4 rotation_xyz(float rx, float ry, float rz)
{
    m4 I = identity();
    m4 a = rotate(I, radians(rx), { 1, 0, 0 });
    m4 b = rotate(I, radians(ry), { 0, 1, 0 });
    m4 c = rotate(I, radians(rz), { 0, 0, 1 });
    return matmul(matmul(a, b), c);
}

// SphericalToWorldCoodinates (Util.h:7-11)
v3 spherical(float longitude, float latitude)
{
    float sint = std::sin(longitude);
    return { std::cos(latitude) * sint, std::sin(latitude) * sint, std::cos(longitude) };
}

void store(const m4& m, float out[16])
{
    for (int c = 0; c < 4; ++c) {
        out[4 * c + 0] = m.c[c].x;
        out[4 * c + 1] = m.c[c].y;
        out[4 * c + 2] = m.c[c].z;
        out[4 * c + 3] = m.c[c].w;
    }
}

// glm::cross
inline v3 cross(const v3& a, const v3& b)
{
    return { a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y };
}

struct quat { float x, y, z, w; };

// glm::tquat(vec3 eulerAngle) (gtc/quaternion.inl:124-136)
quat quat_from_euler(float ex, float ey, float ez)
{
    float cx = std::cos(ex * 0.5f), cy = std::cos(ey * 0.5f), cz = std::cos(ez * 0.5f);
    float sx = std::sin(ex * 0.5f), sy = std::sin(ey * 0.5f), sz = std::sin(ez * 0.5f);
    quat q;
    q.w = cx * cy * cz + sx * sy * sz;
    q.x = sx * cy * cz - cx * sy * sz;
    q.y = cx * sy * cz + sx * cy * sz;
    q.z = cx * cy * sz - sx * sy * cz;
    return q;
}

// glm quat * vec3 (gtc/quaternion.inl:298-309)
v3 rotate_vec(const quat& q, const v3& v)
{
    v3 qv = { q.x, q.y, q.z };
    v3 uv = cross(qv, v);
    v3 uuv = cross(qv, uv);
    return { v.x + ((uv.x * q.w) + uuv.x) * 2.0f,
             v.y + ((uv.y * q.w) + uuv.y) * 2.0f,
             v.z + ((uv.z * q.w) + uuv.z) * 2.0f };
}

}  // namespace

void child_transforms(float child[9][16])
{
    // Sphereflake.cpp:218-231: six children around the equator
    for (unsigned i = 0; i < 6; ++i) {
        float longitude = radians(90.f);
        float latitude = radians(60.0f * (float)i);
        v3 d = normalize(spherical(longitude, latitude));
        m4 t = rotation_xyz(90.0f, (float)(90u + i * 60u), 0.0f);
        t.c[3].x = d.x;
        t.c[3].y = d.y;
        t.c[3].z = d.z;
        store(t, child[i]);
    }
    // Sphereflake.cpp:233-248: three children on the upper cap
    static const float rot[3][3] = { { 325, 45, 15 }, { 145, 230, 165 }, { 60, 0, 0 } };
    for (unsigned i = 0; i < 3; ++i) {
        float longitude = radians(30.0f);
        float latitude = radians(30.0f + 120.0f * (float)i);
        v3 d = normalize(spherical(longitude, latitude));
        m4 t = rotation_xyz(rot[i][0], rot[i][1], rot[i][2]);
        t.c[3].x = d.x;
        t.c[3].y = d.y;
        t.c[3].z = d.z;
        store(t, child[6 + i]);
    }
}

void root_transform(const float o[3], float root[16])
{
    // translate(-o) * CreateRotationMatrix((90, 0, 0))   (Sphereflake.cpp:83)
    m4 T = identity();
    v3 v = { -o[0], -o[1], -o[2] };
    m4 I = identity();
    // glm::translate(m, v): Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3]
    T.c[3] = add(add(add(mul(I.c[0], v.x), mul(I.c[1], v.y)), mul(I.c[2], v.z)), I.c[3]);
    store(matmul(T, rotation_xyz(90.0f, 0.0f, 0.0f)), root);
}

void camera_corners(uint32_t W, uint32_t H, const float pos[3], float pitch, float yaw, float roll,
                    float fov, float o[3], float tl[3], float tr[3], float bl[3])
{
    float aspect = (float)W / (float)H;                       // camera.h:11-12
    // GetScaling (camera.h:111-114): glm vec3::length() is the component count, 3
    float d = std::tan(radians(fov / 2.0f)) / 3;
    quat q = quat_from_euler(yaw, pitch, roll);              // camera.h:65-68
    v3 P = { pos[0], pos[1], pos[2] };
    auto corner = [&](float sx, float sy, float* out) {
        v3 r = rotate_vec(q, { sx, sy, -1.0f });
        out[0] = P.x + r.x;
        out[1] = P.y + r.y;
        out[2] = P.z + r.z;
    };
    corner(-aspect * d, d, tl);                               // camera.h:37-41
    corner(aspect * d, d, tr);                                // camera.h:43-47
    corner(-aspect * d, -d, bl);                              // camera.h:49-53
    o[0] = P.x;
    o[1] = P.y;
    o[2] = P.z;
}

// radius chain: r_0 = 3.0f / 3.0f, r_d = r_{d-1} / 3.0f (Sphereflake.h:97; root call passes 3.0f)
float radius(uint32_t depth)
{
    float p = 3.0f, r = 1.0f;
    for (uint32_t d = 0; d <= depth; ++d) {
        r = p / 3.0f;
        p = r;
    }
    return r;
}

static inline float bits2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// Exact LOD threshold. The reference predicate  sqrtf(t / r) < C || t < 0  (Sphereflake.h:146, C = 70;
// SSE variant Sphereflake.h:129, C = 60) is a composition of correctly rounded monotone operations, so
// for t >= 0 it is true exactly on [0, T) for some float T; for t < 0 it is true. Hence
// pred(t) <=> t < T. Binary search over the ordered bit patterns of non-negative floats finds T.
float lod_threshold(float r, float lod_constant)
{
    auto pred = [r, lod_constant](float t) { return std::sqrt(t / r) < lod_constant || t < 0.0f; };
    uint32_t lo = 0, hi = 0x7f800000u;   // pred(lo) true (t = 0), pred(+inf) false
    while (hi - lo > 1) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (pred(bits2f(mid))) lo = mid; else hi = mid;
    }
    return bits2f(hi);
}

void depth_tables(DepthTables* t, float lod_constant)
{
    for (uint32_t d = 0; d < SF_DEPTH_TABLE; ++d) {
        float r = radius(d);
        float dr = r * 2.0f;
        t->r2_bound[d] = dr * dr;                 // Sphereflake.h:108-110
        t->r2_self[d] = r * r;                    // :180
        t->scale[d] = (4.0f / 3.0f) * r;          // :162
        t->lod[d] = lod_threshold(r, lod_constant);   // :146 (SSE :129)
    }
}

// Leaf threshold of depth d (kernel: skip building/testing the children of a node whose |c|^2 exceeds
// it). Every child C of a depth-d node N lies at |c_C - c_N| = s = (4/3) r_d and has bounding radius
// R = 2 r_{d+1}. A lane's float near root t for C is at least sqrt(|c_C|^2 - R^2 - dl) - sqrt(R^2 + dl),
// dl = 2^-16 |c_C|^2 (the reachability bound of the kernel), hence at least
// |c_N| (1 - 2^-16 - 2^-8) - 2R - s (1 + 2^-8). If |c_N| >= (T_{d+1} (1 + 2^-12) + 2R + s (1 + 2^-8)) / (1 - 2^-7),
// that exceeds T_{d+1} and no child can pass the LOD test (Sphereflake.h:146) for any ray. The extra
// 2^-8 on s and 2^-10 on the square cover the rounding of the unit offsets, the parent rotation and
// the kernel's own |c|^2. Doubles here; the float result rounds up by construction of the slack.
float leaf_threshold(const DepthTables* t, uint32_t d)
{
    if (d + 1u >= SF_DEPTH_TABLE) return INFINITY;
    const double T = t->lod[d + 1u], R = std::sqrt((double)t->r2_bound[d + 1u]), s = t->scale[d];
    const double rhs = T * (1.0 + 0x1p-12) + 2.0 * R + s * (1.0 + 0x1p-8);
    const double th = rhs / (1.0 - 0x1p-7);
    return (float)(th * th * (1.0 + 0x1p-10));
}

// Sobol direction numbers of dims 0 and 1 (the only dims the reference samples, Sphereflake.cpp:139-140),
// generated algorithmically; tests pin them against the reference table (tests/golden/sobol.json).
//   dim 0: van der Corput, M[k] = 2^(31-k) for k < 32, 0 beyond (the table stores 52 entries per dim)
//   dim 1: primitive polynomial x + 1: M[k] = M[k-1] ^ (M[k-1] >> 1), M[0] = 2^31, period 32
void sobol_matrices(uint32_t out[2][52])
{
    uint32_t v = 0x80000000u;
    for (uint32_t k = 0; k < 52; ++k) {
        out[0][k] = k < 32 ? (0x80000000u >> k) : 0u;
        if (k % 32 == 0) v = 0x80000000u;
        else v = v ^ (v >> 1);
        out[1][k] = v;
    }
}

// std::mt19937::seed(value) (init_genrand): state[624] = next index (624 = twist on first draw).
void mt19937_seed(uint32_t seed, uint32_t state[625])
{
    state[0] = seed;
    for (uint32_t i = 1; i < 624; ++i) state[i] = 1812433253u * (state[i - 1] ^ (state[i - 1] >> 30)) + i;
    state[624] = 624;
}

// SSAO::GenerateNoiseTexture (SSAO.cpp:144-164): 64x64 RGBA32F texels, each glm::normalize(vec4) of
// four std::uniform_real_distribution<float>(-1, 1) draws from std::mt19937 seeded 12512. The
// standard library is the same one the reference links (libstdc++ here), so this is the reference's
// own generator; glm 0.9.5 normalize(vec4) = x * (1 / sqrt(((x*x + y*y) + z*z) + w*w))
// (func_geometric.inl:268-277, func_exponential.inl:226-229).
void ssao_noise(float out[SF_NOISE_SIZE * SF_NOISE_SIZE * 4])
{
    std::mt19937 mt;
    mt.seed(12512);
    std::uniform_real_distribution<float> dist(-1, 1);
    for (int i = 0; i < SF_NOISE_SIZE * SF_NOISE_SIZE; ++i) {
        float v[4];
        for (float& x : v) x = dist(mt);
        const float sqr = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
        const float inv = 1.0f / std::sqrt(sqr);
        for (int k = 0; k < 4; ++k) out[4 * i + k] = v[k] * inv;
    }
}

// The final and blur passes sample their RGBA8 sources LINEAR at the fragment centre. In the
// 8-bit-subtexel texture model (sf_post.hip) that is exactly the fragment's own texel iff the centre
// coordinate (i+0.5) * (1/n) * n - 0.5 (post_ssao_blur.glsl:26-29, post_final.glsl:17) snaps to an
// integer for every i < n. Then the blur passes with no accepted tap reduce to a per-pixel weight,
// and the fused post kernel equals the multi-pass one bit for bit.
bool post_centre_exact(uint32_t n)
{
    const float fn = (float)n, ps = 1.0f / fn;
    for (uint32_t i = 0; i < n; ++i) {
        const float fc = (float)i + 0.5f;
        if (std::rint((fc * ps * fn - 0.5f) * 256.0f) != 256.0f * (float)i) return false;
    }
    return true;
}

// Ray generation divides pixel coordinates by the frame size (u = x / W, v = y / H, Sphereflake.cpp:149-150): a
// correctly rounded division, ~11 instructions on the device. With y = RN(1/n), q0 = RN(x y) and the exact
// residual r = x - q0 n (one fma), q = RN(q0 + r y) is RN(x / n) for these operands (Markstein's correction;
// exhaustively true for every n <= 16384 and x in [0, n]); the host checks the frame's own n before the kernels
// use it, so the shortcut never changes a bit.
bool division_by_reciprocal_exact(uint32_t n)
{
    if (n == 0u || n > (1u << 24)) return false;
    const float fn = (float)n, y = 1.0f / fn;
    for (uint32_t x = 0; x <= n; ++x) {
        const float fx = (float)x;
        const float q0 = fx * y;
        const float r = std::fma(-q0, fn, fx);
        const float q = std::fma(r, y, q0);
        const float ref = fx / fn;
        uint32_t a, b;
        std::memcpy(&a, &q, 4);
        std::memcpy(&b, &ref, 4);
        if (a != b) return false;
    }
    return true;
}

}  // namespace sfhost
