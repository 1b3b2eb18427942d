// sf_post.hip -- headless SSAO post-process of the G-buffer on gfx950.
//
// The reference runs three GL fullscreen passes plus a final pass on its G-buffer textures
// (SSAO.cpp:106-142, main.cpp:312-330):
//   SSAO           Shaders/post_ssao.glsl       16 position taps, noise-rotated kernel -> RGBA8 target
//   blur x, blur y Shaders/post_ssao_blur.glsl  depth/normal-aware 5-tap Gaussian -> RGBA8 targets
//   final          Shaders/post_final.glsl      colour = 0.5 + 0.5 (position + camera) times AO
// Here each pass is a kernel over the same data in HBM, with the GL state it depends on restated:
//   - G-buffer textures: RGBA32F, NEAREST, CLAMP_TO_EDGE (main.cpp:181-203)
//   - FBO targets: RGBA8 unorm, LINEAR, CLAMP_TO_EDGE (GLFramebufferObject.cpp:41-45): every pass
//     output is quantised to 8 bits; r = g = b, so one byte per pixel is kept
//   - noise: RGBA32F 64x64, LINEAR, REPEAT (SSAO.cpp:166-174)
// Texture filtering is a model, not a driver emulation: the texel-space coordinate is snapped to
// 8 fractional bits (round to nearest even), NEAREST takes floor, LINEAR the GL bilinear blend
// with those 1/256 weights. Division by a uniform or by a per-tap scalar is evaluated as
// multiplication by the correctly rounded reciprocal, as shader compilers emit vector / scalar.
// oracle/post.py restates the same formulas; the GPU result equals it bit for bit
// (tests/test_gpu_post.py).
//
// With the reference's thresholds (normalThreshold 2.47 > any dot of two unit normals) no blur tap is
// ever accepted, so both blurs collapse to a per-pixel weight: sf_post_fused does SSAO + blurs + final
// in one pass (36 B/pixel of HBM). The host proves the conditions (sf_capi.hip); otherwise the
// multi-pass kernels run.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sf_fastmath.h"
#include "sf_internal.h"

namespace {

__device__ __constant__ float kOffset[3] = { 0.0f, 1.3846153846f, 3.2307692308f };   // post_ssao_blur.glsl:9
__device__ __constant__ float kWeight[3] = { 0.2270270270f, 0.3162162162f, 0.0702702703f };   // :10

__device__ inline float4 ld4(const float* p, uint32_t i) { return reinterpret_cast<const float4*>(p)[i]; }

// texel-space coordinate snapped to 8 fractional bits; the clamp keeps NaN/inf offsets in int range
__device__ inline float snap(float x, float lim) { return rintf(fminf(fmaxf(x, -2.0f), lim + 2.0f) * 256.0f); }

__device__ inline int nearest(float u, float size, int n)   // NEAREST, CLAMP_TO_EDGE
{
    const int t = (int)floorf(snap(u * size, size) * (1.0f / 256.0f));
    return min(max(t, 0), n - 1);
}

// nearest() in fewer operations, the same texel for every u (NaN and infinities included): s256 = 256 size, hi =
// 256 n - 1. (u size) 256 rounds as u (256 size) (a power-of-two scale commutes with rounding; where u size is
// subnormal both snap to texel 0, where they overflow both are +-inf); clamping the snapped coordinate to [0, 256 n -
// 1] before the floor gives the texel clamped to [0, n - 1] after it (below 0 both give texel 0, at or above 256 n - 1
// both give n - 1, NaN: 0 in both); and floor(k / 256) of the integer k = rint(...) is k >> 8.
__device__ inline uint32_t nearest_fast(float u, float s256, float hi)
{
    return (uint32_t)rintf(fminf(fmaxf(u * s256, 0.0f), hi)) >> 8;
}

struct Lin {
    int i0, i1;
    float a;
};

__device__ inline Lin linear_clamp(float u, float size, int n)   // LINEAR, CLAMP_TO_EDGE
{
    const float c = snap(u * size - 0.5f, size);
    const float f = floorf(c * (1.0f / 256.0f));
    const int i = (int)f;
    return { min(max(i, 0), n - 1), min(max(i + 1, 0), n - 1), (c - f * 256.0f) * (1.0f / 256.0f) };
}

__device__ inline float blend(float t00, float t10, float t01, float t11, float a, float b)
{
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    return ((w00 * t00 + w10 * t10) + w01 * t01) + w11 * t11;
}

// k / 255 for every RGBA8 value, correctly rounded (a table instead of 3 full divisions per fragment)
struct UnormTable {
    float v[256];
    constexpr UnormTable() : v()
    {
        for (int k = 0; k < 256; ++k) v[k] = (float)k / 255.0f;
    }
};
__device__ __constant__ UnormTable kUnorm = UnormTable();

__device__ inline float unorm(uint8_t k) { return kUnorm.v[k]; }

__device__ inline uint8_t quant(float x)   // float -> RGBA8 unorm channel (NaN -> 0)
{
    return (uint8_t)floorf(fminf(fmaxf(x, 0.0f), 1.0f) * 255.0f + 0.5f);
}

// texture(source, u, v) of an 8-bit single-channel target
__device__ inline float sample_u8(const uint8_t* t, uint32_t w, uint32_t h, float fw, float fh, float u, float v)
{
    const Lin x = linear_clamp(u, fw, (int)w), y = linear_clamp(v, fh, (int)h);
    return blend(unorm(t[y.i0 * w + x.i0]), unorm(t[y.i0 * w + x.i1]), unorm(t[y.i1 * w + x.i0]),
                 unorm(t[y.i1 * w + x.i1]), x.a, y.a);
}

// texture(noiseTexture, uv * 0.1).xy: LINEAR, REPEAT over 64x64
__device__ inline float2 sample_noise(const float* noise, float u, float v)
{
    const float cs = rintf((u * (float)SF_NOISE_SIZE - 0.5f) * 256.0f);
    const float ct = rintf((v * (float)SF_NOISE_SIZE - 0.5f) * 256.0f);
    const float fs = floorf(cs * (1.0f / 256.0f)), ft = floorf(ct * (1.0f / 256.0f));
    const float a = (cs - fs * 256.0f) * (1.0f / 256.0f), b = (ct - ft * 256.0f) * (1.0f / 256.0f);
    const int m = SF_NOISE_SIZE - 1;
    const int x0 = (int)fs & m, x1 = ((int)fs + 1) & m, y0 = (int)ft & m, y1 = ((int)ft + 1) & m;
    const float4 t00 = ld4(noise, y0 * SF_NOISE_SIZE + x0), t10 = ld4(noise, y0 * SF_NOISE_SIZE + x1);
    const float4 t01 = ld4(noise, y1 * SF_NOISE_SIZE + x0), t11 = ld4(noise, y1 * SF_NOISE_SIZE + x1);
    return make_float2(blend(t00.x, t10.x, t01.x, t11.x, a, b), blend(t00.y, t10.y, t01.y, t11.y, a, b));
}

__device__ inline bool is_background(float4 p) { return p.x * p.x + p.y * p.y + p.z * p.z == 0.0f; }   // length == 0

// post_ssao.glsl:19-25 occlude(), split in two: the tap's texel (NEAREST) and its sample, then the occlusion term
// from the fetched sample -- so that ssao_at can have all 16 samples in flight before it uses the first (the taps
// reach tens of pixels: each fetch is an L2 round trip, and one tap at a time left the kernel latency-bound)
struct TapAxes {
    float sw, hw, sh, hh;   // 256 W, 256 W - 1, 256 H, 256 H - 1 (nearest_fast)
};

__device__ inline uint32_t tap_texel(const PostArgs& a, const TapAxes& ax, float fx, float fy, float ox, float oy,
                                     float rx, float ry)
{
    const uint32_t tx = nearest_fast((fx + ox) * rx, ax.sw, ax.hw);
    const uint32_t ty = nearest_fast((fy + oy) * ry, ax.sh, ax.hh);
    return ty * a.W + tx;
}

__device__ inline float occlude_ieee(const PostArgs& a, float4 s, float4 p, float4 n)
{
    const float dx = s.x - p.x, dy = s.y - p.y, dz = s.z - p.z;
    const float dist = sqrtf(dx * dx + dy * dy + dz * dz);
    const float id = 1.0f / dist;
    const float t = n.x * (dx * id) + n.y * (dy * id) + n.z * (dz * id);
    const float m = t - a.bias;
    const float c = m > 0.0f ? m : 0.0f;   // max(0.0, NaN) -> 0
    return c * (1.0f / (1.0f + dist * dist * a.scale)) * a.intensity;
}

// The range of a fragment's arguments to the short forms, both kinds against the tighter bounds [2^-96, 2^124]
// (the fragment falls back more often than it must only for arguments no frame produces): the min of d2 (a zero d2
// counted as +inf: sqrt(0) is in range) and |1 + dist^2 scale|, and the max of both -- two v_min3/v_max3 per tap.
// (NaN arguments need no flag: a NaN anywhere in a tap makes its term NaN on both paths, and the fragment's 8-bit
// value 0.)
struct TapRange {
    float lo = __builtin_inff(), hi = 0.0f;
    __device__ bool in_range() const { return lo >= SF_SQRT_MID_LO && hi <= SF_RCP_MID_HI; }
};

// occlude_ieee with dist = sqrt(d2), 1 / dist and 1 / (1 + dist^2 scale) by the short correctly rounded forms
// (sf_fastmath.h): the same bits where their arguments are in range (tracked in `rg`; where one is not -- a tiny,
// huge or infinite argument, rare -- the caller recomputes the fragment with occlude_ieee)
__device__ inline float occlude(const PostArgs& a, float4 s, float4 p, float4 n, TapRange& rg)
{
    const float dx = s.x - p.x, dy = s.y - p.y, dz = s.z - p.z;
    const float d2 = dx * dx + dy * dy + dz * dz;
    const float dist = sqrt_rn_mid(d2);
    const float id = d2 == 0.0f ? __builtin_inff() : rcp_rn_mid(dist);   // (d2 in range: dist in [2^-48, 2^62])
    const float arg = 1.0f + dist * dist * a.scale;
    rg.lo = fminf(fminf(rg.lo, d2 == 0.0f ? __builtin_inff() : d2), __builtin_fabsf(arg));
    rg.hi = fmaxf(fmaxf(rg.hi, d2), __builtin_fabsf(arg));
    const float t = n.x * (dx * id) + n.y * (dy * id) + n.z * (dz * id);
    const float c = fmaxf(t - a.bias, 0.0f);   // max(0.0, NaN) -> 0 (a -0 here only adds a zero of either sign)
    return c * rcp_rn_mid(arg) * a.intensity;
}

// post_ssao.glsl:27-61 at SSAO-target fragment (i, j); returns the 8-bit target value
__device__ inline uint8_t ssao_at(const PostArgs& a, uint32_t i, uint32_t j)
{
    const float fx = (float)i + 0.5f, fy = (float)j + 0.5f;
    const float rx = a.rfaw, ry = a.rfah;
    const float u = fx * rx, v = fy * ry;
    const uint32_t px = (uint32_t)nearest(v, a.fh, (int)a.H) * a.W + (uint32_t)nearest(u, a.fw, (int)a.W);
    const float4 p = ld4(a.pos, px);
    if (is_background(p)) return 0;   // vec4(0, 0, 0, 1)
    const float4 n = ld4(a.nrm, px);
    const float R = a.radius >= 0.0f ? a.radius : 8.0f * sf_key_float(a.stats[1]);
    const float rad = R / sqrtf(fabsf(p.z));
    const float2 nz = sample_noise(a.noise, u * 0.1f, v * 0.1f);
    const float qx = nz.x * 2.0f - 1.0f, qy = nz.y * 2.0f - 1.0f;
    const float len = sqrtf(qx * qx + qy * qy);
    const float il = 1.0f / len;
    const float nx = qx * il, ny = qy * il;
    const TapAxes ax{ a.fw * 256.0f, a.fw * 256.0f - 1.0f, a.fh * 256.0f, a.fh * 256.0f - 1.0f };
    // the 16 taps' texels and samples first (post_ssao.glsl:49-55: per kernel direction k, 0.25 c1, 0.75 c1,
    // 0.5 c2, c2), then the terms summed in the shader's order
    float4 s[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float kx = k == 0 ? 1.0f : k == 1 ? -1.0f : 0.0f;   // kernel[4] (post_ssao.glsl:15)
        const float ky = k == 2 ? 1.0f : k == 3 ? -1.0f : 0.0f;
        const float f = 2.0f * (nx * kx + ny * ky);                 // reflect(I, N) = I - 2 dot(N, I) N
        const float c1x = (kx - f * nx) * rad, c1y = (ky - f * ny) * rad;
        const float c2x = c1x * 0.707f - c1y * 0.707f, c2y = c1x * 0.707f + c1y * 0.707f;
        s[4 * k + 0] = ld4(a.pos, tap_texel(a, ax, fx, fy, c1x * 0.25f, c1y * 0.25f, rx, ry));
        s[4 * k + 1] = ld4(a.pos, tap_texel(a, ax, fx, fy, c1x * 0.75f, c1y * 0.75f, rx, ry));
        s[4 * k + 2] = ld4(a.pos, tap_texel(a, ax, fx, fy, c2x * 0.5f, c2y * 0.5f, rx, ry));
        s[4 * k + 3] = ld4(a.pos, tap_texel(a, ax, fx, fy, c2x, c2y, rx, ry));
    }
    float ao = 0.0f;
    TapRange rg;
#pragma unroll
    for (int q = 0; q < 16; ++q) ao += occlude(a, s[q], p, n, rg);
    if (!rg.in_range()) {   // (rare) some tap's argument outside the short forms' ranges: the fragment again, IEEE throughout
        ao = 0.0f;
#pragma unroll 1
        for (int q = 0; q < 16; ++q) {
            const int k = q >> 2, r = q & 3;
            const float kx = k == 0 ? 1.0f : k == 1 ? -1.0f : 0.0f;
            const float ky = k == 2 ? 1.0f : k == 3 ? -1.0f : 0.0f;
            const float f = 2.0f * (nx * kx + ny * ky);
            const float c1x = (kx - f * nx) * rad, c1y = (ky - f * ny) * rad;
            const float c2x = c1x * 0.707f - c1y * 0.707f, c2y = c1x * 0.707f + c1y * 0.707f;
            const float ox = r == 0 ? c1x * 0.25f : r == 1 ? c1x * 0.75f : r == 2 ? c2x * 0.5f : c2x;
            const float oy = r == 0 ? c1y * 0.25f : r == 1 ? c1y * 0.75f : r == 2 ? c2y * 0.5f : c2y;
            ao += occlude_ieee(a, ld4(a.pos, tap_texel(a, ax, fx, fy, ox, oy, rx, ry)), p, n);
        }
    }
    ao = ao / 16.0f;
    return quant(1.0f - ao);
}

// weight the centre tap gets when both taps of both offsets are rejected (post_ssao_blur.glsl:44-63)
__device__ inline float rejected_weight()
{
    float lo = 0.0f;
    lo += kWeight[1];
    lo += kWeight[1];
    lo += kWeight[2];
    lo += kWeight[2];
    return kWeight[0] + lo;
}

// post_final.glsl:15-28 given the AO value sampled at the fragment
__device__ inline void final_store(const PostArgs& a, uint32_t px, float4 p, float ssao)
{
    uchar4 o;
    if (is_background(p)) {
        o = make_uchar4(0, 0, 0, 255);
    } else {
        o.x = quant((0.5f + 0.5f * (p.x + a.cam[0])) * ssao);
        o.y = quant((0.5f + 0.5f * (p.y + a.cam[1])) * ssao);
        o.z = quant((0.5f + 0.5f * (p.z + a.cam[2])) * ssao);
        o.w = 255;
    }
    reinterpret_cast<uchar4*>(a.rgba)[px] = o;
}

// 16x16-pixel workgroups: a wave covers 16x4, so the SSAO taps (a few pixels around) share lines.
// XCD-aware tile order: the dispatcher deals workgroups round-robin over the 8 XCDs (workgroup b on XCD b mod 8),
// each with its own L2. The SSAO taps reach tens of pixels (R / sqrt|z|: median ~11 px, p99 ~70 px at 1080p), so
// with tiles in launch order every XCD's L2 would serve taps all over the frame; here XCD x's workgroups take the
// x-th contiguous eighth of the tiles in row-major order -- a stripe of rows, its taps mostly in its own L2. (A
// bijection of the workgroup index whatever the placement: only locality depends on it.)
__device__ inline bool pixel(uint32_t w, uint32_t h, uint32_t& i, uint32_t& j)
{
    const uint32_t gx = gridDim.x, nb = gx * gridDim.y;
    const uint32_t b = blockIdx.y * gx + blockIdx.x;
    const uint32_t q = nb >> 3, r = nb & 7u, x = b & 7u, k = b >> 3;
    const uint32_t lin = x < r ? x * (q + 1u) + k : r * (q + 1u) + (x - r) * q + k;
    i = (lin % gx) * 16u + (threadIdx.x & 15u);
    j = (lin / gx) * 16u + (threadIdx.x >> 4);
    return i < w && j < h;
}

}  // namespace

// SSAO pass into the SSAO target (aw x ah)
extern "C" __global__ void __launch_bounds__(256) sf_post_ssao(PostArgs a)
{
    uint32_t i, j;
    if (!pixel(a.aw, a.ah, i, j)) return;
    a.ao[j * a.aw + i] = ssao_at(a, i, j);
}

// One blur pass (post_ssao_blur.glsl) over the W x H target: dir 0 = x (source: SSAO target),
// dir 1 = y (source: x-blur target)
extern "C" __global__ void __launch_bounds__(256) sf_post_blur(PostArgs a, uint32_t dir)
{
    uint32_t i, j;
    if (!pixel(a.W, a.H, i, j)) return;
    const uint8_t* src = dir ? a.blur_h : a.ao;
    uint8_t* dst = dir ? a.blur_v : a.blur_h;
    const uint32_t sw = dir ? a.W : a.aw, sh = dir ? a.H : a.ah;
    const float fsw = dir ? a.fw : a.faw, fsh = dir ? a.fh : a.fah;
    const float psx = a.rfw, psy = a.rfh;   // pixelSize = pixelSizeGBuffer (same size)
    const float fx = (float)i + 0.5f, fy = (float)j + 0.5f;
    const float ux = fx * psx, uy = fy * psy;
    const uint32_t px = (uint32_t)nearest(uy, a.fh, (int)a.H) * a.W + (uint32_t)nearest(ux, a.fw, (int)a.W);
    const float4 p = ld4(a.pos, px), n = ld4(a.nrm, px);
    const float dx = dir ? 0.0f : 1.0f, dy = dir ? 1.0f : 0.0f;
    float color = 0.0f, lo = 0.0f;
#pragma unroll
    for (int k = 1; k < 3; ++k) {
        const float ox = dx * kOffset[k] * psx, oy = dy * kOffset[k] * psy;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const float sx = side ? ux - ox : ux + ox, sy = side ? uy - oy : uy + oy;
            const uint32_t q = (uint32_t)nearest(sy, a.fh, (int)a.H) * a.W + (uint32_t)nearest(sx, a.fw, (int)a.W);
            const float4 sp = ld4(a.pos, q), sn = ld4(a.nrm, q);
            if (n.x * sn.x + n.y * sn.y + n.z * sn.z >= a.normal_thr && fabsf(sp.z - p.z) >= a.depth_thr)
                color += sample_u8(src, sw, sh, fsw, fsh, sx, sy) * kWeight[k];
            else
                lo += kWeight[k];
        }
    }
    color += sample_u8(src, sw, sh, fsw, fsh, ux, uy) * (kWeight[0] + lo);
    dst[j * a.W + i] = quant(color);
}

// Final pass (post_final.glsl) from the y-blur target
extern "C" __global__ void __launch_bounds__(256) sf_post_final(PostArgs a)
{
    uint32_t i, j;
    if (!pixel(a.W, a.H, i, j)) return;
    const float u = ((float)i + 0.5f) * a.rfw, v = ((float)j + 0.5f) * a.rfh;
    const uint32_t px = (uint32_t)nearest(v, a.fh, (int)a.H) * a.W + (uint32_t)nearest(u, a.fw, (int)a.W);
    const float4 p = ld4(a.pos, px);
    final_store(a, j * a.W + i, p, is_background(p) ? 0.0f : sample_u8(a.blur_v, a.W, a.H, a.fw, a.fh, u, v));
}

// All four passes in one, valid when the host has proven (sf_capi.hip post_fusable): SSAO target =
// G-buffer size, no blur tap can pass the normal test, and every LINEAR centre sample is the
// fragment's own texel. Each blur is then color = own * weight, and the final samples its own texel.
extern "C" __global__ void __launch_bounds__(256) sf_post_fused(PostArgs a)
{
    uint32_t i, j;
    if (!pixel(a.W, a.H, i, j)) return;
    const uint32_t px = j * a.W + i;
    const uint8_t s = ssao_at(a, i, j);
    if (a.ao) a.ao[px] = s;
    const float w = rejected_weight();
    const uint8_t h = quant(unorm(s) * w);
    const uint8_t v = quant(unorm(h) * w);
    // nearest(own centre) == (i, j) for the final's uv in this regime, as in ssao_at
    const float4 p = ld4(a.pos, px);
    final_store(a, px, p, unorm(v));
}
