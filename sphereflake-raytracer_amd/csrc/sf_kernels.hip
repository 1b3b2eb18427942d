// sf_kernels.hip -- gfx950 (CDNA4) kernels of the Sphereflake primary-ray G-buffer renderer.
//
// Hot path replaced (reference paths relative to /root/reference):
//   ray generation           sphereflake/Sphereflake.cpp:149-150,162-167
//   recursive traversal      sphereflake/Sphereflake.h:86-226 (IntersectSphereflake)
//   packet math              sphereflake/SIMD_AVX.h:59-81 (4x4 product), 163-180 (Dot/Normalize),
//                            236-270 (RaySphereIntersection)
//   G-buffer scatter         sphereflake/Sphereflake.cpp:186-201
//   frame-less sampler       sphereflake/Sphereflake.cpp:86-214, Sobol.cpp:41-55
//
// Numerics: IEEE binary32, the reference's exact operation order, contraction OFF (this file
// and the compile line), correctly rounded division and sqrt (HIP default), denormals kept,
// x86 rsqrtps reproduced from a table. Full frames equal the reference AVX path bit for bit
// under per-ray semantics; the progressive mode reproduces the reference's
// 8-ray packet semantics (packet-wide early-outs, Sphereflake.h:140-153, 207-211,
// SIMD_AVX.h:247-258) bit for bit.
//
// Kernels
//   sf_trace_queue2 -- the product kernel (full frames): a persistent grid of 2-wave workgroups; each wave64
//                      traces one 8x8 pixel tile (or a part of one) per work unit, taken from the previous
//                      render's heavy-first unit order (static first unit, then its block group's atomic
//                      queue). The DFS over the sphereflake is wave-uniform: a node is visited iff at least
//                      one lane of the tile visits it, and each lane keeps exactly its own per-ray visit
//                      semantics through lane masks. When a node expands, 36 lanes build its 9 child
//                      transforms cooperatively (one 4-float column each) into the wave's LDS level,
//                      instead of every ray doing 9 4x4 products per node as the reference packets do.
//                      sf_trace_queue1/4: 1 / 4 waves per workgroup; sf_trace_queue2p: the latency variant
//                      (pipelined child loop) for frames that fill the grid less than twice.
//   sf_order_scan / sf_order_scatter -- the next render's unit order from this render's tile costs.
//   sf_trace_wave{1,2,4} -- the same traversal, one workgroup per tile group (non-persistent A/B path).
//   sf_fixup_wave   -- re-traces the tiles flagged as needing more LDS levels than provisioned, with
//                      SF_MAX_LEVELS levels, and those with an exact tie under the front-first child order,
//                      in index order.
//   sf_trace_ray    -- one thread per ray with a private traversal stack (the straightforward
//                      formulation; cross-check and comparison point).
//   sf_band_unpack  -- packed band slabs of a multi-GPU frame -> the G-buffer at frame positions.
//   sf_mt_draws / sf_packet_* / sf_progressive_* -- frame-less progressive mode.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "sf_internal.h"

#pragma clang fp contract(off)

#define SF_MAX_LEVELS 31         // SF_MAX_DEPTH_LIMIT (ebits is 32 bits)

namespace {

// x86 rsqrtps (SIMD_AVX.h:173), reproduced exactly from the measured table.
__device__ __forceinline__ float rsqrtps_x86(float x, const uint32_t* __restrict__ lut)
{
    const uint32_t b = __float_as_uint(x);
    const uint32_t E = (b >> 23) & 0xffu;
    const uint32_t key = ((E & 1u) << 10) | ((b & 0x7fffffu) >> 13);
    const int32_t E0 = (E & 1u) ? 127 : 128;
    const int32_t k = ((int32_t)E - E0) / 2;
    uint32_t r = (uint32_t)((int32_t)lut[key] - k * (1 << 23));
    if ((b & 0x7fffffffu) > 0x7f800000u) r = b | 0x00400000u;     // NaN -> quiet NaN
    else if (E == 0u) r = (b & 0x80000000u) | 0x7f800000u;        // +-0 / denormal -> +-inf
    else if (b & 0x80000000u) r = 0xffc00000u;                    // negative -> default NaN
    else if (E == 0xffu) r = 0u;                                  // +inf -> +0
    return __uint_as_float(r);
}

// SIMD::Normalize (SIMD_AVX.h:170-180): rsqrt + one Newton-Raphson step.
__device__ __forceinline__ void normalize3(float& x, float& y, float& z, const uint32_t* __restrict__ lut)
{
    const float len = (x * x + y * y) + z * z;
    const float nr = rsqrtps_x86(len, lut);
    const float muls = (len * nr) * nr;
    const float s = (0.5f * nr) * (3.0f - muls);
    x = x * s;
    y = y * s;
    z = z * s;
}

// Ray direction (Sphereflake.cpp:149-150, 162-167): u = x/W, v = y/H at the pixel corner.
__device__ __forceinline__ void ray_dir(const FrameArgs& a, float x, float y, float& dx, float& dy, float& dz,
                                        const uint32_t* __restrict__ lut)
{
    float u, v;
    // (uniform) RN(x / W) as one product and one fma correction (sfhost::division_by_reciprocal_exact); the
    // context's reciprocals by scalar loads from the constant block
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) DeviceConsts* ConstK;
    const ConstK kc = (ConstK)(const void*)a.consts;
    const float rw = kc->rw, rh = kc->rh;
    const uint32_t fast = kc->fast_div;
#else
    const float rw = a.consts->rw, rh = a.consts->rh;
    const uint32_t fast = a.consts->fast_div;
#endif
    if (fast) {
        const float qu = x * rw, qv = y * rh;
        u = __builtin_fmaf(__builtin_fmaf(-qu, a.fw, x), rw, qu);
        v = __builtin_fmaf(__builtin_fmaf(-qv, a.fh, y), rh, qv);
    } else {
        u = x / a.fw;
        v = y / a.fh;
    }
    dx = ((a.tl[0] + a.dh[0] * u) + a.dv[0] * v) - a.o[0];
    dy = ((a.tl[1] + a.dh[1] * u) + a.dv[1] * v) - a.o[1];
    dz = ((a.tl[2] + a.dh[2] * u) + a.dv[2] * v) - a.o[2];
    normalize3(dx, dy, dz, lut);
}

// Near root of RaySphereIntersection (SIMD_AVX.h:260-267); NaN when R2 < d2 (lanes that missed).
__device__ __forceinline__ float near_root(float tca, float d2, float R2)
{
    const float thc = __builtin_sqrtf(R2 - d2);
    const float t0 = tca + thc;
    const float t1 = tca - thc;
    return (t0 <= t1) ? t0 : t1;
}

// One level down the transform chain (Sphereflake.h:162-164, SIMD_AVX.h:59-81 product without FMA): `out` = the
// frame of child i of a depth-p node whose frame is P, both as 3 x 4 {column-major xyz} (xf[3 c + r]). The child's
// unit frame has its translation column scaled by (4/3) r_p. The per-ray kernel and the slab unpack both chain
// with it, so a node's frame is the same float values whichever computes it.
// (child: the 9 unit child frames, scale: the per-depth child translation scales -- from the constant block, or an
// LDS image of them in the slab unpack)
// SF_AFFINE_FMA (round 6): the unit child frames are affine -- row 3 of column c is exactly 0 (c < 3) or 1 (c = 3), as
// glm's translate/rotate make them (Sphereflake.cpp:216-249; sf_set_setup refuses any other) -- so the 4th product
// P[9 + r] * b3 is exact (+-0 or P[9 + r] itself) and s + P[9 + r] * b3 rounds once either way: fma(P[9 + r], b3, s)
// is the same float bit for bit (also for -0, inf and NaN), one VALU instead of two. The traversal's cooperative child
// build (expand) and the slab unpack's centre use the same form.
__device__ __forceinline__ void child_frame(const float (*child)[16], const float* scale, uint32_t p, uint32_t i,
                                            const float* P, float* out)
{
    const float s = scale[p];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float* B = child[i] + 4 * c;
        const float b0 = c == 3 ? B[0] * s : B[0];
        const float b1 = c == 3 ? B[1] * s : B[1];
        const float b2 = c == 3 ? B[2] * s : B[2];
        const float b3 = B[3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
            out[3 * c + r] = __builtin_fmaf(P[9 + r], b3, (P[r] * b0 + P[3 + r] * b1) + P[6 + r] * b2);   // (SF_AFFINE_FMA)
    }
}
__device__ __forceinline__ void child_frame(const DeviceConsts* __restrict__ K, uint32_t p, uint32_t i,
                                            const float* P, float* out)
{
    child_frame(K->child, K->dt.scale, p, i, P, out);
}

struct HitState {
    float minT;
    float cx, cy, cz;     // centre of the nearest accepted sphere
    uint32_t index;       // its heap index (low 32 bits)
    int32_t depth;        // its depth (wave traversal: tie-breaking, see traverse)
    bool hit;
};

// Position and normal of the nearest hit (Sphereflake.h:218-224). Computed once from the winning
// t and centre: the same operations on the same operands as the reference's per-acceptance update.
__device__ __forceinline__ void shade(float dx, float dy, float dz, const HitState& h, const uint32_t* __restrict__ lut,
                                      float& px, float& py, float& pz, float& nx, float& ny, float& nz)
{
    px = py = pz = nx = ny = nz = 0.f;
    if (h.hit) {
        px = dx * h.minT;
        py = dy * h.minT;
        pz = dz * h.minT;
        nx = px - h.cx;
        ny = py - h.cy;
        nz = pz - h.cz;
        normalize3(nx, ny, nz, lut);
    }
}

// max over the wave of a non-negative float (ordered as its bit pattern)
__device__ __forceinline__ float wave_max_pos(float v)
{
    uint32_t b = __float_as_uint(v);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, m, 64));
    return __uint_as_float(__builtin_amdgcn_readfirstlane(b));
}

__device__ __forceinline__ float wave_min(float v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fminf(v, __shfl_xor(v, m, 64));
    return v;
}

// Wave64 ballot straight on the compare mask (no bool -> int -> compare round trip).
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// (lane in m) ? b : a -- one v_cndmask on an SGPR lane mask (a wave ballot), no per-lane bool
__device__ __forceinline__ float sel_mask(float a, float b, uint64_t m)
{
    float r;
    __asm__("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// dst = (lane in m) ? src : dst, in dst's own register (tied operand): one v_cndmask on an SGPR lane
// mask, no per-lane bool materialised and no copy between a pre- and a post-update register
__device__ __forceinline__ void sel_in_place(float& dst, float src, uint64_t m)
{
    __asm__("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(dst) : "v"(src), "s"(m));
}
__device__ __forceinline__ void sel_in_place(uint32_t& dst, uint32_t src, uint64_t m)
{
    __asm__("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(dst) : "v"(src), "s"(m));
}

// Near root with sqrt_rn(x) for x = R2 - d2 >= 2^-96 (finite): the hardware estimate and its +-1 ulp correction
// by two fma residuals -- the sequence the compiler emits for a correctly rounded sqrtf, without the scaling of
// tiny arguments and the zero/inf class fix-up that x >= 2^-96 never needs, so bit for bit its result there.
__device__ __forceinline__ float near_root_big(float tca, float x)
{
    const float s0 = __builtin_amdgcn_sqrtf(x);
    const float sdn = __uint_as_float(__float_as_uint(s0) - 1u);
    const float sup = __uint_as_float(__float_as_uint(s0) + 1u);
    const float rdn = __builtin_fmaf(-sdn, s0, x);
    const float rup = __builtin_fmaf(-sup, s0, x);
    float thc = rdn <= 0.0f ? sdn : s0;
    thc = rup > 0.0f ? sup : thc;
    const float t0 = tca + thc;
    const float t1 = tca - thc;
    return (t0 <= t1) ? t0 : t1;
}

// Exact near root for the rare undecided lanes of the LOD bracket. Inlined: its uniform branch stays a
// real branch (the structurizer leaves wave-uniform regions alone), and without a call no SGPRs are saved
// around it (round 1 kept it out of line so it would not be if-converted into every child test).
__device__ __forceinline__ float near_root_exact(float tca, float d2, float R2)
{
    return near_root(tca, d2, R2);
}

// "Any lane of my group": a group is the lane itself (PW = 0, per-ray semantics) or the PW lanes of a
// reference packet (packet semantics: movemask early-outs, SIMD_AVX.h:247,255, Sphereflake.h:140,149,207;
// PW = 8 for the AVX path, 4 for the SSE path, SIMD_SSE.h).
template <int PW>
__device__ __forceinline__ bool group_any(bool p)
{
    if constexpr (PW != 0) {
        const uint64_t b = wave_ballot(p);
        return ((b >> (threadIdx.x & (64u - PW))) & ((1ull << PW) - 1ull)) != 0ull;
    } else {
        return p;
    }
}

// ------------------------------------------------------------------------------------------
// Wave-coherent traversal of IntersectSphereflake (Sphereflake.h:86-226).
//
// The DFS runs over EXPANDED nodes only (nodes that passed bounding sphere + LOD for at least one
// lane of the wave). When a node expands, the wave
//   1. builds its 9 child world transforms cooperatively into the LDS table of its level
//      (36 lanes: one column each; child translation scaled by (4/3) r, world = parent * child,
//      SIMD_AVX.h:59-81, Sphereflake.h:162-172) plus Dot(centre, centre) of each child;
//   2. culls the children no ray of the tile's cone can reach (9 centre lanes in parallel), then tests
//      the remaining ones one after the other in index order (a uniform loop over a 9-bit mask), giving
//      each lane a 9-bit "child expands" vector E and the wave a 9-bit "pending" mask of children some
//      lane expands.
// Children are then entered in index order. A node's own sphere is tested when the node is entered
// (pre-order) with an ancestor tie-break that reproduces the reference's post-order "first strictly smaller
// t wins" (Sphereflake.h:174-224) -- see self_test. Children that no lane expands cost only their bounding
// test, as in the reference.
//
// Per node (group = the lane itself for per-ray semantics, the 8 lanes of a reference AVX packet
// for packet semantics):
//   bounding   hb = active && any_g(tca >= 0) && any_g(d2 <= (2r)^2)
//   LOD        ex = hb && any_g(t < T_d)          [T_d exact threshold of sqrtf(t/r) < 70 || t < 0]
//   self       hs = active && any_g(tca >= 0) && any_g(d2 <= r^2); accept lanes with d2 <= r^2 && t < minT
// For per-ray groups these are exactly the reference's per-lane tests.
// ------------------------------------------------------------------------------------------
// Per-wave LDS image (floats): [root: 16][cone: 8][per level: table | E 32 | pad 3]. A transform is
// {cx cy cz cc} (cc = Dot(centre, centre)) and its three axis columns. The root keeps them as 4 contiguous
// float4; a level table keeps plane 0 = the 9 children's {centre, cc} float4, then planes 1..3 = their
// column j as float3 (9 x 3 floats each): 117 floats per level instead of 144, so 8 waves fit per SIMD.
struct TraverseLds {
    float* base;
    __device__ __forceinline__ float* root() const { return base; }
    __device__ __forceinline__ float* cone() const { return base + SF_LDS_ROOT; }
    __device__ __forceinline__ float* table(uint32_t lvl) const
    {
        return base + SF_LDS_ROOT + SF_LDS_CONE + lvl * SF_LDS_LEVEL;
    }
    __device__ __forceinline__ uint16_t* E(uint32_t lvl) const
    {
        return reinterpret_cast<uint16_t*>(base + SF_LDS_ROOT + SF_LDS_CONE + lvl * SF_LDS_LEVEL + SF_LDS_TABLE);
    }
};

template <bool B> struct BoolC { static constexpr bool value = B; };

__device__ __forceinline__ void lds_fence()
{
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
}

__device__ __forceinline__ float readlane_f(float v, uint32_t l)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)l));
}
// Lane l of `old` := v (uniform v and l) as a per-lane select: no divergent region, no asm.
__device__ __forceinline__ uint32_t writelane_u(uint32_t v, uint32_t l, uint32_t old)
{
    return (threadIdx.x & 63u) == l ? v : old;
}

// Lane l of `old` := v (uniform v and l): one v_writelane_b32 (traverse_ray's push; a select costs v_cmp, v_mov and
// v_cndmask per word)
__device__ int sf_amdgcn_writelane(int v, int l, int old) __asm("llvm.amdgcn.writelane.i32");   // (no clang builtin)
__device__ __forceinline__ uint32_t writelane_s(uint32_t v, uint32_t l, uint32_t old)
{
    return (uint32_t)sf_amdgcn_writelane((int)v, (int)l, (int)old);
}

// One lane's 64-bit global atomic add on behalf of the wave (EXEC forced to lane 0 inside the asm).
__device__ __forceinline__ void wave_atomic_add_u64(uint64_t* p, uint64_t v)
{
    uint64_t saved;
    const uint32_t zero = 0u;
    __asm__ volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "global_atomic_add_x2 %1, %2, %3\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "s_mov_b64 exec, %0\n\t"
        : "=&s"(saved)
        : "v"(zero), "v"(v), "s"(p)
        : "memory");
}

// Diagnostic build only (make PHASES=1): s_memtime stamps at the DFS segment boundaries, summed per
// segment into 64-bit scalars and added to phase_sums once per wave. Segments: 0->1 push bookkeeping,
// 1->2 expand (node read, build, child tests), 3->4 self test, 4->5 pop; 0 is taken at the loop head (and sums
// what ran since the previous stamp: the child tests no lane passed).
// Never compiled into the product library; read its SHARES, not its run time.
#ifdef SF_PHASE_STAMPS
#define SF_STAMP_DECL uint64_t ph_last = __builtin_amdgcn_s_memtime(), ph_sum[7] = {0, 0, 0, 0, 0, 0, 0}
#define SF_STAMP(k)                                                                            \
    do {                                                                                       \
        uint64_t t_;                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        __asm__ volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        ph_sum[k] += t_ - ph_last;                                                             \
        ph_last = t_;                                                                          \
    } while (0)
#define SF_STAMP_FLUSH(p)                                                                      \
    do {                                                                                       \
        if (p) {                                                                               \
            for (int k_ = 0; k_ < 7; ++k_) wave_atomic_add_u64((uint64_t*)(p) + k_, ph_sum[k_]);  \
        }                                                                                      \
    } while (0)
#elif defined(SF_COUNTS)
// Diagnostic build only (make COUNTS=1): per-wave event counts instead of stamps, summed into
// phase_sums[k]: 0 nodes whose children are tested, 1 child-loop iterations, 2 iterations no lane
// hits (bounding), 3 children entered, 4 leaf skips; lane utilisation: 5 active lanes summed over
// child-loop iterations, 6 bounding-hit lanes summed over them, 7 active lanes summed over expanded
// nodes, 8 inline leaf self tests, 9 their active lanes, 10 child-loop iterations at node depth >= 4,
// 11 their active lanes, 12/13/14 iterations with <= 4 / <= 16 / <= 32 active lanes, 15 waves traced.
#define SF_STAMP_DECL uint64_t ph_sum[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}
#define SF_STAMP(k)
#define SF_COUNT(k, v) (ph_sum[k] += (v))
#define SF_STAMP_FLUSH(p)                                                                      \
    do {                                                                                       \
        if (p) {                                                                               \
            ph_sum[15] = 1;                                                                    \
            for (int k_ = 0; k_ < 16; ++k_) wave_atomic_add_u64((uint64_t*)(p) + k_, ph_sum[k_]); \
        }                                                                                      \
    } while (0)
#else
#define SF_STAMP_DECL
#define SF_STAMP(k)
#define SF_STAMP_FLUSH(p) (void)(p)
#endif
#ifndef SF_COUNT
#define SF_COUNT(k, v)
#endif

// Per-depth constants {(2r)^2, r^2, (4/3) r, T} through the constant address space, so a uniform depth
// gives one s_load_dwordx4 from the scalar cache. Through a generic pointer the compiler cannot rule
// out aliasing with the kernel's global stores and emits a vector load plus a vmcnt wait instead.
__device__ __forceinline__ float4 depth_consts(const DeviceConsts* K, uint32_t d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    // a 32-bit byte offset added to the table base: the scalar load takes it as its SGPR offset, with no
    // 64-bit address arithmetic on the scalar unit per access
    typedef const __attribute__((address_space(4))) float4* ConstF4;
    typedef const __attribute__((address_space(4))) char* ConstC;
    return *(ConstF4)((ConstC)(const void*)K->depth8 + (d << 5));
#else
    return reinterpret_cast<const float4*>(K->depth8)[2u * d];   // host pass: never executed
#endif
}
// depth_consts / depth_cull / depth_far of the depth whose byte offset `o` = d << 5 the caller carries
__device__ __forceinline__ float4 depth_consts_at(const DeviceConsts* K, uint32_t o)
{
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float4* ConstF4;
    typedef const __attribute__((address_space(4))) char* ConstC;
    return *(ConstF4)((ConstC)(const void*)K->depth8 + o);
#else
    return reinterpret_cast<const float4*>(K->depth8)[o >> 4];
#endif
}
__device__ __forceinline__ float depth_word_at(const DeviceConsts* K, uint32_t o, uint32_t w)
{
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float* ConstF;
    typedef const __attribute__((address_space(4))) char* ConstC;
    return *(ConstF)((ConstC)(const void*)K->depth8 + o + 4u * w);
#else
    return reinterpret_cast<const float*>(K->depth8)[(o >> 2) + w];
#endif
}
// {leaf, 0, 0, 0} of depth d (see DeviceConsts::depth8)
__device__ __forceinline__ float depth_leaf(const DeviceConsts* K, uint32_t d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float* ConstF;
    typedef const __attribute__((address_space(4))) char* ConstC;
    return *(ConstF)((ConstC)(const void*)K->depth8 + (d << 5) + 16u);
#else
    return reinterpret_cast<const float4*>(K->depth8)[2u * d + 1u].x;
#endif
}

// {.., cull} of depth d: 2 r_d (1 + 2 SF_OCCL_MARGIN), rounded up (see DeviceConsts::depth8)
__device__ __forceinline__ float depth_cull(const DeviceConsts* K, uint32_t d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float* ConstF;
    typedef const __attribute__((address_space(4))) char* ConstC;
    return *(ConstF)((ConstC)(const void*)K->depth8 + (d << 5) + 20u);
#else
    return reinterpret_cast<const float4*>(K->depth8)[2u * d + 1u].y;
#endif
}

// traverse's status bits: the tile needs more levels than provisioned; an exact tie under the front-first order
#define SF_STATUS_OVERFLOW 1u
#define SF_STATUS_TIE 2u

// {.., far} of depth d: T_d + 2 r_d (1 + 2^-18), rounded up (see DeviceConsts::depth8)
__device__ __forceinline__ float depth_far(const DeviceConsts* K, uint32_t d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float* ConstF;
    typedef const __attribute__((address_space(4))) char* ConstC;
    return *(ConstF)((ConstC)(const void*)K->depth8 + (d << 5) + 24u);
#else
    return reinterpret_cast<const float4*>(K->depth8)[2u * d + 1u].z;
#endif
}

// Root transform -> the wave's LDS image in the transform layout (Sphereflake.cpp:83). The same for
// every tile of a frame: kernels stage it once per wave, before any tile loop.
__device__ __forceinline__ void stage_root(float* __restrict__ Lbase, const float* root)
{
    const uint32_t lane = threadIdx.x & 63u;
    if (lane < 16u) {
        const float rcc = (root[9] * root[9] + root[10] * root[10]) + root[11] * root[11];
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            float rk = 0.f;
            if (k < 3) rk = root[9 + k];
            else if (k == 3) rk = rcc;
            else if ((k & 3) != 3) rk = root[3 * ((k >> 2) - 1) + (k & 3)];
            v = (lane == (uint32_t)k) ? rk : v;
        }
        Lbase[lane] = v;   // TraverseLds::root()
    }
}

// The same staging without a branch on the lane (the multi-frame trace re-stages the root inside its persistent loop,
// where a lane-dependent region made the compiler allocate the whole loop's registers worse: 62 -> 30 SGPR spills):
// lane l writes word l & 15 -- the lanes above 15 repeat a lower lane's store, same address and value.
__device__ __forceinline__ void stage_root_all_lanes(float* __restrict__ Lbase, const float* root)
{
    const uint32_t l = threadIdx.x & 15u;
    const float rcc = (root[9] * root[9] + root[10] * root[10]) + root[11] * root[11];
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        float rk = 0.f;
        if (k < 3) rk = root[9 + k];
        else if (k == 3) rk = rcc;
        else if ((k & 3) != 3) rk = root[3 * ((k >> 2) - 1) + (k & 3)];
        v = (l == (uint32_t)k) ? rk : v;
    }
    Lbase[l] = v;   // TraverseLds::root()
}

// PW: packet width of the semantics (0 per ray, 8 (AVX) or 4 (SSE) frame-less packets); PIPE: the latency
// variant of the per-ray child loop (small frames, whose heaviest tiles' serial DFS is the frame)
// Lane -> (child bi, column bc) of the cooperative child build: lanes 0..26 the axis columns of child lane % 9
// (bc = lane / 9), lanes 27..63 centres (bc = 3) -- lanes 32 + i child i (the ballot lanes), lanes 27..31 child 8,
// the rest repeats. (Lanes 27..31 build child 8 so that traverse_ray can store child 8's centre from the low lane
// group: the centres are 16-B aligned, child i's x at bank 4 i mod 32, so child 8's and child 0's stores from one
// lane group of ds_write_b32 were a 2-way bank conflict on every table store of every expansion.)
__device__ __forceinline__ uint32_t build_child(uint32_t lane)
{
    return lane < 27u ? lane % 9u : lane < 32u ? 8u : (lane - 32u) % 9u;
}

// This lane's column of the cooperative child build (see build_child). Loaded once per wave, before any tile
// loop: a global load in every traversal would wait (vmcnt, in order on this ISA) for the previous tile's
// G-buffer stores.
__device__ __forceinline__ float4 build_column(const DeviceConsts* __restrict__ K)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t bi = build_child(lane);
    const uint32_t bc = lane < 27u ? lane / 9u : 3u;
    const float4 r = make_float4(K->child[bi][4u * bc + 0u], K->child[bi][4u * bc + 1u], K->child[bi][4u * bc + 2u],
                                 K->child[bi][4u * bc + 3u]);
    // retire the loads here (vmcnt(0)): otherwise the wait is placed at the first use inside the traversal,
    // where it would also wait for every tile's G-buffer stores
    __builtin_amdgcn_s_waitcnt(0x0f70);
    return r;
}

template <int PW, bool PIPE = false>
__device__ __forceinline__ void traverse(const DeviceConsts* __restrict__ K, const float* root, float* __restrict__ Lbase,
                                         const float4 bcol, uint32_t levels, float dx, float dy, float dz, bool valid, HitState& h,
                                         int32_t& maxd, uint32_t& status, uint32_t K_flags,
                                         uint64_t* phase_sums = nullptr, uint32_t axl = 36u,
                                         uint64_t* tile_counts = nullptr)
{
    constexpr bool PACKET = PW != 0;
    const uint32_t lane = threadIdx.x & 63u;
    const TraverseLds L{ Lbase };
    const bool cone_cull = (K_flags & SF_FLAG_NO_CONE_CULL) == 0u;
    const bool occl_cull = (K_flags & SF_FLAG_NO_OCCL_CULL) == 0u;
    // front-first child order (per-ray semantics, with the occlusion cull)
    const bool front_first = !PACKET && (K_flags & (SF_FLAG_NO_OCCL_CULL | SF_FLAG_NO_FRONT_FIRST)) == 0u;
    SF_STAMP_DECL;

    h.minT = FLT_MAX;
    h.cx = h.cy = h.cz = 0.f;
    h.index = 0xffffffffu;
    h.depth = -1;
    h.hit = false;   // set on return: hit <=> depth >= 0
    // Lanes whose current best sphere is an ancestor of the node being expanded (see the self test):
    // a wave lane mask, so the tie-break and its updates are scalar mask algebra.
    uint64_t ancm = 0ull;

    // ---- root node (depth 0): bounding sphere + LOD, centre straight from the kernel arguments
    const float rcx = root[9], rcy = root[10], rcz = root[11];
    const float rcc = (rcx * rcx + rcy * rcy) + rcz * rcz;
    bool ex0;
    {
        const float4 dt0 = depth_consts(K, 0u);
        const float tca = (rcx * dx + rcy * dy) + rcz * dz;
        const float d2 = rcc - tca * tca;
        const bool hb = valid && group_any<PW>(tca >= 0.0f) && group_any<PW>(d2 <= dt0.x);
        ex0 = hb && group_any<PW>(near_root(tca, d2, dt0.x) < dt0.w);
    }
    if (!wave_ballot(ex0)) return;
    maxd = 0;

    // ---- the wave's ray cone: axis = lane axl's direction (pixel (4, 4) of the tile), sinT bounds the
    // sine of every lane's angle to it (|d x a| with |d|, |a| = 1 +- 2^-20, plus 2^-16 slack). A wide
    // cone (scattered packets of the frame-less mode, or sinT >= 1/2) disables the child cone cull
    // below through cosT = 0, sinT = 1.
    // Kept in LDS (read with the node in expand): as uniform registers they would spill SGPRs.
    {
    // (half units: axl = the centre pixel of the traced half, (4, 2) or (4, 6))
    const float ax = readlane_f(dx, axl), ay = readlane_f(dy, axl), az = readlane_f(dz, axl);
    float cosT = 0.0f, sinT = 1.0f;
    if (cone_cull) {
        const float cx_ = dy * az - dz * ay, cy_ = dz * ax - dx * az, cz_ = dx * ay - dy * ax;
        const float s2 = (cx_ * cx_ + cy_ * cy_) + cz_ * cz_;
        const bool fwd = (dx * ax + dy * ay) + dz * az > 0.0f;
        const float s2m = fwd ? s2 : 1.0f;
        const float sm = __builtin_amdgcn_sqrtf(wave_max_pos(s2m)) * (1.0f + 0x1p-16f) + 0x1p-16f;
        if (sm < 0.5f) {
            sinT = sm;
            cosT = __builtin_amdgcn_sqrtf(1.0f - sm * sm) * (1.0f - 0x1p-16f);
        }
    }
    if (lane < 5u) L.cone()[lane] = lane == 0u ? ax : lane == 1u ? ay : lane == 2u ? az : lane == 3u ? cosT : sinT;
    }

    // This lane's column of the cooperative child build. The 27 axis columns (column c = lane / 9 of child
    // i = lane % 9) are built by lanes 0..26 of the first 32-lane LDS bank group, the 9 centres (column 3)
    // by lanes 32 + i of the second group. With the column planes skewed by 2 floats (SF_LDS_PLANE) no store of
    // the table build has two distinct addresses on one bank in a group; every other lane repeats a builder
    // (27..31: child 0's centre; 41..63: children (lane - 32) % 9 again) -- the same address and value, merged by
    // the LDS, not a conflict. (Round 2's layout -- centres on lanes 27..35, lanes 36..63 mirroring 0..27 -- put
    // 4.9 M extra cycles per 1080p frame into bank conflicts, 40 % of the LDS instruction cycles.) No divergent
    // region; the build's VALU cost is per wave either way. Lanes 32..40 hold the 9 child centres (read back by
    // v_readlane), and a ballot's per-child mask is bits 0..8 of its high word: one scalar AND (round 3 had the
    // centres on lanes 31..39, whose mask straddled the two words: a 64-bit shift and an AND per ballot).
    const uint32_t bi = build_child(lane);
    const uint32_t bc = lane < 27u ? lane / 9u : 3u;
    // The leaf-threshold skip bounds t from below for every ray. In packet semantics a lane with tca < 0
    // can also pass LOD through another lane's bounding hit (negative t, SIMD_AVX.h:254), which that
    // bound does not cover: there the skip additionally needs every sphere of the child's subtree in
    // front of every lane (leaf_front below).
    const bool lod_cull = (K_flags & SF_FLAG_NO_LOD_CULL) == 0u;
    // Every sphere of a node's subtree lies inside its bounding sphere (radius 2r around its centre c).
    // If c.d >= 2r for every lane's unit direction d, each such sphere (centre c', radius R') has
    // c'.d - R' >= c.d - 2r >= 0, so its near root t >= 0 for every lane: no negative t, and the
    // per-ray leaf threshold applies. Checked as tca >= 0 and tca^2 >= (2r)^2 (1 + 2^-6), the margin
    // covering the rounding of tca, |d| and the threshold.
    auto leaf_front = [&](const float4 pc, float R2b) -> bool {
        if constexpr (!PACKET) return true;
        const float tca = (pc.x * dx + pc.y * dy) + pc.z * dz;
        return wave_ballot(!(tca >= 0.0f && tca * tca >= R2b * (1.0f + 0x1p-6f))) == 0ull;
    };
    const float b[4] = { bcol.x, bcol.y, bcol.z, bcol.w };   // (build_column)
    // where this lane's column goes in a level table: centre lanes (bc = 3) xyz + cc at plane 0, the others
    // xyz in their column plane; the centre lanes' cc store goes to plane 0, the others' to one junk word of
    // the cone block (so both stores are unconditional: no divergent region; one address, no conflict)
    const uint32_t slot = bc == 3u ? bi * 4u : SF_LDS_PLANE + bc * SF_LDS_COLS + bi * 3u;

    uint32_t d = 0;                 // uniform: depth of the open (expanded) node
    uint32_t idxB = 1;              // uniform: 9 x its heap index + 1 mod 2^32 (root 0, child i of n: 9n+1+i),
                                    // i.e. the heap index of its child 0

    // ---- the own sphere of a node (Sphereflake.h:174-224) with centre/|c|^2 `pc`, depth dd, heap index
    // idx, tested when the node opens. The reference tests it after the children (post-order) and
    // accepts strictly smaller t, so on an exact tie the earlier node in post-order wins. Pre-order
    // differs from post-order only for ancestor/descendant pairs, hence: a tie is accepted iff the
    // current best is an ancestor of this node (`anc`). Same result as the reference's order in every case.
    // (actm / actv: the lanes for which the node is visited, as a wave mask (packet semantics) and as a
    // float, +inf on those lanes and -1 on the others (per-ray semantics: one v_min3 folds the visiting
    // lanes into the hit compare, so the hit mask needs no scalar AND)
    auto self_test = [&](const float4 pc, uint32_t dd, uint64_t actm, float actv, uint32_t idx, float R2s) {
        const float tca = (pc.x * dx + pc.y * dy) + pc.z * dz;
        const float d2 = pc.w - tca * tca;
        const bool f0 = tca >= 0.0f, in = d2 <= R2s;
        uint64_t hsm;
        if constexpr (PACKET) hsm = actm & wave_ballot(group_any<PW>(f0) && group_any<PW>(in));
        else hsm = wave_ballot(__builtin_fminf(__builtin_fminf(tca, R2s - d2), actv) >= 0.0f);   // f0 && in (child loop)
        if (hsm) {
#ifndef SF_NO_FAST_SQRT
            // (the general correctly rounded path only when a hitting lane's argument is tiny: a uniform branch)
            const float xs = R2s - d2;
            float ts;
            if ((wave_ballot(!(xs >= 0x1p-96f)) & hsm) != 0ull) ts = near_root_exact(tca, d2, R2s);
            else ts = near_root_big(tca, xs);
#else
            const float ts = near_root(tca, d2, R2s);
#endif
            const uint64_t eqm = wave_ballot(ts == h.minT);
            const uint64_t accm = hsm & (wave_ballot(ts < h.minT) | (eqm & ancm));
            // an exact tie with a best sphere that is not an ancestor: in index order that sphere came first in
            // the reference's post-order too (rejecting is right); with the front-first order it may not have,
            // so the caller re-traces the tile in index order (never seen on the BASELINE views)
            if (front_first && (hsm & eqm & ~ancm) != 0ull) status |= SF_STATUS_TIE;
            sel_in_place(h.minT, ts, accm);
            sel_in_place(h.cx, pc.x, accm);
            sel_in_place(h.cy, pc.y, accm);
            sel_in_place(h.cz, pc.z, accm);
            sel_in_place(h.index, idx, accm);
            uint32_t hd = (uint32_t)h.depth;
            sel_in_place(hd, dd, accm);
            h.depth = (int32_t)hd;
            ancm |= accm;
        }
    };

    // ---- expand the node with centre/|c|^2 `pc` (depth d, columns in LDS): build its 9 child transforms into
    // table(d), then test the children (depth d+1) for the lanes in `act`. Returns this lane's 9-bit
    // "child expands" vector; *pend = the wave's mask of children some lane expands.
    // (pc: the node's {centre, cc}, read by the caller; its columns j = 0..2 (xyz) at col + j * cs: col = node + 4,
    // cs = 4 for the root image; col = the table's column planes + 3 c, cs = SF_LDS_COLS for child c of a level)
    // (the node's own sphere is tested by the caller when the node is entered, before this)
    // (act: the lanes visiting the node, as a per-lane bool for the packet semantics and as the wave mask actm)
    auto expand = [&](const float4 pc, const float* col, uint32_t cs, uint32_t d, bool act, uint64_t actm,
                      float actv, uint32_t& pend, uint32_t& leafm) -> uint32_t {
        d = __builtin_amdgcn_readfirstlane(d);   // wave-uniform: depth constants come by scalar loads
        lds_fence();
        const float3 p0 = *reinterpret_cast<const float3*>(col);
        const float3 p1 = *reinterpret_cast<const float3*>(col + cs);
        const float3 p2 = *reinterpret_cast<const float3*>(col + 2u * cs);
        // the wave's ray cone, read with the node (before this level's stores: the junk cc store below goes
        // to the cone block, so a read after it would wait for a second LDS round trip)
        const float4 cn = *reinterpret_cast<const float4*>(L.cone());
        const float sinT = L.cone()[4];
        const float4 dtn = depth_consts(K, d);        // this node: (4/3) r
        const float4 dtc = depth_consts(K, d + 1u);   // children: (2r)^2, T
        // children's leaf threshold (+inf: no inline leaves when the LOD cull is off), loaded with the others
        const float leaf1 = depth_leaf(K, d + 1u);
        const float leafc = lod_cull ? leaf1 : __builtin_inff();
        // world = parent * child (SIMD_AVX.h:59-81), child translation scaled by (4/3) r (Sphereflake.h:162-172):
        // column 3 lanes multiply b0..b2 by s, the others by 1 (exact)
        const float sm = bc == 3u ? dtn.z : 1.0f;
        const float b0 = b[0] * sm, b1 = b[1] * sm, b2 = b[2] * sm;
        const float x = __builtin_fmaf(pc.x, b[3], (p0.x * b0 + p1.x * b1) + p2.x * b2);
        const float y = __builtin_fmaf(pc.y, b[3], (p0.y * b0 + p1.y * b1) + p2.y * b2);
        const float z = __builtin_fmaf(pc.z, b[3], (p0.z * b0 + p1.z * b1) + p2.z * b2);
        const float w = (x * x + y * y) + z * z;   // Dot(centre, centre) on the centre lanes (bc = 3)
        // table(levels-1) is never read: entering a child of the deepest provisioned level overflows
        // first. Not allocated, not stored (uniform branch).
        if (d + 1u < levels) {
            float* const tb = L.table(d);
            *reinterpret_cast<float3*>(tb + slot) = make_float3(x, y, z);
            *(bc == 3u ? tb + slot + 3u : L.cone() + 5u) = w;
        }
        const float R2b = dtc.x;
        const float T = dtc.w;
        const float Tfar = depth_far(K, d + 1u);
        // Cone cull of child bi (centre c in lanes 32..40): no ray of the wave's cone can hit its bounding
        // sphere. With ca = c.a, q = c - ca a, every lane's angle phi to c is >= alpha - theta, so its
        // line passes at distance |c| sin(phi) >= |q| cosT - ca sinT from c. A float hit
        // (tca >= 0, cc - tca^2 <= R^2, SIMD_AVX.h:247-258) needs |c| sin(phi) <= sqrt(R^2 + dl),
        // dl = 2^-18 |c|^2 covering the rounding of tca, d2, |c|^2 and |d| (~12 ulp + 2^-21); the last
        // terms cover this test's own rounding (hardware sqrt). With beta < 45 deg and theta < 30 deg
        // every lane's phi stays in [beta, 180 - beta], which also covers the 8-lane packet tests.
        // Such a child changes nothing for any lane in the reference: skip it for the whole wave.
        const float ax = cn.x, ay = cn.y, az = cn.z, cosT = cn.w;
        const float dl = w * 0x1p-18f;
        const float ca = (x * ax + y * ay) + z * az;
#ifndef SF_OLD_CONE
        // In squares, with |q| from |c|^2 - ca^2 (no q vector, one hardware sqrt): X = |q| cosT - ca sinT bounds
        // |c| sin(phi) from below; skip when X > 0 and X^2 > R^2 + dl + 2^-19 |c|^2. The added 32 u |c|^2 covers
        // this test's own rounding: |q|^2 = |c|^2 - ca^2 is off by <= 10 u |c|^2 (cancellation), which moves X^2 by
        // <= 2 X dq <= 10 u |c|^2; the sqrt, X and X^2 add <= 7 u |c|^2. (w - ca^2 clamped at 0: no NaN, which
        // the min below would drop.)
        const float sq = __builtin_amdgcn_sqrtf(__builtin_fmaxf(w - ca * ca, 0.0f));
        const float X = sq * cosT - ca * sinT;
        const float Y = X * X - (R2b + w * (0x1p-18f + 0x1p-19f));
        // skip = ca > 0 && w > 2 (R2b + dl) && X > 0 && Y > 0, as compares of a v_min3 and a v_min (with
        // denormals kept, a > b exactly when fl(a - b) > 0; every operand is finite): the kept children from a ballot
        const float mk = __builtin_fminf(__builtin_fminf(ca, w - 2.0f * (R2b + dl)), __builtin_fminf(X, Y));
#else
        const float qx = x - ca * ax, qy = y - ca * ay, qz = z - ca * az;
        const float sq = __builtin_amdgcn_sqrtf((qx * qx + qy * qy) + qz * qz);
        const float lhs = sq * cosT - ca * sinT;
        const float rhs = __builtin_amdgcn_sqrtf(R2b + dl) * (1.0f + 0x1p-18f) + (ca + sq) * 0x1p-18f;
        // skip = ca > 0 && w > 2 (R2b + dl) && lhs > rhs, as ONE compare of a v_min3 (with denormals kept,
        // a > b exactly when fl(a - b) > 0; every operand is finite): the kept children straight from a ballot
        const float mk = __builtin_fminf(__builtin_fminf(ca, w - 2.0f * (R2b + dl)), lhs - rhs);
#endif
        uint32_t M = (uint32_t)(wave_ballot(!(mk > 0.0f)) >> 32) & 0x1ffu;
        M = __builtin_amdgcn_readfirstlane(M);
        SF_STAMP(6);
        uint32_t e = 0, pm = 0;
        if constexpr (!PACKET) {
            // Per-ray semantics. "Any lane" tests are scalar ANDs of ballots of single compares
            // (each ballot is the compare's own lane mask: no bool materialisation); per-lane bools
            // are formed only where a lane's own bit is needed (its E bit).
            SF_COUNT(0, 1);
            SF_COUNT(7, __builtin_popcountll(actm));
            // child i's {centre, cc}: a broadcast LDS read of plane 0 of the table just stored (one LDS
            // instruction instead of four v_readlane on the VALU); the deepest provisioned level keeps no
            // table, there the centre lanes are read back
            // (the loop is instantiated twice, for the LDS and the readlane centres, so the choice is not
            // re-tested in every iteration)
            // actv (+inf on the lanes visiting the node, -1 on the others): ONE v_min3 + compare gives the
            // bounding mask already restricted to the visiting lanes, and the loop branches on it (VCC)
            // without scalar mask algebra
            // one child test: bounding + LOD of child i (centre c, |c|^2 cc) for every lane
            auto test_child = [&](uint32_t i, float cx, float cy, float cz, float cc) {
                SF_COUNT(1, 1);
                const float tca = (cx * dx + cy * dy) + cz * dz;
                const float d2 = cc - tca * tca;
                // bounding (SIMD_AVX.h:247-258): tca >= 0 && d2 <= R2b as ONE compare, min(tca, R2b - d2) >= 0:
                // with denormals kept, fl(R2b - d2) >= 0 exactly when d2 <= R2b (no NaN operands here)
                const float xs = R2b - d2;
                const bool hb = __builtin_fminf(__builtin_fminf(tca, xs), actv) >= 0.0f;
                const uint64_t hbm = wave_ballot(hb);
#ifdef SF_EXP_PAD   // experiment builds only: independent VALU filler per child iteration (issue-bound test)
                {
                    float pad = dx;
#pragma unroll
                    for (int k_ = 0; k_ < SF_EXP_PAD; ++k_) __asm__ volatile("v_mov_b32 %0, %0" : "+v"(pad));
                }
#endif
#ifdef SF_EXP_SPAD  // experiment builds only: SALU filler per child iteration (scalar-unit-bound test)
                {
                    uint32_t spad = i;
#pragma unroll
                    for (int k_ = 0; k_ < SF_EXP_SPAD; ++k_) __asm__ volatile("s_add_u32 %0, %0, 1" : "+s"(spad)::"scc");
                }
#endif
                SF_COUNT(5, __builtin_popcountll(actm));
                SF_COUNT(6, __builtin_popcountll(hbm));
                SF_COUNT(10, d >= 4u ? 1 : 0);
                SF_COUNT(11, d >= 4u ? __builtin_popcountll(actm) : 0);
                SF_COUNT(12, 0);
                SF_COUNT(13, 0);
                SF_COUNT(14, __builtin_popcountll(actm) <= 32 ? 1 : 0);
                if (hbm == 0ull) {
                    SF_COUNT(2, 1);
                    return;
                }
                // Most bounding hits are decided without the root: t = fl(tca - s) <= tca (s >= 0, rounding is
                // monotone), so tca < T expands. And on a bounding hit s <= 2r (1 + 2^-19) + 2^-9.7 tca (d2 can be
                // negative by rounding, down to -2^-19.4 |c|^2, |c|^2 <= tca^2 + R2b), so tca (1 - 2^-8) >= T + 2r
                // (1 + 2^-18) (`Tfar`, rounded up) means t >= T: no expansion. Only lanes in between take the
                // bracket below (rare: a band of width ~2r + 2^-8 tca around T).
                const uint64_t nearm = wave_ballot(tca < T);
                const uint64_t farm = wave_ballot(tca * (1.0f - 0x1p-8f) >= Tfar);
                if ((hbm & ~(nearm | farm)) == 0ull) {
                    const uint64_t exf = hbm & nearm;
                    sel_in_place(e, e | (1u << i), exf);
                    if (exf != 0ull) pm |= 1u << i;
                    SF_COUNT(3, exf != 0ull ? 1 : 0);
                    return;
                }
                // LOD on t = fl(tca - sqrt_rn(R2b - d2)) (SIMD_AVX.h:260-267; t0 <= t1 picks t1 for
                // thc >= 0). Fast bracket: the hardware sqrt is within 2 ulp of sqrt_rn and t is
                // monotone in it, so t_lo = fl(tca - (s + 2ulp)) <= t <= t_hi = fl(tca - (s - 2ulp)):
                // t_hi < T decides "expands", t_lo >= T decides "does not"; the exact path runs only
                // for lanes in between (or with a tiny sqrt argument).
                const float sq = __builtin_amdgcn_sqrtf(xs);
                const float s_lo = __uint_as_float((uint32_t)max((int32_t)__float_as_uint(sq) - 2, 0));
                const float s_hi = __uint_as_float(__float_as_uint(sq) + 2u);
                const float t_hi = tca - s_lo;
                const float t_lo = tca - s_hi;
                // The decision as per-lane values instead of scalar mask algebra: th / tl are t_hi / t_lo on
                // the lanes with a bounding hit and +inf elsewhere; a tiny sqrt argument makes the bracket
                // (-inf, +inf), i.e. undecided. expands: th < T; undecided: tl < T <= th.
                const uint64_t tinym = wave_ballot(xs < 0x1p-96f);
                // (the tiny select is opaque asm, so the hb select below stays one v_cndmask on the VCC of the
                // bounding compare instead of being merged into scalar mask algebra)
                const float thx = sel_mask(t_hi, __builtin_inff(), tinym);
                const float tlx = sel_mask(t_lo, -__builtin_inff(), tinym);
                const float th = hb ? thx : __builtin_inff();
                const float tl = hb ? tlx : __builtin_inff();
                uint64_t exm = wave_ballot(th < T);
                const uint64_t undm = wave_ballot(sel_mask(tl, __builtin_inff(), exm) < T);
                if (undm) {   // rare: exact IEEE root for the undecided lanes (disjoint from exm)
                    const float te = near_root_exact(tca, d2, R2b);
                    exm |= undm & wave_ballot(te < T);
                }
                sel_in_place(e, e | (1u << i), exm);   // the lanes of exm get bit i
                if (exm != 0ull) pm |= 1u << i;
                SF_COUNT(3, exm != 0ull ? 1 : 0);
            };
            auto child_loop = [&](auto tab) {
                const float* ctab = L.table(d);
                if constexpr (PIPE && decltype(tab)::value) {
                    // latency variant (small frames): software-pipelined two ways -- the next child's {centre,
                    // cc} is read into the other register set while this one is tested, so the LDS latency
                    // overlaps the test. Scalar loads are drained first so the waits count LDS reads only.
                    // Child 8 is read again past the last child: harmless.
                    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
                    if (M) {
                        uint32_t i = __builtin_ctz(M);
                        float4 ca = *reinterpret_cast<const float4*>(ctab + i * 4u), cb;
                        for (;;) {
                            uint32_t ci = i;
                            M &= ~(1u << ci);
                            i = __builtin_ctz(M | 0x100u);
                            cb = *reinterpret_cast<const float4*>(ctab + i * 4u);
                            test_child(ci, ca.x, ca.y, ca.z, ca.w);
                            if (!M) break;
                            ci = i;
                            M &= ~(1u << ci);
                            i = __builtin_ctz(M | 0x100u);
                            ca = *reinterpret_cast<const float4*>(ctab + i * 4u);
                            test_child(ci, cb.x, cb.y, cb.z, cb.w);
                            if (!M) break;
                        }
                    }
                }
                else
                while (M) {   // uniform loop over the children some lane can reach, in index order
                    const uint32_t i = __builtin_ctz(M);
                    M &= ~(1u << i);
                    float cx, cy, cz, cc;
                    if constexpr (decltype(tab)::value) {
                        const float4 c4 = *reinterpret_cast<const float4*>(ctab + i * 4u);
                        cx = c4.x, cy = c4.y, cz = c4.z, cc = c4.w;
                    } else {
                        cx = readlane_f(x, 32u + i), cy = readlane_f(y, 32u + i);
                        cz = readlane_f(z, 32u + i), cc = readlane_f(w, 32u + i);
                    }
                    test_child(i, cx, cy, cz, cc);
                }
                // children of a node at the deepest provisioned level (no table) would need a level that does
                // not exist: flag the tile for the deeper re-trace instead of entering them
                if constexpr (!decltype(tab)::value) {
                    if (pm != 0u) status |= SF_STATUS_OVERFLOW;
                    pm = 0u;
                }
            };
            if (d + 1u < levels) child_loop(BoolC<true>{});
            else child_loop(BoolC<false>{});
        } else {
            // Packet semantics (frame-less mode): early-outs over the 8 lanes of a reference packet.
            // (child centres from the LDS table by broadcast reads where the level has one, as in the per-ray
            // loop; the loop is instantiated for both sources)
            auto packet_loop = [&](auto tab) {
            const float* ctab = L.table(d);
            while (M) {
                const uint32_t i = __builtin_ctz(M);
                M &= M - 1u;
                float cx, cy, cz, cc;
                if constexpr (decltype(tab)::value) {
                    const float4 c4 = *reinterpret_cast<const float4*>(ctab + i * 4u);
                    cx = c4.x, cy = c4.y, cz = c4.z, cc = c4.w;
                } else {
                    cx = readlane_f(x, 32u + i), cy = readlane_f(y, 32u + i);
                    cz = readlane_f(z, 32u + i), cc = readlane_f(w, 32u + i);
                }
                const float tca = (cx * dx + cy * dy) + cz * dz;
                const float d2 = cc - tca * tca;
                const bool hb = act & group_any<PW>(tca >= 0.0f) & group_any<PW>(d2 <= R2b);
                if (wave_ballot(hb)) {
                    const float xs = R2b - d2;
                    const float sq = __builtin_amdgcn_sqrtf(xs);
                    const float s_lo = __uint_as_float((uint32_t)max((int32_t)__float_as_uint(sq) - 2, 0));
                    const float s_hi = __uint_as_float(__float_as_uint(sq) + 2u);
                    const float t_hi = tca - s_lo;           // >= t
                    const float t_lo = tca - s_hi;           // <= t
                    float t_dec = t_hi < T ? t_hi : t_lo;    // on the same side of T as t when decided
                    const bool undecided = hb & ((!(t_hi < T) & !(t_lo >= T)) | (xs < 0x1p-96f));
                    if (wave_ballot(undecided)) t_dec = undecided ? near_root_exact(tca, d2, R2b) : t_dec;
                    const bool exi = hb & group_any<PW>(t_dec < T);
                    const uint64_t mi = wave_ballot(exi);
                    e |= exi ? (1u << i) : 0u;
                    pm |= (mi != 0ull ? 1u : 0u) << i;
                }
            }
            };
            if (d + 1u < levels) packet_loop(BoolC<true>{});
            else packet_loop(BoolC<false>{});
            if (d + 1u >= levels) {   // (as in the per-ray loop without a table)
                if (pm != 0u) status |= SF_STATUS_OVERFLOW;
                pm = 0u;
            }
        }
        pend = pm;
        // children none of whose own children can pass LOD for any ray (sfhost::leaf_threshold of their depth;
        // |c|^2 of child i is w on lane 32 + i): entered as inline leaves
        leafm = (uint32_t)(wave_ballot(w > leafc) >> 32) & 0x1ffu;
        // front-first order (per-ray, occlusion cull on): bits 9..17 = the children whose centre lies nearer
        // than this node's along the cone axis; they are entered first, so their hits cull the far ones more
        if constexpr (!PACKET) {
            if (front_first) {
                const float kp = (pc.x * ax + pc.y * ay) + pc.z * az;
                leafm |= ((uint32_t)(wave_ballot(ca < kp) >> 32) & 0x1ffu) << 9;
            }
        }
        return e;
    };

    // DFS stack in VGPR lanes (lane L = level L): {pending children | leaf and front bits << 9}, heap index.
    // Lane selects: no LDS traffic and no lane-0-only region in the loop.
    uint32_t stk_pc = 0u, stk_ix = 0u;
    uint32_t pend = 0u, eN = 0u;
    uint32_t leafN = 0u;            // uniform: the open node's children that are inline leaves (bit i: child i),
                                    // its front children at bits 9..17 (see expand)
    {
        // the root: its own sphere, then -- unless no child of it can pass LOD for any ray
        // (sfhost::leaf_threshold; per-ray semantics only) -- its children
        lds_fence();
        const float4 pc = *reinterpret_cast<const float4*>(L.root());
        const float av0 = ex0 ? __builtin_inff() : -1.0f;
        self_test(pc, 0u, wave_ballot(ex0), av0, 0u, depth_consts(K, 0u).y);
        if (!(lod_cull && __builtin_amdgcn_readfirstlane((int)(pc.w > depth_leaf(K, 0u))) &&
              leaf_front(pc, depth_consts(K, 0u).x)))
            eN = expand(pc, L.root() + 4u, 4u, 0u, ex0, wave_ballot(ex0), av0, pend, leafN);
        else SF_COUNT(4, 1);
    }

    for (;;) {
        d = __builtin_amdgcn_readfirstlane(d);
        SF_STAMP(0);
        if (pend) {
            const uint32_t fp = pend & (leafN >> 9);   // front children still pending first
            const uint32_t c = __builtin_ctz(fp ? fp : pend);
            const uint32_t cbit = 1u << c;
            pend &= ~cbit;
            // (d + 1 < levels here: expand never leaves children pending at the deepest provisioned level)
            const bool a = (eN & cbit) != 0u;
            const uint64_t am = wave_ballot(a);
            const float av = a ? __builtin_inff() : -1.0f;
            const float* node = L.table(d) + c * 4u;
            // enter child c: its own sphere first (pre-order, see self_test), in one place for every child
            maxd = (int32_t)d + 1 > maxd ? (int32_t)d + 1 : maxd;   // Sphereflake.h:157-160
            // (the cull's scalar loads first, so that they are in flight with the LDS read below)
            const float cull_r = depth_cull(K, d + 1u);
            const float cull_t = depth_consts(K, (uint32_t)maxd + 1u).w;
            lds_fence();
            const float4 pc = *reinterpret_cast<const float4*>(node);
            const float4 dc1 = depth_consts(K, d + 1u);
            if constexpr (!PACKET) __asm__ volatile("" ::"s"(cull_r), "s"(cull_t));   // (issued here, not in the branch)
            // Occlusion cull (per-ray semantics): every sphere of the child's subtree, and every bounding sphere
            // the subtree's LOD tests use, lies in the child's bounding ball (radius R = 2r around c). A lane
            // whose float test of any of them accepts has t >= c.d - rho, rho = R + m (|c| + R), m =
            // SF_OCCL_MARGIN covering every rounding of those tests (tca, the d2 cancellation -- the dominant
            // 2^-9.2 (|c| + R) --, the centres' transform chain, |d| != 1). So where c.d - rho > minT the lane
            // can accept nothing in the subtree (ties included: strict), and where c.d - rho >= T of depth
            // maxd + 1 no node of the subtree can pass LOD deeper than the depth already reached (T falls with
            // depth): the max-depth statistic is unchanged. Such lanes do not enter; if none is left, the child
            // is skipped. (The child itself passed LOD for some lane: maxd above counts it either way.)
            uint64_t amx = am;
            float avx = av;
            if constexpr (!PACKET) {
                if (occl_cull) {
                    const float tca = (pc.x * dx + pc.y * dy) + pc.z * dz;
                    const float rho = cull_r + SF_OCCL_MARGIN * __builtin_amdgcn_sqrtf(pc.w);
                    const uint64_t cm = wave_ballot(__builtin_fminf(tca - h.minT, tca - cull_t) > rho);
                    amx = am & ~cm;
                    SF_COUNT(13, 1);
                    SF_COUNT(12, amx == 0ull ? 1 : 0);
                    if (amx == 0ull) continue;
                    avx = sel_mask(av, -1.0f, cm);
                }
            }
            self_test(pc, d + 1u, am, av, idxB + c, dc1.y);
            // A child none of whose children can pass LOD for any ray (sfhost::leaf_threshold) only needs its
            // own sphere: no push, no level, no child build. (leafN: decided for all 9 children when the parent
            // expanded)
            if ((leafN & cbit) != 0u && leaf_front(pc, dc1.x)) {
                SF_COUNT(4, 1);
                SF_COUNT(8, 1);
                SF_COUNT(9, __builtin_popcountll(am));
                ancm &= wave_ballot(h.depth != (int32_t)d + 1);   // the child is finished
                continue;
            }
            // save the open node's state, enter child c
            stk_pc = writelane_u(pend | (leafN << 9), d, stk_pc);
            stk_ix = writelane_u(idxB, d, stk_ix);
            L.E(d)[lane] = (uint16_t)eN;
            idxB = 9u * (idxB + c) + 1u;
            d += 1u;
            SF_STAMP(1);
            eN = expand(pc, L.table(d - 1u) + SF_LDS_PLANE + 3u * c, SF_LDS_COLS, d, a, amx, avx, pend, leafN);
            SF_STAMP(2);
            continue;
        }
        // ---- the node at depth d is finished: a best sphere at depth d is no longer an ancestor
        ancm &= wave_ballot(h.depth != (int32_t)d);
        SF_STAMP(4);
        if (d == 0u) break;
        // ---- back to the parent
        d -= 1u;
        lds_fence();
        {
            const uint32_t pc = __builtin_amdgcn_readlane(stk_pc, d);
            pend = pc & 0x1ffu;
            leafN = pc >> 9;
            idxB = (uint32_t)__builtin_amdgcn_readlane(stk_ix, d);
        }
        eN = L.E(d)[lane];
        (void)__builtin_amdgcn_readfirstlane(eN);   // (stamp builds: close the pop segment after its reads)
        SF_STAMP(5);
    }
    h.hit = h.depth >= 0;
    SF_STAMP_FLUSH(phase_sums);
#ifdef SF_COUNTS
    // per tile (COUNTS=1 builds): expanded nodes | child iterations << 16 | bounding-hit iterations << 32 |
    // inline leaf tests << 48 (16 bits each, saturating)
    if (tile_counts) {
        auto sat = [](uint64_t v) { return v > 0xffffull ? 0xffffull : v; };
        *tile_counts = sat(ph_sum[0]) | (sat(ph_sum[1]) << 16) | (sat(ph_sum[1] - ph_sum[2]) << 32) | (sat(ph_sum[8]) << 48);
    }
#else
    (void)tile_counts;
#endif
}

// ------------------------------------------------------------------------------------------
// Per-ray semantics (full frames), round 3: a child is entered as soon as its own test passes. The reference
// itself recurses into child i before testing child i + 1 (Sphereflake.h:162-172); `traverse` above tests all
// children of a node first, keeps each lane's 9 "expands" bits in LDS and enters the pending children after.
// Per-ray, the tests of child i + 1 do not depend on anything child i's subtree does (bounding and LOD involve
// only the ray and the child; acceptance is the self test's, at entry), so entering at once gives the same
// visits, and the child test's values carry into the entry: its centre and |c|^2 (no second LDS read), tca and
// d2 (the self test's own, not recomputed), the expanding lanes (no per-lane E bits in LDS: no store at the
// push, no load at the pop). A node keeps on the VGPR stack its untested children (the cone-culled mask,
// front children first, as before) instead of its pending ones, and its visiting lanes as one bit per level
// (`actbits`).
// Entry-order mask (bits c and 16 + c, see traverse_ray) of the children c of a node whose child 0 has heap index
// idxB that belong to subtree part q: (idxB + c) mod 4 == q.
__device__ __forceinline__ uint32_t split_mask(uint32_t q, uint32_t idxB)
{
    const uint32_t m9 = (0x111u << ((q - idxB) & 3u)) & 0x1ffu;
    return m9 | (m9 << 16);
}

// SPLIT: a subtree part unit (SF_FLAG_SUBTREE): of the nodes at depth split_depth, only those whose heap index is
// split_q mod 4 are entered (their own sphere and their subtree); everything above is traced as for the whole tile.
template <bool PIPE = false, bool COMPACT = false, bool SPLIT = false>
__device__ __forceinline__ void traverse_ray(const DeviceConsts* __restrict__ K, const float* root, float* __restrict__ Lbase,
                                             const float4 bcol, uint32_t levels, float dx, float dy, float dz, bool valid,
                                             HitState& h, int32_t& maxd, uint32_t& status, uint32_t K_flags,
                                             uint64_t* phase_sums = nullptr, uint32_t axl = 36u,
                                             uint64_t* tile_counts = nullptr, uint32_t split_q = 0u,
                                             uint32_t split_depth = 0u)
{
    const uint32_t lane = threadIdx.x & 63u;
    const TraverseLds L{ Lbase };
    const bool cone_cull = (K_flags & SF_FLAG_NO_CONE_CULL) == 0u;
    const bool occl_cull = (K_flags & SF_FLAG_NO_OCCL_CULL) == 0u;
    const bool front_first = (K_flags & (SF_FLAG_NO_OCCL_CULL | SF_FLAG_NO_FRONT_FIRST)) == 0u;
    SF_STAMP_DECL;

    h.minT = FLT_MAX;
    h.cx = h.cy = h.cz = 0.f;
    h.index = 0xffffffffu;
    h.depth = -1;
    h.hit = false;
    uint64_t ancm = 0ull;   // lanes whose current best sphere is an ancestor of the open node (see self_test)

    // ---- root node (depth 0): bounding sphere + LOD
    const float rcx = root[9], rcy = root[10], rcz = root[11];
    const float rcc = (rcx * rcx + rcy * rcy) + rcz * rcz;
    bool ex0;
    {
        const float4 dt0 = depth_consts(K, 0u);
        const float tca = (rcx * dx + rcy * dy) + rcz * dz;
        const float d2 = rcc - tca * tca;
        const bool hb = valid && tca >= 0.0f && d2 <= dt0.x;
        ex0 = hb && near_root(tca, d2, dt0.x) < dt0.w;
    }
    if (!wave_ballot(ex0)) return;
    maxd = 0;
    float cull_t = depth_consts(K, 1u).w;   // uniform: depth maxd + 1's LOD threshold, reloaded when maxd grows

    // ---- the wave's ray cone (as in traverse)
    {
        const float ax = readlane_f(dx, axl), ay = readlane_f(dy, axl), az = readlane_f(dz, axl);
        float cosT = 0.0f, sinT = 1.0f;
        if (cone_cull) {
            const float cx_ = dy * az - dz * ay, cy_ = dz * ax - dx * az, cz_ = dx * ay - dy * ax;
            const float s2 = (cx_ * cx_ + cy_ * cy_) + cz_ * cz_;
            const bool fwd = (dx * ax + dy * ay) + dz * az > 0.0f;
            const float s2m = fwd ? s2 : 1.0f;
            const float sm = __builtin_amdgcn_sqrtf(wave_max_pos(s2m)) * (1.0f + 0x1p-16f) + 0x1p-16f;
            if (sm < 0.5f) {
                sinT = sm;
                cosT = __builtin_amdgcn_sqrtf(1.0f - sm * sm) * (1.0f - 0x1p-16f);
            }
        }
        if (lane < 5u) L.cone()[lane] = lane == 0u ? ax : lane == 1u ? ay : lane == 2u ? az : lane == 3u ? cosT : sinT;
    }

    // this lane's column of the cooperative child build (see traverse)
    const uint32_t bi = build_child(lane);
    const uint32_t bc = lane < 27u ? lane / 9u : 3u;
    const float b[4] = { bcol.x, bcol.y, bcol.z, bcol.w };
    // child 8's centre is stored by lanes 27..31; the high group's child-8 lanes store into the level's E words,
    // which this traversal does not use, at a float offset of 2 mod 4 (the levels are 32-B aligned): store k then
    // hits bank 2 + k mod 4, no centre store's 4 i + k
    const uint32_t slot = bc == 3u ? (lane >= 32u && bi == 8u ? (uint32_t)SF_LDS_TABLE + 3u : bi * 4u)
                                   : SF_LDS_PLANE + bc * SF_LDS_COLS + bi * 3u;

    uint32_t d = 0;      // uniform: depth of the open node
    uint32_t idxB = 1;   // uniform: the heap index of the open node's child 0 (9 n + 1)

    // ---- the own sphere of a node entered for the lanes of actv (+inf on them, -1 elsewhere), with its tca and
    // d2 already formed by its child test (the same operations: Sphereflake.h:174-224, SIMD_AVX.h:236-270).
    // Pre-order with the ancestor tie rule (see traverse's self_test).
    auto self_test = [&](const float4 pc, float tca, float d2, uint32_t dd, float actv, uint32_t idx, float R2s) {
        const uint64_t hsm = wave_ballot(__builtin_fminf(__builtin_fminf(tca, R2s - d2), actv) >= 0.0f);
        if (hsm) {
            const float xs = R2s - d2;
            float ts;
            if ((wave_ballot(!(xs >= 0x1p-96f)) & hsm) != 0ull) ts = near_root_exact(tca, d2, R2s);
            else ts = near_root_big(tca, xs);
            // strictly nearer lanes accept; exact ties (rare) take a branch of their own: a tie is accepted where
            // the best is an ancestor, and one with a non-ancestor flags the tile (front-first order, see traverse)
            uint64_t accm = hsm & wave_ballot(ts < h.minT);
            const uint64_t tie = hsm & wave_ballot(ts == h.minT);
            if (tie != 0ull) {
                accm |= tie & ancm;
                if (front_first && (tie & ~ancm) != 0ull) status |= SF_STATUS_TIE;
            }
            sel_in_place(h.minT, ts, accm);
            sel_in_place(h.cx, pc.x, accm);
            sel_in_place(h.cy, pc.y, accm);
            sel_in_place(h.cz, pc.z, accm);
            sel_in_place(h.index, idx, accm);
            uint32_t hd = (uint32_t)h.depth;
            sel_in_place(hd, dd, accm);
            h.depth = (int32_t)hd;
            ancm |= accm;
        }
    };

    // ---- LOD of one child whose bounding sphere the lanes of hbm hit (xs = R2b - d2, depth constants R2b, T, Tfar):
    // the lanes that expand it (see traverse's test_child for the fast decisions and the certified bracket)
    auto child_lod = [&](float tca, float d2, float xs, bool hb, uint64_t hbm, float R2b, float T, float Tfar) -> uint64_t {
        const uint64_t nearm = wave_ballot(tca < T);
        const uint64_t farm = wave_ballot(tca * (1.0f - 0x1p-8f) >= Tfar);
        if ((hbm & ~(nearm | farm)) == 0ull) return hbm & nearm;
        const float sq = __builtin_amdgcn_sqrtf(xs);
        const float s_lo = __uint_as_float((uint32_t)max((int32_t)__float_as_uint(sq) - 2, 0));
        const float s_hi = __uint_as_float(__float_as_uint(sq) + 2u);
        const float t_hi = tca - s_lo;
        const float t_lo = tca - s_hi;
        const uint64_t tinym = wave_ballot(xs < 0x1p-96f);
        const float thx = sel_mask(t_hi, __builtin_inff(), tinym);
        const float tlx = sel_mask(t_lo, -__builtin_inff(), tinym);
        const float th = hb ? thx : __builtin_inff();
        const float tl = hb ? tlx : __builtin_inff();
        uint64_t exm = wave_ballot(th < T);
        const uint64_t undm = wave_ballot(sel_mask(tl, __builtin_inff(), exm) < T);
        if (undm) {
            const float te = near_root_exact(tca, d2, R2b);
            exm |= undm & wave_ballot(te < T);
        }
        return exm;
    };

    // ---- expand the node with centre/|c|^2 pc at depth d (axis columns at col + j cs): build its 9 child
    // transforms into table(d) and cull the children no ray of the tile's cone can reach. Returns the children
    // left to test, in entry order (front child i at bit i, the others at 16 + i). At the deepest provisioned level
    // (no table for the children's children) the children are tested here, from the centre lanes: any that some
    // lane expands flags the tile for the deeper re-trace, and none is entered.
    const uint32_t lv32 = __builtin_amdgcn_readfirstlane(levels << 5);   // levels, in depth-constant offset units
    const uint32_t index_order = front_first ? 0u : 0x1ffu;
    // (tb: table(d), ko: d + 1's constants offset -- the caller's carried values, not formed here again)
    auto expand = [&](const float4 pc, const float* col, uint32_t cs, uint32_t d, float actv,
                      float* tb, uint32_t ko, float kp) -> uint32_t {
        d = __builtin_amdgcn_readfirstlane(d);
        SF_COUNT(0, 1);
        SF_COUNT(7, __builtin_popcountll(wave_ballot(actv >= 0.0f)));   // (COUNTS builds: lanes visiting the node)
        lds_fence();
        const float3 p0 = *reinterpret_cast<const float3*>(col);
        const float3 p1 = *reinterpret_cast<const float3*>(col + cs);
        const float3 p2 = *reinterpret_cast<const float3*>(col + 2u * cs);
        const float4 cn = *reinterpret_cast<const float4*>(L.cone());
        const float sinT = L.cone()[4];
        const float4 dtn = depth_consts_at(K, ko - (1u << 5));
        const float4 dtc = depth_consts_at(K, ko);
        const float sm = bc == 3u ? dtn.z : 1.0f;
        const float b0 = b[0] * sm, b1 = b[1] * sm, b2 = b[2] * sm;
        const float x = __builtin_fmaf(pc.x, b[3], (p0.x * b0 + p1.x * b1) + p2.x * b2);
        const float y = __builtin_fmaf(pc.y, b[3], (p0.y * b0 + p1.y * b1) + p2.y * b2);
        const float z = __builtin_fmaf(pc.z, b[3], (p0.z * b0 + p1.z * b1) + p2.z * b2);
        const float w = (x * x + y * y) + z * z;
        const float R2b = dtc.x;
        // cone cull of child bi (centre lanes 32..40), in squares (see traverse). The test is this kernel's own
        // arithmetic, not the reference's, so it fuses: ca, |c|^2 - ca^2, X and Y by fma -- each fused step rounds
        // once where the unfused one rounded twice, so the error bounds behind the slack (traverse) still hold --
        // and the regime condition |c|^2 > 2 (R^2 + 2^-18 |c|^2) as w (1 - 2^-16) > 2 R^2, a slightly stronger
        // one. 15 VALU instead of 23 per expansion. (w itself stays the reference's |c|^2: it is the table's cc.)
        const float ax = cn.x, ay = cn.y, az = cn.z, cosT = cn.w;
        const float ca = __builtin_fmaf(x, ax, __builtin_fmaf(y, ay, z * az));
        const float sq = __builtin_amdgcn_sqrtf(__builtin_fmaxf(__builtin_fmaf(-ca, ca, w), 0.0f));
        const float X = __builtin_fmaf(sq, cosT, -(ca * sinT));
        const float Y = __builtin_fmaf(X, X, -(R2b + w * (0x1p-18f + 0x1p-19f)));
        const float reg = __builtin_fmaf(w, 1.0f - 0x1p-16f, -2.0f * R2b);
        const float mk = __builtin_fminf(__builtin_fminf(ca, reg), __builtin_fminf(X, Y));
        uint32_t M = (uint32_t)(wave_ballot(!(mk > 0.0f)) >> 32) & 0x1ffu;
        M = __builtin_amdgcn_readfirstlane(M);
        // entry order as bit order: the front children (nearer than this node's centre along the cone axis) at
        // bits 0..8, the others at 16..24 -- one find-first-set per child picks the next, and its low 4 bits are
        // the child's number
        // (index order, front_first false: every child "front" -- an OR with a per-traversal mask, not a branch)
        // (kp = (pc.x ax + pc.y ay) + pc.z az, the node's own projection: the caller passes the axis lane's tca of the
        // node, the same operations on the same operands -- the cone axis IS that lane's direction)
        const uint32_t front = ((uint32_t)(wave_ballot(ca < kp) >> 32) & 0x1ffu) | index_order;
        // (one levels test for both outcomes: stored after the cull, the table is read only once this returns)
        if (ko < lv32) {   // (d + 1 < levels)
            *reinterpret_cast<float3*>(tb + slot) = make_float3(x, y, z);
            *(bc == 3u ? tb + slot + 3u : L.cone() + 5u) = w;
            return (M & front) | ((M & ~front) << 16);
        }
        {   // (d + 1 >= levels)
            const float T = dtc.w, Tfar = depth_word_at(K, ko, 6u);   // depth_far(K, d + 1)
            while (M) {
                const uint32_t i = __builtin_ctz(M);
                M &= ~(1u << i);
                const float cx = readlane_f(x, 32u + i), cy = readlane_f(y, 32u + i);
                const float cz = readlane_f(z, 32u + i), cc = readlane_f(w, 32u + i);
                const float tca = (cx * dx + cy * dy) + cz * dz;
                const float d2 = cc - tca * tca;
                const float xs = R2b - d2;
                const bool hb = __builtin_fminf(__builtin_fminf(tca, xs), actv) >= 0.0f;
                const uint64_t hbm = wave_ballot(hb);
                if (hbm != 0ull && child_lod(tca, d2, xs, hb, hbm, R2b, T, Tfar) != 0ull) {
                    status |= SF_STATUS_OVERFLOW;
                    break;
                }
            }
            return 0u;
        }
    };

    uint32_t stk_pc = 0u, stk_ix = 0u;   // VGPR stack, lane k = level k: untested children, idxB
    float* tcur = L.table(0u);           // uniform: L.table(d), moved at push / pop (not formed per child)
    uint32_t kofs = 1u << 5;             // uniform: byte offset of depth d + 1's constants, moved likewise
    float R2c = depth_consts_at(K, kofs).x;   // uniform: depth d + 1's bounding radius^2, reloaded likewise
    uint32_t C = 0u;                     // uniform: the open node's untested children in entry order (child i at bit
                                         // i if it is a front child, else at bit 16 + i)
    float actv;                          // per lane: +inf if the lane visits the open node, -1 otherwise
    uint32_t actbits;                    // per lane: bit k set if the lane visits the open node's level-k ancestor
    {
        lds_fence();
        const float4 pc = *reinterpret_cast<const float4*>(L.root());
        actv = ex0 ? __builtin_inff() : -1.0f;
        actbits = ex0 ? 1u : 0u;
        const float tca = (pc.x * dx + pc.y * dy) + pc.z * dz;
        const float d2 = pc.w - tca * tca;
        self_test(pc, tca, d2, 0u, actv, 0u, depth_consts(K, 0u).y);
        if (!__builtin_amdgcn_readfirstlane((int)(pc.w > depth_leaf(K, 0u))))
            C = expand(pc, L.root() + 4u, 4u, 0u, actv, tcur, kofs, readlane_f(tca, axl));
        else SF_COUNT(4, 1);
        if constexpr (SPLIT) {
            if (split_depth == 1u) C &= split_mask(split_q, 1u);
        }
    }

    // (the scalar unit is shared by the CU's four SIMDs and measured ~3x a VALU op per instruction here: the child
    // loop keeps its scalar bookkeeping to a find-first-set, a clear-lowest and the index)
    for (;;) {
        d = __builtin_amdgcn_readfirstlane(d);
        SF_STAMP(0);
        if (C) {
            const uint32_t p = __builtin_ctz(C);
            __asm__("s_bitset0_b32 %0, %1" : "+s"(C) : "s"(p));   // (one scalar op; C &= C - 1 is two)
            const uint32_t c = p & 15u;   // (front child p, or child p - 16)
            // the children's depth constants (scalar loads, in flight with the centre's LDS read)
            const float4 dc = depth_consts_at(K, kofs);
            lds_fence();
            const float4 pc = *reinterpret_cast<const float4*>(tcur + c * 4u);
            const float tca = (pc.x * dx + pc.y * dy) + pc.z * dz;
            const float d2 = pc.w - tca * tca;
            // bounding (SIMD_AVX.h:247-258) for the visiting lanes: one v_min3 compare, its VCC the branch
            const float xs = R2c - d2;
            const bool hb = __builtin_fminf(__builtin_fminf(tca, xs), actv) >= 0.0f;
            const uint64_t hbm = wave_ballot(hb);
            SF_COUNT(1, 1);
#ifdef SF_COUNTS
            {   // lane utilisation of the child loop (COUNTS builds only)
                const uint32_t na = __builtin_popcountll(wave_ballot(actv >= 0.0f));
                SF_COUNT(5, na);
                SF_COUNT(6, __builtin_popcountll(hbm));
                SF_COUNT(10, d >= 4u ? 1 : 0);
                SF_COUNT(11, d >= 4u ? na : 0);
                SF_COUNT(14, na <= 32u ? 1 : 0);
            }
#endif
            if (hbm == 0ull) {
                SF_COUNT(2, 1);
                continue;
            }
            // depth d + 1's {leaf, cull, far} words: one scalar load
            const float4 dk = depth_consts_at(K, kofs + 16u);
            const float Tfar = dk.z;     // depth_far(K, d + 1)
            const float cull_r = dk.y;   // depth_cull(K, d + 1)
            const uint64_t exm = child_lod(tca, d2, xs, hb, hbm, dc.x, dc.w, Tfar);
            SF_STAMP(2);
            if (exm == 0ull) continue;
            // ---- child c passed bounding + LOD for the lanes of exm: enter it
            SF_COUNT(3, 1);
            if ((int32_t)d + 1 > maxd) {   // Sphereflake.h:157-160
                maxd = (int32_t)d + 1;
                cull_t = depth_consts_at(K, kofs + (1u << 5)).w;
            }
            // occlusion cull (see traverse): lanes for which no sphere of the child's subtree can be accepted or
            // pass LOD deeper than the depth already reached do not enter
            // The fattened radius rho = R (1 + m) + m |c| (see traverse) without |c|: a lane of exm hit the bounding
            // sphere, so |c|^2 = d2 + tca^2 <= R^2 + tca^2 (+ the float test's slack, 2^-9.6 |c|) and
            // |c| <= tca + R (+ 2^-9.6 |c|, whose m multiple is far inside m's safety factor): rho <= R (1 + 2 m) +
            // m tca = cull_r + m tca per lane, no square root.
            uint64_t amx = exm;
            if (occl_cull) {
                const float v = __builtin_fminf(tca - h.minT, tca - cull_t);
                const uint64_t cm = wave_ballot(v - SF_OCCL_MARGIN * tca > cull_r);
                amx = exm & ~cm;
                SF_COUNT(13, 1);
                SF_COUNT(12, amx == 0ull ? 1 : 0);
                if (amx == 0ull) continue;
            }
            const float avx = sel_mask(-1.0f, __builtin_inff(), amx);
            self_test(pc, tca, d2, d + 1u, avx, idxB + c, dc.y);
            SF_STAMP(4);
            // an inline leaf -- its own sphere only (sfhost::leaf_threshold): |c|^2 beyond depth d + 1's leaf
            // threshold; the centre's w is broadcast, so one compare is the branch (round 5: no per-level leaf mask
            // formed at the expansion and carried through the stack)
            // (the leaf skip is always on in this traversal: SF_FLAG_NO_LOD_CULL is the packet traversal's A/B switch)
            if (wave_ballot(pc.w > dk.x) != 0ull) {
                SF_COUNT(4, 1);
                SF_COUNT(8, 1);
                SF_COUNT(9, __builtin_popcountll(amx));
                ancm &= wave_ballot(h.depth != (int32_t)d + 1);   // the child is finished
                continue;
            }
            // push the open node, open child c
            stk_pc = writelane_s(C, d, stk_pc);
            stk_ix = writelane_s(idxB, d, stk_ix);
            {
                const uint32_t bit = 2u << d;   // level d + 1
                uint32_t ab = actbits & ~bit;
                sel_in_place(ab, ab | bit, amx);
                actbits = ab;
            }
            idxB = 9u * (idxB + c) + 1u;
            d += 1u;
            actv = avx;
            SF_STAMP(1);
            const float* const col = tcur + SF_LDS_PLANE + 3u * c;   // the entered child's axis columns
            tcur += SF_LDS_LEVEL;
            kofs += 1u << 5;
            C = expand(pc, col, SF_LDS_COLS, d, avx, tcur, kofs, readlane_f(tca, axl));
            if constexpr (SPLIT) {   // (the children are at depth d + 1)
                if (d + 1u == split_depth) C &= split_mask(split_q, idxB);
            }
            R2c = depth_consts_at(K, kofs).x;
            if (COMPACT && C != 0u) {
                // ---- Active-ray compaction of sparse nodes (north star: "wavefront ballot / prefix-sum active-ray
                // compaction down the recursion"; sf_trace_queue2c, opt-in). Deep in the tree a node is often visited
                // by a handful of the tile's rays, and each of its children then costs a wave-wide test for those few
                // lanes. Where at most 7 lanes visit the node and 3 or more children are left, the visiting rays are
                // packed by their prefix-sum rank (mbcnt of the ballot) into 7 LDS slots, replicated into 9 groups of 7
                // lanes, and group g tests child g: every child's bounding test in ONE wave pass, the same float
                // operations on bit-identical directions. Children no visiting ray hits leave the mask; the loop then
                // tests the others per lane as before. A filter: no decision changes (results bit for bit).
                __builtin_amdgcn_sched_barrier(0);   // (not interleaved with the expansion: register pressure)
                const uint64_t actm = wave_ballot(avx > 0.0f);
                const uint32_t na = (uint32_t)__builtin_popcountll(actm);
                const uint32_t M = (C | (C >> 16)) & 0x1ffu;   // the untested children by index
                if (na <= 7u && __builtin_popcount(M) >= 3) {
                    const float R2b = depth_consts(K, d + 1u).x;
                    // pack through the level's E words (unused by this traversal): visiting lane of rank k writes its
                    // direction to slot k (16 B), the others to a junk slot; every lane reads the slot of its group
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(actm >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)actm, 0u));
                    float* const sc = reinterpret_cast<float*>(L.E(d)) + 1;   // (16-byte aligned; 32 floats)
                    *reinterpret_cast<float4*>(sc + (avx > 0.0f ? 4u * rank : 28u)) = make_float4(dx, dy, dz, 0.0f);
                    lds_fence();
                    uint32_t ln = lane;
                    __asm__ volatile("" : "+v"(ln));   // (formed here, not hoisted and kept live across the DFS)
                    const uint32_t g = (ln * 37u) >> 8;   // lane / 7 (exact for lanes 0..63)
                    const uint32_t sl = ln - 7u * g;      // lane % 7
                    const float4 q = *reinterpret_cast<const float4*>(sc + 4u * sl);
                    const bool ok = sl < na && g < 9u && ((M >> g) & 1u) != 0u;
                    const uint32_t gi = g < 9u ? g : 8u;
                    const float4 cg = *reinterpret_cast<const float4*>(L.table(d) + gi * 4u);   // child g
                    const float tca = (cg.x * q.x + cg.y * q.y) + cg.z * q.z;
                    const float d2 = cg.w - tca * tca;
                    const float xs = R2b - d2;
                    const uint64_t bal =
                        wave_ballot(__builtin_fminf(__builtin_fminf(tca, xs), ok ? __builtin_inff() : -1.0f) >= 0.0f);
                    // child k is hit by some visiting ray iff bits 7k..7k+6 of the ballot are not all zero (lane k asks)
                    const uint32_t kk = ln < 9u ? ln : 0u;
                    const uint64_t grp = (bal >> (7u * kk)) & 0x7full;
                    const uint32_t hitm = (uint32_t)wave_ballot(ln < 9u && grp != 0ull) & 0x1ffu;
                    const uint32_t keep = __builtin_amdgcn_readfirstlane(hitm);
                    C &= keep | (keep << 16);
                }
            }
            SF_STAMP(6);
            continue;
        }
        // ---- the node at depth d is finished: a best sphere at depth d is no longer an ancestor
        ancm &= wave_ballot(h.depth != (int32_t)d);
        if (d == 0u) break;
        d -= 1u;
        tcur -= SF_LDS_LEVEL;
        kofs -= 1u << 5;
        R2c = depth_consts_at(K, kofs).x;
        {
            const uint32_t pw = __builtin_amdgcn_readlane(stk_pc, d);
            C = pw;
            idxB = (uint32_t)__builtin_amdgcn_readlane(stk_ix, d);
        }
        actv = ((actbits >> d) & 1u) ? __builtin_inff() : -1.0f;
        SF_STAMP(5);
    }
    h.hit = h.depth >= 0;
    SF_STAMP_FLUSH(phase_sums);
#ifdef SF_COUNTS
    if (tile_counts) {
        auto sat = [](uint64_t v) { return v > 0xffffull ? 0xffffull : v; };
        *tile_counts = sat(ph_sum[0]) | (sat(ph_sum[1]) << 16) | (sat(ph_sum[1] - ph_sum[2]) << 32) | (sat(ph_sum[8]) << 48);
    }
#else
    (void)tile_counts;
#endif
}

struct Tile {
    uint32_t x, y, orow;
    bool valid;
};

// Tile of a wave: owned tile row k (band sharding) -> frame tile row.
__device__ __forceinline__ Tile tile_of(const FrameArgs& a, uint32_t tile, uint32_t lane, uint32_t part = 0u)
{
    // tile -> (k, tx) and k -> (band, row in band) by multiply-high with host magic numbers and one correction
    // (m = floor((2^32 - 1) / D) underestimates n / D by less than 1 for n < 2^31: q or q + 1), scalar
    auto divmod = [](uint32_t n, uint32_t D, uint32_t m, uint32_t& r) {
        uint32_t q = __umulhi(n, m);
        r = n - q * D;
        if (r >= D) {
            q += 1u;
            r -= D;
        }
        return q;
    };
    uint32_t tx, kr;
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) DeviceConsts* ConstK;
    const uint32_t txm = ((ConstK)(const void*)a.consts)->tx_magic;
#else
    const uint32_t txm = a.consts->tx_magic;
#endif
    const uint32_t k = divmod(tile, a.tiles_x, txm, tx);
    const uint32_t kb = divmod(k, a.tiles_per_band, a.tpb_magic, kr);
    const uint32_t band = a.band_index + kb * a.band_count;
    const uint32_t ty = band * a.tiles_per_band + kr;
    // (opaque copy: recompute the lane's column/row per tile rather than keep them live, or spilled,
    // across a persistent loop)
    uint32_t l = lane;
    __asm__ volatile("" : "+v"(l));
    Tile t;
    t.x = tx * SF_TILE + (l & 7u);
    t.y = ty * SF_TILE + (l >> 3);
    // part unit: only the lanes of pixel rows 0-3 / 4-7 (halves) or of one 4x4 block (quarters) take part
    const uint32_t q = part - SF_PART_QUARTER0;
    const bool in = part == 0u || (part < SF_PART_QUARTER0 ? (l >> 5) + SF_PART_HALF0 == part
                                                           : ((l >> 5) == (q >> 1) && ((l >> 2) & 1u) == (q & 1u)));
    t.valid = t.x < a.W && t.y < a.H && in;
    t.orow = a.compact ? (k * SF_TILE + (l >> 3)) : t.y;
    return t;
}

// G-buffer write (Sphereflake.cpp:186-196): (pos, 1), (nrm, 1); a miss writes (0,0,0,1).
// Packed slabs (multi-GPU bands, a.packed): one float4 (nx, ny, nz, minT) -- the position is dir * minT, which
// the receiving side recomputes bit for bit (sf_unpack_bands), so a band ships 16 B per pixel instead of 32.
__device__ __forceinline__ void write_pixel(const FrameArgs& a, const Tile& t, float dx, float dy, float dz,
                                            const HitState& h, const uint32_t* __restrict__ lut)
{
    float px, py, pz, nx, ny, nz;
    shade(dx, dy, dz, h, lut, px, py, pz, nx, ny, nz);
    const size_t o = (size_t)t.orow * a.W + t.x;
    if (a.packed) {   // (uniform)
        if (a.packed >= SF_PACKED_INDEX) {
            // 4 B: the hit's heap index; the receiver rebuilds the rest. (The host selects this format only where
            // no hit can lie deeper than SF_INDEX_SLAB_DEPTH, whose heap indices are below 2^32; a deeper one would
            // be ambiguous and is written as SF_SLAB_BAD instead.)
            const int32_t lim = a.packed == SF_PACKED_INDEX ? SF_INDEX_SLAB_DEPTH : SF_DIAG_SLAB_DEPTH;   // (tests)
            const bool bad = h.hit && h.depth > lim;
            reinterpret_cast<uint32_t*>(a.pos)[o] = !h.hit ? SF_SLAB_MISS : bad ? SF_SLAB_BAD : h.index;
            // such a pixel counts as unresolved (stats[2]): sf_synchronize then reports SF_EDEPTH instead of the gather
            // silently carrying a NaN pixel (the host's depth proof and the device must never disagree)
            if (bad) atomicAdd(reinterpret_cast<uint32_t*>(a.stats) + 2, 1u);
            return;
        }
        reinterpret_cast<float4*>(a.pos)[o] = make_float4(nx, ny, nz, h.minT);
        return;
    }
    reinterpret_cast<float4*>(a.pos)[o] = make_float4(px, py, pz, 1.0f);
    reinterpret_cast<float4*>(a.nrm)[o] = make_float4(nx, ny, nz, 1.0f);
    if (a.emit_aux) {
        if (a.min_t) a.min_t[o] = h.minT;
        if (a.hit_index) a.hit_index[o] = h.hit ? h.index : 0xffffffffu;
    }
}

struct TileStats {
    int32_t maxd;       // uniform: deepest expanded node (-1: none)
    float closest;      // per lane: its minT (FLT_MAX for invalid lanes); reduced in publish_stats
    bool overflowed;    // uniform: the tile needs more LDS levels than provisioned
};

// One lane's global atomic add on behalf of the wave, result broadcast to every lane. EXEC is set to
// lane 0 inside the asm block, so the compiler's CFG has no lane-0-only region: such regions inside a
// loop let the structurizer run lanes in different iterations, which breaks wave-uniform code.
// A wave-uniform address, said to be so: it can go to an asm "s" operand (an SGPR pair) whatever the compiler's
// divergence analysis concludes about how it was formed (the -fgpu-rdc link's can differ from the compile's).
__device__ __forceinline__ uint32_t* uniform_ptr(uint32_t* p)
{
    const uint64_t pi = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pi), hi = __builtin_amdgcn_readfirstlane((uint32_t)(pi >> 32));
    return reinterpret_cast<uint32_t*>((uint64_t)lo | ((uint64_t)hi << 32));
}

__device__ __forceinline__ uint32_t wave_fetch_add(uint32_t* p, uint32_t v)
{
    p = uniform_ptr(p);   // the address is uniform: say so, so that it can go to the asm in an SGPR pair
    uint32_t r, out;
    uint64_t saved;
    const uint32_t zero = 0u;
    __asm__ volatile(
        "s_mov_b64 %1, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "global_atomic_add %0, %3, %4, %5 sc0\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "s_mov_b64 exec, %1\n\t"
        "s_nop 4\n\t"
        "v_readlane_b32 %2, %0, 0\n\t"
        : "=&v"(r), "=&s"(saved), "=s"(out)
        : "v"(zero), "v"(v), "s"(p)
        : "memory");
    return __builtin_amdgcn_readfirstlane(out);   // asm results count as divergent: say it is uniform
}

// One lane's global atomic increment on behalf of the wave, fire and forget (no return, no wait):
// EXEC is forced to lane 0 inside the asm. The op stays counted in vmcnt, which only makes the
// compiler's own later waits stricter.
__device__ __forceinline__ void wave_atomic_inc_nowait(uint32_t* p)
{
    p = uniform_ptr(p);
    uint64_t saved;
    const uint32_t zero = 0u, one = 1u;
    __asm__ volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "global_atomic_add %1, %2, %3\n\t"
        "s_mov_b64 exec, %0\n\t"
        : "=&s"(saved)
        : "v"(zero), "v"(one), "s"(p)
        : "memory");
}

// One lane's global atomic max on behalf of the wave, completed before it returns (EXEC forced to lane 0).
__device__ __forceinline__ void wave_atomic_max(uint32_t* p, uint32_t v)
{
    p = uniform_ptr(p);
    uint64_t saved;
    const uint32_t zero = 0u;
    __asm__ volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "global_atomic_umax %1, %2, %3\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "s_mov_b64 exec, %0\n\t"
        : "=&s"(saved)
        : "v"(zero), "v"(v), "s"(p)
        : "memory");
}

__device__ __forceinline__ uint32_t cost_bucket(uint32_t c)
{
    const uint32_t k = __float_as_uint((float)(c | 1u)) >> 22;   // exponent and 1 mantissa bit
    const uint32_t b = k - (135u << 1);                            // c < 2^8 -> 0
    return b < SF_ORDER_BUCKETS ? b : (k < (135u << 1) ? 0u : SF_ORDER_BUCKETS - 1u);
}

// The ray-cone axis lane of a unit: the centre pixel of what it traces -- (4, 4) for a whole tile,
// (4, 2) / (4, 6) for the halves, (2 + 4 (q & 1), 2 + 4 (q >> 1)) for quarter q.
__device__ __forceinline__ uint32_t part_axis_lane(uint32_t part)
{
    if (part == 0u) return 36u;
    if (part < SF_PART_QUARTER0) return part == SF_PART_HALF0 ? 20u : 52u;
    const uint32_t q = part - SF_PART_QUARTER0;
    return (2u + 4u * (q >> 1)) * 8u + 2u + 4u * (q & 1u);
}

struct NoPrefetch {
    __device__ void operator()(bool) const {}
};

// `pre` runs right after the traversal, before the tile's shading and stores: the persistent kernel takes
// its next queue ticket there, so the atomic's round trip overlaps the shading instead of following the
// G-buffer stores (whose completion a later wait would otherwise include: vmcnt counts in order).
// Heap index a is n or an ancestor of n (child i of node m is 9 m + 1 + i; indices of depth <= 10, whose heap
// indices fit the 32 bits HitState keeps).
__device__ __forceinline__ bool heap_ancestor(uint32_t a, uint32_t n)
{
    while (n > a) n = (n - 1u) / 9u;
    return n == a;
}

// Subtree part records (SF_FLAG_SUBTREE): part q of split slot s at part_rec + (4 s + q) x 192 u64, three 64-lane
// planes. Stored and loaded with agent scope (sc1: past the writer's and the reader's caches); each part's add to the
// tile's counter follows an agent-scope release fence and the merger (the last to add) acquires before reading them.
__device__ __forceinline__ uint64_t* part_record(const FrameArgs& a, uint32_t slot, uint32_t q)
{
    return a.part_rec + (size_t)(slot * 4u + q) * 192u;
}

template <bool FIXUP, bool PIPE = false, class Prefetch = NoPrefetch, bool COMPACT = false, bool SPLIT = false>
__device__ __forceinline__ TileStats trace_tile(const FrameArgs& a, float* __restrict__ L, const float4 bcol, uint32_t tile,
                                                uint32_t levels, uint32_t* overflow_list, uint32_t* overflow_count,
                                                uint32_t part = 0u, const Prefetch& pre = Prefetch(), uint32_t fl = ~0u,
                                                uint32_t slot = 0u)
{
    // (fl: the launch's flags, with SF_FLAG_REDO_PASS | SF_FLAG_NO_FRONT_FIRST on a re-trace pass; ~0u: flags)
    // (slot: a subtree part unit's split slot -- its position in the unit order / 4)
    const uint32_t flags = fl == ~0u ? a.flags : fl;
    const DeviceConsts* __restrict__ K = a.consts;
    const uint32_t lane = threadIdx.x & 63u;
    if (flags & SF_FLAG_DIAG_HALF) part = (flags & SF_FLAG_DIAG_HALF_SEL) ? 2u : 1u;
    // a subtree part unit: all 64 pixels, the depth-split_depth subtrees of heap index q mod 4 (SF_FLAG_SUBTREE)
    // (only the SPLIT kernel, sf_trace_queue1s, carries the split logic)
    const bool sub = SPLIT && !FIXUP && (flags & SF_FLAG_SUBTREE) != 0u && part >= SF_PART_QUARTER0;
    const Tile t = tile_of(a, tile, lane, sub ? 0u : part);
    const uint64_t t_start = a.tile_trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const uint64_t c_start = (!FIXUP && a.tile_cost) ? __builtin_amdgcn_s_memtime() : 0ull;
    float dx, dy, dz;
    ray_dir(a, (float)t.x, (float)t.y, dx, dy, dz, K->lut);

    HitState h;
    int32_t maxd = -1;
    uint32_t status = 0u;
    uint64_t tile_counts = 0;
    // The main kernels enter children front-first (with the occlusion cull); an exact non-ancestor tie under
    // that order flags the tile like an overflow, and the fixup re-traces it in index order -- the reference's
    // tie rule (see traverse). The fixup kernel always traces in index order.
#ifndef SF_OLD_TRAVERSE
    if constexpr (SPLIT)   // one traversal: the split depth never matches on whole units
        traverse_ray<PIPE, COMPACT, true>(K, a.root, L, bcol, levels, dx, dy, dz, t.valid, h, maxd, status,
                                          FIXUP ? (flags | SF_FLAG_NO_FRONT_FIRST) : flags,
                                          FIXUP ? nullptr : a.phase_sums, part_axis_lane(sub ? 0u : part), &tile_counts,
                                          sub ? part - SF_PART_QUARTER0 : 0u, sub ? a.split_depth : 0xffffffffu);
    else
        traverse_ray<PIPE, COMPACT>(K, a.root, L, bcol, levels, dx, dy, dz, t.valid, h, maxd, status,
                                    FIXUP ? (flags | SF_FLAG_NO_FRONT_FIRST) : flags,
                                    FIXUP ? nullptr : a.phase_sums, part_axis_lane(part), &tile_counts);
#else
    traverse<0, PIPE>(K, a.root, L, bcol, levels, dx, dy, dz, t.valid, h, maxd, status,
                      FIXUP ? (flags | SF_FLAG_NO_FRONT_FIRST) : flags,
                      FIXUP ? nullptr : a.phase_sums, part_axis_lane(part), &tile_counts);
#endif
    if (!FIXUP && (flags & (SF_FLAG_DIAG_FORCE_RETRACE | SF_FLAG_REDO_PASS)) == SF_FLAG_DIAG_FORCE_RETRACE)
        status |= SF_STATUS_TIE;
    bool merger = true;   // this wave writes the tile (a subtree part: only the part that merges)
    if (sub) {
        // ---- subtree part: publish this part's per-pixel result; the part that finishes last merges the four
        // and goes on as a whole tile would (re-trace decision, scheduling cost, G-buffer write)
        const bool rec_cost = a.tile_cost != nullptr && !(flags & SF_FLAG_DIAG_HALF);
        if (rec_cost) {   // the slowest part, in whole-tile terms (x 2, as for quarters)
            const uint64_t cyc = __builtin_amdgcn_s_memtime() - c_start;
            wave_atomic_max(a.part_cost + tile, cyc > 0x7fffffffull ? 0xffffffffu : 2u * (uint32_t)cyc);
        }
        const uint32_t q = part - SF_PART_QUARTER0;
        uint64_t* const R = part_record(a, slot, q);
        __hip_atomic_store(R + lane, ((uint64_t)__float_as_uint(h.cx) << 32) | __float_as_uint(h.minT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(R + 64u + lane, ((uint64_t)__float_as_uint(h.cz) << 32) | __float_as_uint(h.cy),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(R + 128u + lane, ((uint64_t)(uint32_t)h.depth << 32) | h.index,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // release: the records are visible at agent scope before the counter add that publishes them (the
        // memory model, not a hand-placed waitcnt, orders the stores before the add; the merger acquires below)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        // counter: parts done (low byte), parts that flagged an overflow (byte 1), a tie (byte 2)
        const uint32_t add = 1u | ((status & SF_STATUS_OVERFLOW) ? 0x100u : 0u) | ((status & SF_STATUS_TIE) ? 0x10000u : 0u);
        const uint32_t st0 = status;
        const uint32_t old = wave_fetch_add(a.part_done + tile, add);
        merger = (old & 0xffu) == 3u;   // the last part; the others are done with this tile (no write, no flag)
        status = 0u;
      if (merger) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the other parts' records, published before their adds
        a.part_done[tile] = 0u;   // for the next render (uniform value and address)
        // merge: per pixel the nearest sphere over the parts. An exact tie between two parts' spheres is the
        // reference's ancestor rule where one is the other's ancestor (a node's sphere is tested before its
        // subtree, and a tie with an ancestor is accepted, self_test) -- the parts share every node above
        // split_depth, so each part's own result already holds it against the shared spheres -- and otherwise a
        // tie the index-order re-trace resolves, as within a traversal.
        bool tie = false;
#pragma unroll 1
        for (uint32_t p = 0u; p < 4u; ++p) {   // (one part at a time: few registers live)
            if (p == q) continue;
            const uint64_t* const Rp = part_record(a, slot, p);
            const uint64_t r0 = __hip_atomic_load(Rp + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t r1 = __hip_atomic_load(Rp + 64u + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t r2 = __hip_atomic_load(Rp + 128u + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float m = __uint_as_float((uint32_t)r0);
            const uint32_t idx = (uint32_t)r2;
            const int32_t dep = (int32_t)(uint32_t)(r2 >> 32);
            bool take = m < h.minT;
            if (m == h.minT && idx != h.index) {
                const bool both = h.depth >= 0 && dep >= 0 && h.depth <= 10 && dep <= 10;
                if (both && heap_ancestor(h.index, idx)) take = true;          // the deeper sphere wins the tie
                else if (!(both && heap_ancestor(idx, h.index))) tie = true;   // unrelated spheres: re-trace
            }
            if (take) {
                h.minT = m;
                h.cx = __uint_as_float((uint32_t)(r0 >> 32));
                h.cy = __uint_as_float((uint32_t)r1);
                h.cz = __uint_as_float((uint32_t)(r1 >> 32));
                h.index = idx;
                h.depth = dep;
            }
        }
        h.hit = h.depth >= 0;
        status = st0;
        if ((old & 0xff00u) != 0u) status |= SF_STATUS_OVERFLOW;
        if ((old & 0xff0000u) != 0u || wave_ballot(tie) != 0ull) status |= SF_STATUS_TIE;
        if (rec_cost) {
            const uint32_t cost = __builtin_amdgcn_readfirstlane(
                (int)__hip_atomic_load(a.part_cost + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            a.part_cost[tile] = 0u;
            a.tile_cost[tile] = cost;
            if (a.chunk_cnt) {
                const uint32_t cs = __builtin_amdgcn_readfirstlane((tile >> 6) * SF_ORDER_BUCKETS + cost_bucket(cost));
                wave_atomic_inc_nowait(a.chunk_cnt + cs);
            }
        }
      }
    }
    const bool overflowed = status != 0u;
    // a tie under the front-first order with the levels proven (SF_FLAG_TIE_INLINE): this wave re-traces the unit
    // in index order right after (trace_queue_body, told by `pre`); anything else flagged goes to the overflow list
    const bool retrace = !FIXUP && __builtin_amdgcn_readfirstlane(
                                       (int)(status == SF_STATUS_TIE && (flags & SF_FLAG_TIE_INLINE))) != 0;
    pre(retrace);
    if (!FIXUP && a.tile_trace) {
        // diagnostics only: never read by the kernel, never feeds an output value. Every lane stores
        // the same (uniform) words: no lane-0-only region.
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        uint32_t hw;
        __asm__ volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        uint32_t xcc;
        __asm__ volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        a.tile_trace[3u * tile + 0u] = t_start;
        a.tile_trace[3u * tile + 1u] = t_end;
#ifdef SF_COUNTS
        a.tile_trace[3u * tile + 2u] = tile_counts;   // COUNTS=1 builds: the tile's event counts instead
#else
        a.tile_trace[3u * tile + 2u] = ((uint64_t)xcc << 32) | hw;
#endif
    }

    if (!FIXUP && !sub && a.tile_cost && !(flags & (SF_FLAG_DIAG_HALF | SF_FLAG_REDO_PASS))) {
        // scheduling hint for the next render (sf_order_scan / sf_order_scatter); uniform values.
        const uint64_t cyc = __builtin_amdgcn_s_memtime() - c_start;
        uint32_t cost = cyc > 0xffffffffull ? 0xffffffffu : (uint32_t)cyc;
        bool last = true;
        if (part != 0u) {
            // a split tile: the slowest of its parts, in whole-tile terms (x 3/2 for halves, x 2 for
            // quarters), recorded by the part that finishes last
            const uint32_t scaled = part < SF_PART_QUARTER0 ? cost + (cost >> 1) : (cost > 0x7fffffffu ? 0xffffffffu : 2u * cost);
            const uint32_t nparts = part < SF_PART_QUARTER0 ? 2u : 4u;
            wave_atomic_max(a.part_cost + tile, scaled);
            last = wave_fetch_add(a.part_done + tile, 1u) == nparts - 1u;
            if (last) {
                cost = __builtin_amdgcn_readfirstlane(
                    (int)__hip_atomic_load(a.part_cost + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                a.part_cost[tile] = 0u;   // for the next render (uniform values and addresses)
                a.part_done[tile] = 0u;
            }
        }
        if (last) {
            a.tile_cost[tile] = cost;
            if (a.chunk_cnt) {   // (renders that rebuild the order: the histogram for sf_order_scan)
                const uint32_t slot = __builtin_amdgcn_readfirstlane((tile >> 6) * SF_ORDER_BUCKETS + cost_bucket(cost));
                wave_atomic_inc_nowait(a.chunk_cnt + slot);
            }
        }
    }
    if (!FIXUP && overflowed && !retrace) {
        // a deeper (or index-order) re-trace (sf_fixup_wave) rewrites this whole tile
        const uint32_t slot = wave_fetch_add(overflow_count, 1u);
        overflow_list[slot] = tile;   // uniform value and address
    }
    if (t.valid && merger) write_pixel(a, t, dx, dy, dz, h, K->lut);

    // stats: max depth reached, closest sphere distance (Sphereflake.h:157-160, Sphereflake.cpp:197-200)
    TileStats st;
    st.maxd = maxd;
    st.closest = t.valid ? h.minT : FLT_MAX;
    st.overflowed = overflowed;
    return st;
}

// Publish one wave's stats (outside any loop: lane-0 regions are harmless here). `closest` per lane.
// Thousands of waves end together and atomics on one address serialise (~10 ns each), so a wave
// first reads the current value and issues the atomic only if it would change it. The read may be
// stale, never wrong: the values only move one way within a render.
__device__ __forceinline__ void publish_stats(const FrameArgs& a, int32_t maxd, float closest, uint32_t unresolved)
{
    closest = wave_min(closest);
    if ((threadIdx.x & 63u) == 0u) {
        const int32_t key = sf_float_key(closest);
        const int32_t cur_d = __hip_atomic_load(&a.stats[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int32_t cur_k = __hip_atomic_load(&a.stats[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (maxd > cur_d) atomicMax(&a.stats[0], maxd);
        if (key < cur_k) atomicMin(&a.stats[1], key);
        if (unresolved) atomicAdd(&a.stats[2], (int32_t)unresolved);
    }
}

// publish_stats for a call inside a wave-uniform loop (the multi-frame trace publishes a frame's stats when the
// wave leaves the frame): no lane-0 region -- each atomic runs with EXEC forced to lane 0 inside its asm block, as
// wave_atomic_max does (signed max / min: the words start at -1 and at the key of FLT_MAX).
__device__ __forceinline__ void wave_atomic_smax(int32_t* p, int32_t v)
{
    p = reinterpret_cast<int32_t*>(uniform_ptr(reinterpret_cast<uint32_t*>(p)));
    uint64_t saved;
    const uint32_t zero = 0u;
    __asm__ volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "global_atomic_smax %1, %2, %3\n\t"
        "s_mov_b64 exec, %0\n\t"
        : "=&s"(saved)
        : "v"(zero), "v"(v), "s"(p)
        : "memory");
}
__device__ __forceinline__ void wave_atomic_smin(int32_t* p, int32_t v)
{
    p = reinterpret_cast<int32_t*>(uniform_ptr(reinterpret_cast<uint32_t*>(p)));
    uint64_t saved;
    const uint32_t zero = 0u;
    __asm__ volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "global_atomic_smin %1, %2, %3\n\t"
        "s_mov_b64 exec, %0\n\t"
        : "=&s"(saved)
        : "v"(zero), "v"(v), "s"(p)
        : "memory");
}
// Read before the atomic, as publish_stats does: thousands of waves leave a frame together, and atomics on one
// address serialise (~10 ns each) -- issued unconditionally they made a 4-frame launch take twice as long.
__device__ __forceinline__ void publish_stats_in_loop(const FrameArgs& a, int32_t maxd, float closest)
{
    const int32_t key = __builtin_amdgcn_readfirstlane(sf_float_key(wave_min(closest)));
    maxd = __builtin_amdgcn_readfirstlane(maxd);
    const int32_t cur_d = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&a.stats[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const int32_t cur_k = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&a.stats[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (maxd > cur_d) wave_atomic_smax(a.stats + 0, maxd);
    if (key < cur_k) wave_atomic_smin(a.stats + 1, key);
}

}  // namespace

// One wave (one 8x8 tile) per workgroup: LDS is the occupancy limit, so the finest granularity packs best.
// WAVES independent waves per workgroup (adjacent tiles, similar cost); the host picks the variant.
template <int WAVES>
__device__ __forceinline__ void trace_wave_body(const FrameArgs& a, uint32_t* overflow_list, uint32_t* overflow_count)
{
    extern __shared__ float lds[];
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t tile = blockIdx.x * WAVES + wv;
    if (tile >= a.tiles_x * a.tile_rows) return;
    float* const L = lds + wv * SF_LDS_WAVE_FLOATS(a.max_depth);
    stage_root(L, a.root);
    const TileStats st = trace_tile<false>(a, L, build_column(a.consts), tile, a.max_depth, overflow_list, overflow_count);
    publish_stats(a, st.maxd, st.closest, 0u);
}

extern "C" __global__ __launch_bounds__(64) void sf_trace_wave1(FrameArgs a, uint32_t* ol, uint32_t* oc)
{
    trace_wave_body<1>(a, ol, oc);
}
extern "C" __global__ __launch_bounds__(128) void sf_trace_wave2(FrameArgs a, uint32_t* ol, uint32_t* oc)
{
    trace_wave_body<2>(a, ol, oc);
}
extern "C" __global__ __launch_bounds__(256) void sf_trace_wave4(FrameArgs a, uint32_t* ol, uint32_t* oc)
{
    trace_wave_body<4>(a, ol, oc);
}

// Persistent variant: a grid of resident workgroups; each wave pulls 8x8 tiles from a frame-wide
// atomic queue until it runs dry. Dynamic balancing: tile costs vary ~100x (sky vs. deep flake),
// and the in-order workgroup dispatcher otherwise idles CUs behind long tiles. counters: [0,1]
// overflow counts, [2,3] tile queues, alternating per render (this render zeroes the next one's).
template <int WAVES, bool PIPE = false, bool COMPACT = false, bool SPLIT = false>
__device__ __forceinline__ void trace_queue_body(const FrameArgs& a)
{
    extern __shared__ float lds[];
    const uint64_t w_start = __builtin_amdgcn_s_memrealtime();
    const uint32_t wv = threadIdx.x >> 6;
    // measurement: the live shader clock, delta s_memtime / delta s_memrealtime x 100 MHz over this wave's
    // life (the start pair stored now, so nothing stays live across the tile loop; uniform values and
    // addresses; read by sf_kernel_clocks, never by a kernel)
    if (a.clock_probe && wv == 0u && blockIdx.x < SF_CLOCK_WAVES) {
        uint64_t* cp = a.clock_probe + 4u * blockIdx.x;
        cp[0] = __builtin_amdgcn_s_memtime();
        cp[1] = w_start;
    }
    // a.queues (<= SF_QUEUES) tile queues per render, one cache line each: queue k hands out the units
    // after the static first ones with index = k mod a.queues
    // A wave starts on its own XCD's queue and moves on to the next one when it runs dry. One queue
    // for the whole chip serialises ~100 atomics/us on one address (measured: ~11 us per fetch).
    if (blockIdx.x == 0 && threadIdx.x < SF_QUEUES)
        a.counters[SF_QUEUE_WORD(a.parity ^ 1u, threadIdx.x)] = 0u;   // the next render's queues
    if (blockIdx.x == 0 && threadIdx.x == 0) a.counters[a.parity ^ 1u] = 0u;   // and overflow count
    float* const L = lds + wv * SF_LDS_WAVE_FLOATS(a.max_depth);
    const uint32_t ntiles = a.tiles_x * a.tile_rows;
    // work units: tiles in row-major order, or the previous render's heavy-first order in which the
    // heaviest tiles come as two half units (order_meta[0] entries)
    uint32_t nunits = ntiles;
    if (a.tile_order) {
#if defined(__HIP_DEVICE_COMPILE__)
        typedef const __attribute__((address_space(4))) uint32_t* ConstU32;
        nunits = ((ConstU32)(const void*)a.order_meta)[0];
#else
        nunits = a.order_meta[0];
#endif
    } else if (a.flags & SF_FLAG_HALVES) {
        nunits = 2u * ntiles;
    }
    stage_root(L, a.root);
    const float4 bcol = build_column(a.consts);
    // One queue per XCD (a.queues of them); a wave drains its own group's queue and then exits. Stealing
    // from the other queues once the own one ran dry cost every wave up to 7 more atomics on queue words
    // contended chip-wide at the end of the frame: the last wave exited ~60 us after the last tile
    // ended. Every queue still drains: its group's waves only leave when it is empty.
    const uint32_t nq = a.queues, nx = a.xcds;
    // queue k = block group (k % nx) + nx x sub-queue; a group's waves spread over its nq / nx sub-queues by
    // their position in the grid. The group is blockIdx mod nx, not the XCD id: blocks are observed to be
    // dealt round-robin over the XCDs, so a group is one XCD's blocks (its queue word stays in that XCD's
    // traffic), but every group has waves whatever the placement (a CU-masked stream, a partitioned chip):
    // the host keeps nx <= the grid's blocks, so every queue drains.
    uint32_t k = blockIdx.x & (nx - 1u);
    if (nq > nx) {   // (powers of two: shifts, no division)
        const uint32_t lx = __builtin_ctz(nx);
        k += nx * (((blockIdx.x >> lx) * WAVES + wv) & ((nq >> lx) - 1u));
        k = __builtin_amdgcn_readfirstlane(k);
    }
    int32_t maxd = -1;
    float closest = FLT_MAX;   // per lane
    // The first unit of every wave is static: wave w (in dispatch order) takes unit w, so the head of the
    // heavy-first order starts as the waves arrive instead of behind ~900 simultaneous atomics per queue;
    // the queues hand out units nwaves, nwaves + 1, ...
    const uint32_t nwaves = gridDim.x * WAVES;
    uint32_t first = __builtin_amdgcn_readfirstlane(blockIdx.x * WAVES + wv);   // (wv is wave-uniform)
    for (;;) {
        // Re-read the launch arguments every tile (scalar loads from the kernarg segment) instead of
        // keeping ~40 of them live in SGPRs across the whole persistent loop.
        // (FrameArgs is the only kernel argument: offset 0 of the kernarg segment)
        FrameArgs at;
#if defined(__HIP_DEVICE_COMPILE__)
        {
            typedef const __attribute__((address_space(4))) FrameArgs* KernargArgs;
            KernargArgs pa = (KernargArgs)__builtin_amdgcn_kernarg_segment_ptr();
            __asm__ volatile("" : "+s"(pa));
            __builtin_memcpy(&at, (const FrameArgs*)pa, sizeof(FrameArgs));
        }
#else
        at = a;
#endif
        // position in the render's unit order: the static first unit, then the ticket the previous tile
        // took after its traversal (past the end: the XCD's queue is empty)
        // (or, bit 31 set, a unit to re-trace in index order: part << SF_UNIT_PRIO_SHIFT | tile -- a tie under the
        // front-first order with SF_FLAG_TIE_INLINE; the ticket is taken after that pass)
        const uint32_t g = first;
        const bool again = (g >> 31) != 0u;
        if (!again && g >= nunits) break;
        uint32_t t = g, part = 0u;
        if (again) {
            t = g & SF_UNIT_TILE_MASK;
            part = (g >> SF_UNIT_PRIO_SHIFT) & 7u;
        } else if (at.tile_order) {      // heaviest tiles of the previous render first (scalar load)
#if defined(__HIP_DEVICE_COMPILE__)
            typedef const __attribute__((address_space(4))) uint32_t* ConstU32;
            const uint32_t u = ((ConstU32)(const void*)at.tile_order)[g];
#else
            const uint32_t u = at.tile_order[g];
#endif
            t = u & SF_UNIT_TILE_MASK;
            part = u >> SF_UNIT_PART_SHIFT;
            // critical-path tiles (top cost buckets of the last render, order_meta[3]) at raised priority:
            // the SIMD's issue arbitration serves them first, the cheap tiles absorb the wait. Graded: the
            // raised buckets' lowest 3 (1.5 octaves) at 2, the ones above at 3, so the very heaviest tiles
            // also win the arbitration against the merely heavy (8 buckets: 0.1607 -> 0.1578 ms/frame against
            // all raised buckets at one level). The level comes with the unit (sf_order_scatter).
            const uint32_t pr = (u >> SF_UNIT_PRIO_SHIFT) & 3u;
            if (pr == 2u && !(at.flags & SF_FLAG_PRIO_FLAT)) __builtin_amdgcn_s_setprio(3);
            else if (pr != 0u) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(0);
        } else if (at.flags & SF_FLAG_HALVES) {   // (row-major halves: unit g = half g & 1 of tile g / 2)
            t = g >> 1;
            part = SF_PART_HALF0 + (g & 1u);
        }
        const uint64_t u_start = (at.flags & SF_FLAG_DIAG_UNITS) ? __builtin_amdgcn_s_memrealtime() : 0ull;
        // the next unit's ticket, taken when this tile's traversal ends (see trace_tile)
        // (an agent-coherent load of the queue word before the atomic, to skip dry queues, made the frame
        // 1.7x slower: it contends with the atomics on the line)
        // (a subtree part's re-trace is its whole tile's: the part that merged the tile takes it, as part 0)
        auto ticket = [&](bool retrace) {
            const uint32_t rp = ((at.flags & SF_FLAG_SUBTREE) && part >= SF_PART_QUARTER0) ? 0u : part;
            first = retrace ? (0x80000000u | (rp << SF_UNIT_PRIO_SHIFT) | t)
                            : nwaves + wave_fetch_add(at.counters + SF_QUEUE_WORD(at.parity, k), 1u) * nq + k;   // uniform
        };
        const TileStats st = trace_tile<false, PIPE, decltype(ticket), COMPACT, SPLIT>(at, L, bcol, t, at.max_depth, at.overflow_list,
                                                                               at.counters + at.parity, part,
                                               ticket, again ? (at.flags | SF_FLAG_NO_FRONT_FIRST | SF_FLAG_REDO_PASS)
                                                             : at.flags, g >> 2);
        if ((at.flags & SF_FLAG_DIAG_UNITS) && at.tile_trace && (g >> 31) == 0u) {   // diagnostics only (uniform words)
            // (slot g: the unit's position in the order. A re-trace pass -- its ticket word carries bit 31 -- records
            // nothing: its word is no position, and the slot of the unit it repeats already holds that unit's record)
            uint64_t* ut = at.tile_trace + 3u * (at.tiles_x * at.tile_rows) + SF_DIAG_SLOTS + 3u * g;
            ut[0] = u_start;
            ut[1] = __builtin_amdgcn_s_memrealtime();
            ut[2] = t | (part << SF_UNIT_PART_SHIFT);
        }
        maxd = st.maxd > maxd ? st.maxd : maxd;
        closest = fminf(closest, st.closest);
    }
    // the launch arguments again from the kernarg segment, so that none of them is held in a register
    // across the tile loop for the code below
    FrameArgs e;
#if defined(__HIP_DEVICE_COMPILE__)
    {
        typedef const __attribute__((address_space(4))) FrameArgs* KernargArgs;
        KernargArgs pa = (KernargArgs)__builtin_amdgcn_kernarg_segment_ptr();
        __asm__ volatile("" : "+s"(pa));
        __builtin_memcpy(&e, (const FrameArgs*)pa, sizeof(FrameArgs));
    }
#else
    e = a;
#endif
    publish_stats(e, maxd, closest, 0u);
    if (e.clock_probe && wv == 0u && blockIdx.x < SF_CLOCK_WAVES) {   // measurement: the end pair (see above)
        uint64_t* cp = e.clock_probe + 4u * blockIdx.x;
        cp[2] = __builtin_amdgcn_s_memtime();
        cp[3] = __builtin_amdgcn_s_memrealtime();
    }
    if ((e.flags & SF_FLAG_DIAG_UNITS) && e.tile_trace) {   // diagnostics: this wave's {start, end}
        const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * WAVES + wv);
        if (w < SF_DIAG_WAVES) {
            uint64_t* wt = e.tile_trace + (SF_TRACE_WORDS(e.tiles_x * e.tile_rows) - 2u * SF_DIAG_WAVES) + 2u * w;
            wt[0] = w_start;
            wt[1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SF_WAVES_PER_EU, 8))) void sf_trace_queue1(FrameArgs a)
{
    trace_queue_body<1>(a);
}
// the same with subtree-split units (SF_FLAG_SUBTREE): renders whose unit order holds split tiles
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SF_WAVES_PER_EU, 8))) void sf_trace_queue1s(FrameArgs a)
{
    trace_queue_body<1, false, false, true>(a);
}
extern "C" __global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(SF_WAVES_PER_EU, 8))) void sf_trace_queue2(FrameArgs a)
{
    trace_queue_body<2>(a);
}
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SF_WAVES_PER_EU, 8))) void sf_trace_queue4(FrameArgs a)
{
    trace_queue_body<4>(a);
}
// active-ray compaction of sparse nodes (opt-in, SF_COMPACT=1; see traverse_ray): measured against the default
extern "C" __global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(SF_WAVES_PER_EU, 8))) void sf_trace_queue2c(FrameArgs a)
{
    trace_queue_body<2, false, true>(a);
}
// latency variant (pipelined child loop) for frames whose tiles do not fill the persistent grid twice
extern "C" __global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(SF_WAVES_PER_EU, 8))) void sf_trace_queue2p(FrameArgs a)
{
    trace_queue_body<2, true>(a);
}

// Multi-frame persistent trace (round 6, sf_render_frames): ONE resident grid takes the work units of
// up to SF_BATCH_MAX frames -- each a slot context's own view, G-buffer and stats -- from one set of tile queues. A
// wave whose frame runs dry goes on with the next frame's units, so there is no per-frame launch, no hardware queue
// per frame and no frame boundary where waves wait for a successor grid; and the launch's sequence starts with the
// `heavy` heaviest units of EVERY frame of the batch, interleaved (the static first unit of wave w is position w), so
// no frame's heaviest tiles start late and leave a serial tail (the reference's workers likewise trace continuously,
// Sphereflake.cpp:67-74,112-213). Position G of the sequence:
// (units: the shared order's unit count, read on the device like trace_queue_body's; heavy: at most units)
//   G < nframes x heavy:  frame G % nframes, order position G / nframes (the interleaved heads)
//   else (q = G - nframes x heavy): frame q / (units - heavy), order position heavy + q % (units - heavy)
// Per frame everything is as in trace_queue_body<1>: the frame's FrameArgs re-read from the kernel argument segment
// per unit (scalar loads), its root staged in the wave's LDS when the wave's frame changes, its stats published when
// the wave leaves the frame. The frames share the unit order (the camera moves little between frames), the queues
// and their parity (the host gives every frame the first context's); only one frame may record tile costs.
// The batch in the kernel argument segment, through an address the compiler may not reason about: every read is a
// scalar load where it is used, so no batch word stays live in an SGPR across the tile loop (the loop's state is a few
// words: the wave's next position, its frame, its queue, its stats).
__device__ __forceinline__ const __attribute__((address_space(4))) FrameBatch* kernarg_batch()
{
    typedef const __attribute__((address_space(4))) FrameBatch* KernargBatch;
    KernargBatch pa = (KernargBatch)__builtin_amdgcn_kernarg_segment_ptr();
    __asm__ volatile("" : "+s"(pa));
    return pa;
}

__device__ __forceinline__ void load_frame(FrameArgs& at, uint32_t f)
{
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) FrameArgs* KernargArgs;
    KernargArgs pf = &((const __attribute__((address_space(4))) FrameBatch*)__builtin_amdgcn_kernarg_segment_ptr())->f[f];
    __asm__ volatile("" : "+s"(pf));   // (opaque: the fields are loaded where trace_tile uses them, as in trace_queue_body)
    __builtin_memcpy(&at, (const FrameArgs*)pf, sizeof(FrameArgs));
#else
    (void)at;
    (void)f;
#endif
}

template <int WAVES = 1>   // (one wave per workgroup; a template like trace_queue_body, for the shared `lds` declaration)
__device__ __forceinline__ void trace_frames_body()
{
    extern __shared__ float lds[];
    const uint64_t w_start = __builtin_amdgcn_s_memrealtime();
    {
        const auto pb = kernarg_batch();
        if (blockIdx.x == 0 && threadIdx.x < SF_QUEUES)   // the next launch's queues and overflow count
            pb->f[0].counters[SF_QUEUE_WORD(pb->f[0].parity ^ 1u, threadIdx.x)] = 0u;
        if (blockIdx.x == 0 && threadIdx.x == 0) pb->f[0].counters[pb->f[0].parity ^ 1u] = 0u;
        if (pb->f[0].clock_probe && blockIdx.x < SF_CLOCK_WAVES) {   // measurement: the live clock (trace_queue_body)
            uint64_t* cp = pb->f[0].clock_probe + 4u * blockIdx.x;
            cp[0] = __builtin_amdgcn_s_memtime();
            cp[1] = w_start;
        }
    }
    float* const L = lds;
    const float4 bcol = build_column(kernarg_batch()->f[0].consts);   // (the slot contexts' constant blocks are equal)
    uint32_t k;
    {
        const auto pb = kernarg_batch();
        const uint32_t nq = pb->f[0].queues, nx = pb->f[0].xcds;
        k = blockIdx.x & (nx - 1u);
        if (nq > nx) {
            const uint32_t lx = __builtin_ctz(nx);
            k += nx * ((blockIdx.x >> lx) & ((nq >> lx) - 1u));
        }
        k = __builtin_amdgcn_readfirstlane(k);
    }
    // per-frame stats in the lanes of two VGPRs -- lane f: frame f's max depth and closest-hit key so far -- published
    // once per frame when the wave ends: publishing at every frame switch (two agent-scope loads, maybe atomics) put a
    // ~2-us latency on the switch, which a wave of a banded share meets at nearly every unit
    uint32_t stat_d = 0xffffffffu;                  // (int -1)
    uint32_t stat_k = (uint32_t)sf_float_key(FLT_MAX);
    uint32_t cur = 0xffffffffu;   // the frame of the last unit (uniform)
    uint32_t staged = 0xffffffffu;   // the frame whose root is staged in LDS (uniform)
    uint32_t first = __builtin_amdgcn_readfirstlane(blockIdx.x);
    for (;;) {
        const uint32_t G = first;
        const bool again = (G >> 31) != 0u;
        uint32_t f = cur, pos = 0u;
        if (!again) {
            const auto pb = kernarg_batch();
            const uint32_t nframes = pb->nframes;
            // units per frame: the shared order's (order_meta[0]: split tiles count as their parts), else the tiles
            uint32_t units = pb->units;
            if (pb->f[0].tile_order) {
#if defined(__HIP_DEVICE_COMPILE__)
                typedef const __attribute__((address_space(4))) uint32_t* ConstU32;
                units = ((ConstU32)(const void*)pb->f[0].order_meta)[0];
#else
                units = pb->f[0].order_meta[0];
#endif
            }
            const uint32_t heavy = pb->heavy < units ? pb->heavy : units;
            if (G >= nframes * units) break;
            // (no integer division per unit: a division by a uniform value is a ~35-instruction scalar sequence, and
            // four of them per unit measured +18 % SALU against trace_queue_body)
            const uint32_t hh = nframes * heavy;
            if (G < hh) {
                pos = __builtin_amdgcn_readfirstlane(__umulhi(G, pb->magic));   // G / nframes (exact for G < 2^29)
                f = G - pos * nframes;
            } else {
                uint32_t q = G - hh;
                const uint32_t rest = units - heavy;
                f = 0u;
                while (q >= rest) {   // (<= SF_BATCH_MAX - 1 trips)
                    q -= rest;
                    ++f;
                }
                pos = heavy + q;
            }
            f = __builtin_amdgcn_readfirstlane(f);
            pos = __builtin_amdgcn_readfirstlane(pos);
        }
        cur = f;
        FrameArgs at;
        load_frame(at, f);
        if (f != staged) {   // (the frame's root transform into the wave's LDS image)
            stage_root_all_lanes(L, at.root);
            staged = f;
        }
        uint32_t t = pos, part = 0u;
        if (again) {
            t = G & SF_UNIT_TILE_MASK;
            part = (G >> SF_UNIT_PRIO_SHIFT) & 7u;
        } else if (at.tile_order) {
#if defined(__HIP_DEVICE_COMPILE__)
            typedef const __attribute__((address_space(4))) uint32_t* ConstU32;
            const uint32_t u = ((ConstU32)(const void*)at.tile_order)[pos];
#else
            const uint32_t u = at.tile_order[pos];
#endif
            t = u & SF_UNIT_TILE_MASK;
            part = u >> SF_UNIT_PART_SHIFT;
            const uint32_t pr = (u >> SF_UNIT_PRIO_SHIFT) & 3u;
            if (pr == 2u && !(at.flags & SF_FLAG_PRIO_FLAT)) __builtin_amdgcn_s_setprio(3);
            else if (pr != 0u) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(0);
        }
        auto ticket = [&](bool retrace) {
            first = retrace ? (0x80000000u | (part << SF_UNIT_PRIO_SHIFT) | t)
                            : gridDim.x + wave_fetch_add(at.counters + SF_QUEUE_WORD(at.parity, k), 1u) * at.queues + k;
        };
        const TileStats st = trace_tile<false, false, decltype(ticket)>(at, L, bcol, t, at.max_depth, at.overflow_list,
                                                                      at.counters + at.parity, part, ticket,
                                                                      again ? (at.flags | SF_FLAG_NO_FRONT_FIRST |
                                                                               SF_FLAG_REDO_PASS)
                                                                            : at.flags);
        {   // frame cur's stats: the unit's max depth and closest hit into lane cur of the accumulators
            const int32_t ud = __builtin_amdgcn_readfirstlane(st.maxd);
            const int32_t uk = __builtin_amdgcn_readfirstlane(sf_float_key(wave_min(st.closest)));
            const int32_t od = (int32_t)__builtin_amdgcn_readlane(stat_d, cur);
            const int32_t ok = (int32_t)__builtin_amdgcn_readlane(stat_k, cur);
            stat_d = writelane_s((uint32_t)(ud > od ? ud : od), cur, stat_d);
            stat_k = writelane_s((uint32_t)(uk < ok ? uk : ok), cur, stat_k);
        }
    }
    {   // every frame's stats once (read before the atomics: thousands of waves end together, publish_stats)
        const uint32_t nframes = kernarg_batch()->nframes;
        for (uint32_t fr = 0u; fr < nframes; ++fr) {
            const int32_t dd = (int32_t)__builtin_amdgcn_readlane(stat_d, fr);
            const int32_t kk = (int32_t)__builtin_amdgcn_readlane(stat_k, fr);
            if (dd < 0 && kk == sf_float_key(FLT_MAX)) continue;   // (no unit of that frame)
            FrameArgs e;
            load_frame(e, fr);
            publish_stats_in_loop(e, dd, sf_key_float(kk));
        }
    }
    const auto pb = kernarg_batch();
    if (pb->f[0].clock_probe && blockIdx.x < SF_CLOCK_WAVES) {
        uint64_t* cp = pb->f[0].clock_probe + 4u * blockIdx.x;
        cp[2] = __builtin_amdgcn_s_memtime();
        cp[3] = __builtin_amdgcn_s_memrealtime();
    }
}

extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SF_WAVES_PER_EU, 8))) void sf_trace_frames1(FrameBatch b)
{
    (void)b;   // (read through the kernel argument segment, per unit: trace_frames_body)
    trace_frames_body<1>();
}

// Tile order for the next render: tiles sorted by this render's cost, heaviest first (LPT list
// scheduling of the persistent kernel), as a counting sort over SF_ORDER_BUCKETS log-spaced cost
// buckets (2 per octave of cycles). The trace kernel counts every finished tile into its 64-tile
// chunk's bucket histogram (one fire-and-forget atomic); sf_order_scan turns the histograms into
// per-(chunk, bucket) output offsets, heaviest bucket first and chunks in order within a bucket;
// sf_order_scatter (one wave per chunk) writes the permutation and clears the histograms. Stable and
// deterministic. Any permutation gives the same image: only the schedule changes.
// One 64-item chunk c of the scatter, one wave (lane = item within the chunk).
// (rank_out, when not NULL: rank_out[i] = item i's position, the inverse permutation; unsplit orders only)
// (offs: lane b's value is bucket b & 31's output offset for this chunk)
__device__ __forceinline__ void order_scatter_chunk(uint32_t c, uint32_t lane, const uint32_t* __restrict__ cost,
                                                    uint32_t n, uint32_t* __restrict__ chunk_cnt, uint32_t offs,
                                                    uint32_t split_from, uint32_t parts, uint32_t pb,
                                                    uint32_t* __restrict__ order, uint32_t* __restrict__ rank_out)
{
    const uint32_t i = c * 64u + lane;
    const uint32_t first = parts == 4u ? SF_PART_QUARTER0 : SF_PART_HALF0;
    const uint32_t bk = i < n ? cost_bucket(cost[i]) : SF_ORDER_BUCKETS;   // sentinel: no tile
    uint64_t pending = __builtin_amdgcn_ballot_w64(bk < SF_ORDER_BUCKETS);
    while (pending) {   // one round per distinct bucket in the chunk
        const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)bk, (int)__builtin_ctzll(pending));
        const uint64_t m = __builtin_amdgcn_ballot_w64(bk == b);
        const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)offs, (int)b);
        if (bk == b) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            // the unit's wave priority next render (see SF_UNIT_PRIO_SHIFT)
            const uint32_t u = i | ((b >= pb + 3u ? 2u : b >= pb ? 1u : 0u) << SF_UNIT_PRIO_SHIFT);
            if (b >= split_from) {   // `parts` part units, adjacent
                for (uint32_t p = 0; p < parts; ++p) order[off + parts * rank + p] = u | ((first + p) << SF_UNIT_PART_SHIFT);
            } else {
                order[off + rank] = u;
                if (rank_out) rank_out[i] = off + rank;
            }
        }
        pending &= ~m;
    }
    if (lane < SF_ORDER_BUCKETS) chunk_cnt[c * SF_ORDER_BUCKETS + lane] = 0u;   // for the next render
}

// The order's split and priority decisions and the bucket output offsets, by one wave: lane l holds bucket l's
// tile count t (lanes 32..63: 0). Returns the first split bucket and the first raised-priority bucket; X_excl = the
// units of the buckets heavier than l (lane l), units = all the units.
struct OrderPlan {
    int bs, bp;
    uint32_t X_excl, units;
};
__device__ __forceinline__ OrderPlan order_decide(uint32_t t, uint32_t l, uint32_t n_tiles, uint32_t split_buckets,
                                                  uint32_t parts, uint32_t spare, uint32_t waves, uint32_t prio_buckets,
                                                  uint32_t split_cap)
{
    // One wave, lane = bucket (lanes 32..63 hold 0): the split and priority decisions and the bucket
    // offsets from suffix sums over the buckets (heaviest first), instead of serial loops on one thread.
    // Split tiles into `parts` units each, heaviest buckets first (bucket 0 never): automatically as
    // many whole buckets as fit into `spare` idle wave slots, or the top `split_buckets` occupied
    // buckets (at most an eighth of the tiles).
    uint32_t S = t;   // S(l) = sum of tot[bb] over bb >= l
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
        const uint32_t up = (uint32_t)__shfl_down((int)S, o, 64);
        S += l + (uint32_t)o < SF_ORDER_BUCKETS ? up : 0u;
    }
    const uint64_t nz = __builtin_amdgcn_ballot_w64(t != 0u);
    const int btop = nz ? 63 - __builtin_clzll(nz) : 0;   // highest occupied bucket (0 if none)
    int bs = (int)SF_ORDER_BUCKETS;
    if (split_buckets == SF_SPLIT_AUTO) {
        // S is non-increasing in the bucket: the buckets that fit form a suffix
        const uint64_t ok = __builtin_amdgcn_ballot_w64(l >= 1u && l < SF_ORDER_BUCKETS && S * (parts - 1u) <= spare);
        if (ok >> (SF_ORDER_BUCKETS - 1u) & 1ull) bs = __builtin_ctzll(ok);
    } else if (split_buckets == SF_SPLIT_MODEL && waves > 0u) {
        // Makespan model (LPT list scheduling on `waves` slots, the last render's costs): unsplit, the
        // frame takes at least max(C / waves, c_top); splitting buckets >= l into `parts` units adds their
        // work x (parts x rho - 1) and leaves max(the heaviest unsplit bucket, rho x c_top) as the longest
        // unit (rho: the slowest part's share of its tile, measured 0.6 for quarters, 0.68 for halves).
        // Take the l of the least estimate when it is >= 10 % below the unsplit one.
        const float rho = parts == 4u ? 0.6f : 0.68f;
        const uint32_t e = (l + 16u) >> 1;   // bucket l covers [2^e (1 + m/2), ...) cycles, m = (l + 16) & 1
        const float c = l < SF_ORDER_BUCKETS ? __builtin_ldexpf((l + 16u) & 1u ? 1.75f : 1.25f, (int)e) : 0.0f;
        const float w = (float)t * c;   // this bucket's work
        float A = w;                    // A(l) = work of the buckets >= l
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
            const float up = __shfl_down(A, o, 64);
            A += l + (uint32_t)o < SF_ORDER_BUCKETS ? up : 0.0f;
        }
        const float C = __shfl(A, 0, 64);                 // all the work
        const float ctop = __shfl(c, btop, 64);
        const uint64_t below = nz & ((1ull << l) - 1ull);   // occupied buckets under l
        const float cun = below ? __shfl(c, 63 - __builtin_clzll(below), 64) : 0.0f;
        const float Tn = fmaxf(C / (float)waves, ctop);
        float T = fmaxf(fmaxf((C + A * ((float)parts * rho - 1.0f)) / (float)waves, cun), rho * ctop);
        if (!(l >= 1u && (int)l <= btop)) T = __builtin_inff();
        float Tm = T;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) Tm = fminf(Tm, __shfl_xor(Tm, o, 64));
        const uint64_t best = __builtin_amdgcn_ballot_w64(T == Tm);
        if (Tm < 0.9f * Tn && best) bs = 63 - __builtin_clzll(best);   // (ties: the fewest splits)
    } else if (split_buckets != 0u) {
        int b0 = btop - (int)split_buckets + 1;
        if (b0 < 1) b0 = 1;
        // then drop buckets from the bottom of the range while more than an eighth of the tiles split
        const uint64_t ok = __builtin_amdgcn_ballot_w64((int)l >= b0 && l < SF_ORDER_BUCKETS && 8u * S <= n_tiles);
        bs = ok ? __builtin_ctzll(ok) : (int)SF_ORDER_BUCKETS;
    }
    // at most split_cap split tiles (the subtree parts' records are per split slot): S(l) is non-increasing
    {
        const uint64_t capok = __builtin_amdgcn_ballot_w64(l < SF_ORDER_BUCKETS && S <= split_cap);
        const int bcap = capok ? __builtin_ctzll(capok) : (int)SF_ORDER_BUCKETS;
        if (bs < bcap) bs = bcap;
    }
    // the top `prio_buckets` occupied cost buckets run at raised wave priority next render (their
    // serial DFS is the frame's critical path)
    const int bp = btop - (int)prio_buckets + 1;
    // units per bucket -> exclusive offsets, heaviest first: X(l) = sum of units over bb > l
    const uint32_t x = t * ((int)l >= bs ? parts : 1u);
    uint32_t X = x;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
        const uint32_t up = (uint32_t)__shfl_down((int)X, o, 64);
        X += l + (uint32_t)o < SF_ORDER_BUCKETS ? up : 0u;
    }
    OrderPlan r;
    r.bs = bs;
    r.bp = bp;
    r.X_excl = X - x;
    r.units = (uint32_t)__shfl(X, 0, 64);
    return r;
}

#define SF_SCAN_BATCH 16   // chunk counts a scan thread loads at once (independent loads, one wait)

extern "C" __global__ __launch_bounds__(1024) void sf_order_scan(uint32_t* __restrict__ chunk_cnt, uint32_t nc,
                                                                   uint32_t n_tiles, uint32_t split_buckets, uint32_t parts,
                                                                   uint32_t spare, uint32_t waves, uint32_t prio_buckets,
                                                                   uint32_t* __restrict__ chunk_off,
                                                                   uint32_t* __restrict__ order_meta,
                                                                   const uint32_t* __restrict__ fuse_cost,
                                                                   uint32_t* __restrict__ fuse_order, uint32_t split_cap)
{
    // fuse_cost / fuse_order not NULL: this workgroup also does sf_order_scatter's work afterwards (its 16 waves
    // over the chunks), one launch instead of two -- for frames of few chunks, where the second launch's host
    // cost and dispatch latency exceed the scatter itself
    // (with frames in flight this one workgroup shares the CUs with other frames' trace waves, whose heavy
    // tiles run at raised priority: without its own it waited ~125 us instead of ~8 for issue slots)
    __builtin_amdgcn_s_setprio(3);
    // thread = (bucket b = tid % 32, slice k = tid / 32): chunks [k * per, (k + 1) * per) of bucket b
    __shared__ uint32_t part[32][SF_ORDER_BUCKETS + 1];
    __shared__ uint32_t tot[SF_ORDER_BUCKETS];
    const uint32_t tid = threadIdx.x, b = tid % SF_ORDER_BUCKETS, k = tid / SF_ORDER_BUCKETS;
    const uint32_t per = (nc + 31u) / 32u, c0 = k * per, c1 = min(nc, c0 + per);
    uint32_t s_ = 0u;
    uint32_t v0[SF_SCAN_BATCH];   // the first batch stays in registers for the offsets pass below (frames of up
                                  // to 32 x SF_SCAN_BATCH chunks, 1080p included, need no second read)
#pragma unroll
    for (int j = 0; j < SF_SCAN_BATCH; ++j) v0[j] = c0 + j < c1 ? chunk_cnt[(c0 + j) * SF_ORDER_BUCKETS + b] : 0u;
#pragma unroll
    for (int j = 0; j < SF_SCAN_BATCH; ++j) s_ += v0[j];
    for (uint32_t cb = c0 + SF_SCAN_BATCH; cb < c1; cb += SF_SCAN_BATCH) {
        uint32_t v[SF_SCAN_BATCH];
#pragma unroll
        for (int j = 0; j < SF_SCAN_BATCH; ++j) v[j] = cb + j < c1 ? chunk_cnt[(cb + j) * SF_ORDER_BUCKETS + b] : 0u;
#pragma unroll
        for (int j = 0; j < SF_SCAN_BATCH; ++j) s_ += v[j];
    }
    part[k][b] = s_;
    __syncthreads();
    if (tid < SF_ORDER_BUCKETS) {   // per bucket: slices -> exclusive prefix; bucket total
        uint32_t acc = 0u;
        for (uint32_t j = 0; j < 32u; ++j) {
            const uint32_t x = part[j][tid];
            part[j][tid] = acc;
            acc += x;
        }
        tot[tid] = acc;
    }
    __syncthreads();
    __shared__ uint32_t split_from;
    if (tid < 64u) {
        const uint32_t l = tid;
        const uint32_t t = l < SF_ORDER_BUCKETS ? tot[l] : 0u;
        const OrderPlan pl = order_decide(t, l, n_tiles, split_buckets, parts, spare, waves, prio_buckets, split_cap);
        const int bs = pl.bs, bp = pl.bp;
        const uint32_t X = pl.units;
        if (l < SF_ORDER_BUCKETS) tot[l] = pl.X_excl;
        if (l == 0u) {
            split_from = (uint32_t)bs;
            order_meta[0] = X;              // units of the next render
            order_meta[1] = (uint32_t)bs;   // first split bucket
            order_meta[2] = parts;          // units per split tile
            order_meta[3] = prio_buckets == 0u ? SF_ORDER_BUCKETS : (uint32_t)(bp < 0 ? 0 : bp);
        }
    }
    __syncthreads();
    const uint32_t mult = b >= split_from ? parts : 1u;
    uint32_t off = tot[b] + part[k][b] * mult;
#pragma unroll
    for (int j = 0; j < SF_SCAN_BATCH; ++j) {
        if (c0 + j < c1) chunk_off[(c0 + j) * SF_ORDER_BUCKETS + b] = off;
        off += v0[j] * mult;
    }
    for (uint32_t cb = c0 + SF_SCAN_BATCH; cb < c1; cb += SF_SCAN_BATCH) {
        uint32_t v[SF_SCAN_BATCH];
#pragma unroll
        for (int j = 0; j < SF_SCAN_BATCH; ++j) v[j] = cb + j < c1 ? chunk_cnt[(cb + j) * SF_ORDER_BUCKETS + b] : 0u;
#pragma unroll
        for (int j = 0; j < SF_SCAN_BATCH; ++j) {
            if (cb + j < c1) chunk_off[(cb + j) * SF_ORDER_BUCKETS + b] = off;
            off += v[j] * mult;
        }
    }
    if (fuse_order) {
        // chunk_off and the counts were written / read by this workgroup only: a workgroup barrier orders them
        __syncthreads();
        const uint32_t pb = order_meta[3];
        for (uint32_t c = tid >> 6; c < nc; c += blockDim.x >> 6)
            order_scatter_chunk(c, tid & 63u, fuse_cost, n_tiles, chunk_cnt,
                                chunk_off[c * SF_ORDER_BUCKETS + (tid & (SF_ORDER_BUCKETS - 1u))], split_from, parts, pb,
                                fuse_order, nullptr);
    }
}

extern "C" __global__ __launch_bounds__(64) void sf_order_scatter(const uint32_t* __restrict__ cost, uint32_t n,
                                                                    uint32_t* __restrict__ chunk_cnt,
                                                                    const uint32_t* __restrict__ chunk_off,
                                                                    const uint32_t* __restrict__ order_meta,
                                                                    uint32_t* __restrict__ order,
                                                                    uint32_t* __restrict__ rank_out)
{
    __builtin_amdgcn_s_setprio(3);   // (see sf_order_scan)
    order_scatter_chunk(blockIdx.x, threadIdx.x, cost, n, chunk_cnt,
                        chunk_off[blockIdx.x * SF_ORDER_BUCKETS + (threadIdx.x & (SF_ORDER_BUCKETS - 1u))],
                        order_meta[1], order_meta[2], order_meta[3], order, rank_out);
}

// The order rebuild of frames of many chunks in one-wave workgroups only (round 5): with frames in flight the
// persistent trace grids of the other frames refill every wave slot that frees, and sf_order_scan's 16-wave
// workgroup waited for 16 free slots on one CU -- 64 us median, up to 1.6 ms in the bench, its slot's next frame
// queued behind it (profiles/r5/order/). sf_order_bucket_scan: workgroup b (one wave) forms bucket b's per-chunk
// prefix over the chunks (lane l: chunks [l per, (l + 1) per)) and its total; sf_order_scatter_plan: every chunk's
// wave redoes the 32-lane plan (order_decide) from the totals and scatters its chunk.
extern "C" __global__ __launch_bounds__(64) void sf_order_bucket_scan(const uint32_t* __restrict__ chunk_cnt, uint32_t nc,
                                                                        uint32_t* __restrict__ chunk_rel,
                                                                        uint32_t* __restrict__ tot)
{
    __builtin_amdgcn_s_setprio(3);
    const uint32_t b = blockIdx.x, l = threadIdx.x;
    const uint32_t per = (nc + 63u) / 64u, c0 = l * per, c1 = min(nc, c0 + per);
    uint32_t s_ = 0u;
    for (uint32_t cb = c0; cb < c1; cb += SF_SCAN_BATCH) {
        uint32_t v[SF_SCAN_BATCH];
#pragma unroll
        for (int j = 0; j < SF_SCAN_BATCH; ++j) v[j] = cb + j < c1 ? chunk_cnt[(cb + j) * SF_ORDER_BUCKETS + b] : 0u;
#pragma unroll
        for (int j = 0; j < SF_SCAN_BATCH; ++j) s_ += v[j];
    }
    uint32_t incl = s_;   // inclusive prefix over the lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t up = (uint32_t)__shfl_up((int)incl, o, 64);
        incl += l >= (uint32_t)o ? up : 0u;
    }
    uint32_t off = incl - s_;
    for (uint32_t cb = c0; cb < c1; cb += SF_SCAN_BATCH) {
        uint32_t v[SF_SCAN_BATCH];
#pragma unroll
        for (int j = 0; j < SF_SCAN_BATCH; ++j) v[j] = cb + j < c1 ? chunk_cnt[(cb + j) * SF_ORDER_BUCKETS + b] : 0u;
#pragma unroll
        for (int j = 0; j < SF_SCAN_BATCH; ++j) {
            if (cb + j < c1) chunk_rel[(cb + j) * SF_ORDER_BUCKETS + b] = off;
            off += v[j];
        }
    }
    if (l == 63u) tot[b] = incl;
}

extern "C" __global__ __launch_bounds__(64) void sf_order_scatter_plan(const uint32_t* __restrict__ cost, uint32_t n,
                                                                         uint32_t* __restrict__ chunk_cnt,
                                                                         const uint32_t* __restrict__ chunk_rel,
                                                                         const uint32_t* __restrict__ tot,
                                                                         uint32_t split_buckets, uint32_t parts,
                                                                         uint32_t spare, uint32_t waves,
                                                                         uint32_t prio_buckets, uint32_t split_cap,
                                                                         uint32_t* __restrict__ order_meta,
                                                                         uint32_t* __restrict__ order)
{
    __builtin_amdgcn_s_setprio(3);
    const uint32_t l = threadIdx.x, c = blockIdx.x, bl = l & (SF_ORDER_BUCKETS - 1u);
    const uint32_t t = l < SF_ORDER_BUCKETS ? tot[l] : 0u;
    const uint32_t rel = chunk_rel[c * SF_ORDER_BUCKETS + bl];   // (in flight with the plan)
    const OrderPlan pl = order_decide(t, l, n, split_buckets, parts, spare, waves, prio_buckets, split_cap);
    const uint32_t pb = prio_buckets == 0u ? SF_ORDER_BUCKETS : (uint32_t)(pl.bp < 0 ? 0 : pl.bp);
    if (c == 0u && l == 0u) {
        order_meta[0] = pl.units;
        order_meta[1] = (uint32_t)pl.bs;
        order_meta[2] = parts;
        order_meta[3] = pb;
    }
    const uint32_t base = (uint32_t)__shfl((int)pl.X_excl, (int)bl, 64);
    const uint32_t offs = base + rel * ((int)bl >= pl.bs ? parts : 1u);
    order_scatter_chunk(c, l, cost, n, chunk_cnt, offs, (uint32_t)pl.bs, parts, pb, order, nullptr);
}

// Packed band slabs -> the frame G-buffer (multi-GPU gather). `stage` holds `members` slabs
// of members first .. first + members - 1 of a (band_rows, n) band split, each stage_rows x W float4
// (nx, ny, nz, minT) in the compact row order of sf_render_params.compact (member k's bands k, k + n, ...).
// Every pixel is rewritten at its frame position exactly as write_pixel would have: pos = (dir * t, 1) with
// dir recomputed by ray_dir from the same view (t < FLT_MAX: a hit; a miss leaves minT = FLT_MAX) or
// (0, 0, 0, 1), nrm = (n, 1). One thread per staged pixel, consecutive threads along a row: coalesced.
extern "C" __global__ __launch_bounds__(256) void sf_band_unpack(FrameArgs a, const float4* __restrict__ stage,
                                                                  uint32_t stage_rows, uint32_t band_rows, uint32_t n,
                                                                  uint32_t first, uint32_t members, uint32_t row0)
{
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    const uint32_t sr = row0 + blockIdx.y;            // slab row (launches of <= 65535 rows)
    const uint32_t m = blockIdx.z;                    // member first + m
    if (x >= a.W || m >= members) return;
    const uint32_t k = first + m, i = sr / band_rows, r = sr % band_rows;
    const uint32_t y = (i * n + k) * band_rows + r;   // frame row
    if (y >= a.H) return;                             // (rows past this member's slab)
    const float4 v = stage[((size_t)m * stage_rows + sr) * a.W + x];
    float dx, dy, dz;
    ray_dir(a, (float)x, (float)y, dx, dy, dz, a.consts->lut);
    const bool hit = v.w < FLT_MAX;
    const size_t o = (size_t)y * a.W + x;
    reinterpret_cast<float4*>(a.pos)[o] = hit ? make_float4(dx * v.w, dy * v.w, dz * v.w, 1.0f) : make_float4(0.f, 0.f, 0.f, 1.0f);
    reinterpret_cast<float4*>(a.nrm)[o] = make_float4(v.x, v.y, v.z, 1.0f);
}

// Heap index -> its path digits (child numbers), deepest first, 4 bits each, and its depth (the reference's heap
// numbering: child i of node n is 9 n + 1 + i, Sphereflake.h:162-172). Indices of depth <= SF_INDEX_SLAB_DEPTH.
__device__ __forceinline__ uint32_t heap_path(uint32_t n, uint64_t& path)
{
    uint32_t d = 0;
    path = 0;
    while (n) {
        const uint32_t q = (n - 1u) / 9u;
        path |= (uint64_t)(n - 1u - 9u * q) << (4u * d);
        n = q;
        ++d;
    }
    return d;
}

// The frames of every node of depth <= SF_NODE_TABLE_DEPTH under the view's root transform, for the index slab
// unpack: node n's 12 floats (xf layout of child_frame) as 3 float4. One thread per node, chained from the root
// with child_frame -- the same float values the traversal builds (its per-ray form is sf_trace_ray's chain).
extern "C" __global__ __launch_bounds__(256) void sf_node_table(FrameArgs a, float4* __restrict__ table, uint32_t nodes)
{
    const uint32_t n = blockIdx.x * 256u + threadIdx.x;
    if (n >= nodes) return;
    uint64_t path;
    const uint32_t d = heap_path(n, path);
    float xf[12], nx[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) xf[k] = a.root[k];
    for (uint32_t j = 0; j < d; ++j) {
        child_frame(a.consts, j, (uint32_t)(path >> (4u * (d - 1u - j))) & 15u, xf, nx);
#pragma unroll
        for (int k = 0; k < 12; ++k) xf[k] = nx[k];
    }
    table[3u * n + 0u] = make_float4(xf[0], xf[1], xf[2], xf[3]);
    table[3u * n + 1u] = make_float4(xf[4], xf[5], xf[6], xf[7]);
    table[3u * n + 2u] = make_float4(xf[8], xf[9], xf[10], xf[11]);
}

// Index slabs -> the frame G-buffer (multi-GPU gather at 4 B per pixel). `stage` holds `members`
// slabs of uint32 heap indices (SF_SLAB_MISS: no hit) laid out as sf_band_unpack's. A hit's pixel is rebuilt with
// the tracer's own operations: the sphere's frame from the node table (its ancestor at depth <= table_depth) and
// child_frame for the levels below, then the node's self test (Sphereflake.h:174-224: tca, d2, the near root with
// r_d^2) gives minT, and shade's position dir * minT and normal Normalize(position - centre). Coalesced 4-B reads
// along a slab row, 2 x 16-B writes per pixel.
// A grid of resident workgroups, each first copying into LDS the constants every pixel reads at a lane-dependent
// index -- the rsqrtps table (ray_dir, shade), the 9 unit child frames, the depth scales and self radii^2, the first
// heap index of each depth -- then taking 256-pixel segments (member, slab row, x / 256) G = gridDim.x apart.
// Round 6:
//  * two items deep: while item i is rebuilt, item i + G's node-table frame and item i + 2G's slab word are already
//    loading, and no memory operation sits under a branch. gfx9 counts loads and stores on one in-order counter
//    (vmcnt), so a load consumed after a store waits for that store too, and at a join of paths that issued different
//    memory operations the compiler waits for all of them: round 5's loop (a branch around each item's stores, the
//    miss branch) waited for its own stores before every item (`s_waitcnt vmcnt(0)` at the loop head). Here a lane
//    past the frame's width redoes the row's last pixel and an item past a member's slab redoes item 0 -- the same
//    inputs, so the same bits stored twice -- and a miss is rebuilt as the root with its outputs selected after;
//  * the depth of an index from its leading-zero count and one threshold compare (was ten compares), the correctly
//    rounded square root and x86 rsqrtps in their fast forms with a wave-uniform fallback to the general ones (never
//    taken on the views the tests and the bench render), the frame constants read once per launch.
#define SF_DEPTH_MSB_BITS 0x92491249u   // bit k set iff some depth's first heap index (9^d - 1) / 8 has its MSB at k

struct UnpackLds {
    uint32_t lut[2048];
    float child[9][16];
    float scale[SF_DEPTH_TABLE];
    float r2_self[SF_DEPTH_TABLE];
    uint32_t first[12];   // first[c] = (9^(c+1) - 1) / 8: the first heap index of depth c + 1 (first[11]: none)
};

// rsqrtps_x86 for a positive, normal, finite x: the table entry of (exponent parity, mantissa >> 13) less the
// exponent's half -- ((E - E0) / 2) << 23 with E0 = 127 or 128 of E's parity is (E + (E & 1) - 128) << 22
__device__ __forceinline__ float rsqrtps_pos(float x, const uint32_t* __restrict__ lut)
{
    const uint32_t b = __float_as_uint(x);
    const uint32_t E = b >> 23;
    return __uint_as_float(lut[(b >> 13) & 0x7ffu] - ((E + (E & 1u) - 128u) << 22));
}

// normalize3 (SIMD::Normalize) with rsqrtps_pos, falling back to rsqrtps_x86 for the whole wave when a live lane's
// length is zero, denormal, negative, infinite or NaN
__device__ __forceinline__ void normalize3_fast(float& x, float& y, float& z, const uint32_t* __restrict__ lut, bool live)
{
    const float len = (x * x + y * y) + z * z;
    float nr;
    if (wave_ballot(live && !(__float_as_uint(len) - 0x00800000u < 0x7f000000u)) != 0ull) nr = rsqrtps_x86(len, lut);
    else nr = rsqrtps_pos(len, lut);
    const float muls = (len * nr) * nr;
    const float s = (0.5f * nr) * (3.0f - muls);
    x = x * s;
    y = y * s;
    z = z * s;
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void sf_slab_unpack4(
    FrameArgs a, const uint32_t* __restrict__ stage, const float4* __restrict__ table, uint32_t table_depth,
    uint32_t stage_rows, uint32_t band_rows, uint32_t n, uint32_t first, uint32_t members)
{
    __shared__ UnpackLds S;
    const DeviceConsts* __restrict__ K = a.consts;
    {
        for (uint32_t i = threadIdx.x; i < 2048u; i += 256u) S.lut[i] = K->lut[i];
        if (threadIdx.x < 144u) S.child[threadIdx.x >> 4][threadIdx.x & 15u] = K->child[threadIdx.x >> 4][threadIdx.x & 15u];
        if (threadIdx.x < SF_DEPTH_TABLE) {
            S.scale[threadIdx.x] = K->dt.scale[threadIdx.x];
            S.r2_self[threadIdx.x] = K->dt.r2_self[threadIdx.x];
        }
        if (threadIdx.x < 12u) {
            uint32_t f = 1u;
            for (uint32_t k = 0; k < threadIdx.x; ++k) f = 9u * f + 1u;
            S.first[threadIdx.x] = threadIdx.x < 11u ? f : 0xffffffffu;
        }
    }
    // ray_dir's constants (uniform, read once; ray_dir reads them per call)
    const float rw = K->rw, rh = K->rh;
    const bool fast = K->fast_div != 0u;
    __syncthreads();
    const uint32_t segs = (a.W + 255u) >> 8;
    const uint32_t items = members * stage_rows * segs;   // (< 2^32: 16384^2 frames give 2^22)
    const uint32_t G = gridDim.x;
    const uint32_t lane_x = threadIdx.x;
    // item -> its frame row y, its slab row's first word and its segment's first x (uniform, in SGPRs: located once
    // per item); the lane's pixel is x = min(xb + lane, W - 1) -- past the width, the row's last pixel again
    struct Loc { uint32_t y, row, xb; };
    auto locate = [&](uint32_t it) -> Loc {
        const uint32_t seg = it % segs, rest = it / segs;
        const uint32_t sr = rest % stage_rows, m = rest / stage_rows;
        const uint32_t k = first + m, i = sr / band_rows, r = sr % band_rows;
        return Loc{ (i * n + k) * band_rows + r, (m * stage_rows + sr) * a.W, seg << 8 };
    };
    // item 0 has the lowest frame row of the launch: without it no item has a row
    const Loc l0 = locate(0u);
    if (l0.y >= a.H) return;
    // the item it rebuilds: it itself, or item 0 past the items or past a member's slab
    auto item = [&](uint32_t it) -> Loc {
        const Loc l = locate(it < items ? it : 0u);
        return it < items && l.y < a.H ? l : l0;
    };
    auto lane_px = [&](const Loc& l) -> uint32_t { return min(l.xb + lane_x, a.W - 1u); };
    // one item in flight: its location, slab word, and once prepared its depth, table depth, the child digits below
    // the table's depth (the deepest in the highest nibble, depth td + 1's in the lowest) and its ancestor's table frame
    struct Slot {
        Loc l;
        uint32_t idx, d, td, path;
        float4 f0, f1, f2;
    };
    auto prepare = [&](Slot& q) {
        const uint32_t e = q.idx < SF_SLAB_BAD ? q.idx : 0u;   // (a miss: the root, its outputs replaced)
        const uint32_t c = __builtin_popcount(SF_DEPTH_MSB_BITS & (0x7fffffffu >> __builtin_clz(e | 1u)));
        const uint32_t d = c + (e >= S.first[c] ? 1u : 0u);
        const uint32_t td = d < table_depth ? d : table_depth;
        uint32_t anc = e, p = 0u;
        for (uint32_t j = d; j > td; --j) {
            const uint32_t qq = (anc - 1u) / 9u;
            p = (p << 4) | (anc - 1u - 9u * qq);
            anc = qq;
        }
        q.d = d;
        q.td = td;
        q.path = p;
        q.f0 = table[3u * anc];
        q.f1 = table[3u * anc + 1u];
        q.f2 = table[3u * anc + 2u];
    };
    // item it in slot P (its frame loaded), item it + G in slot Q (its slab word loaded): Q's frame loads and item
    // it + 2G's slab word (into P, once P's item is written) go out first, then P's pixel is rebuilt and stored
    auto step = [&](Slot& P, Slot& Q, uint32_t it) {
        prepare(Q);
        const Loc l2 = item(it + 2u * G);
        const uint32_t idx2 = stage[l2.row + lane_px(l2)];

        const uint32_t px_ = lane_px(P.l), py_ = P.l.y;
        float dx, dy, dz;
        {   // ray_dir with the constants read above
            const float fx = (float)px_, fy = (float)py_;
            float u, v;
            if (fast) {
                const float qu = fx * rw, qv = fy * rh;
                u = __builtin_fmaf(__builtin_fmaf(-qu, a.fw, fx), rw, qu);
                v = __builtin_fmaf(__builtin_fmaf(-qv, a.fh, fy), rh, qv);
            } else {
                u = fx / a.fw;
                v = fy / a.fh;
            }
            dx = ((a.tl[0] + a.dh[0] * u) + a.dv[0] * v) - a.o[0];
            dy = ((a.tl[1] + a.dh[1] * u) + a.dv[1] * v) - a.o[1];
            dz = ((a.tl[2] + a.dh[2] * u) + a.dv[2] * v) - a.o[2];
            normalize3_fast(dx, dy, dz, S.lut, true);
        }
        const bool hit = P.idx < SF_SLAB_BAD;
        float xf[12] = { P.f0.x, P.f0.y, P.f0.z, P.f0.w, P.f1.x, P.f1.y, P.f1.z, P.f1.w, P.f2.x, P.f2.y, P.f2.z, P.f2.w };
        uint32_t path = P.path;
        // the frames down to the parent, then only the sphere's centre: child_frame's translation column (the same
        // operations on the same operands)
        for (uint32_t j = P.td; j + 1u < P.d; ++j) {
            float nf[12];
            child_frame(S.child, S.scale, j, path & 15u, xf, nf);
            path >>= 4;
#pragma unroll
            for (int q = 0; q < 12; ++q) xf[q] = nf[q];
        }
        float cx, cy, cz;
        {
            const float sc = S.scale[P.d > 0u ? P.d - 1u : 0u];
            const float* B = S.child[path & 15u] + 12;   // (path & 15 <= 8; 0 where the table holds the sphere)
            const float b0 = B[0] * sc, b1 = B[1] * sc, b2 = B[2] * sc, b3 = B[3];
            const float ex = __builtin_fmaf(xf[9], b3, (xf[0] * b0 + xf[3] * b1) + xf[6] * b2);   // (SF_AFFINE_FMA)
            const float ey = __builtin_fmaf(xf[10], b3, (xf[1] * b0 + xf[4] * b1) + xf[7] * b2);
            const float ez = __builtin_fmaf(xf[11], b3, (xf[2] * b0 + xf[5] * b1) + xf[8] * b2);
            const bool below = P.d > P.td;
            cx = below ? ex : xf[9];
            cy = below ? ey : xf[10];
            cz = below ? ez : xf[11];
        }
        const float tca = (cx * dx + cy * dy) + cz * dz;
        const float d2 = ((cx * cx + cy * cy) + cz * cz) - tca * tca;
        const float R2 = S.r2_self[P.d];
        const float xs = R2 - d2;
        float t;   // (a hit's own self test passed: xs >= 0)
        if (wave_ballot(hit && !(xs >= 0x1p-96f)) != 0ull) t = near_root(tca, d2, R2);
        else t = near_root_big(tca, xs);
        // shade (Sphereflake.h:218-224)
        const float px = dx * t, py = dy * t, pz = dz * t;
        float qx = px - cx, qy = py - cy, qz = pz - cz;
        normalize3_fast(qx, qy, qz, S.lut, hit);
        const float mv = P.idx == SF_SLAB_MISS ? 0.0f : __builtin_nanf("");   // (SF_SLAB_BAD: never made by a correct split)
        const size_t o = (size_t)py_ * a.W + px_;
        reinterpret_cast<float4*>(a.pos)[o] = hit ? make_float4(px, py, pz, 1.0f) : make_float4(mv, mv, mv, 1.0f);
        reinterpret_cast<float4*>(a.nrm)[o] = hit ? make_float4(qx, qy, qz, 1.0f) : make_float4(mv, mv, mv, 1.0f);
        P.l = l2;
        P.idx = idx2;
    };

    Slot A, B;
    A.l = item(blockIdx.x);
    A.idx = stage[A.l.row + lane_px(A.l)];
    B.l = item(blockIdx.x + G);
    B.idx = stage[B.l.row + lane_px(B.l)];
    prepare(A);
    // unrolled twice, so the two slots swap roles without register moves
    for (uint32_t it = blockIdx.x; it < items; it += 2u * G) {
        step(A, B, it);
        if (it + G >= items) break;
        step(B, A, it + G);
    }
}

extern "C" __global__ __launch_bounds__(64) void sf_fixup_wave(FrameArgs a, const uint32_t* overflow_list,
                                                               uint32_t* counters, uint32_t parity)
{
    extern __shared__ float lds[];
    if (blockIdx.x == 0 && threadIdx.x == 0) counters[parity ^ 1u] = 0u;
    const uint32_t n = counters[parity];
    // workgroups without a tile leave at once (the usual case: no tile flagged), before the LDS setup: this
    // kernel sits between a frame's trace and the next render of its slot
    if (blockIdx.x >= n) return;
    int32_t maxd = -1;
    float closest = FLT_MAX;
    uint32_t unresolved = 0u;
    stage_root(lds, a.root);
    const float4 bcol = build_column(a.consts);
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const TileStats st = trace_tile<true>(a, lds, bcol, overflow_list[i], SF_MAX_LEVELS, nullptr, nullptr);
        maxd = st.maxd > maxd ? st.maxd : maxd;
        closest = fminf(closest, st.closest);
        unresolved += st.overflowed ? 1u : 0u;
    }
    publish_stats(a, maxd, closest, unresolved);
}

// ------------------------------------------------------------------------------------------
// One thread per ray, private stack (Sphereflake.h:86-226 restated as an explicit DFS).
// ------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(256) void sf_trace_ray(FrameArgs a)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t tile = blockIdx.x * SF_WAVES_PER_BLOCK + (threadIdx.x >> 6);
    if (tile >= a.tiles_x * a.tile_rows) return;
    const DeviceConsts* __restrict__ K = a.consts;
    const uint32_t* __restrict__ lut = K->lut;
    const Tile t = tile_of(a, tile, lane);
    float dx, dy, dz;
    ray_dir(a, (float)t.x, (float)t.y, dx, dy, dz, lut);

    float xf[SF_MAX_LEVELS + 1][12];
    uint8_t cur[SF_MAX_LEVELS + 1];
#pragma unroll
    for (int k = 0; k < 12; ++k) xf[0][k] = a.root[k];

    HitState h;
    h.minT = FLT_MAX;
    h.cx = h.cy = h.cz = 0.f;
    h.index = 0xffffffffu;
    h.hit = false;
    int32_t maxd = -1;
    bool overflowed = false;

    auto make_child = [&](uint32_t p, uint32_t i) { child_frame(K, p, i, xf[p], xf[p + 1]); };

    if (t.valid) {
        uint32_t d = 0;
        uint64_t idx = 0;
        for (;;) {
            bool ex = false;
            {
                const float cx = xf[d][9], cy = xf[d][10], cz = xf[d][11];
                const float tca = (cx * dx + cy * dy) + cz * dz;
                const float d2 = ((cx * cx + cy * cy) + cz * cz) - tca * tca;
                const float R2b = K->dt.r2_bound[d];
                if (tca >= 0.0f && d2 <= R2b) ex = near_root(tca, d2, R2b) < K->dt.lod[d];
            }
            if (ex) {
                maxd = (int32_t)d > maxd ? (int32_t)d : maxd;
                if (d < SF_MAX_LEVELS) {
                    cur[d] = 0;
                    make_child(d, 0);
                    d += 1;
                    idx = 9u * idx + 1u;
                    continue;
                }
                overflowed = true;
            }
            bool finished = false;
            for (;;) {
                if (d == 0) { finished = true; break; }
                const uint32_t p = d - 1;
                if (cur[p] < 8) {
                    cur[p] += 1;
                    make_child(p, cur[p]);
                    idx += 1u;
                    break;
                }
                idx = (idx - 9u) / 9u;
                d = p;
                const float cx = xf[p][9], cy = xf[p][10], cz = xf[p][11];
                const float tca = (cx * dx + cy * dy) + cz * dz;
                const float d2 = ((cx * cx + cy * cy) + cz * cz) - tca * tca;
                const float R2s = K->dt.r2_self[p];
                if (tca >= 0.0f && d2 <= R2s) {
                    const float ts = near_root(tca, d2, R2s);
                    if (ts < h.minT) {
                        h.minT = ts;
                        h.cx = cx;
                        h.cy = cy;
                        h.cz = cz;
                        h.index = (uint32_t)idx;
                        h.hit = true;
                    }
                }
            }
            if (finished) break;
        }
        write_pixel(a, t, dx, dy, dz, h, lut);
    }
    // wave-level stats
    float closest = wave_min(t.valid ? h.minT : FLT_MAX);
    int32_t md = maxd;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) md = max(md, __shfl_xor(md, m, 64));
    const bool anyov = wave_ballot(overflowed) != 0;
    if (lane == 0u) {
        if (md >= 0) atomicMax(&a.stats[0], md);
        atomicMin(&a.stats[1], sf_float_key(closest));
        if (anyov) atomicAdd(&a.stats[2], 1);
    }
}

// ------------------------------------------------------------------------------------------
// Frame-less progressive mode (Sphereflake.cpp:86-214): random 8-ray packets.
// ------------------------------------------------------------------------------------------

// std::mt19937 continuation: state[0..623] + next index state[624]; writes n tempered 32-bit outputs
// (std::uniform_int_distribution<unsigned>(0) over the full range returns them unchanged).
// One workgroup. The twist runs as 227 independent chains: thread j < 227 makes words j, j + 227 and
// (j < 169) j + 454 of the new block, each from the old block and the chain's own previous word (the
// offset 397 - 624 = -227), in registers -- no barrier inside a twist, one between blocks (there were 3).
// Word 623 of a new block needs new words 0 and 396 (two chains): it is made lazily, in the next twist, by
// the two threads that use it (226: offset 397; 168: offset 1), from the old block's word 623 that the
// buffer being refilled still holds at index 623 (thread 226 writes it back for the twist after).
#define SF_MT_THREADS 256
extern "C" __global__ __launch_bounds__(SF_MT_THREADS) void sf_mt_draws(uint32_t* state, uint32_t* out, uint32_t n)
{
    __shared__ uint32_t buf[2][624];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < 624u; i += SF_MT_THREADS) buf[0][i] = state[i];
    const uint32_t pos0 = min(state[624], 624u);
    __syncthreads();
    auto f = [](uint32_t a, uint32_t b, uint32_t c) {
        const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
        return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    };
    auto temper = [](uint32_t y) {
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    };
    // the rest of the loaded (complete) block
    const uint32_t m0 = min(624u - pos0, n);
    for (uint32_t k = tid; k < m0; k += SF_MT_THREADS) out[k] = temper(buf[0][pos0 + k]);
    uint32_t done = m0;    // outputs written (uniform)
    uint32_t cur = 0;      // buffer of the newest block
    bool full = true;      // the newest block's word 623 is in the buffer (only the loaded block's)
    uint32_t pos = pos0 + m0;
    while (done < n) {
        const uint32_t* sb = buf[cur];
        uint32_t* tb = buf[cur ^ 1u];
        // output index of the new block's word 0: after the newest block's word 623 when that is still due
        const uint32_t o = done + (full ? 0u : 1u);
        if (tid < 227u) {
            const uint32_t j = tid;
            uint32_t x623 = 0u;   // the newest block's word 623 (threads 226 and 168)
            if (j == 226u || j == 168u) {
                x623 = full ? sb[623] : f(tb[623], sb[0], sb[396]);
                if (j == 226u && !full) {
                    buf[cur][623] = x623;                    // for the lazy word 623 of the block made now
                    if (done < n) out[done] = temper(x623);   // its place in the stream
                }
            }
            const uint32_t wa = f(sb[j], sb[j + 1u], j == 226u ? x623 : sb[j + 397u]);
            tb[j] = wa;
            if (o + j < n) out[o + j] = temper(wa);
            const uint32_t wb = f(sb[j + 227u], sb[j + 228u], wa);
            tb[j + 227u] = wb;
            if (o + j + 227u < n) out[o + j + 227u] = temper(wb);
            if (j < 168u || j == 168u) {
                const uint32_t wc = f(sb[j + 454u], j == 168u ? x623 : sb[j + 455u], wb);
                tb[j + 454u] = wc;
                if (o + j + 454u < n) out[o + j + 454u] = temper(wc);
            }
        }
        __syncthreads();
        done = min(n, o + 623u);   // words 0..622 of the new block (623 is due with the next twist)
        pos = done - o;
        cur ^= 1u;
        full = false;
    }
    // state: the newest block, its word 623 made now if it is lazy
    if (!full && tid == 0u) buf[cur][623] = f(buf[cur ^ 1u][623], buf[cur][0], buf[cur][396]);
    __syncthreads();
    for (uint32_t i = tid; i < 624u; i += SF_MT_THREADS) state[i] = buf[cur][i];
    if (tid == 0) state[624] = pos;
}

// ---- parallel mt19937 draws (jump-ahead; host side sf_mtjump.cpp). A batch's n draws: the r = 624 - pos still
// in the loaded buffer, then n - r "post-buffer" draws cut into K segments of L; segment j starts from the window
// V_{jL} = (t^{jL} mod phi)(A) V_0 (V_0 = the buffer), i.e. word k of it is the XOR of x_{i+k} over the set
// coefficients i of the polynomial -- a convolution of the raw sequence x (sf_mt_raw) split over P workgroups
// per segment (sf_mt_jump_partial), then each segment's workgroup XORs its P partial windows and generates its
// draws (sf_mt_segments). Same stream, bit for bit, as the sequential sf_mt_draws.
namespace {
__device__ __forceinline__ uint32_t mt_f(uint32_t a, uint32_t b, uint32_t c)
{
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y)
{
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
// One twist in LDS: nb = the block after ob (both 624 words); 227 threads run the chains (words j, j + 227,
// j + 454) and thread 0 also word 623 = f(ob[623], nb[0], nb[396]): nb[396] is thread 169's second word, which
// thread 0 forms again from ob (two more f) instead of waiting for it behind a barrier. Returns after ONE barrier
// (nb complete), with this thread's words in w[0..2] (w[3]: word 623 on thread 0) for callers that store them
// straight from registers. (Round 4: a barrier before word 623 and a second after it, and the callers re-read nb
// from LDS for their global stores: sf_mt_raw 16.8 us for 33 twists, profiles/r4/final3.)
__device__ __forceinline__ void mt_twist(const uint32_t* ob, uint32_t* nb, uint32_t w[4])
{
    const uint32_t j = threadIdx.x;
    if (j < 227u) {
        const uint32_t a = mt_f(ob[j], ob[j + 1u], ob[j + 397u]);
        nb[j] = a;
        const uint32_t b = mt_f(ob[j + 227u], ob[j + 228u], a);
        nb[j + 227u] = b;
        w[0] = a;
        w[1] = b;
        if (j < 169u) {
            w[2] = mt_f(ob[j + 454u], ob[j + 455u], b);
            nb[j + 454u] = w[2];
        }
        if (j == 0u) {
            const uint32_t a169 = mt_f(ob[169], ob[170], ob[566]);
            const uint32_t b169 = mt_f(ob[396], ob[397], a169);   // nb[396]
            w[3] = mt_f(ob[623], a, b169);
            nb[623] = w[3];
        }
    }
    __syncthreads();
}
}  // namespace

#define SF_MT_PAR_THREADS 256

// The raw sequence x_0..x_{nraw-1} from the state's buffer (x_0..x_623 = the buffer). One workgroup.
extern "C" __global__ __launch_bounds__(SF_MT_PAR_THREADS) void sf_mt_raw(const uint32_t* __restrict__ state,
                                                                           uint32_t* __restrict__ raw, uint32_t blocks)
{
    __shared__ uint32_t buf[2][624];
    for (uint32_t i = threadIdx.x; i < 624u; i += SF_MT_PAR_THREADS) {
        buf[0][i] = state[i];
        raw[i] = state[i];
    }
    __syncthreads();
    const uint32_t j = threadIdx.x;
    for (uint32_t b = 1; b < blocks; ++b) {
        uint32_t w[4];
        mt_twist(buf[(b - 1u) & 1u], buf[b & 1u], w);
        uint32_t* rb = raw + b * 624u;   // this thread's new words, from registers
        if (j < 227u) {
            rb[j] = w[0];
            rb[j + 227u] = w[1];
            if (j < 169u) rb[j + 454u] = w[2];
            if (j == 0u) rb[623] = w[3];
        }
    }
}

// Partial jumped windows: workgroup (s, p) XORs x_{i+k} (k < 624) over the set coefficients i of segment
// s + 1's polynomial within [p C, (p + 1) C), C = ceil(19937 / P); the raw words it needs are staged in LDS.
#define SF_MT_CHUNK ((19937u + SF_MT_PARTS - 1u) / SF_MT_PARTS)
extern "C" __global__ __launch_bounds__(SF_MT_PAR_THREADS) void sf_mt_jump_partial(const uint32_t* __restrict__ raw,
                                                                                    const uint64_t* __restrict__ polys,
                                                                                    uint32_t poly_words,
                                                                                    uint32_t* __restrict__ partial)
{
    // xs: the chunk's raw words, then 624 zeros that the unused slots of an unrolled batch read (XOR 0)
    __shared__ uint32_t xs[SF_MT_CHUNK + 624u + 624u];
    const uint32_t seg = blockIdx.x + 1u, part = blockIdx.y;   // segment 0 needs no jump
    const uint32_t i0 = part * SF_MT_CHUNK, i1 = min(19937u, i0 + SF_MT_CHUNK);
    const uint32_t nx = (i1 - i0) + 624u;
    for (uint32_t i = threadIdx.x; i < nx + 624u; i += SF_MT_PAR_THREADS) xs[i] = i < nx ? raw[i0 + i] : 0u;
    __syncthreads();
    const uint32_t k0 = threadIdx.x, k1 = k0 + 256u, k2 = k0 < 112u ? k0 + 512u : k0;   // window words (k2: 624 total; unused past 112)
    uint32_t a0 = 0u, a1 = 0u, a2 = 0u;
    const uint64_t* pl = polys + (size_t)seg * poly_words;
    for (uint32_t q = i0 >> 6; q <= (i1 - 1u) >> 6; ++q) {
        uint64_t bits = pl[q];   // (uniform)
        const uint32_t lo = q * 64u;
        if (lo < i0) bits &= ~0ull << (i0 - lo);
        if (lo + 64u > i1) bits &= (i1 - lo) >= 64u ? ~0ull : ((1ull << (i1 - lo)) - 1ull);
        // 8 coefficients per batch, their 24 LDS reads issued together (the zero block stands in for the
        // coefficients past the word's last set bit): the loop is LDS-latency bound otherwise
        while (bits) {
            uint32_t ix[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                ix[u] = bits ? lo + (uint32_t)__builtin_ctzll(bits) - i0 : nx;
                bits &= bits - 1ull;
            }
            uint32_t v0[8], v1[8], v2[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                v0[u] = xs[ix[u] + k0];
                v1[u] = xs[ix[u] + k1];
                v2[u] = xs[ix[u] + k2];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                a0 ^= v0[u];
                a1 ^= v1[u];
                a2 ^= v2[u];
            }
        }
    }
    uint32_t* out = partial + ((size_t)blockIdx.x * SF_MT_PARTS + part) * 624u;
    out[k0] = a0;
    out[k1] = a1;
    if (k0 < 112u) out[k0 + 512u] = a2;
}

// Segment j of the batch's n draws: workgroup j builds its window (segment 0: the buffer; others: the XOR of
// their partial windows), then twists and tempers its L post-buffer draws; workgroup 0 also emits the r draws
// left in the buffer. The workgroup holding the last draw stores the generator state after the batch
// (libstdc++ layout) into state_out -- not into `state`, which the other workgroups may still be reading.
extern "C" __global__ __launch_bounds__(SF_MT_PAR_THREADS) void sf_mt_segments(const uint32_t* __restrict__ state,
                                                                                const uint32_t* __restrict__ partial,
                                                                                uint32_t L, uint32_t n,
                                                                                uint32_t* __restrict__ out,
                                                                                uint32_t* __restrict__ state_out)
{
    __shared__ uint32_t buf[2][624];
    const uint32_t j = blockIdx.x, tid = threadIdx.x;
    const uint32_t pos = min(state[624], 624u);
    const uint32_t r = min(624u - pos, n);            // draws still in the buffer
    const uint32_t m = n - r;                         // post-buffer draws
    const uint32_t s0 = j * L;
    if (j == 0u)
        for (uint32_t i = tid; i < r; i += SF_MT_PAR_THREADS) out[i] = mt_temper(state[pos + i]);
    if (m == 0u) {   // the batch ends inside the buffer
        if (j == 0u) {
            for (uint32_t k = tid; k < 624u; k += SF_MT_PAR_THREADS) state_out[k] = state[k];
            if (tid == 0u) state_out[624] = pos + n;
        }
        return;
    }
    if (s0 >= m) return;   // (workgroup-uniform)
    const uint32_t cnt = min(L, m - s0);
    for (uint32_t k = tid; k < 624u; k += SF_MT_PAR_THREADS) {
        uint32_t w;
        if (j == 0u) {
            w = state[k];
        } else {
            const uint32_t* pp = partial + (size_t)(j - 1u) * SF_MT_PARTS * 624u + k;
            w = 0u;
#pragma unroll
            for (uint32_t p = 0; p < SF_MT_PARTS; ++p) w ^= pp[(size_t)p * 624u];
        }
        buf[0][k] = w;
    }
    __syncthreads();
    uint32_t cur = 0, done = 0;
    while (done < cnt) {
        uint32_t w[4];
        mt_twist(buf[cur], buf[cur ^ 1u], w);
        cur ^= 1u;
        const uint32_t take = min(624u, cnt - done);
        uint32_t* ob = out + r + s0 + done;   // this thread's new words, tempered from registers
        if (tid < 227u) {
            if (tid < take) ob[tid] = mt_temper(w[0]);
            if (tid + 227u < take) ob[tid + 227u] = mt_temper(w[1]);
            if (tid < 169u && tid + 454u < take) ob[tid + 454u] = mt_temper(w[2]);
            if (tid == 0u && 623u < take) ob[623] = mt_temper(w[3]);
        }
        done += take;
    }
    if (s0 + cnt == m) {   // the last draw of the batch: the state for the next batch
        for (uint32_t k = tid; k < 624u; k += SF_MT_PAR_THREADS) state_out[k] = buf[cur][k];
        if (tid == 0u) state_out[624] = ((cnt - 1u) % 624u) + 1u;
    }
}

namespace {
// Sobol::Sample (Sobol.cpp:41-55) for dims 0/1.
__device__ __forceinline__ float sobol_sample(uint64_t index, const uint32_t* __restrict__ m, uint32_t scramble)
{
    uint32_t r = scramble;
    for (uint32_t i = 0; index; index >>= 1, ++i)
        if (index & 1u) r ^= m[i];
    return (float)r * (1.f / 4294967296.0f);
}
}  // namespace

// Trace `packets` packets: one 8-lane group per packet, 8 packets per wave. Lane q of packet j uses
// the footprint of Sphereflake.cpp:143-147 around (x0, y0) drawn at Sobol index counter0 + j with
// scrambles draws[2j], draws[2j+1] (Sphereflake.cpp:139-141). Results are staged per lane; the
// owner word of each pixel keeps the highest ticket, so the scatter reproduces sequential order.
// One wave = 64 / PW packets of PW lanes (Sphereflake.cpp:115-160): the AVX footprint is 8 pixels
// around (x0, y0) = 1 + floor(S (W - 2)), 1 + floor(S (H - 2)); the SSE footprint the 2x2 block at
// (x0, y0) = floor(S (W - 1)), floor(S (H - 1)).
template <int PW>
__device__ __forceinline__ void packet_origin(const FrameArgs& a, const DeviceConsts* __restrict__ K,
                                              const uint32_t* draws, uint64_t counter0, uint32_t packet,
                                              float& x0, float& y0)
{
    const uint64_t c = counter0 + packet;
    const float s0 = sobol_sample(c, K->sobol[0], draws[2u * packet]);
    const float s1 = sobol_sample(c, K->sobol[1], draws[2u * packet + 1u]);
    if constexpr (PW == 8) {
        x0 = 1.0f + floorf(s0 * (float)(a.W - 2u));
        y0 = 1.0f + floorf(s1 * (float)(a.H - 2u));
    } else {
        x0 = floorf(s0 * (float)(a.W - 1u));
        y0 = floorf(s1 * (float)(a.H - 1u));
    }
}

// Spatial binning of a batch's packets (the trace order only: results, tickets and the scatter are
// per packet). The reference's packets land uniformly at random, so a wave of 64 / PW consecutive
// packets shares almost no traversal; binned by a square of 2^bin_shift pixels around (x0, y0) they
// share most of it. Counting sort: sf_packet_bin (histogram), sf_packet_scan (exclusive offsets,
// one workgroup), sf_packet_place (slot by atomic cursor; order inside a bin is arbitrary).
template <int PW>
__device__ __forceinline__ uint32_t packet_bin(const FrameArgs& a, const DeviceConsts* __restrict__ K,
                                               const uint32_t* draws, uint64_t counter0, uint32_t packet,
                                               uint32_t bin_shift, uint32_t bins_x)
{
    float x0, y0;
    packet_origin<PW>(a, K, draws, counter0, packet, x0, y0);
    return ((uint32_t)y0 >> bin_shift) * bins_x + ((uint32_t)x0 >> bin_shift);
}

extern "C" __global__ __launch_bounds__(256) void sf_packet_bin(FrameArgs a, const uint32_t* draws, uint64_t counter0,
                                                                 uint32_t packets, uint32_t pw, uint32_t bin_shift,
                                                                 uint32_t bins_x, uint32_t* bin_cnt)
{
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= packets) return;
    const uint32_t b = pw == 8u ? packet_bin<8>(a, a.consts, draws, counter0, p, bin_shift, bins_x)
                                : packet_bin<4>(a, a.consts, draws, counter0, p, bin_shift, bins_x);
    atomicAdd(bin_cnt + b, 1u);
}

extern "C" __global__ __launch_bounds__(1024) void sf_packet_scan(uint32_t* bin_cnt, uint32_t nbins,
                                                                  const uint32_t* __restrict__ rank)
{
    // Counts -> exclusive offsets in place (the place cursors), the bins taken in the order rank[]
    // (heaviest first, from the last batch's per-bin wave cycles) or in index order (rank NULL). Staged
    // through LDS (at the bin's rank) so that global reads and writes are coalesced; thread t scans
    // ranks [t * per, (t + 1) * per) of the staged copy (index padded by 1 per 32 against bank conflicts).
    __shared__ uint32_t cnt[SF_PROG_MAX_BINS + SF_PROG_MAX_BINS / 32u];
    __shared__ uint32_t part[16];
    const uint32_t t = threadIdx.x, per = (nbins + 1023u) / 1024u, b0 = t * per, b1 = min(nbins, b0 + per);
    for (uint32_t i = t; i < nbins; i += 1024u) {
        const uint32_t r = rank ? rank[i] : i;
        cnt[r + (r >> 5)] = bin_cnt[i];
    }
    __syncthreads();
    uint32_t s_ = 0u;
    for (uint32_t b = b0; b < b1; ++b) s_ += cnt[b + (b >> 5)];
    // exclusive scan of the 1024 partials: in-wave shuffles, then the 16 wave totals
    const uint32_t lane = t & 63u, w = t >> 6;
    uint32_t x = s_;
#pragma unroll
    for (uint32_t o = 1u; o < 64u; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        x += lane >= o ? y : 0u;
    }
    if (lane == 63u) part[w] = x;
    __syncthreads();
    if (t == 0u) {
        uint32_t acc = 0u;
        for (uint32_t k = 0; k < 16u; ++k) {
            const uint32_t y = part[k];
            part[k] = acc;
            acc += y;
        }
    }
    __syncthreads();
    uint32_t off = part[w] + x - s_;
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t c = cnt[b + (b >> 5)];
        cnt[b + (b >> 5)] = off;
        off += c;
    }
    __syncthreads();
    for (uint32_t i = t; i < nbins; i += 1024u) {
        const uint32_t r = rank ? rank[i] : i;
        bin_cnt[i] = cnt[r + (r >> 5)];
    }
}

// Frame-less heavy-first order: per 64-bin chunk, the cost-bucket histogram of the bins' last recorded
// wave cycles (input of sf_order_scan / sf_order_scatter, which then rank the bins heaviest first).
extern "C" __global__ __launch_bounds__(64) void sf_bin_hist(const uint32_t* __restrict__ bin_cost, uint32_t nbins,
                                                             uint32_t* __restrict__ chunk_cnt)
{
    const uint32_t c = blockIdx.x, lane = threadIdx.x, i = c * 64u + lane;
    const uint32_t bk = i < nbins ? cost_bucket(bin_cost[i]) : SF_ORDER_BUCKETS;
    uint32_t mine = 0u;
#pragma unroll 1
    for (uint32_t b = 0; b < SF_ORDER_BUCKETS; ++b) {
        const uint32_t n = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(bk == b));
        mine = lane == b ? n : mine;
    }
    if (lane < SF_ORDER_BUCKETS) chunk_cnt[c * SF_ORDER_BUCKETS + lane] = mine;
}

extern "C" __global__ __launch_bounds__(256) void sf_packet_place(FrameArgs a, const uint32_t* draws, uint64_t counter0,
                                                                   uint32_t packets, uint32_t pw, uint32_t bin_shift,
                                                                   uint32_t bins_x, uint32_t* bin_cur, uint32_t* perm)
{
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= packets) return;
    const uint32_t b = pw == 8u ? packet_bin<8>(a, a.consts, draws, counter0, p, bin_shift, bins_x)
                                : packet_bin<4>(a, a.consts, draws, counter0, p, bin_shift, bins_x);
    perm[atomicAdd(bin_cur + b, 1u)] = p;
}

template <int PW>
__device__ __forceinline__ void progressive_trace(const FrameArgs& a, const uint32_t* draws, uint64_t counter0,
                                                  uint32_t packets, uint64_t ticket0, PacketLane* lanes,
                                                  unsigned long long* owner, const uint32_t* perm, uint32_t wave,
                                                  uint32_t levels, uint32_t* ovf_list, uint32_t* ovf_cnt)
{
    extern __shared__ float lds[];
    constexpr uint32_t PPW = 64u / PW;   // packets per wave
    const DeviceConsts* __restrict__ K = a.consts;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t slot = wave * PPW + lane / PW;   // position in the (binned) trace order
    if (wave * PPW >= packets) return;   // wave-uniform
    const uint64_t w_start = (a.flags & SF_FLAG_DIAG_UNITS) ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const uint64_t c_start = a.bin_cost ? __builtin_amdgcn_s_memtime() : 0ull;
    const bool valid = slot < packets;
    const uint32_t packet = valid ? (perm ? perm[slot] : slot) : slot;
    const uint32_t q = lane % PW;
    float x0 = 0.f, y0 = 0.f;
    if (valid) packet_origin<PW>(a, K, draws, counter0, packet, x0, y0);
    float ox, oy;
    if constexpr (PW == 8) {
        // xa = {x0, x0+1, x0+1, x0, x0, x0+1, x0-1, x0-1}, ya = {y0, y0+1, y0, y0+1, y0-1, y0-1, y0, y0-1}
        ox = (q == 1u || q == 2u || q == 5u) ? 1.0f : (q >= 6u ? -1.0f : 0.0f);
        oy = (q == 1u || q == 3u) ? 1.0f : ((q == 4u || q == 5u || q == 7u) ? -1.0f : 0.0f);
    } else {
        // xa = {x0, x0+1, x0, x0+1}, ya = {y0, y0, y0+1, y0+1}
        ox = (q & 1u) ? 1.0f : 0.0f;
        oy = (q & 2u) ? 1.0f : 0.0f;
    }
    const float xf = x0 + ox, yf = y0 + oy;
    float dx, dy, dz;
    ray_dir(a, xf, yf, dx, dy, dz, K->lut);

    HitState h;
    int32_t maxd = -1;
    uint32_t status = 0u;
    stage_root(lds, a.root);
    traverse<PW>(K, a.root, lds, build_column(K), levels, dx, dy, dz, valid, h, maxd, status, a.flags);
    const bool overflowed = (status & SF_STATUS_OVERFLOW) != 0u;

    PacketLane out;
    shade(dx, dy, dz, h, K->lut, out.px, out.py, out.pz, out.nx, out.ny, out.nz);
    out.min_t = h.minT;
    // idx = (size_t)xa + (size_t)ya * W; the reference skips idx > size (Sphereflake.cpp:188-191)
    const uint64_t pix = (uint64_t)xf + (uint64_t)yf * a.W;
    const bool inb = valid && pix < (uint64_t)a.W * a.H;
    out.pixel = inb ? (uint32_t)pix : 0xffffffffu;
    if (valid) lanes[(size_t)packet * PW + q] = out;
    if (inb && !(a.flags & SF_FLAG_DIAG_NO_OWNER)) atomicMax(owner + pix, (unsigned long long)(ticket0 + packet));

    const float closest = wave_min(inb ? h.minT : FLT_MAX);
    const bool anyov = wave_ballot(overflowed) != 0ull;
    if (lane == 0u) {   // read before the atomic: issued only when it changes the word (one address)
        const int32_t key = sf_float_key(closest);
        const int32_t cur_d = __hip_atomic_load(&a.stats[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int32_t cur_k = __hip_atomic_load(&a.stats[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (maxd > cur_d) atomicMax(&a.stats[0], maxd);
        if (key < cur_k) atomicMin(&a.stats[1], key);
        if (anyov && !ovf_list) atomicAdd(&a.stats[2], 1);
    }
    // adaptive levels: a wave that needed more is re-traced whole by sf_progressive_fixup (its partial
    // lanes, owner words and stats are all superseded or implied by the complete traversal)
    if (anyov && ovf_list) {
        const uint32_t k = wave_fetch_add(ovf_cnt, 1u);
        ovf_list[k] = wave;   // uniform value and address
    }
    if (a.bin_cost && perm) {
        // scheduling hint for the next batch (sf_bin_hist): this wave's cycles, for the bin of its first
        // packet (uniform value and address; bins with several waves keep the last one's)
        const uint64_t cyc = __builtin_amdgcn_s_memtime() - c_start;
        const uint32_t p0 = __builtin_amdgcn_readfirstlane(perm[wave * PPW]);
        const uint32_t b = __builtin_amdgcn_readfirstlane(
            packet_bin<PW>(a, K, draws, counter0, p0, a.bin_shift, a.bins_x));
        // quantised to a power of 4: cost classes two octaves wide, so that bins of one class keep their
        // index (screen) order and a wave straddling two bins still gets spatial neighbours
        const uint32_t c32 = cyc > 0x7fffffffull ? 0x7fffffffu : ((uint32_t)cyc | 1u);
        a.bin_cost[b] = 1u << ((31u - (uint32_t)__builtin_clz(c32)) & ~1u);
    }
    if ((a.flags & SF_FLAG_DIAG_UNITS) && a.tile_trace && wave < SF_DIAG_WAVES) {   // diagnostics: this wave's
        // {start, end}, in the per-wave records of the context's trace buffer (sf_set_tile_trace)
        uint64_t* wt = a.tile_trace + (SF_TRACE_WORDS((uint64_t)((a.W + 7u) / 8u) * ((a.H + 7u) / 8u)) - 2u * SF_DIAG_WAVES);
        wt[2u * wave] = w_start;
        wt[2u * wave + 1u] = __builtin_amdgcn_s_memrealtime();
    }
}

template <int PW>
__device__ __forceinline__ void progressive_fixup(const FrameArgs& a, const uint32_t* draws, uint64_t counter0,
                                                  uint32_t packets, uint64_t ticket0, PacketLane* lanes,
                                                  unsigned long long* owner, const uint32_t* perm,
                                                  const uint32_t* ovf_list, uint32_t* counters, uint32_t parity)
{
    if (blockIdx.x == 0 && threadIdx.x == 0) counters[parity ^ 1u] = 0u;   // the next batch's list
    const uint32_t n = counters[parity];
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x)
        progressive_trace<PW>(a, draws, counter0, packets, ticket0, lanes, owner, perm,
                              __builtin_amdgcn_readfirstlane(ovf_list[i]),
                              SF_PROGRESSIVE_LEVELS, nullptr, nullptr);
}

extern "C" __global__ __launch_bounds__(64) void sf_progressive_trace(FrameArgs a, const uint32_t* draws,
                                                                       uint64_t counter0, uint32_t packets,
                                                                       uint64_t ticket0, PacketLane* lanes,
                                                                       unsigned long long* owner, const uint32_t* perm,
                                                                       uint32_t levels, uint32_t* ovf_list,
                                                                       uint32_t* ovf_cnt)
{
    progressive_trace<8>(a, draws, counter0, packets, ticket0, lanes, owner, perm, blockIdx.x, levels, ovf_list,
                         ovf_cnt);
}
extern "C" __global__ __launch_bounds__(64) void sf_progressive_trace_sse(FrameArgs a, const uint32_t* draws,
                                                                           uint64_t counter0, uint32_t packets,
                                                                           uint64_t ticket0, PacketLane* lanes,
                                                                           unsigned long long* owner, const uint32_t* perm,
                                                                           uint32_t levels, uint32_t* ovf_list,
                                                                           uint32_t* ovf_cnt)
{
    progressive_trace<4>(a, draws, counter0, packets, ticket0, lanes, owner, perm, blockIdx.x, levels, ovf_list,
                         ovf_cnt);
}
extern "C" __global__ __launch_bounds__(64) void sf_progressive_fixup(FrameArgs a, const uint32_t* draws,
                                                                       uint64_t counter0, uint32_t packets,
                                                                       uint64_t ticket0, PacketLane* lanes,
                                                                       unsigned long long* owner, const uint32_t* perm,
                                                                       const uint32_t* ovf_list, uint32_t* counters,
                                                                       uint32_t parity)
{
    progressive_fixup<8>(a, draws, counter0, packets, ticket0, lanes, owner, perm, ovf_list, counters, parity);
}
extern "C" __global__ __launch_bounds__(64) void sf_progressive_fixup_sse(FrameArgs a, const uint32_t* draws,
                                                                           uint64_t counter0, uint32_t packets,
                                                                           uint64_t ticket0, PacketLane* lanes,
                                                                           unsigned long long* owner,
                                                                           const uint32_t* perm,
                                                                           const uint32_t* ovf_list,
                                                                           uint32_t* counters, uint32_t parity)
{
    progressive_fixup<4>(a, draws, counter0, packets, ticket0, lanes, owner, perm, ovf_list, counters, parity);
}

// Last writer wins by ticket (= the reference worker's sequential packet order).
extern "C" __global__ __launch_bounds__(256) void sf_progressive_scatter(FrameArgs a, uint32_t packets, uint64_t ticket0,
                                                                         const PacketLane* lanes,
                                                                         const unsigned long long* owner)
{
    const uint32_t pl = a.packet_lanes;   // lanes per packet (8 AVX, 4 SSE)
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= packets * pl) return;
    const PacketLane l = lanes[i];
    if (l.pixel == 0xffffffffu) return;
    if (owner[l.pixel] != (unsigned long long)(ticket0 + i / pl)) return;
    reinterpret_cast<float4*>(a.pos)[l.pixel] = make_float4(l.px, l.py, l.pz, 1.0f);
    reinterpret_cast<float4*>(a.nrm)[l.pixel] = make_float4(l.nx, l.ny, l.nz, 1.0f);
    if (a.emit_aux && a.min_t) a.min_t[l.pixel] = l.min_t;
}
