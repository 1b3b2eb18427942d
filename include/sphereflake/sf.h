/*
 * sf.h -- C ABI of the MI355X (gfx950) Sphereflake primary-ray G-buffer renderer.
 *
 * This is the drop-in boundary for the reference hot path. The reference has no
 * FFI: its boundary is the C++ class SphereflakeRaytracer::Sphereflake
 * (/root/reference/sphereflake/Sphereflake.h:13-58). Each entry point below names
 * the member of that class (or the reference code) it replaces; the C++ class of
 * the same name and surface, layered on this ABI, is
 * sphereflake-raytracer_amd/csrc/Sphereflake.hpp.
 *
 * Conventions
 *   - Every call returns 0 on success and a negative SF_E* code on failure
 *     (sf_strerror() names it). HIP runtime errors map to SF_EHIP; the HIP code
 *     is kept in the context (sf_last_hip_error()).
 *   - The caller owns host buffers; the context owns its device buffers.
 *   - One context per device per host thread. Calls are stream-ordered on the
 *     context stream (or params->stream); sf_download() synchronises. Calls on
 *     different streams of one context run in call order; a caller's stream is
 *     not touched after the call that used it returns (it may be destroyed once
 *     its work is done).
 *   - G-buffer layout is the reference's: float4 (x, y, z, 1) per pixel,
 *     row-major x + y*W, y = 0 is the TOP edge (Sphereflake.cpp:186-196). Misses
 *     are (0, 0, 0, 1), so the GL SSAO post-process consumes it unchanged
 *     (Shaders/post_final.glsl:20, post_ssao.glsl:33).
 *   - Arithmetic is IEEE binary32 reproducing the reference AVX path bit for bit
 *     (per-ray semantics).
 */
#ifndef SPHEREFLAKE_SF_H
#define SPHEREFLAKE_SF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SF_ABI_VERSION 1

enum sf_status {
    SF_OK = 0,
    SF_EINVAL = -1,      /* bad argument (null pointer, zero size, out-of-range band) */
    SF_ENOMEM = -2,      /* device or host allocation failed */
    SF_EHIP = -3,        /* HIP runtime error (see sf_last_hip_error) */
    SF_ENODEV = -4,      /* no such device / not a gfx950 device */
    SF_ENOVIEW = -5,     /* sf_render before sf_set_view */
    SF_EDEPTH = -6,      /* traversal exceeded SF_MAX_DEPTH_LIMIT levels */
    SF_ESTATE = -7,      /* call not valid in the current state (e.g. progressive mode running) */
    SF_ECOMM = -8        /* RCCL error (see sf_dist_last_error) */
};

/* Traversal kernels. */
enum sf_kernel {
    SF_KERNEL_WAVE = 0,      /* default: wave-coherent traversal, one 8x8 pixel tile per wave64,
                                child transforms built cooperatively into LDS */
    SF_KERNEL_PER_RAY = 1    /* one thread per ray, private traversal stack */
};

#define SF_MAX_DEPTH_LIMIT 31   /* traversal levels (expanding depths 0..30) the kernels support */

typedef struct sf_ctx sf_ctx;

/* Per-render options. Zero-initialise and set what you need. */
typedef struct sf_render_params {
    /* Row sharding for multi-GPU. The frame is cut into bands of
       band_rows rows (must be a multiple of 8; 0 = one band = whole frame); this call
       renders the bands b with b % band_count == band_index (band_count 0 or 1 = all). */
    uint32_t band_rows;
    uint32_t band_count;
    uint32_t band_index;
    /* 1: write only the owned bands, packed contiguously (a "slab": band k of this
       rank at rows [k*band_rows, (k+1)*band_rows)); 0: write at frame positions. */
    uint32_t compact;
    uint32_t kernel;          /* enum sf_kernel */
    uint32_t emit_aux;        /* 1: also write minT (float) and hit index (uint32) channels */
    uint32_t max_depth;       /* traversal stack levels to provision (0 = auto: 12, retried at
                                 SF_MAX_DEPTH_LIMIT if a tile needs more) */
    uint32_t packed;          /* band slab formats of the multi-GPU gather (wave kernel only; nrm4 unused):
                                 1: ONE float4 (nx, ny, nz, minT) per pixel into pos4, 16 B/pixel instead of 32;
                                    the receiver forms the position dir * minT bit for bit (sf_unpack_slabs);
                                 2: ONE uint32 per pixel into pos4: the hit sphere's heap index (9n+1+i,
                                    0xffffffff = miss), 4 B/pixel; the receiver rebuilds the sphere's frame, the
                                    self test's minT, position and normal bit for bit. Only where sf_slab_bytes()
                                    is 4 for the view (else SF_EINVAL) */
    void* stream;             /* hipStream_t to launch on; NULL = the context stream */
} sf_render_params;

/* Frame statistics; mirrors Sphereflake::GetMaxDepthReached / GetRaysPerSecond /
   GetClosestSphereDistance (Sphereflake.h:30-58). Accumulated over renders until reset. */
typedef struct sf_stats {
    int32_t max_depth;        /* deepest node that passed bounding + LOD (Sphereflake.h:157-160) */
    float closest;            /* min minT over rays (FLT_MAX if none; may be negative) */
    int64_t rays;             /* rays traced */
    int64_t overflow_tiles;   /* tiles re-rendered because they needed a deeper stack */
} sf_stats;

/* --- lifetime ------------------------------------------------------------ */

/* Replaces Sphereflake::Sphereflake(width, height) (Sphereflake.cpp:43-55): allocates the
   device G-buffer (2 x W*H float4, zeroed like glm's vec4() default) and the aux channels,
   computes the 9 child transforms (ComputeChildTransformations, Sphereflake.cpp:216-249). */
int sf_create(int device, uint32_t width, uint32_t height, sf_ctx** out);

/* Replaces Sphereflake::~Sphereflake (Sphereflake.cpp:57-65). */
void sf_destroy(sf_ctx* ctx);

/* --- view and setup ------------------------------------------------------ */

/* Replaces Sphereflake::SetView (Sphereflake.cpp:76-84): stores the ray origin and image-plane
   corners; root transform = translate(-origin) * CreateRotationMatrix((90,0,0)). */
int sf_set_view(sf_ctx* ctx, const float origin[3], const float top_left[3],
                const float top_right[3], const float bottom_left[3]);

/* Override the host-computed setup constants (root transform and 9 unit child frames,
   glm column-major 4x4). For parity tests against fixture dumps. The child frames must be affine
   (row 3 exactly 0, 0, 0, 1, as Sphereflake.cpp:216-249 makes them): SF_EINVAL otherwise. */
int sf_set_setup(sf_ctx* ctx, const float child[9][16], const float root[16]);

/* Read back the setup constants currently in use. */
int sf_get_setup(const sf_ctx* ctx, float child[9][16], float root[16]);

/* --- rendering ----------------------------------------------------------- */

/* One full-frame (or banded) render into the context's device G-buffer. Replaces the
   std::thread sampling loop Sphereflake::DoImagePart (Sphereflake.cpp:86-214) with a
   deterministic frame. params may be NULL (defaults). Asynchronous on the stream. */
int sf_render(sf_ctx* ctx, const sf_render_params* params);

/* Same, into caller-owned DEVICE buffers (e.g. torch tensors): pos4/nrm4 are float4 arrays
   of rows*W elements, where rows = H (compact = 0) or the slab height (compact = 1);
   min_t / hit_index may be NULL. */
int sf_render_to(sf_ctx* ctx, const sf_render_params* params, float* pos4, float* nrm4,
                 float* min_t, uint32_t* hit_index);

/* Several frames in ONE persistent launch (round 6): frame k is ctxs[k]'s current view, rendered into ctxs[k]'s
   G-buffer and stats exactly as sf_render(ctxs[k], params) would (bit for bit), but one resident grid takes the
   work units of all n frames from one set of tile queues -- a wave whose frame runs dry goes on with the next
   frame's units, and the heaviest tiles of every frame start first -- instead of n launches each ending on its
   own heaviest tiles. For frames of a camera path rendered ahead (the reference's workers trace continuously,
   Sphereflake.cpp:67-74; bench.py's frames in flight). n <= SF_RENDER_FRAMES_MAX contexts on one device, of
   one frame size, each with a view. Launched on params->stream or ctxs[0]'s stream, ordered after every
   context's earlier work; every context's later calls are ordered after it. params: as sf_render, but whole
   frames or bands at frame positions only (compact / packed / per-ray kernel / max_depth: SF_EINVAL). Where the
   batch cannot take one launch (levels not proven for some view, diagnostics on, the subtree-split or
   compaction kernels), the frames are rendered one launch each, with the same results. */
#define SF_RENDER_FRAMES_MAX 8
int sf_render_frames(sf_ctx* const* ctxs, uint32_t n, const sf_render_params* params);

/* Rows of the slab a (band_rows, band_count, band_index) shard owns (compact layout). */
uint32_t sf_slab_rows(uint32_t height, uint32_t band_rows, uint32_t band_count, uint32_t band_index);

/* Bytes per pixel of the smallest lossless band slab for the context's current view: 4 (params.packed = 2, the
   hit index) when the view proves every hit at depth <= 10 -- heap indices below 2^32 --, else 16 (packed = 1);
   0 before sf_set_view. A pure function of the view: every rank of a split computes the same value. */
uint32_t sf_slab_bytes(const sf_ctx* ctx);

/* The receiving end of a banded frame, either slab format: `stage` (device) holds the packed compact slabs of
   members first_member .. first_member + members - 1 of a (band_rows, band_count) split, each stage_rows x W
   pixels of bytes_per_pixel (16: packed = 1, 4: packed = 2) bytes; every pixel is written to the context's G-buffer
   at its frame position, bit for bit what an unbanded render writes (recomputed from the context's current view:
   call it with the view the slabs were traced with). stage_rows must hold every member's slab (SF_EINVAL
   otherwise). Asynchronous on `stream`. */
int sf_unpack_slabs(sf_ctx* ctx, const void* stage, uint32_t bytes_per_pixel, uint32_t stage_rows, uint32_t band_rows,
                    uint32_t band_count, uint32_t first_member, uint32_t members, void* stream);

/* The receiving end of a banded frame: `stage4` (device) holds the packed slabs (params.packed = 1,
   compact = 1) of members first_member .. first_member + members - 1 of a (band_rows, band_count) split, each
   stage_rows x W float4; every pixel is written to the context's G-buffer at its frame position in the
   reference layout, bit for bit what an unbanded render writes (positions recomputed from the context's
   current view: call it with the view the slabs were traced with). Asynchronous on `stream`. */
int sf_unpack_bands(sf_ctx* ctx, const float* stage4, uint32_t stage_rows, uint32_t band_rows, uint32_t band_count,
                    uint32_t first_member, uint32_t members, void* stream);

/* Replaces GetGBuffer() + the GL PBO upload source (Sphereflake.h:25-28,
   GLPixelBufferObject.h:24-29): synchronous D2H copy of the context G-buffer into host
   float4 arrays of W*H elements. Any pointer may be NULL to skip that channel. */
int sf_download(sf_ctx* ctx, float* pos4, float* nrm4, float* min_t, uint32_t* hit_index);

/* Stream-ordered D2H of the context G-buffer (and aux channels) on `stream` (NULL = the context
   stream); returns at once. With page-locked destinations (sf_host_register) it runs at PCIe DMA
   rate and overlaps host work; completion: sf_synchronize (context stream) or the caller's stream. */
int sf_download_async(sf_ctx* ctx, float* pos4, float* nrm4, float* min_t, uint32_t* hit_index, void* stream);

/* Page-lock existing host memory (e.g. the std::vector storage of the C++ class's GBuffer, which the
   reference's PBO upload reads, GLPixelBufferObject.h:24-29) so device copies into it use DMA. */
int sf_host_register(void* ptr, size_t bytes);
int sf_host_unregister(void* ptr);

/* --- reference variant ----------------------------------- */
/* The reference compiles one of two SIMD paths (Sphereflake.cpp:29-33): AVX (SIMD_AVX.h: LOD constant
   70, 8-lane packets, 8-pixel frame-less footprint) or, with __ARCH_NO_AVX (its Linux CMake build),
   SSE (SIMD_SSE.h: LOD constant 60, 4-lane packets, 2x2 footprint, Sphereflake.cpp:115-138). A context
   reproduces either bit for bit; default AVX. Synchronous; later renders use the chosen variant. */
#define SF_VARIANT_AVX 0
#define SF_VARIANT_SSE 1
int sf_set_variant(sf_ctx* ctx, int variant);
int sf_get_variant(const sf_ctx* ctx);   /* SF_VARIANT_* or SF_EINVAL */
/* Exact threshold T: sqrtf(t / r) < lod_constant || t < 0  <=>  t < T (Sphereflake.h:129,146). Host only. */
int sf_lod_threshold(float r, float lod_constant, float* T);
/* 1 when ray generation's u = x / n (Sphereflake.cpp:149-150) may be formed as q0 = RN(x RN(1/n)) corrected by one
   fma residual (RN(q0 + (x - q0 n) RN(1/n))) with the same bits as the division for every integer x in [0, n];
   a context uses the shortcut only for a frame size where this holds (checked at sf_create). Host only. */
int sf_division_by_reciprocal_exact(uint32_t n);

/* --- SSAO post-process ---------------------------------- */
/* The reference's GL passes over the G-buffer (SSAO.cpp:106-142: SSAO, blur x, blur y;
   main.cpp:312-330: final composite), run headless as HIP kernels. Output: RGBA8 image, W*H*4
   bytes, row j = G-buffer row j (GL framebuffer row j counted from the bottom). */
#define SF_POST_GENERAL      1u   /* always run the multi-pass path (A/B; results identical) */
#define SF_POST_UNIT_NORMALS 2u   /* caller's external normals have length <= 1.004 (enables fusion) */

typedef struct sf_post_params {
    float sample_radius;      /* SSAOSampleRadius; < 0: 8 x GetClosestSphereDistance() of this
                                 context, read on the device (main.cpp:316, SSAO.h:15-18) */
    float intensity;          /* SSAO.cpp:51   0.51 */
    float scale;              /* SSAO.cpp:52   3.28 */
    float bias;               /* SSAO.cpp:53   0.23 */
    float normal_threshold;   /* SSAO.cpp:54   2.47 */
    float depth_threshold;    /* SSAO.cpp:55   0.01 */
    float camera_position[3]; /* post_final.glsl cameraPosition (main.cpp:325: the view origin) */
    uint32_t downscale;       /* SSAO target = (W / d, H / d) (SSAO ctor, main.cpp:118 uses 1) */
    uint32_t flags;           /* SF_POST_* */
    void* stream;             /* NULL = the context stream */
} sf_post_params;

/* Reference defaults; camera_position = the context's SetView origin. */
int sf_post_defaults(const sf_ctx* ctx, sf_post_params* params);

/* Post-process a G-buffer on the device. pos4 / nrm4: device float4 G-buffer of W*H pixels (NULL =
   the context's). rgba: device output W*H*4 bytes (NULL = the context's image buffer, see
   sf_download_image). ao: optional device output of the SSAO target before blurring
   ((W/d)*(H/d) bytes, the r channel). Asynchronous on the stream. */
int sf_post_process(sf_ctx* ctx, const sf_post_params* params, const float* pos4, const float* nrm4,
                    uint8_t* rgba, uint8_t* ao);

/* Synchronous D2H of the context image buffer (W*H*4 bytes) written by sf_post_process. */
int sf_download_image(sf_ctx* ctx, uint8_t* rgba);

/* The SSAO noise texture (SSAO.cpp:144-164): 64*64 RGBA32F texels into out[16384]. Host only. */
int sf_ssao_noise(float* out);

/* --- headless image dump ("a PPM/EXR dump for inspection") ------------ */
/* The reference only shows its output in the GL window (main.cpp:306-330); a headless host (no GL)
   inspects a frame through these files. Rows are written top row first (G-buffer row 0 = the top
   edge, Sphereflake.cpp:186-196), so the picture reads the right way up in any viewer. */
#define SF_DUMP_IMAGE         0   /* PPM (P6, 8-bit RGB) of the RGBA8 image of the last sf_post_process;
                                     alpha dropped; SF_ESTATE before any post-process */
#define SF_DUMP_NORMALS       1   /* PPM of the normal channel as clamp(0.5 n + 0.5) * 255, misses black */
#define SF_DUMP_POSITIONS_PFM 2   /* PFM (little-endian float RGB, lossless) of the position channel (x, y, z) */
#define SF_DUMP_NORMALS_PFM   3   /* PFM of the normal channel */
/* Download the context's frame (synchronises) and write it to `path` as `what` (SF_DUMP_*). */
int sf_save_image(sf_ctx* ctx, const char* path, int what);
/* Host-only writers of the same formats: rgba = w*h*4 bytes; v4 = w*h float4 (w component dropped). */
int sf_write_ppm(const char* path, uint32_t width, uint32_t height, const uint8_t* rgba);
int sf_write_pfm(const char* path, uint32_t width, uint32_t height, const float* v4);
/* Frame size of a context. */
int sf_get_size(const sf_ctx* ctx, uint32_t* width, uint32_t* height);

/* Device pointers of the context buffers (any out-pointer may be NULL). */
int sf_device_buffers(sf_ctx* ctx, float** pos4, float** nrm4, float** min_t, uint32_t** hit_index);

/* Block until all work on the context stream is done. */
int sf_synchronize(sf_ctx* ctx);

/* --- stats (Sphereflake.h:30-58) ---------------------------------------- */

int sf_get_stats(sf_ctx* ctx, sf_stats* out);          /* synchronises */
int sf_reset_max_depth(sf_ctx* ctx);                   /* ResetMaxDepthReached */
int sf_reset_rays(sf_ctx* ctx);                        /* ResetRaysPerSecond */
int sf_reset_closest(sf_ctx* ctx);                     /* ResetClosestSphereDistance */

/* --- frame-less progressive mode (Initialize + DoImagePart, Sphereflake.cpp:67-74,86-214) --- */

/* Trace `packets` random 8-ray packets into the context G-buffer, exactly as one reference
   worker thread would: pixel pairs from Sobol dims 0/1 (Sobol.cpp:41-55) scrambled by an
   mt19937 stream seeded with `seed` (std::uniform_int_distribution<unsigned>(0) draws),
   packet footprint of Sphereflake.cpp:143-147, scatter of :186-201, sobol counter starting at
   `counter0`. Packets are traced in parallel; later packets overwrite earlier ones at shared
   pixels, as in the reference's sequential order. */
int sf_progressive(sf_ctx* ctx, uint32_t seed, uint64_t counter0, uint32_t packets, void* stream);

/* --- host setup helpers (reference host math, fixture-pinned) ------------ */

/* Camera corners of reference camera.h:37-53 (FOV, quaternion from (yaw, pitch, roll),
   aspect W/H, scaling tan(fov/2)/3). Angles in radians, fov in degrees. */
int sf_camera_corners(uint32_t width, uint32_t height, const float position[3], float pitch,
                      float yaw, float roll, float fov_deg, float origin[3], float top_left[3],
                      float top_right[3], float bottom_left[3]);

/* The 9 unit child frames of ComputeChildTransformations (Sphereflake.cpp:216-249). */
int sf_child_transforms(float child[9][16]);

/* Root transform of SetView (Sphereflake.cpp:83) for a ray origin. */
int sf_root_transform(const float origin[3], float root[16]);

/* Per-depth constants the kernels use: radius r_d (Sphereflake.h:97), and the exact float
   threshold T_d with  sqrtf(t / r_d) < 70 || t < 0   <=>   t < T_d  (Sphereflake.h:146). */
int sf_depth_constants(uint32_t depth, float* radius, float* lod_threshold);

/* std::mt19937 jump-ahead (host; the frame-less draws' parallel generation): the state (624 words + next
   index, libstdc++ layout: sf_progressive's generator state) after `outputs` more draws, computed with the
   generator's characteristic polynomial (t^m mod phi), not by stepping. */
int sf_mt19937_jump(const uint32_t state_in[625], uint64_t outputs, uint32_t state_out[625]);

/* Reproduction of x86 rsqrtps (the table the kernels use). */
float sf_rsqrtps(float x);

/* --- diagnostics --------------------------------------------------------- */

/* Per-tile timing of the wave kernel (s_memrealtime, 100 MHz) for schedule analysis: when enabled,
   every full-frame render records {start, end, (XCC id << 32) | HW_ID} per 8x8 tile. Off by default;
   never changes results. */
int sf_set_tile_trace(sf_ctx* ctx, int enable);
int sf_get_tile_trace(sf_ctx* ctx, uint64_t* out, size_t n);   /* n >= 3 * tiles; synchronises */
/* Heavy-first tile schedule: the work units the next persistent render takes in order (computed from
   the last render's per-tile costs, heaviest cost bucket first, stable within a bucket; a unit is
   tile | part << 29: part 0 = the whole 8x8 tile, 1/2 = its pixel rows 0-3/4-7, 3..6 = its 4x4 quarters,
   or with env SF_SPLIT_PARTS=subtree its 4 subtree parts -- the tiles of the heaviest buckets may be traced
   as 2 or 4 part units, env SF_SPLIT_BUCKETS / SF_SPLIT_PARTS) and those costs (shader cycles, one per tile
   of the render the order was built for -- a band share's tiles when that render was one; a split tile's
   slowest part, scaled). Either pointer may be NULL; n >= 4 * tiles (order) or tiles (cost only), tiles of
   the whole frame. Returns the unit count, 0 when no order exists yet, or a negative SF_E*. Synchronises. */
int sf_get_tile_order(sf_ctx* ctx, uint32_t* order, uint32_t* cost, size_t n);

/* --- measurement ---------------------------------------------------------- */

/* enable = k > 0: every k-th full-frame render (counting from the call) records HIP events on its
   launch stream around its main trace kernel (the dominant kernel; the roofline in bench.py is priced
   on it). An event pair costs a few us of stream time, so sampling keeps the measurement out of the
   frame rate. enable = 0 turns it off. */
int sf_set_kernel_timing(sf_ctx* ctx, int enable);
/* Durations (ms) of the main trace kernel of the last min(n, 64) timed renders, oldest first;
   returns how many were written (>= 0) or a negative SF_E*. Synchronises. */
int sf_kernel_times(sf_ctx* ctx, float* ms, uint32_t n);
/* Live shader clock (MHz) of the same timed renders, oldest first: per render the median over the first
   wave of 8 workgroups of delta s_memtime / delta s_memrealtime x 100 MHz across that wave's life in the
   trace kernel (it runs for nearly the whole kernel). Returns how many were written; synchronises. */
int sf_kernel_clocks(sf_ctx* ctx, float* mhz, uint32_t n);

/* --- multi-GPU ------------------------------------------ */
/* One process, n member devices (the reference's host thread pool, Sphereflake.cpp:67-74, becomes n
   GPUs). The frame is cut into interleaved bands of band_rows rows, band b traced by member b % n;
   member 0 holds the final G-buffer (its context's buffers): it writes its bands in place; member k > 0
   traces its bands as a packed slab (4 B/pixel hit indices where sf_slab_bytes allows, else 16 B/pixel;
   sf_render_params.packed) and copies it over xGMI into member 0's stage on a copy stream of its own
   (overlapping its next frame's trace); member 0 unpacks the stage into its G-buffer (sf_unpack_slabs) on an
   unpack stream of its own, beside its own trace, and its context stream waits for that. Slabs and stages are
   double-buffered by frame parity, so members run a frame ahead of member 0. A device may appear more than
   once (n contexts on one GPU: the single-GPU test of the path). Stats combine: max depth max, closest min,
   rays and overflow tiles summed. */
typedef struct sf_group sf_group;
int sf_group_create(const int* devices, int n, uint32_t width, uint32_t height, sf_group** out);
void sf_group_destroy(sf_group* group);
int sf_group_size(const sf_group* group);
sf_ctx* sf_group_member(sf_group* group, int k);          /* member k's context (k = 0: the final G-buffer) */
int sf_group_set_view(sf_group* group, const float origin[3], const float top_left[3],
                      const float top_right[3], const float bottom_left[3]);
int sf_group_set_variant(sf_group* group, int variant);
/* One frame across the members (asynchronous; band_rows a multiple of 8, 0 = 8). Work queued on member
   0's context afterwards (sf_download, sf_post_process, ...) sees the whole frame. */
int sf_group_render(sf_group* group, uint32_t band_rows);
int sf_group_synchronize(sf_group* group);
int sf_group_download(sf_group* group, float* pos4, float* nrm4);   /* synchronous D2H of the frame */
int sf_group_get_stats(sf_group* group, sf_stats* out);             /* synchronises */
int sf_group_reset_stats(sf_group* group);                          /* all three counters, every member */
int sf_group_last_hip_error(const sf_group* group);
/* Bytes per pixel a member ships for the current view (sf_slab_bytes of member 0). */
int sf_group_slab_bytes(const sf_group* group);

/* --- multi-GPU, one process per GPU ------------------------------------------------------
   The reference's worker pool (Sphereflake.cpp:67-74) as nranks processes, one GPU each (the torch.distributed /
   MPI model): every rank traces the interleaved bands b = rank (mod nranks) of each frame; ranks k > 0 trace
   theirs as packed slabs (4 B/pixel hit indices where sf_slab_bytes allows, else 16 B/pixel;
   sf_render_params.packed) and send them to rank 0 with RCCL over xGMI (ncclSend behind the trace on the frame's
   stream); rank 0 traces its own bands in place while it receives the others' (one grouped ncclRecv) and unpacks
   them (sf_unpack_slabs) on a receive stream of its own; the slot's context stream then waits for the unpack: the
   frame in rank 0's G-buffer bit for bit the single-GPU frame.
   `slots` frames may be in flight: frame i runs on slot i % slots (its own context, stream, communicator and
   buffers), so a frame's trace fills the GPU while the previous frame's heaviest tiles and gather finish.
   Without ids there is no communicator, whatever nranks: frames in flight on one GPU (nranks = 1), or this rank's
   bands of a distributed G-buffer (sf_dist_render_bands; sf_dist_render returns SF_ESTATE, sf_dist_get_stats this
   rank's stats alone). Every rank must issue the same calls in the same order (set_view, render, get_stats) with
   the same views. */
#define SF_DIST_ID_BYTES 128   /* ncclUniqueId */
#define SF_DIST_MAX_SLOTS 16
typedef struct sf_dist sf_dist;
/* Rank 0 makes one id per slot and hands them to every rank (any channel: MPI, a torch.distributed broadcast). */
int sf_dist_unique_id(uint8_t id[SF_DIST_ID_BYTES]);
/* Collective over the ranks when ids are given (RCCL communicator init per slot). ids: slots x SF_DIST_ID_BYTES,
   or NULL: no communicator at all (bands only, see above); nranks = 1 with ids makes a one-rank communicator.
   band_rows: a multiple of 8 (8 = one tile row). */
int sf_dist_create(int device, uint32_t width, uint32_t height, uint32_t band_rows, int rank, int nranks, int slots,
                   const uint8_t* ids, sf_dist** out);
void sf_dist_destroy(sf_dist* dist);
int sf_dist_slots(const sf_dist* dist);
sf_ctx* sf_dist_context(sf_dist* dist, int slot);     /* slot's context; on rank 0 it holds that slot's frames */
int sf_dist_last_slot(const sf_dist* dist);           /* slot of the last frame issued (SF_ESTATE before any) */
int sf_dist_set_view(sf_dist* dist, const float origin[3], const float top_left[3], const float top_right[3],
                     const float bottom_left[3]);     /* the view of the next frames (kept by the dist and set on
                                                         a slot's context when a frame is rendered on it) */
int sf_dist_render(sf_dist* dist);                    /* one frame, asynchronous (this rank's share + gather;
                                                         SF_ESTATE for nranks > 1 without communicators) */
/* One frame as a distributed G-buffer: this rank's bands into its slot's G-buffer at frame positions (reference
   layout), no gather -- every rank holds its own rows in its own HBM. Asynchronous; no collective. */
int sf_dist_render_bands(sf_dist* dist);

/* The next n frames of a camera path (views[k][0..11] = origin, top-left, top-right, bottom-left) as this rank's
   bands, frame k into slot (frames + k) % slots's G-buffer (n <= slots, n <= SF_RENDER_FRAMES_MAX), in ONE
   multi-frame persistent launch (sf_render_frames): sf_dist_render_bands for n frames without a launch each.
   The views are set on the slots (sf_dist_set_view is not needed). Asynchronous. */
int sf_dist_render_bands_frames(sf_dist* dist, uint32_t n, const float (*views)[12]);
int sf_dist_synchronize(sf_dist* dist);               /* every slot of this rank done */
int sf_dist_download(sf_dist* dist, float* pos4, float* nrm4);   /* rank 0: D2H of the last frame (synchronises) */
int sf_dist_get_stats(sf_dist* dist, sf_stats* out);  /* over slots, and over ranks when made with ids
                                                         (then collective); synchronises */
int sf_dist_reset_stats(sf_dist* dist);
int sf_dist_last_error(const sf_dist* dist, int* hip_error, int* rccl_error);
/* The RCCL communicator of `slot` as RCCL reports it: ncclCommCount, ncclCommUserRank, ncclCommCuDevice
   (SF_ESTATE when the dist was made without ids). */
int sf_dist_comm_info(const sf_dist* dist, int slot, int* count, int* rank, int* device);
/* Bytes per pixel the gather ships for the current view (sf_slab_bytes of the slots' contexts). */
int sf_dist_slab_bytes(const sf_dist* dist);

/* The context's own stream (hipStream_t) -- where calls with a NULL stream are queued. */
void* sf_context_stream(sf_ctx* ctx);

/* --- misc ---------------------------------------------------------------- */

const char* sf_strerror(int status);
int sf_last_hip_error(const sf_ctx* ctx);
int sf_abi_version(void);
/* Hash of the sources this library was built from (scripts/source_hash.py): ties a measurement to a build. */
const char* sf_build_id(void);
int sf_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* SPHEREFLAKE_SF_H */
