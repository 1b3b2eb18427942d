// sf_internal.h -- structures shared by the C ABI layer (sf_capi.hip), the host setup math
// (sf_setup.cpp, g++) and the gfx950 kernels (sf_kernels.hip). Not installed.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define SF_HD __host__ __device__
#else
#define SF_HD
#endif

#define SF_DEPTH_TABLE 33      // depths 0..32 (SF_MAX_DEPTH_LIMIT)
// relative margin of the occlusion cull: a subtree's bounding ball (radius R around c) is fattened to
// R + SF_OCCL_MARGIN (|c| + R). The float tests inside it can start at most sqrt(28 u) (|c| + R) = 2^-9.6 (|c| + R)
// (u = 2^-24; the d2 cancellation, tca and |d| != 1) plus ~25 u (|c| + R) before the ball:
// 3 x 2^-10 is 2.2x that (round 3 started at 2^-7; the wider margin culls fewer deep subtrees)
#ifndef SF_OCCL_MARGIN
#define SF_OCCL_MARGIN 0x1.8p-9f
#endif
#define SF_TILE 8              // a wave64 traces one 8x8 pixel tile
#define SF_WAVES_PER_BLOCK 4   // 256-thread workgroups (per-ray kernel)
#ifndef SF_WAVES_PER_EU
#define SF_WAVES_PER_EU 8      // occupancy target of the persistent trace kernels (waves per SIMD)
#endif
#ifndef SF_TRACE_WAVES
#define SF_TRACE_WAVES 1       // independent waves per workgroup of the wave kernels (round 4: 1 -- 1080p 0.0718-0.0723
                               // -> 0.0697-0.0707 ms against 2, profiles/r4/waves_ab.txt; the pipelined and compaction
                               // variants exist at 2 and take 2)
#endif
// Wave-coherent traversal LDS image, per wave (units: floats):
//   [root: 16][cone: 8][(levels - 1) x (table 144 | E 32)]
// A transform is 4 float4 {cx cy cz cc}, {col0.xyz -}, {col1.xyz -}, {col2.xyz -} (cc = Dot(centre, centre));
// a level table stores them in 4 planes of 9 float4 (plane k = float4 k of children 0..8).
#define SF_LDS_ROOT 16
#define SF_LDS_CONE 8                     // the wave's ray cone {ax, ay, az, cosT, sinT, -, -, -}
// plane 0: {centre, cc} float4 of each of the 9 children (36 floats), 2 floats of skew, then planes 1..3:
// column j (xyz, float3) of each child. The skew puts the column stores of the 27 column builders (lanes
// 0..26, dwords 38 + 3l..) on other banks than child 0's centre store repeated in the same 32-lane LDS group
// (lanes 27..31, dwords 0..3): the table build is free of bank conflicts (sf_kernels.hip, the builder lanes)
#define SF_LDS_PLANE 38
#define SF_LDS_COLS 27                    // planes 1..3: column j (xyz, float3) of each of the 9 children
#define SF_LDS_TABLE (SF_LDS_PLANE + 3 * SF_LDS_COLS)   // the 9 child transforms of the node open at a level
#define SF_LDS_E 32                       // 64 lanes x u16: per-lane child-expand bits of that node
#define SF_LDS_LEVEL (SF_LDS_TABLE + SF_LDS_E + 1)      // (+1: levels stay 16-byte aligned)
// levels - 1 level images: the deepest provisioned level's table is never read (see traverse)
#define SF_LDS_WAVE_FLOATS(levels) (SF_LDS_ROOT + SF_LDS_CONE + ((levels) - 1) * SF_LDS_LEVEL)

// Persistent-kernel tile queues: SF_QUEUES counters per render parity, one 128-byte line each, after
// the two overflow counters (u32 words).
#define SF_QUEUES 32u                     // up to 8 XCDs x 4 queues per XCD
#define SF_QUEUE_STRIDE 32u
#define SF_QUEUE_WORD(parity, k) (SF_QUEUE_STRIDE + ((parity) * SF_QUEUES + (k)) * SF_QUEUE_STRIDE)
#define SF_COUNTER_WORDS (SF_QUEUE_STRIDE + 2u * SF_QUEUES * SF_QUEUE_STRIDE)

// 64-bit diagnostic slots after the per-tile trace (segment sums of PHASES=1, event counts of COUNTS=1)
#define SF_DIAG_SLOTS 16
// per-wave {start, end} records (SF_FLAG_DIAG_UNITS) after the per-tile and per-unit records: waves past
// this many are not recorded
#define SF_DIAG_WAVES 65536u
// tile trace buffer (u64): per tile {start, end, id}, the diagnostic slots, per work unit {start, end,
// unit} (<= 4 units per tile), per wave {start, end}
#define SF_TRACE_WORDS(ntiles) ((size_t)(ntiles) * 15u + SF_DIAG_SLOTS + 2u * SF_DIAG_WAVES)

#define SF_FLAG_NO_LOD_CULL 1u    // disable the leaf-threshold skip (A/B only; results identical; since round 5 the
                                  // frame-less packet traversal only -- the full-frame traversal always skips)
#define SF_FLAG_NO_CONE_CULL 2u   // disable the per-child ray-cone cull (A/B only; results identical)
// diagnostics (schedule studies): trace only one half unit of every 8x8 tile -- pixel rows 0-3, or
// with SF_FLAG_DIAG_HALF_SEL rows 4-7. Other pixels are not written. Never set by the product path.
#define SF_FLAG_DIAG_HALF 4u
#define SF_FLAG_DIAG_HALF_SEL 8u
// diagnostics (schedule studies): with the tile trace on, also record every work unit of the persistent
// kernel by its order position g: {start, end, unit} (s_memrealtime) after the tile trace and the
// diagnostic slots (room for 2 units per tile)
#define SF_FLAG_DIAG_UNITS 0x20u
// diagnostics only, WRONG results: the frame-less trace skips its per-pixel owner atomics (cost study)
#define SF_FLAG_DIAG_NO_OWNER 0x40u
// flat wave priority (A/B): every raised-priority cost bucket at s_setprio 2 (default: graded, see
// trace_queue_body)
#define SF_FLAG_PRIO_FLAT 0x80u
// disable the occlusion cull of the per-ray traversal (A/B only; results identical)
#define SF_FLAG_NO_OCCL_CULL 0x100u
// children in index order only (A/B; results identical): by default the per-ray traversal enters the children
// nearer than their parent's centre along the tile's cone axis first
#define SF_FLAG_NO_FRONT_FIRST 0x200u
// tests only: every tile of the main kernels takes the tie fallback (re-traced in index order: by the same wave
// under SF_FLAG_TIE_INLINE, else by sf_fixup_wave)
#define SF_FLAG_DIAG_FORCE_RETRACE 0x400u
// set by the host, never by a caller: the persistent trace's LDS levels are proven sufficient, so a tile can only be
// flagged for an exact tie under the front-first child order, and the wave that traced it re-traces it in index order
// at once (same levels, no overflow list, no fixup launch after the trace)
#define SF_FLAG_TIE_INLINE 0x800u
// (kernel-internal) the index-order re-trace pass of such a tile: its writes replace the first pass's, its cost is
// not recorded
#define SF_FLAG_REDO_PASS 0x1000u
// set by the host (env SF_SPLIT_PARTS=subtree): the 4 part units of a split tile are SUBTREE parts -- each traces the
// whole 8x8 tile but enters, below FrameArgs.split_depth - 1, only the depth-split_depth nodes whose heap index is its
// part number mod 4; the part that finishes last merges the 4 per-pixel results (nearest, the reference's tie rule)
// and writes the tile (trace_tile). Quarter units (pixel parts) otherwise.
#define SF_FLAG_SUBTREE 0x2000u
// row-major units are tile halves (pixel rows 0-3 / 4-7 of tile u / 2): a frame of fewer tiles than wave slots -- a
// member's share -- then ends on half its heaviest tile's traversal (round 6, A/B: SF_HALVES)
#define SF_FLAG_HALVES 0x4000u

struct DepthTables {
    float r2_bound[SF_DEPTH_TABLE];   // (2 r_d)^2  bounding sphere (Sphereflake.h:108-110)
    float r2_self[SF_DEPTH_TABLE];    // r_d^2      node's own sphere (Sphereflake.h:180)
    float scale[SF_DEPTH_TABLE];      // (4/3) r_d  child translation scale (Sphereflake.h:162)
    float lod[SF_DEPTH_TABLE];        // T_d: sqrtf(t/r_d) < 70 || t < 0  <=>  t < T_d (Sphereflake.h:146)
};

// Per-context read-only device block (global memory; lane-indexed reads hit L1/L2).
struct DeviceConsts {
    float child[9][16];               // unit child frames, glm column-major (Sphereflake.cpp:216-249)
    DepthTables dt;
    // the same interleaved per depth d, one scalar load: {r2_bound, r2_self, scale, lod,
    // leaf, cull, far, 0}; leaf = |c|^2 threshold beyond which no child of a depth-d node centred at c can
    // pass the LOD test for any ray (sfhost::leaf_threshold); cull = 2 r_d (1 + 2 SF_OCCL_MARGIN), rounded
    // up: the occlusion cull's fattened bounding radius without its |c| term (see traverse); far =
    // T_d + 2 r_d (1 + 2^-18), rounded up: a bounding hit with tca (1 - 2^-8) >= far cannot pass LOD
    float depth8[SF_DEPTH_TABLE][8];
    uint32_t lut[2048];               // x86 rsqrtps table (rsqrtps_lut.inc)
    uint32_t sobol[2][52];            // Sobol direction numbers, dims 0 and 1 (Sobol.cpp:34-39, 57-162)
    // per context (its frame size), read by scalar loads where used rather than carried in the launch arguments:
    // {RN(1 / W), RN(1 / H)}: u = x / W as one product and one fma correction, where the host checked it equals
    // x / W for every x in [0, W] and y in [0, H] (fast_div); floor((2^32 - 1) / tiles_x) (tile_of)
    float rw, rh;
    uint32_t fast_div, tx_magic;
};

// Frame-less progressive mode: one traced packet lane (staged between trace and scatter).
struct PacketLane {
    float px, py, pz, nx, ny, nz, min_t;
    uint32_t pixel;                   // x + y*W (Sphereflake.cpp:188), 0xffffffff = skipped
};

// Everything a launch needs, passed by value as the kernel argument.
struct FrameArgs {
    uint32_t W, H;
    float fw, fh;                     // (float)W, (float)H  (Sphereflake.cpp:104-110)
    float o[3], tl[3], dh[3], dv[3];  // origin, top-left, TR-TL, BL-TL (Sphereflake.cpp:162-166)
    float root[12];                   // root transform columns 0..3, xyz (Sphereflake.cpp:83)
    uint32_t tiles_x;                 // ceil(W / 8)
    uint32_t tile_rows;               // tile rows this launch renders
    uint32_t tiles_per_band;          // band_rows / 8
    uint32_t band_count, band_index;
    uint32_t compact;                 // write rows packed into the shard's slab
    uint32_t packed;                  // write one float4 (nx, ny, nz, minT) per pixel to pos only (sf_render_params.packed)
    uint32_t max_depth;               // traversal levels provisioned (<= SF_MAX_DEPTH_LIMIT)
    uint32_t emit_aux;
    uint32_t flags;                   // SF_FLAG_* (A/B switches for diagnostics; 0 = product default)
    const DeviceConsts* consts;
    float* pos;                       // G-buffer positions (float4 x,y,z,1 per pixel)
    float* nrm;                       // G-buffer normals
    float* min_t;                     // optional aux channel
    uint32_t* hit_index;              // optional aux channel (heap index 9n+1+i, 0xffffffff = miss)
    int32_t* stats;                   // [0] max depth (atomicMax), [1] closest key (atomicMin), [2] overflow count
    uint64_t* tile_trace;             // diagnostics (NULL = off): per tile {start, end} s_memrealtime, hw id
    uint64_t* phase_sums;             // diagnostics, stamp builds only (make PHASES=1): 8 segment sums
    uint32_t* counters;               // overflow counts + tile queues (SF_QUEUE_WORD), alternating per render
    uint32_t* overflow_list;          // tiles to re-trace with SF_MAX_DEPTH_LIMIT levels
    uint32_t parity;                  // which half of `counters` this render uses
    uint32_t* tile_cost;              // out (NULL = off): per tile, shader cycles of its traversal
    const uint32_t* tile_order;       // in (NULL = row-major): work units (SF_UNIT_*), heaviest first
    const uint32_t* order_meta;       // with tile_order: [0] units in it, [1] first split bucket
    uint32_t* chunk_cnt;              // out (with tile_cost): per 64-tile chunk, cost-bucket histogram
    uint32_t* part_cost;              // per tile: max cycles over the parts of a split tile (reset by the last part)
    uint32_t* part_done;              // per tile: parts of a split tile finished (reset by the last part)
    uint32_t packet_lanes;            // frame-less mode: 8 (AVX variant) or 4 (SSE variant, 2x2 footprint)
    uint32_t queues;                  // persistent trace: tile queues in use (xcds x queues per XCD, <= SF_QUEUES)
    uint32_t xcds;                    // persistent trace: XCD queue groups (power of 2); queue k serves XCD k % xcds
    uint32_t* bin_cost;               // frame-less mode (NULL = off): per packet bin, cycles of the last wave starting in it
    uint32_t bin_shift, bins_x;       // frame-less mode: the batch's packet bins (squares of 2^bin_shift pixels)
    uint64_t* clock_probe;            // measurement (NULL = off): the first wave of blocks 0..SF_CLOCK_WAVES-1
                                      // writes {s_memtime, s_memrealtime} at its start and at its end
    uint32_t tpb_magic;               // floor((2^32 - 1) / tiles_per_band) (tile_of)
    uint64_t* part_rec;               // SF_FLAG_SUBTREE: per split slot x part, 3 x 64 u64 -- each lane's
                                      // {minT | cx}, {cy | cz}, {index | depth} (merged by the last part)
    uint32_t split_depth;             // SF_FLAG_SUBTREE: depth of the nodes the parts divide (>= 1)
};
#define SF_CLOCK_WAVES 8u             // live shader clock samples per timed render (one per XCD group)

// Multi-frame persistent trace (round 6, sf_render_frames): the frames of one launch, passed by value in the kernel
// argument segment (copied by the runtime at the launch, so the host may build the next batch at once; 4 KB at most:
// 11 FrameArgs). Frame f is one slot context's view into that context's G-buffer and stats. All frames share one
// set of tile queues and one unit order (`units` per frame); the first `heavy` units of every frame's order are
// interleaved across the frames at the head of the launch's sequence (the heaviest tiles of every frame start first),
// the rest follow frame by frame.
#define SF_BATCH_MAX 8u
struct FrameBatch {
    uint32_t nframes, units, heavy;
    uint32_t magic;                   // ceil(2^32 / nframes): G / nframes = mulhi(G, magic) for G < 2^29
    FrameArgs f[SF_BATCH_MAX];
};

// Band slab formats of the multi-GPU gather (FrameArgs.packed / sf_render_params.packed):
//   SF_PACKED_NORMAL  16 B per pixel: float4 (nx, ny, nz, minT); the receiver forms pos = dir * minT
//   SF_PACKED_INDEX    4 B per pixel: the hit's heap index (SF_SLAB_MISS: none); the receiver rebuilds the
//                      sphere's frame (node table + child_frame), its self test's minT, pos and nrm
// The index format needs every hit's heap index below 2^32 -- depth <= SF_INDEX_SLAB_DEPTH -- which the host
// proves from the view (sf_slab_bytes) before choosing it.
#define SF_PACKED_NORMAL 1u
#define SF_PACKED_INDEX 2u
#define SF_INDEX_SLAB_DEPTH 10
// tests only (env SF_DIAG_SLAB_SHALLOW=1): the host launches an index-slab trace as FrameArgs.packed =
// SF_PACKED_INDEX_DIAG, whose slab carries hits only to depth SF_DIAG_SLAB_DEPTH, so a test view's ordinary hits stand
// in for a hit too deep for the format (SF_SLAB_BAD, counted as unresolved: sf_synchronize reports SF_EDEPTH). A packed
// mode, not a flag or a launch argument: write_pixel already holds a.packed, and the product kernel keeps its registers
#define SF_PACKED_INDEX_DIAG 3u
#define SF_DIAG_SLAB_DEPTH 4
#define SF_SLAB_MISS 0xffffffffu
#define SF_SLAB_BAD 0xfffffffeu
// node table of the index unpack: the frames of every node of depth <= SF_NODE_TABLE_DEPTH (3 float4 each; 28.7 MB,
// rebuilt when the root transform changes)
#define SF_NODE_TABLE_DEPTH 6u
#define SF_NODE_TABLE_NODES 597871u   // (9^7 - 1) / 8

// Headless SSAO post-process (Shaders/post_ssao.glsl, post_ssao_blur.glsl,
// post_final.glsl, SSAO.cpp:106-142). Textures are modelled, not emulated: NEAREST/LINEAR filtering
// with the texel coordinate snapped to 8 fractional bits (sf_post.hip).
#define SF_NOISE_SIZE 64               // SSAO.h NOISE_TEXTURE_SIZE
struct PostArgs {
    uint32_t W, H;                    // G-buffer (= blur / final target) size
    uint32_t aw, ah;                  // SSAO target size (W / downscale, H / downscale)
    float fw, fh, faw, fah;
    float rfw, rfh, rfaw, rfah;       // RN(1 / fw) ... RN(1 / fah): the shaders' uniform reciprocals
    const float* pos;                 // float4 per pixel
    const float* nrm;
    const float* noise;               // SF_NOISE_SIZE^2 float4 (.xy read)
    const int32_t* stats;             // [1] closest-hit key, for radius < 0
    float radius;                     // SSAOSampleRadius, or < 0: 8 x closest (SSAO.h:15-18)
    float intensity, scale, bias, normal_thr, depth_thr;
    float cam[3];
    uint8_t* ao;                      // SSAO target (aw x ah); RGBA8 FBO with r = g = b: one channel kept
    uint8_t* blur_h;                  // horizontal blur target (W x H)
    uint8_t* blur_v;                  // vertical blur target (W x H)
    uint8_t* rgba;                    // final image, W x H x RGBA8, row j = G-buffer row j
};

#ifndef SF_PROGRESSIVE_LEVELS
#define SF_PROGRESSIVE_LEVELS 16        // frame-less mode: LDS traversal levels
#endif
#define SF_PROG_FIXUP_BLOCKS 256u      // grid of sf_progressive_fixup (grid-stride over the overflow list)
#ifndef SF_MT_PARTS
#define SF_MT_PARTS 32u                // frame-less mode: workgroups per jump-ahead window (sf_mt_jump_partial)
#endif
#define SF_PROG_MAX_BINS 32768u        // frame-less mode: packet bins (counting sort in one workgroup's LDS)
#define SF_PROG_PREFETCH_MIN 65536u    // frame-less batches from this many packets prefetch the next draws
#define SF_PROG_BIN_MIN 65536u         // frame-less batches below this many packets trace in draw order
                                       // (binning pays once the batch is several waves per slot)
#define SF_ORDER_BUCKETS 32u           // log-spaced cost buckets of sf_tile_order (2 per octave from 2^8 cycles)
// A work unit of the tile order: tile index | prio << SF_UNIT_PRIO_SHIFT | part << SF_UNIT_PART_SHIFT.
// prio (written by sf_order_scatter from the unit's cost bucket, so the trace reads no cost table the same
// launch rewrites): 0 normal, 1 raised (the lowest 3 of the top order_meta[3].. buckets, s_setprio 2),
// 2 raised high (the buckets above, s_setprio 3). Part 0 = the whole 8x8 tile;
// 1, 2 = its pixel rows 0-3 / 4-7 (halves); 3..6 = its 4x4 quarters (q = part - 3: rows 4 (q >> 1).., columns
// 4 (q & 1)..). The heaviest tiles are traced as 2 or 4 part units by as many waves: a tile's serial DFS
// otherwise bounds the frame.
#define SF_UNIT_PART_SHIFT 29u
#define SF_UNIT_PRIO_SHIFT 27u
#define SF_UNIT_TILE_MASK ((1u << SF_UNIT_PRIO_SHIFT) - 1u)   // frames of up to 2^27 8x8 tiles
#define SF_PART_HALF0 1u
#define SF_PART_QUARTER0 3u
// Which tiles are split: env SF_SPLIT_BUCKETS = k splits the top k occupied cost buckets (at most an
// eighth of the tiles). The default (SF_SPLIT_AUTO) splits only into idle wave slots: whole buckets,
// heaviest first, while tiles + split tiles <= the persistent grid's waves. With more tiles than waves
// (1920x1080: 32400 tiles, 7168 waves) nothing is split -- measured: splitting there costs +1.5-3.5 %;
// at 640x360 (3600 tiles) it takes the frame from 0.198 to 0.144 ms.
#define SF_SPLIT_AUTO 0xffffffffu
// tile orders of at most this many 64-tile chunks are scattered by sf_order_scan's own workgroup (8 chunks per
// wave at most); larger ones by sf_order_scatter, one wave per chunk
#ifndef SF_ORDER_FUSE_CHUNKS
#define SF_ORDER_FUSE_CHUNKS 128u
#endif
// env SF_SPLIT_BUCKETS=model: split the buckets a makespan model of the last render's costs says shorten the
// frame (sf_order_scan) -- also on full grids, where the heaviest tile exceeds the slots' fair share
#define SF_SPLIT_MODEL 0xfffffffeu
// split tiles per render at most (sf_order_scan; the subtree parts' records are per split slot)
#define SF_SPLIT_CAP 4096u
// Parts a split tile is traced as (env SF_SPLIT_PARTS): 2 halves or 4 quarters. A split tile's cost for
// the next schedule is its slowest part's, scaled to whole-tile terms (measured: the slowest half takes
// ~0.68 of the whole tile, the slowest quarter ~0.5).

namespace sfhost {
void child_transforms(float child[9][16]);
void root_transform(const float origin[3], float root[16]);
void camera_corners(uint32_t W, uint32_t H, const float pos[3], float pitch, float yaw, float roll,
                    float fov, float o[3], float tl[3], float tr[3], float bl[3]);
float radius(uint32_t depth);
float lod_threshold(float r, float lod_constant = 70.0f);
// true when fma(fma(-q0, n, x), RN(1/n), q0), q0 = RN(x RN(1/n)), equals RN(x / n) for every integer x in [0, n]
bool division_by_reciprocal_exact(uint32_t n);
void depth_tables(DepthTables* t, float lod_constant = 70.0f);
float leaf_threshold(const DepthTables* t, uint32_t depth);
void sobol_matrices(uint32_t out[2][52]);
void mt19937_seed(uint32_t seed, uint32_t state[625]);
// mt19937 jump-ahead (sf_mtjump.cpp): t^(j L) mod phi for j < K (K x mt_poly_words() u64, cached), and the
// host reference jump of a std::mt19937 state by `outputs` draws
int mt_poly_words();
const uint64_t* mt_jump_polys(uint64_t L, uint32_t K);
void mt_jump(const uint32_t in[625], uint64_t outputs, uint32_t out[625]);
void ssao_noise(float out[SF_NOISE_SIZE * SF_NOISE_SIZE * 4]);
bool post_centre_exact(uint32_t n);
}  // namespace sfhost

// Order-preserving map float <-> int32 for atomicMin on floats (negative values included).
SF_HD static inline int32_t sf_float_key(float f)
{
    union { float f; int32_t i; } u;
    u.f = f;
    return u.i >= 0 ? u.i : (int32_t)(u.i ^ 0x7fffffff);
}
SF_HD static inline float sf_key_float(int32_t k)
{
    union { float f; int32_t i; } u;
    u.i = k >= 0 ? k : (int32_t)(k ^ 0x7fffffff);
    return u.f;
}
