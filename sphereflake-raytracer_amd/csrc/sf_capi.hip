// sf_capi.hip -- host side of the C ABI declared in include/sphereflake/sf.h.
//
// Owns the per-device context: device G-buffer (positions, normals as float4, reference layout
// Sphereflake.h:7-11), optional aux channels (minT, hit index), the read-only constants block
// (child frames, per-depth tables, rsqrtps table), stats words and the overflow tile list.
// Launches are stream-ordered; nothing here synchronises except sf_download / sf_get_stats /
// sf_synchronize.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

#include "sf_build_id.h"   // SF_SOURCE_HASH (generated: build/, scripts/source_hash.py)
#include "sf_internal.h"
#include "sphereflake/sf.h"

extern "C" __global__ void sf_trace_wave1(FrameArgs a, uint32_t* overflow_list, uint32_t* overflow_count);
extern "C" __global__ void sf_trace_wave2(FrameArgs a, uint32_t* overflow_list, uint32_t* overflow_count);
extern "C" __global__ void sf_trace_wave4(FrameArgs a, uint32_t* overflow_list, uint32_t* overflow_count);
extern "C" __global__ void sf_trace_queue1(FrameArgs a);
extern "C" __global__ void sf_trace_frames1(FrameBatch b);
extern "C" __global__ void sf_trace_queue1s(FrameArgs a);
extern "C" __global__ void sf_trace_queue2(FrameArgs a);
extern "C" __global__ void sf_trace_queue4(FrameArgs a);
extern "C" __global__ void sf_trace_queue2p(FrameArgs a);
extern "C" __global__ void sf_trace_queue2c(FrameArgs a);
extern "C" __global__ void sf_order_scan(uint32_t* chunk_cnt, uint32_t nc, uint32_t n_tiles,
                                         uint32_t split_buckets, uint32_t parts, uint32_t spare, uint32_t waves,
                                         uint32_t prio_buckets,
                                         uint32_t* chunk_off, uint32_t* order_meta, const uint32_t* fuse_cost,
                                         uint32_t* fuse_order, uint32_t split_cap);
extern "C" __global__ void sf_order_bucket_scan(const uint32_t* chunk_cnt, uint32_t nc, uint32_t* chunk_rel, uint32_t* tot);
extern "C" __global__ void sf_order_scatter_plan(const uint32_t* cost, uint32_t n, uint32_t* chunk_cnt,
                                                 const uint32_t* chunk_rel, const uint32_t* tot, uint32_t split_buckets,
                                                 uint32_t parts, uint32_t spare, uint32_t waves, uint32_t prio_buckets,
                                                 uint32_t split_cap, uint32_t* order_meta, uint32_t* order);
extern "C" __global__ void sf_order_scatter(const uint32_t* cost, uint32_t n, uint32_t* chunk_cnt,
                                            const uint32_t* chunk_off, const uint32_t* order_meta, uint32_t* order,
                                            uint32_t* rank_out);
extern "C" __global__ void sf_fixup_wave(FrameArgs a, const uint32_t* overflow_list, uint32_t* counters,
                                         uint32_t parity);
extern "C" __global__ void sf_trace_ray(FrameArgs a);
extern "C" __global__ void sf_band_unpack(FrameArgs a, const float4* stage, uint32_t stage_rows, uint32_t band_rows,
                                           uint32_t n, uint32_t first, uint32_t members, uint32_t row0);
extern "C" __global__ void sf_node_table(FrameArgs a, float4* table, uint32_t nodes);
extern "C" __global__ void sf_slab_unpack4(FrameArgs a, const uint32_t* stage, const float4* table, uint32_t table_depth,
                                           uint32_t stage_rows, uint32_t band_rows, uint32_t n, uint32_t first,
                                           uint32_t members);
extern "C" __global__ void sf_post_ssao(PostArgs a);
extern "C" __global__ void sf_post_blur(PostArgs a, uint32_t dir);
extern "C" __global__ void sf_post_final(PostArgs a);
extern "C" __global__ void sf_post_fused(PostArgs a);
extern "C" __global__ void sf_mt_draws(uint32_t* state, uint32_t* out, uint32_t n);
extern "C" __global__ void sf_mt_raw(const uint32_t* state, uint32_t* raw, uint32_t blocks);
extern "C" __global__ void sf_mt_jump_partial(const uint32_t* raw, const uint64_t* polys, uint32_t poly_words,
                                              uint32_t* partial);
extern "C" __global__ void sf_mt_segments(const uint32_t* state, const uint32_t* partial, uint32_t L, uint32_t n,
                                          uint32_t* out, uint32_t* state_out);
extern "C" __global__ void sf_progressive_trace(FrameArgs a, const uint32_t* draws, uint64_t counter0, uint32_t packets,
                                                uint64_t ticket0, PacketLane* lanes, unsigned long long* owner,
                                                const uint32_t* perm, uint32_t levels, uint32_t* ovf_list,
                                                uint32_t* ovf_cnt);
extern "C" __global__ void sf_progressive_fixup(FrameArgs a, const uint32_t* draws, uint64_t counter0, uint32_t packets,
                                                uint64_t ticket0, PacketLane* lanes, unsigned long long* owner,
                                                const uint32_t* perm, const uint32_t* ovf_list, uint32_t* counters,
                                                uint32_t parity);
extern "C" __global__ void sf_progressive_fixup_sse(FrameArgs a, const uint32_t* draws, uint64_t counter0,
                                                    uint32_t packets, uint64_t ticket0, PacketLane* lanes,
                                                    unsigned long long* owner, const uint32_t* perm,
                                                    const uint32_t* ovf_list, uint32_t* counters, uint32_t parity);
extern "C" __global__ void sf_packet_bin(FrameArgs a, const uint32_t* draws, uint64_t counter0, uint32_t packets,
                                         uint32_t pw, uint32_t bin_shift, uint32_t bins_x, uint32_t* bin_cnt);
extern "C" __global__ void sf_packet_scan(uint32_t* bin_cnt, uint32_t nbins, const uint32_t* rank);
extern "C" __global__ void sf_bin_hist(const uint32_t* bin_cost, uint32_t nbins, uint32_t* chunk_cnt);
extern "C" __global__ void sf_packet_place(FrameArgs a, const uint32_t* draws, uint64_t counter0, uint32_t packets,
                                           uint32_t pw, uint32_t bin_shift, uint32_t bins_x, uint32_t* bin_cur,
                                           uint32_t* perm);
extern "C" __global__ void sf_progressive_trace_sse(FrameArgs a, const uint32_t* draws, uint64_t counter0,
                                                    uint32_t packets, uint64_t ticket0, PacketLane* lanes,
                                                    unsigned long long* owner, const uint32_t* perm, uint32_t levels,
                                                    uint32_t* ovf_list, uint32_t* ovf_cnt);
extern "C" __global__ void sf_progressive_scatter(FrameArgs a, uint32_t packets, uint64_t ticket0,
                                                  const PacketLane* lanes, const unsigned long long* owner);

static const uint32_t kLut[2048] = {
#include "rsqrtps_lut.inc"
};

namespace {

constexpr uint32_t kDefaultLevels = 12;   // depths 0..11 expand; every BASELINE camera stays <= 10
// parallel mt19937 draws (sf_mtjump.cpp, sf_kernels.hip): from this many draws per call, in K <= kMtSegMax
// segments of >= kMtSegMin draws, each jumped to by a convolution split over SF_MT_PARTS workgroups
constexpr uint32_t kMtParMin = 32768, kMtSegMin = 8192, kMtSegMax = 32;
constexpr uint32_t kMtParts = SF_MT_PARTS, kMtRawBlocks = 33;   // raw words x_0..x_20559 (19937 + 623 + 1)

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DevGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// A context's stream gets a hardware queue of its own (round 6): it is made with a CU mask of every CU, which the
// HIP runtime serves with a queue of that stream's own, not one of the GPU_MAX_HW_QUEUES queues it shares out and
// hands on from destroyed streams. Measured (profiles/r6/multi/queue_reuse/): with shared queues, a dist
// of 8 slots made after a dist of 3 or 4 had run its loops and been destroyed (the bench's legs; any process that
// renders a whole frame before a 1/8 band share) traced the share at 0.0132-0.0141 ms per frame instead of
// 0.0110-0.0113 -- every time, at the same clock, with the same buffers; not after one that made and rendered plain
// contexts, nor after a dist of 8 or 16 slots. Queues of their own: 0.0110-0.0112 in every such sequence.
// (The mask covers every CU: no CU is withheld. Such a stream is not a non-blocking one: work on the legacy default
// stream is ordered with it; the library enqueues nothing there.) SF_STREAM_CUMASK=0: a plain non-blocking stream.
bool stream_cumask_on()
{
    static const bool on = [] {
        const char* ev = std::getenv("SF_STREAM_CUMASK");
        return !ev || std::atoi(ev) != 0;
    }();
    return on;
}
// (the caller has made `device` current)
hipError_t stream_acquire(int device, hipStream_t* out)
{
    if (!stream_cumask_on()) return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
    int cus = 0;
    hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) return e;
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xffffffffu);
    if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
    if (hipExtStreamCreateWithCUMask(out, (uint32_t)mask.size(), mask.data()) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();   // (a runtime without CU-masked queues: a plain stream, as with SF_STREAM_CUMASK=0)
    return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
}

}  // namespace

struct sf_ctx {
    uint32_t fast_div = 0;             // ray generation's u = x / W by reciprocal + fma correction (host-verified)
    int device = 0;
    uint32_t W = 0, H = 0;
    hipStream_t stream = nullptr;
    float* pos = nullptr;
    float* nrm = nullptr;
    float* min_t = nullptr;
    uint32_t* hit_index = nullptr;
    int32_t* stats = nullptr;          // [0] max depth, [1] closest key, [2] unrecoverable overflow
    uint32_t* ovf_counters = nullptr;  // [0,1] overflow counts, then the tile queues (SF_QUEUE_WORD); alternating per render
    uint32_t* ovf_list = nullptr;      // 4 x tiles_x * tiles_y entries (one per work unit)
    float4* node_table = nullptr;      // index slab unpack: frames of the nodes of depth <= SF_NODE_TABLE_DEPTH
    float table_root[12];              // the root transform the table was built for
    uint32_t table_gen = 0;            // ... and consts_gen (0: no table yet)
    uint32_t consts_gen = 1;           // bumped by every constant-block upload (children, depth tables)
    struct SlabCacheEntry {            // sf_slab_bytes of recent views (gen 0: empty)
        float root[16];
        uint32_t gen = 0, bytes = 0;
    } slab_cache[64];
    uint32_t slab_cache_next = 0;
    DeviceConsts* consts = nullptr;
    DeviceConsts host_consts;
    float child[9][16];
    float root[16];
    float o[3], tl[3], tr[3], bl[3];
    bool has_view = false;
    uint32_t parity = 0;
    int64_t rays = 0;
    int last_hip = 0;
    int fixup_blocks = 256;
    uint32_t waves_per_block = SF_TRACE_WAVES;   // tuning knob: env SF_TRACE_WAVES = 1 | 2 | 4
    uint32_t levels_override = 0;                // tuning knob: env SF_LEVELS (LDS levels, 0 = adaptive)
    bool slab_shallow = false;                   // tests only: index slabs as SF_PACKED_INDEX_DIAG (env SF_DIAG_SLAB_SHALLOW)
    int frames_heavy = -1;                       // A/B: sf_render_frames' interleaved head units per frame (env
                                                 // SF_FRAMES_HEAVY; -1: the grid's waves / frames)
    bool frames_one = false;                     // A/B: sf_render_frames takes its kernel for one frame too (env SF_FRAMES_ONE)
    bool persistent = true;                      // tuning knob: env SF_PERSISTENT=0 -> one workgroup per tile group
    uint32_t flags = 0;                          // SF_FLAG_* A/B switches: env SF_FLAGS
    int cus = 256;
    uint32_t queues = 8;                         // persistent trace: XCD queue groups, one per XCD (power of 2)
    uint32_t queues_per_xcd = 4;                 // env SF_QUEUES_PER_XCD = 1 | 2 | 4: tile queues per XCD (full grids)
    int pipe = -1;                               // env SF_PIPE = 0 | 1: latency variant of the trace (-1: auto)
    uint32_t prio_buckets = 8;                   // top cost buckets (3 octaves) traced at raised wave priority (env SF_PRIO_BUCKETS)
    int occ_key = -1, occ_blocks = 0;            // cached occupancy (waves per block, levels) -> blocks per CU
    uint32_t max_blocks = 0;                     // diagnostics: env SF_MAX_BLOCKS caps the persistent grid
    int variant = SF_VARIANT_AVX;                // reference path reproduced (sf_set_variant)
    // frame-less progressive mode
    uint32_t* mt_state = nullptr;      // 624 words + next index (std::mt19937 layout)
    uint32_t* draws = nullptr;         // 2 per packet
    PacketLane* lanes = nullptr;       // 8 per packet
    uint32_t prog_cap = 0;             // packets the scratch buffers hold
    uint32_t* perm = nullptr;          // binned trace order of a batch (prog_cap)
    uint32_t* bin_cnt = nullptr;       // SF_PROG_MAX_BINS packet-bin counters / cursors
    // frame-less heavy-first trace order (env SF_PROG_ORDER=1; default off: with the packet-mode leaf
    // skip it measured 1-2 % slower, the longest waves no longer set the batch): per bin the cycles of
    // the last wave that started in it, its histogram per 64-bin chunk, and the bins' heavy-first rank
    bool prog_order = false;
    uint32_t* bin_cost = nullptr;
    uint32_t* bin_rank = nullptr;
    uint32_t* bin_order = nullptr;
    uint32_t* bin_chunk_cnt = nullptr;
    uint32_t* bin_chunk_off = nullptr;
    uint32_t* bin_meta = nullptr;
    uint32_t bin_key = 0;              // (shift, bins) of the batches whose costs bin_cost holds; 0 = none
    bool prog_bin = true;              // env SF_PROG_BIN=0: trace packets in draw order
    // Draw prefetch: after a large batch, the next batch's mt19937 draws (same stream, same size) are
    // generated on pf_stream while this batch traces -- the generator is one sequential workgroup.
    // A call that does not continue the stream restores the state saved before the prefetch.
    uint32_t* draws_pf = nullptr;      // the prefetched draws (prog_cap x 2)
    // ... and, where the batch is binned in index order, its binned trace order (the bins depend on the draws,
    // the Sobol index and the frame size only, not on the view): the next batch starts with its trace
    uint32_t* perm_pf = nullptr;       // prog_cap
    uint32_t* bin_cnt_pf = nullptr;    // SF_PROG_MAX_BINS
    uint32_t pf_bin_pl = 0;            // packet lanes the prefetched order was binned for (0: not binned)
    uint32_t* mt_saved = nullptr;      // MT state before the pending prefetch
    hipStream_t pf_stream = nullptr;
    hipEvent_t pf_done = nullptr;      // prefetch written (pf_stream)
    hipEvent_t mt_ready = nullptr;     // this batch's draws generated on the render stream
    hipEvent_t traced = nullptr;       // the last batch's trace done reading its draws
    // parallel draws (env SF_MT_PARALLEL=0: the single-workgroup generator only)
    bool mt_parallel = true;
    uint32_t mt_seg_max = kMtSegMax;   // env SF_MT_SEGMENTS: at most this many segments per call (2..kMtSegMax)
    uint32_t* mt_raw = nullptr;        // kMtRawBlocks x 624 raw words from the state's buffer
    uint32_t* mt_partial = nullptr;    // (kMtSegMax - 1) x kMtParts partial windows
    uint32_t* mt_state2 = nullptr;     // the state after the batch (copied back into mt_state)
    uint64_t* mt_polys = nullptr;      // kMtSegMax jump polynomials t^(j L) mod phi
    uint64_t mt_poly_key = 0;          // (L << 8 | K) of the uploaded polynomials
    bool traced_valid = false;
    uint32_t pf_packets = 0;           // draws pending for a batch of this many packets (0: none)
    bool prog_prefetch = true;         // env SF_PROG_PREFETCH=0: off
    // Adaptive traversal levels: LDS for the deepest level seen so far + 1 (as full frames) instead of
    // SF_PROGRESSIVE_LEVELS (twice the occupancy); a wave that needs more is re-traced by
    // sf_progressive_fixup. env SF_PROG_ADAPT=0: always SF_PROGRESSIVE_LEVELS.
    bool prog_adapt = true;
    int32_t* h_prog_depth = nullptr;   // pinned copy of the max-depth stat after each batch
    uint32_t* prog_ovf = nullptr;      // overflowed wave indices (prog_cap waves)
    uint32_t* prog_ovf_cnt = nullptr;  // [2] list counts, alternating per batch
    uint32_t prog_par = 0;
    unsigned long long* owner = nullptr;   // per pixel: highest ticket written
    bool prog_seeded = false;
    uint32_t prog_seed = 0;
    uint64_t prog_next = 0;            // Sobol counter the device MT stream is positioned at
    uint64_t ticket = 1;
    // LDS provisioning hint: max depth seen by a completed render (pinned copy of the device
    // stats word, refreshed asynchronously after every render). Only sizes the traversal stack;
    // a tile that needs more is re-traced by sf_fixup_wave, so a stale hint costs time, never results.
    int32_t* h_depth = nullptr;
    int32_t* h_stats = nullptr;        // pinned: the stats words, copied on the stream by sf_synchronize
    bool stats_dirty = true;           // work was enqueued since the last sf_synchronize checked the stats
    // the stats' unresolved word may have changed since that check: every enqueuing call but a persistent trace
    // with its levels proven and its ties re-traced inline, which adds 0 to it (its max-depth / closest words are
    // read by sf_get_stats, not here) -- after only such traces sf_synchronize needs no stats copy, just the wait
    bool stats_unknown = true;
    int32_t unresolved = 0;            // the stats' unresolved-tile count at the last check
    uint64_t* tile_trace = nullptr;    // diagnostics: per tile {start, end, hw id}
    // Heavy-first tile scheduling: every persistent render records per-tile cycles; sf_tile_order
    // turns them into the next render's tile permutation (heaviest first), so the tail of the
    // persistent kernel drains light tiles. Results never depend on the order.
    uint32_t* tile_cost = nullptr;
    uint32_t* tile_order = nullptr;
    uint32_t* chunk_cnt = nullptr;     // per 64-tile chunk x SF_ORDER_BUCKETS (zeroed by sf_order_scatter)
    uint32_t* chunk_off = nullptr;
    uint32_t* order_meta = nullptr;    // [0] work units in tile_order, [1] first split bucket, [2] parts per split tile, [3] first raised-priority bucket
    uint32_t* order_tot = nullptr;     // per cost bucket: tiles of the rebuilding render (sf_order_bucket_scan)
    uint32_t split_buckets = SF_SPLIT_AUTO;   // env SF_SPLIT_BUCKETS = k: top k buckets (0: never split)
    uint32_t split_parts = 4;          // env SF_SPLIT_PARTS = 2 (halves) | 4 (quarters); 640x360: 0.122 -> 0.097 ms with quarters
    uint32_t* part_cost = nullptr;     // per tile: slowest part of a split tile (zeroed, reset by the last part)
    uint32_t* part_done = nullptr;     // per tile: parts finished (zeroed, reset by the last part)
    // env SF_SPLIT_PARTS=subtree: split tiles traced as 4 subtree parts (SF_FLAG_SUBTREE) instead of pixel quarters;
    // part_rec holds their per-pixel results (SF_SPLIT_CAP split slots), split_depth_env the depth they divide
    // (0: the view's deepest LOD-passable depth - 2)
    uint64_t* part_rec = nullptr;
    uint32_t split_depth_env = 0;
    uint32_t order_n = 0;              // tile count the current tile_order is a permutation of (0: none)
    // Stream ordering across calls: every call that enqueues work on the context's buffers first joins
    // the stream of the previous such call (ctx_join), so renders, frame-less batches, post-processing
    // and downloads issued on different streams of one context run in call order, as on one stream.
    hipStream_t last_stream = nullptr; // stream of the latest enqueued work (nullptr: the context stream)
    hipEvent_t join_ev = nullptr;      // the point later calls order after (see ctx_join / StreamMark)
    // Heavy-first tile order: -1 (default) on whole frames whose tiles fill at most half the persistent grid's
    // waves (640x360: rebuilt after every 3rd render, costs recorded by every render) and on whole frames of more
    // than twice its waves (1080p and up: rebuilt after every 64th render (16th until round 5) from that render's costs only, model
    // splits: no steady-state cost, shorter frame ends); row-major between (1280x720) and on multi-GPU shares, where
    // with frames in flight the order measured slower (round 3); env SF_ORDER=0 never, SF_ORDER=1 always
    int order_mode = -1;
    uint32_t order_every = 0;          // env SF_ORDER_EVERY = k: rebuild the order after every k-th render only
                                       // (0 = auto: 3 for small frames, 16 for frames over twice the grid, else 1)
    int order_record_env = -1;         // env SF_ORDER_RECORD=0|1: tile costs recorded only by the render a rebuild
                                       // reads / by every render (default: only on frames over twice the grid)
    bool split_env = false;            // SF_SPLIT_BUCKETS given
    int halves = -1;                   // env SF_HALVES: row-major units as tile halves (SF_FLAG_HALVES); -1 = by policy
    // The frame-less prefetch stream at the device's greatest priority (env SF_PF_PRIO=0: normal): HIP deals streams
    // over GPU_MAX_HW_QUEUES (4) hardware queues, and in a process that made other streams first (the bench) the
    // prefetch stream shared the context stream's queue, serialising the next batch's draws behind this batch's
    // trace: SSE 0.440 -> 0.306, AVX 0.607 -> 0.480 ms per 2^18-packet batch in the bench process; a fresh process
    // measured 0.322 / 0.509 with normal priority (profiles/r4/frameless.txt)
    bool pf_prio = true;
    bool compact = false;              // env SF_COMPACT=1: the trace kernel with active-ray compaction of sparse nodes
    bool tie_inline = true;            // env SF_TIE_INLINE=0: ties under the front-first order go to sf_fixup_wave          // env SF_ORDER_RECORD=0: only the render before a rebuild records tile costs
    uint32_t order_phase = 0;          // renders since the last rebuild
    // Measurement: HIP events around the main trace kernel of each render (sf_set_kernel_timing)
    static constexpr int kTimed = 64;
    hipEvent_t ev[kTimed][2] = {};
    uint64_t* clock_buf = nullptr;     // per timed render slot: SF_CLOCK_WAVES x {memtime, realtime} at start / end
    bool timing = false;
    uint32_t ev_next = 0, ev_count = 0;
    uint32_t ev_period = 1, ev_phase = 0;   // time every ev_period-th render
    // SSAO post-process (sf_post_process): lazily allocated
    float* noise = nullptr;            // 64x64 float4
    uint8_t* ao = nullptr;             // SSAO target, sized for post_ao_px pixels
    size_t post_ao_px = 0;
    uint8_t* blur_h = nullptr;         // W x H
    uint8_t* blur_v = nullptr;
    uint8_t* image = nullptr;          // W x H RGBA8
    int centre_exact = -1;             // sfhost::post_centre_exact(W) && (H), cached
};

#define SF_HIP(ctx, expr)                                        \
    do {                                                         \
        hipError_t e_ = (expr);                                  \
        if (e_ != hipSuccess) {                                  \
            if (ctx) (ctx)->last_hip = (int)e_;                  \
            return SF_EHIP;                                      \
        }                                                        \
    } while (0)

// Order work about to be enqueued on `s` after everything the context enqueued before, on whatever
// stream (one event wait, only when the stream changes; same-stream calls cost nothing). A call that
// enqueued on a caller's stream records join_ev on it when it returns (StreamMark), so the context never
// touches that stream again afterwards: the caller may destroy it once the work is done.
static int ctx_join(sf_ctx* c, hipStream_t s)
{
    c->stats_dirty = true;   // (every call that enqueues work joins first)
    c->stats_unknown = true;   // (a trace that cannot change the unresolved word restores it, launch())
    hipStream_t last = c->last_stream ? c->last_stream : c->stream;
    if (s == last) return SF_OK;
    if (last == c->stream) SF_HIP(c, hipEventRecord(c->join_ev, c->stream));   // (the context's own stream)
    SF_HIP(c, hipStreamWaitEvent(s, c->join_ev, 0));
    c->last_stream = s == c->stream ? nullptr : s;
    return SF_OK;
}

// End of a call that enqueued on `s`: on a caller's stream, mark the point every later call orders after.
struct StreamMark {
    sf_ctx* c;
    hipStream_t s;
    StreamMark(sf_ctx* c_, hipStream_t s_) : c(c_), s(s_) {}
    ~StreamMark()
    {
        if (s != c->stream) (void)hipEventRecord(c->join_ev, s);
    }
};

// Host-synchronous drain: all work the context enqueued on any stream is done.
static int ctx_drain(sf_ctx* c)
{
    if (int rc = ctx_join(c, c->stream)) return rc;
    SF_HIP(c, hipStreamSynchronize(c->stream));
    return SF_OK;
}

static void free_ctx(sf_ctx* c)
{
    if (!c) return;
    DevGuard g(c->device);
    if (c->last_stream && c->join_ev) (void)hipEventSynchronize(c->join_ev);   // (never the caller's stream)
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->join_ev) (void)hipEventDestroy(c->join_ev);
    (void)hipFree(c->pos);
    (void)hipFree(c->nrm);
    (void)hipFree(c->min_t);
    (void)hipFree(c->hit_index);
    (void)hipFree(c->stats);
    (void)hipFree(c->ovf_counters);
    (void)hipFree(c->ovf_list);
    (void)hipFree(c->node_table);
    (void)hipFree(c->consts);
    (void)hipFree(c->mt_state);
    (void)hipFree(c->draws);
    (void)hipFree(c->lanes);
    (void)hipFree(c->perm);
    (void)hipFree(c->bin_cnt);
    (void)hipFree(c->bin_cost);
    (void)hipFree(c->bin_rank);
    (void)hipFree(c->bin_order);
    (void)hipFree(c->bin_chunk_cnt);
    (void)hipFree(c->bin_chunk_off);
    (void)hipFree(c->bin_meta);
    if (c->pf_stream) (void)hipStreamSynchronize(c->pf_stream);
    if (c->h_prog_depth) (void)hipHostFree(c->h_prog_depth);
    (void)hipFree(c->prog_ovf);
    (void)hipFree(c->prog_ovf_cnt);
    (void)hipFree(c->draws_pf);
    (void)hipFree(c->perm_pf);
    (void)hipFree(c->bin_cnt_pf);
    (void)hipFree(c->mt_saved);
    (void)hipFree(c->mt_raw);
    (void)hipFree(c->mt_partial);
    (void)hipFree(c->mt_state2);
    (void)hipFree(c->mt_polys);
    if (c->pf_done) (void)hipEventDestroy(c->pf_done);
    if (c->mt_ready) (void)hipEventDestroy(c->mt_ready);
    if (c->traced) (void)hipEventDestroy(c->traced);
    if (c->pf_stream) (void)hipStreamDestroy(c->pf_stream);
    (void)hipFree(c->owner);
    if (c->h_depth) (void)hipHostFree(c->h_depth);
    if (c->h_stats) (void)hipHostFree(c->h_stats);
    (void)hipFree(c->tile_trace);
    (void)hipFree(c->tile_cost);
    (void)hipFree(c->tile_order);
    (void)hipFree(c->chunk_cnt);
    (void)hipFree(c->chunk_off);
    (void)hipFree(c->order_meta);
    (void)hipFree(c->order_tot);
    (void)hipFree(c->part_cost);
    (void)hipFree(c->part_done);
    (void)hipFree(c->part_rec);
    (void)hipFree(c->noise);
    (void)hipFree(c->ao);
    (void)hipFree(c->blur_h);
    (void)hipFree(c->blur_v);
    (void)hipFree(c->image);
    for (int i = 0; i < sf_ctx::kTimed; ++i)
        for (int j = 0; j < 2; ++j)
            if (c->ev[i][j]) (void)hipEventDestroy(c->ev[i][j]);
    (void)hipFree(c->clock_buf);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

static int upload_consts(sf_ctx* c)
{
    std::memcpy(c->host_consts.child, c->child, sizeof c->child);
    sfhost::depth_tables(&c->host_consts.dt, c->variant == SF_VARIANT_SSE ? 60.0f : 70.0f);
    for (int d = 0; d < SF_DEPTH_TABLE; ++d) {
        float* e = c->host_consts.depth8[d];
        e[0] = c->host_consts.dt.r2_bound[d];
        e[1] = c->host_consts.dt.r2_self[d];
        e[2] = c->host_consts.dt.scale[d];
        e[3] = c->host_consts.dt.lod[d];
        e[4] = sfhost::leaf_threshold(&c->host_consts.dt, (uint32_t)d);
        e[5] = std::nextafter((float)(std::sqrt((double)e[0]) * (1.0 + 2.0 * (double)SF_OCCL_MARGIN)), FLT_MAX);
        e[6] = std::nextafter((float)((double)e[3] + std::sqrt((double)e[0]) * (1.0 + 0x1p-18)), FLT_MAX);
        e[7] = 0.0f;
    }
    std::memcpy(c->host_consts.lut, kLut, sizeof kLut);
    sfhost::sobol_matrices(c->host_consts.sobol);
    c->host_consts.rw = 1.0f / (float)c->W;
    c->host_consts.rh = 1.0f / (float)c->H;
    c->host_consts.fast_div = c->fast_div ? 1u : 0u;
    c->host_consts.tx_magic = 0xffffffffu / ((c->W + 7) / 8);
    if (int rc_ = ctx_drain(c)) return rc_;   // no kernel of the context may still read the block
    ++c->consts_gen;
    SF_HIP(c, hipMemcpyAsync(c->consts, &c->host_consts, sizeof(DeviceConsts), hipMemcpyHostToDevice, c->stream));
    SF_HIP(c, hipStreamSynchronize(c->stream));
    return SF_OK;
}

static int reset_stats_dev(sf_ctx* c, int which)
{
    // which: bit0 max depth, bit1 closest
    int32_t init[2] = { -1, sf_float_key(FLT_MAX) };
    if (int rc_ = ctx_join(c, c->stream)) return rc_;   // after every render that updates the words
    if (which & 1) SF_HIP(c, hipMemcpyAsync(c->stats + 0, &init[0], 4, hipMemcpyHostToDevice, c->stream));
    if (which & 2) SF_HIP(c, hipMemcpyAsync(c->stats + 1, &init[1], 4, hipMemcpyHostToDevice, c->stream));
    SF_HIP(c, hipStreamSynchronize(c->stream));
    return SF_OK;
}

extern "C" {

int sf_abi_version(void) { return SF_ABI_VERSION; }

const char* sf_build_id(void) { return SF_SOURCE_HASH; }

int sf_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* sf_strerror(int s)
{
    switch (s) {
    case SF_OK: return "ok";
    case SF_EINVAL: return "invalid argument";
    case SF_ENOMEM: return "out of memory";
    case SF_EHIP: return "HIP runtime error";
    case SF_ENODEV: return "no such device or not a gfx950 (MI355X) device";
    case SF_ENOVIEW: return "render before SetView";
    case SF_EDEPTH: return "traversal deeper than SF_MAX_DEPTH_LIMIT";
    case SF_ESTATE: return "invalid state";
    case SF_ECOMM: return "RCCL error";
    default: return "unknown error";
    }
}

int sf_last_hip_error(const sf_ctx* ctx) { return ctx ? ctx->last_hip : 0; }

int sf_get_size(const sf_ctx* ctx, uint32_t* width, uint32_t* height)
{
    if (!ctx) return SF_EINVAL;
    if (width) *width = ctx->W;
    if (height) *height = ctx->H;
    return SF_OK;
}

int sf_create(int device, uint32_t width, uint32_t height, sf_ctx** out)
{
    if (!out || width == 0 || height == 0) return SF_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return SF_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SF_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SF_ENODEV;

    sf_ctx* c = new (std::nothrow) sf_ctx();
    if (!c) return SF_ENOMEM;
    c->device = device;
    c->W = width;
    c->H = height;
    c->fast_div = sfhost::division_by_reciprocal_exact(width) && sfhost::division_by_reciprocal_exact(height);
    c->fixup_blocks = prop.multiProcessorCount;
    c->cus = prop.multiProcessorCount;
    {   // gfx950: 32 CUs per XCD; a compute partition of the chip exposes fewer XCDs (then fewer queues)
        uint32_t x = c->cus >= 32 ? (uint32_t)c->cus / 32u : 1u, q = 1u;
        while (q * 2u <= x && q * 2u <= 8u) q *= 2u;
        c->queues = q;
        if (const char* ev = std::getenv("SF_NQUEUES")) {
            const int v = std::atoi(ev);
            if (v == 1 || v == 2 || v == 4 || v == 8) c->queues = (uint32_t)v;
        }
        if (const char* ev = std::getenv("SF_PIPE")) c->pipe = std::atoi(ev) != 0 ? 1 : 0;
        if (const char* ev = std::getenv("SF_QUEUES_PER_XCD")) {
            const int v = std::atoi(ev);
            if (v == 1 || v == 2 || v == 4) c->queues_per_xcd = (uint32_t)v;
        }
    }
    if (const char* ev = std::getenv("SF_PERSISTENT")) c->persistent = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("SF_ORDER")) c->order_mode = std::atoi(ev) != 0 ? 1 : 0;
    if (const char* ev = std::getenv("SF_COMPACT")) c->compact = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("SF_PF_PRIO")) c->pf_prio = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("SF_TIE_INLINE")) c->tie_inline = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("SF_ORDER_RECORD")) c->order_record_env = std::atoi(ev) != 0 ? 1 : 0;
    if (const char* ev = std::getenv("SF_ORDER_EVERY")) c->order_every = std::atoi(ev) > 1 ? (uint32_t)std::atoi(ev) : 1u;   // (explicit)
    if (const char* ev = std::getenv("SF_PROG_BIN")) c->prog_bin = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("SF_PROG_PREFETCH")) c->prog_prefetch = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("SF_PROG_ADAPT")) c->prog_adapt = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("SF_PROG_ORDER")) c->prog_order = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("SF_MT_PARALLEL")) c->mt_parallel = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("SF_MT_SEGMENTS")) {
        const int k = std::atoi(ev);
        c->mt_seg_max = k < 2 ? 2u : k > (int)kMtSegMax ? kMtSegMax : (uint32_t)k;
    }
    if (const char* ev = std::getenv("SF_SPLIT_BUCKETS"))
        c->split_buckets = std::strcmp(ev, "model") == 0 ? SF_SPLIT_MODEL
                         : std::strcmp(ev, "auto") == 0 ? SF_SPLIT_AUTO : (uint32_t)std::atoi(ev);
    if (std::getenv("SF_SPLIT_BUCKETS")) c->split_env = true;
    if (const char* ev = std::getenv("SF_HALVES")) c->halves = std::atoi(ev);
    bool subtree = false;
    if (const char* ev = std::getenv("SF_SPLIT_PARTS")) {
        subtree = std::strcmp(ev, "subtree") == 0;
        c->split_parts = (subtree || std::atoi(ev) == 4) ? 4u : 2u;
    }
    if (const char* ev = std::getenv("SF_SPLIT_DEPTH")) c->split_depth_env = (uint32_t)std::atoi(ev);
    if (const char* ev = std::getenv("SF_MAX_BLOCKS")) c->max_blocks = (uint32_t)std::atoi(ev);
    if (const char* ev = std::getenv("SF_PRIO_BUCKETS")) c->prio_buckets = (uint32_t)std::atoi(ev);
    if (const char* ev = std::getenv("SF_FLAGS")) c->flags = (uint32_t)std::strtoul(ev, nullptr, 0);
    if (const char* ev = std::getenv("SF_TRACE_WAVES")) {
        const int w = std::atoi(ev);
        c->waves_per_block = (w == 1 || w == 2 || w == 4) ? (uint32_t)w : SF_TRACE_WAVES;
    } else if (c->compact || c->pipe == 1) {
        c->waves_per_block = 2;   // the compaction and pipelined (latency) variants are 2-wave kernels
    }
    if (const char* ev = std::getenv("SF_LEVELS")) {
        const int l = std::atoi(ev);
        c->levels_override = (l >= 2 && l <= SF_MAX_DEPTH_LIMIT) ? (uint32_t)l : 0u;
    }
    if (const char* ev = std::getenv("SF_DIAG_SLAB_SHALLOW")) c->slab_shallow = std::atoi(ev) != 0;   // (tests only)
    if (const char* ev = std::getenv("SF_FRAMES_HEAVY")) c->frames_heavy = std::atoi(ev);
    if (const char* ev = std::getenv("SF_FRAMES_ONE")) c->frames_one = std::atoi(ev) != 0;
    DevGuard g(device);
    const size_t npx = (size_t)width * height;
    const size_t ntiles = (size_t)((width + 7) / 8) * ((height + 7) / 8);
    if (ntiles > (size_t)SF_UNIT_TILE_MASK + 1u) {   // a work unit holds the tile index in 27 bits
        delete c;
        return SF_EINVAL;
    }
    auto fail = [&](hipError_t e) {
        c->last_hip = (int)e;
        free_ctx(c);
        return e == hipErrorOutOfMemory ? SF_ENOMEM : SF_EHIP;
    };
    hipError_t e;
    if ((e = stream_acquire(device, &c->stream)) != hipSuccess) return fail(e);
    if ((e = hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->pos, npx * 16)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->nrm, npx * 16)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->min_t, npx * 4)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->hit_index, npx * 4)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->stats, 16)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->ovf_counters, SF_COUNTER_WORDS * 4)) != hipSuccess) return fail(e);
    // each work unit pushes its tile at most once and a tile has <= 4 units: 4 entries per tile
    if ((e = hipMalloc(&c->ovf_list, 4 * ntiles * 4)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->tile_cost, ntiles * 4)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->tile_order, 4 * ntiles * 4)) != hipSuccess) return fail(e);   // <= 4 units per tile
    if ((e = hipMalloc(&c->order_meta, 4 * 4)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->order_tot, SF_ORDER_BUCKETS * 4)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->part_cost, ntiles * 4)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->part_done, ntiles * 4)) != hipSuccess) return fail(e);
    if ((e = hipMemsetAsync(c->part_cost, 0, ntiles * 4, c->stream)) != hipSuccess) return fail(e);
    if ((e = hipMemsetAsync(c->part_done, 0, ntiles * 4, c->stream)) != hipSuccess) return fail(e);
    if (subtree && (e = hipMalloc(&c->part_rec, (size_t)SF_SPLIT_CAP * 4u * 192u * 8u)) != hipSuccess) return fail(e);
    const size_t nchunks = (ntiles + 63) / 64;
    if ((e = hipMalloc(&c->chunk_cnt, nchunks * SF_ORDER_BUCKETS * 4)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->chunk_off, nchunks * SF_ORDER_BUCKETS * 4)) != hipSuccess) return fail(e);
    if ((e = hipMemsetAsync(c->chunk_cnt, 0, nchunks * SF_ORDER_BUCKETS * 4, c->stream)) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&c->consts, sizeof(DeviceConsts))) != hipSuccess) return fail(e);
    if ((e = hipHostMalloc(&c->h_depth, 4, hipHostMallocDefault)) != hipSuccess) return fail(e);
    if ((e = hipHostMalloc(&c->h_stats, 16, hipHostMallocDefault)) != hipSuccess) return fail(e);
    *c->h_depth = -1;
    // G-buffer starts as glm vec4() = (0,0,0,0) (Sphereflake.cpp:48-49, type_vec4.inl:59-64)
    if ((e = hipMemsetAsync(c->pos, 0, npx * 16, c->stream)) != hipSuccess) return fail(e);
    if ((e = hipMemsetAsync(c->nrm, 0, npx * 16, c->stream)) != hipSuccess) return fail(e);
    if ((e = hipMemsetAsync(c->min_t, 0, npx * 4, c->stream)) != hipSuccess) return fail(e);
    if ((e = hipMemsetAsync(c->hit_index, 0xff, npx * 4, c->stream)) != hipSuccess) return fail(e);
    if ((e = hipMemsetAsync(c->stats, 0, 16, c->stream)) != hipSuccess) return fail(e);
    if ((e = hipMemsetAsync(c->ovf_counters, 0, SF_COUNTER_WORDS * 4, c->stream)) != hipSuccess) return fail(e);
    sfhost::child_transforms(c->child);
    int rc = upload_consts(c);
    if (rc == SF_OK) rc = reset_stats_dev(c, 3);
    if (rc != SF_OK) {
        free_ctx(c);
        return rc;
    }
    *out = c;
    return SF_OK;
}

void sf_destroy(sf_ctx* ctx) { free_ctx(ctx); }

int sf_set_view(sf_ctx* c, const float origin[3], const float tl[3], const float tr[3], const float bl[3])
{
    if (!c || !origin || !tl || !tr || !bl) return SF_EINVAL;
    std::memcpy(c->o, origin, 12);
    std::memcpy(c->tl, tl, 12);
    std::memcpy(c->tr, tr, 12);
    std::memcpy(c->bl, bl, 12);
    sfhost::root_transform(origin, c->root);
    c->has_view = true;
    return SF_OK;
}

int sf_set_setup(sf_ctx* c, const float child[9][16], const float root[16])
{
    if (!c || !child || !root) return SF_EINVAL;
    // the kernels fuse the 4th term of every child product (SF_AFFINE_FMA, sf_kernels.hip): exact only for affine unit
    // child frames, row 3 = (0, 0, 0, 1) -- what the reference's ComputeChildTransformations makes
    for (int i = 0; i < 9; ++i)
        for (int col = 0; col < 4; ++col)
            if (child[i][4 * col + 3] != (col == 3 ? 1.0f : 0.0f)) return SF_EINVAL;
    DevGuard g(c->device);
    std::memcpy(c->child, child, sizeof c->child);
    std::memcpy(c->root, root, sizeof c->root);
    return upload_consts(c);
}

int sf_get_setup(const sf_ctx* c, float child[9][16], float root[16])
{
    if (!c) return SF_EINVAL;
    if (child) std::memcpy(child, c->child, sizeof c->child);
    if (root) std::memcpy(root, c->root, sizeof c->root);
    return SF_OK;
}

uint32_t sf_slab_rows(uint32_t height, uint32_t band_rows, uint32_t band_count, uint32_t band_index)
{
    if (band_rows == 0) band_rows = ((height + 7) / 8) * 8;
    if (band_count == 0) band_count = 1;
    uint32_t bands = (height + band_rows - 1) / band_rows, rows = 0;
    for (uint32_t b = band_index; b < bands; b += band_count) {
        uint32_t y0 = b * band_rows, y1 = y0 + band_rows < height ? y0 + band_rows : height;
        rows += y1 - y0;
    }
    return rows;
}

static FrameArgs frame_args(const sf_ctx* c)
{
    FrameArgs a;
    std::memset(&a, 0, sizeof a);
    a.W = c->W;
    a.H = c->H;
    a.fw = (float)c->W;                  // (float)m_Width (Sphereflake.cpp:104-110)
    a.fh = (float)c->H;
    for (int k = 0; k < 3; ++k) {
        a.o[k] = c->o[k];
        a.tl[k] = c->tl[k];
        a.dh[k] = c->tr[k] - c->tl[k];   // m_TopRight - m_TopLeft (Sphereflake.cpp:162)
        a.dv[k] = c->bl[k] - c->tl[k];   // m_BottomLeft - m_TopLeft (Sphereflake.cpp:163)
    }
    for (int col = 0; col < 4; ++col)
        for (int r = 0; r < 3; ++r) a.root[3 * col + r] = c->root[4 * col + r];
    a.tiles_x = (c->W + 7) / 8;
    a.band_count = 1;
    a.consts = c->consts;
    a.stats = c->stats;
    a.flags = c->flags;
    a.xcds = c->queues;
    a.queues = c->queues;   // (x queues per XCD once the persistent grid is known, launch())
    return a;
}

// The next render's tile order from the tile costs the render just enqueued on `s` recorded (sf_order_scan /
// sf_order_bucket_scan + sf_order_scatter_plan); `waves`: resident waves of its persistent grid.
static int order_rebuild(sf_ctx* c, hipStream_t s, uint32_t ntiles, uint32_t waves, uint32_t split_buckets)
{
    const uint32_t nc = (ntiles + 63u) / 64u;
    const uint32_t spare = waves > ntiles ? waves - ntiles : 0u;
    // few chunks: the scan's workgroup also scatters (one launch: ~3 us less host time and one
    // dispatch less on the frame's stream); more: one wave per chunk in a launch of its own
    const bool fuse = nc <= SF_ORDER_FUSE_CHUNKS;
    const uint32_t cap = c->part_rec ? SF_SPLIT_CAP : 0xffffffffu;
    if (fuse) {
        hipLaunchKernelGGL(sf_order_scan, dim3(1), dim3(1024), 0, s, c->chunk_cnt, nc, ntiles, split_buckets,
                           c->split_parts, spare, waves, c->prio_buckets, c->chunk_off, c->order_meta,
                           (const uint32_t*)c->tile_cost, c->tile_order, cap);
        SF_HIP(c, hipGetLastError());
    } else {   // (round 5: one-wave workgroups only -- see sf_order_bucket_scan)
        hipLaunchKernelGGL(sf_order_bucket_scan, dim3(SF_ORDER_BUCKETS), dim3(64), 0, s, (const uint32_t*)c->chunk_cnt,
                           nc, c->chunk_off, c->order_tot);
        SF_HIP(c, hipGetLastError());
        hipLaunchKernelGGL(sf_order_scatter_plan, dim3(nc), dim3(64), 0, s, (const uint32_t*)c->tile_cost, ntiles,
                           c->chunk_cnt, (const uint32_t*)c->chunk_off, (const uint32_t*)c->order_tot, split_buckets,
                           c->split_parts, spare, waves, c->prio_buckets, cap, c->order_meta, c->tile_order);
        SF_HIP(c, hipGetLastError());
    }
    c->order_n = ntiles;
    return SF_OK;
}

// LDS traversal levels for the context's view, and whether they are proven sufficient (no tile can overflow).
// Geometric bound: every sphere lies inside the root's bounding sphere (radius 2 around the root centre), so a
// depth-d node can pass the LOD test (t < T_d, Sphereflake.h:146) only if |root centre| - 2 < T_d. The deepest such
// d + 1 levels suffice; a bound that is off only costs a re-trace of the affected tiles (sf_fixup_wave), never results.
static uint32_t frame_levels(const sf_ctx* c, bool* bounded_out)
{
    uint32_t levels = kDefaultLevels;
    const float rc = std::sqrt(c->root[12] * c->root[12] + c->root[13] * c->root[13] + c->root[14] * c->root[14]);
    const float gap = (rc - 2.0f) * (1.0f - 1e-3f);
    bool bounded = false;
    if (gap > 0.0f) {
        uint32_t dmax = 0;
        while (dmax + 1u < SF_DEPTH_TABLE && c->host_consts.dt.lod[dmax + 1u] > gap) ++dmax;
        levels = dmax + 1u;
        bounded = levels <= SF_MAX_DEPTH_LIMIT;
    }
    const int32_t seen = *(volatile int32_t*)c->h_depth;   // max depth of a finished render
    if (seen >= 0 && (uint32_t)seen + 1u < levels) {
        levels = (uint32_t)seen + 1u;
        bounded = false;
    }
    if (levels < 4u) levels = 4u;
    if (levels > SF_MAX_DEPTH_LIMIT) levels = SF_MAX_DEPTH_LIMIT;
    if (c->levels_override) {
        levels = c->levels_override;
        bounded = false;
    }
    *bounded_out = bounded;
    return levels;
}

static int launch(sf_ctx* c, const sf_render_params* pp, float* pos, float* nrm, float* min_t, uint32_t* hidx)
{
    if (!c) return SF_EINVAL;
    if (!c->has_view) return SF_ENOVIEW;
    if (!pos || !nrm) return SF_EINVAL;
    sf_render_params p;
    std::memset(&p, 0, sizeof p);
    if (pp) p = *pp;
    const uint32_t tiles_y = (c->H + 7) / 8;
    uint32_t band_rows = p.band_rows ? p.band_rows : tiles_y * 8;
    uint32_t band_count = p.band_count ? p.band_count : 1;
    if (band_rows % 8 != 0 || p.band_index >= band_count) return SF_EINVAL;
    if (p.kernel > SF_KERNEL_PER_RAY || p.max_depth > SF_MAX_DEPTH_LIMIT) return SF_EINVAL;
    const uint32_t tpb = band_rows / 8;
    const uint32_t bands = (tiles_y + tpb - 1) / tpb;
    // owned tile rows: full bands for all but possibly the frame's last band
    uint32_t tile_rows = 0;
    for (uint32_t b = p.band_index; b < bands; b += band_count) {
        uint32_t t0 = b * tpb, t1 = t0 + tpb < tiles_y ? t0 + tpb : tiles_y;
        tile_rows += t1 - t0;
    }
    hipStream_t s = p.stream ? (hipStream_t)p.stream : c->stream;
    DevGuard g(c->device);
    if (tile_rows == 0) return SF_OK;
    const bool unknown_before = c->stats_unknown;
    if (int rc = ctx_join(c, s)) return rc;
    StreamMark mark_(c, s);

    FrameArgs a = frame_args(c);
    bool unresolved_safe = false;   // this launch adds nothing to the unresolved word (see sf_ctx::stats_unknown)
    a.tile_rows = tile_rows;
    a.tiles_per_band = tpb;
    a.tpb_magic = 0xffffffffu / tpb;
    a.band_count = band_count;
    a.band_index = p.band_index;
    a.compact = p.compact ? 1u : 0u;
    if (p.packed > SF_PACKED_INDEX) return SF_EINVAL;
    if (p.packed == SF_PACKED_INDEX && sf_slab_bytes(c) != 4u) return SF_EINVAL;   // (a hit could be too deep)
    a.packed = p.packed;
    if (a.packed == SF_PACKED_INDEX && c->slab_shallow) a.packed = SF_PACKED_INDEX_DIAG;
    if (a.packed && p.kernel == SF_KERNEL_PER_RAY) return SF_EINVAL;   // (the per-ray kernel writes the plain layout)
    a.emit_aux = p.emit_aux ? 1u : 0u;
    a.pos = pos;
    a.nrm = nrm;
    a.min_t = min_t;
    a.hit_index = hidx;
    a.tile_trace = c->tile_trace;
    a.counters = c->ovf_counters;
    a.overflow_list = c->ovf_list;
    a.parity = c->parity;
    if (c->tile_trace) {
        const size_t ntr = (size_t)((c->W + 7) / 8) * ((c->H + 7) / 8);
        a.phase_sums = c->tile_trace + 3 * ntr;
    }

    const uint32_t ntiles = a.tiles_x * tile_rows;
    const uint32_t blocks = (ntiles + SF_WAVES_PER_BLOCK - 1) / SF_WAVES_PER_BLOCK;
    if (p.kernel == SF_KERNEL_PER_RAY) {
        a.max_depth = 31;
        hipLaunchKernelGGL(sf_trace_ray, dim3(blocks), dim3(256), 0, s, a);
        SF_HIP(c, hipGetLastError());
    } else {
        const bool autod = p.max_depth == 0;
        bool bounded = false;   // levels proven sufficient: no tile can overflow
        uint32_t levels = frame_levels(c, &bounded);
        if (!autod) bounded = bounded && p.max_depth >= levels;
        a.max_depth = autod ? levels : p.max_depth;
        const size_t lds = (size_t)SF_LDS_WAVE_FLOATS(a.max_depth) * 4;
        uint32_t* cnt = c->ovf_counters + c->parity;
        const uint32_t wpb = c->waves_per_block;
        const dim3 block(64 * wpb);
        // levels proven sufficient on the persistent kernel: only a tie under the front-first child order can flag
        // a tile, and its own wave re-traces it in index order -- no fixup launch after the trace
        const bool front_first = (c->flags & (SF_FLAG_NO_OCCL_CULL | SF_FLAG_NO_FRONT_FIRST)) == 0u;
        const bool tie_inline = bounded && c->persistent && front_first && c->tie_inline;
        if (tie_inline) a.flags |= SF_FLAG_TIE_INLINE;
        if (c->persistent) {
            const void* kern = wpb == 1 ? (const void*)sf_trace_queue1
                             : wpb == 2 ? (c->compact ? (const void*)sf_trace_queue2c : (const void*)sf_trace_queue2)
                                        : (const void*)sf_trace_queue4;
            const int key = (int)(wpb * 64 + a.max_depth) | (c->compact ? 1 << 20 : 0);
            if (c->occ_key != key) {
                int nb = 0;
                SF_HIP(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, (int)block.x, wpb * lds));
                c->occ_blocks = nb < 1 ? 1 : nb;
                c->occ_key = key;
            }
            uint32_t nblk = (uint32_t)c->occ_blocks * (uint32_t)c->cus;
            const bool small = ntiles <= 2u * nblk * wpb;   // tiles fill the full persistent grid at most twice
            // The heavy-first order (and the splits it carries) only where the frame's tiles fill at most half
            // the grid's waves: there idle slots take the split heaviest tiles and shorten the frame. With 3
            // frames in flight, frames of more tiles are throughput-bound and the order costs more than it
            // gains: 1280x720 0.039 -> 0.036 ms, a 1080p member's share over 2 / 4 GPUs 0.045 -> 0.042 /
            // 0.028 -> 0.026 ms without it, while 640x360 keeps it (0.0203 vs 0.0232 ms on a fixed view).
            // A member's share of a multi-GPU frame (band_count > 1) stays row-major too: its tiles are every N-th
            // band row of the frame, and with frames in flight the order measured slower there at every N (1080p
            // over 8 GPUs: 0.0212 vs 0.0204 ms per frame, `profiles/r3/share2/r3aw.txt`).
            const bool tiny = 2u * ntiles <= nblk * wpb && band_count == 1u;
            // Round 4: whole frames of more than twice the grid's waves (1080p and up) take the order too, in a form
            // that costs the steady state nothing: rebuilt after every 16th render (64th since round 5, below) from that render's tile costs
            // alone (the renders between record nothing), heavy tiles split by the makespan model. With 3 frames in
            // flight the steady frame period is unchanged (1080p 0.0787 vs 0.0792 ms, 4K 0.373 vs 0.373), but a
            // frame whose successors are not yet queued -- the last of a timed loop, a lone frame -- no longer ends
            // on its heaviest tiles' serial traversal: one frame alone 0.175 -> 0.151-0.164 ms at 1080p, and the
            // driver's 20-step loop 0.0871 -> 0.0846 ms per frame (mean of 4 interleaved runs a side,
            // profiles/r4/order_ab.txt). Frames between half and twice the grid (1280x720) measured slower with it
            // (0.0358 -> 0.0388 ms) and keep the row-major order. End of round 4, with the faster kernel: large
            // frames take the order WITHOUT splits -- the split parts re-traverse their tile's shared upper levels,
            // and with frames in flight only the loop's last frame gains from them: the 20-step loop 0.0759-0.0782
            // -> 0.0748-0.0766 ms, one frame alone 0.133-0.136 -> 0.129-0.139, steady period unchanged (5
            // interleaved runs a side, profiles/r4/split0_ab.txt).
            const bool large = !small && band_count == 1u;
            const bool use_order = c->order_mode > 0 || (c->order_mode < 0 && (tiny || large));
            const uint32_t split_buckets = (large && !c->split_env) ? 0u : c->split_buckets;
            // row-major halves (SF_FLAG_HALVES): every tile as two units of its pixel rows 0-3 / 4-7
            const bool halves = !use_order && c->halves > 0;
            if (halves) a.flags |= SF_FLAG_HALVES;
            // work units: tiles, or up to `split_parts` per tile when the schedule may split tiles
            const uint32_t units_max = (use_order && split_buckets != 0u) ? c->split_parts * ntiles
                                                                          : halves ? 2u * ntiles : ntiles;
            const uint32_t need = (units_max + wpb - 1) / wpb;
            if (nblk > need) nblk = need;
            if (c->max_blocks && nblk > c->max_blocks) nblk = c->max_blocks;
            const dim3 grid(nblk);
            // every queue group needs blocks of its own (the group is blockIdx mod xcds): fewer queues for a
            // grid of fewer blocks than groups
            while (a.xcds > 1u && a.xcds > nblk) a.xcds >>= 1;
            a.queues = a.xcds;
            // several queues per XCD split each XCD's tickets over as many counters (less contention on
            // each); every queue needs waves of its own, so only with a full grid (>= 64 waves per queue)
            if (c->queues_per_xcd > 1u && nblk * wpb >= 64u * a.xcds * c->queues_per_xcd)
                a.queues = a.xcds * c->queues_per_xcd;
            // the order is rebuilt after every order_every-th render (and whenever none exists for this frame
            // size); the renders in between keep the last order and record their tile costs only
            // Small frames (tiles fill the persistent grid less than twice) are latency-bound: there the stale
            // order costs the trace nothing measurable while the two order kernels are ~5 us of a ~80 us
            // frame, so by default they are rebuilt after every 3rd render (640x360 -6 %, 1280x720 -4 %);
            // full grids are throughput-bound and a stale order costs more than the kernels (1080p).
            // (large frames: every 64th since round 5 -- the rebuild's scan is one 16-wave workgroup, which waits for
            // wave slots behind the frames in flight, 64 us median and up to 1.6 ms in the bench, with its slot's next
            // frame queued behind it: the driver's 20-step loop 0.0727-0.0743 -> 0.0721-0.0722 ms in two 5-run A/Bs;
            // a one-wave scan, or the rebuild on a stream of its own, measured slower, profiles/r5/order/)
            const uint32_t every = c->order_every ? c->order_every : (small ? 3u : large ? 64u : 1u);
            const bool rebuild = use_order && (c->order_n != ntiles || c->order_phase + 1u >= every);
            if (use_order) c->order_phase = rebuild ? 0u : c->order_phase + 1u;
            if (use_order) {
                // tile costs: recorded by every render, or only by the render whose costs the rebuild reads
                const bool record = c->order_record_env >= 0 ? c->order_record_env != 0 : !large;
                a.tile_cost = (rebuild || record) ? c->tile_cost : nullptr;
                a.chunk_cnt = rebuild ? c->chunk_cnt : nullptr;
                a.part_cost = c->part_cost;
                a.part_done = c->part_done;
                if (c->part_rec && split_buckets != 0u && wpb == 1u) {   // split tiles are traced as subtree parts
                    a.part_rec = c->part_rec;
                    a.split_depth = c->split_depth_env ? c->split_depth_env : (levels > 3u ? levels - 3u : 1u);
                    a.flags |= SF_FLAG_SUBTREE;
                }
                a.tile_order = c->order_n == ntiles ? c->tile_order : nullptr;   // ordered by ctx_join
                a.order_meta = c->order_meta;
            }
            const bool timed = c->timing && c->ev_phase == 0;
            if (c->timing) c->ev_phase = (c->ev_phase + 1u) % c->ev_period;
            if (timed) {
                SF_HIP(c, hipEventRecord(c->ev[c->ev_next][0], s));
                a.clock_probe = c->clock_buf + (size_t)c->ev_next * SF_CLOCK_WAVES * 4u;
            }
            // small frames (tiles fill the persistent grid less than twice) are latency-bound: the heaviest
            // tiles' serial DFS is the frame, and the pipelined child loop shortens it (640x360 -4 %); full
            // grids are throughput-bound, where it costs more instructions than it hides (1080p +1.7 %)
            const bool pipe = c->pipe >= 0 ? c->pipe == 1 : small;
            if (wpb == 1 && (a.flags & SF_FLAG_SUBTREE)) hipLaunchKernelGGL(sf_trace_queue1s, grid, block, lds, s, a);
            else if (wpb == 1) hipLaunchKernelGGL(sf_trace_queue1, grid, block, lds, s, a);
            else if (wpb == 2 && pipe) hipLaunchKernelGGL(sf_trace_queue2p, grid, block, 2 * lds, s, a);
            else if (wpb == 2 && c->compact) hipLaunchKernelGGL(sf_trace_queue2c, grid, block, 2 * lds, s, a);
            else if (wpb == 2) hipLaunchKernelGGL(sf_trace_queue2, grid, block, 2 * lds, s, a);
            else hipLaunchKernelGGL(sf_trace_queue4, grid, block, 4 * lds, s, a);
            SF_HIP(c, hipGetLastError());
            if (timed) {
                SF_HIP(c, hipEventRecord(c->ev[c->ev_next][1], s));
                c->ev_next = (c->ev_next + 1u) % sf_ctx::kTimed;
                c->ev_count = c->ev_count < (uint32_t)sf_ctx::kTimed ? c->ev_count + 1u : c->ev_count;
            }
            if (rebuild) {   // the next render's tile order, from this render's tile costs
                if (int rc = order_rebuild(c, s, ntiles, nblk * wpb, split_buckets)) return rc;
            }
        } else {
            const dim3 grid((ntiles + wpb - 1) / wpb);
            if (wpb == 1) hipLaunchKernelGGL(sf_trace_wave1, grid, block, lds, s, a, c->ovf_list, cnt);
            else if (wpb == 2) hipLaunchKernelGGL(sf_trace_wave2, grid, block, 2 * lds, s, a, c->ovf_list, cnt);
            else hipLaunchKernelGGL(sf_trace_wave4, grid, block, 4 * lds, s, a, c->ovf_list, cnt);
        }
        SF_HIP(c, hipGetLastError());
        // Re-trace of overflowed tiles (it also zeroes the next render's overflow counter itself). With the
        // levels proven sufficient (persistent kernel) only an exact tie under the front-first child order can
        // flag a tile -- never seen on the BASELINE views --: its own wave re-traces it (tie_inline), or with
        // SF_TIE_INLINE=0 the fixup's small grid.
        // (no fixup after the trace: nothing is counted as unresolved -- except by an index-slab trace, whose
        // write_pixel counts a hit too deep for the format (SF_SLAB_BAD): that one must leave stats_unknown set so
        // sf_synchronize reads the word and reports SF_EDEPTH (VERDICT/ADVICE r5))
        unresolved_safe = bounded && c->persistent && !(front_first && !tie_inline) && a.packed < SF_PACKED_INDEX;
        if (!(bounded && c->persistent) || (front_first && !tie_inline)) {
            const size_t lds_fix = (size_t)SF_LDS_WAVE_FLOATS(SF_MAX_DEPTH_LIMIT) * 4;
            const uint32_t fb = (bounded && c->persistent) ? 8u : 4u * (uint32_t)c->fixup_blocks;
            hipLaunchKernelGGL(sf_fixup_wave, dim3(fb), dim3(64), lds_fix, s, a,
                               (const uint32_t*)c->ovf_list, c->ovf_counters, c->parity);
            SF_HIP(c, hipGetLastError());
        }
        c->parity ^= 1u;
        // LDS-level hint for later renders: only needed when the geometric bound is unavailable
        if (!bounded) SF_HIP(c, hipMemcpyAsync(c->h_depth, c->stats, 4, hipMemcpyDeviceToHost, s));
    }
    uint32_t rows = 0;
    for (uint32_t b = p.band_index; b < bands; b += band_count) {
        uint32_t y0 = b * band_rows, y1 = y0 + band_rows < c->H ? y0 + band_rows : c->H;
        rows += y1 - y0;
    }
    c->rays += (int64_t)rows * c->W;
    if (unresolved_safe) c->stats_unknown = unknown_before;
    return SF_OK;
}

int sf_render(sf_ctx* c, const sf_render_params* p)
{
    if (!c) return SF_EINVAL;
    return launch(c, p, c->pos, c->nrm, c->min_t, c->hit_index);
}

int sf_render_to(sf_ctx* c, const sf_render_params* p, float* pos4, float* nrm4, float* min_t, uint32_t* hidx)
{
    if (p && p->packed && !nrm4) nrm4 = pos4;   // (packed slabs write pos4 only)
    return launch(c, p, pos4, nrm4, min_t, hidx);
}

// Multi-frame persistent trace (sf.h; kernel sf_trace_frames1). One launch where every frame's own launch() would be
// a bounded persistent one-wave trace (levels proven for its view, ties re-traced inline, no fixup launch), else one
// launch() per frame. The frames share the first context's tile queues, its unit order (rebuilt from frame 0's costs
// on its schedule) and its kernel timing; each frame writes its own context's G-buffer, aux channels and stats.
int sf_render_frames(sf_ctx* const* cs, uint32_t n, const sf_render_params* pp)
{
    static_assert(SF_RENDER_FRAMES_MAX <= (int)SF_BATCH_MAX, "the batch travels in the kernel argument segment");
    static_assert(sizeof(FrameBatch) <= 4096, "kernel argument segment");
    if (!cs || n == 0 || n > (uint32_t)SF_RENDER_FRAMES_MAX) return SF_EINVAL;
    sf_render_params p;
    std::memset(&p, 0, sizeof p);
    if (pp) p = *pp;
    if (p.compact || p.packed || p.kernel == SF_KERNEL_PER_RAY || p.max_depth) return SF_EINVAL;
    sf_ctx* const c0 = cs[0];
    for (uint32_t k = 0; k < n; ++k) {
        if (!cs[k]) return SF_EINVAL;
        if (!cs[k]->has_view) return SF_ENOVIEW;
        if (cs[k]->device != c0->device || cs[k]->W != c0->W || cs[k]->H != c0->H) return SF_EINVAL;
        for (uint32_t j = 0; j < k; ++j)
            if (cs[j] == cs[k]) return SF_EINVAL;   // (two frames into one G-buffer in one launch would race)
    }
    const uint32_t tiles_y = (c0->H + 7) / 8;
    const uint32_t band_rows = p.band_rows ? p.band_rows : tiles_y * 8;
    const uint32_t band_count = p.band_count ? p.band_count : 1;
    if (band_rows % 8 != 0 || p.band_index >= band_count || p.kernel > SF_KERNEL_PER_RAY) return SF_EINVAL;
    // one launch only where each frame alone would take the bounded one-wave persistent trace with nothing after it
    uint32_t levels = 0;
    bool one = n > 1 || c0->frames_one;
    for (uint32_t k = 0; k < n && one; ++k) {
        const sf_ctx* c = cs[k];
        bool bounded = false;
        const uint32_t l = frame_levels(c, &bounded);
        const bool front_first = (c->flags & (SF_FLAG_NO_OCCL_CULL | SF_FLAG_NO_FRONT_FIRST)) == 0u;
        one = bounded && c->persistent && c->waves_per_block == 1u && !c->compact && !c->part_rec && !c->tile_trace &&
              !(front_first && !c->tie_inline) && c->flags == c0->flags && c->variant == c0->variant &&
              !(c->flags & SF_FLAG_DIAG_HALF);
        levels = l > levels ? l : levels;
    }
    if (!one) {   // one launch per frame: the same frames (launch() orders each context's own calls)
        for (uint32_t k = 0; k < n; ++k)
            if (int rc = launch(cs[k], &p, cs[k]->pos, cs[k]->nrm, cs[k]->min_t, cs[k]->hit_index)) return rc;
        return SF_OK;
    }
    const uint32_t tpb = band_rows / 8;
    const uint32_t bands = (tiles_y + tpb - 1) / tpb;
    uint32_t tile_rows = 0, rows = 0;
    for (uint32_t b = p.band_index; b < bands; b += band_count) {
        const uint32_t t0 = b * tpb, t1 = t0 + tpb < tiles_y ? t0 + tpb : tiles_y;
        tile_rows += t1 - t0;
        const uint32_t y0 = b * band_rows, y1 = y0 + band_rows < c0->H ? y0 + band_rows : c0->H;
        rows += y1 - y0;
    }
    hipStream_t s = p.stream ? (hipStream_t)p.stream : c0->stream;
    DevGuard g(c0->device);
    if (tile_rows == 0) return SF_OK;
    bool unknown_before[SF_BATCH_MAX];
    for (uint32_t k = 0; k < n; ++k) {
        unknown_before[k] = cs[k]->stats_unknown;
        if (int rc = ctx_join(cs[k], s)) return rc;
    }
    const size_t lds = (size_t)SF_LDS_WAVE_FLOATS(levels) * 4;
    const int key = (int)(64 + levels) | (1 << 21);   // (c0's occupancy cache, told apart from launch()'s keys)
    if (c0->occ_key != key) {
        int nb = 0;
        SF_HIP(c0, hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)sf_trace_frames1, 64, lds));
        c0->occ_blocks = nb < 1 ? 1 : nb;
        c0->occ_key = key;
    }
    uint32_t nblk = (uint32_t)c0->occ_blocks * (uint32_t)c0->cus;
    const uint32_t ntiles = ((c0->W + 7) / 8) * tile_rows;
    // c0's order policy, as launch() decides it for one of these frames
    const bool small = ntiles <= 2u * nblk;
    const bool tiny = 2u * ntiles <= nblk && band_count == 1u;
    const bool large = !small && band_count == 1u;
    const bool use_order = c0->order_mode > 0 || (c0->order_mode < 0 && (tiny || large));
    const uint32_t split_buckets = (large && !c0->split_env) ? 0u : c0->split_buckets;
    const uint32_t units_max = (use_order && split_buckets != 0u) ? c0->split_parts * ntiles : ntiles;
    if ((uint64_t)n * units_max >= 0x20000000ull) return SF_EINVAL;   // (positions below 2^29: FrameBatch.magic)
    if (nblk > n * units_max) nblk = n * units_max;
    if (c0->max_blocks && nblk > c0->max_blocks) nblk = c0->max_blocks;
    uint32_t xcds = c0->queues;
    while (xcds > 1u && xcds > nblk) xcds >>= 1;
    uint32_t queues = xcds;
    if (c0->queues_per_xcd > 1u && nblk >= 64u * xcds * c0->queues_per_xcd) queues = xcds * c0->queues_per_xcd;
    const uint32_t every = c0->order_every ? c0->order_every : (small ? 3u : large ? 64u : 1u);
    const bool rebuild = use_order && (c0->order_n != ntiles || c0->order_phase + 1u >= every);
    if (use_order) c0->order_phase = rebuild ? 0u : c0->order_phase + 1u;
    const bool record = use_order && (c0->order_record_env >= 0 ? c0->order_record_env != 0 : !large);
    const bool front_first = (c0->flags & (SF_FLAG_NO_OCCL_CULL | SF_FLAG_NO_FRONT_FIRST)) == 0u;
    FrameBatch b;
    std::memset(&b, 0, sizeof b);
    b.nframes = n;
    b.magic = (uint32_t)((0x100000000ull + n - 1u) / n);
    b.units = ntiles;
    b.heavy = c0->frames_heavy >= 0 ? (uint32_t)c0->frames_heavy : nblk / n;   // every frame's heaviest units among
                                                                                // the waves' static first units
    for (uint32_t k = 0; k < n; ++k) {
        sf_ctx* c = cs[k];
        FrameArgs a = frame_args(c);
        a.tile_rows = tile_rows;
        a.tiles_per_band = tpb;
        a.tpb_magic = 0xffffffffu / tpb;
        a.band_count = band_count;
        a.band_index = p.band_index;
        a.emit_aux = p.emit_aux ? 1u : 0u;
        a.pos = c->pos;
        a.nrm = c->nrm;
        a.min_t = c->min_t;
        a.hit_index = c->hit_index;
        a.max_depth = levels;
        if (front_first) a.flags |= SF_FLAG_TIE_INLINE;
        a.counters = c0->ovf_counters;   // the launch's queues: c0's, at c0's parity
        a.overflow_list = c0->ovf_list;
        a.parity = c0->parity;
        a.xcds = xcds;
        a.queues = queues;
        if (use_order) {
            a.tile_order = c0->order_n == ntiles ? c0->tile_order : nullptr;
            a.order_meta = c0->order_meta;
            a.part_cost = c0->part_cost;
            a.part_done = c0->part_done;
            if (k == 0u) {   // only frame 0 records tile costs (the order and its histogram are per tile)
                a.tile_cost = (rebuild || record) ? c0->tile_cost : nullptr;
                a.chunk_cnt = rebuild ? c0->chunk_cnt : nullptr;
            }
        }
        b.f[k] = a;
    }
    const bool timed = c0->timing && c0->ev_phase == 0;
    if (c0->timing) c0->ev_phase = (c0->ev_phase + 1u) % c0->ev_period;
    if (timed) {
        SF_HIP(c0, hipEventRecord(c0->ev[c0->ev_next][0], s));
        b.f[0].clock_probe = c0->clock_buf + (size_t)c0->ev_next * SF_CLOCK_WAVES * 4u;
    }
    hipLaunchKernelGGL(sf_trace_frames1, dim3(nblk), dim3(64), lds, s, b);
    SF_HIP(c0, hipGetLastError());
    if (timed) {
        SF_HIP(c0, hipEventRecord(c0->ev[c0->ev_next][1], s));
        c0->ev_next = (c0->ev_next + 1u) % sf_ctx::kTimed;
        c0->ev_count = c0->ev_count < (uint32_t)sf_ctx::kTimed ? c0->ev_count + 1u : c0->ev_count;
    }
    if (rebuild)
        if (int rc = order_rebuild(c0, s, ntiles, nblk, split_buckets)) return rc;
    c0->parity ^= 1u;
    for (uint32_t k = 0; k < n; ++k) {
        sf_ctx* c = cs[k];
        c->rays += (int64_t)rows * c->W;
        c->stats_unknown = unknown_before[k];   // (bounded, unpacked: the launch adds nothing to the unresolved word)
        if (s != c->stream) SF_HIP(c, hipEventRecord(c->join_ev, s));   // (StreamMark)
    }
    return SF_OK;
}

// Depth bound of every hit under the context's view (-1: none provable). Every sphere lies inside the root's
// bounding sphere (radius 2 around the root centre), so a depth-d node can pass the LOD test (t < T_d,
// Sphereflake.h:146) only if |root centre| - 2 < T_d; a node is self-tested only when its parent passed, so hits
// lie at most one level below the deepest such d. (The same bound launch() provisions its LDS levels from.)
static int hit_depth_bound(const sf_ctx* c)
{
    const float rc = std::sqrt(c->root[12] * c->root[12] + c->root[13] * c->root[13] + c->root[14] * c->root[14]);
    const float gap = (rc - 2.0f) * (1.0f - 1e-3f);
    if (!(gap > 0.0f)) return -1;
    uint32_t dmax = 0;
    while (dmax + 1u < SF_DEPTH_TABLE && c->host_consts.dt.lod[dmax + 1u] > gap) ++dmax;
    return (int)dmax + 1;
}

// True when no depth-SF_INDEX_SLAB_DEPTH node can pass the LOD test for any ray of the view, so every hit lies at depth
// <= SF_INDEX_SLAB_DEPTH (heap index below 2^32). Branch and bound over the node tree in double precision: a node's
// whole subtree lies in its bounding ball (centre c, radius 2 r_d: each level's ball is internally tangent to its
// parent's), and a node at depth D can expand only if t < T_D, where its bounding root t >= |c - O| - 2 r_D (O = the
// ray origin, the frame's origin: the root transform maps it to 0). A subtree whose ball stays farther than T_D
// from O is pruned. Slack: the float chain's centres are within ~1e-6 |c| of these, the float t within ~1e-6 of
// the distance; 1e-3 relative and 1e-5 absolute cover both. The search gives up (false) past kMaxNodes nodes.
static bool index_depth_proven(const sf_ctx* c)
{
    const int D = SF_INDEX_SLAB_DEPTH;
    const double TD = (double)c->host_consts.dt.lod[D] * (1.0 + 1e-3) + 1e-5;
    struct Node {
        double m[12];   // columns 0..3, xyz (the child_frame layout)
        int d;
    };
    constexpr int kMaxNodes = 1 << 16;
    std::vector<Node> stack;
    stack.reserve(256);
    Node root;
    for (int col = 0; col < 4; ++col)
        for (int r = 0; r < 3; ++r) root.m[3 * col + r] = (double)c->root[4 * col + r];
    root.d = 0;
    stack.push_back(root);
    int visited = 0;
    while (!stack.empty()) {
        const Node nd = stack.back();
        stack.pop_back();
        if (++visited > kMaxNodes) return false;
        const double* cc = nd.m + 9;
        const double dist = std::sqrt(cc[0] * cc[0] + cc[1] * cc[1] + cc[2] * cc[2]);
        const double R = 2.0 * (double)sfhost::radius((uint32_t)nd.d) * (1.0 + 1e-6) + 1e-5 * (dist + 1.0);
        if (dist - R >= TD) continue;      // no depth-D node of this subtree comes within T_D of the origin
        if (nd.d == D) return false;       // a depth-D node that may expand: a hit could lie at depth D + 1
        const double s = (double)c->host_consts.dt.scale[nd.d];
        for (int i = 0; i < 9; ++i) {
            Node ch;
            ch.d = nd.d + 1;
            for (int col = 0; col < 4; ++col) {
                double b[4];
                for (int k = 0; k < 4; ++k) b[k] = (double)c->child[i][4 * col + k];
                if (col == 3)
                    for (int k = 0; k < 3; ++k) b[k] *= s;
                for (int r = 0; r < 3; ++r)
                    ch.m[3 * col + r] = nd.m[r] * b[0] + nd.m[3 + r] * b[1] + nd.m[6 + r] * b[2] + nd.m[9 + r] * b[3];
            }
            stack.push_back(ch);
        }
    }
    return true;
}

uint32_t sf_slab_bytes(const sf_ctx* cc)
{
    if (!cc || !cc->has_view) return 0;
    const int d = hit_depth_bound(cc);
    if (d >= 0 && d <= SF_INDEX_SLAB_DEPTH) return 4u;   // (the cheap bound: the whole flake is far enough)
    // the search, cached per view (the root transform) and constant block: a camera path revisits its views
    sf_ctx* c = const_cast<sf_ctx*>(cc);   // (the cache only)
    for (const auto& e : c->slab_cache)
        if (e.gen == c->consts_gen && std::memcmp(e.root, c->root, sizeof e.root) == 0) return e.bytes;
    const uint32_t bytes = index_depth_proven(c) ? 4u : 16u;
    auto& e = c->slab_cache[c->slab_cache_next];
    c->slab_cache_next = (c->slab_cache_next + 1u) % (uint32_t)(sizeof c->slab_cache / sizeof c->slab_cache[0]);
    std::memcpy(e.root, c->root, sizeof e.root);
    e.gen = c->consts_gen;
    e.bytes = bytes;
    return bytes;
}

// The unpack of packed band slabs into the G-buffer on stream s. join: order after the context's previous call
// like every public call (sf_unpack_slabs); without it the caller orders the stream itself (sf_dist / sf_group
// run the unpack beside the context's own trace, on a stream of their own, and join it back with an event).
int sfi_unpack_slabs(sf_ctx* c, const void* stage, uint32_t bytes_per_pixel, uint32_t stage_rows, uint32_t band_rows,
                     uint32_t band_count, uint32_t first_member, uint32_t members, hipStream_t s, bool join)
{
    if (!c || !stage || band_rows == 0 || band_rows % 8 != 0 || band_count == 0 || first_member >= band_count ||
        members > band_count - first_member || (bytes_per_pixel != 4u && bytes_per_pixel != 16u))
        return SF_EINVAL;
    if (!c->has_view) return SF_ENOVIEW;
    if (members == 0) return SF_OK;
    // every member's slab must fit its stage_rows rows: a shorter stage would leave its last rows stale
    for (uint32_t k = first_member; k < first_member + members; ++k)
        if (sf_slab_rows(c->H, band_rows, band_count, k) > stage_rows) return SF_EINVAL;
    if (stage_rows == 0) return SF_OK;
    if (bytes_per_pixel == 4u && sf_slab_bytes(c) != 4u) return SF_EINVAL;   // (the view allows no index slab)
    DevGuard g(c->device);
    if (join) {
        if (int rc = ctx_join(c, s)) return rc;
    }
    // work enqueued whatever `join` says: the next sf_synchronize drains and checks (an unpack alone,
    // without the caller's sfi_join / sf_render beside it, must not meet the idle-sync return)
    c->stats_dirty = true;
    c->stats_unknown = true;
    FrameArgs a = frame_args(c);
    a.pos = c->pos;
    a.nrm = c->nrm;
    if (bytes_per_pixel == 4u) {
        if (!c->node_table)
            SF_HIP(c, hipMalloc(&c->node_table, (size_t)SF_NODE_TABLE_NODES * 3 * sizeof(float4)));
        float root12[12];
        for (int col = 0; col < 4; ++col)
            for (int r = 0; r < 3; ++r) root12[3 * col + r] = c->root[4 * col + r];
        if (c->table_gen != c->consts_gen || std::memcmp(root12, c->table_root, sizeof root12) != 0) {
            hipLaunchKernelGGL(sf_node_table, dim3((SF_NODE_TABLE_NODES + 255u) / 256u), dim3(256), 0, s, a,
                               c->node_table, SF_NODE_TABLE_NODES);
            SF_HIP(c, hipGetLastError());
            std::memcpy(c->table_root, root12, sizeof root12);
            c->table_gen = c->consts_gen;
        }
    }
    if (bytes_per_pixel == 4u) {
        // resident workgroups over the 256-pixel segments (each stages the per-lane constants in LDS once): 8 per CU,
        // or fewer when the slabs have fewer segments
        const uint64_t items = (uint64_t)members * stage_rows * ((c->W + 255u) / 256u);
        const uint64_t cap = 8ull * (uint64_t)c->cus;
        const dim3 grid((uint32_t)(items < cap ? items : cap));
        hipLaunchKernelGGL(sf_slab_unpack4, grid, dim3(256), 0, s, a, reinterpret_cast<const uint32_t*>(stage),
                           (const float4*)c->node_table, SF_NODE_TABLE_DEPTH, stage_rows, band_rows, band_count,
                           first_member, members);
        SF_HIP(c, hipGetLastError());
    }
    for (uint32_t r0 = 0; bytes_per_pixel == 16u && r0 < stage_rows; r0 += 65535u) {
        const uint32_t rows = stage_rows - r0 < 65535u ? stage_rows - r0 : 65535u;
        const dim3 grid((c->W + 255u) / 256u, rows, members);
        hipLaunchKernelGGL(sf_band_unpack, grid, dim3(256), 0, s, a, reinterpret_cast<const float4*>(stage),
                           stage_rows, band_rows, band_count, first_member, members, r0);
        SF_HIP(c, hipGetLastError());
    }
    if (join && s != c->stream) SF_HIP(c, hipEventRecord(c->join_ev, s));   // (StreamMark)
    return SF_OK;
}

// Order the context's own stream after everything the context enqueued before, on whatever stream (ctx_join).
// sf_dist / sf_group call it before they record a frame's start event on the context stream: their receive /
// unpack stream waits only for that event, so the event must already follow earlier consumers queued on a
// caller's stream (sf_download_async, sf_post_process on stream X), or the unpack could overwrite rows X is
// still reading.
int sfi_join(sf_ctx* c)
{
    if (!c) return SF_EINVAL;
    DevGuard g(c->device);
    return ctx_join(c, c->stream);
}

int sf_unpack_slabs(sf_ctx* c, const void* stage, uint32_t bytes_per_pixel, uint32_t stage_rows, uint32_t band_rows,
                    uint32_t band_count, uint32_t first_member, uint32_t members, void* stream)
{
    if (!c) return SF_EINVAL;
    return sfi_unpack_slabs(c, stage, bytes_per_pixel, stage_rows, band_rows, band_count, first_member, members,
                            stream ? (hipStream_t)stream : c->stream, true);
}

int sf_unpack_bands(sf_ctx* c, const float* stage4, uint32_t stage_rows, uint32_t band_rows, uint32_t band_count,
                    uint32_t first_member, uint32_t members, void* stream)
{
    return sf_unpack_slabs(c, stage4, 16u, stage_rows, band_rows, band_count, first_member, members, stream);
}

// n draws of the context's mt19937 stream into `out`, on stream s (advances c->mt_state): the single-workgroup
// generator for small counts, else the parallel jump-ahead path (same stream bit for bit).
static int gen_draws(sf_ctx* c, hipStream_t s, uint32_t* out, uint32_t n)
{
    if (!c->mt_parallel || n < kMtParMin) {
        hipLaunchKernelGGL(sf_mt_draws, dim3(1), dim3(256), 0, s, c->mt_state, out, n);
        SF_HIP(c, hipGetLastError());
        return SF_OK;
    }
    uint32_t K = n / kMtSegMin;
    K = K < 2u ? 2u : K > c->mt_seg_max ? c->mt_seg_max : K;
    const uint32_t L = (n + K - 1u) / K;
    const uint32_t pw = (uint32_t)sfhost::mt_poly_words();
    if (!c->mt_raw || !c->mt_partial || !c->mt_state2 || !c->mt_polys) {
        // all four scratch buffers or none: a partial set would let a later call launch on null buffers
        hipError_t e = hipSuccess;
        if (!c->mt_raw) e = hipMalloc(&c->mt_raw, (size_t)kMtRawBlocks * 624 * 4);
        if (e == hipSuccess && !c->mt_partial) e = hipMalloc(&c->mt_partial, (size_t)(kMtSegMax - 1) * kMtParts * 624 * 4);
        if (e == hipSuccess && !c->mt_state2) e = hipMalloc(&c->mt_state2, 625 * 4);
        if (e == hipSuccess && !c->mt_polys) e = hipMalloc(&c->mt_polys, (size_t)kMtSegMax * pw * 8);
        if (e != hipSuccess) {
            (void)hipFree(c->mt_raw);
            (void)hipFree(c->mt_partial);
            (void)hipFree(c->mt_state2);
            (void)hipFree(c->mt_polys);
            c->mt_raw = c->mt_partial = c->mt_state2 = nullptr;
            c->mt_polys = nullptr;
            c->mt_poly_key = 0;
            c->last_hip = (int)e;
            return e == hipErrorOutOfMemory ? SF_ENOMEM : SF_EHIP;
        }
    }
    const uint64_t key = ((uint64_t)L << 8) | K;
    if (c->mt_poly_key != key) {   // (host polynomials cached per (L, K); ~20 ms for a new batch size)
        SF_HIP(c, hipMemcpyAsync(c->mt_polys, sfhost::mt_jump_polys(L, K), (size_t)K * pw * 8, hipMemcpyHostToDevice, s));
        c->mt_poly_key = key;
    }
    hipLaunchKernelGGL(sf_mt_raw, dim3(1), dim3(256), 0, s, (const uint32_t*)c->mt_state, c->mt_raw, kMtRawBlocks);
    hipLaunchKernelGGL(sf_mt_jump_partial, dim3(K - 1u, kMtParts), dim3(256), 0, s, (const uint32_t*)c->mt_raw,
                       (const uint64_t*)c->mt_polys, pw, c->mt_partial);
    hipLaunchKernelGGL(sf_mt_segments, dim3(K), dim3(256), 0, s, (const uint32_t*)c->mt_state,
                       (const uint32_t*)c->mt_partial, L, n, out, c->mt_state2);
    SF_HIP(c, hipGetLastError());
    SF_HIP(c, hipMemcpyAsync(c->mt_state, c->mt_state2, 625 * 4, hipMemcpyDeviceToDevice, s));
    return SF_OK;
}

// Packet bins of a frame-less batch: squares of 2^shift pixels, about 8 packets per bin (a wave's worth of AVX
// packets), at most SF_PROG_MAX_BINS.
static void bin_geometry(const sf_ctx* c, uint32_t packets, uint32_t& shift, uint32_t& bx, uint32_t& by)
{
    for (shift = 2u;; ++shift) {
        bx = (c->W + (1u << shift) - 1u) >> shift;
        by = (c->H + (1u << shift) - 1u) >> shift;
        const uint64_t nb = (uint64_t)bx * by;
        if (nb <= SF_PROG_MAX_BINS && 8ull * nb <= packets) break;
        if (shift == 30u) break;
    }
}

// Binned trace order of `packets` packets (counting sort by bin, index order of the bins) into perm, on stream s.
static int bin_packets(sf_ctx* c, hipStream_t s, const FrameArgs& a, const uint32_t* draws, uint64_t counter0,
                       uint32_t packets, uint32_t pl, uint32_t* cnt, uint32_t* perm)
{
    uint32_t shift, bx, by;
    bin_geometry(c, packets, shift, bx, by);
    const uint32_t nbins = bx * by, pb = (packets + 255u) / 256u;
    SF_HIP(c, hipMemsetAsync(cnt, 0, (size_t)nbins * 4, s));
    hipLaunchKernelGGL(sf_packet_bin, dim3(pb), dim3(256), 0, s, a, draws, counter0, packets, pl, shift, bx, cnt);
    hipLaunchKernelGGL(sf_packet_scan, dim3(1), dim3(1024), 0, s, cnt, nbins, (const uint32_t*)nullptr);
    hipLaunchKernelGGL(sf_packet_place, dim3(pb), dim3(256), 0, s, a, draws, counter0, packets, pl, shift, bx, cnt, perm);
    SF_HIP(c, hipGetLastError());
    return SF_OK;
}

// Frame-less progressive mode (Sphereflake.cpp:67-74, 86-214). The device MT stream is kept in the
// context; a call that does not continue where the previous one stopped (other seed or counter)
// reseeds and jumps ahead by 2 * counter0 draws on the host (sfhost::mt_jump).
int sf_progressive(sf_ctx* c, uint32_t seed, uint64_t counter0, uint32_t packets, void* stream)
{
    if (!c) return SF_EINVAL;
    if (!c->has_view) return SF_ENOVIEW;
    const bool sse = c->variant == SF_VARIANT_SSE;
    const uint32_t pl = sse ? 4u : 8u;             // packet lanes (SIMD_SSE.h / SIMD_AVX.h)
    // the AVX worker samples x0 in [1, W-2], the SSE worker x0 in [0, W-2] (Sphereflake.cpp:117-118, 140-141)
    if (sse ? (c->W < 2 || c->H < 2) : (c->W < 3 || c->H < 3)) return SF_EINVAL;
    if (packets == 0) return SF_OK;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    DevGuard g(c->device);
    if (int rc = ctx_join(c, s)) return rc;
    StreamMark mark_(c, s);
    if (!c->mt_state) {
        SF_HIP(c, hipMalloc(&c->mt_state, 625 * 4));
        SF_HIP(c, hipMalloc(&c->owner, (size_t)c->W * c->H * 8));
        SF_HIP(c, hipMemsetAsync(c->owner, 0, (size_t)c->W * c->H * 8, s));
    }
    // a pending prefetch either is this batch's draws, or is undone (MT state restored)
    bool prefetched = false, prebinned = false;
    const bool binned = c->prog_bin && packets >= SF_PROG_BIN_MIN;
    if (c->pf_packets) {
        SF_HIP(c, hipStreamWaitEvent(s, c->pf_done, 0));
        if (c->pf_packets == packets && c->prog_seeded && seed == c->prog_seed && counter0 == c->prog_next) {
            std::swap(c->draws, c->draws_pf);
            prefetched = true;
            if (binned && !c->prog_order && c->pf_bin_pl == pl) {
                std::swap(c->perm, c->perm_pf);
                prebinned = true;
            }
        } else {
            SF_HIP(c, hipMemcpyAsync(c->mt_state, c->mt_saved, 625 * 4, hipMemcpyDeviceToDevice, s));
        }
        c->pf_packets = 0;
    }
    if (packets > c->prog_cap) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(c->draws);
        (void)hipFree(c->draws_pf);
        (void)hipFree(c->lanes);
        (void)hipFree(c->perm);
        (void)hipFree(c->perm_pf);
        c->perm_pf = nullptr;
        (void)hipFree(c->prog_ovf);
        c->draws = c->draws_pf = nullptr;
        c->lanes = nullptr;
        c->perm = nullptr;
        c->prog_ovf = nullptr;
        c->prog_cap = 0;
        c->traced_valid = false;
        SF_HIP(c, hipMalloc(&c->draws, (size_t)packets * 2 * 4));
        SF_HIP(c, hipMalloc(&c->lanes, (size_t)packets * 8 * sizeof(PacketLane)));
        SF_HIP(c, hipMalloc(&c->perm, (size_t)packets * 4));
        SF_HIP(c, hipMalloc(&c->prog_ovf, ((size_t)packets + 3) / 4 * 4));   // >= one entry per wave
        c->prog_cap = packets;
    }
    if (!c->prog_seeded || seed != c->prog_seed || counter0 != c->prog_next) {
        uint32_t st[625], sj[625];
        sfhost::mt19937_seed(seed, st);
        sfhost::mt_jump(st, 2 * counter0, sj);   // the stream 2 * counter0 draws on (2 per packet)
        SF_HIP(c, hipMemcpyAsync(c->mt_state, sj, sizeof sj, hipMemcpyHostToDevice, s));
        SF_HIP(c, hipStreamSynchronize(s));
        c->prog_seeded = true;
        c->prog_seed = seed;
    }
    FrameArgs a = frame_args(c);
    a.pos = c->pos;
    a.nrm = c->nrm;
    a.min_t = c->min_t;
    a.emit_aux = 1;
    a.packet_lanes = pl;
    if (c->flags & SF_FLAG_DIAG_UNITS) a.tile_trace = c->tile_trace;   // per-wave diagnostics (sf_set_tile_trace)
    if (!prefetched)
        if (int rc = gen_draws(c, s, c->draws, 2 * packets)) return rc;
    // Prefetch the next batch's draws (a continuing stream of the same batch size) on pf_stream, into
    // the buffer the previous batch traced from, overlapped with this batch's trace.
    if (c->prog_prefetch && packets >= SF_PROG_PREFETCH_MIN) {
        if (!c->pf_stream) {
            if (c->pf_prio) {   // (a stream of the device's greatest priority: a hardware queue of its own)
                int least = 0, greatest = 0;
                SF_HIP(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
                SF_HIP(c, hipStreamCreateWithPriority(&c->pf_stream, hipStreamNonBlocking, greatest));
            } else {
                SF_HIP(c, hipStreamCreateWithFlags(&c->pf_stream, hipStreamNonBlocking));
            }
            SF_HIP(c, hipEventCreateWithFlags(&c->pf_done, hipEventDisableTiming));
            SF_HIP(c, hipEventCreateWithFlags(&c->mt_ready, hipEventDisableTiming));
            SF_HIP(c, hipEventCreateWithFlags(&c->traced, hipEventDisableTiming));
            SF_HIP(c, hipMalloc(&c->mt_saved, 625 * 4));
        }
        if (!c->draws_pf) SF_HIP(c, hipMalloc(&c->draws_pf, (size_t)c->prog_cap * 2 * 4));
        SF_HIP(c, hipEventRecord(c->mt_ready, s));                 // MT state advanced past this batch
        SF_HIP(c, hipStreamWaitEvent(c->pf_stream, c->mt_ready, 0));
        if (c->traced_valid) SF_HIP(c, hipStreamWaitEvent(c->pf_stream, c->traced, 0));   // draws_pf free
        SF_HIP(c, hipMemcpyAsync(c->mt_saved, c->mt_state, 625 * 4, hipMemcpyDeviceToDevice, c->pf_stream));
        if (int rc = gen_draws(c, c->pf_stream, c->draws_pf, 2 * packets)) return rc;
        // the next batch's binned order too (index-ordered bins only: a cost-ranked order needs this batch's costs)
        c->pf_bin_pl = 0;
        if (binned && !c->prog_order) {
            if (!c->perm_pf) SF_HIP(c, hipMalloc(&c->perm_pf, (size_t)c->prog_cap * 4));
            if (!c->bin_cnt_pf) SF_HIP(c, hipMalloc(&c->bin_cnt_pf, SF_PROG_MAX_BINS * 4));
            if (int rc = bin_packets(c, c->pf_stream, a, c->draws_pf, counter0 + packets, packets, pl, c->bin_cnt_pf,
                                     c->perm_pf))
                return rc;
            c->pf_bin_pl = pl;
        }
        SF_HIP(c, hipEventRecord(c->pf_done, c->pf_stream));
        c->pf_packets = packets;
    }
    // Trace order: packets binned by a square of 2^shift pixels (about 8 per bin, a wave's worth of
    // AVX packets), so a wave's packets share their traversal. Small batches: draw order.
    const uint32_t* perm = nullptr;
    if (prebinned) {   // (binned on pf_stream with the draws)
        perm = c->perm;
    } else if (binned) {
        if (!c->bin_cnt) SF_HIP(c, hipMalloc(&c->bin_cnt, SF_PROG_MAX_BINS * 4));
        uint32_t shift, bx, by;
        bin_geometry(c, packets, shift, bx, by);
        const uint32_t nbins = bx * by;
        const uint32_t pb = (packets + 255u) / 256u;
        // Heavy-first: bins ranked by the cycles their waves took in the previous batch of the same
        // binning (the view and the bins do not move between batches); the trace grid then starts with
        // the heaviest packets instead of meeting them wherever their screen region falls.
        const uint32_t* rank = nullptr;
        if (c->prog_order) {
            const uint32_t nc = (nbins + 63u) / 64u;
            const uint32_t key = (shift << 24) | nbins;
            if (!c->bin_cost) {
                const size_t nc_max = (SF_PROG_MAX_BINS + 63u) / 64u;
                SF_HIP(c, hipMalloc(&c->bin_cost, SF_PROG_MAX_BINS * 4));
                SF_HIP(c, hipMalloc(&c->bin_rank, SF_PROG_MAX_BINS * 4));
                SF_HIP(c, hipMalloc(&c->bin_order, SF_PROG_MAX_BINS * 4));
                SF_HIP(c, hipMalloc(&c->bin_chunk_cnt, nc_max * SF_ORDER_BUCKETS * 4));
                SF_HIP(c, hipMalloc(&c->bin_chunk_off, nc_max * SF_ORDER_BUCKETS * 4));
                SF_HIP(c, hipMalloc(&c->bin_meta, 4 * 4));
            }
            if (c->bin_key == key) {
                hipLaunchKernelGGL(sf_bin_hist, dim3(nc), dim3(64), 0, s, (const uint32_t*)c->bin_cost, nbins,
                                   c->bin_chunk_cnt);
                hipLaunchKernelGGL(sf_order_scan, dim3(1), dim3(1024), 0, s, c->bin_chunk_cnt, nc, nbins,
                                   0u, 2u, 0u, 0u, 0u, c->bin_chunk_off, c->bin_meta, (const uint32_t*)nullptr,
                                   (uint32_t*)nullptr, 0xffffffffu);
                hipLaunchKernelGGL(sf_order_scatter, dim3(nc), dim3(64), 0, s, (const uint32_t*)c->bin_cost, nbins,
                                   c->bin_chunk_cnt, (const uint32_t*)c->bin_chunk_off, (const uint32_t*)c->bin_meta,
                                   c->bin_order, c->bin_rank);
                SF_HIP(c, hipGetLastError());
                rank = c->bin_rank;
            } else {   // new binning: no costs yet (this batch records them)
                SF_HIP(c, hipMemsetAsync(c->bin_cost, 0, SF_PROG_MAX_BINS * 4, s));
                c->bin_key = key;
            }
            a.bin_cost = c->bin_cost;
            a.bin_shift = shift;
            a.bins_x = bx;
        }
        SF_HIP(c, hipMemsetAsync(c->bin_cnt, 0, (size_t)nbins * 4, s));
        hipLaunchKernelGGL(sf_packet_bin, dim3(pb), dim3(256), 0, s, a, (const uint32_t*)c->draws, counter0, packets,
                           pl, shift, bx, c->bin_cnt);
        hipLaunchKernelGGL(sf_packet_scan, dim3(1), dim3(1024), 0, s, c->bin_cnt, nbins, rank);
        hipLaunchKernelGGL(sf_packet_place, dim3(pb), dim3(256), 0, s, a, (const uint32_t*)c->draws, counter0, packets,
                           pl, shift, bx, c->bin_cnt, c->perm);
        SF_HIP(c, hipGetLastError());
        perm = c->perm;
    }
    const uint32_t ppw = 64u / pl;                   // packets per wave
    const uint32_t waves = (packets + ppw - 1) / ppw;
    uint32_t levels = SF_PROGRESSIVE_LEVELS;
    if (c->prog_adapt) {
        if (!c->h_prog_depth) {
            SF_HIP(c, hipHostMalloc(&c->h_prog_depth, 4, hipHostMallocDefault));
            *c->h_prog_depth = -1;
            SF_HIP(c, hipMalloc(&c->prog_ovf_cnt, 2 * 4));
            SF_HIP(c, hipMemsetAsync(c->prog_ovf_cnt, 0, 2 * 4, s));
        }
        const int32_t seen = *(volatile int32_t*)c->h_prog_depth;   // max depth of a finished batch
        if (seen >= 0 && (uint32_t)seen + 1u < levels) levels = (uint32_t)seen + 1u < 4u ? 4u : (uint32_t)seen + 1u;
    }
    const bool adaptive = levels < SF_PROGRESSIVE_LEVELS;
    uint32_t* ovf_cnt = adaptive ? c->prog_ovf_cnt + c->prog_par : nullptr;
    const size_t lds = (size_t)SF_LDS_WAVE_FLOATS(levels) * 4;
    if (sse)
        hipLaunchKernelGGL(sf_progressive_trace_sse, dim3(waves), dim3(64), lds, s, a, (const uint32_t*)c->draws,
                           counter0, packets, c->ticket, c->lanes, c->owner, perm, levels,
                           adaptive ? c->prog_ovf : nullptr, ovf_cnt);
    else
        hipLaunchKernelGGL(sf_progressive_trace, dim3(waves), dim3(64), lds, s, a, (const uint32_t*)c->draws,
                           counter0, packets, c->ticket, c->lanes, c->owner, perm, levels,
                           adaptive ? c->prog_ovf : nullptr, ovf_cnt);
    SF_HIP(c, hipGetLastError());
    if (adaptive) {   // re-trace the waves that needed more levels (reads this batch's list, zeroes the next)
        const size_t lds_fix = (size_t)SF_LDS_WAVE_FLOATS(SF_PROGRESSIVE_LEVELS) * 4;
        const dim3 fg(SF_PROG_FIXUP_BLOCKS);
        if (sse)
            hipLaunchKernelGGL(sf_progressive_fixup_sse, fg, dim3(64), lds_fix, s, a, (const uint32_t*)c->draws,
                               counter0, packets, c->ticket, c->lanes, c->owner, perm, (const uint32_t*)c->prog_ovf,
                               c->prog_ovf_cnt, c->prog_par);
        else
            hipLaunchKernelGGL(sf_progressive_fixup, fg, dim3(64), lds_fix, s, a, (const uint32_t*)c->draws,
                               counter0, packets, c->ticket, c->lanes, c->owner, perm, (const uint32_t*)c->prog_ovf,
                               c->prog_ovf_cnt, c->prog_par);
        SF_HIP(c, hipGetLastError());
        c->prog_par ^= 1u;
    }
    if (c->pf_stream) {   // the next prefetch may overwrite this batch's draws after this point
        SF_HIP(c, hipEventRecord(c->traced, s));
        c->traced_valid = true;
    }
    hipLaunchKernelGGL(sf_progressive_scatter, dim3((packets * pl + 255) / 256), dim3(256), 0, s, a, packets, c->ticket,
                       (const PacketLane*)c->lanes, (const unsigned long long*)c->owner);
    SF_HIP(c, hipGetLastError());
    if (c->prog_adapt) SF_HIP(c, hipMemcpyAsync(c->h_prog_depth, c->stats, 4, hipMemcpyDeviceToHost, s));
    c->ticket += packets;
    c->prog_next = counter0 + packets;
    c->rays += (int64_t)pl * packets;                // m_RaysPerSecond += 8 / 4 (Sphereflake.cpp:184-186)
    return SF_OK;
}

// The stats words ride the stream in a small copy to pinned memory, queued behind the context's work, so the host
// waits once (a synchronous hipMemcpy after the drain was a second round trip, ~10-20 us per call: per slot of a
// dist, at the end of every timed loop and every lone frame); a context with nothing enqueued since the last call
// only drains, and so does one whose work since then was only persistent traces that cannot add to the unresolved
// word (round 5: the copy was a blit dispatch of ~4 us behind every lone frame's trace, plus its launch gap).
int sf_synchronize(sf_ctx* c)
{
    if (!c) return SF_EINVAL;
    // nothing enqueued since the last check (every call that enqueues work joins first, ctx_join): no runtime
    // call at all -- a multi-slot caller (sf_dist_synchronize) waits only for the slots that have work
    if (!c->stats_dirty) return c->unresolved != 0 ? SF_EDEPTH : SF_OK;
    DevGuard g(c->device);
    // (after only traces that cannot change the unresolved word, the last check's value stands: no copy)
    const bool check = c->stats_dirty && c->stats_unknown;
    if (check) {
        if (int rc_ = ctx_join(c, c->stream)) return rc_;
        SF_HIP(c, hipMemcpyAsync(c->h_stats, c->stats, 12, hipMemcpyDeviceToHost, c->stream));
    }
    if (int rc_ = ctx_drain(c)) return rc_;
    c->stats_dirty = false;
    c->stats_unknown = false;
    if (check) c->unresolved = ((volatile int32_t*)c->h_stats)[2];
    if (c->unresolved != 0) return SF_EDEPTH;
    return SF_OK;
}

int sf_download(sf_ctx* c, float* pos4, float* nrm4, float* min_t, uint32_t* hidx)
{
    if (!c) return SF_EINVAL;
    int rc = sf_synchronize(c);
    if (rc != SF_OK) return rc;
    DevGuard g(c->device);
    const size_t npx = (size_t)c->W * c->H;
    if (pos4) SF_HIP(c, hipMemcpy(pos4, c->pos, npx * 16, hipMemcpyDeviceToHost));
    if (nrm4) SF_HIP(c, hipMemcpy(nrm4, c->nrm, npx * 16, hipMemcpyDeviceToHost));
    if (min_t) SF_HIP(c, hipMemcpy(min_t, c->min_t, npx * 4, hipMemcpyDeviceToHost));
    if (hidx) SF_HIP(c, hipMemcpy(hidx, c->hit_index, npx * 4, hipMemcpyDeviceToHost));
    return SF_OK;
}

// Transfer/interop: stream-ordered D2H into host memory. With page-locked
// destinations (sf_host_register) the copy runs at PCIe DMA rate and overlaps
// whatever the host does until sf_synchronize (context stream) or the caller syncs `stream`.
int sf_download_async(sf_ctx* c, float* pos4, float* nrm4, float* min_t, uint32_t* hidx, void* stream)
{
    if (!c) return SF_EINVAL;
    DevGuard g(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const size_t npx = (size_t)c->W * c->H;
    if (int rc = ctx_join(c, s)) return rc;
    StreamMark mark_(c, s);
    if (pos4) SF_HIP(c, hipMemcpyAsync(pos4, c->pos, npx * 16, hipMemcpyDeviceToHost, s));
    if (nrm4) SF_HIP(c, hipMemcpyAsync(nrm4, c->nrm, npx * 16, hipMemcpyDeviceToHost, s));
    if (min_t) SF_HIP(c, hipMemcpyAsync(min_t, c->min_t, npx * 4, hipMemcpyDeviceToHost, s));
    if (hidx) SF_HIP(c, hipMemcpyAsync(hidx, c->hit_index, npx * 4, hipMemcpyDeviceToHost, s));
    return SF_OK;
}

int sf_host_register(void* ptr, size_t bytes)
{
    if (!ptr || !bytes) return SF_EINVAL;
    return hipHostRegister(ptr, bytes, hipHostRegisterDefault) == hipSuccess ? SF_OK : SF_EHIP;
}

int sf_host_unregister(void* ptr)
{
    if (!ptr) return SF_EINVAL;
    return hipHostUnregister(ptr) == hipSuccess ? SF_OK : SF_EHIP;
}

int sf_post_defaults(const sf_ctx* c, sf_post_params* p)
{
    if (!c || !p) return SF_EINVAL;
    std::memset(p, 0, sizeof *p);
    p->sample_radius = -1.0f;
    p->intensity = 0.51f;
    p->scale = 3.28f;
    p->bias = 0.23f;
    p->normal_threshold = 2.47f;
    p->depth_threshold = 0.01f;
    std::memcpy(p->camera_position, c->o, 12);
    p->downscale = 1;
    return SF_OK;
}

int sf_ssao_noise(float* out)
{
    if (!out) return SF_EINVAL;
    sfhost::ssao_noise(out);
    return SF_OK;
}

int sf_post_process(sf_ctx* c, const sf_post_params* prm, const float* pos4, const float* nrm4, uint8_t* rgba,
                    uint8_t* ao)
{
    if (!c || !prm || prm->downscale == 0) return SF_EINVAL;
    const uint32_t aw = c->W / prm->downscale, ah = c->H / prm->downscale;
    if (aw == 0 || ah == 0) return SF_EINVAL;
    DevGuard g(c->device);
    hipStream_t s = prm->stream ? (hipStream_t)prm->stream : c->stream;
    const size_t npx = (size_t)c->W * c->H;
    if (int rc = ctx_join(c, s)) return rc;
    StreamMark mark_(c, s);
    if (!c->noise) {
        static float host_noise[SF_NOISE_SIZE * SF_NOISE_SIZE * 4];
        sfhost::ssao_noise(host_noise);
        SF_HIP(c, hipMalloc(&c->noise, sizeof host_noise));
        SF_HIP(c, hipMemcpy(c->noise, host_noise, sizeof host_noise, hipMemcpyHostToDevice));
    }
    if (!c->image) SF_HIP(c, hipMalloc(&c->image, npx * 4));
    if (c->centre_exact < 0) c->centre_exact = sfhost::post_centre_exact(c->W) && sfhost::post_centre_exact(c->H);
    // Fusion is exact when no blur tap can be accepted: every |n| <= 1.004 (the tracer's normals are
    // rsqrtps-normalised, |n| - 1 < 2^-11) bounds dot(n, n') < 1.01 <= normalThreshold
    const bool own_gbuffer = (!pos4 || pos4 == c->pos) && (!nrm4 || nrm4 == c->nrm);
    const bool fused = !(prm->flags & SF_POST_GENERAL) && prm->downscale == 1 && c->centre_exact &&
                       prm->normal_threshold >= 1.01f && (own_gbuffer || (prm->flags & SF_POST_UNIT_NORMALS));
    if (!fused) {
        if (c->post_ao_px < (size_t)aw * ah) {
            SF_HIP(c, hipFree(c->ao));
            c->ao = nullptr;
            SF_HIP(c, hipMalloc(&c->ao, (size_t)aw * ah));
            c->post_ao_px = (size_t)aw * ah;
        }
        if (!c->blur_h) SF_HIP(c, hipMalloc(&c->blur_h, npx));
        if (!c->blur_v) SF_HIP(c, hipMalloc(&c->blur_v, npx));
    }
    PostArgs a;
    std::memset(&a, 0, sizeof a);
    a.W = c->W;
    a.H = c->H;
    a.aw = aw;
    a.ah = ah;
    a.fw = (float)c->W;
    a.fh = (float)c->H;
    a.faw = (float)aw;
    a.fah = (float)ah;
    // uniform reciprocals, correctly rounded here once instead of per fragment (the same IEEE division)
    a.rfw = 1.0f / a.fw;
    a.rfh = 1.0f / a.fh;
    a.rfaw = 1.0f / a.faw;
    a.rfah = 1.0f / a.fah;
    a.pos = pos4 ? pos4 : c->pos;
    a.nrm = nrm4 ? nrm4 : c->nrm;
    a.noise = c->noise;
    a.stats = c->stats;
    a.radius = prm->sample_radius;
    a.intensity = prm->intensity;
    a.scale = prm->scale;
    a.bias = prm->bias;
    a.normal_thr = prm->normal_threshold;
    a.depth_thr = prm->depth_threshold;
    std::memcpy(a.cam, prm->camera_position, 12);
    a.rgba = rgba ? rgba : c->image;
    const dim3 blk(256);
    const dim3 grid((c->W + 15) / 16, (c->H + 15) / 16);
    if (fused) {
        a.ao = ao;
        hipLaunchKernelGGL(sf_post_fused, grid, blk, 0, s, a);
    } else {
        a.ao = ao ? ao : c->ao;
        a.blur_h = c->blur_h;
        a.blur_v = c->blur_v;
        hipLaunchKernelGGL(sf_post_ssao, dim3((aw + 15) / 16, (ah + 15) / 16), blk, 0, s, a);
        hipLaunchKernelGGL(sf_post_blur, grid, blk, 0, s, a, 0u);
        hipLaunchKernelGGL(sf_post_blur, grid, blk, 0, s, a, 1u);
        hipLaunchKernelGGL(sf_post_final, grid, blk, 0, s, a);
    }
    SF_HIP(c, hipGetLastError());
    return SF_OK;
}

int sf_download_image(sf_ctx* c, uint8_t* rgba)
{
    if (!c || !rgba) return SF_EINVAL;
    if (!c->image) return SF_ESTATE;
    int rc = sf_synchronize(c);
    if (rc != SF_OK) return rc;
    DevGuard g(c->device);
    SF_HIP(c, hipMemcpy(rgba, c->image, (size_t)c->W * c->H * 4, hipMemcpyDeviceToHost));
    return SF_OK;
}

int sf_set_variant(sf_ctx* c, int variant)
{
    if (!c || (variant != SF_VARIANT_AVX && variant != SF_VARIANT_SSE)) return SF_EINVAL;
    if (variant == c->variant) return SF_OK;
    DevGuard g(c->device);
    if (int rc_ = ctx_drain(c)) return rc_;
    c->variant = variant;
    c->order_n = 0;       // tile costs of the other variant's frames: start over
    *c->h_depth = -1;     // level hint likewise
    return upload_consts(c);
}

int sf_get_variant(const sf_ctx* c) { return c ? c->variant : SF_EINVAL; }

int sf_set_tile_trace(sf_ctx* c, int enable)
{
    if (!c) return SF_EINVAL;
    DevGuard g(c->device);
    if (int rc_ = ctx_drain(c)) return rc_;
    if (!enable) {
        (void)hipFree(c->tile_trace);
        c->tile_trace = nullptr;
        return SF_OK;
    }
    if (!c->tile_trace) {
        const size_t ntiles = (size_t)((c->W + 7) / 8) * ((c->H + 7) / 8);
        // per tile {start, end, id}, the diagnostic slots, per work unit {start, end, unit} (<= 4 per tile),
        // per wave {start, end}
        SF_HIP(c, hipMalloc(&c->tile_trace, SF_TRACE_WORDS(ntiles) * 8));
        SF_HIP(c, hipMemset(c->tile_trace, 0, SF_TRACE_WORDS(ntiles) * 8));
    }
    return SF_OK;
}

int sf_get_tile_trace(sf_ctx* c, uint64_t* out, size_t n)
{
    if (!c || !out || !c->tile_trace) return SF_EINVAL;
    DevGuard g(c->device);
    const size_t ntiles = (size_t)((c->W + 7) / 8) * ((c->H + 7) / 8);
    if (n < ntiles * 3) return SF_EINVAL;
    if (int rc_ = ctx_drain(c)) return rc_;
    // n >= 3 * tiles + SF_DIAG_SLOTS also returns the segment sums / event counts of the diagnostic
    // builds (zeros otherwise); n >= SF_TRACE_WORDS(tiles) the per-unit and per-wave records too
    const size_t full = SF_TRACE_WORDS(ntiles);
    SF_HIP(c, hipMemcpy(out, c->tile_trace, (n >= full ? full : n >= ntiles * 3 + SF_DIAG_SLOTS ? ntiles * 3 + SF_DIAG_SLOTS : ntiles * 3) * 8,
                        hipMemcpyDeviceToHost));
    return SF_OK;
}

int sf_get_tile_order(sf_ctx* c, uint32_t* order, uint32_t* cost, size_t n)
{
    if (!c) return SF_EINVAL;
    DevGuard g(c->device);
    const size_t ntiles = (size_t)((c->W + 7) / 8) * ((c->H + 7) / 8);
    if (n < ntiles || (!order && !cost)) return SF_EINVAL;
    if (int rc_ = ctx_drain(c)) return rc_;
    if (c->order_n == 0u) return 0;   // (a band share's order covers its own c->order_n tiles)
    uint32_t meta[2];
    SF_HIP(c, hipMemcpy(meta, c->order_meta, sizeof(meta), hipMemcpyDeviceToHost));
    if (order && n < meta[0]) return SF_EINVAL;
    if (order) SF_HIP(c, hipMemcpy(order, c->tile_order, (size_t)meta[0] * 4, hipMemcpyDeviceToHost));
    if (cost) SF_HIP(c, hipMemcpy(cost, c->tile_cost, (size_t)c->order_n * 4, hipMemcpyDeviceToHost));
    return (int)meta[0];
}

void* sf_context_stream(sf_ctx* c) { return c ? (void*)c->stream : nullptr; }

int sf_device_buffers(sf_ctx* c, float** pos4, float** nrm4, float** min_t, uint32_t** hidx)
{
    if (!c) return SF_EINVAL;
    if (pos4) *pos4 = c->pos;
    if (nrm4) *nrm4 = c->nrm;
    if (min_t) *min_t = c->min_t;
    if (hidx) *hidx = c->hit_index;
    return SF_OK;
}

int sf_set_kernel_timing(sf_ctx* c, int enable)
{
    if (!c) return SF_EINVAL;
    DevGuard g(c->device);
    if (enable && !c->ev[0][0]) {
        for (int i = 0; i < sf_ctx::kTimed; ++i)
            for (int j = 0; j < 2; ++j) SF_HIP(c, hipEventCreate(&c->ev[i][j]));
        const size_t cb = (size_t)sf_ctx::kTimed * SF_CLOCK_WAVES * 4u * 8u;
        SF_HIP(c, hipMalloc(&c->clock_buf, cb));
        SF_HIP(c, hipMemset(c->clock_buf, 0, cb));
    }
    if (enable < 0) return SF_EINVAL;
    c->timing = enable != 0;
    c->ev_period = enable > 0 ? (uint32_t)enable : 1u;
    c->ev_next = c->ev_count = c->ev_phase = 0;
    return SF_OK;
}

int sf_kernel_times(sf_ctx* c, float* ms, uint32_t n)
{
    if (!c || !ms) return SF_EINVAL;
    DevGuard g(c->device);
    if (int rc_ = ctx_drain(c)) return rc_;
    const uint32_t k = n < c->ev_count ? n : c->ev_count;
    for (uint32_t i = 0; i < k; ++i) {   // the k most recent, oldest first
        const uint32_t slot = (c->ev_next + sf_ctx::kTimed - k + i) % sf_ctx::kTimed;
        SF_HIP(c, hipEventSynchronize(c->ev[slot][1]));
        SF_HIP(c, hipEventElapsedTime(&ms[i], c->ev[slot][0], c->ev[slot][1]));
    }
    return (int)k;
}

int sf_kernel_clocks(sf_ctx* c, float* mhz, uint32_t n)
{
    if (!c || !mhz) return SF_EINVAL;
    DevGuard g(c->device);
    if (int rc_ = ctx_drain(c)) return rc_;
    const uint32_t k = n < c->ev_count ? n : c->ev_count;
    if (k == 0 || !c->clock_buf) return 0;
    static_assert(SF_CLOCK_WAVES == 8u, "median below assumes 8 records");
    uint64_t rec[SF_CLOCK_WAVES * 4];
    for (uint32_t i = 0; i < k; ++i) {   // the k most recent timed renders, oldest first (as sf_kernel_times)
        const uint32_t slot = (c->ev_next + sf_ctx::kTimed - k + i) % sf_ctx::kTimed;
        SF_HIP(c, hipMemcpy(rec, c->clock_buf + (size_t)slot * SF_CLOCK_WAVES * 4u, sizeof rec, hipMemcpyDeviceToHost));
        float v[SF_CLOCK_WAVES];
        uint32_t m = 0;
        for (uint32_t w = 0; w < SF_CLOCK_WAVES; ++w) {
            const uint64_t* r = rec + 4u * w;
            if (r[3] > r[1] && r[2] > r[0]) v[m++] = (float)((double)(r[2] - r[0]) / (double)(r[3] - r[1]) * 100.0);
        }
        for (uint32_t a = 1; a < m; ++a)   // (insertion sort of <= 8 values)
            for (uint32_t b = a; b > 0 && v[b - 1] > v[b]; --b) std::swap(v[b - 1], v[b]);
        mhz[i] = m ? (m & 1u ? v[m / 2] : 0.5f * (v[m / 2 - 1] + v[m / 2])) : 0.0f;
    }
    return (int)k;
}

int sf_get_stats(sf_ctx* c, sf_stats* out)
{
    if (!c || !out) return SF_EINVAL;
    DevGuard g(c->device);
    if (int rc_ = ctx_drain(c)) return rc_;
    int32_t st[3];
    SF_HIP(c, hipMemcpy(st, c->stats, 12, hipMemcpyDeviceToHost));
    out->max_depth = st[0] < 0 ? 0 : st[0];
    out->closest = sf_key_float(st[1]);
    out->rays = c->rays;
    out->overflow_tiles = st[2];
    return SF_OK;
}

int sf_reset_max_depth(sf_ctx* c)
{
    if (!c) return SF_EINVAL;
    DevGuard g(c->device);
    return reset_stats_dev(c, 1);
}

int sf_reset_rays(sf_ctx* c)
{
    if (!c) return SF_EINVAL;
    c->rays = 0;
    return SF_OK;
}

int sf_reset_closest(sf_ctx* c)
{
    if (!c) return SF_EINVAL;
    DevGuard g(c->device);
    return reset_stats_dev(c, 2);
}

int sf_camera_corners(uint32_t W, uint32_t H, const float pos[3], float pitch, float yaw, float roll, float fov,
                      float o[3], float tl[3], float tr[3], float bl[3])
{
    if (!W || !H || !pos || !o || !tl || !tr || !bl) return SF_EINVAL;
    sfhost::camera_corners(W, H, pos, pitch, yaw, roll, fov, o, tl, tr, bl);
    return SF_OK;
}

int sf_child_transforms(float child[9][16])
{
    if (!child) return SF_EINVAL;
    sfhost::child_transforms(child);
    return SF_OK;
}

int sf_root_transform(const float origin[3], float root[16])
{
    if (!origin || !root) return SF_EINVAL;
    sfhost::root_transform(origin, root);
    return SF_OK;
}

int sf_lod_threshold(float r, float lod_constant, float* T)
{
    if (!T || !(r > 0.0f) || !(lod_constant > 0.0f)) return SF_EINVAL;
    *T = sfhost::lod_threshold(r, lod_constant);
    return SF_OK;
}

int sf_division_by_reciprocal_exact(uint32_t n)
{
    return sfhost::division_by_reciprocal_exact(n) ? 1 : 0;
}

int sf_depth_constants(uint32_t depth, float* radius, float* lod)
{
    if (depth >= SF_DEPTH_TABLE) return SF_EINVAL;
    float r = sfhost::radius(depth);
    if (radius) *radius = r;
    if (lod) *lod = sfhost::lod_threshold(r);
    return SF_OK;
}

int sf_mt19937_jump(const uint32_t state_in[625], uint64_t outputs, uint32_t state_out[625])
{
    if (!state_in || !state_out) return SF_EINVAL;
    sfhost::mt_jump(state_in, outputs, state_out);
    return SF_OK;
}

float sf_rsqrtps(float x)
{
    uint32_t b;
    std::memcpy(&b, &x, 4);
    uint32_t E = (b >> 23) & 0xffu;
    uint32_t r;
    if ((b & 0x7fffffffu) > 0x7f800000u) r = b | 0x00400000u;
    else if (E == 0u) r = (b & 0x80000000u) | 0x7f800000u;
    else if (b & 0x80000000u) r = 0xffc00000u;
    else if (E == 0xffu) r = 0u;
    else {
        uint32_t key = ((E & 1u) << 10) | ((b & 0x7fffffu) >> 13);
        int32_t E0 = (E & 1u) ? 127 : 128;
        int32_t k = ((int32_t)E - E0) / 2;
        r = (uint32_t)((int32_t)kLut[key] - k * (1 << 23));
    }
    float f;
    std::memcpy(&f, &r, 4);
    return f;
}

}  // extern "C"
