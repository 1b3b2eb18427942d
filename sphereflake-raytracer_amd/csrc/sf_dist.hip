// sf_dist.hip -- one process per GPU: a frame's rows split over the ranks, gathered to rank 0 with RCCL
// over xGMI (north star: "row-tiles across 8 x MI355X with RCCL gather").
//
// The reference's only parallelism is its host thread pool (Sphereflake.cpp:67-74). Here every rank owns a
// context on its own GPU and traces the interleaved 8-row bands b = rank (mod nranks) of each frame: flake rows
// cost ~150 nodes per ray and sky rows ~1, so interleaving balances the ranks without any cost exchange.
//   rank 0   traces its bands straight into its context's G-buffer at frame positions, then receives every
//            other rank's slab and unpacks it into the same G-buffer (sf_unpack_bands);
//   rank k   traces its bands as a PACKED compact slab and sends it: one uint32 hit index per pixel (4 B, an
//            eighth of the G-buffer's 32 B) where the view proves every hit's heap index below 2^32
//            (sf_slab_bytes), else one float4 (nx, ny, nz, minT) -- rank 0 rebuilds the rest bit for bit.
// The gather is a gather to one rank, each peer's slab over its own xGMI link (no ring collective): ncclSend on
// the peer's slot stream right behind its trace; on rank 0 one grouped ncclRecv and the unpack on a receive stream
// of the slot, started at the frame's start, so the peers' slabs land and unpack while rank 0 traces its own bands;
// the slot's context stream then waits for the unpack (the frame complete in rank 0's G-buffer).
//
// Frames in flight: `slots` independent pipelines (context + stream + communicator + slab), frame i on slot
// i % slots. A frame's persistent trace grid then fills the wave slots the previous frame's heaviest tiles
// leave idle, and its trace overlaps the previous frame's gather. Every slot has its own communicator, so
// operations of different slots never share one; all ranks issue frames in the same order.
// Without ids there is no communicator (any nranks): the slots alone -- frames in flight on one GPU, or this rank's
// bands of a distributed G-buffer (sf_dist_render_bands, no collective; sf_dist_render then refuses).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cfloat>
#include <cstring>
#include <new>
#include <vector>

#include "sf_internal.h"
#include "sphereflake/sf.h"

// (sf_capi.hip) the unpack without the context's stream join: the caller orders `s` itself
extern "C" int sfi_unpack_slabs(sf_ctx* c, const void* stage, uint32_t bytes_per_pixel, uint32_t stage_rows, uint32_t band_rows,
                     uint32_t band_count, uint32_t first_member, uint32_t members, hipStream_t s, bool join);
// (sf_capi.hip) join the context stream after the context's previous calls on any stream (ctx_join)
extern "C" int sfi_join(sf_ctx* c);

struct sf_dist {
    int device = 0, rank = 0, nranks = 1;
    uint32_t W = 0, H = 0, band_rows = 8;
    struct Slot {
        sf_ctx* ctx = nullptr;
        ncclComm_t comm = nullptr;
        float* slab = nullptr;       // rank > 0: this rank's packed slab (slab_rows x W x 16 B at most)
        float* stage = nullptr;      // rank 0: the other ranks' packed slabs (nranks - 1) x stage_rows x W x 16 B at most
        hipStream_t recv = nullptr;  // rank 0 with peers: receive + unpack stream
        hipEvent_t start = nullptr;  // rank 0: the frame's start on the context stream (G-buffer free to rewrite)
        hipEvent_t done = nullptr;   // rank 0: the frame's unpack done (on `recv`)
        uint64_t view_gen = 0;       // the dist view (generation) this slot's context holds; 0 = none / its own
    };
    std::vector<Slot> slot;
    uint32_t slab_rows = 0, stage_rows = 0;
    uint64_t frames = 0;             // frames issued
    // the view of the next frames (sf_dist_set_view), applied to a slot's context only when a frame is rendered on it
    // (round 6: setting it on every slot at every frame was `slots` host-side root transforms per frame)
    float view[12] = {};
    uint64_t view_gen = 0;
    int last_hip = 0;
    int last_nccl = 0;
    int64_t* red = nullptr;          // device scratch of sf_dist_get_stats (4 x int64)
};

namespace {

struct Dev {
    int prev = -1;
    explicit Dev(int d)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~Dev()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

#define SFD_HIP(d, expr)                        \
    do {                                        \
        hipError_t e_ = (expr);                 \
        if (e_ != hipSuccess) {                 \
            (d)->last_hip = (int)e_;            \
            return SF_EHIP;                     \
        }                                       \
    } while (0)
#define SFD_NCCL(d, expr)                       \
    do {                                        \
        ncclResult_t r_ = (expr);               \
        if (r_ != ncclSuccess) {                \
            (d)->last_nccl = (int)r_;           \
            return SF_ECOMM;                    \
        }                                       \
    } while (0)

void free_dist(sf_dist* d)
{
    Dev g(d->device);
    for (auto& s : d->slot)
        if (s.ctx) (void)sf_synchronize(s.ctx);
    for (auto& s : d->slot) {
        if (s.recv) (void)hipStreamSynchronize(s.recv);
        if (s.comm) (void)ncclCommDestroy(s.comm);
        (void)hipFree(s.slab);
        (void)hipFree(s.stage);
        if (s.recv) (void)hipStreamDestroy(s.recv);
        if (s.start) (void)hipEventDestroy(s.start);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.ctx) sf_destroy(s.ctx);
    }
    (void)hipFree(d->red);
    delete d;
}

}  // namespace

extern "C" int sf_dist_unique_id(uint8_t id[SF_DIST_ID_BYTES])
{
    static_assert(SF_DIST_ID_BYTES == sizeof(ncclUniqueId), "RCCL unique id size");
    if (!id) return SF_EINVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return SF_ECOMM;
    std::memcpy(id, &u, sizeof u);
    return SF_OK;
}

extern "C" int sf_dist_create(int device, uint32_t width, uint32_t height, uint32_t band_rows, int rank, int nranks,
                              int slots, const uint8_t* ids, sf_dist** out)
{
    if (!out || width == 0 || height == 0 || nranks < 1 || rank < 0 || rank >= nranks || slots < 1 ||
        slots > SF_DIST_MAX_SLOTS || band_rows == 0 || band_rows % 8 != 0)
        return SF_EINVAL;
    *out = nullptr;
    sf_dist* d = new (std::nothrow) sf_dist();
    if (!d) return SF_ENOMEM;
    d->device = device;
    d->rank = rank;
    d->nranks = nranks;
    d->W = width;
    d->H = height;
    d->band_rows = band_rows;
    d->slot.resize(slots);
    const uint32_t n = (uint32_t)nranks;
    d->slab_rows = sf_slab_rows(height, band_rows, n, (uint32_t)rank);
    for (uint32_t k = 1; k < n; ++k) d->stage_rows = std::max(d->stage_rows, sf_slab_rows(height, band_rows, n, k));
    auto fail = [&](int rc) {
        free_dist(d);
        return rc;
    };
    for (auto& s : d->slot)
        if (int rc = sf_create(device, width, height, &s.ctx)) return fail(rc);
    Dev g(device);
    for (int k = 0; k < slots; ++k) {
        auto& s = d->slot[k];
        if (ids) {   // (one rank with ids: a communicator of one, which exercises the RCCL path)
            ncclUniqueId u;
            std::memcpy(&u, ids + (size_t)k * SF_DIST_ID_BYTES, sizeof u);
            const ncclResult_t r = ncclCommInitRank(&s.comm, nranks, u, rank);
            if (r != ncclSuccess) {
                d->last_nccl = (int)r;
                s.comm = nullptr;
                return fail(SF_ECOMM);
            }
        }
        hipError_t e = hipSuccess;
        if (rank > 0 && d->slab_rows) e = hipMalloc(&s.slab, (size_t)d->slab_rows * width * 16);
        if (e == hipSuccess && rank == 0 && nranks > 1 && d->stage_rows) {
            e = hipMalloc(&s.stage, (size_t)(nranks - 1) * d->stage_rows * width * 16);
            if (e == hipSuccess && ids) e = hipStreamCreateWithFlags(&s.recv, hipStreamNonBlocking);
            if (e == hipSuccess && ids) e = hipEventCreateWithFlags(&s.start, hipEventDisableTiming);
            if (e == hipSuccess && ids) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        }
        if (e != hipSuccess) {
            d->last_hip = (int)e;
            return fail(e == hipErrorOutOfMemory ? SF_ENOMEM : SF_EHIP);
        }
    }
    if (hipMalloc(&d->red, 4 * sizeof(int64_t)) != hipSuccess) return fail(SF_ENOMEM);
    *out = d;
    return SF_OK;
}

extern "C" void sf_dist_destroy(sf_dist* d)
{
    if (d) free_dist(d);
}

extern "C" int sf_dist_slots(const sf_dist* d) { return d ? (int)d->slot.size() : SF_EINVAL; }

extern "C" sf_ctx* sf_dist_context(sf_dist* d, int slot)
{
    return (d && slot >= 0 && slot < (int)d->slot.size()) ? d->slot[slot].ctx : nullptr;
}

extern "C" int sf_dist_last_slot(const sf_dist* d)
{
    if (!d) return SF_EINVAL;
    if (d->frames == 0) return SF_ESTATE;
    return (int)((d->frames - 1) % d->slot.size());
}

extern "C" int sf_dist_set_view(sf_dist* d, const float origin[3], const float top_left[3], const float top_right[3],
                                const float bottom_left[3])
{
    if (!d || !origin || !top_left || !top_right || !bottom_left) return SF_EINVAL;
    std::memcpy(d->view, origin, 12);
    std::memcpy(d->view + 3, top_left, 12);
    std::memcpy(d->view + 6, top_right, 12);
    std::memcpy(d->view + 9, bottom_left, 12);
    ++d->view_gen;
    return SF_OK;
}

namespace {
// The dist view into slot s's context, if it does not hold it yet (before a frame is rendered on it)
int apply_view(sf_dist* d, sf_dist::Slot& s)
{
    if (d->view_gen == 0 || s.view_gen == d->view_gen) return SF_OK;   // (no dist view yet: the context's own)
    if (int rc = sf_set_view(s.ctx, d->view, d->view + 3, d->view + 6, d->view + 9)) return rc;
    s.view_gen = d->view_gen;
    return SF_OK;
}
}   // namespace

extern "C" int sf_dist_render(sf_dist* d)
{
    if (!d) return SF_EINVAL;
    const uint32_t n = (uint32_t)d->nranks, W = d->W;
    auto& s = d->slot[d->frames % d->slot.size()];
    if (n > 1 && !s.comm) return SF_ESTATE;   // made without ids: bands only (sf_dist_render_bands)
    if (int rc = apply_view(d, s)) return rc;
    hipStream_t st = (hipStream_t)sf_context_stream(s.ctx);
    // the slab format follows from the view, the same on every rank (every rank sets the same views)
    const uint32_t bytes = sf_slab_bytes(s.ctx);
    if (bytes == 0) return SF_ENOVIEW;
    const size_t words = bytes / 4u;   // 32-bit words per pixel on the wire
    sf_render_params p;
    std::memset(&p, 0, sizeof p);
    p.band_rows = d->band_rows;
    p.band_count = n;
    p.band_index = (uint32_t)d->rank;
    if (d->rank == 0) {
        Dev g(d->device);
        const bool peers = n > 1 && d->stage_rows;
        // the frame starts here on the context stream: earlier work there (the consumers of this slot's previous
        // frame) is done before the receive stream rewrites the G-buffer
        // (joined first: a consumer of the previous frame queued on a caller's stream, e.g. sf_download_async on
        // stream X, is ordered into the context stream before the start event the receive stream waits for)
        if (peers) {
            if (int rc = sfi_join(s.ctx)) return rc;
            SFD_HIP(d, hipEventRecord(s.start, st));
            // The receive is posted BEFORE rank 0's own trace: the persistent trace grid takes every wave slot, and a
            // kernel dispatched behind it gets one only as the grid drains -- a one-wave kernel launched after a 1080p
            // trace started 69 us into its 100-us span, one launched before it at once (scripts/slot_residency_probe.py,
            // profiles/r5/slot_residency.txt). Posted after, the peers' ncclSend (and their next frames queued behind it
            // on their slot streams) would wait for most of rank 0's trace.
            SFD_HIP(d, hipStreamWaitEvent(s.recv, s.start, 0));
            const size_t cnt = (size_t)d->stage_rows * W * words;   // 32-bit words per peer of the stage
            SFD_NCCL(d, ncclGroupStart());
            for (uint32_t k = 1; k < n; ++k) {
                const size_t rows = sf_slab_rows(d->H, d->band_rows, n, k);
                if (!rows) continue;
                SFD_NCCL(d, ncclRecv(reinterpret_cast<uint32_t*>(s.stage) + (k - 1) * cnt, rows * W * words, ncclUint32,
                                     (int)k, s.comm, s.recv));
            }
            SFD_NCCL(d, ncclGroupEnd());
        }
        // rank 0: its bands in place on the context stream ...
        if (int rc = sf_render(s.ctx, &p)) return rc;
        if (peers) {
            // ... while the peers' slabs land and unpack on the receive stream
            if (int rc = sfi_unpack_slabs(s.ctx, s.stage, bytes, d->stage_rows, d->band_rows, n, 1, n - 1, s.recv, false))
                return rc;
            SFD_HIP(d, hipEventRecord(s.done, s.recv));
            SFD_HIP(d, hipStreamWaitEvent(st, s.done, 0));   // the frame is complete on the context stream
        }
    } else {
        p.compact = 1;
        p.packed = bytes == 4u ? SF_PACKED_INDEX : SF_PACKED_NORMAL;
        if (d->slab_rows) {
            if (int rc = sf_render_to(s.ctx, &p, s.slab, nullptr, nullptr, nullptr)) return rc;
            Dev g(d->device);
            SFD_NCCL(d, ncclSend(s.slab, (size_t)d->slab_rows * W * words, ncclUint32, 0, s.comm, st));
        }
    }
    ++d->frames;
    return SF_OK;
}

extern "C" int sf_dist_comm_info(const sf_dist* d, int slot, int* count, int* rank, int* device)
{
    if (!d || slot < 0 || slot >= (int)d->slot.size()) return SF_EINVAL;
    const ncclComm_t c = d->slot[slot].comm;
    if (!c) return SF_ESTATE;
    int v = 0;
    if (count) {
        if (ncclCommCount(c, &v) != ncclSuccess) return SF_ECOMM;
        *count = v;
    }
    if (rank) {
        if (ncclCommUserRank(c, &v) != ncclSuccess) return SF_ECOMM;
        *rank = v;
    }
    if (device) {
        if (ncclCommCuDevice(c, &v) != ncclSuccess) return SF_ECOMM;
        *device = v;
    }
    return SF_OK;
}

extern "C" int sf_dist_slab_bytes(const sf_dist* d)
{
    if (!d) return SF_EINVAL;
    sf_dist* m = const_cast<sf_dist*>(d);   // (only the lazily applied view changes: the next frame's slot gets it now)
    auto& s = m->slot[m->frames % m->slot.size()];
    if (int rc = apply_view(m, s)) return rc;
    return (int)sf_slab_bytes(s.ctx);
}

// This rank's bands of the next frame into its slot's G-buffer at frame positions (reference layout): the frame
// as a distributed G-buffer, every rank holding its own rows in its own HBM -- no gather.
extern "C" int sf_dist_render_bands(sf_dist* d)
{
    if (!d) return SF_EINVAL;
    auto& s = d->slot[d->frames % d->slot.size()];
    if (int rc = apply_view(d, s)) return rc;
    sf_render_params p;
    std::memset(&p, 0, sizeof p);
    p.band_rows = d->band_rows;
    p.band_count = (uint32_t)d->nranks;
    p.band_index = (uint32_t)d->rank;
    if (int rc = sf_render(s.ctx, &p)) return rc;
    ++d->frames;
    return SF_OK;
}

// The next n frames of a camera path (views[k] = {origin, top-left, top-right, bottom-left}) as this rank's bands,
// each into its own slot's G-buffer (slots (frames + k) % slots, n <= slots), in ONE multi-frame persistent launch
// (sf_render_frames) on the first frame's slot stream -- the distributed G-buffer of sf_dist_render_bands without a
// launch per frame.
extern "C" int sf_dist_render_bands_frames(sf_dist* d, uint32_t n, const float (*views)[12])
{
    if (!d || !views || n == 0 || n > (uint32_t)SF_RENDER_FRAMES_MAX || n > d->slot.size()) return SF_EINVAL;
    sf_ctx* cs[SF_RENDER_FRAMES_MAX];
    for (uint32_t k = 0; k < n; ++k) {
        auto& s = d->slot[(d->frames + k) % d->slot.size()];
        cs[k] = s.ctx;
        const float* v = views[k];
        if (int rc = sf_set_view(cs[k], v, v + 3, v + 6, v + 9)) return rc;
        s.view_gen = 0;   // (its own view now, not the dist view)
    }
    sf_render_params p;
    std::memset(&p, 0, sizeof p);
    p.band_rows = d->band_rows;
    p.band_count = (uint32_t)d->nranks;
    p.band_index = (uint32_t)d->rank;
    if (int rc = sf_render_frames(cs, n, &p)) return rc;
    d->frames += n;
    return SF_OK;
}

extern "C" int sf_dist_synchronize(sf_dist* d)
{
    if (!d) return SF_EINVAL;
    int first = SF_OK;
    for (auto& s : d->slot) {
        const int rc = sf_synchronize(s.ctx);
        if (rc != SF_OK && first == SF_OK) first = rc;
    }
    return first;
}

extern "C" int sf_dist_download(sf_dist* d, float* pos4, float* nrm4)
{
    if (!d) return SF_EINVAL;
    if (d->rank != 0 || d->frames == 0) return SF_ESTATE;
    if (int rc = sf_dist_synchronize(d)) return rc;
    return sf_download(d->slot[(d->frames - 1) % d->slot.size()].ctx, pos4, nrm4, nullptr, nullptr);
}

// Collective when the dist has communicators (every rank calls it; without ids: this rank's slots only, the caller
// combines the ranks). Stats of this rank's slots combined, then over the ranks on the device
// (max depth max, closest min, rays and overflow tiles summed: Sphereflake.h:30-58 over the whole frame).
extern "C" int sf_dist_get_stats(sf_dist* d, sf_stats* out)
{
    if (!d || !out) return SF_EINVAL;
    sf_stats t;
    std::memset(&t, 0, sizeof t);
    t.closest = FLT_MAX;
    for (auto& s : d->slot) {
        sf_stats x;
        if (int rc = sf_get_stats(s.ctx, &x)) return rc;
        t.max_depth = std::max(t.max_depth, x.max_depth);
        t.closest = std::min(t.closest, x.closest);
        t.rays += x.rays;
        t.overflow_tiles += x.overflow_tiles;
    }
    if (d->slot[0].comm) {
        Dev g(d->device);
        hipStream_t st = (hipStream_t)sf_context_stream(d->slot[0].ctx);
        // max of {max depth, -closest key}, sum of {rays, overflow tiles}
        int64_t h[4] = { t.max_depth, -(int64_t)sf_float_key(t.closest), t.rays, t.overflow_tiles };
        SFD_HIP(d, hipMemcpyAsync(d->red, h, sizeof h, hipMemcpyHostToDevice, st));
        SFD_NCCL(d, ncclAllReduce(d->red, d->red, 2, ncclInt64, ncclMax, d->slot[0].comm, st));
        SFD_NCCL(d, ncclAllReduce(d->red + 2, d->red + 2, 2, ncclInt64, ncclSum, d->slot[0].comm, st));
        SFD_HIP(d, hipMemcpyAsync(h, d->red, sizeof h, hipMemcpyDeviceToHost, st));
        SFD_HIP(d, hipStreamSynchronize(st));
        t.max_depth = (int32_t)h[0];
        t.closest = sf_key_float((int32_t)(-h[1]));
        t.rays = h[2];
        t.overflow_tiles = h[3];
    }
    *out = t;
    return SF_OK;
}

extern "C" int sf_dist_reset_stats(sf_dist* d)
{
    if (!d) return SF_EINVAL;
    for (auto& s : d->slot) {
        if (int rc = sf_reset_max_depth(s.ctx)) return rc;
        if (int rc = sf_reset_closest(s.ctx)) return rc;
        if (int rc = sf_reset_rays(s.ctx)) return rc;
    }
    return SF_OK;
}

extern "C" int sf_dist_last_error(const sf_dist* d, int* hip_error, int* rccl_error)
{
    if (!d) return SF_EINVAL;
    if (hip_error) *hip_error = d->last_hip;
    if (rccl_error) *rccl_error = d->last_nccl;
    return SF_OK;
}
