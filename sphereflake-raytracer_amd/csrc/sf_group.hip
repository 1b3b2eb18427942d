// sf_group.hip -- single-process multi-GPU rendering behind the C ABI.
//
// The reference's only parallelism is its host thread pool (Sphereflake.cpp:67-74): every thread
// renders into the one shared G-buffer. Here the frame is cut into interleaved bands of band_rows
// rows (band b -> member b mod n: flake rows cost ~150 nodes per ray, sky rows ~1, so contiguous
// halves would be badly unbalanced) and every member device traces its own bands. Member 0 writes its
// bands straight into its own (final) G-buffer at frame positions; member k > 0 traces its bands into a
// PACKED compact slab in its own HBM (one uint32 hit index per pixel where the view allows it, sf_slab_bytes:
// an eighth of the G-buffer's 32 B; else one float4 (nx, ny, nz, minT); member 0 rebuilds the rest bit for bit)
// and ships it with one contiguous peer copy over xGMI into member 0's stage, on a copy stream of its own, so
// the next frame's trace on the member overlaps the copy. Member 0 unpacks the stage into the G-buffer
// (sf_unpack_slabs) on an unpack stream of its own, beside its own trace, after the frame's copies and after
// the frame's start on its context stream; the context stream then waits for the unpack, so work queued on
// member 0's context after sf_group_render (download, post-process) sees the whole frame, and consumers of the
// previous frame queued before it are never overwritten. Slabs and stages are double-buffered by frame
// parity: member k traces frame f + 1 while frame f's copy drains, and frame f + 2's copy into a stage waits
// only for member 0's unpack of frame f from it.
#include <hip/hip_runtime.h>

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

struct sf_group {
    int n = 0;
    uint32_t W = 0, H = 0;
    std::vector<int> device;
    std::vector<sf_ctx*> ctx;
    // per parity b (frame & 1)
    std::vector<float*> slab[2];         // members k > 0: packed compact band slab on their device
    float* stage[2] = { nullptr, nullptr };   // member 0: members 1..n-1's slabs, stage_rows x W float4 each
    std::vector<hipEvent_t> traced[2];   // member k's trace of the frame done (its context stream)
    std::vector<hipEvent_t> copied[2];   // member k's copy into member 0's stage done (its copy stream)
    hipEvent_t unpacked[2] = { nullptr, nullptr };   // member 0 done reading stage[b] (its unpack stream)
    hipEvent_t start0 = nullptr;         // member 0: the frame's start on its context stream
    hipStream_t unpack0 = nullptr;       // member 0: unpack stream
    std::vector<hipStream_t> copy;       // members k > 0: copy stream
    uint32_t band_rows = 0, stage_rows = 0;   // the split the buffers are sized for (0: none yet)
    uint64_t frames = 0;
    bool stage_used[2] = { false, false };
    int last_hip = 0;
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

#define SFG_HIP(g, expr)                        \
    do {                                        \
        hipError_t e_ = (expr);                 \
        if (e_ != hipSuccess) {                 \
            (g)->last_hip = (int)e_;            \
            return SF_EHIP;                     \
        }                                       \
    } while (0)

void free_buffers(sf_group* g)
{
    for (int b = 0; b < 2; ++b) {
        for (int k = 0; k < g->n; ++k) {
            if (k < (int)g->slab[b].size() && g->slab[b][k]) {
                Dev d(g->device[k]);
                (void)hipFree(g->slab[b][k]);
                g->slab[b][k] = nullptr;
            }
        }
        if (g->stage[b]) {
            Dev d(g->device[0]);
            (void)hipFree(g->stage[b]);
            g->stage[b] = nullptr;
        }
        g->stage_used[b] = false;
    }
    g->band_rows = g->stage_rows = 0;
}

void free_group(sf_group* g)
{
    for (int k = 0; k < g->n; ++k)
        if (k < (int)g->ctx.size() && g->ctx[k]) sf_synchronize(g->ctx[k]);
    for (int k = 0; k < g->n; ++k) {
        Dev d(g->device[k]);
        if (k < (int)g->copy.size() && g->copy[k]) (void)hipStreamSynchronize(g->copy[k]);
    }
    free_buffers(g);
    for (int k = 0; k < g->n; ++k) {
        Dev d(g->device[k]);
        for (int b = 0; b < 2; ++b) {
            if (k < (int)g->traced[b].size() && g->traced[b][k]) (void)hipEventDestroy(g->traced[b][k]);
            if (k < (int)g->copied[b].size() && g->copied[b][k]) (void)hipEventDestroy(g->copied[b][k]);
        }
        if (k < (int)g->copy.size() && g->copy[k]) (void)hipStreamDestroy(g->copy[k]);
    }
    {
        Dev d(g->device[0]);
        if (g->unpack0) (void)hipStreamSynchronize(g->unpack0);
        for (int b = 0; b < 2; ++b)
            if (g->unpacked[b]) (void)hipEventDestroy(g->unpacked[b]);
        if (g->start0) (void)hipEventDestroy(g->start0);
        if (g->unpack0) (void)hipStreamDestroy(g->unpack0);
    }
    for (sf_ctx* c : g->ctx) sf_destroy(c);
    delete g;
}

}  // namespace

extern "C" int sf_group_create(const int* devices, int n, uint32_t width, uint32_t height, sf_group** out)
{
    if (!out || !devices || n < 1 || width == 0 || height == 0) return SF_EINVAL;
    *out = nullptr;
    sf_group* g = new (std::nothrow) sf_group();
    if (!g) return SF_ENOMEM;
    g->n = n;
    g->W = width;
    g->H = height;
    g->device.assign(devices, devices + n);
    g->ctx.assign(n, nullptr);
    g->copy.assign(n, nullptr);
    for (int b = 0; b < 2; ++b) {
        g->slab[b].assign(n, nullptr);
        g->traced[b].assign(n, nullptr);
        g->copied[b].assign(n, nullptr);
    }
    for (int k = 0; k < n; ++k) {
        const int rc = sf_create(devices[k], width, height, &g->ctx[k]);
        if (rc != SF_OK) {
            free_group(g);
            return rc;
        }
    }
    // peer access between member 0 and every other device (copies into member 0's stage)
    for (int k = 1; k < n; ++k) {
        if (devices[k] == devices[0]) continue;
        int ok = 0;
        if (hipDeviceCanAccessPeer(&ok, devices[k], devices[0]) != hipSuccess || !ok) {
            free_group(g);
            return SF_ENODEV;
        }
        for (int pass = 0; pass < 2; ++pass) {
            Dev d(pass ? devices[0] : devices[k]);
            const hipError_t e = hipDeviceEnablePeerAccess(pass ? devices[k] : devices[0], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                g->last_hip = (int)e;
                free_group(g);
                return SF_EHIP;
            }
            (void)hipGetLastError();   // clear an "already enabled"
        }
    }
    for (int k = 0; k < n; ++k) {
        Dev d(devices[k]);
        bool ok = true;
        for (int b = 0; b < 2; ++b) {
            if (k == 0) ok = ok && hipEventCreateWithFlags(&g->unpacked[b], hipEventDisableTiming) == hipSuccess;
            if (k > 0) {
                ok = ok && hipEventCreateWithFlags(&g->traced[b][k], hipEventDisableTiming) == hipSuccess;
                ok = ok && hipEventCreateWithFlags(&g->copied[b][k], hipEventDisableTiming) == hipSuccess;
            }
        }
        if (k > 0) ok = ok && hipStreamCreateWithFlags(&g->copy[k], hipStreamNonBlocking) == hipSuccess;
        if (k == 0) ok = ok && hipEventCreateWithFlags(&g->start0, hipEventDisableTiming) == hipSuccess;
        if (k == 0) ok = ok && hipStreamCreateWithFlags(&g->unpack0, hipStreamNonBlocking) == hipSuccess;
        if (!ok) {
            free_group(g);
            return SF_EHIP;
        }
    }
    *out = g;
    return SF_OK;
}

extern "C" void sf_group_destroy(sf_group* g)
{
    if (g) free_group(g);
}

extern "C" int sf_group_size(const sf_group* g) { return g ? g->n : SF_EINVAL; }

extern "C" sf_ctx* sf_group_member(sf_group* g, int k) { return (g && k >= 0 && k < g->n) ? g->ctx[k] : nullptr; }

extern "C" int sf_group_set_view(sf_group* g, const float origin[3], const float top_left[3], const float top_right[3],
                                 const float bottom_left[3])
{
    if (!g) return SF_EINVAL;
    for (sf_ctx* c : g->ctx) {
        const int rc = sf_set_view(c, origin, top_left, top_right, bottom_left);
        if (rc != SF_OK) return rc;
    }
    return SF_OK;
}

extern "C" int sf_group_set_variant(sf_group* g, int variant)
{
    if (!g) return SF_EINVAL;
    for (sf_ctx* c : g->ctx) {
        const int rc = sf_set_variant(c, variant);
        if (rc != SF_OK) return rc;
    }
    return SF_OK;
}

extern "C" int sf_group_render(sf_group* g, uint32_t band_rows)
{
    if (!g) return SF_EINVAL;
    if (band_rows == 0) band_rows = 8;
    if (band_rows % 8 != 0) return SF_EINVAL;
    const uint32_t n = (uint32_t)g->n, W = g->W, H = g->H;
    if (g->band_rows != band_rows) {   // (re)size the slabs and stages for this split
        if (int rc = sf_group_synchronize(g)) return rc;
        for (uint32_t k = 1; k < n; ++k) {
            Dev d(g->device[k]);
            SFG_HIP(g, hipStreamSynchronize(g->copy[k]));
        }
        free_buffers(g);
        uint32_t sr = 0;
        for (uint32_t k = 1; k < n; ++k) sr = std::max(sr, sf_slab_rows(H, band_rows, n, k));
        for (int b = 0; b < 2; ++b) {
            for (uint32_t k = 1; k < n; ++k) {
                const uint32_t rows = sf_slab_rows(H, band_rows, n, k);
                if (!rows) continue;
                Dev d(g->device[k]);
                SFG_HIP(g, hipMalloc(&g->slab[b][k], (size_t)rows * W * 16));
            }
            if (sr) {
                Dev d(g->device[0]);
                SFG_HIP(g, hipMalloc(&g->stage[b], (size_t)(n - 1) * sr * W * 16));
            }
        }
        g->band_rows = band_rows;
        g->stage_rows = sr;
    }
    const int b = (int)(g->frames & 1u);
    const uint32_t bytes = sf_slab_bytes(g->ctx[0]);   // the slab format of this view (the same for every member)
    if (bytes == 0) return SF_ENOVIEW;
    const size_t stage_slab = (size_t)g->stage_rows * W * bytes;   // bytes per member in the stage
    // members k > 0: trace the packed slab, then copy it into member 0's stage on the copy stream
    for (uint32_t k = 1; k < n; ++k) {
        const uint32_t rows = sf_slab_rows(H, band_rows, n, k);
        if (rows == 0) continue;
        Dev d(g->device[k]);
        hipStream_t sk = (hipStream_t)sf_context_stream(g->ctx[k]);
        // slab[b] was last read by the copy of frame f - 2
        if (g->frames >= 2) SFG_HIP(g, hipStreamWaitEvent(sk, g->copied[b][k], 0));
        sf_render_params p;
        std::memset(&p, 0, sizeof p);
        p.band_rows = band_rows;
        p.band_count = n;
        p.band_index = k;
        p.compact = 1;
        p.packed = bytes == 4u ? SF_PACKED_INDEX : SF_PACKED_NORMAL;
        if (int rc = sf_render_to(g->ctx[k], &p, g->slab[b][k], nullptr, nullptr, nullptr)) return rc;
        SFG_HIP(g, hipEventRecord(g->traced[b][k], sk));
        SFG_HIP(g, hipStreamWaitEvent(g->copy[k], g->traced[b][k], 0));
        // stage[b] was last read by member 0's unpack of frame f - 2
        if (g->stage_used[b]) SFG_HIP(g, hipStreamWaitEvent(g->copy[k], g->unpacked[b], 0));
        SFG_HIP(g, hipMemcpyAsync(reinterpret_cast<char*>(g->stage[b]) + (size_t)(k - 1) * stage_slab, g->slab[b][k],
                                  (size_t)rows * W * bytes, hipMemcpyDeviceToDevice, g->copy[k]));
        SFG_HIP(g, hipEventRecord(g->copied[b][k], g->copy[k]));
    }
    // member 0: its bands in place on its context stream, and beside them (after the copies, and after the
    // frame's start on the context stream) the others' unpacked on the unpack stream, which the context stream
    // then waits for
    sf_render_params p;
    std::memset(&p, 0, sizeof p);
    p.band_rows = band_rows;
    p.band_count = n;
    p.band_index = 0;
    const bool peers = n > 1 && g->stage_rows;
    hipStream_t s0 = (hipStream_t)sf_context_stream(g->ctx[0]);
    if (peers) {
        Dev d(g->device[0]);
        // joined first: work queued on member 0 on a caller's stream (sf_download_async, sf_post_process on stream
        // X) is ordered into s0 before start0, which is all the unpack stream waits for
        if (int rc = sfi_join(g->ctx[0])) return rc;
        SFG_HIP(g, hipEventRecord(g->start0, s0));
    }
    if (int rc = sf_render(g->ctx[0], &p)) return rc;
    if (peers) {
        Dev d(g->device[0]);
        SFG_HIP(g, hipStreamWaitEvent(g->unpack0, g->start0, 0));
        for (uint32_t k = 1; k < n; ++k)
            if (sf_slab_rows(H, band_rows, n, k)) SFG_HIP(g, hipStreamWaitEvent(g->unpack0, g->copied[b][k], 0));
        if (int rc = sfi_unpack_slabs(g->ctx[0], g->stage[b], bytes, g->stage_rows, band_rows, n, 1, n - 1, g->unpack0,
                                      false))
            return rc;
        SFG_HIP(g, hipEventRecord(g->unpacked[b], g->unpack0));
        SFG_HIP(g, hipStreamWaitEvent(s0, g->unpacked[b], 0));
        g->stage_used[b] = true;
    }
    ++g->frames;
    return SF_OK;
}

extern "C" int sf_group_synchronize(sf_group* g)
{
    if (!g) return SF_EINVAL;
    int first = SF_OK;
    for (sf_ctx* c : g->ctx) {
        const int rc = sf_synchronize(c);
        if (rc != SF_OK && first == SF_OK) first = rc;
    }
    return first;
}

extern "C" int sf_group_download(sf_group* g, float* pos4, float* nrm4)
{
    if (!g) return SF_EINVAL;
    if (int rc = sf_group_synchronize(g)) return rc;
    return sf_download(g->ctx[0], pos4, nrm4, nullptr, nullptr);
}

extern "C" int sf_group_get_stats(sf_group* g, sf_stats* out)
{
    if (!g || !out) return SF_EINVAL;
    sf_stats t;
    std::memset(&t, 0, sizeof t);
    t.closest = FLT_MAX;
    for (sf_ctx* c : g->ctx) {
        sf_stats s;
        if (int rc = sf_get_stats(c, &s)) return rc;
        t.max_depth = std::max(t.max_depth, s.max_depth);
        t.closest = std::min(t.closest, s.closest);
        t.rays += s.rays;
        t.overflow_tiles += s.overflow_tiles;
    }
    *out = t;
    return SF_OK;
}

extern "C" int sf_group_reset_stats(sf_group* g)
{
    if (!g) return SF_EINVAL;
    for (sf_ctx* c : g->ctx) {
        if (int rc = sf_reset_max_depth(c)) return rc;
        if (int rc = sf_reset_closest(c)) return rc;
        if (int rc = sf_reset_rays(c)) return rc;
    }
    return SF_OK;
}

extern "C" int sf_group_last_hip_error(const sf_group* g) { return g ? g->last_hip : 0; }

extern "C" int sf_group_slab_bytes(const sf_group* g) { return g ? (int)sf_slab_bytes(g->ctx[0]) : SF_EINVAL; }
