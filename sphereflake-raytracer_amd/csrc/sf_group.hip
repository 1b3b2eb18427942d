// sf_group.hip -- single-process multi-GPU rendering behind the C ABI.
//
// The reference's only parallelism is its host thread pool (Sphereflake.cpp:67-74): every thread
// renders into the one shared G-buffer. Here the frame is cut into interleaved bands of band_rows
// rows (band b -> member b mod n: flake rows cost ~150 nodes per ray, sky rows ~1, so contiguous
// halves would be badly unbalanced) and every member device traces its own bands. Member 0 writes its
// bands straight into its own (final) G-buffer at frame positions; member k > 0 traces its bands into
// a compact slab in its own HBM and ships it to member 0 with ONE strided 2D copy per buffer over
// xGMI (slab band i -> frame band i*n + k: source pitch one band, destination pitch n bands), queued
// on its own stream right behind its render, so they overlap the other members' still-running traces. No
// reassembly pass, no staging copy, no host round trip. The copies into member 0's buffers wait for
// the work member 0's stream had queued when the frame was issued (its consumers of the previous
// frame), and member 0's stream waits for every member's copies, so anything queued on member 0's
// context after sf_group_render (download, post-process) sees the whole frame.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstring>
#include <new>
#include <vector>

#include "sf_internal.h"
#include "sphereflake/sf.h"

struct sf_group {
    int n = 0;
    uint32_t W = 0, H = 0;
    std::vector<int> device;
    std::vector<sf_ctx*> ctx;
    std::vector<float*> slab_pos, slab_nrm;   // members k > 0: compact band slabs on their device
    std::vector<uint32_t> slab_rows;
    std::vector<hipEvent_t> copied;      // member k's copies of the frame done (its stream)
    hipEvent_t issued = nullptr;         // member 0's stream at frame issue (its previous consumers)
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

void free_group(sf_group* g)
{
    for (int k = 0; k < g->n; ++k) {
        if (k < (int)g->ctx.size() && g->ctx[k]) sf_synchronize(g->ctx[k]);
    }
    for (int k = 0; k < g->n; ++k) {
        Dev d(g->device[k]);
        if (k < (int)g->copied.size() && g->copied[k]) (void)hipEventDestroy(g->copied[k]);
        if (k < (int)g->slab_pos.size()) (void)hipFree(g->slab_pos[k]);
        if (k < (int)g->slab_nrm.size()) (void)hipFree(g->slab_nrm[k]);
    }
    if (g->issued) {
        Dev d(g->device[0]);
        (void)hipEventDestroy(g->issued);
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
    g->slab_pos.assign(n, nullptr);
    g->slab_nrm.assign(n, nullptr);
    g->slab_rows.assign(n, 0u);
    g->copied.assign(n, nullptr);
    for (int k = 0; k < n; ++k) {
        const int rc = sf_create(devices[k], width, height, &g->ctx[k]);
        if (rc != SF_OK) {
            free_group(g);
            return rc;
        }
    }
    // peer access between member 0 and every other device (copies into member 0's G-buffer)
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
    {
        Dev d(devices[0]);
        if (hipEventCreateWithFlags(&g->issued, hipEventDisableTiming) != hipSuccess) {
            free_group(g);
            return SF_EHIP;
        }
    }
    for (int k = 0; k < n; ++k) {
        Dev d(devices[k]);
        if (hipEventCreateWithFlags(&g->copied[k], hipEventDisableTiming) != hipSuccess) {
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
    const uint32_t bands = (H + band_rows - 1) / band_rows;
    const size_t band_bytes = (size_t)band_rows * W * 16;   // one band of one buffer (float4 per pixel)
    float *pos0 = nullptr, *nrm0 = nullptr;
    if (int rc = sf_device_buffers(g->ctx[0], &pos0, &nrm0, nullptr, nullptr)) return rc;
    for (uint32_t k = 0; k < n; ++k) {
        sf_render_params p;
        std::memset(&p, 0, sizeof p);
        p.band_rows = band_rows;
        p.band_count = n;
        p.band_index = k;
        if (k == 0) {
            // member 0: its bands straight into the final G-buffer, at frame positions
            if (int rc = sf_render(g->ctx[0], &p)) return rc;
            continue;
        }
        p.compact = 1;
        const uint32_t rows = sf_slab_rows(H, band_rows, n, k);
        if (rows == 0) continue;
        Dev d(g->device[k]);
        if (g->slab_rows[k] != rows || !g->slab_pos[k]) {
            // the old slabs may still be copied from
            SFG_HIP(g, hipStreamSynchronize((hipStream_t)sf_context_stream(g->ctx[k])));
            (void)hipFree(g->slab_pos[k]);
            (void)hipFree(g->slab_nrm[k]);
            g->slab_pos[k] = g->slab_nrm[k] = nullptr;
            g->slab_rows[k] = 0;
            SFG_HIP(g, hipMalloc(&g->slab_pos[k], (size_t)rows * W * 16));
            SFG_HIP(g, hipMalloc(&g->slab_nrm[k], (size_t)rows * W * 16));
            g->slab_rows[k] = rows;
        }
        if (int rc = sf_render_to(g->ctx[k], &p, g->slab_pos[k], g->slab_nrm[k], nullptr, nullptr)) return rc;
    }
    // Member 0's stream now ends with this frame's render, behind everything queued on it before
    // (consumers of the previous frame): the copies into its buffers wait for that point.
    hipStream_t s0 = (hipStream_t)sf_context_stream(g->ctx[0]);
    {
        Dev d(g->device[0]);
        SFG_HIP(g, hipEventRecord(g->issued, s0));
    }
    for (uint32_t k = 1; k < n; ++k) {
        const uint32_t rows = sf_slab_rows(H, band_rows, n, k);
        if (rows == 0) continue;
        Dev d(g->device[k]);
        // owned bands: k, k + n, ...; the full ones as one strided copy per buffer, a partial last band apart
        uint32_t nb = 0, full = 0;
        for (uint32_t b = k; b < bands; b += n) {
            ++nb;
            if ((b + 1) * band_rows <= H) ++full;
        }
        hipStream_t sk = (hipStream_t)sf_context_stream(g->ctx[k]);
        SFG_HIP(g, hipStreamWaitEvent(sk, g->issued, 0));   // (the member's render is queued before this)
        for (int buf = 0; buf < 2; ++buf) {
            char* dst = reinterpret_cast<char*>(buf ? nrm0 : pos0);
            const char* src = reinterpret_cast<const char*>(buf ? g->slab_nrm[k] : g->slab_pos[k]);
            if (full)
                SFG_HIP(g, hipMemcpy2DAsync(dst + (size_t)k * band_bytes, (size_t)n * band_bytes, src, band_bytes,
                                            band_bytes, full, hipMemcpyDeviceToDevice, sk));
            if (full < nb) {   // the frame's last band, shorter than band_rows
                const uint32_t b = k + full * n;
                const size_t bytes = (size_t)(H - b * band_rows) * W * 16;
                SFG_HIP(g, hipMemcpyAsync(dst + (size_t)b * band_bytes, src + (size_t)full * band_bytes, bytes,
                                          hipMemcpyDeviceToDevice, sk));
            }
        }
        SFG_HIP(g, hipEventRecord(g->copied[k], sk));
    }
    {   // member 0's stream waits for every member's copies: later work on it sees the whole frame
        Dev d(g->device[0]);
        for (uint32_t k = 1; k < n; ++k)
            if (sf_slab_rows(H, band_rows, n, k)) SFG_HIP(g, hipStreamWaitEvent(s0, g->copied[k], 0));
    }
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
