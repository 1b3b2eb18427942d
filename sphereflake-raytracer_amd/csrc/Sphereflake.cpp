// Sphereflake.cpp -- the reference-compatible C++ class over the C ABI (see Sphereflake.hpp).
// Reference surface: /root/reference/sphereflake/Sphereflake.h:13-58, Sphereflake.cpp:43-84.
#include "Sphereflake.hpp"
#include "SphereflakeSSAO.hpp"

#include <chrono>
#include <cstdio>
#include <cstring>
#include <ctime>

namespace SphereflakeRaytracer {

static void Check(int rc)
{
    if (rc != SF_OK) throw std::runtime_error(std::string("sphereflake: ") + sf_strerror(rc));
}

void Sphereflake::Check(int rc) { SphereflakeRaytracer::Check(rc); }

void Sphereflake::Open(int device, float* positions, float* normals)
{
    Check(sf_create(device, (uint32_t)m_Width, (uint32_t)m_Height, &m_Ctx));
    m_Positions = positions;
    m_Normals = normals;
    // page-lock the vectors' storage (they stay std::vector for the PBO upload, GLPixelBufferObject.h:24-29)
    // so GetGBuffer's D2H runs as DMA straight into them; not fatal when the host refuses to pin
    const size_t bytes = m_Width * m_Height * 16;
    m_Pinned = bytes && sf_host_register(m_Positions, bytes) == SF_OK && sf_host_register(m_Normals, bytes) == SF_OK;
}

void Sphereflake::Close() noexcept
{
    m_Deinitialize = true;
    if (m_Worker.joinable()) m_Worker.join();
    const int rc = m_WorkerError.exchange(SF_OK);
    if (rc != SF_OK) std::fprintf(stderr, "sphereflake: frame-less loop failed: %s\n", sf_strerror(rc));
    sf_destroy(m_Ctx);
    m_Ctx = nullptr;
    if (m_Pinned) {
        sf_host_unregister(m_Positions);
        sf_host_unregister(m_Normals);
        m_Pinned = false;
    }
}

void Sphereflake::SetViewFloats(const float origin[3], const float topLeft[3], const float topRight[3],
                                const float bottomLeft[3])
{
    std::lock_guard<FairMutex> lk(m_Mutex);
    Check(sf_set_view(m_Ctx, origin, topLeft, topRight, bottomLeft));
    m_ViewChange = m_SobolCounter;
}

void Sphereflake::Render(const sf_render_params* params)
{
    std::lock_guard<FairMutex> lk(m_Mutex);
    Check(sf_render(m_Ctx, params));
    m_Stale = true;
}

void Sphereflake::SaveImage(const std::string& path, int what) const
{
    std::lock_guard<FairMutex> lk(m_Mutex);
    Check(sf_save_image(m_Ctx, path.c_str(), what));
}

// Frame-less mode: like the reference's worker threads (seeded from time(NULL), Sphereflake.cpp:88-89),
// a host thread keeps tracing batches of random packets into the persistent G-buffer.
void Sphereflake::Initialize() { Initialize((uint32_t)time(NULL)); }

void Sphereflake::Initialize(uint32_t seed, uint32_t batch)
{
    if (m_Worker.joinable()) {
        if (m_WorkerError.load() == SF_OK) return;   // the loop is running
        m_Worker.join();                             // it stopped on an error: report that error
    }
    if (batch == 0) throw std::runtime_error("sphereflake: Initialize batch must be > 0");
    ThrowWorkerError();
    m_Deinitialize = false;
    {
        std::lock_guard<FairMutex> lk(m_Mutex);
        m_Seed = seed;
        m_SobolCounter = 0;
    }
    m_Worker = std::thread([this, batch] { ProgressiveLoop(batch); });
}

// Batches of 2^18 packets take ~0.6 ms at 1080p (binning + draw prefetch pay from 2^16). Every context
// call is made under m_Mutex (sf.h: one context per host thread at a time), a FIFO lock: a caller's
// SetView / GetGBuffer waits for at most the batch in flight, never for the loop's next one. The first
// failure stops the loop and is kept for the main thread (ThrowWorkerError).
void Sphereflake::ProgressiveLoop(uint32_t batch)
{
    while (!m_Deinitialize) {
        std::lock_guard<FairMutex> lk(m_Mutex);
        int rc = sf_progressive(m_Ctx, m_Seed, m_SobolCounter, batch, nullptr);
        if (rc == SF_OK) rc = sf_synchronize(m_Ctx);
        if (rc != SF_OK) {
            int expected = SF_OK;
            m_WorkerError.compare_exchange_strong(expected, rc);
            return;
        }
        m_SobolCounter += batch;
        m_Stale = true;
    }
}

void Sphereflake::ThrowWorkerError() const
{
    const int rc = m_WorkerError.exchange(SF_OK);
    if (rc != SF_OK) throw std::runtime_error(std::string("sphereflake: frame-less loop failed: ") + sf_strerror(rc));
}

void Sphereflake::Deinitialize()
{
    m_Deinitialize = true;
    if (m_Worker.joinable()) m_Worker.join();
    ThrowWorkerError();
}

uint64_t Sphereflake::GetPacketsTraced() const
{
    std::lock_guard<FairMutex> lk(m_Mutex);
    return m_SobolCounter;
}

uint64_t Sphereflake::GetViewChangePacket() const
{
    std::lock_guard<FairMutex> lk(m_Mutex);
    return m_ViewChange;
}

void Sphereflake::Refresh() const
{
    ThrowWorkerError();
    std::lock_guard<FairMutex> lk(m_Mutex);
    if (m_Stale) {
        Check(sf_download(m_Ctx, m_Positions, m_Normals, nullptr, nullptr));
        m_Stale = false;
    }
}

int Sphereflake::GetMaxDepthReached() const
{
    ThrowWorkerError();
    std::lock_guard<FairMutex> lk(m_Mutex);
    sf_stats s;
    Check(sf_get_stats(m_Ctx, &s));
    return s.max_depth;
}

void Sphereflake::ResetMaxDepthReached()
{
    std::lock_guard<FairMutex> lk(m_Mutex);
    Check(sf_reset_max_depth(m_Ctx));
}

long long Sphereflake::GetRaysPerSecond() const
{
    ThrowWorkerError();
    std::lock_guard<FairMutex> lk(m_Mutex);
    sf_stats s;
    Check(sf_get_stats(m_Ctx, &s));
    return (long long)s.rays;
}

void Sphereflake::ResetRaysPerSecond()
{
    std::lock_guard<FairMutex> lk(m_Mutex);
    Check(sf_reset_rays(m_Ctx));
}

float Sphereflake::GetClosestSphereDistance() const
{
    ThrowWorkerError();
    std::lock_guard<FairMutex> lk(m_Mutex);
    sf_stats s;
    Check(sf_get_stats(m_Ctx, &s));
    return s.closest;
}

void Sphereflake::ResetClosestSphereDistance()
{
    std::lock_guard<FairMutex> lk(m_Mutex);
    Check(sf_reset_closest(m_Ctx));
}

namespace Headless {

SSAO::SSAO(Sphereflake& flake, int downScale) : m_Flake(flake)
{
    if (downScale < 1) throw std::runtime_error("sphereflake: SSAO downScale must be >= 1");
    Check(sf_post_defaults(flake.Context(), &m_Params));
    m_Params.downscale = (uint32_t)downScale;
}

void SSAO::SetCameraPositionFloats(const float p[3])
{
    std::memcpy(m_Params.camera_position, p, sizeof m_Params.camera_position);
    m_CameraSet = true;
}

void SSAO::Render()
{
    if (!m_CameraSet) {
        sf_post_params d;
        Check(sf_post_defaults(m_Flake.Context(), &d));
        std::memcpy(m_Params.camera_position, d.camera_position, sizeof d.camera_position);
    }
    Check(sf_post_process(m_Flake.Context(), &m_Params, nullptr, nullptr, nullptr, nullptr));
}

void SSAO::SaveImage(const std::string& path) const { m_Flake.SaveImage(path, SF_DUMP_IMAGE); }

const std::vector<uint8_t>& SSAO::GetImage() const
{
    m_Image.resize(m_Flake.Width() * m_Flake.Height() * 4);
    Check(sf_download_image(m_Flake.Context(), m_Image.data()));
    return m_Image;
}

}  // namespace Headless

}  // namespace SphereflakeRaytracer
