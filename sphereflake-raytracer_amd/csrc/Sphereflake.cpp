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

Sphereflake::Sphereflake(size_t width, size_t height, int device) : m_Width(width), m_Height(height)
{
    Check(sf_create(device, (uint32_t)width, (uint32_t)height, &m_Ctx));
    // reference: m_GBuffer.positions/normals.resize(W*H) of zero vec4 (Sphereflake.cpp:48-49)
    m_GBuffer.positions.resize(width * height);
    m_GBuffer.normals.resize(width * height);
    // page-lock the vectors' storage (they stay std::vector for the PBO upload, GLPixelBufferObject.h:24-29)
    // so GetGBuffer's D2H runs as DMA straight into them; not fatal when the host refuses to pin
    const size_t bytes = width * height * sizeof(sf_vec4);
    m_Pinned = bytes && sf_host_register(m_GBuffer.positions.data(), bytes) == SF_OK &&
               sf_host_register(m_GBuffer.normals.data(), bytes) == SF_OK;
}

Sphereflake::~Sphereflake()
{
    m_Deinitialize = true;
    if (m_Worker.joinable()) m_Worker.join();
    const int rc = m_WorkerError.exchange(SF_OK);
    if (rc != SF_OK) std::fprintf(stderr, "sphereflake: frame-less loop failed: %s\n", sf_strerror(rc));
    sf_destroy(m_Ctx);
    if (m_Pinned) {
        sf_host_unregister(m_GBuffer.positions.data());
        sf_host_unregister(m_GBuffer.normals.data());
    }
}

void Sphereflake::SetView(const sf_vec3& origin, const sf_vec3& topLeft, const sf_vec3& topRight, const sf_vec3& bottomLeft)
{
    std::lock_guard<FairMutex> lk(m_Mutex);
    const float o[3] = { origin.x, origin.y, origin.z };
    const float tl[3] = { topLeft.x, topLeft.y, topLeft.z };
    const float tr[3] = { topRight.x, topRight.y, topRight.z };
    const float bl[3] = { bottomLeft.x, bottomLeft.y, bottomLeft.z };
    Check(sf_set_view(m_Ctx, o, tl, tr, bl));
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

const GBuffer& Sphereflake::GetGBuffer() const
{
    ThrowWorkerError();
    std::lock_guard<FairMutex> lk(m_Mutex);
    if (m_Stale) {
        Check(sf_download(m_Ctx, &m_GBuffer.positions[0].x, &m_GBuffer.normals[0].x, nullptr, nullptr));
        m_Stale = false;
    }
    return m_GBuffer;
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

void SSAO::SetCameraPosition(const sf_vec3& p)
{
    m_Params.camera_position[0] = p.x;
    m_Params.camera_position[1] = p.y;
    m_Params.camera_position[2] = p.z;
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
