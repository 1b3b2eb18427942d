// Sphereflake.hpp -- drop-in replacement for the reference class
// SphereflakeRaytracer::Sphereflake (/root/reference/sphereflake/Sphereflake.h:13-58), layered on
// the C ABI (include/sphereflake/sf.h). Same names, argument meaning and stats semantics, plus a
// synchronous Render(). The G-buffer keeps the reference layout (std::vector of vec4, row-major,
// y = 0 top, misses (0,0,0,1)), so the reference's GL path (main.cpp:306-310 PBO upload, SSAO)
// consumes it unchanged.
//
// vec3/vec4: when glm is included first (the reference app does, with GLM_FORCE_RADIANS), define
// SF_USE_GLM and the class uses glm::vec3 / glm::vec4 exactly like the reference. Otherwise a
// layout-identical POD is used. The library exports only members whose signatures and bodies do not depend on
// that choice (the Open / Close / SetViewFloats / Refresh members take float pointers); everything that names
// the vector types -- the constructor's resize, the destructor, SetView, GetGBuffer -- is inline here, so a
// glm application links against the same libsphereflake_hip.so and never has its vectors touched as another
// type (tests/test_integration_build.py links the patched reference main.cpp's object against the library).
//
// Differences, all deliberate:
//   - Rendering is an explicit full frame: Render() traces every pixel once, deterministically.
//     Initialize() keeps the reference's frame-less progressive mode (Sphereflake.cpp:67-74) on the
//     device: a host thread keeps launching batches of random 8-ray packets until destruction.
//   - GetGBuffer() downloads the device G-buffer (D2H) when it is stale, by DMA into the vectors'
//     storage, page-locked at construction (sf_host_register).
//   - Errors throw std::runtime_error carrying sf_strerror() (the reference had no error path). A failure
//     of the Initialize() loop stops the loop and is rethrown by the next GetGBuffer(), stats getter or
//     Deinitialize() (the destructor reports it on stderr instead of throwing).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <limits>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "sphereflake/sf.h"

namespace SphereflakeRaytracer {

#ifdef SF_USE_GLM
using sf_vec3 = glm::vec3;
using sf_vec4 = glm::vec4;
#else
struct sf_vec3 {
    float x, y, z;
    sf_vec3(float a = 0.f, float b = 0.f, float c = 0.f) : x(a), y(b), z(c) {}
};
struct sf_vec4 {
    float x, y, z, w;
    sf_vec4(float a = 0.f, float b = 0.f, float c = 0.f, float d = 0.f) : x(a), y(b), z(c), w(d) {}
};
#endif
static_assert(sizeof(sf_vec4) == 16, "vec4 must be 4 packed floats");

struct GBuffer {
    std::vector<sf_vec4> positions;
    std::vector<sf_vec4> normals;
};

// FIFO (ticket) lock: callers are served in arrival order. The frame-less loop re-locks right after each
// batch; with std::mutex (not fair) a caller's per-frame SetView / GetGBuffer could lose to it for many
// batches in a row. Here a waiting caller is always served before the loop's next batch.
class FairMutex {
public:
    void lock()
    {
        std::unique_lock<std::mutex> l(m_);
        const uint64_t t = next_++;
        cv_.wait(l, [&] { return serving_ == t; });
    }
    void unlock()
    {
        {
            std::lock_guard<std::mutex> l(m_);
            ++serving_;
        }
        cv_.notify_all();
    }

private:
    std::mutex m_;
    std::condition_variable cv_;
    uint64_t next_ = 0, serving_ = 0;
};

class Sphereflake {
public:
    // reference: m_GBuffer.positions/normals.resize(W*H) of zero vec4 (Sphereflake.cpp:43-55)
    Sphereflake(size_t width, size_t height, int device = 0) : m_Width(width), m_Height(height)
    {
        m_GBuffer.positions.resize(width * height);
        m_GBuffer.normals.resize(width * height);
        Open(device, &m_GBuffer.positions[0].x, &m_GBuffer.normals[0].x);
    }
    ~Sphereflake() { Close(); }
    Sphereflake(const Sphereflake&) = delete;
    Sphereflake& operator=(const Sphereflake&) = delete;

    // Frame-less progressive mode (reference Initialize(), Sphereflake.cpp:67-74): a host thread keeps
    // tracing batches of `batch` random packets of one worker stream. The reference seeds from time(NULL)
    // (Sphereflake.cpp:88-89); the overload takes an explicit seed (tests, reproducible runs).
    void Initialize();
    void Initialize(uint32_t seed, uint32_t batch = 1u << 18);
    // Stop the frame-less loop and join its thread (the reference does this only in its destructor,
    // Sphereflake.cpp:57-65). Rethrows the first error the loop met, if any.
    void Deinitialize();
    // Packets the frame-less loop has traced so far (= its next Sobol counter).
    uint64_t GetPacketsTraced() const;
    // The frame-less loop's packet counter when the last SetView took effect: batches from that counter on
    // trace the new view (the device loop picks a view up between batches; the reference's workers read
    // it mid-packet, unsynchronised, Sphereflake.cpp:76-84).
    uint64_t GetViewChangePacket() const;

    void SetView(const sf_vec3& origin, const sf_vec3& topLeft, const sf_vec3& topRight, const sf_vec3& bottomLeft)
    {
        const float o[3] = { origin.x, origin.y, origin.z }, tl[3] = { topLeft.x, topLeft.y, topLeft.z };
        const float tr[3] = { topRight.x, topRight.y, topRight.z }, bl[3] = { bottomLeft.x, bottomLeft.y, bottomLeft.z };
        SetViewFloats(o, tl, tr, bl);
    }
    void SetViewFloats(const float origin[3], const float topLeft[3], const float topRight[3], const float bottomLeft[3]);

    // One deterministic full frame into the device G-buffer (new; the reference renders implicitly).
    void Render(const sf_render_params* params = nullptr);

    // the device frame, downloaded into the vectors when it is newer than their contents (Refresh)
    const GBuffer& GetGBuffer() const
    {
        Refresh();
        return m_GBuffer;
    }
    // Headless dump of the device frame (sf_save_image): SF_DUMP_NORMALS / _POSITIONS_PFM / _NORMALS_PFM,
    // or SF_DUMP_IMAGE after an SSAO::Render(). The reference only shows its frame in the GL window.
    void SaveImage(const std::string& path, int what = SF_DUMP_NORMALS) const;

    int GetMaxDepthReached() const;
    void ResetMaxDepthReached();
    long long GetRaysPerSecond() const;   // rays traced since the last reset (reference semantics)
    void ResetRaysPerSecond();
    float GetClosestSphereDistance() const;
    void ResetClosestSphereDistance();

    sf_ctx* Context() const { return m_Ctx; }
    size_t Width() const { return m_Width; }
    size_t Height() const { return m_Height; }

private:
    void Open(int device, float* positions, float* normals);   // sf_create + page-lock the vectors' storage
    void Close() noexcept;                                       // join the frame-less loop, sf_destroy, unpin
    void Refresh() const;                                        // sf_download into m_Positions / m_Normals if stale
    static void Check(int rc);
    void ProgressiveLoop(uint32_t batch);
    void ThrowWorkerError() const;   // rethrows the frame-less loop's first error (held until reported once)

    size_t m_Width, m_Height;
    sf_ctx* m_Ctx = nullptr;
    mutable GBuffer m_GBuffer;
    float* m_Positions = nullptr;   // m_GBuffer's storage as the library sees it (W x H float4 each)
    float* m_Normals = nullptr;
    mutable bool m_Stale = true;
    bool m_Pinned = false;
    mutable FairMutex m_Mutex;
    std::thread m_Worker;
    std::atomic<bool> m_Deinitialize{ false };
    mutable std::atomic<int> m_WorkerError{ SF_OK };   // first failure of the frame-less loop
    uint64_t m_SobolCounter = 0;
    uint64_t m_ViewChange = 0;
    uint32_t m_Seed = 0;
};

}  // namespace SphereflakeRaytracer
