// SphereflakeSSAO.hpp -- headless SSAO + final composite over a Sphereflake's device G-buffer.
//
// Kept out of Sphereflake.hpp on purpose: the reference app (main.cpp:71-72) includes both the renderer
// header and its own GL SSAO class (SSAO.h:6-50, SphereflakeRaytracer::SSAO). The drop-in header must not
// define a second SphereflakeRaytracer::SSAO, so the headless class lives in its own header and its own
// namespace, SphereflakeRaytracer::Headless (tests/test_integration_build.py compiles the patched main.cpp
// against Sphereflake.hpp to hold this).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "Sphereflake.hpp"

namespace SphereflakeRaytracer {
namespace Headless {

// Headless counterpart of the reference's SSAO class (SSAO.h:9-50, SSAO.cpp:49-175) plus the final
// composite pass of main.cpp:321-330, on the device G-buffer of a Sphereflake (sf_post_process).
// The GL texture handle of GetSSAOTexture() becomes the composited RGBA8 image, W*H*4 bytes,
// row j = G-buffer row j.
class SSAO {
public:
    SSAO(Sphereflake& flake, int downScale = 1);

    // SSAO.h:15-18. Until called, the radius is 8 x the closest-hit stat read on the device.
    void SetSampleRadiusMultiplier(float m) { m_Params.sample_radius = 8.0f * m; }
    // post_final.glsl cameraPosition (main.cpp:325); defaults to the SetView origin at Render time.
    void SetCameraPosition(const sf_vec3& p)
    {
        const float f[3] = { p.x, p.y, p.z };
        SetCameraPositionFloats(f);
    }
    void SetCameraPositionFloats(const float p[3]);   // (exported; the vec3 overload is inline, Sphereflake.hpp)

    void Render();                                  // SSAO, blur x, blur y, final (asynchronous)
    const std::vector<uint8_t>& GetImage() const;   // D2H of the last Render's image
    void SaveImage(const std::string& path) const;  // the last Render's image as a PPM

private:
    Sphereflake& m_Flake;
    sf_post_params m_Params;
    bool m_CameraSet = false;
    mutable std::vector<uint8_t> m_Image;
};

}  // namespace Headless
}  // namespace SphereflakeRaytracer
