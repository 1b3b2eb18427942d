// sf_image.cpp -- headless image dump of a context's frame.
//
// The reference has no file output: its frame exists only as GL textures shown in the window
// (main.cpp:306-330, PBO upload of GetGBuffer()). A host without GL inspects a frame through these
// files instead: binary PPM (P6) for the composited RGBA8 image or a normal visualisation, and PFM
// (the float counterpart of PPM) for a lossless dump of the position / normal channels. Pure host
// code over the public C ABI (sf_download / sf_download_image), so it never touches device state.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "sphereflake/sf.h"

namespace {

struct File {
    FILE* f;
    explicit File(const char* path) : f(std::fopen(path, "wb")) {}
    ~File() { if (f) std::fclose(f); }
};

bool valid(const char* path, uint32_t w, uint32_t h, const void* p)
{
    return path && p && w && h && (uint64_t)w * h <= (1ull << 32);
}

}  // namespace

extern "C" {

int sf_write_ppm(const char* path, uint32_t w, uint32_t h, const uint8_t* rgba)
{
    if (!valid(path, w, h, rgba)) return SF_EINVAL;
    File out(path);
    if (!out.f) return SF_EINVAL;
    std::fprintf(out.f, "P6\n%u %u\n255\n", w, h);
    std::vector<uint8_t> row((size_t)w * 3);
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t* src = rgba + (size_t)y * w * 4;
        for (uint32_t x = 0; x < w; ++x) std::memcpy(&row[(size_t)x * 3], src + (size_t)x * 4, 3);
        if (std::fwrite(row.data(), 1, row.size(), out.f) != row.size()) return SF_ENOMEM;
    }
    return std::fflush(out.f) == 0 ? SF_OK : SF_ENOMEM;
}

// PFM stores rows bottom to top; the frame's top row (G-buffer row 0) therefore goes last.
int sf_write_pfm(const char* path, uint32_t w, uint32_t h, const float* v4)
{
    if (!valid(path, w, h, v4)) return SF_EINVAL;
    File out(path);
    if (!out.f) return SF_EINVAL;
    std::fprintf(out.f, "PF\n%u %u\n-1.0\n", w, h);   // negative scale: little-endian floats
    std::vector<float> row((size_t)w * 3);
    for (uint32_t r = 0; r < h; ++r) {
        const float* src = v4 + (size_t)(h - 1 - r) * w * 4;
        for (uint32_t x = 0; x < w; ++x) std::memcpy(&row[(size_t)x * 3], src + (size_t)x * 4, 12);
        if (std::fwrite(row.data(), 4, row.size(), out.f) != row.size()) return SF_ENOMEM;
    }
    return std::fflush(out.f) == 0 ? SF_OK : SF_ENOMEM;
}

int sf_save_image(sf_ctx* ctx, const char* path, int what)
{
    uint32_t w = 0, h = 0;
    if (!path || sf_get_size(ctx, &w, &h) != SF_OK) return SF_EINVAL;
    const size_t npx = (size_t)w * h;
    if (what == SF_DUMP_IMAGE) {
        std::vector<uint8_t> img(npx * 4);
        if (int rc = sf_download_image(ctx, img.data())) return rc;
        return sf_write_ppm(path, w, h, img.data());
    }
    if (what != SF_DUMP_NORMALS && what != SF_DUMP_POSITIONS_PFM && what != SF_DUMP_NORMALS_PFM) return SF_EINVAL;
    std::vector<float> v(npx * 4);
    const bool positions = what == SF_DUMP_POSITIONS_PFM;
    if (int rc = sf_download(ctx, positions ? v.data() : nullptr, positions ? nullptr : v.data(), nullptr, nullptr))
        return rc;
    if (what != SF_DUMP_NORMALS) return sf_write_pfm(path, w, h, v.data());
    // A miss is (0, 0, 0, 1) (Sphereflake.cpp:186-201); a hit's normal has |n| ~ 1, never 0.
    std::vector<uint8_t> img(npx * 4);
    for (size_t i = 0; i < npx; ++i) {
        const float* n = &v[i * 4];
        const bool miss = n[0] == 0.f && n[1] == 0.f && n[2] == 0.f;
        for (int k = 0; k < 3; ++k) {
            float c = miss ? 0.f : std::fmin(std::fmax(0.5f * n[k] + 0.5f, 0.f), 1.f);
            img[i * 4 + k] = (uint8_t)(c * 255.f + 0.5f);
        }
        img[i * 4 + 3] = 255;
    }
    return sf_write_ppm(path, w, h, img.data());
}

}  // extern "C"
