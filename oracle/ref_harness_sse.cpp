// ref_harness_sse.cpp -- TEST INFRASTRUCTURE (oracle side, never shipped).
//
// The reference's SSE variant: the same unmodified sources as ref_harness.cpp,
// compiled with __ARCH_NO_AVX, which selects SIMD_SSE.h (4-lane packets, LOD constant 60,
// SIMD_SSE.h:21) and the 2x2 packet footprint of the frame-less worker (Sphereflake.cpp:115-138).
// The reference's own Linux build defines __ARCH_NO_AVX (CMakeLists.txt). Pinned IEEE flags as for
// the AVX harness (-O2, no FMA, no fast-math); -mavx only because SIMD_SSE.h uses _mm_cmp_ps.
// Nothing from the reference is copied; see oracle/Makefile. Output goes to oracle/_ref/ only.
//
// Modes
//   render W H K out.bin [T] [S]     -> per-ray (broadcast to the 4 lanes) frame, as ref_harness
//   progressive W H K seed P out.bin -> the SSE frame-less worker loop for P packets from mt19937(seed)
#include <functional>
#include <atomic>
#include <thread>
#include <random>
#include <memory>
#include <iostream>
#include <vector>
#include <limits>
#include <chrono>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <immintrin.h>

#ifndef __ARCH_NO_AVX
#define __ARCH_NO_AVX
#endif
#define private public
#include "/root/reference/sphereflake/Sphereflake.cpp"
#include "/root/reference/sphereflake/camera.h"
#include "/root/reference/sphereflake/Sobol.cpp"
#undef private

using namespace SphereflakeRaytracer;

static void hexf(float f) { std::printf("\"%a\"", (double)f); }

// Camera of main.cpp:92-96 with position scaled by K.
static Camera make_camera(size_t W, size_t H, float K)
{
    Camera cam(W, H);
    cam.SetPosition(vec3(-5.4098f, -7.2139f, 1.19006f) * K);
    cam.SetPitch(-1.371f);
    cam.SetYaw(0.921999f);
    cam.SetRoll(0.0f);
    return cam;
}

static void set_view(Sphereflake& sf, const Camera& cam)
{
    sf.SetView(cam.GetPosition(), cam.GetTopLeft(), cam.GetTopRight(), cam.GetBottomLeft());
}

struct RowResult { int maxDepth = 0; float closest = std::numeric_limits<float>::max(); long long hits = 0; };

// Per-ray render of rows [y0, y1): the ray generation of Sphereflake.cpp:149-167 (SSE branch) with
// the 4 lanes broadcast, traversal through the reference IntersectSphereflake (SSE build).
static void render_rows(Sphereflake* sf, size_t W, size_t H, size_t y0, size_t y1, float* out, RowResult* rr)
{
    auto width = _mm_set1_ps((float)W);
    auto height = _mm_set1_ps((float)H);
    float floatMax = std::numeric_limits<float>::max();
    for (size_t y = y0; y < y1; ++y) {
        for (size_t x = 0; x < W; ++x) {
            auto uvx = _mm_div_ps(_mm_set1_ps((float)x), width);
            auto uvy = _mm_div_ps(_mm_set1_ps((float)y), height);
            union { __m128 minT; float minTArray[4]; };
            minT = _mm_set1_ps(floatMax);
            auto directionHorizontalPart = sf->m_TopLeft + (sf->m_TopRight - sf->m_TopLeft) * uvx;
            auto directionVerticalPart = (sf->m_BottomLeft - sf->m_TopLeft) * uvy;
            auto targetDirection = directionHorizontalPart + directionVerticalPart;
            auto rayDirection = targetDirection - sf->m_RayOrigin;
            SIMD::Normalize(rayDirection);
            SIMD::Vec3Packet position, normal;
            position.Set(vec3(0.0f));
            normal.Set(vec3(0.0f));
            auto transform = sf->m_RootTransform;
            sf->IntersectSphereflake(rayDirection, transform, minT, position, normal, 3.0f, 0);
            vec3 p = position.Extract(0), n = normal.Extract(0);
            float* o = out + 7 * (y * W + x);
            o[0] = p.x; o[1] = p.y; o[2] = p.z; o[3] = n.x; o[4] = n.y; o[5] = n.z; o[6] = minTArray[0];
            if (minTArray[0] < rr->closest) rr->closest = minTArray[0];
            if (minTArray[0] != floatMax) rr->hits++;
        }
    }
    rr->maxDepth = sf->m_MaxDepthReached;
}

static int mode_render(size_t W, size_t H, float K, const char* path, unsigned threads, size_t step)
{
    Camera cam = make_camera(W, H, K);
    size_t nrows = (H + step - 1) / step;
    std::vector<float> out(7 * W * nrows);
    std::vector<std::unique_ptr<Sphereflake>> sfs;
    std::vector<RowResult> rr(threads);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < threads; ++t) {
        sfs.emplace_back(new Sphereflake(1, 1));   // one object per thread (m_MaxDepthReached is racy)
        set_view(*sfs.back(), cam);
    }
    std::atomic<size_t> next(0);
    for (unsigned t = 0; t < threads; ++t) {
        th.emplace_back([&, t]() {
            RowResult acc;
            for (;;) {
                size_t k = next.fetch_add(1);
                if (k >= nrows) break;
                size_t y = k * step;
                RowResult r;
                render_rows(sfs[t].get(), W, H, y, y + 1, out.data() + 7 * W * k - 7 * W * y, &r);
                acc.hits += r.hits;
                acc.closest = std::min(acc.closest, r.closest);
            }
            acc.maxDepth = sfs[t]->m_MaxDepthReached;
            rr[t] = acc;
        });
    }
    for (auto& t : th) t.join();
    RowResult tot;
    for (auto& r : rr) { tot.maxDepth = std::max(tot.maxDepth, r.maxDepth); tot.closest = std::min(tot.closest, r.closest); tot.hits += r.hits; }
    FILE* f = std::fopen(path, "wb");
    if (!f) { std::perror("fopen"); return 1; }
    std::fwrite(out.data(), sizeof(float), out.size(), f);
    std::fclose(f);
    std::printf("{\"max_depth\": %d, \"closest\": ", tot.maxDepth); hexf(tot.closest);
    std::printf(", \"hits\": %lld, \"rays\": %zu, \"row_step\": %zu}\n", tot.hits, W * nrows, step);
    return 0;
}

// Body of Sphereflake::DoImagePart (Sphereflake.cpp:86-214, SSE branch) for a fixed packet count, with
// the time(NULL) seed replaced by `seed` and the spin-up sleep / exit flag dropped.
static int mode_progressive(size_t W, size_t H, float K, unsigned seed, unsigned long long packets, const char* path)
{
    Camera cam = make_camera(W, H, K);
    Sphereflake sf(W, H);
    set_view(sf, cam);
    std::mt19937 mt;
    mt.seed((unsigned long)seed);
    std::uniform_int_distribution<unsigned int> rnd(0);
    auto width = _mm_set1_ps((float)sf.m_Width);
    auto height = _mm_set1_ps((float)sf.m_Height);
    SIMD::Vec3Packet position;
    SIMD::Vec3Packet normal;
    float floatMax = std::numeric_limits<float>::max();
    unsigned long long sobolCounter = 0;
    for (unsigned long long p = 0; p < packets; ++p) {
        auto x0 = floorf(Sobol::Sample(sobolCounter, 0, rnd(mt)) * (sf.m_Width - 1));
        auto y0 = floorf(Sobol::Sample(sobolCounter, 1, rnd(mt)) * (sf.m_Height - 1));
        sobolCounter++;
        float xa[4] = { x0, x0 + 1, x0, x0 + 1 };
        float ya[4] = { y0, y0, y0 + 1, y0 + 1 };
        auto x = _mm_set_ps(xa[3], xa[2], xa[1], xa[0]);
        auto y = _mm_set_ps(ya[3], ya[2], ya[1], ya[0]);
        auto uvx = _mm_div_ps(x, width);
        auto uvy = _mm_div_ps(y, height);
        union { __m128 minT; float minTArray[4]; };
        minT = _mm_set1_ps(floatMax);
        auto directionHorizontalPart = sf.m_TopLeft + (sf.m_TopRight - sf.m_TopLeft) * uvx;
        auto directionVerticalPart = (sf.m_BottomLeft - sf.m_TopLeft) * uvy;
        auto targetDirection = directionHorizontalPart + directionVerticalPart;
        auto rayDirection = targetDirection - sf.m_RayOrigin;
        SIMD::Normalize(rayDirection);
        position.Set(vec3(0.0f));
        normal.Set(vec3(0.0f));
        auto transform = sf.m_RootTransform;
        sf.IntersectSphereflake(rayDirection, transform, minT, position, normal, 3.0f, 0);
        sf.m_RaysPerSecond += 4;
        for (auto q = 0u; q < 4; q++) {
            auto idx = (size_t)xa[q] + (size_t)ya[q] * sf.m_Width;
            if (idx >= sf.m_GBuffer.positions.size()) continue;   // the reference's `idx > size` would write OOB at ==
            sf.m_GBuffer.positions[idx] = vec4(position.Extract(q), 1.0f);
            sf.m_GBuffer.normals[idx] = vec4(normal.Extract(q), 1.0f);
            if (minTArray[q] < sf.m_ClosestSphereDistance) sf.m_ClosestSphereDistance = minTArray[q];
        }
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) { std::perror("fopen"); return 1; }
    std::fwrite(&sf.m_GBuffer.positions[0].x, sizeof(float), 4 * W * H, f);
    std::fwrite(&sf.m_GBuffer.normals[0].x, sizeof(float), 4 * W * H, f);
    std::fclose(f);
    std::printf("{\"max_depth\": %d, \"closest\": ", sf.m_MaxDepthReached); hexf(sf.m_ClosestSphereDistance);
    std::printf(", \"rays\": %lld}\n", sf.m_RaysPerSecond);
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    std::string mode = argv[1];
    if (mode == "render" && argc >= 6)
        return mode_render(std::strtoul(argv[2], 0, 10), std::strtoul(argv[3], 0, 10), std::strtof(argv[4], 0), argv[5],
                           argc >= 7 ? (unsigned)std::strtoul(argv[6], 0, 10) : std::max(1u, std::thread::hardware_concurrency()),
                           argc >= 8 ? std::max<size_t>(1, std::strtoul(argv[7], 0, 10)) : 1);
    if (mode == "progressive" && argc >= 8)
        return mode_progressive(std::strtoul(argv[2], 0, 10), std::strtoul(argv[3], 0, 10), std::strtof(argv[4], 0),
                                (unsigned)std::strtoul(argv[5], 0, 10), std::strtoull(argv[6], 0, 10), argv[7]);
    std::fprintf(stderr, "usage: ref_harness_sse render|progressive ...\n");
    return 2;
}
