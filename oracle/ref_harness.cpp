// ref_harness.cpp -- TEST INFRASTRUCTURE (oracle side, never shipped).
//
// Compiles the UNMODIFIED reference hot path where it lies under
// /root/reference (sphereflake/Sphereflake.cpp, Sphereflake.h, SIMD_AVX.h,
// Util.h, camera.h, Sobol.cpp) into a headless driver with pinned IEEE flags
// (-O2 -mavx, no FMA, no fast-math: SURVEY.md §8(c)). Nothing from the
// reference is copied into this repository; see oracle/Makefile for the recipe.
// Output goes to oracle/_ref/ only.
//
// Modes
//   setup  W H K              -> JSON: child transforms (Sphereflake.cpp:216-249),
//                                root transform (Sphereflake.cpp:76-84), camera
//                                corners (camera.h:37-53), radius chain
//   render W H K out.bin [T] [S] -> per-ray (broadcast) frame: for every pixel of
//                                rows y % S == 0 (S = 1 default), pos.xyz nrm.xyz minT
//                                as 7 float32; JSON stats (over those rows) on stdout
//   bench  W H K threads reps -> the reference's own AVX packet path timed as a
//                                deterministic full-frame packet tiling (8-lane
//                                footprint of Sphereflake.cpp:139-147), JSON on stdout
//   progressive W H K seed P out.bin -> the reference's frame-less worker loop (Sphereflake.cpp:86-214)
//                                run for P packets from mt19937(seed), single thread, on a fresh
//                                (zeroed) G-buffer; writes positions+normals (W*H*8 float32), JSON stats
//   sobol                     -> JSON: Sobol dims 0/1 direction numbers + Sample() KATs
//   mt     seed n             -> JSON: libstdc++ mt19937 + uniform_int_distribution<unsigned>(0)
//
// Per-ray semantics: the single ray is broadcast to all 8 lanes, so the packet
// early-outs (Sphereflake.h:140-153, 207-211) act per ray. This is the canonical
// definition the HIP kernels reproduce bit-for-bit.
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

#define private public
#include "/root/reference/sphereflake/Sphereflake.cpp"
#include "/root/reference/sphereflake/camera.h"
#include "/root/reference/sphereflake/Sobol.cpp"
#undef private

using namespace SphereflakeRaytracer;

static void hexf(float f) { std::printf("\"%a\"", (double)f); }

static void hexv(const float* v, int n)
{
    std::printf("[");
    for (int i = 0; i < n; ++i) { if (i) std::printf(", "); hexf(v[i]); }
    std::printf("]");
}

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

static int mode_setup(size_t W, size_t H, float K)
{
    Sphereflake sf(W, H);
    Camera cam = make_camera(W, H, K);
    set_view(sf, cam);
    vec3 o = cam.GetPosition(), tl = cam.GetTopLeft(), tr = cam.GetTopRight(), bl = cam.GetBottomLeft();
    std::printf("{\"W\": %zu, \"H\": %zu, \"K\": ", W, H); hexf(K);
    std::printf(",\n \"children\": [");
    for (int i = 0; i < 9; ++i) {
        if (i) std::printf(",\n   ");
        hexv(&sf.m_ChildTransforms[i].m[0][0], 16);
    }
    std::printf("],\n \"root\": "); hexv(&sf.m_RootTransform.m[0][0], 16);
    std::printf(",\n \"origin\": "); hexv(&o.x, 3);
    std::printf(", \"tl\": "); hexv(&tl.x, 3);
    std::printf(", \"tr\": "); hexv(&tr.x, 3);
    std::printf(", \"bl\": "); hexv(&bl.x, 3);
    std::printf(",\n \"radius\": [");
    float p = 3.0f;
    for (int d = 0; d < 16; ++d) { float r = p / 3.0f; if (d) std::printf(", "); hexf(r); p = r; }
    std::printf("]}\n");
    return 0;
}

struct RowResult { int maxDepth = 0; float closest = std::numeric_limits<float>::max(); long long hits = 0; };

// Per-ray render of rows [y0, y1): ray generation exactly as Sphereflake.cpp:149-167
// with the 8 lanes broadcast, traversal through the reference IntersectSphereflake.
static void render_rows(Sphereflake* sf, size_t W, size_t H, size_t y0, size_t y1, float* out, RowResult* rr)
{
    auto width = _mm256_set1_ps((float)W);
    auto height = _mm256_set1_ps((float)H);
    float floatMax = std::numeric_limits<float>::max();
    for (size_t y = y0; y < y1; ++y) {
        for (size_t x = 0; x < W; ++x) {
            auto xv = _mm256_set1_ps((float)x);
            auto yv = _mm256_set1_ps((float)y);
            auto uvx = _mm256_div_ps(xv, width);
            auto uvy = _mm256_div_ps(yv, height);
            union { __m256 minT; float minTArray[8]; };
            minT = _mm256_broadcast_ss(&floatMax);
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
        sfs.emplace_back(new Sphereflake(1, 1));   // G-buffer unused here; one object per thread (m_MaxDepthReached is racy)
        set_view(*sfs.back(), cam);
    }
    // interleaved row blocks for balance
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

// The reference packet loop (Sphereflake.cpp:139-201, AVX branch) with the random
// Sobol draw replaced by a deterministic stride-3 tiling of packet centres, so a
// frame is covered once (8/9 of the pixels: (x0-1, y0+1) is never in a packet).
static long long bench_packets(Sphereflake* sf, size_t W, size_t H, size_t row0, size_t row1)
{
    auto width = _mm256_set1_ps((float)sf->m_Width);
    auto height = _mm256_set1_ps((float)sf->m_Height);
    SIMD::Vec3Packet position, normal;
    float floatMax = std::numeric_limits<float>::max();
    long long rays = 0;
    for (size_t cy = row0; cy < row1; ++cy) {
        float y0 = (float)(1 + 3 * cy);
        for (size_t cx = 0; 1 + 3 * cx < W - 1; ++cx) {
            float x0 = (float)(1 + 3 * cx);
            float xa[8] = { x0, x0 + 1, x0 + 1, x0, x0, x0 + 1, x0 - 1, x0 - 1 };
            float ya[8] = { y0, y0 + 1, y0, y0 + 1, y0 - 1, y0 - 1, y0, y0 - 1 };
            auto x = _mm256_set_ps(xa[7], xa[6], xa[5], xa[4], xa[3], xa[2], xa[1], xa[0]);
            auto y = _mm256_set_ps(ya[7], ya[6], ya[5], ya[4], ya[3], ya[2], ya[1], ya[0]);
            auto uvx = _mm256_div_ps(x, width);
            auto uvy = _mm256_div_ps(y, height);
            union { __m256 minT; float minTArray[8]; };
            minT = _mm256_broadcast_ss(&floatMax);
            auto directionHorizontalPart = sf->m_TopLeft + (sf->m_TopRight - sf->m_TopLeft) * uvx;
            auto directionVerticalPart = (sf->m_BottomLeft - sf->m_TopLeft) * uvy;
            auto targetDirection = directionHorizontalPart + directionVerticalPart;
            auto rayDirection = targetDirection - sf->m_RayOrigin;
            SIMD::Normalize(rayDirection);
            position.Set(vec3(0.0f));
            normal.Set(vec3(0.0f));
            auto transform = sf->m_RootTransform;
            sf->IntersectSphereflake(rayDirection, transform, minT, position, normal, 3.0f, 0);
            rays += 8;
            for (auto q = 0u; q < 8; q++) {
                auto idx = (size_t)xa[q] + (size_t)ya[q] * sf->m_Width;
                if (idx > sf->m_GBuffer.positions.size()) continue;
                sf->m_GBuffer.positions[idx] = vec4(position.Extract(q), 1.0f);
                sf->m_GBuffer.normals[idx] = vec4(normal.Extract(q), 1.0f);
                if (minTArray[q] < sf->m_ClosestSphereDistance) sf->m_ClosestSphereDistance = minTArray[q];
            }
        }
    }
    return rays;
}

static int mode_bench(size_t W, size_t H, float K, unsigned threads, unsigned reps)
{
    Camera cam = make_camera(W, H, K);
    Sphereflake sf(W, H);   // shared G-buffer, as in the reference (threads write disjoint packets here)
    set_view(sf, cam);
    size_t packetRows = 0;
    while (1 + 3 * packetRows < H - 1) ++packetRows;
    std::vector<double> secs;
    long long raysPerFrame = 0;
    for (unsigned rep = 0; rep < reps; ++rep) {
        std::atomic<size_t> next(0);
        std::atomic<long long> rays(0);
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (unsigned t = 0; t < threads; ++t) {
            th.emplace_back([&]() {
                long long local = 0;
                for (;;) {
                    size_t r0 = next.fetch_add(2);
                    if (r0 >= packetRows) break;
                    local += bench_packets(&sf, W, H, r0, std::min(packetRows, r0 + 2));
                }
                rays += local;
            });
        }
        for (auto& t : th) t.join();
        auto t1 = std::chrono::steady_clock::now();
        secs.push_back(std::chrono::duration<double>(t1 - t0).count());
        raysPerFrame = rays.load();
    }
    std::vector<double> s = secs;
    std::sort(s.begin(), s.end());
    double med = s[s.size() / 2];
    std::printf("{\"W\": %zu, \"H\": %zu, \"K\": %g, \"threads\": %u, \"reps\": %u, \"rays_per_frame\": %lld, "
                "\"median_s\": %.6f, \"best_s\": %.6f, \"mrays_per_s\": %.4f, \"max_depth\": %d}\n",
                W, H, (double)K, threads, reps, raysPerFrame, med, s[0], raysPerFrame / med / 1e6,
                sf.m_MaxDepthReached);
    return 0;
}

// Body of Sphereflake::DoImagePart (Sphereflake.cpp:86-201, AVX branch) for a fixed packet count,
// with the time(NULL) seed replaced by `seed` and the spin-up sleep / exit flag dropped.
static int mode_progressive(size_t W, size_t H, float K, unsigned seed, unsigned long long packets, const char* path)
{
    Camera cam = make_camera(W, H, K);
    Sphereflake sf(W, H);
    set_view(sf, cam);
    std::mt19937 mt;
    mt.seed((unsigned long)seed);
    std::uniform_int_distribution<unsigned int> rnd(0);
    auto width = _mm256_set1_ps((float)sf.m_Width);
    auto height = _mm256_set1_ps((float)sf.m_Height);
    SIMD::Vec3Packet position;
    SIMD::Vec3Packet normal;
    float floatMax = std::numeric_limits<float>::max();
    unsigned long long sobolCounter = 0;
    for (unsigned long long p = 0; p < packets; ++p) {
        auto x0 = 1 + floorf(Sobol::Sample(sobolCounter, 0, rnd(mt)) * (sf.m_Width - 2));
        auto y0 = 1 + floorf(Sobol::Sample(sobolCounter, 1, rnd(mt)) * (sf.m_Height - 2));
        sobolCounter++;
        float xa[8] = { x0, x0 + 1, x0 + 1, x0, x0, x0 + 1, x0 - 1, x0 - 1 };
        float ya[8] = { y0, y0 + 1, y0, y0 + 1, y0 - 1, y0 - 1, y0, y0 - 1 };
        auto x = _mm256_set_ps(xa[7], xa[6], xa[5], xa[4], xa[3], xa[2], xa[1], xa[0]);
        auto y = _mm256_set_ps(ya[7], ya[6], ya[5], ya[4], ya[3], ya[2], ya[1], ya[0]);
        auto uvx = _mm256_div_ps(x, width);
        auto uvy = _mm256_div_ps(y, height);
        union { __m256 minT; float minTArray[8]; };
        minT = _mm256_broadcast_ss(&floatMax);
        auto directionHorizontalPart = sf.m_TopLeft + (sf.m_TopRight - sf.m_TopLeft) * uvx;
        auto directionVerticalPart = (sf.m_BottomLeft - sf.m_TopLeft) * uvy;
        auto targetDirection = directionHorizontalPart + directionVerticalPart;
        auto rayDirection = targetDirection - sf.m_RayOrigin;
        SIMD::Normalize(rayDirection);
        position.Set(vec3(0.0f));
        normal.Set(vec3(0.0f));
        auto transform = sf.m_RootTransform;
        sf.IntersectSphereflake(rayDirection, transform, minT, position, normal, 3.0f, 0);
        sf.m_RaysPerSecond += 8;
        for (auto q = 0u; q < 8; q++) {
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

static int mode_sobol()
{
    std::printf("{\"dim0\": [");
    for (int k = 0; k < 52; ++k) std::printf("%s%u", k ? ", " : "", Sobol::Matrices::matrices[k]);
    std::printf("],\n \"dim1\": [");
    for (int k = 0; k < 52; ++k) std::printf("%s%u", k ? ", " : "", Sobol::Matrices::matrices[52 + k]);
    std::printf("],\n \"samples\": [");
    std::mt19937 mt(777);
    std::uniform_int_distribution<unsigned int> rnd(0);
    bool first = true;
    unsigned long long idxs[] = { 0ull, 1ull, 2ull, 3ull, 7ull, 100ull, 12345ull, 65535ull, 1000003ull,
                                  0xffffffffull, 0x100000000ull, 0x123456789abcull, ~0ull };
    for (unsigned long long idx : idxs) {
        for (unsigned dim = 0; dim < 2; ++dim) {
            for (int s = 0; s < 3; ++s) {
                unsigned scr = s == 0 ? 0u : rnd(mt);
                float v = Sobol::Sample(idx, dim, scr);
                std::printf("%s\n  [%llu, %u, %u, ", first ? "" : ",", idx, dim, scr);
                hexf(v);
                std::printf("]");
                first = false;
            }
        }
    }
    std::printf("]}\n");
    return 0;
}

static int mode_mt(unsigned seed, unsigned n)
{
    std::mt19937 mt;
    mt.seed((unsigned long)seed);
    std::uniform_int_distribution<unsigned int> rnd(0);
    std::printf("{\"seed\": %u, \"draws\": [", seed);
    for (unsigned i = 0; i < n; ++i) std::printf("%s%u", i ? ", " : "", rnd(mt));
    std::printf("]}\n");
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: ref_harness setup|render|bench|sobol|mt ...\n"); return 2; }
    std::string mode = argv[1];
    if (mode == "setup" && argc >= 5) return mode_setup(std::strtoul(argv[2], 0, 10), std::strtoul(argv[3], 0, 10), std::strtof(argv[4], 0));
    if (mode == "render" && argc >= 6)
        return mode_render(std::strtoul(argv[2], 0, 10), std::strtoul(argv[3], 0, 10), std::strtof(argv[4], 0), argv[5],
                           argc >= 7 ? (unsigned)std::strtoul(argv[6], 0, 10) : std::max(1u, std::thread::hardware_concurrency()),
                           argc >= 8 ? std::max<size_t>(1, std::strtoul(argv[7], 0, 10)) : 1);
    if (mode == "bench" && argc >= 7)
        return mode_bench(std::strtoul(argv[2], 0, 10), std::strtoul(argv[3], 0, 10), std::strtof(argv[4], 0),
                          (unsigned)std::strtoul(argv[5], 0, 10), (unsigned)std::strtoul(argv[6], 0, 10));
    if (mode == "progressive" && argc >= 8)
        return mode_progressive(std::strtoul(argv[2], 0, 10), std::strtoul(argv[3], 0, 10), std::strtof(argv[4], 0),
                                (unsigned)std::strtoul(argv[5], 0, 10), std::strtoull(argv[6], 0, 10), argv[7]);
    if (mode == "sobol") return mode_sobol();
    if (mode == "mt" && argc >= 4) return mode_mt((unsigned)std::strtoul(argv[2], 0, 10), (unsigned)std::strtoul(argv[3], 0, 10));
    std::fprintf(stderr, "bad arguments\n");
    return 2;
}
