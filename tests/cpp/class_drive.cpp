// class_drive.cpp -- exercises the reference-compatible C++ class (Sphereflake.hpp) the way the
// reference app drives SphereflakeRaytracer::Sphereflake (main.cpp: construct, SetView each frame,
// GetGBuffer for the PBO upload, the stats getters for the overlay). Used by tests/test_gpu_class.py.
//
// usage: class_drive W H ox oy oz tlx tly tlz trx try trz blx bly blz out.bin [frames [image.bin]]
//   corners as C99 hex floats (bit-exact hand-over); writes positions then normals (W*H vec4 each)
//   of the last frame to out.bin and prints "max_depth rays closest(hex)" on stdout. With image.bin,
//   also runs the headless SSAO chain as main.cpp:312-330 does (radius from GetClosestSphereDistance,
//   camera = origin) and writes the RGBA8 image.
//
// usage: class_drive --initialize-moving W H views.bin out.bin seed batch ms period_us log.txt
//   the frame-less loop under a moving view (main.cpp:304 calls SetView every frame while the workers
//   trace): views.bin holds V views (12 float32 each: origin, TL, TR, BL); view 0 is set before
//   Initialize, then view j % V every period_us. Each SetView's latency is measured; log.txt gets one line
//   "view packet" per call (the loop's counter when it took effect). Latencies are taken once the loop has
//   traced 2 batches. Prints "packets max_depth rays calls max_latency_us elapsed_us batches_in_elapsed".
//
// usage: class_drive --initialize W H corners(12) out.bin seed batch ms
//   the frame-less mode as main.cpp:120-121 starts it: SetView, Initialize(seed, batch), let the loop run
//   `ms` milliseconds (reading GetGBuffer meanwhile, as the render loop does), Deinitialize; writes the
//   G-buffer and prints "packets max_depth rays" (the frame equals `packets / batch` sequential
//   sf_progressive(seed, k * batch, batch) calls, which the test checks).
#include <chrono>
#include <cstdio>
#include <string>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>
#include <vector>

#include "Sphereflake.hpp"
#include "SphereflakeSSAO.hpp"

using namespace SphereflakeRaytracer;

static int initialize_mode(int argc, char** argv)
{
    if (argc < 19) return 2;
    const size_t W = std::strtoul(argv[2], nullptr, 10), H = std::strtoul(argv[3], nullptr, 10);
    float v[12];
    for (int k = 0; k < 12; ++k) v[k] = std::strtof(argv[4 + k], nullptr);
    const uint32_t seed = (uint32_t)std::strtoul(argv[17], nullptr, 0);
    const uint32_t batch = (uint32_t)std::strtoul(argv[18], nullptr, 0);
    const int ms = argc > 19 ? std::atoi(argv[19]) : 200;
    Sphereflake flake(W, H);
    // --initialize-noview: no SetView, so the loop's first batch fails (SF_ENOVIEW); the error must
    // surface in this thread (GetGBuffer / Deinitialize throw), not vanish with the worker
    if (std::strcmp(argv[1], "--initialize-noview") != 0)
        flake.SetView(sf_vec3(v[0], v[1], v[2]), sf_vec3(v[3], v[4], v[5]), sf_vec3(v[6], v[7], v[8]),
                      sf_vec3(v[9], v[10], v[11]));
    flake.Initialize(seed, batch);
    const auto t0 = std::chrono::steady_clock::now();
    size_t reads = 0;
    while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(ms)) {
        const GBuffer& g = flake.GetGBuffer();   // the render loop's per-frame read (main.cpp:306-310)
        if (g.positions.size() != W * H) return 3;
        ++reads;
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    flake.Deinitialize();
    const uint64_t packets = flake.GetPacketsTraced();
    const GBuffer& g = flake.GetGBuffer();
    FILE* out = std::fopen(argv[16], "wb");
    if (!out) return 4;
    std::fwrite(g.positions.data(), sizeof(sf_vec4), g.positions.size(), out);
    std::fwrite(g.normals.data(), sizeof(sf_vec4), g.normals.size(), out);
    std::fclose(out);
    std::printf("%llu %d %lld %zu\n", (unsigned long long)packets, flake.GetMaxDepthReached(),
                flake.GetRaysPerSecond(), reads);
    return 0;
}

static int moving_mode(int argc, char** argv)
{
    if (argc < 11) return 2;
    const size_t W = std::strtoul(argv[2], nullptr, 10), H = std::strtoul(argv[3], nullptr, 10);
    std::vector<float> views;
    {
        FILE* f = std::fopen(argv[4], "rb");
        if (!f) return 4;
        float v[12];
        while (std::fread(v, sizeof v, 1, f) == 1) views.insert(views.end(), v, v + 12);
        std::fclose(f);
    }
    const size_t V = views.size() / 12;
    if (V == 0) return 2;
    const uint32_t seed = (uint32_t)std::strtoul(argv[6], nullptr, 0);
    const uint32_t batch = (uint32_t)std::strtoul(argv[7], nullptr, 0);
    const int ms = std::atoi(argv[8]);
    const int period_us = std::atoi(argv[9]);
    auto set_view = [&](Sphereflake& fl, size_t j) {
        const float* v = &views[12 * j];
        fl.SetView(sf_vec3(v[0], v[1], v[2]), sf_vec3(v[3], v[4], v[5]), sf_vec3(v[6], v[7], v[8]),
                   sf_vec3(v[9], v[10], v[11]));
    };
    Sphereflake flake(W, H);
    set_view(flake, 0);
    FILE* log = std::fopen(argv[10], "w");
    if (!log) return 4;
    std::fprintf(log, "0 0\n");
    flake.Initialize(seed, batch);
    // latencies are measured once the loop runs steadily: its first batches also allocate the frame-less
    // buffers and load the kernels (tens of ms)
    while (flake.GetPacketsTraced() < 2ull * batch) std::this_thread::sleep_for(std::chrono::microseconds(200));
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t p0 = flake.GetPacketsTraced();
    double max_lat = 0.0;
    size_t calls = 0;
    while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(ms)) {
        std::this_thread::sleep_for(std::chrono::microseconds(period_us));
        const size_t j = (calls + 1) % V;
        const auto c0 = std::chrono::steady_clock::now();
        set_view(flake, j);
        const double lat = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count();
        max_lat = lat > max_lat ? lat : max_lat;
        std::fprintf(log, "%zu %llu\n", j, (unsigned long long)flake.GetViewChangePacket());
        ++calls;
    }
    const uint64_t p1 = flake.GetPacketsTraced();
    const double elapsed = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    flake.Deinitialize();
    std::fclose(log);
    const uint64_t packets = flake.GetPacketsTraced();
    const GBuffer& g = flake.GetGBuffer();
    FILE* out = std::fopen(argv[5], "wb");
    if (!out) return 4;
    std::fwrite(g.positions.data(), sizeof(sf_vec4), g.positions.size(), out);
    std::fwrite(g.normals.data(), sizeof(sf_vec4), g.normals.size(), out);
    std::fclose(out);
    std::printf("%llu %d %lld %zu %.1f %.1f %llu\n", (unsigned long long)packets, flake.GetMaxDepthReached(),
                flake.GetRaysPerSecond(), calls, max_lat, elapsed, (unsigned long long)((p1 - p0) / batch));
    return 0;
}

int main(int argc, char** argv)
{
    if (argc > 1 && std::strcmp(argv[1], "--initialize-moving") == 0) {
        try {
            return moving_mode(argc, argv);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "%s\n", e.what());
            return 1;
        }
    }
    if (argc > 1 && std::strncmp(argv[1], "--initialize", 12) == 0) {
        try {
            return initialize_mode(argc, argv);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "%s\n", e.what());
            return 1;
        }
    }
    if (argc < 16) {
        std::fprintf(stderr, "usage: %s W H o.xyz tl.xyz tr.xyz bl.xyz out.bin [frames]\n", argv[0]);
        return 2;
    }
    try {
        const size_t W = std::strtoul(argv[1], nullptr, 10), H = std::strtoul(argv[2], nullptr, 10);
        float v[12];
        for (int k = 0; k < 12; ++k) v[k] = std::strtof(argv[3 + k], nullptr);
        const int frames = argc > 16 ? std::atoi(argv[16]) : 1;
        Sphereflake flake(W, H);
        long long rays = 0;
        for (int f = 0; f < frames; ++f) {
            flake.SetView(sf_vec3(v[0], v[1], v[2]), sf_vec3(v[3], v[4], v[5]), sf_vec3(v[6], v[7], v[8]),
                          sf_vec3(v[9], v[10], v[11]));
            flake.Render();
            const GBuffer& g = flake.GetGBuffer();   // the reference reads it right after (main.cpp:306-310)
            if (g.positions.size() != W * H || g.normals.size() != W * H) return 3;
        }
        rays = flake.GetRaysPerSecond();
        const GBuffer& g = flake.GetGBuffer();
        FILE* out = std::fopen(argv[15], "wb");
        if (!out) return 4;
        std::fwrite(g.positions.data(), sizeof(sf_vec4), g.positions.size(), out);
        std::fwrite(g.normals.data(), sizeof(sf_vec4), g.normals.size(), out);
        std::fclose(out);
        std::printf("%d %lld %a\n", flake.GetMaxDepthReached(), rays, flake.GetClosestSphereDistance());
        if (argc > 17) {
            Headless::SSAO ssao(flake, 1);
            ssao.SetSampleRadiusMultiplier(flake.GetClosestSphereDistance());
            ssao.SetCameraPosition(sf_vec3(v[0], v[1], v[2]));
            ssao.Render();
            const std::vector<uint8_t>& img = ssao.GetImage();
            FILE* f = std::fopen(argv[17], "wb");
            if (!f) return 4;
            std::fwrite(img.data(), 1, img.size(), f);
            std::fclose(f);
            if (argc > 18) {   // headless dumps (sf_save_image) under the prefix argv[18]
                const std::string pre = argv[18];
                ssao.SaveImage(pre + "_image.ppm");
                flake.SaveImage(pre + "_normals.ppm");
                flake.SaveImage(pre + "_pos.pfm", SF_DUMP_POSITIONS_PFM);
                flake.SaveImage(pre + "_nrm.pfm", SF_DUMP_NORMALS_PFM);
            }
        }
        flake.ResetRaysPerSecond();
        flake.ResetMaxDepthReached();
        flake.ResetClosestSphereDistance();
        std::printf("%d %lld %a\n", flake.GetMaxDepthReached(), flake.GetRaysPerSecond(),
                    flake.GetClosestSphereDistance());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
