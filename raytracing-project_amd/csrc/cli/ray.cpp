// ray.cpp — drop-in CLI: ray <scene.json> <output.png> [--paper] [options]
//
// Mirrors raytracer/src/main.cpp:42-94: same usage text, same argv handling
// (paper mode iff argv[3] == "--paper"), same exit codes
// (1 usage, 2 load returned false, 3 exception while loading, 4 PNG write
// failure) and the same final "Wrote <out> (WxH)[ (paper mode)]" line.
// The frame is rendered, converted with toByte and packed on the GPU(s)
// (rt_render_rgb8): 3 bytes per pixel reach the host,
// then the PNG is deflated in parallel bands (rt_write_png).
// Extra options may follow argv[3] (the reference ignores them):
//   --gpus N       render on N GPUs of this node (row strips + RCCL gather); 0 = all
//   --stats        print one JSON line with ray counts and the wall-clock split
//   --threads N    deflate threads for the PNG writer (default 8)
//   --fp32         NON-PARITY FP32 fast path (RT_FLAG_FP32)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "rt.h"
#include "tracer.hpp"

int main(int argc, char** argv) {
    const auto t_start = std::chrono::steady_clock::now();
    if (argc < 3) {
        std::cerr << "Usage: " << argv[0] << " <scene.json> <output.png> [--paper]\n";
        std::cerr << "  --paper: Enable paper rendering mode with crosshatching\n";
        return 1;
    }
    const std::string json_path = argv[1];
    const std::string out_path = argv[2];
    bool paper_mode = false;
    if (argc > 3 && std::string(argv[3]) == "--paper") paper_mode = true;
    bool print_stats = false;
    int png_threads = 8;
    int n_gpus = 1;
    bool fp32 = false;
    for (int i = 3; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--stats")) print_stats = true;
        else if (!std::strcmp(argv[i], "--fp32")) fp32 = true;
        else if (!std::strcmp(argv[i], "--threads") && i + 1 < argc) png_threads = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--gpus") && i + 1 < argc) n_gpus = std::atoi(argv[++i]);
    }

    // one-time host preparation (the jitter tree's tap lists, ~3 ms) on a
    // helper thread while this one loads the scene and initialises HIP
    std::thread warm_host([] { (void)rt_warmup(RT_WARM_HOST); });
    struct Joiner {
        std::thread& t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } join_host{warm_host};
    rtamd::Scene scene;
    rtamd::Camera cam;
    try {
        if (!rtamd::jsonio::load_scene_from_json(json_path, scene, cam)) {
            std::cerr << "Failed to load scene from " << json_path << "\n";
            return 2;
        }
    } catch (const std::exception& e) {
        std::cerr << "[error] " << e.what() << "\n";
        return 3;
    }
    const auto t_loaded = std::chrono::steady_clock::now();

    const int W = cam.nx();
    const int H = cam.ny();
    rtamd::Tracer tracer;
    tracer.scene = &scene;
    tracer.camera = &cam;
    tracer.width = W;
    tracer.height = H;
    tracer.mode = paper_mode ? rtamd::RenderMode::Paper : rtamd::RenderMode::Standard;
    tracer.n_gpus = n_gpus;
    if (fp32) tracer.flags |= RT_FLAG_FP32;

    // device resources (workspaces, RCCL communicators of --gpus N) are
    // released before exit on every path from here on
    struct DeviceTeardown {
        bool done = false;
        ~DeviceTeardown() {
            if (!done) (void)rt_shutdown();
        }
    } teardown;
    // the output bytes are written by the device path into this buffer; its
    // pages are touched here, on a helper thread, while the main thread
    // initialises HIP (page faults of a fresh 25 MB buffer otherwise land on
    // the D2H copy).  Page-locking it as well (rt_host_register) was measured
    // and rejected: registering 25 MB took 47-54 ms and slowed the concurrent
    // scene upload and jitter table; the first pageable D2H costs ~8 ms.
    std::vector<uint8_t> rgb;
    std::thread prefault([&rgb, W, H] { rgb.assign((size_t)W * H * 3, 0); });
    // HIP runtime initialisation (the first HIP call of the process), timed on its own for --stats
    const auto t_hip0 = std::chrono::steady_clock::now();
    (void)rt_device_count();
    const auto t_hip1 = std::chrono::steady_clock::now();
    // the render kernels' code object (~5 ms) loads on a helper thread while
    // this one compiles and uploads the scene and builds the jitter table
    // (RAY_WARM_DEVICE=0: not at all, for measurement)
    const char* wd = std::getenv("RAY_WARM_DEVICE");
    std::thread warm_dev;
    if (!(wd && *wd == '0')) warm_dev = std::thread([] { (void)rt_warmup(RT_WARM_DEVICE); });
    Joiner join_dev{warm_dev};
    if (paper_mode) std::cout << "Rendering in paper mode (" << W << "x" << H << ")\n";
    else std::cout << "Rendering with 8 spp (" << W << "x" << H << ")\n";
    const auto t0 = std::chrono::steady_clock::now();
    prefault.join();
    const auto t_joined = std::chrono::steady_clock::now();
    try {
        tracer.render_rgb8(rgb);
    } catch (const std::exception& e) {
        std::cerr << "[error] " << e.what() << "\n";
        return 5;
    }
    const auto t1 = std::chrono::steady_clock::now();
    std::cout << "Rendering complete!\n";

    if (rt_write_png(out_path.c_str(), rgb.data(), W, H, png_threads) != RT_OK) {
        std::cerr << "Failed to write PNG: " << out_path << "\n";
        return 4;
    }
    const auto t2 = std::chrono::steady_clock::now();
    if (warm_host.joinable()) warm_host.join();
    if (warm_dev.joinable()) warm_dev.join();
    teardown.done = true;
    // With one GPU the library holds no communicators: its device memory is
    // the process's and goes with it at the _Exit below.  Several GPUs:
    // destroy the RCCL communicators first.
    if (n_gpus != 1) (void)rt_shutdown();
    const auto t3 = std::chrono::steady_clock::now();
    std::string mode_str = paper_mode ? " (paper mode)" : "";
    std::cout << "Wrote " << out_path << " (" << W << "x" << H << ")" << mode_str << "\n";
    if (print_stats) {
        const rt_stats& s = tracer.stats;
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        const double ms_render = ms(t0, t1);
        const double rays = (double)(s.rays_intersect + s.rays_occluded);
        double setup[12] = {};
        (void)rt_setup_times(setup, 12);
        // ms_render's host split, in order: output-buffer prefault join,
        // rt_render_rgb8's group setup, rt_frame_begin (scene compile + upload,
        // jitter checkpoint table, jitter launch), the trace launches,
        // rt_frame_end (waits for the device), the D2H copy
        std::printf(
            "{\"ms_hip_init\": %.3f, \"ms_setup_scene\": %.3f, \"ms_setup_jtable\": %.3f, "
            "\"ms_setup_trace_load\": %.3f, \"ms_setup_jitter_load\": %.3f, \"ms_setup_alloc\": %.3f, "
            "\"ms_setup_pinned\": %.3f, \"ms_setup_streams\": %.3f, \"ms_prefault_join\": %.3f, "
            "\"ms_group\": %.3f, \"ms_frame_begin\": %.3f, \"ms_frame_trace\": %.3f, \"ms_frame_end\": %.3f, "
            "\"ms_setup_copy_engine\": %.3f, \"ms_shutdown\": %.3f}\n",
            ms(t_hip0, t_hip1), setup[0], setup[1], setup[2], setup[3], setup[4], setup[5], setup[6],
            ms(t0, t_joined), setup[10], setup[7], setup[8], setup[9], setup[11], ms(t2, t3));
        std::printf(
            "{\"rays_intersect\": %llu, \"rays_occluded\": %llu, \"rays_traced\": %llu, \"n_gpus\": %d, "
            "\"ms_load\": %.3f, \"ms_rng\": %.3f, \"ms_kernel\": %.3f, \"ms_gather\": %.3f, \"ms_tobyte\": %.3f, "
            "\"ms_d2h\": %.3f, \"ms_render\": %.3f, \"ms_png\": %.3f, \"ms_main\": %.3f, \"mrays_per_s\": %.3f}\n",
            (unsigned long long)s.rays_intersect, (unsigned long long)s.rays_occluded,
            (unsigned long long)s.rays_traced, s.n_gpus, ms(t_start, t_loaded), s.ms_rng, s.ms_kernel, s.ms_gather,
            s.ms_tobyte, s.ms_d2h, ms_render, ms(t1, t2), ms(t_start, t2), rays / (ms_render * 1e3));
    }
    // The PNG is closed, the device work is complete and rt_shutdown has
    // released the library's device resources (workspaces, RCCL
    // communicators); what is left at exit is the HIP runtime's own teardown
    // of its static state (~40 ms), which the process does not need: leave
    // without the static destructors, as the kernel driver reclaims the rest.
    // (RT_CLI_NORMAL_EXIT=1: a normal return, for tools that finish their
    // work in the process's exit handlers, e.g. rocprofv3's trace flush)
    std::cout.flush();
    std::fflush(nullptr);
    if (const char* e = std::getenv("RT_CLI_NORMAL_EXIT"); e && *e == '1') return 0;
    std::_Exit(0);
}
