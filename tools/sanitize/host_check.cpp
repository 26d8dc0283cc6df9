// host_check.cpp — AddressSanitizer / UBSan driver for the host C/C++ code
// (sanitizers run on the host restatement, never on the GPU).
//
// Built by tools/sanitize/Makefile from the SOURCES of librt_host (JSON
// parser, schema loader, IR, PNG writer), the device-table compiler
// (scene_compile.cpp) and the C oracle, all with
// -fsanitize=address,undefined; tests/test_sanitize.py runs it over the
// example, torture and deep scenes plus malformed JSON.  Per scene: load,
// compile the device object table, render a band of rows on the oracle in
// both modes, toByte, PNG.  Exit 0 = no sanitizer report.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "oracle.h"
#include "rt.h"
#include "scene_compile.hpp"

static int check_file(const char* path, const char* png_out) {
    rt_scene* s = nullptr;
    const int rc = rt_scene_load_json_file(path, &s);
    if (rc != RT_OK) {
        std::printf("load %s: rc=%d %s\n", path, rc, rt_last_error());
        return 0;   // an error path is a valid outcome (exercised for the sanitizers)
    }
    const rt_scene_desc* d = rt_scene_get_desc(s);
    rtamd::CompiledScene cs = rtamd::compile_scene(*d);
    int W = rt_camera_width(&d->camera), H = rt_camera_height(&d->camera);
    if (W > 64) W = 64;
    if (H > 48) H = 48;
    std::vector<double> fb((size_t)W * H * 3);
    for (int mode = 0; mode < 2; ++mode) {
        oracle_stats st{};
        if (oracle_render_rows(d, W, H, mode, 0, H, fb.data(), &st, 2) != 0) {
            std::printf("oracle failed on %s\n", path);
            rt_scene_destroy(s);
            return 1;
        }
        std::vector<uint8_t> rgb((size_t)W * H * 3);
        rt_framebuffer_to_rgb8(fb.data(), (size_t)W * H, rgb.data());
        if (rt_write_png(png_out, rgb.data(), W, H, 3) != RT_OK) {
            std::printf("png failed\n");
            rt_scene_destroy(s);
            return 1;
        }
    }
    std::printf("ok %s %dx%d objs=%zu ops=%zu fold=%zu\n", path, W, H, cs.objs.size(), cs.ops.size(), cs.fold.size());
    rt_scene_destroy(s);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: host_check <out.png> <scene.json>...\n");
        return 2;
    }
    int bad = 0;
    for (int i = 2; i < argc; ++i) bad += check_file(argv[i], argv[1]);
    // malformed inputs through the text entry point (error paths)
    const char* broken[] = {"", "{", "{\"objects\": [{\"sphere\": {}}]}", "[1, 2", "{\"screen\": {\"dpi\": \"x\"}}",
                            "{\"objects\": [{\"csg\": {\"operator\": \"xor\"}}]}", "\xef\xbb\xbf{}", "nul\0l"};
    for (const char* t : broken) {
        rt_scene* s = nullptr;
        if (rt_scene_load_json_text(t, std::strlen(t), &s) == RT_OK) rt_scene_destroy(s);
    }
    return bad ? 1 : 0;
}
