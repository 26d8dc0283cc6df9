// tracer.hpp — C++17 host mirror of the reference's interface for the hot
// path, implemented on the C-ABI (include/rt.h).  Same names and argument
// meaning as the reference:
//   jsonio::load_scene_from_json[_text]   json_loader.h:27,36 (throws std::runtime_error)
//   Tracer{scene, camera, width, height, mode}.render(std::vector<Color>&)   tracer.h:18-35
// Camera exposes ScreenSpec::nx()/ny() (camera.h:19-21).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt.h"

namespace rtamd {

struct Color {   // core.h:287-305
    double r{}, g{}, b{};
};

enum class RenderMode { Standard, Paper };   // tracer.h:8-11

// Owning scene handle (Scene + the loader's global pools of the reference).
class Scene {
public:
    Scene() = default;
    Scene(const Scene&) = delete;
    Scene& operator=(const Scene&) = delete;
    ~Scene() { reset(); }
    void reset(rt_scene* s = nullptr) {
        if (s_) rt_scene_destroy(s_);
        s_ = s;
    }
    rt_scene* get() const { return s_; }
    const rt_scene_desc* desc() const { return s_ ? rt_scene_get_desc(s_) : nullptr; }

private:
    rt_scene* s_ = nullptr;
};

struct Camera {
    rt_camera c{};
    int nx() const { return rt_camera_width(&c); }
    int ny() const { return rt_camera_height(&c); }
};

namespace jsonio {

inline bool load_scene_from_json_text(const std::string& text, Scene& scene, Camera& cam) {
    rt_scene* s = nullptr;
    int rc = rt_scene_load_json_text(text.data(), text.size(), &s);
    if (rc != RT_OK) throw std::runtime_error(rt_last_error());
    scene.reset(s);
    cam.c = scene.desc()->camera;
    return true;
}

inline bool load_scene_from_json(const std::string& filename, Scene& scene, Camera& cam) {
    rt_scene* s = nullptr;
    int rc = rt_scene_load_json_file(filename.c_str(), &s);
    if (rc != RT_OK) throw std::runtime_error(rt_last_error());
    scene.reset(s);
    cam.c = scene.desc()->camera;
    return true;
}

}  // namespace jsonio

struct Tracer {
    const Scene* scene{nullptr};
    const Camera* camera{nullptr};
    int width{640};
    int height{360};
    RenderMode mode{RenderMode::Standard};
    int flags{RT_FLAG_NONE};
    int n_gpus{1};                 // devices of this process (rt_render_multi); 0 = all visible
    mutable rt_stats stats{};

    // Tracer::render (tracer.cpp:247-305): returns silently when the scene or
    // camera is missing or the size is not positive; throws on device errors
    // (the reference cannot fail there; the device path must fail loudly).
    void render(std::vector<Color>& framebuffer) const {
        if (!scene || !scene->get() || !camera || width <= 0 || height <= 0) return;
        framebuffer.assign((size_t)width * height, Color{});
        int rc = rt_render_multi(scene->get(), width, height,
                                 mode == RenderMode::Paper ? RT_MODE_PAPER : RT_MODE_STANDARD, flags, n_gpus,
                                 reinterpret_cast<double*>(framebuffer.data()), &stats);
        if (rc != RT_OK) throw std::runtime_error(std::string("rt_render failed: ") + rt_last_error());
    }

    // render() + framebuffer_to_mat_bgr8's toByte (main.cpp:19-34) on the
    // device: rgb[(y*W + x)*3 + c], RGB order, top row first.
    void render_rgb8(std::vector<uint8_t>& rgb) const {
        if (!scene || !scene->get() || !camera || width <= 0 || height <= 0) return;
        if (rgb.size() != (size_t)width * height * 3) rgb.assign((size_t)width * height * 3, 0);
        int rc = rt_render_rgb8(scene->get(), width, height,
                                mode == RenderMode::Paper ? RT_MODE_PAPER : RT_MODE_STANDARD, flags, n_gpus,
                                rgb.data(), &stats);
        if (rc != RT_OK) throw std::runtime_error(std::string("rt_render failed: ") + rt_last_error());
    }
};

static_assert(sizeof(Color) == 3 * sizeof(double), "Color must be three packed doubles");

}  // namespace rtamd
