// rt_host.cpp — C-ABI entry points of librt_host.so (scene loading and IR
// access).  No exceptions cross the ABI: failures return an rt_status and
// leave the message in rt_last_error().
#include <atomic>
#include <cmath>
#include <cstring>
#include <new>
#include <string>

#include "rt.h"
#include "rt_internal.hpp"
#include "scene_ir.hpp"

namespace rtamd {
static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }
void clear_last_error() { g_last_error.clear(); }
}  // namespace rtamd

using rtamd::set_last_error;

extern "C" const char* rt_last_error(void) { return rtamd::g_last_error.c_str(); }
extern "C" int rt_abi_version(void) { return RT_ABI_VERSION; }

extern "C" int rt_camera_width(const rt_camera* c) {   // camera.h:19
    if (!c) return 0;
    int n = int(std::round(c->Lx * c->dpi));
    return n > 1 ? n : 1;
}
extern "C" int rt_camera_height(const rt_camera* c) {  // camera.h:21
    if (!c) return 0;
    int n = int(std::round(c->Ly * c->dpi));
    return n > 1 ? n : 1;
}

static std::atomic<uint64_t> g_next_uid{1};

static rt_scene* wrap(rtamd::SceneIR&& ir) {
    rt_scene* s = new (std::nothrow) rt_scene;
    if (!s) return nullptr;
    s->ir = std::move(ir);
    s->d = s->ir.desc();
    s->uid = g_next_uid.fetch_add(1);
    return s;
}

uint64_t rtamd::scene_uid(const rt_scene* s) { return s ? s->uid : 0; }

static int classify(const std::string& msg) {
    if (msg.rfind("JSON parse error: ", 0) == 0) return RT_ERR_PARSE;
    if (msg.rfind("Cannot open JSON file: ", 0) == 0) return RT_ERR_IO;
    return RT_ERR_PROCESSING;
}

extern "C" int rt_scene_load_json_text(const char* text, size_t len, rt_scene** out) {
    if (!out) { set_last_error("rt_scene_load_json_text: out is NULL"); return RT_ERR_INVALID_ARG; }
    *out = nullptr;
    if (!text && len) { set_last_error("rt_scene_load_json_text: text is NULL"); return RT_ERR_INVALID_ARG; }
    try {
        rtamd::SceneIR ir = rtamd::load_scene_from_json_text(std::string(text ? text : "", len));
        *out = wrap(std::move(ir));
        if (!*out) { set_last_error("out of memory"); return RT_ERR_INVALID_ARG; }
        rtamd::clear_last_error();
        return RT_OK;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return classify(e.what());
    }
}

extern "C" int rt_scene_load_json_file(const char* path, rt_scene** out) {
    if (!out || !path) { set_last_error("rt_scene_load_json_file: NULL argument"); return RT_ERR_INVALID_ARG; }
    *out = nullptr;
    try {
        rtamd::SceneIR ir = rtamd::load_scene_from_json_file(path);
        *out = wrap(std::move(ir));
        if (!*out) { set_last_error("out of memory"); return RT_ERR_INVALID_ARG; }
        rtamd::clear_last_error();
        return RT_OK;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return classify(e.what());
    }
}

extern "C" int rt_scene_from_desc(const rt_scene_desc* d, rt_scene** out) {
    if (!out || !d) { set_last_error("rt_scene_from_desc: NULL argument"); return RT_ERR_INVALID_ARG; }
    *out = nullptr;
    std::string why;
    if (!rtamd::validate_desc(*d, &why)) { set_last_error(why); return RT_ERR_INVALID_ARG; }
    *out = wrap(rtamd::SceneIR::from_desc(*d));
    if (!*out) { set_last_error("out of memory"); return RT_ERR_INVALID_ARG; }
    return RT_OK;
}

extern "C" const rt_scene_desc* rt_scene_get_desc(const rt_scene* s) { return s ? &s->d : nullptr; }

extern "C" void rt_scene_destroy(rt_scene* s) { delete s; }

namespace rtamd {

bool validate_desc(const rt_scene_desc& d, std::string* why) {
    auto bad = [&](const std::string& m) { if (why) *why = m; return false; };
    if (d.n_lights < 0 || d.n_materials < 0 || d.n_nodes < 0 || d.n_objects < 0 || d.n_dir_lights < 0)
        return bad("negative count");
    if ((d.n_lights && !d.lights) || (d.n_materials && !d.materials) || (d.n_nodes && !d.nodes) ||
        (d.n_objects && !d.objects) || (d.n_dir_lights && !d.dir_lights))
        return bad("NULL array with non-zero count");
    for (int i = 0; i < d.n_objects; ++i)
        if (d.objects[i] < 0 || d.objects[i] >= d.n_nodes) return bad("object index out of range");
    for (int i = 0; i < d.n_nodes; ++i) {
        const rt_node& n = d.nodes[i];
        auto mat_ok = [&](int m) { return m >= -1 && m < d.n_materials; };
        switch (n.kind) {
            case RT_NODE_SPHERE:
            case RT_NODE_HALFSPACE:
                if (!mat_ok(n.mat)) return bad("material index out of range");
                break;
            case RT_NODE_POKEBALL:
                for (int k = 0; k < 5; ++k)
                    if (!mat_ok(n.mats[k])) return bad("pokeball material index out of range");
                break;
            case RT_NODE_TRANSLATION:
            case RT_NODE_SCALING:
            case RT_NODE_ROTATION:
                if (n.a < 0 || n.a >= d.n_nodes) return bad("transform child out of range");
                break;
            case RT_NODE_CSG:
                if (n.a < 0 || n.a >= d.n_nodes || n.b < 0 || n.b >= d.n_nodes) return bad("csg child out of range");
                if (n.op < 0 || n.op > 2) return bad("bad csg op");
                break;
            default:
                return bad("unknown node kind");
        }
    }
    // The node graph must be a forest (no cycles): children precede parents
    // is not required, but depth must be finite.
    for (int i = 0; i < d.n_nodes; ++i) {
        int depth = 0;
        if (!node_depth_ok(d, i, 0, &depth)) return bad("node graph has a cycle or is too deep");
    }
    return true;
}

bool node_depth_ok(const rt_scene_desc& d, int idx, int level, int* maxdepth) {
    if (level > 4096) return false;
    if (level > *maxdepth) *maxdepth = level;
    const rt_node& n = d.nodes[idx];
    if (n.kind >= RT_NODE_TRANSLATION && n.kind <= RT_NODE_ROTATION)
        return node_depth_ok(d, n.a, level + 1, maxdepth);
    if (n.kind == RT_NODE_CSG)
        return node_depth_ok(d, n.a, level + 1, maxdepth) && node_depth_ok(d, n.b, level + 1, maxdepth);
    return true;
}

}  // namespace rtamd
