// scene_ir.hpp — owning container of the flattened scene IR (include/rt.h).
#pragma once

#include <string>
#include <vector>

#include "rt.h"

namespace rtamd {

// Matrix4 with the reference's semantics (core.h:130-264): rows 0..3, 4 columns.
struct Mat4 {
    double m[4][4];
    Mat4();
    static Mat4 translation(double tx, double ty, double tz);   // core.h:179
    static Mat4 scaling(double sx, double sy, double sz);       // core.h:189
    static Mat4 rotation_x(double a);                           // core.h:199
    static Mat4 rotation_y(double a);                           // core.h:211
    static Mat4 rotation_z(double a);                           // core.h:223
    Mat4 inverse() const;                                       // core.h:239-263
};

struct SceneIR {
    rt_camera camera{};
    double background[3] = {0, 0, 0};
    double ambient[3] = {0, 0, 0};
    double medium_index = 1.0;
    int recursion_limit = 5;
    std::vector<rt_light> lights;
    std::vector<rt_dir_light> dir_lights;
    std::vector<rt_material> materials;
    std::vector<rt_node> nodes;
    std::vector<int32_t> objects;

    SceneIR();
    rt_scene_desc desc() const;       // view with pointers into the vectors
    static SceneIR from_desc(const rt_scene_desc& d);

    int add_material(const rt_material& m);
    int add_node(const rt_node& n);
};

// Material defaults of geometry.h:5-22 (Material{}).
rt_material default_material();
rt_node empty_node(int kind);
// Fill a transform node's forward/inverse matrices.
void set_node_matrix(rt_node& n, const Mat4& M);

// json_loader.cpp semantics.  Throws std::runtime_error with the reference's
// "JSON parse error: " / "JSON processing error: " prefixes.
SceneIR load_scene_from_json_text(const std::string& text);
SceneIR load_scene_from_json_file(const std::string& path);

}  // namespace rtamd

struct rt_scene {
    rtamd::SceneIR ir;
    rt_scene_desc d;
    uint64_t uid = 0;   // process-unique, never reused: keys the device-resident copies (rt_render.hip)
};
