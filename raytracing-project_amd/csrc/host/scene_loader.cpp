// scene_loader.cpp — JSON scene schema -> flattened IR.
//
// Restates the semantics of the reference loader
// (raytracer/src/json_loader.cpp) on top of rtjson::Value:
//   parse_color_block :83-123   parse_screen :133-164   parse_medium :171-184
//   parse_sources :191-204      make_sphere :211-227    make_halfspace :234-248
//   make_pokeball :256-297      make_scaling/translation/rotation :304-345
//   make_csg_binary :354-366    fold_csg_array :375-384 fold_difference_array :392-401
//   parse_object_node :409-434  load_scene_from_json_text :458-490
//   load_scene_from_json :499-503
// Geometry constructors whose arithmetic runs at load time are restated too:
//   HalfSpace normal normalisation (geometry.h:124-134), Pokeball button_dir
//   (Dir3::normalized, core.h:95-101), Matrix4 generators/inverse (core.h:179-263).
#include <cmath>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "json.hpp"
#include "scene_ir.hpp"

namespace rtamd {

using rtjson::Value;

// ------------------------------------------------------------------ Mat4
Mat4::Mat4() {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) m[i][j] = (i == j) ? 1.0 : 0.0;
}
static Mat4 mk(double m00, double m01, double m02, double m03, double m10, double m11, double m12,
               double m13, double m20, double m21, double m22, double m23, double m30, double m31,
               double m32, double m33) {
    Mat4 r;
    r.m[0][0] = m00; r.m[0][1] = m01; r.m[0][2] = m02; r.m[0][3] = m03;
    r.m[1][0] = m10; r.m[1][1] = m11; r.m[1][2] = m12; r.m[1][3] = m13;
    r.m[2][0] = m20; r.m[2][1] = m21; r.m[2][2] = m22; r.m[2][3] = m23;
    r.m[3][0] = m30; r.m[3][1] = m31; r.m[3][2] = m32; r.m[3][3] = m33;
    return r;
}
Mat4 Mat4::translation(double tx, double ty, double tz) {
    return mk(1, 0, 0, tx, 0, 1, 0, ty, 0, 0, 1, tz, 0, 0, 0, 1);
}
Mat4 Mat4::scaling(double sx, double sy, double sz) {
    return mk(sx, 0, 0, 0, 0, sy, 0, 0, 0, 0, sz, 0, 0, 0, 0, 1);
}
Mat4 Mat4::rotation_x(double a) {
    double c = std::cos(a), s = std::sin(a);
    return mk(1, 0, 0, 0, 0, c, -s, 0, 0, s, c, 0, 0, 0, 0, 1);
}
Mat4 Mat4::rotation_y(double a) {
    double c = std::cos(a), s = std::sin(a);
    return mk(c, 0, s, 0, 0, 1, 0, 0, -s, 0, c, 0, 0, 0, 0, 1);
}
Mat4 Mat4::rotation_z(double a) {
    double c = std::cos(a), s = std::sin(a);
    return mk(c, -s, 0, 0, s, c, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1);
}
Mat4 Mat4::inverse() const {
    Mat4 inv;
    double r11 = m[0][0], r12 = m[0][1], r13 = m[0][2], tx = m[0][3];
    double r21 = m[1][0], r22 = m[1][1], r23 = m[1][2], ty = m[1][3];
    double r31 = m[2][0], r32 = m[2][1], r33 = m[2][2], tz = m[2][3];
    double det = r11 * (r22 * r33 - r23 * r32) - r12 * (r21 * r33 - r23 * r31) +
                 r13 * (r21 * r32 - r22 * r31);
    if (std::abs(det) < 1e-12) return Mat4();
    double inv_det = 1.0 / det;
    inv.m[0][0] = (r22 * r33 - r23 * r32) * inv_det;
    inv.m[0][1] = (r13 * r32 - r12 * r33) * inv_det;
    inv.m[0][2] = (r12 * r23 - r13 * r22) * inv_det;
    inv.m[1][0] = (r23 * r31 - r21 * r33) * inv_det;
    inv.m[1][1] = (r11 * r33 - r13 * r31) * inv_det;
    inv.m[1][2] = (r13 * r21 - r11 * r23) * inv_det;
    inv.m[2][0] = (r21 * r32 - r22 * r31) * inv_det;
    inv.m[2][1] = (r12 * r31 - r11 * r32) * inv_det;
    inv.m[2][2] = (r11 * r22 - r12 * r21) * inv_det;
    inv.m[0][3] = -(inv.m[0][0] * tx + inv.m[0][1] * ty + inv.m[0][2] * tz);
    inv.m[1][3] = -(inv.m[1][0] * tx + inv.m[1][1] * ty + inv.m[1][2] * tz);
    inv.m[2][3] = -(inv.m[2][0] * tx + inv.m[2][1] * ty + inv.m[2][2] * tz);
    inv.m[3][0] = 0; inv.m[3][1] = 0; inv.m[3][2] = 0; inv.m[3][3] = 1;
    return inv;
}

// --------------------------------------------------------------- SceneIR
rt_material default_material() {
    rt_material m{};
    m.albedo[0] = m.albedo[1] = m.albedo[2] = 1.0;
    m.ambient[0] = m.ambient[1] = m.ambient[2] = 0.0;
    m.kd = 1.0; m.ks = 0.0; m.kr = 0.0; m.kt = 0.0;
    m.shininess = 32.0;
    m.refractive_index = 1.0;
    return m;
}

rt_node empty_node(int kind) {
    rt_node n{};
    n.kind = kind;
    n.a = n.b = -1;
    n.op = 0;
    n.mat = -1;
    for (int i = 0; i < 5; ++i) n.mats[i] = -1;
    return n;
}

void set_node_matrix(rt_node& n, const Mat4& M) {
    Mat4 inv = M.inverse();   // Transform ctor caches M.inverse() (transform.h:19-20)
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) {
            n.v[i * 4 + j] = M.m[i][j];
            n.v[12 + i * 4 + j] = inv.m[i][j];
        }
}

SceneIR::SceneIR() {
    // Camera{} defaults (camera.h:26-79): eye (0,0,1), P (0,0,0), L 1x1, dpi 72.
    camera.eye[0] = 0; camera.eye[1] = 0; camera.eye[2] = 1;
    camera.P[0] = camera.P[1] = camera.P[2] = 0;
    camera.Lx = 1.0; camera.Ly = 1.0; camera.dpi = 72;
}

int SceneIR::add_material(const rt_material& m) {
    materials.push_back(m);
    return (int)materials.size() - 1;
}
int SceneIR::add_node(const rt_node& n) {
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}

rt_scene_desc SceneIR::desc() const {
    rt_scene_desc d{};
    d.camera = camera;
    for (int i = 0; i < 3; ++i) { d.background[i] = background[i]; d.ambient[i] = ambient[i]; }
    d.medium_index = medium_index;
    d.recursion_limit = recursion_limit;
    d.n_lights = (int32_t)lights.size();
    d.lights = lights.empty() ? nullptr : lights.data();
    d.n_materials = (int32_t)materials.size();
    d.materials = materials.empty() ? nullptr : materials.data();
    d.n_nodes = (int32_t)nodes.size();
    d.nodes = nodes.empty() ? nullptr : nodes.data();
    d.n_objects = (int32_t)objects.size();
    d.objects = objects.empty() ? nullptr : objects.data();
    d.n_dir_lights = (int32_t)dir_lights.size();
    d.dir_lights = dir_lights.empty() ? nullptr : dir_lights.data();
    return d;
}

SceneIR SceneIR::from_desc(const rt_scene_desc& d) {
    SceneIR s;
    s.camera = d.camera;
    for (int i = 0; i < 3; ++i) { s.background[i] = d.background[i]; s.ambient[i] = d.ambient[i]; }
    s.medium_index = d.medium_index;
    s.recursion_limit = d.recursion_limit;
    if (d.n_lights > 0) s.lights.assign(d.lights, d.lights + d.n_lights);
    if (d.n_materials > 0) s.materials.assign(d.materials, d.materials + d.n_materials);
    if (d.n_nodes > 0) s.nodes.assign(d.nodes, d.nodes + d.n_nodes);
    if (d.n_objects > 0) s.objects.assign(d.objects, d.objects + d.n_objects);
    if (d.n_dir_lights > 0) s.dir_lights.assign(d.dir_lights, d.dir_lights + d.n_dir_lights);
    return s;
}

// ---------------------------------------------------------------- loader
namespace {

struct Vec3 { double x, y, z; };

Vec3 as_vec3(const Value& arr) {   // json_loader.cpp:55-58
    if (!arr.is_array() || arr.size() != 3) throw std::runtime_error("Expected array[3]");
    return Vec3{arr[0].get_double(), arr[1].get_double(), arr[2].get_double()};
}

Vec3 as_rgb(const Value& arr) {    // json_loader.cpp:65-68
    if (!arr.is_array() || arr.size() != 3) throw std::runtime_error("Expected color array[3]");
    return Vec3{arr[0].get_double(), arr[1].get_double(), arr[2].get_double()};
}

void ensure_object_1key(const Value& j) {   // json_loader.cpp:71-73
    if (!j.is_object() || j.size() != 1)
        throw std::runtime_error("Each object node must be a one-entry object");
}

double deg2rad(double d) { return d * M_PI / 180.0; }   // json_loader.cpp:76

void set3(double* dst, const Vec3& v) { dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; }

rt_material parse_color_block(const Value& jc) {   // json_loader.cpp:83-123
    if (!jc.is_object()) throw std::runtime_error("color must be an object");
    rt_material m{};
    m.albedo[0] = m.albedo[1] = m.albedo[2] = 0.0;
    m.ambient[0] = m.ambient[1] = m.ambient[2] = 0.0;
    m.kd = 1.0; m.ks = 0.0; m.kr = 0.0; m.kt = 0.0;
    m.shininess = 1.0;
    m.refractive_index = 1.0;
    if (jc.contains("diffuse")) set3(m.albedo, as_rgb(jc.at("diffuse")));
    if (jc.contains("ambient")) set3(m.ambient, as_rgb(jc.at("ambient")));
    if (jc.contains("specular")) { Vec3 s = as_rgb(jc.at("specular")); m.ks = (s.x + s.y + s.z) / 3.0; }
    if (jc.contains("reflected")) { Vec3 r = as_rgb(jc.at("reflected")); m.kr = (r.x + r.y + r.z) / 3.0; }
    if (jc.contains("refracted")) { Vec3 t = as_rgb(jc.at("refracted")); m.kt = (t.x + t.y + t.z) / 3.0; }
    if (jc.contains("shininess")) m.shininess = jc.at("shininess").get_double();
    return m;
}

class Builder {
public:
    explicit Builder(SceneIR& s) : s_(s) {}

    void parse_screen(const Value& root) {   // json_loader.cpp:133-164
        if (!root.contains("screen")) return;
        const Value& j = root.at("screen");
        const int dpi = j.contains("dpi") ? j.at("dpi").get_int() : 72;
        double Lx = 1.0, Ly = 1.0;
        if (j.contains("dimensions")) {
            const Value& d = j.at("dimensions");
            if (!d.is_array() || d.size() != 2)
                throw std::runtime_error("screen.dimensions must be [Lx, Ly]");
            Lx = d[0].get_double();
            Ly = d[1].get_double();
        }
        if (!j.contains("position")) throw std::runtime_error("screen.position is required");
        const Vec3 P = as_vec3(j.at("position"));
        if (!j.contains("observer")) throw std::runtime_error("screen.observer is required");
        const Vec3 eye = as_vec3(j.at("observer"));
        set3(s_.camera.P, P);
        s_.camera.Lx = Lx;
        s_.camera.Ly = Ly;
        s_.camera.dpi = dpi;
        set3(s_.camera.eye, eye);
    }

    void parse_medium(const Value& root) {   // json_loader.cpp:171-184
        if (!root.contains("medium")) return;
        const Value& jm = root.at("medium");
        if (jm.contains("ambient")) set3(s_.ambient, as_rgb(jm.at("ambient")));
        if (jm.contains("index")) s_.medium_index = jm.at("index").get_double();
        if (jm.contains("recursion")) s_.recursion_limit = jm.at("recursion").get_int();
    }

    void parse_sources(const Value& root) {   // json_loader.cpp:191-204
        if (!root.contains("sources")) return;
        const Value& arr = root.at("sources");
        if (!arr.is_array()) throw std::runtime_error("'sources' must be an array");
        for (const Value& js : arr.array_items()) {
            if (!js.contains("position") || !js.contains("intensity"))
                throw std::runtime_error("each source needs 'position' and 'intensity'");
            const Vec3 p = as_vec3(js.at("position"));
            const Vec3 I = as_rgb(js.at("intensity"));
            rt_light L{};
            set3(L.pos, p);
            set3(L.intensity, I);
            s_.lights.push_back(L);
        }
    }

    int parse_object_node(const Value& jnode) {   // json_loader.cpp:409-434
        ensure_object_1key(jnode);
        const auto it = jnode.object_items().begin();
        const std::string& kind = it->first;
        const Value& val = it->second;
        if (kind == "sphere") return make_sphere(val);
        if (kind == "halfSpace") return make_halfspace(val);
        if (kind == "pokeball") return make_pokeball(val);
        if (kind == "scaling") return make_scaling(val);
        if (kind == "translation") return make_translation(val);
        if (kind == "rotation") return make_rotation(val);
        if (kind == "csg") return make_csg_binary(val);
        if (kind == "union") return fold_csg_array(val, RT_CSG_UNION);
        if (kind == "intersection") return fold_csg_array(val, RT_CSG_INTERSECTION);
        if (kind == "difference") return fold_difference_array(val);
        throw std::runtime_error("unknown object kind: " + kind);
    }

private:
    SceneIR& s_;

    int make_sphere(const Value& j) {   // json_loader.cpp:211-227
        if (!j.contains("position") || !j.contains("radius") || !j.contains("color"))
            throw std::runtime_error("sphere requires 'position', 'radius', 'color'");
        const Vec3 c = as_vec3(j.at("position"));
        const double r = j.at("radius").get_double();
        rt_material m = parse_color_block(j.at("color"));
        if (j.contains("index")) m.refractive_index = j.at("index").get_double();
        rt_node n = empty_node(RT_NODE_SPHERE);
        n.mat = s_.add_material(m);
        set3(n.v, c);
        n.v[3] = r;
        return s_.add_node(n);
    }

    int make_halfspace(const Value& j) {   // json_loader.cpp:234-248
        if (!j.contains("position") || !j.contains("normal") || !j.contains("color"))
            throw std::runtime_error("halfSpace requires 'position', 'normal', 'color'");
        const Vec3 p0 = as_vec3(j.at("position"));
        const Vec3 N = as_vec3(j.at("normal"));
        rt_material m = parse_color_block(j.at("color"));
        if (j.contains("index")) m.refractive_index = j.at("index").get_double();
        rt_node n = empty_node(RT_NODE_HALFSPACE);
        n.mat = s_.add_material(m);
        set3(n.v, p0);
        set3(n.aux, N);
        // HalfSpace ctor (geometry.h:124-134)
        const double L2 = N.x * N.x + N.y * N.y + N.z * N.z;
        if (L2 > 0.0) {
            const double invL = 1.0 / std::sqrt(L2);
            n.v[3] = N.x * invL; n.v[4] = N.y * invL; n.v[5] = N.z * invL;
        } else {
            n.v[3] = 0; n.v[4] = 1; n.v[5] = 0;
        }
        return s_.add_node(n);
    }

    int make_pokeball(const Value& jn) {   // json_loader.cpp:256-297
        if (!jn.contains("position") || !jn.contains("radius"))
            throw std::runtime_error("pokeball requires 'position' and 'radius'.");
        const Vec3 c = as_vec3(jn.at("position"));
        const double r = jn.at("radius").get_double();

        rt_material top = default_material(), bottom = default_material(), belt = default_material(),
                    ring = default_material(), button = default_material();
        top.albedo[0] = 0.88; top.albedo[1] = 0.12; top.albedo[2] = 0.20; top.kd = 1.0; top.ks = 0.15; top.shininess = 64;
        bottom.albedo[0] = 0.95; bottom.albedo[1] = 0.95; bottom.albedo[2] = 0.98; bottom.kd = 1.0; bottom.ks = 0.08; bottom.shininess = 32;
        belt.albedo[0] = 0.12; belt.albedo[1] = 0.12; belt.albedo[2] = 0.15; belt.kd = 1.0;
        ring.albedo[0] = 0.35; ring.albedo[1] = 0.35; ring.albedo[2] = 0.40; ring.kd = 1.0;
        button.albedo[0] = 0.96; button.albedo[1] = 0.96; button.albedo[2] = 0.99; button.kd = 1.0; button.ks = 0.25; button.shininess = 64;

        double belt_half = 0.06, btn_outer = 0.28, ring_width = 0.06;
        Vec3 btn_dir{1, 0, 0};
        if (jn.contains("colors")) {
            const Value& jc = jn.at("colors");
            if (jc.contains("top")) top = parse_color_block(jc.at("top"));
            if (jc.contains("bottom")) bottom = parse_color_block(jc.at("bottom"));
            if (jc.contains("belt")) belt = parse_color_block(jc.at("belt"));
            if (jc.contains("ring")) ring = parse_color_block(jc.at("ring"));
            if (jc.contains("button")) button = parse_color_block(jc.at("button"));
        }
        if (jn.contains("belt_half")) belt_half = jn.at("belt_half").get_double();
        if (jn.contains("button_outer")) btn_outer = jn.at("button_outer").get_double();
        if (jn.contains("ring_width")) ring_width = jn.at("ring_width").get_double();
        if (jn.contains("button_dir")) btn_dir = as_vec3(jn.at("button_dir"));

        rt_node n = empty_node(RT_NODE_POKEBALL);
        n.mats[RT_PB_TOP] = s_.add_material(top);
        n.mats[RT_PB_BOTTOM] = s_.add_material(bottom);
        n.mats[RT_PB_BELT] = s_.add_material(belt);
        n.mats[RT_PB_RING] = s_.add_material(ring);
        n.mats[RT_PB_BUTTON] = s_.add_material(button);
        set3(n.v, c);
        n.v[3] = r;
        n.v[4] = belt_half;
        n.v[5] = btn_outer;
        n.v[6] = ring_width;
        set3(n.aux, btn_dir);
        // btnDir(button_dir.normalized()) — Dir3::normalized (core.h:95-101)
        const double L = std::sqrt(btn_dir.x * btn_dir.x + btn_dir.y * btn_dir.y + btn_dir.z * btn_dir.z);
        if (L > 1e-6) {
            n.v[7] = btn_dir.x / L; n.v[8] = btn_dir.y / L; n.v[9] = btn_dir.z / L;
        } else {
            n.v[7] = 0; n.v[8] = 1; n.v[9] = 0;
        }
        return s_.add_node(n);
    }

    int make_transform(int kind, const Mat4& M, int child) {
        rt_node n = empty_node(kind);
        n.a = child;
        set_node_matrix(n, M);
        return s_.add_node(n);
    }

    int make_scaling(const Value& j) {   // json_loader.cpp:304-310
        if (!j.contains("factors") || !j.contains("subject"))
            throw std::runtime_error("scaling requires 'factors' and 'subject'");
        const Vec3 s = as_vec3(j.at("factors"));
        int child = parse_object_node(j.at("subject"));
        int idx = make_transform(RT_NODE_SCALING, Mat4::scaling(s.x, s.y, s.z), child);
        set3(s_.nodes[idx].aux, s);
        return idx;
    }

    int make_translation(const Value& j) {   // json_loader.cpp:317-323
        if (!j.contains("factors") || !j.contains("subject"))
            throw std::runtime_error("translation requires 'factors' and 'subject'");
        const Vec3 t = as_vec3(j.at("factors"));
        int child = parse_object_node(j.at("subject"));
        int idx = make_transform(RT_NODE_TRANSLATION, Mat4::translation(t.x, t.y, t.z), child);
        set3(s_.nodes[idx].aux, t);
        return idx;
    }

    int make_rotation(const Value& j) {   // json_loader.cpp:330-345
        if (!j.contains("angle") || !j.contains("direction") || !j.contains("subject"))
            throw std::runtime_error("rotation requires 'angle', 'direction', and 'subject'");
        const double angle_deg = j.at("angle").get_double();
        const int axis_i = j.at("direction").get_int();
        if (axis_i != 0 && axis_i != 1 && axis_i != 2)
            throw std::runtime_error("rotation direction must be 0 (X), 1 (Y), or 2 (Z)");
        int child = parse_object_node(j.at("subject"));
        const double ang = deg2rad(angle_deg);
        Mat4 M = axis_i == 0 ? Mat4::rotation_x(ang) : axis_i == 1 ? Mat4::rotation_y(ang) : Mat4::rotation_z(ang);
        int idx = make_transform(RT_NODE_ROTATION, M, child);
        s_.nodes[idx].op = axis_i;
        s_.nodes[idx].aux[0] = ang;
        return idx;
    }

    int make_csg(int op, int a, int b) {
        rt_node n = empty_node(RT_NODE_CSG);
        n.op = op;
        n.a = a;
        n.b = b;
        return s_.add_node(n);
    }

    int make_csg_binary(const Value& j) {   // json_loader.cpp:354-366
        if (!j.contains("operator") || !j.contains("left") || !j.contains("right"))
            throw std::runtime_error("csg requires 'operator', 'left', 'right'");
        const std::string op = j.at("operator").get_string();
        int cop;
        if (op == "union") cop = RT_CSG_UNION;
        else if (op == "intersection") cop = RT_CSG_INTERSECTION;
        else if (op == "difference") cop = RT_CSG_DIFFERENCE;
        else throw std::runtime_error("csg.operator must be union/intersection/difference");
        int lhs = parse_object_node(j.at("left"));
        int rhs = parse_object_node(j.at("right"));
        return make_csg(cop, lhs, rhs);
    }

    int fold_csg_array(const Value& arr, int op) {   // json_loader.cpp:375-384
        if (!arr.is_array() || arr.empty())
            throw std::runtime_error("CSG array must be a non-empty array");
        int acc = parse_object_node(arr.at(0));
        for (size_t i = 1; i < arr.size(); ++i) {
            int rhs = parse_object_node(arr.at(i));
            acc = make_csg(op, acc, rhs);
        }
        return acc;
    }

    int fold_difference_array(const Value& arr) {   // json_loader.cpp:392-401
        if (!arr.is_array() || arr.size() < 2)
            throw std::runtime_error("difference array must have at least 2 elements");
        int acc = parse_object_node(arr.at(0));
        for (size_t i = 1; i < arr.size(); ++i) {
            int rhs = parse_object_node(arr.at(i));
            acc = make_csg(RT_CSG_DIFFERENCE, acc, rhs);
        }
        return acc;
    }
};

}  // namespace

SceneIR load_scene_from_json_text(const std::string& text) {   // json_loader.cpp:458-490
    SceneIR s;
    try {
        Value root = Value::parse(text);
        Builder b(s);
        b.parse_screen(root);
        b.parse_medium(root);
        b.parse_sources(root);
        if (root.contains("background")) {
            Vec3 bg = as_rgb(root.at("background"));
            set3(s.background, bg);
        }
        s.objects.clear();
        if (root.contains("objects")) {
            const Value& arr = root.at("objects");
            if (!arr.is_array()) throw std::runtime_error("'objects' must be an array");
            for (const Value& node : arr.array_items()) s.objects.push_back(b.parse_object_node(node));
        }
        return s;
    } catch (const rtjson::parse_error& e) {
        throw std::runtime_error(std::string("JSON parse error: ") + e.what());
    } catch (const std::exception& e) {
        throw std::runtime_error(std::string("JSON processing error: ") + e.what());
    }
}

SceneIR load_scene_from_json_file(const std::string& path) {   // json_loader.cpp:499-503
    std::ifstream ifs(path);
    if (!ifs) throw std::runtime_error("Cannot open JSON file: " + path);
    std::ostringstream ss;
    ss << ifs.rdbuf();
    return load_scene_from_json_text(ss.str());
}

}  // namespace rtamd
