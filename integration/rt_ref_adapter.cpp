// rt_ref_adapter.cpp — see rt_ref_adapter.hpp.
//
// The reference keeps CSG's operator and operands private (csg.h:42-48) and
// exposes no accessor.  A maintainer may add three const getters to CSG; so
// that this file also builds against the UNMODIFIED reference (our tests
// compile it in place, oracle/Makefile), it reads them through the standard
// explicit-instantiation access rule ([temp.explicit]/12: names in an
// explicit instantiation are not access-checked).
#include "rt_ref_adapter.hpp"

#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>

#include "csg.h"
#include "geometry.h"
#include "transform.h"

namespace {

template <class Tag, typename Tag::type M>
struct Grant {
    friend typename Tag::type member(Tag) { return M; }
};
struct CsgOpTag {
    using type = CSGOp CSG::*;
    friend type member(CsgOpTag);
};
struct CsgATag {
    using type = std::shared_ptr<Primitive> CSG::*;
    friend type member(CsgATag);
};
struct CsgBTag {
    using type = std::shared_ptr<Primitive> CSG::*;
    friend type member(CsgBTag);
};
template struct Grant<CsgOpTag, &CSG::op_>;
template struct Grant<CsgATag, &CSG::A_>;
template struct Grant<CsgBTag, &CSG::B_>;

struct Builder {
    std::vector<rt_material> mats;
    std::vector<rt_node> nodes;
    std::map<const Material*, int> mat_id;
    std::map<const Primitive*, int> node_id;

    int material(const Material* m) {
        if (!m) return -1;   // a primitive without material: magenta in shading (shading.cpp:33)
        auto it = mat_id.find(m);
        if (it != mat_id.end()) return it->second;
        rt_material r{};
        r.albedo[0] = m->albedo.r; r.albedo[1] = m->albedo.g; r.albedo[2] = m->albedo.b;
        r.ambient[0] = m->ambient.r; r.ambient[1] = m->ambient.g; r.ambient[2] = m->ambient.b;
        r.kd = m->kd; r.ks = m->ks; r.kr = m->kr; r.kt = m->kt;
        r.shininess = m->shininess;
        r.refractive_index = m->refractive_index;
        mats.push_back(r);
        return mat_id[m] = (int)mats.size() - 1;
    }

    static rt_node blank(int kind) {
        rt_node n;
        std::memset(&n, 0, sizeof(n));
        n.kind = kind;
        n.a = n.b = -1;
        n.mat = -1;
        for (int& k : n.mats) k = -1;
        return n;
    }

    static void matrices(rt_node& n, const Transform& t) {
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 4; ++j) {
                n.v[4 * i + j] = t.transform_matrix.m[i][j];
                n.v[12 + 4 * i + j] = t.inverse_matrix.m[i][j];
            }
    }

    int node(const Primitive* p, int depth = 0) {
        if (!p) throw std::runtime_error("null primitive in the scene graph");
        if (depth > 4096) throw std::runtime_error("scene graph too deep");
        auto it = node_id.find(p);
        if (it != node_id.end()) return it->second;
        rt_node n;
        if (auto pb = dynamic_cast<const Pokeball*>(p)) {   // before Sphere: Pokeball derives from it
            n = blank(RT_NODE_POKEBALL);
            n.v[0] = pb->c.x; n.v[1] = pb->c.y; n.v[2] = pb->c.z; n.v[3] = pb->r;
            n.v[4] = pb->beltHalf; n.v[5] = pb->btnOuter; n.v[6] = pb->ringWidth;
            n.v[7] = pb->btnDir.x; n.v[8] = pb->btnDir.y; n.v[9] = pb->btnDir.z;
            n.aux[0] = pb->btnDir.x; n.aux[1] = pb->btnDir.y; n.aux[2] = pb->btnDir.z;
            n.mats[RT_PB_TOP] = material(&pb->topMat);
            n.mats[RT_PB_BOTTOM] = material(&pb->bottomMat);
            n.mats[RT_PB_BELT] = material(&pb->beltMat);
            n.mats[RT_PB_RING] = material(&pb->ringMat);
            n.mats[RT_PB_BUTTON] = material(&pb->buttonMat);
        } else if (auto s = dynamic_cast<const Sphere*>(p)) {
            n = blank(RT_NODE_SPHERE);
            n.v[0] = s->c.x; n.v[1] = s->c.y; n.v[2] = s->c.z; n.v[3] = s->r;
            n.mat = material(s->mat);
        } else if (auto h = dynamic_cast<const HalfSpace*>(p)) {
            n = blank(RT_NODE_HALFSPACE);
            n.v[0] = h->p0.x; n.v[1] = h->p0.y; n.v[2] = h->p0.z;
            n.v[3] = h->n.x; n.v[4] = h->n.y; n.v[5] = h->n.z;   // already unit (geometry.h:124-134)
            n.aux[0] = h->n.x; n.aux[1] = h->n.y; n.aux[2] = h->n.z;
            n.mat = material(h->mat);
        } else if (auto c = dynamic_cast<const CSG*>(p)) {
            n = blank(RT_NODE_CSG);
            const CSGOp op = c->*member(CsgOpTag{});
            n.op = op == CSGOp::Union ? RT_CSG_UNION : op == CSGOp::Intersection ? RT_CSG_INTERSECTION
                                                                                  : RT_CSG_DIFFERENCE;
            n.a = node((c->*member(CsgATag{})).get(), depth + 1);
            n.b = node((c->*member(CsgBTag{})).get(), depth + 1);
        } else if (auto t = dynamic_cast<const Transform*>(p)) {
            const bool tr = dynamic_cast<const Translation*>(p) != nullptr;
            const bool sc = dynamic_cast<const Scaling*>(p) != nullptr;
            n = blank(tr ? RT_NODE_TRANSLATION : sc ? RT_NODE_SCALING : RT_NODE_ROTATION);
            matrices(n, *t);
            const auto& M = t->transform_matrix.m;
            if (tr) {
                n.aux[0] = M[0][3]; n.aux[1] = M[1][3]; n.aux[2] = M[2][3];
            } else if (sc) {
                n.aux[0] = M[0][0]; n.aux[1] = M[1][1]; n.aux[2] = M[2][2];
            } else {
                // the axis is the one the matrix leaves fixed (core.h:199-233)
                n.op = (M[0][0] == 1.0 && M[0][1] == 0.0 && M[0][2] == 0.0) ? 0
                       : (M[1][1] == 1.0 && M[1][0] == 0.0 && M[1][2] == 0.0) ? 1 : 2;
                const int a = n.op == 0 ? 1 : 0, b = n.op == 2 ? 1 : 2;
                n.aux[0] = std::atan2(n.op == 1 ? M[0][2] : M[b][a], M[a][a]);
            }
            n.a = node(t->child.get(), depth + 1);
        } else {
            throw std::runtime_error("unknown Primitive subtype in the scene graph");
        }
        nodes.push_back(n);
        return node_id[p] = (int)nodes.size() - 1;
    }
};

}  // namespace

namespace rtref {

int scene_from_reference(const Scene& scene, const Camera& cam, rt_scene** out) {
    if (!out) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    Builder B;
    std::vector<int32_t> objects;
    try {
        for (const Primitive* p : scene.objects) objects.push_back(B.node(p));
    } catch (const std::exception&) {
        return RT_ERR_INVALID_ARG;
    }
    std::vector<rt_light> lights;
    for (const PointLight& L : scene.point_lights) {
        rt_light l{};
        l.pos[0] = L.pos.x; l.pos[1] = L.pos.y; l.pos[2] = L.pos.z;
        l.intensity[0] = L.intensity.r; l.intensity[1] = L.intensity.g; l.intensity[2] = L.intensity.b;
        lights.push_back(l);
    }
    std::vector<rt_dir_light> dls;
    for (const DirectionalLight& L : scene.dir_lights) {
        rt_dir_light l{};
        l.dir[0] = L.dir.x; l.dir[1] = L.dir.y; l.dir[2] = L.dir.z;
        l.radiance[0] = L.radiance.r; l.radiance[1] = L.radiance.g; l.radiance[2] = L.radiance.b;
        dls.push_back(l);
    }
    rt_scene_desc d;
    std::memset(&d, 0, sizeof(d));
    d.camera.eye[0] = cam.eye.x; d.camera.eye[1] = cam.eye.y; d.camera.eye[2] = cam.eye.z;
    d.camera.P[0] = cam.screen.P.x; d.camera.P[1] = cam.screen.P.y; d.camera.P[2] = cam.screen.P.z;
    d.camera.Lx = cam.screen.Lx;
    d.camera.Ly = cam.screen.Ly;
    d.camera.dpi = cam.screen.dpi;
    d.background[0] = scene.background.r; d.background[1] = scene.background.g; d.background[2] = scene.background.b;
    d.ambient[0] = scene.ambient.r; d.ambient[1] = scene.ambient.g; d.ambient[2] = scene.ambient.b;
    d.medium_index = scene.medium_index;
    d.recursion_limit = scene.recursion_limit;
    d.n_lights = (int32_t)lights.size();
    d.lights = lights.data();
    d.n_materials = (int32_t)B.mats.size();
    d.materials = B.mats.data();
    d.n_nodes = (int32_t)B.nodes.size();
    d.nodes = B.nodes.data();
    d.n_objects = (int32_t)objects.size();
    d.objects = objects.data();
    d.n_dir_lights = (int32_t)dls.size();
    d.dir_lights = dls.data();
    return rt_scene_from_desc(&d, out);   // deep copy
}

void render_on_gpu(const Scene& scene, const Camera& cam, int width, int height, bool paper,
                   std::vector<Color>& framebuffer, int n_gpus) {
    if (width <= 0 || height <= 0) return;   // tracer.cpp:248
    rt_scene* s = nullptr;
    if (scene_from_reference(scene, cam, &s) != RT_OK)
        throw std::runtime_error(std::string("scene conversion failed: ") + rt_last_error());
    framebuffer.assign((size_t)width * height, Color{0, 0, 0});
    static_assert(sizeof(Color) == 3 * sizeof(double), "Color must be three packed doubles");
    rt_stats st{};
    const int rc = rt_render_multi(s, width, height, paper ? RT_MODE_PAPER : RT_MODE_STANDARD, RT_FLAG_NONE, n_gpus,
                                   reinterpret_cast<double*>(framebuffer.data()), &st);
    rt_scene_destroy(s);
    if (rc != RT_OK) throw std::runtime_error(std::string("rt_render failed: ") + rt_last_error());
}

}  // namespace rtref
