// ref_harness.cpp — OUR harness around the reference's own hot-path sources.
//
// TEST INFRASTRUCTURE ONLY.  oracle/Makefile compiles this file together with
// /root/reference/raytracer/src/{tracer,shading,scene,geometry,csg,transform}.cpp
// (read in place, never copied) into oracle/_ref/libref.so.  It rebuilds the
// reference objects from the flattened IR through their public constructors
// (mirroring json_loader.cpp's make_* functions) and exposes C entry points
// used by tests/golden/make_golden.py to produce fixtures.
//
// Ray counting: Scene::intersect / Scene::occluded are wrapped at link time
// (-Wl,--wrap) so that calls from tracer.o and shading.o are counted without
// modifying the reference sources.
#include <cstdint>
#include <map>
#include <memory>
#include <random>
#include <vector>

#include "camera.h"
#include "csg.h"
#include "geometry.h"
#include "scene.h"
#include "tracer.h"
#include "transform.h"

#include "oracle.h"
#include "rt.h"
#include "rt_ref_adapter.hpp"

static uint64_t g_n_isect = 0, g_n_occl = 0;

extern "C" {
bool __real__ZNK5Scene9intersectERK3RayddR3Hit(const Scene* self, const Ray& r, double tmin, double tmax, Hit& out);
bool __real__ZNK5Scene8occludedERK3Raydd(const Scene* self, const Ray& r, double tmin, double tmax);

bool __wrap__ZNK5Scene9intersectERK3RayddR3Hit(const Scene* self, const Ray& r, double tmin, double tmax,
                                               Hit& out) {
    ++g_n_isect;
    return __real__ZNK5Scene9intersectERK3RayddR3Hit(self, r, tmin, tmax, out);
}
bool __wrap__ZNK5Scene8occludedERK3Raydd(const Scene* self, const Ray& r, double tmin, double tmax) {
    ++g_n_occl;
    return __real__ZNK5Scene8occludedERK3Raydd(self, r, tmin, tmax);
}
}

namespace {

struct Built {
    std::vector<std::shared_ptr<Material>> mats;   // IR material index -> reference Material
    std::vector<std::shared_ptr<Primitive>> nodes; // IR node index -> reference Primitive
    std::map<const Material*, int> mat_id;         // reference Material* -> IR index
    Scene scene;
    Camera cam;
};

Material to_ref(const rt_material& m) {
    Material r;
    r.albedo = Color(m.albedo[0], m.albedo[1], m.albedo[2]);
    r.ambient = Color(m.ambient[0], m.ambient[1], m.ambient[2]);
    r.kd = m.kd; r.ks = m.ks; r.kr = m.kr; r.kt = m.kt;
    r.shininess = m.shininess;
    r.refractive_index = m.refractive_index;
    return r;
}

std::shared_ptr<Primitive> build_node(Built& b, const rt_scene_desc* d, int idx) {
    if (b.nodes[idx]) return b.nodes[idx];
    const rt_node& n = d->nodes[idx];
    std::shared_ptr<Primitive> p;
    switch (n.kind) {
        case RT_NODE_SPHERE:
            p = std::make_shared<Sphere>(Point3(n.v[0], n.v[1], n.v[2]), n.v[3], b.mats[n.mat].get());
            break;
        case RT_NODE_HALFSPACE:
            p = std::make_shared<HalfSpace>(Point3(n.v[0], n.v[1], n.v[2]), Dir3(n.aux[0], n.aux[1], n.aux[2]),
                                            b.mats[n.mat].get());
            break;
        case RT_NODE_POKEBALL: {
            auto pb = std::make_shared<Pokeball>(
                Point3(n.v[0], n.v[1], n.v[2]), n.v[3], to_ref(d->materials[n.mats[RT_PB_TOP]]),
                to_ref(d->materials[n.mats[RT_PB_BOTTOM]]), to_ref(d->materials[n.mats[RT_PB_BELT]]),
                to_ref(d->materials[n.mats[RT_PB_RING]]), to_ref(d->materials[n.mats[RT_PB_BUTTON]]), n.v[4], n.v[5],
                n.v[6], Dir3(n.aux[0], n.aux[1], n.aux[2]));
            b.mat_id[&pb->topMat] = n.mats[RT_PB_TOP];
            b.mat_id[&pb->bottomMat] = n.mats[RT_PB_BOTTOM];
            b.mat_id[&pb->beltMat] = n.mats[RT_PB_BELT];
            b.mat_id[&pb->ringMat] = n.mats[RT_PB_RING];
            b.mat_id[&pb->buttonMat] = n.mats[RT_PB_BUTTON];
            p = pb;
            break;
        }
        case RT_NODE_TRANSLATION:
            p = std::make_shared<Translation>(build_node(b, d, n.a), Vec3(n.aux[0], n.aux[1], n.aux[2]));
            break;
        case RT_NODE_SCALING:
            p = std::make_shared<Scaling>(build_node(b, d, n.a), Vec3(n.aux[0], n.aux[1], n.aux[2]));
            break;
        case RT_NODE_ROTATION:
            p = std::make_shared<Rotation>(build_node(b, d, n.a), (Axis)n.op, n.aux[0]);
            break;
        case RT_NODE_CSG: {
            CSGOp op = n.op == RT_CSG_UNION ? CSGOp::Union
                       : n.op == RT_CSG_INTERSECTION ? CSGOp::Intersection : CSGOp::Difference;
            auto A = build_node(b, d, n.a);
            auto B = build_node(b, d, n.b);
            p = std::make_shared<CSG>(op, A, B);
            break;
        }
    }
    b.nodes[idx] = p;
    return p;
}

std::unique_ptr<Built> build(const rt_scene_desc* d) {
    auto b = std::make_unique<Built>();
    for (int i = 0; i < d->n_materials; ++i) {
        b->mats.push_back(std::make_shared<Material>(to_ref(d->materials[i])));
        b->mat_id[b->mats.back().get()] = i;
    }
    b->nodes.resize(d->n_nodes);
    for (int i = 0; i < d->n_objects; ++i) b->scene.objects.push_back(build_node(*b, d, d->objects[i]).get());
    for (int i = 0; i < d->n_lights; ++i) {
        PointLight L;
        L.pos = Point3(d->lights[i].pos[0], d->lights[i].pos[1], d->lights[i].pos[2]);
        L.intensity = Color(d->lights[i].intensity[0], d->lights[i].intensity[1], d->lights[i].intensity[2]);
        b->scene.point_lights.push_back(L);
    }
    for (int i = 0; i < d->n_dir_lights; ++i) {
        DirectionalLight L;
        L.dir = Dir3(d->dir_lights[i].dir[0], d->dir_lights[i].dir[1], d->dir_lights[i].dir[2]);
        L.radiance = Color(d->dir_lights[i].radiance[0], d->dir_lights[i].radiance[1], d->dir_lights[i].radiance[2]);
        b->scene.dir_lights.push_back(L);
    }
    b->scene.background = Color(d->background[0], d->background[1], d->background[2]);
    b->scene.ambient = Color(d->ambient[0], d->ambient[1], d->ambient[2]);
    b->scene.medium_index = d->medium_index;
    b->scene.recursion_limit = d->recursion_limit;
    b->cam.eye = Point3(d->camera.eye[0], d->camera.eye[1], d->camera.eye[2]);
    b->cam.screen.P = Point3(d->camera.P[0], d->camera.P[1], d->camera.P[2]);
    b->cam.screen.Lx = d->camera.Lx;
    b->cam.screen.Ly = d->camera.Ly;
    b->cam.screen.dpi = d->camera.dpi;
    return b;
}

void export_hit(const Built& b, const Hit& h, oracle_hit* o) {
    o->t = h.t;
    o->p[0] = h.p.x; o->p[1] = h.p.y; o->p[2] = h.p.z;
    o->n[0] = h.n.x; o->n[1] = h.n.y; o->n[2] = h.n.z;
    auto it = b.mat_id.find(h.mat);
    o->mat = h.mat ? (it != b.mat_id.end() ? it->second : -2) : -1;
    o->front_face = h.front_face ? 1 : 0;
}

}  // namespace

extern "C" {

// The reference-side binding (integration/rt_ref_adapter.cpp): IR -> the
// reference's own objects -> rtref::scene_from_reference -> a new rt_scene.
// Tests compare it with the input IR (tests/test_ref_adapter.py).
int ref_roundtrip(const rt_scene_desc* d, void** out_scene) {
    auto b = build(d);
    rt_scene* s = nullptr;
    const int rc = rtref::scene_from_reference(b->scene, b->cam, &s);
    *out_scene = s;
    return rc;
}

// Tracer::render (tracer.cpp:247-305) on the full frame.
int ref_render(const rt_scene_desc* d, int W, int H, int mode, double* fb, uint64_t* n_isect, uint64_t* n_occl) {
    auto b = build(d);
    Tracer t;
    t.scene = &b->scene;
    t.camera = &b->cam;
    t.width = W;
    t.height = H;
    t.mode = mode == RT_MODE_PAPER ? RenderMode::Paper : RenderMode::Standard;
    std::vector<Color> out;
    g_n_isect = g_n_occl = 0;
    t.render(out);
    for (size_t i = 0; i < out.size(); ++i) {
        fb[3 * i + 0] = out[i].r;
        fb[3 * i + 1] = out[i].g;
        fb[3 * i + 2] = out[i].b;
    }
    if (n_isect) *n_isect = g_n_isect;
    if (n_occl) *n_occl = g_n_occl;
    return 0;
}

int ref_node_intersect(const rt_scene_desc* d, int node, const double o[3], const double dir[3], double tmin,
                       double tmax, oracle_hit* out) {
    auto b = build(d);
    auto p = build_node(*b, d, node);
    Ray r(Point3(o[0], o[1], o[2]), Dir3(dir[0], dir[1], dir[2]));
    Hit h;
    bool ok = p->intersect(r, tmin, tmax, h);
    export_hit(*b, h, out);
    return ok ? 1 : 0;
}

int ref_node_interval(const rt_scene_desc* d, int node, const double o[3], const double dir[3], double* t0,
                      double* t1, oracle_hit* h0, oracle_hit* h1) {
    auto b = build(d);
    auto p = build_node(*b, d, node);
    Ray r(Point3(o[0], o[1], o[2]), Dir3(dir[0], dir[1], dir[2]));
    Hit a, c;
    double x0 = 0, x1 = 0;
    bool ok = p->interval(r, x0, x1, a, c);
    *t0 = x0;
    *t1 = x1;
    export_hit(*b, a, h0);
    export_hit(*b, c, h1);
    return ok ? 1 : 0;
}

// Batched primitive queries (one scene build for many rays).
int ref_node_intersect_batch(const rt_scene_desc* d, int node, int n, const double* o, const double* dir,
                             double tmin, double tmax, int* ok, oracle_hit* out) {
    auto b = build(d);
    auto p = build_node(*b, d, node);
    for (int i = 0; i < n; ++i) {
        Ray r(Point3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), Dir3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]));
        Hit h;
        ok[i] = p->intersect(r, tmin, tmax, h) ? 1 : 0;
        export_hit(*b, h, &out[i]);
    }
    return 0;
}

int ref_node_interval_batch(const rt_scene_desc* d, int node, int n, const double* o, const double* dir, int* ok,
                            double* t0, double* t1, oracle_hit* h0, oracle_hit* h1) {
    auto b = build(d);
    auto p = build_node(*b, d, node);
    for (int i = 0; i < n; ++i) {
        Ray r(Point3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), Dir3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]));
        Hit a, c;
        double x0 = 0, x1 = 0;
        ok[i] = p->interval(r, x0, x1, a, c) ? 1 : 0;
        t0[i] = x0;
        t1[i] = x1;
        export_hit(*b, a, &h0[i]);
        export_hit(*b, c, &h1[i]);
    }
    return 0;
}

// Camera::generate_ray / generate_ray_subpixel (camera.h:44-78)
void ref_camera_ray(const rt_scene_desc* d, int i, int j, double dx, double dy, int subpixel, double o[3],
                    double dir[3]) {
    auto b = build(d);
    Ray r = subpixel ? b->cam.generate_ray_subpixel(i, j, dx, dy) : b->cam.generate_ray(i, j);
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z;
    dir[0] = r.d.x; dir[1] = r.d.y; dir[2] = r.d.z;
}

// The real libstdc++ jitter stream (tracer.cpp:284-293).
void ref_jitter(uint64_t first, uint64_t count, double* out) {
    std::mt19937 rng(12345);
    std::uniform_real_distribution<double> uni(-0.5, 0.5);
    rng.discard(2 * first);
    for (uint64_t k = 0; k < count; ++k) out[k] = uni(rng);
}

void ref_mt_words(uint64_t first, uint64_t count, uint32_t* out) {
    std::mt19937 rng(12345);
    rng.discard(first);
    for (uint64_t k = 0; k < count; ++k) out[k] = (uint32_t)rng();
}

}  // extern "C"
