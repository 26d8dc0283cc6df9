/*
 * oracle.c — plain-C CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Every function follows the
 * operation order of the reference so that, compiled with gcc -O2 on x86-64
 * without -march (SSE2 doubles, no FMA contraction), results are bit-identical
 * to the reference build in oracle/_ref.  Citations are
 * raytracer/src/<file>:<line> in the reference repository.
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define kEPS 1e-6      /* core.h:10 */
#define kINF INFINITY  /* core.h:12 */

typedef struct { double x, y, z; } V3;
typedef struct { V3 o, d; } Ray;
typedef struct { double t; V3 p; V3 n; int mat; int ff; } Hit;

typedef struct {
    const rt_scene_desc* s;
    oracle_stats st;
} Ctx;

static inline double dmax(double a, double b) { return (a < b) ? b : a; } /* std::max(a,b) */
static inline double dmin(double a, double b) { return (b < a) ? b : a; } /* std::min(a,b) */

static inline V3 v3(double x, double y, double z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline double dot3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* core.h:50 */

/* Dir3::normalized / Vec4::normalized (core.h:58-64, 95-101) */
static inline V3 normalized(V3 v) {
    double L = sqrt(dot3(v, v));
    if (L > kEPS) return v3(v.x / L, v.y / L, v.z / L);
    return v3(0, 1, 0);
}

/* Ray::Ray (core.h:278) */
static inline Ray make_ray(V3 o, V3 d) { Ray r; r.o = o; r.d = normalized(d); return r; }
/* Ray::at (core.h:280) */
static inline V3 ray_at(const Ray* r, double t) {
    return v3(r->o.x + r->d.x * t, r->o.y + r->d.y * t, r->o.z + r->d.z * t);
}

static inline Hit default_hit(void) { /* Hit{} geometry.h:25-35 */
    Hit h;
    h.t = kINF; h.p = v3(0, 0, 0); h.n = v3(0, 1, 0); h.mat = -1; h.ff = 1;
    return h;
}

/* Hit::set_face_normal (geometry.h:42-45) */
static inline void set_face_normal(Hit* h, const Ray* r, V3 outward) {
    h->ff = dot3(r->d, outward) < 0.0;
    h->n = h->ff ? outward : v3(-outward.x, -outward.y, -outward.z);
}

static inline V3 vget(const double* p) { return v3(p[0], p[1], p[2]); }

/* ------------------------------------------------------------ primitives */

/* Sphere::intersect (geometry.cpp:12-37) */
static int sphere_intersect(Ctx* c, V3 cen, double rad, int mat, const Ray* ray, double tmin,
                            double tmax, Hit* out) {
    c->st.ops[RT_OPC_SPHERE_ISECT]++;
    V3 oc = v3(ray->o.x - cen.x, ray->o.y - cen.y, ray->o.z - cen.z);
    double a = 1.0;
    double half_b = dot3(oc, ray->d);
    double cterm = dot3(oc, oc) - rad * rad;
    double disc = half_b * half_b - a * cterm;
    if (disc < 0.0) return 0;
    double sqrtD = sqrt(disc);
    double t = (-half_b - sqrtD) / a;
    if (t < tmin || t > tmax) {
        t = (-half_b + sqrtD) / a;
        if (t < tmin || t > tmax) return 0;
    }
    c->st.ops[RT_OPC_SPHERE_ISECT_HIT]++;
    out->t = t;
    out->p = ray_at(ray, t);
    V3 outward = v3((out->p.x - cen.x) / rad, (out->p.y - cen.y) / rad, (out->p.z - cen.z) / rad);
    set_face_normal(out, ray, outward);
    out->mat = mat;
    return 1;
}

/* Sphere::interval (geometry.cpp:48-78) */
static int sphere_interval(Ctx* c, V3 cen, double r, int mat, const Ray* ray, double* t0, double* t1,
                           Hit* h0, Hit* h1) {
    c->st.ops[RT_OPC_SPHERE_IVL]++;
    V3 oc = v3(ray->o.x - cen.x, ray->o.y - cen.y, ray->o.z - cen.z);
    double a = 1.0;
    double half_b = dot3(oc, ray->d);
    double cterm = dot3(oc, oc) - r * r;
    double disc = half_b * half_b - a * cterm;
    if (disc < 0.0) return 0;
    c->st.ops[RT_OPC_SPHERE_IVL_HIT]++;
    double s = sqrt(disc);
    *t0 = (-half_b - s) / a;
    *t1 = (-half_b + s) / a;
    if (*t0 > *t1) { double tmp = *t0; *t0 = *t1; *t1 = tmp; }
    h0->t = *t0;
    h0->p = ray_at(ray, *t0);
    set_face_normal(h0, ray, v3((h0->p.x - cen.x) / r, (h0->p.y - cen.y) / r, (h0->p.z - cen.z) / r));
    h0->mat = mat;
    h1->t = *t1;
    h1->p = ray_at(ray, *t1);
    set_face_normal(h1, ray, v3((h1->p.x - cen.x) / r, (h1->p.y - cen.y) / r, (h1->p.z - cen.z) / r));
    h1->mat = mat;
    return 1;
}

/* HalfSpace::intersect (geometry.cpp:90-106) */
static int half_intersect(Ctx* c, V3 p0, V3 n, int mat, const Ray* r, double tmin, double tmax, Hit* out) {
    c->st.ops[RT_OPC_HALF_ISECT]++;
    const double ndotd = dot3(n, r->d);
    if (fabs(ndotd) < 1e-12) return 0;
    V3 diff = v3(p0.x - r->o.x, p0.y - r->o.y, p0.z - r->o.z);
    const double t = dot3(n, diff) / ndotd;
    if (t < tmin || t > tmax) return 0;
    c->st.ops[RT_OPC_HALF_ISECT_HIT]++;
    Hit h = default_hit();
    h.t = t;
    h.p = ray_at(r, t);
    set_face_normal(&h, r, n);
    h.mat = mat;
    *out = h;
    return 1;
}

/* HalfSpace::interval (geometry.cpp:117-147) */
static int half_interval(Ctx* c, V3 p0, V3 n, int mat, const Ray* r, double* tE, double* tX, Hit* hE,
                         Hit* hX) {
    c->st.ops[RT_OPC_HALF_IVL]++;
    const double ndotd = dot3(n, r->d);
    V3 diff = v3(r->o.x - p0.x, r->o.y - p0.y, r->o.z - p0.z);
    const double f0 = dot3(n, diff);
    if (fabs(ndotd) < 1e-12) {
        if (f0 >= 0.0) {
            *tE = -kINF; *tX = kINF;
            hE->t = *tE; hE->p = r->o; set_face_normal(hE, r, n); hE->mat = mat;
            hX->t = *tX; hX->p = r->o; set_face_normal(hX, r, n); hX->mat = mat;
            return 1;
        }
        return 0;
    }
    const double tPlane = -f0 / ndotd;
    if (ndotd > 0.0) {
        *tE = tPlane; *tX = kINF;
        hE->t = *tE; hE->p = ray_at(r, *tE); set_face_normal(hE, r, n); hE->mat = mat;
        hX->t = *tX; hX->p = r->o; set_face_normal(hX, r, n); hX->mat = mat;
    } else {
        *tE = -kINF; *tX = tPlane;
        hE->t = *tE; hE->p = r->o; set_face_normal(hE, r, n); hE->mat = mat;
        hX->t = *tX; hX->p = ray_at(r, *tX); set_face_normal(hX, r, n); hX->mat = mat;
    }
    return 1;
}

static inline double clamp1(double x) { /* geometry.cpp:152-156 */
    if (x < -1.0) return -1.0;
    if (x > 1.0) return 1.0;
    return x;
}

/* Pokeball::pick_region_material (geometry.cpp:163-180) */
static int pick_region(Ctx* c, const rt_node* nd, V3 p) {
    c->st.ops[RT_OPC_POKE_REGION]++;
    const double* v = nd->v;
    double r = v[3];
    V3 u = v3((p.x - v[0]) / r, (p.y - v[1]) / r, (p.z - v[2]) / r);
    const double ang = acos(clamp1(dot3(u, v3(v[7], v[8], v[9]))));
    const double inner = dmax(0.0, v[5] - v[6]);
    if (ang <= v[5]) {
        if (ang >= inner) return nd->mats[RT_PB_RING];
        return nd->mats[RT_PB_BUTTON];
    }
    if (fabs(u.y) <= v[4]) return nd->mats[RT_PB_BELT];
    return (u.y >= 0.0) ? nd->mats[RT_PB_TOP] : nd->mats[RT_PB_BOTTOM];
}

/* Transform::project_t_world (transform.h:76-80) */
static inline double project_t_world(const Ray* r, V3 Pw) {
    V3 v = v3(Pw.x - r->o.x, Pw.y - r->o.y, Pw.z - r->o.z);
    const double dd = r->d.x * r->d.x + r->d.y * r->d.y + r->d.z * r->d.z;
    return dd > 0.0 ? (v.x * r->d.x + v.y * r->d.y + v.z * r->d.z) / dd : kINF;
}

/* Matrix4 * Vec4 (core.h:169-176), rows 0..2 of a 3x4 block */
static inline V3 mat_apply(const double* m, V3 v, double w) {
    return v3(m[0] * v.x + m[1] * v.y + m[2] * v.z + m[3] * w,
              m[4] * v.x + m[5] * v.y + m[6] * v.z + m[7] * w,
              m[8] * v.x + m[9] * v.y + m[10] * v.z + m[11] * w);
}

static int node_intersect(Ctx* c, int idx, const Ray* r, double tmin, double tmax, Hit* out);
static int node_interval(Ctx* c, int idx, const Ray* r, double* t0, double* t1, Hit* h0, Hit* h1);

/* Local ray of a transform node, or 0 when Scaling rejects (transform.cpp). */
static int local_ray(Ctx* c, const rt_node* nd, const Ray* r, Ray* out) {
    c->st.ops[RT_OPC_XFORM]++;
    const double* M = nd->v;
    const double* I = nd->v + 12;
    if (nd->kind == RT_NODE_TRANSLATION) {   /* transform.cpp:24-29 */
        V3 lo = v3(r->o.x - M[3], r->o.y - M[7], r->o.z - M[11]);
        *out = make_ray(lo, r->d);
        return 1;
    }
    if (nd->kind == RT_NODE_SCALING) {       /* transform.cpp:97-111 */
        double sx = M[0], sy = M[5], sz = M[10];
        if (fabs(sx) < kEPS || fabs(sy) < kEPS || fabs(sz) < kEPS) return 0;
        V3 lo = v3(r->o.x / sx, r->o.y / sy, r->o.z / sz);
        V3 ld = v3(r->d.x / sx, r->d.y / sy, r->d.z / sz);
        *out = make_ray(lo, ld);
        return 1;
    }
    /* Rotation (transform.cpp:184-196) */
    V3 lo = mat_apply(I, r->o, 1.0);
    V3 ld = mat_apply(I, r->d, 0.0);
    *out = make_ray(lo, ld);
    return 1;
}

/* Map a child hit point / normal back to world space; returns the world normal
 * BEFORE set_face_normal (translation: unchanged; scaling/rotation: normalised). */
static inline V3 map_point(const rt_node* nd, V3 p) {
    const double* M = nd->v;
    if (nd->kind == RT_NODE_TRANSLATION) return v3(p.x + M[3], p.y + M[7], p.z + M[11]);
    if (nd->kind == RT_NODE_SCALING) return v3(p.x * M[0], p.y * M[5], p.z * M[10]);
    return mat_apply(M, p, 1.0);
}
static inline V3 map_normal(const rt_node* nd, V3 n) {
    const double* M = nd->v;
    if (nd->kind == RT_NODE_TRANSLATION) return n;
    if (nd->kind == RT_NODE_SCALING) return normalized(v3(n.x / M[0], n.y / M[5], n.z / M[10]));
    return normalized(mat_apply(M, n, 0.0));
}

/* Translation/Scaling/Rotation::intersect (transform.cpp:18-44, 95-127, 182-213) */
static int xform_intersect(Ctx* c, const rt_node* nd, const Ray* r, double tmin, double tmax, Hit* out) {
    Ray lr;
    if (!local_ray(c, nd, r, &lr)) return 0;
    Hit h = default_hit();
    if (!node_intersect(c, nd->a, &lr, 0.0, kINF, &h)) return 0;
    V3 wp = map_point(nd, h.p);
    V3 wn = map_normal(nd, h.n);
    double wt = project_t_world(r, wp);
    if (!(wt > tmin && wt < tmax)) return 0;
    *out = h;
    out->p = wp;
    set_face_normal(out, r, wn);
    out->t = wt;
    return 1;
}

/* Translation/Scaling/Rotation::interval (transform.cpp:55-82, 138-169, 224-255) */
static int xform_interval(Ctx* c, const rt_node* nd, const Ray* r, double* tE, double* tX, Hit* hE,
                          Hit* hX) {
    Ray lr;
    if (!local_ray(c, nd, r, &lr)) return 0;
    if (!node_interval(c, nd->a, &lr, tE, tX, hE, hX)) return 0;
    hE->p = map_point(nd, hE->p);
    hX->p = map_point(nd, hX->p);
    V3 nE = map_normal(nd, hE->n);
    V3 nX = map_normal(nd, hX->n);
    set_face_normal(hE, r, nE);
    set_face_normal(hX, r, nX);
    *tE = project_t_world(r, hE->p);
    *tX = project_t_world(r, hX->p);
    return 1;
}

/* ------------------------------------------------------------------ CSG */
typedef struct { double t; int type; int who; Hit h; } Ev;   /* csg.cpp:79; type 0 Enter, 1 Exit */

/* event_less lambda (csg.cpp:87-92) */
static inline int event_less(const Ev* a, const Ev* b) {
    if (fabs(a->t - b->t) > 1e-6) return a->t < b->t;
    if (a->type != b->type) return a->type == 0;
    return a->who < b->who;
}

/* libstdc++ std::sort on <= 16 elements = __insertion_sort
 * (/usr/include/c++/11/bits/stl_algo.h:1819-1871). */
static void sort_events(Ev* ev, int n) {
    for (int i = 1; i < n; ++i) {
        if (event_less(&ev[i], &ev[0])) {
            Ev val = ev[i];
            for (int k = i; k > 0; --k) ev[k] = ev[k - 1];
            ev[0] = val;
        } else {
            Ev val = ev[i];
            int last = i, next = i - 1;
            while (event_less(&val, &ev[next])) {
                ev[last] = ev[next];
                last = next;
                --next;
            }
            ev[last] = val;
        }
    }
}

static inline int csg_combine(int op, int a, int b) {
    switch (op) {
        case RT_CSG_UNION: return a || b;
        case RT_CSG_INTERSECTION: return a && b;
        case RT_CSG_DIFFERENCE: return a && !b;
    }
    return 0;
}

/* CSG::interval (csg.cpp:61-163) */
static int csg_interval(Ctx* c, const rt_node* nd, const Ray* ray, double* tEnter, double* tExit,
                        Hit* enterHit, Hit* exitHit) {
    double ta0 = 0, ta1 = 0, tb0 = 0, tb1 = 0;
    Hit ha0 = default_hit(), ha1 = default_hit(), hb0 = default_hit(), hb1 = default_hit();
    const int hitA = node_interval(c, nd->a, ray, &ta0, &ta1, &ha0, &ha1);
    const int hitB = node_interval(c, nd->b, ray, &tb0, &tb1, &hb0, &hb1);
    if (!hitA && !hitB) return 0;
    c->st.ops[RT_OPC_CSG_COMBINE]++;

    Ev ev[4];
    int n = 0;
#define ADD(T, TY, WHO, H) do { if (isfinite(T)) { ev[n].t = (T); ev[n].type = (TY); ev[n].who = (WHO); ev[n].h = (H); ++n; } } while (0)
    if (hitA) { ADD(ta0, 0, 0, ha0); ADD(ta1, 1, 0, ha1); }
    if (hitB) { ADD(tb0, 0, 1, hb0); ADD(tb1, 1, 1, hb1); }
#undef ADD
    sort_events(ev, n);

    int inA = hitA && ((ta0 < 1e-6) && (ta1 > 1e-6));
    int inB = hitB && ((tb0 < 1e-6) && (tb1 > 1e-6));
    const int op = nd->op;
    int inR = csg_combine(op, inA, inB);

    int haveEnter = 0;
    Hit hEnter = default_hit(), hExit = default_hit();
    double tEnt = 0.0, tExt = kINF;
    if (inR) {
        haveEnter = 1;
        tEnt = 0.0;
        hEnter.t = 0.0;
        hEnter.p = ray->o;
        hEnter.n = v3(0, 0, 0);
        hEnter.mat = (inA && ha0.mat >= 0) ? ha0.mat : (inB ? hb0.mat : -1);
        hEnter.ff = 1;
    }
    for (int k = 0; k < n; ++k) {
        const Ev* e = &ev[k];
        const int before = inR;
        if (e->who == 0) inA = (e->type == 0);
        else inB = (e->type == 0);
        const int after = csg_combine(op, inA, inB);
        if (!before && after) {
            haveEnter = 1;
            tEnt = e->t;
            hEnter = e->h;
            if (op == RT_CSG_DIFFERENCE && e->who == 1 && e->type == 1)
                set_face_normal(&hEnter, ray, v3(-e->h.n.x, -e->h.n.y, -e->h.n.z));
        } else if (before && !after) {
            tExt = e->t;
            hExit = e->h;
            if (op == RT_CSG_DIFFERENCE && e->who == 1 && e->type == 0)
                set_face_normal(&hExit, ray, v3(-e->h.n.x, -e->h.n.y, -e->h.n.z));
            break;
        }
        inR = after;
    }
    if (!haveEnter || !isfinite(tExt)) return 0;
    *tEnter = tEnt;
    *tExit = tExt;
    *enterHit = hEnter;
    *exitHit = hExit;
    return 1;
}

/* CSG::intersect (csg.cpp:169-185) */
static int csg_intersect(Ctx* c, const rt_node* nd, const Ray* r, double tmin, double tmax, Hit* out) {
    double tEnter, tExit;
    Hit hEnter = default_hit(), hExit = default_hit();
    if (!csg_interval(c, nd, r, &tEnter, &tExit, &hEnter, &hExit)) return 0;
    const double t = dmax(tEnter, tmin);
    if (!(t < tExit && t < tmax)) return 0;
    *out = hEnter;
    out->t = t;
    out->p = v3(r->o.x + r->d.x * t, r->o.y + r->d.y * t, r->o.z + r->d.z * t);
    return 1;
}

/* --------------------------------------------------------- dispatch */
static int node_intersect(Ctx* c, int idx, const Ray* r, double tmin, double tmax, Hit* out) {
    const rt_node* nd = &c->s->nodes[idx];
    switch (nd->kind) {
        case RT_NODE_SPHERE:
            return sphere_intersect(c, vget(nd->v), nd->v[3], nd->mat, r, tmin, tmax, out);
        case RT_NODE_HALFSPACE:
            return half_intersect(c, vget(nd->v), vget(nd->v + 3), nd->mat, r, tmin, tmax, out);
        case RT_NODE_POKEBALL:   /* geometry.cpp:190-197 (Sphere base has mat=nullptr) */
            if (!sphere_intersect(c, vget(nd->v), nd->v[3], -1, r, tmin, tmax, out)) return 0;
            out->mat = pick_region(c, nd, out->p);
            return 1;
        case RT_NODE_TRANSLATION:
        case RT_NODE_SCALING:
        case RT_NODE_ROTATION:
            return xform_intersect(c, nd, r, tmin, tmax, out);
        case RT_NODE_CSG:
            return csg_intersect(c, nd, r, tmin, tmax, out);
    }
    return 0;
}

static int node_interval(Ctx* c, int idx, const Ray* r, double* t0, double* t1, Hit* h0, Hit* h1) {
    const rt_node* nd = &c->s->nodes[idx];
    switch (nd->kind) {
        case RT_NODE_SPHERE:
            return sphere_interval(c, vget(nd->v), nd->v[3], nd->mat, r, t0, t1, h0, h1);
        case RT_NODE_HALFSPACE:
            return half_interval(c, vget(nd->v), vget(nd->v + 3), nd->mat, r, t0, t1, h0, h1);
        case RT_NODE_POKEBALL:   /* geometry.cpp:207-217 */
            if (!sphere_interval(c, vget(nd->v), nd->v[3], -1, r, t0, t1, h0, h1)) return 0;
            h0->mat = pick_region(c, nd, h0->p);
            h1->mat = pick_region(c, nd, h1->p);
            return 1;
        case RT_NODE_TRANSLATION:
        case RT_NODE_SCALING:
        case RT_NODE_ROTATION:
            return xform_interval(c, nd, r, t0, t1, h0, h1);
        case RT_NODE_CSG:
            return csg_interval(c, nd, r, t0, t1, h0, h1);
    }
    return 0;
}

/* ---------------------------------------------------------------- scene */
/* Scene::intersect (scene.cpp:10-24) */
static int scene_intersect(Ctx* c, const Ray* r, double tmin, double tmax, Hit* out) {
    c->st.rays_intersect++;
    Hit temp = default_hit();
    int hit_any = 0;
    double closest_t = tmax;
    for (int i = 0; i < c->s->n_objects; ++i) {
        if (node_intersect(c, c->s->objects[i], r, tmin, closest_t, &temp)) {
            hit_any = 1;
            closest_t = temp.t;
            *out = temp;
        }
    }
    return hit_any;
}

/* Scene::occluded (scene.cpp:33-42) */
static int scene_occluded(Ctx* c, const Ray* r, double tmin, double tmax) {
    c->st.rays_occluded++;
    Hit tmp = default_hit();
    for (int i = 0; i < c->s->n_objects; ++i)
        if (node_intersect(c, c->s->objects[i], r, tmin, tmax, &tmp)) return 1;
    return 0;
}

/* combine (shading.cpp:6-12) */
static inline V3 combine(V3 a, V3 b) {
    return v3(1.0 - (1.0 - a.x) * (1.0 - b.x), 1.0 - (1.0 - a.y) * (1.0 - b.y), 1.0 - (1.0 - a.z) * (1.0 - b.z));
}

/* shade_lambert_phong (shading.cpp:31-138): directional lights (:45-76,
 * reachable through rt_scene_from_desc only) then point lights (:79-130). */
static V3 shade(Ctx* c, const Hit* hit, V3 wo) {
    if (hit->mat < 0) return v3(1, 0, 1);
    const rt_scene_desc* s = c->s;
    c->st.ops[RT_OPC_SHADE_CALL]++;
    const rt_material* m = &s->materials[hit->mat];
    const V3 n = hit->n;
    V3 E_total = v3(m->ambient[0] * s->ambient[0], m->ambient[1] * s->ambient[1], m->ambient[2] * s->ambient[2]);
    const double shadow_epsilon = dmax(1e-3, 1e-4 * hit->t);
    for (int li = 0; li < s->n_dir_lights; ++li) {
        const rt_dir_light* L = &s->dir_lights[li];
        c->st.ops[RT_OPC_LIGHT_EVAL]++;
        V3 wi = normalized(v3(-L->dir[0], -L->dir[1], -L->dir[2]));   /* (-light.dir).normalized() */
        double ndotl = dmax(0.0, dot3(n, wi));
        if (ndotl <= 0.0) continue;
        V3 so = v3(hit->p.x + n.x * shadow_epsilon, hit->p.y + n.y * shadow_epsilon, hit->p.z + n.z * shadow_epsilon);
        Ray sr = make_ray(so, wi);
        if (scene_occluded(c, &sr, shadow_epsilon, INFINITY)) continue;
        c->st.ops[RT_OPC_SHADE_LIGHT]++;
        /* scale(mul(albedo, radiance), kd * ndotl) */
        double sd = m->kd * ndotl;
        V3 E_d = v3(m->albedo[0] * L->radiance[0] * sd, m->albedo[1] * L->radiance[1] * sd,
                    m->albedo[2] * L->radiance[2] * sd);
        V3 E_s = v3(0, 0, 0);
        if (m->ks > 0.0) {
            c->st.ops[RT_OPC_SHADE_SPEC]++;
            V3 rr = normalized(v3(2.0 * dot3(n, wi) * n.x - wi.x, 2.0 * dot3(n, wi) * n.y - wi.y,
                                  2.0 * dot3(n, wi) * n.z - wi.z));
            double rdotv = dmax(0.0, dot3(rr, wo));
            double spec = pow(rdotv, m->shininess) * m->ks;
            E_s = v3(L->radiance[0] * spec, L->radiance[1] * spec, L->radiance[2] * spec);
        }
        E_total = combine(E_total, combine(E_d, E_s));
    }
    for (int li = 0; li < s->n_lights; ++li) {
        const rt_light* L = &s->lights[li];
        c->st.ops[RT_OPC_LIGHT_EVAL]++;
        V3 to_light = v3(L->pos[0] - hit->p.x, L->pos[1] - hit->p.y, L->pos[2] - hit->p.z);
        double dist_squared = dot3(to_light, to_light);
        if (dist_squared <= 0.01) dist_squared = 0.01;
        double distance = sqrt(dist_squared);
        V3 wi = v3(to_light.x / distance, to_light.y / distance, to_light.z / distance);
        double ndotl = dmax(0.0, dot3(n, wi));
        if (ndotl <= 0.0) continue;
        double max_shadow_t = distance - shadow_epsilon;
        if (max_shadow_t <= shadow_epsilon) continue;
        V3 so = v3(hit->p.x + n.x * shadow_epsilon, hit->p.y + n.y * shadow_epsilon, hit->p.z + n.z * shadow_epsilon);
        Ray sr = make_ray(so, wi);
        if (scene_occluded(c, &sr, shadow_epsilon, max_shadow_t)) continue;
        c->st.ops[RT_OPC_SHADE_LIGHT]++;
        double effective_dist = dmax(0.5, distance);
        double falloff = 1.0 / (effective_dist * effective_dist);
        double f2 = falloff * 2.0;
        V3 I_L = v3(L->intensity[0] * f2, L->intensity[1] * f2, L->intensity[2] * f2);
        double sd = m->kd * ndotl * 1.5;
        V3 E_d = v3(m->albedo[0] * I_L.x * sd, m->albedo[1] * I_L.y * sd, m->albedo[2] * I_L.z * sd);
        V3 E_s = v3(0, 0, 0);
        if (m->ks > 0.0) {
            c->st.ops[RT_OPC_SHADE_SPEC]++;
            V3 rr = normalized(v3(2.0 * dot3(n, wi) * n.x - wi.x, 2.0 * dot3(n, wi) * n.y - wi.y,
                                  2.0 * dot3(n, wi) * n.z - wi.z));
            double rdotv = dmax(0.0, dot3(rr, wo));
            double spec = pow(rdotv, m->shininess) * m->ks;
            E_s = v3(I_L.x * spec, I_L.y * spec, I_L.z * spec);
        }
        V3 E_light = combine(E_d, E_s);
        E_total = combine(E_total, E_light);
    }
    E_total.x = dmin(1.5, E_total.x);
    E_total.y = dmin(1.5, E_total.y);
    E_total.z = dmin(1.5, E_total.z);
    return E_total;
}

/* Tracer::trace_recursive (tracer.cpp:22-73) */
static V3 trace_recursive(Ctx* c, const Ray* r, int depth) {
    const rt_scene_desc* s = c->s;
    if (depth >= s->recursion_limit) return v3(0, 0, 0);
    Hit h = default_hit();
    if (scene_intersect(c, r, 1e-4, kINF, &h)) {
        V3 wo = normalized(v3(-r->d.x, -r->d.y, -r->d.z));
        V3 direct = shade(c, &h, wo);
        if (h.mat < 0) return direct;
        const rt_material* mat = &s->materials[h.mat];
        V3 total = direct;
        if (mat->kr > 0.0 && depth < s->recursion_limit - 1) {
            c->st.ops[RT_OPC_SECONDARY]++;
            V3 incident = normalized(r->d);
            double k = 2.0 * dot3(incident, h.n);   /* reflect (tracer.cpp:76-78) */
            V3 refl = normalized(v3(incident.x - h.n.x * k, incident.y - h.n.y * k, incident.z - h.n.z * k));
            V3 ro = h.ff ? v3(h.p.x + h.n.x * 1e-6, h.p.y + h.n.y * 1e-6, h.p.z + h.n.z * 1e-6)
                         : v3(h.p.x - h.n.x * 1e-6, h.p.y - h.n.y * 1e-6, h.p.z - h.n.z * 1e-6);
            Ray rr = make_ray(ro, refl);
            V3 Ir = trace_recursive(c, &rr, depth + 1);
            total = combine(total, v3(Ir.x * mat->kr, Ir.y * mat->kr, Ir.z * mat->kr));
        }
        if (mat->kt > 0.0 && depth < s->recursion_limit - 1) {
            double eta = h.ff ? (s->medium_index / mat->refractive_index) : (mat->refractive_index / s->medium_index);
            V3 incident = normalized(r->d);
            double cos_i = -dot3(incident, h.n);   /* has_total_internal_reflection (tracer.cpp:100-104) */
            double sin_t2 = eta * eta * dmax(0.0, 1.0 - cos_i * cos_i);
            if (!(sin_t2 >= 1.0)) {
                c->st.ops[RT_OPC_SECONDARY]++;
                /* refract (tracer.cpp:87-98) */
                double ci = -dot3(incident, h.n);
                double st2 = eta * eta * dmax(0.0, 1.0 - ci * ci);
                V3 rd;
                if (st2 >= 1.0) {
                    rd = v3(0, 0, 0);
                } else {
                    double cos_t = sqrt(1.0 - st2);
                    double k = eta * ci - cos_t;
                    rd = v3(incident.x * eta + h.n.x * k, incident.y * eta + h.n.y * k, incident.z * eta + h.n.z * k);
                }
                V3 refr = normalized(rd);
                V3 ro = h.ff ? v3(h.p.x - h.n.x * 1e-6, h.p.y - h.n.y * 1e-6, h.p.z - h.n.z * 1e-6)
                             : v3(h.p.x + h.n.x * 1e-6, h.p.y + h.n.y * 1e-6, h.p.z + h.n.z * 1e-6);
                Ray tr = make_ray(ro, refr);
                V3 It = trace_recursive(c, &tr, depth + 1);
                total = combine(total, v3(It.x * mat->kt, It.y * mat->kt, It.z * mat->kt));
            }
        }
        return total;
    }
    return v3(s->background[0], s->background[1], s->background[2]);
}

/* ---------------------------------------------------------------- camera */
static int cam_nx(const rt_camera* c) { int n = (int)round(c->Lx * c->dpi); return n > 1 ? n : 1; }
static int cam_ny(const rt_camera* c) { int n = (int)round(c->Ly * c->dpi); return n > 1 ? n : 1; }

/* Camera::generate_ray (camera.h:44-58) */
static Ray generate_ray(const rt_camera* cam, int i, int j) {
    const int nx = cam_nx(cam), ny = cam_ny(cam);
    V3 eye = vget(cam->eye);
    if (i < 0 || i >= nx || j < 0 || j >= ny) return make_ray(eye, v3(0, 0, -1));
    const double sx = ((double)i + 0.5) / (double)nx;
    const int jf = ny - 1 - j;
    const double sy = ((double)jf + 0.5) / (double)ny;
    /* U = (Lx,0,0), V = (0,Ly,0) (camera.h:23-25) */
    V3 S = v3(cam->P[0] + cam->Lx * sx + 0.0 * sy, cam->P[1] + 0.0 * sx + cam->Ly * sy,
              cam->P[2] + 0.0 * sx + 0.0 * sy);
    V3 d = normalized(v3(S.x - eye.x, S.y - eye.y, S.z - eye.z));
    return make_ray(eye, d);
}

/* Camera::generate_ray_subpixel (camera.h:68-78) */
static Ray generate_ray_subpixel(const rt_camera* cam, int i, int j, double dx, double dy) {
    const int nx = cam_nx(cam), ny = cam_ny(cam);
    V3 eye = vget(cam->eye);
    const double sx = (i + 0.5 + dx) / (double)nx;
    const double sy = (j + 0.5 + dy) / (double)ny;
    V3 S = v3(cam->P[0] + cam->Lx * sx + 0.0 * sy, cam->P[1] + 0.0 * sx + cam->Ly * sy,
              cam->P[2] + 0.0 * sx + 0.0 * sy);
    V3 d = normalized(v3(S.x - eye.x, S.y - eye.y, S.z - eye.z));
    return make_ray(eye, d);
}

/* --------------------------------------------------------------- mt19937 */
typedef struct { uint32_t mt[624]; int idx; } MT;

static void mt_seed(MT* g, uint32_t s) {
    g->mt[0] = s;
    for (int i = 1; i < 624; ++i) g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
    g->idx = 624;
}

static void mt_twist(MT* g) {   /* libstdc++ mersenne_twister_engine::_M_gen_rand */
    const uint32_t UM = 0x80000000u, LM = 0x7fffffffu, A = 0x9908b0dfu;
    uint32_t* mt = g->mt;
    for (int k = 0; k < 624 - 397; ++k) {
        uint32_t y = (mt[k] & UM) | (mt[k + 1] & LM);
        mt[k] = mt[k + 397] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    }
    for (int k = 624 - 397; k < 623; ++k) {
        uint32_t y = (mt[k] & UM) | (mt[k + 1] & LM);
        mt[k] = mt[k + (397 - 624)] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    }
    uint32_t y = (mt[623] & UM) | (mt[0] & LM);
    mt[623] = mt[396] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    g->idx = 0;
}

static inline uint32_t mt_next(MT* g) {
    if (g->idx >= 624) mt_twist(g);
    uint32_t y = g->mt[g->idx++];
    y ^= (y >> 11) & 0xffffffffu;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

static void mt_discard(MT* g, uint64_t n) {
    while (n > 0) {
        if (g->idx >= 624) mt_twist(g);
        uint64_t avail = (uint64_t)(624 - g->idx);
        uint64_t take = n < avail ? n : avail;
        g->idx += (int)take;
        n -= take;
    }
}

/* uniform_real_distribution<double>(-0.5,0.5)(rng) (random.h:1870) over
 * generate_canonical<double,53> (random.tcc:3348-3378). */
static inline double uni(MT* g) {
    double sum = 0.0, tmp = 1.0;
    sum += (double)mt_next(g) * tmp;
    tmp *= 4294967296.0;
    sum += (double)mt_next(g) * tmp;
    tmp *= 4294967296.0;
    double ret = sum / tmp;
    if (ret >= 1.0) ret = nextafter(1.0, 0.0);
    return (ret * (0.5 - -0.5)) + -0.5;
}

/* ---------------------------------------------------------------- paper */
static double get_luminance(V3 c) { return 0.299 * c.x + 0.587 * c.y + 0.114 * c.z; }

/* Tracer::get_edge_strength (tracer.cpp:133-178) */
static double edge_strength(Ctx* c, int W, int H, int x, int y) {
    const rt_camera* cam = &c->s->camera;
    const double epsilon = 1e-4;
    Ray center = generate_ray(cam, x, y);
    Hit ch = default_hit();
    int centerHits = scene_intersect(c, &center, epsilon, kINF, &ch);
    static const int dxs[4] = {-1, 1, 0, 0};
    static const int dys[4] = {0, 0, -1, 1};
    double maxEdge = 0.0;
    int valid = 0;
    for (int i = 0; i < 4; ++i) {
        int nx = x + dxs[i], ny = y + dys[i];
        if (nx < 0 || nx >= W || ny < 0 || ny >= H) continue;
        valid++;
        Ray nr = generate_ray(cam, nx, ny);
        Hit nh = default_hit();
        int nHits = scene_intersect(c, &nr, epsilon, kINF, &nh);
        if (centerHits != nHits) { maxEdge = dmax(maxEdge, 0.9); continue; }
        if (centerHits && nHits) {
            double minD = dmin(ch.t, nh.t), maxD = dmax(ch.t, nh.t);
            if (minD > 1e-4 && maxD / minD > 3.0) maxEdge = dmax(maxEdge, 0.6);
            double nd = dot3(ch.n, nh.n);
            if (nd < 0.2) maxEdge = dmax(maxEdge, 0.5);
            if (ch.mat != nh.mat && nd < 0.7) maxEdge = dmax(maxEdge, 0.3);
        }
    }
    if (valid < 4) maxEdge *= 0.5;
    return maxEdge;
}

/* Tracer::apply_crosshatch (tracer.cpp:188-205); C '%' truncates like C++. */
static double crosshatch(double lum, int x, int y) {
    if (lum < 0.15) return 0.0;
    double darkness = 1.0 - lum;
    int diag1 = ((x + y) % 4) < 1;
    int diag2 = ((x - y) % 4) < 1;
    int horizontal = (y % 4) < 1;
    int draw = 0;
    if (darkness > 0.8) draw = (diag1 && diag2) || horizontal;
    else if (darkness > 0.65) draw = (diag1 && diag2) || (horizontal && ((x + y) % 3 == 0));
    else if (darkness > 0.5) draw = (diag1 && diag2) || (horizontal && ((x + y) % 4 == 0));
    else if (darkness > 0.35) draw = diag1 || (horizontal && ((x + y) % 3 == 0));
    else if (darkness > 0.2) draw = diag1;
    else if (darkness > 0.12) draw = diag1 && ((x + y) % 8) < 2;
    return draw ? 0.0 : 1.0;
}

static void paper_pixel(Ctx* c, int W, int H, int x, int y, double* out) {
    const rt_scene_desc* s = c->s;
    Ray r = generate_ray(&s->camera, x, y);
    V3 base;
    Hit h = default_hit();   /* trace_paper (tracer.cpp:111-120) */
    if (scene_intersect(c, &r, 1e-4, kINF, &h)) {
        V3 wo = normalized(v3(-r.d.x, -r.d.y, -r.d.z));
        base = shade(c, &h, wo);
    } else {
        base = v3(1, 1, 1);
    }
    double L = get_luminance(base);
    double edge = edge_strength(c, W, H, x, y);
    double o;
    V3 ov;
    if (edge > 0.8) ov = v3(0, 0, 0);
    else if (edge > 0.5) ov = v3(0.2, 0.2, 0.2);
    else {
        o = crosshatch(L, x, y);
        ov = v3(o, o, o);
        if (edge > 0.3) {
            double darken = (edge - 0.3) * 0.4;
            ov.x *= (1.0 - darken);
            ov.y *= (1.0 - darken);
            ov.z *= (1.0 - darken);
        }
    }
    out[0] = ov.x; out[1] = ov.y; out[2] = ov.z;
}

/* --------------------------------------------------------------- render */
typedef struct {
    const rt_scene_desc* s;
    int W, H, mode;
    int row0, row1;   /* output rows handled by this job */
    int out_row0;     /* first output row of the whole call */
    double* fb;       /* base of the call's buffer */
    oracle_stats st;
} Job;

static void* run_job(void* arg) {
    Job* j = (Job*)arg;
    Ctx c;
    memset(&c, 0, sizeof(c));
    c.s = j->s;
    const int W = j->W, H = j->H;
    if (j->mode == RT_MODE_PAPER) {
        for (int y = j->row0; y < j->row1; ++y)
            for (int x = 0; x < W; ++x)
                paper_pixel(&c, W, H, x, y, j->fb + ((size_t)(y - j->out_row0) * W + x) * 3);
    } else {
        /* output row r <-> loop row yl = H-1-r (tracer.cpp:297).  Iterate loop
         * rows ascending to consume the stream in order. */
        const int yl0 = H - j->row1, yl1 = H - j->row0;
        MT g;
        mt_seed(&g, 12345u);
        mt_discard(&g, (uint64_t)32 * (uint64_t)W * (uint64_t)yl0);
        for (int y = yl0; y < yl1; ++y) {
            for (int x = 0; x < W; ++x) {
                V3 acc = v3(0, 0, 0);
                for (int sidx = 0; sidx < 8; ++sidx) {
                    double dx = uni(&g);
                    double dy = uni(&g);
                    Ray r = generate_ray_subpixel(&c.s->camera, x, y, dx, dy);
                    V3 col = trace_recursive(&c, &r, 0);
                    acc.x += col.x; acc.y += col.y; acc.z += col.z;
                }
                const double inv = 1.0 / (double)8;
                acc.x *= inv; acc.y *= inv; acc.z *= inv;
                const int yy = H - 1 - y;
                double* o = j->fb + ((size_t)(yy - j->out_row0) * W + x) * 3;
                o[0] = acc.x; o[1] = acc.y; o[2] = acc.z;
            }
        }
    }
    j->st = c.st;
    return NULL;
}

int oracle_render_rows(const rt_scene_desc* d, int W, int H, int mode, int row0, int row1, double* fb,
                       oracle_stats* st, int n_threads) {
    if (!d || !fb || W <= 0 || H <= 0 || row0 < 0 || row1 > H || row0 > row1) return -1;
    if (n_threads < 1) n_threads = 1;
    int rows = row1 - row0;
    if (n_threads > rows) n_threads = rows > 0 ? rows : 1;
    Job* jobs = (Job*)calloc((size_t)n_threads, sizeof(Job));
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -1; }
    for (int t = 0; t < n_threads; ++t) {
        jobs[t].s = d; jobs[t].W = W; jobs[t].H = H; jobs[t].mode = mode;
        jobs[t].row0 = row0 + (int)((long long)rows * t / n_threads);
        jobs[t].row1 = row0 + (int)((long long)rows * (t + 1) / n_threads);
        jobs[t].out_row0 = row0;
        jobs[t].fb = fb;
    }
    if (n_threads == 1) {
        run_job(&jobs[0]);
    } else {
        for (int t = 0; t < n_threads; ++t) pthread_create(&th[t], NULL, run_job, &jobs[t]);
        for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    }
    if (st) {
        memset(st, 0, sizeof(*st));
        for (int t = 0; t < n_threads; ++t) {
            st->rays_intersect += jobs[t].st.rays_intersect;
            st->rays_occluded += jobs[t].st.rays_occluded;
            for (int k = 0; k < 16; ++k) st->ops[k] += jobs[t].st.ops[k];
        }
    }
    free(jobs);
    free(th);
    return 0;
}

/* ------------------------------------------------------------- KAT API */
static void export_hit(const Hit* h, oracle_hit* o) {
    o->t = h->t;
    o->p[0] = h->p.x; o->p[1] = h->p.y; o->p[2] = h->p.z;
    o->n[0] = h->n.x; o->n[1] = h->n.y; o->n[2] = h->n.z;
    o->mat = h->mat;
    o->front_face = h->ff;
}

int oracle_node_intersect(const rt_scene_desc* d, int node, const double o[3], const double dir[3], double tmin,
                          double tmax, oracle_hit* out) {
    Ctx c; memset(&c, 0, sizeof(c)); c.s = d;
    Ray r = make_ray(vget(o), vget(dir));
    Hit h = default_hit();
    int ok = node_intersect(&c, node, &r, tmin, tmax, &h);
    if (out) export_hit(&h, out);
    return ok;
}

int oracle_node_interval(const rt_scene_desc* d, int node, const double o[3], const double dir[3], double* t0,
                         double* t1, oracle_hit* h0, oracle_hit* h1) {
    Ctx c; memset(&c, 0, sizeof(c)); c.s = d;
    Ray r = make_ray(vget(o), vget(dir));
    Hit a = default_hit(), b = default_hit();
    double x0 = 0, x1 = 0;
    int ok = node_interval(&c, node, &r, &x0, &x1, &a, &b);
    if (t0) *t0 = x0;
    if (t1) *t1 = x1;
    if (h0) export_hit(&a, h0);
    if (h1) export_hit(&b, h1);
    return ok;
}

int oracle_scene_intersect(const rt_scene_desc* d, const double o[3], const double dir[3], double tmin, double tmax,
                           oracle_hit* out) {
    Ctx c; memset(&c, 0, sizeof(c)); c.s = d;
    Ray r = make_ray(vget(o), vget(dir));
    Hit h = default_hit();
    int ok = scene_intersect(&c, &r, tmin, tmax, &h);
    if (out) export_hit(&h, out);
    return ok;
}

int oracle_scene_occluded(const rt_scene_desc* d, const double o[3], const double dir[3], double tmin, double tmax) {
    Ctx c; memset(&c, 0, sizeof(c)); c.s = d;
    Ray r = make_ray(vget(o), vget(dir));
    return scene_occluded(&c, &r, tmin, tmax);
}

void oracle_camera_ray(const rt_scene_desc* d, int i, int j, double dx, double dy, int subpixel, double o[3],
                       double dir[3]) {
    Ray r = subpixel ? generate_ray_subpixel(&d->camera, i, j, dx, dy) : generate_ray(&d->camera, i, j);
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z;
    dir[0] = r.d.x; dir[1] = r.d.y; dir[2] = r.d.z;
}

void oracle_jitter(uint64_t first, uint64_t count, double* out) {
    MT g;
    mt_seed(&g, 12345u);
    mt_discard(&g, 2 * first);
    for (uint64_t k = 0; k < count; ++k) out[k] = uni(&g);
}

void oracle_mt_words(uint64_t first, uint64_t count, uint32_t* out) {
    MT g;
    mt_seed(&g, 12345u);
    mt_discard(&g, first);
    for (uint64_t k = 0; k < count; ++k) out[k] = mt_next(&g);
}
