/*
 * oracle.h — CPU restatement of the reference ray-trace path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so.  The product path
 * (librtamd.so, the `ray` CLI) never links or calls it.
 *
 * Pinning: oracle/_ref/ is the reference's own hot path
 * (raytracer/src/{tracer,shading,scene,geometry,csg,transform}.cpp) compiled
 * from /root/reference by oracle/Makefile with our harness
 * oracle/ref_harness.cpp; tests/golden/ holds framebuffers, ray counts and
 * per-primitive KAT vectors produced by it (script: tests/golden/make_golden.py).
 * The oracle is checked bit-for-bit against those fixtures.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#include "rt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_stats {
    uint64_t rays_intersect;   /* Scene::intersect calls (scene.cpp:10) */
    uint64_t rays_occluded;    /* Scene::occluded calls  (scene.cpp:33) */
    uint64_t ops[16];          /* rt_op_counter */
} oracle_stats;

typedef struct oracle_hit {    /* geometry.h:25-46 Hit */
    double t;
    double p[3];
    double n[3];
    int32_t mat;               /* material index, -1 = nullptr */
    int32_t front_face;
} oracle_hit;

/* Tracer::render restricted to OUTPUT rows [row0,row1) (top row first).
 * fb receives (row1-row0)*W*3 doubles.  n_threads>1 splits the rows into
 * bands; each band fast-forwards its own mt19937 to the band's first word. */
int oracle_render_rows(const rt_scene_desc* d, int W, int H, int mode, int row0, int row1,
                       double* fb, oracle_stats* st, int n_threads);

/* Primitive-level queries (Primitive::intersect / ::interval) on node `node`.
 * The ray is built as Ray(o, d) (direction normalised, core.h:278). */
int oracle_node_intersect(const rt_scene_desc* d, int node, const double o[3], const double dir[3],
                          double tmin, double tmax, oracle_hit* out);
int oracle_node_interval(const rt_scene_desc* d, int node, const double o[3], const double dir[3],
                         double* t0, double* t1, oracle_hit* h0, oracle_hit* h1);

/* Scene-level queries. */
int oracle_scene_intersect(const rt_scene_desc* d, const double o[3], const double dir[3],
                           double tmin, double tmax, oracle_hit* out);
int oracle_scene_occluded(const rt_scene_desc* d, const double o[3], const double dir[3],
                          double tmin, double tmax);

/* Camera::generate_ray (subpixel=0) / generate_ray_subpixel (subpixel=1). */
void oracle_camera_ray(const rt_scene_desc* d, int i, int j, double dx, double dy, int subpixel,
                       double o[3], double dir[3]);

/* Jitter stream: the n-th uniform(-0.5,0.5) draw of std::mt19937(12345)
 * (tracer.cpp:284-293).  Fills out[k] for k in [first, first+count). */
void oracle_jitter(uint64_t first, uint64_t count, double* out);
/* Raw tempered mt19937(12345) outputs [first, first+count). */
void oracle_mt_words(uint64_t first, uint64_t count, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif
