// rt_device.hpp — FP64 device restatement of the reference trace path for
// gfx950 (CDNA4).  Operation order follows the reference step for step and
// the file is compiled with -ffp-contract=off and IEEE div/sqrt, so every
// rounding matches the x86-64 reference except pow() with a non-integer
// exponent, which comes from the device math library (<= 1 ulp apart; no
// reference scene has one).  The pokeball's acos is never evaluated: its two
// comparisons are thresholds of the host's acos (pick_region).  Citations are
// raytracer/src/<file>:<line> of the reference.
//
// Design:
//   * one lane per (pixel, sample); a wave is 8 pixels x 8 samples,
//   * the scene object loop and the per-object op programs are WAVE-UNIFORM:
//     every lane walks the same sequence, parameters come through the scalar
//     cache, and whole objects are skipped with __any() on a bound test,
//   * transforms / CSG operands live on a ray stack and an interval stack
//     whose top two intervals stay in VGPRs (left-deep folds never spill),
//   * reflection / refraction recursion is an explicit per-lane frame stack.
//
// Precision: the file is compiled once per arithmetic type.  RT_REAL double
// (namespace rtd) is the parity path; RT_REAL float (namespace rtf,
// rt_render_f32.hip, RT_FLAG_FP32) is the optional non-parity fast path of
// the same algorithm on float scene copies.  Literals
// go through RV() so the float build does no double arithmetic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "rt.h"
#include "rt_launch.hpp"
#include "scene_compile.hpp"

#ifndef RT_REAL
#define RT_REAL double
#define RT_NS rtd
#endif

namespace RT_NS {

using rtamd::DevObj;
using rtamd::DevOp;
using real = RT_REAL;
using NodeT = rtamd::NodeR<real>;
using MatT = rtamd::MatR<real>;
using LightT = rtamd::LightR<real>;
using DLightT = rtamd::DLightR<real>;
using FoldT = rtamd::FoldLeafR<real>;
#define RV(x) static_cast<real>(x)
#define RT_INF static_cast<real>(__builtin_inf())

__device__ __forceinline__ double sqrt_r(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ double fabs_r(double x) { return __builtin_fabs(x); }
__device__ __forceinline__ float sqrt_r(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ float fabs_r(float x) { return __builtin_fabsf(x); }

constexpr real kEPS = RV(1e-6);   // core.h:10

#ifdef RT_BIG_STACKS
constexpr int kMaxDepth = rtamd::kBigDepth;
constexpr int kMaxIvlSpill = rtamd::kBigIvlSpill;
constexpr int kMaxRayStack = rtamd::kBigRayStack;
#else
using rtamd::kMaxDepth;
using rtamd::kMaxIvlSpill;
using rtamd::kMaxRayStack;
#endif

struct V3 {
    real x, y, z;
};
__device__ __forceinline__ V3 v3(real x, real y, real z) { return V3{x, y, z}; }
__device__ __forceinline__ real dot3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ real dmax(real a, real b) { return (a < b) ? b : a; }   // std::max
__device__ __forceinline__ real dmin(real a, real b) { return (b < a) ? b : a; }   // std::min
// std::max(c, x) / std::min(c, x) with a non-NaN constant c as one v_max / v_min
// instead of compare + two selects: equal for every x including NaN (both
// give c); for x = -0 against c = +0 the sign of the zero may differ, so these
// are used only where a zero result's sign cannot reach the output (each use
// says why).
__device__ __forceinline__ real cmax(real c, real x) { return __builtin_fmax(c, x); }
__device__ __forceinline__ real cmin(real c, real x) { return __builtin_fmin(c, x); }
__device__ __forceinline__ V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
// The next representable value above x >= 0 (x itself for +inf).
__device__ __forceinline__ double next_up(double x) {
    return x < __builtin_inf() ? __longlong_as_double(__double_as_longlong(x) + 1) : x;
}
__device__ __forceinline__ float next_up(float x) {
    return x < __builtin_inff() ? __int_as_float(__float_as_int(x) + 1) : x;
}

// (a0, a1, a2) / b: three IEEE divisions, bit-identical to the compiler's
// own FP64 division (v_div_scale / v_rcp / two Newton steps / v_div_fmas /
// v_div_fixup, the exact sequence `a / b` lowers to on gfx950), with the
// reciprocal refinement done once when the scaled denominator is the same for
// every numerator and lane (it depends on the numerator only at the extremes
// of the exponent range, where the three divisions are done one by one).
// tests/test_gpu_numerics.py checks it bit for bit against `/`.
struct D3 {
    double x, y, z;
};
__device__ __forceinline__ D3 div3(double a0, double a1, double a2, double b) {
    bool u0, u1, u2;
    const double s0 = __builtin_amdgcn_div_scale(a0, b, false, &u0);
    const double s1 = __builtin_amdgcn_div_scale(a1, b, false, &u1);
    const double s2 = __builtin_amdgcn_div_scale(a2, b, false, &u2);
    const bool same = __double_as_longlong(s0) == __double_as_longlong(s1) &&
                      __double_as_longlong(s0) == __double_as_longlong(s2);
    if (!__all(same)) return D3{a0 / b, a1 / b, a2 / b};
    const double rcp = __builtin_amdgcn_rcp(s0);
    const double f0 = __builtin_fma(-s0, rcp, 1.0);
    const double f1 = __builtin_fma(rcp, f0, rcp);
    const double f2 = __builtin_fma(-s0, f1, 1.0);
    const double f3 = __builtin_fma(f1, f2, f1);
    auto quot = [&](double a) {
        bool vcc;
        const double n = __builtin_amdgcn_div_scale(a, b, true, &vcc);
        const double mul = n * f3;
        const double f4 = __builtin_fma(-s0, mul, n);
        return __builtin_amdgcn_div_fixup(__builtin_amdgcn_div_fmas(f4, f3, mul, vcc), b, a);
    };
    return D3{quot(a0), quot(a1), quot(a2)};
}
__device__ __forceinline__ auto div3(float a0, float a1, float a2, float b) {
    struct F3 { float x, y, z; };
    return F3{a0 / b, a1 / b, a2 / b};
}

// Dir3::normalized (core.h:95-101)
__device__ __forceinline__ V3 normalized(V3 v) {
    real L = sqrt_r(dot3(v, v));
    if (L > kEPS) {
        const auto q = div3(v.x, v.y, v.z, L);
        return v3(q.x, q.y, q.z);
    }
    return v3(RV(0.0), RV(1.0), RV(0.0));
}

struct DRay {
    V3 o, d;
};
// Ray::Ray (core.h:278) normalises the direction.
__device__ __forceinline__ DRay make_ray(V3 o, V3 d) { return DRay{o, normalized(d)}; }
__device__ __forceinline__ V3 ray_at(const DRay& r, real t) {   // core.h:280
    return v3(r.o.x + r.d.x * t, r.o.y + r.d.y * t, r.o.z + r.d.z * t);
}

// Hit without t (interval hits' t is never observed: see DESIGN.md).
struct DHit {
    V3 p, n;
    int mat;
    int ff;
};

// Hit::set_face_normal (geometry.h:42-45)
__device__ __forceinline__ void set_face_normal(DHit& h, const DRay& r, V3 outward) {
    h.ff = dot3(r.d, outward) < RV(0.0);
    h.n = h.ff ? outward : vneg(outward);
}

struct Ivl {
    int ok;
    real t0, t1;
    DHit h0, h1;
};

struct THit {   // intersect-mode hit
    int ok;
    real t;
    DHit h;
};

// Per-lane op counters (RT_FLAG_COUNT_OPS builds only).
//
// Diagnostic builds with -DRT_PHASE_PROF (tools/build_exp.sh, never the
// product library) give the uncounted variant wave-level phase timers:
// pb(k)/pe(k) bracket a phase at points where the whole wave is converged,
// and the accumulated shader-clock cycles of lane 0 land in rt_stats.ops[k]
// (PH_* below).
enum RtPhase {
    PH_SETUP = 0,      // jitter load + camera ray
    PH_PRIMARY,        // scene_intersect(_wave) incl. resolve_hit
    PH_SHADE1,         // light loop pass 1 without the occlusion queries
    PH_SHADOW,         // scene_occluded(_wave)
    PH_SHADOW_CSG,     //   of which compact-CSG object evaluations
    PH_SHADE2,         // light loop pass 2 (accumulation)
    PH_PRIMARY_CSG,    // compact-CSG object evaluations of primary rays
    PH_TAIL,           // sample sum, framebuffer store
    PH_CSG_LEAF,       // run_compact: leaf intervals
    PH_CSG_COMB,       // run_compact: CSG combines
    PH_CHAIN_XF,       // object_hit: transform chain down and back up
    PH_OBJ_PREF,       // wave queries: per-candidate prefilters (leaf masks, ball tests)
    PH_OBJ_HIT,        // wave queries: object_hit calls (all kinds)
    PH_WAVE_SETUP,     // wave queries: bundle setup + transposed object test
    PH_COUNT
};
// Diagnostic builds with -DRT_EVENT_PROF instead count WAVE-level executions
// of the events below (first active lane, so divergent paths count once per
// wave that runs them) into rt_stats.ops[k]; no timers.
enum RtEvent {
    EV_SHQ = 0,        // shadow wave queries with some lane querying
    EV_SH_CAND,        // shadow: candidate objects after the transposed test
    EV_SH_HIT,         // shadow: object_hit calls (after the prefilters)
    EV_SH_CSG,         //   of which CSG objects
    EV_PR_CAND,        // primary: candidate objects
    EV_PR_HIT,         // primary: object_hit calls
    EV_FOLD_LEAF,      // fold_leaf_ivl executions
    EV_COMB,           // csg_c executions past the both-empty test
    EV_COMB_SINGLE,    //   one-operand path
    EV_COMB_EASY,      //   union closed form
    EV_COMB_GEN,       //   general sweep
    EV_LIGHT1,         // light pass 1 iterations with some lane needing a query
    EV_LIGHT2,         // light pass 2 iterations (lit lights)
    EV_BOUNCE,         // trace_wave steps after the first (reflection / refraction bounces)
    EV_COMPACT_LEAF,   // leaf_ivl_c executions (trace_wave scenes: lanes evaluating in bounce steps)
    EV_WAVES,          // waves with an active lane
    EV_COUNT
};
template <bool C>
struct Cnt;
template <>
struct Cnt<false> {
    static constexpr bool kPlain = false;
    __device__ __forceinline__ void inc(int) {}
    __device__ __forceinline__ void gate(bool) {}
#ifdef RT_EVENT_PROF
    __device__ static unsigned long long* acc() {
        __shared__ unsigned long long a[4][EV_COUNT];
        return &a[threadIdx.x >> 6][0];
    }
    __device__ __forceinline__ void init() {
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < EV_COUNT; ++k) acc()[k] = 0;
    }
    __device__ __forceinline__ bool first() {
        return (int)__lane_id() == __builtin_ctzll(__builtin_amdgcn_read_exec());
    }
    __device__ __forceinline__ void ev(int k) {
        if (first()) acc()[k] += 1;
    }
    __device__ __forceinline__ void evn(int k, unsigned n) {   // (wave-uniform n)
        if (first()) acc()[k] += n;
    }
    __device__ __forceinline__ void pb(int) {}
    __device__ __forceinline__ void pe(int) {}
    __device__ __forceinline__ unsigned long long get(int k) { return acc()[k]; }
#elif defined(RT_PHASE_PROF)
    // per-wave accumulators in LDS, updated by the first active lane, so
    // that phases inside divergent code are timed too (256-thread blocks)
    // (start stamps live in LDS too: no VGPRs taken from the kernel)
    __device__ static unsigned long long* acc() {
        __shared__ unsigned long long a[4][2 * PH_COUNT];
        return &a[threadIdx.x >> 6][0];
    }
    __device__ __forceinline__ void init() {
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < PH_COUNT; ++k) acc()[k] = 0;
    }
    __device__ __forceinline__ bool first() {
        return (int)__lane_id() == __builtin_ctzll(__builtin_amdgcn_read_exec());
    }
    __device__ __forceinline__ void pb(int k) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (first()) acc()[PH_COUNT + k] = t;
    }
    __device__ __forceinline__ void pe(int k) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (first()) acc()[k] += t - acc()[PH_COUNT + k];
    }
    __device__ __forceinline__ unsigned long long get(int k) { return acc()[k]; }
    __device__ __forceinline__ void ev(int) {}
    __device__ __forceinline__ void evn(int, unsigned) {}
#else
    __device__ __forceinline__ void init() {}
    __device__ __forceinline__ void pb(int) {}
    __device__ __forceinline__ void pe(int) {}
    __device__ __forceinline__ void ev(int) {}
    __device__ __forceinline__ void evn(int, unsigned) {}
#endif
};
template <>
struct Cnt<true> {
    static constexpr bool kPlain = false;
    uint32_t c[16];
    uint32_t on;   // 0 while a lane evaluates an object only to keep the wave convergent
    __device__ __forceinline__ Cnt() : on(1u) {
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = 0;
    }
    __device__ __forceinline__ void inc(int k) { c[k] += on; }
    __device__ __forceinline__ void gate(bool b) { on = b ? 1u : 0u; }
    __device__ __forceinline__ void ev(int) {}
    __device__ __forceinline__ void evn(int, unsigned) {}
    __device__ __forceinline__ void init() {}
    __device__ __forceinline__ void pb(int) {}
    __device__ __forceinline__ void pe(int) {}
};
// The plain kernels' counter type (no counting, like Cnt<false>): scenes
// whose objects are all spheres, half-spaces and pokeballs (no transform or
// CSG object, SceneView::plain) run kernels compiled without the transform /
// CSG evaluation and the CSG shadow prefilters.  That code, never executed
// for such scenes, still shaped the register allocation of every path: the
// paper kernel spilled 48 B/lane and the recursion kernel 48 B beyond its
// frame stack; without it config 5 runs 4.34 -> 3.78 ms and the recursion row
// 15.33 -> 12.95 ms (profiles/r06_ab/ab_plain.txt).  The type carries the
// choice down every query (each is templated on its counter type).
struct CntPlain : Cnt<false> {
    static constexpr bool kPlain = true;
};
// op-counting builds of a query (Cnt<true>)
template <class CT>
constexpr bool kCounting = std::is_same<CT, Cnt<true>>::value;
// transform / CSG object code compiled in (every kernel but the plain ones)
template <class CT>
constexpr bool kCsg = !CT::kPlain;

struct DevScene {
    const NodeT* nodes;
    const MatT* mats;
    const LightT* lights;
    const DLightT* dlights;
    const DevObj* objs;
    const DevOp* ops;
    const float* gb;    // OP_IVL_GROUP bounds (cx, cy, cz, r), f32-inflated
    const float4* ctab; // per object 2 x float4: wave-level cull record (CompiledScene::ctab)
    const float4* lrec; // [light][object] 2 x float4: light-relative shadow cull records (CompiledScene::lrec / lwrec)
    const float4* lgb;  // [light][gb ball] 2 x float4 (CompiledScene::lgb)
    int n_gb;
    const FoldT* fold;  // fold objects' leaf tables (DevObj::fold0)
    int n_lights, n_objs;
    int n_dlights;
    int n_bounded;   // objects with a bounding ball (wave-level culling pays only when > 0)
    int n_lead;      // CompiledScene::n_lead: unbounded objects ahead of every bounded one (0 in the BVH kernels)
    int cam_nx, cam_ny;
    int rec_limit, cull;
    real eye[3], P[3], Lx, Ly;
    real medium_index;
    // The background colour (the miss value) is the albedo of material slot
    // bg_mat, and every material's ambient term arrives multiplied by the
    // scene's ambient (E_a = K_a I_a, shading.cpp:39: the same single
    // multiplication, done on the host): neither is a kernel argument held in
    // SGPRs through the whole trace.
    int bg_mat;
    // wave BVH kernels only (objs / ctab then hold CompiledScene::wobjs /
    // wctab): each object's index in the reference's order, and the chunk
    // records (2 x float4 per chunk of 64 objects)
    const int32_t* worig;
    const float4* wchunk;
    int n_chunks;
};

__device__ __forceinline__ V3 ld3(const real* p) { return v3(p[0], p[1], p[2]); }
__device__ __forceinline__ V3 background(const DevScene& S) { return ld3(S.mats[S.bg_mat].albedo); }

// --------------------------------------------------------------- primitives
// Sphere::intersect (geometry.cpp:12-37)
template <class CT>
__device__ __forceinline__ bool sphere_intersect(V3 c, real rad, const DRay& ray, real tmin, real tmax,
                                                 real& t_out, DHit& out, CT& cnt) {
    cnt.inc(RT_OPC_SPHERE_ISECT);
    V3 oc = v3(ray.o.x - c.x, ray.o.y - c.y, ray.o.z - c.z);
    real half_b = dot3(oc, ray.d);
    real cterm = dot3(oc, oc) - rad * rad;
    real disc = half_b * half_b - RV(1.0) * cterm;
    if (disc < RV(0.0)) return false;
    real sq = sqrt_r(disc);
    real t = (-half_b - sq) / RV(1.0);
    if (t < tmin || t > tmax) {
        t = (-half_b + sq) / RV(1.0);
        if (t < tmin || t > tmax) return false;
    }
    cnt.inc(RT_OPC_SPHERE_ISECT_HIT);
    t_out = t;
    out.p = ray_at(ray, t);
    V3 outward = v3((out.p.x - c.x) / rad, (out.p.y - c.y) / rad, (out.p.z - c.z) / rad);
    set_face_normal(out, ray, outward);
    return true;
}

// Sphere::interval (geometry.cpp:48-78)
template <class CT>
__device__ __forceinline__ void sphere_interval(V3 c, real r, int mat, const DRay& ray, Ivl& o, CT& cnt) {
    cnt.inc(RT_OPC_SPHERE_IVL);
    V3 oc = v3(ray.o.x - c.x, ray.o.y - c.y, ray.o.z - c.z);
    real half_b = dot3(oc, ray.d);
    real cterm = dot3(oc, oc) - r * r;
    real disc = half_b * half_b - RV(1.0) * cterm;
    o.ok = !(disc < RV(0.0));
    if (!o.ok) return;
    cnt.inc(RT_OPC_SPHERE_IVL_HIT);
    real s = sqrt_r(disc);
    real t0 = (-half_b - s) / RV(1.0);
    real t1 = (-half_b + s) / RV(1.0);
    if (t0 > t1) {
        real tt = t0;
        t0 = t1;
        t1 = tt;
    }
    o.t0 = t0;
    o.t1 = t1;
    o.h0.p = ray_at(ray, t0);
    set_face_normal(o.h0, ray, v3((o.h0.p.x - c.x) / r, (o.h0.p.y - c.y) / r, (o.h0.p.z - c.z) / r));
    o.h0.mat = mat;
    o.h1.p = ray_at(ray, t1);
    set_face_normal(o.h1, ray, v3((o.h1.p.x - c.x) / r, (o.h1.p.y - c.y) / r, (o.h1.p.z - c.z) / r));
    o.h1.mat = mat;
}

// HalfSpace::intersect (geometry.cpp:90-106)
template <class CT>
__device__ __forceinline__ bool half_intersect(V3 p0, V3 n, const DRay& r, real tmin, real tmax, real& t_out,
                                               DHit& out, CT& cnt) {
    cnt.inc(RT_OPC_HALF_ISECT);
    const real ndotd = dot3(n, r.d);
    if (fabs_r(ndotd) < RV(1e-12)) return false;
    V3 diff = v3(p0.x - r.o.x, p0.y - r.o.y, p0.z - r.o.z);
    const real t = dot3(n, diff) / ndotd;
    if (t < tmin || t > tmax) return false;
    cnt.inc(RT_OPC_HALF_ISECT_HIT);
    t_out = t;
    out.p = ray_at(r, t);
    set_face_normal(out, r, n);
    return true;
}

// HalfSpace::interval (geometry.cpp:117-147)
template <class CT>
__device__ __forceinline__ void half_interval(V3 p0, V3 n, int mat, const DRay& r, Ivl& o, CT& cnt) {
    cnt.inc(RT_OPC_HALF_IVL);
    const real ndotd = dot3(n, r.d);
    V3 diff = v3(r.o.x - p0.x, r.o.y - p0.y, r.o.z - p0.z);
    const real f0 = dot3(n, diff);
    o.h0.mat = mat;
    o.h1.mat = mat;
    if (fabs_r(ndotd) < RV(1e-12)) {
        o.ok = f0 >= RV(0.0);
        o.t0 = -RT_INF;
        o.t1 = RT_INF;
        o.h0.p = r.o;
        o.h1.p = r.o;
    } else {
        o.ok = 1;
        const real tPlane = -f0 / ndotd;
        if (ndotd > RV(0.0)) {
            o.t0 = tPlane;
            o.t1 = RT_INF;
            o.h0.p = ray_at(r, tPlane);
            o.h1.p = r.o;
        } else {
            o.t0 = -RT_INF;
            o.t1 = tPlane;
            o.h0.p = r.o;
            o.h1.p = ray_at(r, tPlane);
        }
    }
    set_face_normal(o.h0, r, n);
    set_face_normal(o.h1, r, n);
}

__device__ __forceinline__ real clamp1(real x) {   // geometry.cpp:152-156
    if (x < -RV(1.0)) return -RV(1.0);
    if (x > RV(1.0)) return RV(1.0);
    return x;
}

// Pokeball::pick_region_material (geometry.cpp:163-180) given its local unit
// position u = (p - c) / r (the same three divisions as Sphere's outward
// normal at p, geometry.cpp:31: callers that have that normal pass it)
template <class CT>
__device__ __forceinline__ int pick_region_u(const NodeT* nd, V3 u, CT& cnt) {
    cnt.inc(RT_OPC_POKE_REGION);
    const real* v = nd->v;
    // ang = acos(x) <= btnOuter / ang >= inner as x >= xb / x <= xi: the
    // thresholds of the host's (the reference's) acos, rtamd::pokeball_thresholds
    const real x = clamp1(dot3(u, v3(v[7], v[8], v[9])));
    if (x >= v[rtamd::kPokeXb]) return (x <= v[rtamd::kPokeXi]) ? nd->mats[RT_PB_RING] : nd->mats[RT_PB_BUTTON];
    if (fabs_r(u.y) <= v[4]) return nd->mats[RT_PB_BELT];
    return (u.y >= RV(0.0)) ? nd->mats[RT_PB_TOP] : nd->mats[RT_PB_BOTTOM];
}
template <class CT>
__device__ __forceinline__ int pick_region(const NodeT* nd, V3 p, CT& cnt) {
    const real* v = nd->v;
    const auto uq = div3(p.x - v[0], p.y - v[1], p.z - v[2], v[3]);
    return pick_region_u(nd, v3(uq.x, uq.y, uq.z), cnt);
}

// Leaf Primitive::intersect for the three leaf kinds.
template <class CT>
__device__ __forceinline__ bool leaf_intersect(const NodeT* nd, const DRay& r, real tmin, real tmax,
                                               real& t, DHit& h, CT& cnt) {
    const int kind = nd->kind;
    if (kind == RT_NODE_HALFSPACE) {
        bool ok = half_intersect(ld3(nd->v), ld3(nd->v + 3), r, tmin, tmax, t, h, cnt);
        h.mat = nd->mat;
        return ok;
    }
    bool ok = sphere_intersect(ld3(nd->v), nd->v[3], r, tmin, tmax, t, h, cnt);
    if (kind == RT_NODE_SPHERE) {
        h.mat = nd->mat;
    } else if (ok) {   // Pokeball::intersect (geometry.cpp:190-197)
        h.mat = pick_region(nd, h.p, cnt);
    }
    return ok;
}

template <class CT>
__device__ __forceinline__ void leaf_interval(const NodeT* nd, const DRay& r, Ivl& o, CT& cnt) {
    const int kind = nd->kind;
    if (kind == RT_NODE_HALFSPACE) {
        half_interval(ld3(nd->v), ld3(nd->v + 3), nd->mat, r, o, cnt);
        return;
    }
    sphere_interval(ld3(nd->v), nd->v[3], nd->mat, r, o, cnt);
    if (kind == RT_NODE_POKEBALL && o.ok) {   // geometry.cpp:207-217
        o.h0.mat = pick_region(nd, o.h0.p, cnt);
        o.h1.mat = pick_region(nd, o.h1.p, cnt);
    }
}

// ---------------------------------------------------------------- transforms
// Matrix4 * Vec4 rows 0..2 (core.h:169-176)
__device__ __forceinline__ V3 mat_apply(const real* m, V3 v, real w) {
    return v3(m[0] * v.x + m[1] * v.y + m[2] * v.z + m[3] * w, m[4] * v.x + m[5] * v.y + m[6] * v.z + m[7] * w,
              m[8] * v.x + m[9] * v.y + m[10] * v.z + m[11] * w);
}

// Local ray of Translation / Scaling / Rotation (transform.cpp:24-29, 97-111, 184-196).
// Degenerate Scaling never reaches the device (compiled to OP_NEVER).
__device__ __forceinline__ DRay local_ray(const NodeT* nd, const DRay& r) {
    const real* M = nd->v;
    const int kind = nd->kind;
    if (kind == RT_NODE_TRANSLATION) return make_ray(v3(r.o.x - M[3], r.o.y - M[7], r.o.z - M[11]), r.d);
    if (kind == RT_NODE_SCALING) {
        const real sx = M[0], sy = M[5], sz = M[10];
        return make_ray(v3(r.o.x / sx, r.o.y / sy, r.o.z / sz), v3(r.d.x / sx, r.d.y / sy, r.d.z / sz));
    }
    const real* I = nd->v + 12;
    return make_ray(mat_apply(I, r.o, RV(1.0)), mat_apply(I, r.d, RV(0.0)));
}

__device__ __forceinline__ V3 map_point(const NodeT* nd, V3 p) {
    const real* M = nd->v;
    const int kind = nd->kind;
    if (kind == RT_NODE_TRANSLATION) return v3(p.x + M[3], p.y + M[7], p.z + M[11]);
    if (kind == RT_NODE_SCALING) return v3(p.x * M[0], p.y * M[5], p.z * M[10]);
    return mat_apply(M, p, RV(1.0));
}

__device__ __forceinline__ V3 map_normal(const NodeT* nd, V3 n) {
    const real* M = nd->v;
    const int kind = nd->kind;
    if (kind == RT_NODE_TRANSLATION) return n;
    if (kind == RT_NODE_SCALING) return normalized(v3(n.x / M[0], n.y / M[5], n.z / M[10]));
    return normalized(mat_apply(M, n, RV(0.0)));
}

// Transform::project_t_world (transform.h:76-80)
__device__ __forceinline__ real project_t_world(const DRay& r, V3 Pw) {
    V3 v = v3(Pw.x - r.o.x, Pw.y - r.o.y, Pw.z - r.o.z);
    const real dd = r.d.x * r.d.x + r.d.y * r.d.y + r.d.z * r.d.z;
    return dd > RV(0.0) ? (v.x * r.d.x + v.y * r.d.y + v.z * r.d.z) / dd : RT_INF;
}

// ------------------------------------------------------------------- CSG
__device__ __forceinline__ bool csg_combine(int op, bool a, bool b) {
    return op == RT_CSG_UNION ? (a || b) : op == RT_CSG_INTERSECTION ? (a && b) : (a && !b);
}

// event_less lambda (csg.cpp:87-92); code = who*2 + type (type 0 Enter, 1 Exit)
__device__ __forceinline__ bool ev_less(real ta, int ca, real tb, int cb) {
    if (fabs_r(ta - tb) > RV(1e-6)) return ta < tb;
    const int tya = ca & 1, tyb = cb & 1;
    if (tya != tyb) return tya == 0;
    return (ca >> 1) < (cb >> 1);
}

__device__ __forceinline__ const DHit& sel_hit(int code, const Ivl& a, const Ivl& b) {
    return code == 0 ? a.h0 : code == 1 ? a.h1 : code == 2 ? b.h0 : b.h1;
}

// CSG::interval (csg.cpp:61-163) on the two child intervals already computed.
template <class CT>
__device__ __forceinline__ void csg_interval(int op, const Ivl& A, const Ivl& B, const DRay& ray, Ivl& R,
                                             CT& cnt) {
    R.ok = 0;
    if (!A.ok && !B.ok) return;
    cnt.inc(RT_OPC_CSG_COMBINE);
    // Finite events in push order a0, a1, b0, b1 (csg.cpp:76-81).
    real et[4];
    int ec[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        et[k] = RV(0.0);
        ec[k] = 0;
    }
    int n = 0;
    {
        const bool p0 = A.ok && __builtin_isfinite(A.t0);
        const bool p1 = A.ok && __builtin_isfinite(A.t1);
        const bool p2 = B.ok && __builtin_isfinite(B.t0);
        const bool p3 = B.ok && __builtin_isfinite(B.t1);
        const real tv[4] = {A.t0, A.t1, B.t0, B.t1};
        const bool pv[4] = {p0, p1, p2, p3};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool here = pv[e] && n == k;
                et[k] = here ? tv[e] : et[k];
                ec[k] = here ? e : ec[k];
            }
            n += pv[e] ? 1 : 0;
        }
    }
    // libstdc++ __insertion_sort (stl_algo.h:1819-1871) with the non-strict
    // comparator, unrolled over the fixed <= 4 slots.
#pragma unroll
    for (int i = 1; i < 4; ++i) {
        if (i < n) {
            const real vt = et[i];
            const int vc = ec[i];
            if (ev_less(vt, vc, et[0], ec[0])) {
#pragma unroll
                for (int k = i; k > 0; --k) {
                    et[k] = et[k - 1];
                    ec[k] = ec[k - 1];
                }
                et[0] = vt;
                ec[0] = vc;
            } else {
                bool moving = true;
                int last = i;
#pragma unroll
                for (int k = i; k > 0; --k) {
                    // __unguarded_linear_insert: while (comp(val, *next)) shift
                    if (moving && ev_less(vt, vc, et[k - 1], ec[k - 1])) {
                        et[k] = et[k - 1];
                        ec[k] = ec[k - 1];
                        last = k - 1;
                    } else {
                        moving = false;
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k == last) {
                        et[k] = vt;
                        ec[k] = vc;
                    }
                }
            }
        }
    }
    bool inA = A.ok && (A.t0 < RV(1e-6)) && (A.t1 > RV(1e-6));
    bool inB = B.ok && (B.t0 < RV(1e-6)) && (B.t1 > RV(1e-6));
    bool inR = csg_combine(op, inA, inB);
    bool haveEnter = false;
    int enterCode = -1, exitCode = -1;
    bool flipE = false, flipX = false;
    real tEnt = RV(0.0), tExt = RT_INF;
    int originMat = -1;
    if (inR) {
        haveEnter = true;
        originMat = (inA && A.h0.mat >= 0) ? A.h0.mat : (inB ? B.h0.mat : -1);
    }
    bool done = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < n && !done) {
            const bool before = inR;
            const int code = ec[k];
            const bool enter = (code & 1) == 0;
            if ((code >> 1) == 0) inA = enter;
            else inB = enter;
            const bool after = csg_combine(op, inA, inB);
            if (!before && after) {
                haveEnter = true;
                tEnt = et[k];
                enterCode = code;
                flipE = (op == RT_CSG_DIFFERENCE) && code == 3;
            } else if (before && !after) {
                tExt = et[k];
                exitCode = code;
                flipX = (op == RT_CSG_DIFFERENCE) && code == 2;
                done = true;
            }
            if (!done) inR = after;
        }
    }
    if (!haveEnter || !__builtin_isfinite(tExt)) return;
    R.ok = 1;
    R.t0 = tEnt;
    R.t1 = tExt;
    if (enterCode < 0) {
        R.h0.p = ray.o;
        R.h0.n = v3(RV(0.0), RV(0.0), RV(0.0));
        R.h0.mat = originMat;
        R.h0.ff = 1;
    } else {
        R.h0 = sel_hit(enterCode, A, B);
        if (flipE) set_face_normal(R.h0, ray, vneg(R.h0.n));
    }
    R.h1 = sel_hit(exitCode, A, B);
    if (flipX) set_face_normal(R.h1, ray, vneg(R.h1.n));
}

// ------------------------------------------------------------ interpreter
struct IStack {
    Ivl tos, nos;
    Ivl spill[kMaxIvlSpill];
    int sp;   // number of entries (wave-uniform)

    __device__ __forceinline__ void push(const Ivl& v) {
        if (sp >= 2) spill[sp - 2] = nos;
        if (sp >= 1) nos = tos;
        tos = v;
        ++sp;
    }
    // replace the top two by r
    __device__ __forceinline__ void reduce2(const Ivl& r) {
        tos = r;
        if (sp >= 3) nos = spill[sp - 3];
        --sp;
    }
};

// Evaluate one OBJ_PROG object: Primitive::intersect(root, ray, tmin, tmax).
template <bool EAGER, class CT>
__device__ __forceinline__ bool run_program(const DevScene& S, int pc0, int pc1, const DRay& world, real tmin,
                                         real tmax, real& t_out, DHit& h_out, CT& cnt) {
    DRay cur = world;
    DRay rstk[kMaxRayStack];
    int rsp = 0;
    IStack st;
    st.sp = 0;
    THit hit;
    hit.ok = 0;
    hit.t = RV(0.0);
    for (int pc = pc0; pc < pc1; ++pc) {
        const DevOp op = S.ops[pc];
        const NodeT* nd = &S.nodes[op.node];
        const real lo = op.top == 1 ? tmin : RV(0.0);
        const real hi = op.top == 1 ? tmax : RT_INF;
        switch (op.op) {
            case rtamd::OP_XPUSH:
                cnt.inc(RT_OPC_XFORM);
                rstk[rsp++] = cur;
                cur = local_ray(nd, cur);
                break;
            case rtamd::OP_LEAF_IVL: {
                Ivl v;
                leaf_interval(nd, cur, v, cnt);
                st.push(v);
                break;
            }
            case rtamd::OP_CSG: {
                Ivl r;
                csg_interval(op.csg_op, st.nos, st.tos, cur, r, cnt);
                st.reduce2(r);
                break;
            }
            case rtamd::OP_XPOP_IVL: {
                const DRay parent = rstk[--rsp];
                Ivl& v = st.tos;
                if (v.ok) {   // transform.cpp:55-82 (138-169, 224-255)
                    v.h0.p = map_point(nd, v.h0.p);
                    v.h1.p = map_point(nd, v.h1.p);
                    const V3 nE = map_normal(nd, v.h0.n);
                    const V3 nX = map_normal(nd, v.h1.n);
                    set_face_normal(v.h0, parent, nE);
                    set_face_normal(v.h1, parent, nX);
                    v.t0 = project_t_world(parent, v.h0.p);
                    v.t1 = project_t_world(parent, v.h1.p);
                }
                cur = parent;
                break;
            }
            case rtamd::OP_LEAF_ISECT: {
                real t = RV(0.0);
                hit.ok = leaf_intersect(nd, cur, lo, hi, t, hit.h, cnt);
                hit.t = t;
                break;
            }
            case rtamd::OP_CSG_ISECT: {   // CSG::intersect (csg.cpp:169-185)
                const Ivl& v = st.tos;
                const real t = dmax(v.t0, lo);
                hit.ok = v.ok && (t < v.t1 && t < hi);
                hit.t = t;
                hit.h = v.h0;
                hit.h.p = v3(cur.o.x + cur.d.x * t, cur.o.y + cur.d.y * t, cur.o.z + cur.d.z * t);
                st.sp -= 1;
                break;
            }
            case rtamd::OP_XPOP_HIT: {   // transform.cpp:18-44 (95-127, 182-213)
                const DRay parent = rstk[--rsp];
                if (hit.ok) {
                    const V3 wp = map_point(nd, hit.h.p);
                    const V3 wn = map_normal(nd, hit.h.n);
                    const real wt = project_t_world(parent, wp);
                    hit.ok = (wt > lo && wt < hi);
                    hit.h.p = wp;
                    set_face_normal(hit.h, parent, wn);
                    hit.t = wt;
                }
                cur = parent;
                break;
            }
            case rtamd::OP_NEVER:
            default:
                if (op.top == 2) {
                    Ivl v;
                    v.ok = 0;
                    st.push(v);
                } else {
                    hit.ok = 0;
                }
                break;
        }
    }
    t_out = hit.t;
    h_out = hit.h;
    return hit.ok;
}

// ================================================================ compact
// Lazy hit references (DESIGN.md §Lazy hits).  An interval endpoint in a
// compact CSG program is (t_ref, code): code = op index of the leaf | ROOT1
// (exit root) | FLIP (a CSG difference re-faced it: csg.cpp:140-150 leaves n
// unchanged and sets front_face=false) | ORIGIN (the inside-at-origin entry of
// csg.cpp:113-122: p = ray.o, n = 0, material of the referenced leaf hit).
// The normal / material of a referenced hit is a pure function of (frame
// ray, leaf, t_ref), so it is recomputed bit-identically only for the hit
// that wins.
constexpr int REF_PC_MASK = (1 << 22) - 1;
constexpr int REF_ROOT1 = 1 << 22;
constexpr int REF_FLIP = 1 << 23;
constexpr int REF_ORIGIN = 1 << 24;

struct CIvl {
    int ok;
    real t0, t1;   // interval (event times)
    real s0, s1;   // t_ref of the entry / exit hit references
    int c0, c1;      // codes of the entry / exit hit references
};

// Primitive::interval for a leaf without computing hit points or normals
// (geometry.cpp:48-78, 117-147, 207-217).
template <class CT>
__device__ __forceinline__ void leaf_ivl_c(const NodeT* nd, int pc, const DRay& r, CIvl& o, CT& cnt) {
    cnt.ev(EV_COMPACT_LEAF);
    o.c0 = pc;
    o.c1 = pc | REF_ROOT1;
    if (nd->kind == RT_NODE_HALFSPACE) {
        cnt.inc(RT_OPC_HALF_IVL);
        const V3 n = ld3(nd->v + 3);
        const real ndotd = dot3(n, r.d);
        V3 diff = v3(r.o.x - nd->v[0], r.o.y - nd->v[1], r.o.z - nd->v[2]);
        const real f0 = dot3(n, diff);
        if (fabs_r(ndotd) < RV(1e-12)) {
            o.ok = f0 >= RV(0.0);
            o.t0 = -RT_INF;
            o.t1 = RT_INF;
        } else {
            o.ok = 1;
            const real tPlane = -f0 / ndotd;
            o.t0 = ndotd > RV(0.0) ? tPlane : -RT_INF;
            o.t1 = ndotd > RV(0.0) ? RT_INF : tPlane;
        }
    } else {
        cnt.inc(RT_OPC_SPHERE_IVL);
        const real r0 = nd->v[3];
        V3 oc = v3(r.o.x - nd->v[0], r.o.y - nd->v[1], r.o.z - nd->v[2]);
        const real half_b = dot3(oc, r.d);
        const real cterm = dot3(oc, oc) - r0 * r0;
        const real disc = half_b * half_b - RV(1.0) * cterm;
        o.ok = !(disc < RV(0.0));
        const real s = sqrt_r(o.ok ? disc : RV(0.0));
        real t0 = (-half_b - s) / RV(1.0);
        real t1 = (-half_b + s) / RV(1.0);
        if (t0 > t1) {
            const real tt = t0;
            t0 = t1;
            t1 = tt;
        }
        o.t0 = t0;
        o.t1 = t1;
        if (o.ok) cnt.inc(RT_OPC_SPHERE_IVL_HIT);
    }
    o.s0 = o.t0;
    o.s1 = o.t1;
}

// CSG::interval (csg.cpp:61-163) on two compact child intervals.
template <class CT>
__device__ __forceinline__ void csg_c(int op, const CIvl& A, const CIvl& B, CIvl& R, CT& cnt) {
    R.ok = 0;
    R.t0 = R.t1 = R.s0 = R.s1 = RV(0.0);
    R.c0 = R.c1 = 0;
    if (!A.ok && !B.ok) return;
    cnt.inc(RT_OPC_CSG_COMBINE);
    cnt.ev(EV_COMB);
    if (!(A.ok && B.ok)) {
        cnt.ev(EV_COMB_SINGLE);
        // Exactly one operand has an interval X.  The sweep then sees only X's
        // events: an intersection is never inside; a difference without A is
        // never inside; otherwise the result is X itself, or, when the origin
        // lies inside X, [0, X.t1] with the inside-at-origin entry hit
        // (csg.cpp:113-122).  An infinite exit gives no hit (:158); an
        // infinite entry outside the origin gives no entry (:134-146).
        const bool useA = A.ok;
        if (op == RT_CSG_INTERSECTION || (op == RT_CSG_DIFFERENCE && !useA)) return;
        const CIvl& X = useA ? A : B;
        const bool inX = (X.t0 < RV(1e-6)) && (X.t1 > RV(1e-6));
        R.t1 = X.t1;
        R.s1 = X.s1;
        R.c1 = X.c1;
        if (inX) {
            R.ok = __builtin_isfinite(X.t1);
            R.t0 = RV(0.0);
            R.s0 = X.s0;
            R.c0 = (X.c0 & ~REF_FLIP) | REF_ORIGIN;
        } else {
            // two events sorted by the same epsilon comparator: an exit that
            // sorts first (t1 < t0 - 1e-6, possible for CSG results) never closes
            R.ok = __builtin_isfinite(X.t0) && __builtin_isfinite(X.t1) && !ev_less(X.t1, 1, X.t0, 0);
            R.t0 = X.t0;
            R.s0 = X.s0;
            R.c0 = X.c0;
        }
        return;
    }
    if (op == RT_CSG_UNION) {
        // Closed form of the union sweep when no comparison of the sort can
        // tie: four finite events, every pair farther apart than the
        // comparator's 1e-6 (so event_less is plain '<' and the sorted order
        // is the numeric one) and each interval ordered (t0 < t1).  Then the
        // first event is the earlier entry X; the result is X, extended to
        // the other interval Y's exit when Y enters before X exits - or, when
        // the origin lies inside A or B, the same from t = 0 with the
        // inside-at-origin entry (csg.cpp:98-152).  Other lanes take the
        // general sweep below.
        const real e = RV(1e-6);
        const bool easy = __builtin_isfinite(A.t0) && __builtin_isfinite(A.t1) && __builtin_isfinite(B.t0) &&
                          __builtin_isfinite(B.t1) && (A.t1 - A.t0 > e) && (B.t1 - B.t0 > e) &&
                          (fabs_r(A.t0 - B.t0) > e) && (fabs_r(A.t0 - B.t1) > e) && (fabs_r(A.t1 - B.t0) > e) &&
                          (fabs_r(A.t1 - B.t1) > e);
        if (easy) {
            cnt.ev(EV_COMB_EASY);
            const bool inA = (A.t0 < e) && (A.t1 > e);
            const bool inB = (B.t0 < e) && (B.t1 > e);
            const bool xa = inA || (!inB && A.t0 < B.t0);
            const real x1 = xa ? A.t1 : B.t1;
            const real y0 = xa ? B.t0 : A.t0;
            const real y1 = xa ? B.t1 : A.t1;
            const bool ext_y = (y0 < x1) && (y1 > x1);
            const bool org = inA || inB;
            const int xc0 = xa ? A.c0 : B.c0;
            R.ok = 1;
            R.t0 = org ? RV(0.0) : (xa ? A.t0 : B.t0);
            R.s0 = xa ? A.s0 : B.s0;
            R.c0 = org ? ((xc0 & ~REF_FLIP) | REF_ORIGIN) : xc0;
            R.t1 = ext_y ? y1 : x1;
            R.s1 = (ext_y != xa) ? A.s1 : B.s1;
            R.c1 = (ext_y != xa) ? A.c1 : B.c1;
            return;
        }
    }
    cnt.ev(EV_COMB_GEN);
    // Finite events in push order a0, a1, b0, b1 (csg.cpp:76-81).
    real et[4];
    int ec[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        et[k] = RV(0.0);
        ec[k] = 0;
    }
    int n = 0;
    {
        const real tv[4] = {A.t0, A.t1, B.t0, B.t1};
        const bool pv[4] = {A.ok && __builtin_isfinite(A.t0), A.ok && __builtin_isfinite(A.t1),
                            B.ok && __builtin_isfinite(B.t0), B.ok && __builtin_isfinite(B.t1)};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool here = pv[e] && n == k;
                et[k] = here ? tv[e] : et[k];
                ec[k] = here ? e : ec[k];
            }
            n += pv[e] ? 1 : 0;
        }
    }
    // libstdc++ __insertion_sort (stl_algo.h:1819-1871) with the non-strict
    // comparator, unrolled over the fixed <= 4 slots.
#pragma unroll
    for (int i = 1; i < 4; ++i) {
        if (i < n) {
            const real vt = et[i];
            const int vc = ec[i];
            if (ev_less(vt, vc, et[0], ec[0])) {
#pragma unroll
                for (int k = i; k > 0; --k) {
                    et[k] = et[k - 1];
                    ec[k] = ec[k - 1];
                }
                et[0] = vt;
                ec[0] = vc;
            } else {
                bool moving = true;
                int last = i;
#pragma unroll
                for (int k = i; k > 0; --k) {
                    if (moving && ev_less(vt, vc, et[k - 1], ec[k - 1])) {
                        et[k] = et[k - 1];
                        ec[k] = ec[k - 1];
                        last = k - 1;
                    } else {
                        moving = false;
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k == last) {
                        et[k] = vt;
                        ec[k] = vc;
                    }
            }
        }
    }
    bool inA = A.ok && (A.t0 < RV(1e-6)) && (A.t1 > RV(1e-6));
    bool inB = B.ok && (B.t0 < RV(1e-6)) && (B.t1 > RV(1e-6));
    bool inR = csg_combine(op, inA, inB);
    const bool origin = inR;
    bool haveEnter = inR;
    int enterE = -1, exitE = -1;
    bool flipE = false, flipX = false;
    real tEnt = RV(0.0), tExt = RT_INF;
    const bool originFromA = inA;
    bool done = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < n && !done) {
            const bool before = inR;
            const int e = ec[k];
            const bool enter = (e & 1) == 0;
            if ((e >> 1) == 0) inA = enter;
            else inB = enter;
            const bool after = csg_combine(op, inA, inB);
            if (!before && after) {
                haveEnter = true;
                tEnt = et[k];
                enterE = e;
                flipE = (op == RT_CSG_DIFFERENCE) && e == 3;
            } else if (before && !after) {
                tExt = et[k];
                exitE = e;
                flipX = (op == RT_CSG_DIFFERENCE) && e == 2;
                done = true;
            }
            if (!done) inR = after;
        }
    }
    if (!haveEnter || !__builtin_isfinite(tExt)) return;
    R.ok = 1;
    R.t0 = tEnt;
    R.t1 = tExt;
    if (enterE < 0) {
        // origin hit: material source = A.h0 if inside A else B.h0 (leaf materials are never null here)
        (void)origin;
        R.s0 = originFromA ? A.s0 : B.s0;
        R.c0 = ((originFromA ? A.c0 : B.c0) & ~REF_FLIP) | REF_ORIGIN;
    } else {
        R.s0 = enterE == 0 ? A.s0 : enterE == 1 ? A.s1 : enterE == 2 ? B.s0 : B.s1;
        R.c0 = (enterE == 0 ? A.c0 : enterE == 1 ? A.c1 : enterE == 2 ? B.c0 : B.c1) | (flipE ? REF_FLIP : 0);
    }
    R.s1 = exitE == 0 ? A.s0 : exitE == 1 ? A.s1 : exitE == 2 ? B.s0 : B.s1;
    R.c1 = (exitE == 0 ? A.c0 : exitE == 1 ? A.c1 : exitE == 2 ? B.c0 : B.c1) | (flipX ? REF_FLIP : 0);
}

// ------------------------------------------------------------ f32 culling
// Cull tests run in float (full-rate VALU; the trace itself is FP64).  They
// are conservative: "false" only when the segment [t0, t1] of the ray stays
// farther than r from the ball's centre even after the float rounding of
// every input and operation (the host grows each ball by 1e-6 of its scale,
// float_ball() in scene_compile.cpp; the test adds 4e-6 of the magnitudes it
// works with).  NaN rays always pass.  Culling therefore never changes a
// result, only skips work no lane needs.
constexpr float RT_INF_F = __builtin_inff();

// Square root for the f32 cull tests: the hardware v_sqrt_f32 (~1 ulp, one
// instruction) instead of the correctly rounded sequence (~15): every test
// carries a margin of >= 1e-6 of the magnitudes involved, far above 1 ulp.
__device__ __forceinline__ float sqrt_cull(float x) { return __builtin_amdgcn_sqrtf(x); }

struct FRay {
    float ox, oy, oz, dx, dy, dz;
};

__device__ __forceinline__ FRay to_fray(const DRay& r) {
    return FRay{(float)r.o.x, (float)r.o.y, (float)r.o.z, (float)r.d.x, (float)r.d.y, (float)r.d.z};
}

// The f32 cull tests work on (x, y) pairs as packed two-float vectors: on
// gfx950 v_pk_add/mul/fma_f32 do both halves in one VALU issue, and the
// trace kernels are VALU-issue bound.  Each half rounds exactly like the
// scalar operation (the margins never relied on a particular order).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v f2(float x, float y) { return f2v{x, y}; }
__device__ __forceinline__ f2v f2s(float s) { return f2v{s, s}; }
__device__ __forceinline__ f2v pk_fma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
// |w|^2 and w.a with w = (wxy, wz)
__device__ __forceinline__ float dot_pk(f2v axy, float az, f2v bxy, float bz) {
    const f2v p = axy * bxy;
    return __builtin_fmaf(az, bz, p.x + p.y);
}

__device__ __forceinline__ bool ball_touch(const float* g, const FRay& r, float t0, float t1) {
    const f2v dxy = f2(r.dx, r.dy);
    const f2v oxy = f2(r.ox, r.oy) - f2(g[0], g[1]);
    const float oz = r.oz - g[2];
    const float b = dot_pk(oxy, oz, dxy, r.dz);
    const float t = __builtin_fminf(__builtin_fmaxf(-b, t0), t1);   // closest point of the segment
    const f2v qxy = pk_fma(f2s(t), dxy, oxy);
    const float qz = __builtin_fmaf(t, r.dz, oz);
    const float q2 = dot_pk(qxy, qz, qxy, qz);
    const float e = 4e-6f * (__builtin_fabsf(oxy.x) + __builtin_fabsf(oxy.y) + __builtin_fabsf(oz) + __builtin_fabsf(t) + g[3]);
    const float R = g[3] + e;
    return !(q2 > R * R);
}

// Compact CSG program [pc0, pc1) on the frame ray r: the root interval.
// The top two stack entries are plain locals (VGPRs); only trees that are
// not left-deep folds touch the spill array (scratch), at uniform indices.
//
// Leaf line mask (lmask, wave-uniform; all ones = none): bit k clear means
// that no lane's LINE meets the k-th leaf's ball (k = order of the program's
// OP_LEAF_IVL ops = DevObj::pb0 ball order), so every lane's interval of that
// leaf is empty (Sphere::interval, geometry.cpp:48-78: disc < 0) and the leaf
// is pushed as the empty interval without its FP64 evaluation; an operand
// group whose leaves are all clear is skipped as one empty combine.  Exact by
// construction: an empty interval is what the skipped evaluation returns.
template <bool DEEP, class CT>
__device__ __forceinline__ CIvl run_compact(const DevScene& S, int pc0, int pc1, const DRay& r, CT& cnt,
                                            uint64_t lmask = ~0ull, bool use_mask = false) {
    CIvl tos, nos;
    tos.ok = nos.ok = 0;
    tos.t0 = tos.t1 = tos.s0 = tos.s1 = nos.t0 = nos.t1 = nos.s0 = nos.s1 = RV(0.0);
    tos.c0 = tos.c1 = nos.c0 = nos.c1 = 0;
    constexpr int NSP = DEEP ? kMaxIvlSpill : 1;
    real sp_t0[NSP], sp_t1[NSP], sp_s0[NSP], sp_s1[NSP];
    int sp_ok[NSP], sp_c0[NSP], sp_c1[NSP];
    int sp = 0;   // stack entries (wave-uniform)
    int li = 0;   // leaf ordinal (wave-uniform)
    const FRay fr = to_fray(r);
    for (int pc = pc0; pc < pc1; ++pc) {
        const DevOp op = S.ops[pc];
        if (op.op == rtamd::OP_LEAF_IVL) {
            CIvl v;
            if (use_mask && !((lmask >> (li & 63)) & 1ull)) {
                cnt.inc(RT_OPC_CULLED);
                v.ok = 0;
                v.t0 = v.t1 = v.s0 = v.s1 = RV(0.0);
                v.c0 = v.c1 = 0;
            } else {
                cnt.pb(PH_CSG_LEAF);
                leaf_ivl_c(&S.nodes[op.node], pc, r, v, cnt);
                cnt.pe(PH_CSG_LEAF);
            }
            ++li;
            if (DEEP && sp >= 2) {
                const int k = sp - 2;
                sp_ok[k] = nos.ok; sp_t0[k] = nos.t0; sp_t1[k] = nos.t1; sp_s0[k] = nos.s0; sp_s1[k] = nos.s1;
                sp_c0[k] = nos.c0; sp_c1[k] = nos.c1;
            }
            nos = tos;
            tos = v;
            ++sp;
        } else if (op.op == rtamd::OP_IVL_GROUP) {
            // the full line: Primitive::interval has no range
            const int nl = op.top / 2;   // leaves of the group (leaf + CSG op each)
            const bool skip = use_mask ? ((lmask >> (li & 63)) & ((nl >= 64) ? ~0ull : ((1ull << nl) - 1))) == 0
                                       : (S.cull && !__any(ball_touch(S.gb + 4 * op.node, fr, -RT_INF_F, RT_INF_F)));
            if (skip) {
                li += nl;
                cnt.inc(RT_OPC_CULLED);
                CIvl e, v;
                e.ok = 0;
                e.t0 = e.t1 = e.s0 = e.s1 = RV(0.0);
                e.c0 = e.c1 = 0;
                csg_c(op.csg_op, tos, e, v, cnt);
                tos = v;
                pc += op.top;
            }
        } else {
            CIvl v;
            cnt.pb(PH_CSG_COMB);
            csg_c(op.csg_op, nos, tos, v, cnt);
            cnt.pe(PH_CSG_COMB);
            tos = v;
            if (DEEP && sp >= 3) {
                const int k = sp - 3;
                nos.ok = sp_ok[k]; nos.t0 = sp_t0[k]; nos.t1 = sp_t1[k]; nos.s0 = sp_s0[k]; nos.s1 = sp_s1[k];
                nos.c0 = sp_c0[k]; nos.c1 = sp_c1[k];
            }
            --sp;
        }
    }
    return tos;
}

// Sphere::interval (geometry.cpp:48-78) of a fold leaf, compact form.
template <class CT>
__device__ __forceinline__ void fold_leaf_ivl(const FoldT& L, const DRay& r, CIvl& o, CT& cnt) {
    cnt.inc(RT_OPC_SPHERE_IVL);
    cnt.ev(EV_FOLD_LEAF);
    o.c0 = L.pc;
    o.c1 = L.pc | REF_ROOT1;
    const real r0 = L.r;
    V3 oc = v3(r.o.x - L.c[0], r.o.y - L.c[1], r.o.z - L.c[2]);
    const real half_b = dot3(oc, r.d);
    const real cterm = dot3(oc, oc) - r0 * r0;
    const real disc = half_b * half_b - RV(1.0) * cterm;
    o.ok = !(disc < RV(0.0));
    const real sq = sqrt_r(o.ok ? disc : RV(0.0));
    real t0 = (-half_b - sq) / RV(1.0);
    real t1 = (-half_b + sq) / RV(1.0);
    if (t0 > t1) {
        const real tt = t0;
        t0 = t1;
        t1 = tt;
    }
    o.t0 = o.s0 = t0;
    o.t1 = o.s1 = t1;
    if (o.ok) cnt.inc(RT_OPC_SPHERE_IVL_HIT);
}

// CSG::interval of a fold object (DevObj::nfold > 0): the left-deep fold
// acc = leaf_0 op leaf_1 op ... (csg.cpp:61-163, combined by csg_c exactly
// as run_compact would), with lmask (wave-uniform) naming the leaves some
// lane's line can meet.  A leaf outside the mask has an empty interval in
// every lane, so it is not evaluated; combining with an empty interval is
// idempotent (csg_c: acc op empty = f(acc), f(f(acc)) = f(acc)), so a run of
// such leaves costs one empty combine.  Exact by construction.
template <class CT>
__device__ __forceinline__ CIvl run_fold(const DevScene& S, const DevObj& ob, const DRay& r, uint64_t lmask,
                                         CT& cnt) {
    const FoldT* L = S.fold + ob.fold0;
    CIvl acc, e;
    e.ok = 0;
    e.t0 = e.t1 = e.s0 = e.s1 = RV(0.0);
    e.c0 = e.c1 = 0;
    if (lmask & 1ull) fold_leaf_ivl(L[0], r, acc, cnt);
    else acc = e;
    bool norm = false;   // acc is already a fixed point of the empty combine (wave-uniform)
    for (int k = 1; k < ob.nfold; ++k) {
        CIvl v;
        if (!((lmask >> k) & 1ull)) {
            cnt.inc(RT_OPC_CULLED);
            if (norm) continue;
            norm = true;
            v = e;
        } else {
            fold_leaf_ivl(L[k], r, v, cnt);
            norm = false;
        }
        CIvl R;
        csg_c(ob.fold_op, acc, v, R, cnt);
        acc = R;
    }
    return acc;
}

// Leaf Primitive::intersect without normal (t and acceptance only).
template <class CT>
__device__ __forceinline__ bool leaf_hit_t(const NodeT* nd, const DRay& r, real tmin, real tmax, real& t,
                                           CT& cnt) {
    if (nd->kind == RT_NODE_HALFSPACE) {   // geometry.cpp:90-106
        cnt.inc(RT_OPC_HALF_ISECT);
        const V3 n = ld3(nd->v + 3);
        const real ndotd = dot3(n, r.d);
        if (fabs_r(ndotd) < RV(1e-12)) return false;
        V3 diff = v3(nd->v[0] - r.o.x, nd->v[1] - r.o.y, nd->v[2] - r.o.z);
        t = dot3(n, diff) / ndotd;
        const bool ok = !(t < tmin || t > tmax);
        if (ok) cnt.inc(RT_OPC_HALF_ISECT_HIT);
        return ok;
    }
    cnt.inc(RT_OPC_SPHERE_ISECT);   // geometry.cpp:12-37
    const real rad = nd->v[3];
    V3 oc = v3(r.o.x - nd->v[0], r.o.y - nd->v[1], r.o.z - nd->v[2]);
    const real half_b = dot3(oc, r.d);
    const real cterm = dot3(oc, oc) - rad * rad;
    const real disc = half_b * half_b - RV(1.0) * cterm;
    if (disc < RV(0.0)) return false;
    const real sq = sqrt_r(disc);
    t = (-half_b - sq) / RV(1.0);
    if (t < tmin || t > tmax) {
        t = (-half_b + sq) / RV(1.0);
        if (t < tmin || t > tmax) return false;
    }
    cnt.inc(RT_OPC_SPHERE_ISECT_HIT);
    return true;
}

// Normal / front_face / material of a leaf hit at point p on frame ray r.
template <class CT>
__device__ __forceinline__ void leaf_shading(const NodeT* nd, const DRay& r, V3 p, DHit& h, CT& cnt) {
    if (nd->kind == RT_NODE_HALFSPACE) {
        set_face_normal(h, r, ld3(nd->v + 3));
        h.mat = nd->mat;
        return;
    }
    const real rad = nd->v[3];
    const auto oq = div3(p.x - nd->v[0], p.y - nd->v[1], p.z - nd->v[2], rad);
    const V3 outward = v3(oq.x, oq.y, oq.z);
    set_face_normal(h, r, outward);
    h.mat = nd->kind == RT_NODE_SPHERE ? nd->mat : pick_region_u(nd, outward, cnt);   // (u = the outward normal)
}

// Resolve a compact hit reference on frame ray r into (n, ff, mat).
template <class CT>
__device__ __forceinline__ void resolve_ref(const DevScene& S, const DRay& r, real ts, int code, DHit& h,
                                            CT& cnt) {
    const NodeT* nd = &S.nodes[S.ops[code & REF_PC_MASK].node];
    const V3 p = __builtin_isfinite(ts) ? ray_at(r, ts) : r.o;
    leaf_shading(nd, r, p, h, cnt);
    if (code & REF_ORIGIN) {
        h.n = v3(RV(0.0), RV(0.0), RV(0.0));
        h.ff = 1;
    }
    if (code & REF_FLIP) h.ff = 0;
}

// Ray at depth k of an object's transform chain (k = 0: world).
__device__ __forceinline__ DRay chain_ray(const DevScene& S, int pc0, int k, const DRay& world) {
    DRay r = world;
    for (int i = 0; i < k; ++i) r = local_ray(&S.nodes[S.ops[pc0 + i].node], r);
    return r;
}


// Primitive::intersect(object, ray, tmin, tmax): hit t, hit point p and a lazy
// reference (ts, code) resolved later by resolve_hit().
template <bool EAGER, bool DEEP, class CT>
__device__ __forceinline__ bool object_hit(const DevScene& S, const DevObj& ob, const DRay& world, real tmin,
                                           real tmax, real& t, V3& p, real& ts, int& code, CT& cnt,
                                           uint64_t lmask = ~0ull, bool use_mask = false) {
    if (!kCsg<CT> || ob.kind <= rtamd::OBJ_POKE) {
        const bool ok = leaf_hit_t(&S.nodes[ob.node], world, tmin, tmax, t, cnt);
        p = ray_at(world, t);
        ts = t;
        code = 0;
        return ok;
    }
    if (ob.kind == rtamd::OBJ_CHAIN) {
        // transforms (transform.cpp): local ray, child on [0,inf), map back, project t
        DRay cur = world;
        cnt.pb(PH_CHAIN_XF);
        for (int k = 0; k < ob.m; ++k) {
            cnt.inc(RT_OPC_XFORM);
            cur = local_ray(&S.nodes[S.ops[ob.pc0 + k].node], cur);
        }
        cnt.pe(PH_CHAIN_XF);
        const real lo = ob.m ? RV(0.0) : tmin;
        const real hi = ob.m ? RT_INF : tmax;
        bool ok;
        if (ob.core == 0) {
            ok = leaf_hit_t(&S.nodes[ob.node], cur, lo, hi, t, cnt);
            p = ray_at(cur, t);
            ts = t;
            code = ob.cpc0;
        } else {   // CSG::intersect (csg.cpp:169-185)
            const CIvl R = (use_mask && ob.nfold > 0) ? run_fold(S, ob, cur, lmask, cnt)
                                                      : run_compact<DEEP>(S, ob.cpc0, ob.cpc1, cur, cnt, lmask, use_mask);
            t = dmax(R.t0, lo);
            ok = R.ok && (t < R.t1 && t < hi);
            p = v3(cur.o.x + cur.d.x * t, cur.o.y + cur.d.y * t, cur.o.z + cur.d.z * t);
            ts = R.s0;
            code = R.c0;
        }
        cnt.pb(PH_CHAIN_XF);
        for (int k = ob.m - 1; k >= 0; --k) {
            const DRay parent = (k == 0) ? world : chain_ray(S, ob.pc0, k, world);
            const NodeT* nd = &S.nodes[S.ops[ob.pc0 + k].node];
            const V3 wp = map_point(nd, p);
            const real wt = project_t_world(parent, wp);
            const real l = k ? RV(0.0) : tmin, h = k ? RT_INF : tmax;
            ok = ok && (wt > l && wt < h);
            p = wp;
            t = wt;
        }
        cnt.pe(PH_CHAIN_XF);
        return ok;
    }
    if constexpr (EAGER) {
        if (ob.kind == rtamd::OBJ_EAGER) {
            DHit h;
            const bool ok = run_program<EAGER>(S, ob.pc0, ob.pc1, world, tmin, tmax, t, h, cnt);
            p = h.p;
            ts = t;
            code = 0;
            return ok;
        }
    }
    return false;
}

// Full hit record (p, n, front_face, mat) of the winning object.
template <bool EAGER, class CT>
__device__ __forceinline__ void resolve_hit(const DevScene& S, int obj, const DRay& world, real tmin, V3 p,
                                            real ts, int code, DHit& h, CT& cnt) {
    const DevObj ob = S.objs[obj];
    h.p = p;
    if (!kCsg<CT> || ob.kind <= rtamd::OBJ_POKE) {
        leaf_shading(&S.nodes[ob.node], world, p, h, cnt);
        return;
    }
    if (ob.kind == rtamd::OBJ_CHAIN) {
        const DRay cur = chain_ray(S, ob.pc0, ob.m, world);
        if (ob.core == 0) leaf_shading(&S.nodes[ob.node], cur, ray_at(cur, ts), h, cnt);
        else resolve_ref(S, cur, ts, code, h, cnt);
        for (int k = ob.m - 1; k >= 0; --k) {   // normals back through the chain
            const DRay parent = (k == 0) ? world : chain_ray(S, ob.pc0, k, world);
            const V3 wn = map_normal(&S.nodes[S.ops[ob.pc0 + k].node], h.n);
            set_face_normal(h, parent, wn);
        }
        return;
    }
    if constexpr (EAGER) {   // re-run the eager program (result does not depend on tmax)
        real t;
        run_program<EAGER>(S, ob.pc0, ob.pc1, world, tmin, RT_INF, t, h, cnt);
        h.p = p;
    }
}

// Scene::intersect (scene.cpp:10-24): closest hit; every object applies its
// own accept rule with tmax = closest-so-far, so ties resolve as in the
// reference (Sphere/HalfSpace accept t == tmax, CSG/transforms do not).
template <bool EAGER, bool DEEP, class CT>
__device__ bool scene_intersect(const DevScene& S, const DRay& r, real tmin, real tmax, real& t_best,
                                DHit& best, CT& cnt) {
    real closest = tmax;
    int win = -1;
    V3 wp = v3(RV(0.0), RV(0.0), RV(0.0));
    real wts = RV(0.0);
    int wcode = 0;
    const FRay fr = to_fray(r);
    const float ftmin = (float)tmin;
    for (int o = 0; o < S.n_objs; ++o) {
        const DevObj ob = S.objs[o];
        if (ob.kind == rtamd::OBJ_NEVER) continue;
        if (ob.has_bound && S.cull) {
            // groups skip their members; every bounded object is pre-tested
            if (!__any(ball_touch(ob.fb, fr, ftmin, (float)closest))) {
                cnt.inc(RT_OPC_CULLED);
                if (ob.kind == rtamd::OBJ_GROUP) o += ob.m;
                continue;
            }
        }
        if (ob.kind == rtamd::OBJ_GROUP) continue;
        real t = RV(0.0), ts = RV(0.0);
        V3 p;
        int code = 0;
        if (object_hit<EAGER, DEEP>(S, ob, r, tmin, closest, t, p, ts, code, cnt)) {
            closest = t;
            win = o;
            wp = p;
            wts = ts;
            wcode = code;
        }
    }
    if (win < 0) return false;
    resolve_hit<EAGER>(S, win, r, tmin, wp, wts, wcode, best, cnt);
    t_best = closest;
    return true;
}

// A lane's segment [o + t0 d, o + t1 d] against a bare half-space's plane
// (cull record type 3: c0 = (n, n.p), c1.y = its magnitude): false only if
// both ends lie on the same side by more than the f32 margin, where the
// plane crossing t of HalfSpace::intersect (geometry.cpp:90-106) is outside
// [t0, t1] in every rounding.  NaN passes.
__device__ __forceinline__ bool plane_touch(const float4 c0, const float4 c1, const FRay& r, float t0, float t1) {
    const float ax = __builtin_fmaf(t0, r.dx, r.ox), ay = __builtin_fmaf(t0, r.dy, r.oy), az = __builtin_fmaf(t0, r.dz, r.oz);
    const float bx = __builtin_fmaf(t1, r.dx, r.ox), by = __builtin_fmaf(t1, r.dy, r.oy), bz = __builtin_fmaf(t1, r.dz, r.oz);
    const float sa = __builtin_fmaf(c0.x, ax, __builtin_fmaf(c0.y, ay, c0.z * az)) - c0.w;
    const float sb = __builtin_fmaf(c0.x, bx, __builtin_fmaf(c0.y, by, c0.z * bz)) - c0.w;
    const float mag = __builtin_fabsf(ax) + __builtin_fabsf(ay) + __builtin_fabsf(az) + __builtin_fabsf(bx) +
                      __builtin_fabsf(by) + __builtin_fabsf(bz) + c1.y + 1.0f;
    const float m = 1e-5f * mag;
    return !((sa > m) & (sb > m)) & !((sa < -m) & (sb < -m));
}

// Scene::occluded (scene.cpp:33-42): any hit; per-lane early exit.
// lazy: r.d is the shadow direction BEFORE the Ray constructor's
// re-normalisation (core.h:278); the f32 culls use it as it is (a few FP64
// ulps from the normalised one, far inside their margins) and the exact ray
// is formed only once an object survives them (as scene_occluded_capsule).
template <bool EAGER, bool DEEP, class CT>
__device__ bool scene_occluded(const DevScene& S, const DRay& r0, real tmin, real tmax, CT& cnt, bool lazy = false) {
    bool hit = false;
    DRay r = r0;
    bool r_exact = !lazy;
    const FRay fr = to_fray(r0);
    const float ftmin = (float)tmin, ftmax = (float)tmax;
    for (int o = 0; o < S.n_objs; ++o) {
        if (__all(hit)) break;
        const DevObj ob = S.objs[o];
        if (ob.kind == rtamd::OBJ_NEVER) continue;
        if (ob.has_bound && S.cull) {
            if (!__any(!hit && ball_touch(ob.fb, fr, ftmin, ftmax))) {
                cnt.inc(RT_OPC_CULLED);
                if (ob.kind == rtamd::OBJ_GROUP) o += ob.m;
                continue;
            }
        } else if (S.cull && ob.kind != rtamd::OBJ_GROUP) {
            // a bare half-space: skipped unless some lane's segment crosses its plane
            const float4 c1 = S.ctab[2 * o + 1];
            if (__float_as_int(c1.x) == 3 && !__any(!hit && plane_touch(S.ctab[2 * o], c1, fr, ftmin, ftmax))) {
                cnt.inc(RT_OPC_CULLED);
                continue;
            }
        }
        if (ob.kind == rtamd::OBJ_GROUP) continue;
        if (!r_exact) {   // Ray::Ray (core.h:278) of the shadow ray (shading.cpp:98)
            r.d = normalized(r.d);
            r_exact = true;
        }
        // every lane evaluates (no divergent region between the loop's
        // wave-wide tests, see scene_occluded_wave); op-counting builds take
        // the same path and count only the reference's calls (lanes without
        // a hit yet)
        real t = RV(0.0), ts = RV(0.0);
        V3 p;
        int code = 0;
        cnt.gate(!hit);
        const bool h = object_hit<EAGER, DEEP>(S, ob, r, tmin, tmax, t, p, ts, code, cnt);
        cnt.gate(true);
        hit = hit || h;
    }
    return hit;
}


// ------------------------------------------- wave-level shadow-ray culling
// Every lane of the wave active AT THIS POINT.  The transposed tests (lane j
// tests object / leaf j for the whole wave) and the DPP / readlane bundle
// reductions are valid only then, so each of them checks the exec mask where
// it runs (a convergent read: __builtin_amdgcn_read_exec lowers to
// llvm.amdgcn.ballot(true), which the compiler cannot move across control
// flow) and otherwise falls back to the all-candidates mask.  Culling then
// stays exact whatever the compiler does with the surrounding regions.
__device__ __forceinline__ bool exec_full() { return __builtin_amdgcn_read_exec() == ~0ull; }

__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {   // every lane must be active
    // row_ror:1,2,4,8 (DPP) leaves each row's maximum in all its lanes
    v = umax32(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xf, 0xf, false));
    v = umax32(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xf, 0xf, false));
    v = umax32(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false));
    v = umax32(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false));
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    return umax32(umax32(r0, r1), umax32(r2, r3));
}

__device__ __forceinline__ float rdlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// A wave-uniform float computed by VALU math (which lands in a VGPR) moved
// back to an SGPR.  The shadow-bundle parameters live across the whole query:
// in SGPRs they free VGPRs for the paper kernel (7% faster there, measured);
// in the standard kernel they cost 1% and stay in VGPRs (UO = false).
template <bool On = true>
__device__ __forceinline__ float uni(float v) {
    if constexpr (On) return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
    else return v;
}


// A bundle's cone (or double cone, for lines): origins within rho of o,
// directions within theta of a (cth = cos theta, sth = sin theta).
struct Cone {
    f2v oxy, axy;
    float oz, az, cth, sth, rho, m5;
};
// |x| + |y| + |z| + r of a ball (the records carry it precomputed)
__device__ __forceinline__ float ball_mag(const float4 g) {
    return __builtin_fabsf(g.x) + __builtin_fabsf(g.y) + __builtin_fabsf(g.z) + g.w;
}

// The same bundle seen as LINES (Primitive::interval has no range, so a CSG
// leaf's interval is empty only if its whole line misses the leaf): every
// lane's line lies within rho of a line through o whose direction is within
// theta of +-a, so a ball can be touched only if the angle between w = c - o
// and the axis LINE is <= theta + asin(R / |w|): the double cone, cone_touch
// with |w.a|.  Conservative in f32 like cone_touch.
template <bool LINE>
__device__ __forceinline__ bool cone_touch_t(const float4 g, float gmag, const Cone& K) {
    const f2v wxy = f2(g.x, g.y) - K.oxy;
    const float wz = g.z - K.oz;
    const float m = __builtin_fmaf(1e-5f, gmag, K.m5);
    const float R = g.w + K.rho + m;
    const float L2 = dot_pk(wxy, wz, wxy, wz);
    const float wa0 = dot_pk(wxy, wz, K.axy, K.az);
    const float wa = LINE ? __builtin_fabsf(wa0) : wa0;
    // angle(w, a) <= theta + asin(R / |w|)  <=>  w.a >= cos(theta) sqrt(L2 - R^2) - sin(theta) R;
    // !(L2 > R^2): the bundle's origin region touches the ball (or NaN).  No
    // branch: lanes disagree on the first test.
    const float rhs = K.cth * sqrt_cull(L2 - R * R) - K.sth * R;
    return !(L2 > R * R) | !(wa + m < rhs);
}
__device__ __forceinline__ bool line_touch(const float* g, const Cone& K) {
    const float4 b = *reinterpret_cast<const float4*>(g);
    return cone_touch_t<true>(b, ball_mag(b), K);
}

template <class CT>
__device__ __forceinline__ void cnt_add(CT& cnt, int k, int n) {
    for (int i = 0; i < n; ++i) cnt.inc(k);
}
// Objects a culled BVH chunk holds (op-counting builds: RT_OPC_CULLED counts
// every object a query skipped, whether by its own test or its chunk's)
__device__ __forceinline__ int chunk_objects(const DevScene& S, int base) {
    int n = 0;
    for (int o = base; o < S.n_objs && o < base + 64; ++o) {
        const int k = S.objs[o].kind;
        n += (k != rtamd::OBJ_GROUP && k != rtamd::OBJ_NEVER) ? 1 : 0;
    }
    return n;
}


// ------------------------------------------------- capsule shadow culls
// A shadow query of a whole wave (every lane active; lanes that need no
// query pass need = false) is culled object by object in ONE transposed
// test instead of one wave-uniform ball test per object: the segments
// [o + tmin d, o + tmax d] of all querying lanes lie inside the capsule of
// radius rho around [C0, C1], C0 / C1 the first querying lane's endpoints
// and rho the largest distance of any lane's endpoint from them (a point
// (1-s) A_i + s B_i is within (1-s)|A_i - C0| + s|B_i - C1| of the axis).
// Lane j then tests object j's bounding ball against that capsule, and one
// ballot gives the objects any lane can reach.  Like ball_touch the test is
// conservative in f32 (a margin of 1e-5 of every magnitude involved), so it
// never drops an object some lane's segment touches: results are unchanged.
// The kernels without the wave BVH use it (configs 1-6: at most a few dozen
// objects, one transposed test per query); the BVH kernels use the
// light-centred culls below.
//
// A shadow bundle's capsule (wave-uniform): radius rho around the segment
// [a, b], u = b - a, iuu = 1 / |u|^2 (0 for a point), m5 = 1e-5 * the
// bundle's magnitude and rm5 = rho + m5 (the margins' uniform parts).
struct Capsule {
    f2v axy, bxy, uxy;
    float az, bz, uz, iuu, rho, m5, rm5;
    f2v abx, aby, abz;   // (a.x, b.x), ... for the half-space test
};
__device__ __forceinline__ bool capsule_touch(const float4 g, float gmag, const Capsule& K) {
    const f2v wxy = f2(g.x, g.y) - K.axy;
    const float wz = g.z - K.az;
    const float wu = dot_pk(wxy, wz, K.uxy, K.uz);
    // (iuu = 0 for a point capsule: s = 0; a non-finite wu makes q NaN: passes)
    const float s = __builtin_amdgcn_fmed3f(wu * K.iuu, 0.0f, 1.0f);
    const f2v qxy = pk_fma(f2s(-s), K.uxy, wxy);
    const float qz = __builtin_fmaf(-s, K.uz, wz);
    const float d2 = dot_pk(qxy, qz, qxy, qz);
    const float R = g.w + K.rho + __builtin_fmaf(1e-5f, gmag, K.m5);
    return !(d2 > R * R);   // NaN passes
}
__device__ __forceinline__ bool capsule_touch(const float* g, const Capsule& K) {
    const float4 b = *reinterpret_cast<const float4*>(g);
    return capsule_touch(b, ball_mag(b), K);
}


// Lane j's transposed test of object j's cull record (CompiledScene::ctab)
// against the capsule of radius rho around the segment [a, b] (u = b - a).
// Record word 5 (c1.y) is the magnitude of the record's ball or plane point.
__device__ __forceinline__ bool record_touch(const float4 c0, const float4 c1, const Capsule& K) {
    // Lanes test objects of different types side by side, so both tests run
    // on every lane and the type selects (no divergent branches, no exec
    // bookkeeping between the record's loads and the ballot).
    const int type = __float_as_int(c1.x);
    // a bare half-space: the segments cross its plane only if the capsule
    // does (both axis ends farther than rho on one side: no lane); n.x - n.p
    // in f32 is within 1e-6 of the magnitudes of the signed distance, far
    // inside the margin.  (sa, sb) as one packed pair.
    const f2v sab = pk_fma(f2s(c0.x), K.abx, pk_fma(f2s(c0.y), K.aby, f2s(c0.z) * K.abz)) - f2s(c0.w);
    const float m = __builtin_fmaf(1e-5f, c1.y, K.rm5);
    const bool plane = !((sab.x > m) & (sab.y > m)) & !((sab.x < -m) & (sab.y < -m));   // NaN passes
    const bool ball = capsule_touch(c0, c1.y, K);
    return (type == 1) | ((type == 2) & ball) | ((type == 3) & plane);
}

// Scene::occluded for the querying lanes of a fully active wave.  Returns
// false for lanes with need = false.
//
// r0 is the shadow ray BEFORE the Ray constructor's re-normalisation of its
// direction (core.h:278): the f32 culling works on it directly (the
// re-normalised direction differs by a few FP64 ulps, far inside every cull
// test's 1e-5 margins), and the exact FP64 ray (make_ray, one sqrt and three
// divisions per lane) is formed only when some candidate object survives the
// culls and is evaluated - most shadow queries of a wave end before that.
//
// BV (wave BVH kernels): S.objs is the Morton-ordered list in chunks of 64
// with a cull record per chunk (CompiledScene::wobjs / wchunk); one
// transposed test per 64 chunks skips every chunk no querying segment can
// reach, then each surviving chunk runs the object test below.  Occlusion is
// an OR over objects, so the order is free.
template <bool EAGER, bool DEEP, bool UO, bool BV = false, bool LEAD = false, class CT>
__device__ bool scene_occluded_capsule(const DevScene& S, const DRay& r0, real tmin, real tmax, bool need, bool wave_ok,
                                    CT& cnt) {
#if defined(RT_ABL) && RT_ABL == 1   // diagnostic ablation builds only (wrong images): no shadow queries
    return false;
#endif
    cnt.pb(PH_WAVE_SETUP);
    const FRay fr = to_fray(r0);
    DRay r = r0;           // the exact ray, formed on the first object evaluation (wave-uniform)
    bool r_exact = false;
    const float ftmin = (float)tmin, ftmax = (float)tmax;
    const uint64_t nm = __ballot(need);
    if (!nm) return false;
    cnt.ev(EV_SHQ);
    const int f = __builtin_ctzll(nm);
    // (the segment ends stay scalar: as packed (A, B) pairs they cost config 4
    // 8.51 -> 8.67 ms in register moves)
    const float Ax = __builtin_fmaf(ftmin, fr.dx, fr.ox), Ay = __builtin_fmaf(ftmin, fr.dy, fr.oy),
                Az = __builtin_fmaf(ftmin, fr.dz, fr.oz);
    const float Bx = __builtin_fmaf(ftmax, fr.dx, fr.ox), By = __builtin_fmaf(ftmax, fr.dy, fr.oy),
                Bz = __builtin_fmaf(ftmax, fr.dz, fr.oz);
    const bool fin = __builtin_isfinite(Ax + Ay + Az + Bx + By + Bz);
    // without the capsule (a partially active wave, or unbounded / non-finite
    // segments) every object is a candidate and each bounded one gets the
    // per-lane segment test
    const bool cap = wave_ok && exec_full() && !__any(need && !fin);
    const float ax = rdlane_f(Ax, f), ay = rdlane_f(Ay, f), az = rdlane_f(Az, f);
    const float bx = rdlane_f(Bx, f), by = rdlane_f(By, f), bz = rdlane_f(Bz, f);
    const float da = (Ax - ax) * (Ax - ax) + (Ay - ay) * (Ay - ay) + (Az - az) * (Az - az);
    const float db = (Bx - bx) * (Bx - bx) + (By - by) * (By - by) + (Bz - bz) * (Bz - bz);
    const float d = need ? __builtin_fmaxf(da, db) : 0.0f;
    const float rho = uni<UO>(cap ? sqrt_cull(__uint_as_float(wave_max_u32(__float_as_uint(d)))) : 0.0f);
    const float ux = uni<UO>(bx - ax), uy = uni<UO>(by - ay), uz = uni<UO>(bz - az);
    const float uu = __builtin_fmaf(ux, ux, __builtin_fmaf(uy, uy, uz * uz));
    const float mag = __builtin_fabsf(ax) + __builtin_fabsf(ay) + __builtin_fabsf(az) + __builtin_fabsf(bx) +
                      __builtin_fabsf(by) + __builtin_fabsf(bz) + rho + 1.0f;
    Capsule K;
    K.axy = f2(ax, ay), K.bxy = f2(bx, by), K.uxy = f2(ux, uy);
    K.az = az, K.bz = bz, K.uz = uz;
    K.iuu = uni<UO>(uu > 0.0f ? __builtin_amdgcn_rcpf(uu) : 0.0f);
    K.rho = rho;
    K.m5 = uni<UO>(1e-5f * mag);
    K.rm5 = uni<UO>(rho + 1e-5f * mag);
    K.abx = f2(ax, bx), K.aby = f2(ay, by), K.abz = f2(az, bz);
    const int lane = __lane_id();
    // line bundle for the CSG leaf masks, built on first use (cap only)
    bool lb_ready = false;
    Cone LB{f2(0.0f, 0.0f), f2(0.0f, 0.0f), 0.0f, 0.0f, -1.0f, 1.0f, 0.0f, 0.0f};
    bool hit = false;
    // the lead objects (CompiledScene::n_lead: unbounded, ahead of every
    // bounded one) as pseudo-chunk -1, each tested on its own - a bare
    // half-space by every querying lane's segment against its plane - then
    // the transposed tests over the objects behind them
    const int lead = (BV || !LEAD) ? 0 : S.n_lead;
    const int nch = BV ? S.n_chunks : (S.n_objs - lead + 63) >> 6;
    uint64_t cm = 0;   // (BV) chunks ch & ~63 .. +63 some querying segment can reach
    for (int ch = lead > 0 ? -1 : 0; ch < nch; ++ch) {
        int base;
        uint64_t m;
        if (ch < 0) {
            base = 0;
            m = 0;
            for (int o = 0; o < lead; ++o) {
                const float4 c1 = S.ctab[2 * o + 1];
                const int type = __float_as_int(c1.x);
                const bool pass = type == 1 || (type == 3 && (!(cap && S.cull) ||
                                                               __any(need && plane_touch(S.ctab[2 * o], c1, fr, ftmin, ftmax))));
                if (pass) m |= 1ull << o;
                else if (type != 0 && need) cnt.inc(RT_OPC_CULLED);
            }
            cnt.pe(PH_WAVE_SETUP);
        } else {
        if (ch > 0 || lead > 0) cnt.pb(PH_WAVE_SETUP);   // (phase builds: a later chunk's test timed from here)
        if constexpr (BV) {
            if ((ch & 63) == 0) {
                const int c = ch + lane;
                const int cr = c < nch ? c : nch - 1;
                const float4 k0 = S.wchunk[2 * cr], k1 = S.wchunk[2 * cr + 1];
                const bool pass = (c < nch) & record_touch(k0, k1, K);
                cm = (cap && exec_full()) ? __ballot(pass) : ~0ull;
            }
            if (!((cm >> (ch & 63)) & 1ull)) {
                if constexpr (kCounting<CT>)
                    if (need) cnt_add(cnt, RT_OPC_CULLED, chunk_objects(S, ch << 6));
                continue;
            }
        }
        base = lead + (ch << 6);
        const int nc = S.n_objs - base;
        const int j = base + lane;
        // the object's cull record (CompiledScene::ctab): one 32-byte load on
        // every lane (lanes past the last object re-read it and are masked)
        const int jr = j < S.n_objs ? j : S.n_objs - 1;
        const float4 c0 = S.ctab[2 * jr], c1 = S.ctab[2 * jr + 1];
        const bool pass = (j < S.n_objs) &
                          (cap ? record_touch(c0, c1, K)
                               : __float_as_int(c1.x) != 0);
        // (lane j tests object j only with the whole wave active; otherwise
        // every object of the chunk is a candidate)
        m = (cap && exec_full()) ? __ballot(pass) : (nc >= 64 ? ~0ull : ((1ull << nc) - 1));
        cnt.pe(PH_WAVE_SETUP);
#if defined(RT_ABL) && RT_ABL == 2   // diagnostic: setup + transposed test only
        if (m != 12345) return false;
#endif
        if constexpr (kCounting<CT>) {
            if (need) {
                int skipped = 0;
                for (int o = base; o < S.n_objs && o < base + 64; ++o) {
                    const int k = S.objs[o].kind;
                    if (k != rtamd::OBJ_GROUP && k != rtamd::OBJ_NEVER && !((m >> (o - base)) & 1)) ++skipped;
                }
                cnt_add(cnt, RT_OPC_CULLED, skipped);
            }
        }
        }
        while (m) {
            const int o = base + __builtin_ctzll(m);
            m &= m - 1;
            const DevObj ob = S.objs[o];
            if (ob.kind == rtamd::OBJ_GROUP || ob.kind == rtamd::OBJ_NEVER) continue;
            cnt.ev(EV_SH_CAND);
            cnt.pb(PH_OBJ_PREF);
            // CSG objects: no lane's segment reaches a leaf ball (DevObj::pb0);
            // otherwise the leaves whose balls no querying lane's line meets
            uint64_t lmask = ~0ull;
            bool use_mask = false;
            if (kCsg<CT> && cap && ob.npb > 0 && exec_full()) {
                const float* g = S.gb + 4 * (ob.pb0 + (lane < ob.npb ? lane : 0));
                const bool in = lane < ob.npb;
                const uint64_t cb = __ballot(in && capsule_touch(g, K));   // leaves the capsule reaches
                bool seg = cb != 0;
#ifndef RT_NO_LANE_LEAF_TEST
                // Then each lane's own segment against those leaf balls: the
                // object can occlude a lane only at a point within the slop
                // of one of its leaves' balls (leaf_prefilter,
                // scene_compile.cpp), so unless some lane's segment touches
                // one of them, no lane's query can hit it.  (A shadow ray
                // leaving the object's own surface starts outside every leaf
                // ball by its eps offset, so the self-shadow queries of a
                // wave on the object - whose capsule always reaches the
                // leaves around it - skip the evaluation.)  The exec mask is
                // full here (checked above), so cb is the whole wave's.
                if (seg) {
                    seg = false;
                    for (uint64_t mm = cb; mm && !seg; mm &= mm - 1) {
                        const float* gk = S.gb + 4 * (ob.pb0 + __builtin_ctzll(mm));
                        seg = __any(need && !hit && ball_touch(gk, fr, ftmin, ftmax));
                    }
                }
#endif
                if (!seg) {
                    if (need) cnt.inc(RT_OPC_CULLED);
                    cnt.pe(PH_OBJ_PREF);
                    continue;
                }
                if (!lb_ready) {
                    // line bundle of the querying lanes (lane f's line as the axis)
                    lb_ready = true;
                    const float lox = rdlane_f(fr.ox, f), loy = rdlane_f(fr.oy, f), loz = rdlane_f(fr.oz, f);
                    const float lax = rdlane_f(fr.dx, f), lay = rdlane_f(fr.dy, f), laz = rdlane_f(fr.dz, f);
                    const float dxo = fr.ox - lox, dyo = fr.oy - loy, dzo = fr.oz - loz;
                    const float do2 = need ? dxo * dxo + dyo * dyo + dzo * dzo : 0.0f;
                    const float dc = need ? __builtin_fmaxf(0.0f, 1.0f - __builtin_fmaf(fr.dx, lax, __builtin_fmaf(fr.dy, lay, fr.dz * laz)))
                                          : 0.0f;
                    const float lrho = uni<UO>(sqrt_cull(__uint_as_float(wave_max_u32(__float_as_uint(do2)))));
                    const float dcm = __uint_as_float(wave_max_u32(__float_as_uint(dc))) + 4e-6f;
                    const float lcth = uni<UO>(1.0f - dcm);
                    LB.oxy = f2(lox, loy), LB.axy = f2(lax, lay), LB.oz = loz, LB.az = laz;
                    LB.cth = lcth;
                    LB.sth = uni<UO>(sqrt_cull(__builtin_fmaxf(0.0f, 1.0f - lcth * lcth)) + 1e-6f);
                    LB.rho = lrho;
                    LB.m5 = uni<UO>(1e-5f * (__builtin_fabsf(lox) + __builtin_fabsf(loy) + __builtin_fabsf(loz) + lrho + 1.0f));
                }
#ifdef RT_NO_LEAF_MASK
                use_mask = false;
#else
                use_mask = LB.cth > 0.0f;
#endif
                if (use_mask) {
                    const bool full = exec_full();
                    const uint64_t b = __ballot(in && line_touch(g, LB));
                    lmask = full ? b : ~0ull;
                }
            }
            if (S.cull && ob.has_bound) {   // per-lane segment test (f32, cheaper than an FP64 miss)
                if (!__any(need && !hit && ball_touch(ob.fb, fr, ftmin, ftmax))) {
                    if (need) cnt.inc(RT_OPC_CULLED);
                    cnt.pe(PH_OBJ_PREF);
                    continue;
                }
            }
            cnt.pe(PH_OBJ_PREF);
#if defined(RT_ABL) && RT_ABL == 3   // diagnostic: everything but the shadow object evaluations
            if (m != 12345) continue;
#endif
            const bool csg_obj = ob.kind == rtamd::OBJ_CHAIN && ob.core != 0;
            if (csg_obj) cnt.pb(PH_SHADOW_CSG);
            cnt.pb(PH_OBJ_HIT);
            cnt.ev(EV_SH_HIT);
            if (csg_obj) cnt.ev(EV_SH_CSG);
            if (!r_exact) {   // Ray::Ray (core.h:278) of the shadow ray (shading.cpp:98), in place
                r.d = normalized(r.d);
                r_exact = true;
            }
            {
                // every lane evaluates (the wave runs the object anyway) and
                // only querying lanes without a hit take the result: no
                // divergent region between this loop's wave-wide tests.  The
                // op-counting builds take the same path and count only the
                // reference's calls (querying lanes without a hit yet).
                real t = RV(0.0), ts = RV(0.0);
                V3 p;
                int code = 0;
                const bool take = need && !hit;
                cnt.gate(take);
                const bool h = object_hit<EAGER, DEEP>(S, ob, r, tmin, tmax, t, p, ts, code, cnt, lmask, use_mask);
                cnt.gate(true);
                hit = hit || (take && h);
            }
            cnt.pe(PH_OBJ_HIT);
            if (csg_obj) cnt.pe(PH_SHADOW_CSG);
            if (__all(hit || !need)) return hit;
        }
    }
    return hit;
}


// ------------------------------------------------ light-centred shadow culls
// (the wave-BVH kernels: scenes of many objects, where the per-object cost of
// the transposed test dominates).  Every shadow segment of one light ends at
// that light (shading.cpp:79-104): lane i's ray starts at o_i = p_i + n_i
// eps_i toward wi_i = (L - p_i) / dist_i and runs over t in (eps_i, dist_i -
// eps_i), so each of its points (p_i + t wi_i) + n_i eps_i lies within eps_i
// of the segment [L, p_i].  When every querying lane's hit point lies within
// rho of q (ShadowHull, once per shade() call: q halfway between the first
// querying lane's hit point and the one farthest from it), all of a wave's
// segments for light L lie within emax (the largest eps) of the hull of L
// and the ball B(q, rho): the cone from L with axis a = (q - L) / |q - L| and
// half-angle asin(rho / |q - L|), cut at the ball.  The cull records are
// light-relative and computed once per scene on the host
// (CompiledScene::lrec / lgb: w = c - L and |w|^2 of each ball), so a
// record's transposed test is one dot product and a few compares.  The
// per-lane test of a surviving candidate stays ball_touch on the lane's
// actual segment (its eps offset is what clears the object the lane itself
// lies on); a bare half-space that passes the hull test (hit points on its
// own plane) gets a per-lane test of the segment's start against its plane.
// Conservative in f32 (margins of >= 1e-6 of the magnitudes involved); a wave
// whose hull is not valid (a hit point within 0.1 of the light, where the
// reference clamps the distance, or L inside the hull ball) tests every
// object per lane instead.  Measured against the capsule (profiles/r04_*):
// 4096 random spheres 52.0 -> 41.7 ms, the 576-sphere lattice 7.10 -> 4.88
// ms, paper mode 24.7 -> 19.2 ms; on config 4 / 5 (15 / 65 objects) the
// capsule's per-query setup is no dearer and it needs fewer registers, so the
// kernels without the BVH keep it.
struct ShadowHull {
    float qx, qy, qz, rho, emax;
    bool ok;
};
template <bool UO>
__device__ __forceinline__ ShadowHull shadow_hull(const V3& p, real eps, bool valid, bool wave_ok) {
    ShadowHull H{0.0f, 0.0f, 0.0f, 0.0f, 0.0f, false};
    const float px = (float)p.x, py = (float)p.y, pz = (float)p.z;
    const uint64_t vm = __ballot(valid);
    const bool full = wave_ok && exec_full();
    const int f = vm ? __builtin_ctzll(vm) : 0;
    H.qx = rdlane_f(px, f);
    H.qy = rdlane_f(py, f);
    H.qz = rdlane_f(pz, f);
    const float e = valid ? (float)eps : 0.0f;
    const bool bad = valid && !__builtin_isfinite(px + py + pz);
    if (full && vm && !__any(bad)) {
        // centre: halfway between lane f's hit point and the one farthest
        // from it (about half the radius a corner lane's ball would have)
        float dx = px - H.qx, dy = py - H.qy, dz = pz - H.qz;
        const float d2f = valid ? __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz)) : 0.0f;
        const uint32_t mf = wave_max_u32(__float_as_uint(d2f));
        const uint64_t gm = __ballot(valid && __float_as_uint(d2f) == mf);
        const int g = gm ? __builtin_ctzll(gm) : f;
        H.qx = uni<UO>(0.5f * (H.qx + rdlane_f(px, g)));
        H.qy = uni<UO>(0.5f * (H.qy + rdlane_f(py, g)));
        H.qz = uni<UO>(0.5f * (H.qz + rdlane_f(pz, g)));
        dx = px - H.qx, dy = py - H.qy, dz = pz - H.qz;
        const float d2 = valid ? __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz)) : 0.0f;
        H.rho = uni<UO>(sqrt_cull(__uint_as_float(wave_max_u32(__float_as_uint(d2)))));
        H.emax = uni<UO>(__uint_as_float(wave_max_u32(__float_as_uint(e))) * 1.000001f);
        H.ok = __builtin_isfinite(H.rho);
    }
    return H;
}

// One light's cone over a ShadowHull (wave-uniform): axis a, cos / sin of
// the half-angle beta, the hull ball's distance dq along the axis and radius
// rho; beyond dq the hull is inside the cylinder of radius rend = rho / cb
// up to xe = dq + rho.
struct LightCone {
    float ax, ay, az, cb, sb, dq, xe, rend, rho, emax, qx, qy, qz, mq;
};

// Ball record (w = c - L, |w|^2), (type, r, |w|_1 + r) against the hull: the
// ball grown by emax (r') touches it only if L lies in it, or, with x the
// axial and p the perpendicular coordinate of w: for x < dq (the cone
// body) p cos(beta) <= r' + max(x, 0) sin(beta) and x >= -r'; for x >= dq
// (the end) max(0, x - xe)^2 + max(0, p - rend)^2 <= r'^2.
__device__ __forceinline__ bool lrec_ball_cone(const float4 c0, float r, float magw, const LightCone& K) {
    const float x = dot_pk(f2(c0.x, c0.y), c0.z, f2(K.ax, K.ay), K.az);
    const float p2 = __builtin_fmaxf(0.0f, __builtin_fmaf(-x, x, c0.w));
    const float mw = 4e-6f * magw;
    const float re = r + K.emax + mw;
    const float m2 = 1e-6f * magw * magw;   // (the rounding of W2 - x^2: <= 4e-7 magw^2)
    const float re2 = __builtin_fmaf(re, re, m2);
    const float rhs = __builtin_fmaf(__builtin_fmaxf(x, 0.0f), K.sb, re);
    const bool inside = !(c0.w > re2);
    const bool body = !(p2 * (K.cb * K.cb) > __builtin_fmaf(rhs, rhs, m2)) & !(x < -re - mw);
    const float ex = __builtin_fmaxf(0.0f, x - K.xe);
    const float ep = __builtin_fmaxf(0.0f, sqrt_cull(p2) - K.rend - mw);
    const bool end = !(__builtin_fmaf(ex, ex, ep * ep) > re2);
    return inside | ((x < K.dq) ? body : end);   // NaN passes
}

// Lane j's transposed test of its light-relative record (types: 0 never,
// 1 always, 2 ball, 3 bare half-space plane (n, n.p), (type, n.L - n.p, mag)).
__device__ __forceinline__ bool lrec_touch(const float4 c0, const float4 c1, const LightCone& K) {
    const int type = __float_as_int(c1.x);
    const bool ball = lrec_ball_cone(c0, c1.y, c1.z, K);
    // a plane: every segment point's signed distance lies between the
    // light's (c1.y) and its hit point's (within rho of q's) +- emax
    const float sq = dot_pk(f2(c0.x, c0.y), c0.z, f2(K.qx, K.qy), K.qz) - c0.w;
    const float mp = 1e-5f * (c1.z + K.mq + K.rho) + K.emax;
    const float sl = c1.y;
    const bool plane = !((sl > mp) & (sq - K.rho > mp)) & !((sl < -mp) & (sq + K.rho < -mp));   // NaN passes
    return (type == 1) | ((type == 2) & ball) | ((type == 3) & plane);
}

// A world ball (c, r) (wave BVH chunk records) against the cone, made
// light-relative on the fly.
__device__ __forceinline__ bool ball_cone(const float4 g, const LightCone& K, float Lx, float Ly, float Lz) {
    const float wx = g.x - Lx, wy = g.y - Ly, wz = g.z - Lz;
    const float w2 = __builtin_fmaf(wx, wx, __builtin_fmaf(wy, wy, wz * wz));
    const float magw = __builtin_fabsf(wx) + __builtin_fabsf(wy) + __builtin_fabsf(wz) + g.w;
    return lrec_ball_cone(make_float4(wx, wy, wz, w2), g.w, magw, K);
}

// Sub-bundles of a shadow query (the wave BVH kernels).  Where a tile
// straddles depth edges of an incoherent scene its hull is wide and lets
// dozens of objects through that no segment reaches (a pixel's 8 samples do
// not help: one straddling pixel is as wide as the tile).  So the querying
// lanes are clustered greedily by their ray origins: the first remaining lane
// q and every remaining lane within tau = 1/64 of q's distance to the light
// form a cluster of radius rho_c <= tau, at most kMaxClusters of them (the
// last takes every lane left).  A cluster's segments start within rho_c of
// q_c (plus eps along the ray) and end within 2 eps of L, so they lie within
// 2 emax of the cone from L over B(q_c, rho_c + emax).  Every lane forms its
// own cluster's cone; lane j tests its record (c0, c1) against each cluster's
// cone (read from the cluster's first lane) and the ballot of "any cluster
// reaches it" refines the wave's candidate mask.  Conservative like the wave
// hull; a cluster whose cone is not valid keeps every object.  Every lane
// must be active.
#ifndef RT_SUB_MIN
#define RT_SUB_MIN 1
#endif
constexpr int kSubBundleMin = RT_SUB_MIN;   // candidates before the refinement runs (A/B: RT_SUB_MIN)
#ifndef RT_MAXCL
#define RT_MAXCL 6
#endif
constexpr int kMaxClusters = RT_MAXCL;
__device__ __forceinline__ uint64_t sub_bundle_mask(const float4 c0, const float4 c1, const DRay& r0, real tmin,
                                                    bool need, uint64_t nm, float Lx, float Ly, float Lz) {
    const int lane = __lane_id();
    const float ox = (float)r0.o.x, oy = (float)r0.o.y, oz = (float)r0.o.z;
    const bool bad = need && !__builtin_isfinite(ox + oy + oz);
    if (__any(bad)) return ~0ull;
    const float e = need ? (float)tmin : 0.0f;
    const float emax = __uint_as_float(wave_max_u32(__float_as_uint(e))) * 1.000001f;
    // greedy clusters: each lane ends with its cluster's centre and radius^2
    float cx = ox, cy = oy, cz = oz, cr2 = 0.0f;
    uint64_t rem = nm, leaders = 0;
    for (int k = 0; rem && k < kMaxClusters; ++k) {
        const int f = __builtin_ctzll(rem);
        leaders |= 1ull << f;
        const float qx = rdlane_f(ox, f), qy = rdlane_f(oy, f), qz = rdlane_f(oz, f);
        const float lx = qx - Lx, ly = qy - Ly, lz = qz - Lz;
        const float tau2 = (k + 1 == kMaxClusters) ? __builtin_inff()
                                                   : 2.4414e-4f * __builtin_fmaf(lx, lx, __builtin_fmaf(ly, ly, lz * lz));
        const float dx = ox - qx, dy = oy - qy, dz = oz - qz;
        const float d2 = __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz));
        const bool in = ((rem >> lane) & 1ull) && d2 <= tau2;
        const uint64_t mb = __ballot(in);
        const float r2 = __uint_as_float(wave_max_u32(__float_as_uint(in ? d2 : 0.0f)));
        if (in) {
            cx = qx, cy = qy, cz = qz;
            cr2 = r2;
        }
        rem &= ~mb;
    }
    // the lane's cluster's cone
    const float ux = cx - Lx, uy = cy - Ly, uz = cz - Lz;
    const float dq = sqrt_cull(__builtin_fmaf(ux, ux, __builtin_fmaf(uy, uy, uz * uz)));
    const float mq = __builtin_fabsf(cx) + __builtin_fabsf(cy) + __builtin_fabsf(cz) + __builtin_fabsf(Lx) +
                     __builtin_fabsf(Ly) + __builtin_fabsf(Lz);
    const float rho = __builtin_fmaf(sqrt_cull(cr2) + emax, 1.00001f, 1e-6f * (mq + 1.0f));
    const float inv = __builtin_amdgcn_rcpf(dq);
    const float sb = __builtin_fminf(1.0f, rho * inv * 1.00001f + 1e-6f);
    const float cb = sqrt_cull(__builtin_fmaxf(0.0f, __builtin_fmaf(-sb, sb, 1.0f))) * 0.99999f - 1e-6f;
    const bool ok = (dq > rho * 1.0001f) && (cb > 0.0f) && __builtin_isfinite(rho);
    const float gv[14] = {ux * inv, uy * inv, uz * inv, cb, sb, dq * 0.99999f, (dq + rho) * 1.00001f,
                          rho * __builtin_amdgcn_rcpf(cb) * 1.00001f + 1e-6f * mq, rho, 2.0f * emax, cx, cy, cz, mq};
    bool pass = false;
    while (leaders) {
        const int lg = __builtin_ctzll(leaders);
        leaders &= leaders - 1;
        if (!__builtin_amdgcn_readlane(ok ? 1 : 0, lg)) return ~0ull;   // keep every object
        LightCone K;
        K.ax = rdlane_f(gv[0], lg), K.ay = rdlane_f(gv[1], lg), K.az = rdlane_f(gv[2], lg);
        K.cb = rdlane_f(gv[3], lg), K.sb = rdlane_f(gv[4], lg), K.dq = rdlane_f(gv[5], lg);
        K.xe = rdlane_f(gv[6], lg), K.rend = rdlane_f(gv[7], lg), K.rho = rdlane_f(gv[8], lg);
        K.emax = rdlane_f(gv[9], lg), K.qx = rdlane_f(gv[10], lg), K.qy = rdlane_f(gv[11], lg);
        K.qz = rdlane_f(gv[12], lg), K.mq = rdlane_f(gv[13], lg);
        pass = pass || lrec_touch(c0, c1, K);
    }
    return __ballot(pass);
}

// Scene::occluded (scene.cpp:33-42) for the querying lanes of a fully active
// wave, light li of S.lights.  Returns false for lanes with need = false.
//
// r0 is the shadow ray BEFORE the Ray constructor's re-normalisation of its
// direction (core.h:278; r0.d = wi, unit for every lane whose light distance
// was not clamped, regular = d2 > 0.01): the culls work on it directly, and
// the exact FP64 ray (make_ray, one sqrt and three divisions per lane) is
// formed only when some candidate object survives them and is evaluated -
// most shadow queries of a wave end before that.
//
// BV (wave BVH kernels): S.objs is the Morton-ordered list in chunks of 64
// with a cull record per chunk (CompiledScene::wobjs / wchunk); one
// transposed test per 64 chunks skips every chunk no querying segment can
// reach, then each surviving chunk runs the object test below.  Occlusion is
// an OR over objects, so the order is free.
template <bool EAGER, bool DEEP, bool UO, bool BV = false, class CT>
__device__ bool scene_occluded_wave(const DevScene& S, const DRay& r0, real tmin, real tmax, bool need, bool wave_ok,
                                    CT& cnt, int li, const ShadowHull& H, bool regular) {
#if defined(RT_ABL) && RT_ABL == 1   // diagnostic ablation builds only (wrong images): no shadow queries
    return false;
#endif
    cnt.pb(PH_WAVE_SETUP);
    DRay r = r0;           // the exact ray, formed on the first object evaluation (wave-uniform)
    bool r_exact = false;
    const uint64_t nm = __ballot(need);
    if (!nm) return false;
    cnt.ev(EV_SHQ);
    const int f = __builtin_ctzll(nm);
    const LightT* Lp = &S.lights[li];
    const float Lx = (float)Lp->pos[0], Ly = (float)Lp->pos[1], Lz = (float)Lp->pos[2];
    // the light's cone over the shade call's hull (uniform; shadow_hull)
    LightCone K;
    bool cone = H.ok && wave_ok && exec_full() && !__any(need && !regular);
    {
        const float dx = H.qx - Lx, dy = H.qy - Ly, dz = H.qz - Lz;
        const float dq = sqrt_cull(__builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz)));
        const float mq = __builtin_fabsf(H.qx) + __builtin_fabsf(H.qy) + __builtin_fabsf(H.qz) + __builtin_fabsf(Lx) +
                         __builtin_fabsf(Ly) + __builtin_fabsf(Lz);
        const float rho = __builtin_fmaf(H.rho, 1.00001f, 1e-6f * (mq + 1.0f));
        const float inv = __builtin_amdgcn_rcpf(dq);
        const float sb = __builtin_fminf(1.0f, rho * inv * 1.00001f + 1e-6f);
        const float cb = sqrt_cull(__builtin_fmaxf(0.0f, __builtin_fmaf(-sb, sb, 1.0f))) * 0.99999f - 1e-6f;
        cone = cone && (dq > rho * 1.0001f) && (cb > 0.0f);
        K.ax = uni<UO>(dx * inv), K.ay = uni<UO>(dy * inv), K.az = uni<UO>(dz * inv);
        K.cb = uni<UO>(cb), K.sb = uni<UO>(sb);
        K.dq = uni<UO>(dq * 0.99999f);
        K.xe = uni<UO>((dq + rho) * 1.00001f);
        K.rend = uni<UO>(rho * __builtin_amdgcn_rcpf(cb) * 1.00001f + 1e-6f * mq);
        K.rho = uni<UO>(rho), K.emax = H.emax;
        K.qx = H.qx, K.qy = H.qy, K.qz = H.qz;
        K.mq = uni<UO>(mq);
    }
    const float leps = (float)tmin * 1.0000002f;
    const int lane = __lane_id();
    const float4* lrec = S.lrec + 2 * (size_t)li * S.n_objs;
    const float4* lgb = S.lgb + 2 * (size_t)li * S.n_gb;
    // line bundle for the CSG leaf masks, built on first use (cone only)
    bool lb_ready = false;
    Cone LB{f2(0.0f, 0.0f), f2(0.0f, 0.0f), 0.0f, 0.0f, -1.0f, 1.0f, 0.0f, 0.0f};
    bool hit = false;
    const int nch = BV ? S.n_chunks : (S.n_objs + 63) >> 6;
    uint64_t cm = 0;   // (BV) chunks ch & ~63 .. +63 some querying segment can reach
    for (int ch = 0; ch < nch; ++ch) {
        if (ch > 0) cnt.pb(PH_WAVE_SETUP);   // (phase builds: a later chunk's test timed from here)
        if constexpr (BV) {
            if ((ch & 63) == 0) {
                const int c = ch + lane;
                const int cr = c < nch ? c : nch - 1;
                const float4 k0 = S.wchunk[2 * cr], k1 = S.wchunk[2 * cr + 1];
                const int ktype = __float_as_int(k1.x);
                const bool pass = (c < nch) & ((ktype != 2) | ball_cone(k0, K, Lx, Ly, Lz));
                cm = (cone && exec_full()) ? __ballot(pass) : ~0ull;
                if (cone && __builtin_popcountll(cm) > kSubBundleMin && exec_full()) {
                    // the chunk balls against the per-pixel hulls (light-relative on the fly)
                    const float wx = k0.x - Lx, wy = k0.y - Ly, wz = k0.z - Lz;
                    const float4 q0 = make_float4(wx, wy, wz, __builtin_fmaf(wx, wx, __builtin_fmaf(wy, wy, wz * wz)));
                    const float4 q1 = make_float4(k1.x, k0.w, __builtin_fabsf(wx) + __builtin_fabsf(wy) + __builtin_fabsf(wz) + k0.w,
                                                  0.0f);
                    cm &= sub_bundle_mask(q0, q1, r0, tmin, need, nm, Lx, Ly, Lz);
                }
            }
            if (!((cm >> (ch & 63)) & 1ull)) {
                if constexpr (kCounting<CT>)
                    if (need) cnt_add(cnt, RT_OPC_CULLED, chunk_objects(S, ch << 6));
                continue;
            }
        }
        const int base = ch << 6;
        const int nc = S.n_objs - base;
        const int j = base + lane;
        // the object's light-relative record (CompiledScene::lrec): one
        // 32-byte load on every lane (lanes past the last object re-read it
        // and are masked)
        const int jr = j < S.n_objs ? j : S.n_objs - 1;
        const float4 c0 = lrec[2 * jr], c1 = lrec[2 * jr + 1];
        const bool pass = (j < S.n_objs) & (cone ? lrec_touch(c0, c1, K) : __float_as_int(c1.x) != 0);
        // (lane j tests object j only with the whole wave active; otherwise
        // every object of the chunk is a candidate)
        uint64_t m = (cone && exec_full()) ? __ballot(pass) : (nc >= 64 ? ~0ull : ((1ull << nc) - 1));
        // Sub-bundles: where the wave's hull lets many objects of a chunk
        // through (a tile straddling depth edges of an incoherent scene), each
        // object is tested again against the eight per-pixel hulls (a pixel's
        // 8 samples hit close together) and kept if any of them reaches it.
        if (cone && __builtin_popcountll(m) > kSubBundleMin && exec_full())
            m &= sub_bundle_mask(c0, c1, r0, tmin, need, nm, Lx, Ly, Lz);
        cnt.pe(PH_WAVE_SETUP);
#if defined(RT_ABL) && RT_ABL == 2   // diagnostic: setup + transposed test only
        if (m != 12345) return false;
#endif
        if constexpr (kCounting<CT>) {
            if (need) {
                int skipped = 0;
                for (int o = base; o < S.n_objs && o < base + 64; ++o) {
                    const int k = S.objs[o].kind;
                    if (k != rtamd::OBJ_GROUP && k != rtamd::OBJ_NEVER && !((m >> (o - base)) & 1)) ++skipped;
                }
                cnt_add(cnt, RT_OPC_CULLED, skipped);
            }
        }
        while (m) {
            const int o = base + __builtin_ctzll(m);
            m &= m - 1;
            const DevObj ob = S.objs[o];
            if (ob.kind == rtamd::OBJ_GROUP || ob.kind == rtamd::OBJ_NEVER) continue;
            cnt.ev(EV_SH_CAND);
            cnt.pb(PH_OBJ_PREF);
            // CSG objects: no lane's segment reaches a leaf ball (DevObj::pb0);
            // otherwise the leaves whose balls no querying lane's line meets
            uint64_t lmask = ~0ull;
            bool use_mask = false;
            if (kCsg<CT> && cone && ob.npb > 0 && exec_full()) {
                const int k = ob.pb0 + (lane < ob.npb ? lane : 0);
                const float4 g0 = lgb[2 * k], g1 = lgb[2 * k + 1];
                const bool in = lane < ob.npb;
                const uint64_t cbm = __ballot(in && lrec_ball_cone(g0, g1.y, g1.z, K));
                bool seg = cbm != 0;
#ifndef RT_NO_LANE_LEAF_TEST
                // each lane's own segment against the leaf balls the cone
                // reaches (see scene_occluded_capsule): no touch, no hit
                if (seg) {
                    const FRay sfr = to_fray(r0);
                    const float st0 = (float)tmin, st1 = (float)tmax;
                    seg = false;
                    for (uint64_t mm = cbm; mm && !seg; mm &= mm - 1) {
                        const float* gk = S.gb + 4 * (ob.pb0 + __builtin_ctzll(mm));
                        seg = __any(need && !hit && ball_touch(gk, sfr, st0, st1));
                    }
                }
#endif
                if (!seg) {
                    if (need) cnt.inc(RT_OPC_CULLED);
                    cnt.pe(PH_OBJ_PREF);
                    continue;
                }
                if (!lb_ready) {
                    // line bundle of the querying lanes (lane f's line as the axis)
                    lb_ready = true;
                    const FRay fr = to_fray(r0);
                    const float lox = rdlane_f(fr.ox, f), loy = rdlane_f(fr.oy, f), loz = rdlane_f(fr.oz, f);
                    const float lax = rdlane_f(fr.dx, f), lay = rdlane_f(fr.dy, f), laz = rdlane_f(fr.dz, f);
                    const float dxo = fr.ox - lox, dyo = fr.oy - loy, dzo = fr.oz - loz;
                    const float do2 = need ? dxo * dxo + dyo * dyo + dzo * dzo : 0.0f;
                    const float dc = need ? __builtin_fmaxf(0.0f, 1.0f - __builtin_fmaf(fr.dx, lax, __builtin_fmaf(fr.dy, lay, fr.dz * laz)))
                                          : 0.0f;
                    const float lrho = uni<UO>(sqrt_cull(__uint_as_float(wave_max_u32(__float_as_uint(do2)))));
                    const float dcm = __uint_as_float(wave_max_u32(__float_as_uint(dc))) + 4e-6f;
                    const float lcth = uni<UO>(1.0f - dcm);
                    LB.oxy = f2(lox, loy), LB.axy = f2(lax, lay), LB.oz = loz, LB.az = laz;
                    LB.cth = lcth;
                    LB.sth = uni<UO>(sqrt_cull(__builtin_fmaxf(0.0f, 1.0f - lcth * lcth)) + 1e-6f);
                    LB.rho = lrho;
                    LB.m5 = uni<UO>(1e-5f * (__builtin_fabsf(lox) + __builtin_fabsf(loy) + __builtin_fabsf(loz) + lrho + 1.0f));
                }
#ifdef RT_NO_LEAF_MASK
                use_mask = false;
#else
                use_mask = LB.cth > 0.0f;
#endif
                if (use_mask) {
                    const bool full = exec_full();
                    const uint64_t b = __ballot(in && line_touch(S.gb + 4 * k, LB));
                    lmask = full ? b : ~0ull;
                }
            }
            if (cone && ob.kind == rtamd::OBJ_HALF) {
                // a bare half-space passed the hull test (hit points on or
                // near its plane: the hull cannot tell their sides, the
                // segments can): lane i's segment runs from A_i = o_i + tmin
                // d_i to within 2 eps of L, so it crosses the plane only if
                // A_i's signed distance and the light's (record) allow it
                const float4 o0 = lrec[2 * o], o1 = lrec[2 * o + 1];   // (n, n.p), (type, n.L - n.p, mag)
                const float ax = (float)__builtin_fma(tmin, r0.d.x, r0.o.x), ay = (float)__builtin_fma(tmin, r0.d.y, r0.o.y),
                            az = (float)__builtin_fma(tmin, r0.d.z, r0.o.z);
                const float sa = dot_pk(f2(o0.x, o0.y), o0.z, f2(ax, ay), az) - o0.w;
                const float mp = 1e-5f * (o1.z + __builtin_fabsf(ax) + __builtin_fabsf(ay) + __builtin_fabsf(az));
                const float e2 = 2.0f * leps;   // (the far end: within 2 eps of L)
                const float sl = o1.y;
                const bool cross = !((sa > mp) & (sl - e2 > mp)) & !((sa < -mp) & (sl + e2 < -mp));   // NaN passes
                if (!__any(need && !hit && cross)) {
                    if (need) cnt.inc(RT_OPC_CULLED);
                    cnt.pe(PH_OBJ_PREF);
                    continue;
                }
            }
            if (S.cull && ob.has_bound) {
                // per-lane segment test (f32, cheaper than an FP64 miss) on the
                // lane's actual segment: its eps offset from the hit point is
                // what clears the object a lane itself lies on
                const FRay fr = to_fray(r0);
                if (!__any(need && !hit && ball_touch(ob.fb, fr, (float)tmin, (float)tmax))) {
                    if (need) cnt.inc(RT_OPC_CULLED);
                    cnt.pe(PH_OBJ_PREF);
                    continue;
                }
            }
            cnt.pe(PH_OBJ_PREF);
#if defined(RT_ABL) && RT_ABL == 3   // diagnostic: everything but the shadow object evaluations
            if (m != 12345) continue;
#endif
            const bool csg_obj = ob.kind == rtamd::OBJ_CHAIN && ob.core != 0;
            if (csg_obj) cnt.pb(PH_SHADOW_CSG);
            cnt.pb(PH_OBJ_HIT);
            cnt.ev(EV_SH_HIT);
            if (csg_obj) cnt.ev(EV_SH_CSG);
            if (!r_exact) {   // Ray::Ray (core.h:278) of the shadow ray (shading.cpp:98), in place
                r.d = normalized(r.d);
                r_exact = true;
            }
            {
                // every lane evaluates (the wave runs the object anyway) and
                // only querying lanes without a hit take the result: no
                // divergent region between this loop's wave-wide tests.  The
                // op-counting builds take the same path and count only the
                // reference's calls (querying lanes without a hit yet).
                real t = RV(0.0), ts = RV(0.0);
                V3 p;
                int code = 0;
                const bool take = need && !hit;
                cnt.gate(take);
                const bool h = object_hit<EAGER, DEEP>(S, ob, r, tmin, tmax, t, p, ts, code, cnt, lmask, use_mask);
                cnt.gate(true);
                hit = hit || (take && h);
            }
            cnt.pe(PH_OBJ_HIT);
            if (csg_obj) cnt.pe(PH_SHADOW_CSG);
            if (__all(hit || !need)) return hit;
        }
    }
    return hit;
}


// Scene::intersect for a fully active wave: the closest hit of every lane.
// The lanes' rays form a bundle - origins within rho of lane 0's, directions
// within the cone of half-angle theta around lane 0's - and every ray point
// o_i + t d_i (t >= 0) lies within rho of the cone from lane 0's origin.  One
// transposed test of object j's ball (grown by rho) against that cone, on
// lane j, picks the objects any lane can reach; the per-object loop then runs
// over those, in scene order, exactly as scene_intersect (ties and the
// shrinking closest-so-far included).  Conservative in f32 like
// capsule_touch: results are unchanged.
__device__ __forceinline__ bool cone_touch(const float4 g, float gmag, const Cone& K) {
    return cone_touch_t<false>(g, gmag, K);
}
__device__ __forceinline__ bool cone_touch(const float* g, const Cone& K) {
    const float4 b = *reinterpret_cast<const float4*>(g);
    return cone_touch_t<false>(b, ball_mag(b), K);
}

//
// valid = false: a lane that only keeps the wave fully active (trace_wave's
// finished paths); its ray is left out of the bundle and of every test, its
// result is garbage and its ops are not counted.
//
// BV (wave BVH kernels): the chunk test of scene_occluded_wave with the
// cone.  Objects then come in Morton order, not the reference's, so every
// object is evaluated with the range up to and INCLUDING the closest hit so
// far (each object's hit t does not depend on tmax, only its acceptance),
// and a hit at exactly the closest t is resolved as the reference's in-order
// loop would: of two objects hitting at the same t, the later (in the
// reference's order) wins if it accepts t == tmax (spheres, half-spaces,
// pokeballs: rtamd::accepts_tie), else the earlier one.
template <bool EAGER, bool DEEP, bool BV = false, bool LEAD = false, class CT>
__device__ bool scene_intersect_wave(const DevScene& S, const DRay& r, real tmin, real tmax, real& t_best,
                                     DHit& best, bool wave_ok, CT& cnt, bool valid = true) {
    cnt.pb(PH_WAVE_SETUP);
    const uint64_t vm = __ballot(valid);
    if (!vm) {
        cnt.pe(PH_WAVE_SETUP);
        return false;
    }
    const int f = __builtin_ctzll(vm);   // the bundle's axis lane
    const FRay fr = to_fray(r);
    const bool fin = __builtin_isfinite(fr.ox + fr.oy + fr.oz + fr.dx + fr.dy + fr.dz);
    // no cone for a partially active wave or non-finite rays: every object is
    // a candidate (the per-lane ball test still runs)
    const bool cone = S.cull && wave_ok && exec_full() && !__any(valid && !fin) && tmin >= RV(0.0);
    const float ox = rdlane_f(fr.ox, f), oy = rdlane_f(fr.oy, f), oz = rdlane_f(fr.oz, f);
    const float ax = rdlane_f(fr.dx, f), ay = rdlane_f(fr.dy, f), az = rdlane_f(fr.dz, f);
    const float do2 = valid ? (fr.ox - ox) * (fr.ox - ox) + (fr.oy - oy) * (fr.oy - oy) + (fr.oz - oz) * (fr.oz - oz)
                            : 0.0f;
    // 1 - cos(angle to the axis), >= 0 up to rounding
    const float dc = valid ? __builtin_fmaxf(0.0f, 1.0f - __builtin_fmaf(fr.dx, ax, __builtin_fmaf(fr.dy, ay, fr.dz * az)))
                           : 0.0f;
    const float rho = cone ? sqrt_cull(__uint_as_float(wave_max_u32(__float_as_uint(do2)))) : 0.0f;
    const float dcm = cone ? __uint_as_float(wave_max_u32(__float_as_uint(dc))) + 4e-6f : 2.0f;   // rounding of unit dots
    const float cth = 1.0f - dcm;
    const bool wide = !(cth > 0.0f);   // a bundle wider than 90 degrees (or no cone): no culling
    const float sth = sqrt_cull(__builtin_fmaxf(0.0f, 1.0f - cth * cth)) + 1e-6f;
    const float mag = __builtin_fabsf(ox) + __builtin_fabsf(oy) + __builtin_fabsf(oz) + rho + 1.0f;
    const Cone K{f2(ox, oy), f2(ax, ay), oz, az, cth, sth, rho, 1e-5f * mag};
    const int lane = __lane_id();
    real closest = tmax;
    int win = -1;
    int win_orig = 0;       // (BV) the winner's index in the reference's order
    bool win_tie = false;   // (BV) whether the winner accepts t == tmax
    V3 wp = v3(RV(0.0), RV(0.0), RV(0.0));
    real wts = RV(0.0);
    int wcode = 0;
    const float ftmin = (float)tmin;
    // the lead objects (CompiledScene::n_lead: unbounded, ahead of every
    // bounded one) first, in order, as pseudo-chunk -1; then the transposed
    // tests over the objects behind them (the reference's order throughout)
    const int lead = (BV || !LEAD) ? 0 : S.n_lead;
    const int nch = BV ? S.n_chunks : (S.n_objs - lead + 63) >> 6;
    uint64_t cm = 0;   // (BV) chunks ch & ~63 .. +63 the bundle can reach
    for (int ch = lead > 0 ? -1 : 0; ch < nch; ++ch) {
        int base;
        uint64_t m;
        if (ch < 0) {
            base = 0;
            m = 0;
            for (int o = 0; o < lead; ++o)
                if (__float_as_int(S.ctab[2 * o + 1].x) != 0) m |= 1ull << o;
            cnt.pe(PH_WAVE_SETUP);
        } else {
        if (ch > 0 || lead > 0) cnt.pb(PH_WAVE_SETUP);   // (phase builds: a later chunk's test timed from here)
        if constexpr (BV) {
            if ((ch & 63) == 0) {
                const int c = ch + lane;
                const int cr = c < nch ? c : nch - 1;
                const float4 k0 = S.wchunk[2 * cr], k1 = S.wchunk[2 * cr + 1];
                const int ktype = __float_as_int(k1.x);
                const bool pass = (c < nch) & ((ktype != 2) | wide | cone_touch(k0, k1.y, K));
                cm = (cone && exec_full()) ? __ballot(pass) : ~0ull;
            }
            if (!((cm >> (ch & 63)) & 1ull)) {
                if constexpr (kCounting<CT>)
                    if (valid) cnt_add(cnt, RT_OPC_CULLED, chunk_objects(S, ch << 6));
                continue;
            }
        }
        base = lead + (ch << 6);
        const int j = base + lane;
        const int jr = j < S.n_objs ? j : S.n_objs - 1;   // (see scene_occluded_wave)
        const float4 c0 = S.ctab[2 * jr], c1 = S.ctab[2 * jr + 1];
        const int type = __float_as_int(c1.x);
        const bool pass = (j < S.n_objs) & (type != 0) &
                          ((type != 2) | wide | cone_touch(c0, c1.y, K));
        const int nc = S.n_objs - base;
        m = (cone && exec_full()) ? __ballot(pass) : (nc >= 64 ? ~0ull : ((1ull << nc) - 1));
        cnt.pe(PH_WAVE_SETUP);
        if constexpr (kCounting<CT>) {
            int skipped = 0;
            for (int o = base; o < S.n_objs && o < base + 64; ++o) {
                const int k = S.objs[o].kind;
                if (k != rtamd::OBJ_GROUP && k != rtamd::OBJ_NEVER && !((m >> (o - base)) & 1)) ++skipped;
            }
            if (valid) cnt_add(cnt, RT_OPC_CULLED, skipped);
        }
        }
        while (m) {
            const int o = base + __builtin_ctzll(m);
            m &= m - 1;
            const DevObj ob = S.objs[o];
            if (ob.kind == rtamd::OBJ_GROUP || ob.kind == rtamd::OBJ_NEVER) continue;
            cnt.ev(EV_PR_CAND);
            cnt.pb(PH_OBJ_PREF);
            // CSG objects: the bundle reaches no leaf ball (DevObj::pb0);
            // otherwise the leaves whose balls no lane's line meets
            uint64_t lmask = ~0ull;
#ifdef RT_NO_LEAF_MASK
            const bool use_mask = false;
            if (kCsg<CT> && !wide && ob.npb > 0 && exec_full() && !__any(lane < ob.npb && cone_touch(S.gb + 4 * (ob.pb0 + (lane < ob.npb ? lane : 0)), K))) {
                if (valid) cnt.inc(RT_OPC_CULLED);
                cnt.pe(PH_OBJ_PREF);
                continue;
            }
#else
            const bool use_mask = kCsg<CT> && !wide && ob.npb > 0 && exec_full();
#endif
            if (use_mask) {
                const float* g = S.gb + 4 * (ob.pb0 + (lane < ob.npb ? lane : 0));
                const bool in = lane < ob.npb;
                if (!__any(in && cone_touch(g, K))) {
                    if (valid) cnt.inc(RT_OPC_CULLED);
                    cnt.pe(PH_OBJ_PREF);
                    continue;
                }
                const bool full = exec_full();
                const uint64_t b = __ballot(in && line_touch(g, K));
                lmask = full ? b : ~0ull;
            }
            if (S.cull && ob.has_bound && !__any(valid && ball_touch(ob.fb, fr, ftmin, (float)closest))) {
                if (valid) cnt.inc(RT_OPC_CULLED);
                cnt.pe(PH_OBJ_PREF);
                continue;
            }
            cnt.pe(PH_OBJ_PREF);
            real t = RV(0.0), ts = RV(0.0);
            V3 p;
            int code = 0;
            const bool csg_obj = ob.kind == rtamd::OBJ_CHAIN && ob.core != 0;
            if (csg_obj) cnt.pb(PH_PRIMARY_CSG);
            cnt.pb(PH_OBJ_HIT);
            cnt.ev(EV_PR_HIT);
            cnt.gate(valid);
            if constexpr (BV) {
                const bool ok = object_hit<EAGER, DEEP>(S, ob, r, tmin, next_up(closest), t, p, ts, code, cnt, lmask,
                                                        use_mask);
                const int oo = S.worig[o];
                const bool tie = rtamd::accepts_tie(ob);
                const bool take = ok && ((t < closest) ||
                                         (t == closest && (win < 0 ? tie : (oo > win_orig ? tie : !win_tie))));
                if (take) {
                    closest = t;
                    win = o;
                    win_orig = oo;
                    win_tie = tie;
                    wp = p;
                    wts = ts;
                    wcode = code;
                }
            } else if (object_hit<EAGER, DEEP>(S, ob, r, tmin, closest, t, p, ts, code, cnt, lmask, use_mask)) {
                closest = t;
                win = o;
                wp = p;
                wts = ts;
                wcode = code;
            }
            cnt.gate(true);
            cnt.pe(PH_OBJ_HIT);
            if (csg_obj) cnt.pe(PH_PRIMARY_CSG);
        }
    }
    if (win < 0) return false;
    cnt.gate(valid);
    resolve_hit<EAGER>(S, win, r, tmin, wp, wts, wcode, best, cnt);
    cnt.gate(true);
    t_best = closest;
    return true;
}

// ----------------------------------------------------------------- shading
// std::pow(x, shininess) of the specular term (shading.cpp:120).  The
// reference's glibc pow is correctly rounded in practice; the device
// library's pow is not always, and costs ~10 % of a frame.  Every shininess
// in the reference's scenes is a small integer, so for integer exponents
// 0..1023 x^k is evaluated by left-to-right binary powering in double-double
// arithmetic (exact products by fma, ~2^-100 relative error), and rounded
// once: the correctly rounded x^k.  Other exponents use the library pow.
// The library pow for non-integer exponents (no reference scene has one) is
// kept out of line: inlined, its temporaries set the trace kernel's register
// peak and made the compiler spill ~130 B/lane on the common integer path.
__device__ __attribute__((noinline)) double pow_general(double x, double y) { return pow(x, y); }

__device__ __forceinline__ double pow_spec(double x, double y) {
    const int k = (int)y;
    if (!(y >= 0.0 && y < 1024.0 && (double)k == y)) return pow_general(x, y);
    if (k == 0) return 1.0;   // pow(x, 0) = 1 for every x
    // (h, l): an unnormalised double-double (h the rounded product, l the
    // exact product error by fma plus the cross term), 4 / 3 operations per
    // squaring / multiplication instead of 7 with renormalisation.  Equal bit
    // for bit to the renormalised evaluation except below 2^-1000, where the
    // specular term is 0 to far beyond any tolerance (50 M random (x, k),
    // tools/probe/pow_dd_check.c).
    const int top = 31 - __builtin_clz(k);
    double h = x, l = 0.0;
    for (int i = top - 1; i >= 0; --i) {
        double p = h * h;   // (h, l)^2
        l = __builtin_fma(h + h, l, __builtin_fma(h, h, -p));
        h = p;
        if ((k >> i) & 1) {   // (h, l) * x
            p = h * x;
            l = __builtin_fma(l, x, __builtin_fma(h, x, -p));
            h = p;
        }
    }
    return h + l;
}
__device__ __forceinline__ float pow_spec(float x, float y) { return pow(x, y); }

// Per-lane LDS pool: shade() keeps pass 1's light geometry (wi, dist) of the
// first kLightCache lights of each light chunk there for pass 2, instead of
// recomputing sqrt + three divisions per lit light; flush_counters() reuses
// each wave's own region at the end.  Every wave owns kPoolWave doubles,
// laid out [light][field][lane] (consecutive lanes read consecutive 8-byte
// words: no bank conflicts); the pool is the workgroup's dynamic LDS, sized
// at launch by pool_bytes(threads) (rt_kernels.hpp launches): kLightCache x 4
// x 64 doubles = 10 KiB per wave, 40 KiB per 256-thread workgroup, so four
// workgroups (16 waves) still fit a CU's 160 KiB.
#ifndef RT_LIGHT_CACHE
#define RT_LIGHT_CACHE 5
#endif
constexpr int kLightCache = RT_LIGHT_CACHE;
constexpr int kPoolWave = (kLightCache > 0 ? kLightCache : 1) * 4 * 64;
constexpr size_t pool_bytes(int threads) { return (size_t)(threads / 64) * kPoolWave * sizeof(double); }
__device__ __forceinline__ double* lds_pool() {
    extern __shared__ double rt_lds_pool[];
    return rt_lds_pool;
}
// wave w's region
__device__ __forceinline__ double* wave_pool(int w) { return lds_pool() + (size_t)w * kPoolWave; }

__device__ __forceinline__ V3 combine(V3 a, V3 b) {   // shading.cpp:6-12
    return v3(RV(1.0) - (RV(1.0) - a.x) * (RV(1.0) - b.x), RV(1.0) - (RV(1.0) - a.y) * (RV(1.0) - b.y), RV(1.0) - (RV(1.0) - a.z) * (RV(1.0) - b.z));
}

// shade_lambert_phong (shading.cpp:31-138), point lights only (the loader
// never populates directional lights).
// DL: the scene may have directional lights (the lean kernels, chosen only
// for scenes without, do not carry their code or registers).
#ifndef RT_STD_UO
#define RT_STD_UO false
#endif
// LEAD: the wave queries handle CompiledScene::n_lead (the paper and
// recursion kernels; in the lean standard kernel the extra path cost
// registers: config 4 kernel 7.2 -> 7.6 ms, profiles/r06_ab/ab_lead.txt)
template <bool EAGER, bool DEEP, bool DL, int WV, bool UO = RT_STD_UO, bool LEAD = false, class CT>
__device__ V3 shade(const DevScene& S, real ht, const DHit& hit, V3 wo, uint32_t& n_occl, CT& cnt,
                    bool valid = true) {
    // valid = false: a lane of the wave that has nothing to shade (a primary
    // miss) but keeps the wave fully active for scene_occluded_wave; its
    // result is discarded by the caller.
    const bool has_mat = hit.mat >= 0;
    valid = valid && has_mat;
    if (valid) cnt.inc(RT_OPC_SHADE_CALL);
    // WV (wave-level culling; the host picks it for scenes with >= 4 bounded
    // objects, culling on): the capsule test needs every lane active
    const bool wave_full = WV && __builtin_amdgcn_read_exec() == ~0ull;
    const V3 n = hit.n;
    const real eps = cmax(RV(1e-3), RV(1e-4) * ht);   // (no zeros)
    // the wave's hit points once per call: the light-centred shadow culls
    // of every light start from them (scene_occluded_wave)
    ShadowHull hull{0.0f, 0.0f, 0.0f, 0.0f, 0.0f, false};
    if constexpr (WV == 2) hull = shadow_hull<UO>(hit.p, eps, valid, wave_full);
    // Two passes over the lights so that only (p, n, eps) stay live across
    // the shadow queries (register pressure): pass 1 decides, per light, the
    // reference's early-outs and the occlusion query; pass 2 recomputes the
    // same light geometry (identical operations, identical bits) and
    // accumulates in the reference's order.  Lights beyond 32 are handled in
    // further rounds of the same two passes.
    V3 E = v3(RV(0.0), RV(0.0), RV(0.0));
    {
        const MatT* m = &S.mats[valid ? hit.mat : 0];
        E = v3(m->ambient[0], m->ambient[1], m->ambient[2]);   // (K_a I_a, premultiplied)
    }
    // directional lights first (shading.cpp:45-76): no falloff, shadow ray to infinity
    for (int li = 0; DL && li < S.n_dlights; ++li) {
        if (!valid) break;
        const DLightT* L = &S.dlights[li];
        cnt.inc(RT_OPC_LIGHT_EVAL);
        const V3 wi = normalized(v3(-L->dir[0], -L->dir[1], -L->dir[2]));
        const real ndotl = dmax(RV(0.0), dot3(n, wi));
        if (ndotl <= RV(0.0)) continue;
        const V3 so = v3(hit.p.x + n.x * eps, hit.p.y + n.y * eps, hit.p.z + n.z * eps);
        ++n_occl;
        if (scene_occluded<EAGER, DEEP>(S, make_ray(so, wi), eps, RT_INF, cnt)) continue;
        cnt.inc(RT_OPC_SHADE_LIGHT);
        const MatT* m = &S.mats[hit.mat];
        const real sd = m->kd * ndotl;   // scale(mul(albedo, radiance), kd * ndotl)
        const V3 Ed = v3(m->albedo[0] * L->radiance[0] * sd, m->albedo[1] * L->radiance[1] * sd,
                         m->albedo[2] * L->radiance[2] * sd);
        V3 Es = v3(RV(0.0), RV(0.0), RV(0.0));
        if (m->ks > RV(0.0)) {
            cnt.inc(RT_OPC_SHADE_SPEC);
            const V3 rr = normalized(v3(RV(2.0) * dot3(n, wi) * n.x - wi.x, RV(2.0) * dot3(n, wi) * n.y - wi.y,
                                        RV(2.0) * dot3(n, wi) * n.z - wi.z));
            const real rdotv = dmax(RV(0.0), dot3(rr, wo));
            const real spec = pow_spec(rdotv, m->shininess) * m->ks;
            Es = v3(L->radiance[0] * spec, L->radiance[1] * spec, L->radiance[2] * spec);
        }
        E = combine(E, combine(Ed, Es));
    }
    if (WV) cnt.pb(PH_SHADE2);   // (pass 2 is timed from the end of pass 1; this start is overwritten)
    double* const lc = wave_pool((int)(threadIdx.x >> 6)) + (threadIdx.x & 63);
    for (int l0 = 0; __any(valid) && l0 < S.n_lights; l0 += 32) {
        const int l1 = S.n_lights - l0 < 32 ? S.n_lights : l0 + 32;
        uint32_t lit = 0;
        if (WV) cnt.pb(PH_SHADE1);
        for (int li = l0; li < l1; ++li) {
            const LightT* L = &S.lights[li];
            if (valid) cnt.inc(RT_OPC_LIGHT_EVAL);
            V3 tl = v3(L->pos[0] - hit.p.x, L->pos[1] - hit.p.y, L->pos[2] - hit.p.z);
            real d2 = dot3(tl, tl);
            if (d2 <= RV(0.01)) d2 = RV(0.01);
            const real dist = sqrt_r(d2);
            const auto wq = div3(tl.x, tl.y, tl.z, dist);
            const V3 wi = v3(wq.x, wq.y, wq.z);
            if (li - l0 < kLightCache) {
                double* c = lc + (li - l0) * 4 * 64;
                c[0] = wi.x;
                c[64] = wi.y;
                c[2 * 64] = wi.z;
                c[3 * 64] = dist;
            }
            const real ndotl = cmax(RV(0.0), dot3(n, wi));   // (only compared with 0)
            const real max_t = dist - eps;
            // shading.cpp:86-103: back-facing lights and lights closer than
            // the shadow epsilon are skipped before the occlusion query
            const bool need = valid && ndotl > RV(0.0) && max_t > eps;
            if (!__any(need)) continue;
            cnt.ev(EV_LIGHT1);
            const V3 so = v3(hit.p.x + n.x * eps, hit.p.y + n.y * eps, hit.p.z + n.z * eps);
            bool occ = false;
            if constexpr (WV == 2) {
                cnt.pb(PH_SHADOW);
                // (the direction's re-normalisation happens inside, when needed)
                occ = scene_occluded_wave<EAGER, DEEP, UO, true>(S, DRay{so, wi}, eps, max_t, need, wave_full, cnt, li,
                                                                 hull, d2 > RV(0.01));
                cnt.pe(PH_SHADOW);
            } else if constexpr (WV) {
                cnt.pb(PH_SHADOW);
                occ = scene_occluded_capsule<EAGER, DEEP, UO, false, LEAD>(S, DRay{so, wi}, eps, max_t, need, wave_full, cnt);
                cnt.pe(PH_SHADOW);
            } else if (need) {
                // (the direction's re-normalisation happens inside, when needed)
                occ = scene_occluded<EAGER, DEEP>(S, DRay{so, wi}, eps, max_t, cnt, true);
            }
            if (need) {
                ++n_occl;
                if (!occ) lit |= 1u << (li - l0);
            }
        }
        if (WV) {
            cnt.pe(PH_SHADE1);
            cnt.pb(PH_SHADE2);
        }
#if defined(RT_ABL) && RT_ABL == 4   // diagnostic: no pass-2 accumulation
        if (lit != 12345u) continue;
#endif
        if (!lit) continue;
        const MatT* m = &S.mats[hit.mat];
        const real kd = m->kd, ks = m->ks, shin = m->shininess;
        const V3 alb = ld3(m->albedo);
        for (int li = l0; li < l1; ++li) {
            if (!((lit >> (li - l0)) & 1u)) continue;
            cnt.ev(EV_LIGHT2);
            const LightT* L = &S.lights[li];
            V3 wi;
            real dist;
            if (li - l0 < kLightCache) {   // pass 1's values (same lane)
                const double* c = lc + (li - l0) * 4 * 64;
                wi = v3((real)c[0], (real)c[64], (real)c[2 * 64]);
                dist = (real)c[3 * 64];
            } else {
                V3 tl = v3(L->pos[0] - hit.p.x, L->pos[1] - hit.p.y, L->pos[2] - hit.p.z);
                real d2 = dot3(tl, tl);
                if (d2 <= RV(0.01)) d2 = RV(0.01);
                dist = sqrt_r(d2);
                const auto wq = div3(tl.x, tl.y, tl.z, dist);
                wi = v3(wq.x, wq.y, wq.z);
            }
            const real ndotl = cmax(RV(0.0), dot3(n, wi));   // (> 0: a lit light)
            cnt.inc(RT_OPC_SHADE_LIGHT);
            const real ed = cmax(RV(0.5), dist);
            const real falloff = RV(1.0) / (ed * ed);
            const real f2 = falloff * RV(2.0);
            const V3 IL = v3(L->intensity[0] * f2, L->intensity[1] * f2, L->intensity[2] * f2);
            const real sd = kd * ndotl * RV(1.5);
            const V3 Ed = v3(alb.x * IL.x * sd, alb.y * IL.y * sd, alb.z * IL.z * sd);
            V3 Es = v3(RV(0.0), RV(0.0), RV(0.0));
            if (ks > RV(0.0)) {
                cnt.inc(RT_OPC_SHADE_SPEC);
                const V3 rr = normalized(v3(RV(2.0) * dot3(n, wi) * n.x - wi.x, RV(2.0) * dot3(n, wi) * n.y - wi.y,
                                            RV(2.0) * dot3(n, wi) * n.z - wi.z));
                const real rdotv = cmax(RV(0.0), dot3(rr, wo));
                const real spec = pow_spec(rdotv, shin) * ks;   // (a -0 here gives Es = -0: combine ignores the sign)
                Es = v3(IL.x * spec, IL.y * spec, IL.z * spec);
            }
            E = combine(E, combine(Ed, Es));
        }
    }
    if (WV) cnt.pe(PH_SHADE2);
    E.x = cmin(RV(1.5), E.x);   // (keeps a zero's sign)
    E.y = cmin(RV(1.5), E.y);
    E.z = cmin(RV(1.5), E.z);
    return has_mat ? E : v3(RV(1.0), RV(0.0), RV(1.0));   // magenta for a null material (shading.cpp:33)
}

// ---------------------------------------------------------------- tracing
struct Frame {
    V3 total;
    DRay refr;
    int mat;
    int stage;      // 0 = reflection child pending, 1 = refraction child pending
    int want_refr;
};

// Tracer::trace_recursive (tracer.cpp:22-73) as an explicit frame stack,
// wave-synchronous (WV kernels with reflection / refraction): every lane of
// the wave runs every step until the whole wave is done, and a lane whose
// path has finished rides along with valid = false.  The exec mask therefore
// stays full at the closest-hit and shadow queries of every bounce, so their
// wave-level culls apply to secondary rays too (a lane-divergent loop would
// leave only the lanes still bouncing active and every query would fall back
// to testing all objects).  Each lane's arithmetic is the one of trace()
// below, step for step.
//
// A step's children (the reflected and refracted rays, tracer.cpp:38-68) are
// formed and pushed BEFORE the step is shaded: they depend only on the hit,
// and after shade() the step then needs nothing but its direct colour and
// the stack (the next ray is read back from the frame).  So the ray, the hit
// point and the normal are dead across shade(), whose shadow queries set the
// kernel's register peak; kept live there they cost ~320 B/lane of spill slots
// and 32 % on a frame without bounces.
// trace_wave's frame: the colour so far and the material; the children's
// rays live in the ray slots (two per level), so a frame is 32 bytes.  The
// stack sits in scratch, and every resident wave's stack lines travel
// through the L2 (profiles/r05u_pmc_mem_cfg6.txt): frames are kept small and
// nothing is copied between slots.
struct WFrame {
    V3 total;
    int mat;
    int sf;   // bit 0: stage (0 = reflection child pending, 1 = refraction child pending); bit 1: refraction wanted
};

// The lead-object path (CompiledScene::n_lead) in trace_wave's closest-hit /
// shadow queries: on in the plain kernel, off in the general one.  Compiled
// into the general kernel its extra code cost the recursion row more than its
// culling saved (15.33 ms without it in either query, 15.91 with both;
// profiles/r06_ab/ab_lead_split.txt); the plain kernel has the registers for
// it (12.77 vs 13.00 ms, profiles/r06_ab/ab_plain_tune.txt).  The paper
// kernels keep both.
#ifndef RT_SEC_LEAD_I
#define RT_SEC_LEAD_I false
#endif
#ifndef RT_SEC_LEAD_S
#define RT_SEC_LEAD_S false
#endif
#ifndef RT_PLAIN_SEC_LEAD
#define RT_PLAIN_SEC_LEAD true
#endif
template <bool EAGER, bool DEEP, bool DL, int WV, class CT>
__device__ __forceinline__ V3 trace_wave(const DevScene& S, DRay r0, uint32_t& n_isect, uint32_t& n_occl, CT& cnt) {
    WFrame stk[kMaxDepth];
    // The ray each step traces lives in memory, not registers: slots 2k and
    // 2k + 1 hold frame k's reflected and refracted children.  A step after
    // the camera ray's loads its ray from slot rsel (lanes with nothing to
    // evaluate load nothing), and it is dead by the time the step is shaded
    // (a loop-carried register copy stayed live across shade() on every path).
    DRay nxt[2 * kMaxDepth];
    int rsel = 0;
    int sp = 0;
    int depth = 0;
    const int limit = S.rec_limit;
    // (a finished path's colour is parked in stk[0].total: every lane's path
    // finishes, so the slot is always written before the final read)
    bool alive = true;
    const bool wave_ok = __builtin_amdgcn_read_exec() == ~0ull;
    // One step of the wave, inlined twice: FIRST is the camera ray's step,
    // peeled off the loop, so a wave none of whose lanes descends never enters
    // the loop and the loop's live state does not shape that step's code (the
    // no-bounce frame 9.81 -> 9.18 ms, the recursion row 19.16 -> 18.43 ms;
    // profiles/r05_ab/ab_secw_peel.txt).
    auto step = [&](auto first_tag) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(first_tag)::value;
        // ---- evaluate node (r, depth) on the lanes still tracing
        const bool eval = alive && depth < limit;
        DRay r;
        if constexpr (FIRST) {
            r = r0;
        } else {
            r = DRay{v3(RV(0.0), RV(0.0), RV(0.0)), v3(RV(0.0), RV(0.0), -RV(1.0))};   // (riders: never traced)
            if (eval) r = nxt[rsel];
        }
        if (!FIRST) {
            cnt.ev(EV_BOUNCE);
            cnt.evn(EV_COMPACT_LEAF, (unsigned)__builtin_popcountll(__ballot(eval)));
        }
        real ht = RV(0.0);
        DHit h;
        h.p = h.n = v3(RV(0.0), RV(0.0), RV(0.0));
        h.mat = -1;
        h.ff = 1;
        if (eval) ++n_isect;
        cnt.pb(PH_PRIMARY);
        const bool hit = scene_intersect_wave<EAGER, DEEP, (WV == 2), kCsg<CT> ? RT_SEC_LEAD_I : RT_PLAIN_SEC_LEAD>(S, r, RV(1e-4), RT_INF, ht, h, wave_ok, cnt, eval);
        cnt.pe(PH_PRIMARY);
        const bool sh = eval && hit;
        // ---- the step's children, pushed before shading (tracer.cpp:38-68)
        bool descend = false;
        if (sh && h.mat >= 0) {
            const MatT* mat = &S.mats[h.mat];
            const bool can = depth < limit - 1;
            const bool want_refl = mat->kr > RV(0.0) && can;
            bool want_refr = false;
            DRay refr;
            if (mat->kt > RV(0.0) && can) {
                const real eta = h.ff ? (S.medium_index / mat->refractive_index)
                                      : (mat->refractive_index / S.medium_index);
                const V3 inc = normalized(r.d);
                const real cos_i = -dot3(inc, h.n);   // tracer.cpp:100-104
                const real st2 = eta * eta * dmax(RV(0.0), RV(1.0) - cos_i * cos_i);
                if (!(st2 >= RV(1.0))) {
                    want_refr = true;
                    const real cos_t = sqrt_r(RV(1.0) - st2);   // tracer.cpp:87-98
                    const real k = eta * cos_i - cos_t;
                    const V3 rd = normalized(v3(inc.x * eta + h.n.x * k, inc.y * eta + h.n.y * k,
                                                inc.z * eta + h.n.z * k));
                    const V3 ro = h.ff ? v3(h.p.x - h.n.x * RV(1e-6), h.p.y - h.n.y * RV(1e-6), h.p.z - h.n.z * RV(1e-6))
                                       : v3(h.p.x + h.n.x * RV(1e-6), h.p.y + h.n.y * RV(1e-6), h.p.z + h.n.z * RV(1e-6));
                    refr = make_ray(ro, rd);
                }
            }
            if (want_refl || want_refr) {
                WFrame& fr = stk[sp];
                fr.mat = h.mat;
                if (want_refr) nxt[2 * sp + 1] = refr;
                cnt.inc(RT_OPC_SECONDARY);
                if (want_refl) {
                    const V3 inc = normalized(r.d);
                    const real k = RV(2.0) * dot3(inc, h.n);   // reflect (tracer.cpp:76-78)
                    const V3 rd = normalized(v3(inc.x - h.n.x * k, inc.y - h.n.y * k, inc.z - h.n.z * k));
                    const V3 ro = h.ff ? v3(h.p.x + h.n.x * RV(1e-6), h.p.y + h.n.y * RV(1e-6), h.p.z + h.n.z * RV(1e-6))
                                       : v3(h.p.x - h.n.x * RV(1e-6), h.p.y - h.n.y * RV(1e-6), h.p.z - h.n.z * RV(1e-6));
                    fr.sf = want_refr ? 2 : 0;
                    nxt[2 * sp] = make_ray(ro, rd);
                } else {
                    fr.sf = 1;
                }
                ++sp;
                descend = true;
            }
        }
        const V3 wo = normalized(vneg(r.d));
        V3 direct = v3(RV(0.0), RV(0.0), RV(0.0));
        if (__any(sh)) direct = shade<EAGER, DEEP, DL, WV, RT_STD_UO, kCsg<CT> ? RT_SEC_LEAD_S : RT_PLAIN_SEC_LEAD>(S, ht, h, wo, n_occl, cnt, sh);
        // the step's value (a finished lane's colour is in memory, so nothing
        // but the stack state is carried across steps)
        V3 ret = v3(RV(0.0), RV(0.0), RV(0.0));
        if (eval && !hit) ret = background(S);
        if (sh) {
            if (descend) {
                stk[sp - 1].total = direct;
                rsel = 2 * (sp - 1) + (stk[sp - 1].sf & 1);
                depth = sp;
            } else {
                ret = direct;
            }
        }
        if (alive && !descend) {
            // ---- unwind
            bool resumed = false;
            while (sp > 0) {
                WFrame& fr = stk[sp - 1];
                const MatT* mat = &S.mats[fr.mat];
                const int sf = fr.sf;
                if ((sf & 1) == 0) {
                    fr.total = combine(fr.total, v3(ret.x * mat->kr, ret.y * mat->kr, ret.z * mat->kr));
                    if (sf & 2) {
                        cnt.inc(RT_OPC_SECONDARY);
                        fr.sf = sf | 1;
                        rsel = 2 * (sp - 1) + 1;
                        depth = sp;
                        resumed = true;
                        break;
                    }
                    ret = fr.total;
                    --sp;
                } else {
                    fr.total = combine(fr.total, v3(ret.x * mat->kt, ret.y * mat->kt, ret.z * mat->kt));
                    ret = fr.total;
                    --sp;
                }
            }
            if (!resumed) {
                alive = false;
                stk[0].total = ret;   // (sp == 0: the stack is free)
            }
        }
        return ret;
    };
    // (a wave none of whose lanes descends: every lane's colour is the first
    // step's value, returned from registers)
    const V3 first = step(std::true_type{});
    if (!__any(alive)) return first;
    while (__any(alive)) step(std::false_type{});
    return stk[0].total;
}

// Tracer::trace_recursive (tracer.cpp:22-73) as an explicit frame stack.
template <bool EAGER, bool DEEP, bool SECONDARY, bool DL, int WV, class CT>
__device__ __forceinline__ V3 trace(const DevScene& S, DRay r, uint32_t& n_isect, uint32_t& n_occl, CT& cnt) {
#ifndef RT_OLD_TRACE
    if constexpr (SECONDARY && WV) return trace_wave<EAGER, DEEP, DL, WV>(S, r, n_isect, n_occl, cnt);
#endif
    if constexpr (!SECONDARY) {
        // No material reflects or refracts (or recursion <= 1): trace_recursive
        // reduces to one closest hit + local shading (tracer.cpp:22-37, 72).
        if (S.rec_limit <= 0) return v3(RV(0.0), RV(0.0), RV(0.0));
        real ht = RV(0.0);
        DHit h;
        h.mat = -1;
        ++n_isect;
        if constexpr (WV) {
            // miss lanes stay in shade() (valid = false) so that the wave
            // stays fully active for the wave-level shadow queries
            cnt.pb(PH_PRIMARY);
            const bool hit = scene_intersect_wave<EAGER, DEEP, (WV == 2)>(S, r, RV(1e-4), RT_INF, ht, h,
                                                               __builtin_amdgcn_read_exec() == ~0ull, cnt);
            cnt.pe(PH_PRIMARY);
            if (!__any(hit)) return background(S);
#if defined(RT_ABL) && RT_ABL == 5   // diagnostic: primary hit only, no shading
            if (S.n_objs != 12345) return hit ? h.n : background(S);
#endif
            const V3 E = shade<EAGER, DEEP, DL, WV>(S, ht, h, normalized(vneg(r.d)), n_occl, cnt, hit);
            return hit ? E : background(S);
        } else {
            if (!scene_intersect<EAGER, DEEP>(S, r, RV(1e-4), RT_INF, ht, h, cnt)) return background(S);
            return shade<EAGER, DEEP, DL, WV>(S, ht, h, normalized(vneg(r.d)), n_occl, cnt);
        }
    }
    Frame stk[kMaxDepth];
    int sp = 0;
    int depth = 0;
    const int limit = S.rec_limit;
    V3 ret;
    for (;;) {
        // ---- evaluate node (r, depth)
        bool descend = false;
        if (depth >= limit) {
            ret = v3(RV(0.0), RV(0.0), RV(0.0));
        } else {
            real ht = RV(0.0);
            DHit h;
            ++n_isect;
            if (!scene_intersect<EAGER, DEEP>(S, r, RV(1e-4), RT_INF, ht, h, cnt)) {
                ret = background(S);
            } else {
                const V3 wo = normalized(vneg(r.d));
                const V3 direct = shade<EAGER, DEEP, DL, WV>(S, ht, h, wo, n_occl, cnt);
                if (h.mat < 0) {
                    ret = direct;
                } else {
                    const MatT* mat = &S.mats[h.mat];
                    const bool can = depth < limit - 1;
                    const bool want_refl = mat->kr > RV(0.0) && can;
                    bool want_refr = false;
                    DRay refr;
                    if (mat->kt > RV(0.0) && can) {
                        const real eta = h.ff ? (S.medium_index / mat->refractive_index)
                                                : (mat->refractive_index / S.medium_index);
                        const V3 inc = normalized(r.d);
                        const real cos_i = -dot3(inc, h.n);   // tracer.cpp:100-104
                        const real st2 = eta * eta * dmax(RV(0.0), RV(1.0) - cos_i * cos_i);
                        if (!(st2 >= RV(1.0))) {
                            want_refr = true;
                            const real cos_t = sqrt_r(RV(1.0) - st2);   // tracer.cpp:87-98
                            const real k = eta * cos_i - cos_t;
                            const V3 rd = normalized(v3(inc.x * eta + h.n.x * k, inc.y * eta + h.n.y * k,
                                                        inc.z * eta + h.n.z * k));
                            const V3 ro = h.ff ? v3(h.p.x - h.n.x * RV(1e-6), h.p.y - h.n.y * RV(1e-6), h.p.z - h.n.z * RV(1e-6))
                                               : v3(h.p.x + h.n.x * RV(1e-6), h.p.y + h.n.y * RV(1e-6), h.p.z + h.n.z * RV(1e-6));
                            refr = make_ray(ro, rd);
                        }
                    }
                    if (want_refl || want_refr) {
                        Frame f;
                        f.total = direct;
                        f.mat = h.mat;
                        f.want_refr = want_refr;
                        f.refr = refr;
                        if (want_refl) {
                            cnt.inc(RT_OPC_SECONDARY);
                            const V3 inc = normalized(r.d);
                            const real k = RV(2.0) * dot3(inc, h.n);   // reflect (tracer.cpp:76-78)
                            const V3 rd = normalized(v3(inc.x - h.n.x * k, inc.y - h.n.y * k, inc.z - h.n.z * k));
                            const V3 ro = h.ff ? v3(h.p.x + h.n.x * RV(1e-6), h.p.y + h.n.y * RV(1e-6), h.p.z + h.n.z * RV(1e-6))
                                               : v3(h.p.x - h.n.x * RV(1e-6), h.p.y - h.n.y * RV(1e-6), h.p.z - h.n.z * RV(1e-6));
                            f.stage = 0;
                            stk[sp++] = f;
                            r = make_ray(ro, rd);
                        } else {
                            cnt.inc(RT_OPC_SECONDARY);
                            f.stage = 1;
                            stk[sp++] = f;
                            r = refr;
                        }
                        depth = sp;
                        descend = true;
                    } else {
                        ret = direct;
                    }
                }
            }
        }
        if (descend) continue;
        // ---- unwind
        bool resumed = false;
        while (sp > 0) {
            Frame& f = stk[sp - 1];
            const MatT* mat = &S.mats[f.mat];
            if (f.stage == 0) {
                f.total = combine(f.total, v3(ret.x * mat->kr, ret.y * mat->kr, ret.z * mat->kr));
                if (f.want_refr) {
                    cnt.inc(RT_OPC_SECONDARY);
                    f.stage = 1;
                    r = f.refr;
                    depth = sp;
                    resumed = true;
                    break;
                }
                ret = f.total;
                --sp;
            } else {
                f.total = combine(f.total, v3(ret.x * mat->kt, ret.y * mat->kt, ret.z * mat->kt));
                ret = f.total;
                --sp;
            }
        }
        if (!resumed) return ret;
    }
}

// ------------------------------------------------------------------ camera
// Camera::generate_ray_subpixel (camera.h:68-78)
__device__ __forceinline__ DRay gen_ray_subpixel(const DevScene& S, int i, int j, real dx, real dy) {
    const real sx = (i + RV(0.5) + dx) / (real)S.cam_nx;
    const real sy = (j + RV(0.5) + dy) / (real)S.cam_ny;
    const V3 Sp = v3(S.P[0] + S.Lx * sx + RV(0.0) * sy, S.P[1] + RV(0.0) * sx + S.Ly * sy, S.P[2] + RV(0.0) * sx + RV(0.0) * sy);
    const V3 e = ld3(S.eye);
    return make_ray(e, normalized(v3(Sp.x - e.x, Sp.y - e.y, Sp.z - e.z)));
}

// Camera::generate_ray (camera.h:44-58)
__device__ __forceinline__ DRay gen_ray(const DevScene& S, int i, int j) {
    const int nx = S.cam_nx, ny = S.cam_ny;
    const V3 e = ld3(S.eye);
    if (i < 0 || i >= nx || j < 0 || j >= ny) return make_ray(e, v3(RV(0.0), RV(0.0), -RV(1.0)));
    const real sx = ((real)i + RV(0.5)) / (real)nx;
    const int jf = ny - 1 - j;
    const real sy = ((real)jf + RV(0.5)) / (real)ny;
    const V3 Sp = v3(S.P[0] + S.Lx * sx + RV(0.0) * sy, S.P[1] + RV(0.0) * sx + S.Ly * sy, S.P[2] + RV(0.0) * sx + RV(0.0) * sy);
    return make_ray(e, normalized(v3(Sp.x - e.x, Sp.y - e.y, Sp.z - e.z)));
}

}  // namespace RT_NS
