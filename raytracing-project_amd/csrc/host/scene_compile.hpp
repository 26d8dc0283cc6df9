// scene_compile.hpp — lowers the scene IR (include/rt.h) to the device form.
//
// Every top-level object becomes one DevObj, evaluated with WAVE-UNIFORM
// control flow (every lane walks the same op sequence; only data differs),
// replacing the reference's virtual recursion (Primitive::intersect /
// ::interval, geometry.h:62-75):
//   OBJ_SPHERE / OBJ_HALF / OBJ_POKE  a bare leaf primitive,
//   OBJ_CHAIN  a chain of m >= 0 transforms over either one leaf or a CSG tree
//              whose operands are leaves / CSG nodes only.  Intervals carry
//              lazy hit references; normals and materials are resolved once
//              for the winning hit (DESIGN.md §Lazy hits),
//   OBJ_EAGER  anything else (a transform inside a CSG operand): a general
//              post-order program with full hit records (rare; its own
//              kernel variant so it never costs the common case registers),
//   OBJ_NEVER  can never report a hit (degenerate Scaling, transform.cpp:97).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "rt.h"

namespace rtamd {

enum DevObjKind : int32_t {
    OBJ_SPHERE = 0,
    OBJ_HALF = 1,
    OBJ_POKE = 2,
    OBJ_CHAIN = 3,
    OBJ_EAGER = 4,
    OBJ_NEVER = 5,
    OBJ_GROUP = 6       // cull header: the next m objects lie inside bound (skipped when no lane touches it)
};

enum DevOpCode : int32_t {
    OP_XPUSH = 0,       // push current ray, current = local ray of transform node
    OP_LEAF_IVL = 1,    // push Primitive::interval(leaf, current ray)
    OP_CSG = 2,         // pop b, pop a, push CSG::interval combine(op)
    OP_XPOP_IVL = 3,    // (eager) map top interval back through transform node, pop ray
    OP_LEAF_ISECT = 4,  // hit = Primitive::intersect(leaf, current ray, range)
    OP_CSG_ISECT = 5,   // hit = CSG::intersect from top interval, range
    OP_XPOP_HIT = 6,    // (eager) map hit back through transform node, check range, pop ray
    OP_NEVER = 7,       // the subtree can never hit (degenerate Scaling, transform.cpp:97)
    OP_IVL_GROUP = 8    // compact: the next `top` ops fold sphere leaves into the stack top with csg_op;
                        // skipped (one combine with an empty interval) when no lane's line meets ball `node`
};

struct DevObj {
    int32_t kind;
    int32_t node;       // leaf node (bare leaves; CHAIN with a leaf core)
    int32_t pc0;        // CHAIN: first XPUSH op; EAGER: program start
    int32_t m;          // CHAIN: number of transforms in the chain; GROUP: member count
    int32_t core;       // CHAIN: 0 = leaf core, 1 = CSG core
    int32_t cpc0, cpc1; // CHAIN: leaf core -> cpc0 = its LEAF_ISECT op; CSG core -> [cpc0,cpc1) compact program
    int32_t pc1;        // EAGER: program end
    int32_t has_bound;  // conservative world-space bounding sphere present
    int32_t pb0;        // CHAIN with a compact CSG core: first leaf prefilter ball in gbounds (units of 4 floats)
    int32_t npb;        //   and their count (0 = none): world balls of every leaf, grown by the CSG epsilon slop
    int32_t fold0;      // CHAIN whose CSG core is a left-deep fold of one operator over sphere / pokeball
    int32_t nfold;      //   leaves (the loader's n-ary arrays): first FoldLeaf and leaf count (0 = not a fold)
    int32_t fold_op;    //   the fold's rt_csg_op
    int32_t pad;
    double bc[3];       // bound centre
    double br;          // bound radius (already inflated)
    float fb[4];        // the same ball in float (cx, cy, cz, r), inflated for the f32 cull test
};

// One leaf of a fold object (DevObj::fold0), in fold order = the order of the
// object's OP_LEAF_IVL ops and of its prefilter balls.  pc is the leaf's
// OP_LEAF_IVL op index (its lazy hit-reference code).
struct FoldLeaf {
    double c[3];
    double r;
    int32_t pc;
    int32_t pad;
};

struct DevOp {
    int32_t op;
    int32_t node;       // IR node index (leaf / transform / csg)
    int32_t top;        // eager: 1 = range is the query's (tmin,tmax); 0 = nested (0,inf); 2 = NEVER in interval mode
    int32_t csg_op;
};

struct CompiledScene {
    std::vector<DevObj> objs;
    std::vector<DevOp> ops;
    std::vector<FoldLeaf> fold;    // leaves of the fold objects (DevObj::fold0)
    // Wave-level cull record of every object (8 floats, objs order), read by
    // lane j for object j in the transposed tests: (c, r) of the f32 bound
    // ball or, for a bare half-space, (n, n.p) of its plane; then the type
    // (0 never a candidate: group / never-hit, 1 always, 2 ball, 3 plane)
    // and, for a plane, |px| + |py| + |pz| (the f32 margin's scale).
    std::vector<float> ctab;
    std::vector<float> gbounds;    // OP_IVL_GROUP bounds: (cx, cy, cz, r) per group, in the CSG frame, f32-inflated;
                                   // then the leaf prefilter balls of CHAIN objects (world frame, see DevObj::pb0)
    // Wave BVH (scenes with more than kWaveBvhMin = 256 objects and no eager
    // programs; DESIGN.md §Wave BVH): the wave kernels' object list - every
    // object except group headers and never-hit objects, unbounded ones
    // first, the rest in Morton order of their bound centres - with its cull
    // records, each object's index in objs (the reference's order, which
    // decides closest-hit ties) and one cull record per chunk of kWaveChunk
    // consecutive objects (the enclosing ball; type 1 = always a candidate
    // for a chunk with an unbounded member).  Empty: no BVH.
    std::vector<DevObj> wobjs;
    std::vector<float> wctab;
    std::vector<int32_t> worig;
    std::vector<float> wchunk;
    // Light-relative shadow cull records (light_records, scene_compile.cpp):
    // [light][record] x 8 floats for ctab (lrec), wctab (lwrec) and every
    // gbounds ball (lgb); the shadow-query culls of scene_occluded_wave.
    std::vector<float> lrec, lwrec, lgb;
    int max_ray_depth = 0;   // transform nesting on any path of an eager program (chains need no stack)
    int max_ivl_depth = 0;   // interval stack depth on any path
    bool has_eager = false;  // some object needs the eager interpreter
    // Unbounded objects (ctab type 1 / 3) that precede every bounded one in
    // objs order (0 if an unbounded object follows a bounded one, or more
    // than 64 lead).  The wave kernels without the BVH test these one by one
    // before the transposed tests, which then cover only the objects behind
    // them: a floor plus 64 spheres (config 5) is one 64-object chunk, not
    // two.  Visiting them first keeps the reference's order (closest-hit ties).
    int n_lead = 0;
    bool has_pokeball = false;
};

constexpr int kWaveChunk = 64;   // objects per transposed test (one wave)
constexpr int kWaveBvhMin = 4 * kWaveChunk;   // the wave BVH is built for scenes of more objects

// Closest-hit tie rule of Scene::intersect (scene.cpp:10-24) for an object:
// does it accept a hit at t == tmax (a later such object replaces an earlier
// one at the same t)?  Spheres, half-spaces and pokeballs do (geometry.cpp
// range tests), a CSG or a transform does not (strict t < tmax).
#ifdef __HIP__
__host__ __device__
#endif
inline bool accepts_tie(const DevObj& o) {
    return o.kind == OBJ_SPHERE || o.kind == OBJ_HALF || o.kind == OBJ_POKE ||
           (o.kind == OBJ_CHAIN && o.m == 0 && o.core == 0);
}

// Throws std::runtime_error on malformed IR.
CompiledScene compile_scene(const rt_scene_desc& d);

// Pokeball::pick_region_material (geometry.cpp:163-180) decides its button /
// ring regions by comparing ang = std::acos(x), x = clamp1(u . btnDir), with
// btnOuter and inner = max(0, btnOuter - ringWidth).  The host's acos (glibc,
// the reference's own) is monotone non-increasing, so
//   ang <= btnOuter  <=>  x >= xb   (xb: the least double in [-1, 1] with acos(x) <= btnOuter)
//   ang >= inner     <=>  x <= xi   (xi: the greatest double in [-1, 1] with acos(x) >= inner)
// and the device compares x with these two thresholds instead of evaluating
// acos: the reference's decision exactly (the device math library's acos
// could differ from glibc's in the last bit).  No such x: xb = 2 / xi = -2.
// Device node slots of a pokeball (rt_render.hip frame_begin fills them in
// the device copy of the nodes; the IR's v[10..23] of a pokeball are unused).
constexpr int kPokeXb = 20, kPokeXi = 21;
void pokeball_thresholds(double btn_outer, double ring_width, double& xb, double& xi);

}  // namespace rtamd
