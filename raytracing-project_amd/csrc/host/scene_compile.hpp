// scene_compile.hpp — lowers the scene IR (include/rt.h) to the device form.
//
// Every top-level object becomes one DevObj.  Leaf primitives are evaluated
// directly; any object involving a transform or a CSG node becomes a short
// post-order program of DevOps that the device interprets with WAVE-UNIFORM
// control flow (every lane runs the same op sequence; only data differs),
// replacing the reference's virtual recursion (Primitive::intersect /
// ::interval, geometry.h:62-75) with an explicit ray stack (transforms) and
// interval stack (CSG operands).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "rt.h"

namespace rtamd {

enum DevObjKind : int32_t { OBJ_SPHERE = 0, OBJ_HALF = 1, OBJ_POKE = 2, OBJ_PROG = 3, OBJ_NEVER = 4 };

enum DevOpCode : int32_t {
    OP_XPUSH = 0,       // push current ray, current = local ray of transform node
    OP_LEAF_IVL = 1,    // push Primitive::interval(leaf, current ray)
    OP_CSG = 2,         // pop b, pop a, push CSG::interval combine(op)
    OP_XPOP_IVL = 3,    // map top interval back through transform node, pop ray
    OP_LEAF_ISECT = 4,  // hit = Primitive::intersect(leaf, current ray, range)
    OP_CSG_ISECT = 5,   // hit = CSG::intersect from top interval, range
    OP_XPOP_HIT = 6,    // map hit back through transform node, check range, pop ray
    OP_NEVER = 7        // the subtree can never hit (degenerate Scaling, transform.cpp:97)
};

struct DevObj {
    int32_t kind;
    int32_t node;       // IR node index (leaf kinds)
    int32_t pc0, pc1;   // program range (OBJ_PROG)
    int32_t has_bound;  // conservative world-space bounding sphere present
    int32_t strict;     // 1 = accepts only t < tmax (CSG / transforms), 0 = t <= tmax
    int32_t pad[2];
    double bc[3];       // bound centre
    double br;          // bound radius (already inflated)
};

struct DevOp {
    int32_t op;
    int32_t node;       // IR node index (leaf / transform / csg)
    int32_t top;        // 1 = range is the query's (tmin,tmax); 0 = nested (0,inf)
    int32_t csg_op;
};

struct CompiledScene {
    std::vector<DevObj> objs;
    std::vector<DevOp> ops;
    int max_ray_depth = 0;   // transform nesting on any path
    int max_ivl_depth = 0;   // interval stack depth on any path
};

// Throws std::runtime_error on malformed IR.
CompiledScene compile_scene(const rt_scene_desc& d);

}  // namespace rtamd
