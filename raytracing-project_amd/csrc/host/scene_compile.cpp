// scene_compile.cpp — IR -> device object table + wave-uniform programs.
//
// Bounds: every node gets a conservative bounding sphere in the frame of the
// ray it is queried with, or "unbounded" (half-spaces and anything whose
// result can extend along them), or "empty" (can never report an interval
// or a hit: degenerate Scaling, transform.cpp:97).  The bound of a CSG node
// follows from the reference's interval semantics (csg.cpp:61-163): a union
// is inside only where a child is; an intersection only where BOTH are; a
// difference only where A is; the result's events are child events or the
// origin (which then lies inside a child).  A ray whose [tmin,tmax] segment
// misses an inflated bound therefore gets "no hit" from that subtree, which
// lets the device skip it when no lane of the wave needs it.
#include "scene_compile.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace rtamd {
namespace {

struct Bound {
    enum Kind { Empty, Unbounded, Ball } kind = Unbounded;
    double c[3] = {0, 0, 0};
    double r = 0;
};

Bound ball(double x, double y, double z, double r) {
    Bound b;
    b.kind = Bound::Ball;
    b.c[0] = x; b.c[1] = y; b.c[2] = z;
    b.r = std::fabs(r);
    return b;
}

Bound merge_union(const Bound& a, const Bound& b) {
    if (a.kind == Bound::Empty) return b;
    if (b.kind == Bound::Empty) return a;
    if (a.kind == Bound::Unbounded || b.kind == Bound::Unbounded) return Bound{};
    double d[3] = {b.c[0] - a.c[0], b.c[1] - a.c[1], b.c[2] - a.c[2]};
    double dist = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    if (dist + b.r <= a.r) return a;
    if (dist + a.r <= b.r) return b;
    double R = 0.5 * (dist + a.r + b.r);
    Bound o;
    o.kind = Bound::Ball;
    double k = (dist > 0) ? (R - a.r) / dist : 0.0;
    for (int i = 0; i < 3; ++i) o.c[i] = a.c[i] + d[i] * k;
    o.r = R;
    return o;
}

// A ball in float for the device's f32 cull tests (rt_device.hpp ball_touch):
// the double ball grown by 1e-6 of its scale, rounded outward, so that the
// float centre's rounding error stays inside it.
void float_ball(const double c[3], double r, float out[4]) {
    const double mag = std::fabs(c[0]) + std::fabs(c[1]) + std::fabs(c[2]) + r;
    for (int k = 0; k < 3; ++k) out[k] = (float)c[k];
    out[3] = std::nextafter((float)(r + 1e-6 * (1.0 + mag)), INFINITY);
}

// |x| + |y| + |z| + r of a float ball, rounded up: the magnitude a cull record
// carries (record word 5) for the device tests' margins, so the transposed
// tests do not re-add it per lane.
float float_ball_mag(const float b[4]) {
    const double m = std::fabs((double)b[0]) + std::fabs((double)b[1]) + std::fabs((double)b[2]) + (double)b[3];
    return std::nextafter((float)m, INFINITY);
}

// Light-relative shadow cull records (CompiledScene::lrec / lwrec / lgb):
// for every point light L, one 8-float record per input record (ctab layout:
// c0 = ball (c, r) or plane (n, n.p); c1.x = type; c1.y = magnitude).  A ball
// becomes (w = c - L, |w|^2) + (type, r, |w.x|+|w.y|+|w.z|+r); a bare
// half-space's plane (n, n.p) + (type, n.L - n.p, |p| + |L|); other types are
// copied.  `stride` floats per input record (8 for ctab, 4 for bare balls of
// gbounds, which are all type 2).  Computed in double, rounded to nearest:
// the device tests carry margins of >= 4e-6 of these magnitudes.
void light_records(const float* rec, size_t n, int stride, const rt_light* lights, int n_lights,
                   std::vector<float>& out) {
    out.assign((size_t)std::max(0, n_lights) * n * 8, 0.0f);
    for (int l = 0; l < n_lights; ++l) {
        const double* L = lights[l].pos;
        for (size_t j = 0; j < n; ++j) {
            const float* r = rec + (size_t)stride * j;
            float* o = &out[((size_t)l * n + j) * 8];
            int type = 2;
            if (stride == 8) std::memcpy(&type, &r[4], sizeof(int));
            if (type == 2) {
                const double w[3] = {(double)r[0] - L[0], (double)r[1] - L[1], (double)r[2] - L[2]};
                for (int k = 0; k < 3; ++k) o[k] = (float)w[k];
                o[3] = (float)(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
                o[5] = r[3];
                o[6] = std::nextafter((float)(std::fabs(w[0]) + std::fabs(w[1]) + std::fabs(w[2]) + (double)r[3]), INFINITY);
            } else if (type == 3) {
                for (int k = 0; k < 4; ++k) o[k] = r[k];
                o[5] = (float)((double)r[0] * L[0] + (double)r[1] * L[1] + (double)r[2] * L[2] - (double)r[3]);
                o[6] = std::nextafter((float)((double)r[5] + std::fabs(L[0]) + std::fabs(L[1]) + std::fabs(L[2])), INFINITY);
            }
            std::memcpy(&o[4], &type, sizeof(int));
        }
    }
}

bool is_degenerate_scaling(const rt_node& n) {
    const double kEPS = 1e-6;   // core.h:10, checked at transform.cpp:97
    return n.kind == RT_NODE_SCALING &&
           (std::fabs(n.v[0]) < kEPS || std::fabs(n.v[5]) < kEPS || std::fabs(n.v[10]) < kEPS);
}

// The ball b of a transform node's child, in the node's parent frame.
Bound xform_ball(const rt_node& n, const Bound& b) {
    if (b.kind != Bound::Ball) return b;
    if (n.kind == RT_NODE_TRANSLATION) return ball(b.c[0] + n.v[3], b.c[1] + n.v[7], b.c[2] + n.v[11], b.r);
    if (n.kind == RT_NODE_SCALING) {
        double s = std::max(std::fabs(n.v[0]), std::max(std::fabs(n.v[5]), std::fabs(n.v[10])));
        return ball(b.c[0] * n.v[0], b.c[1] * n.v[5], b.c[2] * n.v[10], b.r * s);
    }
    const double* M = n.v;   // rotation
    return ball(M[0] * b.c[0] + M[1] * b.c[1] + M[2] * b.c[2] + M[3],
                M[4] * b.c[0] + M[5] * b.c[1] + M[6] * b.c[2] + M[7],
                M[8] * b.c[0] + M[9] * b.c[1] + M[10] * b.c[2] + M[11], b.r);
}

class Compiler {
public:
    explicit Compiler(const rt_scene_desc& d) : d_(d) {}

    // Height of the CSG tree rooted at idx (0 for a leaf).
    int csg_height(int idx, int level = 0) {
        if (level > 4096) throw std::runtime_error("scene graph too deep");
        const rt_node& n = d_.nodes[idx];
        if (n.kind != RT_NODE_CSG) return 0;
        return 1 + std::max(csg_height(n.a, level + 1), csg_height(n.b, level + 1));
    }

    // Leaf prefilter of a CHAIN object with a compact CSG core (ops
    // [cpc0, cpc1)): a hit of the object lies at a point of the CSG's first
    // interval, and every point of a CSG interval is within height x 1e-6 (the
    // event comparator's tie width, once per level) of some leaf interval,
    // i.e. of a leaf's ball - the result's events are leaf events or the
    // origin, which then lies inside a leaf (csg.cpp:61-163).  So a segment
    // that passes no leaf ball grown by that slop cannot hit the object.  The
    // balls are mapped through the transform chain to the world frame.
    void leaf_prefilter(DevObj& o, const std::vector<int>& chain, int core, CompiledScene& cs) {
        std::vector<int> leaves;
        for (int pc = o.cpc0; pc < o.cpc1; ++pc)
            if (cs.ops[pc].op == OP_LEAF_IVL) leaves.push_back(cs.ops[pc].node);
        if (leaves.empty() || leaves.size() > 64) return;
        const double slop = (csg_height(core) + 2) * 1e-6;
        std::vector<float> balls;
        for (int lf : leaves) {
            Bound b = bound(lf);
            if (b.kind != Bound::Ball) return;   // a half-space leaf: no prefilter
            b.r += slop;
            for (size_t k = chain.size(); k-- > 0;) b = xform_ball(d_.nodes[chain[k]], b);
            float fb[4];
            float_ball(b.c, b.r, fb);
            balls.insert(balls.end(), fb, fb + 4);
        }
        o.pb0 = (int)(cs.gbounds.size() / 4);
        o.npb = (int)leaves.size();
        cs.gbounds.insert(cs.gbounds.end(), balls.begin(), balls.end());
    }

    // A compact CSG core that is a left-deep fold of ONE operator whose
    // operands are all sphere / pokeball leaves (the loader's n-ary
    // union / intersection / difference arrays, json_loader.cpp:375-401, and
    // binary csg chains of that shape) gets a flat leaf table: the device
    // evaluates it as acc = leaf_0; acc = acc op leaf_k (csg.cpp:61-163)
    // without the op interpreter, skipping leaves by the wave's line mask
    // (rt_device.hpp run_fold).  Needs the leaf prefilter balls (same order).
    void fold_leaves(DevObj& o, int core, CompiledScene& cs) {
        if (o.npb <= 0) return;
        const int op = d_.nodes[core].op;
        std::vector<int> rhs;
        int cur = core;
        while (d_.nodes[cur].kind == RT_NODE_CSG && d_.nodes[cur].op == op) {
            rhs.push_back(d_.nodes[cur].b);
            cur = d_.nodes[cur].a;
        }
        auto is_ball = [&](int i) {
            const int k = d_.nodes[i].kind;
            return k == RT_NODE_SPHERE || k == RT_NODE_POKEBALL;
        };
        if (!is_ball(cur)) return;
        for (int b : rhs)
            if (!is_ball(b)) return;
        std::vector<int> leaves{cur};
        for (size_t k = rhs.size(); k-- > 0;) leaves.push_back(rhs[k]);   // innermost first
        std::vector<int> pcs;
        for (int pc = o.cpc0; pc < o.cpc1; ++pc)
            if (cs.ops[pc].op == OP_LEAF_IVL) pcs.push_back(pc);
        if (pcs.size() != leaves.size() || (int)leaves.size() != o.npb || leaves.size() > 64) return;
        o.fold0 = (int)cs.fold.size();
        o.nfold = (int)leaves.size();
        o.fold_op = op;
        for (size_t k = 0; k < leaves.size(); ++k) {
            const rt_node& n = d_.nodes[leaves[k]];
            if (cs.ops[pcs[k]].node != leaves[k]) throw std::runtime_error("fold leaf order mismatch");
            FoldLeaf f{};
            for (int i = 0; i < 3; ++i) f.c[i] = n.v[i];
            f.r = n.v[3];
            f.pc = pcs[k];
            cs.fold.push_back(f);
        }
    }

    Bound bound(int idx, int level = 0) {
        if (level > 4096) throw std::runtime_error("scene graph too deep");
        const rt_node& n = d_.nodes[idx];
        switch (n.kind) {
            case RT_NODE_SPHERE:
            case RT_NODE_POKEBALL:
                return ball(n.v[0], n.v[1], n.v[2], n.v[3]);
            case RT_NODE_HALFSPACE:
                return Bound{};
            case RT_NODE_TRANSLATION:
            case RT_NODE_SCALING:
            case RT_NODE_ROTATION:
                if (is_degenerate_scaling(n)) { Bound e; e.kind = Bound::Empty; return e; }
                return xform_ball(n, bound(n.a, level + 1));
            case RT_NODE_CSG: {
                Bound a = bound(n.a, level + 1), b = bound(n.b, level + 1);
                if (n.op == RT_CSG_UNION) return merge_union(a, b);
                if (n.op == RT_CSG_INTERSECTION) {
                    if (a.kind == Bound::Empty || b.kind == Bound::Empty) { Bound e; e.kind = Bound::Empty; return e; }
                    if (a.kind == Bound::Ball && b.kind == Bound::Ball) return a.r <= b.r ? a : b;
                    if (a.kind == Bound::Ball) return a;
                    if (b.kind == Bound::Ball) return b;
                    return Bound{};
                }
                return a;   // difference: inside only where A is
            }
        }
        throw std::runtime_error("unknown node kind");
    }

    void emit_isect(int idx, int top, int level) {
        if (level > 4096) throw std::runtime_error("scene graph too deep");
        const rt_node& n = d_.nodes[idx];
        switch (n.kind) {
            case RT_NODE_SPHERE:
            case RT_NODE_HALFSPACE:
            case RT_NODE_POKEBALL:
                op(OP_LEAF_ISECT, idx, top);
                return;
            case RT_NODE_TRANSLATION:
            case RT_NODE_SCALING:
            case RT_NODE_ROTATION:
                if (is_degenerate_scaling(n)) { op(OP_NEVER, idx, top); return; }
                op(OP_XPUSH, idx, top);
                ray_push();
                emit_isect(n.a, 0, level + 1);
                op(OP_XPOP_HIT, idx, top);
                --rdepth_;
                return;
            case RT_NODE_CSG:
                emit_ivl(idx, level + 1);
                op(OP_CSG_ISECT, idx, top);
                --idepth_;
                return;
        }
        throw std::runtime_error("unknown node kind");
    }

    void emit_ivl(int idx, int level) {
        if (level > 4096) throw std::runtime_error("scene graph too deep");
        const rt_node& n = d_.nodes[idx];
        switch (n.kind) {
            case RT_NODE_SPHERE:
            case RT_NODE_HALFSPACE:
            case RT_NODE_POKEBALL:
                op(OP_LEAF_IVL, idx, 0);
                ivl_push();
                return;
            case RT_NODE_TRANSLATION:
            case RT_NODE_SCALING:
            case RT_NODE_ROTATION:
                if (is_degenerate_scaling(n)) {
                    op(OP_NEVER, idx, 2);   // top == 2: push an empty interval
                    ivl_push();
                    return;
                }
                op(OP_XPUSH, idx, 0);
                ray_push();
                emit_ivl(n.a, level + 1);
                op(OP_XPOP_IVL, idx, 0);
                --rdepth_;
                return;
            case RT_NODE_CSG: {
                emit_ivl(n.a, level + 1);
                emit_ivl(n.b, level + 1);
                DevOp& o = op(OP_CSG, idx, 0);
                o.csg_op = n.op;
                --idepth_;   // two popped, one pushed
                return;
            }
        }
        throw std::runtime_error("unknown node kind");
    }

    // CSG subtree made of CSG nodes and leaves only, every leaf with a material.
    bool compact_csg(int idx, int level) {
        if (level > 4096) throw std::runtime_error("scene graph too deep");
        const rt_node& n = d_.nodes[idx];
        switch (n.kind) {
            case RT_NODE_SPHERE:
            case RT_NODE_HALFSPACE:
                return n.mat >= 0;
            case RT_NODE_POKEBALL:
                for (int k = 0; k < 5; ++k)
                    if (n.mats[k] < 0) return false;
                return true;
            case RT_NODE_CSG:
                return compact_csg(n.a, level + 1) && compact_csg(n.b, level + 1);
            default:
                return false;
        }
    }

    // Compact interval program of a CSG subtree.  A left-deep fold of one
    // operator (the loader's n-ary arrays, json_loader.cpp:375-401) is
    // emitted as a0, b1, CSG, b2, CSG, ...; runs of consecutive sphere /
    // pokeball operands b_i..b_j may get an OP_IVL_GROUP header.  Skipping a
    // run is exact: a leaf whose line misses its sphere has an empty
    // interval, and combining the running interval with an empty one is
    // idempotent (csg_c: A op empty = f(A) with f(f(A)) = f(A)), so m skipped
    // steps equal one combine with an empty interval.
    //
    // The runs are chosen by dynamic programming over the fold order with the
    // cost model "a header costs one leaf test and is passed by a fraction
    // (R_group / R_fold)^2 of the rays that reach the fold", R_fold being the
    // ball around every bounded operand.
    void emit_compact_ivl(int idx) {
        const rt_node& n = d_.nodes[idx];
        if (n.kind != RT_NODE_CSG) {
            op(OP_LEAF_IVL, idx, 0);
            ivl_push();
            return;
        }
        std::vector<int> spine, rhs;   // fold steps, innermost first
        int cur = idx;
        while (d_.nodes[cur].kind == RT_NODE_CSG && d_.nodes[cur].op == n.op) {
            spine.push_back(cur);
            rhs.push_back(d_.nodes[cur].b);
            cur = d_.nodes[cur].a;
        }
        std::reverse(spine.begin(), spine.end());
        std::reverse(rhs.begin(), rhs.end());
        emit_compact_ivl(cur);

        const size_t m = rhs.size();
        std::vector<char> ball_leaf(m);
        Bound fold;
        fold.kind = Bound::Empty;
        {
            const Bound b0 = bound(cur);
            if (b0.kind == Bound::Ball) fold = b0;
        }
        for (size_t k = 0; k < m; ++k) {
            const int kind = d_.nodes[rhs[k]].kind;
            ball_leaf[k] = kind == RT_NODE_SPHERE || kind == RT_NODE_POKEBALL;
            const Bound b = bound(rhs[k]);
            if (b.kind == Bound::Ball) fold = merge_union(fold, b);
        }
        // best[k] = cost of operands [0, k); from[k] = start of the last run
        // (a header is an f32 line test, ~1/4 of an FP64 sphere interval)
        constexpr size_t kMaxRun = 32;
        constexpr double kHeader = 0.25;
        std::vector<double> best(m + 1, 0.0);
        std::vector<size_t> from(m + 1, 0);
        std::vector<char> hdr(m + 1, 0), grouped(m + 1, 0);
        for (size_t k = 1; k <= m; ++k) {
            best[k] = best[k - 1] + 1.0;
            from[k] = k - 1;
            if (!ball_leaf[k - 1] || fold.kind != Bound::Ball || fold.r <= 0.0) continue;
            Bound g = bound(rhs[k - 1]);
            for (size_t i = k; i-- > 0 && k - i <= kMaxRun;) {
                if (!ball_leaf[i]) break;
                if (i + 1 < k) g = merge_union(g, bound(rhs[i]));
                const double f = std::min(1.0, g.r / fold.r);
                const double c = best[i] + kHeader + f * f * (double)(k - i);
                if (c < best[k]) {
                    best[k] = c;
                    from[k] = i;
                    hdr[k] = 1;
                }
            }
        }
        std::vector<std::pair<size_t, size_t>> runs;
        for (size_t k = m; k > 0; k = from[k]) {
            runs.emplace_back(from[k], k);
            if (hdr[k]) grouped[from[k]] = 1;
        }
        std::reverse(runs.begin(), runs.end());
        for (const auto& run : runs) {
            const size_t i = run.first, j = run.second;
            if (j - i >= 2 || grouped[i]) {
                Bound g = bound(rhs[i]);
                for (size_t k = i + 1; k < j; ++k) g = merge_union(g, bound(rhs[k]));
                DevOp& h = op(OP_IVL_GROUP, (int)(gb_->size() / 4), 2 * (int)(j - i));
                h.csg_op = n.op;
                float fb[4];
                float_ball(g.c, g.r, fb);
                gb_->insert(gb_->end(), fb, fb + 4);
            }
            for (size_t k = i; k < j; ++k) {
                emit_compact_ivl(rhs[k]);
                DevOp& o = op(OP_CSG, spine[k], 0);
                o.csg_op = n.op;
                --idepth_;
            }
        }
    }

    CompiledScene run() {
        CompiledScene cs;
        ops_ = &cs.ops;
        gb_ = &cs.gbounds;
        for (int k = 0; k < d_.n_nodes; ++k)
            if (d_.nodes[k].kind == RT_NODE_POKEBALL) cs.has_pokeball = true;
        for (int i = 0; i < d_.n_objects; ++i) {
            int idx = d_.objects[i];
            DevObj o{};
            o.node = idx;
            o.pc0 = o.pc1 = o.cpc0 = o.cpc1 = (int)cs.ops.size();
            Bound b = bound(idx);
            // transform chain above the core
            std::vector<int> chain;
            int core = idx;
            bool degenerate = false;
            while (d_.nodes[core].kind >= RT_NODE_TRANSLATION && d_.nodes[core].kind <= RT_NODE_ROTATION) {
                if (is_degenerate_scaling(d_.nodes[core])) degenerate = true;
                chain.push_back(core);
                core = d_.nodes[core].a;
            }
            const rt_node& cn = d_.nodes[core];
            const bool leaf_core = cn.kind == RT_NODE_SPHERE || cn.kind == RT_NODE_HALFSPACE || cn.kind == RT_NODE_POKEBALL;
            if (b.kind == Bound::Empty || degenerate) {
                o.kind = OBJ_NEVER;
            } else if (chain.empty() && leaf_core) {
                o.kind = cn.kind == RT_NODE_SPHERE ? OBJ_SPHERE : cn.kind == RT_NODE_HALFSPACE ? OBJ_HALF : OBJ_POKE;
            } else if (leaf_core || (cn.kind == RT_NODE_CSG && compact_csg(core, 0))) {
                o.kind = OBJ_CHAIN;
                o.m = (int)chain.size();
                rdepth_ = idepth_ = 0;
                // (a chain maps its ray level by level in registers: no ray stack)
                for (int t : chain) op(OP_XPUSH, t, 0);
                o.node = core;
                o.cpc0 = (int)cs.ops.size();
                if (leaf_core) {
                    o.core = 0;
                    op(OP_LEAF_ISECT, core, 0);
                } else {
                    o.core = 1;
                    emit_compact_ivl(core);
                }
                o.cpc1 = (int)cs.ops.size();
                o.pc1 = o.cpc1;
                if (!leaf_core) {
                    leaf_prefilter(o, chain, core, cs);
                    fold_leaves(o, core, cs);
                }
            } else {
                o.kind = OBJ_EAGER;
                cs.has_eager = true;
                o.pc0 = (int)cs.ops.size();
                rdepth_ = idepth_ = 0;
                emit_isect(idx, 1, 0);
                o.pc1 = (int)cs.ops.size();
            }
            if (b.kind == Bound::Ball) {
                o.has_bound = 1;
                double mag = std::fabs(b.c[0]) + std::fabs(b.c[1]) + std::fabs(b.c[2]) + b.r;
                for (int k = 0; k < 3; ++k) o.bc[k] = b.c[k];
                o.br = b.r * (1.0 + 1e-7) + 1e-7 * (1.0 + mag);
                float_ball(b.c, b.r, o.fb);
            }
            cs.objs.push_back(o);
        }
        cs.max_ray_depth = max_r_;
        cs.max_ivl_depth = max_i_;
        cs.objs = insert_groups(cs.objs);
        cs.ctab.assign(cs.objs.size() * 8, 0.0f);
        for (size_t j = 0; j < cs.objs.size(); ++j) {
            const DevObj& o = cs.objs[j];
            float* c = &cs.ctab[8 * j];
            int type = 1;
            if (o.kind == OBJ_GROUP || o.kind == OBJ_NEVER) {
                type = 0;
            } else if (o.has_bound) {
                type = 2;
                for (int k = 0; k < 4; ++k) c[k] = o.fb[k];
                c[5] = float_ball_mag(c);
            } else if (o.kind == OBJ_HALF) {
                type = 3;
                const double* v = d_.nodes[o.node].v;   // point v[0..2], unit normal v[3..5]
                for (int k = 0; k < 3; ++k) c[k] = (float)v[3 + k];
                c[3] = (float)(v[3] * v[0] + v[4] * v[1] + v[5] * v[2]);
                c[5] = (float)(std::fabs(v[0]) + std::fabs(v[1]) + std::fabs(v[2]));
            }
            std::memcpy(&c[4], &type, sizeof(int));
        }
        {
            auto type_of = [&](size_t j) {
                int t;
                std::memcpy(&t, &cs.ctab[8 * j + 4], sizeof t);
                return t;
            };
            size_t lead = 0;
            while (lead < cs.objs.size() && (type_of(lead) == 1 || type_of(lead) == 3)) ++lead;
            bool ok = lead <= 64;
            for (size_t j = lead; ok && j < cs.objs.size(); ++j) ok = type_of(j) != 1 && type_of(j) != 3;
            cs.n_lead = ok ? (int)lead : 0;
        }
        build_wave_bvh(cs);
        light_records(cs.ctab.data(), cs.objs.size(), 8, d_.lights, d_.n_lights, cs.lrec);
        light_records(cs.wctab.data(), cs.wobjs.size(), 8, d_.lights, d_.n_lights, cs.lwrec);
        light_records(cs.gbounds.data(), cs.gbounds.size() / 4, 4, d_.lights, d_.n_lights, cs.lgb);
        return cs;
    }

    // The wave BVH (CompiledScene::wobjs ...).  Morton order of the f32 bound
    // centres over their bounding box (10 bits per axis) puts nearby objects
    // in the same chunk, so a chunk's enclosing ball is tight and one
    // transposed test over the chunk records skips whole chunks of objects.
    static void build_wave_bvh(CompiledScene& cs) {
        std::vector<int> ids;
        for (size_t j = 0; j < cs.objs.size(); ++j)
            if (cs.objs[j].kind != OBJ_GROUP && cs.objs[j].kind != OBJ_NEVER) ids.push_back((int)j);
        // (up to four chunks the transposed object test alone is as cheap:
        // 145 objects ran 8 % slower with the BVH, profiles/r03g_bvh_perf.txt)
        static const int bvh_min = [] {   // RT_BVH_MIN: measurement override of kWaveBvhMin
            const char* e = std::getenv("RT_BVH_MIN");
            return e && *e ? std::atoi(e) : kWaveBvhMin;
        }();
        if (cs.has_eager || (int)ids.size() <= bvh_min) return;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int j : ids)
            if (cs.objs[j].has_bound)
                for (int k = 0; k < 3; ++k) {
                    lo[k] = std::min(lo[k], cs.objs[j].bc[k]);
                    hi[k] = std::max(hi[k], cs.objs[j].bc[k]);
                }
        auto spread = [](uint32_t v) {   // 10 bits -> every third bit
            v &= 0x3ffu;
            v = (v | (v << 16)) & 0x030000ffu;
            v = (v | (v << 8)) & 0x0300f00fu;
            v = (v | (v << 4)) & 0x030c30c3u;
            v = (v | (v << 2)) & 0x09249249u;
            return v;
        };
        auto morton = [&](const DevObj& o) -> uint64_t {
            if (!o.has_bound) return 0;   // unbounded objects first (their chunks are never skipped)
            uint32_t code = 0;
            for (int k = 0; k < 3; ++k) {
                const double ext = hi[k] - lo[k];
                const double u = ext > 0 ? (o.bc[k] - lo[k]) / ext : 0.0;
                const uint32_t q = (uint32_t)std::min(1023.0, std::max(0.0, std::floor(u * 1024.0)));
                code |= spread(q) << k;
            }
            return 1 + (uint64_t)code;
        };
        std::vector<std::pair<uint64_t, int>> keyed;
        for (int j : ids) keyed.emplace_back(morton(cs.objs[j]), j);
        std::stable_sort(keyed.begin(), keyed.end(),
                         [](const std::pair<uint64_t, int>& a, const std::pair<uint64_t, int>& b) { return a.first < b.first; });
        // the unbounded objects fill the first chunk(s), padded with
        // never-hit entries so that every later chunk is all balls
        size_t n_unb = 0;
        while (n_unb < keyed.size() && keyed[n_unb].first == 0) ++n_unb;
        const size_t pad = n_unb % kWaveChunk ? kWaveChunk - n_unb % kWaveChunk : 0;
        const size_t n = keyed.size() + pad;
        cs.wobjs.assign(n, DevObj{});
        cs.worig.assign(n, -1);
        cs.wctab.assign(n * 8, 0.0f);   // (type 0: never a candidate)
        for (size_t i = n_unb; i < n_unb + pad; ++i) cs.wobjs[i].kind = OBJ_NEVER;
        for (size_t k = 0; k < keyed.size(); ++k) {
            const size_t i = k < n_unb ? k : k + pad;
            const int j = keyed[k].second;
            cs.wobjs[i] = cs.objs[j];
            cs.worig[i] = j;
            std::memcpy(&cs.wctab[8 * i], &cs.ctab[8 * (size_t)j], 8 * sizeof(float));
        }
        const size_t nch = (n + kWaveChunk - 1) / kWaveChunk;
        cs.wchunk.assign(nch * 8, 0.0f);
        for (size_t c = 0; c < nch; ++c) {
            const size_t a = c * kWaveChunk, b = std::min(n, a + kWaveChunk);
            bool all_bounded = true;
            double C[3] = {0.0, 0.0, 0.0};
            size_t cnt = 0;
            for (size_t i = a; i < b; ++i) {
                if (cs.wobjs[i].kind == OBJ_NEVER) continue;   // (padding)
                all_bounded = all_bounded && cs.wobjs[i].has_bound;
                for (int k = 0; k < 3; ++k) C[k] += cs.wobjs[i].bc[k];
                ++cnt;
            }
            float* rec = &cs.wchunk[8 * c];
            int type = 1;
            if (all_bounded && cnt > 0) {
                for (int k = 0; k < 3; ++k) C[k] /= (double)cnt;
                double R = 0.0;
                for (size_t i = a; i < b; ++i) {
                    const DevObj& o = cs.wobjs[i];
                    if (o.kind == OBJ_NEVER) continue;
                    const double dx = o.bc[0] - C[0], dy = o.bc[1] - C[1], dz = o.bc[2] - C[2];
                    R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz) + o.br);
                }
                const double mag = std::fabs(C[0]) + std::fabs(C[1]) + std::fabs(C[2]) + R;
                R = R * (1.0 + 1e-7) + 1e-7 * (1.0 + mag);
                float_ball(C, R, rec);
                rec[5] = float_ball_mag(rec);
                type = 2;
            }
            std::memcpy(&rec[4], &type, sizeof(int));
        }
    }

    // Wave-uniform cull groups over runs of consecutive bounded objects.  A run
    // grows while its bounding ball stays within 2x the largest member radius
    // (so it is worth testing) and has at most 8 members; only runs of >= 2
    // members get a header.  Skipping a run is exact: no object in it can
    // report a hit for a lane whose segment misses the bound.
    static std::vector<DevObj> insert_groups(const std::vector<DevObj>& in) {
        std::vector<DevObj> out;
        size_t i = 0;
        while (i < in.size()) {
            if (!in[i].has_bound) { out.push_back(in[i]); ++i; continue; }
            Bound g = ball(in[i].bc[0], in[i].bc[1], in[i].bc[2], in[i].br);
            double rmax = in[i].br;
            size_t j = i + 1;
            while (j < in.size() && in[j].has_bound && j - i < 8) {
                Bound b = ball(in[j].bc[0], in[j].bc[1], in[j].bc[2], in[j].br);
                Bound m = merge_union(g, b);
                const double r2 = std::max(rmax, in[j].br);
                if (m.r > 2.0 * r2) break;
                g = m;
                rmax = r2;
                ++j;
            }
            if (j - i >= 2) {
                DevObj h{};
                h.kind = OBJ_GROUP;
                h.m = (int)(j - i);
                h.has_bound = 1;
                const double mag = std::fabs(g.c[0]) + std::fabs(g.c[1]) + std::fabs(g.c[2]) + g.r;
                for (int k = 0; k < 3; ++k) h.bc[k] = g.c[k];
                h.br = g.r * (1.0 + 1e-7) + 1e-7 * (1.0 + mag);
                float_ball(g.c, g.r, h.fb);
                out.push_back(h);
            }
            for (size_t k = i; k < j; ++k) out.push_back(in[k]);
            i = j;
        }
        return out;
    }

private:
    const rt_scene_desc& d_;
    std::vector<DevOp>* ops_ = nullptr;
    std::vector<float>* gb_ = nullptr;
    int rdepth_ = 0, idepth_ = 0, max_r_ = 0, max_i_ = 0;

    DevOp& op(int code, int node, int top) {
        DevOp o{};
        o.op = code;
        o.node = node;
        o.top = top;
        ops_->push_back(o);
        return ops_->back();
    }
    void ray_push() { ++rdepth_; max_r_ = std::max(max_r_, rdepth_); }
    void ivl_push() { ++idepth_; max_i_ = std::max(max_i_, idepth_); }
};

}  // namespace

namespace {
// doubles of [-1, 1] in order <-> integers (sign-magnitude to two's order)
int64_t dkey(double x) {
    int64_t i;
    std::memcpy(&i, &x, sizeof i);
    return i >= 0 ? i : -(i & INT64_MAX);
}
double dval(int64_t k) {
    const int64_t i = k >= 0 ? k : ((-k) | INT64_MIN);
    double x;
    std::memcpy(&x, &i, sizeof x);
    return x;
}
// least x in [-1, 1] with pred(x), pred monotone (false ... false true ... true)
template <class P>
double least_true(P pred) {
    int64_t lo = dkey(-1.0), hi = dkey(1.0);
    if (!pred(dval(hi))) return 2.0;
    if (pred(dval(lo))) return -1.0;
    while (hi - lo > 1) {   // pred(lo) false, pred(hi) true
        const int64_t mid = lo + (hi - lo) / 2;
        (pred(dval(mid)) ? hi : lo) = mid;
    }
    return dval(hi);
}
}  // namespace

void pokeball_thresholds(double btn_outer, double ring_width, double& xb, double& xi) {
    const double inner = std::max(0.0, btn_outer - ring_width);
    xb = least_true([&](double x) { return std::acos(x) <= btn_outer; });
    // greatest x with acos(x) >= inner = (least x with acos(x) < inner) - 1 ulp
    const double lt = least_true([&](double x) { return std::acos(x) < inner; });
    xi = lt == 2.0 ? 1.0 : lt == -1.0 ? -2.0 : dval(dkey(lt) - 1);
}

CompiledScene compile_scene(const rt_scene_desc& d) {
    Compiler c(d);
    return c.run();
}

}  // namespace rtamd

// rt_test.h: the pokeball acos thresholds (CPU)
extern "C" int rt_test_pokeball_thresholds(double btn_outer, double ring_width, double* out2) {
    if (!out2) return -1;
    rtamd::pokeball_thresholds(btn_outer, ring_width, out2[0], out2[1]);
    return 0;
}
