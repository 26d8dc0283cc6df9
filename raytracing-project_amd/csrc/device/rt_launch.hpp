// rt_launch.hpp — what the host side of librtamd hands to the render kernels.
//
// The kernels exist twice: namespace rtd (FP64, the parity path) and
// namespace rtf (FP32, RT_FLAG_FP32, rt_render_f32.hip).  Both are built from
// rt_device.hpp + rt_kernels.hpp; this header holds the precision-neutral
// launch interface: device pointers, the camera/medium in double, and the
// per-launch parameter blocks.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt.h"
#include "scene_compile.hpp"

namespace rtamd {

// Scene records in a given precision.  The double instances are
// layout-identical to the C-ABI structs of rt.h; the float ones are the
// converted copies the FP32 kernels read.
template <class T>
struct NodeR {
    int32_t kind;
    int32_t a, b;
    int32_t op;
    int32_t mat;
    int32_t mats[5];
    T v[24];
    T aux[4];
};
template <class T>
struct MatR {
    T albedo[3];
    T ambient[3];
    T kd, ks, kr, kt;
    T shininess;
    T refractive_index;
};
template <class T>
struct LightR {
    T pos[3];
    T intensity[3];
};
template <class T>
struct DLightR {
    T dir[3];
    T radiance[3];
};
template <class T>
struct FoldLeafR {   // FoldLeaf (scene_compile.hpp) in the launching precision
    T c[3];
    T r;
    int32_t pc;
    int32_t pad;
};
static_assert(sizeof(FoldLeafR<double>) == sizeof(FoldLeaf), "FoldLeafR<double> must mirror FoldLeaf");
static_assert(sizeof(NodeR<double>) == sizeof(rt_node), "NodeR<double> must mirror rt_node");
static_assert(sizeof(MatR<double>) == sizeof(rt_material), "MatR<double> must mirror rt_material");
static_assert(sizeof(LightR<double>) == sizeof(rt_light), "LightR<double> must mirror rt_light");
static_assert(sizeof(DLightR<double>) == sizeof(rt_dir_light), "DLightR<double> must mirror rt_dir_light");

// Device-resident scene, precision-neutral (records are NodeR/MatR/... of
// the launching precision).
struct SceneView {
    const void* nodes;
    const void* mats;
    const void* lights;
    const void* dlights;
    const DevObj* objs;
    const DevOp* ops;
    const float* gb;
    const float* ctab;   // CompiledScene::ctab
    const float* lrec;   // CompiledScene::lrec / lwrec / lgb: light-relative shadow cull records
    const float* lwrec;
    const float* lgb;
    int n_gb;
    const void* fold;   // FoldLeafR of the launching precision
    // wave BVH (CompiledScene::wobjs, wctab, worig, wchunk); n_chunks = 0: none
    const DevObj* wobjs;
    const float* wctab;
    const int32_t* worig;
    const float* wchunk;
    int n_wobjs, n_chunks;
    int n_lights, n_dlights, n_objs;
    int n_bounded;
    int wave_cull;   // wave-level culls: cull && n_bounded >= wave_cull_min() (host-decided)
    int n_lead;      // CompiledScene::n_lead (0: none / RT_LEAD=0)
    int plain;       // only sphere / half-space / pokeball objects: the plain kernels (CntPlain, rt_device.hpp)
    int cam_nx, cam_ny;
    int rec_limit, cull;
    double eye[3], P[3], Lx, Ly;
    double medium_index;
    int bg_mat;   // the background colour: albedo of material slot bg_mat (appended after the scene's)
};

struct StdParams {
    int W, H;
    int n_rows;
    const int32_t* rows;
    const int32_t* jrow;   // jitter row of every listed row
    const double* jit;     // 16 draws per pixel: (dx, dy) of samples 0..7
    double* fb;
    unsigned long long* counters;
};

struct PaperParams {
    int W, H;
    int n_ext;
    int n_rows;
    int n_list;                  // primary pass: ext indices ext_list[0..n_list) of this launch
    const int32_t* ext_list;
    const int32_t* ext_rows;     // rows needing a primary hit
    const int32_t* ext_shade;    // 1 = row is rendered by this call (shade it)
    const int32_t* nbr;          // per rendered row: ext index of r-1, r, r+1 (-1 = outside frame)
    const int32_t* rows;         // rendered rows
    int* mat;                    // [n_ext*W]: primary hit's material (kPaperMiss for none) | crosshatch band << 24
    double* t;
    double* nx;
    double* ny;
    double* nz;
    double* fb;
    uint8_t* code;               // non-null: k_paper_finish writes paper_code bytes [n_rows*W] instead of fb
    unsigned int* gtime;         // non-null: a timed launch; primary waves store (start, end) wall-clock ticks (paper_wave_slot)
    unsigned long long* counters;
};

// Paper mode's output alphabet (tracer.cpp:258-281): every pixel is grey
// (r = g = b) and a function of the edge strength - the max of the constants
// {0.9, 0.6, 0.5, 0.3} over the neighbour tests, or 0, halved when a
// neighbour lies outside the frame (tracer.cpp:133-178) - and of the hatch
// bit apply_crosshatch returns (tracer.cpp:188-205).  So one byte holds a
// pixel exactly: bits 0-2 the index of the max in {0, 0.3, 0.5, 0.6, 0.9},
// bit 3 the halving, bit 4 the hatch bit (white).  The distributed frame
// gathers these bytes (1 B/px instead of 24) and the root decodes them with
// the reference's own FP64 expression, bit for bit.
__host__ __device__ inline double paper_code_value(unsigned code) {
    const unsigned i = code & 7;
    double edge = i == 1 ? 0.3 : i == 2 ? 0.5 : i == 3 ? 0.6 : i == 4 ? 0.9 : 0.0;
    if (code & 8) edge *= 0.5;
    if (edge > 0.8) return 0.0;
    if (edge > 0.5) return 0.2;
    double o = (code & 16) ? 1.0 : 0.0;
    if (edge > 0.3) {
        const double darken = (edge - 0.3) * 0.4;
        o *= (1.0 - darken);
    }
    return o;
}

// Per-lane stacks of the render kernels (checked on the host per scene).
// The common kernels carry small ones; scenes beyond them run on the
// "big-stack" build of the general kernels (namespace rtdb,
// rt_kernels_big.hip), whose stacks live in scratch memory.
constexpr int kMaxRayStack = 8;   // transform nesting inside CSG operands (eager programs)
constexpr int kMaxIvlSpill = 6;   // CSG interval stack entries beyond the top two
constexpr int kMaxDepth = 16;     // reflection/refraction frames (medium.recursion <= 17)
constexpr int kBigRayStack = 64;
constexpr int kBigIvlSpill = 62;
constexpr int kBigDepth = 128;    // medium.recursion <= 129

// Scenes with at least this many bounded objects take the wave-level culling
// kernels (WV >= 1).  RT_WV_MIN overrides it (measurement A/B; default 4).
int wave_cull_min();

constexpr int kCounterWords = 2 + 16;   // isect, occl, ops[16]
constexpr int kCounterSlots = 512;      // spread of the per-block counter atomics

}  // namespace rtamd

// Kernel variants (rt_kernels.hpp): E = scene has eager (transform-inside-CSG)
// objects, D = general compact CSG (deep stacks, directional lights),
// SEC = reflection/refraction frames, C = op counting, pl = plain scene
// (SceneView::plain: the lean / recursion / paper kernels without transform
// and CSG code).
#define RT_DECLARE_LAUNCHERS(NS)                                                                                  \
    namespace NS {                                                                                                \
    void launch_std(bool e, bool d, bool sec, bool c, hipStream_t st, const rtamd::SceneView& V,                 \
                    const rtamd::StdParams& P);                                                                   \
    void launch_paper(bool e, bool d, bool c, dim3 grid, hipStream_t st, const rtamd::SceneView& V,               \
                      const rtamd::PaperParams& P);                                                               \
    void launch_paper_finish(dim3 grid, hipStream_t st, const rtamd::PaperParams& P);                             \
    const void* std_kernel(bool e, bool d, bool sec, bool wv, bool bv, bool pl);                                  \
    const void* paper_kernel(bool e, bool d, bool wv, bool bv, bool pl);                                          \
    int kernel_block_threads(bool paper);                                                                         \
    size_t kernel_pool_bytes(bool paper);                                                                         \
    }
RT_DECLARE_LAUNCHERS(rtd)
RT_DECLARE_LAUNCHERS(rtf)
RT_DECLARE_LAUNCHERS(rtdb)
