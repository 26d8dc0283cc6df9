// rt_render.hip — gfx950 render kernels and the librtamd C-ABI.
//
// Standard mode (Tracer::render, tracer.cpp:282-300):
//   k_std: one lane per (pixel, sample); a wave covers 4x2 pixels x 8 samples,
//   a 256-thread block 8x4 pixels.  Samples are summed in order s = 0..7
//   across the 8 lanes of a pixel (cross-lane shuffles), then x 1/8.
// Paper mode (tracer.cpp:258-281):
//   k_paper_primary: one lane per pixel: the primary intersect (shared by
//   trace_paper, the centre probe and the four neighbour probes of
//   get_edge_strength, which all re-trace identical rays) + shading.
//   k_paper_finish: edge strength from the stored neighbour hits + hatch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "mt_jump.hpp"
#include "mt_poly.hpp"
#include "rt.h"
#include "rt_device.hpp"
#include "rt_internal.hpp"
#include "scene_compile.hpp"

using namespace rtd;

namespace {

constexpr int kCounterWords = 2 + 16;   // isect, occl, ops[16]
constexpr int kCounterSlots = 512;      // spread of the per-block counter atomics
constexpr int kJitterKMax = 1024;       // twist blocks per jitter segment, upper bound
constexpr int kJitterKMin = 64;

// Segment length for a jitter job.  A segment is regenerated serially by one
// workgroup (latency ~ K twist blocks, ~0.6 us each); a checkpoint costs one
// GF(2) jump (a ~10k-tap correlation over 20k words in LDS).  Aim at a few
// hundred segments for the words the job needs: enough workgroups to fill
// the chip, few enough that the jumps stay cheap (measured with
// tools/sim_ranks.py on config 4: 1024 for a 4K frame, 256-512 for a
// 1/8-frame rank; small frames get short segments).  RT_JITTER_K overrides
// (diagnostics).
int jitter_k(int64_t words_needed) {
    static const int env_k = [] {
        const char* e = std::getenv("RT_JITTER_K");
        return e ? std::atoi(e) : 0;
    }();
    if (env_k > 0) return env_k;
    int K = kJitterKMax;
    while (K > kJitterKMin && words_needed / (624 * 128) < K) K >>= 1;
    return K;
}

struct StdParams {
    int W, H;
    int n_rows;
    const int32_t* rows;
    const int32_t* jrow;   // jitter row of every listed row
    const double* jit;     // 16 draws per pixel: (dx, dy) of samples 0..7
    double* fb;
    unsigned long long* counters;
};

// Ray / op counters: wave reduction by shuffles, block reduction through LDS,
// then one atomic per block and counter into one of kCounterSlots slots
// (blockIdx-hashed).  A single hot address would serialize ~2M atomics at the
// L2 (~6 ns each, MI355X_MICROARCH.md fan-in row) - 12 ms per 4K frame.
template <bool C>
__device__ __forceinline__ void flush_counters(unsigned long long* ctr, uint32_t ni, uint32_t no, Cnt<C>& cnt) {
    constexpr int NW = C ? 18 : 2;
    __shared__ unsigned long long red[4][NW];
    unsigned long long v[NW];
    v[0] = ni;
    v[1] = no;
    if constexpr (C) {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[2 + k] = cnt.c[k];
    }
#pragma unroll
    for (int k = 0; k < NW; ++k)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NW; ++k) red[wave][k] = v[k];
    __syncthreads();
    if (threadIdx.x < NW) {
        const unsigned long long sum = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                       red[3][threadIdx.x];
        const unsigned slot = (blockIdx.x + blockIdx.y * gridDim.x) % kCounterSlots;
        if (sum) atomicAdd(&ctr[(size_t)slot * kCounterWords + threadIdx.x], sum);
    }
}

// Occupancy target of the lean variants (E = D = SEC = false): 4 waves/SIMD
// caps them at 128 VGPRs; the few values the compiler then spills are
// long-lived (stored once, reloaded once), and the extra wave per SIMD hides
// FP64 latency (measured 21.6 -> 19.2 ms on config 4; 5 and 6 are slower).
#ifndef RT_LEAN_WAVES
#define RT_LEAN_WAVES 4
#endif

template <bool E, bool D, bool SEC, bool C, bool DL = true>
__device__ __forceinline__ void std_body(const DevScene& S, const StdParams& P) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int s = lane & 7;
    const int pix = lane >> 3;
    const int x = blockIdx.x * 8 + (wave & 1) * 4 + (pix & 3);
    const int ri = blockIdx.y * 4 + (wave >> 1) * 2 + (pix >> 2);
    const bool active = x < P.W && ri < P.n_rows;
    uint32_t ni = 0, no = 0;
    Cnt<C> cnt;
    V3 c = v3(0.0, 0.0, 0.0);
    if (active) {
        const int r = P.rows[ri];
        const int y = P.H - 1 - r;   // loop row (tracer.cpp:297 writes row ny-1-y)
        // draws 16p+2s, 16p+2s+1 of the stream: dx, dy (tracer.cpp:293)
        const double2 j = *reinterpret_cast<const double2*>(P.jit + ((size_t)P.jrow[ri] * P.W + x) * 16 + 2 * s);
        const DRay ray = gen_ray_subpixel(S, x, y, j.x, j.y);
        c = trace<E, D, SEC, DL>(S, ray, ni, no, cnt);
    }
    // acc += trace(...) for s = 0..7 in order (tracer.cpp:290-296)
    const int base = lane & ~7;
    V3 acc = v3(0.0, 0.0, 0.0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const double cx = __shfl(c.x, base + k);
        const double cy = __shfl(c.y, base + k);
        const double cz = __shfl(c.z, base + k);
        acc.x += cx;
        acc.y += cy;
        acc.z += cz;
    }
    if (active && s == 0) {
        const double inv = 1.0 / (double)8;
        double* o = P.fb + ((size_t)ri * P.W + x) * 3;
        o[0] = acc.x * inv;
        o[1] = acc.y * inv;
        o[2] = acc.z * inv;
    }
    flush_counters(P.counters, ni, no, cnt);
}

template <bool E, bool D, bool SEC, bool C>
__global__ __launch_bounds__(256) void k_std(DevScene S, StdParams P) {
    std_body<E, D, SEC, C>(S, P);
}

template <bool C>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_LEAN_WAVES))) void k_std_lean(DevScene S,
                                                                                                       StdParams P) {
    std_body<false, false, false, C, false>(S, P);
}

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
    int* hit;                    // [n_ext*W]
    int* mat;
    double* t;
    double* nx;
    double* ny;
    double* nz;
    double* lum;
    double* fb;
    unsigned long long* counters;
};

template <bool E, bool D, bool C, bool DL = true>
__device__ __forceinline__ void paper_primary_body(const DevScene& S, const PaperParams& P) {
    // block 16x16 pixels, wave 8x8
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int li = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const bool active = x < P.W && li < P.n_list;
    uint32_t ni = 0, no = 0;
    Cnt<C> cnt;
    if (active) {
        const int ei = P.ext_list[li];
        const int y = P.ext_rows[ei];
        const DRay r = gen_ray(S, x, y);
        double ht = 0.0;
        DHit h;
        ++ni;
        const bool hits = scene_intersect<E, D>(S, r, 1e-4, RT_INF, ht, h, cnt);
        const size_t idx = (size_t)ei * P.W + x;
        P.hit[idx] = hits ? 1 : 0;
        P.t[idx] = ht;
        P.nx[idx] = h.n.x;
        P.ny[idx] = h.n.y;
        P.nz[idx] = h.n.z;
        P.mat[idx] = hits ? h.mat : -3;
        if (P.ext_shade[ei]) {
            // trace_paper (tracer.cpp:111-120) + get_luminance (:123-125)
            V3 base = v3(1.0, 1.0, 1.0);
            if (hits) base = shade<E, D, DL>(S, ht, h, normalized(vneg(r.d)), no, cnt);
            P.lum[idx] = 0.299 * base.x + 0.587 * base.y + 0.114 * base.z;
        }
    }
    flush_counters(P.counters, ni, no, cnt);
}

template <bool E, bool D, bool C>
__global__ __launch_bounds__(256) void k_paper_primary(DevScene S, PaperParams P) {
    paper_primary_body<E, D, C>(S, P);
}

template <bool C>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_LEAN_WAVES))) void k_paper_primary_lean(
    DevScene S, PaperParams P) {
    paper_primary_body<false, false, C, false>(S, P);
}

// apply_crosshatch (tracer.cpp:188-205); C++ '%' truncation toward zero.
__device__ __forceinline__ double crosshatch(double lum, int x, int y) {
    if (lum < 0.15) return 0.0;
    const double darkness = 1.0 - lum;
    const bool diag1 = ((x + y) % 4) < 1;
    const bool diag2 = ((x - y) % 4) < 1;
    const bool horizontal = (y % 4) < 1;
    bool draw = false;
    if (darkness > 0.8) draw = (diag1 && diag2) || horizontal;
    else if (darkness > 0.65) draw = (diag1 && diag2) || (horizontal && ((x + y) % 3 == 0));
    else if (darkness > 0.5) draw = (diag1 && diag2) || (horizontal && ((x + y) % 4 == 0));
    else if (darkness > 0.35) draw = diag1 || (horizontal && ((x + y) % 3 == 0));
    else if (darkness > 0.2) draw = diag1;
    else if (darkness > 0.12) draw = diag1 && ((x + y) % 8) < 2;
    return draw ? 0.0 : 1.0;
}

__global__ __launch_bounds__(256) void k_paper_finish(PaperParams P) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int ri = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= P.W || ri >= P.n_rows) return;
    const int y = P.rows[ri];
    const int e_up = P.nbr[3 * ri + 0], e_c = P.nbr[3 * ri + 1], e_dn = P.nbr[3 * ri + 2];
    const size_t ci = (size_t)e_c * P.W + x;
    const bool ch = P.hit[ci] != 0;
    const double ct = P.t[ci];
    const V3 cn = v3(P.nx[ci], P.ny[ci], P.nz[ci]);
    const int cm = P.mat[ci];
    // get_edge_strength (tracer.cpp:133-178): neighbours (-1,0) (1,0) (0,-1) (0,1)
    double maxEdge = 0.0;
    int valid = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int dx = (i == 0) ? -1 : (i == 1) ? 1 : 0;
        const int dy = (i == 2) ? -1 : (i == 3) ? 1 : 0;
        const int nxp = x + dx, nyp = y + dy;
        if (nxp < 0 || nxp >= P.W || nyp < 0 || nyp >= P.H) continue;
        ++valid;
        const int er = (dy < 0) ? e_up : (dy > 0) ? e_dn : e_c;
        const size_t ni = (size_t)er * P.W + nxp;
        const bool nh = P.hit[ni] != 0;
        if (ch != nh) {
            maxEdge = dmax(maxEdge, 0.9);
            continue;
        }
        if (ch && nh) {
            const double nt = P.t[ni];
            const double minD = dmin(ct, nt), maxD = dmax(ct, nt);
            if (minD > 1e-4 && maxD / minD > 3.0) maxEdge = dmax(maxEdge, 0.6);
            const double nd = dot3(cn, v3(P.nx[ni], P.ny[ni], P.nz[ni]));
            if (nd < 0.2) maxEdge = dmax(maxEdge, 0.5);
            if (cm != P.mat[ni] && nd < 0.7) maxEdge = dmax(maxEdge, 0.3);
        }
    }
    if (valid < 4) maxEdge *= 0.5;
    const double edge = maxEdge;
    V3 o;
    if (edge > 0.8) {
        o = v3(0.0, 0.0, 0.0);
    } else if (edge > 0.5) {
        o = v3(0.2, 0.2, 0.2);
    } else {
        const double h = crosshatch(P.lum[ci], x, y);
        o = v3(h, h, h);
        if (edge > 0.3) {
            const double darken = (edge - 0.3) * 0.4;
            o.x *= (1.0 - darken);
            o.y *= (1.0 - darken);
            o.z *= (1.0 - darken);
        }
    }
    double* dst = P.fb + ((size_t)ri * P.W + x) * 3;
    dst[0] = o.x;
    dst[1] = o.y;
    dst[2] = o.z;
}

__global__ void k_scatter_rows(const double* __restrict__ src, const int32_t* __restrict__ rows, int n_rows, int W,
                               double* __restrict__ dst) {
    const size_t row_len = (size_t)W * 3;
    const size_t total = row_len * n_rows;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / row_len, k = i - r * row_len;
        const int32_t d = rows[r];
        if (d >= 0) dst[(size_t)d * row_len + k] = src[i];
    }
}

__global__ void k_to_rgb8(const double* __restrict__ fb, size_t n, uint8_t* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double v = fb[i];
        double c = (v < 1.0) ? v : 1.0;   // std::min(1.0, v)
        c = (0.0 < c) ? c : 0.0;          // std::max(0.0, .)
        out[i] = (uint8_t)(int)round(c * 255.0);   // round half away from zero (core.h:316)
    }
}

// Kernel variants: E = scene has eager (transform-inside-CSG) objects,
// D = some compact CSG needs an interval stack deeper than 2 (not a left-deep
// fold), SEC = reflection/refraction frames needed, C = op counting.  Eager
// scenes always use D.  Each variant gets its own register allocation.
template <bool E, bool D, bool SEC>
void launch_std_c(bool c, dim3 grid, hipStream_t st, const DevScene& S, const StdParams& P) {
    if (c) hipLaunchKernelGGL((k_std<E, D, SEC, true>), grid, dim3(256), 0, st, S, P);
    else hipLaunchKernelGGL((k_std<E, D, SEC, false>), grid, dim3(256), 0, st, S, P);
}
void launch_std(bool e, bool d, bool sec, bool c, dim3 grid, hipStream_t st, const DevScene& S, const StdParams& P) {
    if (e) {
        if (sec) launch_std_c<true, true, true>(c, grid, st, S, P);
        else launch_std_c<true, true, false>(c, grid, st, S, P);
    } else if (d) {
        if (sec) launch_std_c<false, true, true>(c, grid, st, S, P);
        else launch_std_c<false, true, false>(c, grid, st, S, P);
    } else {
        if (sec) launch_std_c<false, false, true>(c, grid, st, S, P);
        else if (c) hipLaunchKernelGGL((k_std_lean<true>), grid, dim3(256), 0, st, S, P);
        else hipLaunchKernelGGL((k_std_lean<false>), grid, dim3(256), 0, st, S, P);
    }
}
template <bool E, bool D>
void launch_paper_c(bool c, dim3 grid, hipStream_t st, const DevScene& S, const PaperParams& P) {
    if (c) hipLaunchKernelGGL((k_paper_primary<E, D, true>), grid, dim3(256), 0, st, S, P);
    else hipLaunchKernelGGL((k_paper_primary<E, D, false>), grid, dim3(256), 0, st, S, P);
}
void launch_paper(bool e, bool d, bool c, dim3 grid, hipStream_t st, const DevScene& S, const PaperParams& P) {
    if (e) launch_paper_c<true, true>(c, grid, st, S, P);
    else if (d) launch_paper_c<false, true>(c, grid, st, S, P);
    else if (c) hipLaunchKernelGGL((k_paper_primary_lean<true>), grid, dim3(256), 0, st, S, P);
    else hipLaunchKernelGGL((k_paper_primary_lean<false>), grid, dim3(256), 0, st, S, P);
}

// ------------------------------------------------------------ host side
#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) {                                                                  \
            rtamd::set_last_error(std::string(#expr) + " failed: " + hipGetErrorString(e_));     \
            return RT_ERR_HIP;                                                                   \
        }                                                                                        \
    } while (0)

// Growable device buffer.
struct DBuf {
    void* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        size_t want = bytes + bytes / 8 + 256;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) n = want;
        return e;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

// Per-device workspace (one render at a time per device; guarded by a mutex).
struct Workspace {
    std::mutex mu;
    DBuf nodes, mats, lights, dlights, objs, ops, gb;
    DBuf rows, jit, ckpt, jscratch, counters;
    DBuf paper_i, paper_d, paper_aux, fb;
    std::map<int, rtamd::JitterPlan> jplan;   // per segment length K
    rtamd::JitterJob jjob;
    std::vector<rtamd::JRange> jranges;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    std::vector<hipEvent_t> tev;   // one per rt_frame_trace call of the open frame (pool)
};

Workspace& workspace(int dev) {
    static std::mutex gm;
    static std::vector<Workspace*> ws;
    std::lock_guard<std::mutex> lk(gm);
    if ((int)ws.size() <= dev) ws.resize(dev + 1, nullptr);
    if (!ws[dev]) ws[dev] = new Workspace;
    return *ws[dev];
}

template <class T>
hipError_t upload(DBuf& b, const std::vector<T>& v, hipStream_t st) {
    size_t bytes = v.size() * sizeof(T);
    hipError_t e = b.ensure(bytes ? bytes : 16);
    if (e != hipSuccess || !bytes) return e;
    return hipMemcpyAsync(b.p, v.data(), bytes, hipMemcpyHostToDevice, st);
}

}  // namespace

// One frame in flight on one device (rt_frame_begin .. rt_frame_end).  Holds
// the device workspace lock for its lifetime; every launch is stream-ordered
// on `st`, and every host buffer an async upload reads stays alive here
// until rt_frame_end has synchronised the stream.
struct rt_frame {
    Workspace* ws = nullptr;
    std::unique_lock<std::mutex> lock;
    hipStream_t st = nullptr;
    DevScene S;
    int W = 0, H = 0, mode = 0, n_rows = 0;
    bool eager = false, deep = false, secondary = false, count_ops = false;
    bool traced = false;
    std::vector<int32_t> rows;
    std::vector<int32_t> rows_jrow;            // standard mode: rows | jitter row of each
    std::chrono::steady_clock::time_point t_start;
    uint64_t logical_isect = 0;
    // paper mode: ext = rendered rows and their vertical neighbours
    int n_ext = 0;
    std::vector<int32_t> ext_pos;              // output row -> ext index (-1: none)
    std::vector<char> ext_done;                // primary hit already launched
    int list_used = 0;                         // ext-list entries consumed in the aux buffer
    int n_tev = 0;                             // trace events recorded (ws.tev[0 .. n_tev))
    hipStream_t last_st = nullptr;             // stream of the previous trace call
    std::vector<std::vector<int32_t>> stage;   // host sources of async uploads
    rtamd::CompiledScene cs;
    std::vector<rt_node> nodes;
    std::vector<rt_material> mats;
    std::vector<rt_light> lights;
    std::vector<rt_dir_light> dlights;
};

namespace {

int frame_begin(const rt_scene* s, int W, int H, int mode, int flags, const int32_t* rows_host, int n_rows,
                hipStream_t st, rt_frame** out) {
    const auto t_start = std::chrono::steady_clock::now();
    if (!out) { rtamd::set_last_error("rt_frame_begin: out is NULL"); return RT_ERR_INVALID_ARG; }
    *out = nullptr;
    if (!s) { rtamd::set_last_error("rt_render: scene is NULL"); return RT_ERR_INVALID_ARG; }
    if (W <= 0 || H <= 0) { rtamd::set_last_error("rt_render: W and H must be > 0"); return RT_ERR_INVALID_ARG; }
    if (mode != RT_MODE_STANDARD && mode != RT_MODE_PAPER) { rtamd::set_last_error("rt_render: bad mode"); return RT_ERR_INVALID_ARG; }
    if (n_rows < 0 || (n_rows > 0 && !rows_host)) { rtamd::set_last_error("rt_render: bad rows"); return RT_ERR_INVALID_ARG; }
    {
        std::vector<char> seen(H, 0);
        for (int i = 0; i < n_rows; ++i) {
            if (rows_host[i] < 0 || rows_host[i] >= H) { rtamd::set_last_error("rt_render: row out of range"); return RT_ERR_INVALID_ARG; }
            if (seen[rows_host[i]]++) { rtamd::set_last_error("rt_render: duplicate row"); return RT_ERR_INVALID_ARG; }
        }
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        rtamd::set_last_error("rt_render: no HIP device available");
        return RT_ERR_NO_DEVICE;
    }
    const rt_scene_desc& d = *rt_scene_get_desc(s);
    rtamd::CompiledScene cs;
    try {
        cs = rtamd::compile_scene(d);
    } catch (const std::exception& e) {
        rtamd::set_last_error(std::string("scene compile: ") + e.what());
        return RT_ERR_INVALID_ARG;
    }
    if (cs.max_ray_depth > kMaxRayStack || cs.max_ivl_depth > kMaxIvlSpill + 2) {
        rtamd::set_last_error("scene nesting exceeds the device stacks (transforms <= 8, CSG operand depth <= 8)");
        return RT_ERR_UNSUPPORTED;
    }
    bool secondary = false;
    for (int i = 0; i < d.n_materials; ++i)
        if (d.materials[i].kr > 0.0 || d.materials[i].kt > 0.0) secondary = true;
    if (d.recursion_limit < 2) secondary = false;   // depth < limit-1 never holds (tracer.cpp:38,51)
    if (secondary && mode == RT_MODE_STANDARD && d.recursion_limit - 1 > kMaxDepth) {
        rtamd::set_last_error("medium.recursion exceeds the device frame stack (17)");
        return RT_ERR_UNSUPPORTED;
    }
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::unique_ptr<rt_frame> f(new rt_frame);
    f->ws = &workspace(dev);
    f->lock = std::unique_lock<std::mutex>(f->ws->mu);
    Workspace& ws = *f->ws;
    f->st = st;
    f->W = W;
    f->H = H;
    f->mode = mode;
    f->n_rows = n_rows;
    f->eager = cs.has_eager;
    // the lean kernels carry no directional-light code: such scenes take the
    // general (D) variants
    f->deep = cs.max_ivl_depth > 2 || d.n_dir_lights > 0;
    f->secondary = secondary;
    f->count_ops = (flags & RT_FLAG_COUNT_OPS) != 0;
    f->rows.assign(rows_host, rows_host + n_rows);
    f->t_start = t_start;
    if (!ws.ev[0])
        for (int i = 0; i < 4; ++i) HIP_TRY(hipEventCreate(&ws.ev[i]));

    // --- upload the scene (a few KB; the frame keeps the host copies alive)
    f->nodes.assign(d.nodes, d.nodes + d.n_nodes);
    f->mats.assign(d.materials, d.materials + d.n_materials);
    f->lights.assign(d.lights, d.lights + d.n_lights);
    f->dlights.assign(d.dir_lights, d.dir_lights + d.n_dir_lights);
    f->cs = std::move(cs);
    HIP_TRY(upload(ws.nodes, f->nodes, st));
    HIP_TRY(upload(ws.mats, f->mats, st));
    HIP_TRY(upload(ws.lights, f->lights, st));
    HIP_TRY(upload(ws.dlights, f->dlights, st));
    HIP_TRY(upload(ws.objs, f->cs.objs, st));
    HIP_TRY(upload(ws.ops, f->cs.ops, st));
    HIP_TRY(upload(ws.gb, f->cs.gbounds, st));
    const size_t ctr_bytes = (size_t)kCounterSlots * kCounterWords * sizeof(unsigned long long);
    HIP_TRY(ws.counters.ensure(ctr_bytes));
    HIP_TRY(hipMemsetAsync(ws.counters.p, 0, ctr_bytes, st));

    DevScene& S = f->S;
    S.nodes = ws.nodes.as<rt_node>();
    S.mats = ws.mats.as<rt_material>();
    S.lights = ws.lights.as<rt_light>();
    S.dlights = ws.dlights.as<rt_dir_light>();
    S.n_dlights = d.n_dir_lights;
    S.objs = ws.objs.as<DevObj>();
    S.ops = ws.ops.as<DevOp>();
    S.gb = ws.gb.as<float>();
    S.n_lights = d.n_lights;
    S.n_objs = (int)f->cs.objs.size();
    S.cam_nx = rt_camera_width(&d.camera);
    S.cam_ny = rt_camera_height(&d.camera);
    S.rec_limit = d.recursion_limit;
    S.cull = (flags & RT_FLAG_NO_CULL) ? 0 : 1;
    for (int i = 0; i < 3; ++i) {
        S.eye[i] = d.camera.eye[i];
        S.P[i] = d.camera.P[i];
        S.bg[i] = d.background[i];
        S.amb[i] = d.ambient[i];
    }
    S.Lx = d.camera.Lx;
    S.Ly = d.camera.Ly;
    S.medium_index = d.medium_index;

    HIP_TRY(hipEventRecord(ws.ev[0], st));
    if (n_rows > 0 && mode == RT_MODE_STANDARD) {
        // Loop row y = H-1-rows[ri] consumes outputs [32Wy, 32W(y+1))
        // (tracer.cpp:284-293).  Jitter rows are laid out in stream order
        // (jrow = rank of y), so runs of consecutive loop rows - a strip, or
        // the whole frame - are one range for the generator.
        const int64_t row_q = (int64_t)32 * W;
        std::vector<int32_t> order(n_rows);
        for (int ri = 0; ri < n_rows; ++ri) order[ri] = ri;
        std::sort(order.begin(), order.end(), [&](int a, int b) { return f->rows[a] > f->rows[b]; });
        f->rows_jrow.assign(f->rows.begin(), f->rows.end());
        f->rows_jrow.resize(2 * (size_t)n_rows);
        ws.jranges.clear();
        for (int k = 0; k < n_rows; ++k) {
            const int ri = order[k];
            f->rows_jrow[n_rows + ri] = k;
            const int64_t y = H - 1 - f->rows[ri];
            if (!ws.jranges.empty() && ws.jranges.back().qb == row_q * y)
                ws.jranges.back().qb += row_q;
            else
                ws.jranges.push_back(rtamd::JRange{row_q * y, row_q * (y + 1), (int64_t)k * 16 * W});
        }
        const int64_t q1 = ws.jranges.back().qb;
        const int K = jitter_k(row_q * n_rows);
        rtamd::JitterPlan& plan = ws.jplan[K];
        const int levels = rtamd::mt_levels_needed(K, q1);
        if (plan.K != K || plan.levels < levels) {
            try {
                HIP_TRY(plan.build(K, levels));
            } catch (const std::exception& ex) {
                rtamd::set_last_error(std::string("jitter plan: ") + ex.what());
                return RT_ERR_PROCESSING;
            }
        }
        HIP_TRY(ws.ckpt.ensure(rtamd::mt_ckpt_words(K, q1) * sizeof(uint32_t)));
        HIP_TRY(ws.jit.ensure((size_t)n_rows * 16 * W * sizeof(double)));
        HIP_TRY(ws.jscratch.ensure(rtamd::mt_scratch_bytes(K, ws.jranges)));
        HIP_TRY(upload(ws.rows, f->rows_jrow, st));
        HIP_TRY(rtamd::mt_launch_jitter(plan, ws.jranges, ws.jjob, ws.jscratch.p, ws.ckpt.as<uint32_t>(),
                                        ws.jit.as<double>(), st));
    } else if (n_rows > 0) {
        // rows needing a primary hit: rendered rows and their vertical neighbours
        std::vector<char> need(H, 0), shade_row(H, 0);
        for (int r : f->rows) {
            need[r] = 1;
            shade_row[r] = 1;
            if (r > 0) need[r - 1] = 1;
            if (r + 1 < H) need[r + 1] = 1;
        }
        std::vector<int32_t> ext, ext_shade;
        f->ext_pos.assign(H, -1);
        for (int r = 0; r < H; ++r)
            if (need[r]) {
                f->ext_pos[r] = (int)ext.size();
                ext.push_back(r);
                ext_shade.push_back(shade_row[r]);
            }
        std::vector<int32_t> nbr(3 * (size_t)n_rows);
        for (int i = 0; i < n_rows; ++i) {
            const int r = f->rows[i];
            nbr[3 * i + 0] = r > 0 ? f->ext_pos[r - 1] : -1;
            nbr[3 * i + 1] = f->ext_pos[r];
            nbr[3 * i + 2] = r + 1 < H ? f->ext_pos[r + 1] : -1;
            // logical Scene::intersect calls: trace_paper + centre + valid neighbours
            f->logical_isect += (uint64_t)W * 2 + (uint64_t)(W > 1 ? 2 * (W - 1) : 0) +
                                (uint64_t)W * ((r > 0) + (r + 1 < H));
        }
        f->n_ext = (int)ext.size();
        f->ext_done.assign(f->n_ext, 0);
        // aux: ext_rows | ext_shade | nbr | rows | ext lists (n_ext, filled per trace call)
        f->stage.emplace_back();
        std::vector<int32_t>& ints = f->stage.back();
        ints.insert(ints.end(), ext.begin(), ext.end());
        ints.insert(ints.end(), ext_shade.begin(), ext_shade.end());
        ints.insert(ints.end(), nbr.begin(), nbr.end());
        ints.insert(ints.end(), f->rows.begin(), f->rows.end());
        HIP_TRY(ws.paper_aux.ensure((ints.size() + f->n_ext) * sizeof(int32_t)));
        HIP_TRY(hipMemcpyAsync(ws.paper_aux.p, ints.data(), ints.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
        const size_t npx = (size_t)f->n_ext * W;
        HIP_TRY(ws.paper_i.ensure(npx * 2 * sizeof(int)));
        HIP_TRY(ws.paper_d.ensure(npx * 5 * sizeof(double)));
    }
    HIP_TRY(hipEventRecord(ws.ev[1], st));
    *out = f.release();
    return RT_OK;
}

int frame_trace(rt_frame* f, int ri0, int ri1, double* fb, hipStream_t hs) {
    if (!f) { rtamd::set_last_error("rt_frame_trace: frame is NULL"); return RT_ERR_INVALID_ARG; }
    if (ri0 < 0 || ri1 < ri0 || ri1 > f->n_rows) { rtamd::set_last_error("rt_frame_trace: bad row range"); return RT_ERR_INVALID_ARG; }
    if (ri1 == ri0) return RT_OK;
    if (!fb) { rtamd::set_last_error("rt_frame_trace: fb is NULL"); return RT_ERR_INVALID_ARG; }
    Workspace& ws = *f->ws;
    const hipStream_t st = hs ? hs : f->st;
    const int W = f->W, n = ri1 - ri0;
    unsigned long long* ctr = ws.counters.as<unsigned long long>();
    // another stream first waits for the scene upload and jitter (begin); in
    // paper mode a chunk also reads primary hits an earlier chunk computed,
    // so chunks on different streams are chained
    if (st != f->st) HIP_TRY(hipStreamWaitEvent(st, ws.ev[1], 0));
    if (f->mode == RT_MODE_PAPER && f->n_tev > 0 && f->last_st != st)
        HIP_TRY(hipStreamWaitEvent(st, ws.tev[f->n_tev - 1], 0));
    if (f->mode == RT_MODE_STANDARD) {
        StdParams P;
        P.W = W;
        P.H = f->H;
        P.n_rows = n;
        P.rows = ws.rows.as<int32_t>() + ri0;
        P.jrow = ws.rows.as<int32_t>() + f->n_rows + ri0;
        P.jit = ws.jit.as<double>();
        P.fb = fb;
        P.counters = ctr;
        dim3 grid((W + 7) / 8, (n + 3) / 4);
        launch_std(f->eager, f->deep, f->secondary, f->count_ops, grid, st, f->S, P);
        HIP_TRY(hipGetLastError());
    } else {
        // primary hits of the ext rows this chunk reads that no earlier chunk computed
        std::vector<int32_t> list;
        for (int i = ri0; i < ri1; ++i) {
            const int r = f->rows[i];
            for (int rr = r - 1; rr <= r + 1; ++rr) {
                if (rr < 0 || rr >= f->H) continue;
                const int e = f->ext_pos[rr];
                if (e >= 0 && !f->ext_done[e]) {
                    f->ext_done[e] = 1;
                    list.push_back(e);
                }
            }
        }
        const int32_t* aux = ws.paper_aux.as<int32_t>();
        const int n_ext = f->n_ext, n_rows = f->n_rows;
        PaperParams P;
        P.W = W;
        P.H = f->H;
        P.n_ext = n_ext;
        P.ext_rows = aux;
        P.ext_shade = aux + n_ext;
        P.nbr = aux + 2 * n_ext + 3 * (size_t)ri0;
        P.rows = aux + 2 * n_ext + 3 * (size_t)n_rows + ri0;
        int32_t* d_list = ws.paper_aux.as<int32_t>() + 2 * n_ext + 4 * (size_t)n_rows + f->list_used;
        P.ext_list = d_list;
        P.n_list = (int)list.size();
        P.n_rows = n;
        const size_t npx = (size_t)n_ext * W;
        P.hit = ws.paper_i.as<int>();
        P.mat = P.hit + npx;
        double* dd = ws.paper_d.as<double>();
        P.t = dd;
        P.nx = dd + npx;
        P.ny = dd + 2 * npx;
        P.nz = dd + 3 * npx;
        P.lum = dd + 4 * npx;
        P.fb = fb;
        P.counters = ctr;
        if (!list.empty()) {
            f->list_used += (int)list.size();
            f->stage.push_back(std::move(list));
            const std::vector<int32_t>& L = f->stage.back();
            HIP_TRY(hipMemcpyAsync(d_list, L.data(), L.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
            dim3 g1((W + 15) / 16, (P.n_list + 15) / 16);
            launch_paper(f->eager, f->deep, f->count_ops, g1, st, f->S, P);
            HIP_TRY(hipGetLastError());
        }
        dim3 g2((W + 63) / 64, (n + 3) / 4);
        hipLaunchKernelGGL(k_paper_finish, g2, dim3(256), 0, st, P);
        HIP_TRY(hipGetLastError());
    }
    if ((int)ws.tev.size() <= f->n_tev) {
        hipEvent_t e = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ws.tev.push_back(e);
    }
    HIP_TRY(hipEventRecord(ws.tev[f->n_tev], st));
    ++f->n_tev;
    f->last_st = st;
    f->traced = true;
    return RT_OK;
}

int frame_end(rt_frame* f, rt_stats* stats) {
    if (!f) { rtamd::set_last_error("rt_frame_end: frame is NULL"); return RT_ERR_INVALID_ARG; }
    std::unique_ptr<rt_frame> own(f);
    Workspace& ws = *f->ws;
    const hipStream_t st = f->st;
    for (int i = 0; i < f->n_tev; ++i) HIP_TRY(hipStreamWaitEvent(st, ws.tev[i], 0));   // join trace streams
    HIP_TRY(hipEventRecord(ws.ev[2], st));
    const size_t ctr_bytes = (size_t)kCounterSlots * kCounterWords * sizeof(unsigned long long);
    std::vector<unsigned long long> slots((size_t)kCounterSlots * kCounterWords);
    HIP_TRY(hipMemcpyAsync(slots.data(), ws.counters.p, ctr_bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    unsigned long long hc[kCounterWords] = {};
    for (int sl = 0; sl < kCounterSlots; ++sl)
        for (int k = 0; k < kCounterWords; ++k) hc[k] += slots[(size_t)sl * kCounterWords + k];
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->rays_intersect = f->mode == RT_MODE_PAPER ? f->logical_isect : hc[0];
        stats->rays_occluded = hc[1];
        stats->rays_traced = hc[0] + hc[1];
        stats->pixels = (uint64_t)f->n_rows * f->W;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, ws.ev[0], ws.ev[1]) == hipSuccess) stats->ms_rng = ms;
        if (hipEventElapsedTime(&ms, ws.ev[1], ws.ev[2]) == hipSuccess) stats->ms_kernel = ms;
        for (int k = 0; k < 16; ++k) stats->ops[k] = hc[2 + k];
        stats->ms_total =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - f->t_start).count();
    }
    return RT_OK;
}

int render_rows_impl(const rt_scene* s, int W, int H, int mode, int flags, const int32_t* rows_host, int n_rows,
                     double* fb_dev, hipStream_t st, rt_stats* stats) {
    if (n_rows > 0 && !fb_dev) { rtamd::set_last_error("rt_render: bad rows/fb"); return RT_ERR_INVALID_ARG; }
    rt_frame* f = nullptr;
    int rc = frame_begin(s, W, H, mode, flags, rows_host, n_rows, st, &f);
    if (rc != RT_OK) return rc;
    rc = frame_trace(f, 0, n_rows, fb_dev, nullptr);
    const int rc2 = frame_end(f, stats);
    return rc != RT_OK ? rc : rc2;
}

}  // namespace

// ------------------------------------------------------------------ C-ABI
extern "C" int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int rt_render_rows_device(const rt_scene* s, int W, int H, int mode, int flags, const int32_t* rows_host,
                                     int n_rows, double* fb_rows_dev, void* hip_stream, rt_stats* stats) {
    return render_rows_impl(s, W, H, mode, flags, rows_host, n_rows, fb_rows_dev, (hipStream_t)hip_stream, stats);
}

extern "C" int rt_frame_begin(const rt_scene* s, int W, int H, int mode, int flags, const int32_t* rows_host,
                              int n_rows, void* hip_stream, rt_frame** out) {
    return frame_begin(s, W, H, mode, flags, rows_host, n_rows, (hipStream_t)hip_stream, out);
}

extern "C" int rt_frame_trace(rt_frame* f, int ri0, int ri1, double* fb_rows_dev, void* hip_stream) {
    return frame_trace(f, ri0, ri1, fb_rows_dev, (hipStream_t)hip_stream);
}

extern "C" int rt_frame_end(rt_frame* f, rt_stats* stats) { return frame_end(f, stats); }

extern "C" int rt_render(const rt_scene* s, int W, int H, int mode, int flags, double* fb_host, rt_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!fb_host) { rtamd::set_last_error("rt_render: fb is NULL"); return RT_ERR_INVALID_ARG; }
    if (W <= 0 || H <= 0) { rtamd::set_last_error("rt_render: W and H must be > 0"); return RT_ERR_INVALID_ARG; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        rtamd::set_last_error("rt_render: no HIP device available");
        return RT_ERR_NO_DEVICE;
    }
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::vector<int32_t> rows(H);
    for (int r = 0; r < H; ++r) rows[r] = r;
    static std::mutex fbm;
    static DBuf fb;
    std::lock_guard<std::mutex> lk(fbm);
    const size_t bytes = (size_t)W * H * 3 * sizeof(double);
    HIP_TRY(fb.ensure(bytes));
    int rc = render_rows_impl(s, W, H, mode, flags, rows.data(), H, fb.as<double>(), nullptr, stats);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipMemcpy(fb_host, fb.p, bytes, hipMemcpyDeviceToHost));
    if (stats)
        stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

extern "C" int rt_scatter_rows_device(const double* src_dev, const int32_t* rows_dev, int n_rows, int W,
                                      double* fb_dev, void* hip_stream) {
    if (n_rows <= 0) return RT_OK;
    if (!src_dev || !rows_dev || !fb_dev || W <= 0) { rtamd::set_last_error("rt_scatter_rows_device: bad args"); return RT_ERR_INVALID_ARG; }
    const size_t total = (size_t)W * 3 * n_rows;
    const unsigned blocks = (unsigned)std::min<size_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(k_scatter_rows, dim3(blocks), dim3(256), 0, (hipStream_t)hip_stream, src_dev, rows_dev, n_rows,
                       W, fb_dev);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

extern "C" int rt_framebuffer_to_rgb8_device(const double* fb_dev, size_t n_pixels, uint8_t* rgb8_dev,
                                             void* hip_stream) {
    if (!n_pixels) return RT_OK;
    if (!fb_dev || !rgb8_dev) { rtamd::set_last_error("rt_framebuffer_to_rgb8_device: NULL"); return RT_ERR_INVALID_ARG; }
    const size_t n = n_pixels * 3;
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_to_rgb8, dim3(blocks), dim3(256), 0, (hipStream_t)hip_stream, fb_dev, n, rgb8_dev);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

// ------------------------------------------------------------- test hooks
#include "rt_test.h"

extern "C" int rt_test_mt_jump_cpu(int K_blocks, int levels) {
    // Every radix-8 tree polynomial x^(624*K*m*8^j) applied to the seed
    // window must equal advancing it m*8^j*K twist blocks sequentially.
    try {
        std::vector<uint32_t> polys = rtamd::mt_tree_polys(K_blocks, levels);
        uint32_t base[624];
        rtamd::mt_first_window(12345u, base);
        int bad = 0;
        for (int j = 0; j < levels; ++j) {
            uint32_t seq[624];
            std::memcpy(seq, base, sizeof(seq));
            const uint64_t step = (uint64_t)K_blocks << (3 * j);
            for (int m = 1; m < rtamd::kMTRadix; ++m) {
                rtamd::mt_advance_blocks_cpu(seq, step);
                uint32_t jumped[624];
                rtamd::mt_apply_jump_cpu(polys.data() + ((size_t)j * 7 + (m - 1)) * 624, base, jumped);
                // bit 31..0 of words 1..623 and the top bit of word 0 define the state
                bool ok = (jumped[0] & 0x80000000u) == (seq[0] & 0x80000000u);
                for (int k = 1; k < 624; ++k) ok = ok && jumped[k] == seq[k];
                if (!ok) ++bad;
            }
        }
        return bad;
    } catch (...) {
        return -1;
    }
}

extern "C" int rt_test_jitter_device(int K, int64_t q0, int64_t q1, int64_t first, int64_t count,
                                     double* out_host) {
    if (K <= 0 || q0 < 0 || q1 <= q0 || (q0 & 1) || (q1 & 1) || !out_host || first * 2 < q0 || (first + count) * 2 > q1)
        return RT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
    rtamd::JitterPlan plan;
    HIP_TRY(plan.build(K, rtamd::mt_levels_needed(K, q1)));
    DBuf dc, dj, ds;
    const std::vector<rtamd::JRange> ranges{rtamd::JRange{q0, q1, 0}};
    rtamd::JitterJob job;
    HIP_TRY(dc.ensure(rtamd::mt_ckpt_words(K, q1) * 4));
    HIP_TRY(dj.ensure((size_t)(q1 - q0) / 2 * sizeof(double)));
    HIP_TRY(ds.ensure(rtamd::mt_scratch_bytes(K, ranges)));
    HIP_TRY(rtamd::mt_launch_jitter(plan, ranges, job, ds.p, dc.as<uint32_t>(), dj.as<double>(), nullptr));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out_host, dj.as<double>() + (first - q0 / 2), (size_t)count * sizeof(double),
                      hipMemcpyDeviceToHost));
    plan.release();
    (void)hipFree(dc.p);
    (void)hipFree(dj.p);
    (void)hipFree(ds.p);
    return RT_OK;
}

extern "C" int rt_test_compile_info(const rt_scene* s, int32_t* out) {
    if (!s || !out) return RT_ERR_INVALID_ARG;
    try {
        const rtamd::CompiledScene cs = rtamd::compile_scene(*rt_scene_get_desc(s));
        int groups = 0, members = 0, ivl_groups = 0, ivl_members = 0;
        for (const auto& o : cs.objs)
            if (o.kind == rtamd::OBJ_GROUP) { ++groups; members += o.m; }
        for (const auto& op : cs.ops)
            if (op.op == rtamd::OP_IVL_GROUP) { ++ivl_groups; ivl_members += op.top / 2; }
        out[0] = (int32_t)cs.objs.size();
        out[1] = groups;
        out[2] = members;
        out[3] = (int32_t)cs.ops.size();
        out[4] = ivl_groups;
        out[5] = ivl_members;
        out[6] = cs.has_eager ? 1 : 0;
        out[7] = cs.max_ivl_depth;
        return RT_OK;
    } catch (const std::exception& e) {
        rtamd::set_last_error(std::string("scene compile: ") + e.what());
        return RT_ERR_INVALID_ARG;
    }
}
