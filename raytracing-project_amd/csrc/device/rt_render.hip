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

#include <cstdio>

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
#include "pinned.hpp"
#include "mt_poly.hpp"
#include "rt.h"
#include "rt_launch.hpp"
#include "rt_internal.hpp"
#include "scene_compile.hpp"

using rtamd::kCounterSlots;
using rtamd::kMaxDepth;
using rtamd::kMaxIvlSpill;
using rtamd::kMaxRayStack;
using rtamd::kCounterWords;
using rtamd::PaperParams;
using rtamd::SceneView;

namespace {
// SceneView::plain: every object a sphere, half-space or pokeball (no
// transform or CSG object: the plain kernels, rt_device.hpp CntPlain)
bool plain_scene(const rtamd::CompiledScene& cs) {
    for (const auto& o : cs.objs)
        if (o.kind != rtamd::OBJ_SPHERE && o.kind != rtamd::OBJ_HALF && o.kind != rtamd::OBJ_POKE &&
            o.kind != rtamd::OBJ_NEVER && o.kind != rtamd::OBJ_GROUP)
            return false;
    return true;
}
}  // namespace
using rtamd::StdParams;

namespace {

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

// The frame's op counters: kCounterSlots x kCounterWords partial sums reduced
// on the device and stored straight into page-locked host memory, so that
// rt_frame_end reads 144 B after one event instead of copying 72 KiB through
// the runtime's pageable staging (which waited ~115 us after the last kernel
// before the copy even started: profiles/r04t_api_timeline.txt).
__global__ void __launch_bounds__(64) k_reduce_counters(unsigned long long* __restrict__ slots,
                                                        unsigned long long* __restrict__ out,
                                                        const unsigned int* __restrict__ gtime, int wpg) {
    // block k < kCounterWords sums word k over the slots (8 independent loads
    // per lane); block kCounterWords + g sums paper-mode list group g's wave
    // times (end - start, mod 2^32) over its wpg waves
    const int k = blockIdx.x, lane = threadIdx.x;
    if (k >= rtamd::kCounterWords) {
        const size_t g = k - rtamd::kCounterWords;
        unsigned v = 0;
        for (int xt = lane; xt < wpg; xt += 64) {
            const unsigned* t = gtime + 2 * (g * wpg + xt);
            v += t[1] - t[0];
        }
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) reinterpret_cast<unsigned int*>(out + rtamd::kCounterWords)[g] = v;
        return;
    }
    // (and leaves the slots zero for the next frame: Workspace::counters_zero)
    unsigned long long v = 0;
#pragma unroll
    for (int sl = lane; sl < rtamd::kCounterSlots; sl += 64) {
        unsigned long long* w = slots + (size_t)sl * rtamd::kCounterWords + k;
        v += *w;
        *w = 0ull;
    }
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) out[k] = v;
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
        rtamd::SetupTimer tm(rtamd::kSetupAlloc);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) n = want;
        return e;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// The device-resident copy of one scene (compiled object table + records in
// the launching precision).  A scene handle is immutable, so the copy is
// keyed by its process-unique id and reused by every later frame of that
// scene on the device: the inputs stay resident in HBM between frames.
struct SceneCache {
    bool valid = false;
    uint64_t uid = 0;
    // Wave BVH on or off, decided per scene by measurement (scenes that have
    // one: > kWaveBvhMin objects).  Exact either way (the BVH kernels equal
    // the flat-list ones bit for bit), so the first frame of a frame shape
    // runs with the BVH, the second without, and later frames take the one
    // whose trace kernels were faster: a scene bound by its closest-hit ties
    // ran 0.85x with the BVH (profiles/r04fin_bvh_perf.txt).
    int bvh_trial = 0;       // 0: next frame tries the BVH, 1: tries without, 2: decided
    float bvh_ms[2] = {0.f, 0.f};
    bool bvh_off = false;
    uint64_t bvh_key = 0;    // frame shape of the trial (W, H, mode, rows, flags)
    bool fp32 = false;
    rtamd::CompiledScene cs;
    std::vector<rt_node> nodes;   // host sources of the uploads (kept alive)
    std::vector<rt_material> mats;
    std::vector<rt_light> lights;
    std::vector<rt_dir_light> dlights;
    std::vector<rtamd::NodeR<float>> nodes_f;
    std::vector<rtamd::MatR<float>> mats_f;
    std::vector<rtamd::LightR<float>> lights_f;
    std::vector<rtamd::DLightR<float>> dlights_f;
    std::vector<rtamd::FoldLeafR<float>> fold_f;
};

// RT_BVH_AB (measurement A/B; default 1): 0 = a scene with a wave BVH always
// uses it (no trial frames, SceneCache::bvh_trial).
bool bvh_ab() {
    static const bool on = [] { const char* e = std::getenv("RT_BVH_AB"); return !(e && *e == '0'); }();
    return on;
}

// Per-device workspace (one render at a time per device; guarded by a mutex).
struct Workspace {
    std::mutex mu;
    DBuf nodes, mats, lights, dlights, objs, ops, gb, ctab, lrec, lwrec, lgb;
    DBuf wobjs, wctab, worig, wchunk;   // wave BVH (CompiledScene::wobjs ...)
    DBuf fold;
    DBuf nodes_f, mats_f, lights_f, dlights_f, fold_f;   // float copies (RT_FLAG_FP32)
    DBuf rows, jit, ckpt, jscratch, counters;
    DBuf paper_i, paper_d, paper_aux, fb;
    rtamd::JitterTable jtab;                  // mt19937(12345) checkpoint table (resident)
    rtamd::JitterJob jjob;
    rtamd::PinnedArena up;                    // page-locked staging of a frame's uploads (pinned.hpp)
    DBuf gtime;                               // paper mode: primary waves' (start, end) ticks (paper_wave_slot)
    unsigned long long* ctr_host = nullptr;   // page-locked: the frame's reduced counters (k_reduce_counters)
    size_t ctr_host_words = 0;                //   + the paper-mode list-group costs behind them
    // paper mode: measured primary-pass cost of each 8-entry list group of a
    // frame, by the group's first ext index, per frame key (scene, size,
    // mode, flags, rows): the next frame of that key launches its groups
    // costliest first (order_paper_groups)
    std::map<uint64_t, std::vector<uint32_t>> paper_cost;
    std::vector<rtamd::JRange> jranges;
    std::vector<int32_t> rows_cached;   // what `rows` holds (a frame with the same rows skips the upload)
    bool counters_zero = false;         // the last frame's k_reduce_counters left `counters` zero (no memset)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    std::vector<hipEvent_t> tev;   // one per rt_frame_trace call of the open frame (pool)
    std::vector<hipEvent_t> pev;   // paper mode: the end of each call's primary pass (pool)
    hipStream_t aux_st = nullptr;  // render_rows_impl: a paper frame's odd chunks
    SceneCache sc;
};

// Workspaces by (device, slot).  Slot 0 is the process's own; the simulated
// ranks of rt_test_dist_threads run on one device concurrently, each on its
// own host thread with its own slot (rtamd::set_workspace_slot), as separate
// processes would hold separate workspaces.  Never deleted (frames hold
// pointers); emptied by rt_shutdown.
std::mutex g_ws_mu;
std::map<std::pair<int, int>, Workspace*> g_ws;
thread_local int t_ws_slot = 0;

Workspace& workspace(int dev) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    Workspace*& w = g_ws[{dev, t_ws_slot}];
    if (!w) w = new Workspace;
    return *w;
}

// One-time setup costs of this process (rt_setup_times): host wall time of
// the scene compile + upload enqueue, the jitter checkpoint-table builds, and
// the first launch of the trace kernels and of the jitter fill (a code
// object is loaded onto the device at its first kernel launch).
struct SetupTimes {
    std::mutex mu;
    double scene_ms = 0.0, jtable_ms = 0.0, trace_launch_ms = 0.0, jitter_launch_ms = 0.0;
    double extra[rtamd::kSetupSlots] = {};   // rtamd::note_setup_ms slots (4..)
    bool trace_launched = false, jitter_launched = false;
};
SetupTimes g_setup;
using SClock = std::chrono::steady_clock;
double ms_since(SClock::time_point t) { return std::chrono::duration<double, std::milli>(SClock::now() - t).count(); }

// rt_render's staging frame (host-output path), one per process
std::mutex g_fb_mu;
DBuf g_fb;
int g_fb_dev = 0;

template <class T>
hipError_t upload(DBuf& b, const std::vector<T>& v, hipStream_t st, rtamd::PinnedArena* up = nullptr) {
    size_t bytes = v.size() * sizeof(T);
    hipError_t e = b.ensure(bytes ? bytes : 16);
    if (e != hipSuccess || !bytes) return e;
    return rtamd::upload_async(up, b.p, v.data(), bytes, st);
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
    SceneView S;
    int W = 0, H = 0, mode = 0, n_rows = 0;
    bool eager = false, deep = false, secondary = false, count_ops = false, fp32 = false;
    bool big = false;                          // big-stack kernels (rtdb)
    bool traced = false;
    bool timed = false;                        // paper mode: a launch stored its waves' ticks (PaperParams::gtime)
    int bvh_trial = -1;                        // SceneCache::bvh_trial this frame measures (-1: none)
    std::vector<int32_t> rows;
    std::vector<int32_t> rows_jrow;            // standard mode: rows | jitter row of each
    std::chrono::steady_clock::time_point t_start;
    uint64_t logical_isect = 0;
    // paper mode: ext = rendered rows and their vertical neighbours
    int n_ext = 0;
    std::vector<int32_t> ext_pos;              // output row -> ext index (-1: none)
    std::vector<int> ext_done;                 // primary hit launched by trace call (value - 1); 0 = not yet
    std::vector<hipStream_t> call_st;          // stream of each trace call
    int list_used = 0;                         // ext-list entries consumed in the aux buffer (a multiple of 16)
    uint64_t key = 0;                          // paper mode: Workspace::paper_cost key
    std::vector<std::pair<int, int>> calls;    // paper mode: (list offset, f->stage index) of each launched list
    int n_tev = 0;                             // trace events recorded (ws.tev[0 .. n_tev))
    hipStream_t last_st = nullptr;             // stream of the previous trace call
    std::vector<std::vector<int32_t>> stage;   // host sources of async uploads
};

namespace {

template <size_t N>
void to_float(float (&dst)[N], const double (&src)[N]) {
    for (size_t i = 0; i < N; ++i) dst[i] = (float)src[i];
}

// Float copies of the scene records for the FP32 kernels (RT_FLAG_FP32).
void make_float_scene(SceneCache& f) {
    f.nodes_f.resize(f.nodes.size());
    for (size_t i = 0; i < f.nodes.size(); ++i) {
        const rt_node& s = f.nodes[i];
        rtamd::NodeR<float>& o = f.nodes_f[i];
        o.kind = s.kind;
        o.a = s.a;
        o.b = s.b;
        o.op = s.op;
        o.mat = s.mat;
        for (int k = 0; k < 5; ++k) o.mats[k] = s.mats[k];
        to_float(o.v, s.v);
        to_float(o.aux, s.aux);
    }
    f.mats_f.resize(f.mats.size());
    for (size_t i = 0; i < f.mats.size(); ++i) {
        const rt_material& s = f.mats[i];
        rtamd::MatR<float>& o = f.mats_f[i];
        to_float(o.albedo, s.albedo);
        to_float(o.ambient, s.ambient);
        o.kd = (float)s.kd;
        o.ks = (float)s.ks;
        o.kr = (float)s.kr;
        o.kt = (float)s.kt;
        o.shininess = (float)s.shininess;
        o.refractive_index = (float)s.refractive_index;
    }
    f.lights_f.resize(f.lights.size());
    for (size_t i = 0; i < f.lights.size(); ++i) {
        to_float(f.lights_f[i].pos, f.lights[i].pos);
        to_float(f.lights_f[i].intensity, f.lights[i].intensity);
    }
    f.dlights_f.resize(f.dlights.size());
    for (size_t i = 0; i < f.dlights.size(); ++i) {
        to_float(f.dlights_f[i].dir, f.dlights[i].dir);
        to_float(f.dlights_f[i].radiance, f.dlights[i].radiance);
    }
    f.fold_f.resize(f.cs.fold.size());
    for (size_t i = 0; i < f.cs.fold.size(); ++i) {
        to_float(f.fold_f[i].c, f.cs.fold[i].c);
        f.fold_f[i].r = (float)f.cs.fold[i].r;
        f.fold_f[i].pc = f.cs.fold[i].pc;
        f.fold_f[i].pad = 0;
    }
}

// Paper mode launch order.  A wave of k_paper_primary covers one 8-entry
// group of the ext list; a group's cost varies ~10x over a frame (sky rows
// against crowded ones, profiles/r04s_strips5.json).  Launched in row order,
// the costly rows of the lower frame start last and their waves form the
// launch's tail: one launch of a rank's rows of an 8-way config-5 frame took
// 0.858 ms in row order, 0.799 ms costliest strips first, 0.994 ms cheapest
// first (profiles/r04y_order5.jsonl).  So every primary wave stores its
// start and end ticks (PaperParams::gtime), rt_frame_end sums them per group
// and keeps them per frame key, and the next frame of that key launches its
// 16-entry blocks (workgroup rows) costliest first.  Measured: one GPU
// 5.37 -> 5.33 ms, the slowest of 8 ranks' trace 0.95 -> 0.93 ms
// (profiles/r04_ab/ab_order.jsonl).  Groups keep their entries (each wave
// stays on 8 consecutive rows of one strip); only the launch order changes,
// which no pixel depends on.  A frame with no history runs in row order.
// primary waves per 8-entry list group (k_paper_primary: 16-column blocks of 2x2 waves)
int paper_waves_per_group(int W) { return 2 * ((W + 15) / 16); }

uint64_t paper_frame_key(uint64_t uid, int W, int H, int mode, int flags, const int32_t* rows, int n_rows) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](uint64_t v) {
        for (int i = 0; i < 8; ++i) {
            h ^= (v >> (8 * i)) & 0xff;
            h *= 1099511628211ull;
        }
    };
    mix(uid);
    mix((uint64_t)(uint32_t)W << 32 | (uint32_t)H);
    mix((uint64_t)(uint32_t)mode << 32 | (uint32_t)flags);
    mix((uint64_t)n_rows);
    for (int i = 0; i < n_rows; ++i) mix((uint64_t)(uint32_t)rows[i]);
    return h;
}

// Reorders the 16-entry blocks of list (one workgroup row: its four waves
// share the workgroup's culls, so a block stays one piece) costliest first
// when every 8-entry group with an entry has a measured cost (else leaves the
// row order); padding blocks go last.
void order_paper_groups(std::vector<int32_t>& list, const std::vector<uint32_t>* cost) {
    if (!cost) return;
    const size_t nb = list.size() / 16;
    std::vector<std::pair<uint64_t, size_t>> key(nb);
    for (size_t b = 0; b < nb; ++b) {
        uint64_t c = 0;
        for (size_t g = 2 * b; g < 2 * b + 2; ++g) {
            int32_t e = -1;
            for (size_t i = 0; i < 8 && e < 0; ++i) e = list[8 * g + i];
            if (e < 0) continue;
            if ((size_t)e >= cost->size() || (*cost)[e] == 0) return;   // not measured: row order
            c += (*cost)[e];
        }
        key[b] = {c, b};
    }
    std::stable_sort(key.begin(), key.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    std::vector<int32_t> out(list.size());
    for (size_t j = 0; j < nb; ++j) std::copy_n(list.begin() + 16 * key[j].second, 16, out.begin() + 16 * j);
    list.swap(out);
}

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
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::unique_ptr<rt_frame> f(new rt_frame);
    f->ws = &workspace(dev);
    f->lock = std::unique_lock<std::mutex>(f->ws->mu);
    // a failure below may leave uploads of this frame queued on st (some read
    // the page-locked staging arena the next frame_begin resets): drain st
    // before the workspace lock goes (destroyed before f)
    struct DrainOnFail {
        hipStream_t st;
        bool armed = true;
        ~DrainOnFail() {
            if (armed) (void)hipStreamSynchronize(st);
        }
    } drain{st};
    Workspace& ws = *f->ws;
    const bool fp32 = (flags & RT_FLAG_FP32) != 0;
    SceneCache& sc = ws.sc;
    ws.up.reset();   // (the previous frame's uploads completed: its rt_frame_end synchronised)
    if (!sc.valid || sc.uid != rtamd::scene_uid(s) || sc.fp32 != fp32) {
        // compile + upload the scene once; later frames of it find it resident
        // (uploads from the page-locked arena: plain DMA, no pageable staging)
        const auto t_sc = SClock::now();
        struct AddTime {
            SClock::time_point t;
            ~AddTime() {
                std::lock_guard<std::mutex> lk(g_setup.mu);
                g_setup.scene_ms += ms_since(t);
            }
        } add_scene_time{t_sc};
        sc.valid = false;
        try {
            sc.cs = rtamd::compile_scene(d);
        } catch (const std::exception& e) {
            rtamd::set_last_error(std::string("scene compile: ") + e.what());
            return RT_ERR_INVALID_ARG;
        }
        sc.nodes.assign(d.nodes, d.nodes + d.n_nodes);
        for (rt_node& n : sc.nodes)   // pick_region's acos thresholds (device copy only)
            if (n.kind == RT_NODE_POKEBALL) rtamd::pokeball_thresholds(n.v[5], n.v[6], n.v[rtamd::kPokeXb], n.v[rtamd::kPokeXi]);
        sc.mats.assign(d.materials, d.materials + d.n_materials);
        // device material table: K_a premultiplied by the scene's I_a (the
        // reference's E_a = mul(m.ambient, scene.ambient), one double product
        // per channel, shading.cpp:39), and one extra slot whose albedo is the
        // background colour (DevScene::bg_mat)
        for (rt_material& m : sc.mats)
            for (int c = 0; c < 3; ++c) m.ambient[c] = m.ambient[c] * d.ambient[c];
        {
            rt_material bgm{};
            for (int c = 0; c < 3; ++c) bgm.albedo[c] = d.background[c];
            sc.mats.push_back(bgm);
        }
        sc.lights.assign(d.lights, d.lights + d.n_lights);
        sc.dlights.assign(d.dir_lights, d.dir_lights + d.n_dir_lights);
        if (fp32) {
            make_float_scene(sc);
            HIP_TRY(upload(ws.nodes_f, sc.nodes_f, st, &ws.up));
            HIP_TRY(upload(ws.mats_f, sc.mats_f, st, &ws.up));
            HIP_TRY(upload(ws.lights_f, sc.lights_f, st, &ws.up));
            HIP_TRY(upload(ws.dlights_f, sc.dlights_f, st, &ws.up));
            HIP_TRY(upload(ws.fold_f, sc.fold_f, st, &ws.up));
        } else {
            HIP_TRY(upload(ws.nodes, sc.nodes, st, &ws.up));
            HIP_TRY(upload(ws.mats, sc.mats, st, &ws.up));
            HIP_TRY(upload(ws.lights, sc.lights, st, &ws.up));
            HIP_TRY(upload(ws.dlights, sc.dlights, st, &ws.up));
            HIP_TRY(upload(ws.fold, sc.cs.fold, st, &ws.up));
        }
        HIP_TRY(upload(ws.objs, sc.cs.objs, st, &ws.up));
        HIP_TRY(upload(ws.ops, sc.cs.ops, st, &ws.up));
        HIP_TRY(upload(ws.gb, sc.cs.gbounds, st, &ws.up));
        HIP_TRY(upload(ws.ctab, sc.cs.ctab, st, &ws.up));
        HIP_TRY(upload(ws.lrec, sc.cs.lrec, st, &ws.up));
        HIP_TRY(upload(ws.lwrec, sc.cs.lwrec, st, &ws.up));
        HIP_TRY(upload(ws.lgb, sc.cs.lgb, st, &ws.up));
        HIP_TRY(upload(ws.wobjs, sc.cs.wobjs, st, &ws.up));
        HIP_TRY(upload(ws.wctab, sc.cs.wctab, st, &ws.up));
        HIP_TRY(upload(ws.worig, sc.cs.worig, st, &ws.up));
        HIP_TRY(upload(ws.wchunk, sc.cs.wchunk, st, &ws.up));
        sc.uid = rtamd::scene_uid(s);
        sc.fp32 = fp32;
        sc.valid = true;
        sc.bvh_trial = 0;   // (a new scene: its own BVH trial)
        sc.bvh_key = 0;
    }
    const rtamd::CompiledScene& cs = sc.cs;
    bool secondary = false;
    for (int i = 0; i < d.n_materials; ++i)
        if (d.materials[i].kr > 0.0 || d.materials[i].kt > 0.0) secondary = true;
    if (d.recursion_limit < 2) secondary = false;   // depth < limit-1 never holds (tracer.cpp:38,51)
    // Stack tiers: the common kernels, else the big-stack build (rtdb), else refuse.
    const int frames = (secondary && mode == RT_MODE_STANDARD) ? d.recursion_limit - 1 : 0;
    bool big = false;
    if (cs.max_ray_depth > kMaxRayStack || cs.max_ivl_depth > kMaxIvlSpill + 2 || frames > kMaxDepth) {
        if (cs.max_ray_depth > rtamd::kBigRayStack || cs.max_ivl_depth > rtamd::kBigIvlSpill + 2 ||
            frames > rtamd::kBigDepth) {
            rtamd::set_last_error("scene exceeds the device stacks: transform nesting inside CSG operands " +
                                  std::to_string(cs.max_ray_depth) + " (max " + std::to_string(rtamd::kBigRayStack) +
                                  "), CSG operand depth " + std::to_string(cs.max_ivl_depth) + " (max " +
                                  std::to_string(rtamd::kBigIvlSpill + 2) + "), medium.recursion " +
                                  std::to_string(d.recursion_limit) + " with reflection/refraction (max " +
                                  std::to_string(rtamd::kBigDepth + 1) + ")");
            return RT_ERR_UNSUPPORTED;
        }
        if (fp32) {
            rtamd::set_last_error("the FP32 fast path has only the common device stacks; render this scene in FP64");
            return RT_ERR_UNSUPPORTED;
        }
        big = true;
    }
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
    f->fp32 = fp32;
    f->big = big;
    f->rows.assign(rows_host, rows_host + n_rows);
    f->t_start = t_start;
    if (!ws.ev[0]) {
        rtamd::SetupTimer tm(rtamd::kSetupStreams);
        for (int i = 0; i < 4; ++i) HIP_TRY(hipEventCreate(&ws.ev[i]));
    }
    const size_t ctr_bytes = (size_t)kCounterSlots * kCounterWords * sizeof(unsigned long long);
    {
        const void* before = ws.counters.p;
        HIP_TRY(ws.counters.ensure(ctr_bytes));
        if (!ws.counters_zero || ws.counters.p != before) HIP_TRY(hipMemsetAsync(ws.counters.p, 0, ctr_bytes, st));
        ws.counters_zero = false;   // (until this frame's reduction has run)
    }

    SceneView& S = f->S;
    S.nodes = fp32 ? ws.nodes_f.p : ws.nodes.p;
    S.mats = fp32 ? ws.mats_f.p : ws.mats.p;
    S.lights = fp32 ? ws.lights_f.p : ws.lights.p;
    S.dlights = fp32 ? ws.dlights_f.p : ws.dlights.p;
    S.fold = fp32 ? ws.fold_f.p : ws.fold.p;
    S.n_dlights = d.n_dir_lights;
    S.objs = ws.objs.as<rtamd::DevObj>();
    S.ops = ws.ops.as<rtamd::DevOp>();
    S.gb = ws.gb.as<float>();
    S.ctab = ws.ctab.as<float>();
    S.lrec = ws.lrec.as<float>();
    S.lwrec = ws.lwrec.as<float>();
    S.lgb = ws.lgb.as<float>();
    S.n_gb = (int)(sc.cs.gbounds.size() / 4);
    S.wobjs = ws.wobjs.as<rtamd::DevObj>();
    S.wctab = ws.wctab.as<float>();
    S.worig = ws.worig.as<int32_t>();
    S.wchunk = ws.wchunk.as<float>();
    S.n_wobjs = (int)cs.wobjs.size();
    S.n_chunks = (flags & RT_FLAG_NO_BVH) ? 0 : (int)(cs.wchunk.size() / 8);
    f->bvh_trial = -1;
    if (S.n_chunks > 0 && !(flags & (RT_FLAG_NO_CULL | RT_FLAG_FORCE_BVH)) && bvh_ab()) {
        const uint64_t key = ((uint64_t)(uint32_t)W << 40) ^ ((uint64_t)(uint32_t)H << 20) ^ ((uint64_t)n_rows << 2) ^
                             ((uint64_t)mode << 1) ^ ((uint64_t)(uint32_t)flags << 48);
        if (sc.bvh_key != key) {
            sc.bvh_key = key;
            sc.bvh_trial = 0;
        }
        if (sc.bvh_trial < 2) f->bvh_trial = sc.bvh_trial;
        if (sc.bvh_trial == 1 || (sc.bvh_trial == 2 && sc.bvh_off)) S.n_chunks = 0;
    }
    S.n_lights = d.n_lights;
    S.n_objs = (int)cs.objs.size();
    S.n_bounded = 0;
    for (const auto& o : cs.objs)
        if (o.has_bound && o.kind != rtamd::OBJ_GROUP) ++S.n_bounded;
    S.cam_nx = rt_camera_width(&d.camera);
    S.cam_ny = rt_camera_height(&d.camera);
    S.rec_limit = d.recursion_limit;
    S.cull = (flags & RT_FLAG_NO_CULL) ? 0 : 1;
    S.wave_cull = S.cull && S.n_bounded >= rtamd::wave_cull_min();
    {
        static const bool lead_on = [] { const char* e = std::getenv("RT_LEAD"); return !(e && *e == '0'); }();
        S.n_lead = lead_on ? cs.n_lead : 0;   // (RT_LEAD=0: measurement A/B)
        static const bool plain_on = [] { const char* e = std::getenv("RT_PLAIN"); return !(e && *e == '0'); }();
        S.plain = plain_on && plain_scene(cs) ? 1 : 0;   // (RT_PLAIN=0: measurement A/B)
    }
    for (int i = 0; i < 3; ++i) {
        S.eye[i] = d.camera.eye[i];
        S.P[i] = d.camera.P[i];
    }
    S.Lx = d.camera.Lx;
    S.Ly = d.camera.Ly;
    S.medium_index = d.medium_index;
    S.bg_mat = d.n_materials;

    if (n_rows > 0 && mode == RT_MODE_STANDARD) {
        // the checkpoint table must reach the last loop row's stream words
        // (built on the first frame, extended only for a larger frame)
        int max_y = 0;
        for (int i = 0; i < n_rows; ++i) max_y = std::max(max_y, H - 1 - rows_host[i]);
        const int64_t q_end = (int64_t)32 * W * (max_y + 1);
        try {   // (the jump polynomials: file read or GF(2) arithmetic, may throw)
            const int64_t n_need = (q_end - 1) / ((int64_t)rtamd::kTableK * 624) + 1;
            if (n_need > ws.jtab.n_ck) {   // a build or an extension: synchronous
                const auto t_j = SClock::now();
                HIP_TRY(ws.jtab.ensure(n_need, st));
                std::lock_guard<std::mutex> lk(g_setup.mu);
                g_setup.jtable_ms += ms_since(t_j);
            }
        } catch (const std::exception& e) {
            rtamd::set_last_error(std::string("jitter checkpoint table: ") + e.what());
            return RT_ERR_PROCESSING;
        }
    }
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
        HIP_TRY(ws.jit.ensure((size_t)n_rows * 16 * W * sizeof(double)));
        HIP_TRY(ws.jscratch.ensure(rtamd::mt_fill_scratch_bytes(ws.jranges)));
        // (the rows / jitter-row lists of the previous frame of this
        // workspace are still on the device: the same row set skips the copy)
        if (!(ws.rows.p && ws.rows_cached == f->rows_jrow)) {
            HIP_TRY(upload(ws.rows, f->rows_jrow, st, &ws.up));
            ws.rows_cached = f->rows_jrow;
        }
        ws.jjob.up = &ws.up;
        const auto t_l = SClock::now();
        HIP_TRY(rtamd::mt_launch_fill(ws.jtab, ws.jranges, ws.jjob, ws.jscratch.p, ws.jit.as<double>(), st));
        {
            std::lock_guard<std::mutex> lk(g_setup.mu);
            if (!g_setup.jitter_launched) g_setup.jitter_launch_ms = ms_since(t_l);
            g_setup.jitter_launched = true;
        }
        (void)q1;
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
        // (+ the ext lists of the trace calls: every entry once, each run padded
        // by < 8 to a group boundary and each call's list by < 16 to a block)
        HIP_TRY(ws.paper_aux.ensure((ints.size() + 24 * (size_t)f->n_ext) * sizeof(int32_t)));
        f->key = paper_frame_key(rtamd::scene_uid(s), W, H, mode, flags, rows_host, n_rows);
        // primary waves' (start, end) ticks: <= 3 list groups per ext row (the
        // list capacity / 8), 2 * ceil(W / 16) waves per group
        HIP_TRY(ws.gtime.ensure((size_t)3 * f->n_ext * paper_waves_per_group(W) * 2 * sizeof(unsigned)));
        HIP_TRY(rtamd::upload_async(&ws.up, ws.paper_aux.p, ints.data(), ints.size() * sizeof(int32_t), st));
        const size_t npx = (size_t)f->n_ext * W;
        HIP_TRY(ws.paper_i.ensure(npx * sizeof(int)));
        HIP_TRY(ws.paper_d.ensure(npx * 4 * sizeof(double)));
    }
    HIP_TRY(hipEventRecord(ws.ev[1], st));
    drain.armed = false;
    *out = f.release();
    rtamd::note_setup_ms(rtamd::kLastBegin, ms_since(t_start));
    {
        std::lock_guard<std::mutex> lk(g_setup.mu);
        g_setup.extra[rtamd::kLastTrace] = 0.0;   // (this frame's trace calls add to it)
    }
    return RT_OK;
}

// fb: FP64 rows; codes (paper mode, FP64 kernels only): one paper_code byte
// per pixel instead (rtamd::frame_trace_paper_codes).
int frame_trace(rt_frame* f, int ri0, int ri1, double* fb, hipStream_t hs, uint8_t* codes = nullptr) {
    if (!f) { rtamd::set_last_error("rt_frame_trace: frame is NULL"); return RT_ERR_INVALID_ARG; }
    if (ri0 < 0 || ri1 < ri0 || ri1 > f->n_rows) { rtamd::set_last_error("rt_frame_trace: bad row range"); return RT_ERR_INVALID_ARG; }
    if (ri1 == ri0) return RT_OK;
    if (!fb && !codes) { rtamd::set_last_error("rt_frame_trace: fb is NULL"); return RT_ERR_INVALID_ARG; }
    if (codes && (f->mode != RT_MODE_PAPER || f->fp32)) {
        rtamd::set_last_error("rt_frame_trace: paper codes need a paper-mode FP64 frame");
        return RT_ERR_INVALID_ARG;
    }
    Workspace& ws = *f->ws;
    const hipStream_t st = hs ? hs : f->st;
    const int W = f->W, n = ri1 - ri0;
    unsigned long long* ctr = ws.counters.as<unsigned long long>();
    // another stream first waits for the scene upload and jitter (begin).  In
    // paper mode a chunk whose finish pass reads primary hits that an earlier
    // call computed on another stream waits for that call's PRIMARY pass
    // (adjacent strips share a neighbour row: one GPU's chunked frame, or
    // adjacent strips of one rank), and only its finish waits: its primary
    // computes new entries only, so it overlaps the earlier call's finish
    // (latency-bound) on the other stream.
    const auto t_launch = SClock::now();
    if (st != f->st) HIP_TRY(hipStreamWaitEvent(st, ws.ev[1], 0));
    std::vector<char> wait;
    if (f->mode == RT_MODE_PAPER && f->n_tev > 0) {
        wait.assign(f->n_tev, 0);
        for (int i = ri0; i < ri1; ++i) {
            const int r = f->rows[i];
            for (int rr = r - 1; rr <= r + 1; ++rr) {
                if (rr < 0 || rr >= f->H) continue;
                const int e = f->ext_pos[rr];
                if (e >= 0 && f->ext_done[e]) {
                    const int c = f->ext_done[e] - 1;   // the call that computed it
                    if (f->call_st[c] != st) wait[c] = 1;
                }
            }
        }
    }
    // paper mode: the ext entries this call marks as its own (ext_done) are
    // unmarked again if the call fails before its event is recorded, so that a
    // later call never waits on an event that was not recorded
    struct Unmark {
        std::vector<int>& done;
        std::vector<int32_t> marked;
        bool keep = false;
        ~Unmark() {
            if (!keep)
                for (int32_t e : marked) done[e] = 0;
        }
    } unmark{f->ext_done, {}};
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
        if (f->fp32) rtf::launch_std(f->eager, f->deep, f->secondary, f->count_ops, st, f->S, P);
        else if (f->big) rtdb::launch_std(true, true, f->secondary, f->count_ops, st, f->S, P);
        else rtd::launch_std(f->eager, f->deep, f->secondary, f->count_ops, st, f->S, P);
        HIP_TRY(hipGetLastError());
    } else {
        // primary hits of the ext rows this chunk reads that no earlier chunk
        // computed.  k_paper_primary's waves are 8 list entries tall: each run
        // of consecutive rows starts on a wave boundary (entries -1 pad), so no
        // wave mixes rows of different strips (the wave-level culls need
        // coherent rays).
        std::vector<int32_t> list;
        int prev_row = -2;
        for (int i = ri0; i < ri1; ++i) {
            const int r = f->rows[i];
            for (int rr = r - 1; rr <= r + 1; ++rr) {
                if (rr < 0 || rr >= f->H) continue;
                const int e = f->ext_pos[rr];
                if (e >= 0 && !f->ext_done[e]) {
                    f->ext_done[e] = f->n_tev + 1;   // (this call's index + 1)
                    unmark.marked.push_back(e);
                    if (rr != prev_row + 1)
                        while (list.size() % 8) list.push_back(-1);
                    list.push_back(e);
                    prev_row = rr;
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
        P.mat = ws.paper_i.as<int>();
        double* dd = ws.paper_d.as<double>();
        P.t = dd;
        P.nx = dd + npx;
        P.ny = dd + 2 * npx;
        P.nz = dd + 3 * npx;
        P.fb = fb;
        P.code = codes;
        P.gtime = nullptr;
        P.counters = ctr;
        if (!list.empty()) {
            while (list.size() % 16) list.push_back(-1);   // whole blocks: the group index is li / 8
            if ((size_t)f->list_used + list.size() > 24 * (size_t)n_ext) {
                rtamd::set_last_error("rt_frame_trace: paper-mode list overflow");
                return RT_ERR_PROCESSING;
            }
            // RT_PAPER_ORDER (measurement A/B): 0 = row order, untimed; 1 = row
            // order, every frame timed; 2 (default) = costliest blocks first,
            // from the wave times of the first frame of the scene and row set
            // (later frames untimed: a timed launch reads the clock ahead of
            // the scene loads, which costs it its scalar loads, k_paper_primary_lean)
            static const int order_mode = [] { const char* e = std::getenv("RT_PAPER_ORDER"); return e && *e ? std::atoi(e) : 2; }();
            const auto cost_it = ws.paper_cost.find(f->key);
            const bool have_cost = cost_it != ws.paper_cost.end();
            if (order_mode >= 2) order_paper_groups(list, have_cost ? &cost_it->second : nullptr);
            P.n_list = (int)list.size();
            if (!f->count_ops && (order_mode == 1 || (order_mode >= 2 && !have_cost))) {
                P.gtime = ws.gtime.as<unsigned>() + (size_t)(f->list_used / 8) * paper_waves_per_group(W) * 2;
                f->timed = true;
            }
            f->calls.emplace_back(f->list_used, (int)f->stage.size());
            f->list_used += (int)list.size();
            f->stage.push_back(std::move(list));
            const std::vector<int32_t>& L = f->stage.back();
            HIP_TRY(rtamd::upload_async(&ws.up, d_list, L.data(), L.size() * sizeof(int32_t), st));
            dim3 g1((W + 15) / 16, (P.n_list + 15) / 16);
            if (f->fp32) rtf::launch_paper(f->eager, f->deep, f->count_ops, g1, st, f->S, P);
            else if (f->big) rtdb::launch_paper(true, true, f->count_ops, g1, st, f->S, P);
            else rtd::launch_paper(f->eager, f->deep, f->count_ops, g1, st, f->S, P);
            HIP_TRY(hipGetLastError());
        }
        if ((int)ws.pev.size() <= f->n_tev) {
            hipEvent_t e = nullptr;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            ws.pev.push_back(e);
        }
        HIP_TRY(hipEventRecord(ws.pev[f->n_tev], st));
        for (size_t c = 0; c < wait.size(); ++c)
            if (wait[c]) HIP_TRY(hipStreamWaitEvent(st, ws.pev[c], 0));
        dim3 g2((W + 63) / 64, (n + 3) / 4);
        if (f->fp32) rtf::launch_paper_finish(g2, st, P);
        else rtd::launch_paper_finish(g2, st, P);
        HIP_TRY(hipGetLastError());
    }
    {
        std::lock_guard<std::mutex> lk(g_setup.mu);
        if (!g_setup.trace_launched) g_setup.trace_launch_ms = ms_since(t_launch);
        g_setup.trace_launched = true;
    }
    if ((int)ws.tev.size() <= f->n_tev) {
        hipEvent_t e = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ws.tev.push_back(e);
    }
    HIP_TRY(hipEventRecord(ws.tev[f->n_tev], st));
    rtamd::note_setup_ms(rtamd::kLastTrace, ms_since(t_launch));
    HIP_TRY(rtamd::warm_copy_engine(st));   // (once per process, while the trace runs)
    unmark.keep = true;
    f->call_st.push_back(st);
    ++f->n_tev;
    f->last_st = st;
    f->traced = true;
    return RT_OK;
}

int frame_end_body(rt_frame* f, rt_stats* stats);

int frame_end(rt_frame* f, rt_stats* stats) {
    if (!f) { rtamd::set_last_error("rt_frame_end: frame is NULL"); return RT_ERR_INVALID_ARG; }
    std::unique_ptr<rt_frame> own(f);   // (holds the workspace lock)
    const auto t_end = SClock::now();
    const int rc = frame_end_body(f, stats);
    rtamd::note_setup_ms(rtamd::kLastEnd, ms_since(t_end));
    if (rc != RT_OK) {
        // an early return left this frame's work queued: drain every stream it
        // used before the lock goes (the next frame_begin resets the
        // page-locked staging its copies read, and reuses its buffers)
        (void)hipStreamSynchronize(f->st);
        for (hipStream_t s : f->call_st) (void)hipStreamSynchronize(s);
    }
    return rc;
}

int frame_end_body(rt_frame* f, rt_stats* stats) {
    Workspace& ws = *f->ws;
    const hipStream_t st = f->st;
    // join the other trace streams: one wait on each one's last call (stream
    // order covers its earlier ones; every wait is a barrier packet on st)
    for (int i = 0; i < f->n_tev; ++i) {
        if (f->call_st[i] == st) continue;
        bool last = true;
        for (int j = i + 1; j < f->n_tev; ++j) last = last && f->call_st[j] != f->call_st[i];
        if (last) HIP_TRY(hipStreamWaitEvent(st, ws.tev[i], 0));
    }
    HIP_TRY(hipEventRecord(ws.ev[2], st));
    const int n_groups = f->list_used / 8;
    const size_t host_words = kCounterWords + ((size_t)n_groups + 1) / 2;
    if (!ws.ctr_host || ws.ctr_host_words < host_words) {
        if (ws.ctr_host) (void)hipHostFree(ws.ctr_host);   // (the previous frame's readback is done)
        ws.ctr_host = nullptr;
        ws.ctr_host_words = 0;
        rtamd::SetupTimer tm(rtamd::kSetupPinned);
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ws.ctr_host), host_words * sizeof(unsigned long long),
                              hipHostMallocDefault));
        ws.ctr_host_words = host_words;
    }
    unsigned long long* ctr = ws.counters.as<unsigned long long>();
    const bool timed = f->timed;   // (some launch of this frame stored its waves' ticks)
    hipLaunchKernelGGL(k_reduce_counters, dim3(kCounterWords + (timed ? n_groups : 0)), dim3(64), 0, st, ctr, ws.ctr_host,
                       ws.gtime.as<unsigned>(), paper_waves_per_group(f->W));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ws.ev[3], st));
    HIP_TRY(rtamd::spin_wait(ws.ev[3]));
    ws.counters_zero = true;
    unsigned long long hc[kCounterWords];
    for (int k = 0; k < kCounterWords; ++k) hc[k] = ((volatile unsigned long long*)ws.ctr_host)[k];
    if (timed) {
        // this frame's group costs, by each group's first ext index
        if (ws.paper_cost.size() >= 64 && !ws.paper_cost.count(f->key)) ws.paper_cost.clear();
        std::vector<uint32_t>& cost = ws.paper_cost[f->key];
        cost.resize(f->n_ext, 0);
        const volatile unsigned int* gc = reinterpret_cast<const volatile unsigned int*>(ws.ctr_host + kCounterWords);
        for (const auto& c : f->calls) {
            const std::vector<int32_t>& L = f->stage[c.second];
            for (size_t g = 0; g < L.size() / 8; ++g) {
                int32_t e = -1;
                for (size_t i = 0; i < 8 && e < 0; ++i) e = L[8 * g + i];
                if (e >= 0) cost[e] = std::max(1u, (unsigned)gc[c.first / 8 + g]);
            }
        }
    }
    if (f->bvh_trial >= 0) {
        // the BVH trial frames: their trace kernels' time decides later frames
        SceneCache& sc = ws.sc;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, ws.ev[1], ws.ev[2]) == hipSuccess && sc.bvh_trial == f->bvh_trial) {
            sc.bvh_ms[f->bvh_trial] = ms;
            if (++sc.bvh_trial == 2) sc.bvh_off = sc.bvh_ms[1] < sc.bvh_ms[0];
        }
    }
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
        stats->n_gpus = 1;
    }
    return RT_OK;
}

int render_rows_impl(const rt_scene* s, int W, int H, int mode, int flags, const int32_t* rows_host, int n_rows,
                     double* fb_dev, hipStream_t st, rt_stats* stats) {
    if (n_rows > 0 && !fb_dev) { rtamd::set_last_error("rt_render: bad rows/fb"); return RT_ERR_INVALID_ARG; }
    rt_frame* f = nullptr;
    int rc = frame_begin(s, W, H, mode, flags, rows_host, n_rows, st, &f);
    if (rc != RT_OK) return rc;
    // paper mode: row chunks alternating between a second stream and the
    // frame's (rtamd::row_chunks), so that each chunk's finish overlaps the
    // next chunk's primary; the last chunk runs on the frame stream
    std::vector<std::pair<int, int>> bounds{{0, n_rows}};
    if (mode == RT_MODE_PAPER && rtamd::paper_chunks_1gpu() > 1) {
        Workspace& ws = *f->ws;
        if (!ws.aux_st && hipStreamCreateWithFlags(&ws.aux_st, hipStreamNonBlocking) != hipSuccess) ws.aux_st = nullptr;
        if (ws.aux_st) bounds = rtamd::row_chunks(n_rows, rtamd::paper_chunks_1gpu(), RT_PAPER_STRIP_ROWS);
    }
    for (size_t k = 0; k < bounds.size() && rc == RT_OK; ++k) {
        const hipStream_t cst = ((bounds.size() - 1 - k) & 1) ? f->ws->aux_st : nullptr;
        rc = frame_trace(f, bounds[k].first, bounds[k].second, fb_dev + (size_t)bounds[k].first * W * 3, cst);
    }
    const int rc2 = frame_end(f, stats);
    return rc != RT_OK ? rc : rc2;
}

}  // namespace

void rtamd::set_workspace_slot(int slot) { t_ws_slot = slot; }

namespace {
// dst <- page-locked host src, 16-byte words (+ a byte tail), read by the GPU over PCIe
__global__ void k_host_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16, int tail) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < tail)
        reinterpret_cast<unsigned char*>(dst + n16)[threadIdx.x] = reinterpret_cast<const unsigned char*>(src + n16)[threadIdx.x];
}
}  // namespace

hipError_t rtamd::host_copy_async(void* dst, const void* src, size_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15)
        return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
    const size_t n16 = n / 16;
    const int tail = (int)(n - n16 * 16);
    const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(1024, (n16 + 255) / 256));
    hipLaunchKernelGGL(k_host_copy, dim3(blocks), dim3(256), 0, st, static_cast<const uint4*>(src),
                       static_cast<uint4*>(dst), n16, tail);
    return hipGetLastError();
}

extern "C" int rt_warmup(int what) {
    if (what & ~(RT_WARM_HOST | RT_WARM_DEVICE)) {
        rtamd::set_last_error("rt_warmup: unknown bits");
        return RT_ERR_INVALID_ARG;
    }
    if (what & RT_WARM_HOST) {
        try {
            rtamd::mt_prefetch_host_taps();
        } catch (const std::exception& e) {
            rtamd::set_last_error(std::string("rt_warmup: ") + e.what());
            return RT_ERR_PROCESSING;
        }
    }
    if (what & RT_WARM_DEVICE) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
            rtamd::set_last_error("rt_warmup: no HIP device available");
            return RT_ERR_NO_DEVICE;
        }
        // the FP64 render kernels' code object (one per fat binary and
        // device, loaded at its first use; hipFuncGetAttributes loads it)
        hipFuncAttributes a{};
        HIP_TRY(hipFuncGetAttributes(&a, rtd::std_kernel(false, false, false, true, false, false)));
    }
    return RT_OK;
}

hipError_t rtamd::warm_copy_engine(hipStream_t st) {
    static std::mutex mu;
    static bool done = false;
    static void* dev = nullptr;
    static std::vector<char> host;
    std::lock_guard<std::mutex> lk(mu);
    if (done) return hipSuccess;
    done = true;   // (one attempt: the copy is an optimisation only)
    // a 1 MiB read-back into pageable memory takes the same runtime path as
    // a frame's read-back (its staging set-up is the ~8 ms first-copy cost);
    // issued behind the first trace launch, the host spends that time while
    // the trace runs (the call returns when the copy has run)
    constexpr size_t kBytes = (size_t)1 << 20;
    rtamd::SetupTimer tm(rtamd::kSetupCopyEngine);
    if (hipMalloc(&dev, kBytes) != hipSuccess) return hipSuccess;
    host.resize(kBytes);
    return hipMemcpyAsync(host.data(), dev, kBytes, hipMemcpyDeviceToHost, st);
}

int rtamd::wave_cull_min() {
    static const int v = [] {
        const char* e = std::getenv("RT_WV_MIN");
        return e && *e ? std::max(1, std::atoi(e)) : 4;
    }();
    return v;
}

void rtamd::note_setup_ms(int slot, double ms) {
    if (slot < 4 || slot >= kSetupSlots) return;
    std::lock_guard<std::mutex> lk(g_setup.mu);
    if (slot < kLastBegin || slot == kLastTrace || slot == kSetupCopyEngine) g_setup.extra[slot] += ms;
    else g_setup.extra[slot] = ms;
}

// Row chunks of a frame or a rank's share (see rt_internal.hpp).
std::vector<std::pair<int, int>> rtamd::row_chunks(int m, int chunks, int S) {
    const int64_t units = (m + S - 1) / S;
    chunks = (int)std::max<int64_t>(1, std::min<int64_t>(chunks, units));
    const int64_t wsum = (int64_t)chunks * (chunks + 1) / 2;
    std::vector<std::pair<int, int>> out;
    int64_t acc = 0;
    for (int k = 0; k < chunks; ++k) {
        const int64_t u0 = acc * units / wsum;
        acc += chunks - k;
        const int64_t u1 = acc * units / wsum;
        const int a = (int)std::min<int64_t>(m, u0 * S), b = (int)std::min<int64_t>(m, u1 * S);
        if (b > a) out.emplace_back(a, b);
    }
    if (out.empty()) out.emplace_back(0, 0);
    return out;
}

// RT_PAPER_CHUNKS_1GPU (measurement A/B; 1 .. 4, default 1): row chunks of a
// paper frame rendered by one GPU, alternating between two streams so that
// chunk k's finish pass overlaps chunk k+1's primary.  Measured on config 5
// (profiles/r05_ab/ab_paper_chunks_1gpu.txt): 1 chunk 5.34 ms, 2 chunks 5.37,
// 4 chunks 5.57 - the chunks' own tails and their separate costliest-first
// orders cost more than the overlapped finish saves - so one launch pair.
int rtamd::paper_chunks_1gpu() {
    static const int c = [] {
        const char* e = std::getenv("RT_PAPER_CHUNKS_1GPU");
        return e && *e ? std::max(1, std::min(4, std::atoi(e))) : 1;
    }();
    return c;
}

int rtamd::release_device_workspaces(int min_slot) {
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) return RT_ERR_NO_DEVICE;
    if (min_slot <= 0) {
        std::lock_guard<std::mutex> lk(g_fb_mu);
        if (g_fb.p) {
            (void)hipSetDevice(g_fb_dev);
            g_fb.release();
        }
    }
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (auto& kv : g_ws) {
        Workspace* w = kv.second;
        const int dev = kv.first.first;
        if (!w || kv.first.second < min_slot) continue;
        std::lock_guard<std::mutex> wl(w->mu);   // waits for an open frame of this device
        (void)hipSetDevice(dev);
        (void)hipDeviceSynchronize();
        for (DBuf* b : {&w->nodes, &w->mats, &w->lights, &w->dlights, &w->objs, &w->ops, &w->gb, &w->ctab, &w->lrec,
                        &w->lwrec, &w->lgb, &w->fold,
                        &w->wobjs, &w->wctab, &w->worig, &w->wchunk,
                        &w->nodes_f, &w->mats_f, &w->lights_f, &w->dlights_f, &w->fold_f, &w->rows, &w->jit, &w->ckpt,
                        &w->jscratch, &w->counters, &w->paper_i, &w->paper_d, &w->paper_aux, &w->fb, &w->gtime})
            b->release();
        w->jtab.release();
        w->rows_cached.clear();
        w->counters_zero = false;
        w->up.release();
        if (w->ctr_host) (void)hipHostFree(w->ctr_host);
        w->ctr_host = nullptr;
        w->ctr_host_words = 0;
        w->paper_cost.clear();
        for (auto& e : w->ev) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
        for (auto& e : w->tev)
            if (e) (void)hipEventDestroy(e);
        w->tev.clear();
        for (auto& e : w->pev)
            if (e) (void)hipEventDestroy(e);
        w->pev.clear();
        if (w->aux_st) (void)hipStreamDestroy(w->aux_st);
        w->aux_st = nullptr;
        w->sc = SceneCache();
    }
    (void)hipSetDevice(prev);
    return RT_OK;
}

// ------------------------------------------------------------------ C-ABI
extern "C" int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int rt_setup_times(double* out, int n) {
    if (!out || n < 0) return RT_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(g_setup.mu);
    const double v[4] = {g_setup.scene_ms, g_setup.jtable_ms, g_setup.trace_launch_ms, g_setup.jitter_launch_ms};
    for (int i = 0; i < n && i < rtamd::kSetupSlots; ++i) out[i] = i < 4 ? v[i] : g_setup.extra[i];
    return RT_OK;
}

extern "C" int rt_set_device(int device) {
    HIP_TRY(hipSetDevice(device));
    return RT_OK;
}

extern "C" int rt_device_alloc(size_t bytes, void** dev_out) {
    if (!dev_out) { rtamd::set_last_error("rt_device_alloc: NULL"); return RT_ERR_INVALID_ARG; }
    *dev_out = nullptr;
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, bytes ? bytes : 1));
    const hipError_t e = hipMemset(p, 0, bytes ? bytes : 1);
    if (e != hipSuccess) {
        (void)hipFree(p);
        rtamd::set_last_error(std::string("rt_device_alloc: hipMemset failed: ") + hipGetErrorString(e));
        return RT_ERR_HIP;
    }
    *dev_out = p;
    return RT_OK;
}

extern "C" int rt_device_free(void* dev) {
    if (dev) HIP_TRY(hipFree(dev));
    return RT_OK;
}

extern "C" int rt_memcpy_h2d(void* dev, const void* host, size_t bytes) {
    if (!bytes) return RT_OK;
    if (!dev || !host) { rtamd::set_last_error("rt_memcpy_h2d: NULL"); return RT_ERR_INVALID_ARG; }
    HIP_TRY(hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice));
    return RT_OK;
}

extern "C" int rt_memcpy_d2h(void* host, const void* dev, size_t bytes) {
    if (!bytes) return RT_OK;
    if (!dev || !host) { rtamd::set_last_error("rt_memcpy_d2h: NULL"); return RT_ERR_INVALID_ARG; }
    HIP_TRY(hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost));
    return RT_OK;
}

extern "C" int rt_device_synchronize(void) {
    HIP_TRY(hipDeviceSynchronize());
    return RT_OK;
}

extern "C" int rt_stream_create(void** stream_out) {
    if (!stream_out) { rtamd::set_last_error("rt_stream_create: NULL"); return RT_ERR_INVALID_ARG; }
    hipStream_t st = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    *stream_out = st;
    return RT_OK;
}

extern "C" int rt_stream_destroy(void* stream) {
    if (stream) HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return RT_OK;
}

extern "C" int rt_host_register(void* host, size_t bytes) {
    if (!host || !bytes) { rtamd::set_last_error("rt_host_register: NULL or empty"); return RT_ERR_INVALID_ARG; }
    HIP_TRY(hipHostRegister(host, bytes, hipHostRegisterDefault));
    return RT_OK;
}

extern "C" int rt_host_unregister(void* host) {
    if (!host) { rtamd::set_last_error("rt_host_unregister: NULL"); return RT_ERR_INVALID_ARG; }
    HIP_TRY(hipHostUnregister(host));
    return RT_OK;
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

int rtamd::frame_trace_paper_codes(rt_frame* f, int ri0, int ri1, uint8_t* codes_rows_dev, void* hip_stream) {
    return frame_trace(f, ri0, ri1, nullptr, (hipStream_t)hip_stream, codes_rows_dev);
}

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
    std::lock_guard<std::mutex> lk(g_fb_mu);
    DBuf& fb = g_fb;
    const size_t bytes = (size_t)W * H * 3 * sizeof(double);
    if (fb.p && g_fb_dev != dev) fb.release();   // (a staging frame lives on one device)
    HIP_TRY(fb.ensure(bytes));
    g_fb_dev = dev;
    int rc = render_rows_impl(s, W, H, mode, flags, rows.data(), H, fb.as<double>(), nullptr, stats);
    if (rc != RT_OK) return rc;
    const auto t1 = std::chrono::steady_clock::now();
    HIP_TRY(hipMemcpy(fb_host, fb.p, bytes, hipMemcpyDeviceToHost));
    if (stats) {
        const auto t2 = std::chrono::steady_clock::now();
        stats->ms_d2h = std::chrono::duration<double, std::milli>(t2 - t1).count();
        stats->ms_total = std::chrono::duration<double, std::milli>(t2 - t0).count();
    }
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

extern "C" int rt_test_paper_order(int32_t* list, int n, const uint32_t* cost, int n_cost) {
    if (n < 0 || n % 16 || (n && !list) || n_cost < 0 || (n_cost && !cost)) return RT_ERR_INVALID_ARG;
    std::vector<int32_t> L(list, list + n);
    const std::vector<uint32_t> c(cost, cost + n_cost);
    order_paper_groups(L, &c);
    std::copy(L.begin(), L.end(), list);
    return RT_OK;
}

extern "C" int rt_test_mt_jump_cpu(int K_blocks, int levels) {
    // Every radix-R tree polynomial x^(624*K*m*R^j) applied to the seed
    // window must equal advancing it m*R^j*K twist blocks sequentially.
    try {
        std::vector<uint32_t> polys = rtamd::mt_tree_polys(K_blocks, levels);
        uint32_t base[624];
        rtamd::mt_first_window(12345u, base);
        int bad = 0;
        for (int j = 0; j < levels; ++j) {
            uint32_t seq[624];
            std::memcpy(seq, base, sizeof(seq));
            const uint64_t step = (uint64_t)K_blocks << (rtamd::kMTRadixBits * j);
            for (int m = 1; m < rtamd::kMTRadix; ++m) {
                rtamd::mt_advance_blocks_cpu(seq, step);
                uint32_t jumped[624];
                rtamd::mt_apply_jump_cpu(polys.data() + ((size_t)j * (rtamd::kMTRadix - 1) + (m - 1)) * 624, base,
                                         jumped);
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

extern "C" int rt_test_mt_poly_file(const char* path, int levels) {
    if (!path || levels <= 0) return RT_ERR_INVALID_ARG;
    try {
        std::vector<uint32_t> from_file;
        if (!rtamd::mt_load_tree_polys(path, rtamd::kTableK, levels, from_file)) return 2;
        return from_file == rtamd::mt_tree_polys_computed(rtamd::kTableK, levels) ? 0 : 1;
    } catch (...) {
        return -1;
    }
}

extern "C" int rt_test_jitter_device(int K, int64_t q0, int64_t q1, int64_t first, int64_t count,
                                     double* out_host) {
    if (K < 0 || q0 < 0 || q1 <= q0 || (q0 & 1) || (q1 & 1) || !out_host || first * 2 < q0 || (first + count) * 2 > q1)
        return RT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
    if (K == 0) {   // the frame path: checkpoint table + one-wave fill
        rtamd::JitterTable T;
        HIP_TRY(T.ensure((q1 - 1) / ((int64_t)rtamd::kTableK * 624) + 1, nullptr));
        DBuf dj, ds;
        const std::vector<rtamd::JRange> ranges{rtamd::JRange{q0, q1, 0}};
        rtamd::JitterJob job;
        HIP_TRY(dj.ensure((size_t)(q1 - q0) / 2 * sizeof(double)));
        HIP_TRY(ds.ensure(rtamd::mt_fill_scratch_bytes(ranges)));
        HIP_TRY(rtamd::mt_launch_fill(T, ranges, job, ds.p, dj.as<double>(), nullptr));
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemcpy(out_host, dj.as<double>() + (first - q0 / 2), (size_t)count * sizeof(double),
                          hipMemcpyDeviceToHost));
        T.release();
        (void)hipFree(dj.p);
        (void)hipFree(ds.p);
        return RT_OK;
    }
    rtamd::JitterPlan plan;
    HIP_TRY(plan.build(K, rtamd::mt_levels_needed(K, q1), nullptr));
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

extern "C" int rt_test_kernel_name(const rt_scene* s, int mode, int flags, char* out, int cap) {
    if (!s || !out || cap <= 0) return RT_ERR_INVALID_ARG;
    try {
        const rt_scene_desc& d = *rt_scene_get_desc(s);
        const rtamd::CompiledScene cs = rtamd::compile_scene(d);
        bool secondary = false;
        for (int i = 0; i < d.n_materials; ++i)
            if (d.materials[i].kr > 0.0 || d.materials[i].kt > 0.0) secondary = true;
        if (d.recursion_limit < 2) secondary = false;
        const bool eager = cs.has_eager;
        const bool deep = eager || cs.max_ivl_depth > 2 || d.n_dir_lights > 0;
        int n_bounded = 0;
        for (const auto& o : cs.objs)
            if (o.has_bound && o.kind != rtamd::OBJ_GROUP) ++n_bounded;
        const bool f32 = (flags & RT_FLAG_FP32) != 0;
        const bool wv = !(flags & RT_FLAG_NO_CULL) && n_bounded >= rtamd::wave_cull_min();
        const bool bv = wv && !cs.wchunk.empty() && !(flags & RT_FLAG_NO_BVH);
        const bool cnt = (flags & RT_FLAG_COUNT_OPS) != 0;
        const int frames = (secondary && mode == RT_MODE_STANDARD) ? d.recursion_limit - 1 : 0;
        const bool big = !f32 && (cs.max_ray_depth > kMaxRayStack || cs.max_ivl_depth > kMaxIvlSpill + 2 ||
                                  frames > kMaxDepth);
        const char* ns = big ? "rtdb" : f32 ? "rtf" : "rtd";
        auto tf = [](bool b) { return b ? "true" : "false"; };
        // (the plain variants: FP64 only, never op-counting)
        const bool pl = !big && !f32 && !cnt && plain_scene(cs) && [] {
            const char* e = std::getenv("RT_PLAIN");
            return !(e && *e == '0');
        }();
        std::string name;
        if (mode == RT_MODE_PAPER) {
            if (!big && !eager && !deep)
                name = std::string("k_paper_primary_lean<") + tf(cnt) + ", " + (bv ? "2" : wv ? "1" : "0") + ", false, " +
                       tf(pl) + ">";
            else
                name = std::string("k_paper_primary<") + tf(big || eager) + ", " + tf(big || deep) + ", " + tf(cnt) + ">";
        } else if (!big && !eager && !deep && !secondary) {
            name = std::string("k_std_lean<") + tf(cnt) + ", " + (bv ? "2" : wv ? "1" : "0") + ", " + tf(pl) + ">";
        } else if (!big && !eager && !deep && wv) {   // (secondary here)
            name = std::string("k_std_secw<") + tf(cnt) + ", " + (bv ? "2" : "1") + ", " + tf(pl) + ">";
        } else {
            name = std::string("k_std<") + tf(big || eager) + ", " + tf(big || deep) + ", " + tf(secondary) + ", " +
                   tf(cnt) + ", false>";
        }
        std::snprintf(out, (size_t)cap, "%s::%s", ns, name.c_str());
        return RT_OK;
    } catch (const std::exception& e) {
        rtamd::set_last_error(std::string("scene compile: ") + e.what());
        return RT_ERR_INVALID_ARG;
    }
}

extern "C" int rt_test_kernel_info(const rt_scene* s, int mode, int flags, int32_t* out) {
    if (!s || !out) return RT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
    try {
        const rt_scene_desc& d = *rt_scene_get_desc(s);
        const rtamd::CompiledScene cs = rtamd::compile_scene(d);
        bool secondary = false;
        for (int i = 0; i < d.n_materials; ++i)
            if (d.materials[i].kr > 0.0 || d.materials[i].kt > 0.0) secondary = true;
        if (d.recursion_limit < 2) secondary = false;
        const bool deep = cs.max_ivl_depth > 2 || d.n_dir_lights > 0;
        int n_bounded = 0;
        for (const auto& o : cs.objs)
            if (o.has_bound && o.kind != rtamd::OBJ_GROUP) ++n_bounded;
        const bool wv = !(flags & RT_FLAG_NO_CULL) && n_bounded >= rtamd::wave_cull_min();
        const bool bv = wv && !cs.has_eager && !deep && !cs.wchunk.empty() && !(flags & RT_FLAG_NO_BVH);
        const bool f32 = (flags & RT_FLAG_FP32) != 0;
        const int frames = (secondary && mode == RT_MODE_STANDARD) ? d.recursion_limit - 1 : 0;
        const bool big = !f32 && (cs.max_ray_depth > kMaxRayStack || cs.max_ivl_depth > kMaxIvlSpill + 2 ||
                                  frames > kMaxDepth);
        const bool pl = plain_scene(cs);
        const void* fn = big ? (mode == RT_MODE_PAPER ? rtdb::paper_kernel(true, true, false, false, false)
                                                      : rtdb::std_kernel(true, true, secondary, false, false, false))
                       : mode == RT_MODE_PAPER
                             ? (f32 ? rtf::paper_kernel(cs.has_eager, deep, wv, bv, pl)
                                    : rtd::paper_kernel(cs.has_eager, deep, wv, bv, pl))
                             : (f32 ? rtf::std_kernel(cs.has_eager, deep, secondary, wv, bv, pl)
                                    : rtd::std_kernel(cs.has_eager, deep, secondary, wv, bv, pl));
        hipFuncAttributes a{};
        HIP_TRY(hipFuncGetAttributes(&a, fn));
        int blocks = 0;
        const bool paper = mode == RT_MODE_PAPER;
        const int threads = big ? rtdb::kernel_block_threads(paper)
                                : f32 ? rtf::kernel_block_threads(paper) : rtd::kernel_block_threads(paper);
        const size_t pool = big ? rtdb::kernel_pool_bytes(paper)
                                : f32 ? rtf::kernel_pool_bytes(paper) : rtd::kernel_pool_bytes(paper);
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, threads, pool));
        out[0] = a.numRegs;                      // VGPRs per lane
        out[1] = (int32_t)a.localSizeBytes;      // scratch (spill) bytes per lane
        out[2] = (int32_t)(a.sharedSizeBytes + pool);   // LDS per workgroup (static + the shading pool)
        out[3] = blocks;                                 // resident workgroups per CU
        out[4] = blocks * (threads / 64) / 4;            // waves per SIMD (4 SIMDs per CU)
        out[5] = a.maxThreadsPerBlock;
        out[6] = wv ? 1 : 0;
        out[7] = secondary ? 1 : 0;
        return RT_OK;
    } catch (const std::exception& e) {
        rtamd::set_last_error(std::string("scene compile: ") + e.what());
        return RT_ERR_INVALID_ARG;
    }
}

extern "C" int rt_test_wave_bvh(const rt_scene* s, int32_t* counts, int32_t* worig, float* wctab, int cap_objs,
                                float* wchunk, int cap_chunks) {
    if (!s || !counts || cap_objs < 0 || cap_chunks < 0) return RT_ERR_INVALID_ARG;
    try {
        const rtamd::CompiledScene cs = rtamd::compile_scene(*rt_scene_get_desc(s));
        const int n = (int)cs.wobjs.size(), nch = (int)(cs.wchunk.size() / 8);
        counts[0] = n;
        counts[1] = nch;
        for (int i = 0; i < std::min(n, cap_objs); ++i) {
            if (worig) worig[i] = cs.worig[i];
            if (wctab) std::memcpy(wctab + 8 * (size_t)i, &cs.wctab[8 * (size_t)i], 8 * sizeof(float));
        }
        if (wchunk) std::memcpy(wchunk, cs.wchunk.data(), (size_t)std::min(nch, cap_chunks) * 8 * sizeof(float));
        return RT_OK;
    } catch (const std::exception& e) {
        rtamd::set_last_error(std::string("scene compile: ") + e.what());
        return RT_ERR_INVALID_ARG;
    }
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
