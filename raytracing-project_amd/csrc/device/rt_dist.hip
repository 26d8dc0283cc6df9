// rt_dist.hip — frames on several GPUs and the device output path.
//
// pixels are independent, so a frame is partitioned by OUTPUT
// ROWS: strips of RT_STRIP_ROWS rows (paper mode: RT_PAPER_STRIP_ROWS) are
// dealt to the ranks interleaved (strip_owners: balances cheap sky rows
// against expensive geometry rows).  Every rank runs
// the ordinary trace (rt_frame_* of rt_render.hip) on its rows, chunk by
// chunk, and each chunk is handed to ONE RCCL collective, ncclGather to rank
// 0 over xGMI, on a high-priority stream so it overlaps the tracing of the
// next chunk; rank 0 places the gathered strips into its frame.  Paper-mode
// ranks gather one byte per pixel (the output alphabet, paper_code_value),
// which rank 0 decodes into its FP64 or RGB8 frame.  The jitter
// stream of every row is taken at that row's own stream offset, so the frame
// is bit-identical to a one-GPU render (tracer.cpp:284-299).
//
// toByte (core.h:313-316, main.cpp:19-34) runs on the
// device before the gather, so only 3 bytes per pixel cross xGMI and PCIe on
// the CLI's path.
//
// Two ways in:
//   rt_render_multi / rt_render_rgb8   one process, n devices (ncclCommInitAll,
//                                      one host thread per device)
//   rt_dist_create + rt_render_dist    one process per device (torchrun/MPI)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "rccl_dyn.hpp"   // (RCCL is dlopened on first use: after rccl.h, before any ncclXxx call)

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rt.h"
#include "rt_internal.hpp"
#include "rt_launch.hpp"
#include "rt_test.h"

namespace {

constexpr int kChunks = 4;
// Paper frames gather one code byte per pixel, so their chunks hide little
// transfer, while every chunk adds a launch tail of the costly paper waves:
// 2 chunks project config 5 at 8 ranks 5.21-5.23x -> 5.46-5.56x, at 4 ranks
// 3.04 -> 3.12-3.18x (1: 4.58x, 3: 5.30x; profiles/r06_ab/ab_dist_chunks.txt).
constexpr int kPaperChunks = 2;
constexpr int kSplitSlots = 10;   // rt_dist_frame_split (include/rt.h)   // pipeline units per rank (chunk k gathered while k+1 is traced)

#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) {                                                                  \
            rtamd::set_last_error(std::string(#expr) + " failed: " + hipGetErrorString(e_));     \
            return RT_ERR_HIP;                                                                   \
        }                                                                                        \
    } while (0)

#define NCCL_TRY(expr)                                                                           \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess) {                                                                 \
            rtamd::set_last_error(std::string(#expr) + " failed: " + ncclGetErrorString(r_));    \
            return RT_ERR_HIP;                                                                   \
        }                                                                                        \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        const size_t want = bytes + bytes / 16 + 256;
        rtamd::SetupTimer tm(rtamd::kSetupAlloc);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) n = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

// ------------------------------------------------------------- partition
// Strip height per mode: standard mode RT_STRIP_ROWS (8); paper mode
// RT_PAPER_STRIP_ROWS (30): each strip's primary hits are traced with its two
// neighbour rows (the edge probes, tracer.cpp:133-178), and 30 + 2 = 32 rows
// keep every 8-row wave of k_paper_primary inside one strip (coherent rays
// for the wave-level culls) at 1/15 halo overhead (8-row strips: 1/4 extra
// rows and waves straddling strips 16+ rows apart).
int strip_height(int mode) { return mode == RT_MODE_PAPER ? RT_PAPER_STRIP_ROWS : RT_STRIP_ROWS; }

// Which rank renders strip s.  Interleaved so that every rank samples the
// whole frame (cheap sky rows against expensive geometry rows), by a smooth
// weighted round robin: every strip, each rank's credit grows by its weight
// and the rank with the most credit takes the strip (and pays the total).
//  * Ties go to the rank first in a per-round rotation (round k = strips
//    [k*world, (k+1)*world) starts at rank k mod world), so a rank's strips do
//    not all sit at the same phase of a world*S-row period: config 5's sphere
//    rows have structure on that scale (a plain s mod world split left the
//    slowest of 8 paper-mode ranks 11 % above the mean).
//  * Rank 0 also places every gathered strip into the frame (the FP64 frame:
//    24 B/px written; paper mode decodes one byte per pixel into 24), so it
//    renders fewer strips: weight 1 - c*world (per mille: c = 45 paper, 8
//    standard, 0 for RGB8 output; from per-rank timings, profiles/r04*; the
//    paper value raised 30 -> 45 with the plain paper kernel, whose faster
//    trace left the root's placement the longest leg: 8-rank frame
//    0.726 -> 0.708 ms, profiles/r06_ab/ab_dist_shed_plain.txt).
// The partition is a pure function of (H, world, mode, kind), all of which
// the ranks check against each other before the first gather.
constexpr int kRootShedPaper = 45, kRootShedStd = 8;
// (RT_ROOT_SHED_PAPER / RT_ROOT_SHED_STD: measurement A/B only.  Both values
// travel in the frame descriptor, so ranks that see different ones refuse the
// frame together instead of tracing another partition than the root places.)
int64_t root_shed(int mode) {
    static const int shed_paper = [] { const char* e = std::getenv("RT_ROOT_SHED_PAPER"); return e && *e ? std::atoi(e) : kRootShedPaper; }();
    static const int shed_std = [] { const char* e = std::getenv("RT_ROOT_SHED_STD"); return e && *e ? std::atoi(e) : kRootShedStd; }();
    return mode == RT_MODE_PAPER ? shed_paper : shed_std;
}
std::vector<int> strip_owners(int n_strips, int world, int64_t c) {
    std::vector<int> own((size_t)std::max(0, n_strips), 0);
    if (world <= 1) return own;
    std::vector<int64_t> w((size_t)world, 1000), cur((size_t)world, 0);
    w[0] = std::max<int64_t>(500, 1000 - c * world);
    int64_t total = 0;
    for (int64_t v : w) total += v;
    for (int s = 0; s < n_strips; ++s) {
        for (int r = 0; r < world; ++r) cur[r] += w[r];
        const int rot = (s / world) % world;
        int best = rot;
        for (int i = 1; i < world; ++i) {
            const int r = (rot + i) % world;
            if (cur[r] > cur[best]) best = r;
        }
        own[s] = best;
        cur[best] -= total;
    }
    return own;
}

// Output rows of every rank (ascending per rank), strips of strip_height(mode).
// (A partition balanced on measured strip costs - the strips' summed primary
// wave ticks, exchanged in the trace-status agreement, longest processing
// time first - was measured and rejected: slower at 2 ranks, no better at 4
// and 8, profiles/r05_ab/ab_cost_partition.txt.)
// shed: the root's per-mille shed for this frame (0 for RGB8 output; else
// root_shed(mode), which every rank checks in the frame descriptor).
std::vector<std::vector<int32_t>> partition_rows(int H, int world, int mode, int64_t shed) {
    const int S = strip_height(mode);
    const int n_strips = (H + S - 1) / S;
    std::vector<std::vector<int32_t>> rows((size_t)world);
    const std::vector<int> own = strip_owners(n_strips, world, shed);
    for (int st = 0; st < n_strips; ++st)
        for (int r = st * S; r < std::min(H, (st + 1) * S); ++r) rows[own[st]].push_back(r);
    return rows;
}

uint64_t fnv_bytes(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}

// Content hash of a scene (the IR arrays and camera fields; no padding bytes),
// equal on every rank that loaded the same JSON: part of the frame descriptor
// the ranks check, and of the key their strip costs belong to.
int64_t scene_hash(const rt_scene* s) {
    if (!s) return 0;
    const rt_scene_desc& d = *rt_scene_get_desc(s);
    uint64_t h = 1469598103934665603ull;
    h = fnv_bytes(h, d.camera.eye, sizeof d.camera.eye);
    h = fnv_bytes(h, d.camera.P, sizeof d.camera.P);
    h = fnv_bytes(h, &d.camera.Lx, sizeof(double));
    h = fnv_bytes(h, &d.camera.Ly, sizeof(double));
    h = fnv_bytes(h, &d.camera.dpi, sizeof(int32_t));
    h = fnv_bytes(h, d.background, sizeof d.background);
    h = fnv_bytes(h, d.ambient, sizeof d.ambient);
    h = fnv_bytes(h, &d.medium_index, sizeof(double));
    h = fnv_bytes(h, &d.recursion_limit, sizeof(int32_t));
    h = fnv_bytes(h, d.lights, sizeof(rt_light) * (size_t)d.n_lights);
    h = fnv_bytes(h, d.materials, sizeof(rt_material) * (size_t)d.n_materials);
    h = fnv_bytes(h, d.nodes, sizeof(rt_node) * (size_t)d.n_nodes);
    h = fnv_bytes(h, d.objects, sizeof(int32_t) * (size_t)d.n_objects);
    h = fnv_bytes(h, d.dir_lights, sizeof(rt_dir_light) * (size_t)d.n_dir_lights);
    return (int64_t)(h >> 2);   // (62 bits: v and -v both representable)
}

// Row chunks of a rank's share: rtamd::row_chunks (rt_render.hip), whole
// strips of S rows (a chunk never splits a strip, so a paper-mode strip's
// rows and halo are traced by one launch), of decreasing size (4 chunks:
// 40/30/20/10 %).  Chunk k is gathered while chunk k+1 is traced, so only the
// last, smallest chunk's gather is exposed.
std::vector<std::pair<int, int>> chunk_bounds(int m, int chunks, int S = 1) { return rtamd::row_chunks(m, chunks, S); }

// Gathered slot i (row_bytes bytes) -> row rows[i] of dst; rows[i] < 0 is padding.
template <class V>
__global__ void k_place_rows(const V* __restrict__ src, const int32_t* __restrict__ rows, int n_slots, size_t row_v,
                             V* __restrict__ dst) {
    const size_t total = row_v * (size_t)n_slots;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t slot = i / row_v, k = i - slot * row_v;
        const int32_t d = rows[slot];
        if (d >= 0) dst[(size_t)d * row_v + k] = src[i];
    }
}

hipError_t place_rows(const void* src, const int32_t* rows_dev, int n_slots, size_t row_bytes, void* dst,
                      hipStream_t st) {
    if (n_slots <= 0) return hipSuccess;
    const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
    auto launch = [&](auto tag) {
        using V = decltype(tag);
        const size_t row_v = row_bytes / sizeof(V);
        const size_t total = row_v * (size_t)n_slots;
        const unsigned blocks = (unsigned)std::min<size_t>((total + 255) / 256, 16384);
        hipLaunchKernelGGL(k_place_rows<V>, dim3(blocks), dim3(256), 0, st, static_cast<const V*>(src), rows_dev,
                           n_slots, row_v, static_cast<V*>(dst));
        return hipGetLastError();
    };
    if (row_bytes % 16 == 0 && al % 16 == 0) return launch(uint4{});
    if (row_bytes % 8 == 0 && al % 8 == 0) return launch(uint2{});
    if (row_bytes % 4 == 0 && al % 4 == 0) return launch(uint32_t{});
    return launch(uint8_t{});
}

// Paper-mode distributed frames gather one paper-code byte per pixel
// (rtamd::paper_code_value): gathered slot i (W codes) -> row rows[i] of dst,
// decoded to FP64 RGB (kind 0) or to toByte'd RGB8 (kind 1, core.h:313-316).
template <bool RGB8>
__global__ void k_place_codes(const uint8_t* __restrict__ src, const int32_t* __restrict__ rows, int n_slots, int W,
                              void* __restrict__ dst) {
    const size_t total = (size_t)W * n_slots;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t slot = i / W, x = i - slot * W;
        const int32_t d = rows[slot];
        if (d < 0) continue;
        const double v = rtamd::paper_code_value(src[i]);
        const size_t o = ((size_t)d * W + x) * 3;
        if constexpr (RGB8) {
            double c = (v < 1.0) ? v : 1.0;
            c = (0.0 < c) ? c : 0.0;
            const uint8_t b = (uint8_t)(int)round(c * 255.0);
            uint8_t* q = static_cast<uint8_t*>(dst) + o;
            q[0] = b;
            q[1] = b;
            q[2] = b;
        } else {
            double* q = static_cast<double*>(dst) + o;
            q[0] = v;
            q[1] = v;
            q[2] = v;
        }
    }
}

hipError_t place_codes(const uint8_t* src, const int32_t* rows_dev, int n_slots, int W, int kind, void* dst,
                       hipStream_t st) {
    if (n_slots <= 0) return hipSuccess;
    const size_t total = (size_t)W * n_slots;
    const unsigned blocks = (unsigned)std::min<size_t>((total + 255) / 256, 16384);
    if (kind) hipLaunchKernelGGL(k_place_codes<true>, dim3(blocks), dim3(256), 0, st, src, rows_dev, n_slots, W, dst);
    else hipLaunchKernelGGL(k_place_codes<false>, dim3(blocks), dim3(256), 0, st, src, rows_dev, n_slots, W, dst);
    return hipGetLastError();
}

// ------------------------------------------------------ test transport
// rt_test_dist_threads: the ranks of a distributed frame simulated on ONE
// device, concurrently, one host thread per rank with its own streams and its
// own device workspace (as separate processes would have them).  Their
// collectives keep RCCL's contract - every rank issues the same sequence, and
// each collective is ordered on the rank's collective stream - through host
// rendezvous plus device work on the ranks' own streams:
//   all-reduce (max): each rank records "input ready"; rendezvous (input
//     pointers posted); each rank waits for every input and reduces all of
//     them into a private temporary, records "read"; rendezvous; each rank
//     waits until every rank has read its input, then copies the temporary
//     over its buffer (in place, as the agreement reductions use it).
//   gather: each rank records "send ready"; rendezvous (send pointers
//     posted); the root waits for every send and copies it into its receive
//     buffer, records "copied"; rendezvous; the other ranks' streams wait for
//     "copied" (a send completes once the root holds the data).
// Every device wait refers to an event recorded before the rendezvous that
// publishes it, so no stream can wait on work queued behind it.  A rendezvous
// waits at most the rank's timeout: a rank that times out (a peer that never
// arrives) or aborts marks the group aborted, and its peers see that as the
// communicator's asynchronous error (dist_wait) or at their next rendezvous.
constexpr int kSimMaxWorld = 16;

struct SimGroup {
    explicit SimGroup(int w) : world(w), posted((size_t)w, nullptr), in((size_t)w, nullptr), rd((size_t)w, nullptr) {}
    int world;
    std::mutex mu;
    std::condition_variable cv;
    int count = 0;
    uint64_t gen = 0;
    bool aborted = false;
    std::string why;
    std::vector<const void*> posted;        // one pointer per rank, posted at a collective's first rendezvous
    std::vector<hipEvent_t> in, rd;         // per rank: input / send ready, all-reduce inputs read
    hipEvent_t copied = nullptr;            // the root's gather copies
    // Rendezvous of every rank (post: this rank's pointer, or nullptr at a
    // collective's second rendezvous).  Returns "" or why it failed.
    std::string meet(int rank, const void* post, double timeout_ms, const char* what) {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return "the group was aborted (" + why + ")";
        if (post) posted[rank] = post;
        const uint64_t g = gen;
        if (++count == world) {
            count = 0;
            ++gen;
            cv.notify_all();
            return "";
        }
        const bool done = cv.wait_for(lk, std::chrono::duration<double, std::milli>(timeout_ms),
                                      [&] { return gen != g || aborted; });
        if (gen != g) return "";
        if (!done) {
            aborted = true;
            why = "rank " + std::to_string(rank) + " timed out after " + std::to_string((long)timeout_ms) +
                  " ms waiting for " + what + " (a peer rank did not take part)";
            cv.notify_all();
            return why;
        }
        return "the group was aborted (" + why + ")";
    }
    void abort(const std::string& w) {
        std::lock_guard<std::mutex> lk(mu);
        if (!aborted) why = w;
        aborted = true;
        cv.notify_all();
    }
    bool is_aborted(std::string* w) {
        std::lock_guard<std::mutex> lk(mu);
        if (aborted && w) *w = why;
        return aborted;
    }
};

struct I64Ptrs {
    const int64_t* p[kSimMaxWorld];
};

__global__ void k_sim_max_i64(I64Ptrs in, int world, int n, int64_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t v = in.p[0][i];
    for (int r = 1; r < world; ++r) v = std::max(v, in.p[r][i]);
    out[i] = v;
}

}  // namespace

// One rank of a frame distribution (also the single-device case, world 1).
struct rt_dist {
    int world = 1, rank = 0, device = 0;
    ncclComm_t comm = nullptr;
    bool own_comm = false;
    hipStream_t comm_st = nullptr;            // collectives + placement (high priority)
    hipStream_t alt_st = nullptr;             // odd trace chunks (a chunk's tail overlaps the next chunk)
    DevBuf mine, mine8, stage, rowtab;
    hipEvent_t ev_chunk[kChunks] = {};
    hipEvent_t ev_gs[kChunks] = {}, ev_ge[kChunks] = {};   // each collective + its placement (comm_st)
    hipEvent_t ev_gm[kChunks] = {};           // between each collective and its placement (comm_st)
    hipEvent_t ev_a0 = nullptr, ev_a1 = nullptr;   // around the frame agreement's reduction (comm_st)
    double split[kSplitSlots] = {};           // rt_dist_frame_split: this rank's last collective frame
    hipEvent_t ev_alt = nullptr;              // end of alt_st's work in a frame (joined into st)
    hipEvent_t ev_tb[2 * kChunks] = {};
    std::vector<int32_t> rowtab_host;          // source of the async row-table upload
    std::mutex mu;                            // one frame at a time per rank
    DevBuf* sim_stage = nullptr;              // rt_test_dist_sim_rank: shared stage, copies instead of RCCL
    size_t xchg_cap = 0;                      // int64 slots of xchg / xchg_host
    SimGroup* simg = nullptr;                 // rt_test_dist_threads: concurrent ranks, same-device transport
    DevBuf simtmp;                            //   its all-reduce temporary
    bool force_collective = false;            // rt_test_dist_create_rccl1: world 1 through ncclGather
    DevBuf red;                               // rt_dist_reduce_max scratch
    // Per-frame agreement (collective frames): the frame descriptor + each
    // rank's setup status before the first gather, each rank's trace status
    // before the last one (int64 slots, ncclMax), read back through pinned
    // host memory.
    DevBuf xchg;
    int64_t* xchg_host = nullptr;
    hipEvent_t ev_desc = nullptr;
    bool dead = false;                        // communicator aborted: the handle renders no more frames
    std::string dead_why;
    std::thread abort_th;                     // ncclCommAbort runs here (it can wait for the stream to drain)
    std::atomic<double> abort_ms{-1.0};       //   its duration once done
    double timeout_ms = 120000.0;             // RT_DIST_TIMEOUT_MS / rt_dist_set_timeout
    int inject = 0;                           // rt_test_dist_inject (next frame only)
    int shed_delta = 0;                       // rt_test_dist_threads fault DESC_SHED (next frame only)
    // content hashes by rtamd::scene_uid (process-unique, never reused: a scene
    // loaded after another was destroyed may get its address, never its uid)
    std::map<uint64_t, int64_t> scene_hashes;
    bool collective() const { return world > 1 || force_collective; }
};

namespace {

// A rank's streams and events, created on first need: the collective stream
// only for collective frames, the alternate chunk stream only for frames of
// more than one chunk (a one-GPU frame of the `ray` CLI creates neither: the
// first stream creations of a process cost ~30 ms of setup,
// profiles/r05_cli_split.txt).
int dist_init_events(rt_dist& D) {
    for (auto& e : D.ev_chunk) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : D.ev_tb) HIP_TRY(hipEventCreate(&e));
    for (auto& e : D.ev_gs) HIP_TRY(hipEventCreate(&e));
    for (auto& e : D.ev_gm) HIP_TRY(hipEventCreate(&e));
    for (auto& e : D.ev_ge) HIP_TRY(hipEventCreate(&e));
    HIP_TRY(hipEventCreate(&D.ev_a0));
    HIP_TRY(hipEventCreate(&D.ev_a1));
    HIP_TRY(hipEventCreateWithFlags(&D.ev_desc, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&D.ev_alt, hipEventDisableTiming));
    return RT_OK;
}

int dist_init_streams(rt_dist& D, bool coll, bool alt) {
    rtamd::SetupTimer tm(rtamd::kSetupStreams);
    if (!D.ev_alt) {
        const int re = dist_init_events(D);
        if (re != RT_OK) return re;
    }
    if (coll && !D.comm_st) {
        int lo = 0, hi = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_TRY(hipStreamCreateWithPriority(&D.comm_st, hipStreamNonBlocking, hi));
    }
    if (alt && !D.alt_st) HIP_TRY(hipStreamCreateWithFlags(&D.alt_st, hipStreamNonBlocking));
    return RT_OK;
}

// ------------------------------------------------ frame agreement + waits
// A rank that fails on its own (a launch error, an allocation, a bad frame
// argument) must not leave its peers blocked in a collective it never joins.
// So every rank of a collective frame issues every collective of the frame
// whatever happened locally, and the ranks agree on the outcome through two
// small max-reductions of int64 slots on the collective stream:
//   before the first gather: the frame descriptor (W, H, mode, kind, flags as
//     v and -v: all ranks equal iff max(v) == v and max(-v) == -v) and one
//     setup-failure slot per rank.  The host waits for it while the first
//     chunk traces; on a mismatch or a failure no rank issues a gather;
//   before the last gather: one trace-failure slot per rank (the last chunk
//     traces meanwhile), read back after the frame.
// Waits on the collective stream poll with a deadline and the communicator's
// asynchronous error; on either the communicator is aborted (ncclCommAbort)
// and the handle refuses further frames: a rank whose peer died returns
// RT_ERR_HIP instead of hanging.
// Descriptor: W, H, mode, output kind, flags, the scene's content hash
// (ranks that loaded different scenes refuse the frame together) and the
// root's strip shed of each mode (strip_owners: a rank that saw another
// RT_ROOT_SHED_* value would trace another partition than the root places).
constexpr int kDescFields = 8;

// slots: the agreement 1 descriptor (v, -v) + setup status per rank, then the
// trace status per rank
int dist_init_xchg(rt_dist& D, size_t slots) {
    if (slots <= D.xchg_cap && D.xchg_host) return RT_OK;
    const size_t bytes = slots * sizeof(int64_t);
    HIP_TRY(D.xchg.ensure(bytes));
    if (D.xchg_host) (void)hipHostFree(D.xchg_host);   // (the previous frame's readbacks are done)
    D.xchg_host = nullptr;
    D.xchg_cap = 0;
    rtamd::SetupTimer tm(rtamd::kSetupPinned);
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&D.xchg_host), bytes, hipHostMallocDefault));
    D.xchg_cap = slots;
    return RT_OK;
}



// The communicator is aborted on a helper thread: ncclCommAbort can wait
// for work already queued on the collective stream (a held stream kept it
// 1.9 s, gpurun_out/r04c_dist_tests.log), and the rank must return near its
// deadline, not when its stream drains.  release_rank joins the thread; its
// duration is reported with the handle's later refusals.
void dist_abort(rt_dist& D, const std::string& why) {
    if (D.simg) D.simg->abort("rank " + std::to_string(D.rank) + ": " + why);
    if (D.comm && D.own_comm) {
        if (D.abort_th.joinable()) D.abort_th.join();
        ncclComm_t c = D.comm;
        std::atomic<double>* ms = &D.abort_ms;
        D.abort_th = std::thread([c, ms] {
            const auto t0 = std::chrono::steady_clock::now();
            (void)ncclCommAbort(c);
            ms->store(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        });
    }
    D.comm = nullptr;
    D.own_comm = false;
    D.dead = true;
    D.dead_why = why;
}

std::string abort_note(const rt_dist& D) {
    const double ms = D.abort_ms.load();
    if (!D.abort_th.joinable() && ms < 0) return "";
    char buf[96];
    if (ms < 0) std::snprintf(buf, sizeof buf, "; ncclCommAbort still running");
    else std::snprintf(buf, sizeof buf, "; ncclCommAbort took %.1f ms", ms);
    return buf;
}

int dist_wait(rt_dist& D, hipEvent_t ev, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return RT_OK;
        if (q != hipErrorNotReady) {
            rtamd::set_last_error(std::string("rt_render_dist: ") + what + ": " + hipGetErrorString(q));
            return RT_ERR_HIP;
        }
        if (D.comm) {
            ncclResult_t ae = ncclSuccess;
            if (ncclCommGetAsyncError(D.comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                const std::string why = std::string("RCCL asynchronous error during ") + what + ": " +
                                        ncclGetErrorString(ae);
                dist_abort(D, why);
                rtamd::set_last_error("rt_render_dist: " + why + " (communicator abort started)");
                return RT_ERR_HIP;
            }
        }
        std::string gw;
        if (D.simg && D.simg->is_aborted(&gw)) {
            const std::string why = std::string("the group was aborted during ") + what + " (" + gw + ")";
            dist_abort(D, why);
            rtamd::set_last_error("rt_render_dist: " + why);
            return RT_ERR_HIP;
        }
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms > D.timeout_ms) {
            const std::string why = std::string("timed out after ") + std::to_string((long)D.timeout_ms) +
                                    " ms waiting for " + what + " (a peer rank did not take part)";
            dist_abort(D, why);
            char buf[64];
            std::snprintf(buf, sizeof buf, " (gave up at %.1f ms)", ms);
            rtamd::set_last_error("rt_render_dist: " + why + buf + "; communicator abort started");
            return RT_ERR_HIP;
        }
        if (it < 4096) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// The frame's collectives.  RCCL, or one of the two test stand-ins: the
// concurrent same-device transport (D.simg, rt_test_dist_threads) and the
// one-rank-at-a-time timing stand-in (D.sim_stage, rt_test_dist_sim_rank:
// reductions are the identity, a gather is a copy into the shared stage).
// Each returns "" or why it could not be issued.
std::string coll_max_i64(rt_dist& D, int64_t* buf, size_t n, const char* what) {
    if (D.sim_stage) return "";
    if (D.simg) {
        SimGroup& G = *D.simg;
        const int w = G.world;
        if (D.simtmp.ensure(n * sizeof(int64_t)) != hipSuccess) return "all-reduce temporary allocation failed";
        if (hipEventRecord(G.in[D.rank], D.comm_st) != hipSuccess) return "event record failed";
        std::string e = G.meet(D.rank, buf, D.timeout_ms, what);
        if (!e.empty()) return e;
        I64Ptrs P{};
        for (int r = 0; r < w; ++r) {
            P.p[r] = static_cast<const int64_t*>(G.posted[r]);
            if (r != D.rank && hipStreamWaitEvent(D.comm_st, G.in[r], 0) != hipSuccess) return "stream wait failed";
        }
        hipLaunchKernelGGL(k_sim_max_i64, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, D.comm_st, P, w, (int)n,
                           D.simtmp.as<int64_t>());
        if (hipGetLastError() != hipSuccess || hipEventRecord(G.rd[D.rank], D.comm_st) != hipSuccess)
            return "all-reduce launch failed";
        e = G.meet(D.rank, nullptr, D.timeout_ms, what);
        if (!e.empty()) return e;
        for (int r = 0; r < w; ++r)
            if (r != D.rank && hipStreamWaitEvent(D.comm_st, G.rd[r], 0) != hipSuccess) return "stream wait failed";
        if (hipMemcpyAsync(buf, D.simtmp.p, n * sizeof(int64_t), hipMemcpyDeviceToDevice, D.comm_st) != hipSuccess)
            return "all-reduce copy failed";
        return "";
    }
    const ncclResult_t r = ncclAllReduce(buf, buf, n, ncclInt64, ncclMax, D.comm, D.comm_st);
    return r == ncclSuccess ? "" : std::string("ncclAllReduce failed: ") + ncclGetErrorString(r);
}

// Gather `bytes` from every rank into recv (root only: world * bytes, rank
// order).  bytes_type: the payload is bytes (RGB8 / paper codes), else doubles.
std::string coll_gather(rt_dist& D, const void* send, void* recv, size_t bytes, bool bytes_type, const char* what) {
    if (D.sim_stage) {
        if (hipMemcpyAsync(static_cast<char*>(recv) + (size_t)D.rank * bytes, send, bytes, hipMemcpyDeviceToDevice,
                           D.comm_st) != hipSuccess)
            return "simulated gather copy failed";
        return "";
    }
    if (D.simg) {
        SimGroup& G = *D.simg;
        if (hipEventRecord(G.in[D.rank], D.comm_st) != hipSuccess) return "event record failed";
        std::string e = G.meet(D.rank, send, D.timeout_ms, what);
        if (!e.empty()) return e;
        if (D.rank == 0) {
            for (int r = 0; r < G.world; ++r) {
                if (r != 0 && hipStreamWaitEvent(D.comm_st, G.in[r], 0) != hipSuccess) return "stream wait failed";
                if (bytes && hipMemcpyAsync(static_cast<char*>(recv) + (size_t)r * bytes, G.posted[r], bytes,
                                            hipMemcpyDeviceToDevice, D.comm_st) != hipSuccess)
                    return "gather copy failed";
            }
            if (hipEventRecord(G.copied, D.comm_st) != hipSuccess) return "event record failed";
        }
        e = G.meet(D.rank, nullptr, D.timeout_ms, what);
        if (!e.empty()) return e;
        if (D.rank != 0 && hipStreamWaitEvent(D.comm_st, G.copied, 0) != hipSuccess) return "stream wait failed";
        return "";
    }
    const ncclResult_t r = ncclGather(send, D.rank == 0 ? recv : nullptr, bytes_type ? bytes : bytes / 8,
                                      bytes_type ? ncclUint8 : ncclFloat64, 0, D.comm, D.comm_st);
    return r == ncclSuccess ? "" : std::string("ncclGather failed: ") + ncclGetErrorString(r);
}

// rt_test_dist_inject: a kernel that holds the collective stream for a bounded
// time (every wave leaves after max_ticks of the 100 MHz wall clock), standing
// in for a peer that never arrives.
__global__ void k_test_stall(unsigned long long max_ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < max_ticks) __builtin_amdgcn_s_sleep(127);
}

enum { kInjectTraceFail = 1, kInjectStall = 2, kInjectSetupFail = 3 };

// Row chunks per rank and frame (each one gather): kChunks (paper: kPaperChunks), or
// RT_DIST_CHUNKS (standard mode) / RT_DIST_CHUNKS_PAPER from the environment
// (measurement A/B; 1 .. kChunks).
int frame_chunks(int mode) {
    static const int c[2] = {
        [] { const char* e = std::getenv("RT_DIST_CHUNKS"); return e && *e ? std::atoi(e) : kChunks; }(),
        [] { const char* e = std::getenv("RT_DIST_CHUNKS_PAPER"); return e && *e ? std::atoi(e) : kPaperChunks; }()};
    return std::min(kChunks, std::max(1, c[mode == RT_MODE_PAPER ? 1 : 0]));
}

// RT_DIST_TIMEOUT_MS: how long a rank waits for its peers inside one frame
// before it aborts the communicator (default 120 s).
double env_timeout_ms() {
    const char* e = std::getenv("RT_DIST_TIMEOUT_MS");
    if (e && *e) {
        const double v = std::atof(e);
        if (v > 0) return v;
    }
    return 120000.0;
}

// One rank's part of a frame.  kind 0: FP64 frame (W*H*3 doubles); kind 1:
// toByte'd RGB8 frame (W*H*3 bytes).  out_root: the root's device output
// (ignored on other ranks).  Blocks until this rank's work (and, on the
// root, the whole frame) is complete.
int dist_frame(rt_dist& D, const rt_scene* s, int W, int H, int mode, int flags, int kind, void* out_root,
               hipStream_t st, rt_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> lk(D.mu);
    if (D.dead) {
        rtamd::set_last_error("rt_render_dist: this rank's communicator was aborted (" + D.dead_why +
                              abort_note(D) + "); destroy the handle and create a new one");
        return RT_ERR_HIP;
    }
    const bool root = D.rank == 0;
    const bool coll = D.collective();
    const int inject = D.inject;
    D.inject = 0;
    const int64_t shed_std = root_shed(RT_MODE_STANDARD) + D.shed_delta, shed_paper = root_shed(RT_MODE_PAPER) + D.shed_delta;
    D.shed_delta = 0;
    // Local argument checks.  Without a collective they return at once; in a
    // collective frame a failing rank still joins the frame's agreement (below)
    // so that no peer waits for it.
    int rc = RT_OK;
    if (!s) { rtamd::set_last_error("rt_render_dist: scene is NULL"); rc = RT_ERR_INVALID_ARG; }
    else if (W <= 0 || H <= 0) { rtamd::set_last_error("rt_render_dist: W and H must be > 0"); rc = RT_ERR_INVALID_ARG; }
    else if (mode != RT_MODE_STANDARD && mode != RT_MODE_PAPER) { rtamd::set_last_error("rt_render_dist: bad mode"); rc = RT_ERR_INVALID_ARG; }
    else if (root && !out_root) { rtamd::set_last_error("rt_render_dist: the root needs an output buffer"); rc = RT_ERR_INVALID_ARG; }
    if (rc != RT_OK && !coll) return rc;
    {
        // (the collective stream itself: without it nothing can be joined)
        const int rs = dist_init_streams(D, coll, coll || (mode == RT_MODE_PAPER && rtamd::paper_chunks_1gpu() > 1));
        if (rs != RT_OK) return rs;
    }
    const int Wc = std::max(W, 1), Hc = std::max(H, 1);
    const int S = strip_height(mode == RT_MODE_PAPER ? RT_MODE_PAPER : RT_MODE_STANDARD);
    int64_t shash = 0;   // (the scene's content hash, checked with the descriptor)
    if (s) {
        const uint64_t uid = rtamd::scene_uid(s);
        auto it = D.scene_hashes.find(uid);
        if (it == D.scene_hashes.end()) {
            if (D.scene_hashes.size() > 64) D.scene_hashes.clear();
            it = D.scene_hashes.emplace(uid, scene_hash(s)).first;
        }
        shash = it->second;
    }
    const size_t n_desc = 2 * kDescFields + (size_t)D.world;
    const size_t n_stat = (size_t)D.world;
    if (coll) {
        const int rx = dist_init_xchg(D, n_desc + n_stat);
        if (rx != RT_OK) return rx;
    }
    const std::vector<std::vector<int32_t>> part =
        partition_rows(Hc, D.world, mode, kind ? 0 : (mode == RT_MODE_PAPER ? shed_paper : shed_std));
    const std::vector<int32_t>& rows = part[D.rank];
    const int n = (int)rows.size();
    int m = 0;
    for (const auto& pr : part) m = std::max(m, (int)pr.size());
    const size_t row_elems = (size_t)Wc * 3;
    // paper mode (FP64) across ranks: each rank produces one paper-code byte
    // per pixel, 1 B/px crosses xGMI, and the root decodes (k_place_codes)
    const bool codes = coll && mode == RT_MODE_PAPER && !(flags & RT_FLAG_FP32);
    const size_t row_bytes = codes ? (size_t)Wc : row_elems * (kind ? 1 : sizeof(double));   // gathered per row
    // (one GPU: paper frames in chunks too, so that each chunk's finish pass
    // overlaps the next chunk's primary on the other stream)
    // (kChunks bounds the per-chunk event arrays)
    const auto bounds = chunk_bounds(
        m, std::min(kChunks, coll ? frame_chunks(mode) : (mode == RT_MODE_PAPER ? rtamd::paper_chunks_1gpu() : 1)), S);
    const bool direct = !coll && kind == 0;   // trace straight into the caller's frame
    DevBuf& stage = D.sim_stage ? *D.sim_stage : D.stage;
    auto fail = [&](int code, const char* what) {
        if (rc == RT_OK) {
            rc = code;
            if (what) rtamd::set_last_error(std::string("rt_render_dist: ") + what);
        }
    };
    // setup: buffers, the root's placement table, the frame
    if (rc == RT_OK && !direct &&
        D.mine.ensure(std::max<size_t>(1, (size_t)m * (codes ? (size_t)Wc : row_elems * sizeof(double)))) != hipSuccess)
        fail(RT_ERR_HIP, "row buffer allocation failed");
    if (rc == RT_OK && kind == 1 && coll && !codes && D.mine8.ensure(std::max<size_t>(1, (size_t)m * row_elems)) != hipSuccess)
        fail(RT_ERR_HIP, "RGB8 row buffer allocation failed");
    if (rc == RT_OK && coll && (root || D.sim_stage) && stage.ensure((size_t)D.world * m * row_bytes) != hipSuccess)
        fail(RT_ERR_HIP, "gather stage allocation failed");
    if (rc == RT_OK && coll && root) {
        // placement table: chunk k occupies slots [world*a, world*b) as [rank][b-a]
        D.rowtab_host.assign((size_t)D.world * m, -1);
        for (int r = 0; r < D.world; ++r) {
            const std::vector<int32_t>& rr = part[r];
            for (const auto& ab : bounds)
                for (int i = ab.first; i < ab.second; ++i)
                    D.rowtab_host[(size_t)D.world * ab.first + (size_t)r * (ab.second - ab.first) + (i - ab.first)] =
                        i < (int)rr.size() ? rr[i] : -1;
        }
        if (D.rowtab.ensure(D.rowtab_host.size() * sizeof(int32_t)) != hipSuccess ||
            hipMemcpyAsync(D.rowtab.p, D.rowtab_host.data(), D.rowtab_host.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice, D.comm_st) != hipSuccess)
            fail(RT_ERR_HIP, "placement table upload failed");
    }
    if (rc == RT_OK && inject == kInjectSetupFail) fail(RT_ERR_HIP, "injected setup failure (rt_test_dist_inject)");
    rt_frame* f = nullptr;
    if (rc == RT_OK) {
        const int rb = rt_frame_begin(s, W, H, mode, flags, rows.data(), n, st, &f);
        if (rb != RT_OK) rc = rb;   // (rt_frame_begin set the message)
    }
    if (!coll && rc != RT_OK) return rc;

    // agreement 1 (collective frames): descriptor + setup status of every
    // rank, issued right after chunk 0's trace is enqueued (so that the
    // trace starts without waiting for these host calls) and awaited before
    // the first gather.  A failure of chunk 0's own launch is reported here
    // too.
    int64_t* xd = D.xchg.as<int64_t>();
    int64_t* xh = D.xchg_host;
    bool a_timed = false;
    auto issue_agreement = [&]() -> bool {
        const int64_t v[kDescFields] = {W, H, mode, kind, flags, shash, shed_std, shed_paper};
        for (int i = 0; i < kDescFields; ++i) {
            xh[i] = v[i];
            xh[kDescFields + i] = -v[i];
        }
        for (int r = 0; r < D.world; ++r) xh[2 * kDescFields + r] = (r == D.rank && rc != RT_OK) ? 1 : 0;
        std::string why;
        bool ok = hipMemcpyAsync(xd, xh, n_desc * sizeof(int64_t), hipMemcpyHostToDevice, D.comm_st) == hipSuccess;
        if (!ok) why = "descriptor upload failed";
        if (ok) {
            a_timed = hipEventRecord(D.ev_a0, D.comm_st) == hipSuccess;
            why = coll_max_i64(D, xd, n_desc, "the frame agreement");
            ok = why.empty();
            a_timed = a_timed && ok && hipEventRecord(D.ev_a1, D.comm_st) == hipSuccess;
        }
        if (ok) ok = hipMemcpyAsync(xh, xd, n_desc * sizeof(int64_t), hipMemcpyDeviceToHost, D.comm_st) == hipSuccess;
        if (ok && inject == kInjectStall) {
            int rate_khz = 100000;
            (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, D.device);
            // bounded (the wave always leaves), and far longer than the timeout:
            // the rank must give up at its deadline, not when the stream drains
            const double stall_ms = std::min(std::max(10000.0, 4 * D.timeout_ms), 30000.0);
            const unsigned long long ticks = (unsigned long long)rate_khz * (unsigned long long)stall_ms;
            hipLaunchKernelGGL(k_test_stall, dim3(1), dim3(64), 0, D.comm_st, ticks);
            ok = hipGetLastError() == hipSuccess;
        }
        if (ok) ok = hipEventRecord(D.ev_desc, D.comm_st) == hipSuccess;
        if (!ok) {
            // this rank cannot take part in the frame's collectives: its peers
            // will time out; abort so that nothing is left queued on them here
            if (f) (void)rt_frame_end(f, nullptr);
            if (why.empty()) why = "HIP call failed";
            dist_abort(D, "frame agreement could not be issued: " + why);
            rtamd::set_last_error("rt_render_dist: the frame agreement could not be issued (" + why +
                                  "); communicator aborted");
        }
        return ok;
    };
    double* fb_rows = direct ? static_cast<double*>(out_root) : D.mine.as<double>();
    int n_tb = 0, n_g = 0;
    double agree_wait_ms = 0.0;
    bool gm_ok[kChunks] = {};
    bool status_sent = false, issued = false;
    // Pass 1: every chunk's trace (and toByte) enqueued on its stream and the
    // chunk's end recorded (ev_chunk[k]); agreement 1 issued right after
    // chunk 0.  Pass 2 (collective frames): agreement 1's verdict, agreement 2
    // (this rank's trace status: every enqueue is known by then, so the
    // reduction sits on the collective stream ahead of the gathers, in the
    // shadow of the trace, not between the last two gathers at the frame's
    // tail), then one gather (+ the root's placement) per chunk.
    bool chunk_ev[kChunks] = {};
    for (size_t k = 0; k < bounds.size(); ++k) {
        const int a = bounds[k].first, b = bounds[k].second, hi = std::min(b, n);
        (void)b;
        // chunks alternate between two streams, the last one on st: the frame's
        // end (rt_frame_end on st) then follows it in stream order instead of
        // through a cross-queue wait (~40 us, profiles/r04u_api_timeline.txt)
        const hipStream_t cst = ((bounds.size() - 1 - k) & 1) ? D.alt_st : st;
        if (rc == RT_OK && inject == kInjectTraceFail && k == bounds.size() / 2) {
            rtamd::set_last_error("rt_render_dist: injected trace failure (rt_test_dist_inject)");
            rc = RT_ERR_HIP;
        }
        if (rc == RT_OK && hi > a)
            rc = codes ? rtamd::frame_trace_paper_codes(f, a, hi, D.mine.as<uint8_t>() + (size_t)a * row_bytes, cst)
                       : rt_frame_trace(f, a, hi, fb_rows + (size_t)a * row_elems, cst);
        if (rc == RT_OK && kind == 1 && hi > a && !codes) {
            // (one GPU: rows are the frame's, in order, so chunk rows land at their own place)
            uint8_t* dst8 = (coll ? D.mine8.as<uint8_t>() : static_cast<uint8_t*>(out_root)) + (size_t)a * row_elems;
            if (hipEventRecord(D.ev_tb[n_tb++], cst) != hipSuccess) fail(RT_ERR_HIP, "event record failed");
            if (rc == RT_OK) rc = rt_framebuffer_to_rgb8_device(fb_rows + (size_t)a * row_elems, (size_t)(hi - a) * W, dst8, cst);
            if (rc == RT_OK && hipEventRecord(D.ev_tb[n_tb++], cst) != hipSuccess) fail(RT_ERR_HIP, "event record failed");
        }
        if (!coll) {
            if (rc != RT_OK) break;
            continue;
        }
        // chunk k's end, for its gather (none after a local failure: the
        // gather is still issued - the peers are waiting for it)
        if (rc == RT_OK) {
            chunk_ev[k] = hipEventRecord(D.ev_chunk[k], cst) == hipSuccess;
            if (!chunk_ev[k]) fail(RT_ERR_HIP, "event chaining failed");
        }
        if (!issued) {
            if (!issue_agreement()) return RT_ERR_HIP;
            issued = true;
        }
    }
    if (coll && !issued) {
        if (!issue_agreement()) return RT_ERR_HIP;
        issued = true;
    }
    if (coll) {
        // (the descriptor reduction ran while the chunks trace)
        const auto t_aw = std::chrono::steady_clock::now();
        const int rw = dist_wait(D, D.ev_desc, "the frame agreement");
        agree_wait_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_aw).count();
        if (rw != RT_OK) {
            if (f) (void)rt_frame_end(f, nullptr);
            return rw;
        }
        std::string bad;
        for (int i = 0; i < kDescFields; ++i) {
            static const char* names[kDescFields] = {"W", "H", "mode", "output kind", "flags", "scene",
                                                     "RT_ROOT_SHED_STD", "RT_ROOT_SHED_PAPER"};
            if (xh[i] != -xh[kDescFields + i]) bad += std::string(bad.empty() ? "" : ", ") + names[i];
        }
        std::string failed;
        for (int r = 0; r < D.world; ++r)
            if (xh[2 * kDescFields + r]) failed += (failed.empty() ? "" : ",") + std::to_string(r);
        if (!bad.empty() || !failed.empty()) {
            // every rank reaches this same verdict: no gather is issued anywhere
            const int rl = rc;
            const int re = f ? rt_frame_end(f, nullptr) : RT_OK;
            (void)re;
            if (rl != RT_OK) return rl;   // this rank's own failure (message already set)
            if (!bad.empty()) {
                rtamd::set_last_error("rt_render_dist: the ranks disagree on the frame (" + bad + ")");
                return RT_ERR_INVALID_ARG;
            }
            rtamd::set_last_error("rt_render_dist: rank(s) " + failed + " failed to set up or start the frame");
            return RT_ERR_HIP;
        }
        // agreement 2: this rank's trace status (every chunk is enqueued or skipped)
        {
            int64_t* sd = xd + n_desc;
            int64_t* sh = xh + n_desc;
            for (int r = 0; r < D.world; ++r) sh[r] = (r == D.rank && rc != RT_OK) ? 1 : 0;
            bool ok = hipMemcpyAsync(sd, sh, n_stat * sizeof(int64_t), hipMemcpyHostToDevice, D.comm_st) == hipSuccess;
            std::string why = ok ? coll_max_i64(D, sd, n_stat, "the trace status reduction") : "status upload failed";
            ok = why.empty();
            if (ok) ok = hipMemcpyAsync(sh, sd, n_stat * sizeof(int64_t), hipMemcpyDeviceToHost, D.comm_st) == hipSuccess;
            if (!ok) fail(RT_ERR_HIP, ("trace status reduction could not be issued: " + why).c_str());
            status_sent = ok;
        }
        for (size_t k = 0; k < bounds.size(); ++k) {
            const int a = bounds[k].first, b = bounds[k].second;
            // chunk k -> root: ONE collective, ordered after the chunk's trace
            // (issued whatever happened locally: the peers are waiting for it)
            if (chunk_ev[k] && hipStreamWaitEvent(D.comm_st, D.ev_chunk[k], 0) != hipSuccess)
                fail(RT_ERR_HIP, "event chaining failed");
            const bool timed = hipEventRecord(D.ev_gs[n_g], D.comm_st) == hipSuccess;
            const char* send = (kind && !codes ? D.mine8.as<char>() : D.mine.as<char>()) + (size_t)a * row_bytes;
            const size_t chunk_bytes = (size_t)(b - a) * row_bytes;
            char* recv = stage.as<char>() + (size_t)D.world * a * row_bytes;
            {
                const std::string why = coll_gather(D, send, (root || D.sim_stage) ? recv : nullptr, chunk_bytes,
                                                    kind || codes, "a gather");
                if (!why.empty()) {
                    fail(RT_ERR_HIP, why.c_str());
                    if (D.simg && D.simg->is_aborted(nullptr)) dist_abort(D, why);
                }
            }
            gm_ok[n_g] = timed && hipEventRecord(D.ev_gm[n_g], D.comm_st) == hipSuccess;
            if (root) {
                const int32_t* slots = D.rowtab.as<int32_t>() + (size_t)D.world * a;
                const hipError_t pe = codes ? place_codes(reinterpret_cast<const uint8_t*>(recv), slots, D.world * (b - a),
                                                          Wc, kind, out_root, D.comm_st)
                                            : place_rows(recv, slots, D.world * (b - a), row_bytes, out_root, D.comm_st);
                if (pe != hipSuccess) fail(RT_ERR_HIP, "row placement failed");
            }
            if (timed && hipEventRecord(D.ev_ge[n_g], D.comm_st) == hipSuccess) ++n_g;
        }
    }
    const auto t_tail = std::chrono::steady_clock::now();
    // alt_st's last work (a chunk's toByte) into st, which rt_frame_end
    // synchronises (without toByte, rt_frame_end joins alt_st's last trace call)
    if (n_tb > 0 && D.alt_st &&
        (hipEventRecord(D.ev_alt, D.alt_st) != hipSuccess || hipStreamWaitEvent(st, D.ev_alt, 0) != hipSuccess))
        fail(RT_ERR_HIP, "stream join failed");
    const int rc_end = f ? rt_frame_end(f, stats) : RT_OK;   // joins and synchronises the trace streams
    if (coll) {
        if (hipEventRecord(D.ev_desc, D.comm_st) != hipSuccess) {
            dist_abort(D, "could not record the end of the frame's collectives");
            rtamd::set_last_error("rt_render_dist: could not record the end of the frame's collectives; communicator aborted");
            return RT_ERR_HIP;
        }
        const int rw = dist_wait(D, D.ev_desc, "the frame's gathers");
        if (rw != RT_OK) return rw;
    }
    if (rc != RT_OK) return rc;
    if (rc_end != RT_OK) return rc_end;
    if (coll && status_sent) {
        std::string failed;
        for (int r = 0; r < D.world; ++r)
            if (xh[n_desc + r]) failed += (failed.empty() ? "" : ",") + std::to_string(r);
        if (!failed.empty()) {
            rtamd::set_last_error("rt_render_dist: rank(s) " + failed + " failed while tracing the frame" +
                                  (root ? " (the gathered frame is incomplete)" : ""));
            return RT_ERR_HIP;
        }
    }
    if (stats) {
        float ms = 0.f;
        // the collectives and placements themselves (each waits for its
        // chunk's trace first; the waits are not counted)
        double g = 0.0;
        for (int i = 0; i < n_g; ++i)
            if (hipEventElapsedTime(&ms, D.ev_gs[i], D.ev_ge[i]) == hipSuccess) g += ms;
        stats->ms_gather = g;
        if (coll) {
            // this rank's split of the frame (rt_dist_frame_split)
            double* sp = D.split;
            std::fill(sp, sp + kSplitSlots, 0.0);
            if (a_timed && hipEventElapsedTime(&ms, D.ev_a0, D.ev_a1) == hipSuccess) sp[1] = ms;
            sp[2] = agree_wait_ms;
            for (int i = 0; i < n_g; ++i) {
                float mg = 0.f, mp = 0.f;
                if (!gm_ok[i] || hipEventElapsedTime(&mg, D.ev_gs[i], D.ev_gm[i]) != hipSuccess ||
                    hipEventElapsedTime(&mp, D.ev_gm[i], D.ev_ge[i]) != hipSuccess)
                    continue;
                sp[3] += mg;
                sp[4] += mp;
                if (i == n_g - 1) {
                    sp[5] = mg;
                    sp[6] = mp;
                }
            }
            sp[7] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_tail).count();
            int cw = D.simg ? D.simg->world : D.world;
            if (D.comm && ncclCommCount(D.comm, &cw) != ncclSuccess) cw = -1;
            sp[8] = cw;
            sp[9] = n;
        }
        double tb = 0.0;
        for (int i = 0; i + 1 < n_tb; i += 2)
            if (hipEventElapsedTime(&ms, D.ev_tb[i], D.ev_tb[i + 1]) == hipSuccess) tb += ms;
        stats->ms_tobyte = tb;
        stats->n_gpus = D.world;
        stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (coll) D.split[0] = stats->ms_total;
    }
    return RT_OK;
}

// Everything a rank holds on its device: the communicator (if owned),
// buffers, streams and events.  The rank object itself stays valid (empty).
void release_rank(rt_dist& d) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(d.device);
    if (d.abort_th.joinable()) d.abort_th.join();
    if (d.comm_st) (void)hipStreamSynchronize(d.comm_st);
    if (d.comm && d.own_comm) (void)ncclCommDestroy(d.comm);
    d.comm = nullptr;
    d.own_comm = false;
    d.mine.release();
    d.mine8.release();
    d.stage.release();
    d.rowtab.release();
    d.red.release();
    d.simtmp.release();
    d.xchg.release();
    if (d.xchg_host) (void)hipHostFree(d.xchg_host);
    d.xchg_host = nullptr;
    if (d.comm_st) (void)hipStreamDestroy(d.comm_st);
    if (d.alt_st) (void)hipStreamDestroy(d.alt_st);
    d.comm_st = d.alt_st = nullptr;
    auto drop = [](hipEvent_t& e) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
    };
    for (auto& e : d.ev_chunk) drop(e);
    for (auto& e : d.ev_tb) drop(e);
    for (auto& e : d.ev_gs) drop(e);
    for (auto& e : d.ev_gm) drop(e);
    for (auto& e : d.ev_ge) drop(e);
    drop(d.ev_a0);
    drop(d.ev_a1);
    drop(d.ev_alt);
    drop(d.ev_desc);
    (void)hipSetDevice(prev);
}

// --------------------------------------------- one process, n devices
struct LocalGroup {
    std::mutex mu;   // one rt_render_multi / rt_render_rgb8 call at a time per group (comms, root buffers)
    int n = 0;
    std::vector<std::unique_ptr<rt_dist>> ranks;
    DevBuf out;      // root frame (device 0)
    DevBuf out8;
};

std::mutex g_groups_mu;
std::map<int, std::unique_ptr<LocalGroup>> g_groups;
std::vector<std::unique_ptr<LocalGroup>> g_dropped;   // emptied groups whose lock may still be held

// rt_shutdown: destroy every cached group (RCCL communicators, streams,
// buffers).  Groups are created again on the next multi-GPU call.
int shutdown_groups() {
    std::lock_guard<std::mutex> lk(g_groups_mu);
    int n = 0;
    for (auto& kv : g_groups) {
        LocalGroup& G = *kv.second;
        std::lock_guard<std::mutex> glk(G.mu);
        for (auto& r : G.ranks) release_rank(*r);
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(0);
        G.out.release();
        G.out8.release();
        (void)hipSetDevice(prev);
        ++n;
    }
    g_groups.clear();
    g_dropped.clear();
    return n;
}

// Called with G->mu held by the caller (render_multi); takes the registry lock.
void drop_group(int n, LocalGroup* G) {
    for (auto& r : G->ranks) release_rank(*r);
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(0);
    G->out.release();
    G->out8.release();
    (void)hipSetDevice(prev);
    std::lock_guard<std::mutex> lk(g_groups_mu);
    auto it = g_groups.find(n);
    if (it != g_groups.end() && it->second.get() == G) g_dropped.push_back(std::move(it->second));   // freed at rt_shutdown
    if (it != g_groups.end()) g_groups.erase(it);
}

int local_group(int n, LocalGroup** out) {
    std::lock_guard<std::mutex> lk(g_groups_mu);
    auto it = g_groups.find(n);
    if (it != g_groups.end()) {
        *out = it->second.get();
        return RT_OK;
    }
    std::unique_ptr<LocalGroup> G(new LocalGroup);
    G->n = n;
    std::vector<ncclComm_t> comms(n, nullptr);
    if (n > 1) {
        std::vector<int> devs(n);
        for (int i = 0; i < n; ++i) devs[i] = i;
        NCCL_TRY(ncclCommInitAll(comms.data(), n, devs.data()));
    }
    for (int i = 0; i < n; ++i) {
        std::unique_ptr<rt_dist> D(new rt_dist);
        D->world = n;
        D->rank = i;
        D->device = i;
        D->timeout_ms = env_timeout_ms();
        D->comm = comms[i];
        D->own_comm = n > 1;
        G->ranks.push_back(std::move(D));
    }
    *out = G.get();
    g_groups[n] = std::move(G);
    return RT_OK;
}

int render_multi(const rt_scene* s, int W, int H, int mode, int flags, int n_gpus, int kind, void* out_host,
                 rt_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!out_host) { rtamd::set_last_error("rt_render_multi: output is NULL"); return RT_ERR_INVALID_ARG; }
    if (!s) { rtamd::set_last_error("rt_render_multi: scene is NULL"); return RT_ERR_INVALID_ARG; }
    if (W <= 0 || H <= 0) { rtamd::set_last_error("rt_render: W and H must be > 0"); return RT_ERR_INVALID_ARG; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        rtamd::set_last_error("rt_render: no HIP device available");
        return RT_ERR_NO_DEVICE;
    }
    const int n = n_gpus <= 0 ? ndev : n_gpus;
    if (n > ndev) {
        rtamd::set_last_error("rt_render_multi: " + std::to_string(n) + " GPUs requested, " + std::to_string(ndev) +
                              " visible");
        return RT_ERR_INVALID_ARG;
    }
    int prev_dev = 0;
    HIP_TRY(hipGetDevice(&prev_dev));
    LocalGroup* G = nullptr;
    int rc = local_group(n, &G);
    if (rc != RT_OK) return rc;
    // the whole call under the group's lock: buffer ensure, the per-device
    // threads (their ncclGather calls must not interleave with another
    // call's on the same communicators) and the D2H copy
    std::lock_guard<std::mutex> glk(G->mu);
    const size_t out_bytes = (size_t)W * H * 3 * (kind ? 1 : sizeof(double));
    HIP_TRY(hipSetDevice(0));
    DevBuf& out = kind ? G->out8 : G->out;
    HIP_TRY(out.ensure(out_bytes));
    rtamd::note_setup_ms(rtamd::kLastGroup,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    std::vector<rt_stats> st(n);
    std::vector<int> rcs(n, RT_OK);
    std::vector<std::string> errs(n);
    auto work = [&](int i) {
        if (hipSetDevice(i) != hipSuccess) {
            rcs[i] = RT_ERR_HIP;
            errs[i] = "hipSetDevice failed";
            return;
        }
        std::memset(&st[i], 0, sizeof(rt_stats));
        rcs[i] = dist_frame(*G->ranks[i], s, W, H, mode, flags, kind, i == 0 ? out.p : nullptr, nullptr, &st[i]);
        if (rcs[i] != RT_OK) errs[i] = rt_last_error();
    };
    if (n == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int i = 0; i < n; ++i) th.emplace_back(work, i);
        for (auto& t : th) t.join();
    }
    (void)hipSetDevice(0);
    for (int i = 0; i < n; ++i)
        if (rcs[i] != RT_OK) {
            // a rank whose communicator was aborted leaves the group unusable:
            // drop it (the next call creates the communicators again)
            bool dead = false;
            for (auto& r : G->ranks) dead = dead || r->dead;
            if (dead) drop_group(n, G);
            rtamd::set_last_error("device " + std::to_string(i) + ": " + errs[i]);
            (void)hipSetDevice(prev_dev);
            return rcs[i];
        }
    const auto t1 = std::chrono::steady_clock::now();
    HIP_TRY(hipMemcpy(out_host, out.p, out_bytes, hipMemcpyDeviceToHost));
    const auto t2 = std::chrono::steady_clock::now();
    (void)hipSetDevice(prev_dev);
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        for (int i = 0; i < n; ++i) {
            stats->rays_intersect += st[i].rays_intersect;
            stats->rays_occluded += st[i].rays_occluded;
            stats->rays_traced += st[i].rays_traced;
            stats->pixels += st[i].pixels;
            stats->ms_rng = std::max(stats->ms_rng, st[i].ms_rng);
            stats->ms_kernel = std::max(stats->ms_kernel, st[i].ms_kernel);
            stats->ms_tobyte = std::max(stats->ms_tobyte, st[i].ms_tobyte);
            for (int k = 0; k < 16; ++k) stats->ops[k] += st[i].ops[k];
        }
        stats->ms_gather = st[0].ms_gather;
        stats->ms_d2h = std::chrono::duration<double, std::milli>(t2 - t1).count();
        stats->ms_total = std::chrono::duration<double, std::milli>(t2 - t0).count();
        stats->n_gpus = n;
    }
    return RT_OK;
}

}  // namespace

// ------------------------------------------------------------------ C-ABI
extern "C" int rt_dist_rows_mode(int H, int world, int rank, int mode, int32_t* rows_out) {
    if (H <= 0 || world <= 0 || rank < 0 || rank >= world || !rows_out ||
        (mode != RT_MODE_STANDARD && mode != RT_MODE_PAPER))
        return RT_ERR_INVALID_ARG;
    const std::vector<int32_t> r = partition_rows(H, world, mode, root_shed(mode))[rank];
    std::copy(r.begin(), r.end(), rows_out);
    return (int)r.size();
}

extern "C" int rt_dist_frame_split(rt_dist* d, double* out, int n) {
    if (!d || !out || n < 0) { rtamd::set_last_error("rt_dist_frame_split: bad arguments"); return RT_ERR_INVALID_ARG; }
    std::lock_guard<std::mutex> lk(d->mu);
    for (int i = 0; i < n && i < kSplitSlots; ++i) out[i] = d->split[i];
    return std::min(n, kSplitSlots);
}

extern "C" int rt_dist_rows(int H, int world, int rank, int32_t* rows_out) {
    return rt_dist_rows_mode(H, world, rank, RT_MODE_STANDARD, rows_out);
}

extern "C" int rt_render_multi(const rt_scene* s, int W, int H, int mode, int flags, int n_gpus, double* fb_host,
                               rt_stats* stats) {
    if (n_gpus == 1) return rt_render(s, W, H, mode, flags, fb_host, stats);
    return render_multi(s, W, H, mode, flags, n_gpus, 0, fb_host, stats);
}

extern "C" int rt_render_rgb8(const rt_scene* s, int W, int H, int mode, int flags, int n_gpus, uint8_t* rgb8_host,
                              rt_stats* stats) {
    return render_multi(s, W, H, mode, flags, n_gpus, 1, rgb8_host, stats);
}

extern "C" int rt_dist_get_id(uint8_t id[RT_DIST_ID_BYTES]) {
    if (!id) { rtamd::set_last_error("rt_dist_get_id: NULL"); return RT_ERR_INVALID_ARG; }
    static_assert(sizeof(ncclUniqueId) == RT_DIST_ID_BYTES, "RT_DIST_ID_BYTES must match ncclUniqueId");
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return RT_OK;
}

extern "C" int rt_dist_create(const uint8_t id[RT_DIST_ID_BYTES], int world, int rank, rt_dist** out) {
    if (!out || !id || world <= 0 || rank < 0 || rank >= world) {
        rtamd::set_last_error("rt_dist_create: bad arguments");
        return RT_ERR_INVALID_ARG;
    }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        rtamd::set_last_error("rt_dist_create: no HIP device available");
        return RT_ERR_NO_DEVICE;
    }
    std::unique_ptr<rt_dist> D(new rt_dist);
    D->world = world;
    D->rank = rank;
    D->timeout_ms = env_timeout_ms();
    HIP_TRY(hipGetDevice(&D->device));
    if (world > 1) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        NCCL_TRY(ncclCommInitRank(&D->comm, world, u, rank));
        D->own_comm = true;
    }
    *out = D.release();
    return RT_OK;
}

extern "C" int rt_dist_set_timeout(rt_dist* d, int timeout_ms) {
    if (!d || timeout_ms <= 0) { rtamd::set_last_error("rt_dist_set_timeout: bad arguments"); return RT_ERR_INVALID_ARG; }
    std::lock_guard<std::mutex> lk(d->mu);
    d->timeout_ms = timeout_ms;
    return RT_OK;
}

extern "C" void rt_dist_destroy(rt_dist* d) {
    if (!d) return;
    release_rank(*d);
    delete d;
}

extern "C" int rt_render_dist(rt_dist* d, const rt_scene* s, int W, int H, int mode, int flags, double* fb_root_dev,
                              void* hip_stream, rt_stats* stats) {
    if (!d) { rtamd::set_last_error("rt_render_dist: dist is NULL"); return RT_ERR_INVALID_ARG; }
    return dist_frame(*d, s, W, H, mode, flags, 0, fb_root_dev, (hipStream_t)hip_stream, stats);
}

extern "C" int rt_render_dist_rgb8(rt_dist* d, const rt_scene* s, int W, int H, int mode, int flags,
                                   uint8_t* rgb8_root_dev, void* hip_stream, rt_stats* stats) {
    if (!d) { rtamd::set_last_error("rt_render_dist_rgb8: dist is NULL"); return RT_ERR_INVALID_ARG; }
    return dist_frame(*d, s, W, H, mode, flags, 1, rgb8_root_dev, (hipStream_t)hip_stream, stats);
}

// ------------------------------------------------------------- test hook
// The ranks of a distributed frame on the current device, CONCURRENTLY: one
// host thread per rank, each with its own frame stream, collective and
// alternate streams and device workspace (workspace slot rank + 1), through
// dist_frame with the same-device transport (SimGroup) in place of RCCL, so
// every line of the world >= 2 protocol runs: partition, chunks, the frame
// agreement and trace-status reductions and their verdicts, gathers, the
// root's placement, and the timeouts.  Ranks run their frames freely, as
// processes would (no barrier between frames).  See rt_test.h.
extern "C" int rt_test_dist_threads(const rt_scene* s, int W, int H, int mode, int flags, rt_test_dist_run* run,
                                    double* fb_host, uint8_t* rgb8_host) {
    if (!s || !run || W <= 0 || H <= 0 || run->world <= 0 || run->world > kSimMaxWorld || run->frames <= 0 ||
        !run->rc || !run->ms)
        return RT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    const int world = run->world, frames = run->frames;
    const int kind = run->rgb8 ? 1 : 0;
    const size_t frame_bytes = (size_t)W * H * 3 * (kind ? 1 : sizeof(double));
    DevBuf out;
    HIP_TRY(out.ensure((size_t)W * (H + 1) * 3 * (kind ? 1 : sizeof(double))));   // (+1 row: a rank may be given H + 1)
    SimGroup G(world);
    std::vector<std::unique_ptr<rt_dist>> ranks;
    int rc = RT_OK;
    for (int r = 0; r < world && rc == RT_OK; ++r) {
        ranks.emplace_back(new rt_dist);
        rt_dist& D = *ranks.back();
        D.world = world;
        D.rank = r;
        D.device = dev;
        D.simg = world > 1 ? &G : nullptr;
        D.timeout_ms = run->timeout_ms > 0 ? run->timeout_ms : env_timeout_ms();
        if (hipEventCreateWithFlags(&G.in[r], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&G.rd[r], hipEventDisableTiming) != hipSuccess)
            rc = RT_ERR_HIP;
    }
    if (rc == RT_OK && hipEventCreateWithFlags(&G.copied, hipEventDisableTiming) != hipSuccess) rc = RT_ERR_HIP;
    if (rc == RT_OK) {
        auto body = [&](int r) {
            rt_dist& D = *ranks[r];
            (void)hipSetDevice(dev);
            rtamd::set_workspace_slot(r + 1);
            hipStream_t st = nullptr;
            const bool have_st = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
            for (int fr = 0; fr < frames; ++fr) {
                const size_t o = (size_t)fr * world + r;
                run->ms[o] = 0.0;
                if (run->msgs && run->msg_cap > 0) run->msgs[o * run->msg_cap] = 0;
                const bool hit = fr == run->fault_frame && r == run->fault_rank;
                if (hit && run->fault == RT_TEST_FAULT_ABSENT) {
                    run->rc[o] = RT_TEST_RANK_ABSENT;
                    continue;
                }
                if (!have_st) {
                    run->rc[o] = RT_ERR_HIP;
                    continue;
                }
                int Hr = H, fl = flags;
                const rt_scene* sf = run->frame_scenes && run->frame_scenes[fr] ? run->frame_scenes[fr] : s;
                if (hit) {
                    if (run->fault == RT_TEST_FAULT_DESC_SCENE && run->alt_scene) sf = run->alt_scene;
                    if (run->fault == RT_TEST_FAULT_DESC_SHED) D.shed_delta = 1;
                    if (run->fault == RT_TEST_FAULT_TRACE) D.inject = kInjectTraceFail;
                    if (run->fault == RT_TEST_FAULT_SETUP) D.inject = kInjectSetupFail;
                    if (run->fault == RT_TEST_FAULT_DESC_H) Hr = H + 1;
                    if (run->fault == RT_TEST_FAULT_DESC_FLAGS) fl ^= RT_FLAG_NO_CULL;
                }
                if (r == 0) {   // every output byte must be written by this frame's placement
                    (void)hipMemsetAsync(out.p, 0xff, out.n, st);
                    (void)hipStreamSynchronize(st);
                }
                const auto t0 = std::chrono::steady_clock::now();
                rt_stats stt{};
                const int rr = dist_frame(D, sf, W, Hr, mode, fl, kind, r == 0 ? out.p : nullptr, st, &stt);
                run->ms[o] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                run->rc[o] = rr;
                if (rr == RT_OK && run->split) std::copy(D.split, D.split + kSplitSlots, run->split + o * kSplitSlots);
                if (rr != RT_OK && run->msgs && run->msg_cap > 0)
                    std::snprintf(run->msgs + o * run->msg_cap, (size_t)run->msg_cap, "%s", rt_last_error());
                if (r == 0 && rr == RT_OK) {
                    void* dst = kind ? (void*)(rgb8_host ? rgb8_host + (size_t)fr * frame_bytes : nullptr)
                                     : (void*)(fb_host ? reinterpret_cast<char*>(fb_host) + (size_t)fr * frame_bytes : nullptr);
                    if (dst && hipMemcpy(dst, out.p, frame_bytes, hipMemcpyDeviceToHost) != hipSuccess)
                        run->rc[o] = RT_ERR_HIP;
                }
            }
            if (have_st) {
                (void)hipStreamSynchronize(st);
                (void)hipStreamDestroy(st);
            }
            rtamd::set_workspace_slot(0);
        };
        std::vector<std::thread> th;
        for (int r = 0; r < world; ++r) th.emplace_back(body, r);
        for (auto& t : th) t.join();
    }
    (void)hipSetDevice(dev);
    for (auto& d : ranks) release_rank(*d);
    for (hipEvent_t e : G.in) if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : G.rd) if (e) (void)hipEventDestroy(e);
    if (G.copied) (void)hipEventDestroy(G.copied);
    out.release();
    (void)rtamd::release_device_workspaces(1);   // the simulated ranks' workspaces
    (void)hipSetDevice(dev);
    return rc;
}

// ------------------------------------------------------------- test hook
// rt_test_dist_threads for one fault-free frame (the root's frame only).
extern "C" int rt_test_render_dist_sim(const rt_scene* s, int W, int H, int mode, int flags, int world, int rgb8,
                                       double* fb_host, uint8_t* rgb8_host) {
    if (!s || W <= 0 || H <= 0 || world <= 0 || world > kSimMaxWorld || (rgb8 ? !rgb8_host : !fb_host))
        return RT_ERR_INVALID_ARG;
    std::vector<int> rcs((size_t)world, RT_OK);
    std::vector<double> ms((size_t)world, 0.0);
    std::vector<char> msgs((size_t)world * 256, 0);
    rt_test_dist_run run{};
    run.world = world;
    run.rgb8 = rgb8;
    run.frames = 1;
    run.fault_rank = -1;
    run.rc = rcs.data();
    run.ms = ms.data();
    run.msgs = msgs.data();
    run.msg_cap = 256;
    const int rc = rt_test_dist_threads(s, W, H, mode, flags, &run, fb_host, rgb8_host);
    if (rc != RT_OK) return rc;
    for (int r = 0; r < world; ++r)
        if (rcs[r] != RT_OK) {
            rtamd::set_last_error("simulated rank " + std::to_string(r) + ": " + std::string(&msgs[(size_t)r * 256]));
            return rcs[r];
        }
    return RT_OK;
}

// ------------------------------------------------------------- test hook
// One simulated rank of a world-`world` frame on the current device, through
// the product's rank path (dist_frame: partition, chunks on two streams,
// paper codes, the gather stage and, on rank 0, the placement), the RCCL
// gather replaced by a device copy into a shared stage.  Ranks are cached per
// (world, rank), so repeated calls time a warm rank (tools/sim_ranks.py).
extern "C" int rt_test_dist_sim_rank(const rt_scene* s, int W, int H, int mode, int flags, int world, int rank,
                                     int rgb8, rt_stats* stats) {
    if (!s || W <= 0 || H <= 0 || world <= 0 || rank < 0 || rank >= world) return RT_ERR_INVALID_ARG;
    static std::mutex mu;
    static std::map<std::pair<int, int>, std::unique_ptr<rt_dist>> ranks;
    static DevBuf stage, out;
    std::lock_guard<std::mutex> lk(mu);
    // every simulated rank on the same two extra streams, as a real rank's
    // process has them (per-rank streams here would outnumber the device's
    // hardware queues and serialise a rank's two chunk streams on one queue)
    static rt_dist streams;
    auto& d = ranks[{world, rank}];
    if (!d) {
        d.reset(new rt_dist);
        d->world = world;
        d->rank = rank;
        d->sim_stage = &stage;
        HIP_TRY(hipGetDevice(&d->device));
        const int rs = dist_init_streams(streams, true, true);
        if (rs != RT_OK) return rs;
        d->comm_st = streams.comm_st;
        d->alt_st = streams.alt_st;
        const int re = dist_init_events(*d);
        if (re != RT_OK) return re;
    }
    void* o = nullptr;
    if (rank == 0) {
        HIP_TRY(out.ensure((size_t)W * H * 3 * (rgb8 ? 1 : sizeof(double))));
        o = out.p;
    }
    return dist_frame(*d, s, W, H, mode, flags, rgb8 ? 1 : 0, o, nullptr, stats);
}

// ---------------------------------------- launcher plumbing over RCCL
// Max-reduction of a few doubles over every rank of d (host in, host out):
// the bench's max-over-ranks timing and its barrier, for launchers without a
// collective layer of their own.  World 1 without a communicator: identity.
extern "C" int rt_dist_reduce_max(rt_dist* d, double* vals_host, int n) {
    if (!d || n < 0 || (n > 0 && !vals_host)) { rtamd::set_last_error("rt_dist_reduce_max: bad arguments"); return RT_ERR_INVALID_ARG; }
    if (!d->comm || n == 0) return RT_OK;
    std::lock_guard<std::mutex> lk(d->mu);
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(d->device));
    int rc = dist_init_streams(*d, true, false);
    if (rc == RT_OK) {
        const size_t bytes = (size_t)n * sizeof(double);
        if (d->red.ensure(bytes) != hipSuccess ||
            hipMemcpyAsync(d->red.p, vals_host, bytes, hipMemcpyHostToDevice, d->comm_st) != hipSuccess) {
            rtamd::set_last_error("rt_dist_reduce_max: device buffer failed");
            rc = RT_ERR_HIP;
        } else {
            const ncclResult_t r = ncclAllReduce(d->red.p, d->red.p, (size_t)n, ncclFloat64, ncclMax, d->comm, d->comm_st);
            if (r != ncclSuccess) {
                rtamd::set_last_error(std::string("ncclAllReduce failed: ") + ncclGetErrorString(r));
                rc = RT_ERR_HIP;
            } else if (hipMemcpyAsync(vals_host, d->red.p, bytes, hipMemcpyDeviceToHost, d->comm_st) != hipSuccess ||
                       hipStreamSynchronize(d->comm_st) != hipSuccess) {
                rtamd::set_last_error("rt_dist_reduce_max: copy back failed");
                rc = RT_ERR_HIP;
            }
        }
    }
    (void)hipSetDevice(prev);
    return rc;
}

extern "C" int rt_dist_barrier(rt_dist* d) {
    double z = 0.0;
    return rt_dist_reduce_max(d, &z, 1);
}

// Release every device resource the library caches: the per-device
// workspaces of rt_render* (scene copies, jitter table, frame buffers) and
// the device groups of rt_render_multi / rt_render_rgb8 (RCCL communicators,
// streams, buffers).  rt_dist handles are the caller's (rt_dist_destroy).
// No render may be in flight; later calls re-create what they need.
extern "C" int rt_shutdown(void) {
    shutdown_groups();
    return rtamd::release_device_workspaces();
}

// ------------------------------------------------------------- test hook
// A world-1 rank WITH a real RCCL communicator (ncclCommInitRank over one
// rank) whose frames take the collective path: row chunks, ncclGather to
// root 0, placement.  On a one-GPU machine this runs the collective API
// surface of the multi-GPU frame (arguments, counts, datatypes, root, the
// communicator's lifetime) through RCCL itself.
extern "C" int rt_test_dist_create_rccl1(rt_dist** out) {
    if (!out) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    uint8_t id[RT_DIST_ID_BYTES];
    int rc = rt_dist_get_id(id);
    if (rc != RT_OK) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
    std::unique_ptr<rt_dist> D(new rt_dist);
    D->world = 1;
    D->rank = 0;
    D->force_collective = true;
    D->timeout_ms = env_timeout_ms();
    HIP_TRY(hipGetDevice(&D->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    NCCL_TRY(ncclCommInitRank(&D->comm, 1, u, 0));
    D->own_comm = true;
    *out = D.release();
    return RT_OK;
}

// ------------------------------------------------------------- test hook
// Fault injection on the next frame of d: 1 = this rank's trace fails at its
// middle chunk (a rank-local failure after the frame agreement), 2 = the
// collective stream is held past the rank's timeout (a peer that never
// arrives: the wait times out and the communicator is aborted).
extern "C" int rt_test_dist_inject(rt_dist* d, int what) {
    if (!d || what < 0 || what > 3) return RT_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(d->mu);
    d->inject = what;
    return RT_OK;
}

// ------------------------------------------------------------- test hook
// The paper-code decoder the root runs after the gather (host build of the
// same inline function), for the CPU tests: value of one code byte.
extern "C" double rt_test_paper_code_value(int code) { return rtamd::paper_code_value((unsigned)code & 31u); }
