// rt_dist.hip — frames on several GPUs and the device output path.
//
// pixels are independent, so a frame is partitioned by OUTPUT
// ROWS: strip s of RT_STRIP_ROWS rows (paper mode: RT_PAPER_STRIP_ROWS) goes
// to rank s mod N (interleaving balances cheap sky rows against expensive
// geometry rows).  Every rank runs
// the ordinary trace (rt_frame_* of rt_render.hip) on its rows, chunk by
// chunk, and each chunk is handed to ONE RCCL collective, ncclGather to rank
// 0 over xGMI, on a high-priority stream so it overlaps the tracing of the
// next chunk; rank 0 places the gathered strips into its frame.  The jitter
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

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rt.h"
#include "rt_internal.hpp"
#include "rt_test.h"

namespace {

constexpr int kChunks = 4;   // pipeline units per rank (chunk k gathered while k+1 is traced)

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

std::vector<int32_t> strip_rows(int H, int world, int rank, int S = RT_STRIP_ROWS) {
    std::vector<int32_t> rows;
    for (int s = 0; s * S < H; ++s)
        if (s % world == rank)
            for (int r = s * S; r < std::min(H, (s + 1) * S); ++r) rows.push_back(r);
    return rows;
}

int max_rows(int H, int world, int S = RT_STRIP_ROWS) {
    int m = 0;
    for (int r = 0; r < world; ++r) m = std::max(m, (int)strip_rows(H, world, r, S).size());
    return m;
}

// `chunks` contiguous pieces of [0, m), each a whole number of strips of S
// rows (a chunk never splits a strip, so a paper-mode strip's rows and halo
// are traced by one launch), of decreasing size: weights chunks, chunks-1,
// ..., 1 (4 chunks: 40/30/20/10 %).  Chunk k is gathered while chunk k+1 is
// traced, so only the last, smallest chunk's gather is exposed.
std::vector<std::pair<int, int>> chunk_bounds(int m, int chunks, int S = 1) {
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
    hipEvent_t ev_alt = nullptr;              // end of alt_st's work in a frame (joined into st)
    hipEvent_t ev_tb[2 * kChunks] = {};
    std::vector<int32_t> rowtab_host;          // source of the async row-table upload
    std::mutex mu;                            // one frame at a time per rank
    DevBuf* sim_stage = nullptr;              // rt_test_render_dist_sim: shared stage, copies instead of RCCL
    bool force_collective = false;            // rt_test_dist_create_rccl1: world 1 through ncclGather
    DevBuf red;                               // rt_dist_reduce_max scratch
    bool collective() const { return world > 1 || force_collective; }
};

namespace {

int dist_init_streams(rt_dist& D) {
    if (D.comm_st) return RT_OK;
    int lo = 0, hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_TRY(hipStreamCreateWithPriority(&D.comm_st, hipStreamNonBlocking, hi));
    HIP_TRY(hipStreamCreateWithFlags(&D.alt_st, hipStreamNonBlocking));
    for (auto& e : D.ev_chunk) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : D.ev_tb) HIP_TRY(hipEventCreate(&e));
    for (auto& e : D.ev_gs) HIP_TRY(hipEventCreate(&e));
    for (auto& e : D.ev_ge) HIP_TRY(hipEventCreate(&e));
    HIP_TRY(hipEventCreateWithFlags(&D.ev_alt, hipEventDisableTiming));
    return RT_OK;
}

// One rank's part of a frame.  kind 0: FP64 frame (W*H*3 doubles); kind 1:
// toByte'd RGB8 frame (W*H*3 bytes).  out_root: the root's device output
// (ignored on other ranks).  Blocks until this rank's work (and, on the
// root, the whole frame) is complete.
int dist_frame(rt_dist& D, const rt_scene* s, int W, int H, int mode, int flags, int kind, void* out_root,
               hipStream_t st, rt_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!s) { rtamd::set_last_error("rt_render_dist: scene is NULL"); return RT_ERR_INVALID_ARG; }
    if (W <= 0 || H <= 0) { rtamd::set_last_error("rt_render_dist: W and H must be > 0"); return RT_ERR_INVALID_ARG; }
    const bool root = D.rank == 0;
    if (root && !out_root) { rtamd::set_last_error("rt_render_dist: the root needs an output buffer"); return RT_ERR_INVALID_ARG; }
    std::lock_guard<std::mutex> lk(D.mu);
    int rc = dist_init_streams(D);
    if (rc != RT_OK) return rc;
    const int S = strip_height(mode);
    const std::vector<int32_t> rows = strip_rows(H, D.world, D.rank, S);
    const int n = (int)rows.size();
    const int m = max_rows(H, D.world, S);
    const size_t row_elems = (size_t)W * 3;
    const size_t row_bytes = row_elems * (kind ? 1 : sizeof(double));
    const bool coll = D.collective();
    const auto bounds = chunk_bounds(m, coll ? kChunks : 1, S);
    const bool direct = !coll && kind == 0;   // trace straight into the caller's frame
    if (!direct) HIP_TRY(D.mine.ensure(std::max<size_t>(1, (size_t)m * row_elems * sizeof(double))));
    if (kind == 1 && coll) HIP_TRY(D.mine8.ensure(std::max<size_t>(1, (size_t)m * row_elems)));
    DevBuf& stage = D.sim_stage ? *D.sim_stage : D.stage;
    if (coll && (root || D.sim_stage)) HIP_TRY(stage.ensure((size_t)D.world * m * row_bytes));
    if (coll && root) {
        // placement table: chunk k occupies slots [world*a, world*b) as [rank][b-a]
        D.rowtab_host.assign((size_t)D.world * m, -1);
        for (int r = 0; r < D.world; ++r) {
            const std::vector<int32_t> rr = strip_rows(H, D.world, r, S);
            for (const auto& ab : bounds)
                for (int i = ab.first; i < ab.second; ++i)
                    D.rowtab_host[(size_t)D.world * ab.first + (size_t)r * (ab.second - ab.first) + (i - ab.first)] =
                        i < (int)rr.size() ? rr[i] : -1;
        }
        HIP_TRY(D.rowtab.ensure(D.rowtab_host.size() * sizeof(int32_t)));
        HIP_TRY(hipMemcpyAsync(D.rowtab.p, D.rowtab_host.data(), D.rowtab_host.size() * sizeof(int32_t),
                               hipMemcpyHostToDevice, D.comm_st));
    }
    rt_frame* f = nullptr;
    rc = rt_frame_begin(s, W, H, mode, flags, rows.data(), n, st, &f);
    if (rc != RT_OK) return rc;
    double* fb_rows = direct ? static_cast<double*>(out_root) : D.mine.as<double>();
    int n_tb = 0, n_g = 0;
    for (size_t k = 0; k < bounds.size() && rc == RT_OK; ++k) {
        const int a = bounds[k].first, b = bounds[k].second, hi = std::min(b, n);
        const hipStream_t cst = (k & 1) ? D.alt_st : st;   // chunks alternate between two streams
        if (hi > a) rc = rt_frame_trace(f, a, hi, fb_rows + (size_t)a * row_elems, cst);
        if (rc != RT_OK) break;
        if (kind == 1 && hi > a) {
            uint8_t* dst8 = coll ? D.mine8.as<uint8_t>() + (size_t)a * row_elems : static_cast<uint8_t*>(out_root);
            if (hipEventRecord(D.ev_tb[n_tb++], cst) != hipSuccess) { rc = RT_ERR_HIP; break; }
            rc = rt_framebuffer_to_rgb8_device(fb_rows + (size_t)a * row_elems, (size_t)(hi - a) * W, dst8, cst);
            if (rc != RT_OK) break;
            if (hipEventRecord(D.ev_tb[n_tb++], cst) != hipSuccess) { rc = RT_ERR_HIP; break; }
        }
        if (!coll) continue;
        // chunk k -> root: ONE collective, ordered after the chunk's trace
        if (hipEventRecord(D.ev_chunk[k], cst) != hipSuccess || hipStreamWaitEvent(D.comm_st, D.ev_chunk[k], 0) != hipSuccess) {
            rtamd::set_last_error("rt_render_dist: event chaining failed");
            rc = RT_ERR_HIP;
            break;
        }
        if (hipEventRecord(D.ev_gs[n_g], D.comm_st) != hipSuccess) { rc = RT_ERR_HIP; break; }
        const char* send = (kind ? D.mine8.as<char>() : D.mine.as<char>()) + (size_t)a * row_bytes;
        const size_t chunk_bytes = (size_t)(b - a) * row_bytes;
        char* recv = stage.as<char>() + (size_t)D.world * a * row_bytes;
        if (D.sim_stage) {
            if (hipMemcpyAsync(recv + (size_t)D.rank * chunk_bytes, send, chunk_bytes, hipMemcpyDeviceToDevice,
                               D.comm_st) != hipSuccess) {
                rtamd::set_last_error("rt_test_render_dist_sim: copy failed");
                rc = RT_ERR_HIP;
                break;
            }
        } else {
            const ncclResult_t r = ncclGather(send, root ? recv : nullptr, kind ? chunk_bytes : chunk_bytes / 8,
                                              kind ? ncclUint8 : ncclFloat64, 0, D.comm, D.comm_st);
            if (r != ncclSuccess) {
                rtamd::set_last_error(std::string("ncclGather failed: ") + ncclGetErrorString(r));
                rc = RT_ERR_HIP;
                break;
            }
        }
        if (root && place_rows(recv, D.rowtab.as<int32_t>() + (size_t)D.world * a, D.world * (b - a), row_bytes,
                               out_root, D.comm_st) != hipSuccess) {
            rtamd::set_last_error("rt_render_dist: row placement failed");
            rc = RT_ERR_HIP;
            break;
        }
        if (hipEventRecord(D.ev_ge[n_g++], D.comm_st) != hipSuccess) { rc = RT_ERR_HIP; break; }
    }
    // alt_st's last work (a chunk's toByte) into st, which rt_frame_end synchronises
    if (hipEventRecord(D.ev_alt, D.alt_st) != hipSuccess || hipStreamWaitEvent(st, D.ev_alt, 0) != hipSuccess) {
        if (rc == RT_OK) rc = RT_ERR_HIP;
    }
    const int rc_end = rt_frame_end(f, stats);   // joins and synchronises the trace streams
    if (coll && hipStreamSynchronize(D.comm_st) != hipSuccess && rc == RT_OK) {
        rtamd::set_last_error("rt_render_dist: gather stream failed");
        rc = RT_ERR_HIP;
    }
    if (rc != RT_OK) return rc;
    if (rc_end != RT_OK) return rc_end;
    if (stats) {
        float ms = 0.f;
        // the collectives and placements themselves (each waits for its
        // chunk's trace first; the waits are not counted)
        double g = 0.0;
        for (int i = 0; i < n_g; ++i)
            if (hipEventElapsedTime(&ms, D.ev_gs[i], D.ev_ge[i]) == hipSuccess) g += ms;
        stats->ms_gather = g;
        double tb = 0.0;
        for (int i = 0; i + 1 < n_tb; i += 2)
            if (hipEventElapsedTime(&ms, D.ev_tb[i], D.ev_tb[i + 1]) == hipSuccess) tb += ms;
        stats->ms_tobyte = tb;
        stats->n_gpus = D.world;
        stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return RT_OK;
}

// Everything a rank holds on its device: the communicator (if owned),
// buffers, streams and events.  The rank object itself stays valid (empty).
void release_rank(rt_dist& d) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(d.device);
    if (d.comm_st) (void)hipStreamSynchronize(d.comm_st);
    if (d.comm && d.own_comm) (void)ncclCommDestroy(d.comm);
    d.comm = nullptr;
    d.own_comm = false;
    d.mine.release();
    d.mine8.release();
    d.stage.release();
    d.rowtab.release();
    d.red.release();
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
    for (auto& e : d.ev_ge) drop(e);
    drop(d.ev_alt);
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
    return n;
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
    const std::vector<int32_t> r = strip_rows(H, world, rank, strip_height(mode));
    std::copy(r.begin(), r.end(), rows_out);
    return (int)r.size();
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
extern "C" int rt_test_render_dist_sim(const rt_scene* s, int W, int H, int mode, int flags, int world, int rgb8,
                                       double* fb_host, uint8_t* rgb8_host) {
    if (!s || W <= 0 || H <= 0 || world <= 0 || (rgb8 ? !rgb8_host : !fb_host)) return RT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
    const size_t out_bytes = (size_t)W * H * 3 * (rgb8 ? 1 : sizeof(double));
    DevBuf out, stage;
    HIP_TRY(out.ensure(out_bytes));
    HIP_TRY(hipMemset(out.p, 0xff, out_bytes));   // every byte must be written by the placement
    std::vector<std::unique_ptr<rt_dist>> ranks;
    for (int r = 0; r < world; ++r) {
        ranks.emplace_back(new rt_dist);
        ranks.back()->world = world;
        ranks.back()->rank = r;
        ranks.back()->sim_stage = world > 1 ? &stage : nullptr;
        HIP_TRY(hipGetDevice(&ranks.back()->device));
    }
    int rc = RT_OK;
    // non-root ranks first (they deposit their chunks), then the root places
    for (int r = world - 1; r >= 0 && rc == RT_OK; --r) {
        rt_stats st{};
        rc = dist_frame(*ranks[r], s, W, H, mode, flags, rgb8 ? 1 : 0, r == 0 ? out.p : nullptr, nullptr, &st);
    }
    if (rc == RT_OK && hipMemcpy(rgb8 ? (void*)rgb8_host : (void*)fb_host, out.p, out_bytes, hipMemcpyDeviceToHost) != hipSuccess)
        rc = RT_ERR_HIP;
    for (auto& d : ranks) release_rank(*d);
    stage.release();
    out.release();
    return rc;
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
    int rc = dist_init_streams(*d);
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
    HIP_TRY(hipGetDevice(&D->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    NCCL_TRY(ncclCommInitRank(&D->comm, 1, u, 0));
    D->own_comm = true;
    *out = D.release();
    return RT_OK;
}
