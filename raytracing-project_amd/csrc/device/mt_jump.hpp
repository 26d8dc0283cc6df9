// mt_jump.hpp — the parallel mt19937 jitter stream (mt_jump.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace rtamd {

// Checkpoint c (segment c of K twist blocks) is stored as up to kMTParts
// partial windows whose XOR is the window: a jump is split across several
// workgroups by tap ranges, each writing its own partial.
constexpr int kMTParts = 8;
constexpr int kMTMaxLevels = 8;

// Host-built plan for one segment length K: the radix-64 tree's tap lists
// (exponents with coefficient 1 in x^(624*K*m*64^j) mod phi, csrc/host/
// mt_poly.cpp) and the seed window, resident on the device.
struct JitterPlan {
    int K = 0;
    int levels = 0;
    uint16_t* d_taps = nullptr;
    uint32_t* d_base = nullptr;        // window at n = 624 for seed 12345
    std::vector<int32_t> off;          // taps of (j, m) at [off[j*R+m], off[j*R+m+1]), m in 1..R-1
    // Uploads the taps and the seed window on `stream` from page-locked
    // staging (h_stage: freed by drop_stage() once the stream has passed the
    // copies).  A pageable synchronous copy of the ~4.6 MB of taps took ~7.6
    // ms of the CLI's one-time setup (profiles/r06c_cli_prof.txt).
    hipError_t build(int K_blocks, int levels_needed, hipStream_t stream);
    void* h_stage = nullptr;
    void drop_stage();
    void release();
};

// A run of stream outputs: the draw made of outputs q, q+1 (q even, in
// [qa, qb)) is stored at jit[dst + (q - qa)/2].  Ranges passed to the
// launcher are sorted by qa and disjoint.  A rendered loop row y of width W
// is the range [32*W*y, 32*W*(y+1)) (tracer.cpp:284-293: 8 samples x 2
// draws x 2 words).
struct JRange {
    int64_t qa, qb, dst;
};

// mt19937 tempering (libstdc++ random.tcc operator()).
__host__ __device__ __forceinline__ uint32_t mt_temper_word(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// One jitter draw from two raw (untempered) words: tempering, generate_canonical<double,
// 53> over the two outputs (random.tcc:3348-3378), then
// uniform_real_distribution(-0.5, 0.5): (u * (b - a)) + a (random.h:1870).
// Callers compile without FP contraction, so every step rounds as on x86-64.
__host__ __device__ __forceinline__ double jitter_draw(uint32_t raw0, uint32_t raw1) {
    double sum = 0.0;
    sum += (double)mt_temper_word(raw0) * 1.0;
    sum += (double)mt_temper_word(raw1) * 4294967296.0;
    double ret = sum / 18446744073709551616.0;
    if (ret >= 1.0) ret = 0x1.fffffffffffffp-1;   // nextafter(1, 0)
    return (ret * (0.5 - -0.5)) + -0.5;
}

// Host-side state of one launch: device lists (segments to regenerate,
// checkpoints per tree level, ranges) are staged here and uploaded into the
// caller's device scratch; the host copy stays alive until the stream is
// synchronised.
struct PinnedArena;
struct JitterJob {
    std::vector<char> stage;
    int64_t qmax = 0;
    PinnedArena* up = nullptr;   // page-locked staging of the job's upload (pinned.hpp), if set
};

// Only the checkpoints the requested ranges need are computed (the needed
// segments and their tree ancestors) and only the segments that overlap a
// range are regenerated, so a rank rendering 1/N of the rows does ~1/N of
// the jump work.  d_scratch must hold mt_scratch_bytes(ranges) bytes, d_ckpt
// mt_ckpt_words(K, qmax) words; plan.levels >= mt_levels_needed(K, qmax).
hipError_t mt_launch_jitter(const JitterPlan& plan, const std::vector<JRange>& ranges, JitterJob& job,
                            void* d_scratch, uint32_t* d_ckpt, double* d_jit, hipStream_t stream);
size_t mt_scratch_bytes(int K, const std::vector<JRange>& ranges);
size_t mt_ckpt_words(int K, int64_t q1);
int mt_levels_needed(int K, int64_t q1);

// Checkpoint table: the generator's window at every kTableK-th twist block
// from the start of the stream, i.e. constants of std::mt19937(12345) in the
// same sense as the jump polynomials.  Computed once per device with the
// GF(2) jump tree (k_mt_jump, on first use and again only when a frame needs
// checkpoints beyond the table) and kept resident; every frame then
// regenerates ALL of its jitter draws from it (k_mt_fill_w: one wavefront
// per kTableK-block segment, no per-frame jumps).
// 16 twist blocks per segment: the fill's floor is one wave's sequential walk
// through a segment, so shorter segments cut a rank's jitter time at N > 1
// (8-rank share of config 4: 0.174 -> 0.086 ms) at 4x the table (66 MB for
// a 4K frame, built once per device).  bin/mt_polygen writes the tree
// polynomials for this K (tests/test_mt_poly_file.py keeps the two in step).
#ifndef RT_TABLE_K
#define RT_TABLE_K 16
#endif
constexpr int kTableK = RT_TABLE_K;   // (RT_TABLE_K: measurement A/B; lib/mt19937_tree.polys must be written for it)
struct JitterTable {
    JitterPlan plan;                  // K = kTableK
    uint32_t* d_table = nullptr;      // [cap][624] windows
    int64_t n_ck = 0, cap = 0;        // checkpoints present / allocated
    float ms_last_build = 0.f;        // device time of the last extension (diagnostics)
    hipError_t ensure(int64_t n_need, hipStream_t stream);   // synchronous when it grows
    void release();
};
// Host-only: the checkpoint tree's tap lists for every level the shipped
// polynomial file holds, cached for the process (rt_warmup RT_WARM_HOST runs
// it on a helper thread while the caller initialises HIP).
void mt_prefetch_host_taps();
// Scratch for mt_launch_fill's segment/range lists.
size_t mt_fill_scratch_bytes(const std::vector<JRange>& ranges);
// Regenerate the draws of `ranges` from the table (table.ensure must cover them).
hipError_t mt_launch_fill(const JitterTable& T, const std::vector<JRange>& ranges, JitterJob& job, void* d_scratch,
                          double* d_jit, hipStream_t stream);

}  // namespace rtamd
