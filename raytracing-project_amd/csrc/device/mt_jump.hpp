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

// Host-built plan for one segment length K: the radix-8 tree's tap lists
// (exponents with coefficient 1 in x^(624*K*m*8^j) mod phi, csrc/host/
// mt_poly.cpp) and the seed window, resident on the device.
struct JitterPlan {
    int K = 0;
    int levels = 0;
    uint16_t* d_taps = nullptr;
    uint32_t* d_base = nullptr;        // window at n = 624 for seed 12345
    std::vector<int32_t> off;          // taps of (j, m) at [off[j*8+m], off[j*8+m+1]), m in 1..7
    hipError_t build(int K_blocks, int levels_needed);   // synchronous upload
    void release();
};

// Writes jit[(q - q0)/2] for even q in [q0, q1) (q0, q1 even).  d_ckpt must
// hold mt_ckpt_words(K, q1) words; plan.levels >= mt_levels_needed(K, q1).
hipError_t mt_launch_jitter(const JitterPlan& plan, int64_t q0, int64_t q1, uint32_t* d_ckpt, double* d_jit,
                            hipStream_t stream);
size_t mt_ckpt_words(int K, int64_t q1);
int mt_levels_needed(int K, int64_t q1);

}  // namespace rtamd
