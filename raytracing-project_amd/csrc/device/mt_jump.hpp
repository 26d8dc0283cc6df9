// mt_jump.hpp — launchers for the parallel mt19937 jitter stream (mt_jump.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtamd {

// Writes jit[(q - q0)/2] for even q in [q0, q1) (q0, q1 even).  d_ckpt must
// hold mt_num_checkpoints(K, q1) * 624 words.  d_taps holds, for level j,
// the exponents i with coefficient 1 in P_j = x^(624*K*2^j) mod phi at
// [tap_off[j], tap_off[j+1]) (tap_off is a HOST array of levels+1 entries).
hipError_t mt_launch_jitter(const uint32_t* d_base_win, const uint32_t* d_taps, const int32_t* tap_off, int levels,
                            int K, int64_t q0, int64_t q1, uint32_t* d_ckpt, double* d_jit, hipStream_t stream);
int64_t mt_num_checkpoints(int K, int64_t q1);
int mt_levels_needed(int K, int64_t q1);

}  // namespace rtamd
