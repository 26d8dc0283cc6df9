// mt_jump.hip — parallel generation of the reference's jitter stream.
//
// The reference consumes ONE serial std::mt19937(12345) stream through
// uniform_real_distribution<double>(-0.5,0.5) (raytracer/src/tracer.cpp:
// 284-293; libstdc++ generate_canonical, random.tcc:3348-3378).  Here the
// stream is cut into segments of K twist blocks.  Kernel 1 jumps the
// generator to every segment start (GF(2) jump polynomials from
// csrc/host/mt_poly.cpp: window' = XOR_i p_i * window shifted by i); kernel 2
// regenerates each segment sequentially inside one workgroup (the twist is
// split into its three dependent phases of 227/227/170 words) and writes the
// jitter doubles.  Output: jit[(q - q0)/2] = uniform(w_q, w_{q+1}) for every
// even output index q in [q0, q1).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mt_jump.hpp"

namespace {

constexpr int N = 624;
constexpr int DEG = 19937;
constexpr int JUMP_BUF = DEG + N;           // raw words w_n .. w_{n+DEG+N-1}
constexpr int JUMP_THREADS = 640;
constexpr int FILL_THREADS = 320;

__device__ __forceinline__ uint32_t twist_word(uint32_t wk, uint32_t wk1, uint32_t wk397) {
    const uint32_t y = (wk & 0x80000000u) | (wk1 & 0x7fffffffu);
    return wk397 ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// generate_canonical<double,53> over two outputs, then
// uniform_real_distribution(-0.5,0.5): (u * (b - a)) + a (random.h:1870).
__device__ __forceinline__ double jitter_from(uint32_t w0, uint32_t w1) {
    double sum = 0.0;
    sum += (double)w0 * 1.0;
    sum += (double)w1 * 4294967296.0;
    double ret = sum / 18446744073709551616.0;
    if (ret >= 1.0) ret = 0x1.fffffffffffffp-1;   // nextafter(1, 0)
    return (ret * (0.5 - -0.5)) + -0.5;
}

// Generate buf[N .. N + 624*nblocks) from the window in buf[0..N) with the
// three-phase twist (phase 2 reads phase-1 outputs through the +397 tap).
__device__ __forceinline__ void twist_blocks(uint32_t* buf, int nblocks, int limit) {
    for (int b = 0; b < nblocks; ++b) {
        uint32_t* w = buf + b * N;
        for (int j = threadIdx.x; j < 227; j += blockDim.x)
            if (N + b * N + j < limit) w[N + j] = twist_word(w[j], w[j + 1], w[j + 397]);
        __syncthreads();
        for (int j = 227 + threadIdx.x; j < 454; j += blockDim.x)
            if (N + b * N + j < limit) w[N + j] = twist_word(w[j], w[j + 1], w[j + 397]);
        __syncthreads();
        for (int j = 454 + threadIdx.x; j < N; j += blockDim.x)
            if (N + b * N + j < limit) w[N + j] = twist_word(w[j], w[j + 1], w[j + 397]);
        __syncthreads();
    }
}

// One workgroup per segment: window(c) = jumps for every set bit of c applied
// to the base window (outputs 0..623).
__global__ __launch_bounds__(JUMP_THREADS) void k_mt_jump(const uint32_t* __restrict__ base_win,
                                                          const uint32_t* __restrict__ polys, int levels,
                                                          int64_t c0, uint32_t* __restrict__ ckpt) {
    __shared__ uint32_t buf[JUMP_BUF + 8];
    const int64_t c = c0 + blockIdx.x;
    const int tid = threadIdx.x;
    uint32_t win = (tid < N) ? base_win[tid] : 0u;
    for (int k = 0; k < levels; ++k) {
        if (!((c >> k) & 1)) continue;   // wave-uniform
        if (tid < N) buf[tid] = win;
        __syncthreads();
        twist_blocks(buf, (JUMP_BUF - N + N - 1) / N, JUMP_BUF);
        // correlation: out[j] = XOR_{i: p_i = 1} w[i + j]
        const uint32_t* P = polys + (size_t)k * N;
        uint32_t acc = 0;
        if (tid < N) {
            for (int wi = 0; wi < N; ++wi) {
                uint32_t bits = P[wi];   // uniform -> scalar load
                const uint32_t* src = buf + wi * 32 + tid;
                while (bits) {
                    const int b = __builtin_ctz(bits);
                    acc ^= src[b];
                    bits &= bits - 1u;
                }
            }
        }
        __syncthreads();
        win = acc;
    }
    if (tid < N) ckpt[(size_t)blockIdx.x * N + tid] = win;
}

// One workgroup per segment: regenerate K blocks from the checkpoint and
// write jitter for outputs in [q0, q1).
__global__ __launch_bounds__(FILL_THREADS) void k_mt_fill(const uint32_t* __restrict__ ckpt, int K, int64_t c0,
                                                          int64_t q0, int64_t q1, double* __restrict__ jit) {
    __shared__ uint32_t buf[2 * N + 8];
    const int tid = threadIdx.x;
    for (int j = tid; j < N; j += blockDim.x) buf[j] = ckpt[(size_t)blockIdx.x * N + j];
    __syncthreads();
    const int64_t seg_q = (c0 + blockIdx.x) * (int64_t)K * N;
    for (int b = 0; b < K; ++b) {
        const int64_t bq = seg_q + (int64_t)b * N;   // output index of buf[0]
        if (bq >= q1) break;                          // uniform
        if (bq + N > q0) {
            for (int i = tid; i < N / 2; i += blockDim.x) {
                const int64_t q = bq + 2 * i;
                if (q >= q0 && q < q1)
                    jit[(q - q0) >> 1] = jitter_from(temper(buf[2 * i]), temper(buf[2 * i + 1]));
            }
        }
        if (b + 1 < K && bq + N < q1) {
            twist_blocks(buf, 1, 2 * N);
            for (int j = tid; j < N; j += blockDim.x) buf[j] = buf[N + j];
            __syncthreads();
        }
    }
}

}  // namespace

namespace rtamd {

hipError_t mt_launch_jitter(const uint32_t* d_base_win, const uint32_t* d_polys, int levels, int K,
                            int64_t q0, int64_t q1, uint32_t* d_ckpt, double* d_jit, hipStream_t stream) {
    if (q1 <= q0) return hipSuccess;
    const int64_t seg = (int64_t)K * N;
    const int64_t c0 = q0 / seg, c1 = (q1 - 1) / seg;
    const int64_t nseg = c1 - c0 + 1;
    hipLaunchKernelGGL(k_mt_jump, dim3((unsigned)nseg), dim3(JUMP_THREADS), 0, stream, d_base_win, d_polys, levels,
                       c0, d_ckpt);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_mt_fill, dim3((unsigned)nseg), dim3(FILL_THREADS), 0, stream, d_ckpt, K, c0, q0, q1, d_jit);
    return hipGetLastError();
}

int64_t mt_num_segments(int K, int64_t q0, int64_t q1) {
    if (q1 <= q0) return 0;
    const int64_t seg = (int64_t)K * N;
    return (q1 - 1) / seg - q0 / seg + 1;
}

int mt_levels_needed(int K, int64_t q1) {
    const int64_t seg = (int64_t)K * N;
    int64_t cmax = q1 > 0 ? (q1 - 1) / seg : 0;
    int L = 0;
    while ((cmax >> L) > 0) ++L;
    return L < 1 ? 1 : L;
}

}  // namespace rtamd
