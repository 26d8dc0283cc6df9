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

#include <algorithm>

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

// Tree doubling, level j: ckpt[c] = jump(ckpt[c - 2^j]) by x^(624*K*2^j) for
// c in [lo, lo + gridDim.x).  The jump is the correlation
// out[j] = XOR_{i in taps} w[i + j] over the raw words regenerated from the
// source window; taps = exponents with a 1 coefficient (host-built list,
// staged in LDS as 16-bit offsets and read 8 at a time by broadcast).
constexpr int MAX_TAPS = DEG + 8;
__global__ __launch_bounds__(JUMP_THREADS) void k_mt_jump_level(const uint32_t* __restrict__ taps, int ntaps,
                                                                int64_t lo, int64_t stride,
                                                                uint32_t* __restrict__ ckpt) {
    __shared__ uint32_t buf[JUMP_BUF + 8];
    __shared__ __attribute__((aligned(16))) uint16_t tp[MAX_TAPS];
    const int64_t c = lo + blockIdx.x;
    const int tid = threadIdx.x;
    for (int j = tid; j < N; j += blockDim.x) buf[j] = ckpt[(size_t)(c - stride) * N + j];
    const int n8 = ntaps & ~7;
    for (int i = tid; i < ntaps; i += blockDim.x) tp[i] = (uint16_t)taps[i];
    __syncthreads();
    twist_blocks(buf, (JUMP_BUF - 1) / N, JUMP_BUF);
    if (tid < N) {
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        const uint32_t* src = buf + tid;
        for (int i = 0; i < n8; i += 8) {
            const uint4 q = *reinterpret_cast<const uint4*>(tp + i);   // uniform address: broadcast
            a0 ^= src[q.x & 0xffffu];
            a1 ^= src[q.x >> 16];
            a2 ^= src[q.y & 0xffffu];
            a3 ^= src[q.y >> 16];
            a0 ^= src[q.z & 0xffffu];
            a1 ^= src[q.z >> 16];
            a2 ^= src[q.w & 0xffffu];
            a3 ^= src[q.w >> 16];
        }
        for (int i = n8; i < ntaps; ++i) a0 ^= src[tp[i]];
        ckpt[(size_t)c * N + tid] = a0 ^ a1 ^ a2 ^ a3;
    }
}

// One workgroup per segment: regenerate K blocks from the checkpoint and
// write jitter for outputs in [q0, q1).  buf is a 2-block ring: the block at
// offset `base` is converted to jitter while the first twist phase of the
// next block (written at base + 624, mod 1248) runs; no copies.
__global__ __launch_bounds__(FILL_THREADS) void k_mt_fill(const uint32_t* __restrict__ ckpt, int K, int64_t c0,
                                                          int64_t q0, int64_t q1, double* __restrict__ jit) {
    __shared__ uint32_t buf[2 * N];
    const int tid = threadIdx.x;
    for (int j = tid; j < N; j += blockDim.x) buf[j] = ckpt[(size_t)(c0 + blockIdx.x) * N + j];
    __syncthreads();
    const int64_t seg_q = (c0 + blockIdx.x) * (int64_t)K * N;
    int base = 0;
    for (int b = 0; b < K; ++b) {
        const int64_t bq = seg_q + (int64_t)b * N;   // output index of the block at `base`
        if (bq >= q1) break;                          // uniform
        const bool more = b + 1 < K && bq + N < q1;   // uniform
        const int nb = base ^ N;                      // ring slot of the next block (0 <-> 624)
        auto R = [&](int k) { return buf[(base + k) % (2 * N)]; };
        // phase 1 of the next block + conversion of this block
        if (more)
            for (int j = tid; j < 227; j += blockDim.x) buf[nb + j] = twist_word(R(j), R(j + 1), R(j + 397));
        if (bq + N > q0) {
            for (int i = tid; i < N / 2; i += blockDim.x) {
                const int64_t q = bq + 2 * i;
                if (q >= q0 && q < q1) jit[(q - q0) >> 1] = jitter_from(temper(R(2 * i)), temper(R(2 * i + 1)));
            }
        }
        __syncthreads();
        if (more) {
            for (int j = 227 + tid; j < 454; j += blockDim.x) buf[nb + j] = twist_word(R(j), R(j + 1), R(j + 397));
            __syncthreads();
            for (int j = 454 + tid; j < N; j += blockDim.x) buf[nb + j] = twist_word(R(j), R(j + 1), R(j + 397));
            __syncthreads();
        }
        base = nb;
    }
}

}  // namespace

namespace rtamd {

hipError_t mt_launch_jitter(const uint32_t* d_base_win, const uint32_t* d_taps, const int32_t* tap_off, int levels,
                            int K, int64_t q0, int64_t q1, uint32_t* d_ckpt, double* d_jit, hipStream_t stream) {
    if (q1 <= q0) return hipSuccess;
    const int64_t seg = (int64_t)K * N;
    const int64_t c0 = q0 / seg, c1 = (q1 - 1) / seg;
    hipError_t e = hipMemcpyAsync(d_ckpt, d_base_win, N * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) return e;
    for (int j = 0; j < levels; ++j) {
        const int64_t lo = (int64_t)1 << j;
        if (lo > c1) break;
        const int64_t hi = std::min<int64_t>((int64_t)2 << j, c1 + 1);
        hipLaunchKernelGGL(k_mt_jump_level, dim3((unsigned)(hi - lo)), dim3(JUMP_THREADS), 0, stream,
                           d_taps + tap_off[j], tap_off[j + 1] - tap_off[j], lo, lo, d_ckpt);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_mt_fill, dim3((unsigned)(c1 - c0 + 1)), dim3(FILL_THREADS), 0, stream, d_ckpt, K, c0, q0,
                       q1, d_jit);
    return hipGetLastError();
}

int64_t mt_num_checkpoints(int K, int64_t q1) {
    if (q1 <= 0) return 1;
    return (q1 - 1) / ((int64_t)K * N) + 1;
}

int mt_levels_needed(int K, int64_t q1) {
    const int64_t seg = (int64_t)K * N;
    int64_t cmax = q1 > 0 ? (q1 - 1) / seg : 0;
    int L = 0;
    while ((cmax >> L) > 0) ++L;
    return L < 1 ? 1 : L;
}

}  // namespace rtamd
