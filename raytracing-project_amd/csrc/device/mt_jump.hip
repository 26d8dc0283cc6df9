// mt_jump.hip — parallel generation of the reference's jitter stream.
//
// The reference consumes ONE serial std::mt19937(12345) stream through
// uniform_real_distribution<double>(-0.5,0.5) (raytracer/src/tracer.cpp:
// 284-293; libstdc++ generate_canonical, random.tcc:3348-3378).  Here the
// stream is cut into segments of K twist blocks.  k_mt_jump computes the
// window at every segment start with a radix-64 tree of GF(2) jumps
// (csrc/host/mt_poly.cpp: window' = XOR_i p_i * window shifted by i), each
// jump split over S workgroups by tap ranges; k_mt_fill regenerates every
// segment inside one workgroup and writes the jitter doubles.  Output:
// jit[(q - q0)/2] = uniform(w_q, w_{q+1}) for every even output index q in
// [q0, q1).
//
// Twist with one barrier per block: thread t < 227 owns words t, 227+t and
// 454+t of the new block.  Word 227+t reads new word t through the +397 tap
// and word 454+t reads new word 227+t, so both come from the same thread's
// registers; only word 623 needs new word 0 (its +1 neighbour), which
// thread 169 recomputes.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <memory>
#include <mutex>
#include <string>
#include <stdint.h>

#include <algorithm>
#include <cstring>

#include "mt_jump.hpp"
#include "pinned.hpp"
#include "mt_poly.hpp"

namespace {

constexpr int N = 624;
constexpr int DEG = 19937;
constexpr int JUMP_BUF = DEG + N;   // raw words w_n .. w_{n+DEG+N-1}
constexpr int JUMP_THREADS = 320;   // 312 correlation lanes x 2 outputs
// k_mt_fill roles: waves 0-3 twist the next block (227 lanes), waves 4-8
// convert the current one (312 output pairs, one per lane), so the two
// latency chains of a block overlap instead of running back to back.
constexpr int FILL_TWIST = 256;
constexpr int FILL_THREADS = FILL_TWIST + 320;
constexpr int MAX_LEVELS = rtamd::kMTMaxLevels;

__device__ __forceinline__ uint32_t twist_word(uint32_t wk, uint32_t wk1, uint32_t wk397) {
    const uint32_t y = (wk & 0x80000000u) | (wk1 & 0x7fffffffu);
    return wk397 ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// One twist block: nw[0..N) from the previous block o[0..N) (disjoint LDS
// ranges).  Called by every thread; words at index >= lim are not stored.
__device__ __forceinline__ void twist_block(const uint32_t* o, uint32_t* nw, int lim) {
    const int t = threadIdx.x;
    if (t < 227) {
        const uint32_t n0 = twist_word(o[t], o[t + 1], o[t + 397]);
        const uint32_t n1 = twist_word(o[227 + t], o[228 + t], n0);
        if (t < lim) nw[t] = n0;
        if (227 + t < lim) nw[227 + t] = n1;
        if (t < 170) {
            const uint32_t nx = (t == 169) ? twist_word(o[0], o[1], o[397]) : o[455 + t];
            const uint32_t n2 = twist_word(o[454 + t], nx, n1);
            if (454 + t < lim) nw[454 + t] = n2;
        }
    }
}

// Workgroup barrier ordering LDS only.  __syncthreads() also orders global
// memory, i.e. waits for the jitter stores of the iteration to complete,
// which put an HBM write round trip into every twist block of k_mt_fill.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ int ckpt_parts(int64_t c, const int8_t* parts) {
    if (c == 0) return 1;
    const int j = (63 - __builtin_clzll((unsigned long long)c)) / rtamd::kMTRadixBits;   // c in [R^j, R^(j+1))
    return parts[j];
}

struct JumpArgs {
    int64_t div;                // partial-window slot of checkpoint c: c / div (1, or R for the coarse table tree)
    int64_t lo;                 // R^j: this level computes checkpoints in [lo, R*lo)
    const int64_t* list;        // the checkpoints of this level to compute (gridDim.x of them)
    int S;                      // partial jumps per checkpoint (gridDim.y)
    int32_t off[rtamd::kMTRadix], len[rtamd::kMTRadix];   // tap slice of x^(624*K*m*R^j), m = c / lo
    int8_t parts[MAX_LEVELS];   // partial count of the checkpoints of every level
};

// Tree level j: ckpt[c] = jump(ckpt[c - m*lo]) by x^(624*K*m*lo), partial
// s of S over the taps [s*len/S, (s+1)*len/S).  The jump is the correlation
// out[k] = XOR_{i in taps} w[i + k] over the raw words regenerated from the
// source window; taps are staged in LDS as 16-bit exponents and read 8 at a
// time by broadcast.
constexpr int MAX_TAPS = DEG + 8;
__global__ __launch_bounds__(JUMP_THREADS) void k_mt_jump(const uint16_t* __restrict__ taps, JumpArgs A,
                                                          uint32_t* __restrict__ ckpt) {
    __shared__ uint32_t buf[JUMP_BUF + 8];
    __shared__ __attribute__((aligned(16))) uint16_t tp[MAX_TAPS];
    const int64_t c = A.list[blockIdx.x];
    const int s = blockIdx.y;
    const int m = (int)(c / A.lo);
    const int64_t r = c - (int64_t)m * A.lo;
    const int tid = threadIdx.x;
    const int np = ckpt_parts(r, A.parts);
    for (int k = tid; k < N; k += blockDim.x) {
        uint32_t v = 0;
        for (int p = 0; p < np; ++p) v ^= ckpt[((size_t)(r / A.div) * rtamd::kMTParts + p) * N + k];
        buf[k] = v;
    }
    const int n_all = A.len[m];
    const int t0 = (int)((int64_t)s * n_all / A.S), t1 = (int)((int64_t)(s + 1) * n_all / A.S);
    const int ntaps = t1 - t0;
    const uint16_t* src_taps = taps + A.off[m] + t0;
    for (int i = tid; i < ntaps; i += blockDim.x) tp[i] = src_taps[i];
    __syncthreads();
    for (int b = N; b < JUMP_BUF; b += N) {
        twist_block(buf + b - N, buf + b, JUMP_BUF - b);
        lds_barrier();
    }
    if (tid < N / 2) {
        uint32_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
        const uint32_t* sa = buf + tid;
        const uint32_t* sb = buf + tid + N / 2;
        const int n8 = ntaps & ~7;
        for (int i = 0; i < n8; i += 8) {
            const uint4 q = *reinterpret_cast<const uint4*>(tp + i);   // uniform address: broadcast
            const uint32_t e0 = q.x & 0xffffu, e1 = q.x >> 16, e2 = q.y & 0xffffu, e3 = q.y >> 16;
            const uint32_t e4 = q.z & 0xffffu, e5 = q.z >> 16, e6 = q.w & 0xffffu, e7 = q.w >> 16;
            a0 ^= sa[e0]; b0 ^= sb[e0];
            a1 ^= sa[e1]; b1 ^= sb[e1];
            a0 ^= sa[e2]; b0 ^= sb[e2];
            a1 ^= sa[e3]; b1 ^= sb[e3];
            a0 ^= sa[e4]; b0 ^= sb[e4];
            a1 ^= sa[e5]; b1 ^= sb[e5];
            a0 ^= sa[e6]; b0 ^= sb[e6];
            a1 ^= sa[e7]; b1 ^= sb[e7];
        }
        for (int i = n8; i < ntaps; ++i) {
            a0 ^= sa[tp[i]];
            b0 ^= sb[tp[i]];
        }
        uint32_t* out = ckpt + ((size_t)(c / A.div) * rtamd::kMTParts + s) * N;
        out[tid] = a0 ^ a1;
        out[tid + N / 2] = b0 ^ b1;
    }
}

struct FillArgs {
    int K;
    int nr;                      // number of ranges
    const rtamd::JRange* R;      // sorted, disjoint output ranges
    const int64_t* segs;         // per workgroup: (segment c, first range overlapping it)
    int8_t parts[MAX_LEVELS];
    // k_mt_fill_w with ONE range (a whole frame, or one strip): segs = R =
    // nullptr, the range travels here and workgroup b takes segment c0 + b -
    // nothing to upload before the fill
    rtamd::JRange one;
    int64_t c0;
};

// Where the draws of one block go: output pair i (outputs bq+2i, bq+2i+1)
// is stored at p0[i] for i in [a0, b0) and at p1[i] for i in [a1, b1)
// (block-uniform); rows narrower than 20 pixels put more than two ranges
// into a block and take the generic path.
struct BlockDst {
    double* p0;
    double* p1;
    int a0, b0, a1, b1;
    bool generic;
};

__device__ __forceinline__ int clampP(int64_t v) { return v < 0 ? 0 : v > N / 2 ? N / 2 : (int)v; }

__device__ __forceinline__ BlockDst block_dst(double* jit, int64_t bq, const rtamd::JRange& g0,
                                              const rtamd::JRange& g1, int r, int nr) {
    BlockDst d;
    d.a0 = clampP((g0.qa - bq) >> 1);
    d.b0 = clampP((g0.qb - bq) >> 1);
    d.a1 = clampP((g1.qa - bq) >> 1);
    d.b1 = clampP((g1.qb - bq) >> 1);
    d.p0 = jit + (g0.dst - ((g0.qa - bq) >> 1));
    d.p1 = jit + (g1.dst - ((g1.qa - bq) >> 1));
    d.generic = g1.qb - bq < N && r + 2 < nr;
    return d;
}

__device__ __forceinline__ int64_t generic_dst(int64_t q, const FillArgs& A, int r) {
    for (int k = r; k < A.nr && q >= A.R[k].qa; ++k)
        if (q < A.R[k].qb) return A.R[k].dst + ((q - A.R[k].qa) >> 1);
    return -1;
}

// generate_canonical<double,53> over two tempered outputs, then
// uniform_real_distribution(-0.5,0.5) (mt_jump.hpp jitter_draw).
__device__ __forceinline__ double jitter_from(uint32_t raw0, uint32_t raw1) { return rtamd::jitter_draw(raw0, raw1); }

// One workgroup per needed segment: regenerate its blocks from the
// checkpoint and write the jitter of every output that falls in a range.
// Blocks live in a 2-block LDS ring with one barrier per block: while the
// twist waves compute block b+1 from block b, the convert waves turn block b
// into draws and store them.  The range cursor r is workgroup-uniform (scalar registers).
__global__ __launch_bounds__(FILL_THREADS) void k_mt_fill(const uint32_t* __restrict__ ckpt, FillArgs A,
                                                          double* __restrict__ jit) {
    __shared__ uint32_t buf[2 * N];
    const int tid = threadIdx.x;
    const int64_t c = A.segs[2 * blockIdx.x];
    int r = (int)A.segs[2 * blockIdx.x + 1];
    const int np = ckpt_parts(c, A.parts);
    const int64_t seg_q = c * (int64_t)A.K * N;
    const int64_t q_last = A.R[A.nr - 1].qb;
    // ranges r and r+1 cached in scalar registers
    rtamd::JRange g0 = A.R[r];
    rtamd::JRange g1 = r + 1 < A.nr ? A.R[r + 1] : rtamd::JRange{q_last, q_last, 0};
    for (int k = tid; k < N; k += blockDim.x) {   // block 0 = the checkpoint window
        uint32_t v = 0;
        for (int p = 0; p < np; ++p) v ^= ckpt[((size_t)c * rtamd::kMTParts + p) * N + k];
        buf[k] = v;
    }
    __syncthreads();
    int base = 0;   // ring slot of block b
    for (int b = 0; b < A.K; ++b) {
        const int64_t bq = seg_q + (int64_t)b * N;   // first output fed by block b
        if (bq >= q_last) break;
        while (g0.qb <= bq) {                         // uniform
            if (++r >= A.nr) break;
            g0 = g1;
            g1 = r + 1 < A.nr ? A.R[r + 1] : rtamd::JRange{q_last, q_last, 0};
        }
        if (r >= A.nr) break;
        const uint32_t* o = buf + base;
        if (tid < FILL_TWIST) {
            if (b + 1 < A.K && bq + N < q_last) twist_block(o, buf + (base ^ N), N);
        } else if (g0.qa < bq + N) {
            const int i = tid - FILL_TWIST;   // output pair i of the block
            if (i < N / 2) {
                const BlockDst d = block_dst(jit, bq, g0, g1, r, A.nr);
                double* dst = nullptr;
                if (d.generic) {
                    const int64_t q = generic_dst(bq + 2 * i, A, r);
                    if (q >= 0) dst = jit + q;
                } else if (i >= d.a0 && i < d.b0) {
                    dst = d.p0 + i;
                } else if (i >= d.a1 && i < d.b1) {
                    dst = d.p1 + i;
                }
                if (dst) *dst = jitter_from(o[2 * i], o[2 * i + 1]);
            }
        }
        lds_barrier();
        base ^= N;
    }
}

int level_parts(int64_t n_level) {
    const int64_t want = (512 + n_level - 1) / n_level;
    return (int)std::min<int64_t>(rtamd::kMTParts, std::max<int64_t>(1, want));
}

// Level of checkpoint c >= 1 in the radix-R tree and its parent.
inline int ckpt_level(int64_t c) { return (63 - __builtin_clzll((unsigned long long)c)) / rtamd::kMTRadixBits; }
inline int64_t ckpt_parent(int64_t c) {
    const int64_t lo = (int64_t)1 << (rtamd::kMTRadixBits * ckpt_level(c));
    return c - (c / lo) * lo;
}

// Table expansion: ONE wavefront per coarse checkpoint c' (window at table
// entry R*c', from the jump tree's partial windows) walks the stream forward
// sequentially and stores the window at every kTableK-th block, i.e. table
// entries R*c' .. R*c' + R-1 (< n).  Sequential twisting of R*kTableK blocks
// per wave replaces R-1 GF(2) jumps of ~10^4 taps each.
__global__ __launch_bounds__(64) void k_mt_expand(const uint32_t* __restrict__ ckpt, JumpArgs A, int64_t n,
                                                  uint32_t* __restrict__ table) {
    __shared__ uint32_t buf[2 * N];
    const int lane = threadIdx.x;
    const int64_t cc = blockIdx.x;               // coarse slot
    const int64_t c0 = cc * rtamd::kMTRadix;     // its table entry
    const int np = ckpt_parts(c0, A.parts);
    for (int k = lane; k < N; k += 64) {
        uint32_t v = 0;
        for (int p = 0; p < np; ++p) v ^= ckpt[((size_t)cc * rtamd::kMTParts + p) * N + k];
        buf[k] = v;
    }
    lds_barrier();
    int base = 0;
    for (int e = 0; e < rtamd::kMTRadix && c0 + e < n; ++e) {
        uint32_t* dst = table + (size_t)(c0 + e) * N;
        for (int k = lane; k < N; k += 64) dst[k] = buf[base + k];
        if (e + 1 == rtamd::kMTRadix || c0 + e + 1 >= n) break;
        for (int b = 0; b < rtamd::kTableK; ++b) {   // advance one segment
            const uint32_t* o = buf + base;
            uint32_t* nw = buf + (base ^ N);
            for (int t = lane; t < 227; t += 64) {
                const uint32_t n0 = twist_word(o[t], o[t + 1], o[t + 397]);
                const uint32_t n1 = twist_word(o[227 + t], o[228 + t], n0);
                nw[t] = n0;
                nw[227 + t] = n1;
                if (t < 170) {
                    const uint32_t nx = (t == 169) ? twist_word(o[0], o[1], o[397]) : o[455 + t];
                    nw[454 + t] = twist_word(o[454 + t], nx, n1);
                }
            }
            lds_barrier();
            base ^= N;
        }
    }
}

// Workgroup = ONE wavefront per segment of kTableK blocks.  The segment's
// window comes from the checkpoint table; per block the wave converts the
// current block into draws (312 output pairs, ~5 per lane) and twists the
// next block into the other half of a 2-block LDS ring (227 lanes' worth of
// the three-word recurrence, ~4 per lane).  A single wave needs no
// workgroup barrier, only LDS ordering, so blocks follow each other at the
// wave's instruction rate and many segments share a SIMD.
constexpr int FILLW_THREADS = 64;
__global__ __launch_bounds__(FILLW_THREADS) void k_mt_fill_w(const uint32_t* __restrict__ table, FillArgs A,
                                                             double* __restrict__ jit) {
    __shared__ uint32_t buf[2 * N];
    const int lane = threadIdx.x;
    const bool one = A.segs == nullptr;   // (kernel-uniform)
    const int64_t c = one ? A.c0 + blockIdx.x : A.segs[2 * blockIdx.x];
    int r = one ? 0 : (int)A.segs[2 * blockIdx.x + 1];
    const int64_t seg_q = c * (int64_t)A.K * N;
    const int64_t q_last = one ? A.one.qb : A.R[A.nr - 1].qb;
    rtamd::JRange g0 = one ? A.one : A.R[r];
    rtamd::JRange g1 = !one && r + 1 < A.nr ? A.R[r + 1] : rtamd::JRange{q_last, q_last, 0};
    for (int k = lane; k < N; k += FILLW_THREADS) buf[k] = table[(size_t)c * N + k];
    lds_barrier();
    int base = 0;
    for (int b = 0; b < A.K; ++b) {
        const int64_t bq = seg_q + (int64_t)b * N;
        if (bq >= q_last) break;
        while (g0.qb <= bq) {   // uniform
            if (++r >= A.nr) break;
            g0 = g1;
            g1 = !one && r + 1 < A.nr ? A.R[r + 1] : rtamd::JRange{q_last, q_last, 0};
        }
        if (r >= A.nr) break;
        const uint32_t* o = buf + base;
        if (g0.qa < bq + N) {
            const BlockDst d = block_dst(jit, bq, g0, g1, r, A.nr);   // (one range: never generic)
            for (int i = lane; i < N / 2; i += FILLW_THREADS) {
                double* dst = nullptr;
                if (d.generic) {
                    const int64_t q = generic_dst(bq + 2 * i, A, r);
                    if (q >= 0) dst = jit + q;
                } else if (i >= d.a0 && i < d.b0) {
                    dst = d.p0 + i;
                } else if (i >= d.a1 && i < d.b1) {
                    dst = d.p1 + i;
                }
                if (dst) *dst = jitter_from(o[2 * i], o[2 * i + 1]);
            }
        }
        if (b + 1 < A.K && bq + N < q_last) {
            uint32_t* nw = buf + (base ^ N);
            for (int t = lane; t < 227; t += FILLW_THREADS) {
                const uint32_t n0 = twist_word(o[t], o[t + 1], o[t + 397]);
                const uint32_t n1 = twist_word(o[227 + t], o[228 + t], n0);
                nw[t] = n0;
                nw[227 + t] = n1;
                if (t < 170) {
                    const uint32_t nx = (t == 169) ? twist_word(o[0], o[1], o[397]) : o[455 + t];
                    nw[454 + t] = twist_word(o[454 + t], nx, n1);
                }
            }
        }
        lds_barrier();
        base ^= N;
    }
}

// Needed segments of a job (with the first range overlapping each), in the
// layout FillArgs::segs expects.
std::vector<int64_t> job_segments(const std::vector<rtamd::JRange>& ranges, int64_t seg) {
    std::vector<int64_t> segs;
    size_t r = 0;
    int64_t last = -1;
    for (const rtamd::JRange& g : ranges) {
        for (int64_t c = std::max(last + 1, g.qa / seg); c <= (g.qb - 1) / seg; ++c) {
            while (r < ranges.size() && ranges[r].qb <= c * seg) ++r;
            segs.push_back(c);
            segs.push_back((int64_t)r);
            last = c;
        }
    }
    return segs;
}

}  // namespace

namespace rtamd {

hipError_t JitterTable::ensure(int64_t n_need, hipStream_t stream) {
    if (n_need <= n_ck) return hipSuccess;
    const int64_t n_new = std::max<int64_t>(n_need, n_ck + n_ck / 4);
    const int64_t q1 = n_new * (int64_t)kTableK * N;
    const int levels = mt_levels_needed(kTableK, q1);
    if (levels > MAX_LEVELS) return hipErrorInvalidValue;
    hipError_t e = hipSuccess;
    if (plan.K != kTableK || plan.levels < levels) {
        e = plan.build(kTableK, levels, stream);
        if (e != hipSuccess) return e;
    }
    // The coarse checkpoints (every R-th table entry: c = R*c') by the jump
    // tree's levels >= 1 (each from a coarse parent, c mod R^j), as partial
    // windows in slot c' of d_ckpt; then one wave per coarse checkpoint fills
    // the R entries behind it by sequential twisting (k_mt_expand).
    const int64_t R = rtamd::kMTRadix;
    const int64_t n_coarse = (n_new + R - 1) / R;
    std::vector<int64_t> lists;
    int64_t lvl_off[MAX_LEVELS + 1] = {0};
    for (int j = 0; j < plan.levels; ++j) {
        const int64_t lo = (int64_t)1 << (kMTRadixBits * j);
        if (j >= 1)
            for (int64_t c = lo; c < std::min(n_coarse * R, lo * R); c += R) lists.push_back(c);
        lvl_off[j + 1] = (int64_t)lists.size();
    }
    uint32_t* d_ckpt = nullptr;
    int64_t* d_list = nullptr;
    uint32_t* d_tab = nullptr;
    int64_t* h_list = nullptr;   // page-locked staging of the lists (host_copy_async)
    hipEvent_t e0 = nullptr, e1 = nullptr;
    e = hipMalloc(&d_ckpt, (size_t)n_coarse * kMTParts * N * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&d_list, std::max<size_t>(1, lists.size()) * sizeof(int64_t));
    if (e == hipSuccess) e = hipMalloc(&d_tab, (size_t)n_new * N * sizeof(uint32_t));
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess && !lists.empty()) {
        e = hipHostMalloc(reinterpret_cast<void**>(&h_list), lists.size() * sizeof(int64_t), hipHostMallocDefault);
        if (e == hipSuccess) {
            std::copy(lists.begin(), lists.end(), h_list);
            e = host_copy_async(d_list, h_list, lists.size() * sizeof(int64_t), stream);
        } else {
            h_list = nullptr;
        }
    }
    if (e == hipSuccess) e = hipEventRecord(e0, stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d_ckpt, plan.d_base, N * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream);
    int8_t parts[MAX_LEVELS] = {1, 1, 1, 1, 1, 1, 1, 1};
    for (int j = 0; j < plan.levels; ++j) {
        const int64_t n_j = lvl_off[j + 1] - lvl_off[j];
        if (n_j > 0) parts[j] = (int8_t)level_parts(n_j);
    }
    JumpArgs A{};
    A.div = R;
    for (int k = 0; k < MAX_LEVELS; ++k) A.parts[k] = parts[k];
    for (int j = 1; j < plan.levels && e == hipSuccess; ++j) {
        const int64_t n_j = lvl_off[j + 1] - lvl_off[j];
        if (n_j <= 0) continue;
        A.lo = (int64_t)1 << (kMTRadixBits * j);
        A.list = d_list + lvl_off[j];
        A.S = parts[j];
        for (int m = 0; m < kMTRadix; ++m) {
            A.off[m] = plan.off[(size_t)j * kMTRadix + m];
            A.len[m] = plan.off[(size_t)j * kMTRadix + m + 1] - A.off[m];
        }
        hipLaunchKernelGGL(k_mt_jump, dim3((unsigned)n_j, (unsigned)A.S), dim3(JUMP_THREADS), 0, stream, plan.d_taps,
                           A, d_ckpt);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_mt_expand, dim3((unsigned)n_coarse), dim3(64), 0, stream, d_ckpt, A, n_new, d_tab);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(e1, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    else (void)hipStreamSynchronize(stream);   // (nothing queued may read what is freed below)
    plan.drop_stage();
    if (h_list) (void)hipHostFree(h_list);
    if (e == hipSuccess) (void)hipEventElapsedTime(&ms_last_build, e0, e1);
    if (d_ckpt) (void)hipFree(d_ckpt);
    if (d_list) (void)hipFree(d_list);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (e != hipSuccess) {
        if (d_tab) (void)hipFree(d_tab);
        return e;
    }
    if (d_table) (void)hipFree(d_table);
    d_table = d_tab;
    n_ck = cap = n_new;
    return hipSuccess;
}

void JitterTable::release() {
    if (d_table) (void)hipFree(d_table);
    d_table = nullptr;
    n_ck = cap = 0;
    plan.release();
}

size_t mt_fill_scratch_bytes(const std::vector<JRange>& ranges) {
    if (ranges.empty()) return 64;
    const int64_t n_ck = (ranges.back().qb - 1) / ((int64_t)kTableK * N) + 1;
    return ranges.size() * sizeof(JRange) + (size_t)n_ck * 2 * sizeof(int64_t) + 64;
}

hipError_t mt_launch_fill(const JitterTable& T, const std::vector<JRange>& ranges, JitterJob& job, void* d_scratch,
                          double* d_jit, hipStream_t stream) {
    if (ranges.empty()) return hipSuccess;
    for (size_t i = 0; i < ranges.size(); ++i) {
        const JRange& g = ranges[i];
        if (g.qa < 0 || g.qb <= g.qa || (g.qa & 1) || (g.qb & 1) || g.dst < 0 || (i && g.qa < ranges[i - 1].qb))
            return hipErrorInvalidValue;
    }
    const int64_t seg = (int64_t)kTableK * N;
    if ((ranges.back().qb - 1) / seg >= T.n_ck) return hipErrorInvalidValue;   // table too short
    if (ranges.size() == 1) {
        // one range: the segments are c0 .. c1, the range goes by value
        FillArgs F{};
        F.K = kTableK;
        F.nr = 1;
        F.one = ranges[0];
        F.c0 = ranges[0].qa / seg;
        const int64_t n_seg = (ranges[0].qb - 1) / seg - F.c0 + 1;
        job.qmax = ranges[0].qb;
        hipLaunchKernelGGL(k_mt_fill_w, dim3((unsigned)n_seg), dim3(FILLW_THREADS), 0, stream, T.d_table, F, d_jit);
        return hipGetLastError();
    }
    const std::vector<int64_t> segs = job_segments(ranges, seg);
    const size_t b_r = ranges.size() * sizeof(JRange), b_s = segs.size() * sizeof(int64_t);
    job.stage.resize(b_r + b_s);
    std::memcpy(job.stage.data(), ranges.data(), b_r);
    std::memcpy(job.stage.data() + b_r, segs.data(), b_s);
    job.qmax = ranges.back().qb;
    char* dsc = static_cast<char*>(d_scratch);
    hipError_t e = upload_async(job.up, dsc, job.stage.data(), job.stage.size(), stream);
    if (e != hipSuccess) return e;
    FillArgs F{};
    F.K = kTableK;
    F.nr = (int)ranges.size();
    F.R = reinterpret_cast<const JRange*>(dsc);
    F.segs = reinterpret_cast<const int64_t*>(dsc + b_r);
    hipLaunchKernelGGL(k_mt_fill_w, dim3((unsigned)(segs.size() / 2)), dim3(FILLW_THREADS), 0, stream, T.d_table, F,
                       d_jit);
    return hipGetLastError();
}

// The precomputed tree polynomials live next to this library
// (lib/mt19937_tree.polys, written by the build's bin/mt_polygen).
static void locate_poly_file() {
    static std::once_flag once;
    std::call_once(once, [] {
        Dl_info info{};
        if (dladdr(reinterpret_cast<void*>(&locate_poly_file), &info) && info.dli_fname) {
            std::string dir(info.dli_fname);
            const size_t slash = dir.rfind('/');
            dir = slash == std::string::npos ? std::string(".") : dir.substr(0, slash);
            mt_set_poly_file(dir + "/mt19937_tree.polys");
        }
    });
}

// The tree's tap lists (host only, cached per process): level-major, so a
// plan of fewer levels uses a prefix.  rt_warmup(RT_WARM_HOST) computes them
// on a helper thread while the process initialises HIP.
namespace {
struct HostTaps {
    int K = 0, levels = 0;
    std::vector<uint16_t> taps;
    std::vector<int32_t> off;
};
std::mutex g_taps_mu;
std::shared_ptr<const HostTaps> g_taps;
}  // namespace

std::shared_ptr<const HostTaps> host_taps(int K_blocks, int levels_needed) {
    std::lock_guard<std::mutex> lk(g_taps_mu);
    if (g_taps && g_taps->K == K_blocks && g_taps->levels >= levels_needed) return g_taps;
    locate_poly_file();
    std::vector<uint32_t> polys = mt_tree_polys(K_blocks, levels_needed);
    // the set coefficients of every polynomial, in order (~2.3 M taps for 4
    // levels): sized by popcount, then one ctz walk per word (a bit-by-bit
    // scan took ~40 ms of the CLI's one-time setup)
    auto T = std::make_shared<HostTaps>();
    T->K = K_blocks;
    T->levels = levels_needed;
    const size_t n_poly = (size_t)levels_needed * (kMTRadix - 1);
    size_t n_taps = 0;
    for (size_t k = 0; k < n_poly * kPolyWords32; ++k) n_taps += (size_t)__builtin_popcount(polys[k]);
    T->taps.resize(n_taps);
    size_t o = 0;
    T->off.assign(1, 0);
    for (int j = 0; j < levels_needed; ++j)
        for (int m = 0; m < kMTRadix; ++m) {
            if (m > 0) {
                const uint32_t* P = polys.data() + ((size_t)j * (kMTRadix - 1) + (m - 1)) * kPolyWords32;
                for (int w = 0; w < kPolyWords32; ++w)
                    for (uint32_t b = P[w]; b; b &= b - 1) {
                        const int i = w * 32 + __builtin_ctz(b);
                        if (i < kMTDeg) T->taps[o++] = (uint16_t)i;
                    }
            }
            T->off.push_back((int32_t)o);
        }
    T->taps.resize(o);
    g_taps = T;
    return T;
}

void mt_prefetch_host_taps() {
    locate_poly_file();
    const int levels = std::min(MAX_LEVELS, mt_poly_file_levels(kTableK));
    if (levels > 0) (void)host_taps(kTableK, levels);   // (never the slow computed path here)
}

hipError_t JitterPlan::build(int K_blocks, int levels_needed, hipStream_t stream) {
    release();
    const std::shared_ptr<const HostTaps> T = host_taps(K_blocks, levels_needed);
    // page-locked staging: [seed window | taps of the first levels_needed levels]
    const size_t win_bytes = (size_t)N * sizeof(uint32_t);
    const size_t o = (size_t)T->off[(size_t)levels_needed * kMTRadix];
    const size_t taps_cap = o + 8;
    hipError_t e = hipHostMalloc(&h_stage, win_bytes + taps_cap * sizeof(uint16_t), hipHostMallocDefault);
    if (e != hipSuccess) {
        h_stage = nullptr;
        return e;
    }
    uint32_t* win = static_cast<uint32_t*>(h_stage);
    uint16_t* taps = reinterpret_cast<uint16_t*>(static_cast<char*>(h_stage) + win_bytes);
    std::memcpy(taps, T->taps.data(), o * sizeof(uint16_t));
    off.assign(T->off.begin(), T->off.begin() + (size_t)levels_needed * kMTRadix + 1);
    for (int k = 0; k < 8; ++k) taps[o + k] = 0;
    const size_t n_up = o + 8;
    mt_first_window(12345u, win);
    e = hipMalloc(&d_taps, n_up * sizeof(uint16_t));
    if (e == hipSuccess) e = hipMalloc(&d_base, win_bytes);
    if (e == hipSuccess) e = host_copy_async(d_taps, taps, n_up * sizeof(uint16_t), stream);
    if (e == hipSuccess) e = host_copy_async(d_base, win, win_bytes, stream);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(stream);
        release();
        return e;
    }
    K = K_blocks;
    levels = levels_needed;
    return hipSuccess;
}

void JitterPlan::drop_stage() {
    if (h_stage) (void)hipHostFree(h_stage);
    h_stage = nullptr;
}

void JitterPlan::release() {
    drop_stage();
    if (d_taps) (void)hipFree(d_taps);
    if (d_base) (void)hipFree(d_base);
    d_taps = nullptr;
    d_base = nullptr;
    K = levels = 0;
    off.clear();
}

size_t mt_scratch_bytes(int K, const std::vector<JRange>& ranges) {
    if (ranges.empty()) return 64;
    const int64_t n_ck = (ranges.back().qb - 1) / ((int64_t)K * N) + 1;
    return ranges.size() * sizeof(JRange) + (size_t)n_ck * 3 * sizeof(int64_t) + 64;
}

hipError_t mt_launch_jitter(const JitterPlan& plan, const std::vector<JRange>& ranges, JitterJob& job,
                            void* d_scratch, uint32_t* d_ckpt, double* d_jit, hipStream_t stream) {
    if (ranges.empty()) return hipSuccess;
    for (size_t i = 0; i < ranges.size(); ++i) {
        const JRange& g = ranges[i];
        if (g.qa < 0 || g.qb <= g.qa || (g.qa & 1) || (g.qb & 1) || g.dst < 0 ||
            (i && g.qa < ranges[i - 1].qb))
            return hipErrorInvalidValue;
    }
    const int K = plan.K;
    const int64_t seg = (int64_t)K * N;
    const int64_t qmax = ranges.back().qb;
    const int64_t c1 = (qmax - 1) / seg;
    if (plan.levels < mt_levels_needed(K, qmax) || plan.levels > MAX_LEVELS) return hipErrorInvalidValue;

    // needed segments (with their first overlapping range) and the tree
    // ancestors of each: checkpoint c is one jump from ckpt_parent(c)
    std::vector<int64_t> segs;
    std::vector<char> need((size_t)c1 + 1, 0);
    {
        size_t r = 0;
        int64_t last = -1;
        for (const JRange& g : ranges) {
            for (int64_t c = std::max(last + 1, g.qa / seg); c <= (g.qb - 1) / seg; ++c) {
                while (r < ranges.size() && ranges[r].qb <= c * seg) ++r;
                segs.push_back(c);
                segs.push_back((int64_t)r);
                for (int64_t a = c; a > 0 && !need[a]; a = ckpt_parent(a)) need[a] = 1;
                last = c;
            }
        }
    }
    std::vector<int64_t> lists;
    int64_t lvl_off[MAX_LEVELS + 1] = {0};
    for (int j = 0; j < plan.levels; ++j) {
        const int64_t lo = (int64_t)1 << (kMTRadixBits * j);
        for (int64_t c = lo; c <= std::min(c1, lo * kMTRadix - 1); ++c)
            if (need[c]) lists.push_back(c);
        lvl_off[j + 1] = (int64_t)lists.size();
    }
    // stage: ranges | segs | per-level lists
    const size_t b_r = ranges.size() * sizeof(JRange), b_s = segs.size() * sizeof(int64_t),
                 b_l = lists.size() * sizeof(int64_t);
    job.stage.resize(b_r + b_s + b_l);
    std::memcpy(job.stage.data(), ranges.data(), b_r);
    std::memcpy(job.stage.data() + b_r, segs.data(), b_s);
    if (b_l) std::memcpy(job.stage.data() + b_r + b_s, lists.data(), b_l);
    job.qmax = qmax;
    char* dsc = static_cast<char*>(d_scratch);
    hipError_t e = upload_async(job.up, dsc, job.stage.data(), job.stage.size(), stream);
    if (e != hipSuccess) return e;
    const JRange* dR = reinterpret_cast<const JRange*>(dsc);
    const int64_t* dS = reinterpret_cast<const int64_t*>(dsc + b_r);
    const int64_t* dL = reinterpret_cast<const int64_t*>(dsc + b_r + b_s);

    e = hipMemcpyAsync(d_ckpt, plan.d_base, N * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) return e;
    int8_t parts[MAX_LEVELS] = {1, 1, 1, 1, 1, 1, 1, 1};
    for (int j = 0; j < plan.levels; ++j) {
        const int64_t n_j = lvl_off[j + 1] - lvl_off[j];
        if (n_j > 0) parts[j] = (int8_t)level_parts(n_j);
    }
    for (int j = 0; j < plan.levels; ++j) {
        const int64_t n_j = lvl_off[j + 1] - lvl_off[j];
        if (n_j <= 0) continue;
        JumpArgs A;
        A.div = 1;
        A.lo = (int64_t)1 << (kMTRadixBits * j);
        A.list = dL + lvl_off[j];
        A.S = parts[j];
        for (int m = 0; m < kMTRadix; ++m) {
            A.off[m] = plan.off[(size_t)j * kMTRadix + m];
            A.len[m] = plan.off[(size_t)j * kMTRadix + m + 1] - A.off[m];
        }
        for (int k = 0; k < MAX_LEVELS; ++k) A.parts[k] = parts[k];
        hipLaunchKernelGGL(k_mt_jump, dim3((unsigned)n_j, (unsigned)A.S), dim3(JUMP_THREADS), 0, stream,
                           plan.d_taps, A, d_ckpt);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    FillArgs F;
    F.K = K;
    F.nr = (int)ranges.size();
    F.R = dR;
    F.segs = dS;
    for (int k = 0; k < MAX_LEVELS; ++k) F.parts[k] = parts[k];
    hipLaunchKernelGGL(k_mt_fill, dim3((unsigned)(segs.size() / 2)), dim3(FILL_THREADS), 0, stream, d_ckpt, F,
                       d_jit);
    return hipGetLastError();
}

size_t mt_ckpt_words(int K, int64_t q1) {
    const int64_t n = q1 > 0 ? (q1 - 1) / ((int64_t)K * N) + 1 : 1;
    return (size_t)n * kMTParts * N;
}

int mt_levels_needed(int K, int64_t q1) {
    const int64_t seg = (int64_t)K * N;
    const int64_t cmax = q1 > 0 ? (q1 - 1) / seg : 0;   // highest checkpoint index
    int L = 1;
    while (((int64_t)1 << (kMTRadixBits * L)) <= cmax) ++L;
    return L;
}

}  // namespace rtamd
