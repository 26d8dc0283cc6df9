// mt_poly.hpp — GF(2) jump-ahead polynomials for std::mt19937.
//
// The reference draws its sub-pixel jitter from ONE serial std::mt19937(12345)
// stream (raytracer/src/tracer.cpp:284-293): pixel p (loop order), sample s
// consumes outputs 32p+4s .. 32p+4s+3.  To generate that stream on the GPU in
// parallel we jump the generator to checkpoints.  Raw (untempered) words obey
// a linear recurrence over GF(2) whose characteristic polynomial phi has
// degree 19937; for every bit position, w[n+J] = XOR_i p_i * w[n+i] with
// p = x^J mod phi.  phi is recovered here with Berlekamp-Massey and the jump
// polynomials for J = 624*K*2^k by repeated squaring modulo phi.
//
// Conventions: raw word w_k, k >= 0, w_0..w_623 = seeding (init_genrand),
// w_{k+624} = w_{k+397} ^ twist(w_k, w_{k+1}); output q = temper(w_{624+q}).
// A "window at n" is w_n .. w_{n+623}.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace rtamd {

constexpr int kMTN = 624;
constexpr int kMTDeg = 19937;
constexpr int kPolyWords32 = 624;   // 19968 coefficient bits >= 19937

// Window at n = 624 (raw words feeding outputs 0..623) for the given seed.
void mt_first_window(uint32_t seed, uint32_t win[kMTN]);

// Characteristic polynomial phi (bit i = coefficient of x^i), degree 19937.
const std::vector<uint64_t>& mt_charpoly();

// P_k = x^(624*K*2^k) mod phi for k in [0, levels), each kPolyWords32 words.
// Cached per (K, levels) in the process.
std::vector<uint32_t> mt_jump_table(int K_blocks, int levels);

// Radix-64 checkpoint tree (mt_jump.hip): level j computes checkpoints
// c in [64^j, 64^(j+1)) as ONE jump from c - m*64^j, m = c / 64^j, by
// x^(624*K*m*64^j) mod phi.  Returns those polynomials for j < levels and
// m = 1..63 at index (j*63 + m-1)*kPolyWords32.  Cached per (K, levels).
// (Radix 64: two levels reach 4096 segments - every frame up to 8K - so a
// frame's checkpoints take two dependent jump launches.)
constexpr int kMTRadixBits = 6;
constexpr int kMTRadix = 1 << kMTRadixBits;
std::vector<uint32_t> mt_tree_polys(int K_blocks, int levels);

// The tree polynomials are constants of mt19937: the build writes them once
// (bin/mt_polygen -> lib/mt19937_tree.polys, next to librtamd.so) and
// mt_tree_polys() reads the levels it needs from that file instead of
// computing them (~0.5-2 s of GF(2) arithmetic on the first frame of a
// process).  File: "MTJPOLY1", u32 K, u32 levels, u32 words per polynomial,
// u32 0, the polynomials in mt_tree_polys order, u64 FNV-1a of the payload.
// A missing, short or corrupt file is ignored (the polynomials are computed).
void mt_set_poly_file(const std::string& path);
bool mt_save_tree_polys(const std::string& path, int K_blocks, int levels);
// Levels the configured poly file holds for K (0: none / unusable header).
int mt_poly_file_levels(int K_blocks);
// Reads the first `levels` levels from `path` into out; false if unusable.
bool mt_load_tree_polys(const std::string& path, int K_blocks, int levels, std::vector<uint32_t>& out);
// mt_tree_polys computed in this process, ignoring the file (tests).
std::vector<uint32_t> mt_tree_polys_computed(int K_blocks, int levels);

// x^J mod phi for an arbitrary J (kPolyWords32 words).
std::vector<uint32_t> mt_jump_poly(uint64_t J);

// CPU application of a jump polynomial to a window (tests / validation).
void mt_apply_jump_cpu(const uint32_t* poly, const uint32_t win[kMTN], uint32_t out[kMTN]);

// Advance a window by whole blocks sequentially (CPU, tests).
void mt_advance_blocks_cpu(uint32_t win[kMTN], uint64_t blocks);

inline uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

}  // namespace rtamd
