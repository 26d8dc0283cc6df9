// mt_poly.cpp — see mt_poly.hpp.
#include "mt_poly.hpp"

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>

namespace rtamd {
namespace {

constexpr uint32_t UM = 0x80000000u, LM = 0x7fffffffu, MA = 0x9908b0dfu;

inline uint32_t twist_word(uint32_t wk, uint32_t wk1, uint32_t wk397) {
    uint32_t y = (wk & UM) | (wk1 & LM);
    return wk397 ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
}

// Raw words w_n .. w_{n+count-1} starting from a window at n.
void gen_raw(const uint32_t win[kMTN], size_t count, std::vector<uint32_t>& out) {
    out.resize(count < (size_t)kMTN ? (size_t)kMTN : count);
    std::memcpy(out.data(), win, sizeof(uint32_t) * kMTN);
    for (size_t k = kMTN; k < count; ++k) out[k] = twist_word(out[k - 624], out[k - 623], out[k - 227]);
}

constexpr int kW64 = (2 * kMTDeg + 128) / 64 + 2;   // words for products

struct Poly {
    std::vector<uint64_t> w;
    explicit Poly(size_t n = kW64) : w(n, 0) {}
    bool bit(size_t i) const { return (w[i >> 6] >> (i & 63)) & 1u; }
    void flip(size_t i) { w[i >> 6] ^= (uint64_t)1 << (i & 63); }
};

// Berlekamp-Massey over GF(2) on bit 0 of raw words starting at w_624.
std::vector<uint64_t> compute_charpoly() {
    const size_t N = 2 * (size_t)kMTDeg + 256;
    uint32_t win[kMTN];
    mt_first_window(5489u, win);
    std::vector<uint32_t> raw;
    gen_raw(win, N, raw);
    // rs = reversed bit sequence: rs[k] = s[N-1-k]
    const size_t NW = N / 64 + 2;
    std::vector<uint64_t> rs(NW + 2, 0);
    for (size_t k = 0; k < N; ++k)
        if (raw[N - 1 - k] & 1u) rs[k >> 6] |= (uint64_t)1 << (k & 63);
    auto rs_word = [&](size_t off) -> uint64_t {   // 64 bits of rs starting at bit off
        size_t q = off >> 6, r = off & 63;
        uint64_t lo = rs[q] >> r;
        uint64_t hi = (r && q + 1 < rs.size()) ? (rs[q + 1] << (64 - r)) : 0;
        return lo | hi;
    };
    std::vector<uint64_t> Cp(NW + 2, 0), Bp(NW + 2, 0), T;
    Cp[0] = 1; Bp[0] = 1;
    size_t L = 0, m = 1;
    for (size_t n = 0; n < N; ++n) {
        // d = sum_{i=0..L} C_i s[n-i] = sum_i C_i rs[N-1-n+i]
        const size_t off = N - 1 - n;
        uint64_t acc = 0;
        const size_t nwords = L / 64 + 1;
        for (size_t w = 0; w < nwords; ++w) {
            uint64_t c = Cp[w];
            if (w == nwords - 1) {
                size_t rem = (L & 63) + 1;
                if (rem < 64) c &= (((uint64_t)1 << rem) - 1);
            }
            acc ^= c & rs_word(off + 64 * w);
        }
        int d = __builtin_parityll(acc);
        if (!d) { ++m; continue; }
        const bool grow = 2 * L <= n;
        if (grow) T = Cp;
        // C ^= B << m
        const size_t ws = m >> 6, bs = m & 63;
        for (size_t w = Cp.size(); w-- > 0;) {
            if (w < ws) break;
            uint64_t v = Bp[w - ws] << bs;
            if (bs && w - ws >= 1) v |= Bp[w - ws - 1] >> (64 - bs);
            Cp[w] ^= v;
        }
        if (grow) { L = n + 1 - L; Bp = T; m = 1; } else { ++m; }
    }
    if (L != (size_t)kMTDeg) throw std::runtime_error("mt19937 Berlekamp-Massey: unexpected linear complexity");
    // phi_j = C_{L-j}
    std::vector<uint64_t> phi((kMTDeg + 64) / 64 + 1, 0);
    for (size_t j = 0; j <= L; ++j) {
        size_t i = L - j;
        if ((Cp[i >> 6] >> (i & 63)) & 1u) phi[j >> 6] |= (uint64_t)1 << (j & 63);
    }
    return phi;
}

// Reducer: phi shifted by 0..63 bits for word-granular XOR.
struct Reducer {
    std::vector<std::vector<uint64_t>> sh;   // sh[b] = phi << b, (PW+1) words
    size_t PW;
    explicit Reducer(const std::vector<uint64_t>& phi) {
        PW = phi.size();
        sh.resize(64);
        for (int b = 0; b < 64; ++b) {
            sh[b].assign(PW + 1, 0);
            for (size_t w = 0; w < PW; ++w) {
                sh[b][w] ^= phi[w] << b;
                if (b) sh[b][w + 1] ^= phi[w] >> (64 - b);
            }
        }
    }
    // Reduce p (degree < 2*deg) modulo phi in place.
    void reduce(std::vector<uint64_t>& p) const {
        for (size_t d = (size_t)2 * kMTDeg; d >= (size_t)kMTDeg; --d) {
            if (!((p[d >> 6] >> (d & 63)) & 1u)) continue;
            const size_t s = d - kMTDeg;
            const size_t ws = s >> 6;
            const auto& v = sh[s & 63];
            for (size_t w = 0; w < v.size() && ws + w < p.size(); ++w) p[ws + w] ^= v[w];
        }
    }
};

uint64_t spread32(uint32_t x) {   // interleave zeros: bit i -> bit 2i
    uint64_t v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
}

// p := p^2 mod phi (p has degree < deg).
void square_mod(std::vector<uint64_t>& p, const Reducer& R) {
    std::vector<uint64_t> q(kW64, 0);
    for (size_t w = 0; w < p.size() && 2 * w + 1 < q.size(); ++w) {
        q[2 * w] = spread32((uint32_t)p[w]);
        q[2 * w + 1] = spread32((uint32_t)(p[w] >> 32));
    }
    R.reduce(q);
    for (size_t w = 0; w < p.size(); ++w) p[w] = q[w];
}

// p := p * x mod phi
void mulx_mod(std::vector<uint64_t>& p) {
    const auto& phi = mt_charpoly();
    uint64_t carry = 0;
    for (size_t w = 0; w < p.size(); ++w) {
        uint64_t nc = p[w] >> 63;
        p[w] = (p[w] << 1) | carry;
        carry = nc;
    }
    if ((p[kMTDeg >> 6] >> (kMTDeg & 63)) & 1u)
        for (size_t w = 0; w < phi.size() && w < p.size(); ++w) p[w] ^= phi[w];
}

std::vector<uint32_t> to_words32(const std::vector<uint64_t>& p) {
    std::vector<uint32_t> out(kPolyWords32, 0);
    for (int j = 0; j < kPolyWords32; ++j) {
        uint64_t w = (j / 2 < (int)p.size()) ? p[j / 2] : 0;
        out[j] = (uint32_t)((j & 1) ? (w >> 32) : w);
    }
    return out;
}

std::mutex g_mu;

}  // namespace

void mt_first_window(uint32_t seed, uint32_t win[kMTN]) {
    uint32_t mt[kMTN];
    mt[0] = seed;
    for (int i = 1; i < kMTN; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    // one twist: w_624..w_1247 (libstdc++ _M_gen_rand, in place)
    for (int k = 0; k < kMTN; ++k) {
        uint32_t wk397 = (k + 397 < kMTN) ? mt[k + 397] : mt[k + 397 - kMTN];
        uint32_t wk1 = (k + 1 < kMTN) ? mt[k + 1] : mt[0];
        mt[k] = twist_word(mt[k], wk1, wk397);
    }
    std::memcpy(win, mt, sizeof(mt));
}

const std::vector<uint64_t>& mt_charpoly() {
    static std::vector<uint64_t> phi;
    static std::once_flag once;
    std::call_once(once, [] { phi = compute_charpoly(); });
    return phi;
}

std::vector<uint32_t> mt_jump_poly(uint64_t J) {
    const auto& phi = mt_charpoly();
    static Reducer* R = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!R) R = new Reducer(phi);
    }
    std::vector<uint64_t> p(phi.size(), 0);
    p[0] = 1;   // x^0
    int top = 63;
    while (top >= 0 && !((J >> top) & 1u)) --top;
    for (int b = top; b >= 0; --b) {
        square_mod(p, *R);
        if ((J >> b) & 1u) mulx_mod(p);
    }
    return to_words32(p);
}

std::vector<uint32_t> mt_jump_table(int K_blocks, int levels) {
    static std::map<std::pair<int, int>, std::vector<uint32_t>> cache;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = cache.find({K_blocks, levels});
        if (it != cache.end()) return it->second;
    }
    const auto& phi = mt_charpoly();
    static Reducer* R = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!R) R = new Reducer(phi);
    }
    // P_0 = x^(624*K): start from x^624 and square log2(K) times when K is a
    // power of two, otherwise use the general exponentiation.
    std::vector<uint64_t> p(phi.size(), 0);
    if (K_blocks > 0 && (K_blocks & (K_blocks - 1)) == 0) {
        p[624 >> 6] = (uint64_t)1 << (624 & 63);
        for (int k = K_blocks; k > 1; k >>= 1) square_mod(p, *R);
    } else {
        std::vector<uint32_t> w = mt_jump_poly((uint64_t)624 * (uint64_t)K_blocks);
        for (int j = 0; j < kPolyWords32; ++j) p[j / 2] |= (uint64_t)w[j] << ((j & 1) * 32);
    }
    std::vector<uint32_t> table;
    table.reserve((size_t)levels * kPolyWords32);
    for (int l = 0; l < levels; ++l) {
        std::vector<uint32_t> w = to_words32(p);
        table.insert(table.end(), w.begin(), w.end());
        square_mod(p, *R);
    }
    std::lock_guard<std::mutex> lk(g_mu);
    cache[{K_blocks, levels}] = table;
    return table;
}

namespace {

// a * b mod phi (both of degree < 19937), schoolbook carry-less product.
std::vector<uint64_t> mul_mod(const std::vector<uint64_t>& a, const std::vector<uint64_t>& b, const Reducer& R) {
    std::vector<uint64_t> q(kW64, 0);
    const size_t nb = b.size();
    for (size_t i = 0; i < (size_t)kMTDeg; ++i) {
        if (!((a[i >> 6] >> (i & 63)) & 1u)) continue;
        const size_t ws = i >> 6, bs = i & 63;
        for (size_t w = 0; w < nb && ws + w < q.size(); ++w) {
            q[ws + w] ^= b[w] << bs;
            if (bs && ws + w + 1 < q.size()) q[ws + w + 1] ^= b[w] >> (64 - bs);
        }
    }
    R.reduce(q);
    q.resize(a.size());
    return q;
}

std::vector<uint64_t> from_words32(const uint32_t* w, size_t n64) {
    std::vector<uint64_t> p(n64, 0);
    for (int j = 0; j < kPolyWords32; ++j)
        if ((size_t)(j / 2) < n64) p[j / 2] |= (uint64_t)w[j] << ((j & 1) * 32);
    return p;
}

}  // namespace

namespace {
std::string g_poly_file;   // guarded by g_mu

uint64_t fnv1a(const uint32_t* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    const unsigned char* b = reinterpret_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n * 4; ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}
}  // namespace

void mt_set_poly_file(const std::string& path) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_poly_file = path;
}

bool mt_load_tree_polys(const std::string& path, int K_blocks, int levels, std::vector<uint32_t>& out) {
    if (path.empty() || levels <= 0) return false;
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    char magic[8];
    uint32_t hdr[4];
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "MTJPOLY1", 8) == 0 &&
              std::fread(hdr, 4, 4, f) == 4 && (int)hdr[0] == K_blocks && (int)hdr[1] >= levels &&
              hdr[2] == (uint32_t)kPolyWords32;
    std::vector<uint32_t> all;
    // the level count comes from the file: bound it (a jump of 64^16 blocks is
    // far past any frame) and by the file's own size before sizing the buffer
    constexpr uint32_t kMaxLevels = 16;
    if (ok) {
        long here = std::ftell(f);
        ok = hdr[1] <= kMaxLevels && here >= 0 && std::fseek(f, 0, SEEK_END) == 0;
        const long end = ok ? std::ftell(f) : -1;
        ok = ok && end >= here && std::fseek(f, here, SEEK_SET) == 0 &&
             (uint64_t)(end - here) == (uint64_t)hdr[1] * (kMTRadix - 1) * kPolyWords32 * 4 + 8;
    }
    if (ok) {
        all.resize((size_t)hdr[1] * (kMTRadix - 1) * kPolyWords32);
        uint64_t sum = 0;
        ok = std::fread(all.data(), 4, all.size(), f) == all.size() && std::fread(&sum, 8, 1, f) == 1 &&
             sum == fnv1a(all.data(), all.size());
    }
    std::fclose(f);
    if (!ok) return false;
    out.assign(all.begin(), all.begin() + (size_t)levels * (kMTRadix - 1) * kPolyWords32);
    return true;
}

int mt_poly_file_levels(int K_blocks) {
    std::string file;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        file = g_poly_file;
    }
    if (file.empty()) return 0;
    FILE* f = std::fopen(file.c_str(), "rb");
    if (!f) return 0;
    char magic[8];
    uint32_t hdr[4];
    const bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "MTJPOLY1", 8) == 0 &&
                    std::fread(hdr, 4, 4, f) == 4 && (int)hdr[0] == K_blocks && hdr[1] <= 16 &&
                    hdr[2] == (uint32_t)kPolyWords32;
    std::fclose(f);
    return ok ? (int)hdr[1] : 0;
}

bool mt_save_tree_polys(const std::string& path, int K_blocks, int levels) {
    const std::vector<uint32_t> p = mt_tree_polys_computed(K_blocks, levels);
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const uint32_t hdr[4] = {(uint32_t)K_blocks, (uint32_t)levels, (uint32_t)kPolyWords32, 0u};
    const uint64_t sum = fnv1a(p.data(), p.size());
    bool ok = std::fwrite("MTJPOLY1", 1, 8, f) == 8 && std::fwrite(hdr, 4, 4, f) == 4 &&
              std::fwrite(p.data(), 4, p.size(), f) == p.size() && std::fwrite(&sum, 8, 1, f) == 1;
    ok = (std::fclose(f) == 0) && ok;
    return ok;
}

std::vector<uint32_t> mt_tree_polys(int K_blocks, int levels) {
    static std::map<std::pair<int, int>, std::vector<uint32_t>> cache;
    std::string file;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = cache.find({K_blocks, levels});
        if (it != cache.end()) return it->second;
        file = g_poly_file;
    }
    std::vector<uint32_t> out;
    if (!mt_load_tree_polys(file, K_blocks, levels, out)) out = mt_tree_polys_computed(K_blocks, levels);
    std::lock_guard<std::mutex> lk(g_mu);
    cache[{K_blocks, levels}] = out;
    return out;
}

std::vector<uint32_t> mt_tree_polys_computed(int K_blocks, int levels) {
    const auto& phi = mt_charpoly();
    static Reducer* R = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!R) R = new Reducer(phi);
    }
    // base = x^(624*K*R^j), level by level (R^j -> R^(j+1): log2(R) squarings)
    std::vector<uint32_t> b0 = mt_jump_table(K_blocks, 1);
    std::vector<uint64_t> base = from_words32(b0.data(), phi.size());
    std::vector<uint32_t> out;
    out.reserve((size_t)levels * (kMTRadix - 1) * kPolyWords32);
    for (int j = 0; j < levels; ++j) {
        std::vector<uint64_t> pm = base;
        for (int m = 1; m < kMTRadix; ++m) {
            if (m > 1) pm = mul_mod(pm, base, *R);
            std::vector<uint32_t> w = to_words32(pm);
            out.insert(out.end(), w.begin(), w.end());
        }
        for (int k = 1; k < kMTRadix; k <<= 1) square_mod(base, *R);
    }
    return out;
}

void mt_apply_jump_cpu(const uint32_t* poly, const uint32_t win[kMTN], uint32_t out[kMTN]) {
    std::vector<uint32_t> raw;
    gen_raw(win, (size_t)kMTDeg + kMTN + 1, raw);
    for (int j = 0; j < kMTN; ++j) out[j] = 0;
    for (int i = 0; i <= kMTDeg; ++i) {
        if (!((poly[i >> 5] >> (i & 31)) & 1u)) continue;
        for (int j = 0; j < kMTN; ++j) out[j] ^= raw[i + j];
    }
}

void mt_advance_blocks_cpu(uint32_t win[kMTN], uint64_t blocks) {
    uint32_t buf[2 * kMTN];
    for (uint64_t b = 0; b < blocks; ++b) {
        std::memcpy(buf, win, sizeof(uint32_t) * kMTN);
        for (int k = 0; k < kMTN; ++k) buf[kMTN + k] = twist_word(buf[k], buf[k + 1], buf[k + 397]);
        std::memcpy(win, buf + kMTN, sizeof(uint32_t) * kMTN);
    }
}

}  // namespace rtamd
