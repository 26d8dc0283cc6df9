// rt_kernels.hpp — the render kernels, built once per precision right after
// rt_device.hpp (RT_NS = rtd: FP64 parity path, rt_render.hip; RT_NS = rtf:
// FP32 fast path, rt_render_f32.hip).
//
// Standard mode (Tracer::render, tracer.cpp:282-300):
//   k_std: one lane per (pixel, sample); a wave covers 4x2 pixels x 8 samples,
//   a 256-thread block 8x4 pixels.  Samples are summed in order s = 0..7
//   across the 8 lanes of a pixel (cross-lane shuffles), then x 1/8.
// Paper mode (tracer.cpp:258-281):
//   k_paper_primary: one lane per pixel: the primary intersect (shared by
//   trace_paper, the centre probe and the four neighbour probes of
//   get_edge_strength, which all re-trace identical rays) + shading.
//   k_paper_finish: edge strength from the stored neighbour hits + hatch.
// The framebuffer, jitter draws and paper hit records stay double in both
// precisions (the float kernels convert on load / store).

namespace RT_NS {

using rtamd::kCounterSlots;
using rtamd::kCounterWords;
using rtamd::PaperParams;
using rtamd::SceneView;
using rtamd::StdParams;

namespace {

// Ray / op counters: wave reduction by shuffles, block reduction through LDS,
// then one atomic per block and counter into one of kCounterSlots slots
// (blockIdx-hashed).  A single hot address would serialize ~2M atomics at the
// L2 (~6 ns each, MI355X_MICROARCH.md fan-in row) - 12 ms per 4K frame.
// Standard-mode workgroup: RT_STD_WPB waves of 2x4 pixels x 8 samples.
// Default 1 (round 6): one-wave workgroups, each with its own 10 KiB of
// dynamic LDS (lds_pool).  A workgroup's LDS is released only when its last
// wave ends, so with 4-wave workgroups a wave that finished early left its
// SIMD slot empty until the slowest wave of its group was done; single-wave
// groups let the dispatcher refill each slot as soon as its wave exits.
// Measured: recursion row 12.77 -> 10.69 ms (waves of one group take
// different numbers of bounces), config 4 6.41 -> 6.33 ms
// (profiles/r06_ab/ab_wpb.txt).
#ifndef RT_STD_WPB
#define RT_STD_WPB 1
#endif
constexpr int kStdWPB = RT_STD_WPB;
constexpr int kStdThreads = 64 * kStdWPB;
// RT_STD_TW: a wave's pixel tile is TW x (8 / TW) pixels (default 2 x 4: the 4 x 2 tile of rounds 1-4
// measured config 4 8.45 -> 8.39 ms and the recursion row 17.55 -> 15.83 ms, profiles/r05_ab/ab_std_tile.txt)
#ifndef RT_STD_TW
#define RT_STD_TW 2
#endif
constexpr int kStdTW = RT_STD_TW, kStdTH = 8 / RT_STD_TW;
static_assert(kStdTW * kStdTH == 8, "a wave holds 8 pixels");
constexpr int kStdBlockX = kStdWPB >= 2 ? 2 * kStdTW : kStdTW;            // pixels per workgroup in x
constexpr int kStdBlockY = kStdWPB >= 4 ? 2 * kStdTH : kStdTH;            // output rows per workgroup

template <bool C, int NWAVES = 4>
__device__ __forceinline__ void flush_counters(unsigned long long* ctr, uint32_t ni, uint32_t no, Cnt<C>& cnt) {
#if defined(RT_EVENT_PROF)
    constexpr int NW = C ? 18 : 2 + EV_COUNT;
#elif defined(RT_PHASE_PROF)
    constexpr int NW = C ? 18 : 2 + PH_COUNT;
#else
    constexpr int NW = C ? 18 : 2;
#endif
    // red(w)[k] lives in wave w's own region of the LDS pool (its lanes are
    // done with shading when their wave gets here)
    static_assert(NW <= 64 && 64 <= kPoolWave, "counter slots");
    auto red = [](int w) { return reinterpret_cast<unsigned long long*>(wave_pool(w)); };
    unsigned long long v[NW];
    v[0] = ni;
    v[1] = no;
    if constexpr (C) {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[2 + k] = cnt.c[k];
    }
#if defined(RT_EVENT_PROF)
    if constexpr (!C) {
#pragma unroll
        for (int k = 0; k < EV_COUNT; ++k) v[2 + k] = (threadIdx.x & 63) == 0 ? cnt.get(k) : 0ull;
    }
#elif defined(RT_PHASE_PROF)
    if constexpr (!C) {
#pragma unroll
        for (int k = 0; k < PH_COUNT; ++k) v[2 + k] = (threadIdx.x & 63) == 0 ? cnt.get(k) : 0ull;
    }
#endif
#pragma unroll
    for (int k = 0; k < NW; ++k)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NW; ++k) red(wave)[k] = v[k];
    if constexpr (NWAVES > 1) __syncthreads();
    if (threadIdx.x < NW) {
        unsigned long long sum = 0;
#pragma unroll
        for (int w = 0; w < NWAVES; ++w) sum += red(w)[threadIdx.x];
        const unsigned slot = (blockIdx.x + blockIdx.y * gridDim.x) % kCounterSlots;
        if (sum) atomicAdd(&ctr[(size_t)slot * kCounterWords + threadIdx.x], sum);
    }
}

// Occupancy target of the lean variants (E = D = SEC = false): 4 waves/SIMD
// caps them at 128 VGPRs; the few values the compiler then spills are
// long-lived (stored once, reloaded once), and the extra wave per SIMD hides
// FP64 latency (measured 21.6 -> 19.2 ms on config 4; 5 and 6 are slower).
#ifndef RT_LEAN_WAVES
#define RT_LEAN_WAVES 4
#endif

// PL: the plain kernels (CntPlain: no transform / CSG code)
template <bool E, bool D, bool SEC, bool C, bool DL = true, int WV = 0, bool PL = false>
__device__ __forceinline__ void std_body(const DevScene& S, const StdParams& P) {
    static_assert(!(PL && C), "plain kernels do not count");
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int s = lane & 7;
    const int pix = lane >> 3;
    const int x = blockIdx.x * kStdBlockX + (wave & 1) * kStdTW + (pix % kStdTW);
    const int ri = blockIdx.y * kStdBlockY + (wave >> 1) * kStdTH + (pix / kStdTW);
    const bool active = x < P.W && ri < P.n_rows;
    uint32_t ni = 0, no = 0;
    std::conditional_t<PL, CntPlain, Cnt<C>> cnt;
    cnt.init();
    V3 c = v3(RV(0.0), RV(0.0), RV(0.0));
    if (active) {
        cnt.ev(EV_WAVES);
        cnt.pb(PH_SETUP);
        const int r = P.rows[ri];
        const int y = P.H - 1 - r;   // loop row (tracer.cpp:297 writes row ny-1-y)
        // draws 16p+2s, 16p+2s+1 of the stream: dx, dy (tracer.cpp:293)
        const double2 j = *reinterpret_cast<const double2*>(P.jit + ((size_t)P.jrow[ri] * P.W + x) * 16 + 2 * s);
        const DRay ray = gen_ray_subpixel(S, x, y, RV(j.x), RV(j.y));
        cnt.pe(PH_SETUP);
        c = trace<E, D, SEC, DL, WV>(S, ray, ni, no, cnt);
    }
    cnt.pb(PH_TAIL);
    // acc += trace(...) for s = 0..7 in order (tracer.cpp:290-296)
    const int base = lane & ~7;
    V3 acc = v3(RV(0.0), RV(0.0), RV(0.0));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const real cx = __shfl(c.x, base + k);
        const real cy = __shfl(c.y, base + k);
        const real cz = __shfl(c.z, base + k);
        acc.x += cx;
        acc.y += cy;
        acc.z += cz;
    }
    if (active && s == 0) {
        const real inv = RV(1.0) / (real)8;
        double* o = P.fb + ((size_t)ri * P.W + x) * 3;
        o[0] = acc.x * inv;
        o[1] = acc.y * inv;
        o[2] = acc.z * inv;
    }
    cnt.pe(PH_TAIL);
    flush_counters<C, kStdWPB>(P.counters, ni, no, cnt);
}

// WV: wave-level culling (scene_occluded_wave / scene_intersect_wave), picked
// by the host for scenes with >= 4 bounded objects and culling on.
template <bool E, bool D, bool SEC, bool C, bool WV = false>
__global__ __launch_bounds__(kStdThreads) void k_std(DevScene S, StdParams P) {
    std_body<E, D, SEC, C, true, WV>(S, P);
}

// Occupancy targets of the plain variants (PL): 4 waves/SIMD (128 VGPRs),
// as the general kernels.  (A 5-wave target caps the registers at 96 and
// spills: config 3 1.10 -> 1.22 ms once the LDS pool became dynamic and no
// longer capped the compiler's occupancy estimate itself; with a static
// 40 KiB pool the target had been inert, profiles/r06_ab/ab_wpb.txt,
// ab_light_cache.txt, ab_plain_tune.txt.)
#ifndef RT_PLAIN_LEAN_WAVES
#define RT_PLAIN_LEAN_WAVES 4
#endif
// WV: 0 = per-lane culls, 1 = wave-level culls, 2 = wave-level culls over the
// wave BVH (CompiledScene::wobjs / wchunk)
template <bool C, int WV, bool PL = false>
__global__ __launch_bounds__(kStdThreads) __attribute__((amdgpu_waves_per_eu(PL ? RT_PLAIN_LEAN_WAVES : RT_LEAN_WAVES))) void k_std_lean(DevScene S,
                                                                                                       StdParams P) {
    std_body<false, false, false, C, false, WV, PL>(S, P);
}

// Reflection / refraction with wave-level culling (trace_wave): the wave
// runs every bounce in lockstep.  Occupancy target RT_SEC_WAVES waves/SIMD.
#ifndef RT_SEC_WAVES
#define RT_SEC_WAVES 4
#endif
#ifndef RT_PLAIN_SEC_WAVES
#define RT_PLAIN_SEC_WAVES RT_SEC_WAVES
#endif
template <bool C, int WV = 1, bool PL = false>
__global__ __launch_bounds__(kStdThreads) __attribute__((amdgpu_waves_per_eu(PL ? RT_PLAIN_SEC_WAVES : RT_SEC_WAVES))) void k_std_secw(DevScene S,
                                                                                                      StdParams P) {
    std_body<false, false, true, C, false, WV, PL>(S, P);   // (no directional lights: those scenes take D)
}

// apply_crosshatch (tracer.cpp:188-205) in two halves.  Its FP64 part - the
// luminance tests - depends on the pixel's own shading only, so the primary
// pass reduces it to a band (0: lum < 0.15, black; 1..6: the darkness branch
// taken; 7: no branch, white; a NaN luminance takes none, as in the
// reference) stored with the material (4 bits instead of an 8-byte
// luminance); the finish pass applies the band's (x, y) pattern.  C++ '%'
// truncation toward zero.
__device__ __forceinline__ int hatch_band(real lum) {
    if (lum < RV(0.15)) return 0;
    const real darkness = RV(1.0) - lum;
    if (darkness > RV(0.8)) return 1;
    if (darkness > RV(0.65)) return 2;
    if (darkness > RV(0.5)) return 3;
    if (darkness > RV(0.35)) return 4;
    if (darkness > RV(0.2)) return 5;
    if (darkness > RV(0.12)) return 6;
    return 7;
}
__device__ __forceinline__ real crosshatch(int band, int x, int y) {
    if (band == 0) return RV(0.0);
    const bool diag1 = ((x + y) % 4) < 1;
    const bool diag2 = ((x - y) % 4) < 1;
    const bool horizontal = (y % 4) < 1;
    bool draw = false;
    if (band == 1) draw = (diag1 && diag2) || horizontal;
    else if (band == 2) draw = (diag1 && diag2) || (horizontal && ((x + y) % 3 == 0));
    else if (band == 3) draw = (diag1 && diag2) || (horizontal && ((x + y) % 4 == 0));
    else if (band == 4) draw = diag1 || (horizontal && ((x + y) % 3 == 0));
    else if (band == 5) draw = diag1;
    else if (band == 6) draw = diag1 && ((x + y) % 8) < 2;
    return draw ? RV(0.0) : RV(1.0);
}
// material slot: material (>= -3) in the low 24 bits, band in bits 24-27
__device__ __forceinline__ int paper_mat_pack(int mat, int band) { return (mat & 0xffffff) | (band << 24); }
__device__ __forceinline__ int paper_mat(int slot) {   // (sign-extends the material's 24 bits)
    return static_cast<int>(static_cast<unsigned>(slot) << 8) >> 8;
}
__device__ __forceinline__ int paper_band(int slot) { return (slot >> 24) & 15; }

// Paper-mode primary records: the material slot of a pixel whose ray hit
// nothing (a hit's material is an index >= 0, or -1 for none).
constexpr int kPaperMiss = -3;



#ifndef RT_PAPER_UO
#define RT_PAPER_UO true
#endif
// The plain paper kernel keeps the shadow bundle's wave-uniform parameters in
// VGPRs (it has the registers: config 5 3.55 -> 3.51 ms,
// profiles/r06_ab/ab_uo.txt); the general one moves them to SGPRs.
#ifndef RT_PLAIN_PAPER_UO
#define RT_PLAIN_PAPER_UO false
#endif
// Paper-mode primary workgroup: RT_PAPER_WPB waves of 8x8 pixels (4: 16x16
// pixels per 256-thread workgroup; 1, the default since round 6: one wave per
// workgroup with its own 10 KiB of dynamic LDS, as RT_STD_WPB; config 5
// 3.78 -> 3.56 ms, profiles/r06_ab/ab_wpb.txt).  The host's grid is in 16x16
// units either way (launch_paper remaps it), and wave (start, end) slots stay
// per 8x8 tile.
#ifndef RT_PAPER_WPB
#define RT_PAPER_WPB 1
#endif
constexpr int kPaperWPB = RT_PAPER_WPB;
static_assert(kPaperWPB == 1 || kPaperWPB == 4, "paper workgroups of 1 or 4 waves");
constexpr int kPaperThreads = 64 * kPaperWPB;
// a wave's 8x8 tile: (tile column, list group of 8 entries)
__device__ __forceinline__ int paper_tile_x() {
    return kPaperWPB == 4 ? (int)blockIdx.x * 2 + (int)((threadIdx.x >> 6) & 1) : (int)blockIdx.x;
}
__device__ __forceinline__ int paper_tile_y() {
    return kPaperWPB == 4 ? (int)blockIdx.y * 2 + (int)(threadIdx.x >> 7) : (int)blockIdx.y;
}
// A primary wave's (start, end) tick slot: group-major, one per 8-column tile
// (2 * ceil(W / 16) of them, rt_render.hip paper_waves_per_group) per 8-entry
// list group.
__device__ __forceinline__ unsigned* paper_wave_slot(const PaperParams& P) {
    const unsigned g = __builtin_amdgcn_readfirstlane(paper_tile_y()), xt = __builtin_amdgcn_readfirstlane(paper_tile_x());
    const unsigned tiles = kPaperWPB == 4 ? 2 * gridDim.x : gridDim.x;
    return P.gtime + 2 * ((size_t)g * tiles + xt);
}
#ifndef RT_PAPER_LEAD_I   // (A/B switches: lead objects in the paper closest-hit / shadow queries)
#define RT_PAPER_LEAD_I true
#endif
#ifndef RT_PAPER_LEAD_S
#define RT_PAPER_LEAD_S true
#endif
template <bool E, bool D, bool C, bool DL = true, int WV = 0, bool T = false, bool PL = false>
__device__ __forceinline__ void paper_primary_body(const DevScene& S, const PaperParams& P) {
    static_assert(!(PL && C), "plain kernels do not count");
    // wave 8x8 pixels (block 16x16 or one wave, RT_PAPER_WPB)
    const int lane = threadIdx.x & 63;
    const int x = paper_tile_x() * 8 + (lane & 7);
    const int li = paper_tile_y() * 8 + (lane >> 3);
    // (list entries < 0 pad a run of consecutive rows to a wave boundary)
    const int ei = li < P.n_list ? P.ext_list[li] : -1;
    const bool active = x < P.W && ei >= 0;
    // T (timed launches, P.gtime set): the wave's cost for later frames'
    // launch order (rt_render.hip order_paper_groups), its start and end
    // wall-clock ticks, stored into its own slot at the end (one-address
    // atomics per list group serialised the waves: +18 % frame time).  Every
    // store of this kernel comes after its last scene read, and only timed
    // launches read the clock at the start: a global store or the clock read
    // (an intrinsic with side effects) ahead of a load from the scene's arrays
    // takes away the compiler's proof that the load sees unmodified memory,
    // and the wave-uniform object and node reads of every shadow query then
    // become vector loads instead of scalar ones (config 5 4.61 vs 5.30 ms).
    unsigned t_start = 0u;
    if constexpr (T) t_start = (unsigned)wall_clock64();
    uint32_t ni = 0, no = 0;
    std::conditional_t<PL, CntPlain, Cnt<C>> cnt;
    cnt.init();
    DRay r{v3(RV(0.0), RV(0.0), RV(0.0)), v3(RV(0.0), RV(0.0), -RV(1.0))};
    real ht = RV(0.0);
    DHit h;
    h.mat = -1;
    h.p = h.n = v3(RV(0.0), RV(0.0), RV(0.0));
    h.ff = 1;
    bool hits = false, sh = false;
    size_t idx = 0;
    if (active) {
        const int y = P.ext_rows[ei];
        r = gen_ray(S, x, y);
        ++ni;
        if constexpr (WV)
            hits = scene_intersect_wave<E, D, (WV == 2), RT_PAPER_LEAD_I>(S, r, RV(1e-4), RT_INF, ht, h, __builtin_amdgcn_read_exec() == ~0ull,
                                              cnt);
        else
            hits = scene_intersect<E, D>(S, r, RV(1e-4), RT_INF, ht, h, cnt);
        idx = (size_t)ei * P.W + x;
        sh = P.ext_shade[ei] != 0;   // (a neighbour-only row needs the hit, not the shading)
    }
    int band = 0;   // the pixel's crosshatch band (hatch_band; neighbour-only rows: unused)
    // trace_paper (tracer.cpp:111-120) + get_luminance (:123-125).  shade()
    // runs with the whole wave (lanes with nothing to shade pass valid =
    // false) so that the wave-level shadow culls keep a full wave even when
    // it mixes shaded rows and neighbour-only rows (strip edges of a
    // multi-GPU partition) or inactive lanes.
    if (__any(sh)) {
        V3 base = shade<E, D, DL, WV, PL ? RT_PLAIN_PAPER_UO : RT_PAPER_UO, RT_PAPER_LEAD_S>(S, ht, h, normalized(vneg(r.d)), no,
                                                                                     cnt, sh && hits);
        if (sh) {
            if (!hits) base = v3(RV(1.0), RV(1.0), RV(1.0));
            band = hatch_band(RV(0.299) * base.x + RV(0.587) * base.y + RV(0.114) * base.z);
        }
    }
    // the material slot: the material (kPaperMiss for no hit: the finish
    // pass's hit flag) in the low 24 bits, the crosshatch band above
    if (active) {
        P.t[idx] = ht;
        P.nx[idx] = h.n.x;
        P.ny[idx] = h.n.y;
        P.nz[idx] = h.n.z;
        P.mat[idx] = paper_mat_pack(hits ? h.mat : kPaperMiss, band);
    }
    flush_counters<C, kPaperWPB>(P.counters, ni, no, cnt);
    if constexpr (T) {
        if (__lane_id() == 0) {
            unsigned* slot = paper_wave_slot(P);
            slot[0] = t_start;
            slot[1] = (unsigned)wall_clock64();
        }
    }
}

template <bool E, bool D, bool C, bool T = false>
__global__ __launch_bounds__(kPaperThreads) void k_paper_primary(DevScene S, PaperParams P) {
    paper_primary_body<E, D, C, true, 0, T>(S, P);
}

#ifndef RT_PAPER_WAVES
#define RT_PAPER_WAVES RT_LEAN_WAVES
#endif
#ifndef RT_PLAIN_PAPER_WAVES
#define RT_PLAIN_PAPER_WAVES RT_PAPER_WAVES
#endif
template <bool C, int WV, bool T = false, bool PL = false>
__global__ __launch_bounds__(kPaperThreads) __attribute__((amdgpu_waves_per_eu(PL ? RT_PLAIN_PAPER_WAVES : RT_PAPER_WAVES))) void k_paper_primary_lean(
    DevScene S, PaperParams P) {
    paper_primary_body<false, false, C, false, WV, T, PL>(S, P);
}

// One paper pixel (tracer.cpp:258-281) from its primary record and its four
// neighbours' (-1,0) (1,0) (0,-1) (0,1), already loaded.  CODES: a
// distributed frame's rank writes a paper_code byte (P.code) instead of FP64.
template <bool CODES>
__device__ __forceinline__ void paper_pixel(const PaperParams& P, int x, int y, int ri, int cm, real ct, V3 cn,
                                            int cband, const int (&nm)[4], const real (&nt)[4], const real (&nnx)[4],
                                            const real (&nny)[4], const real (&nnz)[4]) {
    const bool ch = cm != kPaperMiss;
    // get_edge_strength (tracer.cpp:133-178)
    real maxEdge = RV(0.0);
    int eidx = 0;   // index of maxEdge in {0, 0.3, 0.5, 0.6, 0.9} (rtamd::paper_code)
    int valid = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int dx = (i == 0) ? -1 : (i == 1) ? 1 : 0;
        const int dy = (i == 2) ? -1 : (i == 3) ? 1 : 0;
        const int nxp = x + dx, nyp = y + dy;
        if (nxp < 0 || nxp >= P.W || nyp < 0 || nyp >= P.H) continue;
        ++valid;
        const bool nh = nm[i] != kPaperMiss;
        if (ch != nh) {
            maxEdge = dmax(maxEdge, RV(0.9));
            eidx = max(eidx, 4);
            continue;
        }
        if (ch && nh) {
            const real minD = dmin(ct, nt[i]), maxD = dmax(ct, nt[i]);
            if (minD > RV(1e-4) && maxD / minD > RV(3.0)) {
                maxEdge = dmax(maxEdge, RV(0.6));
                eidx = max(eidx, 3);
            }
            const real nd = dot3(cn, v3(nnx[i], nny[i], nnz[i]));
            if (nd < RV(0.2)) {
                maxEdge = dmax(maxEdge, RV(0.5));
                eidx = max(eidx, 2);
            }
            if (cm != nm[i] && nd < RV(0.7)) {
                maxEdge = dmax(maxEdge, RV(0.3));
                eidx = max(eidx, 1);
            }
        }
    }
    if (valid < 4) maxEdge *= RV(0.5);
    const real edge = maxEdge;
    if constexpr (CODES) {
        // distributed frames: the pixel's place in the output alphabet
        // (rtamd::paper_code), decoded bit-exactly on the root after the gather
        const bool h = edge <= RV(0.5) && crosshatch(cband, x, y) != RV(0.0);
        P.code[(size_t)ri * P.W + x] = (uint8_t)(eidx | (valid < 4 ? 8 : 0) | (h ? 16 : 0));
        return;
    }
    V3 o;
    if (edge > RV(0.8)) {
        o = v3(RV(0.0), RV(0.0), RV(0.0));
    } else if (edge > RV(0.5)) {
        o = v3(RV(0.2), RV(0.2), RV(0.2));
    } else {
        const real h = crosshatch(cband, x, y);
        o = v3(h, h, h);
        if (edge > RV(0.3)) {
            const real darken = (edge - RV(0.3)) * RV(0.4);
            o.x *= (RV(1.0) - darken);
            o.y *= (RV(1.0) - darken);
            o.z *= (RV(1.0) - darken);
        }
    }
    double* dst = P.fb + ((size_t)ri * P.W + x) * 3;
    dst[0] = o.x;
    dst[1] = o.y;
    dst[2] = o.z;
}

// A pixel pair's record in one ext row (x even, W even: 8/16-byte loads)
struct FinRec {
    int2 m;
    double2 t, nx, ny, nz;
};
__device__ __forceinline__ FinRec fin_load(const PaperParams& P, size_t i) {
    FinRec r;
    r.m = *reinterpret_cast<const int2*>(P.mat + i);
    r.t = *reinterpret_cast<const double2*>(P.t + i);
    r.nx = *reinterpret_cast<const double2*>(P.nx + i);
    r.ny = *reinterpret_cast<const double2*>(P.ny + i);
    r.nz = *reinterpret_cast<const double2*>(P.nz + i);
    return r;
}
// Pixels x and x + 1 of output row ri (frame row y) from the pair's records
// in the centre (ext index at ci), up and down rows, and their outer
// x-neighbours (loaded here).
template <bool CODES>
__device__ __forceinline__ void paper_finish_pair(const PaperParams& P, int x, int y, int ri, size_t ci, const FinRec& c,
                                                  const FinRec& u, const FinRec& d) {
    const size_t li = ci - (x > 0 ? 1 : 0), rj = ci + 1 + (x + 2 < P.W ? 1 : 0);
    const int ml = paper_mat(P.mat[li]), mr = paper_mat(P.mat[rj]);
    const real tl = P.t[li], tr = P.t[rj];
    const real xl = P.nx[li], xr = P.nx[rj], yl = P.ny[li], yr = P.ny[rj], zl = P.nz[li], zr = P.nz[rj];
    {
        const int nm[4] = {ml, paper_mat(c.m.y), paper_mat(u.m.x), paper_mat(d.m.x)};
        const real nt[4] = {tl, RV(c.t.y), RV(u.t.x), RV(d.t.x)};
        const real nnx[4] = {xl, RV(c.nx.y), RV(u.nx.x), RV(d.nx.x)}, nny[4] = {yl, RV(c.ny.y), RV(u.ny.x), RV(d.ny.x)},
                   nnz[4] = {zl, RV(c.nz.y), RV(u.nz.x), RV(d.nz.x)};
        paper_pixel<CODES>(P, x, y, ri, paper_mat(c.m.x), RV(c.t.x), v3(RV(c.nx.x), RV(c.ny.x), RV(c.nz.x)),
                           paper_band(c.m.x), nm, nt, nnx, nny, nnz);
    }
    {
        const int nm[4] = {paper_mat(c.m.x), mr, paper_mat(u.m.y), paper_mat(d.m.y)};
        const real nt[4] = {RV(c.t.x), tr, RV(u.t.y), RV(d.t.y)};
        const real nnx[4] = {RV(c.nx.x), xr, RV(u.nx.y), RV(d.nx.y)}, nny[4] = {RV(c.ny.x), yr, RV(u.ny.y), RV(d.ny.y)},
                   nnz[4] = {RV(c.nz.x), zr, RV(u.nz.y), RV(d.nz.y)};
        paper_pixel<CODES>(P, x + 1, y, ri, paper_mat(c.m.y), RV(c.t.y), v3(RV(c.nx.y), RV(c.ny.y), RV(c.nz.y)),
                           paper_band(c.m.y), nm, nt, nnx, nny, nnz);
    }
}

// The finish pass: 64x4 threads per block.  Every operand is loaded up front
// in one round of independent loads (neighbours outside the frame clamped
// onto the centre and skipped by paper_pixel; hit/miss is the material slot
// against kPaperMiss).  PAIR (even W): a thread takes two adjacent pixels
// with 8/16-byte loads of both, and their outer x-neighbours.
template <bool CODES, bool PAIR>
__device__ __forceinline__ void paper_finish_px(const PaperParams& P, int x, int ri) {
    const int y = P.rows[ri];
    const int e_up = P.nbr[3 * ri + 0], e_c = P.nbr[3 * ri + 1], e_dn = P.nbr[3 * ri + 2];
    const size_t ci = (size_t)e_c * P.W + x;
    const size_t ui = (size_t)(e_up >= 0 ? e_up : e_c) * P.W + x, di = (size_t)(e_dn >= 0 ? e_dn : e_c) * P.W + x;
    if constexpr (!PAIR) {
        const size_t nidx[4] = {ci - (x > 0 ? 1 : 0), ci + (x + 1 < P.W ? 1 : 0), ui, di};
        int nm[4];
        real nt[4], nnx[4], nny[4], nnz[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            nm[i] = paper_mat(P.mat[nidx[i]]);
            nt[i] = P.t[nidx[i]];
            nnx[i] = P.nx[nidx[i]];
            nny[i] = P.ny[nidx[i]];
            nnz[i] = P.nz[nidx[i]];
        }
        const int mc = P.mat[ci];
        paper_pixel<CODES>(P, x, y, ri, paper_mat(mc), P.t[ci], v3(P.nx[ci], P.ny[ci], P.nz[ci]), paper_band(mc), nm, nt,
                           nnx, nny, nnz);
    } else {
        // rows: c = centre, u = up, d = down; pixels x and x + 1 (x even, W even:
        // every pair is 8/16-byte aligned)
        paper_finish_pair<CODES>(P, x, y, ri, ci, fin_load(P, ci), fin_load(P, ui), fin_load(P, di));
    }
}

// RT_FINISH_RPT row rounds per block: a 64x4-thread block finishes 4 rows per
// round, so a round's up / down neighbour records were the previous round's
// centre rows (L1 / L2-hot) and only a block's first and last rows are read
// again by another block.
#ifndef RT_FINISH_RPT
#define RT_FINISH_RPT 1
#endif
// RT_FINISH_BR rows per block (64 x BR threads): a block's rows share their
// neighbour rows, only its first and last rows' are read by another block.
// (Measured and rejected in round 6: one wave walking down a 128-pixel column
// strip, its up / centre / down records kept in registers so that every
// record row is read once: config 5 3.58 -> 3.65-3.68 ms for 8-32 rows per
// wave, profiles/r06_ab/ab_finish_walk.txt.)
#ifndef RT_FINISH_BR
#define RT_FINISH_BR 4
#endif
constexpr int kFinishRounds = RT_FINISH_RPT;
constexpr int kFinishRows = RT_FINISH_BR;
template <bool CODES, bool PAIR>
__global__ __launch_bounds__(64 * kFinishRows) void k_paper_finish(PaperParams P) {
    const int xt = blockIdx.x * 64 + (threadIdx.x & 63);
    const int x = PAIR ? 2 * xt : xt;
    if (x >= P.W) return;
    for (int k = 0; k < kFinishRounds; ++k) {
        const int ri = (blockIdx.y * kFinishRounds + k) * kFinishRows + (threadIdx.x >> 6);
        if (ri >= P.n_rows) return;
        paper_finish_px<CODES, PAIR>(P, x, ri);
    }
}

// bv: the wave BVH kernels, whose object list is the Morton-ordered one
DevScene make_scene(const SceneView& V, bool bv = false) {
    DevScene S;
    S.nodes = static_cast<const NodeT*>(V.nodes);
    S.mats = static_cast<const MatT*>(V.mats);
    S.lights = static_cast<const LightT*>(V.lights);
    S.dlights = static_cast<const DLightT*>(V.dlights);
    S.objs = bv ? V.wobjs : V.objs;
    S.ops = V.ops;
    S.gb = V.gb;
    S.ctab = reinterpret_cast<const float4*>(bv ? V.wctab : V.ctab);
    S.lrec = reinterpret_cast<const float4*>(bv ? V.lwrec : V.lrec);
    S.lgb = reinterpret_cast<const float4*>(V.lgb);
    S.n_gb = V.n_gb;
    S.fold = static_cast<const FoldT*>(V.fold);
    S.worig = bv ? V.worig : nullptr;
    S.wchunk = reinterpret_cast<const float4*>(bv ? V.wchunk : nullptr);
    S.n_chunks = bv ? V.n_chunks : 0;
    S.n_lights = V.n_lights;
    S.n_dlights = V.n_dlights;
    S.n_bounded = V.n_bounded;
    S.n_lead = bv ? 0 : V.n_lead;
    S.n_objs = bv ? V.n_wobjs : V.n_objs;
    S.cam_nx = V.cam_nx;
    S.cam_ny = V.cam_ny;
    S.rec_limit = V.rec_limit;
    S.cull = V.cull;
    for (int i = 0; i < 3; ++i) {
        S.eye[i] = (real)V.eye[i];
        S.P[i] = (real)V.P[i];
    }
    S.Lx = (real)V.Lx;
    S.Ly = (real)V.Ly;
    S.medium_index = (real)V.medium_index;
    S.bg_mat = V.bg_mat;
    return S;
}

// Dynamic LDS of the kernels that shade (lds_pool): one region per wave
constexpr size_t kStdPool = pool_bytes(kStdThreads), kPaperPool = pool_bytes(kPaperThreads);
// the paper primary's grid from the host's 16x16-pixel units
inline dim3 pgrid(dim3 g) { return kPaperWPB == 4 ? g : dim3(2 * g.x, 2 * g.y); }

// The plain kernels (PL) are built for the FP64 namespace only (RT_NO_PLAIN:
// the FP32 diagnostic build keeps one variant per choice).
#ifdef RT_NO_PLAIN
constexpr bool kPlainKernels = false;
#else
constexpr bool kPlainKernels = true;
#endif
template <int WV>
void launch_lean(bool c, bool pl, dim3 grid, hipStream_t st, const DevScene& S, const StdParams& P) {
    if (c) hipLaunchKernelGGL((k_std_lean<true, WV>), grid, dim3(kStdThreads), kStdPool, st, S, P);
    else if (kPlainKernels && pl) hipLaunchKernelGGL((k_std_lean<false, WV, kPlainKernels>), grid, dim3(kStdThreads), kStdPool, st, S, P);
    else hipLaunchKernelGGL((k_std_lean<false, WV>), grid, dim3(kStdThreads), kStdPool, st, S, P);
}
template <int WV>
void launch_secw(bool c, bool pl, dim3 grid, hipStream_t st, const DevScene& S, const StdParams& P) {
    if (c) hipLaunchKernelGGL((k_std_secw<true, WV>), grid, dim3(kStdThreads), kStdPool, st, S, P);
    else if (kPlainKernels && pl) hipLaunchKernelGGL((k_std_secw<false, WV, kPlainKernels>), grid, dim3(kStdThreads), kStdPool, st, S, P);
    else hipLaunchKernelGGL((k_std_secw<false, WV>), grid, dim3(kStdThreads), kStdPool, st, S, P);
}
template <int WV>
void launch_paper_lean(bool c, bool pl, dim3 grid, hipStream_t st, const DevScene& S, const PaperParams& P) {
    // (timed launches: never op-counting ones, rt_frame_trace)
    if (c) hipLaunchKernelGGL((k_paper_primary_lean<true, WV>), pgrid(grid), dim3(kPaperThreads), kPaperPool, st, S, P);
    else if (kPlainKernels && pl) {
        if (P.gtime) hipLaunchKernelGGL((k_paper_primary_lean<false, WV, true, kPlainKernels>), pgrid(grid), dim3(kPaperThreads), kPaperPool, st, S, P);
        else hipLaunchKernelGGL((k_paper_primary_lean<false, WV, false, kPlainKernels>), pgrid(grid), dim3(kPaperThreads), kPaperPool, st, S, P);
    } else if (P.gtime) hipLaunchKernelGGL((k_paper_primary_lean<false, WV, true>), pgrid(grid), dim3(kPaperThreads), kPaperPool, st, S, P);
    else hipLaunchKernelGGL((k_paper_primary_lean<false, WV>), pgrid(grid), dim3(kPaperThreads), kPaperPool, st, S, P);
}

template <bool E, bool D, bool SEC, bool WV = false>
void launch_std_c(bool c, dim3 grid, hipStream_t st, const DevScene& S, const StdParams& P) {
    if (c) hipLaunchKernelGGL((k_std<E, D, SEC, true, WV>), grid, dim3(kStdThreads), kStdPool, st, S, P);
    else hipLaunchKernelGGL((k_std<E, D, SEC, false, WV>), grid, dim3(kStdThreads), kStdPool, st, S, P);
}

template <bool E, bool D>
void launch_paper_c(bool c, dim3 grid, hipStream_t st, const DevScene& S, const PaperParams& P) {
    // (timed launches: never op-counting ones, rt_frame_trace)
    if (c) hipLaunchKernelGGL((k_paper_primary<E, D, true>), pgrid(grid), dim3(kPaperThreads), kPaperPool, st, S, P);
    else if (P.gtime) hipLaunchKernelGGL((k_paper_primary<E, D, false, true>), pgrid(grid), dim3(kPaperThreads), kPaperPool, st, S, P);
    else hipLaunchKernelGGL((k_paper_primary<E, D, false>), pgrid(grid), dim3(kPaperThreads), kPaperPool, st, S, P);
}

}  // namespace

// Eager scenes always use D.  Each variant gets its own register allocation.
void launch_std(bool e, bool d, bool sec, bool c, hipStream_t st, const SceneView& V, const StdParams& P) {
    const bool bv = !e && !d && V.wave_cull && V.n_chunks > 0;
    const DevScene S = make_scene(V, bv);
    const dim3 grid((P.W + kStdBlockX - 1) / kStdBlockX, (P.n_rows + kStdBlockY - 1) / kStdBlockY);
#ifdef RT_GENERAL_ONLY
    // big-stack build: only the general variants (every feature, scratch stacks)
    (void)e;
    (void)d;
    if (sec) launch_std_c<true, true, true>(c, grid, st, S, P);
    else launch_std_c<true, true, false>(c, grid, st, S, P);
#else
    const bool wv = V.wave_cull;
    const bool pl = V.plain != 0;
    if (e) {
        if (sec) launch_std_c<true, true, true>(c, grid, st, S, P);
        else launch_std_c<true, true, false>(c, grid, st, S, P);
    } else if (d) {
        if (sec) launch_std_c<false, true, true>(c, grid, st, S, P);
        else launch_std_c<false, true, false>(c, grid, st, S, P);
    } else {
        if (sec) {
            if (bv) launch_secw<2>(c, pl, grid, st, S, P);
            else if (wv) launch_secw<1>(c, pl, grid, st, S, P);
            else launch_std_c<false, false, true>(c, grid, st, S, P);
        } else if (bv) {
            launch_lean<2>(c, pl, grid, st, S, P);
        } else if (wv) {
            launch_lean<1>(c, pl, grid, st, S, P);
        } else {
            launch_lean<0>(c, pl, grid, st, S, P);
        }
    }
#endif
}

void launch_paper(bool e, bool d, bool c, dim3 grid, hipStream_t st, const SceneView& V, const PaperParams& P) {
    const bool bv = !e && !d && V.wave_cull && V.n_chunks > 0;
    const DevScene S = make_scene(V, bv);
#ifdef RT_GENERAL_ONLY
    (void)e;
    (void)d;
    launch_paper_c<true, true>(c, grid, st, S, P);
#else
    const bool wv = V.wave_cull;
    const bool pl = V.plain != 0;
    if (e) launch_paper_c<true, true>(c, grid, st, S, P);
    else if (d) launch_paper_c<false, true>(c, grid, st, S, P);
    else if (bv) launch_paper_lean<2>(c, pl, grid, st, S, P);
    else if (wv) launch_paper_lean<1>(c, pl, grid, st, S, P);
    else launch_paper_lean<0>(c, pl, grid, st, S, P);
#endif
}

// The kernel launch_std / launch_paper pick for a variant (resource queries).
const void* std_kernel(bool e, bool d, bool sec, bool wv, bool bv, bool pl) {
#ifdef RT_GENERAL_ONLY
    (void)e, (void)d, (void)wv, (void)bv, (void)pl;
    return sec ? (const void*)k_std<true, true, true, false> : (const void*)k_std<true, true, false, false>;
#else
    if (e) return sec ? (const void*)k_std<true, true, true, false> : (const void*)k_std<true, true, false, false>;
    if (d) return sec ? (const void*)k_std<false, true, true, false> : (const void*)k_std<false, true, false, false>;
    pl = pl && kPlainKernels;
    if (sec) {
        if (bv) return pl ? (const void*)k_std_secw<false, 2, kPlainKernels> : (const void*)k_std_secw<false, 2>;
        if (wv) return pl ? (const void*)k_std_secw<false, 1, kPlainKernels> : (const void*)k_std_secw<false, 1>;
        return (const void*)k_std<false, false, true, false>;
    }
    if (bv) return pl ? (const void*)k_std_lean<false, 2, kPlainKernels> : (const void*)k_std_lean<false, 2>;
    if (wv) return pl ? (const void*)k_std_lean<false, 1, kPlainKernels> : (const void*)k_std_lean<false, 1>;
    return pl ? (const void*)k_std_lean<false, 0, kPlainKernels> : (const void*)k_std_lean<false, 0>;
#endif
}

// The trace kernels' workgroup size and dynamic LDS (resource queries)
int kernel_block_threads(bool paper) { return paper ? kPaperThreads : kStdThreads; }
size_t kernel_pool_bytes(bool paper) { return paper ? kPaperPool : kStdPool; }

const void* paper_kernel(bool e, bool d, bool wv, bool bv, bool pl) {
#ifdef RT_GENERAL_ONLY
    (void)e, (void)d, (void)wv, (void)bv, (void)pl;
    return (const void*)k_paper_primary<true, true, false>;
#else
    if (e) return (const void*)k_paper_primary<true, true, false>;
    if (d) return (const void*)k_paper_primary<false, true, false>;
    pl = pl && kPlainKernels;
    if (bv) return pl ? (const void*)k_paper_primary_lean<false, 2, false, kPlainKernels> : (const void*)k_paper_primary_lean<false, 2>;
    if (wv) return pl ? (const void*)k_paper_primary_lean<false, 1, false, kPlainKernels> : (const void*)k_paper_primary_lean<false, 1>;
    return pl ? (const void*)k_paper_primary_lean<false, 0, false, kPlainKernels> : (const void*)k_paper_primary_lean<false, 0>;
#endif
}

void launch_paper_finish(dim3 grid, hipStream_t st, const PaperParams& P) {
    // (grid.x covers W pixels one per thread; even W: two per thread; grid.y
    // kFinishRows * kFinishRounds rows per block)
    grid.y = (P.n_rows + kFinishRows * kFinishRounds - 1) / (kFinishRows * kFinishRounds);
    const dim3 blk(64 * kFinishRows);
    if (P.W % 2 == 0) {
        const dim3 g2((P.W / 2 + 63) / 64, grid.y);
        if (P.code) hipLaunchKernelGGL((k_paper_finish<true, true>), g2, blk, 0, st, P);
        else hipLaunchKernelGGL((k_paper_finish<false, true>), g2, blk, 0, st, P);
    } else {
        if (P.code) hipLaunchKernelGGL((k_paper_finish<true, false>), grid, blk, 0, st, P);
        else hipLaunchKernelGGL((k_paper_finish<false, false>), grid, blk, 0, st, P);
    }
}

}  // namespace RT_NS
