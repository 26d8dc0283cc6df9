/*
 * rt_test.h — test hooks exported by librtamd.so (not part of the drop-in
 * boundary; used by tests/ to check the jitter-stream machinery in isolation).
 */
#ifndef RT_TEST_H
#define RT_TEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* CPU check of the GF(2) jump polynomials (csrc/host/mt_poly.cpp): for
 * tree levels j < levels and m = 1..7, applying x^(624*K*m*8^j) mod phi to
 * the seed window must equal advancing it m*8^j*K twist blocks
 * sequentially.  Returns the number of mismatching polynomials (0 = all
 * good), -1 on error. */
int rt_test_mt_jump_cpu(int K_blocks, int levels);

/* GPU: generate the jitter stream for output indices [q0, q1) (even) with the
 * device jump/fill kernels at segment length K_blocks twist blocks and copy
 * uniform draws [first, first+count) (draw index = output index / 2) to
 * out_host.  K_blocks == 0 selects the frame path instead: the resident
 * checkpoint table (every 64 twist blocks, built by the same jump tree) and
 * the one-wavefront fill kernel.  Returns an rt_status. */
int rt_test_jitter_device(int K_blocks, int64_t q0, int64_t q1, int64_t first, int64_t count, double* out_host);

/* Host-only: compile a scene to its device object table and report
 * out[8] = {objects incl. cull headers, object cull groups, their members,
 * program ops, CSG operand groups (OP_IVL_GROUP), their members, has eager
 * programs, max CSG operand depth}.  No device is touched. */
struct rt_scene;
int rt_test_compile_info(const struct rt_scene* s, int32_t* out);

/* Host-only: the wave BVH of a scene (CompiledScene::wobjs ...).  counts[2] =
 * {objects in the wave list, chunks} (both 0: no BVH); up to cap_objs
 * entries of worig (each listed object's index in the compiled object table)
 * and of wctab (8 floats per object: its cull record), up to cap_chunks
 * chunk records (8 floats each). */
int rt_test_wave_bvh(const struct rt_scene* s, int32_t* counts, int32_t* worig, float* wctab, int cap_objs,
                     float* wchunk, int cap_chunks);

/* Resources of the trace kernel rt_render would launch for this scene, mode
 * and flags (hipFuncGetAttributes + occupancy query): out[8] = {VGPRs per
 * lane, scratch bytes per lane, LDS bytes per workgroup (static + the
 * dynamic shading pool of 10 KiB per wave), resident
 * workgroups per CU, waves per SIMD, max threads per block, wave-level
 * culling variant, reflection/refraction variant}.  Needs a device. */
int rt_test_kernel_info(const struct rt_scene* s, int mode, int flags, int32_t* out);

/* The name of that kernel as rocprofv3 reports it (e.g. "rtd::k_std_lean<false, true>"),
 * NUL-terminated into out[0 .. cap).  Host only. */
int rt_test_kernel_name(const struct rt_scene* s, int mode, int flags, char* out, int cap);

/* GPU: the shared-denominator division of the device code (rt_device.hpp
 * div3) next to the compiler's own division on the same inputs:
 * div3_host[3i+k] and plain_host[3i+k] = a[3i+k] / b[i].  Tests require the
 * two to be bit-identical. */
int rt_test_div3(const double* a_host, const double* b_host, int n, double* div3_host, double* plain_host);

/* Host only: the precomputed mt19937 tree jump polynomials in `path` (the
 * build's lib/mt19937_tree.polys, read by the jitter generator) against the
 * same polynomials computed in this process, first `levels` levels.
 * Returns 0 equal, 1 different, 2 file missing / short / corrupt. */
int rt_test_mt_poly_file(const char* path, int levels);

/* GPU, one device: the distributed frame of rt_render_dist with `world`
 * (<= 16) simulated ranks running CONCURRENTLY on the current device, one
 * host thread per rank with its own streams and device workspace, through the
 * product's rank path (dist_frame) with RCCL replaced by a same-device
 * transport that keeps its contract (host rendezvous + device copies / max
 * reduction on each rank's collective stream, timeouts): partition, row
 * chunks, both frame agreements and their verdicts, gathers, placement on the
 * root.  run->frames consecutive frames; in frame run->fault_frame rank
 * run->fault_rank gets run->fault:
 *   TRACE       its trace fails at its middle chunk (after the agreement)
 *   SETUP       it fails before its frame begins (reported in the agreement)
 *   DESC_H      it is given H + 1 (the ranks disagree on the descriptor)
 *   DESC_FLAGS  it is given flags ^ RT_FLAG_NO_CULL
 *   ABSENT      it does not take part in that frame (a dead peer; the others
 *               time out after run->timeout_ms)
 *   DESC_SCENE  it renders run->alt_scene instead (another scene content)
 *   DESC_SHED   its root strip shed (RT_ROOT_SHED_*) is one per mille higher
 * run->frame_scenes (may be NULL; entries may be NULL): frame fr renders
 * frame_scenes[fr] instead of s, on the same ranks (a rank handle reused
 * across scenes).
 * Per frame fr and rank r: run->rc[fr*world + r] (an rt_status, or
 * RT_TEST_RANK_ABSENT), run->ms[...] (the call's wall time), and the error
 * text in run->msgs[(fr*world + r) * msg_cap ...] (may be NULL).  The root's
 * frame of every successful frame fr goes to fb_host + fr*W*H*3 (doubles) or,
 * with run->rgb8, rgb8_host + fr*W*H*3 (either may be NULL).  timeout_ms <= 0:
 * RT_DIST_TIMEOUT_MS / 120 s.  Returns an rt_status for the harness itself. */
enum {
    RT_TEST_FAULT_NONE = 0,
    RT_TEST_FAULT_TRACE = 1,
    RT_TEST_FAULT_SETUP = 2,
    RT_TEST_FAULT_DESC_H = 3,
    RT_TEST_FAULT_DESC_FLAGS = 4,
    RT_TEST_FAULT_ABSENT = 5,
    RT_TEST_FAULT_DESC_SCENE = 6,
    RT_TEST_FAULT_DESC_SHED = 7
};
#define RT_TEST_RANK_ABSENT 1
typedef struct rt_test_dist_run {
    int world, rgb8, frames;
    int fault_rank, fault, fault_frame;
    int timeout_ms;
    int msg_cap;
    int* rc;
    double* ms;
    char* msgs;
    const struct rt_scene* const* frame_scenes;
    const struct rt_scene* alt_scene;
    double* split;   /* may be NULL: rt_dist_frame_split of rank r after frame fr at
                        split[(fr*world + r) * 10 ...] (successful frames) */
} rt_test_dist_run;
int rt_test_dist_threads(const struct rt_scene* s, int W, int H, int mode, int flags, rt_test_dist_run* run,
                         double* fb_host, uint8_t* rgb8_host);
/* rt_test_dist_threads for one fault-free frame: the root's frame to fb_host
 * (W*H*3 doubles) or, with rgb8, rgb8_host. */
int rt_test_render_dist_sim(const struct rt_scene* s, int W, int H, int mode, int flags, int world, int rgb8,
                            double* fb_host, uint8_t* rgb8_host);

/* GPU, one device: a world-1 rt_dist WITH a real RCCL communicator
 * (ncclCommInitRank over one rank) whose rt_render_dist frames take the
 * multi-GPU collective path (row chunks, ncclGather to root 0, placement).
 * Free with rt_dist_destroy. */
struct rt_dist;
int rt_test_dist_create_rccl1(struct rt_dist** out);
/* Fault injection on the next frame of d (rt_render_dist): 1 = this rank's
 * trace fails at its middle chunk, 2 = the collective stream is held past the
 * rank's timeout (bounded, >= 10 s: the holding kernel always ends), 3 = this
 * rank fails before its frame begins. */
int rt_test_dist_inject(struct rt_dist* d, int what);
/* CPU: Pokeball::pick_region_material's acos comparisons as thresholds
 * (rtamd::pokeball_thresholds, scene_compile.hpp): out2[0] = xb, the least x
 * in [-1, 1] with acos(x) <= btn_outer (2: none), out2[1] = xi, the greatest
 * x with acos(x) >= max(0, btn_outer - ring_width) (-2: none).  Returns 0. */
int rt_test_pokeball_thresholds(double btn_outer, double ring_width, double* out2);
/* CPU: the paper-mode output code decoder of distributed frames
 * (rtamd::paper_code_value): bits 0-2 edge index in {0, 0.3, 0.5, 0.6, 0.9},
 * bit 3 halved at the frame border, bit 4 the hatch bit (white). */
double rt_test_paper_code_value(int code);
/* CPU: the paper-mode primary launch order (rt_render.hip order_paper_groups)
 * applied in place to list[0, n) (n a multiple of 16; entries are ext
 * indices, -1 padding), given the measured cost of the 8-entry group whose
 * first entry is e in cost[e] (0 = unmeasured).  Returns 0. */
int rt_test_paper_order(int32_t* list, int n, const uint32_t* cost, int n_cost);
/* GPU: one simulated rank (rank of world) of a distributed frame on the
 * current device through the product's rank path, the RCCL gather replaced by
 * a device copy (rank 0 also places every slot).  Ranks are cached, so a
 * repeated call times a warm rank.  For per-rank timing (tools/sim_ranks.py). */
int rt_test_dist_sim_rank(const struct rt_scene* s, int W, int H, int mode, int flags, int world, int rank, int rgb8,
                          struct rt_stats* stats);

#ifdef __cplusplus
}
#endif
#endif
