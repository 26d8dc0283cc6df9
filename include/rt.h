/*
 * rt.h — C-ABI of the MI355X-native per-pixel ray-trace path.
 *
 * This is the drop-in boundary for the reference's hot path
 * (alp-aydin/Raytracing-Project).  Every entry point is plain C: pointers,
 * sizes and integer error codes, no C++ types, no exceptions, no torch types.
 *
 * Reference seams replaced (paths relative to the reference repo root):
 *   rt_scene_load_json_text  <- jsonio::load_scene_from_json_text
 *                               raytracer/src/json_loader.cpp:458-490
 *   rt_scene_load_json_file  <- jsonio::load_scene_from_json
 *                               raytracer/src/json_loader.cpp:499-503
 *   rt_render                <- Tracer::render (standard + paper mode)
 *                               raytracer/src/tracer.cpp:247-305, tracer.h:18-35
 *   rt_render_multi          <- Tracer::render over the GPUs of one node (row
 *                               strips + RCCL gather)
 *   rt_render_rgb8           <- Tracer::render + framebuffer_to_mat_bgr8
 *                               (main.cpp:19-34, 74-89) on the device
 *   rt_dist_* / rt_render_dist <- the same for one process per GPU
 *   rt_render_rows_device    <- the same loop restricted to a set of output
 *                               rows (multi-GPU row tiling)
 *   rt_frame_begin/trace/end <- the same loop, split so that row chunks can
 *                               be gathered while later chunks are traced
 *   rt_scatter_rows_device   <- (no reference equivalent: places gathered row
 *                               bands into the full framebuffer on rank 0)
 *   rt_framebuffer_to_rgb8   <- framebuffer_to_mat_bgr8 / toByte
 *                               raytracer/src/main.cpp:19-34, core.h:313-316
 *   rt_write_png             <- cv::imwrite (main.cpp:86-89)
 *
 * The scene is held in a flattened intermediate representation
 * (rt_scene_desc) produced by the host loader.  The same struct is consumed
 * by the GPU renderer and by the CPU oracle under oracle/ (test only).
 *
 * Library split:
 *   librt_host.so — loader, IR, PNG writer (pure host C++17, no HIP).
 *   librtamd.so   — HIP/gfx950 renderer; links librt_host.so.
 */
#ifndef RT_H
#define RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 6   /* 2: rt_scene_desc gained directional lights
                              3: rt_stats gained the output-path timings; multi-GPU
                                 and device-output entry points (rt_render_multi,
                                 rt_render_rgb8, rt_dist_*)
                              4: rt_shutdown, device-buffer utilities, rt_dist_reduce_max /
                                 rt_dist_barrier
                              5: rt_dist_set_timeout, per-frame rank agreement,
                                 rt_host_register / rt_host_unregister
                              6: rt_dist_frame_split, rt_warmup; the frame descriptor
                                 carries the scene hash and the root strip shed */

/* ---------------------------------------------------------------- errors */
enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = -1,   /* null pointer / bad size                      */
    RT_ERR_PARSE = -2,         /* "JSON parse error: ..." (json_loader.cpp:485) */
    RT_ERR_PROCESSING = -3,    /* "JSON processing error: ..." (:487)          */
    RT_ERR_IO = -4,            /* "Cannot open JSON file: ..." (:501) / PNG write */
    RT_ERR_HIP = -5,           /* HIP runtime failure (message in rt_last_error) */
    RT_ERR_UNSUPPORTED = -6,   /* scene exceeds a compiled device limit          */
    RT_ERR_NO_DEVICE = -7      /* no HIP device / extension missing             */
};

/* Last error message of the calling thread ("" if none). */
const char* rt_last_error(void);
int rt_abi_version(void);

/* -------------------------------------------------------- scene IR types */
enum rt_node_kind {
    RT_NODE_SPHERE = 0,       /* geometry.h:79-109     Sphere                    */
    RT_NODE_HALFSPACE = 1,    /* geometry.h:112-158    HalfSpace                 */
    RT_NODE_POKEBALL = 2,     /* geometry.h:161-242    Pokeball                  */
    RT_NODE_TRANSLATION = 3,  /* transform.h:87-111    Translation               */
    RT_NODE_SCALING = 4,      /* transform.h:117-141   Scaling                   */
    RT_NODE_ROTATION = 5,     /* transform.h:150-185   Rotation                  */
    RT_NODE_CSG = 6           /* csg.h:13-49           CSG                       */
};

enum rt_csg_op { RT_CSG_UNION = 0, RT_CSG_INTERSECTION = 1, RT_CSG_DIFFERENCE = 2 };

enum rt_pokeball_region {
    RT_PB_TOP = 0, RT_PB_BOTTOM = 1, RT_PB_BELT = 2, RT_PB_RING = 3, RT_PB_BUTTON = 4
};

/* Material — geometry.h:5-22.  Every JSON colour block instance (and each
 * of a pokeball's five region materials) gets its own index: the paper-mode
 * edge detector compares material identity (tracer.cpp:170). */
typedef struct rt_material {
    double albedo[3];
    double ambient[3];
    double kd, ks, kr, kt;
    double shininess;
    double refractive_index;
} rt_material;

/* Parameter layout of rt_node.v per kind:
 *   SPHERE      v[0..2]=centre  v[3]=radius
 *   HALFSPACE   v[0..2]=p0      v[3..5]=unit normal (normalised as geometry.h:124-134)
 *   POKEBALL    v[0..2]=centre  v[3]=radius  v[4]=belt_half  v[5]=button_outer
 *               v[6]=ring_width v[7..9]=unit button_dir (Dir3::normalized)
 *   TRANSLATION/SCALING/ROTATION
 *               v[0..11]  = forward matrix rows 0..2 (4 columns, row-major)
 *               v[12..23] = inverse matrix rows 0..2 (Matrix4::inverse, core.h:239)
 *   CSG         (no parameters; op in rt_node.op)
 * aux[] keeps the raw constructor inputs (used only to rebuild reference
 * objects in oracle/_ref): HALFSPACE aux[0..2]=normal as given,
 * POKEBALL aux[0..2]=button_dir as given, ROTATION aux[0]=angle in radians,
 * TRANSLATION/SCALING aux[0..2]=factors.
 * Children: a (transform subject / CSG left), b (CSG right); -1 if unused.
 * Materials: mat (sphere / halfspace), mats[5] (pokeball, rt_pokeball_region order). */
typedef struct rt_node {
    int32_t kind;
    int32_t a, b;
    int32_t op;        /* rt_csg_op for CSG; axis 0/1/2 for ROTATION */
    int32_t mat;
    int32_t mats[5];
    double v[24];
    double aux[4];
} rt_node;

typedef struct rt_light {      /* scene.h:21-26 PointLight */
    double pos[3];
    double intensity[3];
} rt_light;

/* scene.h:10-15 DirectionalLight.  The JSON loader never creates one
 * (json_loader.cpp has no key for it); they are reachable through
 * rt_scene_from_desc, as the reference's Scene::dir_lights is through its API,
 * and shaded before the point lights (shading.cpp:45-76). */
typedef struct rt_dir_light {
    double dir[3];             /* direction from the light toward the scene (incident) */
    double radiance[3];
} rt_dir_light;

typedef struct rt_camera {     /* camera.h:7-79 Camera + ScreenSpec */
    double eye[3];
    double P[3];
    double Lx, Ly;
    int32_t dpi;
    int32_t pad_;
} rt_camera;

typedef struct rt_scene_desc {
    rt_camera camera;
    double background[3];      /* scene.h:40 */
    double ambient[3];         /* scene.h:43 */
    double medium_index;       /* scene.h:45 */
    int32_t recursion_limit;   /* scene.h:47 (default 5) */
    int32_t n_lights;
    const rt_light* lights;
    int32_t n_materials;
    int32_t n_nodes;
    const rt_material* materials;
    const rt_node* nodes;
    int32_t n_objects;         /* top-level objects, in JSON order */
    int32_t pad_;
    const int32_t* objects;    /* node index of each top-level object */
    int32_t n_dir_lights;      /* scene.h:36 dir_lights (ABI 2) */
    int32_t pad2_;
    const rt_dir_light* dir_lights;
} rt_scene_desc;

/* ScreenSpec::nx/ny (camera.h:19-21): max(1, int(round(L * dpi))). */
int rt_camera_width(const rt_camera* cam);
int rt_camera_height(const rt_camera* cam);

/* -------------------------------------------------------- scene handles */
typedef struct rt_scene rt_scene;   /* opaque: owns the IR arrays */

/* Parse JSON text with the reference schema.  On failure *out is NULL and
 * rt_last_error() holds the message (same prefixes as the reference). */
int rt_scene_load_json_text(const char* text, size_t len, rt_scene** out);
int rt_scene_load_json_file(const char* path, rt_scene** out);
/* Deep-copy a caller-built IR into an owned scene. */
int rt_scene_from_desc(const rt_scene_desc* desc, rt_scene** out);
const rt_scene_desc* rt_scene_get_desc(const rt_scene* s);
void rt_scene_destroy(rt_scene* s);

/* ------------------------------------------------------------- render */
enum rt_mode { RT_MODE_STANDARD = 0, RT_MODE_PAPER = 1 };

typedef struct rt_stats {
    uint64_t rays_intersect;   /* Scene::intersect calls, reference definition (scene.cpp:10) */
    uint64_t rays_occluded;    /* Scene::occluded calls (scene.cpp:33)                         */
    uint64_t rays_traced;      /* intersect+occluded queries actually evaluated on device      */
    uint64_t pixels;
    double ms_rng;             /* jitter-stream generation (device)                             */
    double ms_kernel;          /* trace kernels (device)                                        */
    double ms_total;           /* whole call, host wall clock                                   */
    uint64_t ops[16];          /* per-op counters when RT_FLAG_COUNT_OPS is set (rt_op_counter) */
    /* ABI 3: the rest of the frame's wall clock */
    double ms_gather;          /* multi-GPU: RCCL gather of the row strips + placement on the root (device) */
    double ms_tobyte;          /* device toByte + RGB packing (rt_render_rgb8)                      */
    double ms_d2h;             /* device -> host copy of the result                                 */
    int32_t n_gpus;            /* devices that rendered                                             */
    int32_t pad_;
} rt_stats;

/* Op counters used by the FLOP model. */
enum rt_op_counter {
    RT_OPC_SPHERE_ISECT = 0,    /* Sphere::intersect calls                 */
    RT_OPC_SPHERE_ISECT_HIT,    /*   ... that hit                          */
    RT_OPC_SPHERE_IVL,          /* Sphere::interval calls (incl. pokeball)  */
    RT_OPC_SPHERE_IVL_HIT,      /*   ... that produced an interval         */
    RT_OPC_HALF_ISECT,          /* HalfSpace::intersect calls              */
    RT_OPC_HALF_ISECT_HIT,
    RT_OPC_HALF_IVL,
    RT_OPC_POKE_REGION,         /* Pokeball::pick_region_material          */
    RT_OPC_CSG_COMBINE,         /* CSG::interval combine steps             */
    RT_OPC_XFORM,               /* transform ray mappings                  */
    RT_OPC_SHADE_LIGHT,         /* per-light shading evaluations           */
    RT_OPC_SHADE_SPEC,          /* ... with a specular pow()               */
    RT_OPC_SECONDARY,           /* reflection/refraction spawns            */
    RT_OPC_CULLED,              /* subtree evaluations skipped by a wave-uniform bound cull */
    RT_OPC_LIGHT_EVAL,          /* point-light loop iterations in shading  */
    RT_OPC_SHADE_CALL           /* shade_lambert_phong calls with a material */
};

enum rt_flags {
    RT_FLAG_NONE = 0,
    RT_FLAG_COUNT_OPS = 1,      /* fill rt_stats.ops (slower, instrumented kernels) */
    RT_FLAG_NO_CULL = 2,        /* disable wave-uniform bounding-sphere culling    */
    RT_FLAG_FP32 = 4,           /* NON-PARITY fast path: trace in
                                   FP32 on float copies of the scene; framebuffer stays
                                   double.  Not within the 1e-5 parity tolerance.   */
    RT_FLAG_NO_BVH = 8,         /* scenes of more than 256 top-level objects (the wave
                                   BVH threshold kWaveBvhMin, scene_compile.hpp) and no
                                   eager programs: wave-level culling without the wave
                                   BVH (A/B; results are identical).  No effect on
                                   smaller scenes, which never build the BVH.        */
    RT_FLAG_FORCE_BVH = 16      /* a scene that has a wave BVH uses it on every frame.
                                   Without this flag (or RT_FLAG_NO_BVH) the first two
                                   frames of a frame shape try it on and off and later
                                   frames take the faster (identical results). */
};

/* Tracer::render: render the whole frame into a caller-owned host buffer of
 * W*H*3 doubles (row-major, top row first, RGB), exactly like the
 * reference's std::vector<Color>.  W,H must be > 0 (the reference returns
 * silently otherwise, tracer.cpp:248 — here RT_ERR_INVALID_ARG).
 * Uses the current HIP device; blocks until done. */
int rt_render(const rt_scene* s, int W, int H, int mode, int flags,
              double* fb_host, rt_stats* stats);

/* Tracer::render over n_gpus HIP devices of THIS process (n_gpus <= 0: all
 * visible devices): every device renders interleaved strips of RT_STRIP_ROWS
 * (paper mode: RT_PAPER_STRIP_ROWS) output rows (a weighted round robin over the strips, rotated every
 * round, device 0 lighter for its placement work: rt_dist_rows_mode), and the strips reach
 * device 0 through RCCL ncclGather over xGMI (one collective per row chunk,
 * overlapped with the tracing of the next chunk) before the one D2H copy into
 * fb_host.  The result is bit-identical to rt_render (same kernels, same
 * jitter-stream offsets).  n_gpus == 1 is rt_render. */
int rt_render_multi(const rt_scene* s, int W, int H, int mode, int flags, int n_gpus, double* fb_host,
                    rt_stats* stats);

/* Tracer::render followed by framebuffer_to_mat_bgr8's toByte
 * (main.cpp:19-34, core.h:313-316) on the device(s), RGB order, top row
 * first: only 3 bytes per pixel cross xGMI and PCIe.
 * This is the CLI's path (`ray ... --gpus N`). */
int rt_render_rgb8(const rt_scene* s, int W, int H, int mode, int flags, int n_gpus, uint8_t* rgb8_host,
                   rt_stats* stats);

/* ------------------------------------------- one process per GPU (RCCL)
 * For launchers that start one process per device (torchrun, MPI): rank 0
 * calls rt_dist_get_id and hands the RT_DIST_ID_BYTES bytes to every rank,
 * each rank binds its current HIP device with rt_dist_create, and every
 * frame each rank calls rt_render_dist[_rgb8]: it renders its strips
 * (rt_dist_rows) and rank 0 receives the whole frame in its device buffer
 * (the ncclGather of rt_render_multi).  Non-root ranks pass NULL.  The call
 * returns when this rank's part (and on rank 0 the whole frame) is done;
 * stats are this rank's (ray counts of its rows). */
#define RT_STRIP_ROWS 8          /* standard mode */
#define RT_PAPER_STRIP_ROWS 30   /* paper mode: + 2 neighbour rows per strip = 32, four 8-row waves */
#define RT_DIST_ID_BYTES 128
typedef struct rt_dist rt_dist;
int rt_dist_get_id(uint8_t id[RT_DIST_ID_BYTES]);
int rt_dist_create(const uint8_t id[RT_DIST_ID_BYTES], int world, int rank, rt_dist** out);
void rt_dist_destroy(rt_dist* d);
int rt_render_dist(rt_dist* d, const rt_scene* s, int W, int H, int mode, int flags, double* fb_root_dev,
                   void* hip_stream, rt_stats* stats);
int rt_render_dist_rgb8(rt_dist* d, const rt_scene* s, int W, int H, int mode, int flags, uint8_t* rgb8_root_dev,
                        void* hip_stream, rt_stats* stats);
/* Max-reduction of n doubles over all ranks of d, in place on the host
 * (ncclAllReduce on the rank's collective stream; world 1 without a
 * communicator: unchanged), and a barrier built on it.  Launcher plumbing
 * for callers without a collective layer of their own (bench.py's max-over-
 * ranks timing). */
int rt_dist_reduce_max(rt_dist* d, double* vals_host, int n);
int rt_dist_barrier(rt_dist* d);
/* Failure behaviour of rt_render_dist[_rgb8] with more than one rank.  Every
 * rank issues every collective of a frame whatever happens locally, and the
 * ranks agree twice per frame through small RCCL max-reductions: before the
 * first gather on the frame descriptor (W, H, mode, output kind, flags) and
 * on each rank's setup status; before the last gather on each rank's trace
 * status.  So a rank-local failure makes EVERY rank return an error (the
 * failing rank its own; the others RT_ERR_INVALID_ARG for a descriptor
 * mismatch, RT_ERR_HIP naming the failed ranks otherwise) and the next frame
 * renders normally.  A wait for peers that exceeds the rank's timeout (or an
 * RCCL asynchronous error) aborts the communicator (ncclCommAbort) and returns
 * RT_ERR_HIP; that handle then refuses frames and must be destroyed.  The
 * timeout is RT_DIST_TIMEOUT_MS from the environment at creation (default
 * 120000) or rt_dist_set_timeout. */
int rt_dist_set_timeout(rt_dist* d, int timeout_ms);
/* This rank's split of its last successful collective frame (world > 1, or a
 * forced-collective world 1), in ms, for diagnosing a multi-GPU run from one
 * line (bench.py puts every rank's split into its JSON):
 *   out[0] the whole call (host)        out[1] the frame agreement's reduction (device)
 *   out[2] host wait for its verdict    out[3] this rank's gathers (device, sum)
 *   out[4] the root's placements (device, sum; 0 elsewhere)
 *   out[5] the last chunk's gather      out[6] the last chunk's placement (device)
 *   out[7] host time from the last enqueue to the call's return
 *   out[8] the communicator's rank count (ncclCommCount)
 *   out[9] output rows this rank traced
 * Writes min(n, 10) entries and returns that count. */
int rt_dist_frame_split(rt_dist* d, double* out, int n);
/* The partition of an FP64 frame: writes the output rows of `rank`
 * (ascending) to rows_out (room for H entries) and returns their count; <0
 * on bad arguments.  (RGB8 frames weight every rank equally.)
 * rt_dist_rows is the standard-mode partition (RT_STRIP_ROWS); paper mode
 * uses RT_PAPER_STRIP_ROWS strips (rt_dist_rows_mode). */
int rt_dist_rows(int H, int world, int rank, int32_t* rows_out);
int rt_dist_rows_mode(int H, int world, int rank, int mode, int32_t* rows_out);

/* Render an arbitrary set of OUTPUT rows (top-row-first indices) into a
 * compact device buffer fb_rows_dev[n_rows][W][3] on the given HIP stream
 * (NULL = default stream).  rows_host lists the rows, distinct, in any order
 * (a duplicate is RT_ERR_INVALID_ARG).  Only the jitter-stream segments those
 * rows consume are generated.  Blocks until done. */
int rt_render_rows_device(const rt_scene* s, int W, int H, int mode, int flags,
                          const int32_t* rows_host, int n_rows,
                          double* fb_rows_dev, void* hip_stream, rt_stats* stats);

/* Frame pipeline: rt_render_rows_device split into an asynchronous begin /
 * trace / end, so that a multi-GPU rank can hand finished row chunks to a
 * collective (RCCL on its own stream) while the next chunks are traced
 * (SURVEY.md §8e).  rt_frame_begin validates the rows (as
 * rt_render_rows_device), uploads the scene and enqueues the jitter stream of
 * ALL the listed rows; rt_frame_trace enqueues the trace of list entries
 * [ri0, ri1) into fb_rows_dev[0 .. ri1-ri0) (each list entry traced once)
 * on trace_stream (NULL = the frame's stream; another stream first waits for
 * begin's work, so consecutive chunks on two streams overlap their launch
 * tails); rt_frame_end joins every stream used, waits, fills stats and frees
 * the frame — call it exactly once per begun frame, also after an error.
 * begin/trace only enqueue work.  One frame per device at a time (begin
 * blocks while another frame of the same device is open). */
typedef struct rt_frame rt_frame;
int rt_frame_begin(const rt_scene* s, int W, int H, int mode, int flags, const int32_t* rows_host, int n_rows,
                   void* hip_stream, rt_frame** out);
int rt_frame_trace(rt_frame* f, int ri0, int ri1, double* fb_rows_dev, void* trace_stream);
int rt_frame_end(rt_frame* f, rt_stats* stats);

/* fb_dev[rows[i]][*] = src_dev[i][*] for i < n_rows (device copy, W*3 doubles per row);
 * slots with rows[i] < 0 (padding) are skipped. */
int rt_scatter_rows_device(const double* src_dev, const int32_t* rows_dev, int n_rows,
                           int W, double* fb_dev, void* hip_stream);

/* Device-side toByte + RGB packing: rgb8_dev[W*H*3]. */
int rt_framebuffer_to_rgb8_device(const double* fb_dev, size_t n_pixels,
                                  uint8_t* rgb8_dev, void* hip_stream);

/* ------------------------------------------------------------ host I/O */
/* toByte(v) = round(clamp01(v)*255) (core.h:316), RGB order. */
void rt_framebuffer_to_rgb8(const double* fb, size_t n_pixels, uint8_t* rgb8);
/* Write an 8-bit RGB PNG (zlib deflate, n_threads > 1 parallelises the deflate). */
int rt_write_png(const char* path, const uint8_t* rgb8, int W, int H, int n_threads);

/* Number of HIP devices visible (0 when none / driver not loaded). */
int rt_device_count(void);

/* ------------------------------------------ device buffers and teardown
 * For callers with no device-memory layer of their own (a cgo / JNI / ctypes
 * binding, tests, bench.py): plain HIP allocations and copies on the
 * library's own HIP runtime, so a process needs no second one.  All return
 * an rt_status; sizes are bytes. */
int rt_set_device(int device);                       /* hipSetDevice for this thread        */
int rt_device_alloc(size_t bytes, void** dev_out);   /* hipMalloc, zero-filled              */
int rt_device_free(void* dev);
int rt_memcpy_h2d(void* dev, const void* host, size_t bytes);
int rt_memcpy_d2h(void* host, const void* dev, size_t bytes);
int rt_device_synchronize(void);
int rt_stream_create(void** stream_out);             /* non-blocking HIP stream              */
int rt_stream_destroy(void* stream);
/* Page-lock an existing host buffer (hipHostRegister) so that the output
 * copies of rt_render_rgb8 / rt_render_multi into it run as direct DMA
 * instead of through the runtime's pageable staging: for callers that render
 * many frames into the same buffer (registering 25 MB costs ~50 ms, so the
 * one-frame `ray` CLI does not).  Unregister before freeing it. */
int rt_host_register(void* host, size_t bytes);
int rt_host_unregister(void* host);
/* One-time setup costs of this process so far, host wall clock in ms:
 * out[0] scene compile + upload (first frame of each scene), out[1] jitter
 * checkpoint-table builds / extensions, out[2] first trace-kernel launch
 * (loads the kernels' code object onto the device), out[3] first jitter-fill
 * launch (its code object), out[4] device allocations (hipMalloc), out[5]
 * page-locked host allocations, out[6] stream / event creation; and the
 * split of the LAST frame (not cumulative): out[7] rt_frame_begin, out[8]
 * its rt_frame_trace calls, out[9] rt_frame_end, out[10] the device-group
 * setup of the last rt_render_multi / rt_render_rgb8 call; out[11] the
 * one-time copy-engine warm-up (host time, overlapped with the first
 * frame's trace).  min(n, 12) entries are written. */
int rt_setup_times(double* out, int n);
/* One-time preparation a caller can start early, e.g. on a helper thread
 * while its main thread initialises HIP or parses the scene:
 *   RT_WARM_HOST    host-only: the jitter stream's jump-tree tap lists (read
 *                   from lib/mt19937_tree.polys; ~3 ms), cached for the process
 *   RT_WARM_DEVICE  loads the FP64 render kernels' code object onto the
 *                   current device (~5 ms at a process's first trace launch)
 * Thread-safe; the frames that follow find the work done. */
enum { RT_WARM_HOST = 1, RT_WARM_DEVICE = 2 };
int rt_warmup(int what);
/* Release every device resource the library caches (per-device workspaces,
 * resident scenes and jitter tables, the rt_render_multi device groups with
 * their RCCL communicators).  No render may be in flight; later calls
 * re-create what they need.  The `ray` CLI calls it before exit when it
 * rendered on several GPUs (RCCL communicators); a one-GPU run leaves the
 * device memory to process exit. */
int rt_shutdown(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_H */
