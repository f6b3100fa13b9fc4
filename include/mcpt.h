/* mcpt.h -- C ABI of libmcpt_hip.so, the MI355X (gfx950) path tracer.
 *
 * Drop-in boundary for the reference's per-pixel radiance loop (luotong96/Monte_Carlo_Path_Tracing).
 * The reference has no plugin/FFI seam: its loop is inlined in main() (main.cpp:547-588) and
 * calls `veach.closet_ray_intersect(eye, dir, triangle(-1,-1))` then
 * `shade_with_mis` / `shade_with_brdf` on the globals `Myobj veach` / `Mylight lights`
 * (main.cpp:23-24).  Each entry point below names the reference interface it replaces.
 *
 * Conventions: every function returns 0 (MCPT_OK) or a negative MCPT_E_* code; no exception
 * crosses the ABI (the reference instead exit(1)s on load errors, Myobj.cpp:15-20,
 * Mylight.cpp:16-20, and throws std::out_of_range on a bad material, main.cpp:425);
 * mcpt_last_error() returns a thread-local message.  Callers own host buffers; the library owns
 * device memory.  One render at a time per scene handle.  Results are deterministic for a fixed
 * (seed, spp, width, height) independent of how the sample range is split across calls / GPUs,
 * up to fp64 summation order.
 */
#ifndef MCPT_H
#define MCPT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCPT_VERSION 20200 /* 2.2.0: mcpt_stats gains comm_init_seconds, device_setup_seconds and
                               * device_seconds[MCPT_STATS_MAX_DEVICES] (appended): where a multi-device call's
                               * time went; mcpt_render_opts gains stats_size (appended: a caller built against
                               * an older header is refused by struct_size instead of having its smaller
                               * mcpt_stats overrun);
                               * 2.1.0: mcpt_stats gains prep_exact_nodes, cache_build_seconds and prep_band_nodes
                               * (appended);
                               * 2.0.0: mcpt_render_opts carries struct_size (checked first), a device list
                               * and a multi-process communicator; debug entry points moved to mcpt_debug.h */

enum {
    MCPT_OK = 0,
    MCPT_E_INVALID = -1,  /* bad argument */
    MCPT_E_IO = -2,       /* file not found / parse error */
    MCPT_E_SCENE = -3,    /* scene violates the reference's assumptions (e.g. facet without material) */
    MCPT_E_DEVICE = -4,   /* HIP error */
    MCPT_E_OVERFLOW = -5, /* reserved (since 2.0 a generation larger than the queue is processed in slices) */
    MCPT_E_CANCELLED = -6, /* the progress callback asked to stop */
};

/* shade_with_mis main.cpp:402 / shade_with_brdf :348 / shade :269 (the one main() calls, :575) with
 * the spherical-triangle light sampler (main.cpp:297) / shade with the uniform-area light sampler
 * select_a_point_from_lights (Mylight.cpp:102-160, the alternative commented out at main.cpp:296:
 * a light by radiance, a triangle by area, a uniform point; no O(N_L) light prep) */
enum { MCPT_MODE_MIS = 0, MCPT_MODE_BRDF = 1, MCPT_MODE_SHADE = 2, MCPT_MODE_SHADE_AREA = 3 };

/* closest-hit acceleration: the BVH (default; the true closest hit) or the reference's own uniform
 * grid with its in-cell acceptance rule (Myobj.cpp:78-162, 334-622), crack included -- hit for hit
 * the reference's traversal, for parity studies (much slower). */
enum { MCPT_ACCEL_BVH = 0, MCPT_ACCEL_GRID = 1 };
/* mcpt_closest_hit flags */
enum { MCPT_HIT_LIGHT_ONLY = 1, MCPT_HIT_GRID = 2 };

typedef struct mcpt_scene mcpt_scene;

/* Flattened scene (host pointers, copied by mcpt_scene_create).  Facets in the reference's
 * (shape, face) order; light table in Mylight::lightsTriangles order (material name, then facet,
 * Mylight.cpp:88). */
typedef struct {
    int32_t nfacets, nmaterials, nlights;
    const float* positions;      /* nfacets*9: v0 v1 v2 (tinyobj real_t = float) */
    const float* normals;        /* nfacets*9: vertex normals */
    const int32_t* material_id;  /* nfacets */
    const float* materials;      /* nmaterials*7: Kd[3] Ks[3] Ns */
    const int32_t* light_facet;  /* nlights: facet of each light triangle */
    const double* light_radiance; /* nlights*3: radiance of its <light> material */
    const int32_t* light_group;  /* optional, nlights: index of its <light> (ascending; the lights of
                                  * select_a_point_from_lights, Mylight.cpp:102-160); NULL = each run of
                                  * equal radiance is one light */
} mcpt_scene_desc;

/* Camera of main.cpp:507-510,547-564 generalised to width x height:
 * pixellen = tan(fovy/360)*|w|/(height/2) (the reference's /360 quirk kept), eye pulled back by
 * dist_scale (2 in the reference). */
typedef struct {
    double eye[3], lookat[3], up[3];
    double fovy;
    double dist_scale;
    int32_t width, height;
} mcpt_camera;

/* progress callback (replaces the reference's per-row progress / EasyX display, main.cpp:539-592):
 * called on the rendering host thread after every wavefront generation with the camera samples
 * dispatched so far and the call's total; return nonzero to cancel the render (MCPT_E_CANCELLED,
 * the framebuffer then holds a partial sum). */
typedef int (*mcpt_progress_fn)(void* user, uint64_t samples_dispatched, uint64_t samples_total);

/* Multi-process communicator (one process per GPU, e.g. torchrun): rank 0 creates an id with
 * mcpt_comm_unique_id, the caller broadcasts its MCPT_COMM_ID_BYTES bytes (any channel), every rank
 * calls mcpt_comm_init_rank (RCCL ncclCommInitRank on `device`; collective over all ranks).  The
 * library owns the RCCL communicator. */
typedef struct mcpt_comm mcpt_comm;
#define MCPT_COMM_ID_BYTES 128

typedef struct {
    uint32_t struct_size;   /* sizeof(mcpt_render_opts) of the caller's header (mcpt_render_opts_init sets
                             * it); checked before any other field -- a mismatch is MCPT_E_INVALID */
    int32_t spp;            /* samples per pixel of the whole frame (the 1/spp weight) */
    int32_t sample_begin;   /* render global sample indices [sample_begin, sample_end) */
    int32_t sample_end;     /*   (0,0 = all); with devices / comm this is the JOB's range, split below */
    int32_t mode;           /* MCPT_MODE_MIS / MCPT_MODE_BRDF / MCPT_MODE_SHADE */
    uint64_t seed;          /* counter-RNG seed (reference default 20240430 in bench/tests) */
    int32_t samples_per_launch; /* wavefront working set: the node queue is refilled with camera samples
                                 * up to samples_per_launch x width x height nodes per generation
                                 * (0 = auto: 48 Mi nodes, at most the call's camera samples and at
                                 * most half the free HBM) */
    int32_t queue_factor;   /* wavefront queue capacity = factor * batch roots (0 = 2); a generation with
                             * more nodes than the children buffer can take is processed in slices, the
                             * rest parked on a spill stack in HBM (never an overflow error) */
    int32_t device;         /* HIP device ordinal (-1 = current); ignored when num_devices > 0 */
    int32_t accel;          /* MCPT_ACCEL_BVH / MCPT_ACCEL_GRID (grid over the scene and this camera's
                             * eye with n0 = 100000, main.cpp:501-504; rebuilt when the eye changes) */
    mcpt_progress_fn progress; /* optional (NULL = none); with several devices it is called from the
                                * devices' worker threads, serialised by the library */
    void* progress_user;
    int32_t flags;          /* MCPT_RENDER_* bits (0 = defaults) */
    /* One process, several GPUs: num_devices > 0 splits [sample_begin, sample_end)
     * into num_devices contiguous, balanced shards, shard k rendered on devices[k] (a device may be
     * listed more than once: its shards run one after another into that device's buffer), one host
     * thread and stream per distinct device, no exchange while rendering; then ONE RCCL
     * ncclReduce(sum) over the distinct devices (ncclCommInitAll, cached per scene handle) into the
     * root devices[0].  mcpt_render: the result lands in out_rgb; mcpt_render_device: dev_out_rgb
     * lives on devices[0].  The image equals the single-device render up to fp64 summation order. */
    int32_t num_devices;
    const int32_t* devices;
    /* One process per GPU: this process renders rank's share of [sample_begin, sample_end) on the
     * communicator's device and the call ends with ONE ncclReduce(sum, root rank 0): the whole job's
     * sum is ADDED to rank 0's buffer; other ranks' buffers are left unchanged (their shard goes
     * through a library buffer).  Every rank must make the same call.  Exclusive with devices.
     * Failures: a rank whose render fails (out of memory, its own cancel, ...) still joins the reduce with
     * a failure flag, so rank 0 returns MCPT_E_DEVICE "k of N ranks failed" and nobody blocks.  The one
     * exception is a rank that cannot take part in the reduce at all -- it cannot allocate its
     * (W*H*3 + 1)-double reduce buffer (done first, before any other allocation of the call, and kept
     * for later calls of the same frame size) or its device can no longer enqueue work: it aborts the
     * communicator and returns, and under RCCL its peers then block in ncclReduce (RCCL has no way to
     * release them from one rank).  Leave that buffer's room free on every device. */
    mcpt_comm* comm;
    uint32_t stats_size;    /* sizeof(mcpt_stats) of the caller's header (mcpt_render_opts_init sets it): the
                             * library writes at most this many bytes of the stats (0: none) */
} mcpt_render_opts;
/* mcpt_render_opts.flags: skip the light-side cull statistic in the hot loop of the split light cull;
 * mcpt_stats.light_evals_culled_backface then reads 0 and _culled_plane holds both cheap-stage culls
 * (every prep variant reports it that way).  Images and all other statistics are unchanged. */
enum { MCPT_RENDER_NO_BACKFACE_STATS = 1 };
/* mcpt_render_opts.flags: shade_with_mis evaluates the BRDF branch's light pdf with the node's OWN
 * light prep instead of the reference's stale sampler state (main.cpp:443 vs :487: the state the
 * last prep inside the light branch's recursion left, Mylight.cpp:484-493).  The default follows
 * the reference; this flag is the "fixed" estimator (4.6e-3 relative L2 from the reference's on the
 * Veach stand-in, profiles/stale_pdf_delta.json). */
enum { MCPT_RENDER_FRESH_PDF = 2 };
/* mcpt_render_opts.flags: precision of the light prep's full stage (SURVEY.md §8(b) FP32_STABLE,
 * opt-in).  Default (flag clear) = FP64_LIGHT: the reference's fp64, required for parity.  With the
 * flag, the spherical-triangle weights (Mylight.cpp:360-413) are evaluated two lights per lane in
 * packed fp32 by a cancellation-free Van Oosterom-Strackee form (p - x1 with x1 split hi + lo, the
 * triple product against a precomputed area normal) and summed in fp64: weights within ~1e-6 of the
 * fp64 ones, rendered frames within the 1e-3 relative L2 tolerance of the fp64 render; the edge-length
 * and vertex-angle culls below 1e-8 rad reduce to "sA > 0".  Applies to scenes with more than 64
 * light triangles (the split prep); cheap culls, pick, sampling, pdf and shading stay fp64. */
enum { MCPT_RENDER_PRECISION_FP32 = 4 };

/* zero-fills *opts and sets struct_size, stats_size, device = -1, seed = 20240430, spp = 10 (main.cpp:567),
 * mode = MCPT_MODE_MIS */
void mcpt_render_opts_init(mcpt_render_opts* opts);

#define MCPT_STATS_MAX_DEVICES 16
typedef struct {
    double seconds;         /* device time of the render (HIP events) */
    uint64_t camera_samples;
    uint64_t shading_nodes; /* nodes that passed entry + RR (prep nodes in MIS) */
    uint64_t light_evals_survived; /* light triangles surviving the cull chain (MIS prep) */
    uint64_t rays;          /* extension rays traced */
    uint64_t light_rays;    /* light-only rays traced (MIS light pdf) */
    uint64_t generations;   /* wavefront generations launched */
    double prep_seconds;    /* device time inside the light-prep kernel (HIP events, its stream) */
    uint64_t prep_launches;
    uint64_t light_evals_total;           /* prep_full_nodes x light triangles (MIS, shade) */
    uint64_t light_evals_culled_backface; /* culled by the light-side test (Mylight.cpp:340-345) */
    uint64_t light_evals_culled_plane;    /* culled by the tangent-plane test (Mylight.cpp:347-357) */
    uint64_t light_evals_candidates;      /* passed both; evaluated in full (Mylight.cpp:360-413) */
    uint64_t prep_full_nodes;   /* prep nodes that ran the O(N_L) stages (incl. root-cache builds) */
    uint64_t prep_cached_nodes; /* root nodes served by the per-pixel root-point cache (pick only) */
    uint64_t prep_cache_points; /* root points whose prep built the cache (included in prep_full_nodes) */
    uint64_t spilled_nodes; /* nodes parked on the spill stack (generations larger than the queue) */
    double reduce_seconds;  /* the RCCL reduce of a multi-device / multi-rank call (0 otherwise) */
    int32_t devices_used;   /* distinct devices (or 1 per rank) that rendered */
    double trace_seconds;   /* device time in the traversal kernel (k_mis_rays; BRDF-only: k_extend_brdf) */
    uint64_t trace_launches;
    uint64_t node_visits;   /* BVH node visits and ray/triangle tests of that kernel -- counted only when */
    uint64_t tri_tests;     /* the render sets MCPT_DEBUG_COUNT_TRAVERSAL (mcpt_debug.h), else 0 */
    uint64_t prep_exact_nodes; /* light preps whose pick lay within the rounding band of a cumulative-weight
                                * boundary and were redone with the reference's literal formulas and
                                * summation order (Mylight.cpp:335-438), so the pick is the reference's.
                                * The band's constants are calibrated, not a proven bound (DESIGN.md
                                * §4.3.3: tools/prep_error_study.py on the stand-in, tools/band_margin_study.py
                                * on the stress scenes: margins x2.1 (slivers, 32 seeds) to x111, x10 on the
                                * stand-in; tests/test_band_margin.py) */
    double cache_build_seconds; /* device time building the per-pixel root-point cache (in prep_seconds) */
    uint64_t prep_band_nodes;   /* light preps whose slack the whole-table band bound could not clear and
                                 * that took the per-chunk band test (prep_exact_nodes of them failed it) */
    /* ABI 2.2: where a multi-device / multi-rank call's time went */
    double comm_init_seconds;    /* device list: wall time of ncclCommInitAll in THIS call (first call over a
                                  * device set; 0 when the cached communicator is reused).  Created on the
                                  * calling thread before any device work starts.  0 for single-device and
                                  * mcpt_comm calls (mcpt_comm_init_rank is the caller's) */
    double device_setup_seconds; /* device list: max over devices of the worker's setup wall time (device state:
                                  * scene upload + BVH on first use; framebuffer) */
    double device_seconds[MCPT_STATS_MAX_DEVICES]; /* per rank of the call's communicator (distinct devices
                                  * in order of first appearance; entries beyond 16 not recorded): wall time of
                                  * its shards, setup and reduce excluded -- max/min is the load imbalance.
                                  * Single device / mcpt_comm rank: [0] = this call's render time */
} mcpt_stats;
/* With several devices, `seconds` is the wall time of the whole call (setup + shards + reduce; comm init
 * excluded), counts are summed over devices and prep_seconds is summed device time. */

int mcpt_version(void);
const char* mcpt_last_error(void);

/* Myobj::read + Mylight::read + gather_light_triangles (Myobj.cpp:10-28, Mylight.cpp:11-100):
 * OBJ/MTL via the tinyobjloader-compatible reader, <light mtlname radiance> via the XML reader. */
int mcpt_scene_load(const char* obj_path, const char* xml_path, mcpt_scene** out);
/* flattened-array form of the same (the reference's data after loading) */
int mcpt_scene_create(const mcpt_scene_desc* desc, mcpt_scene** out);
void mcpt_scene_destroy(mcpt_scene* scene);
int mcpt_scene_counts(const mcpt_scene* scene, int32_t* nfacets, int32_t* nmaterials, int32_t* nlights);
/* device bytes of the acceleration structures the traversal reads (both BVHs' 4-wide nodes and leaf
 * triangles; the reference's counterpart is its uniform grid, Myobj.cpp:110-162) */
int mcpt_scene_accel_bytes(const mcpt_scene* scene, uint64_t* bytes);
/* host copies of the loaded, flattened scene (any pointer may be NULL): the reference's data
 * after Myobj::read / gather_light_triangles, plus Myobj::get_unique_normal_of_facet (Myobj.cpp:680) */
int mcpt_scene_arrays(const mcpt_scene* scene, float* positions, float* normals, int32_t* material_id,
                      float* materials, int32_t* light_facet, double* light_radiance, double* unique_normals);
/* the XML's <camera> block (README.md:339-343; ignored by the reference main.cpp:507-510) */
int mcpt_scene_camera(const mcpt_scene* scene, mcpt_camera* cam);

/* main.cpp:547-588: render samples [sample_begin, sample_end) of an spp-sample frame and ADD
 * sum_k L_k * (1/spp) into out_rgb (caller-owned host buffer, height*width*3 doubles, row 0 =
 * top image row).  Devices: opts->device, or opts->devices / opts->comm (see mcpt_render_opts). */
int mcpt_render(mcpt_scene* scene, const mcpt_camera* cam, const mcpt_render_opts* opts, double* out_rgb,
                mcpt_stats* stats);
/* same, accumulating into a DEVICE buffer (height*width*3 doubles on opts->device, devices[0] or the
 * comm's device), without any host round trip.  The buffer must be coarse-grained device memory
 * (hipMalloc, or the torch caching allocator): the framebuffer is updated with hardware fp64
 * atomics, which do not work on fine-grained / managed (hipMallocManaged, hipHostMalloc) memory --
 * such buffers are rejected with MCPT_E_INVALID. */
int mcpt_render_device(mcpt_scene* scene, const mcpt_camera* cam, const mcpt_render_opts* opts,
                       double* dev_out_rgb, mcpt_stats* stats);

/* Myobj::cal_scene_boundingbox(eye) + Myobj::meshing(n0) (Myobj.cpp:78-162): build the scene's
 * uniform grid (box of every vertex and `eye`; cell edge = largest extent / n0^(1/3)) for
 * MCPT_HIT_GRID queries.  Renders with MCPT_ACCEL_GRID build their own for their camera. */
int mcpt_scene_meshing(mcpt_scene* scene, const double eye[3], int32_t n0);
/* the current grid: box_and_cell = (xmin, xmax, ymin, ymax, zmin, zmax, cell edge), cells per axis */
int mcpt_scene_grid_info(const mcpt_scene* scene, double* box_and_cell, int32_t* cells);

/* Myobj::closet_ray_intersect (Myobj.cpp:334) / closet_ray_intersect_light_triangle (:476) for a
 * batch of n rays (host arrays): ro/rd n*3, exclude n (origin facet, -1 none) ->
 * facet (or -1) and t, beta, gamma (n*3).  flags: MCPT_HIT_LIGHT_ONLY (the light-only query),
 * MCPT_HIT_GRID (the reference's grid of mcpt_scene_meshing instead of the BVH). */
int mcpt_closest_hit(mcpt_scene* scene, int32_t n, const double* ro, const double* rd, const int32_t* exclude,
                     int32_t flags, int32_t* facet, double* tbg);
/* Mylight::prepared_for_lights_spherical_triangle_sampling (Mylight.cpp:322) at n shading points
 * (x1, normal) -> weights_sum, survivor count, and the FACET of the light triangle picked by the
 * counter-RNG rule for uniform u[k] (first survivor with cumulative weight >= u*weights_sum;
 * -1 if empty or weights_sum < 1e-8). */
int mcpt_light_prep(mcpt_scene* scene, int32_t n, const double* x1, const double* normal, const double* u,
                    double* weights_sum, int32_t* count, int32_t* pick);
/* primary-hit map of main.cpp:563-572 for a camera: facet (or -1), t, beta, gamma per pixel */
int mcpt_primary_hits(mcpt_scene* scene, const mcpt_camera* cam, int32_t* facet, double* tbg);

/* RadianceRGB::tone_mapping (RadianceRGB.cpp:51-67) of an HDR frame + the EasyX saveimage BMP
 * layout (32-bpp BI_RGB, bottom-up) of main.cpp:583-596 */
int mcpt_tone_map(const double* rgb, int32_t width, int32_t height, double max_radiance, double gamma,
                  uint8_t* out_rgb8);
int mcpt_write_bmp(const char* path, const uint8_t* rgb8, int32_t width, int32_t height);

/* Multi-process communicator (see mcpt_comm above): ncclGetUniqueId / ncclCommInitRank /
 * ncclCommDestroy.  device -1 = the current device. */
int mcpt_comm_unique_id(uint8_t id[MCPT_COMM_ID_BYTES]);
int mcpt_comm_init_rank(int32_t nranks, int32_t rank, const uint8_t id[MCPT_COMM_ID_BYTES], int32_t device,
                        mcpt_comm** out);
void mcpt_comm_destroy(mcpt_comm* comm);

#ifdef __cplusplus
}
#endif
#endif
