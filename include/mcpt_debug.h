/* mcpt_debug.h -- diagnostics and A/B switches of libmcpt_hip.so.  NOT part of the drop-in boundary
 * (include/mcpt.h): kernel-variant timing and render switches used by tools/ for same-box A/B
 * experiments.  No reference interface corresponds to these. */
#ifndef MCPT_DEBUG_H
#define MCPT_DEBUG_H
#include "mcpt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* mcpt_render_opts.flags bits for A/B experiments (the library accepts them; images are unchanged):
 * MCPT_DEBUG_SPLIT_BRDF runs BRDF-only renders as gen / rays / combine kernels instead of the fused
 * k_extend_brdf; MCPT_DEBUG_NO_ROOT_CACHE disables the per-pixel root-point light-prep cache. */
enum {
    MCPT_DEBUG_SPLIT_BRDF = 1 << 16,
    MCPT_DEBUG_NO_ROOT_CACHE = 1 << 17,
    MCPT_DEBUG_COUNT_TRAVERSAL = 1 << 18,
    MCPT_DEBUG_SHARD_RANKS = 1 << 19,
    MCPT_DEBUG_RAYS_PERSIST = 1 << 20,
    MCPT_DEBUG_RAYS_CW8 = 1 << 21,
    MCPT_DEBUG_FUSED_CULL = 1 << 22,
    MCPT_DEBUG_NO_EXACT_DEFER = 1 << 23
};
/* MCPT_DEBUG_NO_EXACT_DEFER: k_prep_exact recomputes a root's literal sums even when another wave of the same
 * launch is computing its pixel's, instead of deferring the root to the follow-up launch that only searches the
 * stored sums (the default since round 6; picks and sums are the same either way). */
/* MCPT_DEBUG_FUSED_CULL: the MIS children's light prep runs its cheap stages inside k_prep_pk2, one wave per
 * node (prep variant 8, chunks below the node's tangent plane skipped), instead of k_prep_cull_lanes' lane per
 * node writing candidate words that k_prep_pk2 reads back (variant 17). */
/* MCPT_DEBUG_RAYS_PERSIST: the MIS / shade ray sets of every scene go through the persistent refilling
 * traversal (by default only trees beyond an XCD's L2 do; smaller ones take k_mis_rays, one ray per thread).
 * MCPT_DEBUG_RAYS_CW8: the persistent traversal walks the 8-wide compressed trees (k_rays_cw8) instead of the
 * 4-wide ones (k_rays_persistent).  mcpt_closest_hit flag MCPT_DEBUG_HIT_CW8: trace the batch through the
 * 8-wide trees (one ray per thread, k_rays_cw8's traversal). */
enum { MCPT_DEBUG_HIT_CW8 = 1 << 8 };
/* MCPT_DEBUG_COUNT_TRAVERSAL runs the traversal kernel's counting instance, which fills
 * mcpt_stats.node_visits / tri_tests (the events of the traversal roofline; slower, for untimed
 * replays).
 * MCPT_DEBUG_SHARD_RANKS (device lists, mcpt_render_opts.devices): every list entry becomes its own rank
 * of the ncclCommInitAll communicator, a repeated device included (normally repeated devices are merged
 * into one rank).  Real RCCL refuses a device twice; with mcpt_debug_set_collective_lib pointing at the
 * test collective (tests/collshim) it runs the multi-rank group reduce on a one-GPU box. */

/* Test infrastructure: load the NCCL-API collective library at `path` instead of librccl.so.1.  Must
 * be called before the first communicator of the process (mcpt_comm_unique_id / _init_rank or a device
 * list render), else MCPT_E_INVALID.  tests/collshim/libmcpt_collshim.so implements the entry points the
 * library binds (ncclGetUniqueId, ncclCommInitRank, ncclCommInitAll, ncclReduce, ncclGroupStart/End,
 * ncclCommDestroy, ncclCommAbort, ncclGetErrorString) over host shared memory, so 2-8 processes can
 * share one GPU -- the multi-rank protocol of mcpt_render_opts.comm then runs in CI as it does over
 * xGMI.  Not part of the drop-in boundary. */
int mcpt_debug_set_collective_lib(const char* path);

/* diagnostics: run the light-prep kernel variant `variant` `iters` times on the n points and report
 * the mean device time per launch; outputs like those of mcpt_light_prep, pick = facet.  Variants: -1 auto
 * (9 if N_L <= 64, else 17, else 0 when the candidate list does not fit in LDS); 0 k_prep (per-wave
 * LDS candidate queue, any N_L); 8 k_prep_pk2 (packed-fp32 cheap stages, stored LDS candidate list,
 * branch-free fp64 batches, lane-parallel batch search in one kernel); 9 k_prep_lane (lane per
 * node, small light sets); 17 k_prep_cull_lanes (lane per node, light table in scalar registers)
 * + k_prep_pk2's fp64 phase (the renderer's form: the cull's lanes take the nodes bucketed by their
 * tangent-plane chunk classes and skip the work a class decides, k_cull_classify); 18 variant 17 without
 * that order and without the chunk classes (its candidate words must be identical).  Other values:
 * MCPT_E_DEVICE (invalid value). */
int mcpt_debug_prep_bench(mcpt_scene* scene, int32_t n, const double* x1, const double* normal, const double* u,
                          int32_t variant, int32_t iters, double* ms_per_launch, double* weights_sum, int32_t* pick);

/* diagnostics: mcpt_light_prep with every point through the exact fallback alone (k_prep_exact: the
 * reference's literal cull chain and weights, Mylight.cpp:335-413, summed in index order, and the
 * counter-RNG pick over those sums) -- the arithmetic the renderer uses for picks inside the
 * ambiguity band.  Scenes with more than 64 light triangles (else MCPT_E_INVALID). */
int mcpt_debug_light_prep_exact(mcpt_scene* scene, int32_t n, const double* x1, const double* normal, const double* u,
                                double* weights_sum, int32_t* count, int32_t* pick);

/* diagnostics: the reference's literal cull chain (Mylight.cpp:335-413, light_tri_stage) for every light
 * at one point, 20 doubles per light: stage (0 survives, 1/2 cheap culls, 3 full-stage cull), A, B, C
 * (after the orientation swap), a, b, c, alpha, beta, gamma, alpha+beta+gamma-pi, w (-1 if culled),
 * alpha's acos argument, B.C.  For checking the GPU's fp64 sqrt / division / acos against the host's. */
int mcpt_debug_light_literal(mcpt_scene* scene, const double x1[3], const double normal[3], double* out20);

/* diagnostics (host only, no GPU): the traversal's fp32 triangle pre-test (tri_filter in render.hip)
 * on n (triangle, ray) pairs -- tri: 9 floats per triangle (a, b, c), ro / rd: 3 doubles per ray,
 * tlim: the traversal's current limit per pair (FLT_MAX: none).  verdict: 0 the reference's fp64 test
 * (Myobj.cpp:165-192) surely rejects, or the hit lies surely beyond tlim; 2 it surely accepts, with
 * tup >= its t; 1 undecided.  Lets a CPU test check the bound's soundness against the fp64 test. */
int mcpt_debug_tri_filter(int32_t n, const float* tri, const double* ro, const double* rd, const float* tlim,
                          int32_t* verdict, float* tup);

/* diagnostics (host only): checks the 8-wide compressed tree of the scene (light_only: the light-only tree)
 * against its binary tree.  out[6] = nodes reached, triangles reached, facets of the binary tree,
 * facets reached more than once, errors (bad indices, or a triangle vertex outside the decoded box of a slot
 * on its path), depth. */
int mcpt_debug_bvh8_check(mcpt_scene* scene, int32_t light_only, int64_t out[6]);
// The 4-wide tree of every traversal kernel (collapse_bvh4) and its quantized form (quantize_bvh4), walked on
// the host: out = {nodes, facets reached, facets in the binary tree, facets reached twice, errors (a vertex
// outside an ancestor slot's box, a quantized slot box not containing its fp32 box, a bad index), depth}.
int mcpt_debug_bvh4_check(mcpt_scene* scene, int32_t light_only, int64_t out[6]);

#ifdef __cplusplus
}
#endif
#endif
