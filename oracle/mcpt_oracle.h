/* TEST INFRASTRUCTURE ONLY -- CPU oracle for the MI355X path tracer.
 *
 * A plain-C, single-file restatement of the reference's per-pixel radiance loop
 * (luotong96/Monte_Carlo_Path_Tracing): OBJ/MTL/XML loading (Myobj.cpp:10-28, Mylight.cpp:11-100,
 * the vendored tinyobjloader number parser tiny_obj_loader.h:897-1028), the uniform grid + 3D-DDA
 * closest hit (Myobj.cpp:78-162,334-622), staged spherical-triangle light sampling
 * (Mylight.cpp:322-493) and its non-staged form (:163-318), the Phong BRDF (BRDF.cpp:17-133), the
 * three integrators (shade main.cpp:269-344, shade_with_brdf :348-399, shade_with_mis :402-494)
 * and the camera/frame loop (main.cpp:507-588).  All arithmetic is fp64 in the reference's
 * evaluation order, built with -ffp-contract=off.
 *
 * Parity pin: tests/test_oracle_golden.py checks every function against golden vectors produced by
 * the compiled reference (oracle/ref_harness.cpp, `make -C oracle golden`).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / CPU baseline -- never as a product path.
 */
#ifndef MCPT_ORACLE_H
#define MCPT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

/* main.cpp:402 / :348 / :269; SHADE_AREA = shade() with the uniform-area light sampler
 * select_a_point_from_lights (Mylight.cpp:102-160, the alternative commented out at main.cpp:296) */
enum { ORC_MODE_MIS = 0, ORC_MODE_BRDF = 1, ORC_MODE_SHADE = 2, ORC_MODE_SHADE_AREA = 3 };
/* With the counter RNG, shade_with_mis evaluates the BRDF branch's light pdf like the reference:
 * with the light-sampler state the LAST prep left, after the light branch's recursion (main.cpp:443
 * vs :487, Mylight.cpp:484-493 -- the "stale-pdf" behaviour, which the RefRng replay has too).
 * ORC_FLAG_FRESH_PDF, or-ed into the mode, uses the node's own prep instead (a fix of the
 * reference; tools/stale_pdf_delta.py measures the difference). */
enum { ORC_FLAG_FRESH_PDF = 0x200 };
enum { ORC_RNG_REF = 0, ORC_RNG_COUNTER = 1 };

/* camera: eye, lookat, up, fovy parameter (the reference's tan(fovy/360) quirk), eye pull-back
 * factor (2 in main.cpp:509-510), image size */
typedef struct {
    double eye[3], lookat[3], up[3];
    double fovy;
    double dist_scale;
    int width, height;
} orc_camera;

/* returns NULL on failure; orc_last_error() has the reason */
orc_scene* orc_scene_load(const char* obj_path, const char* xml_path);
void orc_scene_free(orc_scene* s);
const char* orc_last_error(void);
void orc_scene_counts(const orc_scene* s, int* nfacets, int* nmaterials, int* nlights);
/* per facet: v0 v1 v2 n0 n1 n2 (float x18), material id, light index (-1 = not a light) */
void orc_scene_facets(const orc_scene* s, float* v18, int* mat, int* light_of_facet, double* unique_n3);
void orc_scene_materials(const orc_scene* s, float* kd_ks_ns7);
/* light table in reference order (Mylight.cpp:88 map order): facet, area, radiance rgb */
void orc_scene_lights(const orc_scene* s, int* facet, double* area_rgb4);
int orc_scene_camera(const orc_scene* s, orc_camera* cam); /* 0 if the XML had a <camera> */

/* uniform grid of Myobj::cal_scene_boundingbox + meshing (Myobj.cpp:78-162) */
void orc_grid_build(orc_scene* s, const double camera_pos[3], int n0);
void orc_grid_info(const orc_scene* s, double* bbox6_cellw);

/* one ray -> hit facet (or -1), t, beta, gamma.  exclude = origin facet (-1 none) */
int orc_closest_hit(const orc_scene* s, const double ro[3], const double rd[3], int exclude, double* tbg3);
int orc_closest_light_hit(const orc_scene* s, const double ro[3], const double rd[3], int exclude, double* tbg3);
int orc_intersect_triangle(const orc_scene* s, const double ro[3], const double rd[3], int facet, double* tbg3);

/* Phong BRDF (BRDF.cpp:17-25, 107-133) */
void orc_brdf_phong(const double n[3], const double wi[3], const double wr[3], const double kd[3],
                    const double ks[3], double ns, double rgb[3]);
double orc_phong_pdf(const double n[3], const double wi[3], const double wr[3], const double kd[3],
                     const double ks[3], double ns);
/* sample_from_phong (BRDF.cpp:28-104) with the reference RNG replayed from clock counter `ctr` */
void orc_sample_phong_ref(uint64_t ctr, const double n[3], const double wr[3], const double kd[3],
                          const double ks[3], double ns, double dir_pdf4[4]);
/* sample_from_phong with explicit uniforms (lobe pick u0, xi1, xi2) -- the counter-RNG form */
void orc_sample_phong_u(const double n[3], const double wr[3], const double kd[3], const double ks[3],
                        double ns, double u0, double u1, double u2, double dir_pdf4[4]);

/* light prep at (x1, n) -> weights_sum, survivor count; optional survivors' light-order indices
 * and weights (arrays of size nlights) */
double orc_light_prep(const orc_scene* s, const double x1[3], const double n[3], int* count,
                      int* survivor_idx, double* survivor_w);
/* prep + lights_spherical_triangle_sampling with reference RNG from clock counter ctr.
 * out: facet (or -1 dummy), coord xyz, prob, clock draws consumed */
void orc_light_sample_ref(const orc_scene* s, uint64_t ctr, const double x1[3], const double n[3], double out6[6]);
/* same with explicit uniforms (pick u, xi1, xi2) -> facet, coord, prob, weights_sum */
void orc_light_sample_u(const orc_scene* s, const double x1[3], const double n[3], double u, double xi1,
                        double xi2, double out6[6]);
/* eval_spherical_triangle_sampling_pdf of `facet` with a fresh prep at (x1, n) */
double orc_light_pdf(const orc_scene* s, const double x1[3], const double n[3], int facet);

void orc_tone_map(const double rgb[3], double max_radiance, double gamma, int out[3]);

/* primary ray of pixel (i, j) -- main.cpp:547-564 generalised to W x H */
void orc_camera_ray(const orc_camera* cam, int i, int j, double eye[3], double dir[3]);

/* one camera sample of pixel (i, j):  RefRng replay from clock ctr (stale-pdf quirk as in the
 * reference DFS), or the counter RNG keyed by (seed, pixel, sample, node) with fresh pdf.
 * returns radiance (not scaled by 1/spp); *draws = clock ticks consumed (RefRng). */
void orc_shade_sample(const orc_scene* s, const orc_camera* cam, int mode, int rng, uint64_t ctr_or_seed,
                      int i, int j, int sample, double rgb[3], uint64_t* draws);

/* full render (counter RNG), samples [s0, s1) of spp, accumulated as sum += L * (1/spp):
 * out_rgb[H*W*3] (row-major, row i = image row from the top).  Pixel subset: stride (every
 * `stride`-th pixel in x and y, starting at offset); other pixels untouched. nthreads >= 1. */
int orc_render(const orc_scene* s, const orc_camera* cam, int mode, uint64_t seed, int spp, int s0, int s1,
               int stride, int offset, int nthreads, double* out_rgb, uint64_t* stats4);

/* depth-cap study: the MIS frame with the tree cut below depth max_depth (<= 62) and the nodes per depth
 * (hist[64], [63] = nodes cut), see mcpt_oracle.c */
int orc_depth_study(const orc_scene* s, const orc_camera* cam, uint64_t seed, int spp, int stride, int offset,
                    int nthreads, int max_depth, double* out_rgb, uint64_t* hist);

/* debugging aid: per-node records of one MIS camera sample (counter RNG), see mcpt_oracle.c */
int orc_debug_mis_sample(const orc_scene* s, const orc_camera* cam, int mode, uint64_t seed, int i, int j, int sample,
                         double* rec, int max_nodes);

/* counter RNG: uniform in [0,1) for (seed, pixel, sample, node, dim) -- shared with the GPU */
double orc_counter_uniform(uint64_t seed, uint64_t pixel, uint64_t sample, uint64_t node, uint32_t dim);

#ifdef __cplusplus
}
#endif
#endif
