// MI355X (gfx950) wavefront path tracer for the reference's per-pixel radiance loop
// (main.cpp:547-588 -> shade_with_mis main.cpp:402-494 / shade_with_brdf :348-399 / shade :269-344).
//
// The recursion is flattened into generations of a persistent SoA node queue in HBM:
//
//   k_primary          lane per pixel : camera ray (main.cpp:547-564) + closest hit, once per call
//   k_root_table       lane per pixel : a root's point, normal, wo and kind, once per call
//   k_roots_t          8 roots per lane : a camera sample's root from that table (RR) -> queue
//                                       (path regeneration)
//   k_root_points      lane per pixel : root shading points for the per-pixel root-point cache
//   k_prep_cull_lanes  lane per node  : light prep phase A -- the light-side and tangent-plane culls
//                                       of Mylight.cpp:340-357 against every light (light table
//                                       in scalar registers) -> candidate words
//   k_prep_pk2         WAVE per node  : phase B -- fp64 spherical-triangle weights of the candidates
//                                       (Mylight.cpp:360-413) in dense 64-wide batches -> weights_sum
//                                       and the inverse-CDF pick; in build mode fills the cache
//   k_prep_pick_g      16 LANES per root : the pick of a root from the root-point cache (k_prep_pick,
//                      a wave per root, for tables of more than 64 chunks)
//   k_prep / k_prep_lane              : the same prep for huge / tiny light sets
//   k_mis_gen / k_shade_gen / k_brdf_gen, k_mis_rays (BVH or the reference grid), k_*_combine:
//                                       light + BRDF samples, their closest hits, MIS weights and the
//                                       children's entry checks -> next generation's queue
//   k_extend_brdf      lane per node  : the BRDF-only vertex in one kernel
//
// A node's value is the sum over its subtree's emitter hits of (throughput x emit); contributions
// are accumulated straight into an fp64 framebuffer with hardware fp64 atomics.
// RNG: counter hash of (seed, pixel, sample, heap node id, dim) -- identical to the CPU oracle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "comm.h"
#include "device_math.h"
#include "mcpt.h"
#include "mcpt_debug.h"
#include "mcpt_internal.h"

using namespace mcpt;

// ============================================================================================
// device scene
// ============================================================================================
// two consecutive light triangles (2q, 2q+1) for the lane-per-node cull, every field as an (A, B)
// float pair so that one v_pk_fma_f32 with a scalar operand serves both lights: nl = unique normal,
// d = float(nl . p0 + 1e-8) (the threshold folded in), p[3k+i] = coordinate i of vertex k.  Padding
// lights (index >= N_L) have nl = 0, d = 1e30 (light-side culled).  128 B = two s_load_dwordx16.
struct LightPair {
    float2 nl[3];
    float2 d;      // nl . p0 + 1e-8 of both lights
    float2 p[9];
    float pad[6];
};

struct DScene {
    int F, NL;
    const float4* tri_v;      // F*3, original facet order
    const float* tri_n;       // F*9 vertex normals
    const int* tri_mat;       // F
    const int* tri_light;     // F -> light index or -1
    const float* mtl;         // M*7
    const double* light_rad;  // NL*3
    const double* light_sum;  // NL
    const int* light_facet;   // NL
    const float4* lt_v;       // NL*3 light vertices (reference order); .w = float(unique normal)
    float light_bound;        // max |coordinate| over light vertices
    const double4* lt_n;      // NL: unique normal xyz, w = RadianceRGB::sum()
    const float4* lt_pk;      // NL*3: (p0.x, p1.x, p2.x, nl.x), (.. .y), (.. .z) -- packed cheap stages
    const float* lt_d;        // NL: float(nl . p0)
    const double2* lt_w;      // NL*5: p0, p1, p2 (fp64), 2 RadianceRGB::sum()
    const float4* lt_f;       // NL*4: fp32 records of MCPT_RENDER_PRECISION_FP32 (LightF32: p0, p1, p2 with the
                              // area normal in .w, then 2 RadianceRGB::sum() as fp64 bits)
    const struct LightPair* lt_pair;  // 32*nchunks light pairs for k_prep_cull_lanes (scalar loads)
    // exact-pick band: per 64-light chunk a bounding sphere (centre, radius) of its
    // vertices and (max sum L, max sum L / shortest edge) of its lights; the same over the whole table
    const float4* chunk_sph;  // nchunks
    const float2* chunk_sk;   // nchunks
    double band_ctr[3], band_R, band_S, band_K;
    const float4* leaf_v;     // per leaf slot: 3 float4 (w of the first = facet id bits)
    const BvhNode4* bvh4;     // 4-wide collapse of bvh (same leaves), breadth-first node order
    const BvhNode4* lbvh4;
    const BvhNode4Q* bvh4q;   // the same trees as 64-B compressed nodes (k_rays_persistent)
    const BvhNode4Q* lbvh4q;
    int nbvh4, nlbvh4;        // node counts
    const float4* lleaf_v;
    // 8-wide compressed trees (BvhNode8Q, k_rays_cw8) and their triangle slots (3 float4 each, w of the
    // first = facet id bits; unused slots are never read); null when a tree does not fit the 24-bit base
    const BvhNode8Q* bvh8;
    const BvhNode8Q* lbvh8;
    const float4* tri8_v;
    const float4* ltri8_v;
    // select_a_point_from_lights (MCPT_MODE_SHADE_AREA): the lightsRadiance map in name order --
    // RadianceRGB::sum() per light and its running sum, the light-table run of its triangles -- and
    // the triangles' areas (Mylight.cpp:66-69) with their running sum within their light
    int ngroups;
    const double* grp_sum;
    const double* grp_cum;
    const int2* grp_range;    // (first light-table index, count)
    const double* l_area;
    const double* l_area_cum;
    // reference uniform grid (MCPT_ACCEL_GRID; null until mcpt_scene_meshing / a grid render)
    const int* g_start;       // CSR cell -> facets
    const int* g_tri;
    double g_mn[3], g_inv_d;
    int g_lim[3], g_gd[3];
};

struct CamFrame {
    d3 eye, U, V, N;
    double wlen, pixellen;
    int W, H;
};

// camera of main.cpp:507-510,547-553 (host, fp64, same operation order as the oracle)
static CamFrame cam_setup(const mcpt_camera& c) {
    auto sub3 = [](d3 a, d3 b) { return d3{a.x - b.x, a.y - b.y, a.z - b.z}; };
    auto mul3 = [](d3 a, double s) { return d3{a.x * s, a.y * s, a.z * s}; };
    auto nrm = [](d3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); };
    auto unit = [&](d3 a) {
        double l = nrm(a);
        return d3{a.x / l, a.y / l, a.z / l};
    };
    auto cr = [](d3 a, d3 b) { return d3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; };
    CamFrame f;
    d3 start{c.eye[0], c.eye[1], c.eye[2]};
    d3 w = sub3(d3{c.lookat[0], c.lookat[1], c.lookat[2]}, start);
    start = sub3(start, mul3(w, c.dist_scale - 1));
    w = mul3(w, c.dist_scale);
    f.eye = start;
    f.wlen = nrm(w);
    f.pixellen = std::tan(c.fovy / 360) * nrm(w) / (c.height / 2.0);
    f.N = unit(w);
    f.V = unit(cr(f.N, d3{c.up[0], c.up[1], c.up[2]}));
    f.U = unit(cr(f.V, f.N));
    f.W = c.width;
    f.H = c.height;
    return f;
}

__device__ inline d3 cam_dir(const CamFrame& f, int i, int j) {  // main.cpp:563-564
    d3 delta = mk3(-f.pixellen * (i - (f.H - 1) / 2.0), f.pixellen * (j - (f.W - 1) / 2.0), 0);
    return normalized(cols_mul(f.U, f.V, f.N, add(delta, mk3(0, 0, f.wlen))));
}

// ============================================================================================
// BVH traversal: fp32 slab tests on conservatively enlarged boxes (prune only), fp64 reference
// triangle test on every candidate.  Stack in LDS, [depth][thread] layout (conflict-free).
// ============================================================================================
constexpr int kStack = 48;
constexpr int kLeafBits = 5;  // leaf code ~((first slot << kLeafBits) | count)
constexpr int kRayBlock = 256;
constexpr int kRayLds = 16;  // LDS stack entries per lane of trace4_ww (16 KB per 256 lanes)
// k_mis_rays: the first kRayTop nodes of the traversed BVH4 (breadth-first numbering: its top
// levels) staged in LDS per workgroup; 0 = off.  A/B builds: -DMCPT_RAY_TOP=N -DMCPT_RAY_LDS=M.
// k_mis_rays stages the BVH's top four levels (1 + 4 + 16 + 64 = 85 nodes, 10.9 KB) in LDS per
// block and reads them with ds_read when the whole wave is in them, with an 8-entry LDS stack per
// lane (same-box A/B on Veach, profiles/round2b_ab_ray_top.txt: traversal 0.82-0.84 -> 0.735-0.745 ms
// per launch; 21 nodes: 0.76; the earlier per-lane generic-pointer select: 0.79-0.84)
// minimum waves per SIMD of the wavefront kernels' launch bounds (1 = the compiler's choice);
// A/B in profiles/round2b_ab_launch_bounds.txt
#ifndef MCPT_LB_CULL
#define MCPT_LB_CULL 1
#endif
#ifndef MCPT_LB_PICK
#define MCPT_LB_PICK 7  // 72 VGPRs: k_prep_pick 427 -> 396 ms per profile run (round 3, same box)
#endif
#ifndef MCPT_LB_GEN
#define MCPT_LB_GEN 1
#endif
#ifndef MCPT_LB_RAYS
#define MCPT_LB_RAYS 6  // 6 waves/SIMD (80 VGPRs, fewer spills) on the round-5 trees: k_mis_rays 3.54 -> 3.41 ms (was 7)
#endif
// 4: 128 VGPRs (141 / 140 without: the literal survival chain of state_light_pdf; 44 / 12 B of
// scratch): k_mis_combine<true> 314 -> 308, k_mis_complete 121 -> 110 ms per profile run, MIS +0.6%
// (round 3, same box, profiles/round3_ab_exact_pick.txt block 7)
#ifndef MCPT_LB_COMBINE
#define MCPT_LB_COMBINE 4
#endif
#ifndef MCPT_LB_COMPLETE
#define MCPT_LB_COMPLETE 4
#endif
#ifndef MCPT_LB_SHADE_GEN
#define MCPT_LB_SHADE_GEN 1
#endif
#ifndef MCPT_RAY_TOP
#define MCPT_RAY_TOP 85
#endif
#ifndef MCPT_RAY_LDS
#define MCPT_RAY_LDS 8
#endif
constexpr int kRayTop = MCPT_RAY_TOP;
constexpr int kRayTopLds = MCPT_RAY_LDS;
constexpr int kTraceBlock = 128;

struct Hit {
    int f;
    double t, beta, gamma;
};

// one node visit's loads: the four children's boxes (lo[axis][child], hi) and child codes
__device__ inline void load_node(const BvhNode4* nd, float (&lo)[3][4], float (&hi)[3][4], int (&ch)[4]) {
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float4 l = *reinterpret_cast<const float4*>(nd->lo[a]), h = *reinterpret_cast<const float4*>(nd->hi[a]);
        lo[a][0] = l.x, lo[a][1] = l.y, lo[a][2] = l.z, lo[a][3] = l.w;
        hi[a][0] = h.x, hi[a][1] = h.y, hi[a][2] = h.z, hi[a][3] = h.w;
    }
    const int4 c = *reinterpret_cast<const int4*>(nd->child);
    ch[0] = c.x, ch[1] = c.y, ch[2] = c.z, ch[3] = c.w;
}
// compressed node (k_rays_persistent): the slab distances of the 24 planes directly,
//   t = fma(byte, 2^(ex - 127) * inv, fma(org, inv, -o * inv))
// -- the same plane (org + byte * scale, quantize_bvh4 rounds it outward) with a few more fp32
// roundings, each ~1 ulp of |plane - origin| * |inv|, far inside the boxes' 1e-5-of-the-scene
// margins; 2 VALU per plane (v_cvt_f32_ubyteN + v_fma_f32) plus 2 per axis
// The planes come out as near (tn) and far (tf) per axis: the byte arrays are swapped by the sign of
// the inverse direction (neg[a]), as m = scale * inv carries that sign and fma(q, m, b) is monotone
// in q -- tn / tf are exactly the fminf / fmaxf of the two slab distances.
__device__ inline void node_tplanes(const BvhNode4Q* nd, const float (&inv)[3], const float (&oi)[3], const bool (&neg)[3],
                                    float (&tn)[3][4], float (&tf)[3][4], int (&ch)[4]) {
    const float4 v0 = *reinterpret_cast<const float4*>(nd->org);
    const uint4 v1 = *reinterpret_cast<const uint4*>(nd->q);
    const uint2 v2 = *reinterpret_cast<const uint2*>(nd->q + 4);
    const int4 c = *reinterpret_cast<const int4*>(nd->child);
    const unsigned ex = __float_as_uint(v0.w);
    const float org[3] = {v0.x, v0.y, v0.z};
    const unsigned ql[3] = {v1.x, v1.z, v2.x}, qh[3] = {v1.y, v1.w, v2.y};
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float m = __uint_as_float(((ex >> (8 * a)) & 0xffu) << 23) * inv[a];
        const float b = fmaf(org[a], inv[a], -oi[a]);
        const unsigned qn = neg[a] ? qh[a] : ql[a], qf = neg[a] ? ql[a] : qh[a];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            tn[a][k] = fmaf((float)((qn >> (8 * k)) & 0xffu), m, b);
            tf[a][k] = fmaf((float)((qf >> (8 * k)) & 0xffu), m, b);
        }
    }
    ch[0] = c.x, ch[1] = c.y, ch[2] = c.z, ch[3] = c.w;
}

// fp32 pre-test of the reference's triangle test (Myobj.cpp:165-192) with a rigorous error bound.
// The four determinants (detA, nb, ng, nt of tri_hit) are evaluated in fp32 as triple products
// sharing two cross products, p = ac x rd and q = ab x ar:
//   detA = ab.p, nb = ar.p, ng = rd.q, nt = -(ac.q)
// -- the same exact values as tri_hit's det3 forms (cyclic permutations).  Each fp32 value is
// within E = 16 * 6 * u32 * Wx * Wy * Wz of the fp64 one, W = max |component| of the operand (a
// triple product has 6 terms of at most Wx Wy Wz; the fma evaluation rounds <= 6 u32 of their sum,
// the inputs carry <= u32 relative error -- ab, ac: fp32 differences of the fp32 vertices, rd: its
// fp32 rounding -- and ar = a - (float)ro carries <= 2 u32 (|ar| + |ro|), so W_ar = M_ar + M_ro;
// the fp64 evaluation's own error is ~1e-16 of the same sum).  Verdicts:
//   0: tri_hit rejects for sure: a numerator of the opposite sign to detA beyond its bound, beta +
//      gamma > 1 beyond the bounds, |detA| < 1e-8 for sure, or t above `tlim` for sure (tlim is at
//      least the t of a triangle tri_hit accepts: this one cannot be the closest hit);
//   2: tri_hit accepts for sure, *tup >= its t;
//   1: undecided -- the fp64 test decides.
// Nothing tri_hit would accept as the closest hit is rejected, so hits stay bit-identical.
struct RayF {
    float ox, oy, oz, dx, dy, dz;
    float mo;  // max |ro| component (rounded up)
    float kd;  // 96 u32 * max |rd| component
};
__host__ __device__ inline RayF ray_f(d3 ro, d3 rd) {
    RayF r;
    r.ox = (float)ro.x, r.oy = (float)ro.y, r.oz = (float)ro.z;
    r.dx = (float)rd.x, r.dy = (float)rd.y, r.dz = (float)rd.z;
    r.mo = fmaxf(fmaxf(fabsf(r.ox), fabsf(r.oy)), fabsf(r.oz)) * 1.0000002f;
    r.kd = 96.0f * 5.9604645e-8f * 1.0001f * fmaxf(fmaxf(fabsf(r.dx), fabsf(r.dy)), fabsf(r.dz));
    return r;
}
__host__ __device__ inline int tri_filter(float4 a4, float4 b4, float4 c4, const RayF& r, float tlim, float* tup) {
    const float abx = a4.x - b4.x, aby = a4.y - b4.y, abz = a4.z - b4.z;
    const float acx = a4.x - c4.x, acy = a4.y - c4.y, acz = a4.z - c4.z;
    const float arx = a4.x - r.ox, ary = a4.y - r.oy, arz = a4.z - r.oz;
    const float px = fmaf(acy, r.dz, -acz * r.dy), py = fmaf(acz, r.dx, -acx * r.dz), pz = fmaf(acx, r.dy, -acy * r.dx);
    const float qx = fmaf(aby, arz, -abz * ary), qy = fmaf(abz, arx, -abx * arz), qz = fmaf(abx, ary, -aby * arx);
    const float dA = fmaf(abx, px, fmaf(aby, py, abz * pz));
    const float nb = fmaf(arx, px, fmaf(ary, py, arz * pz));
    const float ng = fmaf(r.dx, qx, fmaf(r.dy, qy, r.dz * qz));
    const float nt = -fmaf(acx, qx, fmaf(acy, qy, acz * qz));
    const float wab = fmaxf(fmaxf(fabsf(abx), fabsf(aby)), fabsf(abz));
    const float wac = fmaxf(fmaxf(fabsf(acx), fabsf(acy)), fabsf(acz));
    const float war = fmaxf(fmaxf(fabsf(arx), fabsf(ary)), fabsf(arz)) + r.mo;
    // bounds (+1e-30 keeps them positive under flush-to-zero; the products round well inside the x16)
    const float eA = fmaf(wab * wac, r.kd, 1e-30f);
    const float eB = fmaf(war * wac, r.kd, 1e-30f);
    const float eG = fmaf(wab * war, r.kd, 1e-30f);
    const float eT = fmaf(wab * wac * war, 96.0f * 5.9604645e-8f * 1.0001f, 1e-30f);
    const float aA = fabsf(dA);
    if (aA <= eA) return aA + eA < 0.999f * (float)MCPT_EPS ? 0 : 1;  // sign of detA unknown
    const float sb = dA < 0 ? -nb : nb, sg = dA < 0 ? -ng : ng, st = dA < 0 ? -nt : nt;  // numerators over |detA|
    if (sb < -eB || sg < -eG || st < -eT) return 0;  // beta, gamma or t < 0 for sure
    const float over = (sb + sg) - aA, eover = (eB + eG + eA) * 1.0001f + 1e-6f * aA;
    if (over > eover) return 0;                                         // beta + gamma > 1 for sure
    if ((aA + eA) * 1.000001f < (float)MCPT_EPS) return 0;              // |detA| < 1e-8 for sure
    if ((st - eT) * 0.999999f > tlim * (aA + eA) * 1.000001f) return 0;  // farther than a sure hit
    const float lo = aA - eA;
    if (sb > eB && sg > eG && -over > eover && (st - eT) * 0.999999f > (float)MCPT_EPS * 1.001f * (aA + eA) &&
        lo > 1.001f * (float)MCPT_EPS) {
        *tup = (st + eT) * 1.000001f / (lo * 0.999999f);
        return 2;
    }
    return 1;
}
// trace4_ww's fp32 pre-filter with deferred fp64 tests (kFilter), per kernel.  Same-box A/B
// (profiles/round2h_ab_traversal.txt): BRDF-only traversal (k_extend_brdf) 2.19 -> 2.10 ms per
// launch (+3% C2); k_mis_rays alone 4.62 -> 4.64 ms (+-0: its light rays mostly end on the light
// they aim at, so the deferred fp64 slots run in nearly every wave), but with the light-ray seed
// (tlimit known from the start, so the fp32 test also rejects triangles behind the light)
// 4.04 -> 3.95 ms, shade-area +1.3%
// Rejected round-3 traversal variants (same-box, profiles/round3_ab_traversal.txt; removed from the
// source in round 4): node loads as 32-bit byte offsets (neutral); near / far planes picked once per
// ray by the inverse direction's sign (97 -> 63 VALU per visit, but k_mis_rays 3.81 -> 4.02 ms); the
// near / far planes selected after the usual loads (MIS 464.3 -> 463.2, BRDF-only 5 831 -> 5 760).
#ifndef MCPT_FILTER_MIS
#define MCPT_FILTER_MIS 1
#endif
#ifndef MCPT_FILTER_BRDF
#define MCPT_FILTER_BRDF 1
#endif

// Closest hit over the 4-wide BVH (Myobj::closet_ray_intersect semantics without the grid):
//  * Aila & Laine's "while-while" loop: a lane descends through inner nodes until it holds a leaf
//    (postponed), and the wave tests triangles only once every active lane has one (or ran out of
//    nodes), so the fp64 triangle tests run with few idle lanes; leaves travel on the stack as
//    ~((first << kLeafBits) | count) (kLeafBits = 5: SAH leaves hold up to 16 triangles);
//  * four slab tests per node visit as one FMA per plane (origin * inverse precomputed; the boxes'
//    conservative margins absorb the extra rounding), hits ordered near-to-far by a 5-comparator
//    network, the nearest followed and the rest pushed far-first;
//  * a short LDS stack of kLds entries per lane with a private (scratch) overflow up to kStack;
//  * every triangle of a hit leaf gets the reference's fp64 Cramer test (Myobj.cpp:165-192) behind
//    a sign pre-test that rejects beta < 0, gamma < 0 and t < 0 before the three divisions (a
//    nonzero quotient has the sign of its operands; the divisions of the surviving candidates are
//    exactly tri_hit's, so accepted hits are bit-identical); origin facet excluded, t > 1e-8, ties
//    to the lower facet id (a total order on (t, facet): the result does not depend on test order);
//  * kFilter: tri_filter's fp32 pre-test first; triangles it cannot reject wait in two per-lane
//    slots and get the fp64 test after the traversal, wave-wide (a third survivor is tested at
//    once); a sure hit lowers tlimit by its fp32 upper bound.
// kCount: also count node visits and triangle tests into *visits / *tests (the traversal roofline's
// events; only the untimed statistics replay instantiates it)
// kTop > 0: nodes [0, kTop) are read from `top` (an LDS copy of the tree's top levels) through a
// generic pointer, the rest from `nodes`
// MCPT_TRACE_DIAG (diagnostics only, with kCount): *witer / *wleaf count the WAVE's iterations of the
// node-visit loop and of the triangle loop (added by the wave's first active lane), so that visits /
// (64 witer) is the traversal's SIMD lane utilisation
#ifndef MCPT_PERSIST_SHADE_AREA
#define MCPT_PERSIST_SHADE_AREA 1
#endif
#ifndef MCPT_TRACE_DIAG
#define MCPT_TRACE_DIAG 0
#endif
// kLazyBG: the running best keeps its leaf slot instead of (beta, gamma) -- 1 VGPR for 4 across the whole
// traversal -- and the winner's (beta, gamma) are recomputed once at the end by the same operations on the same
// triangle, so they are bit-identical (MCPT_RAYS_LAZY_BG, k_mis_rays)
template <int kLds, bool kCount = false, int kTop = 0, bool kFilter = true, bool kLazyBG = false>
__device__ inline Hit trace4_ww(const BvhNode4* __restrict__ nodes, const float4* __restrict__ leafv, d3 ro, d3 rd,
                                int exclude, int* __restrict__ lds, int stride, unsigned* visits = nullptr,
                                unsigned* tests = nullptr, const BvhNode4* top = nullptr, float tlimit0 = FLT_MAX,
                                unsigned* witer = nullptr, unsigned* wleaf = nullptr) {
    auto first_lane = []() { return (int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1; };
    (void)first_lane;
    constexpr int kDone = 0x7fffffff;
    Hit best{-1, DBL_MAX, 0, 0};
    if (isnan(rd.x) || isnan(rd.y) || isnan(rd.z)) return best;  // reference: UB (Myobj.cpp:463-468)
    int spill[kStack - kLds];
    auto inv = [](double d) {
        float f = (float)d;
        if (fabsf(f) < 1e-30f) f = copysignf(1e-30f, f);
        return 1.0f / f;
    };
    const float ix = inv(rd.x), iy = inv(rd.y), iz = inv(rd.z);
    const float oix = (float)ro.x * ix, oiy = (float)ro.y * iy, oiz = (float)ro.z * iz;
    // tlimit0: at least the t of a triangle tri_hit accepts (or FLT_MAX) -- boxes beyond it hold no
    // closest hit
    float tlimit = tlimit0;
    int best_q = -1;  // kLazyBG: the winner's leaf slot
    // the reference's fp64 test of leaf triangle q (the facet is not `exclude`): a sign pre-test
    // rejects beta < 0, gamma < 0 and t < 0 before the three divisions, which are tri_hit's
    auto exact = [&](int q) {
        const float4 a4 = leafv[3 * q], b4 = leafv[3 * q + 1], c4 = leafv[3 * q + 2];
        const int fac = __float_as_int(a4.w);
        const d3 a = f3(a4), ab = sub(a, f3(b4)), ac = sub(a, f3(c4)), ar = sub(a, ro);
        const double detA = det3(ab, ac, rd);
        if (fabs(detA) < MCPT_EPS) return;
        const double nb = det3(ar, ac, rd), ng = det3(ab, ar, rd), nt = det3(ab, ac, ar);
        const bool neg = detA < 0;
        if ((nb != 0 && ((nb < 0) != neg)) || (ng != 0 && ((ng < 0) != neg)) || (nt != 0 && ((nt < 0) != neg)))
            return;
        const double beta = nb / detA, gamma = ng / detA, tt = nt / detA;
        if (beta < 0 || gamma < 0 || beta + gamma > 1 || tt < 0 || fabs(tt) < MCPT_EPS) return;
        if (tt < best.t || (tt == best.t && fac < best.f)) {
            best.f = fac;
            best.t = tt;
            if (kLazyBG) {
                best_q = q;
            } else {
                best.beta = beta;
                best.gamma = gamma;
            }
            tlimit = fminf(tlimit, (float)tt * 1.0001f + 1e-5f);
        }
    };
    const RayF rf = kFilter ? ray_f(ro, rd) : RayF{};
    int pend0 = -1, pend1 = -1;
    int sp = 0;
    auto push = [&](int v) {
        if (sp < kLds) lds[sp * stride] = v;
        else if (sp < kStack) spill[sp - kLds] = v;
        sp = sp < kStack ? sp + 1 : sp;
    };
    auto pop = [&]() -> int {
        if (sp == 0) return kDone;
        --sp;
        return sp < kLds ? lds[sp * stride] : spill[sp - kLds];
    };
    int node = 0;
    int leaf = 0;
    while (node != kDone || leaf < 0) {
        while (node >= 0 && node != kDone) {
            if (kCount) ++*visits;
            if (kCount && MCPT_TRACE_DIAG && witer && first_lane()) ++*witer;
            float t[4];
            int code[4];
            // the tree's top levels from LDS when the whole wave is in them (a wave-uniform branch)
            {
                float lo[3][4], hi[3][4];
                int chs[4];
                if (kTop > 0 && __all(node < kTop)) load_node(top + node, lo, hi, chs);
                else load_node(nodes + node, lo, hi, chs);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float tx0 = fmaf(lo[0][k], ix, -oix), tx1 = fmaf(hi[0][k], ix, -oix);
                    const float ty0 = fmaf(lo[1][k], iy, -oiy), ty1 = fmaf(hi[1][k], iy, -oiy);
                    const float tz0 = fmaf(lo[2][k], iz, -oiz), tz1 = fmaf(hi[2][k], iz, -oiz);
                    const float t0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
                    const float t1 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tlimit));
                    const bool h = chs[k] != kBvh4Empty && t0 <= t1 * 1.00001f + 1e-6f;
                    t[k] = h ? t0 : FLT_MAX;
                    code[k] = h ? chs[k] : kDone;
                }
            }
            // sort (t, code) ascending; misses (FLT_MAX, kDone) sink to the end
            auto cs = [&](int a, int b) {
                const bool sw = t[b] < t[a];
                const float ta = t[a], tb = t[b];
                const int ca = code[a], cb = code[b];
                t[a] = sw ? tb : ta, t[b] = sw ? ta : tb;
                code[a] = sw ? cb : ca, code[b] = sw ? ca : cb;
            };
            cs(0, 1), cs(2, 3), cs(0, 2), cs(1, 3), cs(1, 2);
            if (code[3] != kDone) push(code[3]);
            if (code[2] != kDone) push(code[2]);
            if (code[1] != kDone) push(code[1]);
            node = code[0] != kDone ? code[0] : pop();
            if (node < 0 && leaf >= 0) {  // postpone the leaf, keep descending
                leaf = node;
                node = pop();
            }
            if (!__any(leaf >= 0)) break;
        }
        while (leaf < 0) {
            const int packed = ~leaf, first = packed >> kLeafBits, cnt = packed & ((1 << kLeafBits) - 1);
            for (int q = first; q < first + cnt; q++) {
                const float4 a4 = leafv[3 * q], b4 = leafv[3 * q + 1], c4 = leafv[3 * q + 2];
                const int fac = __float_as_int(a4.w);
                if (kCount && MCPT_TRACE_DIAG && wleaf && first_lane()) ++*wleaf;
                if (fac == exclude) continue;
                if (kCount) ++*tests;
                if (kFilter) {
                    // fp32 pre-test; survivors wait in two slots for the fp64 test (run wave-wide at
                    // the end, or at once for a third survivor), so the fp64 work has few idle lanes
                    float tup;
                    const int v = tri_filter(a4, b4, c4, rf, tlimit, &tup);
                    if (v == 0) continue;
                    if (v == 2) tlimit = fminf(tlimit, tup * 1.0001f + 1e-5f);
                    if (pend0 < 0) pend0 = q;
                    else if (pend1 < 0) pend1 = q;
                    else exact(q);
                } else {
                    exact(q);
                }
            }
            leaf = node;
            if (node < 0) node = pop();
        }
    }
    if (kFilter && pend0 >= 0) exact(pend0);
    if (kFilter && pend1 >= 0) exact(pend1);
    if (kLazyBG && best_q >= 0) {  // the winner's (beta, gamma): exact()'s operations on its triangle
        const float4 a4 = leafv[3 * best_q], b4 = leafv[3 * best_q + 1], c4 = leafv[3 * best_q + 2];
        const d3 a = f3(a4), ab = sub(a, f3(b4)), ac = sub(a, f3(c4)), ar = sub(a, ro);
        const double detA = det3(ab, ac, rd);
        best.beta = det3(ar, ac, rd) / detA;
        best.gamma = det3(ab, ar, rd) / detA;
    }
    return best;
}

// ---- 8-wide traversal over BvhNode8Q (the compressed wide BVH, mcpt_internal.h) ----
// Per lane: a node group (nb << 8 | the hit bits of the node's inner children in near-to-far order: the
// bit of slot s at position s ^ oct, oct = the octant code of the ray's direction, so that the lowest bit
// is the nearest child), a triangle group (base triangle slot tb, 16-bit mask tw) and a stack of node
// groups (one word each).  No sorting and no child codes to load: child = base + slot.  Closest hit by the
// reference's fp64 test (Myobj.cpp:165-192) with ties to the lower facet id, on conservatively pruned
// boxes -- the same hits as trace4_ww, visited in another order.
struct Cw8Frame {  // per-ray constants of the slab tests
    float inv[3], oi[3];
    unsigned oct;  // bit a set iff the ray goes +a: near children (negative side) come first
};
__device__ inline Cw8Frame cw8_frame(d3 ro, d3 rd) {
    Cw8Frame F;
    auto inv = [](double d) {
        float f = (float)d;
        if (fabsf(f) < 1e-30f) f = copysignf(1e-30f, f);
        return 1.0f / f;
    };
    F.inv[0] = inv(rd.x), F.inv[1] = inv(rd.y), F.inv[2] = inv(rd.z);
    F.oi[0] = (float)ro.x * F.inv[0], F.oi[1] = (float)ro.y * F.inv[1], F.oi[2] = (float)ro.z * F.inv[2];
    F.oct = (F.inv[0] < 0 ? 0u : 1u) | (F.inv[1] < 0 ? 0u : 2u) | (F.inv[2] < 0 ? 0u : 4u);
    return F;
}
// one node visit: the eight children's slab tests on the decoded byte planes (near / far planes picked per
// axis by the direction's sign, as node_tplanes), then the new node group (inner hits in key order) and
// triangle group (leaf hits spread over their two triangle slots, masked by the used slots)
__device__ inline void cw8_visit(const BvhNode8Q* __restrict__ nd, const Cw8Frame& F, float tlimit, unsigned* ng, int* tb,
                                 unsigned* tw) {
    const float4 v0 = *reinterpret_cast<const float4*>(nd->org);
    const uint4 v1 = *reinterpret_cast<const uint4*>(&nd->qlo[0][0]);
    const uint4 v2 = *reinterpret_cast<const uint4*>(&nd->qlo[2][0]);
    const uint4 v3 = *reinterpret_cast<const uint4*>(&nd->qhi[1][0]);
    const int4 v4 = *reinterpret_cast<const int4*>(&nd->base_inner);
    const unsigned ex = __float_as_uint(v0.w);
    const float org[3] = {v0.x, v0.y, v0.z};
    const unsigned ql[3][2] = {{v1.x, v1.y}, {v1.z, v1.w}, {v2.x, v2.y}};
    const unsigned qh[3][2] = {{v2.z, v2.w}, {v3.x, v3.y}, {v3.z, v3.w}};
    float m[3], b[3];
    unsigned qn[3][2], qf[3][2];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        m[a] = __uint_as_float(((ex >> (8 * a)) & 0xffu) << 23) * F.inv[a];
        b[a] = fmaf(org[a], F.inv[a], -F.oi[a]);
        const bool neg = F.inv[a] < 0;
#pragma unroll
        for (int h = 0; h < 2; h++) qn[a][h] = neg ? qh[a][h] : ql[a][h], qf[a][h] = neg ? ql[a][h] : qh[a][h];
    }
    unsigned hit = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int h = k >> 2, sh = 8 * (k & 3);
        float tn[3], tf[3];
#pragma unroll
        for (int a = 0; a < 3; a++) {
            tn[a] = fmaf((float)((qn[a][h] >> sh) & 0xffu), m[a], b[a]);
            tf[a] = fmaf((float)((qf[a][h] >> sh) & 0xffu), m[a], b[a]);
        }
        const float t0 = fmaxf(fmaxf(tn[0], tn[1]), fmaxf(tn[2], 0.0f));
        const float t1 = fminf(fminf(tf[0], tf[1]), fminf(tf[2], tlimit));
        hit |= (t0 <= fmaf(t1, 1.00001f, 1e-6f)) ? 1u << k : 0u;
    }
    const unsigned imask = ex >> 24;
    unsigned ih = hit & imask;  // slot s -> bit s ^ oct
    ih = (F.oct & 1) ? ((ih & 0x55u) << 1) | ((ih >> 1) & 0x55u) : ih;
    ih = (F.oct & 2) ? ((ih & 0x33u) << 2) | ((ih >> 2) & 0x33u) : ih;
    ih = (F.oct & 4) ? ((ih & 0x0fu) << 4) | ((ih >> 4) & 0x0fu) : ih;
    *ng = ((unsigned)v4.x << 8) | ih;
    unsigned lh = hit & ~imask & 0xffu;  // slot s -> triangle slots 2 s, 2 s + 1
    lh = (lh | (lh << 4)) & 0x0f0fu;
    lh = (lh | (lh << 2)) & 0x3333u;
    lh = (lh | (lh << 1)) & 0x5555u;
    *tb = v4.y;
    *tw = (lh | (lh << 1)) & (unsigned)v4.z;
}
// the next child of a node group (its nearest remaining hit), removed from the group
__device__ inline int cw8_next(unsigned* ng, unsigned oct) {
    const unsigned bit = (unsigned)__builtin_ctz(*ng & 0xffu);
    *ng &= ~(1u << bit);
    return (int)((*ng >> 8) + (bit ^ oct));
}
// the reference's fp64 test of triangle slot q against the best hit so far (origin facet excluded)
__device__ inline void cw8_tri(const float4* __restrict__ triv, int q, d3 ro, d3 rd, int excl, Hit* best, float* tlimit) {
    const float4 a4 = triv[3 * q], b4 = triv[3 * q + 1], c4 = triv[3 * q + 2];
    const int fac = __float_as_int(a4.w);
    if (fac == excl) return;
    const d3 a = f3(a4), ab = sub(a, f3(b4)), ac = sub(a, f3(c4)), ar = sub(a, ro);
    const double detA = det3(ab, ac, rd);
    if (fabs(detA) < MCPT_EPS) return;
    const double nb = det3(ar, ac, rd), ng = det3(ab, ar, rd), nt = det3(ab, ac, ar);
    const bool neg = detA < 0;
    if ((nb != 0 && ((nb < 0) != neg)) || (ng != 0 && ((ng < 0) != neg)) || (nt != 0 && ((nt < 0) != neg))) return;
    const double beta = nb / detA, gamma = ng / detA, tt = nt / detA;
    if (beta < 0 || gamma < 0 || beta + gamma > 1 || tt < 0 || fabs(tt) < MCPT_EPS) return;
    if (tt < best->t || (tt == best->t && fac < best->f)) {
        *best = Hit{fac, tt, beta, gamma};
        *tlimit = fminf(*tlimit, (float)tt * 1.0001f + 1e-5f);
    }
}
// the root's node group: its only "child" is node 0 (slot 0, bit oct)
__device__ inline unsigned cw8_root(unsigned oct) { return 1u << oct; }
// closest hit of one ray per lane through an 8-wide tree (while-while: the wave descends until every lane
// holds a triangle group or is done, then tests the groups); stack of node groups: kLds entries in LDS
// ([entry][lane], stride) and a private overflow up to kStack
template <int kLds, bool kCount = false>
__device__ inline Hit trace_cw8(const BvhNode8Q* __restrict__ nodes, const float4* __restrict__ triv, d3 ro, d3 rd, int excl,
                                unsigned* __restrict__ lds, int stride, float tlimit = FLT_MAX, unsigned* visits = nullptr,
                                unsigned* tests = nullptr) {
    Hit best{-1, DBL_MAX, 0, 0};
    if (isnan(rd.x) || isnan(rd.y) || isnan(rd.z)) return best;  // reference: UB (Myobj.cpp:463-468)
    unsigned spill[kStack - kLds];
    int sp = 0;
    const Cw8Frame F = cw8_frame(ro, rd);
    unsigned ng = cw8_root(F.oct), tw = 0;
    int tb = 0;
    while (true) {
        while (true) {
            const bool want = tw == 0 && ((ng & 0xffu) != 0 || sp > 0);
            if (!__any(want)) break;
            if (want) {
                if ((ng & 0xffu) == 0) {
                    --sp;
                    ng = sp < kLds ? lds[sp * stride] : spill[sp - kLds];
                }
                const int child = cw8_next(&ng, F.oct);
                if (ng & 0xffu) {
                    if (sp < kLds) lds[sp * stride] = ng;
                    else if (sp < kStack) spill[sp - kLds] = ng;
                    sp = sp < kStack ? sp + 1 : sp;
                }
                if (kCount) ++*visits;
                cw8_visit(nodes + child, F, tlimit, &ng, &tb, &tw);
            }
        }
        if (tw == 0) break;
        while (tw != 0) {
            const int bit = __builtin_ctz(tw);
            tw &= tw - 1;
            if (kCount) ++*tests;
            cw8_tri(triv, tb + bit, ro, rd, excl, &best, &tlimit);
        }
    }
    return best;
}

// The picked triangle's spherical triangle for Arvo's sampler (Mylight.cpp:453-461): the reference's
// literal chain (light_tri_stage -- sqrt / division unit vectors, correctly rounded acos for
// alpha, beta, gamma and c, alpha + beta + gamma - pi), so the sampled direction follows the oracle's arithmetic; light_full's
// rsqrt / atan2 form differs by up to ~1e-10 relative in sA for small triangles.  One triangle per
// node, so the literal chain costs little here.  light_full stays as the fallback for a pick the
// literal chain would cull (a pick from the fp32 prep's weights).
__device__ inline void pick_sph(const DScene& S, int pick, d3 p, d3 N, SphTri* sph) {
    const double4 ln = S.lt_n[pick];
    const d3 p0 = f3(S.lt_v[3 * pick]), p1 = f3(S.lt_v[3 * pick + 1]), p2 = f3(S.lt_v[3 * pick + 2]);
    if (light_tri_stage<true>(p0, p1, p2, mk3(ln.x, ln.y, ln.z), S.light_sum[pick], p, N, sph) != 0)
        light_full(p0, p1, p2, 2.0 * ln.w, p, N, sph);
}

// x86 cvttsd2si semantics for (int)floor(x) of the reference (out of range -> INT_MIN)
__device__ inline int icvt(double f) { return (f >= -2147483648.0 && f < 2147483648.0) ? (int)f : (int)0x80000000u; }
__device__ inline int ifloor(double x) { return icvt(floor(x)); }
// Myobj::closet_ray_intersect (Myobj.cpp:334-474) and closet_ray_intersect_light_triangle (:476-622)
// on the reference's uniform grid, in its arithmetic: a 3D-DDA from the cell holding the origin
// (no clipping to the box: an origin outside it, or rounding to cell -1 on the box's min face, is a
// miss -- the reference's "crack"); in each cell every listed facet except the origin facet gets
// the fp64 Cramer test, and a hit counts only if its point lies in the current cell; the first
// cell with a counted hit returns its nearest (first listed on ties).  light_only skips non-light
// facets and steps every axis whose crossing ties the nearest within 1e-8 (:576-604).
__device__ inline Hit grid_trace(const DScene& S, d3 ro, d3 rd, int exclude, bool light_only) {
    Hit best{-1, DBL_MAX, 0, 0};
    if (isnan(rd.x) || isnan(rd.y) || isnan(rd.z)) return best;  // reference: UB (Myobj.cpp:463-468)
    const d3 mn = mk3(S.g_mn[0], S.g_mn[1], S.g_mn[2]);
    const d3 x0 = mul(sub(ro, mn), S.g_inv_d);
    const double xyz0[3] = {x0.x, x0.y, x0.z}, dir[3] = {rd.x, rd.y, rd.z};
    int xyz[3], sign[3], nxyz[3];
    double ts[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        xyz[i] = ifloor(xyz0[i]);
        sign[i] = dir[i] < 0 ? -1 : 1;
        if (fabs(dir[i]) < MCPT_EPS) sign[i] = 0;
        if (sign[i]) {
            if (fabs(floor(xyz0[i]) - xyz0[i]) < MCPT_EPS) nxyz[i] = xyz[i] + sign[i];
            else nxyz[i] = sign[i] > 0 ? icvt(ceil(xyz0[i])) : ifloor(xyz0[i]);
            ts[i] = (nxyz[i] - xyz0[i]) / dir[i];
        } else {
            nxyz[i] = -1;
            ts[i] = DBL_MAX;
        }
    }
    for (;;) {
        for (int i = 0; i < 3; i++)
            if (xyz[i] < 0 || xyz[i] > S.g_lim[i]) return best;
        const size_t c = ((size_t)xyz[0] * S.g_gd[1] + xyz[1]) * S.g_gd[2] + xyz[2];
        const int q1 = S.g_start[c + 1];
        for (int q = S.g_start[c]; q < q1; q++) {
            const int f = S.g_tri[q];
            if (light_only && S.tri_light[f] < 0) continue;
            if (f == exclude) continue;
            const TriHit h = tri_hit(f3(S.tri_v[3 * f]), f3(S.tri_v[3 * f + 1]), f3(S.tri_v[3 * f + 2]), ro, rd);
            if (!h.hit) continue;
            const d3 cp = mul(sub(add(ro, mul(rd, h.t)), mn), S.g_inv_d);
            if (ifloor(cp.x) != xyz[0] || ifloor(cp.y) != xyz[1] || ifloor(cp.z) != xyz[2]) continue;
            if (h.t < best.t) best = Hit{f, h.t, h.beta, h.gamma};
        }
        if (best.f >= 0) return best;
        if (!light_only) {
            double t = DBL_MAX;
            int ind = -1;
            for (int i = 0; i < 3; i++)
                if (sign[i] != 0 && ts[i] < t) {
                    ind = i;
                    t = ts[i];
                }
            if (ind < 0) return best;
            xyz[ind] += sign[ind];
            nxyz[ind] += sign[ind];
            ts[ind] = (nxyz[ind] - xyz0[ind]) / dir[ind];
        } else {
            double t = DBL_MAX;
            for (int i = 0; i < 3; i++)
                if (ts[i] < t) t = ts[i];
            if (t == DBL_MAX) return best;
            for (int i = 0; i < 3; i++)
                if (fabs(t - ts[i]) < MCPT_EPS) {
                    xyz[i] += sign[i];
                    nxyz[i] += sign[i];
                    ts[i] = (nxyz[i] - xyz0[i]) / dir[i];
                }
        }
    }
}

// ============================================================================================
// wavefront queue (SoA)
// ============================================================================================
// 3-vectors (the queue's p, n, wo, tp, Aux's directions and throughputs, the prep kernels' node inputs)
// are interleaved, [cap][3] (node i's y at p[3 i + 1]): a wave's loads of one vector cover 1 536
// contiguous bytes, fully coalesced, and a vector is one dwordx4 + dwordx2 pair.  The component-major
// form (x[cap] y[cap] z[cap]) was measured slower in round 3 (BRDF-only 5 893 interleaved vs 5 637,
// MIS 454.8 vs 453.5; profiles/round3_ab_queue_layout.txt) and removed.
__host__ __device__ inline size_t idx3(size_t, size_t i, int k) { return 3 * i + (size_t)k; }
template <class T>
__device__ inline d3 ld3(const T* a, size_t cap, size_t i) {
    return mk3(a[idx3(cap, i, 0)], a[idx3(cap, i, 1)], a[idx3(cap, i, 2)]);
}
__device__ inline void st3(double* a, size_t cap, size_t i, d3 v) {
    a[idx3(cap, i, 0)] = v.x, a[idx3(cap, i, 1)] = v.y, a[idx3(cap, i, 2)] = v.z;
}
struct Queue {
    double* p;      // 3-vectors (idx3): shading point
    double* n;      // interpolated normal
    double* wo;
    double* tp;     // path throughput
    int* f;         // cap
    int* pixel;     // cap
    int* sample;    // cap
    uint64_t* node; // cap   heap id (MIS) / depth+1 (BRDF)
    int* par;       // cap   MIS tree reduction: parent slot * 2 + (0 light, 1 BRDF child), -1 root
    double* wsum;   // cap   (MIS prep output)
    int* pick;      // cap   (MIS prep output)
    unsigned* count;
    int cap;
};

// the ray sets of a generation: persistent waves with ray refill (k_rays_persistent) over the BVH,
// one thread per ray (k_mis_rays) over the reference grid
// (-1 auto: persistent when the acceleration structures exceed an XCD's 4 MiB L2 -- long, cache-
// missing rays: Cornell-1M traversal -13%, the frame +9%; Veach's short L2-resident rays run 5%
// faster one per thread at 8 waves/SIMD; profiles/round2b_ab_rays_persistent.txt)
#ifndef MCPT_RAYS_PERSISTENT
#define MCPT_RAYS_PERSISTENT -1
#endif
// k_rays_persistent reads the 64-B compressed nodes (BvhNode4Q): Cornell-1M traversal -6%; the
// L2-resident kernels keep the 128-B fp32 nodes (their decode VALU costs more than the lines save:
// Veach MIS -1.5%, BRDF -5%; profiles/round2b_ab_bvh_quant.txt)
#ifndef MCPT_BAND_DIAG
#define MCPT_BAND_DIAG 0
#endif
#ifndef MCPT_EXACT_PICK
#define MCPT_EXACT_PICK 1
#endif
#ifndef MCPT_WORKING_SET
#define MCPT_WORKING_SET (48 << 20)  // default wavefront working set (nodes per generation)
#endif
#ifndef MCPT_ROOT_GROUP
#define MCPT_ROOT_GROUP 2  // small scenes: consecutive roots take this many samples of a pixel (A/B: 1 / 2 / 4 / 8 -> 437 / 442 / 437 / 430)
#endif
#ifndef MCPT_ROOT_MINOR
#define MCPT_ROOT_MINOR -1  // -1 auto (by acceleration-structure size), 0 sample-major, 1 sample-minor
#endif
struct Params {
    DScene S;
    uint64_t seed;
    double inv_spp;
    double* fb;                  // W*H*3 fp64
    unsigned long long* stats;   // [0] cached root preps [1] light survivors [2] rays [3] light rays [4] overflow
                                 // [5] prep candidates [6] light-side culls [7] full preps
    int mode;
    // BRDF-only (k_extend_brdf): root entries (node id 1) carry only facet, pixel and sample; their
    // point, normal and wo come from the per-pixel root table ([npx][9], k_root_table) and their
    // throughput is 1 -- so k_roots_t does not copy a per-pixel constant into every sample's entry
    const double* root_pnw;
};

__device__ inline int lane_id() { return __lane_id(); }

// wave-aggregated append: returns this lane's slot (or -1 if !want)
__device__ inline int wave_append(unsigned* counter, bool want) {
    const uint64_t m = __ballot(want);
    if (m == 0) return -1;
    const int leader = __ffsll((unsigned long long)m) - 1;
    const int lane = lane_id();
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(m));
    base = __shfl(base, leader);
    const uint64_t below = lane == 0 ? 0ull : (m & ((~0ull) >> (64 - lane)));
    return want ? (int)(base + __popcll(below)) : -1;
}

// workgroup-aggregated append: ONE atomic per workgroup.  The queue counter is a single word, and
// one device-scope word saturates at ~88 atomic adds per microsecond (MI355X_MICROARCH.md,
// "dequeue"), so per-wave appends capped the root and extension kernels at ~5.6 G nodes/s.
// Must be called by every thread of the workgroup (it contains barriers).
__device__ inline int block_append(unsigned* counter, bool want) {
    __shared__ unsigned s_cnt[16];  // per wave, up to 1024 threads
    __shared__ unsigned s_base;
    const int lane = lane_id(), wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const uint64_t m = __ballot(want);
    if (lane == 0) s_cnt[wid] = (unsigned)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned tot = 0;
        for (int w = 0; w < nw; w++) {
            const unsigned c = s_cnt[w];
            s_cnt[w] = tot;
            tot += c;
        }
        s_base = tot ? atomicAdd(counter, tot) : 0u;
    }
    __syncthreads();
    const unsigned base = s_base + s_cnt[wid];
    __syncthreads();  // s_cnt / s_base are reused by the next call
    const uint64_t below = lane == 0 ? 0ull : (m & ((~0ull) >> (64 - lane)));
    return want ? (int)(base + __popcll(below)) : -1;
}

// workgroup-aggregated statistics counters: adds the sums of a and b (each 0..3) over the
// workgroup to ca / cb with one atomic each (per-lane or per-wave atomics on a shared counter
// serialise at wavefront node rates).  Must be called by ALL threads of the workgroup.
__device__ inline void block_count(unsigned long long* ca, unsigned a, unsigned long long* cb = nullptr,
                                   unsigned b = 0) {
    __shared__ unsigned s_sum[2][16];
    const int lane = lane_id(), wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const unsigned na = (unsigned)__popcll(__ballot(a & 1)) + 2u * (unsigned)__popcll(__ballot(a & 2));
    const unsigned nb = (unsigned)__popcll(__ballot(b & 1)) + 2u * (unsigned)__popcll(__ballot(b & 2));
    if (lane == 0) { s_sum[0][wid] = na; s_sum[1][wid] = nb; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long ta = 0, tb = 0;
        for (int w = 0; w < nw; w++) { ta += s_sum[0][w]; tb += s_sum[1][w]; }
        if (ta) atomicAdd(ca, ta);
        if (cb && tb) atomicAdd(cb, tb);
    }
    __syncthreads();  // s_sum is reused by the next call
}

// the statistics block: words 0..15 (the render's counters), then kStatShards 128-B lines for the
// ray counts (rays, light_rays), which every wavefront workgroup adds to -- one line per 8 workgroups
// round robin instead of one word for all (the host sums the shards)
constexpr int kStatShards = 8;
constexpr int kStatBytes = 128 * (1 + kStatShards);
template <class P_>
__device__ inline unsigned long long* ray_stats(const P_& P) {
    return P.stats + 16 * (1 + (blockIdx.x & (kStatShards - 1)));
}

// shading point and normal of a hit (main.cpp:406-407: interpolated position, normalised
// interpolation of the vertex normals)
__device__ inline void node_point(const DScene& S, int f, double beta, double gamma, d3* p, d3* N) {
    const float4* v = S.tri_v + 3 * f;
    const float* nv = S.tri_n + 9 * f;
    const double a0 = 1.0 - beta - gamma;
    *p = add(add(mul(f3(v[0]), a0), mul(f3(v[1]), beta)), mul(f3(v[2]), gamma));
    *N = normalized(add(add(mul(mk3(nv[0], nv[1], nv[2]), a0), mul(mk3(nv[3], nv[4], nv[5]), beta)),
                        mul(mk3(nv[6], nv[7], nv[8]), gamma)));
}

// node entry of shade_with_* (main.cpp:406-437 / :351-383): interpolate, back-face -> 0,
// emitter -> its emission, Russian roulette (MIS / BRDF: dim 0; shade() draws it later); kind:
// 0 contributes nothing, 1 emitter (light index li), 2 shading node (p, N) to push.
struct Entry {
    int kind, li;
    d3 p, N;
};
__device__ inline Entry entry_eval(const Params& P, bool active, int f, double beta, double gamma, d3 wo, int pixel,
                                   int sample, uint64_t node) {
    const DScene& S = P.S;
    Entry e{0, -1, mk3(0, 0, 0), mk3(0, 0, 0)};
    if (!active) return e;
    // MIS: heap ids (root 1, children 2n, 2n+1); BRDF / shade: paths (node = depth + 1)
    const bool too_deep = P.mode == MCPT_MODE_MIS ? node >= (2ull << MCPT_MAX_DEPTH) : node > MCPT_MAX_DEPTH + 1;
    if (too_deep) return e;
    node_point(S, f, beta, gamma, &e.p, &e.N);
    if (dot(e.N, wo) < 0) return e;
    const int li = S.tri_light[f];
    if (li >= 0) {
        e.kind = 1;
        e.li = li;
    } else if (P.mode == MCPT_MODE_SHADE || P.mode == MCPT_MODE_SHADE_AREA) {
        e.kind = 2;  // shade() samples direct light before its RR draw (main.cpp:295-327)
    } else {
        const uint64_t key = counter_key(P.seed, (uint64_t)pixel, (uint64_t)sample, node);
        e.kind = counter_u(key, 0) > MCPT_P_RR ? 0 : 2;
    }
    return e;
}
// writes a shading node at queue position slot (from an append), or flags the overflow
__device__ inline void queue_write(const Params& P, bool push, int slot, const Entry& e, int f, d3 wo, d3 tp, int pixel,
                                   int sample, uint64_t node, int par, Queue& q, bool write_tp = true) {
    if (!push) return;
    if (slot >= q.cap) {
        atomicOr((unsigned long long*)(P.stats + 4), 1ull);
        return;
    }
    const size_t s = (size_t)slot;
    st3(q.p, q.cap, s, e.p);
    st3(q.n, q.cap, s, e.N);
    st3(q.wo, q.cap, s, wo);
    if (write_tp) st3(q.tp, q.cap, s, tp);
    q.f[s] = f;
    q.pixel[s] = pixel;
    q.sample[s] = sample;
    q.node[s] = node;
    q.par[s] = par;
}
// appends a shading node to q.  Must be called by ALL threads of the workgroup (block_append).
__device__ inline void queue_push(const Params& P, bool push, const Entry& e, int f, d3 wo, d3 tp, int pixel, int sample,
                                  uint64_t node, int par, Queue& q) {
    const int slot = block_append(q.count, push);
    if (!push) return;
    if (slot >= q.cap) {
        atomicOr((unsigned long long*)(P.stats + 4), 1ull);
        return;
    }
    const size_t s = (size_t)slot;
    st3(q.p, q.cap, s, e.p);
    st3(q.n, q.cap, s, e.N);
    st3(q.wo, q.cap, s, wo);
    st3(q.tp, q.cap, s, tp);
    q.f[s] = f;
    q.pixel[s] = pixel;
    q.sample[s] = sample;
    q.node[s] = node;
    q.par[s] = par;
}
// entry + push with forward throughput: emitters add tp x emission to the framebuffer (BRDF-only,
// shade() and the fresh-pdf MIS path).  Must be called by ALL threads of the workgroup.
__device__ inline void node_entry(const Params& P, bool active, int f, double beta, double gamma, d3 wo, d3 tp,
                                  int pixel, int sample, uint64_t node, Queue& q, int par = -1) {
    const Entry e = entry_eval(P, active, f, beta, gamma, wo, pixel, sample, node);
    if (e.kind == 1) {
        const DScene& S = P.S;
        double* px = P.fb + 3 * (size_t)pixel;
        unsafeAtomicAdd(px + 0, tp.x * S.light_rad[3 * e.li + 0] * P.inv_spp);
        unsafeAtomicAdd(px + 1, tp.y * S.light_rad[3 * e.li + 1] * P.inv_spp);
        unsafeAtomicAdd(px + 2, tp.z * S.light_rad[3 * e.li + 2] * P.inv_spp);
    }
    queue_push(P, e.kind == 2, e, f, wo, tp, pixel, sample, node, par, q);
}

// ============================================================================================
// kernels
// ============================================================================================
template <bool kGrid>
__global__ __launch_bounds__(kTraceBlock) void k_primary(DScene S, CamFrame cam, int* hit_f, double* hit_tbg) {
    __shared__ int stack[kRayLds * kTraceBlock];
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int npx = cam.W * cam.H;
    if (idx >= npx) return;
    const int i = idx / cam.W, j = idx % cam.W;
    const d3 dir = cam_dir(cam, i, j);
    const Hit h = kGrid ? grid_trace(S, cam.eye, dir, -1, false)
                        : trace4_ww<kRayLds>(S.bvh4, S.leaf_v, cam.eye, dir, -1, stack + threadIdx.x, kTraceBlock);
    hit_f[idx] = h.f;
    hit_tbg[3 * idx] = h.f >= 0 ? h.t : 0.0;
    hit_tbg[3 * idx + 1] = h.f >= 0 ? h.beta : 0.0;
    hit_tbg[3 * idx + 2] = h.f >= 0 ? h.gamma : 0.0;
}

// roots: r in [0, nroots): pixel = r % npx, sample = s0 + r / npx
// root order: the call's nsamp samples in blocks of `group` consecutive samples; within a block,
// pixel-major with the block's samples of a pixel consecutive (group 1 = sample-major over the frame,
// group nsamp = fully sample-minor: a pixel's samples leave one point, coherent traversal of a BVH
// that misses L2)
// Per-pixel root table (k_root_table, once per call): a root's entry (main.cpp:406-437 at the primary
// hit) is the same for every sample of its pixel except the Russian roulette draw, so the point, normal
// and wo (9 doubles) and the kind (-2 nothing: miss or back face, -1 shading, >= 0 emitter li) are
// computed once per pixel with the same functions, and k_roots_t only draws RR and appends.
// Roots from the per-pixel table by k_roots_t (kRootsPT roots per thread, one queue atomic per 2 048
// roots).  The table alone in round 3's k_roots (node_entry per root, one atomic per 256 roots) changed
// nothing (111-112 ms per profile run, profiles/round3_ab_acos_dpp_roottab.txt): it was bound by the
// queue counter's atomic rate; with k_roots_t 112 -> 55 ms, MIS +1.7% same-box
// (profiles/round3_ab_roots_batched.txt).
struct RootTab {
    double* pnw;  // [npx][9]: p, N, wo
    int* kind;    // [npx]
};
__global__ __launch_bounds__(256) void k_root_table(DScene S, CamFrame cam, const int* hit_f, const double* hit_tbg, RootTab rt) {
    const int px = blockIdx.x * blockDim.x + threadIdx.x;
    if (px >= cam.W * cam.H) return;
    const int f = hit_f[px];
    d3 p = mk3(0, 0, 0), N = mk3(0, 0, 0), wo = mk3(0, 0, 0);
    int kind = -2;
    if (f >= 0) {
        wo = mul(cam_dir(cam, px / cam.W, px % cam.W), -1);
        node_point(S, f, hit_tbg[3 * px + 1], hit_tbg[3 * px + 2], &p, &N);
        if (!(dot(N, wo) < 0)) kind = S.tri_light[f] >= 0 ? S.tri_light[f] : -1;
    }
    double* o = rt.pnw + 9 * (size_t)px;
    o[0] = p.x, o[1] = p.y, o[2] = p.z, o[3] = N.x, o[4] = N.y, o[5] = N.z, o[6] = wo.x, o[7] = wo.y, o[8] = wo.z;
    rt.kind[px] = kind;
}

// pixel and sample of root rg (the call's root index; order above)
__device__ inline void root_of(long long rg, int npx, int s0, int group, int nsamp, int* pixel, int* sample) {
    const long long full = (long long)(nsamp / group) * group * npx;  // roots in whole blocks
    if (full < (1ll << 31)) {  // uniform: 32-bit division (a 64-bit one is a long emulated sequence)
        const unsigned gn = (unsigned)group * (unsigned)npx, ur = (unsigned)rg;
        if (rg < full) {
            const unsigned blk = ur / gn, idx = ur - blk * gn;
            *pixel = (int)(idx / (unsigned)group);
            *sample = s0 + (int)blk * group + (int)(idx - (unsigned)*pixel * (unsigned)group);
        } else {
            const unsigned gt = (unsigned)(nsamp % group), idx = ur - (unsigned)full;
            *pixel = (int)(idx / gt);
            *sample = s0 + (nsamp / group) * group + (int)(idx - (unsigned)*pixel * gt);
        }
    } else if (rg < full) {
        const long long blk = rg / ((long long)group * npx), idx = rg - blk * group * npx;
        *pixel = (int)(idx / group);
        *sample = s0 + (int)blk * group + (int)(idx % group);
    } else {
        const int gt = nsamp % group;
        const long long idx = rg - full;
        *pixel = (int)(idx / gt);
        *sample = s0 + (nsamp / group) * group + (int)(idx % gt);
    }
}

// Roots from the per-pixel table, kRootsPT per thread: the queue's single counter word takes ~88
// atomic adds per microsecond (MI355X_MICROARCH.md), and one block_append per 256 roots held k_roots at
// that rate (~160 k appends, ~1.8 ms per 41 M-root refill).  Here a 256-thread block takes 256 x
// kRootsPT roots with ONE atomic; sub-batch j (roots base + 256 j + thread) is compacted in order
// and placed after sub-batches < j, so the queue order equals k_roots' and every store is coalesced.
#ifndef MCPT_ROOTS_PT
#define MCPT_ROOTS_PT 8
#endif
constexpr int kRootsPT = MCPT_ROOTS_PT;
// lite (BRDF-only with P.root_pnw): the entries' point, normal, wo and throughput are not written
// (k_extend_brdf reads them from the root table)
__global__ __launch_bounds__(256) void k_roots_t(Params P, const int* __restrict__ hit_f, int npx, int s0, long long rbase,
                                                 int nroots, Queue q, int group, int nsamp, RootTab rt, int lite) {
    __shared__ unsigned s_w[kRootsPT][4];
    __shared__ unsigned s_base;
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const int base = blockIdx.x * 256 * kRootsPT;
    int px[kRootsPT], sm[kRootsPT];
    uint64_t wm[kRootsPT];
#pragma unroll
    for (int j = 0; j < kRootsPT; j++) {
        const int r = base + 256 * j + (int)threadIdx.x;
        bool want = false;
        px[j] = 0, sm[j] = 0;
        if (r < nroots) {
            root_of(rbase + r, npx, s0, group, nsamp, &px[j], &sm[j]);
            const int kind = rt.kind[px[j]];
            if (kind >= 0) {  // emitter: its emission (main.cpp:411-412 with throughput 1)
                double* fb = P.fb + 3 * (size_t)px[j];
                unsafeAtomicAdd(fb + 0, P.S.light_rad[3 * kind + 0] * P.inv_spp);
                unsafeAtomicAdd(fb + 1, P.S.light_rad[3 * kind + 1] * P.inv_spp);
                unsafeAtomicAdd(fb + 2, P.S.light_rad[3 * kind + 2] * P.inv_spp);
            } else if (kind == -1) {  // shading node; RR dim 0 (MIS / BRDF), shade() draws it later
                want = (P.mode == MCPT_MODE_SHADE || P.mode == MCPT_MODE_SHADE_AREA) ||
                       !(counter_u(counter_key(P.seed, (uint64_t)px[j], (uint64_t)sm[j], 1), 0) > MCPT_P_RR);
            }
        }
        wm[j] = __ballot(want);
        if (lane == 0) s_w[j][wid] = (unsigned)__popcll(wm[j]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned run = 0;
        for (int j = 0; j < kRootsPT; j++)
            for (int w = 0; w < 4; w++) {
                const unsigned c = s_w[j][w];
                s_w[j][w] = run;
                run += c;
            }
        s_base = run ? atomicAdd(q.count, run) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRootsPT; j++) {
        if (!((wm[j] >> lane) & 1)) continue;
        const unsigned rk = __builtin_amdgcn_mbcnt_hi((unsigned)(wm[j] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)wm[j], 0u));
        const size_t slot = (size_t)s_base + s_w[j][wid] + rk;
        if (slot >= (size_t)q.cap) {
            atomicOr((unsigned long long*)(P.stats + 4), 1ull);
            continue;
        }
        if (!lite) {
            const double* t = rt.pnw + 9 * (size_t)px[j];
            st3(q.p, q.cap, slot, mk3(t[0], t[1], t[2]));
            st3(q.n, q.cap, slot, mk3(t[3], t[4], t[5]));
            st3(q.wo, q.cap, slot, mk3(t[6], t[7], t[8]));
            st3(q.tp, q.cap, slot, mk3(1, 1, 1));
        }
        q.f[slot] = hit_f[px[j]];
        q.pixel[slot] = px[j];
        q.sample[slot] = sm[j];
        q.node[slot] = 1;
        q.par[slot] = -1;
    }
}

// moves nodes [sb, sb + m) of src to [db, db + m) of dst (every field a generation carries into the
// next: point, normal, wo, throughput, facet, pixel, sample, node id) -- the spill stack's push and
// pop when a generation is larger than its children buffer can take (render_on_device)
__global__ __launch_bounds__(256) void k_queue_move(Queue src, int sb, Queue dst, int db, int m) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const size_t s = (size_t)sb + k, d = (size_t)db + k;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        dst.p[idx3(dst.cap, d, c)] = src.p[idx3(src.cap, s, c)];
        dst.n[idx3(dst.cap, d, c)] = src.n[idx3(src.cap, s, c)];
        dst.wo[idx3(dst.cap, d, c)] = src.wo[idx3(src.cap, s, c)];
        dst.tp[idx3(dst.cap, d, c)] = src.tp[idx3(src.cap, s, c)];
    }
    dst.f[d] = src.f[s];
    dst.pixel[d] = src.pixel[s];
    dst.sample[d] = src.sample[s];
    dst.node[d] = src.node[s];
    dst.par[d] = src.par[s];
}

// root shading points of the pixels whose primary hit is a front-facing non-emitter (the nodes
// that reach the light prep at the root), compacted into q for the root-cache build
__global__ __launch_bounds__(256) void k_root_points(DScene S, CamFrame cam, const int* hit_f, const double* hit_tbg,
                                                     Queue q) {
    const int px = blockIdx.x * blockDim.x + threadIdx.x;
    const int npx = cam.W * cam.H;
    bool want = false;
    d3 p = mk3(0, 0, 0), N = mk3(0, 0, 0);
    if (px < npx) {
        const int f = hit_f[px];
        if (f >= 0 && S.tri_light[f] < 0) {
            node_point(S, f, hit_tbg[3 * px + 1], hit_tbg[3 * px + 2], &p, &N);
            want = !(dot(N, mul(cam_dir(cam, px / cam.W, px % cam.W), -1)) < 0);
        }
    }
    const int slot = block_append(q.count, want);
    if (want && slot < q.cap) {
        st3(q.p, q.cap, slot, p);
        st3(q.n, q.cap, slot, N);
        q.pixel[slot] = px;
    }
}

// Light prep for scenes with few light triangles (N_L <= kSmallNL, e.g. the 2-triangle Cornell
// light): lane per node, a sequential loop over the light table in index order -- exactly the
// oracle's loop (the reference's literal cull chain and weight, light_tri_stage), the sum in index
// order and the pick "first survivor whose running sum >= u * weights_sum" (last survivor on
// rounding): exact by construction, no ambiguity band needed.  A wave per node would leave 62 of 64
// lanes idle here.
constexpr int kSmallNL = 64;
__device__ inline unsigned long long wave_sum_u64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ inline int wave_sum_int(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
// adds a and b summed over the wave to ca / cb, one atomic each (every lane of the wave must call)
__device__ inline void wave_count2(unsigned long long* ca, unsigned a, unsigned long long* cb, unsigned b) {
    const unsigned long long sa = wave_sum_u64(a), sb = wave_sum_u64(b);
    if (__lane_id() == 0) {
        if (sa) atomicAdd(ca, sa);
        if (sb) atomicAdd(cb, sb);
    }
}
// Root-point cache of the small-table prep (k_prep_lane's scenes, N_L <= kSmallNL; the large tables'
// cache is PrepCache): a root's (x1, n) is its pixel's, so its literal running sums are a function of the
// pixel (main.cpp:563-572 re-traces the same primary ray for every sample).  Per pixel: the running sum
// after each light (-1 where the light does not survive), weights_sum and the last survivor; a root's
// pick is then a search of its pixel's row -- the same comparisons on the same values as k_prep_lane's
// pick loop, so weights_sum and the pick are bit-identical.
struct SmallCache {
    double* cum;   // [npx][NL]
    double* wsum;  // [npx]
    int* last;     // [npx]
};
// kKeep > 0 (N_L <= kKeep): the running sums of pass 1 stay in registers and the pick searches them,
// instead of re-running the literal chain (six acos per light) up to the picked light.  kBuild: the
// nodes are root points (qpixel = their pixels); their rows go to the SmallCache, no pick.
template <int kKeep, bool kBuild>
__global__ __launch_bounds__(256) void k_prep_lane(DScene S, uint64_t seed, int n, const double* __restrict__ qp,
                                                   const double* __restrict__ qn, int qs, const int* __restrict__ qpixel,
                                                   const int* __restrict__ qsample, const uint64_t* __restrict__ qnode,
                                                   const double* __restrict__ u_override, double* __restrict__ wsum_out,
                                                   int* __restrict__ pick_out, int* __restrict__ count_out,
                                                   unsigned long long* stats, SmallCache C) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < n;
    unsigned long long surv = 0, cand = 0, c1 = 0;
    if (active) {
        const d3 x1 = ld3(qp, qs, i);
        const d3 nn = ld3(qn, qs, i);
        // the reference's literal chain (light_tri_stage: Mylight.cpp:335-413, six acos), so weights,
        // weights_sum (summed in index order below) and the pick are the reference's bit for bit
        auto eval = [&](int li, bool* ok) -> double {
            const double2* w = S.lt_w + 5 * li;
            const double2 a = w[0], b = w[1], c = w[2], d = w[3], e = w[4];
            const d3 p0 = mk3(a.x, a.y, b.x), p1 = mk3(b.y, c.x, c.y), p2 = mk3(d.x, d.y, e.x);
            const double4 ln = S.lt_n[li];
            SphTri o;
            const int st = light_tri_stage(p0, p1, p2, mk3(ln.x, ln.y, ln.z), S.light_sum[li], x1, nn, &o);
            *ok = st == 0;
            return st == 0 ? o.w : (double)st;  // culled: 1 or 2 = the cheap stage, 3 = the full stage
        };
        double* row = kBuild ? C.cum + (size_t)qpixel[i] * S.NL : nullptr;
        double cw[kKeep > 0 ? kKeep : 1];  // running sum after light li, -1 if it does not survive
        double wsum = 0;
        int last = -1;
        auto visit = [&](int li) {
            bool ok;
            const double r = eval(li, &ok);
            if (ok) {
                wsum += r;
                surv++;
                last = li;
            }
            const bool culled = !ok && (r == 1.0 || r == 2.0);
            c1 += culled && r == 1.0;
            cand += !culled;
            return ok ? wsum : -1.0;
        };
        if (kKeep > 0) {
#pragma unroll
            for (int li = 0; li < kKeep; li++) cw[li] = li < S.NL ? visit(li) : -1.0;
        } else {
            for (int li = 0; li < S.NL; li++) {
                const double c = visit(li);
                if (kBuild) row[li] = c;
            }
        }
        if (kBuild) {
            if (kKeep > 0) {
#pragma unroll
                for (int li = 0; li < kKeep; li++)
                    if (li < S.NL) row[li] = cw[li];
            }
            C.wsum[qpixel[i]] = wsum;
            C.last[qpixel[i]] = last;
        } else {
            int pick = -1;
            if (!(fabs(wsum) < MCPT_EPS)) {
                const double u = u_override ? u_override[i]
                                            : counter_u(counter_key(seed, (uint64_t)qpixel[i], (uint64_t)qsample[i], qnode[i]), 1);
                const double target = u * wsum;
                if (kKeep > 0) {  // first survivor whose running sum reaches the target (culled: -1 never does)
#pragma unroll
                    for (int li = kKeep - 1; li >= 0; li--)
                        if (cw[li] >= target) pick = li;
                } else {
                    double cum = 0;
                    for (int li = 0; li < S.NL; li++) {
                        bool ok;
                        const double r = eval(li, &ok);
                        if (!ok) continue;
                        cum += r;
                        if (cum >= target) {
                            pick = li;
                            break;
                        }
                    }
                }
                if (pick < 0) pick = last;
            }
            wsum_out[i] = wsum;
            pick_out[i] = pick;
            if (count_out) count_out[i] = (int)surv;
        }
    }
    if (stats) {  // launch-uniform: one atomic per counter per workgroup (per-wave atomics on one word
                  // serialise at ~88 per us)
        __shared__ unsigned long long s_st[4][4];  // [counter][wave], 256 threads
        const int wid = threadIdx.x >> 6;
        const unsigned long long ss = wave_sum_u64(surv), cs = wave_sum_u64(cand), c1s = wave_sum_u64(c1);
        const unsigned long long full = __popcll(__ballot(active));
        if (lane_id() == 0) s_st[0][wid] = ss, s_st[1][wid] = cs, s_st[2][wid] = c1s, s_st[3][wid] = full;
        __syncthreads();
        if (threadIdx.x < 4) {
            const unsigned long long t = s_st[threadIdx.x][0] + s_st[threadIdx.x][1] + s_st[threadIdx.x][2] + s_st[threadIdx.x][3];
            constexpr int kIdx[4] = {1, 5, 6, 7};
            if (t) atomicAdd(stats + kIdx[threadIdx.x], t);
        }
    }
}

// cached roots of a small-table scene (SmallCache): the pick searches the pixel's row of running sums
// (lane per root); weights_sum is the cached one
__global__ __launch_bounds__(256) void k_prep_lane_pick(DScene S, uint64_t seed, int n, const int* __restrict__ qpixel,
                                                        const int* __restrict__ qsample, const uint64_t* __restrict__ qnode,
                                                        double* __restrict__ wsum_out, int* __restrict__ pick_out,
                                                        unsigned long long* stats, SmallCache C) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < n;
    if (active) {
        const int px = qpixel[i];
        const double wsum = C.wsum[px];
        int pick = -1;
        if (!(fabs(wsum) < MCPT_EPS)) {
            const double target = counter_u(counter_key(seed, (uint64_t)px, (uint64_t)qsample[i], qnode[i]), 1) * wsum;
            const double* row = C.cum + (size_t)px * S.NL;
            for (int li = 0; li < S.NL; li++)
                if (row[li] >= target) {
                    pick = li;
                    break;
                }
            if (pick < 0) pick = C.last[px];
        }
        wsum_out[i] = wsum;
        pick_out[i] = pick;
    }
    if (stats) {
        const unsigned long long c = __popcll(__ballot(active));
        if (lane_id() == 0 && c) atomicAdd(stats + 0, c);
    }
}

// Light prep, one wave per node (Mylight.cpp:322-422).
//  pass 1: chunks of 64 light triangles run the cheap cull stages (light side, tangent plane);
//          candidates are compacted into a per-wave LDS queue, and every 64 queued candidates are
//          evaluated densely (full stage, fp64) as one batch: wave inclusive scan -> batch total.
//          weights_sum = sequential sum of the batch totals (index order is preserved).
//  pass 2: the inverse-CDF pick (first survivor whose cumulative weight >= u*weights_sum, u = dim
//          1) re-runs the cheap stages to rebuild only the batch that holds the target and
//          re-evaluates those <= 64 candidates.
// u_override / count_out: test entry (mcpt_light_prep).
// Inclusive wave64 prefix sum of doubles with DPP (GFX9 row_shr / row_bcast; no LDS traffic).
// Out-of-range sources read 0 (update_dpp's `old` operand), so every step is a plain add.
template <int kCtrl, int kRowMask>
__device__ inline double dpp_shift(double v) {
    const unsigned long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, kCtrl, kRowMask, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), kCtrl, kRowMask, 0xf, false);
    return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}
// row_shr with bound_ctrl: every lane is written (source or 0), so no `old` register is needed
template <int kCtrl>
__device__ inline double dpp_shr(double v) {
    const unsigned long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, kCtrl, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), kCtrl, 0xf, 0xf, true);
    return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ inline double wave_incl_scan(double v, int lane) {
    (void)lane;
    v += dpp_shr<0x111>(v);  // row_shr:1
    v += dpp_shr<0x112>(v);  // row_shr:2
    v += dpp_shr<0x114>(v);  // row_shr:4
    v += dpp_shr<0x118>(v);  // row_shr:8
    v += dpp_shift<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
    v += dpp_shift<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
    return v;
}

__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Totals of four 64-lane batches a, b, c, d (gfx950 permlane swaps + one row reduction instead of
// four full wave scans): returns, in lanes 15 / 31 / 47 / 63, the totals of a / b / c / d.
//   permlane32_swap(a, c), (b, d): lanes 0-31 of a + c hold a's pair sums (lane l, l+32), lanes
//   32-63 c's; likewise b + d.  permlane16_swap(p, q) then gathers row r (16 lanes) of p + q =
//   batch r's sums of four lanes; a row_shr 1/2/4/8 scan leaves each row's total in its lane 15.
__device__ inline void swap32(double& x, double& y) {
    const unsigned long long bx = __double_as_longlong(x), by = __double_as_longlong(y);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)bx, (unsigned)by, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(bx >> 32), (unsigned)(by >> 32), false, false);
    x = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
    y = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}
__device__ inline void swap16(double& x, double& y) {
    const unsigned long long bx = __double_as_longlong(x), by = __double_as_longlong(y);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)bx, (unsigned)by, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(bx >> 32), (unsigned)(by >> 32), false, false);
    x = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
    y = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}
__device__ inline double batch_totals4(double a, double b, double c, double d) {
    swap32(a, c);
    swap32(b, d);
    double p = a + c, q = b + d;
    swap16(p, q);
    double r = p + q;
    r += dpp_shr<0x111>(r);  // row_shr:1
    r += dpp_shr<0x112>(r);  // row_shr:2
    r += dpp_shr<0x114>(r);  // row_shr:4
    r += dpp_shr<0x118>(r);  // row_shr:8
    return r;
}

// ---- exact pick: the ambiguity band ------------------------------------------
// The GPU's weights differ from the reference's (oracle's) by rounding, so a pick whose target u W
// lies within that difference of a cumulative-weight boundary may differ.  Each pick therefore
// computes its margin -- the distance of the target from the two boundaries around the picked
// candidate -- and compares it with a band that bounds the prefix sums' difference (calibrated with
// tools/prep_error_study.py on 60 000 shading points and tools/band_margin_study.py on the stress
// scenes: the band is >= 2x the largest difference measured anywhere, sliver scene included): kappa u sqrt(sum_c n_c m_c^2) over the 64-light chunks (m_c = S_c + K_c (|x1 - c_c| + R_c),
// the chunk's largest sum L and sum L / shortest edge, scaled by the distance bound) + the flagged
// slivers' own terms + the GPU's summation-order rounding.  A node inside the band goes to the exact
// fallback (k_prep_exact: the reference's literal formulas, summed in the reference's order).
#ifndef MCPT_BAND_KAPPA
#define MCPT_BAND_KAPPA 8.0
#endif
#ifndef MCPT_BAND_SLIVER
#define MCPT_BAND_SLIVER 0.5  // round 6: 0.25 with tau 1000 was exceeded 1.5x on the sliver scene
#endif
constexpr double kU53 = 0x1.0p-53;
constexpr int kExactHead = 16;  // exact list: [0] count, entries from [kExactHead]
// rounding of the GPU's own sums (batch trees instead of a sequential sum) and of its formulas
__device__ inline double band_round(int ncand, double wsum) { return (2.0 * ncand + 4096.0) * kU53 * fabs(wsum); }
// the slivers' terms: sum over flagged candidates of lsum2 sqrt(2x)/num (sliver_term), to band units
__device__ inline double band_sliver(double acc) { return MCPT_BAND_SLIVER * 0.5 * kU53 * acc; }
// upper bound of band_base for a node with ncand candidates (sum of n_c = ncand; every chunk's m_c within
// the scene sphere's and the table's maxima)
__device__ inline double band_base_upper(const DScene& S, d3 x1, int ncand) {
    const double dx = x1.x - S.band_ctr[0], dy = x1.y - S.band_ctr[1], dz = x1.z - S.band_ctr[2];
    const double m = S.band_S + S.band_K * (sqrt(dx * dx + dy * dy + dz * dz) + S.band_R);
    return MCPT_BAND_KAPPA * kU53 * sqrt((double)ncand) * m * 1.0001;
}
// the per-chunk term of the band for one node (this lane): n_c = set bits of the node's candidate word c
// (mrow), or 64 without words
__device__ inline double band_base(const DScene& S, d3 x1, const uint64_t* mrow, int nchunks) {
    double b2 = 0;
    for (int c = 0; c < nchunks; c++) {
        const int nc = mrow ? __popcll(mrow[c]) : 64;
        if (nc == 0) continue;
        const float4 sp = S.chunk_sph[c];
        const float2 sk = S.chunk_sk[c];
        const double dx = x1.x - sp.x, dy = x1.y - sp.y, dz = x1.z - sp.z;
        const double m = (double)sk.x + (double)sk.y * (sqrt(dx * dx + dy * dy + dz * dz) + (double)sp.w);
        b2 += (double)nc * m * m;
    }
    return MCPT_BAND_KAPPA * kU53 * sqrt(b2) * 1.0001;
}
// distance of target = u W from the boundaries around the picked candidate (lane pl of the batch whose
// exclusive prefix is base; sc = this lane's inclusive in-batch scan): below, the cumulative weight
// before it (none if that is 0: no earlier weight); above, the cumulative weight including it
// (pl is wave-uniform -- it comes from a ballot -- so the two values are read with v_readlane into
// SGPRs rather than an LDS permute)
__device__ inline double readlane_f64(double v, int l) {  // l: wave-uniform
    l = __builtin_amdgcn_readfirstlane(l);
    const unsigned long long b = __double_as_longlong(v);
    return __longlong_as_double(((long long)(unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l) << 32) |
                                (unsigned)__builtin_amdgcn_readlane((int)b, l));
}
__device__ inline double pick_margin(double base, double sc, int pl, double target) {
    const int l = __builtin_amdgcn_readfirstlane(pl);
    const double c_hi = base + readlane_f64(sc, l);
    const double c_lo = l > 0 ? base + readlane_f64(sc, l - 1) : base;
    const double m_lo = c_lo == 0.0 ? INFINITY : target - c_lo;
    return fmin(m_lo, c_hi - target);
}
// the room a pick leaves for the band: its margin, and the distance of weights_sum from the empty-set
// threshold 1e-8 (Mylight.cpp:427); a pick is exact if its slack exceeds the band (NaN: not exact)
__device__ inline double pick_slack(double margin, double wsum) {
    const double s = fmin(margin, fabs(fabs(wsum) - MCPT_EPS));
    return s == s ? s : -INFINITY;
}
// one lane per node: a slack the whole-table bound of the per-chunk term cannot clear is stored and the
// node listed (maybe: count in [0], entries from kExactHead) for k_prep_band's per-chunk test
__device__ inline void band_candidate(const DScene& S, double* slack, int* maybe, int idx, double sl, d3 x1, int ncand) {
    if (!(sl > band_base_upper(S, x1, ncand))) {
        slack[idx] = sl;
        const int q = atomicAdd(maybe, 1);
        maybe[kExactHead + q] = idx;
    }
}

struct PrepLight {
    d3 p0, p1, p2, nl;
    double lsum2;  // 2 RadianceRGB::sum()
};
__device__ inline PrepLight load_light(const DScene& S, int li) {
    const double4 ln = S.lt_n[li];
    return PrepLight{f3(S.lt_v[3 * li]), f3(S.lt_v[3 * li + 1]), f3(S.lt_v[3 * li + 2]), mk3(ln.x, ln.y, ln.z), 2.0 * ln.w};
}
// The cheap stages evaluated in fp32 with a rigorous rounding-error bound `err`, falling back to
// the exact fp64 reference arithmetic only when a value lies within err of the 1e-8 threshold:
// the decisions are exactly those of Mylight.cpp:340-357.  Light-side test: culled iff
// nl.(x1-p0) < 1e-8; tangent-plane test: culled iff n.(pi-x1) < 1e-8 for all three vertices.
// lt_v[3l+k].w holds float(nl[k]).
struct NodeF {
    float x, y, z, nx, ny, nz, err;
};
__device__ inline NodeF node_f(d3 x1, d3 n, float scene_bound) {
    const float X = fmaxf(fmaxf(fabsf((float)x1.x), fabsf((float)x1.y)), fabsf((float)x1.z));
    // |t_f32 - t| <= 15 u (X + P) for u = 2^-24 (DESIGN.md "light prep numerics"); 2^-19 (X+P) bounds it
    return NodeF{(float)x1.x, (float)x1.y, (float)x1.z, (float)n.x, (float)n.y, (float)n.z,
                 0x1.0p-19f * (X + scene_bound) + 1e-30f};
}
__device__ inline int prep_stage_regs(const DScene& S, int li, float4 a, float4 b, float4 c, d3 x1, d3 n,
                                      const NodeF& nf) {
    if (li >= S.NL) return 3;
    constexpr float kEps = 1e-8f;
    const float s1 = fmaf(a.w, nf.x - a.x, fmaf(b.w, nf.y - a.y, c.w * (nf.z - a.z)));
    if (s1 < kEps - nf.err) return 1;
    const float t0 = fmaf(nf.nx, a.x - nf.x, fmaf(nf.ny, a.y - nf.y, nf.nz * (a.z - nf.z)));
    const float t1 = fmaf(nf.nx, b.x - nf.x, fmaf(nf.ny, b.y - nf.y, nf.nz * (b.z - nf.z)));
    const float t2 = fmaf(nf.nx, c.x - nf.x, fmaf(nf.ny, c.y - nf.y, nf.nz * (c.z - nf.z)));
    const float tm = fmaxf(fmaxf(t0, t1), t2);
    if (s1 > kEps + nf.err) {
        if (tm < kEps - nf.err) return 2;
        if (tm > kEps + nf.err) return 0;
    }
    const double4 ln = S.lt_n[li];  // ambiguous: exact reference arithmetic
    return light_cheap_stage(f3(a), f3(b), f3(c), mk3(ln.x, ln.y, ln.z), x1, n);
}
__device__ inline int prep_stage(const DScene& S, int li, d3 x1, d3 n, const NodeF& nf) {
    if (li >= S.NL) return 3;
    return prep_stage_regs(S, li, S.lt_v[3 * li], S.lt_v[3 * li + 1], S.lt_v[3 * li + 2], x1, n, nf);
}

constexpr int kPrepQueue = 128;  // per-wave candidate queue (ints)
#ifndef MCPT_LB_EXACT
#define MCPT_LB_EXACT 4  // k_prep_exact: 4 waves/SIMD (128 VGPRs)
#endif
#ifndef MCPT_EXACT_DEFER
#define MCPT_EXACT_DEFER 1  // k_prep_exact: a root whose pixel another wave of the launch computes waits for a follow-up launch
#endif
#ifndef MCPT_PREP_GRAB
#define MCPT_PREP_GRAB 8  // A/B (profiles/round3_ab_launch_params.txt): 4 -> 8 lowers the prep launch 20.65 -> 20.37-20.52 ms
#endif
constexpr int kPrepGrab = MCPT_PREP_GRAB;  // nodes a wave takes per work-counter atomic

__global__ __launch_bounds__(256) void k_prep(DScene S, uint64_t seed, int n, const double* __restrict__ qp,
                                              const double* __restrict__ qn, int qs, const int* __restrict__ qpixel,
                                              const int* __restrict__ qsample, const uint64_t* __restrict__ qnode,
                                              const double* __restrict__ u_override, double* __restrict__ wsum_out,
                                              int* __restrict__ pick_out, int* __restrict__ count_out,
                                              unsigned long long* stats, int nchunks, unsigned* __restrict__ work,
                                              double* __restrict__ slack, int exact_off, int exact_counts,
                                              int* __restrict__ maybe) {
    extern __shared__ double prep_lds[];
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
    // per wave: [nchunks doubles batch totals][kPrepQueue ints]
    double* bt = prep_lds + (size_t)wib * (nchunks + kPrepQueue / 2);
    int* q = reinterpret_cast<int*>(bt + nchunks);
    const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    unsigned long long surv_acc = 0, cand_acc = 0, c1_acc = 0;
    int grab = 0, left = 0;
    while (true) {
        // dynamic distribution: a wave grabs kPrepGrab nodes per atomic (node costs vary ~10x)
        if (left == 0) {
            unsigned b = 0;
            if (lane == 0) b = atomicAdd(work, (unsigned)kPrepGrab);
            grab = __shfl((int)b, 0);
            left = kPrepGrab;
        }
        const int node = grab++;
        left--;
        if (node >= n) break;
        const d3 x1 = ld3(qp, qs, node);
        const d3 nn = ld3(qn, qs, node);
        const NodeF nf = node_f(x1, nn, S.light_bound);
        int qcnt = 0, nb = 0, survivors = 0, candidates = 0, culled1 = 0;
        double sacc = 0;  // flagged slivers' band terms (exact pick)
        bool degen = false;
        // ---- pass 1 ----
        for (int c = 0; c < nchunks; c++) {
            const int li = c * 64 + lane;
            const int stage = prep_stage(S, li, x1, nn, nf);
            const bool cand = stage == 0;
            const uint64_t m = __ballot(cand);
            if (cand) q[qcnt + __popcll(m & lt_mask)] = li;
            qcnt += __popcll(m);
            candidates += __popcll(m);
            culled1 += __popcll(__ballot(stage == 1));
            const bool last = (c == nchunks - 1);
            while (qcnt >= 64 || (last && qcnt > 0)) {
                wave_lds_sync();
                const bool act = lane < qcnt;
                const int lj = act ? q[lane] : 0;
                double w = 0;
                bool ok = false;
                if (act) {
                    const PrepLight L = load_light(S, lj);
                    const WeightBx r = light_weight_bx(L.p0, L.p1, L.p2, L.lsum2, x1);
                    ok = r.ok;
                    w = r.w;
                    if (ok && r.sliver) {
                        const double t = sliver_term(r.num, r.den) * L.lsum2;
                        sacc += t;
                        degen |= 2.0 * w < 64.0 * kU53 * t;
                    }
                    degen |= !ok;
                }
                const double sc = wave_incl_scan(w, lane);
                survivors += __popcll(__ballot(ok));
                if (lane == 63) bt[nb] = sc;
                nb++;
                const int rem = qcnt > 64 ? qcnt - 64 : 0;
                const int mv = lane < rem ? q[64 + lane] : 0;
                wave_lds_sync();
                if (lane < rem) q[lane] = mv;
                qcnt = rem;
            }
        }
        wave_lds_sync();
        double wsum = 0;
        for (int b = 0; b < nb; b++) wsum += bt[b];
        // ---- pass 2: inverse-CDF pick ----
        int pick = -1;
        double margin = INFINITY;
        if (!(fabs(wsum) < MCPT_EPS)) {
            double u;
            if (u_override) u = u_override[node];
            else u = counter_u(counter_key(seed, (uint64_t)qpixel[node], (uint64_t)qsample[node], qnode[node]), 1);
            const double target = u * wsum;
            int kb = -1, lastpos = -1;
            double cum = 0, base = 0;
            for (int b = 0; b < nb; b++) {
                const double nxt = cum + bt[b];
                if (bt[b] > 0) lastpos = b;
                if (kb < 0 && nxt >= target && bt[b] > 0) {
                    kb = b;
                    base = cum;
                }
                cum = nxt;
            }
            if (kb < 0) {  // rounding: fall back to the last batch with weight
                kb = lastpos;
                base = 0;
                for (int b = 0; b < kb; b++) base += bt[b];
            }
            // rebuild the candidate queue up to batch kb
            qcnt = 0;
            int formed = 0;
            for (int c = 0; c < nchunks; c++) {
                const int li = c * 64 + lane;
                const bool cand = prep_stage(S, li, x1, nn, nf) == 0;
                const uint64_t m = __ballot(cand);
                if (cand) q[qcnt + __popcll(m & lt_mask)] = li;
                qcnt += __popcll(m);
                if (qcnt >= 64 || (c == nchunks - 1 && qcnt > 0)) {
                    if (formed == kb) break;
                    const int rem = qcnt > 64 ? qcnt - 64 : 0;
                    wave_lds_sync();
                    const int mv = lane < rem ? q[64 + lane] : 0;
                    wave_lds_sync();
                    if (lane < rem) q[lane] = mv;
                    qcnt = rem;
                    formed++;
                    if (c == nchunks - 1 && qcnt > 0 && formed == kb) break;
                }
            }
            wave_lds_sync();
            const bool act = lane < qcnt && lane < 64;
            const int lj = act ? q[lane] : 0;
            double w = 0;
            bool ok = false;
            if (act) {
                const PrepLight L = load_light(S, lj);
                ok = light_weight(L.p0, L.p1, L.p2, L.lsum2, x1, &w);
                if (!ok) w = 0;
            }
            const double sc = wave_incl_scan(w, lane);
            const uint64_t candm = __ballot(ok && (base + sc >= target));
            const uint64_t okm = __ballot(ok);
            int pl = -1;
            if (candm) pl = __ffsll((unsigned long long)candm) - 1;
            else if (okm) pl = 63 - __clzll((long long)okm);
            if (pl >= 0) {
                pick = __shfl(lj, pl);
                margin = pick_margin(base, sc, pl, target);
            }
        }
        if (lane == 0) {
            wsum_out[node] = wsum;
            pick_out[node] = pick;
            if (count_out) count_out[node] = survivors;
        }
        if (slack) {  // exact pick (k_prep_band: no candidate words here, every chunk counts as full)
            double sl = pick_slack(margin, wsum) - (band_sliver(__shfl(wave_incl_scan(sacc, lane), 63)) +
                                                    band_round(candidates, wsum));
            if (exact_counts && __ballot(degen)) sl = -INFINITY;
            if (lane == 0) band_candidate(S, slack, maybe, exact_off + node, sl, x1, candidates);
        }
        surv_acc += survivors;
        cand_acc += candidates;
        c1_acc += culled1;
        wave_lds_sync();
    }
    if (lane == 0 && stats) {
        if (surv_acc) atomicAdd(stats + 1, surv_acc);
        if (cand_acc) atomicAdd(stats + 5, cand_acc);
        if (c1_acc) atomicAdd(stats + 6, c1_acc);
    }
}

// Cheap stages of the light prep in packed fp32 (v_pk_fma_f32): lt_pk[3l..3l+2] = X, Y, Z with
// X = (p0.x, p1.x, p2.x, nl.x) etc. and lt_d[l] = float(nl.p0), so that (t0, t1) = n.(p0, p1) - n.x1
// and (t2, s1) = (n.p2 - n.x1, nl.x1 - nl.p0) are four packed FMA chains; n.x1 is rounded once per
// node.  The error bound of node_f still holds (DESIGN.md "light prep numerics").  The sure
// outcomes are predicates; the ambiguous lanes (a value within err of the 1e-8 threshold) take one
// rarely-taken branch into the exact fp64 reference arithmetic.
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ inline int prep_stage_pk_bf(const DScene& S, int li, float4 X, float4 Y, float4 Z, float dl, v2f nx2,
                                       v2f ny2, v2f nz2, v2f nxs, v2f nys, v2f nzs, float cn, d3 x1, d3 n, float err) {
    constexpr float kEps = 1e-8f;
    const v2f tab = __builtin_elementwise_fma(nx2, v2f{X.x, X.y}, __builtin_elementwise_fma(ny2, v2f{Y.x, Y.y}, nz2 * v2f{Z.x, Z.y})) - v2f{cn, cn};
    const v2f tcs = __builtin_elementwise_fma(nxs, v2f{X.z, X.w}, __builtin_elementwise_fma(nys, v2f{Y.z, Y.w}, nzs * v2f{Z.z, Z.w})) - v2f{cn, dl};
    const float s1 = tcs.y;
    const float tm = fmaxf(fmaxf(tab.x, tab.y), tcs.x);
    const float lo = kEps - err, hi = kEps + err;
    const bool s1_out = s1 < lo, s1_in = s1 > hi, t_out = tm < lo, t_in = tm > hi;
    int stage = li >= S.NL ? 3 : s1_out ? 1 : (s1_in && t_out) ? 2 : (s1_in && t_in) ? 0 : -1;
    if (stage < 0) {
        const double4 ln = S.lt_n[li];  // ambiguous: exact reference arithmetic
        stage = light_cheap_stage(mk3(X.x, Y.x, Z.x), mk3(X.y, Y.y, Z.y), mk3(X.z, Y.z, Z.z), mk3(ln.x, ln.y, ln.z), x1, n);
    }
    return stage;
}

// Light-table loads through buffer descriptors (32-bit offsets, immediate offsets per vertex row,
// hardware bounds check returning 0 past the table, so no index clamp).
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
constexpr int kBufFlags = 0x00020000;  // gfx9 raw buffer descriptor word 3
__device__ inline float4 u4f(v4u v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ inline double u2d(unsigned lo, unsigned hi) {
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// structured (idxen) buffer load: address = base + vindex * stride (from the descriptor) + offset,
// so a light index from the candidate list needs no VALU address arithmetic (hipcc has no builtin
// for the struct form; this binds the LLVM intrinsic by name)
__device__ v4u struct_load_b128(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.ptr.buffer.load.v4i32");
constexpr int kLtW = 80;  // bytes per light record in lt_w (the descriptor's stride)
// the light-record descriptor for k_prep_pk2 / prep_select: stride kLtW, the whole padded table
// plus the sentinel records (lt_w has nl_pad + kSentinelPad records)
constexpr int kSentinelPad = 64;
__device__ inline __amdgpu_buffer_rsrc_t light_record_rsrc(const DScene& S, int ngroups4) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)S.lt_w, kLtW, (ngroups4 * 256 + kSentinelPad) * kLtW, kBufFlags);
}
__device__ inline double prep_weight_buf(__amdgpu_buffer_rsrc_t rw, int li, d3 x1, bool* ok) {
    const v4u a = struct_load_b128(rw, li, 0, 0, 0);
    const v4u b = struct_load_b128(rw, li, 16, 0, 0);
    const v4u c = struct_load_b128(rw, li, 32, 0, 0);
    const v4u d = struct_load_b128(rw, li, 48, 0, 0);
    const v4u e = struct_load_b128(rw, li, 64, 0, 0);
    return light_weight_bf<true>(mk3(u2d(a.x, a.y), u2d(a.z, a.w), u2d(b.x, b.y)),
                           mk3(u2d(b.z, b.w), u2d(c.x, c.y), u2d(c.z, c.w)),
                           mk3(u2d(d.x, d.y), u2d(d.z, d.w), u2d(e.x, e.y)), u2d(e.z, e.w), x1, ok);
}
// prep_weight_buf with the exact-pick bookkeeping (light_weight_bx); *lsum2 = the record's 2 sum L
__device__ inline WeightBx prep_weight_buf_bx(__amdgpu_buffer_rsrc_t rw, int li, d3 x1, double* lsum2) {
    const v4u a = struct_load_b128(rw, li, 0, 0, 0);
    const v4u b = struct_load_b128(rw, li, 16, 0, 0);
    const v4u c = struct_load_b128(rw, li, 32, 0, 0);
    const v4u d = struct_load_b128(rw, li, 48, 0, 0);
    const v4u e = struct_load_b128(rw, li, 64, 0, 0);
    *lsum2 = u2d(e.z, e.w);
    return light_weight_bx<true>(mk3(u2d(a.x, a.y), u2d(a.z, a.w), u2d(b.x, b.y)),
                                 mk3(u2d(b.z, b.w), u2d(c.x, c.y), u2d(c.z, c.w)),
                                 mk3(u2d(d.x, d.y), u2d(d.z, d.w), u2d(e.x, e.y)), u2d(e.z, e.w), x1);
}
// fp32 records (MCPT_RENDER_PRECISION_FP32, LightF32): 10 floats at a 64-B stride (a record never
// straddles a cache line), the same padding and sentinels as lt_w
constexpr int kLtF = 64;
__device__ inline __amdgpu_buffer_rsrc_t light_record_f32_rsrc(const DScene& S, int ngroups4) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)S.lt_f, kLtF, (ngroups4 * 256 + kSentinelPad) * kLtF, kBufFlags);
}
__device__ v2u struct_load_b64(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.ptr.buffer.load.v2i32");
__device__ inline LightF32 load_light_f32(__amdgpu_buffer_rsrc_t rf, int li) {
    const v4u a = struct_load_b128(rf, li, 0, 0, 0);
    const v4u b = struct_load_b128(rf, li, 16, 0, 0);
    const v2u c = struct_load_b64(rf, li, 32, 0, 0);
    return LightF32{__builtin_bit_cast(v4f_t, a), __builtin_bit_cast(v4f_t, b), __builtin_bit_cast(v2f_t, c)};
}
// x1 split into float hi + lo per component (wave-uniform), for light_weight_f32x2
struct NodeF32 {
    v2f_t xh, yh, zh, xl, yl, zl;
};
__device__ inline NodeF32 node_f32(d3 x1) {
    const float hx = (float)x1.x, hy = (float)x1.y, hz = (float)x1.z;
    const float lx = (float)(x1.x - hx), ly = (float)(x1.y - hy), lz = (float)(x1.z - hz);
    return NodeF32{v2f_t{hx, hx}, v2f_t{hy, hy}, v2f_t{hz, hz}, v2f_t{lx, lx}, v2f_t{ly, ly}, v2f_t{lz, lz}};
}
__device__ inline void prep_weight_f32x2(__amdgpu_buffer_rsrc_t rf, int li, int lj, const NodeF32& X, double* w0,
                                         double* w1, bool* ok0, bool* ok1) {
    light_weight_f32x2(load_light_f32(rf, li), load_light_f32(rf, lj), X.xh, X.yh, X.zh, X.xl, X.yl, X.zl, w0, w1, ok0,
                       ok1);
}

__device__ inline int lane_rank(uint64_t m) {  // set bits of m below this lane
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// lst[base + rank] = idx for the lanes whose bit is set in m (rank = set bits of m below the lane),
// with exec = m for the store instead of a per-lane bit test: 2 v_mbcnt + 1 v_lshl_add per word.
// exec is restored before the block ends; the LDS store is ordered with the kernel's other LDS
// accesses (in-order per wave; the caller's wave_lds_sync follows the rebuild).
__device__ inline void append_masked(uint64_t m, unsigned lo, unsigned hi, unsigned base_bytes, unsigned idx) {
    uint64_t saved;
    unsigned t;
    asm volatile(
        "s_and_saveexec_b64 %[sv], %[m]\n\t"
        "v_mbcnt_lo_u32_b32 %[t], %[lo], 0\n\t"
        "v_mbcnt_hi_u32_b32 %[t], %[hi], %[t]\n\t"
        "v_lshl_add_u32 %[t], %[t], 1, %[b]\n\t"
        "ds_write_b16 %[t], %[x]\n\t"
        "s_mov_b64 exec, %[sv]"
        : [sv] "=&s"(saved), [t] "=&v"(t)
        : [m] "s"(m), [lo] "s"(lo), [hi] "s"(hi), [b] "s"(base_bytes), [x] "v"(idx)
        : "memory", "scc");  // s_and_saveexec writes SCC
}

// Root-point cache.  Every camera sample of a pixel starts at the same shading point (the
// reference re-traces the identical primary ray per sample, main.cpp:572), so the light prep of a
// root node (x1, n) -- batch totals and candidate list -- is a function of the pixel alone; only the
// pick (u, dim 1) differs per sample.  A render call with >= 2 samples per pixel builds the cache
// once over the pixels (build = 1) and root nodes then take the pick-only path (use = 1): the same
// scan over the same batch totals and the same batch re-evaluation as the full path, so results
// are identical.
struct PrepCache {
    double* bt;           // [npx][nchunks] the batch totals' inclusive scan (raw totals when nb > 64)
    unsigned short* lst;  // [npx][lstride] candidate list (light indices, index order)
    double* w;            // [npx][lstride] in-batch inclusive prefix of the candidate weights (wave scan);
                          // a candidate the full stage culls: its prefix with the sign bit set
    int4* info;           // [npx] (nb, ncand, survivors, 0)
    int lstride;
    int build;            // this launch builds entries of pixel qpixel[node] (qpixel == nullptr: node)
    int use;              // host side: root nodes go to k_prep_pick
    // exact pick: the pick's slack -- its margin less the band's terms known here
    // (flagged slivers, summation rounding) -- is compared with the whole-table upper bound of the
    // band's per-chunk term right away (band_candidate); only a node it does not clear has its slack
    // stored (slack[exact_off + node]) and is listed for k_prep_band.  k_prep_pick holds the whole band
    // (cached) and lists an ambiguous root on the exact list directly.  null: no band (the opt-in fp32 precision, benches of
    // the prep alone).  exact_counts: -inf also for nodes whose survivor count may differ (a candidate
    // the full stage culls, a near-degenerate sliver) -- the mcpt_light_prep entry reports counts.
    double* slack;
    int exact_off;
    int exact_counts;
    int* maybe;  // nodes whose slack the whole-table bound cannot clear (band_candidate), for k_prep_band
    int* exact;  // k_prep_pick: roots inside the cached band go straight to the exact list
};

// inverse-CDF pick from the batch totals bt[0, nb) and candidate list lst (LDS or global): returns
// weights_sum and the picked light (-1 if weights_sum < eps) and the pick's margin (pick_margin; +inf
// without a pick).  u_of() gives dim 1 when needed.
template <bool kF32 = false, class U>
__device__ inline double prep_select(const double* bt, const unsigned short* lst, int nb, int ncand, int lane,
                                     __amdgpu_buffer_rsrc_t rw, d3 x1, U u_of, int* pick_out, double* margin_out) {
    double wsum = 0;
    int pick = -1;
    int kb = -1;
    double base = 0, target = 0;
    if (nb <= 64) {
        const double v = lane < nb ? bt[lane] : 0.0;
        const double cum = wave_incl_scan(v, lane);
        wsum = __shfl(cum, 63);
        if (!(fabs(wsum) < MCPT_EPS)) {
            target = u_of() * wsum;
            const uint64_t hitm = __ballot(cum >= target && v > 0);
            const uint64_t posm = __ballot(v > 0);
            kb = hitm ? __ffsll((unsigned long long)hitm) - 1 : 63 - __clzll((long long)posm);
            const double exc = __shfl_up(cum, 1);
            base = kb == 0 ? 0.0 : __shfl(exc, kb);
        }
    } else {  // more than 64 batches (N_L > 4096 with many candidates): sequential search
        for (int b = 0; b < nb; b++) wsum += bt[b];
        if (!(fabs(wsum) < MCPT_EPS)) {
            target = u_of() * wsum;
            int lastpos = -1;
            double cum = 0;
            for (int b = 0; b < nb; b++) {
                const double nxt = cum + bt[b];
                if (bt[b] > 0) lastpos = b;
                if (kb < 0 && nxt >= target && bt[b] > 0) {
                    kb = b;
                    base = cum;
                }
                cum = nxt;
            }
            if (kb < 0) {
                kb = lastpos;
                base = 0;
                for (int b = 0; b < kb; b++) base += bt[b];
            }
        }
    }
    double margin = INFINITY;
    if (kb >= 0) {
        const int k = 64 * kb + lane;
        const bool act = k < ncand;
        const int lj = act ? (int)lst[k] : 0;
        bool ok;
        double w;
        if (kF32) {  // the same packed evaluation as the batch (both halves this candidate)
            bool ok1;
            double w1;
            prep_weight_f32x2(rw, lj, lj, node_f32(x1), &w, &w1, &ok, &ok1);
        } else {
            w = prep_weight_buf(rw, lj, x1, &ok);
        }
        ok = ok && act;
        w = act ? w : 0.0;
        const double sc = wave_incl_scan(w, lane);
        const uint64_t candm = __ballot(ok && (base + sc >= target));
        const uint64_t okm = __ballot(ok);
        int pl = -1;
        if (candm) pl = __ffsll((unsigned long long)candm) - 1;
        else if (okm) pl = 63 - __clzll((long long)okm);
        if (pl >= 0) {
            pick = __shfl(lj, pl);
            margin = pick_margin(base, sc, pl, target);
        }
    }
    *pick_out = pick;
    *margin_out = margin;
    return wsum;
}

constexpr int kChunkUnroll = 2;
// candidate words, node-major: word (node, chunk) at node * mask_stride + chunk, the row padded to
// whole 64-B lines (zero words past nchunks), so k_prep_pk2 reads a node's words as s_load_dwordx16
// of whole lines (each line fetched once) and the cull writes them two chunks (16 B) at a time
constexpr int kMaskLine = 8;  // words per 64-B line
__host__ __device__ inline int mask_stride(int nchunks) { return (nchunks + kMaskLine - 1) / kMaskLine * kMaskLine; }
// chunk splits of k_prep_cull_lanes over blockIdx.y (more waves in flight to hide the table's
// scalar-load latency), each a whole number of bursts: a lane keeps kCullBurst words in registers
// and stores them back to back, so the node's 64-B line is written whole before L2 can evict it
// (stored a pair at a time, lines were written back partially: 707 instead of ~400 B per node).
// Same-box A/B (profiles/round2b_ab_cull_burst.txt): burst 2 / 4 splits 423.4, burst 4 428.1,
// burst 8 with 6 splits 429.2, burst 8 with 3 splits 424.5 Msamples/s.
#ifndef MCPT_CULL_BURST
#define MCPT_CULL_BURST 8
#endif
constexpr int kCullBurst = MCPT_CULL_BURST;  // candidate words a cull lane stores back to back (even, <= kMaskLine)
static_assert(kCullBurst % 2 == 0 && kMaskLine % kCullBurst == 0, "cull burst");
#ifndef MCPT_CULL_SPLITS
#define MCPT_CULL_SPLITS 6
#endif
inline int cull_splits(int nchunks) { return std::max(1, std::min(MCPT_CULL_SPLITS, nchunks / 4)); }
// Phase A with a lane per shading node and the light table in scalar registers: each light pair
// (LightPair, two s_load_dwordx16) is read once per 64 nodes from the scalar cache, and the two
// cheap stages of both lights run as 13 v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 with one
// scalar operand each -- no vector memory traffic at all in the light loop.  A lane shifts its
// candidate bit into a 32-bit word with one v_addc_co_u32 (carry-in = the wave's compare mask);
// after 32 lights v_bfrev puts light j at bit j, so the stored word per (node, chunk) is the same
// as k_prep_cull's.  Values within err of the 1e-8 threshold take the exact fp64 stage, so the
// decisions are the reference's (err as in node_f; the threshold is folded into d and cn).
// raw v_max3_f32 / v_min_f32 (the builtins canonicalise operands that came out of packed ops
// first; NaN handling is irrelevant here: a NaN light value never reaches the cull)
__device__ inline float max3_raw(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ inline float min_raw(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ inline float min_abs_raw(float a, float b) {
    float r;
    asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ inline float min3_abs_raw(float a, float b, float c) {  // min(a, |b|, |c|)
    float r;
    asm("v_min3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ inline unsigned shift_in(unsigned w, uint64_t carry) {
    unsigned r;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(w), "s"(carry));
    return r;
}

// Chunk classes of the tangent-plane test (Mylight.cpp:347-357) from the chunk's vertex sphere
// (chunk_sph: centre c, radius r rounded up): h = n . c - (n . x1 + 1e-8) in the same fp32 form as the
// cull's t (|c| <= light_bound, so its rounding error is within err too).  ABOVE: h - r > 4 err, so every
// vertex has t > err in fp32 and t > 0 exactly -- the plane test passes every light of the chunk without
// ambiguity and the candidate bit is the light-side test alone.  BELOW: h + r < -4 err -- every light is
// plane-culled exactly and in fp32, so the chunk's word is 0.  (4 err covers err for h, err for t and the
// rounding of h -+ r.)  Else STRADDLE: the full two-stage cull.
enum { kChunkStraddle = 0, kChunkAbove = 1, kChunkBelow = 2 };
__device__ inline unsigned chunk_class(float nx, float ny, float nz, float ncn, float err, float4 sp) {
    const float h = fmaf(nx, sp.x, fmaf(ny, sp.y, fmaf(nz, sp.z, ncn)));
    const float m = 4.0f * err;
    return h - sp.w > m ? kChunkAbove : h + sp.w < -m ? kChunkBelow : kChunkStraddle;
}

// the two cheap stages of light pair T (lights A, B) for this lane's node, threshold folded in:
// s = nl . x1 - (nl . p0 + 1e-8), t[k] = n . p_k - (n . x1 + 1e-8)
struct CullLane {
    v2f xx, yy, zz, nxx, nyy, nzz, ncn;
    __device__ inline v2f eval_s(const LightPair& L) const {  // the light-side value alone
        const v2f nlx{L.nl[0].x, L.nl[0].y}, nly{L.nl[1].x, L.nl[1].y}, nlz{L.nl[2].x, L.nl[2].y};
        return __builtin_elementwise_fma(xx, nlx, __builtin_elementwise_fma(yy, nly, zz * nlz)) - v2f{L.d.x, L.d.y};
    }
    __device__ inline void eval(const LightPair& L, v2f* s, v2f* t) const {
        const v2f nlx{L.nl[0].x, L.nl[0].y}, nly{L.nl[1].x, L.nl[1].y}, nlz{L.nl[2].x, L.nl[2].y};
        // (the subtraction stays separate: a packed FMA reads at most one scalar operand)
        *s = __builtin_elementwise_fma(xx, nlx, __builtin_elementwise_fma(yy, nly, zz * nlz)) - v2f{L.d.x, L.d.y};
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const v2f px{L.p[3 * k].x, L.p[3 * k].y}, py{L.p[3 * k + 1].x, L.p[3 * k + 1].y},
                pz{L.p[3 * k + 2].x, L.p[3 * k + 2].y};
            t[k] = __builtin_elementwise_fma(nxx, px, __builtin_elementwise_fma(nyy, py, __builtin_elementwise_fma(nzz, pz, ncn)));
        }
    }
};

// one chunk (64 lights, two halves of 32) of the cull for this lane's node: the candidate word
// (bit j = light 64 c + j)
template <bool kCountC1>
__device__ inline uint64_t cull_chunk(const DScene& S, const CullLane& cl, const LightPair* __restrict__ T, int c,
                                      float err, uint64_t actm, bool act, d3 x1, d3 nn, unsigned long long& c1,
                                      bool classes) {
    // wave-uniform chunk classes (chunk_class; the nodes arrive sorted by their classes, k_cull_order):
    // every lane BELOW -- the word is 0 (not in the counting instance, which counts the light-side culls);
    // every lane ABOVE -- the light-side test alone.  Inactive lanes agree with anything.
    bool above = false;
    if (classes) {
        const unsigned cls = chunk_class(cl.nxx[0], cl.nyy[0], cl.nzz[0], cl.ncn[0], err, S.chunk_sph[c]);
        if (!kCountC1 && (__ballot(cls != kChunkBelow) & actm) == 0) return 0ull;
        above = (__ballot(cls != kChunkAbove) & actm) == 0;
    }
    unsigned word[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const LightPair* __restrict__ Th = T + 32 * c + 16 * h;
        unsigned w = 0, c1w = 0;
        float amin = __builtin_inff();  // min over the 32 lights of min(|s|, |min(s, max t)|)
        // pairs holding real lights (the table's last chunk is partial: N_L = 3012 leaves 4 of 64)
        const int qend = kCountC1 ? 16 : min(16, max(0, (S.NL - (64 * c + 32 * h) + 1) >> 1));
        // ABOVE: every fp32 t > err, so min(s, max t) > err iff s > err and |min(s, max t)| <= err iff
        // |s| <= err -- the same bits and the same fallback trigger as pair() without the t terms.  A NaN
        // s (a degenerate light's normal) passes the light-side test as in the reference (Mylight.cpp:342
        // culls only tmp < eps) and as in pair(), whose v_min_f32 returns max t for it: !(s <= err).
        auto pair_s = [&](int q) {
            const v2f s1 = cl.eval_s(Th[q]);
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const float sv = s1[e];
                amin = min_abs_raw(amin, sv);
                if (kCountC1) c1w += __popcll(__ballot(sv < -err) & actm);  // statistic only
                w = shift_in(w, __ballot(!(sv <= err)));
            }
        };
        auto pair = [&](int q) {
            v2f s1, t[3];
            cl.eval(Th[q], &s1, t);
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const float sv = s1[e];
                const float mn = min_raw(sv, max3_raw(t[0][e], t[1][e], t[2][e]));
                // ambiguous lanes (a value within err of the threshold) have s >= -err and a clear bit here
                amin = min3_abs_raw(amin, sv, mn);
                if (kCountC1) c1w += __popcll(__ballot(sv < -err) & actm);  // statistic only
                w = shift_in(w, __ballot(mn > err));
            }
        };
        if (qend == 16) {
            if (above) {
#pragma unroll 2
                for (int q = 0; q < 16; q++) pair_s(q);
            } else {
#pragma unroll 2
                for (int q = 0; q < 16; q++) pair(q);
            }
        } else {  // the padding lights' bits stay clear; light j's bit back at 31 - j
            for (int q = 0; q < qend; q++) pair(q);
            w = qend == 0 ? 0u : w << (32 - 2 * qend);
        }
        if (__ballot(amin <= err) & actm) {  // rare: the reference's exact fp64 stages for the ambiguous (node, light) pairs
            for (int q = 0; q < 16; q++) {
                v2f s1, t[3];
                cl.eval(Th[q], &s1, t);
                for (int e = 0; e < 2; e++) {
                    const float sv = s1[e];
                    const float mn = min_raw(sv, max3_raw(t[0][e], t[1][e], t[2][e]));
                    const int li = 64 * c + 32 * h + 2 * q + e;
                    int st = -1;
                    if (act && min_abs_raw(sv, mn) <= err && li < S.NL) {
                        const LightPair& L = Th[q];
                        auto pc = [&](int i) { return (double)(e ? L.p[i].y : L.p[i].x); };
                        const double4 ln = S.lt_n[li];
                        st = light_cheap_stage(mk3(pc(0), pc(1), pc(2)), mk3(pc(3), pc(4), pc(5)),
                                               mk3(pc(6), pc(7), pc(8)), mk3(ln.x, ln.y, ln.z), x1, nn);
                        if (st == 0) w |= 1u << (31 - (2 * q + e));
                    }
                    if (kCountC1) c1w += __popcll(__ballot(st == 1));  // uniform: every lane of the wave
                }
            }
        }
        c1 += c1w;
        word[h] = __builtin_bitreverse32(w);
    }
    return ((uint64_t)word[1] << 32) | word[0];
}

template <bool kCountC1>
__global__ __launch_bounds__(256, MCPT_LB_CULL) void k_prep_cull_lanes(DScene S, int n, const double* __restrict__ qp,
                                                         const double* __restrict__ qn, int qs, uint64_t* __restrict__ masks,
                                                         int nchunks, unsigned long long* stats,
                                                         const int* __restrict__ order) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = idx < n;
    const int nd = order ? order[act ? idx : n - 1] : (act ? idx : n - 1);  // the node this lane culls
    const d3 x1 = ld3(qp, qs, nd);
    const d3 nn = ld3(qn, qs, nd);
    const NodeF f = node_f(x1, nn, S.light_bound);
    const float cn = (float)(dot(nn, x1) + MCPT_EPS);
    CullLane cl;
    cl.xx = v2f{f.x, f.x};
    cl.yy = v2f{f.y, f.y};
    cl.zz = v2f{f.z, f.z};
    cl.nxx = v2f{f.nx, f.nx};
    cl.nyy = v2f{f.ny, f.ny};
    cl.nzz = v2f{f.nz, f.nz};
    cl.ncn = v2f{-cn, -cn};
    const float err = f.err;
    const uint64_t actm = __ballot(act);
    unsigned long long c1 = 0;
    const LightPair* __restrict__ T = S.lt_pair;
    // blockIdx.y splits the chunks (whole bursts of kCullBurst words): more waves per SIMD to hide
    // the scalar-load latency of the table.  A burst's words are stored back to back (16 B per
    // store) into the node's row.
    const int bursts = (nchunks + kCullBurst - 1) / kCullBurst;
    const int per = (bursts + gridDim.y - 1) / gridDim.y;
    const int pb = blockIdx.y * per, pe = min(bursts, pb + per);
    uint4* __restrict__ row = reinterpret_cast<uint4*>(masks + (size_t)nd * mask_stride(nchunks));
    for (int p = pb; p < pe; p++) {
        uint64_t w[kCullBurst];
#pragma unroll
        for (int i = 0; i < kCullBurst; i++) {
            const int c = kCullBurst * p + i;
            w[i] = c < nchunks ? cull_chunk<kCountC1>(S, cl, T, c, err, actm, act, x1, nn, c1, order != nullptr) : 0ull;
        }
        if (act)
#pragma unroll
            for (int i = 0; i < kCullBurst; i += 2)
                row[(kCullBurst * p + i) / 2] = make_uint4((unsigned)w[i], (unsigned)(w[i] >> 32), (unsigned)w[i + 1],
                                                           (unsigned)(w[i + 1] >> 32));
    }
    // zero words past the last burst up to the row's last whole line (k_prep_pk2 reads whole lines)
    if (act && pe == bursts)
        for (int p = bursts * kCullBurst / 2; p < mask_stride(nchunks) / 2; p++) row[p] = make_uint4(0, 0, 0, 0);
    // padding lights (index >= N_L, d = 1e30) were counted as light-side culled by every active lane
    if (kCountC1 && pe == bursts) c1 -= (unsigned long long)(64 * nchunks - S.NL) * (unsigned long long)__popcll(actm);
    if ((threadIdx.x & 63) == 0 && stats && c1) atomicAdd(stats + 6, c1);
}

// ---- the cull's node order (k_cull_classify + k_cull_scatter) ----
// A chunk's class skips work in k_prep_cull_lanes only when every lane of the wave agrees, and a
// generation's nodes come in no spatial order.  The class pattern over the chunks depends on the node's
// tangent plane alone (every node of a flat surface has the same one), so the nodes are bucketed by a
// hash of it: k_cull_classify hashes each node's pattern into one of kCullBuckets buckets and counts
// them, k_cull_scatter writes the order (bucket by bucket) that the cull's lanes read their nodes in.
// The candidate words do not depend on the order (each lane writes its node's row), only the work does.
constexpr int kCullBuckets = 64;
constexpr int kCullPer = 8;  // nodes per thread of the two order kernels
__device__ inline unsigned cull_pattern_bucket(const DScene& S, d3 x1, d3 nn, int nchunks) {
    const NodeF f = node_f(x1, nn, S.light_bound);
    const float ncn = -(float)(dot(nn, x1) + MCPT_EPS);  // as in k_prep_cull_lanes
    unsigned h = 2166136261u;
    for (int c = 0; c < nchunks; c++) h = (h ^ chunk_class(f.nx, f.ny, f.nz, ncn, f.err, S.chunk_sph[c])) * 16777619u;
    h ^= h >> 15;
    h *= 0x2c1b3c6du;
    h ^= h >> 12;
    return h & (kCullBuckets - 1);
}
// LDS histogram add of bucket b for the active lanes, one atomic per distinct bucket of the wave in the
// common case (a wave of one surface); returns this lane's rank among the block's nodes of its bucket
__device__ inline unsigned hist_add(unsigned* hist, unsigned b) {
    const unsigned b0 = __builtin_amdgcn_readfirstlane(b);
    const uint64_t m = __ballot(b == b0);
    const int lead = __ffsll((unsigned long long)m) - 1;
    unsigned base = 0;
    if ((int)(threadIdx.x & 63) == lead) base = atomicAdd(&hist[b0], (unsigned)__popcll(m));
    base = __builtin_amdgcn_readlane(base, lead);
    return b == b0 ? base + (unsigned)lane_rank(m) : atomicAdd(&hist[b], 1u);
}
__global__ __launch_bounds__(256) void k_cull_classify(DScene S, int n, const double* __restrict__ qp,
                                                       const double* __restrict__ qn, int qs, int nchunks,
                                                       unsigned char* __restrict__ keys, unsigned* __restrict__ count) {
    __shared__ unsigned hist[kCullBuckets];
    if (threadIdx.x < kCullBuckets) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int k = 0; k < kCullPer; k++) {
        const int node = (blockIdx.x * kCullPer + k) * 256 + threadIdx.x;
        if (node < n) {
            const unsigned b = cull_pattern_bucket(S, ld3(qp, qs, node), ld3(qn, qs, node), nchunks);
            keys[node] = (unsigned char)b;
            (void)hist_add(hist, b);
        }
    }
    __syncthreads();
    if (threadIdx.x < kCullBuckets && hist[threadIdx.x]) atomicAdd(&count[threadIdx.x], hist[threadIdx.x]);
}
// count[0, kCullBuckets): nodes per bucket (k_cull_classify); count[kCullBuckets, 2 kCullBuckets): the
// buckets' fill cursors (zero before the launch); order[bucket start + cursor] = node
__global__ __launch_bounds__(256) void k_cull_scatter(int n, const unsigned char* __restrict__ keys,
                                                      unsigned* __restrict__ count, int* __restrict__ order) {
    __shared__ unsigned hist[kCullBuckets], start[kCullBuckets];
    if (threadIdx.x < kCullBuckets) {
        hist[threadIdx.x] = 0;
        start[threadIdx.x] = count[threadIdx.x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive scan of the bucket sizes
        unsigned s = 0;
        for (int b = 0; b < kCullBuckets; b++) {
            const unsigned v = start[b];
            start[b] = s;
            s += v;
        }
    }
    unsigned rank[kCullPer], key[kCullPer];
    for (int k = 0; k < kCullPer; k++) {
        const int node = (blockIdx.x * kCullPer + k) * 256 + threadIdx.x;
        if (node < n) {
            key[k] = keys[node];
            rank[k] = hist_add(hist, key[k]);
        }
    }
    __syncthreads();
    if (threadIdx.x < kCullBuckets && hist[threadIdx.x])
        start[threadIdx.x] += atomicAdd(&count[kCullBuckets + threadIdx.x], hist[threadIdx.x]);
    __syncthreads();
    for (int k = 0; k < kCullPer; k++) {
        const int node = (blockIdx.x * kCullPer + k) * 256 + threadIdx.x;
        if (node < n) order[start[key[k]] + rank[k]] = node;
    }
}
// device scratch of the cull's node order: keys u8[n], order int[n], count u32[2 kCullBuckets]
struct CullOrder {
    unsigned char* keys = nullptr;
    int* order = nullptr;
    unsigned* count = nullptr;
};

#ifndef MCPT_FUSED_CLASSES
#define MCPT_FUSED_CLASSES 1
#endif
// an all-zero candidate word skips its list append by a scalar branch (same-box A/B: 410.6 / 425.0 /
// 425.1 vs 423.8 / 415.8 / 421.9 Msamples/s, profiles/round2b_ab_zero_words.txt)
constexpr int kMaskBatch = kMaskLine;  // candidate words per batch of scalar loads (k_prep_pk2): one line
template <int kMinWavesPerSimd, bool kBuild, bool kMaskIn = false, bool kF32 = false>
__global__ __launch_bounds__(256, kMinWavesPerSimd) void k_prep_pk2(DScene S, uint64_t seed, int n, const double* __restrict__ qp,
                                                  const double* __restrict__ qn, int qs, const int* __restrict__ qpixel,
                                                  const int* __restrict__ qsample, const uint64_t* __restrict__ qnode,
                                                  const double* __restrict__ u_override, double* __restrict__ wsum_out,
                                                  int* __restrict__ pick_out, int* __restrict__ count_out,
                                                  unsigned long long* stats, int nchunks, int wave_bytes,
                                                  unsigned* __restrict__ work, PrepCache C,
                                                  const uint64_t* __restrict__ masks = nullptr) {
    extern __shared__ double prep_lds[];
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
    double* bt = reinterpret_cast<double*>(reinterpret_cast<char*>(prep_lds) + (size_t)wib * wave_bytes);
    unsigned short* lst = reinterpret_cast<unsigned short*>(bt + nchunks);
    const int ngroups4 = (nchunks + 3) / 4;
    const __amdgpu_buffer_rsrc_t rpk = __builtin_amdgcn_make_buffer_rsrc((void*)S.lt_pk, 0, ngroups4 * 4 * 3072, kBufFlags);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)S.lt_d, 0, ngroups4 * 4 * 256, kBufFlags);
    const __amdgpu_buffer_rsrc_t rw = kF32 ? light_record_f32_rsrc(S, ngroups4) : light_record_rsrc(S, ngroups4);
    // list padding: the entries [ncand, 64 nb) of the last batch name a sentinel record past the
    // table, which the full stage always culls, so a batch needs no k < ncand test
    const unsigned short sentinel = (unsigned short)(ngroups4 * 256);
    unsigned long long cand_acc = 0, c1_acc = 0, full_acc = 0, pad_acc = 0;
    unsigned bad_acc = 0;  // per lane: culled lanes of phase B, padding included
    int grab = 0, left = 0;
    while (true) {
        if (left == 0) {
            unsigned b = 0;
            if (lane == 0) b = atomicAdd(work, (unsigned)kPrepGrab);
            grab = __shfl((int)b, 0);
            left = kPrepGrab;
        }
        const int node = __builtin_amdgcn_readfirstlane(grab++);
        left--;
        if (node >= n) break;
        const d3 x1 = ld3(qp, qs, node);
        auto u_of = [&]() {
            return u_override ? u_override[node]
                              : counter_u(counter_key(seed, (uint64_t)qpixel[node], (uint64_t)qsample[node], qnode[node]), 1);
        };
        int ncand = 0, nb = 0, survivors = 0, culled1 = 0;
        const uint64_t* __restrict__ mrow = kMaskIn ? masks + (size_t)node * mask_stride(nchunks) : nullptr;
        if (kMaskIn) {  // phase A done by k_prep_cull_lanes: rebuild the list from the candidate words
            // The node's words are wave-uniform: scalar loads of whole 64-B lines (s_load_dwordx16,
            // kMaskBatch words each, the row zero-padded to whole lines) put them straight into SGPRs,
            // so a word costs 3 VALU (2 v_mbcnt + 1 v_lshl_add) + 1 v_add for the index.
            const unsigned lds_lst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lst);  // LDS offset (low half of the flat address)
            for (int c0 = 0; c0 < nchunks; c0 += kMaskBatch) {
                uint64_t mw[kMaskBatch];
#pragma unroll
                for (int q = 0; q < kMaskBatch; q++) mw[q] = mrow[c0 + q];
#pragma unroll
                for (int q = 0; q < kMaskBatch; q++) {
                    const uint64_t m = mw[q];
                    if (m != 0) {  // wave-uniform (SGPR word): an empty chunk costs no VALU
                        append_masked(m, (unsigned)m, (unsigned)(m >> 32), lds_lst + 2u * (unsigned)ncand,
                                      (unsigned)lane + 64u * (unsigned)(c0 + q));
                        ncand += __popcll(m);
                    }
                }
            }
        } else {
        const d3 nn = ld3(qn, qs, node);
        const NodeF nf = node_f(x1, nn, S.light_bound);
        const float cn = (float)dot(nn, x1);
        const v2f nx2{nf.nx, nf.nx}, ny2{nf.ny, nf.ny}, nz2{nf.nz, nf.nz};
        const v2f nxs{nf.nx, nf.x}, nys{nf.ny, nf.y}, nzs{nf.nz, nf.z};
        // phase A: cheap stages over all chunks, kChunkUnroll chunks' table loads in flight at a
        // time (the loop is L2-latency-bound; the tables are padded to whole groups of 4 chunks).
        // MCPT_FUSED_CLASSES: a chunk wholly below the node's tangent plane (chunk_class, the node is the
        // wave's, so the class is wave-uniform) holds no candidate and is skipped, loads included
        const float ncls = -(float)(dot(nn, x1) + MCPT_EPS);  // chunk_class's form, as k_prep_cull_lanes
        for (int c = 0; c < nchunks; c += kChunkUnroll) {
            float4 X[kChunkUnroll], Y[kChunkUnroll], Z[kChunkUnroll];
            float dl[kChunkUnroll];
            bool skip[kChunkUnroll];
#pragma unroll
            for (int q = 0; q < kChunkUnroll; q++) {
                const int cq = c + q;
                skip[q] = MCPT_FUSED_CLASSES && cq < nchunks &&
                          __builtin_amdgcn_readfirstlane(chunk_class(nf.nx, nf.ny, nf.nz, ncls, nf.err, S.chunk_sph[cq])) ==
                              kChunkBelow;
                if (skip[q]) continue;
                X[q] = u4f(__builtin_amdgcn_raw_buffer_load_b128(rpk, lane * 48, cq * 3072, 0));
                Y[q] = u4f(__builtin_amdgcn_raw_buffer_load_b128(rpk, lane * 48 + 16, cq * 3072, 0));
                Z[q] = u4f(__builtin_amdgcn_raw_buffer_load_b128(rpk, lane * 48 + 32, cq * 3072, 0));
                dl[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rd, lane * 4, cq * 256, 0));
            }
#pragma unroll
            for (int q = 0; q < kChunkUnroll; q++) {
                if (skip[q]) continue;
                const int li = (c + q) * 64 + lane;
                const int stage = prep_stage_pk_bf(S, li, X[q], Y[q], Z[q], dl[q], nx2, ny2, nz2, nxs, nys, nzs, cn, x1, nn, nf.err);
                const uint64_t m = __ballot(stage == 0);
                if (stage == 0) lst[ncand + lane_rank(m)] = (unsigned short)li;
                ncand += __popcll(m);
                culled1 += __popcll(__ballot(stage == 1));
            }
        }
        }
        nb = (ncand + 63) >> 6;
        if (ncand + lane < 64 * nb) lst[ncand + lane] = sentinel;  // pad the last batch
        wave_lds_sync();
        // phase B: dense fp64 batches of 64 consecutive candidates, four at a time (batch_totals4).
        // Culled lanes (the full stage's rare culls and the sentinel padding) are counted by a
        // branch on the exec mask that is almost never taken except for the padding, instead of a
        // ballot per batch; survivors = ncand - (culled lanes - padding).
        int nbad = 0;
        double sacc = 0;  // flagged slivers' error terms (this lane's candidates)
        int ndeg = 0;     // near-degenerate slivers (this lane's)
        const NodeF32 xf = node_f32(x1);
        for (int b0 = 0; b0 < nb; b0 += 4) {
            double w4[4];
            if (kF32) {  // batches (b0, b0+1) and (b0+2, b0+3) as the two halves of packed fp32 evaluations
#pragma unroll
                for (int i = 0; i < 4; i += 2) {
                    w4[i] = w4[i + 1] = 0.0;
                    if (b0 + i < nb) {  // wave-uniform
                        const int k0 = 64 * (b0 + i) + lane, k1 = k0 + 64;
                        const bool has1 = b0 + i + 1 < nb;
                        bool ok0, ok1;
                        double w0, w1;
                        prep_weight_f32x2(rw, (int)lst[k0], has1 ? (int)lst[k1] : (int)sentinel, xf, &w0, &w1, &ok0, &ok1);
                        if (kBuild) {  // in-batch inclusive prefixes, culled with the sign bit (PrepCache::w)
                            const size_t row = (size_t)(qpixel ? qpixel[node] : node) * C.lstride;
                            const double s0 = wave_incl_scan(ok0 ? w0 : 0.0, lane);
                            const double s1 = has1 ? wave_incl_scan(ok1 ? w1 : 0.0, lane) : 0.0;
                            if (k0 < ncand) C.w[row + k0] = ok0 ? s0 : copysign(s0, -1.0);
                            if (k1 < ncand) C.w[row + k1] = ok1 ? s1 : copysign(s1, -1.0);
                        }
                        w4[i] = w0;
                        w4[i + 1] = w1;
                        if (!ok0) asm volatile("v_add_u32 %0, 1, %0" : "+v"(nbad));
                        if (has1 && !ok1) asm volatile("v_add_u32 %0, 1, %0" : "+v"(nbad));
                    }
                }
            } else {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                w4[i] = 0.0;
                if (b0 + i < nb) {  // wave-uniform
                    const int k = 64 * (b0 + i) + lane;
                    double l2;
                    const WeightBx r = prep_weight_buf_bx(rw, (int)lst[k], x1, &l2);  // w = 0 if culled
                    if (kBuild) {  // in-batch inclusive prefix, culled with the sign bit (PrepCache::w)
                        const double sc = wave_incl_scan(r.ok ? r.w : 0.0, lane);
                        if (k < ncand) C.w[(size_t)(qpixel ? qpixel[node] : node) * C.lstride + k] = r.ok ? sc : copysign(sc, -1.0);
                    }
                    w4[i] = r.w;
                    // a real branch (SALU only when no lane is culled or a sliver): culled lanes (the
                    // padding included) are counted, slivers add their term to the band
                    if (!r.ok | r.sliver) {
                        if (!r.ok) {
                            asm volatile("v_add_u32 %0, 1, %0" : "+v"(nbad));
                        } else {
                            const double t = sliver_term(r.num, r.den) * l2;
                            sacc += t;
                            if (2.0 * r.w < 64.0 * kU53 * t)  // sA within the reference's error of 0
                                asm volatile("v_add_u32 %0, 1, %0" : "+v"(ndeg));
                        }
                    }
                }
            }
            }
            const double t = batch_totals4(w4[0], w4[1], w4[2], w4[3]);
            if ((lane & 15) == 15 && b0 + (lane >> 4) < nb) bt[b0 + (lane >> 4)] = t;
        }
        wave_lds_sync();
        const int npad = 64 * nb - ncand;
        if (kBuild || count_out) survivors = ncand - (wave_sum_int(nbad) - npad);
        bad_acc += nbad;
        pad_acc += npad;
        full_acc++;
        cand_acc += ncand;
        c1_acc += culled1;
        // the flagged slivers' band term (wave-uniform; almost always 0 without a wave reduction)
        double band_sl = 0;
        if (!kF32 && __ballot(sacc > 0.0)) band_sl = band_sliver(__shfl(wave_incl_scan(sacc, lane), 63));
        if (kBuild) {  // store the entry of this pixel (C.build), with the node's band for k_prep_pick
            const int px = qpixel ? qpixel[node] : node;
            if (nb <= 64) {  // the batch totals' inclusive scan -- the same scan k_prep_pick used to redo per root
                const double cum = wave_incl_scan(lane < nb ? bt[lane] : 0.0, lane);
                if (lane < nb) C.bt[(size_t)px * nchunks + lane] = cum;
            } else {  // k_prep_pick sums these sequentially
                for (int b = lane; b < nb; b += 64) C.bt[(size_t)px * nchunks + b] = bt[b];
            }
            for (int k = lane; k < ncand; k += 64) C.lst[(size_t)px * C.lstride + k] = lst[k];
            if (lane == 0) {
                const double band = kF32 ? 0.0 : band_sl + band_base(S, x1, mrow, nchunks);
                C.info[px] = make_int4(nb, ncand, survivors, __float_as_int((float)band * 1.001f));
            }
            wave_lds_sync();
            continue;
        }
        int pick;
        double margin;
        const double wsum = prep_select<kF32>(bt, lst, nb, ncand, lane, rw, x1, u_of, &pick, &margin);
        if (lane == 0) {
            wsum_out[node] = wsum;
            pick_out[node] = pick;
            if (count_out) count_out[node] = survivors;
        }
        if (!kF32 && C.slack) {  // exact pick: the slack against the band (band_candidate, k_prep_band)
            double sl = pick_slack(margin, wsum) - (band_sl + band_round(ncand, wsum));
            // survivor counts: a candidate the full stage culls (the reference may keep it) or a
            // near-degenerate sliver (the reference may cull it) -- survivors < ncand without padding
            if (C.exact_counts && (survivors < ncand || __ballot(ndeg != 0))) sl = -INFINITY;
            if (lane == 0) band_candidate(S, C.slack, C.maybe, C.exact_off + node, sl, x1, ncand);
        }
        wave_lds_sync();
    }
    if (stats) {
        const unsigned long long surv_acc = cand_acc - (wave_sum_u64(bad_acc) - pad_acc);
        if (lane == 0) {
            if (surv_acc) atomicAdd(stats + 1, surv_acc);
            if (cand_acc) atomicAdd(stats + 5, cand_acc);
            if (c1_acc) atomicAdd(stats + 6, c1_acc);
            if (full_acc) atomicAdd(stats + 7, full_acc);
        }
    }
}

// root nodes (node id 1) from the root-point cache: prep_select's search with the cached batch
// totals and candidate weights -- the same scans over the same values, so the same pick -- and no
// light-triangle arithmetic at all.  One wave per node, kPickNodes nodes per wave at a time: a root
// is a chain of three dependent loads (pixel -> batch totals -> one batch of weights), so the wave
// issues each link for all of its nodes before waiting on any of them (the kernel is bound by
// that latency, not by bandwidth).  No LDS.
#ifndef MCPT_PICK_NODES
#define MCPT_PICK_NODES 4
#endif
constexpr int kPickNodes = MCPT_PICK_NODES;
__global__ __launch_bounds__(256, MCPT_LB_PICK) void k_prep_pick(DScene S, uint64_t seed, int n, const int* __restrict__ qpixel,
                                                   const int* __restrict__ qsample, const uint64_t* __restrict__ qnode,
                                                   double* __restrict__ wsum_out, int* __restrict__ pick_out,
                                                   unsigned long long* stats, int nchunks, PrepCache C) {
    const int lane = threadIdx.x & 63;
    const int waves = gridDim.x * (blockDim.x >> 6);
    const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    unsigned long long cached = 0;
    // static assignment: a root costs ~the same everywhere, and a shared work counter would
    // serialise on its one address at this node rate
    for (int n0 = gw * kPickNodes; n0 < n; n0 += waves * kPickNodes) {
        int px[kPickNodes], smp[kPickNodes];
        uint64_t nid[kPickNodes];
#pragma unroll
        for (int k = 0; k < kPickNodes; k++) {
            const int node = min(n0 + k, n - 1);
            px[k] = qpixel[node];
            smp[k] = qsample[node];
            nid[k] = qnode[node];
        }
        double vraw[kPickNodes];
        int4 inf[kPickNodes];
#pragma unroll
        for (int k = 0; k < kPickNodes; k++) {
            vraw[k] = lane < nchunks ? C.bt[(size_t)px[k] * nchunks + lane] : 0.0;
            inf[k] = C.info[px[k]];
        }
        // the roots' pick uniforms (dim 1), one root per lane 0..kPickNodes-1: the 64-bit hash chain
        // runs once for all of them instead of once per root on every lane
        double ul;
        {
            const int kk = lane & (kPickNodes - 1);
            int pxs = px[0], sms = smp[0];
            uint64_t nds = nid[0];
#pragma unroll
            for (int k = 1; k < kPickNodes; k++) {
                pxs = kk == k ? px[k] : pxs;
                sms = kk == k ? smp[k] : sms;
                nds = kk == k ? nid[k] : nds;
            }
            ul = counter_u(counter_key(seed, (uint64_t)pxs, (uint64_t)sms, nds), 1);
        }
        double wsum[kPickNodes], base[kPickNodes], target[kPickNodes];
        int kb[kPickNodes];
#pragma unroll
        for (int k = 0; k < kPickNodes; k++) {
            const int nb = inf[k].x;
            const double* bt = C.bt + (size_t)px[k] * nchunks;
            const double u = __longlong_as_double(
                ((long long)__builtin_amdgcn_readlane((int)(__double_as_longlong(ul) >> 32), k) << 32) |
                (unsigned)__builtin_amdgcn_readlane((int)__double_as_longlong(ul), k));
            wsum[k] = 0;
            kb[k] = -1;
            base[k] = 0;
            target[k] = 0;
            if (nb <= 64) {  // vraw = the cached inclusive scan of the batch totals (cache build)
                const double W = nb > 0 ? readlane_f64(vraw[k], nb - 1) : 0.0;
                const double cum = lane < nb ? vraw[k] : W;
                wsum[k] = W;
                if (!(fabs(wsum[k]) < MCPT_EPS)) {
                    target[k] = u * wsum[k];
                    // the first batch whose running total reaches the target (and is positive: for a
                    // target > 0 that batch's own total is positive, as "cum >= target && v > 0" required;
                    // for target 0 it is the first positive batch); target <= W, so one exists
                    const uint64_t hitm = __ballot(lane < nb && cum >= target[k] && cum > 0.0);
                    kb[k] = hitm ? __ffsll((unsigned long long)hitm) - 1 : -1;
                    base[k] = kb[k] > 0 ? readlane_f64(cum, kb[k] - 1) : 0.0;
                }
            } else {  // more than 64 batches (N_L > 4096 with many candidates): sequential search
                double ws = 0;
                for (int b = 0; b < nb; b++) ws += bt[b];
                wsum[k] = ws;
                if (!(fabs(ws) < MCPT_EPS)) {
                    target[k] = u * ws;
                    int lastpos = -1, kk = -1;
                    double cum = 0, bs = 0;
                    for (int b = 0; b < nb; b++) {
                        const double nxt = cum + bt[b];
                        if (bt[b] > 0) lastpos = b;
                        if (kk < 0 && nxt >= target[k] && bt[b] > 0) {
                            kk = b;
                            bs = cum;
                        }
                        cum = nxt;
                    }
                    if (kk < 0) {
                        kk = lastpos;
                        bs = 0;
                        for (int b = 0; b < kk; b++) bs += bt[b];
                    }
                    kb[k] = kk;
                    base[k] = bs;
                }
            }
        }
        double wc[kPickNodes];
#pragma unroll
        for (int k = 0; k < kPickNodes; k++) {
            const int j = 64 * kb[k] + lane;
            const bool act = kb[k] >= 0 && j < inf[k].y;
            wc[k] = act ? C.w[(size_t)px[k] * C.lstride + j] : -0.0;  // signed in-batch prefix
        }
        // the picked lane's light index only (one uniform load per root, issued for all roots
        // before waiting) instead of the batch's 64 list entries
        int pls[kPickNodes];
        double margin[kPickNodes];
#pragma unroll
        for (int k = 0; k < kPickNodes; k++) {
            pls[k] = -1;
            margin[k] = INFINITY;
            if (kb[k] >= 0) {
                // the cache build stored each batch's inclusive scan (the scan this pick used to redo):
                // survivors as is, culled candidates with the sign bit set
                const bool ok = !signbit(wc[k]);
                const double sc = fabs(wc[k]);
                const uint64_t candm = __ballot(ok && (base[k] + sc >= target[k]));
                const uint64_t okm = __ballot(ok);
                if (candm) pls[k] = __ffsll((unsigned long long)candm) - 1;
                else if (okm) pls[k] = 63 - __clzll((long long)okm);
                if (pls[k] >= 0) margin[k] = pick_margin(base[k], sc, pls[k], target[k]);
            }
        }
        if (C.exact) {  // exact pick: the band stored by the cache build (same weights) + this sum's rounding
#pragma unroll
            for (int k = 0; k < kPickNodes; k++) {
                const double band = (double)__int_as_float(inf[k].w) + band_round(inf[k].y, wsum[k]);
                if (lane == 0 && n0 + k < n && !(pick_slack(margin[k], wsum[k]) > band)) {
                    const int q = atomicAdd(C.exact, 1);
                    C.exact[kExactHead + q] = C.exact_off + n0 + k;
                }
            }
        }
        int pk[kPickNodes];
#pragma unroll
        for (int k = 0; k < kPickNodes; k++)
            pk[k] = pls[k] >= 0 ? (int)C.lst[(size_t)px[k] * C.lstride + 64 * kb[k] + pls[k]] : -1;
#pragma unroll
        for (int k = 0; k < kPickNodes; k++) {
            const int pick = pk[k];
            if (lane == 0 && n0 + k < n) {
                wsum_out[n0 + k] = wsum[k];
                pick_out[n0 + k] = pick;
            }
        }
        cached += (unsigned long long)min(kPickNodes, n - n0);
    }
    if (lane == 0 && stats && cached) atomicAdd(stats + 0, cached);
}

// k_prep_pick with a 16-lane group per root (nchunks <= 64): the same search over the same cached
// values, so the same pick, margin and exact-list decision.  k_prep_pick spends a whole wave per root
// for a batch-total row of nchunks values and a batch of 64 weights, so its 72 VGPRs hold only four
// roots' chains and the kernel waits on latency at ~2 TB/s (round 3 PMC: 478 B and four dependent
// hops per root).  Here lane (g, l) of a wave holds entries l, l + 16, l + 32, l + 48 of root g's row
// and batch -- each 16-lane load is one whole 128-B line -- so a wave keeps 4 * kPickSlots roots in
// flight, and the batch's 64 list entries (one more line) come with its weights instead of one
// dependent load after the search.  Cross-lane reads inside a group are ds_bpermute.
#ifndef MCPT_PICK_SLOTS
#define MCPT_PICK_SLOTS 4  // roots per wave = 4 x slots (A/B: 2 slots at 7 waves 476.8-478.2, 4 slots at 4 waves 480.2-480.5)
#endif
#ifndef MCPT_PICK_GROUPS
#define MCPT_PICK_GROUPS 1  // 0: k_prep_pick (wave per root) for every table size (A/B)
#endif
#ifndef MCPT_LB_PICKG
#define MCPT_LB_PICKG 4  // 121 VGPRs at 4 slots, no spills
#endif
constexpr int kPickSlots = MCPT_PICK_SLOTS;
__device__ inline int bperm_i32(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
__device__ inline double bperm_f64(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)b);
    const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// v[k], k uniform within the lane's group: two levels of selects on k's bits (written on the four
// values rather than the array, which the compiler otherwise turns into an indexed scratch load)
template <class T>
__device__ inline T sel4v(T v0, T v1, T v2, T v3, int k) {
    const T lo = (k & 1) ? v1 : v0, hi = (k & 1) ? v3 : v2;
    return (k & 2) ? hi : lo;
}
template <class T>
__device__ inline T sel4(const T (&v)[4], int k) { return sel4v(v[0], v[1], v[2], v[3], k); }
// first / last searches within a 16-lane group by a row reduction (DPP row_ror butterflies: four VALU
// each) on per-lane candidate indices, instead of decoding ballot masks lane by lane (round 3, +1.1%)
__device__ inline unsigned row_min_u32(unsigned v) {
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false));  // row_ror:8
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false));  // row_ror:4
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xf, 0xf, false));  // row_ror:2
    return min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xf, 0xf, false));  // row_ror:1
}
__device__ inline int row_max_i32(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x124, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x122, 0xf, 0xf, false));
    return max(v, __builtin_amdgcn_update_dpp(0, v, 0x121, 0xf, 0xf, false));
}
__global__ __launch_bounds__(256, MCPT_LB_PICKG) void k_prep_pick_g(DScene S, uint64_t seed, int n, const int* __restrict__ qpixel,
                                                     const int* __restrict__ qsample, const uint64_t* __restrict__ qnode,
                                                     double* __restrict__ wsum_out, int* __restrict__ pick_out,
                                                     unsigned long long* stats, int nchunks, PrepCache C) {
    constexpr int kR = 4 * kPickSlots;  // roots per wave and iteration
    static_assert((kR & (kR - 1)) == 0 && kR <= 64, "pick slots");
    const int lane = threadIdx.x & 63, g = lane >> 4, gl = lane & 15, g0 = lane & 48;
    const int waves = gridDim.x * (blockDim.x >> 6);
    const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int nq = (nchunks + 15) >> 4;  // row entries per lane (<= 4)
    unsigned long long cached = 0;
    // lane r < kR: root n0 + r (coalesced queue loads), fetched one iteration ahead so that the queue
    // hop overlaps the previous roots' cache hops (round 3: +0.6%)
    int f_px = 0, f_smp = 0;
    uint64_t f_nid = 0;
    auto fetch = [&](int m0) {
        const int node = min(m0 + (lane & (kR - 1)), n - 1);
        f_px = qpixel[node];
        f_smp = qsample[node];
        f_nid = qnode[node];
    };
    // slot s: group g takes root 4 s + g; its row of batch totals (inclusive scan) and info
    int px[kPickSlots];
    int4 inf[kPickSlots];
    double bv[kPickSlots][4];
    auto load_rows = [&](int pxl_, int (&px_)[kPickSlots], int4 (&inf_)[kPickSlots], double (&bv_)[kPickSlots][4]) {
#pragma unroll
        for (int s = 0; s < kPickSlots; s++) {
            px_[s] = bperm_i32(pxl_, 4 * s + g);
            const double* row = C.bt + (size_t)px_[s] * nchunks + gl;
#pragma unroll
            for (int k = 0; k < 4; k++) bv_[s][k] = k < nq && 16 * k + gl < nchunks ? row[16 * k] : 0.0;
            inf_[s] = C.info[px_[s]];
        }
    };
    if (gw * kR < n) fetch(gw * kR);
    for (int n0 = gw * kR; n0 < n; n0 += waves * kR) {
        const int pxl = f_px;
        const double ul = counter_u(counter_key(seed, (uint64_t)pxl, (uint64_t)f_smp, f_nid), 1);  // dim 1
        if (n0 + waves * kR < n) fetch(n0 + waves * kR);
        load_rows(pxl, px, inf, bv);
        double wsum[kPickSlots], base[kPickSlots], target[kPickSlots];
        int kb[kPickSlots];
#pragma unroll
        for (int s = 0; s < kPickSlots; s++) {
            const int nb = inf[s].x;
            const int lw = max(nb - 1, 0);
            const double W = bperm_f64(sel4(bv[s], lw >> 4), g0 + (lw & 15));
            wsum[s] = nb > 0 ? W : 0.0;
            const bool valid = !(fabs(wsum[s]) < MCPT_EPS);
            target[s] = bperm_f64(ul, 4 * s + g) * wsum[s];
            {
                unsigned c = 64;
#pragma unroll
                for (int k = 3; k >= 0; k--)
                    c = valid && 16 * k + gl < nb && bv[s][k] >= target[s] && bv[s][k] > 0.0 ? 16 * k + gl : c;
                c = row_min_u32(c);
                kb[s] = c < 64 ? (int)c : -1;
            }
            const int lb = max(kb[s] - 1, 0);
            const double b = bperm_f64(sel4(bv[s], lb >> 4), g0 + (lb & 15));
            base[s] = kb[s] > 0 ? b : 0.0;
        }
        // the picked batch's signed in-batch prefixes and its 64 list entries
        double wc[kPickSlots][4];
        int lj[kPickSlots][4];
#pragma unroll
        for (int s = 0; s < kPickSlots; s++) {
            const size_t off = (size_t)px[s] * C.lstride + 64 * max(kb[s], 0) + gl;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const bool act = kb[s] >= 0 && 64 * kb[s] + 16 * k + gl < inf[s].y;
                wc[s][k] = act ? C.w[off + 16 * k] : -0.0;
                lj[s][k] = act ? (int)C.lst[off + 16 * k] : -1;
            }
        }
#pragma unroll
        for (int s = 0; s < kPickSlots; s++) {
            int pl;
            {
                unsigned cf = 64;
                int cl = -1;
#pragma unroll
                for (int k = 3; k >= 0; k--) {
                    const bool ok = !signbit(wc[s][k]);
                    cf = ok && (base[s] + fabs(wc[s][k]) >= target[s]) ? 16 * k + gl : cf;
                    cl = ok && cl < 0 ? 16 * k + gl : cl;  // the highest k wins
                }
                cf = row_min_u32(cf);
                const int lastv = row_max_i32(cl);  // every lane of the row takes part in the DPP steps
                pl = cf < 64 ? (int)cf : lastv;
            }
            double margin = INFINITY;
            int pick = -1;
            {
                const int l1 = max(pl, 0), l0 = max(pl - 1, 0);
                double sc[4];
#pragma unroll
                for (int k = 0; k < 4; k++) sc[k] = fabs(wc[s][k]);
                const double s1 = bperm_f64(sel4(sc, l1 >> 4), g0 + (l1 & 15));
                const double s0 = bperm_f64(sel4(sc, l0 >> 4), g0 + (l0 & 15));
                const int pk = bperm_i32(sel4(lj[s], l1 >> 4), g0 + (l1 & 15));
                if (pl >= 0) {  // pick_margin's terms
                    const double c_hi = base[s] + s1;
                    const double c_lo = pl > 0 ? base[s] + s0 : base[s];
                    const double m_lo = c_lo == 0.0 ? INFINITY : target[s] - c_lo;
                    margin = fmin(m_lo, c_hi - target[s]);
                    pick = pk;
                }
            }
            const int node = n0 + 4 * s + g;
            bool amb = false;
            if (gl == 0 && node < n) {
                wsum_out[node] = wsum[s];
                pick_out[node] = pick;
                if (C.exact) {  // exact pick: the band stored by the cache build + this sum's rounding
                    const double band = (double)__int_as_float(inf[s].w) + band_round(inf[s].y, wsum[s]);
                    amb = !(pick_slack(margin, wsum[s]) > band);
                }
            }
            if (C.exact) {  // one list atomic per wave (C.exact is launch-uniform)
                const int q = wave_append(reinterpret_cast<unsigned*>(C.exact), amb);
                if (amb) C.exact[kExactHead + q] = C.exact_off + node;
            }
        }
        cached += (unsigned long long)min(kR, n - n0);
    }
    if (lane == 0 && stats && cached) atomicAdd(stats + 0, cached);
}

// Exact pick, the band test's second half (lane per listed node): the per-chunk term
// of the band against the slack of each node band_candidate listed (k_prep_pk2 / k_prep: margin less
// the slivers' and the rounding terms, not above the whole-table bound), from the node's candidate
// words.  Nodes inside the band are appended to the exact list (count in list[0], wave-aggregated).
// Only nodes [0, nmask) have candidate words (the prep variant that ran wrote them); any other node is
// tested with every chunk counted as full (band_base without words: 64 candidates per chunk, an upper
// bound), never with stale words.
constexpr int kBandBlocks = 128;
__global__ __launch_bounds__(256) void k_prep_band(DScene S, const int* __restrict__ maybe, const double* __restrict__ slack,
                                                  const double* __restrict__ qp, int qs, const uint64_t* __restrict__ masks,
                                                  int nmask, int nchunks, int* __restrict__ list, unsigned long long* stats) {
    const int cnt = maybe[0];
    if (blockIdx.x == 0 && threadIdx.x == 0 && stats && cnt) atomicAdd(stats + 11, (unsigned long long)cnt);
    for (int j0 = blockIdx.x * blockDim.x; j0 < cnt; j0 += gridDim.x * blockDim.x) {  // block-uniform trip count
        const int j = j0 + threadIdx.x;
        bool amb = false;
        int i = 0;
        if (j < cnt) {
            i = maybe[kExactHead + j];
            const double sl = slack[i];
            if (!(sl > 0.0)) {
                amb = true;
            } else {
                const d3 x1 = ld3(qp, qs, i);
                amb = !(sl > band_base(S, x1, masks && i < nmask ? masks + (size_t)i * mask_stride(nchunks) : nullptr, nchunks));
            }
        }
        const int q = wave_append(reinterpret_cast<unsigned*>(list), amb);
        if (amb) list[kExactHead + q] = i;
    }
}

// Exact fallback of the light prep's pick.  For the nodes the prep kernels put on
// the exact list (list[kExactHead + j] = node index, count in list[0]): the reference's own arithmetic
// end to end -- the cheap culls (light_cheap_stage, Mylight.cpp:340-357; for a node whose candidate
// words k_prep_cull_lanes wrote, those words, and for a root its pixel's cached candidate list: the same
// decisions), the literal full stage (light_tri_stage: sqrt / division unit vectors, acos_cr vertex
// angles, alpha + beta + gamma - pi, Mylight.cpp:360-413), weights_sum summed candidate by candidate in
// index order (Mylight.cpp:415-418) and the pick "first survivor whose running sum >= u weights_sum,
// else the last survivor" -- so weights_sum, the survivor count and the pick are the oracle's bit for
// bit (acos_cr: correctly rounded, so up to glibc's acos on the ~5e-4 of arguments it rounds the other
// way).
// One wave per node, with enough waves for 4 per SIMD (a launch holds ~10^3-10^4 listed nodes; with one
// wave per SIMD the serial running sum ran at the latency of every instruction -- ~100 us per node).
// The running sum is the one sequential part: each 64-candidate chunk's weights sit one per lane and
// are added in order through v_readlane (culled candidates contribute +0, which leaves an fp64 sum
// unchanged), fully unrolled, lane q keeping the sum after candidate q; the pick is a ballot search
// over the stored running sums.
constexpr int kExactBlock = 256;
inline int exact_waves(int NL) {  // grid-stride; scratch (2 x 8 B per light per wave) kept <= 1 GiB
    const long long per = 16ll * ((NL + 63) & ~63);
    return (int)std::max(256ll, std::min(8192ll, (1ll << 30) / per)) & ~3;
}
inline int exact_blocks(int NL) { return exact_waves(NL) / (kExactBlock / 64); }
// Roots' literal sums, per pixel and per render call: a root's (x1, n) is its pixel's, so the literal
// running sums of its candidates are the same for every sample; the first exact root of a pixel stores
// them (pool entry: the running sum after each cached candidate, -1 if culled, then weights_sum) and
// later ones only search.  slot[16 + px]: -1 none, -2 being computed, -3 no room, else
// (launch << 20) | entry; an entry is read only by later launches (kernel boundaries order it).
// slot[0]: the pool's allocation counter.
struct RootLit {
    int* slot;
    double* pool;
    int cap, stride, launch;
};
__global__ __launch_bounds__(kExactBlock, MCPT_LB_EXACT) void k_prep_exact(DScene S, uint64_t seed, const int* __restrict__ list,
                                                         const double* __restrict__ qp, const double* __restrict__ qn, int qs,
                                                         const int* __restrict__ qpixel, const int* __restrict__ qsample,
                                                         const uint64_t* __restrict__ qnode,
                                                         const double* __restrict__ u_override, double* __restrict__ wsum_out,
                                                         int* __restrict__ pick_out, int* __restrict__ count_out,
                                                         unsigned long long* stats, double* __restrict__ scratch,
                                                         const uint64_t* __restrict__ masks, int nmask, int nchunks,
                                                         const unsigned short* __restrict__ clst, const int4* __restrict__ cinfo,
                                                         int lstride, int root_off, RootLit RL, int* __restrict__ defer) {
    const int lane = threadIdx.x & 63;
    const int waves = gridDim.x * (kExactBlock / 64);
    const int gw = blockIdx.x * (kExactBlock / 64) + (threadIdx.x >> 6);
    const int nlp = (S.NL + 63) & ~63;
    double* wsc = scratch + (size_t)gw * nlp;                  // candidates' weights, then running sums
    int* lst = reinterpret_cast<int*>(scratch + (size_t)waves * nlp) + (size_t)gw * nlp;  // candidate list
    const int cnt = list[0];
    if (gw == 0 && lane == 0 && stats && cnt) atomicAdd(stats + 10, (unsigned long long)cnt);
    for (int j = gw; j < cnt; j += waves) {
        const int node = list[kExactHead + j];
        const d3 x1 = ld3(qp, qs, node);
        const d3 nn = ld3(qn, qs, node);
#if MCPT_BAND_DIAG
        const unsigned long long t0 = wall_clock64();
#endif
        const bool root = clst && node >= root_off;
        const int px = root ? qpixel[node] : -1;
        const double* cum = wsc;  // the running sums searched by the pick
        double run = 0;           // the reference's weights_sum, in its order (wave-uniform)
        int ncand = 0, surv = -1;
        bool claimed = false;
        if (root) {
            ncand = cinfo[px].y;
            if (RL.slot) {
                const int sv = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(RL.slot + 16 + px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                bool later = false;  // another wave of this launch has the pixel (claimed or already stored)
                if (sv >= 0 && (sv >> 20) < RL.launch) {  // stored by an earlier launch of this call
                    cum = RL.pool + (size_t)(sv & 0xfffff) * RL.stride;
                    run = cum[lstride];
                } else if (sv == -1) {
                    int old = 0;
                    if (lane == 0) old = atomicCAS(RL.slot + 16 + px, -1, -2);
                    old = __shfl(old, 0);
                    claimed = old == -1;
                    later = !claimed && old != -3;
                } else {
                    later = sv != -3;
                }
                // MCPT_EXACT_DEFER: rather than redo the literal sums another wave of this launch is computing,
                // the root waits for the follow-up launch (defer list), which only searches them
                if (later && defer) {
                    if (lane == 0) defer[kExactHead + atomicAdd(defer, 1)] = node;
                    continue;
                }
            }
        }
        if (cum == wsc) {
            if (root) {  // a root: its pixel's cached candidate list
#if MCPT_BAND_DIAG  // exact roots per pixel, in the scratch's unused last quarter
                if (lane == 0) atomicAdd(reinterpret_cast<int*>(scratch + (size_t)waves * nlp * 3 / 2) + px, 1);
#endif
                for (int k = lane; k < ncand; k += 64) lst[k] = clst[(size_t)px * lstride + k];
            } else if (masks && node < nmask) {  // the node's candidate words
                const uint64_t* mrow = masks + (size_t)node * mask_stride(nchunks);
                for (int c = 0; c < nchunks; c++) {
                    const uint64_t m = mrow[c];
                    if ((m >> lane) & 1) lst[ncand + __popcll(m & ((1ull << lane) - 1))] = 64 * c + lane;
                    ncand += __popcll(m);
                }
            } else {
                for (int c = 0; c < S.NL; c += 64) {  // cheap stages, candidates compacted in index order
                    const int li = c + lane;
                    bool cand = false;
                    if (li < S.NL) {
                        const double4 ln = S.lt_n[li];
                        cand = light_cheap_stage(f3(S.lt_v[3 * li]), f3(S.lt_v[3 * li + 1]), f3(S.lt_v[3 * li + 2]),
                                                 mk3(ln.x, ln.y, ln.z), x1, nn) == 0;
                    }
                    const uint64_t m = __ballot(cand);
                    if (cand) lst[ncand + lane_rank(m)] = li;
                    ncand += __popcll(m);
                }
            }
            wave_lds_sync();
#if MCPT_BAND_DIAG
            const unsigned long long t1 = wall_clock64();
#endif
            for (int k0 = 0; k0 < ncand; k0 += 64) {  // the literal full stage, 64 candidates at a time
                const int k = k0 + lane;
                if (k < ncand) {
                    const int li = lst[k];
                    const double4 ln = S.lt_n[li];
                    SphTri o;
                    const int st = light_tri_stage(f3(S.lt_v[3 * li]), f3(S.lt_v[3 * li + 1]), f3(S.lt_v[3 * li + 2]),
                                                   mk3(ln.x, ln.y, ln.z), S.light_sum[li], x1, nn, &o);
                    wsc[k] = st == 0 ? o.w : -1.0;
                }
            }
            wave_lds_sync();
#if MCPT_BAND_DIAG
            const unsigned long long t2 = wall_clock64();
            if (lane == 0 && stats) {
                atomicAdd(stats + 12, t1 - t0);
                atomicAdd(stats + 13, t2 - t1);
            }
#endif
            surv = 0;
            for (int k0 = 0; k0 < ncand; k0 += 64) {
                const bool in = k0 + lane < ncand;
                const double w = in ? wsc[k0 + lane] : -1.0;
                const bool ok = w >= 0.0;
                surv += __popcll(__ballot(ok));
                const double wz = ok ? w : 0.0;
                double mine = 0.0;
#pragma unroll 8
                for (int q = 0; q < 64; q++) {
                    run += readlane_f64(wz, q);
                    mine = lane == q ? run : mine;
                }
                if (in) wsc[k0 + lane] = ok ? mine : -1.0;  // running sum after this survivor, -1 if culled
            }
            wave_lds_sync();
            if (claimed) {  // publish this pixel's sums for the later launches of the call
                int e = 0;
                if (lane == 0) e = atomicAdd(RL.slot, 1);
                e = __shfl(e, 0);
                if (e < RL.cap) {
                    double* dst = RL.pool + (size_t)e * RL.stride;
                    for (int k = lane; k < ncand; k += 64) dst[k] = wsc[k];
                    if (lane == 0) dst[lstride] = run;
                }
                if (lane == 0) atomicExch(RL.slot + 16 + px, e < RL.cap ? (RL.launch << 20) | e : -3);
            }
        }
#if MCPT_BAND_DIAG
        const unsigned long long t3 = wall_clock64();
#endif
        int pick = -1;
        if (!(fabs(run) < MCPT_EPS)) {
            const double u = u_override ? u_override[node]
                                        : counter_u(counter_key(seed, (uint64_t)qpixel[node], (uint64_t)qsample[node], qnode[node]), 1);
            const double target = u * run;
            int found = -1, last = -1;
            for (int k0 = 0; k0 < ncand && found < 0; k0 += 64) {
                const bool in = k0 + lane < ncand;
                const double rv = in ? cum[k0 + lane] : -1.0;
                const uint64_t hm = __ballot(rv >= 0.0 && rv >= target);
                const uint64_t sm = __ballot(rv >= 0.0);
                if (hm) found = k0 + __ffsll((unsigned long long)hm) - 1;
                if (sm) last = k0 + 63 - __clzll((long long)sm);
            }
            const int at = found >= 0 ? found : last;
            if (at >= 0) pick = root ? (int)clst[(size_t)px * lstride + at] : lst[at];
        }
        if (lane == 0) {
            wsum_out[node] = run;
            pick_out[node] = pick;
            if (count_out) count_out[node] = surv >= 0 ? surv : cinfo[px].z;
#if MCPT_BAND_DIAG  // wall-clock ticks (100 MHz) summed over nodes: lists, literal (above), sum + pick
            if (stats) {
                const unsigned long long t4 = wall_clock64();
                atomicAdd(stats + 14, t3 - t0);
                atomicAdd(stats + 15, t4 - t3);
            }
#endif
        }
        wave_lds_sync();
    }
}
// diagnostics (mcpt_debug_light_literal): the literal chain's intermediates for every light at one point,
// 20 doubles per light: stage, A, B, C (after the orientation swap), a, b, c, alpha, beta, gamma, sA, w
__global__ void k_light_literal(DScene S, d3 x1, d3 nn, double* out) {
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= S.NL) return;
    const double4 ln = S.lt_n[li];
    const d3 p0 = f3(S.lt_v[3 * li]), p1 = f3(S.lt_v[3 * li + 1]), p2 = f3(S.lt_v[3 * li + 2]);
    double* o = out + 20 * (size_t)li;
    for (int k = 0; k < 20; k++) o[k] = 0;
    SphTri t;
    o[0] = light_tri_stage(p0, p1, p2, mk3(ln.x, ln.y, ln.z), S.light_sum[li], x1, nn, &t);
    // recompute the angles the same way (light_tri_stage keeps only alpha, c)
    d3 A = normalized(sub(p0, x1)), B = normalized(sub(p1, x1)), C = normalized(sub(p2, x1));
    if (dot(cross(normalized(sub(C, A)), normalized(sub(B, A))), nn) < 0) {
        const d3 tt = B;
        B = C;
        C = tt;
    }
    o[1] = A.x, o[2] = A.y, o[3] = A.z, o[4] = B.x, o[5] = B.y, o[6] = B.z, o[7] = C.x, o[8] = C.y, o[9] = C.z;
    o[10] = acos_cr(fmax(-1.0, fmin(1.0, dot(B, C))));
    o[11] = acos_cr(fmax(-1.0, fmin(1.0, dot(A, C))));
    o[12] = acos_cr(fmax(-1.0, fmin(1.0, dot(A, B))));
    o[13] = acos_cr(fmax(-1.0, fmin(1.0, -dot(normalized(cross(B, A)), normalized(cross(A, C))))));
    o[14] = acos_cr(fmax(-1.0, fmin(1.0, -dot(normalized(cross(C, B)), normalized(cross(B, A))))));
    o[15] = acos_cr(fmax(-1.0, fmin(1.0, -dot(normalized(cross(A, C)), normalized(cross(C, B))))));
    o[16] = o[13] + o[14] + o[15] - MCPT_PI;
    o[17] = o[0] == 0 ? t.w : -1.0;
    o[18] = -dot(normalized(cross(B, A)), normalized(cross(A, C)));  // alpha's acos argument
    o[19] = dot(B, C);
}
// scratch doubles k_prep_exact needs (per wave: weights + list)
inline size_t exact_scratch_doubles(int NL) { return (size_t)exact_waves(NL) * 2 * (size_t)((NL + 63) & ~63); }

// ---- MIS node split into three kernels (ray generation / traversal / combination) -------------
// (one MIS node per lane with three inlined traversals measured 152 VGPRs, 3 waves/SIMD.)  Split,
// the traversal kernel runs at high occupancy on a short LDS stack, and the shading kernels carry
// no traversal state.  Per node in `Aux` (capacity = queue capacity):
//   d1, d2   light / BRDF directions (3 doubles each)
//   w1       tp * f(wl) * cos / (p_light + p_phong) / 0.6  -- the light child's throughput
//   w2       tp * f(wi); c2 = (pdf, cos) of the BRDF sample -- the BRDF child's throughput needs
//            the light pdf of the light-only hit (main.cpp:482-487)
//   flags    bit 0 trace d1, bit 1 trace d2, bit 2 trace d2 against the light BVH
//   hf/hbg   ray set k in [k*cap, (k+1)*cap): hit facet, (beta, gamma)
struct Aux {
    double *d1, *d2, *w1, *w2, *c2, *hbg, *s1;
    int *flags, *hf;
    int cap;
};

// ---- shade_with_mis as a bottom-up tree reduction (the reference's stale light pdf) ------------
// The reference evaluates the BRDF branch's light pdf with the light sampler's state after the
// light branch's recursion: the prep of the LAST node that ran one in DFS order inside the light
// child's subtree (main.cpp:443 vs :487, Mylight.cpp:484-493).  That node is the end of the path
// from the light child that steps to the BRDF child when it is a shading node (passes entry + RR),
// else to the light child when it is, else stops -- known only once the subtree below has been
// expanded.  So the radiance is reduced bottom-up, as the reference's recursion returns it: a node
// with shading children holds a slot until both have reported their radiance and their path end's
// prep state (x, N, weights_sum); then L = L_light + L_brdf with the reference's operation order
// (main.cpp:464, :491) and the node reports to its parent (the root splats L / spp).  Expansion is
// unchanged (it needs no weights), so the wavefront stays as wide as before.
// A slot's fields that k_mis_combine writes together and k_mis_complete reads together share one
// 128-B record (one line per slot instead of five scattered int arrays plus an 80-B w straddling two
// lines; slot ids from the free ring are random, so every field touched costs a line):
//   int [0] par  parent code: slot * 4 + role * 2 (0 light, 1 BRDF child) + need; -1 = root (need: some
//                ancestor will evaluate a light pdf at this subtree's path-end state)
//   int [1] pix  pixel (root splat)
//   int [2] fl   bit0 light child shading, bit1 BRDF child shading, bit2 BRDF child emitter, bit3 BRDF
//                edge, bit4 this node's path-end state is needed (its own parent code's need bit)
//   int [3] li   light triangle along the BRDF direction (light-only ray) or -1
//   double [2, 12)  w: brdf of the light edge [3], its scalar s1, brdf of the BRDF edge [3], pdf, cos, s2
//   double [12, 15) Lb: BRDF child's radiance (or its emitter's emission)
constexpr int kSlotRec = 16;  // doubles per slot record
struct Slots {
    double* rec;   // kSlotRec doubles per slot (above)
    int* pend;     // shading children still to report (atomics: its own array)
    double* Ll;    // 3: light child's radiance (or the light edge's finished contribution)
    double* last;  // 14: path-end prep state (x, N, weights_sum) reported by the light / BRDF child
    // Allocation, freeing and the ready lists are split over kSlotShards shards, each with its own
    // counters on its own 64-B line: a single counter word saturates at ~88 atomics/us
    // (MI355X_MICROARCH.md), and a generation makes ~10^5 of these appends.  Slot ids carry their
    // allocating shard in the low bits (bump allocation: local << 5 | shard); a workgroup allocates
    // from shard blockIdx & 31, a wave frees and appends to shard (global wave index) & 31.
    int* ring;     // per shard: free slot ids (FIFO), rcap_ring entries each
    int* ready0;   // per shard: slots whose children have all reported, rcap_ready entries each (parity 0)
    int* ready1;   //   (parity 1)
    unsigned* ctrl;  // per shard, 16 words: [0] bump [1] ring head [2] ring tail [3] ring end this pass [4..5] ready counts
    int cap;       // slot ids < cap (= rcap << 5)
    int rcap;      // slots per shard
    int ring_cap, ready_cap;  // entries per shard of ring / ready lists
};
constexpr int kSlotShards = 32;
constexpr int kCtrlBytes = kSlotShards * 16 * 4;
__device__ inline int wave_shard() {  // the shard of this wave (global wave index)
    return (int)((blockIdx.y * gridDim.x + blockIdx.x) * ((blockDim.x + 63) >> 6) + (threadIdx.x >> 6)) & (kSlotShards - 1);
}

// the light pdf of light triangle li at a prep state (x, N, weights_sum) -- Mylight.cpp:484-493: sum L
// / weights_sum if li survived that prep, else 0.  Survival by the reference's literal cull chain
// (light_tri_eval: acos-based edge and vertex angles, alpha + beta + gamma - pi >= 0), not the
// prep's Van Oosterom-Strackee form: the two agree except on spherical triangles of ~zero area
// (seen edge-on, e.g. on a sphere light's silhouette), whose weight is negligible in weights_sum but
// whose survival decides whether this pdf is sum L / weights_sum or 0 -- one triangle per node, so
// the exact chain is cheap here.
__device__ inline double state_light_pdf(const DScene& S, int li, const double* st) {
    if (li < 0 || fabs(st[6]) < MCPT_EPS) return 0.0;
    const d3 x = mk3(st[0], st[1], st[2]), N = mk3(st[3], st[4], st[5]);
    const PrepLight L = load_light(S, li);
    // the literal chain only where the quick test cannot decide (slivers, near-degenerate triangles)
    const double lsum = S.light_sum[li];
    const int q = literal_survival_quick(L.p0, L.p1, L.p2, L.nl, lsum, x, N);
    if (q > 0 || (q < 0 && light_tri_eval(L.p0, L.p1, L.p2, L.nl, lsum, x, N, nullptr)))
        return lsum / st[6];
    return 0.0;
}

// a finished node reports radiance L -- and, when its parent code's need bit asks for it, its path-end
// state st -- to its parent slot; the parent goes to ready list rp once both children have (one
// append per wave: a single counter word saturates at ~88 atomics/us, MI355X_MICROARCH.md); a root
// adds L / spp to its pixel.  Every lane of the wave that reaches the call must make it.
__device__ inline void mis_report(const Params& P, const Slots& T, bool act, int par, int pixel, d3 L, const double* st,
                                  int rp) {
    bool ready = false;
    int ps = 0;
    if (act && par < 0) {
        // a zero component adds nothing (the framebuffer is never -0), so its device-scope fp64 atomic
        // is skipped -- the same image bit for bit
        double* px = P.fb + 3 * (size_t)pixel;
        if (L.x != 0.0) unsafeAtomicAdd(px + 0, L.x * P.inv_spp);
        if (L.y != 0.0) unsafeAtomicAdd(px + 1, L.y * P.inv_spp);
        if (L.z != 0.0) unsafeAtomicAdd(px + 2, L.z * P.inv_spp);
    } else if (act) {
        ps = par >> 2;
        const int role = (par >> 1) & 1;
        double* dl = role ? T.rec + kSlotRec * (size_t)ps + 12 : T.Ll + 3 * (size_t)ps;
        dl[0] = L.x, dl[1] = L.y, dl[2] = L.z;
        if (par & 1) {
            double* ds = T.last + 14 * (size_t)ps + 7 * role;
#pragma unroll
            for (int k = 0; k < 7; k++) ds[k] = st[k];
        }
        // the parent's fields are read by a LATER kernel (the next k_mis_complete), so kernel
        // boundaries order these stores before those reads; only the count needs an atomic
        ready = atomicSub(&T.pend[ps], 1) == 1;
    }
    const int sh = wave_shard();
    const int q = wave_append(&T.ctrl[16 * sh + 4 + rp], ready);
    if (ready) (rp ? T.ready1 : T.ready0)[(size_t)sh * T.ready_cap + q] = ps;
}

// The seed of a light ray (p, wl) aimed at light facet fac: tri_hit's t for that facet (a hit the
// closest-hit query must accept unless it is the origin facet), else -1.  Written by the generation
// kernels into the set-0 hit slot A.hbg[2 i], read by k_mis_rays before it overwrites the slot.
// (A/B: -DMCPT_SEED_LIGHT=0)
#ifndef MCPT_SEED_LIGHT
#define MCPT_SEED_LIGHT 1
#endif
__device__ inline double seed_light_t(const DScene& S, int fac, int origin, d3 p, d3 wl) {
    if (!MCPT_SEED_LIGHT || fac < 0 || fac == origin) return -1;
    const TriHit h = tri_hit(f3(S.tri_v[3 * fac]), f3(S.tri_v[3 * fac + 1]), f3(S.tri_v[3 * fac + 2]), p, wl);
    return h.hit ? h.t : -1;
}

// kStale: the tree-reduction form (Slots) -- w1 / w2 hold the edges' BRDF values and s1 the light
// edge's scalar, applied bottom-up; else w1 / w2 are forward throughputs (fresh-pdf path)
template <bool kStale>
__global__ __launch_bounds__(256, MCPT_LB_GEN) void k_mis_gen(Params P, Queue cur, int n, Aux A) {
    const DScene& S = P.S;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const d3 p = ld3(cur.p, cur.cap, i);
    const d3 N = ld3(cur.n, cur.cap, i);
    const uint64_t key = counter_key(P.seed, (uint64_t)cur.pixel[i], (uint64_t)cur.sample[i], cur.node[i]);
    const double wsum = cur.wsum[i];
    const int pick = cur.pick[i];
    int flags = 0;
    // ---- light branch (main.cpp:443-466); the BRDF inputs are loaded after it (the picked light's
    // literal chain is the register peak: 132 -> 116 VGPRs, 3 -> 4 waves per SIMD) ----
    d3 coord;
    double lprob = 1;
    if (pick >= 0) {
        SphTri sph;
        pick_sph(S, pick, p, N, &sph);
        const d3 Pd = arvo_sample(sph, counter_u(key, 2), counter_u(key, 3));
        TriHit th = tri_hit(f3(S.lt_v[3 * pick]), f3(S.lt_v[3 * pick + 1]), f3(S.lt_v[3 * pick + 2]), p, Pd);
        coord = add(p, mul(Pd, th.hit ? th.t : 0.0));  // miss: t = 0 (Mylight.cpp:475-481)
        lprob = S.light_sum[pick] / wsum;
    } else {
        coord = add(mul(N, -1), p);  // Mylight.cpp:427-430
    }
    const d3 wl = normalized(sub(coord, p));
    const d3 wo = ld3(cur.wo, cur.cap, i);
    const d3 tp = ld3(cur.tp, cur.cap, i);
    const int f = cur.f[i];
    const float* m = S.mtl + 7 * S.tri_mat[f];
    const d3 kd = mk3(m[0], m[1], m[2]), ks = mk3(m[3], m[4], m[5]);
    const double sh = m[6];
    d3 w1 = mk3(0, 0, 0);
    double s1 = 0;
    if (dot(wl, N) > 0) {
        flags |= 1;
        A.hbg[2 * (size_t)i] = seed_light_t(S, pick >= 0 ? S.light_facet[pick] : -1, f, p, wl);
        const d3 b = brdf_phong(N, wl, wo, kd, ks, sh);
        const double pp = phong_pdf(N, wl, wo, kd, ks, sh);
        s1 = dot(wl, N) / (lprob + pp) / MCPT_P_RR;
        w1 = kStale ? b : mul(hmul(tp, b), s1);
    }
    // ---- BRDF branch (main.cpp:469-493) ----
    double pdf;
    const d3 wi = sample_phong(N, wo, kd, ks, sh, counter_u(key, 4), counter_u(key, 5), counter_u(key, 6), &pdf);
    d3 w2 = mk3(0, 0, 0);
    if (!(dot(wi, N) < 0)) {
        flags |= 2;
        if (!(fabs(wsum) < MCPT_EPS)) flags |= 4;  // light pdf can only be nonzero with a light set
        w2 = kStale ? brdf_phong(N, wi, wo, kd, ks, sh) : hmul(tp, brdf_phong(N, wi, wo, kd, ks, sh));
    }
    st3(A.d1, A.cap, i, wl);
    st3(A.d2, A.cap, i, wi);
    st3(A.w1, A.cap, i, w1);
    st3(A.w2, A.cap, i, w2);
    A.c2[2 * i] = pdf, A.c2[2 * i + 1] = dot(wi, N);
    if (kStale) A.s1[i] = s1;
    A.flags[i] = flags;
}

#ifndef MCPT_RAYS_LAZY_BG
#define MCPT_RAYS_LAZY_BG 1
#endif
// closest hits of ray set blockIdx.y (0: d1, 1: d2, 2: d2 against the light-only BVH) from the
// queue's shading points, excluding the origin facet
// kCount: counts node visits / triangle tests into cnt[0] / cnt[1] (statistics replay only)
template <bool kGrid, bool kCount = false>
__global__ __launch_bounds__(kRayBlock, MCPT_LB_RAYS) void k_mis_rays(DScene S, Queue cur, int n, Aux A, int first_set,
                                                          unsigned long long* cnt = nullptr, int seeded = 0,
                                                          int compact = 0) {
    constexpr int kTop = kGrid ? 0 : kRayTop;
    __shared__ int stack[kRayTopLds * kRayBlock];
    __shared__ BvhNode4 top[kTop > 0 ? kTop : 1];
    const int set = blockIdx.y + first_set;
    // compact (shade() modes): the block's nodes regrouped stably -- the nodes that trace this set
    // first, in their order, the others in the block's last waves, which then exit at once.  shade-area
    // +6% (its light rays are traced by a minority of nodes); MIS, whose three sets are traced densely or
    // by half of the nodes, ran 3.5% slower traversal with it (profiles/round4_ab_cull_classes.txt)
    __shared__ int s_wc[kRayBlock / 64][2], s_off[kRayBlock / 64][2], s_ord[kRayBlock];
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (compact) {  // uniform
        const int i0 = i;
        const int key = i0 < n && (A.flags[i0] & (1 << set)) ? 0 : 1;
        const int w = threadIdx.x >> 6;
        const uint64_t m0 = __ballot(key == 0);
        const int rank = key == 0 ? lane_rank(m0) : lane_rank(~m0);
        if (lane_id() == 0) {
            s_wc[w][0] = __popcll(m0);
            s_wc[w][1] = 64 - __popcll(m0);
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // offsets: traced nodes first, waves in order within a key
            int t = 0;
            for (int b = 0; b < 2; b++)
                for (int ww = 0; ww < kRayBlock / 64; ww++) {
                    s_off[ww][b] = t;
                    t += s_wc[ww][b];
                }
        }
        __syncthreads();
        s_ord[s_off[w][key] + rank] = i0;
        __syncthreads();
        i = s_ord[threadIdx.x];
    }
    if (kTop > 0) {  // the tree's top levels into LDS (uniform per block: blockIdx.y picks the tree)
        const BvhNode4* src = set == 2 ? S.lbvh4 : S.bvh4;
        const int cnt4 = min(kTop, set == 2 ? S.nlbvh4 : S.nbvh4) * (int)(sizeof(BvhNode4) / sizeof(float4));
        for (int k = threadIdx.x; k < cnt4; k += blockDim.x)
            reinterpret_cast<float4*>(top)[k] = reinterpret_cast<const float4*>(src)[k];
        __syncthreads();
    }
    if (!kCount && i >= n) return;
    const int fl = i < n ? A.flags[i] : 0;
    int f = -1;
    double beta = 0, gamma = 0;
    unsigned visits = 0, tests = 0, witer = 0, wleaf = 0;
    if (fl & (1 << set)) {
        const double* d = set == 0 ? A.d1 : A.d2;
        const d3 ro = ld3(cur.p, cur.cap, i);
        const d3 rd = ld3(d, A.cap, i);
        const float4* leafv = set == 2 ? S.lleaf_v : S.leaf_v;  // uniform per block
        Hit h;
        if (kGrid)
            h = grid_trace(S, ro, rd, cur.f[i], set == 2);
        else {
            // set 0 aims at a sampled light triangle: the generation kernel left that triangle's
            // exact t along the ray in the set-0 hit slot (seed_light_t), so boxes behind the light
            // are pruned from the start
            float tl0 = FLT_MAX;
            if (set == 0 && (seeded & 1)) {
                const double t0 = A.hbg[2 * ((size_t)set * A.cap + i)];
                if (t0 > 0) tl0 = (float)t0 * 1.0001f + 1e-5f;
            }
            h = trace4_ww<kRayTopLds, kCount, kTop, MCPT_FILTER_MIS, MCPT_RAYS_LAZY_BG>(set == 2 ? S.lbvh4 : S.bvh4, leafv, ro, rd, cur.f[i],
                                                    stack + threadIdx.x, kRayBlock, &visits, &tests, top, tl0, &witer, &wleaf);
        }
        f = h.f;
        beta = h.beta;
        gamma = h.gamma;
    }
    if (kCount) {
        wave_count2(cnt, visits, cnt + 1, tests);
        if (MCPT_TRACE_DIAG) wave_count2(cnt + 6, witer, cnt + 7, wleaf);
        if (i >= n) return;
    }
    // only a traced set's slots are written (its consumers test the node's flags first), and (beta,
    // gamma) only for a hit: 4 B per miss instead of 20 B per node and set
    if (fl & (1 << set)) {
        const size_t o = (size_t)set * A.cap + i;
        A.hf[o] = f;
        if (set < 2 && f >= 0) {
            A.hbg[2 * o] = beta;
            A.hbg[2 * o + 1] = gamma;
        }
    }
}

// workgroup-aggregated slot allocation (ring entries freed by earlier passes first, then new slots from the
// bump counter) and k_mis_combine's two child appends (light children first, then BRDF children, as two
// block_append calls would order them) in ONE barrier phase: the workgroup's three counts are reduced
// together and thread 0 issues the queue atomic and the slot-ring atomics back to back, so the workgroup
// waits for one round of device-scope atomics instead of three.  Must be called by ALL threads.
__device__ inline void block_alloc_slot_push2(const Slots& T, bool want, bool push1, bool push2, unsigned* qcount, int* slot_out,
                                              int* q1_out, int* q2_out) {
    __shared__ unsigned s_cnt[3][16];
    __shared__ unsigned s_base, s_ring, s_bump, s_q;
    const int lane = lane_id(), wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const uint64_t m = __ballot(want), m1 = __ballot(push1), m2 = __ballot(push2);
    if (lane == 0) s_cnt[0][wid] = (unsigned)__popcll(m), s_cnt[1][wid] = (unsigned)__popcll(m1), s_cnt[2][wid] = (unsigned)__popcll(m2);
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned tot[3] = {0, 0, 0};
        for (int k = 0; k < 3; k++)
            for (int w = 0; w < nw; w++) {
                const unsigned c = s_cnt[k][w];
                s_cnt[k][w] = tot[k];
                tot[k] += c;
            }
        for (int w = 0; w < nw; w++) s_cnt[2][w] += tot[1];  // BRDF children after all light children
        const unsigned np = tot[1] + tot[2];
        unsigned q = 0, base = 0, from_ring = 0, bump = 0;
        unsigned* c = T.ctrl + 16 * (blockIdx.x & (kSlotShards - 1));
        if (np) q = atomicAdd(qcount, np);
        if (tot[0]) {
            base = atomicAdd(&c[1], tot[0]);
            const unsigned end = c[3];
            from_ring = base >= end ? 0u : min(tot[0], end - base);
            if (tot[0] > from_ring) bump = atomicAdd(&c[0], tot[0] - from_ring);
        }
        s_base = base, s_ring = from_ring, s_bump = bump, s_q = q;
    }
    __syncthreads();
    const uint64_t below = lane == 0 ? 0ull : ((~0ull) >> (64 - lane));
    const unsigned j = s_cnt[0][wid] + (unsigned)__popcll(m & below);
    const int sh = blockIdx.x & (kSlotShards - 1);
    int slot = -1;
    if (want)
        slot = j < s_ring ? T.ring[(size_t)sh * T.ring_cap + (s_base + j) % (unsigned)T.ring_cap]
                          : (int)(((s_bump + (j - s_ring)) << 5) | (unsigned)sh);
    *slot_out = slot;
    *q1_out = push1 ? (int)(s_q + s_cnt[1][wid] + (unsigned)__popcll(m1 & below)) : -1;
    *q2_out = push2 ? (int)(s_q + s_cnt[2][wid] + (unsigned)__popcll(m2 & below)) : -1;
    __syncthreads();
}

// The same three ray sets as k_mis_rays, traced by PERSISTENT waves that refill lanes whose ray has
// finished with the next ray of a shared pool (Aila & Laine's persistent while-while with dynamic
// ray fetch): a wave of one-ray-per-lane runs as long as its longest ray, and rays differ ~10x in
// length (and a ray set's untraced nodes leave lanes idle from the start).  Pool item t = set-major
// (t / n = set - first_set, t % n = node); a wave fetches items for all its idle lanes with one
// atomic once at least kRefill lanes are idle; items whose set is not flagged for their node are
// answered (-1) at once.  Each round is one iteration of trace4_ww's outer loop for every lane in
// flight; the per-lane state (ray, stack pointer, LDS + private stack, best hit) lives across
// rounds.  Hits are bit-identical to k_mis_rays (the closest hit, ties to the lower facet id, by the
// same tests on conservatively pruned boxes); only the order of visits, and so their count, differs.
#ifndef MCPT_RAYS_REFILL
#define MCPT_RAYS_REFILL 8  // A/B on Cornell-1M: 16 -> 1220, 8 -> 1231-1237, 4 -> 1203, 32 -> 1179 (profiles/round2b_ab_rays_persistent.txt)
#endif
constexpr int kRefill = MCPT_RAYS_REFILL;
#ifndef MCPT_PERSIST_LDS
#define MCPT_PERSIST_LDS 16  // LDS stack entries per lane of k_rays_persistent (private stack beyond)
#endif
constexpr int kPersistLds = MCPT_PERSIST_LDS;
#ifndef MCPT_RAY_CHUNK
#define MCPT_RAY_CHUNK 256
#endif
constexpr int kRayChunk = MCPT_RAY_CHUNK;  // pool items a wave takes per atomic
template <bool kCount = false>
#ifndef MCPT_RAYS_WAVES
#define MCPT_RAYS_WAVES 6
#endif
__global__ __launch_bounds__(kRayBlock, MCPT_RAYS_WAVES) void k_rays_persistent(DScene S, Queue cur, int n, Aux A, int first_set,
                                                                  int nsets, unsigned* __restrict__ pool,
                                                                  unsigned long long* cnt = nullptr, int seeded = 0) {
    constexpr int kDone = 0x7fffffff;
    __shared__ int stack[kPersistLds * kRayBlock];
    int* __restrict__ lds = stack + threadIdx.x;
    constexpr int stride = kRayBlock;
    const int lane = threadIdx.x & 63;
    const unsigned total = (unsigned)nsets * (unsigned)n;
    int spill[kStack - kPersistLds];
    unsigned visits = 0, tests = 0, witer = 0, wleaf = 0;
    bool busy = false, exhausted = false;
    unsigned wnext = 0, wend = 0;  // the wave's private range of pool items (wave-uniform)
    int set = 0, ii = 0, excl = -1;
    d3 ro = mk3(0, 0, 0), rd = mk3(0, 0, 0);
    float ix = 0, iy = 0, iz = 0, oix = 0, oiy = 0, oiz = 0, tlimit = FLT_MAX;
    int sp = 0, node = kDone, leaf = 0;
    Hit best{-1, DBL_MAX, 0, 0};
    auto push = [&](int v) {
        if (sp < kPersistLds) lds[sp * stride] = v;
        else if (sp < kStack) spill[sp - kPersistLds] = v;
        sp = sp < kStack ? sp + 1 : sp;
    };
    auto pop = [&]() -> int {
        if (sp == 0) return kDone;
        --sp;
        return sp < kPersistLds ? lds[sp * stride] : spill[sp - kPersistLds];
    };
    auto finish = [&]() {  // the lane's traced ray is done: store its hit ((beta, gamma) only for a hit)
        const size_t o = (size_t)set * A.cap + ii;
        A.hf[o] = best.f;
        if (set < 2 && best.f >= 0) {
            A.hbg[2 * o] = best.beta;
            A.hbg[2 * o + 1] = best.gamma;
        }
        busy = false;
    };
    while (true) {
        // refill the idle lanes (all of them at the start, then whenever kRefill are idle) from the
        // wave's private chunk of kRayChunk consecutive items; one pool atomic per chunk (a single
        // counter word saturates at ~88 atomics per us)
        while (!exhausted) {
            const uint64_t idle = __ballot(!busy);
            if (idle == 0 || (__popcll(idle) < kRefill && __ballot(busy) != 0)) break;
            if (wnext >= wend) {
                unsigned base = 0;
                if (lane == 0) base = atomicAdd(pool, (unsigned)kRayChunk);
                base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
                if (base >= total) {
                    exhausted = true;
                    break;
                }
                wnext = base;
                wend = min(base + (unsigned)kRayChunk, total);
            }
            const unsigned take = min((unsigned)__popcll(idle), wend - wnext);
            const unsigned rk = (unsigned)lane_rank(idle);
            const unsigned base = wnext;
            wnext += take;
            if (!busy && rk < take) {
                const unsigned it = base + rk;
                {
                    set = first_set + (int)(it / (unsigned)n);
                    ii = (int)(it % (unsigned)n);
                    best = Hit{-1, DBL_MAX, 0, 0};
                    if (A.flags[ii] & (1 << set)) {
                        const double* d = set == 0 ? A.d1 : A.d2;
                        ro = ld3(cur.p, cur.cap, ii);
                        rd = ld3(d, A.cap, ii);
                        excl = cur.f[ii];
                        if (isnan(rd.x) || isnan(rd.y) || isnan(rd.z)) {  // reference: UB (Myobj.cpp:463-468)
                            finish();
                        } else {
                            auto inv = [](double v) {
                                float f = (float)v;
                                if (fabsf(f) < 1e-30f) f = copysignf(1e-30f, f);
                                return 1.0f / f;
                            };
                            ix = inv(rd.x), iy = inv(rd.y), iz = inv(rd.z);
                            oix = (float)ro.x * ix, oiy = (float)ro.y * iy, oiz = (float)ro.z * iz;
                            tlimit = FLT_MAX;
                            // set 0: the light triangle's exact t (seed_light_t)
                            if (set == 0 && (seeded & 1)) {
                                const double t0 = A.hbg[2 * ((size_t)set * A.cap + ii)];
                                if (t0 > 0) tlimit = (float)t0 * 1.0001f + 1e-5f;
                            }
                            sp = 0;
                            node = 0;
                            leaf = 0;
                            busy = true;
                        }
                    } else {
                        busy = false;  // this set is not traced for this node: nothing to store
                    }
                }
            }
        }
        if (__ballot(busy) == 0) break;  // pool exhausted and no ray in flight
        // one round of trace4_ww's outer loop on every lane in flight
        if (busy) {
            const BvhNode4Q* __restrict__ nodes = set == 2 ? S.lbvh4q : S.bvh4q;
            const float4* __restrict__ leafv = set == 2 ? S.lleaf_v : S.leaf_v;
            const float inv3[3] = {ix, iy, iz}, oi3[3] = {oix, oiy, oiz};
            const bool neg3[3] = {ix < 0, iy < 0, iz < 0};
            while (node >= 0 && node != kDone) {
                if (kCount) ++visits;
                if (kCount && MCPT_TRACE_DIAG && (int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) ++witer;
                float tn[3][4], tf[3][4];  // near / far slab distances per axis and child
                int chs[4];
                node_tplanes(nodes + node, inv3, oi3, neg3, tn, tf, chs);
                float t[4];
                int code[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float t0 = fmaxf(fmaxf(tn[0][k], tn[1][k]), fmaxf(tn[2][k], 0.0f));
                    const float t1 = fminf(fminf(tf[0][k], tf[1][k]), fminf(tf[2][k], tlimit));
                    // empty slots keep their test here: a quantized empty slot's planes (255, 0) can
                    // fall inside the margin when the node's scale is tiny
                    const bool h = chs[k] != kBvh4Empty && t0 <= fmaf(t1, 1.00001f, 1e-6f);
                    t[k] = h ? t0 : FLT_MAX;
                    code[k] = h ? chs[k] : kDone;
                }
                auto cs = [&](int a, int b) {
                    const bool sw = t[b] < t[a];
                    const float ta = t[a], tb = t[b];
                    const int ca = code[a], cb = code[b];
                    t[a] = sw ? tb : ta, t[b] = sw ? ta : tb;
                    code[a] = sw ? cb : ca, code[b] = sw ? ca : cb;
                };
                cs(0, 1), cs(2, 3), cs(0, 2), cs(1, 3), cs(1, 2);
                if (code[3] != kDone) push(code[3]);
                if (code[2] != kDone) push(code[2]);
                if (code[1] != kDone) push(code[1]);
                node = code[0] != kDone ? code[0] : pop();
                if (node < 0 && leaf >= 0) {  // postpone the leaf, keep descending
                    leaf = node;
                    node = pop();
                }
                if (!__any(leaf >= 0)) break;
            }
            while (leaf < 0) {
                const int packed = ~leaf, first = packed >> kLeafBits, cnt4 = packed & ((1 << kLeafBits) - 1);
                for (int q = first; q < first + cnt4; q++) {
                    if (kCount && MCPT_TRACE_DIAG && (int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) ++wleaf;
                    const float4 a4 = leafv[3 * q], b4 = leafv[3 * q + 1], c4 = leafv[3 * q + 2];
                    const int fac = __float_as_int(a4.w);
                    if (fac == excl) continue;
                    if (kCount) ++tests;
                    const d3 a = f3(a4), ab = sub(a, f3(b4)), ac = sub(a, f3(c4)), ar = sub(a, ro);
                    const double detA = det3(ab, ac, rd);
                    if (fabs(detA) < MCPT_EPS) continue;
                    const double nb = det3(ar, ac, rd), ng = det3(ab, ar, rd), nt = det3(ab, ac, ar);
                    const bool neg = detA < 0;
                    if ((nb != 0 && ((nb < 0) != neg)) || (ng != 0 && ((ng < 0) != neg)) || (nt != 0 && ((nt < 0) != neg)))
                        continue;
                    const double beta = nb / detA, gamma = ng / detA, tt = nt / detA;
                    if (beta < 0 || gamma < 0 || beta + gamma > 1 || tt < 0 || fabs(tt) < MCPT_EPS) continue;
                    if (tt < best.t || (tt == best.t && fac < best.f)) {
                        best.f = fac;
                        best.t = tt;
                        best.beta = beta;
                        best.gamma = gamma;
                        tlimit = fminf(tlimit, (float)tt * 1.0001f + 1e-5f);
                    }
                }
                leaf = node;
                if (node < 0) node = pop();
            }
            if (!(node != kDone || leaf < 0)) finish();
        }
    }
    if (kCount) wave_count2(cnt, visits, cnt + 1, tests);
    if (kCount && MCPT_TRACE_DIAG) wave_count2(cnt + 6, witer, cnt + 7, wleaf);
}

// k_rays_persistent over the 8-wide compressed trees (BvhNode8Q): the same refilling persistent waves,
// pool and hit slots; a round is, for every lane in flight, node visits until the lane holds a triangle
// group (while-while: the wave descends until every lane does or has run out of nodes), then that group's
// triangles.  Hits are bit-identical to k_rays_persistent / k_mis_rays (same tests, same total order on
// (t, facet), conservative boxes); visits and their order differ.
#ifndef MCPT_RAYS_CW8
// 1: the persistent traversal uses the 8-wide trees by default.  Off: measured slower on C5 (round 5, same
// binary, profiles/round5_ab_cornell_cw8.txt): 22.1 node visits per ray instead of 30.8, but 8.0 triangle
// tests instead of 6.7 (octant order instead of sorted hits) and twice the box tests per visit --
// k_rays_cw8 5.18 vs k_rays_persistent 3.91 ms per launch, C5 1 651 vs 2 044 Msamples/s
#define MCPT_RAYS_CW8 0
#endif
#ifndef MCPT_CW8_WAVES
#define MCPT_CW8_WAVES 6
#endif
template <bool kCount = false>
__global__ __launch_bounds__(kRayBlock, MCPT_CW8_WAVES) void k_rays_cw8(DScene S, Queue cur, int n, Aux A, int first_set, int nsets,
                                                                  unsigned* __restrict__ pool, unsigned long long* cnt = nullptr,
                                                                  int seeded = 0) {
    __shared__ unsigned stack[kPersistLds * kRayBlock];
    unsigned* __restrict__ lds = stack + threadIdx.x;
    constexpr int stride = kRayBlock;
    const int lane = threadIdx.x & 63;
    const unsigned total = (unsigned)nsets * (unsigned)n;
    unsigned spill[kStack - kPersistLds];
    unsigned visits = 0, tests = 0, witer = 0, wleaf = 0;
    bool busy = false, exhausted = false;
    unsigned wnext = 0, wend = 0;
    int set = 0, ii = 0, excl = -1;
    d3 ro = mk3(0, 0, 0), rd = mk3(0, 0, 0);
    Cw8Frame F{};
    float tlimit = FLT_MAX;
    unsigned ng = 0, tw = 0;
    int tb = 0, sp = 0;
    Hit best{-1, DBL_MAX, 0, 0};
    auto push = [&](unsigned v) {
        if (sp < kPersistLds) lds[sp * stride] = v;
        else if (sp < kStack) spill[sp - kPersistLds] = v;
        sp = sp < kStack ? sp + 1 : sp;
    };
    auto pop = [&]() -> unsigned {
        --sp;
        return sp < kPersistLds ? lds[sp * stride] : spill[sp - kPersistLds];
    };
    auto finish = [&]() {
        const size_t o = (size_t)set * A.cap + ii;
        A.hf[o] = best.f;
        if (set < 2 && best.f >= 0) {
            A.hbg[2 * o] = best.beta;
            A.hbg[2 * o + 1] = best.gamma;
        }
        busy = false;
    };
    while (true) {
        while (!exhausted) {  // refill, as k_rays_persistent
            const uint64_t idle = __ballot(!busy);
            if (idle == 0 || (__popcll(idle) < kRefill && __ballot(busy) != 0)) break;
            if (wnext >= wend) {
                unsigned base = 0;
                if (lane == 0) base = atomicAdd(pool, (unsigned)kRayChunk);
                base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
                if (base >= total) {
                    exhausted = true;
                    break;
                }
                wnext = base;
                wend = min(base + (unsigned)kRayChunk, total);
            }
            const unsigned take = min((unsigned)__popcll(idle), wend - wnext);
            const unsigned rk = (unsigned)lane_rank(idle);
            const unsigned base = wnext;
            wnext += take;
            if (!busy && rk < take) {
                const unsigned it = base + rk;
                set = first_set + (int)(it / (unsigned)n);
                ii = (int)(it % (unsigned)n);
                best = Hit{-1, DBL_MAX, 0, 0};
                if (A.flags[ii] & (1 << set)) {
                    const double* d = set == 0 ? A.d1 : A.d2;
                    ro = ld3(cur.p, cur.cap, ii);
                    rd = ld3(d, A.cap, ii);
                    excl = cur.f[ii];
                    if (isnan(rd.x) || isnan(rd.y) || isnan(rd.z)) {  // reference: UB (Myobj.cpp:463-468)
                        finish();
                    } else {
                        F = cw8_frame(ro, rd);
                        tlimit = FLT_MAX;
                        if (set == 0 && (seeded & 1)) {  // set 0: the light triangle's exact t (seed_light_t)
                            const double t0 = A.hbg[2 * ((size_t)set * A.cap + ii)];
                            if (t0 > 0) tlimit = (float)t0 * 1.0001f + 1e-5f;
                        }
                        ng = cw8_root(F.oct);
                        tw = 0;
                        sp = 0;
                        busy = true;
                    }
                } else {
                    busy = false;
                }
            }
        }
        if (__ballot(busy) == 0) break;  // pool exhausted and no ray in flight
        if (busy) {
            const BvhNode8Q* __restrict__ nodes = set == 2 ? S.lbvh8 : S.bvh8;
            const float4* __restrict__ triv = set == 2 ? S.ltri8_v : S.tri8_v;
            while (true) {  // descend until every lane holds a triangle group or is out of nodes
                const bool want = tw == 0 && ((ng & 0xffu) != 0 || sp > 0);
                if (!__any(want)) break;
                if (want) {
                    if (kCount && MCPT_TRACE_DIAG && (int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) ++witer;
                    if ((ng & 0xffu) == 0) ng = pop();
                    const int child = cw8_next(&ng, F.oct);
                    if (ng & 0xffu) push(ng);
                    if (kCount) ++visits;
                    cw8_visit(nodes + child, F, tlimit, &ng, &tb, &tw);
                }
            }
            while (tw != 0) {
                if (kCount && MCPT_TRACE_DIAG && (int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) ++wleaf;
                const int bit = __builtin_ctz(tw);
                tw &= tw - 1;
                if (kCount) ++tests;
                cw8_tri(triv, tb + bit, ro, rd, excl, &best, &tlimit);
            }
            if ((ng & 0xffu) == 0 && sp == 0) finish();
        }
    }
    if (kCount) wave_count2(cnt, visits, cnt + 1, tests);
    if (kCount && MCPT_TRACE_DIAG) wave_count2(cnt + 6, witer, cnt + 7, wleaf);
}

#ifndef MCPT_COMBINE_LAZY
#define MCPT_COMBINE_LAZY 1
#endif
template <bool kStale>
__global__ __launch_bounds__(256, MCPT_LB_COMBINE) void k_mis_combine(Params P, Queue cur, int n, Aux A, Queue nxt, Slots T, int rp) {
    const DScene& S = P.S;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < n;
    const int ii = active ? i : 0;
    const int fl = A.flags[ii];
    const int pixel = cur.pixel[ii], sample = cur.sample[ii];
    const uint64_t node = cur.node[ii];
    const size_t o1 = ii, o2 = (size_t)A.cap + ii, ol = 2 * (size_t)A.cap + ii;
    // the three hit slots are loaded with the flags, not after them (a slot of a set the node did not
    // trace holds a stale value, which the flag tests below mask): one dependent hop less
    const int h1 = A.hf[o1], h2 = A.hf[o2], hl = A.hf[ol];
    const bool c1 = active && (fl & 1) && h1 >= 0;
    const bool c2 = active && (fl & 2) && h2 >= 0;
    const d3 p = ld3(cur.p, cur.cap, ii);
    const d3 N = ld3(cur.n, cur.cap, ii);
    const int li = (c2 && (fl & 4) && hl >= 0) ? S.tri_light[hl] : -1;
    const double own[7] = {p.x, p.y, p.z, N.x, N.y, N.z, cur.wsum[ii]};
    // a ray set's direction, throughput and (pdf, cos) matter only when that set hit (c1 / c2): the stale
    // form reads them under that predicate, so a lane whose ray missed fetches none of its 48-104 B
    // (MCPT_COMBINE_LAZY; the fresh form reads them all, as before)
    const bool lz = MCPT_COMBINE_LAZY && kStale;
    const d3 z3 = mk3(0, 0, 0);
    const d3 d1 = (!lz || c1) ? ld3(A.d1, A.cap, ii) : z3;
    const d3 w1 = (!lz || c1) ? ld3(A.w1, A.cap, ii) : z3;
    const d3 d2 = (!lz || c2) ? ld3(A.d2, A.cap, ii) : z3;
    const d3 w2 = (!lz || c2) ? ld3(A.w2, A.cap, ii) : z3;
    const double pdf = (!lz || c2) ? A.c2[2 * ii] : 0.0, cosb = (!lz || c2) ? A.c2[2 * ii + 1] : 0.0;
    if (!kStale) {  // fresh light pdf (this node's own prep) and forward throughputs
        d3 tp2 = mk3(0, 0, 0);
        if (c2) tp2 = mul(w2, cosb / (pdf + state_light_pdf(S, li, own)) / MCPT_P_RR);
        node_entry(P, c1, c1 ? h1 : -1, A.hbg[2 * o1], A.hbg[2 * o1 + 1], mul(d1, -1), w1, pixel, sample, 2 * node, nxt);
        node_entry(P, c2, c2 ? h2 : -1, A.hbg[2 * o2], A.hbg[2 * o2 + 1], mul(d2, -1), tp2, pixel, sample,
                   2 * node + 1, nxt);
    } else {
        const int f1 = c1 ? h1 : -1, f2 = c2 ? h2 : -1;
        const double b1 = c1 ? A.hbg[2 * o1] : 0.0, g1 = c1 ? A.hbg[2 * o1 + 1] : 0.0;
        const double b2 = c2 ? A.hbg[2 * o2] : 0.0, g2 = c2 ? A.hbg[2 * o2 + 1] : 0.0;
        const double s1 = (!lz || c1) ? A.s1[ii] : 0.0;
        const Entry e1 = entry_eval(P, c1, f1, b1, g1, mul(d1, -1), pixel, sample, 2 * node);
        const Entry e2 = entry_eval(P, c2, f2, b2, g2, mul(d2, -1), pixel, sample, 2 * node + 1);
        const bool lsh = e1.kind == 2, bsh = e2.kind == 2;
        // light edge: an emitter child finishes it now (main.cpp:464 with the child's emission)
        d3 Llight = mk3(0, 0, 0);
        if (e1.kind == 1) Llight = mul(hmul(mk3(S.light_rad[3 * e1.li], S.light_rad[3 * e1.li + 1], S.light_rad[3 * e1.li + 2]), w1), s1);
        // BRDF edge scalar: without a shading light child the sampler state is this node's own
        double s2 = 0;
        if (c2 && !lsh) s2 = cosb / (pdf + state_light_pdf(S, li, own)) / MCPT_P_RR;
        const bool hold = lsh || bsh;
        // the slot and both child appends in one barrier phase (round 5; three phases before: ±0, one
        // phase kept, profiles/round5_ab_combine_phase.txt)
        int slot, qp1, qp2;
        block_alloc_slot_push2(T, hold, lsh, bsh, nxt.count, &slot, &qp1, &qp2);
        const int pc = cur.par[ii];
        const bool need = pc >= 0 && (pc & 1);  // this subtree's path end is needed above
        d3 Lbr = mk3(0, 0, 0);
        if (e2.kind == 1) Lbr = mul(hmul(mk3(S.light_rad[3 * e2.li], S.light_rad[3 * e2.li + 1], S.light_rad[3 * e2.li + 2]), w2), s2);
        // finished now (no shading child): L = L_light + L_brdf (main.cpp:493); its path end is itself
        mis_report(P, T, active && !hold, pc, pixel, add(Llight, Lbr), own, rp);
        if (active && hold) {
            const size_t q = (size_t)slot;
            T.pend[q] = (int)lsh + (int)bsh;
            double* r = T.rec + kSlotRec * q;
            *reinterpret_cast<int4*>(r) = make_int4(pc, pixel,
                                                    (int)lsh | ((int)bsh << 1) | ((e2.kind == 1) << 2) | ((int)c2 << 3) | ((int)need << 4),
                                                    li);
            double* w = r + 2;
            w[0] = w1.x, w[1] = w1.y, w[2] = w1.z, w[3] = s1;
            w[4] = w2.x, w[5] = w2.y, w[6] = w2.z, w[7] = pdf, w[8] = cosb, w[9] = s2;
            if (!lsh) T.Ll[3 * q] = Llight.x, T.Ll[3 * q + 1] = Llight.y, T.Ll[3 * q + 2] = Llight.z;
            if (e2.kind == 1) r[12] = S.light_rad[3 * e2.li], r[13] = S.light_rad[3 * e2.li + 1], r[14] = S.light_rad[3 * e2.li + 2];
        }
        // the light child's path end is needed by this node's stale BRDF-edge pdf, and by whoever
        // needs this node's path end when the light child is on this node's path (no shading BRDF child)
        const bool need_l = (c2 && li >= 0) || (need && !bsh);
        const bool need_b = need;
        const d3 z = mk3(0, 0, 0);
        // the stale form never reads a node's forward throughput (w1 / w2 carry the edges), so it is not written
        queue_write(P, lsh, qp1, e1, f1, mul(d1, -1), z, pixel, sample, 2 * node, 4 * slot + (int)need_l, nxt, false);
        queue_write(P, bsh, qp2, e2, f2, mul(d2, -1), z, pixel, sample, 2 * node + 1, 4 * slot + 2 + (int)need_b, nxt, false);
    }
    block_count(ray_stats(P), active ? (unsigned)((fl & 1) + ((fl >> 1) & 1)) : 0u, ray_stats(P) + 1,
                (active && c2) ? 1u : 0u);
}

// the slots whose children have all reported (ready list rp_in): L = L_light + L_brdf with the BRDF
// edge's light pdf at the light child's path-end state, the slot goes back to the free ring, and the
// node reports to its parent (ready list 1 - rp_in) -- one tree level per pass, in step with the
// wavefront; grid-stride over the device-side count
// grid: x blocks per shard, y = ready-list shard
// (round 3: evaluating the stale pdf in a separate kernel so that this one runs at 8 waves/SIMD was
// measured slower, MIS 488.0-491.0 vs 492.0-493.0; profiles/round3_ab_slot_rec.txt)
__global__ __launch_bounds__(256, MCPT_LB_COMPLETE) void k_mis_complete(Params P, Slots T, int rp_in) {
    const DScene& S = P.S;
    const unsigned n = T.ctrl[16 * blockIdx.y + 4 + rp_in];
    const int* ready = (rp_in ? T.ready1 : T.ready0) + (size_t)blockIdx.y * T.ready_cap;
    const unsigned stride = gridDim.x * blockDim.x;
    // whole waves iterate together (wave-level appends inside)
    for (unsigned base = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < n; base += stride) {
        const unsigned i = base + lane_id();
        const bool act = i < n;
        const size_t q = act ? (size_t)ready[i] : 0;
        const double* rc = T.rec + kSlotRec * q;
        const int4 hdr = act ? *reinterpret_cast<const int4*>(rc) : make_int4(-1, 0, 0, -1);
        const int fl = hdr.z;
        const double* w = rc + 2;
        const bool lsh = fl & 1, bsh = fl & 2;
        d3 L = mk3(0, 0, 0);
        double stc[7] = {0, 0, 0, 0, 0, 0, 0};
        int par = -1, pix = 0;
        if (act) {
            const d3 Ll = mk3(T.Ll[3 * q], T.Ll[3 * q + 1], T.Ll[3 * q + 2]);
            const d3 Llight = lsh ? mul(hmul(Ll, mk3(w[0], w[1], w[2])), w[3]) : Ll;
            const double* last_l = T.last + 14 * q;
            double s2 = w[9];
            if (lsh && (fl & 8))  // the light child's path-end state
                s2 = w[8] / (w[7] + state_light_pdf(S, hdr.w, last_l)) / MCPT_P_RR;
            d3 Lbr = mk3(0, 0, 0);
            if (bsh || (fl & 4)) Lbr = mul(hmul(mk3(rc[12], rc[13], rc[14]), mk3(w[4], w[5], w[6])), s2);
            L = add(Llight, Lbr);
            if (fl & 16) {  // this subtree's path end, for an ancestor
                const double* st = bsh ? last_l + 7 : last_l;
#pragma unroll
                for (int k = 0; k < 7; k++) stc[k] = st[k];
            }
            par = hdr.x;
            pix = hdr.y;
        }
        const int fs = wave_shard();
        const int r = wave_append(&T.ctrl[16 * fs + 2], act);  // free the slot
        if (act) T.ring[(size_t)fs * T.ring_cap + (unsigned)r % (unsigned)T.ring_cap] = (int)q;
        mis_report(P, T, act, par, pix, L, stc, 1 - rp_in);
    }
}

// between passes: ring entries freed so far become allocatable, unconsumed reservations are returned,
// and the consumed ready list is emptied
__global__ void k_slot_fixup(Slots T, int rp_consumed) {  // one thread per shard
    unsigned* c = T.ctrl + 16 * threadIdx.x;
    c[1] = min(c[1], c[3]);
    c[3] = c[2];
    c[4 + rp_consumed] = 0;
}

// first index of the running sums cum[0..n) that is >= target (n - 1 if none): the counter-RNG
// inverse CDF, equal to the oracle's linear scan (the same running sums)
__device__ inline int cdf_search(const double* cum, int n, double target) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cum[mid] >= target) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}
// Mylight::select_a_point_from_lights (Mylight.cpp:102-160) with the counter RNG: a light of the
// lightsRadiance map by RadianceRGB::sum() (dim 1), one of its triangles by area (dim 7), a uniform
// point beta = 1 - sqrt(1 - ksi1), gamma = (1 - beta) ksi2 (dims 2, 3); proba = p(light) p(triangle) /
// area, an area-measure pdf.  Fewer than two choices: index 0, probability 1 (libstdc++'s
// discrete_distribution).  Returns the light-table index, or -1 if the light has no triangles (the
// reference throws std::out_of_range, Mylight.cpp:128).  The oracle's area_light_sample, op for op.
__device__ inline int area_light_sample(const DScene& S, uint64_t key, d3* coord, double* prob) {
    const int G = S.ngroups;
    if (G == 0) return -1;
    int k = 0;
    double p1 = 1.0;
    if (G >= 2) {
        const double tot = S.grp_cum[G - 1];
        k = cdf_search(S.grp_cum, G, counter_u(key, 1) * tot);
        p1 = S.grp_sum[k] / tot;
    }
    const int2 r = S.grp_range[k];
    if (r.y == 0) return -1;
    int jj = 0;
    double p2 = 1.0;
    if (r.y >= 2) {
        const double tot = S.l_area_cum[r.x + r.y - 1];
        jj = cdf_search(S.l_area_cum + r.x, r.y, counter_u(key, 7) * tot);
        p2 = S.l_area[r.x + jj] / tot;
    }
    const int j = r.x + jj;
    const double ksi1 = counter_u(key, 2), ksi2 = counter_u(key, 3);
    const double beta = 1 - sqrt(1 - ksi1);
    const double gamma = (1 - beta) * ksi2;
    const double alpha = 1 - beta - gamma;
    *coord = add(add(mul(f3(S.lt_v[3 * j]), alpha), mul(f3(S.lt_v[3 * j + 1]), beta)), mul(f3(S.lt_v[3 * j + 2]), gamma));
    double proba = 1.0;
    proba *= p1;
    proba *= p2;
    proba *= 1.0 / S.l_area[j];
    *prob = proba;
    return j;
}

__global__ __launch_bounds__(256, MCPT_LB_SHADE_GEN) void k_shade_gen(Params P, Queue cur, int n, Aux A) {
    const DScene& S = P.S;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const d3 p = ld3(cur.p, cur.cap, i);
    const d3 N = ld3(cur.n, cur.cap, i);
    const d3 wo = ld3(cur.wo, cur.cap, i);
    const d3 tp = ld3(cur.tp, cur.cap, i);
    const int f = cur.f[i];
    const uint64_t key = counter_key(P.seed, (uint64_t)cur.pixel[i], (uint64_t)cur.sample[i], cur.node[i]);
    const float* m = S.mtl + 7 * S.tri_mat[f];
    const d3 kd = mk3(m[0], m[1], m[2]), ks = mk3(m[3], m[4], m[5]);
    const double sh = m[6];
    int pick = -1;
    int flags = 0;
    // ---- direct light (main.cpp:295-316) ----
    d3 coord, n1 = N, w1 = mk3(0, 0, 0);
    double lprob = 1;
    if (P.mode == MCPT_MODE_SHADE_AREA) {  // main.cpp:296: select_a_point_from_lights
        pick = area_light_sample(S, key, &coord, &lprob);
        if (pick >= 0) {
            const double4 ln = S.lt_n[pick];
            n1 = mk3(ln.x, ln.y, ln.z);
        } else {
            coord = add(mul(N, -1), p);
        }
    } else if ((pick = cur.pick[i]) >= 0) {
        const double4 ln = S.lt_n[pick];
        SphTri sph;
        pick_sph(S, pick, p, N, &sph);
        const d3 Pd = arvo_sample(sph, counter_u(key, 2), counter_u(key, 3));
        TriHit th = tri_hit(f3(S.lt_v[3 * pick]), f3(S.lt_v[3 * pick + 1]), f3(S.lt_v[3 * pick + 2]), p, Pd);
        coord = add(p, mul(Pd, th.hit ? th.t : 0.0));  // miss: t = 0 (Mylight.cpp:311-317)
        lprob = S.light_sum[pick] / cur.wsum[i];
        n1 = mk3(ln.x, ln.y, ln.z);
    } else {
        coord = add(mul(N, -1), p);  // empty set: x1 - n (Mylight.cpp:263-266); wl = -N never passes wl.N > 0
    }
    const d3 wl = normalized(sub(coord, p));
    if (pick >= 0 && dot(wl, N) > 0 && dot(mul(wl, -1), n1) > 0) {
        flags |= 1;
        A.hbg[2 * (size_t)i] = seed_light_t(S, S.light_facet[pick], f, p, wl);
        const d3 b = brdf_phong(N, wl, wo, kd, ks, sh);
        const d3 d = sub(coord, p);
        const d3 I = mk3(S.light_rad[3 * pick], S.light_rad[3 * pick + 1], S.light_rad[3 * pick + 2]);
        const d3 Ld = mul(hmul(I, b), dot(wl, N) * dot(mul(wl, -1), n1) / dot(d, d) / lprob);
        w1 = mk3(tp.x * Ld.x * P.inv_spp, tp.y * Ld.y * P.inv_spp, tp.z * Ld.z * P.inv_spp);
    }
    // ---- indirect (main.cpp:318-343) ----
    d3 wi = mk3(0, 0, 0), w2 = mk3(0, 0, 0);
    if (!(counter_u(key, 0) > MCPT_P_RR)) {
        double pdf;
        wi = sample_phong(N, wo, kd, ks, sh, counter_u(key, 4), counter_u(key, 5), counter_u(key, 6), &pdf);
        if (!(dot(wi, N) < 0)) {
            flags |= 2;
            w2 = mul(hmul(tp, brdf_phong(N, wi, wo, kd, ks, sh)), dot(wi, N) / pdf / MCPT_P_RR);
        }
    }
    st3(A.d1, A.cap, i, wl);
    st3(A.d2, A.cap, i, wi);
    st3(A.w1, A.cap, i, w1);
    st3(A.w2, A.cap, i, w2);
    A.hf[2 * (size_t)A.cap + i] = pick >= 0 ? S.light_facet[pick] : -1;
    A.flags[i] = flags;
}

__global__ __launch_bounds__(256) void k_shade_combine(Params P, Queue cur, int n, Aux A, Queue nxt) {
    const DScene& S = P.S;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < n;
    const int ii = active ? i : 0;
    const int fl = A.flags[ii];
    const size_t o1 = ii, o2 = (size_t)A.cap + ii;
    if (active && (fl & 1) && A.hf[o1] >= 0 && A.hf[o1] == A.hf[2 * (size_t)A.cap + ii]) {
        double* px = P.fb + 3 * (size_t)cur.pixel[ii];
        unsafeAtomicAdd(px + 0, A.w1[idx3(A.cap, ii, 0)]);
        unsafeAtomicAdd(px + 1, A.w1[idx3(A.cap, ii, 1)]);
        unsafeAtomicAdd(px + 2, A.w1[idx3(A.cap, ii, 2)]);
    }
    const int h2 = A.hf[o2];
    const bool c = active && (fl & 2) && h2 >= 0 && S.tri_light[h2] < 0;
    const d3 d2 = ld3(A.d2, A.cap, ii);
    const d3 w2 = ld3(A.w2, A.cap, ii);
    node_entry(P, c, c ? h2 : -1, A.hbg[2 * o2], A.hbg[2 * o2 + 1], mul(d2, -1), w2, cur.pixel[ii], cur.sample[ii],
               cur.node[ii] + 1, nxt);
    block_count(ray_stats(P), active ? (unsigned)((fl & 1) + ((fl >> 1) & 1)) : 0u);
}

// shade_with_brdf (main.cpp:385-396): gen samples the bounce, combine spawns the child on any hit
__global__ __launch_bounds__(256) void k_brdf_gen(Params P, Queue cur, int n, Aux A) {
    const DScene& S = P.S;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const d3 N = ld3(cur.n, cur.cap, i);
    const d3 wo = ld3(cur.wo, cur.cap, i);
    const d3 tp = ld3(cur.tp, cur.cap, i);
    const uint64_t key = counter_key(P.seed, (uint64_t)cur.pixel[i], (uint64_t)cur.sample[i], cur.node[i]);
    const float* m = S.mtl + 7 * S.tri_mat[cur.f[i]];
    const d3 kd = mk3(m[0], m[1], m[2]), ks = mk3(m[3], m[4], m[5]);
    const double sh = m[6];
    double pdf;
    const d3 wi = sample_phong<true>(N, wo, kd, ks, sh, counter_u(key, 4), counter_u(key, 5), counter_u(key, 6), &pdf);
    int flags = 0;
    d3 w2 = mk3(0, 0, 0);
    if (!(dot(wi, N) < 0)) {
        flags = 2;
        w2 = mul(hmul(tp, brdf_phong<false, true>(N, wi, wo, kd, ks, sh)), dot(wi, N) / pdf / MCPT_P_RR);
    }
    st3(A.d2, A.cap, i, wi);
    st3(A.w2, A.cap, i, w2);
    A.flags[i] = flags;
}

__global__ __launch_bounds__(256) void k_brdf_combine(Params P, Queue cur, int n, Aux A, Queue nxt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < n;
    const int ii = active ? i : 0;
    const int fl = A.flags[ii];
    const size_t o2 = (size_t)A.cap + ii;
    const int h2 = A.hf[o2];
    const bool c = active && (fl & 2) && h2 >= 0;
    const d3 d2 = ld3(A.d2, A.cap, ii);
    const d3 w2 = ld3(A.w2, A.cap, ii);
    node_entry(P, c, c ? h2 : -1, A.hbg[2 * o2], A.hbg[2 * o2 + 1], mul(d2, -1), w2, cur.pixel[ii], cur.sample[ii],
               cur.node[ii] + 1, nxt);
    block_count(ray_stats(P), (active && (fl & 2)) ? 1u : 0u);
}

// one BRDF-only path vertex (main.cpp:385-396)
// BRDF-only extension: 256-thread blocks with the BVH4's top levels in LDS (MCPT_BRDF_TOP nodes, 0 =
// none: 128-thread blocks with a 16-entry stack)
#ifndef MCPT_BRDF_TOP
#define MCPT_BRDF_TOP 21
#endif
constexpr int kBrdfTop = MCPT_BRDF_TOP;
constexpr int kBrdfBlock = kBrdfTop > 0 ? 256 : kTraceBlock;
constexpr int kBrdfLds = kBrdfTop > 0 ? 8 : kRayLds;
#ifndef MCPT_BRDF_TIMING
#define MCPT_BRDF_TIMING 0  // A/B only: 1 = sampling twice, 2 = traversal twice (cost shares, timing builds)
#endif
#ifndef MCPT_BRDF_PARK
#define MCPT_BRDF_PARK 1  // the child throughput in LDS during the traversal: 14 spilled VGPRs -> 0, C2 +6% (profiles/round5_ab_brdf_park.txt)
#endif
#ifndef MCPT_BRDF_WAVES
#define MCPT_BRDF_WAVES 5  // 96 VGPRs (10 spilled): 4 -> 5 waves/SIMD, +5% BRDF-only (profiles/round2b_ab_brdf.txt)
#endif
template <bool kCount = false>
__global__ __launch_bounds__(kBrdfBlock, MCPT_BRDF_WAVES) void k_extend_brdf(Params P, Queue cur, int n, Queue nxt) {
    __shared__ int stack[kBrdfLds * kBrdfBlock];
#if MCPT_BRDF_PARK
    // the child's throughput waits out the traversal in LDS, not in VGPRs (MCPT_BRDF_PARK)
    __shared__ double park[3 * kBrdfBlock];
#endif
    __shared__ BvhNode4 top[kBrdfTop > 0 ? kBrdfTop : 1];
    const DScene& S = P.S;
    if (kBrdfTop > 0) {  // the tree's top levels into LDS (as k_mis_rays)
        const int cnt4 = min(kBrdfTop, S.nbvh4) * (int)(sizeof(BvhNode4) / sizeof(float4));
        for (int k = threadIdx.x; k < cnt4; k += blockDim.x)
            reinterpret_cast<float4*>(top)[k] = reinterpret_cast<const float4*>(S.bvh4)[k];
        __syncthreads();
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < n;
    const int ii = active ? i : 0;
    const int f = cur.f[ii], pixel = cur.pixel[ii], sample = cur.sample[ii];
    const uint64_t node = cur.node[ii];
    d3 p, N, wo, tp;
    if (P.root_pnw && node == 1) {  // a root: the per-pixel table (k_roots_t wrote no point / normal / wo)
        const double* t = P.root_pnw + 9 * (size_t)pixel;
        p = mk3(t[0], t[1], t[2]), N = mk3(t[3], t[4], t[5]), wo = mk3(t[6], t[7], t[8]), tp = mk3(1, 1, 1);
    } else {
        p = ld3(cur.p, cur.cap, ii), N = ld3(cur.n, cur.cap, ii), wo = ld3(cur.wo, cur.cap, ii), tp = ld3(cur.tp, cur.cap, ii);
    }
    bool c = false;
    unsigned traced = 0, visits = 0, tests = 0, witer = 0, wleaf = 0;
    Hit h{-1, 0, 0, 0};
    d3 wi = mk3(0, 0, 0), tpc = mk3(0, 0, 0);
    if (active) {
        const uint64_t key = counter_key(P.seed, (uint64_t)pixel, (uint64_t)sample, node);
        const float* m = S.mtl + 7 * S.tri_mat[f];
        const d3 kd = mk3(m[0], m[1], m[2]), ks = mk3(m[3], m[4], m[5]);
        const double sh = m[6];
        double pdf;
        wi = sample_phong<true>(N, wo, kd, ks, sh, counter_u(key, 4), counter_u(key, 5), counter_u(key, 6), &pdf);
#if MCPT_BRDF_TIMING == 1  // timing-only build: the sampling and shading run twice (cost share of that region)
        {
            double pdf2;
            const d3 wi2 = sample_phong<true>(N, wo, kd, ks, sh, counter_u(key, 7), counter_u(key, 8), counter_u(key, 9), &pdf2);
            const d3 b2 = brdf_phong<false, true>(N, wi2, wo, kd, ks, sh);
            if (P.mode == 12345) wi = wi2, pdf = pdf2 + b2.x;
        }
#endif
        if (!(dot(wi, N) < 0)) {
            traced = 1;
            // the child's throughput does not depend on the hit: computed before the traversal, so
            // the shading state (N, wo, material, tp, pdf) is dead during it (fewer VGPRs)
            const d3 b = brdf_phong<false, true>(N, wi, wo, kd, ks, sh);
            tpc = mul(hmul(tp, b), dot(wi, N) / pdf / MCPT_P_RR);
#if MCPT_BRDF_PARK
            park[threadIdx.x] = tpc.x, park[kBrdfBlock + threadIdx.x] = tpc.y, park[2 * kBrdfBlock + threadIdx.x] = tpc.z;
#endif
            h = trace4_ww<kBrdfLds, kCount, kBrdfTop, MCPT_FILTER_BRDF>(S.bvh4, S.leaf_v, p, wi, f, stack + threadIdx.x, kBrdfBlock, &visits,
                                                      &tests, top, FLT_MAX, &witer, &wleaf);
#if MCPT_BRDF_TIMING == 2  // timing-only build: the traversal runs twice
            {
                const Hit h2 = trace4_ww<kBrdfLds, kCount, kBrdfTop, MCPT_FILTER_BRDF>(S.bvh4, S.leaf_v, p, wi, f, stack + threadIdx.x,
                                                                                    kBrdfBlock, &visits, &tests, top);
                if (P.mode == 12345) h = h2;
            }
#endif
            c = h.f >= 0;
        }
    }
#if MCPT_BRDF_PARK
    if (traced) tpc = mk3(park[threadIdx.x], park[kBrdfBlock + threadIdx.x], park[2 * kBrdfBlock + threadIdx.x]);
#endif
    node_entry(P, c, h.f, h.beta, h.gamma, mul(wi, -1), tpc, pixel, sample, node + 1, nxt);
    block_count(ray_stats(P), traced);
    if (kCount) wave_count2(P.stats + 8, visits, P.stats + 9, tests);
    if (kCount && MCPT_TRACE_DIAG) wave_count2(P.stats + 14, witer, P.stats + 15, wleaf);
}

// batch closest hit (test / FFI entry mcpt_closest_hit)
template <bool kGrid>
__global__ __launch_bounds__(kTraceBlock) void k_trace_batch(DScene S, int n, const double* ro, const double* rd,
                                                             const int* ex, int light_only, int* f_out,
                                                             double* tbg) {
    __shared__ int stack[kRayLds * kTraceBlock];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Hit h = kGrid ? grid_trace(S, mk3(ro[3 * i], ro[3 * i + 1], ro[3 * i + 2]), mk3(rd[3 * i], rd[3 * i + 1], rd[3 * i + 2]),
                                     ex[i], light_only != 0)
                        : trace4_ww<kRayLds>(light_only ? S.lbvh4 : S.bvh4, light_only ? S.lleaf_v : S.leaf_v, mk3(ro[3 * i], ro[3 * i + 1], ro[3 * i + 2]),
                  mk3(rd[3 * i], rd[3 * i + 1], rd[3 * i + 2]), ex[i], stack + threadIdx.x, kTraceBlock);
    f_out[i] = h.f;
    tbg[3 * i] = h.f >= 0 ? h.t : 0.0;
    tbg[3 * i + 1] = h.f >= 0 ? h.beta : 0.0;
    tbg[3 * i + 2] = h.f >= 0 ? h.gamma : 0.0;
}

// batch closest hit through the 8-wide trees, one ray per thread (mcpt_closest_hit with MCPT_HIT_CW8,
// include/mcpt_debug.h): the traversal of k_rays_cw8 for tests against the reference goldens
__global__ __launch_bounds__(kTraceBlock) void k_trace_batch_cw8(DScene S, int n, const double* ro_, const double* rd_,
                                                                const int* ex, int light_only, int* f_out, double* tbg) {
    __shared__ unsigned stack[kRayLds * kTraceBlock];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Hit best = trace_cw8<kRayLds>(light_only ? S.lbvh8 : S.bvh8, light_only ? S.ltri8_v : S.tri8_v,
                                        mk3(ro_[3 * i], ro_[3 * i + 1], ro_[3 * i + 2]), mk3(rd_[3 * i], rd_[3 * i + 1], rd_[3 * i + 2]),
                                        ex[i], stack + threadIdx.x, kTraceBlock);
    f_out[i] = best.f;
    tbg[3 * i] = best.f >= 0 ? best.t : 0.0;
    tbg[3 * i + 1] = best.f >= 0 ? best.beta : 0.0;
    tbg[3 * i + 2] = best.f >= 0 ? best.gamma : 0.0;
}

// ============================================================================================
// host side
// ============================================================================================
#define HIP_OK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            set_error("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return MCPT_E_DEVICE;                                                              \
        }                                                                                      \
    } while (0)

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct DeviceState {
    int device = -1;
    DScene d{};
    std::vector<void*> allocs;
    hipStream_t stream = nullptr;
    // reusable work buffers
    DevBuf hit_f, hit_tbg, root_pnw, root_kind, fb, rank_fb, stats, work, qa[14], qb[14], qs[14], aux[9], sl[13], cache_bt, cache_lst, cache_info, cache_w, masks;
    DevBuf cull_keys, cull_order, cull_count;  // the cull's node order (CullOrder)
    DevBuf exact, exact_scr, slack;  // exact pick: list, k_prep_exact's scratch, per-node slack
    DevBuf lit_slot, lit_pool;        // exact pick: roots' literal sums per pixel (RootLit)
    DevBuf sc_cum, sc_wsum, sc_last;  // small-table root-point cache (SmallCache)
    int spill_cap = 0;  // nodes the spill stack qs holds (grown on demand)
    bool bvh8_tried = false;  // ensure_bvh8 ran on this device
    DevBuf g_start, g_tri;  // the scene's uniform grid (MCPT_ACCEL_GRID), version grid_version
    int grid_version = 0;
    unsigned* pinned_count = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evp0 = nullptr, evp1 = nullptr, evr0 = nullptr, evr1 = nullptr;
};

}  // namespace

struct mcpt_scene {
    HostScene host;
    Bvh bvh, lbvh;
    Bvh8 bvh8, lbvh8;  // 8-wide compressed trees of bvh / lbvh (k_rays_cw8), built on first use (ensure_bvh8)
    bool bvh8_built = false;
    std::mutex bvh8_mu;
    Grid grid;             // Myobj::cal_scene_boundingbox(eye) + meshing(n0) (mcpt_scene_meshing)
    int grid_version = 0;  // bumped by every rebuild; devices re-upload on mismatch
    std::vector<std::unique_ptr<DeviceState>> devs;
    std::mutex devs_mu;             // devs (render_multi creates device states on its worker threads)
    std::vector<int> comm_devices;  // distinct devices of the cached ncclCommInitAll communicators
    std::vector<void*> comms;
    std::mutex mu;
};

namespace {

// n 3-vectors [n][3] -> the kernels' node-input layout (idx3 with stride n)
std::vector<double> soa3(const double* v, int n) {
    std::vector<double> o(3 * (size_t)n);
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) o[idx3((size_t)n, i, k)] = v[3 * (size_t)i + k];
    return o;
}

int ensure(DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return MCPT_OK;
    if (b.p) HIP_OK(hipFree(b.p));
    b.p = nullptr;
    HIP_OK(hipMalloc(&b.p, std::max<size_t>(bytes, 256)));
    b.bytes = std::max<size_t>(bytes, 256);
    return MCPT_OK;
}
// the cull's node-order scratch for up to n nodes
int cull_order_bufs(DeviceState& D, size_t n, CullOrder* co) {
    int rc;
    if ((rc = ensure(D.cull_keys, n)) || (rc = ensure(D.cull_order, 4 * n)) || (rc = ensure(D.cull_count, 8 * kCullBuckets)))
        return rc;
    *co = CullOrder{(unsigned char*)D.cull_keys.p, (int*)D.cull_order.p, (unsigned*)D.cull_count.p};
    return MCPT_OK;
}

template <class T>
int upload(DeviceState& D, const std::vector<T>& v, const T** out) {
    void* p = nullptr;
    HIP_OK(hipMalloc(&p, std::max<size_t>(v.size() * sizeof(T), 64)));
    D.allocs.push_back(p);  // owned by D from here on, even if the copy fails
    if (!v.empty()) HIP_OK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = static_cast<const T*>(p);
    return MCPT_OK;
}

// the deepest the traversal stacks (trace4_ww, k_rays_persistent) can get on a 4-wide tree: at each node a
// lane pushes every hit child but the nearest, which it follows, so the stack never holds more than the sum
// over a root-to-node path of (children - 1).  A tree that could overflow the kStack entries is refused at
// device setup (a dropped push would lose a subtree, and with it possibly the closest hit), so no traversal
// ever drops one: the builder's depth cap keeps real scenes far below (Veach 8 levels, Cornell-1M 12: at
// most 33 entries)
int bvh4_stack_need(const std::vector<BvhNode4>& t) {
    if (t.empty()) return 0;
    int need = 0;
    std::vector<std::pair<int, int>> st{{0, 0}};  // (node, entries its ancestors may have pushed)
    while (!st.empty()) {
        const auto [v, above] = st.back();
        st.pop_back();
        int used = 0;
        for (int k = 0; k < 4; k++) used += t[v].child[k] != kBvh4Empty;
        const int here = above + std::max(used - 1, 0);
        need = std::max(need, here);
        for (int k = 0; k < 4; k++)
            if (t[v].child[k] >= 0 && t[v].child[k] != kBvh4Empty) st.push_back({t[v].child[k], here});
    }
    return need;
}

// renumbers a 4-wide BVH breadth-first (root 0, then each level in order), so the first nodes are
// its top levels (k_mis_rays stages them in LDS); inner-child indices are remapped
std::vector<BvhNode4> bfs_order(const std::vector<BvhNode4>& in) {
    if (in.empty()) return in;
    std::vector<int32_t> order, newidx(in.size(), -1);
    order.reserve(in.size());
    order.push_back(0);
    newidx[0] = 0;
    for (size_t h = 0; h < order.size(); h++)
        for (int k = 0; k < 4; k++) {
            const int32_t c = in[order[h]].child[k];
            if (c >= 0 && c != kBvh4Empty && newidx[c] < 0) {
                newidx[c] = (int32_t)order.size();
                order.push_back(c);
            }
        }
    std::vector<BvhNode4> out(order.size());
    for (size_t h = 0; h < order.size(); h++) {
        out[h] = in[order[h]];
        for (int k = 0; k < 4; k++) {
            const int32_t c = out[h].child[k];
            if (c >= 0 && c != kBvh4Empty) out[h].child[k] = newidx[c];
        }
    }
    return out;
}

// leaf children as the traversal stack code ~((first leaf slot << 3) | count), so a node visit needs
// no count load or decode (trace4_ww)
int pack_leaf_codes(std::vector<BvhNode4>& nodes) {
    for (BvhNode4& n : nodes)
        for (int k = 0; k < 4; k++)
            if (n.child[k] < 0) {
                const int first = ~n.child[k];
                if (n.count[k] >= (1 << kLeafBits) || first >= (1 << (31 - kLeafBits))) {
                    set_error("BVH leaf (%d triangles at slot %d) does not fit the traversal's leaf code", n.count[k], first);
                    return MCPT_E_SCENE;
                }
                n.child[k] = ~((first << kLeafBits) | n.count[k]);
            }
    return MCPT_OK;
}

std::vector<float4> leaf_vertices(const HostScene& s, const Bvh& b) {
    std::vector<float4> v(3 * std::max<size_t>(b.leaf_facets.size(), 1));
    for (size_t q = 0; q < b.leaf_facets.size(); q++) {
        const int f = b.leaf_facets[q];
        for (int k = 0; k < 3; k++) {
            float4 x;
            x.x = s.pos[9 * f + 3 * k];
            x.y = s.pos[9 * f + 3 * k + 1];
            x.z = s.pos[9 * f + 3 * k + 2];
            int fb = f;
            float w;
            std::memcpy(&w, &fb, 4);
            x.w = k == 0 ? w : 0.0f;
            v[3 * q + k] = x;
        }
    }
    return v;
}

int prep_chunks(int NL);

// the device's scene state, created (scene, light tables and BVHs uploaded) on first use.  Thread-safe
// for distinct devices: render_multi's workers create theirs concurrently (the lookup and the insertion
// hold devs_mu, the uploads do not)
int get_device_state(mcpt_scene* sc, int device, DeviceState** out) {
    if (device < 0) HIP_OK(hipGetDevice(&device));
    {
        std::lock_guard<std::mutex> lk(sc->devs_mu);
        for (auto& d : sc->devs)
            if (d->device == device) {
                HIP_OK(hipSetDevice(device));
                *out = d.get();
                return MCPT_OK;
            }
    }
    HIP_OK(hipSetDevice(device));
    auto D = std::make_unique<DeviceState>();
    D->device = device;
    const HostScene& s = sc->host;
    DScene& d = D->d;
    d.F = s.F;
    d.NL = s.NL;
    d.light_bound = 0.0f;
    std::vector<float4> tv(3 * std::max(s.F, 1));
    for (int f = 0; f < s.F; f++)
        for (int k = 0; k < 3; k++) tv[3 * f + k] = make_float4(s.pos[9 * f + 3 * k], s.pos[9 * f + 3 * k + 1], s.pos[9 * f + 3 * k + 2], 0.f);
    int rc;
    if ((rc = upload(*D, tv, &d.tri_v))) return rc;
    if ((rc = upload(*D, s.nrm, &d.tri_n))) return rc;
    if ((rc = upload(*D, s.mat, &d.tri_mat))) return rc;
    if ((rc = upload(*D, s.light_of, &d.tri_light))) return rc;
    if ((rc = upload(*D, s.mtl, &d.mtl))) return rc;
    if ((rc = upload(*D, s.light_rad, &d.light_rad))) return rc;
    if ((rc = upload(*D, s.light_sum, &d.light_sum))) return rc;
    if ((rc = upload(*D, s.light_facet, &d.light_facet))) return rc;
    std::vector<float4> lv(3 * std::max(s.NL, 1));
    std::vector<double4> ln(std::max(s.NL, 1));
    for (int l = 0; l < s.NL; l++) {
        const int f = s.light_facet[l];
        for (int k = 0; k < 3; k++) {
            lv[3 * l + k] = tv[3 * f + k];
            lv[3 * l + k].w = (float)s.unique_n[3 * f + k];
            d.light_bound = std::max({d.light_bound, std::fabs(lv[3 * l + k].x), std::fabs(lv[3 * l + k].y),
                                      std::fabs(lv[3 * l + k].z)});
        }
        ln[l] = make_double4(s.unique_n[3 * f], s.unique_n[3 * f + 1], s.unique_n[3 * f + 2], s.light_sum[l]);
    }
    if ((rc = upload(*D, lv, &d.lt_v))) return rc;
    if ((rc = upload(*D, ln, &d.lt_n))) return rc;
    {  // select_a_point_from_lights tables (MCPT_MODE_SHADE_AREA): running sums in table order, as the oracle
        d.ngroups = (int)s.group_rsum.size();
        std::vector<double> gcum(d.ngroups), acum(s.NL);
        std::vector<int2> gr(d.ngroups);
        double c = 0;
        for (int k = 0; k < d.ngroups; k++) {
            c += s.group_rsum[k];
            gcum[k] = c;
            gr[k] = make_int2(s.group_start[k], s.group_count[k]);
            double a = 0;
            for (int j = s.group_start[k]; j < s.group_start[k] + s.group_count[k]; j++) {
                a += s.light_area[j];
                acum[j] = a;
            }
        }
        if ((rc = upload(*D, s.group_rsum, &d.grp_sum)) || (rc = upload(*D, gcum, &d.grp_cum)) || (rc = upload(*D, gr, &d.grp_range)) ||
            (rc = upload(*D, s.light_area, &d.l_area)) || (rc = upload(*D, acum, &d.l_area_cum)))
            return rc;
    }
    const int nl_pad = 256 * ((prep_chunks(s.NL) + 3) / 4);  // whole groups of 4 chunks: the prep kernel reads past N_L unchecked
    std::vector<float4> lpk(3 * nl_pad, make_float4(0, 0, 0, 0));
    std::vector<float> ld(nl_pad, 0.0f);
    // + kSentinelPad sentinel records (zero vertices, lsum2 = -1): k_prep_pk2 pads its candidate
    // batches with index nl_pad; the full stage culls them for any x1, as sA > 0 gives w < 0 and
    // sA <= 0 or NaN fail directly (a zero lsum could pass with w = 0), and sA stays on the atan
    // fast path (|y| ~ 0, x ~ 4)
    std::vector<double2> lw(5 * (nl_pad + kSentinelPad), make_double2(0, 0));
    for (int l = nl_pad; l < nl_pad + kSentinelPad; l++) lw[5 * (size_t)l + 4] = make_double2(0.0, -1.0);
    // fp32 records (same padding and sentinels: a zero record gives e1 = e2 = 0, so sA = 0, culled)
    std::vector<float4> lf(4 * (nl_pad + kSentinelPad), make_float4(0, 0, 0, 0));
    for (int l = 0; l < s.NL; l++) {
        const float4 a = lv[3 * l], b = lv[3 * l + 1], c = lv[3 * l + 2];
        lpk[3 * l] = make_float4(a.x, b.x, c.x, a.w);
        lpk[3 * l + 1] = make_float4(a.y, b.y, c.y, b.w);
        lpk[3 * l + 2] = make_float4(a.z, b.z, c.z, c.w);
        ld[l] = (float)(ln[l].x * a.x + ln[l].y * a.y + ln[l].z * a.z);
        lw[5 * l] = make_double2(a.x, a.y);
        lw[5 * l + 1] = make_double2(a.z, b.x);
        lw[5 * l + 2] = make_double2(b.y, b.z);
        lw[5 * l + 3] = make_double2(c.x, c.y);
        lw[5 * l + 4] = make_double2(c.z, 2.0 * ln[l].w);
        // edges p1 - p0, p2 - p0 from the float vertices in fp64, rounded once (exact for nearby vertices)
        const float e1[3] = {(float)((double)b.x - a.x), (float)((double)b.y - a.y), (float)((double)b.z - a.z)};
        const float e2[3] = {(float)((double)c.x - a.x), (float)((double)c.y - a.y), (float)((double)c.z - a.z)};
        lf[4 * (size_t)l] = make_float4(a.x, a.y, a.z, e1[0]);
        lf[4 * (size_t)l + 1] = make_float4(e1[1], e1[2], e2[0], e2[1]);
        lf[4 * (size_t)l + 2] = make_float4(e2[2], (float)(2.0 * ln[l].w), 0, 0);
    }
    std::vector<LightPair> lpr(32 * (size_t)std::max(prep_chunks(s.NL), 1));
    for (size_t q = 0; q < lpr.size(); q++) {
        LightPair& P = lpr[q];
        memset((void*)&P, 0, sizeof P);
        float* nl = &P.nl[0].x;
        float* dd = &P.d.x;
        float* pp = &P.p[0].x;
        for (int h = 0; h < 2; h++) {
            const int l = (int)(2 * q) + h;
            if (l >= s.NL) {
                dd[h] = 1e30f;  // padding: always culled by the light-side test
                continue;
            }
            const float4 v[3] = {lv[3 * l], lv[3 * l + 1], lv[3 * l + 2]};
            nl[h] = (float)ln[l].x;
            nl[2 + h] = (float)ln[l].y;
            nl[4 + h] = (float)ln[l].z;
            dd[h] = (float)((ln[l].x * v[0].x + ln[l].y * v[0].y + ln[l].z * v[0].z) + MCPT_EPS);
            for (int k = 0; k < 3; k++) {
                pp[2 * (3 * k) + h] = v[k].x;
                pp[2 * (3 * k + 1) + h] = v[k].y;
                pp[2 * (3 * k + 2) + h] = v[k].z;
            }
        }
    }
    if ((rc = upload(*D, lpr, &d.lt_pair))) return rc;
    {  // exact-pick band tables: the chunk spheres are conservative (radius rounded up by 1e-6 relative)
        const int nch = prep_chunks(s.NL);
        std::vector<float4> sph(nch, make_float4(0, 0, 0, 0));
        std::vector<float2> sk(nch, make_float2(0, 0));
        double lo_s[3] = {1e300, 1e300, 1e300}, hi_s[3] = {-1e300, -1e300, -1e300};
        double smax = 0, kmax = 0;
        for (int c = 0; c < nch; c++) {
            double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
            const int l0 = 64 * c, l1 = std::min(s.NL, 64 * c + 64);
            for (int l = l0; l < l1; l++)
                for (int k = 0; k < 3; k++) {
                    const double p[3] = {lv[3 * l + k].x, lv[3 * l + k].y, lv[3 * l + k].z};
                    for (int a = 0; a < 3; a++) {
                        lo[a] = std::min(lo[a], p[a]);
                        hi[a] = std::max(hi[a], p[a]);
                        lo_s[a] = std::min(lo_s[a], p[a]);
                        hi_s[a] = std::max(hi_s[a], p[a]);
                    }
                }
            if (l1 <= l0) continue;
            // the centre as stored (float), so R bounds the distances from the centre the kernels read
            const double ctr[3] = {(double)(float)(0.5 * (lo[0] + hi[0])), (double)(float)(0.5 * (lo[1] + hi[1])),
                                   (double)(float)(0.5 * (lo[2] + hi[2]))};
            double R = 0, S = 0, K = 0;
            for (int l = l0; l < l1; l++) {
                double lmin = 1e300;
                for (int k = 0; k < 3; k++) {
                    const float4 a = lv[3 * l + k], b = lv[3 * l + (k + 1) % 3];
                    const double dx = (double)a.x - ctr[0], dy = (double)a.y - ctr[1], dz = (double)a.z - ctr[2];
                    R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz));
                    const double ex = (double)b.x - a.x, ey = (double)b.y - a.y, ez = (double)b.z - a.z;
                    lmin = std::min(lmin, std::sqrt(ex * ex + ey * ey + ez * ez));
                }
                S = std::max(S, s.light_sum[l]);
                K = std::max(K, lmin > 0 ? s.light_sum[l] / lmin : 1e30);
            }
            sph[c] = make_float4((float)ctr[0], (float)ctr[1], (float)ctr[2], (float)(R * (1 + 1e-6) + 1e-6));
            sk[c] = make_float2((float)(S * (1 + 1e-6)), (float)std::min(K * (1 + 1e-6), 1e30));
            smax = std::max(smax, S);
            kmax = std::max(kmax, K);
        }
        double Rs = 0;
        for (int a = 0; a < 3; a++) d.band_ctr[a] = s.NL > 0 ? 0.5 * (lo_s[a] + hi_s[a]) : 0.0;
        for (int c = 0; c < nch; c++) {  // the scene sphere contains every chunk sphere
            const double dx = sph[c].x - d.band_ctr[0], dy = sph[c].y - d.band_ctr[1], dz = sph[c].z - d.band_ctr[2];
            Rs = std::max(Rs, std::sqrt(dx * dx + dy * dy + dz * dz) + sph[c].w);
        }
        d.band_R = Rs * (1 + 1e-6) + 1e-6;
        d.band_S = smax * (1 + 1e-6);
        d.band_K = std::min(kmax * (1 + 1e-6), 1e30);
        if ((rc = upload(*D, sph, &d.chunk_sph)) || (rc = upload(*D, sk, &d.chunk_sk))) return rc;
    }
    if ((rc = upload(*D, lpk, &d.lt_pk))) return rc;
    if ((rc = upload(*D, ld, &d.lt_d))) return rc;
    if ((rc = upload(*D, lw, &d.lt_w))) return rc;
    if ((rc = upload(*D, lf, &d.lt_f))) return rc;
    if ((rc = upload(*D, leaf_vertices(s, sc->bvh), &d.leaf_v))) return rc;
    std::vector<BvhNode4> b4 = bfs_order(collapse_bvh4(sc->bvh)), lb4 = bfs_order(collapse_bvh4(sc->lbvh));
    for (const auto* t : {&b4, &lb4}) {
        const int need = bvh4_stack_need(*t);
        if (need > kStack) {
            set_error("the scene's %sBVH needs %d traversal stack entries, more than the %d the kernels hold "
                      "(degenerate geometry: too many coincident triangles)", t == &lb4 ? "light-only " : "", need, kStack);
            return MCPT_E_SCENE;
        }
    }
    if ((rc = pack_leaf_codes(b4)) || (rc = pack_leaf_codes(lb4))) return rc;
    d.nbvh4 = (int)b4.size();
    d.nlbvh4 = (int)lb4.size();
    if ((rc = upload(*D, b4, &d.bvh4))) return rc;
    if ((rc = upload(*D, lb4, &d.lbvh4))) return rc;
    if ((rc = upload(*D, quantize_bvh4(b4), &d.bvh4q))) return rc;
    if ((rc = upload(*D, quantize_bvh4(lb4), &d.lbvh4q))) return rc;
    if ((rc = upload(*D, leaf_vertices(s, sc->lbvh), &d.lleaf_v))) return rc;
    HIP_OK(hipStreamCreateWithFlags(&D->stream, hipStreamNonBlocking));
    HIP_OK(hipHostMalloc(&D->pinned_count, 64 + kCtrlBytes));
    HIP_OK(hipEventCreate(&D->ev0));
    HIP_OK(hipEventCreate(&D->ev1));
    HIP_OK(hipEventCreate(&D->evp0));
    HIP_OK(hipEventCreate(&D->evp1));
    HIP_OK(hipEventCreate(&D->evr0));
    HIP_OK(hipEventCreate(&D->evr1));
    *out = D.get();
    std::lock_guard<std::mutex> lk(sc->devs_mu);
    sc->devs.push_back(std::move(D));
    return MCPT_OK;
}

int alloc_aux(DevBuf* b, int cap, Aux& a) {
    const size_t c = (size_t)cap;
    const size_t sz[9] = {24 * c, 24 * c, 24 * c, 24 * c, 16 * c, 2 * 16 * c, 4 * c, 3 * 4 * c, 8 * c};
    for (int k = 0; k < 9; k++) {
        int rc = ensure(b[k], sz[k]);
        if (rc) return rc;
    }
    a.d1 = (double*)b[0].p;
    a.d2 = (double*)b[1].p;
    a.w1 = (double*)b[2].p;
    a.w2 = (double*)b[3].p;
    a.c2 = (double*)b[4].p;
    a.hbg = (double*)b[5].p;
    a.flags = (int*)b[6].p;
    a.hf = (int*)b[7].p;
    a.s1 = (double*)b[8].p;
    a.cap = cap;
    return MCPT_OK;
}

// the MIS tree-reduction slot pool (Slots): per-slot arrays, per-shard free rings and ready lists,
// control words.  grow = true keeps the contents of a smaller pool (called between passes, stream
// idle: each shard's ring entries [head, tail) are re-packed from 0, its ready list rp keeps its
// entries; slot ids stay valid).
constexpr int kSlotArrays = 13;
int slot_bytes_per(int k) {  // rec - pend - - - Ll - last (arrays 1, 3, 4, 5, 7 unused)
    static const int b[9] = {8 * kSlotRec, 0, 4, 0, 0, 0, 24, 0, 112};
    return b[k];
}
size_t slot_array_bytes(int k, int rcap) {
    const size_t cap = (size_t)rcap * kSlotShards;
    if (k < 9) return (size_t)slot_bytes_per(k) * cap;
    if (k == 9) return 4 * cap * kSlotShards;                    // rings: cap entries per shard
    if (k < 12) return 4ull * kSlotShards * (2ull * rcap + 256);  // ready lists
    return kCtrlBytes;
}
void slots_view(DevBuf* b, int rcap, Slots& T) {
    T.rec = (double*)b[0].p, T.pend = (int*)b[2].p, T.Ll = (double*)b[6].p, T.last = (double*)b[8].p;
    T.ring = (int*)b[9].p, T.ready0 = (int*)b[10].p, T.ready1 = (int*)b[11].p, T.ctrl = (unsigned*)b[12].p;
    T.rcap = rcap;
    T.cap = rcap * kSlotShards;
    T.ring_cap = T.cap;
    T.ready_cap = 2 * rcap + 256;
}
int alloc_slots(DevBuf* b, int rcap, Slots& T, hipStream_t st, bool grow, int rp, const unsigned* ctrl_host) {
    if (!grow) {
        for (int k = 0; k < kSlotArrays; k++) {
            int rc = ensure(b[k], slot_array_bytes(k, rcap));
            if (rc) return rc;
        }
        slots_view(b, rcap, T);
        HIP_OK(hipMemsetAsync(T.ctrl, 0, kCtrlBytes, st));
        return MCPT_OK;
    }
    const Slots old = T;
    DevBuf nb[kSlotArrays];
    for (int k = 0; k < kSlotArrays; k++) {
        int rc = ensure(nb[k], slot_array_bytes(k, rcap));
        if (rc) return rc;
    }
    Slots nt{};
    slots_view(nb, rcap, nt);
    for (int k = 0; k < 9; k++)  // per-slot data keep their slot ids
        HIP_OK(hipMemcpyAsync(nb[k].p, b[k].p, (size_t)slot_bytes_per(k) * old.cap, hipMemcpyDeviceToDevice, st));
    std::vector<unsigned> c(kSlotShards * 16, 0u);
    for (int sh = 0; sh < kSlotShards; sh++) {
        const unsigned* oc = ctrl_host + 16 * sh;
        const unsigned head = oc[1], nfree = oc[2] - oc[1], nready = oc[4 + rp];
        for (unsigned k = 0; k < nfree;) {  // this shard's ring, in contiguous pieces of the old circle
            const unsigned from = (head + k) % (unsigned)old.ring_cap, len = std::min(nfree - k, (unsigned)old.ring_cap - from);
            HIP_OK(hipMemcpyAsync(nt.ring + (size_t)sh * nt.ring_cap + k, old.ring + (size_t)sh * old.ring_cap + from, 4ull * len,
                                  hipMemcpyDeviceToDevice, st));
            k += len;
        }
        if (nready)
            HIP_OK(hipMemcpyAsync((rp ? nt.ready1 : nt.ready0) + (size_t)sh * nt.ready_cap,
                                  (rp ? old.ready1 : old.ready0) + (size_t)sh * old.ready_cap, 4ull * nready,
                                  hipMemcpyDeviceToDevice, st));
        unsigned* w = &c[16 * sh];
        w[0] = oc[0], w[1] = 0, w[2] = nfree, w[3] = nfree, w[4 + rp] = nready;
    }
    HIP_OK(hipMemcpyAsync(nt.ctrl, c.data(), kCtrlBytes, hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
    for (int k = 0; k < kSlotArrays; k++) {
        if (b[k].p) HIP_OK(hipFree(b[k].p));
        b[k] = nb[k];
    }
    T = nt;
    return MCPT_OK;
}

int alloc_queue(DevBuf* b, int cap, Queue& q) {
    const size_t c = (size_t)cap;
    const size_t sz[14] = {24 * c, 24 * c, 24 * c, 24 * c, 4 * c, 4 * c, 4 * c, 8 * c, 8 * c, 4 * c, 64, 4 * c, 0, 0};
    for (int k = 0; k < 12; k++) {
        int rc = ensure(b[k], sz[k]);
        if (rc) return rc;
    }
    q.p = (double*)b[0].p;
    q.n = (double*)b[1].p;
    q.wo = (double*)b[2].p;
    q.tp = (double*)b[3].p;
    q.f = (int*)b[4].p;
    q.pixel = (int*)b[5].p;
    q.sample = (int*)b[6].p;
    q.node = (uint64_t*)b[7].p;
    q.wsum = (double*)b[8].p;
    q.pick = (int*)b[9].p;
    q.count = (unsigned*)b[10].p;
    q.par = (int*)b[11].p;
    q.cap = cap;
    return MCPT_OK;
}

int validate_camera(const mcpt_camera* cam) {
    if (!cam || cam->width <= 0 || cam->height <= 0 || cam->dist_scale <= 0) {
        set_error("invalid camera");
        return MCPT_E_INVALID;
    }
    return MCPT_OK;
}

int prep_chunks(int NL) { return std::max(1, (NL + 63) / 64); }
size_t prep_lds_bytes(int nchunks) { return 4 * ((size_t)nchunks * sizeof(double) + kPrepQueue * sizeof(int)); }
// per-wave LDS bytes of k_prep_pk2: batch totals + uint16 candidate list, 16-byte aligned
int prep_list_wave_bytes(int nchunks) { return (int)((nchunks * 8 + nchunks * 64 * 2 + 15) / 16 * 16); }
constexpr int kPrepListMaxLds = 64 * 1024;  // per 4-wave block

// Light-prep dispatch.  variant: -1 auto; 0 k_prep (per-wave LDS candidate queue: any N_L); 8
// k_prep_pk2 (cheap stages + stored LDS candidate list + fp64 batches in one kernel); 9 k_prep_lane
// (lane per node, N_L <= kSmallNL); 17 k_prep_cull_lanes + k_prep_pk2<mask-in> (the renderer's
// form: needs the candidate-word scratch `masks`).  Auto: 9 for few lights, else 17 with masks, 8
// without, 0 when the candidate list does not fit in LDS.  Cache builds run 8 or 17.
// work: a device word, zeroed here before the launch (the kernel's dynamic node counter)
// the fp32 variant's launch bound: 5 waves/SIMD (81 VGPRs; 6 forces 80: -0.8% same-box)
#ifndef MCPT_PK2_F32_WAVES
#define MCPT_PK2_F32_WAVES 5
#endif
constexpr int kPk2F32Waves = MCPT_PK2_F32_WAVES;
// the fp64 split form's launch bound (waves/SIMD): 6 keeps it at 72 VGPRs (7 waves by registers)
// since the exact-pick bookkeeping; 5 let it grow to 75 (same-box A/B with the pick at 7: +1.2%)
#ifndef MCPT_PK2_WAVES
#define MCPT_PK2_WAVES 6
#endif
constexpr int kPk2Waves = MCPT_PK2_WAVES;
// whether launch_prep(-1, ...) with these masks takes the split form (variant 17), which writes every
// node's candidate words (k_prep_exact reads them instead of redoing the cheap stages)
inline bool prep_writes_masks(const DScene& d, const uint64_t* masks) {
    return masks && d.NL > kSmallNL && d.NL <= 65535 && 4 * prep_list_wave_bytes(prep_chunks(d.NL)) <= kPrepListMaxLds;
}
// k_prep_lane (N_L <= kSmallNL) with its running sums kept in registers up to 16 lights; build: the nodes
// are root points whose rows go to the SmallCache
hipError_t launch_prep_lane(const DScene& d, uint64_t seed, int n, const double* qp, const double* qn, int qs,
                            const int* qpixel, const int* qsample, const uint64_t* qnode, const double* u, double* wsum,
                            int* pick, int* count, unsigned long long* stats, hipStream_t st, const SmallCache& C, bool build) {
    if (n <= 0) return hipSuccess;
    const dim3 g((n + 255) / 256), b(256);
#define MCPT_LANE(K)                                                                                                     \
    do {                                                                                                                 \
        if (build)                                                                                                       \
            hipLaunchKernelGGL((k_prep_lane<K, true>), g, b, 0, st, d, seed, n, qp, qn, qs, qpixel, qsample, qnode, u, wsum, \
                               pick, count, stats, C);                                                                   \
        else                                                                                                             \
            hipLaunchKernelGGL((k_prep_lane<K, false>), g, b, 0, st, d, seed, n, qp, qn, qs, qpixel, qsample, qnode, u,      \
                               wsum, pick, count, stats, C);                                                             \
    } while (0)
    if (d.NL <= 4) MCPT_LANE(4);
    else if (d.NL <= 16) MCPT_LANE(16);
    else MCPT_LANE(0);
#undef MCPT_LANE
    return hipGetLastError();
}
hipError_t launch_prep(int variant, const DScene& d, uint64_t seed, int n, const double* qp, const double* qn, int qs,
                       const int* qpixel, const int* qsample, const uint64_t* qnode, const double* u, double* wsum,
                       int* pick, int* count, unsigned long long* stats, unsigned* work, hipStream_t st,
                       const PrepCache& cache = PrepCache{}, uint64_t* masks = nullptr, bool count_c1 = true,
                       bool fp32 = false, const CullOrder& co = CullOrder{}) {
    const int nchunks = prep_chunks(d.NL);
    const int wb = prep_list_wave_bytes(nchunks);
    const bool list_ok = d.NL <= 65535 && 4 * wb <= kPrepListMaxLds;
    if (variant < 0) variant = d.NL <= kSmallNL ? 9 : list_ok ? (masks ? 17 : 8) : 0;  // A/B: tools/prep_variants.py
    if (variant != 0 && variant != 8 && variant != 9 && variant != 17 && variant != 18) return hipErrorInvalidValue;
    const bool ordered = variant == 17;  // 18: variant 17 without the node order and the chunk classes (A/B, tests)
    if (variant == 18) variant = 17;
    if (variant == 9) return launch_prep_lane(d, seed, n, qp, qn, qs, qpixel, qsample, qnode, u, wsum, pick, count, stats, st,
                                              SmallCache{}, false);
    if (variant > 0 && !list_ok) variant = 0;
    if (variant == 17 && !masks) variant = 8;  // the split form needs the candidate-word scratch
    if (cache.build && variant != 8 && variant != 17) return hipErrorInvalidValue;
    // enough 4-wave blocks to fill every CU twice over; the work counter balances the load
    const int blocks = std::max(1, std::min((n + 4 * kPrepGrab - 1) / (4 * kPrepGrab), 2048));
    hipError_t e = hipMemsetAsync(work, 0, sizeof(unsigned), st);
    if (e != hipSuccess) return e;
    if (variant == 0) {
        hipLaunchKernelGGL(k_prep, dim3(blocks), dim3(256), prep_lds_bytes(nchunks), st, d, seed, n, qp, qn, qs, qpixel,
                           qsample, qnode, u, wsum, pick, count, stats, nchunks, work, cache.slack, cache.exact_off,
                           cache.exact_counts, cache.maybe);
    } else if (variant == 17) {  // phase A lane per node (light table in scalar registers), then phase B
        const int* order = nullptr;
        if (co.order && ordered) {  // the nodes bucketed by their chunk-class pattern
            e = hipMemsetAsync(co.count, 0, 8 * kCullBuckets, st);
            if (e != hipSuccess) return e;
            const dim3 go((n + 256 * kCullPer - 1) / (256 * kCullPer));
            hipLaunchKernelGGL(k_cull_classify, go, dim3(256), 0, st, d, n, qp, qn, qs, nchunks, co.keys, co.count);
            hipLaunchKernelGGL(k_cull_scatter, go, dim3(256), 0, st, n, (const unsigned char*)co.keys, co.count, co.order);
            order = co.order;
        }
        if (count_c1 || !stats)
            hipLaunchKernelGGL(k_prep_cull_lanes<true>, dim3((n + 255) / 256, cull_splits(nchunks)), dim3(256), 0, st, d,
                               n, qp, qn, qs, masks, nchunks, stats, order);
        else
            hipLaunchKernelGGL(k_prep_cull_lanes<false>, dim3((n + 255) / 256, cull_splits(nchunks)), dim3(256), 0, st, d,
                               n, qp, qn, qs, masks, nchunks, stats, order);
        // fp32: MCPT_RENDER_PRECISION_FP32's packed-fp32 full stage (light_weight_f32x2)
        auto kern = cache.build ? (fp32 ? k_prep_pk2<kPk2F32Waves, true, true, true> : k_prep_pk2<kPk2Waves, true, true, false>)
                                : (fp32 ? k_prep_pk2<kPk2F32Waves, false, true, true> : k_prep_pk2<kPk2Waves, false, true, false>);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 4 * wb, st, d, seed, n, qp, qn, qs, qpixel, qsample, qnode, u, wsum,
                           pick, count, stats, nchunks, wb, work, cache, masks);
    } else if (cache.build) {
        hipLaunchKernelGGL((k_prep_pk2<5, true>), dim3(blocks), dim3(256), 4 * wb, st, d, seed, n, qp, qn, qs, qpixel,
                           qsample, qnode, u, wsum, pick, count, stats, nchunks, wb, work, cache);
    } else {
        hipLaunchKernelGGL((k_prep_pk2<5, false>), dim3(blocks), dim3(256), 4 * wb, st, d, seed, n, qp, qn, qs, qpixel,
                           qsample, qnode, u, wsum, pick, count, stats, nchunks, wb, work, cache);
    }
    return hipGetLastError();
}

// builds the scene's uniform grid for (eye, n0) unless it already is (host side; NOT thread-safe:
// render_multi calls it on the calling thread before its device workers start, so the workers only
// find an up-to-date grid and read it)
int ensure_host_grid(mcpt_scene* sc, const double eye[3], int n0) {
    Grid& g = sc->grid;
    if (!g.ok || g.n0 != n0 || g.eye[0] != eye[0] || g.eye[1] != eye[1] || g.eye[2] != eye[2]) {
        g = build_grid(sc->host, eye, n0);
        sc->grid_version++;
    }
    if (!g.ok) {
        set_error("the scene's bounding box has zero or non-finite extent: no uniform grid (Myobj.cpp:110-162)");
        return MCPT_E_SCENE;
    }
    return MCPT_OK;
}

// ensure_host_grid, then brings D's copy up to date
int use_grid(mcpt_scene* sc, DeviceState& D, const double eye[3], int n0) {
    int rg;
    if ((rg = ensure_host_grid(sc, eye, n0))) return rg;
    const Grid& g = sc->grid;
    if (D.grid_version != sc->grid_version) {
        int rc;
        if ((rc = ensure(D.g_start, g.cell_start.size() * 4)) || (rc = ensure(D.g_tri, g.cell_tri.size() * 4))) return rc;
        HIP_OK(hipMemcpy(D.g_start.p, g.cell_start.data(), g.cell_start.size() * 4, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(D.g_tri.p, g.cell_tri.data(), g.cell_tri.size() * 4, hipMemcpyHostToDevice));
        D.d.g_start = (const int*)D.g_start.p;
        D.d.g_tri = (const int*)D.g_tri.p;
        for (int i = 0; i < 3; i++) {
            D.d.g_mn[i] = g.mn[i];
            D.d.g_lim[i] = g.lim[i];
            D.d.g_gd[i] = g.gd[i];
        }
        D.d.g_inv_d = g.inv_d;
        D.grid_version = sc->grid_version;
    }
    return MCPT_OK;
}

// every option a render checks before it starts (spp, sample range, mode, acceleration, flags) --
// called first by every path, and by every rank of a communicator before any collective, so that a
// bad option fails on all ranks alike instead of leaving some of them in the reduce
// the 8-wide trees (k_rays_cw8, MCPT_DEBUG_RAYS_CW8 / MCPT_DEBUG_HIT_CW8, mcpt_debug_bvh8_check): built on the
// host on first use (1.2 s for the 1 M-triangle scene, so only runs that ask for them pay it) and uploaded to
// a device on its first use there; a tree whose reserved node slots exceed the 24-bit stack base stays null
void ensure_bvh8_host(mcpt_scene* sc) {
    std::lock_guard<std::mutex> lk(sc->bvh8_mu);
    if (sc->bvh8_built) return;
    sc->bvh8 = build_bvh8(sc->host, sc->bvh);
    sc->lbvh8 = build_bvh8(sc->host, sc->lbvh);
    sc->bvh8_built = true;
}
int ensure_bvh8(mcpt_scene* sc, DeviceState* D) {
    ensure_bvh8_host(sc);
    if (D->bvh8_tried) return MCPT_OK;
    DScene& d = D->d;
    const HostScene& s = sc->host;
    int rc;
    HIP_OK(hipSetDevice(D->device));
    // a failed upload (e.g. out of memory) leaves no half-uploaded tree behind and is retried by the next call,
    // so its error is reported each time instead of a later "no 8-wide tree"; only success marks the device tried
    // (a tree too large for the 24-bit stack base then stays null by design)
    struct Undo {
        DScene& d;
        bool armed = true;
        ~Undo() {
            if (armed) d.bvh8 = d.lbvh8 = nullptr, d.tri8_v = d.ltri8_v = nullptr;
        }
    } undo{d};
    for (int t = 0; t < 2; t++) {
        const Bvh8& b8 = t == 0 ? sc->bvh8 : sc->lbvh8;
        // trace_cw8 / k_rays_cw8 push at most one node group per level: a tree deeper than kStack could drop one
        if (b8.nodes.empty() || b8.nodes.size() >= (1u << 24) || b8.depth > kStack) continue;
        std::vector<float4> tv8(3 * std::max<size_t>(b8.tri_facets.size(), 1), make_float4(0.f, 0.f, 0.f, 0.f));
        for (size_t q = 0; q < b8.tri_facets.size(); q++) {
            const int f = b8.tri_facets[q];
            if (f < 0) continue;
            for (int k = 0; k < 3; k++) {
                float w;
                std::memcpy(&w, &f, 4);
                tv8[3 * q + k] = make_float4(s.pos[9 * f + 3 * k], s.pos[9 * f + 3 * k + 1], s.pos[9 * f + 3 * k + 2], k == 0 ? w : 0.0f);
            }
        }
        if ((rc = upload(*D, b8.nodes, t == 0 ? &d.bvh8 : &d.lbvh8))) return rc;
        if ((rc = upload(*D, tv8, t == 0 ? &d.tri8_v : &d.ltri8_v))) return rc;
    }
    undo.armed = false;
    D->bvh8_tried = true;
    return MCPT_OK;
}

int validate_render(const mcpt_render_opts* o) {
    const int s0 = (o->sample_begin == 0 && o->sample_end == 0) ? 0 : o->sample_begin;
    const int s1 = (o->sample_begin == 0 && o->sample_end == 0) ? o->spp : o->sample_end;
    if (o->spp <= 0 || s0 < 0 || s1 < s0 || s1 > o->spp ||
        (o->mode != MCPT_MODE_MIS && o->mode != MCPT_MODE_BRDF && o->mode != MCPT_MODE_SHADE && o->mode != MCPT_MODE_SHADE_AREA) ||
        (o->accel != MCPT_ACCEL_BVH && o->accel != MCPT_ACCEL_GRID)) {
        set_error("invalid render options (spp %d, range [%d,%d), mode %d, accel %d)", o->spp, s0, s1, o->mode, o->accel);
        return MCPT_E_INVALID;
    }
    if (o->flags & ~(MCPT_RENDER_NO_BACKFACE_STATS | MCPT_RENDER_FRESH_PDF | MCPT_RENDER_PRECISION_FP32 |
                     MCPT_DEBUG_SPLIT_BRDF | MCPT_DEBUG_NO_ROOT_CACHE | MCPT_DEBUG_COUNT_TRAVERSAL |
                     MCPT_DEBUG_SHARD_RANKS | MCPT_DEBUG_RAYS_PERSIST | MCPT_DEBUG_RAYS_CW8 | MCPT_DEBUG_FUSED_CULL |
                     MCPT_DEBUG_NO_EXACT_DEFER)) {
        set_error("unknown mcpt_render_opts.flags bits 0x%x", (unsigned)o->flags);
        return MCPT_E_INVALID;
    }
    return MCPT_OK;
}

// the wavefront render into a device framebuffer already resident on D's device
int render_on_device(mcpt_scene* sc, DeviceState& D, const mcpt_camera* cam, const mcpt_render_opts* o,
                     double* dfb, mcpt_stats* stats) {
    const CamFrame cf = cam_setup(*cam);
    const int W = cam->width, H = cam->height, npx = W * H;
    const int s0 = (o->sample_begin == 0 && o->sample_end == 0) ? 0 : o->sample_begin;
    const int s1 = (o->sample_begin == 0 && o->sample_end == 0) ? o->spp : o->sample_end;
    {
        const int rv = validate_render(o);
        if (rv) return rv;
    }
    // MCPT_ACCEL_GRID: the reference's uniform grid over the scene and this camera's eye, n0 =
    // 100000 (main.cpp:501-504), built here unless the scene already holds that grid
    const bool grid = o->accel == MCPT_ACCEL_GRID;
    if (grid) {
        const double eye[3] = {cf.eye.x, cf.eye.y, cf.eye.z};
        int rg;
        if ((rg = use_grid(sc, D, eye, 100000))) return rg;
    }
    // Path regeneration (wavefront with refill): before every generation the current queue is
    // topped up with fresh camera samples (roots) to `target` nodes, so every prep/extend launch
    // is large until the final drain; roots are taken in global order r = (sample - s0) * npx +
    // pixel.  samples_per_launch (if set) sets target = samples_per_launch * npx.
    const long long R = (long long)(s1 - s0) * npx;
    // root order: sample-minor when the acceleration structures exceed an XCD's 4 MiB L2 (the
    // secondary rays of consecutive roots then share their origin and top-down paths: C5 +10%),
    // sample-major otherwise (Veach: the root-point cache's per-pixel reads spread; -3% minor)
    const uint64_t accel = (uint64_t)(D.d.nbvh4 + D.d.nlbvh4) * sizeof(BvhNode4) +
                           (uint64_t)(sc->bvh.leaf_facets.size() + sc->lbvh.leaf_facets.size()) * 3 * sizeof(float4);
    const int nminor = (MCPT_ROOT_MINOR > 0 || (MCPT_ROOT_MINOR < 0 && accel > (4ull << 20))) ? s1 - s0
                                                                                              : std::min(MCPT_ROOT_GROUP, s1 - s0);
    const int qf = o->queue_factor > 0 ? o->queue_factor : 2;
    // default working set: MCPT_WORKING_SET nodes (48 Mi: fewer, larger generations amortise each
    // launch's tail -- measured +6% Veach, +21% Cornell-1M over 4 Mi), but no more than the call's
    // camera samples (a small render holds all its roots at once) and no more than half the free
    // HBM (the other half is left to the root-point cache and the caller)
    size_t ws_held = D.masks.bytes, ws_free = 0, ws_total = 0;
    for (int k = 0; k < 14; k++) ws_held += D.qa[k].bytes + D.qb[k].bytes;
    for (int k = 0; k < 9; k++) ws_held += D.aux[k].bytes;
    for (int k = 0; k < 13; k++) ws_held += D.sl[k].bytes;
    HIP_OK(hipMemGetInfo(&ws_free, &ws_total));
    const size_t ws_node_bytes = 2 * 132 + 152 + 8 * (size_t)mask_stride(prep_chunks(D.d.NL)) + 280;  // queues aux words slots
    const long long ws_mem = (long long)((ws_free + ws_held) / 2 / ((size_t)qf * ws_node_bytes));
    const long long target_ll =
        o->samples_per_launch > 0
            ? (long long)o->samples_per_launch * npx
            : std::min<long long>({(long long)MCPT_WORKING_SET, std::max<long long>(R, 1024), std::max<long long>(ws_mem, 1 << 20)});
    if (target_ll > (1ll << 29)) {
        set_error("batch too large");
        return MCPT_E_INVALID;
    }
    const int target = (int)std::max<long long>(target_ll, 1);
    const int cap = (int)std::min<long long>((long long)qf * target + 1024, (1ll << 30));
    int rc;
    if ((rc = ensure(D.hit_f, 4ull * npx)) || (rc = ensure(D.hit_tbg, 24ull * npx)) ||
        (rc = ensure(D.root_pnw, 72ull * npx)) || (rc = ensure(D.root_kind, 4ull * npx)) || (rc = ensure(D.stats, kStatBytes)) ||
        (rc = ensure(D.work, 256)))
        return rc;
    Queue qa, qb;
    if ((rc = alloc_queue(D.qa, cap, qa)) || (rc = alloc_queue(D.qb, cap, qb))) return rc;
    // extension kernels: MIS and shade split into gen / rays / combine (measured faster), BRDF-only
    // keeps the single kernel (one ray per node; measured faster).  A/B switches:
    const bool count_trav = (o->flags & MCPT_DEBUG_COUNT_TRAVERSAL) != 0;
#define K_MIS_RAYS (grid ? k_mis_rays<true> : count_trav ? k_mis_rays<false, true> : k_mis_rays<false>)

    const bool split_brdf = (o->flags & MCPT_DEBUG_SPLIT_BRDF) != 0;
    // the O(N_L) light prep runs for shade_with_mis and for shade() with the spherical sampler
    const bool needs_prep = o->mode == MCPT_MODE_MIS || o->mode == MCPT_MODE_SHADE;
    const bool fused = !grid && o->mode == MCPT_MODE_BRDF && !split_brdf;  // BRDF-only: k_extend_brdf (the grid runs split)
    Aux aux{};
    if (!fused && (rc = alloc_aux(D.aux, cap, aux))) return rc;
    // shade_with_mis reduces its trees bottom-up to evaluate the BRDF branch's light pdf with the
    // reference's (stale) sampler state, unless MCPT_RENDER_FRESH_PDF asks for the node's own
    const bool stale = o->mode == MCPT_MODE_MIS && !(o->flags & MCPT_RENDER_FRESH_PDF);
    Slots T{};
    int rp = 0;  // ready list being filled
    const unsigned* hctrl = D.pinned_count + 16;  // slot control words, read back with the queue count
    hipStream_t st = D.stream;
    if (stale && (rc = alloc_slots(D.sl, std::max(cap, 1 << 16) / kSlotShards + 1, T, st, false, 0, nullptr))) return rc;
    Params P;
    P.S = D.d;
    P.seed = o->seed;
    P.inv_spp = 1.0 / o->spp;
    P.fb = dfb;
    P.stats = (unsigned long long*)D.stats.p;
    P.mode = o->mode;
    P.root_pnw = nullptr;
    const int nchunks = prep_chunks(D.d.NL);
    const size_t prep_lds = prep_lds_bytes(nchunks);
    if (prep_lds > 160 * 1024) {
        set_error("too many light triangles for the LDS chunk table (%d)", D.d.NL);
        return MCPT_E_SCENE;
    }
    const bool count_c1 = !(o->flags & MCPT_RENDER_NO_BACKFACE_STATS);
    const bool fp32 = (o->flags & MCPT_RENDER_PRECISION_FP32) != 0;
    double prep_ms = 0, trace_ms = 0, cache_ms = 0;
    uint64_t gens = 0, prep_launches = 0, nodes_total = 0, cache_points = 0, trace_launches = 0, cached_roots = 0;
    // candidate words of the split light prep (k_prep_cull -> k_prep_pk2<mask-in>): per node and chunk
    uint64_t* masks = nullptr;
    CullOrder corder{};
    if (needs_prep && D.d.NL > kSmallNL) {
        if ((rc = ensure(D.masks, (size_t)std::max(cap, npx) * mask_stride(nchunks) * 8))) return rc;
        masks = (uint64_t*)D.masks.p;
        if ((rc = cull_order_bufs(D, (size_t)std::max(cap, npx), &corder))) return rc;
    }
    // exact pick: nodes inside the ambiguity band go to k_prep_exact; the opt-in fp32
    // precision makes no exactness claim, and the small-table prep (k_prep_lane) is exact by construction
    // MCPT_EXACT_PICK=0 builds the pre-round-3 prep (VOS weights' own pick) for the cost A/B only
    const bool exact_pick = MCPT_EXACT_PICK && needs_prep && !fp32 && D.d.NL > kSmallNL;
    int *exact_list = nullptr, *maybe_list = nullptr;  // [0] count, entries from kExactHead
    double *exact_scr = nullptr, *slack = nullptr;
    if (exact_pick) {
        if ((rc = ensure(D.exact, 8ull * ((size_t)cap + kExactHead))) ||
            (rc = ensure(D.exact_scr, 8 * exact_scratch_doubles(D.d.NL))) || (rc = ensure(D.slack, 8ull * cap)))
            return rc;
        exact_list = (int*)D.exact.p;
        maybe_list = exact_list + cap + kExactHead;
#if MCPT_BAND_DIAG
        HIP_OK(hipMemset((double*)D.exact_scr.p + (size_t)exact_waves(D.d.NL) * ((D.d.NL + 63) & ~63) * 3 / 2, 0,
                         4ull * cam->width * cam->height));
#endif
        exact_scr = (double*)D.exact_scr.p;
        slack = (double*)D.slack.p;
    }
    // root-point cache (see PrepCache): built here when the call has >= 2 samples per pixel and the
    // entries fit in the free HBM less a 16 GiB reserve (800x600 with N_L = 3012: 15 GB; 1600x1200:
    // 60 GB -- sized for the 288 GB of an MI355X)
    PrepCache pc{};
    const int lstride = 64 * nchunks;
    const size_t cache_bytes = (size_t)npx * ((size_t)nchunks * 8 + (size_t)lstride * 10 + 16);
    size_t free_b = 0, total_b = 0;
    HIP_OK(hipMemGetInfo(&free_b, &total_b));
    const size_t held = D.cache_bt.bytes + D.cache_lst.bytes + D.cache_info.bytes + D.cache_w.bytes;
    const size_t budget = free_b + held > (16ull << 30) ? free_b + held - (16ull << 30) : 0;
    const bool no_cache = (o->flags & MCPT_DEBUG_NO_ROOT_CACHE) != 0;  // A/B switch
    if (needs_prep && s1 - s0 >= 2 && cache_bytes <= budget && !no_cache && D.d.NL > kSmallNL &&
        prep_list_wave_bytes(nchunks) * 4 <= kPrepListMaxLds && D.d.NL <= 65535) {
        if ((rc = ensure(D.cache_bt, (size_t)npx * nchunks * 8)) || (rc = ensure(D.cache_lst, (size_t)npx * lstride * 2)) ||
            (rc = ensure(D.cache_info, (size_t)npx * 16)) || (rc = ensure(D.cache_w, (size_t)npx * lstride * 8)))
            return rc;
        pc.w = (double*)D.cache_w.p;
        pc.bt = (double*)D.cache_bt.p;
        pc.lst = (unsigned short*)D.cache_lst.p;
        pc.info = (int4*)D.cache_info.p;
        pc.lstride = lstride;
        pc.use = 1;  // built below, inside the timed region
    }
    // the small-table prep's root-point cache (SmallCache: N_L <= kSmallNL, e.g. the Cornell scene's
    // 2-triangle light): (N_L + 1.5) x 8 B per pixel
    SmallCache scache{};
    bool small_use = false;
    if (needs_prep && s1 - s0 >= 2 && !no_cache && D.d.NL > 0 && D.d.NL <= kSmallNL &&
        (size_t)npx * (8ull * D.d.NL + 12) <= budget) {
        if ((rc = ensure(D.sc_cum, 8ull * npx * D.d.NL)) || (rc = ensure(D.sc_wsum, 8ull * npx)) ||
            (rc = ensure(D.sc_last, 4ull * npx)))
            return rc;
        scache.cum = (double*)D.sc_cum.p;
        scache.wsum = (double*)D.sc_wsum.p;
        scache.last = (int*)D.sc_last.p;
        small_use = true;
    }
    RootLit rl{};  // roots' literal sums per pixel (k_prep_exact), up to 2 GiB of entries
    if (exact_pick && pc.use) {
        rl.stride = (lstride + 8 + 7) & ~7;
        rl.cap = (int)std::min<long long>({(long long)npx, (2ll << 30) / (8ll * rl.stride), 1ll << 20});
        if ((rc = ensure(D.lit_slot, 4ull * (npx + 16))) || (rc = ensure(D.lit_pool, 8ull * rl.stride * rl.cap))) return rc;
        rl.slot = (int*)D.lit_slot.p;
        rl.pool = (double*)D.lit_pool.p;
    }
    if ((MCPT_RAYS_CW8 || (o->flags & MCPT_DEBUG_RAYS_CW8)) && (rc = ensure_bvh8(sc, &D))) return rc;
    // which traversal the MIS / shade ray sets take: the persistent refilling waves for trees beyond an XCD's
    // 4 MiB L2 and for shade-area's rays (k_rays_persistent, or k_rays_cw8 on the 8-wide trees), else one ray
    // per thread (k_mis_rays)
    const bool rays_pers = !grid && ((o->flags & MCPT_DEBUG_RAYS_PERSIST) || MCPT_RAYS_PERSISTENT > 0 ||
                                     (MCPT_RAYS_PERSISTENT < 0 && accel > (4ull << 20)) ||
                                     (MCPT_PERSIST_SHADE_AREA && o->mode == MCPT_MODE_SHADE_AREA));
    // (round 6: k_rays_persistent handing the combine its hit points instead of (beta, gamma) was measured slower,
    // C5 -2..-6%, shade-area -9%: profiles/round6_ab_hit_points.txt)
    const bool rays_cw8 = rays_pers && (MCPT_RAYS_CW8 || (o->flags & MCPT_DEBUG_RAYS_CW8)) && D.d.bvh8 && D.d.lbvh8;
    // every buffer is allocated above (first-call hipMalloc of the cache is not device work); the
    // timed region (seconds, HIP events) starts at the primary-hit kernel
    HIP_OK(hipMemsetAsync(D.stats.p, 0, kStatBytes, st));
    HIP_OK(hipEventRecord(D.ev0, st));
    hipLaunchKernelGGL(grid ? k_primary<true> : k_primary<false>, dim3((npx + kTraceBlock - 1) / kTraceBlock), dim3(kTraceBlock),
                       0, st, D.d, cf, (int*)D.hit_f.p, (double*)D.hit_tbg.p);
    HIP_OK(hipGetLastError());
    RootTab rtab{(double*)D.root_pnw.p, (int*)D.root_kind.p};
    hipLaunchKernelGGL(k_root_table, dim3((npx + 255) / 256), dim3(256), 0, st, D.d, cf, (const int*)D.hit_f.p,
                       (const double*)D.hit_tbg.p, rtab);
    HIP_OK(hipGetLastError());
    if (fused) P.root_pnw = rtab.pnw;  // BRDF-only: lite root entries (Params::root_pnw)
    if (pc.use || small_use) {
        HIP_OK(hipMemsetAsync(qb.count, 0, 4, st));
        hipLaunchKernelGGL(k_root_points, dim3((npx + 255) / 256), dim3(256), 0, st, D.d, cf, (const int*)D.hit_f.p,
                           (const double*)D.hit_tbg.p, qb);
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpyAsync(D.pinned_count, qb.count, 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        int nr = (int)std::min<unsigned>(D.pinned_count[0], (unsigned)cap);
        if (D.pinned_count[0] > (unsigned)cap) {
            // more root points than the queue holds (a frame of more pixels than the working set under memory
            // pressure): k_root_points dropped some, and their pixels' cache rows would be stale -- no root cache
            // in this call, every root runs the full prep (same image, slower)
            pc.use = 0;
            small_use = false;
            rl = RootLit{};
            nr = 0;
        }
        if (nr > 0 && small_use) {
            HIP_OK(hipEventRecord(D.evp0, st));
            HIP_OK(launch_prep_lane(D.d, o->seed, nr, qb.p, qb.n, qb.cap, qb.pixel, nullptr, nullptr, nullptr, nullptr, nullptr,
                                    nullptr, P.stats, st, scache, true));
            HIP_OK(hipEventRecord(D.evp1, st));
            HIP_OK(hipEventSynchronize(D.evp1));
            float ms = 0;
            HIP_OK(hipEventElapsedTime(&ms, D.evp0, D.evp1));
            prep_ms += ms;
            cache_ms = ms;
            prep_launches++;
            cache_points = (uint64_t)nr;
        } else if (nr > 0) {
            pc.build = 1;
            HIP_OK(hipEventRecord(D.evp0, st));
            HIP_OK(launch_prep(masks ? 17 : 8, D.d, o->seed, nr, qb.p, qb.n, qb.cap, qb.pixel, nullptr, nullptr, nullptr, nullptr,
                               nullptr, nullptr, P.stats, (unsigned*)D.work.p, st, pc, masks, count_c1, fp32, corder));
            HIP_OK(hipEventRecord(D.evp1, st));
            HIP_OK(hipEventSynchronize(D.evp1));
            float ms = 0;
            HIP_OK(hipEventElapsedTime(&ms, D.evp0, D.evp1));
            prep_ms += ms;
            cache_ms = ms;
            prep_launches++;
            cache_points = (uint64_t)nr;
        }
        pc.build = 0;
        if (rl.slot) {  // a fresh set of per-pixel literal sums for this call's cache
            HIP_OK(hipMemsetAsync(rl.slot, 0, 64, st));
            HIP_OK(hipMemsetAsync(rl.slot + 16, 0xff, 4ull * npx, st));
        }
    }
    Queue* cur = &qa;
    Queue* nxt = &qb;
    HIP_OK(hipMemsetAsync(cur->count, 0, 4, st));
    long long rnext = 0;
    // Slicing: an MIS node has up to 2 children (shade / BRDF: 1), so a generation of at most `slice`
    // nodes always fits its children into nxt.  A larger generation (supercritical trees, e.g. occluded
    // lights: 2 x RR 0.6 = 1.2 children per node) parks its excess on a spill stack in HBM (grown on
    // demand) and takes it back, last in first out, before fresh roots -- so deep subtrees drain
    // first and the stack stays bounded by ~depth x slice.  The image does not depend on the order.
    const int branch = o->mode == MCPT_MODE_MIS ? 2 : 1;
    const int slice = cap / branch;
    const int fill = std::min(target, slice);  // refill / pop up to this many nodes per generation
    Queue qs{};
    long long spill_n = 0;
    uint64_t spilled = 0;
    auto grow_spill = [&](long long need) -> int {
        if (need <= D.spill_cap && qs.p) return MCPT_OK;
        if (need > (1ll << 30)) {
            set_error("spill stack beyond 2^30 nodes");
            return MCPT_E_DEVICE;
        }
        const int ncap = (int)std::min<long long>(std::max<long long>(need, 2ll * D.spill_cap), 1ll << 30);
        DevBuf nb[14];
        Queue nq;
        int r;
        if ((r = alloc_queue(nb, ncap, nq))) return r;
        if (spill_n > 0 && qs.p)
            hipLaunchKernelGGL(k_queue_move, dim3((unsigned)((spill_n + 255) / 256)), dim3(256), 0, st, qs, 0, nq, 0, (int)spill_n);
        HIP_OK(hipStreamSynchronize(st));
        for (int k = 0; k < 14; k++) {
            if (D.qs[k].p) HIP_OK(hipFree(D.qs[k].p));
            D.qs[k] = nb[k];
        }
        D.spill_cap = ncap;
        qs = nq;
        return MCPT_OK;
    };
    if (D.spill_cap > 0) {  // the stack of an earlier call (empty)
        int r;
        if ((r = alloc_queue(D.qs, D.spill_cap, qs))) return r;
    }
    auto read_count = [&](unsigned* out) -> int {  // cur's node count; fails on a queue overflow
        HIP_OK(hipMemcpyAsync(D.pinned_count, cur->count, 4, hipMemcpyDeviceToHost, st));
        HIP_OK(hipMemcpyAsync(D.pinned_count + 2, (char*)D.stats.p + 32, 8, hipMemcpyDeviceToHost, st));
        if (stale) HIP_OK(hipMemcpyAsync(D.pinned_count + 16, T.ctrl, kCtrlBytes, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        if (*(unsigned long long*)(D.pinned_count + 2)) {
            set_error("wavefront queue overflow (capacity %d); raise queue_factor", cap);
            return MCPT_E_OVERFLOW;
        }
        *out = std::min<unsigned>(D.pinned_count[0], (unsigned)cap);
        return MCPT_OK;
    };
    while (true) {
        unsigned n = 0;
        if ((rc = read_count(&n))) return rc;
        if (n > (unsigned)slice) {  // push the excess children onto the spill stack
            const int m = (int)n - slice;
            if ((rc = grow_spill(spill_n + m))) return rc;
            hipLaunchKernelGGL(k_queue_move, dim3((m + 255) / 256), dim3(256), 0, st, *cur, slice, qs, (int)spill_n, m);
            HIP_OK(hipGetLastError());
            spill_n += m;
            spilled += (uint64_t)m;
            n = (unsigned)slice;
            HIP_OK(hipMemsetD32Async((hipDeviceptr_t)cur->count, (int)n, 1, st));
        } else if (spill_n > 0 && n < (unsigned)fill) {  // pop spilled children before new roots
            const int m = (int)std::min<long long>((long long)fill - n, spill_n);
            spill_n -= m;
            hipLaunchKernelGGL(k_queue_move, dim3((m + 255) / 256), dim3(256), 0, st, qs, (int)spill_n, *cur, (int)n, m);
            HIP_OK(hipGetLastError());
            n += (unsigned)m;
            HIP_OK(hipMemsetD32Async((hipDeviceptr_t)cur->count, (int)n, 1, st));
        }
        const unsigned n_children = n;  // [0, n_children) children, [n_children, n) fresh roots
        if (rnext < R && n < (unsigned)fill) {  // refill with roots (appended through node_entry)
            const int m = (int)std::min<long long>((long long)fill - n, R - rnext);
            hipLaunchKernelGGL(k_roots_t, dim3((m + 256 * kRootsPT - 1) / (256 * kRootsPT)), dim3(256), 0, st, P,
                               (const int*)D.hit_f.p, npx, s0, rnext, m, *cur, std::max(1, nminor), s1 - s0, rtab,
                               P.root_pnw ? 1 : 0);
            HIP_OK(hipGetLastError());
            rnext += m;
            if ((rc = read_count(&n))) return rc;
        }
        if (n == 0) {
            if (rnext >= R && spill_n == 0) break;
            continue;  // every root of the refill terminated at entry: refill again
        }
        if (stale) {  // a shard serves at most ceil(blocks / 32) workgroups of 256 nodes per generation
            const unsigned per_shard = ((n + 255) / 256 + kSlotShards - 1) / kSlotShards * 256;
            unsigned bump = 0;
            for (int sh = 0; sh < kSlotShards; sh++) bump = std::max(bump, hctrl[16 * sh]);
            if (bump + per_shard > (unsigned)T.rcap) {
                const long long nr = std::max<long long>(2ll * T.rcap, (long long)bump + per_shard + 4096);
                if (nr * kSlotShards > (1ll << 30)) {
                    set_error("MIS reduction slot pool beyond 2^30 slots");
                    return MCPT_E_DEVICE;
                }
                if ((rc = alloc_slots(D.sl, (int)nr, T, st, true, rp, hctrl))) return rc;
            }
        }
        gens++;
        nodes_total += (uint64_t)n;
        const int ni = (int)n;
        // prep_seconds / prep_launches time the full light-prep kernel (k_prep_pk2) launches only
        bool timed = false;
        if (needs_prep) {
            PrepCache cx{};  // the children's full prep: no cache, the picks' slack
            int nmask = 0;   // nodes [0, nmask) have candidate words (k_prep_exact)
            int root_off = INT_MAX;  // nodes [root_off, ni) are roots with a cached candidate list
            cx.slack = slack;
            cx.maybe = maybe_list;
            if (exact_pick) {
                HIP_OK(hipMemsetAsync(exact_list, 0, 4, st));
                HIP_OK(hipMemsetAsync(maybe_list, 0, 4, st));
            }
            if (pc.use || small_use) {  // children: full prep; roots: pick from the root-point cache
                const int nc = (int)n_children, nr = ni - nc;
                if (nc > 0) {
                    // MCPT_DEBUG_FUSED_CULL (A/B): the cheap stages inside k_prep_pk2, wave per node (variant 8)
                    uint64_t* cmasks = (o->flags & MCPT_DEBUG_FUSED_CULL) ? nullptr : masks;
                    nmask = prep_writes_masks(D.d, cmasks) ? nc : 0;
                    HIP_OK(hipEventRecord(D.evp0, st));
                    HIP_OK(launch_prep(-1, D.d, o->seed, nc, cur->p, cur->n, cur->cap, cur->pixel, cur->sample, cur->node, nullptr,
                                       cur->wsum, cur->pick, nullptr, P.stats, (unsigned*)D.work.p, st, cx, cmasks,
                                       count_c1, fp32, corder));
                    HIP_OK(hipEventRecord(D.evp1, st));
                    timed = true;
                }
                // the cached roots are counted here (nr is known): the pick kernels' per-wave atomics on
                // one statistics word serialised at ~88 per us -- 2.3 of k_prep_lane_pick's 2.5 ms per C5 launch
                if (nr > 0) cached_roots += (uint64_t)nr;
                if (nr > 0 && small_use) {
                    hipLaunchKernelGGL(k_prep_lane_pick, dim3((nr + 255) / 256), dim3(256), 0, st, D.d, o->seed, nr,
                                       cur->pixel + nc, cur->sample + nc, cur->node + nc, cur->wsum + nc, cur->pick + nc,
                                       nullptr, scache);
                    HIP_OK(hipGetLastError());
                } else if (nr > 0) {
                    root_off = nc;
                    PrepCache pr = pc;
                    pr.exact = exact_list;
                    pr.exact_off = nc;
                    if (MCPT_PICK_GROUPS && nchunks <= 64) {  // 16 lanes per root
                        const int blocks = std::max(1, std::min((nr + 16 * kPickSlots - 1) / (16 * kPickSlots), 8192));
                        hipLaunchKernelGGL(k_prep_pick_g, dim3(blocks), dim3(256), 0, st, D.d, o->seed, nr, cur->pixel + nc,
                                           cur->sample + nc, cur->node + nc, cur->wsum + nc, cur->pick + nc, nullptr,
                                           nchunks, pr);
                    } else {
                        const int blocks = std::max(1, std::min((nr + 4 * kPickNodes - 1) / (4 * kPickNodes), 8192));
                        hipLaunchKernelGGL(k_prep_pick, dim3(blocks), dim3(256), 0, st, D.d, o->seed, nr, cur->pixel + nc,
                                           cur->sample + nc, cur->node + nc, cur->wsum + nc, cur->pick + nc, nullptr,
                                           nchunks, pr);
                    }
                    HIP_OK(hipGetLastError());
                }
            } else {
                nmask = prep_writes_masks(D.d, masks) ? ni : 0;
                HIP_OK(hipEventRecord(D.evp0, st));
                HIP_OK(launch_prep(-1, D.d, o->seed, ni, cur->p, cur->n, cur->cap, cur->pixel, cur->sample, cur->node, nullptr,
                                   cur->wsum, cur->pick, nullptr, P.stats, (unsigned*)D.work.p, st, cx, masks,
                                   count_c1, fp32, corder));
                HIP_OK(hipEventRecord(D.evp1, st));
                timed = true;
            }
            prep_launches += timed;
            if (exact_pick) {  // the band's nodes: the reference's literal prep and pick
                hipLaunchKernelGGL(k_prep_band, dim3(kBandBlocks), dim3(256), 0, st, D.d, maybe_list, slack, cur->p, cur->cap,
                                   masks, nmask, nchunks, exact_list, P.stats);
                // launch ids 2g and 2g + 1 (generation g): the follow-up launch reads what the first one stored
                const int lid = (int)std::min<uint64_t>(2 * gens, 2046);
                int* defer = MCPT_EXACT_DEFER && rl.slot && !(o->flags & MCPT_DEBUG_NO_EXACT_DEFER) ? maybe_list
                                                                                                    : nullptr;  // k_prep_band has consumed it
                if (defer) HIP_OK(hipMemsetAsync(defer, 0, 4, st));
                hipLaunchKernelGGL(k_prep_exact, dim3(exact_blocks(D.d.NL)), dim3(kExactBlock), 0, st, D.d, o->seed, exact_list,
                                   cur->p, cur->n, cur->cap, cur->pixel, cur->sample, cur->node, nullptr, cur->wsum, cur->pick,
                                   nullptr, P.stats, exact_scr, masks, nmask, nchunks, pc.use ? pc.lst : nullptr,
                                   pc.use ? pc.info : nullptr, pc.lstride, root_off,
                                   RootLit{rl.slot, rl.pool, rl.cap, rl.stride, lid}, defer);
                if (defer)  // the deferred roots (counted above already: no stats)
                    hipLaunchKernelGGL(k_prep_exact, dim3(exact_blocks(D.d.NL)), dim3(kExactBlock), 0, st, D.d, o->seed, defer,
                                       cur->p, cur->n, cur->cap, cur->pixel, cur->sample, cur->node, nullptr, cur->wsum,
                                       cur->pick, nullptr, nullptr, exact_scr, masks, nmask, nchunks, pc.use ? pc.lst : nullptr,
                                       pc.use ? pc.info : nullptr, pc.lstride, root_off,
                                       RootLit{rl.slot, rl.pool, rl.cap, rl.stride, lid + 1}, nullptr);
                HIP_OK(hipGetLastError());
            }
        }
        HIP_OK(hipMemsetAsync(nxt->count, 0, 4, st));
        const dim3 g256((ni + 255) / 256), b256(256);
        unsigned long long* tcnt = P.stats + 8;  // node visits, triangle tests (MCPT_DEBUG_COUNT_TRAVERSAL)
    auto launch_rays = [&](int first_set, int nsets, int seeded) {
        // shade() with uniform-area light points: its shadow and bounce rays run 4% faster on the refilling
        // persistent waves even on the small stand-in (shade_area 2 104-2 126 -> 2 185-2 191 Msamples/s, same
        // binary, profiles/round5_ab_persistent_veach.txt); MIS and shade() are slower there (-1%, -1%)
        if (rays_pers) {
            unsigned* pool = (unsigned*)D.work.p + 8;
            (void)hipMemsetAsync(pool, 0, sizeof(unsigned), st);
            const long long items = (long long)nsets * ni;
            const int blocks = (int)std::max<long long>(1, std::min<long long>((items + kRayBlock - 1) / kRayBlock, 2048));
            if (rays_cw8) {
                if (count_trav)
                    hipLaunchKernelGGL(k_rays_cw8<true>, dim3(blocks), dim3(kRayBlock), 0, st, D.d, *cur, ni, aux, first_set, nsets,
                                       pool, tcnt, MCPT_SEED_LIGHT ? seeded : 0);
                else
                    hipLaunchKernelGGL(k_rays_cw8<false>, dim3(blocks), dim3(kRayBlock), 0, st, D.d, *cur, ni, aux, first_set, nsets,
                                       pool, tcnt, MCPT_SEED_LIGHT ? seeded : 0);
            } else if (count_trav)
                hipLaunchKernelGGL(k_rays_persistent<true>, dim3(blocks), dim3(kRayBlock), 0, st, D.d, *cur, ni, aux,
                                   first_set, nsets, pool, tcnt, MCPT_SEED_LIGHT ? seeded : 0);
            else
                hipLaunchKernelGGL(k_rays_persistent<false>, dim3(blocks), dim3(kRayBlock), 0, st, D.d, *cur, ni, aux,
                                   first_set, nsets, pool, tcnt, MCPT_SEED_LIGHT ? seeded : 0);
        } else {
            hipLaunchKernelGGL(K_MIS_RAYS, dim3((ni + kRayBlock - 1) / kRayBlock, nsets), dim3(kRayBlock), 0, st, D.d,
                               *cur, ni, aux, first_set, tcnt, MCPT_SEED_LIGHT ? seeded : 0,
                               o->mode == MCPT_MODE_MIS ? 0 : 1);
        }
    };
        // trace_seconds: HIP events around the traversal kernel (k_mis_rays; BRDF-only: k_extend_brdf)
        if (!fused && o->mode == MCPT_MODE_MIS) {
            hipLaunchKernelGGL(stale ? k_mis_gen<true> : k_mis_gen<false>, g256, b256, 0, st, P, *cur, ni, aux);
            HIP_OK(hipEventRecord(D.evr0, st));
            launch_rays(0, 3, 1);
            HIP_OK(hipEventRecord(D.evr1, st));
            hipLaunchKernelGGL(stale ? k_mis_combine<true> : k_mis_combine<false>, g256, b256, 0, st, P, *cur, ni, aux,
                               *nxt, T, rp);
            if (stale) {  // one level of the bottom-up reduction per generation
                hipLaunchKernelGGL(k_mis_complete, dim3(32, kSlotShards), dim3(256), 0, st, P, T, rp);
                hipLaunchKernelGGL(k_slot_fixup, dim3(1), dim3(kSlotShards), 0, st, T, rp);
                rp ^= 1;
            }
        } else if (!fused && (o->mode == MCPT_MODE_SHADE || o->mode == MCPT_MODE_SHADE_AREA)) {
            hipLaunchKernelGGL(k_shade_gen, g256, b256, 0, st, P, *cur, ni, aux);
            HIP_OK(hipEventRecord(D.evr0, st));
            launch_rays(0, 2, 1);
            HIP_OK(hipEventRecord(D.evr1, st));
            hipLaunchKernelGGL(k_shade_combine, g256, b256, 0, st, P, *cur, ni, aux, *nxt);
        } else if (!fused) {
            hipLaunchKernelGGL(k_brdf_gen, g256, b256, 0, st, P, *cur, ni, aux);
            HIP_OK(hipEventRecord(D.evr0, st));
            launch_rays(1, 1, 0);
            HIP_OK(hipEventRecord(D.evr1, st));
            hipLaunchKernelGGL(k_brdf_combine, g256, b256, 0, st, P, *cur, ni, aux, *nxt);
        } else {
            HIP_OK(hipEventRecord(D.evr0, st));
            hipLaunchKernelGGL(count_trav ? k_extend_brdf<true> : k_extend_brdf<false>, dim3((ni + kBrdfBlock - 1) / kBrdfBlock),
                               dim3(kBrdfBlock), 0, st, P, *cur, ni, *nxt);
            HIP_OK(hipEventRecord(D.evr1, st));
        }
        HIP_OK(hipGetLastError());
        trace_launches++;
        if (timed) {
            float ms = 0;
            HIP_OK(hipEventSynchronize(D.evp1));
            HIP_OK(hipEventElapsedTime(&ms, D.evp0, D.evp1));
            prep_ms += ms;
        }
        {
            float ms = 0;
            HIP_OK(hipEventSynchronize(D.evr1));
            HIP_OK(hipEventElapsedTime(&ms, D.evr0, D.evr1));
            trace_ms += ms;
        }
        std::swap(cur, nxt);
        if (o->progress && o->progress(o->progress_user, (uint64_t)rnext, (uint64_t)R)) {
            HIP_OK(hipStreamSynchronize(st));
            set_error("render cancelled by the progress callback after %lld of %lld camera samples", rnext, R);
            return MCPT_E_CANCELLED;
        }
    }
    while (stale) {  // drain the reduction: the trees' remaining levels up to their roots
        HIP_OK(hipMemcpyAsync(D.pinned_count + 16, T.ctrl, kCtrlBytes, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        unsigned pending = 0;
        for (int sh = 0; sh < kSlotShards; sh++) pending += hctrl[16 * sh + 4 + rp];
        if (pending == 0) break;
        hipLaunchKernelGGL(k_mis_complete, dim3(32, kSlotShards), dim3(256), 0, st, P, T, rp);
        hipLaunchKernelGGL(k_slot_fixup, dim3(1), dim3(kSlotShards), 0, st, T, rp);
        rp ^= 1;
    }
    HIP_OK(hipEventRecord(D.ev1, st));
    HIP_OK(hipEventSynchronize(D.ev1));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, D.ev0, D.ev1));
    if (stats) {
        unsigned long long hs[kStatBytes / 8] = {0};
        HIP_OK(hipMemcpy(hs, D.stats.p, kStatBytes, hipMemcpyDeviceToHost));
        for (int k = 1; k <= kStatShards; k++) hs[2] += hs[16 * k], hs[3] += hs[16 * k + 1];  // ray_stats shards
        stats->seconds = ms * 1e-3;
        stats->device_seconds[0] = stats->seconds;
        stats->camera_samples = (uint64_t)(s1 - s0) * npx;
        stats->light_evals_survived = hs[1];
        stats->rays = hs[2];
        stats->light_rays = hs[3];
        stats->generations = gens;
        stats->shading_nodes = nodes_total;

        // k_prep_pk2 counts its full-prep nodes (hs[7]) and k_prep_pick the cached roots (hs[0]);
        // k_prep / k_prep_lane (huge / tiny light sets) run every node in full
        const uint64_t full = hs[7] ? hs[7] : (needs_prep ? nodes_total : 0);
        stats->prep_full_nodes = full;
        stats->prep_cached_nodes = hs[0] + cached_roots;
        stats->prep_cache_points = cache_points;
        stats->light_evals_total = full * (uint64_t)D.d.NL;
        stats->light_evals_culled_backface = count_c1 ? hs[6] : 0;
        stats->light_evals_candidates = hs[5];
        stats->light_evals_culled_plane = stats->light_evals_total - hs[5] - stats->light_evals_culled_backface;
        stats->spilled_nodes = spilled;
        stats->trace_seconds = trace_ms * 1e-3;
        stats->trace_launches = trace_launches;
        stats->node_visits = hs[8];
        stats->tri_tests = hs[9];
        stats->reduce_seconds = 0;
        stats->devices_used = 1;
        stats->prep_seconds = prep_ms * 1e-3;
        stats->prep_launches = prep_launches;
        stats->prep_exact_nodes = hs[10];
        stats->prep_band_nodes = hs[11];
#if MCPT_TRACE_DIAG
        if (hs[8])
            fprintf(stderr, "trace diag: %llu visits over %llu wave node-iterations (lane use %.3f), %llu tests over %llu wave "
                            "leaf-iterations (lane use %.3f)\n", hs[8], hs[14], hs[8] / (64.0 * std::max<unsigned long long>(hs[14], 1)),
                    hs[9], hs[15], hs[9] / (64.0 * std::max<unsigned long long>(hs[15], 1)));
#endif
#if MCPT_BAND_DIAG
        fprintf(stderr, "exact diag (10 ns ticks summed over nodes): lists %llu literal %llu lists+literal+sum %llu pick %llu\n",
                hs[12], hs[13], hs[14], hs[15]);
        if (exact_scr) {
            const int nlp = (D.d.NL + 63) & ~63;
            std::vector<int> pc(npx);
            HIP_OK(hipMemcpy(pc.data(), reinterpret_cast<int*>(exact_scr + (size_t)exact_waves(D.d.NL) * nlp * 3 / 2),
                             4ull * npx, hipMemcpyDeviceToHost));
            long long tot = 0, distinct = 0, mx = 0;
            for (int v : pc) tot += v, distinct += v > 0, mx = std::max<long long>(mx, v);
            fprintf(stderr, "exact diag: roots %lld over %lld pixels (max %lld per pixel)\n", tot, distinct, mx);
        }
#endif
        stats->cache_build_seconds = cache_ms * 1e-3;
    }
    return MCPT_OK;
}

int check_opts(const mcpt_render_opts* o) {
    if (o->struct_size != sizeof(mcpt_render_opts)) {
        set_error("mcpt_render_opts.struct_size is %u, this library expects %zu (use mcpt_render_opts_init / the "
                  "mcpt.h of MCPT_VERSION %d)", o->struct_size, sizeof(mcpt_render_opts), MCPT_VERSION);
        return MCPT_E_INVALID;
    }
    if (o->num_devices < 0 || (o->num_devices > 0 && !o->devices) || (o->num_devices > 0 && o->comm)) {
        set_error("invalid device list (num_devices %d, devices %p, comm %p)", o->num_devices, (const void*)o->devices,
                  (const void*)o->comm);
        return MCPT_E_INVALID;
    }
    if (o->num_devices > 0) {
        int nd = 0;
        HIP_OK(hipGetDeviceCount(&nd));
        for (int k = 0; k < o->num_devices; k++)
            if (o->devices[k] < 0 || o->devices[k] >= nd) {
                set_error("devices[%d] = %d: no such device (%d visible)", k, o->devices[k], nd);
                return MCPT_E_INVALID;
            }
    }
    return MCPT_OK;
}

// the caller's framebuffer must be device memory of `device` (fp64 hardware atomics are lost on
// host / managed memory, and a host pointer the runtime does not know would fault the GPU)
int check_device_buffer(const void* p, int device) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        set_error("dev_out_rgb is not coarse-grained device memory (unknown to the HIP runtime)");
        return MCPT_E_INVALID;
    }
    if (a.type != hipMemoryTypeDevice || a.isManaged) {
        set_error("dev_out_rgb is not coarse-grained device memory (memory type %d, managed %d)", (int)a.type, a.isManaged);
        return MCPT_E_INVALID;
    }
    if (a.device != device) {
        set_error("dev_out_rgb lives on device %d, the render's root device is %d", a.device, device);
        return MCPT_E_INVALID;
    }
    return MCPT_OK;
}

// [s0, s1) of the whole job (0,0 = [0, spp))
void job_range(const mcpt_render_opts* o, int* s0, int* s1) {
    const bool all = o->sample_begin == 0 && o->sample_end == 0;
    *s0 = all ? 0 : o->sample_begin;
    *s1 = all ? o->spp : o->sample_end;
}

// shard k of n of [s0, s1): contiguous and balanced (sizes differ by at most one sample)
void shard_range(int s0, int s1, int k, int n, int* a, int* b) {
    const long long len = (long long)s1 - s0;
    *a = s0 + (int)(len * k / n);
    *b = s0 + (int)(len * (k + 1) / n);
}

void add_stats(mcpt_stats& t, const mcpt_stats& x) {
    t.camera_samples += x.camera_samples;
    t.shading_nodes += x.shading_nodes;
    t.light_evals_survived += x.light_evals_survived;
    t.rays += x.rays;
    t.light_rays += x.light_rays;
    t.generations += x.generations;
    t.prep_seconds += x.prep_seconds;
    t.prep_launches += x.prep_launches;
    t.light_evals_total += x.light_evals_total;
    t.light_evals_culled_backface += x.light_evals_culled_backface;
    t.light_evals_culled_plane += x.light_evals_culled_plane;
    t.light_evals_candidates += x.light_evals_candidates;
    t.prep_full_nodes += x.prep_full_nodes;
    t.prep_cached_nodes += x.prep_cached_nodes;
    t.prep_cache_points += x.prep_cache_points;
    t.spilled_nodes += x.spilled_nodes;
    t.trace_seconds += x.trace_seconds;
    t.trace_launches += x.trace_launches;
    t.node_visits += x.node_visits;
    t.tri_tests += x.tri_tests;
    t.prep_exact_nodes += x.prep_exact_nodes;
    t.prep_band_nodes += x.prep_band_nodes;
    t.cache_build_seconds += x.cache_build_seconds;
}

// progress of a multi-device call: the shards' dispatched counts are summed and the caller's callback
// is invoked under a lock (it may be called from any device's worker thread); a cancel stops every
// shard at its next generation
struct MultiProgress {
    const mcpt_render_opts* o;
    uint64_t total = 0;
    std::mutex mu;
    std::vector<uint64_t> done;  // per shard
    std::atomic<bool> cancel{false};
};
struct ShardProgress {
    MultiProgress* m;
    int shard;
};
int multi_progress_cb(void* user, uint64_t dispatched, uint64_t) {
    ShardProgress* sp = static_cast<ShardProgress*>(user);
    MultiProgress* m = sp->m;
    if (m->cancel.load()) return 1;
    if (!m->o->progress) return 0;
    std::lock_guard<std::mutex> lk(m->mu);
    m->done[sp->shard] = dispatched;
    uint64_t sum = 0;
    for (uint64_t d : m->done) sum += d;
    if (m->o->progress(m->o->progress_user, sum, m->total)) m->cancel.store(true);
    return m->cancel.load() ? 1 : 0;
}

// One process, several devices (mcpt_render_opts.devices): shards of the sample range rendered
// concurrently -- one host thread and stream per distinct device, shards on a repeated device run in
// order into that device's buffer -- then ONE ncclReduce(sum) into the root devices[0].
// root_out: the root's framebuffer (device memory on devices[0]); host_out (mcpt_render): when
// non-null, root_out is the library's buffer, loaded from and stored back to host_out.
// MCPT_DEBUG_SHARD_RANKS (include/mcpt_debug.h): every list entry is its own rank of the communicator,
// repeated devices included -- with a collective library that accepts a device twice (tests/collshim)
// this runs the multi-rank group reduce on a one-GPU box.  Ranks on the same device render one after
// another (they share its DeviceState) into framebuffers of their own.
int render_multi(mcpt_scene* sc, const mcpt_camera* cam, const mcpt_render_opts* o, double* root_out,
                 double* host_out, mcpt_stats* stats) {
    const int nshards = o->num_devices;
    const bool per_shard = (o->flags & MCPT_DEBUG_SHARD_RANKS) != 0;
    std::vector<int> uniq;  // the communicator's ranks: distinct devices in order of first appearance; uniq[0] = root
    std::vector<int> shard_dev(nshards);
    for (int k = 0; k < nshards; k++) {
        const int d = o->devices[k];
        auto it = per_shard ? uniq.end() : std::find(uniq.begin(), uniq.end(), d);
        shard_dev[k] = (int)(it - uniq.begin());
        if (it == uniq.end()) uniq.push_back(d);
    }
    const int nu = (int)uniq.size();
    std::vector<int> lock_of(nu);  // ranks on one device share its state: one lock per device
    for (int u = 0; u < nu; u++) lock_of[u] = (int)(std::find(uniq.begin(), uniq.end(), uniq[u]) - uniq.begin());
    std::vector<std::mutex> dev_mu(nu);
    struct OwnBufs {  // per-rank framebuffers of repeated devices (MCPT_DEBUG_SHARD_RANKS), freed on return
        std::vector<void*> p;
        ~OwnBufs() {
            for (void* q : p)
                if (q) (void)hipFree(q);
        }
    } own;
    own.p.assign(nu, nullptr);
    const size_t nfb = 3ull * cam->width * cam->height;
    int rc;
    if ((rc = validate_render(o))) return rc;
    // the reference grid (MCPT_ACCEL_GRID) is built here, before the workers, which then only read it
    if (o->accel == MCPT_ACCEL_GRID) {
        const CamFrame cf = cam_setup(*cam);
        const double eye[3] = {cf.eye.x, cf.eye.y, cf.eye.z};
        if ((rc = ensure_host_grid(sc, eye, 100000))) return rc;
    }
    std::vector<DeviceState*> Ds(nu, nullptr);
    std::vector<double*> fbs(nu, nullptr);
    int s0, s1;
    job_range(o, &s0, &s1);
    MultiProgress mp;
    mp.o = o;
    mp.total = (uint64_t)(s1 - s0) * cam->width * cam->height;
    mp.done.assign(nshards, 0);
    std::vector<ShardProgress> sp(nshards);
    std::vector<mcpt_stats> sst(nshards);
    std::vector<int> urc(nu, MCPT_OK);
    std::vector<std::string> uerr(nu);
    std::vector<double> setup_s(nu, 0.0), render_s(nu, 0.0);
    // the RCCL communicators over exactly these devices (cached per scene handle), created on this thread
    // BEFORE any worker touches a device: ncclCommInitAll allocates and launches on every device of the
    // clique, and never runs concurrently with the workers' scene uploads and queue allocations
    double comm_init_s = 0.0;
    if (sc->comm_devices != uniq) {
        const auto c0 = std::chrono::steady_clock::now();
        comm_all_destroy(sc->comms);
        sc->comm_devices.clear();
        if ((rc = comm_all_init(uniq, sc->comms))) return rc;  // nothing rendered yet: a clean failure
        sc->comm_devices = uniq;
        comm_init_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
    }
    const auto t0 = std::chrono::steady_clock::now();
    // one worker thread per distinct device: its scene state (the uploads of a 1M-triangle scene run
    // on all devices at once, not one after another), its framebuffer, then its shards in order
    auto worker = [&](int u) {
        auto fail = [&](int r) {
            urc[u] = r;
            uerr[u] = mcpt_last_error();
            mp.cancel.store(true);
        };
        int r;
        std::lock_guard<std::mutex> dev_lock(dev_mu[lock_of[u]]);
        const auto w0 = std::chrono::steady_clock::now();
        if ((r = get_device_state(sc, uniq[u], &Ds[u]))) return fail(r);
        DeviceState& D = *Ds[u];
        if (hipDeviceSynchronize() != hipSuccess) {  // the caller's buffers may still be written by other streams
            set_error("hipDeviceSynchronize failed");
            return fail(MCPT_E_DEVICE);
        }
        if (u == 0 && !host_out) {
            fbs[0] = root_out;
        } else {
            if (lock_of[u] != u) {  // a repeated device: a buffer of this rank's own
                if (hipMalloc(&own.p[u], nfb * sizeof(double)) != hipSuccess) {
                    own.p[u] = nullptr;
                    set_error("framebuffer of rank %d on device %d: out of memory", u, uniq[u]);
                    return fail(MCPT_E_DEVICE);
                }
                fbs[u] = (double*)own.p[u];
            } else {
                if ((r = ensure(D.fb, nfb * sizeof(double)))) return fail(r);
                fbs[u] = (double*)D.fb.p;
            }
            const hipError_t e = u == 0 ? hipMemcpyAsync(fbs[0], host_out, nfb * sizeof(double), hipMemcpyHostToDevice, D.stream)
                                        : hipMemsetAsync(fbs[u], 0, nfb * sizeof(double), D.stream);
            if (e != hipSuccess || hipStreamSynchronize(D.stream) != hipSuccess) {
                set_error("framebuffer setup on device %d failed", uniq[u]);
                return fail(MCPT_E_DEVICE);
            }
        }
        const auto w1 = std::chrono::steady_clock::now();
        setup_s[u] = std::chrono::duration<double>(w1 - w0).count();
        struct RenderClock {  // the rank's shard time, recorded on every way out of the loop
            double& out;
            std::chrono::steady_clock::time_point a;
            ~RenderClock() { out = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count(); }
        } rclock{render_s[u], w1};
        for (int k = 0; k < nshards; k++) {
            if (shard_dev[k] != u) continue;
            int a, b;
            shard_range(s0, s1, k, nshards, &a, &b);
            if (a == b) continue;  // more shards than samples
            mcpt_render_opts ok = *o;
            ok.sample_begin = a;
            ok.sample_end = b;
            ok.num_devices = 0;
            ok.devices = nullptr;
            ok.device = uniq[u];
            sp[k] = ShardProgress{&mp, k};
            ok.progress = multi_progress_cb;
            ok.progress_user = &sp[k];
            if ((r = render_on_device(sc, D, cam, &ok, fbs[u], &sst[k]))) return fail(r);
        }
    };
    std::vector<std::thread> th;
    for (int u = 0; u < nu; u++) th.emplace_back(worker, u);
    for (auto& t : th) t.join();
    // report the first real failure: a shard stopped by another's failure reports MCPT_E_CANCELLED,
    // which is the answer only when the user's progress callback asked for it
    int fu = -1;
    for (int u = 0; u < nu; u++)
        if (urc[u] && (fu < 0 || (urc[fu] == MCPT_E_CANCELLED && urc[u] != MCPT_E_CANCELLED))) fu = u;
    if (fu >= 0) {
        set_error("device %d: %s", uniq[fu], uerr[fu].c_str());
        return urc[fu];
    }
    const auto t1 = std::chrono::steady_clock::now();
    std::vector<hipStream_t> streams(nu);
    for (int u = 0; u < nu; u++) streams[u] = Ds[u]->stream;
    if ((rc = comm_all_reduce_sum(sc->comms, uniq, fbs, streams, nfb))) return rc;
    for (int u = 0; u < nu; u++) {
        HIP_OK(hipSetDevice(uniq[u]));
        HIP_OK(hipStreamSynchronize(Ds[u]->stream));
    }
    const auto t2 = std::chrono::steady_clock::now();
    HIP_OK(hipSetDevice(uniq[0]));
    if (host_out) {
        HIP_OK(hipMemcpyAsync(host_out, fbs[0], nfb * sizeof(double), hipMemcpyDeviceToHost, Ds[0]->stream));
        HIP_OK(hipStreamSynchronize(Ds[0]->stream));
    }
    if (stats) {
        mcpt_stats t{};
        for (int k = 0; k < nshards; k++) add_stats(t, sst[k]);
        t.seconds = std::chrono::duration<double>(t2 - t0).count();
        t.reduce_seconds = std::chrono::duration<double>(t2 - t1).count();
        t.devices_used = nu;
        t.comm_init_seconds = comm_init_s;
        for (int u = 0; u < nu; u++) {
            t.device_setup_seconds = std::max(t.device_setup_seconds, setup_s[u]);
            if (u < MCPT_STATS_MAX_DEVICES) t.device_seconds[u] = render_s[u];
        }
        *stats = t;
    }
    return MCPT_OK;
}

// adds src into dst (n doubles): rank 0's share of the reduced job onto the caller's buffer
__global__ void k_add_fb(double* __restrict__ dst, const double* __restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] += src[i];
}

// One process per device (mcpt_render_opts.comm): this rank's shard of the job's sample range, then ONE
// ncclReduce(sum) to rank 0.  Every rank renders into a zeroed library buffer of W*H*3 + 1 doubles whose
// last slot carries the rank's status (0 ok, 1 failed), so the one reduce also tells rank 0 whether any
// rank failed; rank 0 then adds the reduced frame to its `out` (or leaves it unchanged and fails).
// Failures never skip the collective: options are validated identically on every rank before it
// (validate_render), and every later failure on this rank -- the buffer setup, the render (out of
// memory, spill cap, a cancel from its own progress callback: cancelling is per rank), zeroing the
// partial frame -- is recorded and the rank still joins the reduce with the failure flag, then returns
// its error.  The flag is written by a kernel after the zeroing; if even that cannot be enqueued (a
// sticky device error) the rank still enqueues the reduce, and its peers see whatever its buffer holds:
// the one failure mode that can reach rank 0 unflagged is a device that can no longer run kernels, and
// then its ncclReduce fails to enqueue too.  In that case (the reduce itself cannot be enqueued) the
// communicator is aborted and the peers block in their reduce: RCCL has no way to release them from
// one rank.  Other ranks' buffers (`out`) are left unchanged.
__global__ void k_rank_status(double* fb, size_t nfb, double status) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nfb; i += (size_t)gridDim.x * blockDim.x) fb[i] = 0.0;
    if (blockIdx.x == 0 && threadIdx.x == 0) fb[nfb] = status;
}
int render_rank(mcpt_scene* sc, DeviceState& D, const mcpt_camera* cam, const mcpt_render_opts* o, double* out,
                mcpt_stats* stats) {
    int nranks, rank, device;
    int rc;
    if ((rc = comm_rank_info(o->comm, &nranks, &rank, &device))) return rc;
    if ((rc = validate_render(o))) return rc;  // same outcome on every rank: nobody enters the reduce
    const size_t nfb = 3ull * cam->width * cam->height;
    int local = MCPT_OK;
    std::string lerr;
    auto fail = [&](int r, const char* what) {
        if (local) return;
        local = r;
        lerr = what ? what : mcpt_last_error();
        (void)hipGetLastError();
    };
    double* fb = nullptr;
    if ((rc = ensure(D.rank_fb, (nfb + 1) * sizeof(double)))) {
        // no buffer of our own: the caller's is the only device memory at hand.  Rank 0 cannot lend it
        // (it is the result); another rank's `out` is left unchanged by contract, so a rank without a
        // buffer cannot join -- abort instead (below)
        fail(rc, nullptr);
    } else {
        fb = (double*)D.rank_fb.p;
        if (hipMemsetAsync(fb, 0, (nfb + 1) * sizeof(double), D.stream) != hipSuccess) fail(MCPT_E_DEVICE, "hipMemsetAsync of the rank buffer failed");
    }
    int s0, s1, a, b;
    job_range(o, &s0, &s1);
    shard_range(s0, s1, rank, nranks, &a, &b);
    mcpt_stats st{};
    if (!local && a < b) {
        mcpt_render_opts ok = *o;
        ok.sample_begin = a;
        ok.sample_end = b;
        ok.comm = nullptr;
        ok.device = device;
        const int r = render_on_device(sc, D, cam, &ok, fb, &st);
        if (r) fail(r, nullptr);
    }
    if (local && fb) {  // join the reduce anyway, with a zero frame and the failure flag
        hipLaunchKernelGGL(k_rank_status, dim3(1024), dim3(256), 0, D.stream, fb, nfb, 1.0);
        (void)hipGetLastError();
    }
    int rrc = fb ? MCPT_OK : MCPT_E_DEVICE;
    if (fb) {
        (void)hipEventRecord(D.ev0, D.stream);
        rrc = comm_rank_reduce_sum(o->comm, fb, nfb + 1, D.stream);
        (void)hipEventRecord(D.ev1, D.stream);
    }
    if (rrc) {  // this rank cannot take part in the collective: release what RCCL holds for it
        const std::string why = mcpt_last_error();
        comm_rank_abort(o->comm);
        set_error("rank %d could not join the frame reduce (%s)%s%s; the communicator is aborted", rank, why.c_str(),
                  local ? " after: " : "", local ? lerr.c_str() : "");
        return local ? local : rrc;
    }
    double failed = 0;
    if (rank == 0 && !local) HIP_OK(hipMemcpyAsync(&failed, fb + nfb, sizeof(double), hipMemcpyDeviceToHost, D.stream));
    const hipError_t se = hipStreamSynchronize(D.stream);
    if (local) {
        set_error("rank %d: %s", rank, lerr.c_str());
        return local;
    }
    if (se != hipSuccess) {
        set_error("rank %d: the frame reduce failed on the device (%s)", rank, hipGetErrorString(se));
        return MCPT_E_DEVICE;
    }
    if (failed > 0) {
        set_error("%d of %d ranks failed their shard; the frame is not added", (int)failed, nranks);
        return MCPT_E_DEVICE;
    }
    if (rank == 0) {
        hipLaunchKernelGGL(k_add_fb, dim3(1024), dim3(256), 0, D.stream, out, (const double*)fb, nfb);
        HIP_OK(hipGetLastError());
        HIP_OK(hipStreamSynchronize(D.stream));
    }
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, D.ev0, D.ev1));
    if (stats) {
        *stats = st;
        stats->seconds += ms * 1e-3;
        stats->reduce_seconds = ms * 1e-3;
        stats->devices_used = 1;
    }
    return MCPT_OK;
}

// mcpt_light_prep (all_exact = false: the renderer's prep kernels, the band's nodes redone by
// k_prep_exact, which also takes the nodes whose survivor count may differ) and
// mcpt_debug_light_prep_exact (all_exact: every node through k_prep_exact alone)
int light_prep_query(mcpt_scene* sc, int32_t n, const double* x1, const double* nrm, const double* u, double* wsum,
                     int32_t* count, int32_t* pick, bool all_exact) {
    if (!sc || n < 0 || (n && (!x1 || !nrm || !u || !wsum || !count || !pick))) {
        set_error("invalid argument");
        return MCPT_E_INVALID;
    }
    if (n == 0) return MCPT_OK;
    std::lock_guard<std::mutex> lk(sc->mu);
    DeviceState* D;
    int rc;
    if ((rc = get_device_state(sc, -1, &D))) return rc;
    const bool exact = D->d.NL > kSmallNL;  // k_prep_lane is exact by construction
    if (all_exact && !exact) {
        set_error("the exact prep applies to scenes with more than %d light triangles", kSmallNL);
        return MCPT_E_INVALID;
    }
    void *dp, *dn, *du, *dw, *dc, *dk, *dm, *dl = nullptr, *ds = nullptr, *dsl = nullptr;
    HIP_OK(hipMalloc(&dm, 8ull * n * mask_stride(prep_chunks(D->d.NL))));  // candidate words of the split prep (variant 17)
    HIP_OK(hipMalloc(&dp, 24ull * n));
    HIP_OK(hipMalloc(&dn, 24ull * n));
    HIP_OK(hipMalloc(&du, 8ull * n));
    HIP_OK(hipMalloc(&dw, 8ull * n));
    HIP_OK(hipMalloc(&dc, 4ull * n));
    HIP_OK(hipMalloc(&dk, 4ull * n));
    if (exact) {
        HIP_OK(hipMalloc(&dl, 8ull * (n + kExactHead)));  // exact list, then the band's candidate list
        HIP_OK(hipMalloc(&ds, 8 * exact_scratch_doubles(D->d.NL)));
        HIP_OK(hipMalloc(&dsl, 8ull * n));
        HIP_OK(hipMemset(dl, 0, 4));
        HIP_OK(hipMemset((int*)dl + n + kExactHead, 0, 4));
    }
    {  // node coordinates in the kernels' 3-vector layout (idx3, like the wavefront queue)
        const std::vector<double> px = soa3(x1, n), pn = soa3(nrm, n);
        HIP_OK(hipMemcpy(dp, px.data(), 24ull * n, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(dn, pn.data(), 24ull * n, hipMemcpyHostToDevice));
    }
    HIP_OK(hipMemcpy(du, u, 8ull * n, hipMemcpyHostToDevice));
    if ((rc = ensure(D->work, 256))) return rc;
    CullOrder co{};
    if ((rc = cull_order_bufs(*D, (size_t)n, &co))) return rc;
    if (all_exact) {
        std::vector<int> all(n + kExactHead, 0);
        all[0] = n;
        for (int k = 0; k < n; k++) all[kExactHead + k] = k;
        HIP_OK(hipMemcpy(dl, all.data(), 4ull * all.size(), hipMemcpyHostToDevice));
    } else {
        PrepCache cx{};
        cx.slack = (double*)dsl;
        cx.exact_counts = 1;
        cx.maybe = exact ? (int*)dl + n + kExactHead : nullptr;
        HIP_OK(launch_prep(-1, D->d, 0, n, (const double*)dp, (const double*)dn, n, nullptr, nullptr, nullptr,
                           (const double*)du, (double*)dw, (int*)dk, (int*)dc, nullptr, (unsigned*)D->work.p, D->stream,
                           cx, (uint64_t*)dm, true, false, co));
        if (exact)
            hipLaunchKernelGGL(k_prep_band, dim3(kBandBlocks), dim3(256), 0, D->stream, D->d, (const int*)cx.maybe,
                               (const double*)dsl, (const double*)dp, n, (const uint64_t*)dm,
                               prep_writes_masks(D->d, (const uint64_t*)dm) ? n : 0, prep_chunks(D->d.NL), (int*)dl, nullptr);
    }
    if (exact)
        hipLaunchKernelGGL(k_prep_exact, dim3(exact_blocks(D->d.NL)), dim3(kExactBlock), 0, D->stream, D->d, (uint64_t)0,
                           (const int*)dl, (const double*)dp, (const double*)dn, n, nullptr, nullptr, nullptr,
                           (const double*)du, (double*)dw, (int*)dk, (int*)dc, nullptr, (double*)ds,
                           all_exact ? nullptr : (const uint64_t*)dm, prep_writes_masks(D->d, (const uint64_t*)dm) ? n : 0,
                           prep_chunks(D->d.NL), nullptr, nullptr, 0, INT_MAX, RootLit{}, nullptr);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(D->stream));
    HIP_OK(hipMemcpy(wsum, dw, 8ull * n, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(count, dc, 4ull * n, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(pick, dk, 4ull * n, hipMemcpyDeviceToHost));
    for (int k = 0; k < n; k++) pick[k] = pick[k] >= 0 ? sc->host.light_facet[pick[k]] : -1;
    void* bufs[] = {dp, dn, du, dw, dc, dk, dm, dl, ds, dsl};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    return MCPT_OK;
}

}  // namespace

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" {

int mcpt_version(void) { return MCPT_VERSION; }

static int finish_scene(HostScene&& hs, mcpt_scene** out) {
    auto* sc = new mcpt_scene();
    sc->host = std::move(hs);
    std::vector<int32_t> all(sc->host.F), lights(sc->host.light_facet);
    for (int f = 0; f < sc->host.F; f++) all[f] = f;
    // SAH leaves of at most 2 triangles unless the SAH prefers a bigger one (up to 8): each leaf
    // triangle costs a fp64 Cramer test, a box only fp32 slabs (same-box A/B of the leaf bound:
    // 1 -> Veach MIS -1% / Cornell-1M +20%, 2 -> +1.5% / +16%, 3 -> +1% / +7%, 8 -> -5% / -24%,
    // each against 4)
#ifndef MCPT_BVH_MAX_LEAF
#define MCPT_BVH_MAX_LEAF 2
#endif
    constexpr int kMaxLeaf = MCPT_BVH_MAX_LEAF;
    sc->bvh = build_bvh(sc->host, all, kMaxLeaf);
    sc->lbvh = build_bvh(sc->host, lights, kMaxLeaf);
    *out = sc;
    return MCPT_OK;
}

int mcpt_scene_load(const char* obj_path, const char* xml_path, mcpt_scene** out) {
    if (!obj_path || !xml_path || !out) {
        set_error("null argument");
        return MCPT_E_INVALID;
    }
    HostScene hs;
    std::vector<LightDef> lights;
    std::string err;
    if (!load_obj_mtl(obj_path, hs, err) || !load_light_xml(xml_path, hs, lights, err)) {
        set_error("%s", err.c_str());
        return MCPT_E_IO;
    }
    if (!finalize_scene(hs, lights, err)) {
        set_error("%s", err.c_str());
        return MCPT_E_SCENE;
    }
    return finish_scene(std::move(hs), out);
}

int mcpt_scene_create(const mcpt_scene_desc* d, mcpt_scene** out) {
    if (!d || !out || d->nfacets < 0 || d->nmaterials < 0 || d->nlights < 0 || !d->positions || !d->normals ||
        !d->material_id || !d->materials || (d->nlights && (!d->light_facet || !d->light_radiance))) {
        set_error("invalid scene descriptor");
        return MCPT_E_INVALID;
    }
    HostScene hs;
    hs.F = d->nfacets;
    hs.M = d->nmaterials;
    hs.pos.assign(d->positions, d->positions + 9 * (size_t)hs.F);
    hs.nrm.assign(d->normals, d->normals + 9 * (size_t)hs.F);
    hs.mat.assign(d->material_id, d->material_id + hs.F);
    hs.mtl.assign(d->materials, d->materials + 7 * (size_t)hs.M);
    for (int m = 0; m < hs.M; m++) hs.mtl_names.push_back("m" + std::to_string(m));
    // lights are given directly: synthesise one light "material" per light triangle in order
    std::vector<LightDef> none;
    std::string err;
    if (!finalize_scene(hs, none, err)) {
        set_error("%s", err.c_str());
        return MCPT_E_SCENE;
    }
    hs.NL = d->nlights;
    hs.light_facet.assign(d->light_facet, d->light_facet + hs.NL);
    hs.light_rad.assign(d->light_radiance, d->light_radiance + 3 * (size_t)hs.NL);
    hs.light_sum.resize(hs.NL);
    hs.light_of.assign(hs.F, -1);
    for (int l = 0; l < hs.NL; l++) {
        if (hs.light_facet[l] < 0 || hs.light_facet[l] >= hs.F) {
            set_error("light %d: facet out of range", l);
            return MCPT_E_INVALID;
        }
        hs.light_sum[l] = hs.light_rad[3 * l] + hs.light_rad[3 * l + 1] + hs.light_rad[3 * l + 2];
        hs.light_of[hs.light_facet[l]] = l;
        hs.light_area.push_back(light_triangle_area(hs, hs.light_facet[l]));
        // lights (select_a_point_from_lights): desc->light_group, or runs of equal radiance
        const bool same = l > 0 && (d->light_group ? d->light_group[l] == d->light_group[l - 1]
                                                   : std::equal(&hs.light_rad[3 * l], &hs.light_rad[3 * l + 3],
                                                                &hs.light_rad[3 * (l - 1)]));
        if (!same) {
            if (d->light_group && l > 0 && d->light_group[l] < d->light_group[l - 1]) {
                set_error("light_group must be ascending");
                return MCPT_E_INVALID;
            }
            hs.group_rsum.push_back(hs.light_sum[l]);
            hs.group_start.push_back(l);
            hs.group_count.push_back(0);
        }
        hs.group_count.back()++;
    }
    return finish_scene(std::move(hs), out);
}

void mcpt_scene_destroy(mcpt_scene* sc) {
    if (!sc) return;
    comm_all_destroy(sc->comms);
    for (auto& D : sc->devs) {
        (void)hipSetDevice(D->device);
        for (void* p : D->allocs) (void)hipFree(p);
        std::vector<DevBuf*> bufs = {&D->hit_f, &D->hit_tbg, &D->fb, &D->rank_fb, &D->stats, &D->work, &D->cache_bt, &D->cache_lst,
                                     &D->cache_info, &D->cache_w, &D->masks, &D->g_start, &D->g_tri, &D->root_pnw,
                                     &D->root_kind, &D->exact, &D->exact_scr, &D->slack, &D->lit_slot, &D->lit_pool,
                                     &D->sc_cum, &D->sc_wsum, &D->sc_last, &D->cull_keys, &D->cull_order, &D->cull_count};
        for (int k = 0; k < 14; k++) bufs.insert(bufs.end(), {&D->qa[k], &D->qb[k], &D->qs[k]});
        for (int k = 0; k < 9; k++) bufs.push_back(&D->aux[k]);
        for (int k = 0; k < 13; k++) bufs.push_back(&D->sl[k]);
        for (DevBuf* b : bufs)
            if (b->p) (void)hipFree(b->p);
        if (D->pinned_count) (void)hipHostFree(D->pinned_count);
        if (D->stream) (void)hipStreamDestroy(D->stream);
        hipEvent_t evs[] = {D->ev0, D->ev1, D->evp0, D->evp1, D->evr0, D->evr1};
        for (hipEvent_t e : evs)
            if (e) (void)hipEventDestroy(e);
    }
    delete sc;
}

int mcpt_scene_accel_bytes(const mcpt_scene* sc, uint64_t* bytes) {
    if (!sc || !bytes) return MCPT_E_INVALID;
    // 4-wide nodes (128 B) of both BVHs plus their leaf triangles (3 float4 = 48 B)
    auto nodes4 = [](const Bvh& b) { return (uint64_t)collapse_bvh4(b).size(); };
    *bytes = (nodes4(sc->bvh) + nodes4(sc->lbvh)) * sizeof(BvhNode4) +
             (uint64_t)(sc->bvh.leaf_facets.size() + sc->lbvh.leaf_facets.size()) * 3 * sizeof(float4);
    return MCPT_OK;
}

int mcpt_scene_counts(const mcpt_scene* sc, int32_t* nf, int32_t* nm, int32_t* nl) {
    if (!sc) return MCPT_E_INVALID;
    if (nf) *nf = sc->host.F;
    if (nm) *nm = sc->host.M;
    if (nl) *nl = sc->host.NL;
    return MCPT_OK;
}

int mcpt_scene_arrays(const mcpt_scene* sc, float* pos, float* nrm, int32_t* mat, float* mtl, int32_t* lf,
                      double* lrad, double* un) {
    if (!sc) return MCPT_E_INVALID;
    const HostScene& h = sc->host;
    if (pos) std::copy(h.pos.begin(), h.pos.end(), pos);
    if (nrm) std::copy(h.nrm.begin(), h.nrm.end(), nrm);
    if (mat) std::copy(h.mat.begin(), h.mat.end(), mat);
    if (mtl) std::copy(h.mtl.begin(), h.mtl.end(), mtl);
    if (lf) std::copy(h.light_facet.begin(), h.light_facet.end(), lf);
    if (lrad) std::copy(h.light_rad.begin(), h.light_rad.end(), lrad);
    if (un) std::copy(h.unique_n.begin(), h.unique_n.end(), un);
    return MCPT_OK;
}

int mcpt_scene_camera(const mcpt_scene* sc, mcpt_camera* cam) {
    if (!sc || !cam) return MCPT_E_INVALID;
    if (!sc->host.has_cam) {
        set_error("scene XML has no <camera>");
        return MCPT_E_SCENE;
    }
    *cam = sc->host.cam;
    return MCPT_OK;
}

void mcpt_render_opts_init(mcpt_render_opts* o) {
    if (!o) return;
    std::memset((void*)o, 0, sizeof *o);
    o->struct_size = sizeof *o;
    o->stats_size = sizeof(mcpt_stats);
    o->spp = 10;  // main.cpp:567
    o->mode = MCPT_MODE_MIS;
    o->seed = 20240430;
    o->device = -1;
}

// the caller's stats: at most opts->stats_size bytes of the library's (a caller built against an older mcpt.h
// passes a smaller struct; its prefix is the same fields)
static void copy_stats(const mcpt_render_opts* o, const mcpt_stats& st, mcpt_stats* out) {
    if (out) std::memcpy((void*)out, &st, std::min<size_t>(o->stats_size, sizeof st));
}
static int render_device_impl(mcpt_scene* sc, const mcpt_camera* cam, const mcpt_render_opts* o, double* dev_out,
                              mcpt_stats* stats);
static int render_impl(mcpt_scene* sc, const mcpt_camera* cam, const mcpt_render_opts* o, double* out_rgb,
                       mcpt_stats* stats);
int mcpt_render_device(mcpt_scene* sc, const mcpt_camera* cam, const mcpt_render_opts* o, double* dev_out,
                       mcpt_stats* stats) {
    mcpt_stats st{};
    const int rc = render_device_impl(sc, cam, o, dev_out, &st);
    if (rc == MCPT_OK) copy_stats(o, st, stats);
    return rc;
}
int mcpt_render(mcpt_scene* sc, const mcpt_camera* cam, const mcpt_render_opts* o, double* out_rgb, mcpt_stats* stats) {
    mcpt_stats st{};
    const int rc = render_impl(sc, cam, o, out_rgb, &st);
    if (rc == MCPT_OK) copy_stats(o, st, stats);
    return rc;
}
static int render_device_impl(mcpt_scene* sc, const mcpt_camera* cam, const mcpt_render_opts* o, double* dev_out,
                              mcpt_stats* stats) {
    if (!sc || !o || !dev_out) {
        set_error("null argument");
        return MCPT_E_INVALID;
    }
    int rc;
    if ((rc = check_opts(o)) || (rc = validate_camera(cam))) return rc;
    std::lock_guard<std::mutex> lk(sc->mu);
    if (o->num_devices > 0) {
        if ((rc = check_device_buffer(dev_out, o->devices[0]))) return rc;
        return render_multi(sc, cam, o, dev_out, nullptr, stats);
    }
    int device = o->device;
    if (o->comm) {
        int nr, r;
        if ((rc = comm_rank_info(o->comm, &nr, &r, &device))) return rc;
    }
    DeviceState* D;
    if ((rc = get_device_state(sc, device, &D))) return rc;
    if ((rc = check_device_buffer(dev_out, D->device))) return rc;
    // the caller's buffer may still be written by work on other streams (e.g. torch's)
    HIP_OK(hipDeviceSynchronize());
    if (o->comm) return render_rank(sc, *D, cam, o, dev_out, stats);
    return render_on_device(sc, *D, cam, o, dev_out, stats);
}

static int render_impl(mcpt_scene* sc, const mcpt_camera* cam, const mcpt_render_opts* o, double* out_rgb,
                       mcpt_stats* stats) {
    if (!sc || !o || !out_rgb) {
        set_error("null argument");
        return MCPT_E_INVALID;
    }
    int rc;
    if ((rc = check_opts(o)) || (rc = validate_camera(cam))) return rc;
    std::lock_guard<std::mutex> lk(sc->mu);
    if (o->num_devices > 0) return render_multi(sc, cam, o, nullptr, out_rgb, stats);
    int device = o->device;
    if (o->comm) {
        int nr, r;
        if ((rc = comm_rank_info(o->comm, &nr, &r, &device))) return rc;
    }
    DeviceState* D;
    if ((rc = get_device_state(sc, device, &D))) return rc;
    const size_t n = 3ull * cam->width * cam->height;
    if ((rc = ensure(D->fb, n * sizeof(double)))) return rc;
    HIP_OK(hipMemcpyAsync(D->fb.p, out_rgb, n * sizeof(double), hipMemcpyHostToDevice, D->stream));
    if (o->comm)
        rc = render_rank(sc, *D, cam, o, (double*)D->fb.p, stats);
    else
        rc = render_on_device(sc, *D, cam, o, (double*)D->fb.p, stats);
    if (rc) return rc;
    int nr = 1, rank = 0, dv;
    if (o->comm && (rc = comm_rank_info(o->comm, &nr, &rank, &dv))) return rc;
    if (rank != 0) return MCPT_OK;  // the job total lands on rank 0; this rank's out_rgb is unchanged
    HIP_OK(hipMemcpyAsync(out_rgb, D->fb.p, n * sizeof(double), hipMemcpyDeviceToHost, D->stream));
    HIP_OK(hipStreamSynchronize(D->stream));
    return MCPT_OK;
}

int mcpt_scene_meshing(mcpt_scene* sc, const double eye[3], int32_t n0) {
    if (!sc || !eye || n0 <= 0 || !std::isfinite(eye[0]) || !std::isfinite(eye[1]) || !std::isfinite(eye[2])) {
        set_error("invalid argument");
        return MCPT_E_INVALID;
    }
    std::lock_guard<std::mutex> lk(sc->mu);
    sc->grid = build_grid(sc->host, eye, n0);
    sc->grid_version++;
    if (!sc->grid.ok) {
        set_error("the scene's bounding box has zero or non-finite extent: no uniform grid (Myobj.cpp:110-162)");
        return MCPT_E_SCENE;
    }
    return MCPT_OK;
}

int mcpt_scene_grid_info(const mcpt_scene* sc, double* box_and_cell, int32_t* cells) {
    if (!sc || !sc->grid.ok) {
        set_error(sc ? "no grid (call mcpt_scene_meshing first)" : "null scene");
        return MCPT_E_INVALID;
    }
    const Grid& g = sc->grid;
    if (box_and_cell) {
        for (int i = 0; i < 3; i++) {
            box_and_cell[2 * i] = g.mn[i];
            box_and_cell[2 * i + 1] = g.mx[i];
        }
        box_and_cell[6] = g.d;
    }
    if (cells)
        for (int i = 0; i < 3; i++) cells[i] = g.gd[i];
    return MCPT_OK;
}

int mcpt_closest_hit(mcpt_scene* sc, int32_t n, const double* ro, const double* rd, const int32_t* ex,
                     int32_t flags, int32_t* facet, double* tbg) {
    if (!sc || n < 0 || (n && (!ro || !rd || !ex || !facet || !tbg)) ||
        (flags & ~(MCPT_HIT_LIGHT_ONLY | MCPT_HIT_GRID | MCPT_DEBUG_HIT_CW8)) ||
        ((flags & MCPT_HIT_GRID) && (flags & MCPT_DEBUG_HIT_CW8))) {
        set_error("invalid argument");
        return MCPT_E_INVALID;
    }
    if (n == 0) return MCPT_OK;
    std::lock_guard<std::mutex> lk(sc->mu);
    DeviceState* D;
    int rc;
    if ((rc = get_device_state(sc, -1, &D))) return rc;
    const bool grid = (flags & MCPT_HIT_GRID) != 0;
    if (grid) {
        if (!sc->grid.ok) {
            set_error("MCPT_HIT_GRID: no grid (call mcpt_scene_meshing first)");
            return MCPT_E_INVALID;
        }
        if ((rc = use_grid(sc, *D, sc->grid.eye, sc->grid.n0))) return rc;
    }
    const int light_only = (flags & MCPT_HIT_LIGHT_ONLY) != 0;
    void *dro, *drd, *dex, *df, *dt;
    HIP_OK(hipMalloc(&dro, 24ull * n));
    HIP_OK(hipMalloc(&drd, 24ull * n));
    HIP_OK(hipMalloc(&dex, 4ull * n));
    HIP_OK(hipMalloc(&df, 4ull * n));
    HIP_OK(hipMalloc(&dt, 24ull * n));
    HIP_OK(hipMemcpy(dro, ro, 24ull * n, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(drd, rd, 24ull * n, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(dex, ex, 4ull * n, hipMemcpyHostToDevice));
    if (flags & MCPT_DEBUG_HIT_CW8) {
        if ((rc = ensure_bvh8(sc, D))) return rc;
        if (!D->d.bvh8 || !D->d.lbvh8) {
            set_error("MCPT_DEBUG_HIT_CW8: no 8-wide tree for this scene");
            return MCPT_E_INVALID;
        }
        hipLaunchKernelGGL(k_trace_batch_cw8, dim3((n + kTraceBlock - 1) / kTraceBlock), dim3(kTraceBlock), 0, D->stream, D->d, n,
                           (const double*)dro, (const double*)drd, (const int*)dex, light_only, (int*)df, (double*)dt);
    } else {
        hipLaunchKernelGGL(grid ? k_trace_batch<true> : k_trace_batch<false>, dim3((n + kTraceBlock - 1) / kTraceBlock), dim3(kTraceBlock), 0,
                           D->stream, D->d, n, (const double*)dro, (const double*)drd, (const int*)dex, light_only, (int*)df, (double*)dt);
    }
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(D->stream));
    HIP_OK(hipMemcpy(facet, df, 4ull * n, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(tbg, dt, 24ull * n, hipMemcpyDeviceToHost));
    (void)hipFree(dro);
    (void)hipFree(drd);
    (void)hipFree(dex);
    (void)hipFree(df);
    (void)hipFree(dt);
    return MCPT_OK;
}

int mcpt_light_prep(mcpt_scene* sc, int32_t n, const double* x1, const double* nrm, const double* u, double* wsum,
                    int32_t* count, int32_t* pick) {
    return light_prep_query(sc, n, x1, nrm, u, wsum, count, pick, false);
}

int mcpt_debug_light_prep_exact(mcpt_scene* sc, int32_t n, const double* x1, const double* nrm, const double* u,
                                double* wsum, int32_t* count, int32_t* pick) {
    return light_prep_query(sc, n, x1, nrm, u, wsum, count, pick, true);
}

int mcpt_debug_light_literal(mcpt_scene* sc, const double* x1, const double* nrm, double* out) {
    if (!sc || !x1 || !nrm || !out) {
        set_error("invalid argument");
        return MCPT_E_INVALID;
    }
    std::lock_guard<std::mutex> lk(sc->mu);
    DeviceState* D;
    int rc;
    if ((rc = get_device_state(sc, -1, &D))) return rc;
    const int NL = D->d.NL;
    if (NL == 0) return MCPT_OK;
    void* dout;
    HIP_OK(hipMalloc(&dout, 160ull * NL));
    hipLaunchKernelGGL(k_light_literal, dim3((NL + 255) / 256), dim3(256), 0, D->stream, D->d, mk3(x1[0], x1[1], x1[2]),
                       mk3(nrm[0], nrm[1], nrm[2]), (double*)dout);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(D->stream));
    HIP_OK(hipMemcpy(out, dout, 160ull * NL, hipMemcpyDeviceToHost));
    (void)hipFree(dout);
    return MCPT_OK;
}

// host-only check of an 8-wide tree (include/mcpt_debug.h): every facet of the binary tree is reached exactly
// once, and every reached triangle's vertices lie inside the decoded box of every slot on its path (the
// traversal prunes with those boxes, so this is what keeps its hits the binary tree's)
// references beyond the first of each facet in a binary tree's leaf list (spatial splits repeat facets)
static int64_t dup_refs(const Bvh& b) {
    std::vector<int32_t> f(b.leaf_facets);
    std::sort(f.begin(), f.end());
    return (int64_t)(f.size() - (std::unique(f.begin(), f.end()) - f.begin()));
}
// A facet may sit in several leaves (spatial splits, each reference with its triangle clipped to one side):
// then its references' regions (the intersection of the slot boxes on each one's path) must together cover
// the triangle -- checked at the vertices, edge points and interior points; a facet with one reference
// needs all three vertices inside every box on its path.
struct RefRegion {
    int32_t f;
    float lo[3], hi[3];
};
static int64_t check_coverage(const HostScene& hs, std::vector<RefRegion>& refs) {
    std::sort(refs.begin(), refs.end(), [](const RefRegion& x, const RefRegion& y) { return x.f < y.f; });
    int64_t bad = 0;
    static const double kW[][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {.5, .5, 0}, {0, .5, .5}, {.5, 0, .5}, {1. / 3, 1. / 3, 1. / 3},
                                   {.8, .1, .1}, {.1, .8, .1}, {.1, .1, .8}, {.25, .75, 0}, {.75, .25, 0}, {0, .25, .75},
                                   {0, .75, .25}, {.25, 0, .75}, {.75, 0, .25}};
    for (size_t i = 0; i < refs.size();) {
        size_t j = i;
        while (j < refs.size() && refs[j].f == refs[i].f) j++;
        const float* v = &hs.pos[9 * (size_t)refs[i].f];
        const int npts = j - i == 1 ? 3 : (int)(sizeof(kW) / sizeof(kW[0]));
        for (int w = 0; w < npts; w++) {
            float x[3];
            for (int a = 0; a < 3; a++)
                x[a] = j - i == 1 ? v[3 * w + a] : (float)(kW[w][0] * v[a] + kW[w][1] * v[3 + a] + kW[w][2] * v[6 + a]);
            bool in = false;
            for (size_t r = i; r < j && !in; r++)
                in = x[0] >= refs[r].lo[0] && x[0] <= refs[r].hi[0] && x[1] >= refs[r].lo[1] && x[1] <= refs[r].hi[1] &&
                     x[2] >= refs[r].lo[2] && x[2] <= refs[r].hi[2];
            if (!in) bad++;
        }
        i = j;
    }
    return bad;
}
// the 4-wide tree every traversal kernel reads (collapse_bvh4 of the binary tree) and its quantized form
// (quantize_bvh4), walked on the host: every facet of the binary tree reached, each reference's triangle
// covered by the slot boxes on its path (check_coverage), and every quantized slot box containing its fp32
// box (the conservative rounding the persistent traversal relies on)
int mcpt_debug_bvh4_check(mcpt_scene* sc, int32_t light_only, int64_t* out) {
    if (!sc || !out) {
        set_error("invalid argument");
        return MCPT_E_INVALID;
    }
    std::lock_guard<std::mutex> lk(sc->mu);
    const Bvh& bb = light_only ? sc->lbvh : sc->bvh;
    const std::vector<BvhNode4> b4 = collapse_bvh4(bb);
    const std::vector<BvhNode4Q> q4 = quantize_bvh4(b4);
    const HostScene& hs = sc->host;
    int64_t nodes = 0, tris = 0, dup = 0, bad = 0, maxd = 0;
    std::vector<int> seen(hs.F, 0);
    std::vector<RefRegion> refs;
    RefRegion cur{0, {-FLT_MAX, -FLT_MAX, -FLT_MAX}, {FLT_MAX, FLT_MAX, FLT_MAX}};
    std::function<void(int32_t, int)> walk = [&](int32_t ni, int depth) {
        if (ni < 0 || (size_t)ni >= b4.size()) {
            bad++;
            return;
        }
        nodes++;
        maxd = std::max<int64_t>(maxd, depth);
        const BvhNode4& n = b4[ni];
        const BvhNode4Q& q = q4[ni];
        for (int k = 0; k < 4; k++) {
            if (n.child[k] == kBvh4Empty || (n.child[k] < 0 && n.count[k] == 0)) continue;
            const RefRegion saved = cur;
            for (int a = 0; a < 3; a++) {
                cur.lo[a] = std::max(cur.lo[a], n.lo[a][k]), cur.hi[a] = std::min(cur.hi[a], n.hi[a][k]);
                const uint32_t bits = ((q.ex >> (8 * a)) & 0xffu) << 23;
                float sc_;
                std::memcpy(&sc_, &bits, 4);
                const float ql = std::fmaf((float)((q.q[2 * a] >> (8 * k)) & 0xffu), sc_, q.org[a]);
                const float qh = std::fmaf((float)((q.q[2 * a + 1] >> (8 * k)) & 0xffu), sc_, q.org[a]);
                if (!(ql <= n.lo[a][k] && qh >= n.hi[a][k])) bad++;
            }
            if (n.child[k] >= 0) {
                walk(n.child[k], depth + 1);
            } else {
                const int32_t first = ~n.child[k];
                for (int32_t j = first; j < first + n.count[k]; j++) {
                    if (j < 0 || (size_t)j >= bb.leaf_facets.size() || bb.leaf_facets[j] < 0 || bb.leaf_facets[j] >= hs.F) {
                        bad++;
                        continue;
                    }
                    const int f = bb.leaf_facets[j];
                    tris++;
                    if (seen[f]++) dup++;
                    cur.f = f;
                    refs.push_back(cur);
                }
            }
            cur = saved;
        }
    };
    if (!b4.empty()) walk(0, 1);
    bad += check_coverage(hs, refs);
    out[0] = nodes;
    out[1] = tris - dup;  // distinct facets reached
    out[2] = (int64_t)bb.leaf_facets.size() - dup_refs(bb);
    out[3] = dup;
    out[4] = bad;
    out[5] = maxd;
    return MCPT_OK;
}

int mcpt_debug_bvh8_check(mcpt_scene* sc, int32_t light_only, int64_t* out) {
    if (!sc || !out) {
        set_error("invalid argument");
        return MCPT_E_INVALID;
    }
    std::lock_guard<std::mutex> lk(sc->mu);
    ensure_bvh8_host(sc);
    const Bvh8& b = light_only ? sc->lbvh8 : sc->bvh8;
    const Bvh& bb = light_only ? sc->lbvh : sc->bvh;
    const HostScene& hs = sc->host;
    int64_t nodes = 0, tris = 0, dup = 0, bad = 0, maxd = 0;
    std::vector<int> seen(hs.F, 0);
    struct Box {
        float lo[3], hi[3];
    };
    std::vector<Box> path;
    std::vector<RefRegion> refs;
    auto decode = [](const BvhNode8Q& n, int a, int k, bool hi) {
        const uint32_t w = hi ? n.qhi[a][k >> 2] : n.qlo[a][k >> 2];
        const uint32_t bits = ((n.ex >> (8 * a)) & 0xffu) << 23;
        float sc_;
        std::memcpy(&sc_, &bits, 4);
        return std::fmaf((float)((w >> (8 * (k & 3))) & 0xffu), sc_, n.org[a]);
    };
    std::function<void(int32_t, int)> walk = [&](int32_t ni, int depth) {
        if (ni < 0 || (size_t)ni >= b.nodes.size()) {
            bad++;
            return;
        }
        nodes++;
        maxd = std::max<int64_t>(maxd, depth);
        const BvhNode8Q& n = b.nodes[ni];
        const uint32_t imask = n.ex >> 24;
        for (int k = 0; k < 8; k++) {
            Box bx;
            for (int a = 0; a < 3; a++) bx.lo[a] = decode(n, a, k, false), bx.hi[a] = decode(n, a, k, true);
            path.push_back(bx);
            if (imask & (1u << k)) {
                walk(n.base_inner + k, depth + 1);
            } else {
                for (int j = 0; j < 2; j++) {
                    if (!(n.tvalid & (1u << (2 * k + j)))) continue;
                    const int64_t q = (int64_t)n.base_tri + 2 * k + j;
                    if (q < 0 || (size_t)q >= b.tri_facets.size() || b.tri_facets[q] < 0 || b.tri_facets[q] >= hs.F) {
                        bad++;
                        continue;
                    }
                    const int f = b.tri_facets[q];
                    tris++;
                    if (seen[f]++) dup++;
                    RefRegion r{f, {-FLT_MAX, -FLT_MAX, -FLT_MAX}, {FLT_MAX, FLT_MAX, FLT_MAX}};
                    for (const Box& p : path)
                        for (int a = 0; a < 3; a++) r.lo[a] = std::max(r.lo[a], p.lo[a]), r.hi[a] = std::min(r.hi[a], p.hi[a]);
                    refs.push_back(r);
                }
            }
            path.pop_back();
        }
    };
    if (!b.nodes.empty()) walk(0, 1);
    bad += check_coverage(hs, refs);
    out[0] = nodes;
    out[1] = tris - dup;  // distinct facets reached
    out[2] = (int64_t)bb.leaf_facets.size() - dup_refs(bb);
    out[3] = dup;
    out[4] = bad;
    out[5] = maxd;
    return MCPT_OK;
}

// the 4-wide tree every traversal kernel reads (collapse_bvh4 of the binary tree) and its quantized form
// (quantize_bvh4), walked on the host: every facet of the binary tree reached exactly once, each vertex
// inside every ancestor slot's box, and every quantized slot box containing its fp32 box (the conservative
// rounding the persistent traversal relies on)
int mcpt_debug_tri_filter(int32_t n, const float* tri, const double* ro, const double* rd, const float* tlim,
                          int32_t* verdict, float* tup) {
    if (n < 0 || (n > 0 && (!tri || !ro || !rd || !tlim || !verdict || !tup))) return MCPT_E_INVALID;
    for (int32_t k = 0; k < n; k++) {
        const float* v = tri + 9 * (size_t)k;
        const RayF r = ray_f(mk3(ro[3 * k], ro[3 * k + 1], ro[3 * k + 2]), mk3(rd[3 * k], rd[3 * k + 1], rd[3 * k + 2]));
        float t = 0;
        verdict[k] = tri_filter(make_float4(v[0], v[1], v[2], 0), make_float4(v[3], v[4], v[5], 0),
                                make_float4(v[6], v[7], v[8], 0), r, tlim[k], &t);
        tup[k] = t;
    }
    return MCPT_OK;
}

int mcpt_debug_prep_bench(mcpt_scene* sc, int32_t n, const double* x1, const double* nrm, const double* u,
                          int32_t variant, int32_t iters, double* ms, double* wsum, int32_t* pick) {
    if (!sc || n <= 0 || !x1 || !nrm || !u || iters <= 0 || !ms || !wsum || !pick) {
        set_error("invalid argument");
        return MCPT_E_INVALID;
    }
    std::lock_guard<std::mutex> lk(sc->mu);
    DeviceState* D;
    int rc;
    if ((rc = get_device_state(sc, -1, &D))) return rc;
    void *dp, *dn, *du, *dw, *dk, *dm;
    HIP_OK(hipMalloc(&dm, 8ull * n * mask_stride(prep_chunks(D->d.NL))));
    HIP_OK(hipMalloc(&dp, 24ull * n));
    HIP_OK(hipMalloc(&dn, 24ull * n));
    HIP_OK(hipMalloc(&du, 8ull * n));
    HIP_OK(hipMalloc(&dw, 8ull * n));
    HIP_OK(hipMalloc(&dk, 4ull * n));
    {  // node coordinates in the kernels' 3-vector layout (idx3, like the wavefront queue)
        const std::vector<double> px = soa3(x1, n), pn = soa3(nrm, n);
        HIP_OK(hipMemcpy(dp, px.data(), 24ull * n, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(dn, pn.data(), 24ull * n, hipMemcpyHostToDevice));
    }
    HIP_OK(hipMemcpy(du, u, 8ull * n, hipMemcpyHostToDevice));
    if ((rc = ensure(D->work, 256))) return rc;
    CullOrder co{};
    if ((rc = cull_order_bufs(*D, (size_t)n, &co))) return rc;
    HIP_OK(launch_prep(variant, D->d, 0, n, (const double*)dp, (const double*)dn, n, nullptr, nullptr, nullptr,
                       (const double*)du, (double*)dw, (int*)dk, nullptr, nullptr, (unsigned*)D->work.p, D->stream,
                       PrepCache{}, (uint64_t*)dm, true, false, co));
    HIP_OK(hipEventRecord(D->ev0, D->stream));
    for (int it = 0; it < iters; it++)
        HIP_OK(launch_prep(variant, D->d, 0, n, (const double*)dp, (const double*)dn, n, nullptr, nullptr, nullptr,
                           (const double*)du, (double*)dw, (int*)dk, nullptr, nullptr, (unsigned*)D->work.p, D->stream,
                       PrepCache{}, (uint64_t*)dm, true, false, co));
    HIP_OK(hipEventRecord(D->ev1, D->stream));
    HIP_OK(hipEventSynchronize(D->ev1));
    float t = 0;
    HIP_OK(hipEventElapsedTime(&t, D->ev0, D->ev1));
    *ms = t / iters;
    HIP_OK(hipMemcpy(wsum, dw, 8ull * n, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(pick, dk, 4ull * n, hipMemcpyDeviceToHost));
    for (int k = 0; k < n; k++) pick[k] = pick[k] >= 0 ? sc->host.light_facet[pick[k]] : -1;
    void* bufs[] = {dp, dn, du, dw, dk, dm};
    for (void* b : bufs) (void)hipFree(b);
    return MCPT_OK;
}

int mcpt_primary_hits(mcpt_scene* sc, const mcpt_camera* cam, int32_t* facet, double* tbg) {
    if (!sc || !facet || !tbg) {
        set_error("null argument");
        return MCPT_E_INVALID;
    }
    int rc = validate_camera(cam);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(sc->mu);
    DeviceState* D;
    if ((rc = get_device_state(sc, -1, &D))) return rc;
    const int npx = cam->width * cam->height;
    if ((rc = ensure(D->hit_f, 4ull * npx)) || (rc = ensure(D->hit_tbg, 24ull * npx))) return rc;
    hipLaunchKernelGGL(k_primary<false>, dim3((npx + kTraceBlock - 1) / kTraceBlock), dim3(kTraceBlock), 0, D->stream, D->d,
                       cam_setup(*cam), (int*)D->hit_f.p, (double*)D->hit_tbg.p);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(D->stream));
    HIP_OK(hipMemcpy(facet, D->hit_f.p, 4ull * npx, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(tbg, D->hit_tbg.p, 24ull * npx, hipMemcpyDeviceToHost));
    return MCPT_OK;
}

}  // extern "C"
