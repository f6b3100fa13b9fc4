// Device-side fp64 vector math with the reference's evaluation order (vec.cpp, matrix3d.cpp,
// BRDF.cpp, Mylight.cpp), plus the counter RNG shared bit-for-bit with the CPU oracle.
// Compiled with -ffp-contract=off: +, -, *, / and sqrt round exactly like the x86 reference.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "acos_cr.h"

namespace mcpt {

#define MCPT_EPS 1e-8
#define MCPT_PI 3.141592653589793
#define MCPT_P_RR 0.6
#define MCPT_MAX_DEPTH 48  // counter-RNG trees: deeper nodes contribute 0 (oracle COUNTER_MAX_DEPTH)
#ifndef MCPT_PHONG_SKIP_ZERO
#define MCPT_PHONG_SKIP_ZERO 1  // brdf_phong / phong_pdf: no pow for a specular term that is exactly zero
#endif
#ifndef MCPT_PHONG_SQRT
#define MCPT_PHONG_SQRT 1  // BRDF-only sample_phong<true>: sin / cos of theta by identities (see there)
#endif
#ifndef MCPT_PHONG_SINCOSPI
#define MCPT_PHONG_SINCOSPI 1  // BRDF-only sample_phong<true>: phi's sin / cos as sincospi(2 k2)
#endif

struct d3 {
    double x, y, z;
};
__device__ __host__ inline d3 mk3(double a, double b, double c) { return d3{a, b, c}; }
__device__ inline d3 add(d3 a, d3 b) { return d3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ inline d3 sub(d3 a, d3 b) { return d3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ inline d3 mul(d3 a, double c) { return d3{a.x * c, a.y * c, a.z * c}; }
__device__ inline d3 hmul(d3 a, d3 b) { return d3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ inline double dot(d3 a, d3 b) {  // vec.cpp:73-81 (ans = 0; ans += ...)
    double s = 0;
    s += a.x * b.x;
    s += a.y * b.y;
    s += a.z * b.z;
    return s;
}
__device__ inline d3 cross(d3 a, d3 b) {
    return d3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ inline double norm2(d3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
// vec.cpp:99-103: a.x / l, a.y / l, a.z / l with l = sqrt(x^2 + y^2 + z^2), each quotient correctly
// rounded.  The backend's fp64 division is v_div_scale (x2), v_rcp_f64, two Newton steps on the
// reciprocal, q = n y, r = fma(-l, q, n), v_div_fmas (= fma(r, y, q) unscaled) and v_div_fixup; the
// reciprocal part depends on l alone, so for the three quotients by one l it is done once here.  In the
// range where v_div_scale leaves its operands alone and v_div_fixup returns its input (l and the
// quotients' exponents far from the limits: l in [2^-500, 2^500], each nonzero |n| >= l 2^-500) this is
// the same arithmetic, so the quotients are the same correctly rounded values (a zero numerator keeps
// its sign through r == 0); outside it, plain division.
// MCPT_NORMALIZE_SHARED=1 (A/B only): the shared-reciprocal form above; measured slower than the three
// divisions the compiler emits (BRDF-only 5 652 -> 5 477 Msamples/s, MIS 449.5 -> 446.0, same box),
// so plain division is the default
#ifndef MCPT_NORMALIZE_SHARED
#define MCPT_NORMALIZE_SHARED 0
#endif
__device__ inline d3 normalized(d3 a) {
    const double l = norm2(a);
    const double lo = l * 0x1.0p-500;
    const bool fast = l >= 0x1.0p-500 && l <= 0x1.0p500 && (a.x == 0.0 || fabs(a.x) >= lo) &&
                      (a.y == 0.0 || fabs(a.y) >= lo) && (a.z == 0.0 || fabs(a.z) >= lo);
    if (!MCPT_NORMALIZE_SHARED || !fast) return d3{a.x / l, a.y / l, a.z / l};
    const double y0 = __builtin_amdgcn_rcp(l);
    const double y1 = fma(y0, fma(-l, y0, 1.0), y0);
    const double y = fma(y1, fma(-l, y1, 1.0), y1);
    auto q = [&](double n) {
        const double q0 = n * y;
        const double r = fma(-l, q0, n);
        return r == 0.0 ? q0 : fma(r, y, q0);
    };
    return d3{q(a.x), q(a.y), q(a.z)};
}
__device__ inline double det3(d3 a, d3 b, d3 c) { return dot(cross(a, b), c); }
__device__ inline d3 cols_mul(d3 c0, d3 c1, d3 c2, d3 x) {  // matrix3d(c0,c1,c2) * x
    double b0 = 0, b1 = 0, b2 = 0;
    b0 += c0.x * x.x;
    b0 += c1.x * x.y;
    b0 += c2.x * x.z;
    b1 += c0.y * x.x;
    b1 += c1.y * x.y;
    b1 += c2.y * x.z;
    b2 += c0.z * x.x;
    b2 += c1.z * x.y;
    b2 += c2.z * x.z;
    return d3{b0, b1, b2};
}
__device__ inline d3 f3(float4 v) { return d3{(double)v.x, (double)v.y, (double)v.z}; }

// ---- counter RNG (identical to oracle/mcpt_oracle.c counter_key / counter_u) -------------
__device__ __host__ inline uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}
__device__ __host__ inline uint64_t counter_key(uint64_t seed, uint64_t pixel, uint64_t sample, uint64_t node) {
    uint64_t k = mix64(seed + 0x9E3779B97F4A7C15ull * (pixel + 1));
    k = mix64(k ^ (0xD1B54A32D192ED03ull * (sample + 1)));
    return mix64(k ^ (0xA24BAED4963EE407ull * node));
}
__device__ __host__ inline double counter_u(uint64_t key, uint32_t dim) {
    return (double)(mix64(key + 0x9FB21C651E98DF25ull * (dim + 1)) >> 11) * 0x1.0p-53;
}

// ---- Phong BRDF (BRDF.cpp) --------------------------------------------------------------
// a specular term that is exactly zero: with c <= 1 + 1e-9 (unit vectors give c <= 1 + a few ulp) and
// 0 <= sh <= 1e6, pow(c, sh) lies in [0, 1.002), so a zero factor (ks = 0, or the pdf's lobe weight 0) makes the
// term +-0, and x + +-0 = x for the non-negative diffuse part -- skipping the fp64 pow (~220 VALU) there is
// bit-exact; a wave of diffuse-only lanes (the stand-in's floor and backdrop) branches round it.  kSkip = false in
// the BRDF-only kernels, where the branch cost more than it saved (C2 -1.7%; C3 +0.35%, C5 +0.5%:
// profiles/round5_ab_phong_skip.txt)
__device__ inline bool phong_pow_bounded(double c, double sh) { return c <= 1.000000001 && sh >= 0 && sh <= 1e6; }
// x^y as exp2(y log2 x) for the BRDF-only kernels (MCPT_PHONG_EXP2LOG; x > 0 or x = 0 with y > 0): relative
// error ~ln 2 |y log2 x| 2^-53 on top of two ~1-ulp functions -- a few ulp for these arguments (Phong lobes:
// |y log2 x| <~ 50) -- against ~220 fp64 VALU for pow's double-double logarithm
#ifndef MCPT_PHONG_BASIS
#define MCPT_PHONG_BASIS 1  // BRDF-only sample_phong<true>: the frame's constant cross products written out
#endif
#ifndef MCPT_PHONG_EXP2LOG
#define MCPT_PHONG_EXP2LOG 1
#endif
template <bool kFast>
__device__ inline double phong_pow(double x, double y) {
    return (kFast && MCPT_PHONG_EXP2LOG) ? exp2(y * log2(x)) : pow(x, y);
}
template <bool kSkip = true, bool kFast = false>
__device__ inline d3 brdf_phong(d3 n, d3 wi, d3 wr, d3 kd, d3 ks, double sh) {  // BRDF.cpp:17-25
    d3 R = add(mul(wi, -1), mul(n, 2 * dot(wi, n)));
    d3 ans = mul(kd, 1.0 / MCPT_PI);
    double c = dot(wr, R);
    if (c > 0 && !(kSkip && MCPT_PHONG_SKIP_ZERO && ks.x == 0 && ks.y == 0 && ks.z == 0 && phong_pow_bounded(c, sh))) ans = add(ans, mul(ks, (sh + 1) * phong_pow<kFast>(c, sh) / (2 * MCPT_PI)));
    return ans;
}
__device__ inline double phong_pdf(d3 n, d3 wi, d3 wr, d3 kd, d3 ks, double sh) {  // BRDF.cpp:107-133
    double d = dot(kd, mk3(1, 1, 1)) / 3;
    double s = dot(ks, mk3(1, 1, 1)) / 3;
    double sum = d + s;
    double pd = d / sum, ps = s / sum;
    double ct = dot(wi, n);
    if (ct < 0) pd *= 0;
    else pd *= ct / MCPT_PI;
    d3 R = normalized(add(mul(wr, -1), mul(n, 2 * dot(wr, n))));
    double cs = dot(wi, R);
    if (cs < 0) ps *= 0;
    else if (!(MCPT_PHONG_SKIP_ZERO && ps == 0 && phong_pow_bounded(cs, sh))) ps *= (sh + 1) / (2 * MCPT_PI) * pow(cs, sh);  // else +0 stays
    return pd + ps;
}
// sample_from_phong (BRDF.cpp:28-104) with explicit uniforms: lobe pick u0 (lower_bound on the
// normalised {p0, 1}), xi1, xi2.  May return directions below the surface (reference).
// kIdent (the BRDF-only kernels): theta's and phi's sin / cos without acos / sincos (MCPT_PHONG_SQRT,
// MCPT_PHONG_SINCOSPI), a few ulp from the reference's chain.  The MIS and shade() kernels keep the chain:
// there a sampled direction that hits a sliver light feeds the light pdf's ill-conditioned solid angle,
// and a few-ulp direction change moved two C1 MIS pixels by 2.9e-3 (tests/test_c1_frame.py)
template <bool kIdent = false>
__device__ inline d3 sample_phong(d3 n, d3 wr, d3 kd, d3 ks, double sh, double u0, double k1, double k2,
                                  double* pdf_out) {
    double d = dot(kd, mk3(1, 1, 1)) / 3;
    double s = dot(ks, mk3(1, 1, 1)) / 3;
    double sum = 0.0;
    sum += d;
    sum += s;
    double p0 = d / sum, p1 = s / sum;
    int ind = (p0 >= u0) ? 0 : 1;
    double pdf = 1;
    pdf *= ind == 0 ? p0 : p1;
    d3 axis = n;
    double theta, st, ct, sp, cp;
    double phi = 2 * MCPT_PI * k2;
    // the lobes' acos and sincos(theta) taken once after the lobe-specific argument (the same values:
    // theta = 0.5 acos(1 - 2 k1) or acos(k1^(1/(sh+1))); a wave with both lobes runs them once)
    double carg;
    if (ind == 0) carg = 1 - 2 * k1;
    else carg = phong_pow<kIdent>(k1, 1 / (sh + 1));
    if (kIdent && MCPT_PHONG_SQRT) {
        // sin / cos of theta by the identities instead of acos + sincos (~180 fp64 VALU): for the cosine lobe
        // theta = acos(x) / 2 with cos = sqrt((1 + x) / 2), sin = sqrt((1 - x) / 2); for the specular lobe
        // theta = acos(c) with cos = c, sin = sqrt((1 - c)(1 + c)) (1 - c exact near c = 1, no cancellation).
        // Equal to the reference's acos -> sin / cos chain (BRDF.cpp:51-54, 71, 80, 99) up to a few ulp
        const double c = fmax(-1.0, fmin(1.0, carg));
        st = sqrt(ind == 0 ? (1 - c) * 0.5 : (1 - c) * (1 + c));
        ct = ind == 0 ? sqrt((1 + c) * 0.5) : c;
    } else {
        theta = acos(fmax(-1.0, fmin(1.0, carg)));
        if (ind == 0) theta = 0.5 * theta;
        sincos(theta, &st, &ct);
    }
    if (ind == 0) {
        pdf *= ct / MCPT_PI;
    } else {
        // k1^(sh/(sh+1)) = k1 / k1^(1/(sh+1)) = k1 / carg: one fp64 pow (~220 VALU) instead of two, equal up to
        // ~2 ulp (BRDF.cpp:97 evaluates the pow; pow(0, y > 0) = 0).  C2 +0.9%, C3 +0.2% same-box
        // (profiles/round5_ab_pow_margin.txt).  Every kernel uses it (kIdent or not); the identity holds only
        // for sh > 0 with carg > 0, so anything else -- sh <= 0 (pow(0, 0) = 1; sh in (-1, 0) where carg can
        // underflow while k1 > 0) or k1 = 0 -- takes the reference's pow itself
        pdf *= (sh + 1) / (2 * MCPT_PI) * (sh > 0 && carg > 0 ? k1 / carg : pow(k1, sh / (sh + 1)));
        axis = normalized(add(mul(wr, -1), mul(n, 2 * dot(wr, n))));
    }
    if (kIdent && MCPT_PHONG_SINCOSPI) sincospi(2 * k2, &sp, &cp);
    else sincos(phi, &sp, &cp);
    d3 nx, ny;
    if (kIdent && MCPT_PHONG_BASIS) {
        // the same frame with the constant cross products written out (axis x e_x = (0, a.z, -a.y), axis x e_y =
        // (-a.z, 0, a.x)) and ny = axis x nx left unnormalised (unit up to rounding: axis and nx are orthonormal)
        const bool ex = fabs(axis.x - 1) > MCPT_EPS;  // dot(axis, e_x) is axis.x
        nx = normalized(ex ? mk3(0.0, axis.z, -axis.y) : mk3(-axis.z, 0.0, axis.x));
        ny = cross(axis, nx);
    } else {
        if (fabs(dot(axis, mk3(1, 0, 0)) - 1) > MCPT_EPS) nx = normalized(cross(axis, mk3(1, 0, 0)));
        else nx = normalized(cross(axis, mk3(0, 1, 0)));
        ny = normalized(cross(axis, nx));
    }
    *pdf_out = pdf;
    return normalized(cols_mul(nx, ny, axis, mk3(st * cp, st * sp, ct)));
}

// ---- ray / triangle: the reference's Cramer rule in fp64 (Myobj.cpp:165-192) -------------
struct TriHit {
    bool hit;
    double beta, gamma, t;
};
__device__ inline TriHit tri_hit(d3 a, d3 b, d3 c, d3 ro, d3 rd) {
    TriHit h{false, 0, 0, 0};
    d3 ab = sub(a, b), ac = sub(a, c), ar = sub(a, ro);
    double detA = det3(ab, ac, rd);
    if (fabs(detA) < MCPT_EPS) return h;
    double beta = det3(ar, ac, rd) / detA;
    double gamma = det3(ab, ar, rd) / detA;
    double t = det3(ab, ac, ar) / detA;
    if (beta < 0 || gamma < 0 || beta + gamma > 1 || t < 0 || fabs(t) < MCPT_EPS) return h;
    h.hit = true;
    h.beta = beta;
    h.gamma = gamma;
    h.t = t;
    return h;
}

// ---- spherical triangle of one light triangle at (x1, n): Mylight.cpp:335-413 -------------
struct SphTri {
    d3 A, B, C;
    double alpha, c, sA, w;
};
// cull stage reached: 0 = survives the reference's cull chain, 1 = culled by the light-side test
// (Mylight.cpp:340-345), 2 = by the tangent-plane test (:347-357), 3 = by a later degeneracy test.
// The edge-length culls a, b, c < 1e-8 (:372-374) need no acos: acos(x) < 1e-8 iff the clamped x is
// 1 (acos of the largest double below 1 is 1.49e-8, for glibc as for the correctly rounded acos_cr;
// NaN clamps to 1 as well), so the chain takes three acos (alpha, beta, gamma) plus c = acos(A.B)
// when Arvo's sampler needs it (kArvo: o->alpha, o->c).  w = sA lsum.
template <bool kArvo = false>
__device__ inline int light_tri_stage(d3 p0, d3 p1, d3 p2, d3 nl, double lsum, d3 x1, d3 n, SphTri* o) {
    double tmp = dot(nl, sub(x1, p0));
    if (tmp < 0 || fabs(tmp) < MCPT_EPS) return 1;
    double t0 = dot(n, sub(p0, x1)), t1 = dot(n, sub(p1, x1)), t2 = dot(n, sub(p2, x1));
    if ((t0 < 0 || fabs(t0) < MCPT_EPS) && (t1 < 0 || fabs(t1) < MCPT_EPS) && (t2 < 0 || fabs(t2) < MCPT_EPS))
        return 2;
    d3 A = normalized(sub(p0, x1)), B = normalized(sub(p1, x1)), C = normalized(sub(p2, x1));
    if (dot(cross(normalized(sub(C, A)), normalized(sub(B, A))), n) < 0) {
        d3 t = B;
        B = C;
        C = t;
    }
    const double ca = fmax(-1.0, fmin(1.0, dot(B, C)));
    const double cb = fmax(-1.0, fmin(1.0, dot(A, C)));
    const double cc = fmax(-1.0, fmin(1.0, dot(A, B)));
    if (ca == 1.0 || cb == 1.0 || cc == 1.0) return 3;  // a, b or c < 1e-8
    const d3 uBA = normalized(cross(B, A)), uAC = normalized(cross(A, C)), uCB = normalized(cross(C, B));
    // one angle at a time with its test (the same outcome as the reference's three acos and one
    // test: every failing test returns 3): the branches keep the three acos_cr from interleaving,
    // which caps the register peak of the kernels that inline this chain
    const double alpha = acos_cr(fmax(-1.0, fmin(1.0, -dot(uBA, uAC))));
    if (alpha < MCPT_EPS) return 3;
    const double beta = acos_cr(fmax(-1.0, fmin(1.0, -dot(uCB, uBA))));
    if (beta < MCPT_EPS) return 3;
    const double gamma = acos_cr(fmax(-1.0, fmin(1.0, -dot(uAC, uCB))));
    if (gamma < MCPT_EPS) return 3;
    double sA = alpha + beta + gamma - MCPT_PI;
    if (sA < 0) return 3;
    double w = sA * lsum;
    if (w < 0) return 3;
    if (isinf(w) || isnan(w)) return 3;
    if (o) {
        o->A = A;
        o->B = B;
        o->C = C;
        o->alpha = alpha;
        o->c = kArvo ? acos_cr(cc) : 0.0;
        o->sA = sA;
        o->w = w;
    }
    return 0;
}
__device__ inline bool light_tri_eval(d3 p0, d3 p1, d3 p2, d3 nl, double lsum, d3 x1, d3 n, SphTri* o) {
    return light_tri_stage(p0, p1, p2, nl, lsum, x1, n, o) == 0;
}

// ---- light prep, GPU formulation ---------------------------------------------------------
// Stage 1+2 (cheap, exact reference arithmetic): the light-side test (Mylight.cpp:340-345) and
// the tangent-plane test (:347-357).  Returns true if the triangle is a candidate.
// 0 = candidate, 1 = culled by the light-side test, 2 = culled by the tangent-plane test
__device__ inline int light_cheap_stage(d3 p0, d3 p1, d3 p2, d3 nl, d3 x1, d3 n) {
    double tmp = dot(nl, sub(x1, p0));
    if (tmp < 0 || fabs(tmp) < MCPT_EPS) return 1;
    double t0 = dot(n, sub(p0, x1)), t1 = dot(n, sub(p1, x1)), t2 = dot(n, sub(p2, x1));
    return ((t0 < 0 || fabs(t0) < MCPT_EPS) && (t1 < 0 || fabs(t1) < MCPT_EPS) && (t2 < 0 || fabs(t2) < MCPT_EPS)) ? 2 : 0;
}
__device__ inline bool light_cheap(d3 p0, d3 p1, d3 p2, d3 nl, d3 x1, d3 n) {
    return light_cheap_stage(p0, p1, p2, nl, x1, n) == 0;
}

__device__ inline double fdot(d3 a, d3 b) { return fma(a.x, b.x, fma(a.y, b.y, a.z * b.z)); }
__device__ inline d3 fcross(d3 a, d3 b) {
    return d3{fma(a.y, b.z, -a.z * b.y), fma(a.z, b.x, -a.x * b.z), fma(a.x, b.y, -a.y * b.x)};
}
// a * b + c with a wave-uniform c taken from SGPRs: one v_fma_f64 (the compiler otherwise keeps
// fp64 constants in VGPRs and copies each into a v_fmac accumulator first)
__device__ inline double fma_s(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

// 1/sqrt(s) by the hardware rsqrt estimate plus one second-order Newton step, y (1 + e/2) with
// e = 1 - s y^2: relative error ~1.5 e0^2 ~ 1e-14 for the estimate's e0 (weights agree with the
// third-order refinement to ~1e-13 relative, measured; a third-order step costs one more fp64
// FMA per vector in the prep's hottest loop).  No zero/inf fix-ups: a zero vector gives NaN,
// which every caller culls.
__device__ inline double frsq(double s) {
    const double y = __builtin_amdgcn_rsq(s);
    const double e = fma(-s * y, y, 1.0);  // 1 - s y^2
    return fma(y * e, 0.5, y);
}
// a / |a|
__device__ inline d3 funit(d3 a) {
    const double r = frsq(fdot(a, a));
    return d3{a.x * r, a.y * r, a.z * r};
}
// num / den for den > 0 (finite): hardware reciprocal estimate plus one second-order step
// r (1 + e), e = 1 - den r, then one rounding in the product (~1e-14 relative)
__device__ inline double fdiv_pos(double num, double den) {
    const double r = __builtin_amdgcn_rcp(den);
    const double e = fma(-den, r, 1.0);
    return num * fma(r, e, r);
}
__device__ inline double clamp1(double x) { return fmax(-1.0, fmin(1.0, x)); }

// atan2(y, x) for y >= 0 in fp64 (<= ~5 ulp): one division and a degree-9 polynomial in z^2 on
// |z| <= tan(pi/8), fitted in extended precision (tools/fit_atan.py); ~40 instructions instead of
// ocml's ~100.  Octant reduction: y <= k|x|: z = y/|x|; |x| <= k y: z = -|x|/y (+pi/2);
// otherwise z = (y-|x|)/(y+|x|) (+pi/4); then pi - r for x < 0.
// atan(z) for |z| <= tan(pi/8): z + z^3 P(z^2)
// The Horner chain is ONE asm block: between two separate asm statements the compiler's hazard
// recognizer cannot see the instructions and pads each boundary with an s_nop (8 per call); a
// dependent v_fma_f64 chain needs no software wait states on gfx950.
__device__ inline double atan_core(double z) {
    const double s = z * z;
    double p;
    asm("v_fma_f64 %0, %2, %1, %3\n\t"
        "v_fma_f64 %0, %0, %1, %4\n\t"
        "v_fma_f64 %0, %0, %1, %5\n\t"
        "v_fma_f64 %0, %0, %1, %6\n\t"
        "v_fma_f64 %0, %0, %1, %7\n\t"
        "v_fma_f64 %0, %0, %1, %8\n\t"
        "v_fma_f64 %0, %0, %1, %9\n\t"
        "v_fma_f64 %0, %0, %1, %10\n\t"
        "v_fma_f64 %0, %0, %1, %11"
        : "=&v"(p)
        : "v"(s), "v"(0.023022964535612277), "s"(-0.045054138438556275), "s"(0.05743860627393907),
          "s"(-0.0665101622857059), "s"(0.07691210259772996), "s"(-0.09090862908839843),
          "s"(0.11111110041613353), "s"(-0.14285714274661848), "s"(0.19999999999980458),
          "s"(-0.33333333333333476));
    return fma(z * s, p, z);
}
__device__ inline double atan2_pos(double y, double x) {
    constexpr double k = 0.41421356237309503;  // tan(pi/8)
    const double ax = fabs(x);
    const bool A = y <= k * ax, D = !A && ax <= k * y;
    // (num, den, r0) = A: (y, ax, 0); D: (-ax, y, pi/2); else (y - ax, y + ax, pi/4), as
    // num = p y - q ax, den = q y + p ax, r0 = q (pi/2 - p pi/4) with p, q in {0, 1} (exact)
    const double pc = D ? 0.0 : 1.0, qc = A ? 0.0 : 1.0;
    const double num = fma(pc, y, -(qc * ax));
    const double den = fma(qc, y, pc * ax);
    const double r0 = qc * fma(-pc, 0.7853981633974483, 1.5707963267948966);
    const double a = r0 + atan_core(fdiv_pos(num, den));
    return x < 0 ? 3.141592653589793 - a : a;
}
// atan2_pos with a wave-uniform fast path: when every active lane is in the first octant (x > 0,
// y <= tan(pi/8) x -- the spherical triangles of all but the nearest lights), z = y / x directly,
// without the octant selects.  Bit-identical to atan2_pos there (num = y, den = x, r0 = 0 exactly).
__device__ inline double atan2_pos_wave(double y, double x) {
    constexpr double k = 0.41421356237309503;
    if (__ballot(!(x > 0.0 && y <= k * x)) == 0) return atan_core(fdiv_pos(y, x));
    return atan2_pos(y, x);
}

// atan(z) for |z| <= 0.03 by its Taylor series to z^9: the truncation is below z^10/11 <= 5.4e-17
// relative, under half an ulp, so this agrees with atan_core to rounding (5 instructions instead of
// 11).  In the light prep almost every spherical triangle is small (tan(sA/2) ~ 1e-4..1e-2).
#ifdef MCPT_ATAN_SHORT5  // A/B: to z^11, |z| <= 0.05 (truncation <= 0.05^12/13 = 1.9e-17)
constexpr double kAtanShortMax = 0.05;
__device__ inline double atan_short(double z) {
    const double s = z * z;
    double p;
    asm("v_fma_f64 %0, %1, %2, %3\n\t"
        "v_fma_f64 %0, %0, %1, %4\n\t"
        "v_fma_f64 %0, %0, %1, %5\n\t"
        "v_fma_f64 %0, %0, %1, %6"
        : "=&v"(p)
        : "v"(s), "v"(-0.09090909090909091), "s"(0.1111111111111111), "s"(-0.14285714285714285), "s"(0.2),
          "s"(-0.3333333333333333));
    return fma(z * s, p, z);
}
#else
constexpr double kAtanShortMax = 0.03;
__device__ inline double atan_short(double z) {
    const double s = z * z;
    double p;
    asm("v_fma_f64 %0, %1, %2, %3\n\t"
        "v_fma_f64 %0, %0, %1, %4\n\t"
        "v_fma_f64 %0, %0, %1, %5"
        : "=&v"(p)
        : "v"(s), "v"(0.1111111111111111), "s"(-0.14285714285714285), "s"(0.2), "s"(-0.3333333333333333));
    return fma(z * s, p, z);
}
#endif
// atan2_pos_wave with a second wave-uniform fast path for the light prep's batches: when every
// lane has x > 0 and y <= 0.03 x, atan_short.  Only the prep's batch evaluation uses it, where the
// wave's lanes are one node's candidate batch (fixed by the node), so a weight never depends on
// how nodes were batched.
__device__ inline double atan2_pos_prep(double y, double x) {
    if (__ballot(!(x > 0.0 && y <= kAtanShortMax * x)) == 0) return atan_short(fdiv_pos(y, x));
    return atan2_pos_wave(y, x);
}

// Stage 3 (Mylight.cpp:360-413) in fp64 with fewer instructions than the reference's literal
// formulation; identical up to rounding (DESIGN.md "light prep numerics"):
//  * unit vectors A, B, C by rsqrt instead of sqrt + 3 divisions;
//  * the spherical excess sA = alpha + beta + gamma - pi by the Van Oosterom-Strackee identity
//    sA = 2 atan2(|A.(B x C)|, 1 + A.B + B.C + C.A) (one atan2 instead of six acos, and free of
//    the cancellation of alpha+beta+gamma-pi for small triangles);
//  * the edge-length culls a,b,c < 1e-8 rad as cos >= 1 (NaN included): in fp64, acos(x) < 1e-8
//    iff x rounds to 1 (acos of the largest double below 1 is 1.49e-8), so no acos is needed;
//  * the vertex-angle culls alpha, beta, gamma < 1e-8 (a degenerate, zero-area spherical
//    triangle) as sA <= 0.
// Every consumer (the prep batches, the small-N_L lane prep, the pdf's survival test in
// k_mis_combine and the picked triangle's Arvo setup in k_mis_gen / k_shade_gen) goes through
// sph_excess on the same unswapped vectors, so they agree bit for bit on survival; sA agrees bit
// for bit except that the prep's batches (kPrepBatch) may take atan_short, equal to rounding.
struct SphEx {
    d3 A, B, C;     // unit vectors towards p0, p1, p2 (reference vertex order)
    double ab;      // A.B
    double half;    // sA / 2
    double num;     // |A.(B x C)|
    double den;     // 1 + A.B + B.C + C.A = 4 - (the three edges' 1 - cos)
    bool edges_ok;  // A.B, B.C, C.A < 1
};
template <bool kPrepBatch = false>
__device__ inline SphEx sph_excess(d3 a, d3 b, d3 c) {
    SphEx e;
    e.A = funit(a);
    e.B = funit(b);
    e.C = funit(c);
    const double ab = fdot(e.A, e.B), bc = fdot(e.B, e.C), ca = fdot(e.C, e.A);
    e.ab = ab;
    e.edges_ok = (ab < 1.0) & (bc < 1.0) & (ca < 1.0);
    const double num = fabs(fdot(e.A, fcross(e.B, e.C))), den = 1.0 + ab + bc + ca;
    e.num = num;
    e.den = den;
    e.half = kPrepBatch ? atan2_pos_prep(num, den) : atan2_pos_wave(num, den);
    return e;
}

// Weight of one light triangle (Mylight.cpp:360-413) without branches: every lane evaluates
// straight through and the culls become one predicate.  lsum2 = 2 RadianceRGB::sum(), so
// w = (sA/2) lsum2 rounds exactly like the reference's sA * sum (scaling by 2 is exact) without
// the doubling of sA; 0 <= w <= DBL_MAX is one v_cmp_class (-0, +0, +denormal, +normal).
// Returns w, or 0 if culled (*ok = false).
template <bool kPrepBatch = false>
__device__ inline double light_weight_bf(d3 p0, d3 p1, d3 p2, double lsum2, d3 x1, bool* ok) {
    const SphEx e = sph_excess<kPrepBatch>(sub(p0, x1), sub(p1, x1), sub(p2, x1));
    const double w = e.half * lsum2;
    const bool good = e.edges_ok & (e.half > 0) & __builtin_amdgcn_class(w, 0x1e0);
    *ok = good;
    return good ? w : 0.0;
}
// ---- exact pick: light_weight_bf plus the error bookkeeping of the pick band ----
// The reference's weight (alpha + beta + gamma - pi from six acos, Mylight.cpp:375-396) differs from
// this one by its own rounding, ~u / (edge angle) for ordinary triangles and ~u sqrt(2x) / num for
// slivers (a spherical triangle seen nearly edge-on: an angle near 0 or pi, where acos is
// ill-conditioned).  Slivers -- 4 - den > kBandTau num, i.e. the sum of 1/sin of the angles above
// ~2 kBandTau -- are flagged here (one FMA and one compare per candidate) and carry their error term
// into the band; the others are covered by the per-chunk bound.  tau 300 (round 6; was 1000): many
// near-slivers just below 1000 together exceeded the per-chunk bound (tools/band_margin_study.py).
#ifndef MCPT_BAND_TAU
#define MCPT_BAND_TAU 300.0
#endif
struct WeightBx {
    double w;     // weight (0 if culled)
    double num;   // |A.(B x C)|
    double den;   // 1 + A.B + B.C + C.A
    bool ok;      // survives the full stage
    bool sliver;  // 4 - den > kBandTau num
};
template <bool kPrepBatch = false>
__device__ inline WeightBx light_weight_bx(d3 p0, d3 p1, d3 p2, double lsum2, d3 x1) {
    const SphEx e = sph_excess<kPrepBatch>(sub(p0, x1), sub(p1, x1), sub(p2, x1));
    const double w = e.half * lsum2;
    const bool good = e.edges_ok & (e.half > 0) & __builtin_amdgcn_class(w, 0x1e0);
    return WeightBx{good ? w : 0.0, e.num, e.den, good, fma(MCPT_BAND_TAU, e.num, e.den) < 4.0};
}
// the sliver's error term (without the factor u lsum2 / 2 applied by the caller): sqrt(2x) / num,
// x = 4 - den, from the hardware rsqrt / rcp estimates (~1e-7 relative), rounded up by 1% (a bound
// only; no IEEE sqrt / division sequence and its constants in the prep's hot loop)
__device__ inline double sliver_term(double num, double den) {
    const double x2 = fmax(2.0 * (4.0 - den), 1e-300);
    return x2 * __builtin_amdgcn_rsq(x2) * __builtin_amdgcn_rcp(num) * 1.01;
}
// Survival of one light triangle under the reference's literal chain (light_tri_stage == 0) decided
// without it where that is safe: 0 = culled (the exact cheap stages), 1 = survives, -1 = undecided (run
// the literal chain).  From the rsqrt unit vectors (~1e-13 from the literal's sqrt / division ones):
//  * every edge 1 - cos > 1e-9, so the literal's clamped cosines are < 1 (no edge-length cull);
//  * 4 - den <= 1000 num (not a sliver): the spherical law of sines gives 1 / sin(alpha) = sin b sin c / num
//    <= (1 - cos b) + (1 - cos c) <= 4 - den (sin^2 <= 2 (1 - cos)), so every vertex angle has
//    sin >= 1e-3 -- far from the 1e-8 angle culls, and acos is well conditioned (the literal angles are
//    within ~1e-12 of the true ones);
//  * num > 1e-9 max(den, 0), i.e. tan(sA / 2) > 1e-9: the literal sA = alpha + beta + gamma - pi is far
//    above its rounding, so sA > 0;
//  * 0 <= sum L < 1e300 (sA <= 2 pi): w = sA sum L is >= 0 and finite, so the literal chain's w < 0 / inf /
//    NaN culls (Mylight.cpp:405-411) cannot fire.  A negative, huge or NaN radiance is left to the chain.
__device__ inline int literal_survival_quick(d3 p0, d3 p1, d3 p2, d3 nl, double lsum, d3 x1, d3 n) {
    if (light_cheap_stage(p0, p1, p2, nl, x1, n) != 0) return 0;
    const d3 A = funit(sub(p0, x1)), B = funit(sub(p1, x1)), C = funit(sub(p2, x1));
    const double ab = fdot(A, B), bc = fdot(B, C), ca = fdot(C, A);
    const double num = fabs(fdot(A, fcross(B, C))), den = 1.0 + ab + bc + ca;
    const bool clear = fmax(ab, fmax(bc, ca)) < 1.0 - 1e-9 && 4.0 - den <= 1000.0 * num && num > 1e-9 * fmax(den, 0.0) &&
                       lsum >= 0.0 && lsum < 1e300;
    return clear ? 1 : -1;
}
__device__ inline bool light_weight(d3 p0, d3 p1, d3 p2, double lsum2, d3 x1, double* w_out) {
    bool ok;
    *w_out = light_weight_bf(p0, p1, p2, lsum2, x1, &ok);
    return ok;
}

// ---- MCPT_RENDER_PRECISION_FP32 (opt-in): the full stage of two candidates in packed fp32 ----
// The same Van Oosterom-Strackee excess, evaluated for two light triangles per lane with
// v_pk_fma/mul/add_f32 (two lights per VALU instruction) from 10-float records: p0, the edges
// e1 = p1 - p0, e2 = p2 - p0 (differences of nearby floats, exact in fp32 for small triangles),
// 2 RadianceRGB::sum().  Three record loads per light instead of five (the fp64 batch loop is
// co-limited by its light-record load instructions):
//  * a = p0 - x1 with x1 split into float hi + lo parts (~1e-7 relative even next to a light);
//    b = a + e1, c = a + e2;
//  * the triple product as a . (e1 x e2) (= a . (b x c) exactly in real arithmetic), free of the
//    cancellation of b x c for small, distant triangles;
//  * tan(sA/2) = |a.n| / (|a||b||c| + (a.b)|c| + (b.c)|a| + (c.a)|b|) from rsqrt of the squared
//    lengths (no Newton step) and atan by its series to z^7 when the wave's z <= 0.1 (else atanf);
//  * w = double(sA/2) * double(2 sum), accumulated in fp64 like the default path.
// Weights agree with the fp64 path to ~1e-6 relative.  Culls: w finite, sA > 0; the reference's
// edge-length and vertex-angle culls (< 1e-8 rad) are not resolvable in fp32 and are subsumed by
// sA > 0 for degenerate triangles (a nondegenerate triangle below 1e-8 rad keeps its ~1e-16 weight).
typedef float v2f_t __attribute__((ext_vector_type(2)));
typedef float v4f_t __attribute__((ext_vector_type(4)));
struct LightF32 {  // one record as loaded: (p0, e1.x), (e1.y, e1.z, e2.x, e2.y), (e2.z, 2 sum)
    v4f_t q0, q1;
    v2f_t q2;
};
__device__ inline v2f_t pk_fma(v2f_t a, v2f_t b, v2f_t c) { return __builtin_elementwise_fma(a, b, c); }
// weights of lights I, J for the node at x1 = xh + xl (floats per component)
__device__ inline void light_weight_f32x2(const LightF32& I, const LightF32& J, v2f_t xh, v2f_t yh, v2f_t zh,
                                          v2f_t xl, v2f_t yl, v2f_t zl, double* w0, double* w1, bool* ok0, bool* ok1) {
    // {light I, light J} pairs of each record float (v_pk_mov_b32 from the two loads)
    const v2f_t ax = (__builtin_shufflevector(I.q0, J.q0, 0, 4) - xh) - xl,
                ay = (__builtin_shufflevector(I.q0, J.q0, 1, 5) - yh) - yl,
                az = (__builtin_shufflevector(I.q0, J.q0, 2, 6) - zh) - zl;
    const v2f_t e1x = __builtin_shufflevector(I.q0, J.q0, 3, 7), e1y = __builtin_shufflevector(I.q1, J.q1, 0, 4),
                e1z = __builtin_shufflevector(I.q1, J.q1, 1, 5);
    const v2f_t e2x = __builtin_shufflevector(I.q1, J.q1, 2, 6), e2y = __builtin_shufflevector(I.q1, J.q1, 3, 7),
                e2z = __builtin_shufflevector(I.q2, J.q2, 0, 2);
    const v2f_t bx = ax + e1x, by = ay + e1y, bz = az + e1z;
    const v2f_t cx = ax + e2x, cy = ay + e2y, cz = az + e2z;
    const v2f_t nx = pk_fma(e1y, e2z, -(e1z * e2y)), ny = pk_fma(e1z, e2x, -(e1x * e2z)), nz = pk_fma(e1x, e2y, -(e1y * e2x));
    const v2f_t aa = pk_fma(ax, ax, pk_fma(ay, ay, az * az));
    const v2f_t bb = pk_fma(bx, bx, pk_fma(by, by, bz * bz));
    const v2f_t cc = pk_fma(cx, cx, pk_fma(cy, cy, cz * cz));
    const v2f_t ra = v2f_t{__builtin_amdgcn_rsqf(aa.x), __builtin_amdgcn_rsqf(aa.y)};
    const v2f_t rb = v2f_t{__builtin_amdgcn_rsqf(bb.x), __builtin_amdgcn_rsqf(bb.y)};
    const v2f_t rc = v2f_t{__builtin_amdgcn_rsqf(cc.x), __builtin_amdgcn_rsqf(cc.y)};
    const v2f_t ab = pk_fma(ax, bx, pk_fma(ay, by, az * bz));
    const v2f_t bc = pk_fma(bx, cx, pk_fma(by, cy, bz * cz));
    const v2f_t ca = pk_fma(cx, ax, pk_fma(cy, ay, cz * az));
    const v2f_t t = pk_fma(ax, nx, pk_fma(ay, ny, az * nz));
    const v2f_t rab = ra * rb;
    const v2f_t den = pk_fma(ab, rab, pk_fma(bc, rb * rc, pk_fma(ca, rc * ra, v2f_t{1.0f, 1.0f})));
    const v2f_t num = __builtin_elementwise_abs(t) * (rab * rc);
    float h0, h1;
    if (__ballot(!(den.x > 0.0f && num.x <= 0.1f * den.x && den.y > 0.0f && num.y <= 0.1f * den.y)) == 0) {
        // atan(z) = z - z^3/3 + z^5/5 - z^7/7 for z <= 0.1 (truncation z^8/9 < 1.2e-9)
        const v2f_t z = num * v2f_t{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
        const v2f_t sq = z * z;
        const v2f_t p = pk_fma(sq, pk_fma(sq, v2f_t{-0.14285714f, -0.14285714f}, v2f_t{0.2f, 0.2f}),
                               v2f_t{-0.33333334f, -0.33333334f});
        const v2f_t h = pk_fma(z * sq, p, z);
        h0 = h.x;
        h1 = h.y;
    } else {
        h0 = atan2f(num.x, den.x);
        h1 = atan2f(num.y, den.y);
    }
    const double v0 = (double)h0 * (double)I.q2.y, v1 = (double)h1 * (double)J.q2.y;
    *ok0 = (h0 > 0.0f) & __builtin_amdgcn_class(v0, 0x1e0);
    *ok1 = (h1 > 0.0f) & __builtin_amdgcn_class(v1, 0x1e0);
    *w0 = *ok0 ? v0 : 0.0;
    *w1 = *ok1 ? v1 : 0.0;
}

// The picked triangle's spherical triangle for Arvo's sampler: the same survival and sA as
// light_weight_bf (lsum2 = 2 RadianceRGB::sum()), plus unit vectors in the reference's orientation (B, C swapped so that the
// triangle winds counter-clockwise about n, Mylight.cpp:366-371; the test runs on the
// un-normalised edge vectors, normalising by positive lengths cannot change its sign), alpha
// (the angle at A between the great arcs AB and AC, Mylight.cpp:385) and c = acos(A.B).
// Returns true if the triangle survives; fills o.
__device__ inline bool light_full(d3 p0, d3 p1, d3 p2, double lsum2, d3 x1, d3 n, SphTri* o, bool* sliver = nullptr) {
    const SphEx e = sph_excess(sub(p0, x1), sub(p1, x1), sub(p2, x1));
    if (sliver) *sliver = fma(MCPT_BAND_TAU, e.num, e.den) < 4.0;
    const double w = e.half * lsum2;
    if (!(e.edges_ok & (e.half > 0) & __builtin_amdgcn_class(w, 0x1e0))) return false;
    const d3 A = e.A;
    d3 B = e.B, C = e.C;
    double ab = e.ab;
    if (fdot(fcross(sub(C, A), sub(B, A)), n) < 0) {
        const d3 t = B;
        B = C;
        C = t;
        ab = fdot(A, B);
    }
    o->A = A;
    o->B = B;
    o->C = C;
    const d3 u1 = fcross(B, A), u2 = fcross(A, C);
    o->alpha = acos(clamp1(-(fdot(u1, u2) * rsqrt(fdot(u1, u1)) * rsqrt(fdot(u2, u2)))));
    o->c = acos(clamp1(ab));
    o->sA = 2.0 * e.half;
    o->w = w;
    return true;
}

// Arvo SampleTriangle (Mylight.cpp:453-461)
__device__ inline d3 arvo_sample(const SphTri& st, double ksi1, double ksi2) {
    double sA1 = ksi1 * st.sA;
    double ss, tt, sa, ca;
    sincos(sA1 - st.alpha, &ss, &tt);
    sincos(st.alpha, &sa, &ca);
    double u = tt - ca;
    double v = ss + sa * cos(st.c);
    double q = ((v * tt - u * ss) * ca - v) / ((v * ss + u * tt) * sa);
    d3 C1 = normalized(add(mul(st.A, q), mul(normalized(sub(st.C, mul(st.A, dot(st.C, st.A)))), sqrt(1 - q * q))));
    double z = 1 - ksi2 * (1 - dot(C1, st.B));
    return normalized(add(mul(st.B, z), mul(normalized(sub(C1, mul(st.B, dot(C1, st.B)))), sqrt(1 - z * z))));
}

}  // namespace mcpt
