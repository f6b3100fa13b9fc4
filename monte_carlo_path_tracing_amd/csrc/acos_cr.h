// acos to ~2^-100 before its final rounding, for the reference's literal light chain (Mylight.cpp:375-396:
// six acos per light triangle, alpha + beta + gamma - pi).  The chain's sA cancels: a 1-ulp change in
// one angle moves sA by ~4e-16 absolute, which flips the sign test sA < 0 on spherical triangles of
// ~zero area (seen edge-on) and so decides whether such a light survives -- and a survivor's light pdf
// is sum L / weights_sum however small its weight (Mylight.cpp:484-493).  ocml's acos is within 1 ulp
// but differs from glibc's on ~9% of the chain's vertex-angle arguments (tools/literal_check.py);
// glibc's acos is correctly rounded on all but ~2e-4 of them, so a correctly rounded acos on the GPU
// reproduces the reference's angles bit for bit on all but that fraction.
//
// Method: one Newton step on cos(y) = x from the libm result y0, with the residual x - cos(y0)
// evaluated in double-double: x - cos(y0) = (x - 1) + (1 - cos y0), where x - 1 is exact (two_sum)
// and 1 - cos y0 = z (1/2 - z/24 + z^2/720 - ...) with z = y0^2 as a double-double (the first four
// coefficients as double-doubles, the rest in double: their terms are < 1e-5 of the sum).  The series
// runs to z^15 / 30!: at the largest z (x = 0, y0 = pi/2, z = 2.47) the first dropped term z^16 / 32!
// is ~7e-30 absolute (the round-3 form stopped at z^13 / 26!, leaving ~1e-24 = 2^-80 relative there:
// a misrounding chance of ~1e-8 per argument near 0 instead of ~1e-14 now); elsewhere the truncation is
// far smaller and the double-double arithmetic's ~1e-32 dominates.  y = y0 - residual / sin(y0),
// sin(y0) = sqrt((1 - x)(1 + x))
// (on the GPU through v_rsq_f64: the step is ~1 ulp, so its own few-ulp error is irrelevant).
// Negative x: acos(x) = pi - acos(-x) with pi as a double-double.  The last step adds a correction of
// ~1 ulp to y0 in one rounding, so the result is correctly rounded unless the true value lies within
// ~5e-30 relative of a rounding boundary.
//
// Host and device: plain C++ (tools/acos_cr_check.cpp builds it with g++ against mpmath values).
#pragma once
#include <cmath>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace mcpt {

struct DD {
    double h, l;
};
__host__ __device__ inline DD dd_two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return DD{s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline DD dd_fast_sum(double a, double b) {  // |a| >= |b|
    const double s = a + b;
    return DD{s, b - (s - a)};
}
__host__ __device__ inline DD dd_mul(DD a, DD b) {
    const double p = a.h * b.h;
    double e = fma(a.h, b.h, -p);
    e = fma(a.h, b.l, e);
    e = fma(a.l, b.h, e);
    return dd_fast_sum(p, e);
}
__host__ __device__ inline DD dd_add(DD a, DD b) {
    const DD s = dd_two_sum(a.h, b.h);
    return dd_fast_sum(s.h, s.l + (a.l + b.l));
}

// y0 = libm acos(x) and a correction c with acos(x) = y0 + c to <= ~7e-30 absolute, for 0 <= x < 1
__host__ __device__ inline double acos_newton_corr(double x, double y0) {
    const DD z = dd_mul(DD{y0, 0.0}, DD{y0, 0.0});
    // (-1)^k / (2k + 2)!, k = 4..14 in double (Horner in z.h)
    double t = 0x1.3932c5047d60ep-108;
    t = fma(t, z.h, -0x1.0a18a2635085dp-98);
    t = fma(t, z.h, 0x1.88e85fc6a4e5ap-89);
    t = fma(t, z.h, -0x1.f2cf01972f578p-80);
    t = fma(t, z.h, 0x1.0ce396db7f853p-70);
    t = fma(t, z.h, -0x1.e542ba4020225p-62);
    t = fma(t, z.h, 0x1.6827863b97d97p-53);
    t = fma(t, z.h, -0x1.ae7f3e733b81fp-45);
    t = fma(t, z.h, 0x1.93974a8c07c9dp-37);
    t = fma(t, z.h, -0x1.1eed8eff8d898p-29);
    t = fma(t, z.h, 0x1.27e4fb7789f5cp-22);
    // k = 3..0 as double-doubles
    DD p = dd_add(DD{-0x1.a01a01a01a01ap-16, -0x1.a01a01a01a01ap-76}, dd_mul(z, DD{t, 0.0}));
    p = dd_add(DD{0x1.6c16c16c16c17p-10, -0x1.f49f49f49f49fp-65}, dd_mul(z, p));
    p = dd_add(DD{-0x1.5555555555555p-5, -0x1.5555555555555p-59}, dd_mul(z, p));
    p = dd_add(DD{0.5, 0.0}, dd_mul(z, p));
    const DD omc = dd_mul(z, p);                 // 1 - cos(y0)
    const DD xm1 = dd_two_sum(x, -1.0);          // x - 1, exactly
    const double r = (xm1.h + omc.h) + (xm1.l + omc.l);  // x - cos(y0); the first sum is exact (Sterbenz)
    // 1 / sin(y0): the step is ~1 ulp of y0, so ~1e-6 relative accuracy of it is plenty -- the
    // hardware reciprocal square root on the GPU instead of sqrt and a division
    const double s2 = (1.0 - x) * (1.0 + x);
#ifdef __HIP_DEVICE_COMPILE__
    return -r * __builtin_amdgcn_rsq(s2);
#else
    return -r / sqrt(s2);
#endif
}

// Both signs share one libm acos and one correction on |x| (a SIMD wave with lanes of both signs ran
// two of each when the sign picked a branch); the sign selects only the final combination.
__host__ __device__ inline double acos_cr(double x) {
    if (x >= 1.0) return 0.0;
    if (x <= -1.0) return 0x1.921fb54442d18p+1;  // pi rounded, = acos(-1)
    if (!(x == x)) return x;
    const double ax = fabs(x);
    const double y0 = acos(ax);
    const double c = acos_newton_corr(ax, y0);
    // x < 0: (pi_hi - y0) exactly as a two_sum, + pi_lo - c; x >= 0 the same expression with pi and the
    // signs replaced (two_sum(0, y0) = (y0, 0) exactly, so it is y0 + c): one path, no second result live
    const bool neg = x < 0.0;
    const DD d = dd_two_sum(neg ? 0x1.921fb54442d18p+1 : 0.0, neg ? -y0 : y0);
    return d.h + ((d.l + (neg ? 0x1.1a62633145c07p-53 : 0.0)) + (neg ? -c : c));
}

}  // namespace mcpt
