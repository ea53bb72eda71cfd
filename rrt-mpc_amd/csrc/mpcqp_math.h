// mpcqp_math.h -- the planner's elementary functions, made to agree with the host bit for bit.
//
// RRT* decisions sit on knife edges: the first segment check of every iteration tests a segment
// whose length is the step (3 px) up to an ulp, and the number of np.linspace samples is
// ceil(length / 0.75) -- 4 or 5 depending on that last ulp.  The device library's hypot / atan2 /
// cos / sin differ from the host's in the last ulp for 3-27 % of arguments, which grew a different
// tree for ~1 % of plans.  So:
//   py_hypot   math.hypot as CPython computes it (Modules/mathmodule.c vector_norm, 3.10: the
//              coordinates scaled by a power of two, split 26/27 bits, squares summed with
//              compensation, a square root and one correction step) -- the same operations in the
//              same order, uncontracted, so the result equals CPython's bit for bit;
//   cr_atan2, cr_sincos
//              the correctly rounded values: double-double series (|r| <= pi/4 after a
//              triple-double pi/2 reduction) and one Newton step on the device's atan2 in
//              double-double, rounded once (cr_steer: the angle and its cos / sin).  glibc's are within ~0.55 ulp, so they agree with these
//              on ~99.87 % of arguments; oracle/rrt_oracle.py (CR_TRIG) evaluates the same correctly
//              rounded functions exactly, which is what the parity tests hold the device to.
// All device functions; one thread calls them per RRT* iteration.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>

namespace mpcqp_math {

// ---------------------------------------------------------------- CPython's math.hypot (2 args)
__device__ inline double hypot_scaled(double a, double b, double mx) {
#pragma clang fp contract(off)
  constexpr double T27 = 134217729.0;  // 2^27 + 1
  int max_e;
  frexp(mx, &max_e);
  const double scale = ldexp(1.0, -max_e);
  double csum = 1.0, frac1 = 0.0, frac2 = 0.0, frac3 = 0.0;
  const double v[2] = {a, b};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    double x = v[i] * scale;
    double t = x * T27;
    double hi = t - (t - x);
    double lo = x - hi;
    x = hi * hi;
    double old = csum;
    csum += x;
    frac1 += (old - csum) + x;
    x = 2.0 * hi * lo;
    old = csum;
    csum += x;
    frac2 += (old - csum) + x;
    frac3 += lo * lo;
  }
  const double h = sqrt(csum - 1.0 + (frac1 + frac2 + frac3));
  double x = h;
  double t = x * T27;
  const double hi = t - (t - x);
  const double lo = x - hi;
  x = -hi * hi;
  double old = csum;
  csum += x;
  frac1 += (old - csum) + x;
  x = -2.0 * hi * lo;
  old = csum;
  csum += x;
  frac2 += (old - csum) + x;
  x = -lo * lo;
  old = csum;
  csum += x;
  frac3 += (old - csum) + x;
  x = csum - 1.0 + (frac1 + frac2 + frac3);
  return (h + x / (2.0 * h)) / scale;  // scale is a power of two
}

__device__ inline double py_hypot(double dx, double dy) {
  const double a = fabs(dx), b = fabs(dy);
  if (isinf(a) || isinf(b)) return INFINITY;
  if (isnan(a) || isnan(b)) return NAN;
  const double mx = fmax(a, b);
  if (mx == 0.0) return mx;
  int max_e;
  frexp(mx, &max_e);
  if (max_e >= -1023) return hypot_scaled(a, b, mx);
  // subnormal maximum: lossless scaling back to normals first (CPython does the same)
  return DBL_MIN * hypot_scaled(a / DBL_MIN, b / DBL_MIN, mx / DBL_MIN);
}

// ---------------------------------------------------------------- double-double arithmetic
struct dd {
  double hi, lo;
};

__device__ inline dd two_sum(double a, double b) {
#pragma clang fp contract(off)
  const double s = a + b;
  const double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
__device__ inline dd fast_two_sum(double a, double b) {  // |a| >= |b|
#pragma clang fp contract(off)
  const double s = a + b;
  return {s, b - (s - a)};
}
__device__ inline dd two_prod(double a, double b) {
  const double p = a * b;
  return {p, fma(a, b, -p)};
}
__device__ inline dd dd_add(dd a, dd b) {
#pragma clang fp contract(off)
  dd s = two_sum(a.hi, b.hi);
  const dd t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return fast_two_sum(s.hi, s.lo);
}
__device__ inline dd dd_neg(dd a) { return {-a.hi, -a.lo}; }
__device__ inline dd dd_mul(dd a, dd b) {
#pragma clang fp contract(off)
  dd p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return fast_two_sum(p.hi, p.lo);
}
__device__ inline dd dd_mul_d(dd a, double b) {
#pragma clang fp contract(off)
  dd p = two_prod(a.hi, b);
  p.lo += a.lo * b;
  return fast_two_sum(p.hi, p.lo);
}
__device__ inline dd dd_div_d(dd a, double d) {
#pragma clang fp contract(off)
  const double q1 = a.hi / d;
  const dd p = two_prod(q1, d);
  const double r = ((a.hi - p.hi) - p.lo) + a.lo;
  return fast_two_sum(q1, r / d);
}

// pi/2 as a triple double (159 bits)
constexpr double kPio2A = 0x1.921fb54442d18p+0;
constexpr double kPio2B = 0x1.1a62633145c07p-54;
constexpr double kPio2C = -0x1.f1976b7ed8fbcp-110;

// sin r / cos r Taylor coefficients (-1)^j / (2j+1)! and (-1)^j / (2j)!: j = 1..7 as double-doubles,
// j = 8..14 as doubles (those terms are below 2^-48 of the sum for |r| <= pi/4)
__device__ constexpr double kSinHi[7] = {-0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13,
                                         0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33,
                                         -0x1.ae7f3e733b81fp-41};
__device__ constexpr double kSinLo[7] = {-0x1.5555555555555p-57, 0x1.1111111111111p-63, -0x1.a01a01a01a01ap-73,
                                         -0x1.c154f8ddc6c00p-73, 0x1.c062e06d1f209p-80, 0x1.f28e0cc748ebep-87,
                                         -0x1.1d8656b0ee8cbp-97};
__device__ constexpr double kSinTail[7] = {0x1.952c77030ad4ap-49, -0x1.2f49b46814157p-57, 0x1.71b8ef6dcf572p-66,
                                           -0x1.761b41316381ap-75, 0x1.3f3ccdd165fa9p-84, -0x1.d1ab1c2dccea3p-94,
                                           0x1.259f98b4358adp-103};
__device__ constexpr double kCosHi[7] = {-0x1.0000000000000p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10,
                                         0x1.a01a01a01a01ap-16, -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29,
                                         -0x1.93974a8c07c9dp-37};
__device__ constexpr double kCosLo[7] = {0.0, 0x1.5555555555555p-59, 0x1.f49f49f49f49fp-65, 0x1.a01a01a01a01ap-76,
                                         -0x1.cbbc05b4fa99ap-76, -0x1.2aec959e14c06p-83, -0x1.05d6f8a2efd1fp-92};
__device__ constexpr double kCosTail[7] = {0x1.ae7f3e733b81fp-45, -0x1.6827863b97d97p-53, 0x1.e542ba4020225p-62,
                                           -0x1.0ce396db7f853p-70, 0x1.f2cf01972f578p-80, -0x1.88e85fc6a4e5ap-89,
                                           0x1.0a18a2635085dp-98};

// sum_{j>=1} a_j r2^j: the tail in double, then Horner in double-double
__device__ inline dd dd_series(dd r2, const double* hi, const double* lo, const double* tail) {
  double t = tail[6];
#pragma unroll
  for (int j = 5; j >= 0; --j) t = fma(t, r2.hi, tail[j]);
  dd acc{t, 0.0};
#pragma unroll
  for (int j = 6; j >= 0; --j) acc = dd_add(dd_mul(acc, r2), dd{hi[j], lo[j]});
  return dd_mul(acc, r2);
}

// sin and cos of a double t in double-double (relative error ~2^-100 away from multiples of pi/2)
__device__ inline void dd_sincos(double t, dd& s_out, dd& c_out) {
#pragma clang fp contract(off)
  const double k = rint(t * 0x1.45f306dc9c883p-1);  // 2/pi
  // r = t - k pi/2: k A and k B are exact as double-double products
  dd r{t, 0.0};
  r = dd_add(r, dd_neg(two_prod(k, kPio2A)));
  r = dd_add(r, dd_neg(two_prod(k, kPio2B)));
  r = dd_add(r, dd{-k * kPio2C, 0.0});
  const dd r2 = dd_mul(r, r);
  const dd S = dd_add(r, dd_mul(r, dd_series(r2, kSinHi, kSinLo, kSinTail)));
  const dd C = dd_add(dd{1.0, 0.0}, dd_series(r2, kCosHi, kCosLo, kCosTail));
  const int q = ((int)fmod(k, 4.0) + 4) & 3;
  switch (q) {
    case 0: s_out = S; c_out = C; break;
    case 1: s_out = C; c_out = dd_neg(S); break;
    case 2: s_out = dd_neg(S); c_out = dd_neg(C); break;
    default: s_out = dd_neg(C); c_out = S; break;
  }
}

// correctly rounded sin / cos of t (one rounding of the double-double)
__device__ inline void cr_sincos(double t, double& s, double& c) {
  if (!isfinite(t)) {
    s = c = NAN;
    return;
  }
  if (t == 0.0) {
    s = t;
    c = 1.0;
    return;
  }
  dd S, C;
  dd_sincos(t, S, C);
  s = S.hi + S.lo;
  c = C.hi + C.lo;
}

// correctly rounded atan2(y, x): one Newton step from the device's atan2 on
// f(th) = x sin th - y cos th, in double-double.  t0 and its double-double sin / cos are handed
// back (the steer reuses them when the rounded angle is t0).
__device__ inline double cr_atan2_sc(double y, double x, double& t0, dd& S, dd& C) {
#pragma clang fp contract(off)
  t0 = atan2(y, x);
  if (!isfinite(x) || !isfinite(y) || x == 0.0 || y == 0.0) {  // exact special values
    const double th = t0;
    t0 = NAN;  // no sin / cos handed back
    S = C = dd{0.0, 0.0};
    return th;
  }
  dd_sincos(t0, S, C);
  const dd num = dd_add(dd_mul_d(S, x), dd_neg(dd_mul_d(C, y)));
  const double den = x * C.hi + y * S.hi;
  const double delta = (num.hi + num.lo) / den;
  const dd t1 = two_sum(t0, -delta);
  return t1.hi + t1.lo;
}

__device__ inline double cr_atan2(double y, double x) {
  double t0;
  dd S, C;
  return cr_atan2_sc(y, x, t0, S, C);
}

// RRTStarPlanner._steer's angle and its cos / sin, all three correctly rounded
__device__ inline void cr_steer(double dy, double dx, double& th, double& c, double& s) {
  double t0;
  dd S, C;
  th = cr_atan2_sc(dy, dx, t0, S, C);
  if (th == t0) {
    s = S.hi + S.lo;
    c = C.hi + C.lo;
  } else {
    cr_sincos(th, s, c);
  }
}

}  // namespace mpcqp_math
