// Exact arithmetic for the H3 route (the near-tie slow path of point -> cell), shared by
// the HIP kernels (device) and the host library.
//
// The reference's cell id comes from H3 v3.7 C code (H3-Java 3.7.0's JNI library,
// reached from H3IndexSystem.pointToIndex, H3IndexSystem.scala:168-170) compiled for
// x86-64: double arithmetic on SSE2, glibc libm for sin/cos/tan/acos/atan2, and five
// expressions on H3's long-double constants (constants.h: M_2PI, M_SQRT7, M_SQRT3_2,
// M_AP7_ROT_RADS, EPSILON) evaluated on the x87 unit in 80-bit extended precision and
// rounded to double on assignment.  This header makes both parts exact on any IEEE
// double machine:
//
//  * x87 extended precision is emulated in integers: a value is (-1)^s * m * 2^e with
//    a 64-bit significand; +, -, *, / are computed exactly in 128-bit integers and
//    rounded to nearest-even at 64 bits (the x87 default precision control on Linux),
//    then again at 53 bits when stored to a double -- the double rounding x87 does.
//    Checked against the host's real `long double` by tests/test_h3_exact_host.py.
//
//  * The libm functions are evaluated in double-double (~2^-100 relative) and rounded
//    once: the correctly rounded result, unless the exact value lies within ~2^-100 of a
//    rounding midpoint (never observed; it would need ~2^47 samples).  glibc 2.35's dbl-64
//    sin/cos/tan/acos/atan2 aim at correct rounding (IBM Accurate Mathematical Library,
//    < 0.55 ulp); tests/test_h3_exact_host.py measures the agreement on the arguments the
//    H3 route produces.
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>

#ifdef __HIPCC__
#define MGPU_XD __host__ __device__ __forceinline__
#else
#define MGPU_XD inline
#endif

namespace mgpu {
namespace exact {

// ------------------------------------------------------------------ x87 extended

typedef unsigned __int128 u128;

struct X80 {
  uint64_t m;  // significand, bit 63 set unless the value is zero
  int e;       // value = (-1)^s * m * 2^e
  int s;
};

// H3 constants.h long-double literals, rounded to 64 bits as gcc does
// (tests/test_h3_exact_host.py compares them with the compiler's own literals)
constexpr X80 kX2Pi = {0xc90fdaa22168c235ULL, -61, 0};          // M_2PI
constexpr X80 kXEpsilon = {0xe69594bec44de15bULL, -117, 0};     // EPSILON 1e-16
constexpr X80 kXSin60 = {0xddb3d742c265539eULL, -64, 0};        // M_SIN60 = M_SQRT3_2
constexpr X80 kXAp7Rot = {0xaabcfee1d47a0aeaULL, -65, 0};       // M_AP7_ROT_RADS
constexpr X80 kXSqrt7 = {0xa953fd4e97c74dbcULL, -62, 0};        // M_SQRT7

MGPU_XD uint64_t dbits(double d) {
  uint64_t b;
  memcpy(&b, &d, 8);
  return b;
}
MGPU_XD double bitsd(uint64_t b) {
  double d;
  memcpy(&d, &b, 8);
  return d;
}

MGPU_XD int clz128(u128 v) {
  const uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
  return hi ? __builtin_clzll(hi) : 64 + __builtin_clzll(lo);
}

MGPU_XD X80 x80_from_double(double d) {
  const uint64_t b = dbits(d);
  X80 x;
  x.s = (int)(b >> 63);
  const int ex = (int)((b >> 52) & 0x7ff);
  uint64_t f = b & 0xfffffffffffffULL;
  if (ex == 0) {
    if (f == 0) {
      x.m = 0;
      x.e = 0;
      return x;
    }
    const int lz = __builtin_clzll(f);
    x.m = f << lz;
    x.e = -1074 - lz;
    return x;
  }
  x.m = (f | (1ULL << 52)) << 11;
  x.e = ex - 1075 - 11;
  return x;
}

// v * 2^e (+ a nonzero tail below bit 0 when `sticky`) rounded to nearest-even at 64 bits
MGPU_XD X80 x80_round(u128 v, int e, bool sticky, int s) {
  X80 x;
  x.s = s;
  if (v == 0) {
    x.m = 0;
    x.e = 0;
    return x;
  }
  const int lz = clz128(v);
  v <<= lz;
  e -= lz;
  uint64_t hi = (uint64_t)(v >> 64);
  const uint64_t lo = (uint64_t)v;
  const bool guard = (lo >> 63) != 0;
  const bool rest = (lo << 1) != 0 || sticky;
  if (guard && (rest || (hi & 1))) {
    ++hi;
    if (hi == 0) {
      hi = 1ULL << 63;
      ++e;
    }
  }
  x.m = hi;
  x.e = e + 64;
  return x;
}

// the store to a double: nearest-even at 53 bits (normal range: the H3 route's values)
MGPU_XD double x80_to_double(X80 x) {
  if (x.m == 0) return x.s ? -0.0 : 0.0;
  uint64_t keep = x.m >> 11;
  const uint64_t rem = x.m & 0x7ff;
  int e = x.e + 11;
  if ((rem > 0x400) || (rem == 0x400 && (keep & 1))) {
    ++keep;
    if (keep == (1ULL << 53)) {
      keep >>= 1;
      ++e;
    }
  }
  // keep in [2^52, 2^53): biased exponent e + 52 + 1023
  const uint64_t be = (uint64_t)(e + 52 + 1023);
  return bitsd(((uint64_t)x.s << 63) | (be << 52) | (keep & 0xfffffffffffffULL));
}

MGPU_XD X80 x80_neg(X80 a) {
  a.s ^= 1;
  return a;
}

// |a| >= |b| (both normalized or zero)
MGPU_XD bool x80_mag_ge(X80 a, X80 b) {
  if (b.m == 0) return true;
  if (a.m == 0) return false;
  return a.e != b.e ? a.e > b.e : a.m >= b.m;
}

MGPU_XD X80 x80_add(X80 a, X80 b) {
  if (a.m == 0) return b;
  if (b.m == 0) return a;
  if (!x80_mag_ge(a, b)) {
    X80 t = a;
    a = b;
    b = t;
  }
  // a's significand at bits 62..125 (two bits of headroom), b aligned below it
  const u128 A = (u128)a.m << 62;
  const int d = a.e - b.e;
  u128 B;
  bool sticky = false;
  if (d >= 126) {
    B = 0;
    sticky = true;
  } else {
    const u128 Bf = (u128)b.m << 62;
    B = Bf >> d;
    sticky = d > 0 && (Bf << (128 - d)) != 0;
  }
  u128 S;
  if (a.s == b.s) {
    S = A + B;
  } else {
    // A - (B + tail): the tail borrows one unit, the remainder stays sticky
    S = A - B - (sticky ? 1 : 0);
  }
  return x80_round(S, a.e - 62, sticky, a.s);
}

MGPU_XD X80 x80_mul(X80 a, X80 b) {
  if (a.m == 0 || b.m == 0) return X80{0, 0, a.s ^ b.s};
  const u128 P = (u128)a.m * (u128)b.m;
  return x80_round(P, a.e + b.e, false, a.s ^ b.s);
}

MGPU_XD X80 x80_div(X80 a, X80 b) {
  if (a.m == 0) return X80{0, 0, a.s ^ b.s};
#if !defined(__HIP_DEVICE_COMPILE__) && defined(__x86_64__)
  {
    // host: the same 67 quotient bits by two native 128-bit divisions (the builder
    // divides by M_SQRT7 once per resolution per cell vertex)
    const u128 num = (u128)a.m << 63;
    const u128 q1 = num / b.m, r1 = num % b.m;
    const u128 n2 = r1 << 3;
    const u128 q = (q1 << 3) | (n2 / b.m);
    return x80_round(q, a.e - b.e - 66, (n2 % b.m) != 0, a.s ^ b.s);
  }
#endif
  // 67 quotient bits of a.m / b.m (1 integer bit + 66 fraction bits) by long division
  u128 rem = a.m;
  u128 q = 0;
  if (rem >= b.m) {
    rem -= b.m;
    q = 1;
  }
  for (int i = 0; i < 66; ++i) {
    rem <<= 1;
    q <<= 1;
    if (rem >= b.m) {
      rem -= b.m;
      q |= 1;
    }
  }
  return x80_round(q, a.e - b.e - 66, rem != 0, a.s ^ b.s);
}

// exact comparisons of a double with an extended value
MGPU_XD int x80_cmp(X80 a, X80 b) {
  if (a.m == 0 && b.m == 0) return 0;
  const int sa = a.m == 0 ? 0 : (a.s ? -1 : 1);
  const int sb = b.m == 0 ? 0 : (b.s ? -1 : 1);
  if (sa != sb) return sa < sb ? -1 : 1;
  const int mag = (a.e != b.e) ? (a.e > b.e ? 1 : -1) : (a.m == b.m ? 0 : (a.m > b.m ? 1 : -1));
  return sa > 0 ? mag : -mag;
}

// (double)((long double)a OP c).  On an x86-64 host `long double` IS the x87 format:
// there the hardware does it (the chip-table builder runs these per cell vertex); the
// device -- and the tests, through the x80_* functions -- use the emulation.
#if !defined(__HIP_DEVICE_COMPILE__) && defined(__x86_64__) && (__LDBL_MANT_DIG__ == 64)
#define MGPU_NATIVE_X87 1
inline long double x80_ld(X80 c) {
  const long double v = __builtin_ldexpl((long double)c.m, c.e);
  return c.s ? -v : v;
}
inline double ld_add(double a, X80 c) { return (double)((long double)a + x80_ld(c)); }
inline double ld_sub(double a, X80 c) { return (double)((long double)a - x80_ld(c)); }
inline double ld_mul(double a, X80 c) { return (double)((long double)a * x80_ld(c)); }
inline double ld_div(double a, X80 c) { return (double)((long double)a / x80_ld(c)); }
inline bool ld_lt(double a, X80 c) { return (long double)a < x80_ld(c); }
inline bool ld_ge(double a, X80 c) { return (long double)a >= x80_ld(c); }
#else
MGPU_XD double ld_add(double a, X80 c) { return x80_to_double(x80_add(x80_from_double(a), c)); }
MGPU_XD double ld_sub(double a, X80 c) { return x80_to_double(x80_add(x80_from_double(a), x80_neg(c))); }
MGPU_XD double ld_mul(double a, X80 c) { return x80_to_double(x80_mul(x80_from_double(a), c)); }
MGPU_XD double ld_div(double a, X80 c) { return x80_to_double(x80_div(x80_from_double(a), c)); }
MGPU_XD bool ld_lt(double a, X80 c) { return x80_cmp(x80_from_double(a), c) < 0; }
MGPU_XD bool ld_ge(double a, X80 c) { return x80_cmp(x80_from_double(a), c) >= 0; }
#endif

// ------------------------------------------------------------------ double-double

struct DD {
  double hi, lo;
};

MGPU_XD DD two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return DD{s, (a - (s - bb)) + (b - bb)};
}
MGPU_XD DD quick_two_sum(double a, double b) {
  const double s = a + b;
  return DD{s, b - (s - a)};
}
MGPU_XD DD two_prod(double a, double b) {
  const double p = a * b;
  return DD{p, fma(a, b, -p)};
}
MGPU_XD DD dd_neg(DD a) { return DD{-a.hi, -a.lo}; }
// accurate addition (relative error ~3 * 2^-106 of the sum)
MGPU_XD DD dd_add(DD a, DD b) {
  DD s = two_sum(a.hi, b.hi);
  const DD t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = quick_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return quick_two_sum(s.hi, s.lo);
}
MGPU_XD DD dd_sub(DD a, DD b) { return dd_add(a, dd_neg(b)); }
MGPU_XD DD dd_mul(DD a, DD b) {
  DD p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return quick_two_sum(p.hi, p.lo);
}
MGPU_XD DD dd_mul_d(DD a, double b) {
  DD p = two_prod(a.hi, b);
  p.lo += a.lo * b;
  return quick_two_sum(p.hi, p.lo);
}
MGPU_XD DD dd_div(DD a, DD b) {
  const double q1 = a.hi / b.hi;
  DD r = dd_sub(a, dd_mul_d(b, q1));
  const double q2 = r.hi / b.hi;
  r = dd_sub(r, dd_mul_d(b, q2));
  const double q3 = r.hi / b.hi;
  return dd_add(quick_two_sum(q1, q2), DD{q3, 0.0});
}
MGPU_XD DD dd_sqrt(DD a) {
  if (!(a.hi > 0.0)) return DD{0.0, 0.0};
  const double s = sqrt(a.hi);
  const DD e = dd_sub(a, two_prod(s, s));
  return quick_two_sum(s, e.hi / (2.0 * s));
}

// pi/2 as three doubles (163 bits), pi and pi/2 as double-double
constexpr double kPio2_1 = 0x1.921fb54442d18p+0;
constexpr double kPio2_2 = 0x1.1a62633145c07p-54;
constexpr double kPio2_3 = -0x1.f1976b7ed8fbcp-110;
constexpr double kPi_1 = 0x1.921fb54442d18p+1;
constexpr double kPi_2 = 0x1.1a62633145c07p-53;

// 1/n! as double-double, n = 0..29 (generated with exact rationals)
#define MGPU_INVF_TABLE                                                                    \
  {{1.0, 0.0},                                                                             \
   {1.0, 0.0},                                                                             \
   {0x1.0000000000000p-1, 0.0},                                                            \
   {0x1.5555555555555p-3, 0x1.5555555555555p-57},                                          \
   {0x1.5555555555555p-5, 0x1.5555555555555p-59},                                          \
   {0x1.1111111111111p-7, 0x1.1111111111111p-63},                                          \
   {0x1.6c16c16c16c17p-10, -0x1.f49f49f49f49fp-65},                                        \
   {0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-73},                                         \
   {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},                                         \
   {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},                                        \
   {0x1.27e4fb7789f5cp-22, 0x1.cbbc05b4fa99ap-76},                                         \
   {0x1.ae64567f544e4p-26, -0x1.c062e06d1f209p-80},                                        \
   {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83},                                        \
   {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},                                         \
   {0x1.93974a8c07c9dp-37, 0x1.05d6f8a2efd1fp-92},                                         \
   {0x1.ae7f3e733b81fp-41, 0x1.1d8656b0ee8cbp-97},                                         \
   {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101},                                        \
   {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103},                                        \
   {0x1.6827863b97d97p-53, 0x1.eec01221a8b0bp-107},                                        \
   {0x1.2f49b46814157p-57, 0x1.2650f61dbdcb4p-112},                                        \
   {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120},                                        \
   {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120},                                       \
   {0x1.0ce396db7f853p-70, -0x1.aebcdbd20331cp-124},                                       \
   {0x1.761b41316381ap-75, -0x1.3423c7d91404fp-130},                                       \
   {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135},                                       \
   {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139},                                       \
   {0x1.88e85fc6a4e5ap-89, -0x1.71c37ebd16540p-143},                                       \
   {0x1.d1ab1c2dccea3p-94, 0x1.054d0c78aea14p-149},                                        \
   {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153},                                        \
   {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157}}

#ifndef H3T_QUAL
#define H3T_QUAL static const
#endif
H3T_QUAL double kInvFact[30][2] = MGPU_INVF_TABLE;
MGPU_XD DD inv_fact(int n) { return DD{kInvFact[n][0], kInvFact[n][1]}; }

// sin and cos of a double-double |x| <= ~8: x = k pi/2 + r, Taylor series of r to r^29
MGPU_XD void dd_sincos(DD x, DD* s, DD* c) {
  const double kf = rint(x.hi * 0.63661977236758134308);
  DD r = dd_sub(x, two_prod(kf, kPio2_1));
  r = dd_sub(r, two_prod(kf, kPio2_2));
  r = dd_sub(r, DD{kf * kPio2_3, 0.0});
  const DD r2 = dd_mul(r, r);
  // sin r = r (1 - r^2/3! + r^4/5! - ... + r^28/29!)
  DD ps = inv_fact(29);
  for (int n = 27; n >= 3; n -= 2) {
    const DD f = inv_fact(n);
    ps = dd_add(dd_mul(ps, r2), ((n - 1) / 2) & 1 ? dd_neg(f) : f);
  }
  ps = dd_add(dd_mul(ps, r2), DD{1.0, 0.0});
  const DD sr = dd_mul(ps, r);
  // cos r = 1 - r^2/2! + ... + r^28/28!
  DD pc = inv_fact(28);
  for (int n = 26; n >= 2; n -= 2) {
    const DD f = inv_fact(n);
    pc = dd_add(dd_mul(pc, r2), (n / 2) & 1 ? dd_neg(f) : f);
  }
  const DD cr = dd_add(dd_mul(pc, r2), DD{1.0, 0.0});
  const int q = ((int)kf) & 3;
  const DD ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
  *s = (q & 2) ? dd_neg(ss) : ss;
  *c = ((q + 1) & 2) ? dd_neg(cc) : cc;
}

// asin of a double-double |s| <= 0.75: two Newton steps on sin from the libm value
MGPU_XD DD dd_asin_small(DD s) {
  DD phi{asin(s.hi), 0.0};
  for (int it = 0; it < 2; ++it) {
    DD sp, cp;
    dd_sincos(phi, &sp, &cp);
    phi = dd_sub(phi, dd_div(dd_sub(sp, s), cp));
  }
  return phi;
}

// correctly rounded libm (see the header comment)
MGPU_XD void cr_sincos(double a, double* s, double* c) {
  if (!isfinite(a)) {
    *s = *c = a - a;
    return;
  }
  DD ds, dc;
  dd_sincos(DD{a, 0.0}, &ds, &dc);
  *s = ds.hi;
  *c = dc.hi;
}
MGPU_XD double cr_sin(double a) {
  double s, c;
  cr_sincos(a, &s, &c);
  return s;
}
MGPU_XD double cr_cos(double a) {
  double s, c;
  cr_sincos(a, &s, &c);
  return c;
}
MGPU_XD double cr_tan(double a) {
  if (!isfinite(a)) return a - a;
  DD s, c;
  dd_sincos(DD{a, 0.0}, &s, &c);
  return dd_div(s, c).hi;
}
MGPU_XD double cr_acos(double a) {
  if (!(a >= -1.0 && a <= 1.0)) return (a - a) / (a - a);
  if (a >= 0.5) {
    const double d = (1.0 - a) * 0.5;  // exact (Sterbenz)
    if (d == 0.0) return 0.0;
    const DD h = dd_asin_small(dd_sqrt(DD{d, 0.0}));
    return quick_two_sum(2.0 * h.hi, 2.0 * h.lo).hi;
  }
  if (a <= -0.5) {
    const double d = (1.0 + a) * 0.5;
    const DD h = dd_asin_small(dd_sqrt(DD{d, 0.0}));
    return dd_sub(DD{kPi_1, kPi_2}, DD{2.0 * h.hi, 2.0 * h.lo}).hi;
  }
  return dd_sub(DD{kPio2_1, kPio2_2}, dd_asin_small(DD{a, 0.0})).hi;
}
MGPU_XD double cr_atan2(double y, double x) {
  const double t0 = atan2(y, x);
  if (!isfinite(x) || !isfinite(y) || (x == 0.0 && y == 0.0) || t0 == 0.0) return t0;
  // Newton on f(t) = x sin t - y cos t (f' = x cos t + y sin t = hypot(x, y) near the root)
  DD t{t0, 0.0};
  for (int it = 0; it < 2; ++it) {
    DD s, c;
    dd_sincos(t, &s, &c);
    const DD f = dd_sub(dd_mul_d(s, x), dd_mul_d(c, y));
    const double fp = x * c.hi + y * s.hi;
    t = dd_sub(t, DD{f.hi / fp, 0.0});
  }
  return t.hi;
}

}  // namespace exact
}  // namespace mgpu
