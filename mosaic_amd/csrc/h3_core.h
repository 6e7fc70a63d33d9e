// H3 v3.7 point -> cell (geoToH3) for the MI355X path, shared by the HIP kernels
// (device) and the chip-table builder (host).
//
// Replaces: H3IndexSystem.pointToIndex -> H3Core.geoToH3(lat, lon, res)
//   /root/reference/src/main/scala/com/databricks/labs/mosaic/core/index/H3IndexSystem.scala:168-170
// H3 (com.uber:h3:3.7.0, pom.xml:91-97) is not vendored in the reference; the
// published v3.7 algorithm is restated: nearest icosahedron face by squared chord
// distance -> gnomonic projection into that face's hex2d plane -> hex rounding ->
// aperture-7 digit extraction from res down to 0 -> base cell lookup + rotations.
//
// Numerics.  The H3 route (route_face_ijk, the reference formulation) is exact to the
// JVM path's native H3 by construction: IEEE double with FMA contraction disabled (the
// library is compiled with -ffp-contract=off) for every + - * /, H3's five x87
// long-double expressions emulated bit for bit, and correctly rounded
// sin/cos/tan/acos/atan2 (h3_exact.h).  The fast path (fast_hex2d) is an
// approximation trusted only outside a tie band: every point whose hex2d coordinates
// fall near a decision threshold (`margin` below: distance to the nearest threshold,
// in hex units, relative to the coordinate magnitude) is a near-tie and takes the route.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define MGPU_HD __host__ __device__ __forceinline__
#else
#define MGPU_HD inline
#endif

#include <math.h>

#ifndef H3T_QUAL
#define H3T_QUAL static const
#endif
#include "h3_tables.inc"
#include "h3_exact.h"

namespace mgpu {
namespace h3 {

constexpr double kTwoPi = 6.28318530717958647692528676655900576839433;
constexpr double kEpsilon = 1e-16;
constexpr double kSin60 = 0.8660254037844386467637231707529361834714;
constexpr double kAp7Rot = 0.333473172251832115336090755351601070065900389;
constexpr double kRes0UGnomonic = 0.38196601125010500003;
constexpr double kSqrt7 = 2.6457513110645905905016157536392604257102;
constexpr int kMaxRes = 15;
constexpr uint64_t kInit = 35184372088831ULL;  // H3_INIT: all 15 digits = 7
constexpr int kMaxFaceCoord = 2;
// near-tie threshold: decision margins below kTieRel * |hex2d coordinate| are
// reported (the fast path's error is ~1e-15 relative, this is 2^-40 ~ 9e-13)
constexpr double kTieRel = 9.094947017729282e-13;

struct IJK {
  int i, j, k;
};

// libm entry points of the H3 route.  On the device each is its own out-of-line
// function: the route runs for ~1 point in 1e6, and inlining ocml's polynomials
// into it made the route -- and with it every kernel that calls it -- allocate 120
// VGPRs.
#ifdef __HIP_DEVICE_COMPILE__
#define MGPU_LIBM static __device__ __attribute__((noinline))
#else
#define MGPU_LIBM static inline
#endif
// other pieces of the route, out of line on the device for the same reason
#ifdef __HIP_DEVICE_COMPILE__
#define MGPU_COLD_FN static __host__ __device__ __attribute__((noinline))
#else
#define MGPU_COLD_FN static inline
#endif
// correctly rounded (h3_exact.h), the same on the host and the device
MGPU_LIBM void lm_sincos(double a, double* s, double* c) { exact::cr_sincos(a, s, c); }
MGPU_LIBM double lm_acos(double a) { return exact::cr_acos(a); }
MGPU_LIBM double lm_atan2(double y, double x) { return exact::cr_atan2(y, x); }
MGPU_LIBM double lm_tan(double a) { return exact::cr_tan(a); }
MGPU_LIBM double lm_sin(double a) { return exact::cr_sin(a); }
MGPU_LIBM double lm_cos(double a) { return exact::cr_cos(a); }

// _posAngleRads: `rads + M_2PI` and `tmp -= M_2PI` are x87 long-double expressions
MGPU_HD double pos_angle(double rads) {
  double tmp = (rads < 0.0) ? exact::ld_add(rads, exact::kX2Pi) : rads;
  if (exact::ld_ge(rads, exact::kX2Pi)) tmp = exact::ld_sub(tmp, exact::kX2Pi);
  return tmp;
}

MGPU_HD void ijk_normalize(IJK& c) {
  if (c.i < 0) { c.j -= c.i; c.k -= c.i; c.i = 0; }
  if (c.j < 0) { c.i -= c.j; c.k -= c.j; c.j = 0; }
  if (c.k < 0) { c.i -= c.k; c.j -= c.k; c.k = 0; }
  int m = c.i;
  if (c.j < m) m = c.j;
  if (c.k < m) m = c.k;
  if (m > 0) { c.i -= m; c.j -= m; c.k -= m; }
}

MGPU_HD double dmin(double a, double b) { return a < b ? a : b; }

// _hex2dToCoordIJK; *margin receives the smallest distance between a quantity and
// the threshold it was compared against (fractional parts, integer truncation,
// the quadrant folds).
MGPU_COLD_FN IJK hex2d_to_ijk(double vx, double vy, double* margin) {
  IJK h;
  h.k = 0;
  double a1 = fabs(vx), a2 = fabs(vy);
  double x2 = exact::ld_div(a2, exact::kXSin60);  // a2 / M_SIN60 in long double
  double x1 = a1 + x2 / 2.0;
  int m1 = (int)x1, m2 = (int)x2;
  double r1 = x1 - m1, r2 = x2 - m2;
  double mg = dmin(dmin(r1, 1.0 - r1), dmin(r2, 1.0 - r2));
  if (r1 < 0.5) {
    if (r1 < 1.0 / 3.0) {
      mg = dmin(mg, dmin(fabs(r1 - 0.5), fabs(r1 - 1.0 / 3.0)));
      double t = (1.0 + r1) / 2.0;
      mg = dmin(mg, fabs(r2 - t));
      if (r2 < t) { h.i = m1; h.j = m2; } else { h.i = m1; h.j = m2 + 1; }
    } else {
      mg = dmin(mg, dmin(fabs(r1 - 0.5), fabs(r1 - 1.0 / 3.0)));
      double t = 1.0 - r1, u = 2.0 * r1;
      mg = dmin(mg, dmin(fabs(r2 - t), fabs(r2 - u)));
      h.j = (r2 < t) ? m2 : m2 + 1;
      h.i = ((t <= r2) && (r2 < u)) ? m1 + 1 : m1;
    }
  } else {
    if (r1 < 2.0 / 3.0) {
      mg = dmin(mg, dmin(fabs(r1 - 0.5), fabs(r1 - 2.0 / 3.0)));
      double t = 1.0 - r1, u = 2.0 * r1 - 1.0;
      mg = dmin(mg, dmin(fabs(r2 - t), fabs(r2 - u)));
      h.j = (r2 < t) ? m2 : m2 + 1;
      h.i = ((u < r2) && (r2 < t)) ? m1 : m1 + 1;
    } else {
      mg = dmin(mg, fabs(r1 - 2.0 / 3.0));
      double t = r1 / 2.0;
      mg = dmin(mg, fabs(r2 - t));
      h.i = m1 + 1;
      h.j = (r2 < t) ? m2 : m2 + 1;
    }
  }
  if (vx < 0.0) {
    if ((h.j % 2) == 0) {
      long long axisi = h.j / 2;
      long long diff = h.i - axisi;
      h.i = (int)(h.i - 2.0 * diff);
    } else {
      long long axisi = (h.j + 1) / 2;
      long long diff = h.i - axisi;
      h.i = (int)(h.i - (2.0 * diff + 1));
    }
  }
  if (vy < 0.0) {
    h.i = h.i - (2 * h.j + 1) / 2;
    h.j = -1 * h.j;
  }
  ijk_normalize(h);
  mg = dmin(mg, dmin(a1, a2));  // quadrant folds on the signs of vx, vy
  *margin = mg;
  return h;
}

// _geoToHex2d (via _geoToClosestFace).  *face_gap = second-smallest minus
// smallest squared chord distance (face-choice margin).
MGPU_COLD_FN void geo_to_hex2d(double lat, double lon, int res, int* face, double* vx, double* vy, double* face_gap) {
  double slat, clat, slon, clon;
  lm_sincos(lat, &slat, &clat);
  lm_sincos(lon, &slon, &clon);
  double x = clon * clat, y = slon * clat, z = slat;
  int f0 = 0;
  double best = 5.0, second = 5.0;
  for (int f = 0; f < H3T_NUM_FACES; ++f) {
    double dx = H3T_FACE_CENTER_POINT[f][0] - x;
    double dy = H3T_FACE_CENTER_POINT[f][1] - y;
    double dz = H3T_FACE_CENTER_POINT[f][2] - z;
    double s = dx * dx + dy * dy + dz * dz;
    if (s < best) {
      second = best;
      best = s;
      f0 = f;
    } else if (s < second) {
      second = s;
    }
  }
  *face = f0;
  *face_gap = second - best;
  double r = lm_acos(1 - best / 2);
  if (exact::ld_lt(r, exact::kXEpsilon)) {
    *vx = *vy = 0.0;
    return;
  }
  // _geoAzimuthRads(faceCenterGeo[face], g)
  double flat = H3T_FACE_CENTER_GEO[f0][0], flon = H3T_FACE_CENTER_GEO[f0][1];
  double sdl, cdl;
  lm_sincos(lon - flon, &sdl, &cdl);
  double az = lm_atan2(clat * sdl, lm_cos(flat) * slat - lm_sin(flat) * clat * cdl);
  double theta = pos_angle(H3T_FACE_AXES_AZ_CII[f0][0] - pos_angle(az));
  if (res % 2) theta = pos_angle(exact::ld_sub(theta, exact::kXAp7Rot));
  r = lm_tan(r);
  r /= kRes0UGnomonic;
  for (int i = 0; i < res; i++) r = exact::ld_mul(r, exact::kXSqrt7);
  double st, ct;
  lm_sincos(theta, &st, &ct);
  *vx = r * ct;
  *vy = r * st;
}

// lround(n / 7.0) done in integers (n / 7 is never a tie)
MGPU_HD int round_div7(int n) {
  return n >= 0 ? (2 * n + 7) / 14 : -((-2 * n + 7) / 14);
}

MGPU_HD void up_ap7(IJK& c) {
  int i = c.i - c.k, j = c.j - c.k;
  c.i = round_div7(3 * i - j);
  c.j = round_div7(i + 2 * j);
  c.k = 0;
  ijk_normalize(c);
}
MGPU_HD void up_ap7r(IJK& c) {
  int i = c.i - c.k, j = c.j - c.k;
  c.i = round_div7(2 * i + j);
  c.j = round_div7(3 * j - i);
  c.k = 0;
  ijk_normalize(c);
}
MGPU_HD void down_ap7(IJK& c) {
  int i = c.i, j = c.j, k = c.k;
  c.i = 3 * i + j;
  c.j = 3 * j + k;
  c.k = i + 3 * k;
  ijk_normalize(c);
}
MGPU_HD void down_ap7r(IJK& c) {
  int i = c.i, j = c.j, k = c.k;
  c.i = 3 * i + k;
  c.j = i + 3 * j;
  c.k = j + 3 * k;
  ijk_normalize(c);
}

// ccw 60-degree digit rotation: K1->IK5->I4->IJ6->J2->JK3->K1 (table in a u32)
MGPU_HD int rot60ccw(int d) { return (int)((0x72461350u >> (4 * d)) & 0xF); }
// cw: 1->3, 3->2, 2->6, 6->4, 4->5, 5->1
MGPU_HD int rot60cw(int d) { return (int)((0x74152630u >> (4 * d)) & 0xF); }

MGPU_HD int digit_at(uint64_t h, int r) { return (int)((h >> ((kMaxRes - r) * 3)) & 7); }
MGPU_HD uint64_t with_digit(uint64_t h, int r, int d) {
  int s = (kMaxRes - r) * 3;
  return (h & ~(7ULL << s)) | ((uint64_t)d << s);
}
// (no exit inside the loop: an early return here gave wrong per-lane results in waves
// whose lanes took different paths, h3_ring.h)
MGPU_HD int leading_nonzero(uint64_t h, int res) {
  int lead = 0;
  for (int r = kMaxRes; r >= 1; r--) {
    const int d = digit_at(h, r);
    lead = (r <= res && d != 0) ? d : lead;
  }
  return lead;
}
MGPU_HD uint64_t rotate_ccw(uint64_t h, int res) {
  for (int r = 1; r <= res; r++) h = with_digit(h, r, rot60ccw(digit_at(h, r)));
  return h;
}
MGPU_HD uint64_t rotate_cw(uint64_t h, int res) {
  for (int r = 1; r <= res; r++) h = with_digit(h, r, rot60cw(digit_at(h, r)));
  return h;
}
MGPU_HD uint64_t rotate_pent_ccw(uint64_t h, int res) {
  bool found = false;
  for (int r = 1; r <= res; r++) {
    h = with_digit(h, r, rot60ccw(digit_at(h, r)));
    if (!found && digit_at(h, r) != 0) {
      found = true;
      if (leading_nonzero(h, res) == 1) h = rotate_ccw(h, res);
    }
  }
  return h;
}

// _faceIjkToH3
MGPU_HD uint64_t face_ijk_to_h3(int face, IJK ijk, int res) {
  uint64_t h = kInit | (1ULL << 59) | ((uint64_t)res << 52);
  if (res == 0) {
    if (ijk.i > kMaxFaceCoord || ijk.j > kMaxFaceCoord || ijk.k > kMaxFaceCoord) return 0;
    int bc = H3T_FACE_IJK_BASE_CELLS[face][ijk.i][ijk.j][ijk.k] & 0xff;
    return h | ((uint64_t)bc << 45);
  }
  for (int r = res - 1; r >= 0; r--) {
    IJK last = ijk, center;
    if ((r + 1) & 1) {
      up_ap7(ijk);
      center = ijk;
      down_ap7(center);
    } else {
      up_ap7r(ijk);
      center = ijk;
      down_ap7r(center);
    }
    IJK d = {last.i - center.i, last.j - center.j, last.k - center.k};
    ijk_normalize(d);
    int digit = (d.i <= 1 && d.j <= 1 && d.k <= 1) ? (d.i * 4 + d.j * 2 + d.k) : 7;
    h = with_digit(h, r + 1, digit);
  }
  if (ijk.i > kMaxFaceCoord || ijk.j > kMaxFaceCoord || ijk.k > kMaxFaceCoord) return 0;
  unsigned e = H3T_FACE_IJK_BASE_CELLS[face][ijk.i][ijk.j][ijk.k];
  int bc = (int)(e & 0xff), rots = (int)(e >> 8);
  h |= (uint64_t)bc << 45;
  if (H3T_BASE_CELL_DATA[bc][4]) {
    if (leading_nonzero(h, res) == 1) {
      if (H3T_BASE_CELL_DATA[bc][5] == face || H3T_BASE_CELL_DATA[bc][6] == face)
        h = rotate_cw(h, res);
      else
        h = rotate_ccw(h, res);
    }
    for (int i = 0; i < rots; i++) h = rotate_pent_ccw(h, res);
  } else {
    for (int i = 0; i < rots; i++) h = rotate_ccw(h, res);
  }
  return h;
}

// _faceIjkToH3, restated for throughput (bit-identical to face_ijk_to_h3; checked by
// tests/test_h3_digits_host.py on every base cell and resolution):
//  * the walk from `res` to 0 runs in axial coordinates (a, b) = (i - k, j - k), where
//    up_ap7 / down_ap7 are plain linear maps and no ijk normalisation is needed; the
//    digit is a 9-entry lookup of the difference to the parent's centre;
//  * the base-cell rotations permute every 3-bit digit at once with bit-plane logic
//    (rot60ccw: 1->5->4->6->2->3->1, 0 and 7 fixed) instead of a loop per digit.
//  Pentagon base cells keep face_ijk_to_h3's digit-by-digit path.
constexpr uint64_t kDigitPlane = 0x49249249249ULL;  // bit 0 of each of the 15 digit fields
MGPU_HD uint64_t rotate60ccw_all(uint64_t f) {
  const uint64_t b0 = f & kDigitPlane, b1 = (f >> 1) & kDigitPlane, b2 = (f >> 2) & kDigitPlane;
  const uint64_t t = b0 & b1 & b2;
  const uint64_t n2 = ((~b1 & (b0 | b2)) | t) & kDigitPlane;
  const uint64_t n1 = ((~b0 & (b1 | b2)) | t) & kDigitPlane;
  const uint64_t n0 = ((~b2 & (b0 | b1)) | t) & kDigitPlane;
  return n0 | (n1 << 1) | (n2 << 2);
}

MGPU_HD uint64_t face_ijk_to_h3_fast(int face, IJK ijk, int res) {
  uint64_t h = kInit | (1ULL << 59) | ((uint64_t)res << 52);
  int a = ijk.i - ijk.k, b = ijk.j - ijk.k;
  uint64_t digits = kInit;  // 15 digits of 7
  for (int r = res - 1; r >= 0; r--) {
    int na, nb, ca, cb;
    if ((r + 1) & 1) {  // Class III child: up_ap7 / down_ap7
      na = round_div7(3 * a - b);
      nb = round_div7(a + 2 * b);
      ca = 2 * na + nb;
      cb = 3 * nb - na;
    } else {  // Class II child: up_ap7r / down_ap7r
      na = round_div7(2 * a + b);
      nb = round_div7(3 * b - a);
      ca = 3 * na - nb;
      cb = na + 2 * nb;
    }
    const int da = a - ca + 1, db = b - cb + 1;
    const int digit = ((unsigned)da < 3u && (unsigned)db < 3u)
                          ? (int)((0x647205731ULL >> (4 * (da * 3 + db))) & 0xF)
                          : 7;
    const int sh = (kMaxRes - (r + 1)) * 3;
    digits = (digits & ~(7ULL << sh)) | ((uint64_t)digit << sh);
    a = na;
    b = nb;
  }
  IJK base{a, b, 0};
  ijk_normalize(base);
  if (base.i > kMaxFaceCoord || base.j > kMaxFaceCoord || base.k > kMaxFaceCoord) return 0;
  const unsigned e = H3T_FACE_IJK_BASE_CELLS[face][base.i][base.j][base.k];
  const int bc = (int)(e & 0xff), rots = (int)(e >> 8);
  h = (h & ~kInit) | digits | ((uint64_t)bc << 45);
  if (H3T_BASE_CELL_DATA[bc][4]) {  // pentagon: digit-by-digit rotations
    if (leading_nonzero(h, res) == 1) {
      if (H3T_BASE_CELL_DATA[bc][5] == face || H3T_BASE_CELL_DATA[bc][6] == face)
        h = rotate_cw(h, res);
      else
        h = rotate_ccw(h, res);
    }
    for (int i = 0; i < rots; i++) h = rotate_pent_ccw(h, res);
    return h;
  }
  uint64_t f = h & kInit;
  for (int i = 0; i < rots; i++) f = rotate60ccw_all(f);
  return (h & ~kInit) | f;
}

// java.lang.Math.toRadians as on the reference's JDK 8 toolchain
MGPU_HD double to_radians(double deg) { return deg / 180.0 * 3.14159265358979323846; }

// Relative error band of the H3 route's hex2d coordinates: acos(1 - sqd/2) loses
// precision near a face centre (dr = eps / sin r), so H3's own result -- and any
// ulp-level libm difference -- carries a relative error ~eps / sin^2(r).  Decisions
// closer than 2^-40 * (1 + 1/sin^2 r) * |coordinate| to a threshold are near-ties.
MGPU_HD double tie_band(double vx, double vy, double sin2r) {
  double scale = fabs(vx) > fabs(vy) ? fabs(vx) : fabs(vy);
  if (scale < 1.0) scale = 1.0;
  double amp = 1.0 + (sin2r > 1e-300 ? 1.0 / sin2r : 1e300);
  return kTieRel * amp * scale;
}

// H3IndexSystem.pointToIndex(lon, lat, res) by the H3 route (the near-tie slow path
// and the reference for the fast path).  Returns 0 for non-finite input (H3-Java
// then throws IllegalArgumentException).
#ifdef __HIPCC__
// the route's libm polynomials must not be hoisted into the caller's point loop
// (that pins ~70 extra VGPRs for a path taken by ~1e-7 of the points)
#define MGPU_COLD static __host__ __device__ __attribute__((noinline))
#else
#define MGPU_COLD static inline
#endif
MGPU_COLD bool route_face_ijk(double lat, double lon, int res, int* face, IJK* ijk, bool* near_tie) {
  if (!isfinite(lat) || !isfinite(lon)) return false;
  double vx, vy, gap;
  geo_to_hex2d(lat, lon, res, face, &vx, &vy, &gap);
  double margin;
  *ijk = hex2d_to_ijk(vx, vy, &margin);
  double cx = H3T_FACE_CENTER_POINT[*face][0], cy = H3T_FACE_CENTER_POINT[*face][1],
         cz = H3T_FACE_CENTER_POINT[*face][2];
  double slat, clat, slon, clon;
  lm_sincos(lat, &slat, &clat);
  lm_sincos(lon, &slon, &clon);
  double cosr = cx * clon * clat + cy * slon * clat + cz * slat;
  *near_tie = (margin < tie_band(vx, vy, 1.0 - cosr * cosr)) || (gap < 1e-12);
  return true;
}

MGPU_HD uint64_t point_to_cell(double lon_deg, double lat_deg, int res, bool* near_tie) {
  double lat = to_radians(lat_deg), lon = to_radians(lon_deg);
  int face;
  IJK ijk;
  *near_tie = false;
  if (!route_face_ijk(lat, lon, res, &face, &ijk, near_tie)) return 0;
  return face_ijk_to_h3(face, ijk, res);
}

// ------------------------------------------------------------------ fast path
//
// The closed form of H3's projection: with v the unit vector of the point and
// (a, b, c) the face's gnomonic frame (H3T_FACE_FRAME, generated), H3's
//   r = acos(1 - |c - v|^2 / 2), theta = az0 - azimuth(c -> v), R = tan(r) * sqrt7^res / U
//   x = R cos(theta), y = R sin(theta)
// equals  x = K (v.a) / (v.c),  y = K (v.b) / (v.c)  with K = sqrt7^res / U.
// sin / cos of lat and lon come from a k/64-rad table plus a degree-9 Taylor series
// of the remainder (exact by Sterbenz).  The result differs from H3's by rounding
// only; every decision within tie_band() of a threshold goes to the H3 route.

// Fast-path arithmetic: explicit FMAs and a refined reciprocal instead of IEEE
// division.  Only the fast path uses these; its result is trusted only outside the
// tie band, which is ~1e3 x wider than the few-ulp differences they introduce.
MGPU_HD double fma_(double a, double b, double c) { return fma(a, b, c); }
MGPU_HD double recip(double d) {
#ifdef __HIP_DEVICE_COMPILE__
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
#else
  return 1.0 / d;
#endif
}
constexpr double kDegToRad = 0.017453292519943295769236907684886;
constexpr double kInvSin60 = 1.1547005383792515290182975610039149112953;
MGPU_HD double to_radians_fast(double deg) { return deg * kDegToRad; }

// sin and cos of |a| <= 3.15 without tables: a = k pi/2 + r (two-part Cody-Waite,
// |r| <= pi/4 + 1e-15), Taylor series to r^15 / r^16 (truncation < 5e-17), then the
// quadrant of k.  Absolute error ~3e-16: far inside the tie band.
MGPU_HD void sincos_fast(double a, double* s, double* c) {
  const double kf = rint(a * 0.63661977236758134308);
  const double r0 = fma_(kf, -1.5707963267948965580, a);
  const double r = fma_(kf, -6.1232339957367658e-17, r0);
  const double r2 = r * r;
  double ps = fma_(r2, -7.6471637318198164759e-13, 1.6059043836821614599e-10);
  ps = fma_(r2, ps, -2.5052108385441718775e-08);
  ps = fma_(r2, ps, 2.7557319223985890653e-06);
  ps = fma_(r2, ps, -1.9841269841269841270e-04);
  ps = fma_(r2, ps, 8.3333333333333333333e-03);
  ps = fma_(r2, ps, -1.6666666666666666667e-01);
  const double sr = fma_(r * r2, ps, r);
  double pc = fma_(r2, 4.7794773323873852974e-14, -1.1470745597729724714e-11);
  pc = fma_(r2, pc, 2.0876756987868098979e-09);
  pc = fma_(r2, pc, -2.7557319223985890653e-07);
  pc = fma_(r2, pc, 2.4801587301587301587e-05);
  pc = fma_(r2, pc, -1.3888888888888888889e-03);
  pc = fma_(r2, pc, 4.1666666666666666667e-02);
  pc = fma_(r2, pc, -0.5);
  const double cr = fma_(r2, pc, 1.0);
  const int q = (int)kf & 3;
  const double ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
  *s = (q & 2) ? -ss : ss;
  *c = ((q + 1) & 2) ? -cc : cc;
}

// _hex2dToCoordIJK with the fast path's multiply-by-reciprocal and the decision
// margin (same folds and thresholds as hex2d_to_ijk)
MGPU_HD IJK hex2d_to_ijk_fast(double vx, double vy, double* margin) {
  IJK h;
  h.k = 0;
  double a1 = fabs(vx), a2 = fabs(vy);
  double x2 = a2 * kInvSin60;
  double x1 = fma_(x2, 0.5, a1);
  int m1 = (int)x1, m2 = (int)x2;
  double r1 = x1 - m1, r2 = x2 - m2;
  double mg = dmin(dmin(r1, 1.0 - r1), dmin(r2, 1.0 - r2));
  double t, u;
  if (r1 < 0.5) {
    if (r1 < 1.0 / 3.0) {
      t = (1.0 + r1) * 0.5;
      u = t;
      h.i = m1;
      h.j = (r2 < t) ? m2 : m2 + 1;
      mg = dmin(mg, fabs(r1 - 1.0 / 3.0));
    } else {
      t = 1.0 - r1;
      u = 2.0 * r1;
      h.j = (r2 < t) ? m2 : m2 + 1;
      h.i = ((t <= r2) && (r2 < u)) ? m1 + 1 : m1;
      mg = dmin(mg, fabs(r1 - 1.0 / 3.0));
    }
    mg = dmin(mg, fabs(r1 - 0.5));
  } else {
    if (r1 < 2.0 / 3.0) {
      t = 1.0 - r1;
      u = 2.0 * r1 - 1.0;
      h.j = (r2 < t) ? m2 : m2 + 1;
      h.i = ((u < r2) && (r2 < t)) ? m1 : m1 + 1;
      mg = dmin(mg, fabs(r1 - 0.5));
    } else {
      t = r1 * 0.5;
      u = t;
      h.i = m1 + 1;
      h.j = (r2 < t) ? m2 : m2 + 1;
    }
    mg = dmin(mg, fabs(r1 - 2.0 / 3.0));
  }
  mg = dmin(mg, dmin(fabs(r2 - t), fabs(r2 - u)));
  if (vx < 0.0) {
    if ((h.j % 2) == 0) {
      int axisi = h.j / 2;
      int diff = h.i - axisi;
      h.i = h.i - 2 * diff;
    } else {
      int axisi = (h.j + 1) / 2;
      int diff = h.i - axisi;
      h.i = h.i - (2 * diff + 1);
    }
  }
  if (vy < 0.0) {
    h.i = h.i - (2 * h.j + 1) / 2;
    h.j = -1 * h.j;
  }
  ijk_normalize(h);
  mg = dmin(mg, dmin(a1, a2));
  *margin = mg;
  return h;
}

struct FastHex {
  int face;
  IJK ijk;
  bool tie;   // a decision may differ from the H3 route: recompute with route_face_ijk
  bool deep;  // not a tie, and inside the cell's hexagon scaled by 0.9 about its centre
};

// k_res = sqrt7^res / RES0_U_GNOMONIC; `faces` = the faces to consider (bit mask);
// lat, lon in radians (to_radians_fast is fine: a 1-ulp input change is far inside
// the tie band)
MGPU_HD FastHex fast_hex2d(double lat, double lon, int res, double k_res, uint32_t faces) {
  FastHex o;
  // sincos_fast's reduction is exact for |angle| <= 3.15: beyond, the H3 route
  const bool in_table = fabs(lat) <= 3.14 && fabs(lon) <= 3.14;
  if (!in_table) lat = lon = 0.0;
  double slat, clat, slon, clon;
  sincos_fast(lat, &slat, &clat);
  sincos_fast(lon, &slon, &clon);
  double vx = clon * clat, vy = slon * clat, vz = slat;
  double best = 5.0, second = 5.0;
  int f0 = 0;
  for (uint32_t m = faces; m; m &= m - 1) {
    int f = __builtin_ctz(m);
#ifdef __HIP_DEVICE_COMPILE__
    // keep the face table in memory: hoisting all 20 rows out of the caller's point
    // loop would pin 120 registers
    asm volatile("" : "+s"(f));
#endif
    double dx = H3T_FACE_CENTER_POINT[f][0] - vx;
    double dy = H3T_FACE_CENTER_POINT[f][1] - vy;
    double dz = H3T_FACE_CENTER_POINT[f][2] - vz;
    double s = fma_(dx, dx, fma_(dy, dy, dz * dz));
    if (s < best) {
      second = best;
      best = s;
      f0 = f;
    } else if (s < second) {
      second = s;
    }
  }
  o.face = f0;
  double dc, da, db;
#ifdef __HIP_DEVICE_COMPILE__
  // one face for the whole wave (the usual case): the frame comes in by scalar loads
  const int fu = __builtin_amdgcn_readfirstlane(f0);
  if (__all(f0 == fu)) {
    const double(*F)[3] = H3T_FACE_FRAME[fu][res & 1];
    dc = fma_(vx, F[2][0], fma_(vy, F[2][1], vz * F[2][2]));
    da = fma_(vx, F[0][0], fma_(vy, F[0][1], vz * F[0][2]));
    db = fma_(vx, F[1][0], fma_(vy, F[1][1], vz * F[1][2]));
  } else
#endif
  {
    const double(*F)[3] = H3T_FACE_FRAME[f0][res & 1];
    dc = fma_(vx, F[2][0], fma_(vy, F[2][1], vz * F[2][2]));
    da = fma_(vx, F[0][0], fma_(vy, F[0][1], vz * F[0][2]));
    db = fma_(vx, F[1][0], fma_(vy, F[1][1], vz * F[1][2]));
  }
  double q = k_res * recip(dc);
  double x = da * q, y = db * q;
  double margin;
  o.ijk = hex2d_to_ijk_fast(x, y, &margin);
  {
    // inside the hexagon scaled by 0.9 about the centre: the offset's projections on the
    // three edge normals (0, 60, 120 degrees) within 0.45 (the apothem is 0.5)
    const double ci = (double)(o.ijk.i - o.ijk.k), cj = (double)(o.ijk.j - o.ijk.k);
    const double ex = x - (ci - 0.5 * cj), ey = y - cj * 0.8660254037844386;
    const double p60 = 0.5 * ex + 0.8660254037844386 * ey, p120 = -0.5 * ex + 0.8660254037844386 * ey;
    o.deep = fabs(ex) < 0.45 && fabs(p60) < 0.45 && fabs(p120) < 0.45;
  }
  // margin < tie_band(x, y, sin2r) without the division: with sin2r = 1 - dc^2 > 0,
  //   margin < kTieRel * (1 + 1/sin2r) * scale  <=>  margin * sin2r < kTieRel * (sin2r + 1) * scale
  double scale = fabs(x) > fabs(y) ? fabs(x) : fabs(y);
  if (scale < 1.0) scale = 1.0;
  double sin2r = fma_(-dc, dc, 1.0);
  o.tie = !in_table || (second - best < 1e-12) || !(dc > 0.5) || !(sin2r > 1e-300) ||
          (margin * sin2r < kTieRel * (sin2r + 1.0) * scale);
  o.deep = o.deep && !o.tie;
  return o;
}

// lattice key of (face, ijk): face in bits 56..60, (i - k) and (j - k) biased by 2^27
MGPU_HD uint64_t lattice_key(int face, IJK c) {
  uint64_t a = (uint64_t)(uint32_t)(c.i - c.k + (1 << 27)) & 0xFFFFFFFULL;
  uint64_t b = (uint64_t)(uint32_t)(c.j - c.k + (1 << 27)) & 0xFFFFFFFULL;
  return ((uint64_t)face << 56) | (a << 28) | b;
}

// K(res) = sqrt7^res / RES0_U_GNOMONIC
MGPU_HD double k_of_res(int res) {
  double r = 1.0 / kRes0UGnomonic;
  for (int i = 0; i < res; i++) r *= kSqrt7;
  return r;
}

// ------------------------------------------------------------------ inverse (host)

MGPU_HD void ijk_to_hex2d(IJK h, double* x, double* y) {
  int i = h.i - h.k, j = h.j - h.k;
  *x = i - 0.5 * j;
  *y = j * kSin60;
}

// _hex2dToGeo (substrate 0): hex2d on `face` at `res` -> (lat, lon) radians
MGPU_HD void hex2d_to_geo(double vx, double vy, int face, int res, double* lat, double* lon) {
  double r = sqrt(vx * vx + vy * vy);
  double lat0 = H3T_FACE_CENTER_GEO[face][0], lon0 = H3T_FACE_CENTER_GEO[face][1];
  if (r < kEpsilon) {
    *lat = lat0;
    *lon = lon0;
    return;
  }
  double theta = atan2(vy, vx);
  for (int i = 0; i < res; i++) r = exact::ld_div(r, exact::kXSqrt7);
  r *= kRes0UGnomonic;
  r = atan(r);
  if (res % 2) theta = pos_angle(exact::ld_add(theta, exact::kXAp7Rot));
  double az = pos_angle(H3T_FACE_AXES_AZ_CII[face][0] - theta);
  double sinlat = sin(lat0) * cos(r) + cos(lat0) * sin(r) * cos(az);
  if (sinlat > 1.0) sinlat = 1.0;
  if (sinlat < -1.0) sinlat = -1.0;
  *lat = asin(sinlat);
  double sinlon = sin(az) * sin(r) / cos(*lat);
  double coslon = (cos(r) - sin(lat0) * sin(*lat)) / cos(lat0) / cos(*lat);
  if (sinlon > 1.0) sinlon = 1.0;
  if (sinlon < -1.0) sinlon = -1.0;
  if (coslon > 1.0) coslon = 1.0;
  if (coslon < -1.0) coslon = -1.0;
  double l = lon0 + atan2(sinlon, coslon);
  while (l > 3.14159265358979323846) l -= 2 * 3.14159265358979323846;
  while (l < -3.14159265358979323846) l += 2 * 3.14159265358979323846;
  *lon = l;
}

// _h3ToFaceIjkWithInitializedFijk without the overage adjustment: the cell's
// centre in its base cell's home-face lattice.  Returns false for pentagon base
// cells (their digit space is rotated; callers fall back to cell-id probing).
MGPU_HD bool h3_home_face_ijk(uint64_t h, int* face, IJK* ijk, int* res_out) {
  int res = (int)((h >> 52) & 15);
  int bc = (int)((h >> 45) & 127);
  if (bc >= H3T_NUM_BASE_CELLS || H3T_BASE_CELL_DATA[bc][4]) return false;
  *face = H3T_BASE_CELL_DATA[bc][0];
  IJK c{H3T_BASE_CELL_DATA[bc][1], H3T_BASE_CELL_DATA[bc][2], H3T_BASE_CELL_DATA[bc][3]};
  for (int r = 1; r <= res; r++) {
    if (r & 1) down_ap7(c);
    else down_ap7r(c);
    int d = digit_at(h, r);
    if (d == 7) return false;
    if (d) {
      c.i += (d >> 2) & 1;
      c.j += (d >> 1) & 1;
      c.k += d & 1;
      ijk_normalize(c);
    }
  }
  *ijk = c;
  *res_out = res;
  return true;
}

}  // namespace h3
}  // namespace mgpu
