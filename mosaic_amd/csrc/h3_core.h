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
// Numerics.  All arithmetic is IEEE double with FMA contraction disabled (the
// library is compiled with -ffp-contract=off), so every + - * / rounds exactly as
// in the JVM path's native H3.  Two things can differ from that path by an ulp:
// the libm transcendentals (ocml here, glibc there) and the five H3 expressions
// that use x87 long-double constants.  Both only matter for points whose hex2d
// coordinates fall within a few ulps of a cell edge; every such point is detected
// by `margin` below (distance to the nearest decision threshold, in hex units,
// relative to the coordinate magnitude) and is reported as a near-tie.
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

MGPU_HD double pos_angle(double rads) {
  double tmp = (rads < 0.0) ? rads + kTwoPi : rads;
  if (rads >= kTwoPi) tmp -= kTwoPi;
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
MGPU_HD IJK hex2d_to_ijk(double vx, double vy, double* margin) {
  IJK h;
  h.k = 0;
  double a1 = fabs(vx), a2 = fabs(vy);
  double x2 = a2 / kSin60;
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
MGPU_HD void geo_to_hex2d(double lat, double lon, int res, int* face, double* vx, double* vy, double* face_gap) {
  double slat, clat, slon, clon;
  sincos(lat, &slat, &clat);
  sincos(lon, &slon, &clon);
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
  double r = acos(1 - best / 2);
  if (r < kEpsilon) {
    *vx = *vy = 0.0;
    return;
  }
  // _geoAzimuthRads(faceCenterGeo[face], g)
  double flat = H3T_FACE_CENTER_GEO[f0][0], flon = H3T_FACE_CENTER_GEO[f0][1];
  double sdl, cdl;
  sincos(lon - flon, &sdl, &cdl);
  double az = atan2(clat * sdl, cos(flat) * slat - sin(flat) * clat * cdl);
  double theta = pos_angle(H3T_FACE_AXES_AZ_CII[f0][0] - pos_angle(az));
  if (res % 2) theta = pos_angle(theta - kAp7Rot);
  r = tan(r);
  r /= kRes0UGnomonic;
  for (int i = 0; i < res; i++) r *= kSqrt7;
  double st, ct;
  sincos(theta, &st, &ct);
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
MGPU_HD int leading_nonzero(uint64_t h, int res) {
  for (int r = 1; r <= res; r++) {
    int d = digit_at(h, r);
    if (d) return d;
  }
  return 0;
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

// java.lang.Math.toRadians as on the reference's JDK 8 toolchain
MGPU_HD double to_radians(double deg) { return deg / 180.0 * 3.14159265358979323846; }

// H3IndexSystem.pointToIndex(lon, lat, res).  Returns 0 for non-finite input
// (H3-Java then throws IllegalArgumentException).  *near_tie is set when the
// result sits within the fast path's error band of a cell edge.
MGPU_HD uint64_t point_to_cell(double lon_deg, double lat_deg, int res, bool* near_tie) {
  double lat = to_radians(lat_deg), lon = to_radians(lon_deg);
  *near_tie = false;
  if (!isfinite(lat) || !isfinite(lon)) return 0;
  int face;
  double vx, vy, gap;
  geo_to_hex2d(lat, lon, res, &face, &vx, &vy, &gap);
  double margin;
  IJK ijk = hex2d_to_ijk(vx, vy, &margin);
  double scale = fabs(vx) > fabs(vy) ? fabs(vx) : fabs(vy);
  if (scale < 1.0) scale = 1.0;
  *near_tie = (margin < kTieRel * scale) || (gap < 1e-12);
  return face_ijk_to_h3(face, ijk, res);
}

}  // namespace h3
}  // namespace mgpu
