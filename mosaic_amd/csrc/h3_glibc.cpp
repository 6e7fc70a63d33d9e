// The H3 route with the reference's own arithmetic, for the near-tie points only.
//
// Replaces: H3IndexSystem.pointToIndex -> H3Core.geoToH3(lat, lon, res)
//   /root/reference/src/main/scala/com/databricks/labs/mosaic/core/index/H3IndexSystem.scala:168-170
// H3-Java 3.7.0 (pom.xml:91-97) runs H3 C v3.7's geoToH3 in its JNI library on the
// executor's host: SSE2 doubles, the platform glibc's sin / cos / tan / acos / atan2, and
// the five expressions whose operand is one of H3's long-double constants (M_2PI, M_SQRT7,
// M_SIN60, M_AP7_ROT_RADS, EPSILON) in x87 extended precision.  This file is that route,
// built by g++ for the host with -ffp-contract=off (no FMA contraction), so that:
//   * a point the device resolved inside its 2^-40 tie band (h3_core.h route_face_ijk) gets
//     exactly the cell the reference computes, libm rounding included -- the device's
//     route is correctly rounded, glibc is not;
//   * it is called only for those points (a few per 1e8 on uniform data): capi.cpp
//     recomputes them here after the join and, when a cell moves, reruns the join with the
//     corrected (face, ijk) as an override.
// Integer steps (_faceIjkToH3) are shared with the device code (h3_core.h).
#include "h3_glibc.h"

#include <math.h>

#include "h3_core.h"

namespace mgpu {
namespace h3glibc {
namespace {

// H3's constants.h literals (long double on x86-64)
constexpr long double kL2Pi = 6.28318530717958647692528676655900576839433L;
constexpr long double kLEpsilon = 0.0000000000000001L;
constexpr long double kLSin60 = 0.8660254037844386467637231707529361834714L;
constexpr long double kLAp7Rot = 0.333473172251832115336090755351601070065900389L;
constexpr long double kLSqrt7 = 2.6457513110645905905016157536392604257102L;
constexpr double kRes0U = 0.38196601125010500003;

// _posAngleRads: the conditional is a long-double expression, rounded once on assignment
double pos_angle(double rads) {
  double tmp = (rads < 0.0L) ? rads + kL2Pi : rads;
  if (rads >= kL2Pi) tmp -= kL2Pi;
  return tmp;
}

double sq(double x) { return x * x; }

// Each libm call as H3's source writes it: through pointers the compiler cannot see
// through, so no pair sin(a), cos(a) is fused into one sincos call (glibc's sincos
// rounds differently from sin and cos in a few ulps; the oracle calls them separately)
double (*volatile f_sin)(double) = ::sin;
double (*volatile f_cos)(double) = ::cos;
double (*volatile f_tan)(double) = ::tan;
double (*volatile f_acos)(double) = ::acos;
double (*volatile f_atan2)(double, double) = ::atan2;

// _geoAzimuthRads(p1, p2)
double azimuth(double lat1, double lon1, double lat2, double lon2) {
  return f_atan2(f_cos(lat2) * f_sin(lon2 - lon1),
                 f_cos(lat1) * f_sin(lat2) - f_sin(lat1) * f_cos(lat2) * f_cos(lon2 - lon1));
}

// _hex2dToCoordIJK
h3::IJK hex2d_to_ijk(double vx, double vy) {
  h3::IJK h{0, 0, 0};
  const double a1 = fabsl(vx), a2 = fabsl(vy);
  const double x2 = a2 / kLSin60;
  const double x1 = a1 + x2 / 2.0;
  const int m1 = (int)x1, m2 = (int)x2;
  const double r1 = x1 - m1, r2 = x2 - m2;
  if (r1 < 0.5) {
    if (r1 < 1.0 / 3.0) {
      h.i = m1;
      h.j = (r2 < (1.0 + r1) / 2.0) ? m2 : m2 + 1;
    } else {
      h.j = (r2 < (1.0 - r1)) ? m2 : m2 + 1;
      h.i = ((1.0 - r1) <= r2 && r2 < (2.0 * r1)) ? m1 + 1 : m1;
    }
  } else {
    if (r1 < 2.0 / 3.0) {
      h.j = (r2 < (1.0 - r1)) ? m2 : m2 + 1;
      h.i = ((2.0 * r1 - 1.0) < r2 && r2 < (1.0 - r1)) ? m1 : m1 + 1;
    } else {
      h.i = m1 + 1;
      h.j = (r2 < (r1 / 2.0)) ? m2 : m2 + 1;
    }
  }
  if (vx < 0.0) {
    if ((h.j % 2) == 0) {
      const long long axisi = h.j / 2;
      const long long diff = h.i - axisi;
      h.i = (int)(h.i - 2.0 * diff);
    } else {
      const long long axisi = (h.j + 1) / 2;
      const long long diff = h.i - axisi;
      h.i = (int)(h.i - (2.0 * diff + 1));
    }
  }
  if (vy < 0.0) {
    h.i = h.i - (2 * h.j + 1) / 2;
    h.j = -1 * h.j;
  }
  h3::ijk_normalize(h);
  return h;
}

}  // namespace

bool face_ijk(double lon_deg, double lat_deg, int res, int* face, h3::IJK* ijk) {
  if (res < 0 || res > 15 || !isfinite(lon_deg) || !isfinite(lat_deg)) return false;
  // java.lang.Math.toRadians on the reference's JDK 8: deg / 180.0 * PI
  const double lat = lat_deg / 180.0 * 3.14159265358979323846, lon = lon_deg / 180.0 * 3.14159265358979323846;
  // _geoToVec3d, _geoToClosestFace (strict <: the first minimum wins)
  const double r0 = f_cos(lat);
  const double vz = f_sin(lat), vx = f_cos(lon) * r0, vy = f_sin(lon) * r0;
  int f0 = 0;
  double sqd = 5.0;
  for (int f = 0; f < H3T_NUM_FACES; f++) {
    const double d = sq(H3T_FACE_CENTER_POINT[f][0] - vx) + sq(H3T_FACE_CENTER_POINT[f][1] - vy) +
                     sq(H3T_FACE_CENTER_POINT[f][2] - vz);
    if (d < sqd) {
      f0 = f;
      sqd = d;
    }
  }
  *face = f0;
  // _geoToHex2d
  double r = f_acos(1 - sqd / 2);
  double hx = 0.0, hy = 0.0;
  if (!(r < kLEpsilon)) {
    double theta = pos_angle(H3T_FACE_AXES_AZ_CII[f0][0] -
                             pos_angle(azimuth(H3T_FACE_CENTER_GEO[f0][0], H3T_FACE_CENTER_GEO[f0][1], lat, lon)));
    if (res % 2) theta = pos_angle(theta - kLAp7Rot);
    r = f_tan(r);
    r /= kRes0U;
    for (int i = 0; i < res; i++) r *= kLSqrt7;
    hx = r * f_cos(theta);
    hy = r * f_sin(theta);
  }
  *ijk = hex2d_to_ijk(hx, hy);
  return true;
}

uint64_t point_to_cell(double lon_deg, double lat_deg, int res) {
  int face;
  h3::IJK ijk;
  if (!face_ijk(lon_deg, lat_deg, res, &face, &ijk)) return 0;
  return h3::face_ijk_to_h3(face, ijk, res);
}

uint64_t lattice_key(double lon_deg, double lat_deg, int res) {
  int face;
  h3::IJK ijk;
  if (!face_ijk(lon_deg, lat_deg, res, &face, &ijk)) return 0;
  return h3::lattice_key(face, ijk);
}

}  // namespace h3glibc
}  // namespace mgpu
