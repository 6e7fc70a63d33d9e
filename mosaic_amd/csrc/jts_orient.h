// CGAlgorithmsDD.orientationIndex (JTS 1.20, a Maven dependency: pom.xml:98-102): the
// 1e-15 filter, then the DoubleDouble determinant.  Shared by st_contains (pip_core.h,
// host + device) and the host buffer restatement (jts_buffer.h).  Built with
// -ffp-contract=off: every product is rounded separately as on the JVM.
#pragma once
#include "chip_table.h"

namespace mgpu {
namespace pip {

struct DD {
  double hi, lo;
};

MGPU_HDI DD dd_add(DD a, double yhi, double ylo) {
  double S = a.hi + yhi;
  double T = a.lo + ylo;
  double e = S - a.hi;
  double f = T - a.lo;
  double s = S - e;
  double t = T - f;
  s = (yhi - e) + (a.hi - s);
  t = (ylo - f) + (a.lo - t);
  e = s + T;
  double H = S + e;
  double h = e + (S - H);
  e = t + h;
  DD z;
  z.hi = H + e;
  z.lo = e + (H - z.hi);
  return z;
}

MGPU_HDI DD dd_mul(DD a, double yhi, double ylo) {
  const double SPLIT = 134217729.0;
  double C = SPLIT * a.hi;
  double hx = C - a.hi;
  double c = SPLIT * yhi;
  hx = C - hx;
  double tx = a.hi - hx;
  double hy = c - yhi;
  C = a.hi * yhi;
  hy = c - hy;
  double ty = yhi - hy;
  c = ((((hx * hy - C) + hx * ty) + tx * hy) + tx * ty) + (a.hi * ylo + a.lo * yhi);
  DD z;
  z.hi = C + c;
  hx = C - z.hi;
  z.lo = c + hx;
  return z;
}

MGPU_HDI int sgn(double x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }

// CGAlgorithmsDD.orientationIndex(p1, p2, q)
MGPU_HDI int orientation(double p1x, double p1y, double p2x, double p2y, double qx, double qy) {
  double detleft = (p1x - qx) * (p2y - qy);
  double detright = (p1y - qy) * (p2x - qx);
  double det = detleft - detright;
  double detsum;
  if (detleft > 0.0) {
    if (detright <= 0.0) return sgn(det);
    detsum = detleft + detright;
  } else if (detleft < 0.0) {
    if (detright >= 0.0) return sgn(det);
    detsum = -detleft - detright;
  } else {
    return sgn(det);
  }
  double errbound = 1e-15 * detsum;
  if ((det >= errbound) || (-det >= errbound)) return sgn(det);
  DD dx1 = dd_add(DD{p2x, 0.0}, -p1x, 0.0);
  DD dy1 = dd_add(DD{p2y, 0.0}, -p1y, 0.0);
  DD dx2 = dd_add(DD{qx, 0.0}, -p2x, 0.0);
  DD dy2 = dd_add(DD{qy, 0.0}, -p2y, 0.0);
  DD a = dd_mul(dx1, dy2.hi, dy2.lo);
  DD b = dd_mul(dy1, dx2.hi, dx2.lo);
  DD d = dd_add(a, -b.hi, -b.lo);
  if (d.hi > 0) return 1;
  if (d.hi < 0) return -1;
  if (d.lo > 0) return 1;
  if (d.lo < 0) return -1;
  return 0;
}

}  // namespace pip
}  // namespace mgpu
