// mosaicFill's two buffers, restated from JTS 1.20's BufferOp (host code, used by the
// tessellator to flag chips):
//
//   carved = geometry.buffer(-r)                          (core/Mosaic.scala:71)
//   band   = geometry.boundary.buffer(1.01 r).simplify(0.01 r), or, when carved is
//            empty, geometry.buffer(1.01 r).simplify(0.01 r)    (core/Mosaic.scala:75-84)
//   core   = polyfill(carved); border = polyfill(band) diff core (:92-93)
//
// MosaicGeometryJTS.buffer (core/geometry/MosaicGeometryJTS.scala:86-115) runs a default
// BufferOp: round joins, 8 quadrant segments.  JTS (a Maven dependency, not in the
// reference tree; pom.xml:98-102) builds a buffer as
//   1. OffsetCurveSetBuilder: per ring, CoordinateArrays.removeRepeatedPoints; shells
//      that isErodedCompletely are skipped; ring side and Left/Right labels from the
//      ring's orientation (addRingSide); for a closed line (the boundary's rings)
//      addRingBothSides;
//   2. OffsetCurveBuilder.computeRingBufferCurve: BufferInputLineSimplifier (shallow
//      concavities on the non-buffered side removed, tolerance 0.01 * distance), then
//      OffsetSegmentGenerator: offset segments joined by a circular fillet of chords at
//      outside turns (nSegs = round(angle / (pi/16)) equal steps, vertices ON the
//      circle), by the offset segments' intersection at inside turns (else closing
//      segments toward the vertex, closingSegLengthFactor 80), near-duplicate points
//      dropped (1e-6 * distance);
//   3. BufferBuilder: the raw curves noded into a planar graph, each face's depth = the
//      sum of the labels crossed from the outside (Left/Right INTERIOR/EXTERIOR), the
//      result = the faces of depth >= 1.
// Step 3's depth is the curves' signed winding number, so a point off every curve is
// in the buffer iff  sum_curves sign * winding(curve, p) >= 1  -- which is what is
// evaluated here, per queried cell centre, without building the noded polygon.  The
// simplification of the band (DouglasPeuckerSimplifier, 0.01 r) moves its outline by
// < 0.01 r: a centre within that of a band curve is reported as DP-sensitive (its
// membership follows the unsimplified band).  A centre within 1e-9 r of a curve is
// reported unresolved.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "jts_orient.h"

namespace mgpu {
namespace jtsbuf {

struct XY {
  double x, y;
};
inline bool same(XY a, XY b) { return a.x == b.x && a.y == b.y; }
inline double dist(XY a, XY b) {  // Coordinate.distance
  const double dx = a.x - b.x, dy = a.y - b.y;
  return std::sqrt(dx * dx + dy * dy);
}
enum { kCW = -1, kCollinear = 0, kCCW = 1 };
enum { kLeft = 1, kRight = 2 };
enum { kInterior = 0, kExterior = 2 };
inline int opposite(int side) { return side == kLeft ? kRight : kLeft; }
// Orientation.index = CGAlgorithmsDD.orientationIndex
inline int orient(XY a, XY b, XY c) { return mgpu::pip::orientation(a.x, a.y, b.x, b.y, c.x, c.y); }

// Distance.pointToSegment
inline double point_to_segment(XY p, XY a, XY b) {
  if (a.x == b.x && a.y == b.y) return dist(p, a);
  const double len2 = (b.x - a.x) * (b.x - a.x) + (b.y - a.y) * (b.y - a.y);
  const double r = ((p.x - a.x) * (b.x - a.x) + (p.y - a.y) * (b.y - a.y)) / len2;
  if (r <= 0.0) return dist(p, a);
  if (r >= 1.0) return dist(p, b);
  const double s = ((a.y - p.y) * (b.x - a.x) - (a.x - p.x) * (b.y - a.y)) / len2;
  return std::fabs(s) * std::sqrt(len2);
}

// CoordinateArrays.removeRepeatedPoints
inline std::vector<XY> remove_repeated(const std::vector<XY>& in) {
  std::vector<XY> o;
  o.reserve(in.size());
  for (auto& p : in)
    if (o.empty() || !same(o.back(), p)) o.push_back(p);
  return o;
}

// the ring's orientation (shoelace sign: Orientation.isCCW and isCCWArea agree on the
// valid rings a polygon holds)
inline bool is_ccw(const std::vector<XY>& r) {
  if (r.size() < 4) return false;
  double a = 0;
  for (size_t i = 0; i + 1 < r.size(); i++) a += (r[i].x - r[0].x) * (r[i + 1].y - r[0].y) - (r[i + 1].x - r[0].x) * (r[i].y - r[0].y);
  return a > 0;
}

// BufferInputLineSimplifier.simplify(line, signedTol): deletes, until nothing changes,
// middle vertices of consecutive triples that turn toward the side being removed
// (CCW for tol > 0, CW for tol < 0) and lie within |tol| of the triple's chord, then
// pass isShallowSampled -- whose call passes the middle vertex where its parameter list
// names the section end, so the sampled test is the distance from the middle vertex to
// the segments (p0, line[i]) for i in [i0, i2) in steps of max(1, (i2 - i0) / 10).  The
// first vertex is never a middle one (the window starts at index 1).
inline std::vector<XY> simplify_input(const std::vector<XY>& line, double signed_tol) {
  const double tol = std::fabs(signed_tol);
  const int angle = signed_tol < 0 ? kCW : kCCW;
  const int n = (int)line.size();
  std::vector<uint8_t> del(n, 0);
  auto next = [&](int i) {
    int k = i + 1;
    while (k < n && del[k]) k++;
    return k;
  };
  auto shallow = [&](XY p0, XY p1, XY p2) { return point_to_segment(p1, p0, p2) < tol; };
  auto deletable = [&](int i0, int i1, int i2) {
    const XY p0 = line[i0], p1 = line[i1], p2 = line[i2];
    if (orient(p0, p1, p2) != angle) return false;
    if (!shallow(p0, p1, p2)) return false;
    int inc = (i2 - i0) / 10;
    if (inc <= 0) inc = 1;
    for (int i = i0; i < i2; i += inc)
      if (!shallow(p0, p1, line[i])) return false;
    return true;
  };
  bool changed;
  do {
    changed = false;
    int i = 1, mid = next(i), last = next(mid);
    while (last < n) {
      bool d = false;
      if (deletable(i, mid, last)) {
        del[mid] = 1;
        d = changed = true;
      }
      i = d ? last : mid;
      mid = next(i);
      last = next(mid);
    }
  } while (changed);
  std::vector<XY> o;
  o.reserve(n);
  for (int i = 0; i < n; i++)
    if (!del[i]) o.push_back(line[i]);
  return o;
}

// OffsetSegmentGenerator (round joins, 8 quadrant segments) over one closed ring
struct OffsetRing {
  double d;
  int side = kLeft;
  double quantum = M_PI / 2.0 / 8.0;
  double closing = 80.0;  // closingSegLengthFactor (quadrantSegments >= 8, round joins)
  double min_vd;
  std::vector<XY> pts;
  XY s0{}, s1{}, s2{};
  XY o0a{}, o0b{}, o1a{}, o1b{};  // offset0 = (o0a, o0b), offset1 = (o1a, o1b)

  explicit OffsetRing(double dist_) : d(dist_), min_vd(dist_ * 1.0e-6) {}

  void add(XY p) {  // OffsetSegmentString.addPt: near-duplicates dropped
    if (!pts.empty() && dist(p, pts.back()) < min_vd) return;
    pts.push_back(p);
  }
  void offset(XY a, XY b, XY* oa, XY* ob) const {  // computeOffsetSegment
    const double sign = side == kLeft ? 1.0 : -1.0;
    const double dx = b.x - a.x, dy = b.y - a.y, len = std::sqrt(dx * dx + dy * dy);
    const double ux = sign * d * dx / len, uy = sign * d * dy / len;
    *oa = {a.x - uy, a.y + ux};
    *ob = {b.x - uy, b.y + ux};
  }
  void init(XY a, XY b, int side_) {
    side = side_;
    s1 = a;
    s2 = b;
    offset(s1, s2, &o1a, &o1b);
  }
  void fillet(XY p, XY p0, XY p1, int dir, double radius) {  // addCornerFillet
    double start = std::atan2(p0.y - p.y, p0.x - p.x);
    const double end = std::atan2(p1.y - p.y, p1.x - p.x);
    if (dir == kCW) {
      if (start <= end) start += 2.0 * M_PI;
    } else if (start >= end) {
      start -= 2.0 * M_PI;
    }
    add(p0);
    // addDirectedFillet
    const double f = dir == kCW ? -1.0 : 1.0;
    const double total = std::fabs(start - end);
    const int nseg = (int)(total / quantum + 0.5);
    if (nseg >= 1) {
      const double inc = total / nseg;
      for (int i = 0; i < nseg; i++) {
        const double a = start + f * i * inc;
        add({p.x + radius * std::cos(a), p.y + radius * std::sin(a)});
      }
    }
    add(p1);
  }
  // RobustLineIntersector.computeIntersection(p1, p2, q1, q2) for two offset segments
  // of an inside turn (never collinear: the turn is not): the intersection point if any
  static bool intersect(XY p1, XY p2, XY q1, XY q2, XY* out) {
    const int a1 = orient(p1, p2, q1), a2 = orient(p1, p2, q2);
    if ((a1 > 0 && a2 > 0) || (a1 < 0 && a2 < 0)) return false;
    const int b1 = orient(q1, q2, p1), b2 = orient(q1, q2, p2);
    if ((b1 > 0 && b2 > 0) || (b1 < 0 && b2 < 0)) return false;
    if (a1 == 0 && a2 == 0 && b1 == 0 && b2 == 0) return false;
    // endpoint touches: the shared endpoint
    if (a1 == 0) { *out = q1; return true; }
    if (a2 == 0) { *out = q2; return true; }
    if (b1 == 0) { *out = p1; return true; }
    if (b2 == 0) { *out = p2; return true; }
    const double dxp = p2.x - p1.x, dyp = p2.y - p1.y, dxq = q2.x - q1.x, dyq = q2.y - q1.y;
    const double den = dxp * dyq - dyp * dxq;
    const double t = ((q1.x - p1.x) * dyq - (q1.y - p1.y) * dxq) / den;
    *out = {p1.x + t * dxp, p1.y + t * dyp};
    return true;
  }
  void next_segment(XY p, bool add_start) {  // addNextSegment
    s0 = s1;
    s1 = s2;
    s2 = p;
    offset(s0, s1, &o0a, &o0b);
    offset(s1, s2, &o1a, &o1b);
    if (same(s1, s2)) return;
    const int o = orient(s0, s1, s2);
    const bool outside = (o == kCW && side == kLeft) || (o == kCCW && side == kRight);
    if (o == kCollinear) {
      // addCollinear: a reversal (s2 back along s0-s1) gets an end-cap fillet; same
      // direction adds nothing
      const bool reversing = (s2.x - s1.x) * (s1.x - s0.x) + (s2.y - s1.y) * (s1.y - s0.y) < 0;
      if (reversing) fillet(s1, o0b, o1a, kCW, d);
    } else if (outside) {
      if (dist(o0b, o1a) < d * 1.0e-3) {  // OFFSET_SEGMENT_SEPARATION_FACTOR
        add(o0b);
        return;
      }
      if (add_start) add(o0b);
      fillet(s1, o0b, o1a, o, d);
      add(o1a);
    } else {
      XY ip;
      if (intersect(o0a, o0b, o1a, o1b, &ip)) {
        add(ip);
      } else if (dist(o0b, o1a) < d * 1.0e-3) {  // INSIDE_TURN_VERTEX_SNAP_DISTANCE_FACTOR
        add(o0b);
      } else {
        add(o0b);
        add({(closing * o0b.x + s1.x) / (closing + 1), (closing * o0b.y + s1.y) / (closing + 1)});
        add({(closing * o1a.x + s1.x) / (closing + 1), (closing * o1a.y + s1.y) / (closing + 1)});
        add(o1a);
      }
    }
  }
};

// OffsetCurveBuilder.getRingCurve (ring closed, >= 4 points, distance > 0)
inline std::vector<XY> ring_curve(const std::vector<XY>& ring, int side, double distance, bool simplify = true) {
  const double tol = distance * 0.01;  // BufferParameters simplifyFactor
  const std::vector<XY> simp = simplify ? simplify_input(ring, side == kRight ? -tol : tol) : ring;
  OffsetRing g(distance);
  const int n = (int)simp.size() - 1;
  if (n < 1) return {};
  g.init(simp[n - 1], simp[0], side);
  for (int i = 1; i <= n; i++) g.next_segment(simp[i], i != 1);
  if (!g.pts.empty() && !same(g.pts.front(), g.pts.back())) g.pts.push_back(g.pts.front());  // closeRing
  return g.pts;
}

// OffsetCurveSetBuilder.isErodedCompletely (shell, negative distance)
inline bool eroded_completely(const std::vector<XY>& ring, double buffer_distance) {
  if (ring.size() < 4) return buffer_distance < 0;
  if (ring.size() == 4) {  // isTriangleErodedCompletely: the incircle is smaller than |distance|
    const XY a = ring[0], b = ring[1], c = ring[2];
    const double la = dist(b, c), lb = dist(a, c), lc = dist(a, b), s = la + lb + lc;
    const XY inc{(la * a.x + lb * b.x + lc * c.x) / s, (la * a.y + lb * b.y + lc * c.y) / s};
    return point_to_segment(inc, a, b) < std::fabs(buffer_distance);
  }
  double minx = INFINITY, maxx = -INFINITY, miny = INFINITY, maxy = -INFINITY;
  for (auto& p : ring) {
    minx = std::min(minx, p.x);
    maxx = std::max(maxx, p.x);
    miny = std::min(miny, p.y);
    maxy = std::max(maxy, p.y);
  }
  return buffer_distance < 0.0 && 2 * std::fabs(buffer_distance) > std::min(maxy - miny, maxx - minx);
}

// OffsetCurveSetBuilder.isRingCurveInverted (rings of 4..8 points): a curve none of whose
// vertices or segment midpoints is farther than 0.99 * distance from the ring is an
// inverted artefact and is skipped
inline bool curve_inverted(const std::vector<XY>& ring, double distance, const std::vector<XY>& curve) {
  if (distance == 0.0 || ring.size() <= 3 || ring.size() >= 9) return false;
  if (curve.size() > 4 * ring.size()) return false;
  const double tol = 0.99 * std::fabs(distance);
  auto far = [&](XY p) {
    double best = INFINITY;
    for (size_t i = 0; i + 1 < ring.size(); i++) best = std::min(best, point_to_segment(p, ring[i], ring[i + 1]));
    return best > tol;
  };
  for (size_t i = 0; i + 1 < curve.size(); i++) {
    if (far(curve[i])) return false;
    if (far({(curve[i].x + curve[i + 1].x) / 2, (curve[i].y + curve[i + 1].y) / 2})) return false;
  }
  return true;
}

// The depth field of a set of raw curves: depth(p) = sum over curves of sign * winding
struct DepthField {
  struct Seg {
    XY a, b;
    int sign;
  };
  std::vector<Seg> segs;
  // bucket grid (rows x cols), each bucket listing the segments whose box meets it
  double x0 = 0, y0 = 0, s = 1, inv = 1;
  long nx = 0, ny = 0;
  std::vector<uint32_t> start, items;
  bool empty() const { return segs.empty(); }

  // addRingSide: labels from the ring's orientation; sign +1 when the curve's left is
  // INTERIOR, -1 when its right is
  void add_ring_side(const std::vector<XY>& coord, double dist_, int side, int cw_left, int cw_right) {
    int left = cw_left, right = cw_right;
    if (coord.size() >= 4 && is_ccw(coord)) {
      std::swap(left, right);
      side = opposite(side);
    }
    (void)right;
    const auto curve = ring_curve(coord, side, dist_, simplify_rings);
    if (curve.size() < 2 || curve_inverted(coord, dist_, curve)) return;
    const int sign = left == kInterior ? 1 : -1;
    for (size_t i = 0; i + 1 < curve.size(); i++)
      if (!same(curve[i], curve[i + 1])) segs.push_back({curve[i], curve[i + 1], sign});
  }
  bool simplify_rings = true;

  void build_index(double cell) {
    if (segs.empty()) return;
    double minx = INFINITY, miny = INFINITY, maxx = -INFINITY, maxy = -INFINITY;
    for (auto& g : segs) {
      minx = std::min({minx, g.a.x, g.b.x});
      maxx = std::max({maxx, g.a.x, g.b.x});
      miny = std::min({miny, g.a.y, g.b.y});
      maxy = std::max({maxy, g.a.y, g.b.y});
    }
    s = std::max({cell, (maxx - minx) / 512.0, (maxy - miny) / 512.0, 1e-300});
    inv = 1.0 / s;
    x0 = minx;
    y0 = miny;
    nx = (long)((maxx - minx) * inv) + 1;
    ny = (long)((maxy - miny) * inv) + 1;
    start.assign((size_t)(nx * ny + 1), 0);
    for (int pass = 0; pass < 2; pass++) {
      std::vector<uint32_t> fill;
      if (pass) {
        for (size_t q = 1; q < start.size(); q++) start[q] += start[q - 1];
        items.assign(start.back(), 0);
        fill.assign(start.begin(), start.end() - 1);
      }
      for (size_t k = 0; k < segs.size(); k++) {
        const long i0 = col(std::min(segs[k].a.x, segs[k].b.x)), i1 = col(std::max(segs[k].a.x, segs[k].b.x));
        const long j0 = row(std::min(segs[k].a.y, segs[k].b.y)), j1 = row(std::max(segs[k].a.y, segs[k].b.y));
        for (long j = j0; j <= j1; j++)
          for (long i = i0; i <= i1; i++) {
            const size_t q = (size_t)(j * nx + i);
            if (pass) items[fill[q]++] = (uint32_t)k;
            else start[q + 1]++;
          }
      }
    }
  }
  long col(double x) const { return std::min(std::max((long)std::floor((x - x0) * inv), 0L), nx - 1); }
  long row(double y) const { return std::min(std::max((long)std::floor((y - y0) * inv), 0L), ny - 1); }

  // signed winding count of the rightward ray from p (half-open in y), each crossing
  // counted in the bucket that holds its x
  int depth(XY p) const {
    if (segs.empty() || p.y < y0 || p.y > y0 + ny * s) return 0;
    const long j = row(p.y);
    int w = 0;
    for (long i = col(p.x); i < nx; i++) {
      const double bx0 = x0 + i * s, bx1 = i + 1 < nx ? x0 + (i + 1) * s : INFINITY;
      const size_t c = (size_t)(j * nx + i);
      for (uint32_t k = start[c]; k < start[c + 1]; k++) {
        const Seg& g = segs[items[k]];
        const bool up = g.a.y <= p.y && g.b.y > p.y, down = g.b.y <= p.y && g.a.y > p.y;
        if (!up && !down) continue;
        const double xi = (g.b.x - g.a.x) * (p.y - g.a.y) / (g.b.y - g.a.y) + g.a.x;
        if (p.x < xi && xi >= std::max(bx0, p.x) && xi < bx1) w += up ? g.sign : -g.sign;
      }
    }
    return w;
  }
  // distance from p to the nearest curve segment, or INFINITY when none is within q
  double min_dist(XY p, double q) const {
    if (segs.empty()) return INFINITY;
    double best = INFINITY;
    for (long j = row(p.y - q); j <= row(p.y + q); j++)
      for (long i = col(p.x - q); i <= col(p.x + q); i++) {
        const size_t c = (size_t)(j * nx + i);
        for (uint32_t k = start[c]; k < start[c + 1]; k++)
          best = std::min(best, point_to_segment(p, segs[items[k]].a, segs[items[k]].b));
      }
    return best <= q ? best : INFINITY;
  }
  // distance from p to the result's outline -- the pieces of curve segments (split where
  // other segments cross them) with depth >= 1 on exactly one side -- or INFINITY when no
  // outline piece is within q.  Curve pieces inside the result or outside it (the raw
  // curves' loops, the closing segments of inside turns) are not outline.
  double outline_dist(XY p, double q, double eps) const {
    if (segs.empty()) return INFINITY;
    std::vector<uint32_t> near;
    for (long j = row(p.y - q); j <= row(p.y + q); j++)
      for (long i = col(p.x - q); i <= col(p.x + q); i++) {
        const size_t c = (size_t)(j * nx + i);
        for (uint32_t k = start[c]; k < start[c + 1]; k++)
          if (point_to_segment(p, segs[items[k]].a, segs[items[k]].b) <= q) near.push_back(items[k]);
      }
    std::sort(near.begin(), near.end());
    near.erase(std::unique(near.begin(), near.end()), near.end());
    double best = INFINITY;
    std::vector<double> ts;
    std::vector<uint32_t> others;
    for (uint32_t k : near) {
      const Seg& g = segs[k];
      // every segment crossing g splits it
      ts.assign({0.0, 1.0});
      others.clear();
      for (long j = row(std::min(g.a.y, g.b.y)); j <= row(std::max(g.a.y, g.b.y)); j++)
        for (long i = col(std::min(g.a.x, g.b.x)); i <= col(std::max(g.a.x, g.b.x)); i++) {
          const size_t c = (size_t)(j * nx + i);
          for (uint32_t m = start[c]; m < start[c + 1]; m++)
            if (items[m] != k) others.push_back(items[m]);
        }
      std::sort(others.begin(), others.end());
      others.erase(std::unique(others.begin(), others.end()), others.end());
      const double dx = g.b.x - g.a.x, dy = g.b.y - g.a.y;
      for (uint32_t m : others) {
        const Seg& h = segs[m];
        const double ex = h.b.x - h.a.x, ey = h.b.y - h.a.y, den = dx * ey - dy * ex;
        if (den == 0) continue;
        const double t = ((h.a.x - g.a.x) * ey - (h.a.y - g.a.y) * ex) / den;
        const double u = ((h.a.x - g.a.x) * dy - (h.a.y - g.a.y) * dx) / den;
        if (t > 0 && t < 1 && u >= 0 && u <= 1) ts.push_back(t);
      }
      std::sort(ts.begin(), ts.end());
      const double len = std::sqrt(dx * dx + dy * dy);
      if (!(len > 0)) continue;
      const double ux = -dy / len * eps, uy = dx / len * eps;
      for (size_t a = 0; a + 1 < ts.size(); a++) {
        if (!(ts[a + 1] > ts[a])) continue;
        const XY pa{g.a.x + ts[a] * dx, g.a.y + ts[a] * dy}, pb{g.a.x + ts[a + 1] * dx, g.a.y + ts[a + 1] * dy};
        const double dd = point_to_segment(p, pa, pb);
        if (!(dd < best) || dd > q) continue;
        const XY m{(pa.x + pb.x) / 2, (pa.y + pb.y) / 2};
        const bool l = depth({m.x + ux, m.y + uy}) >= 1, r = depth({m.x - ux, m.y - uy}) >= 1;
        if (l != r) best = dd;
      }
    }
    return best;
  }
  // is {depth >= 1} non-empty?  Every face of the arrangement is bounded by curve
  // segments, so probing both sides of every segment at a few points finds one
  bool any_positive(double eps) const {
    for (auto& g : segs) {
      const double dx = g.b.x - g.a.x, dy = g.b.y - g.a.y, len = std::sqrt(dx * dx + dy * dy);
      if (!(len > 0)) continue;
      const double nx_ = -dy / len * eps, ny_ = dx / len * eps;
      for (double t : {0.5, 0.25, 0.75}) {
        const XY m{g.a.x + t * dx, g.a.y + t * dy};
        if (depth({m.x + nx_, m.y + ny_}) >= 1 || depth({m.x - nx_, m.y - ny_}) >= 1) return true;
      }
    }
    return false;
  }
};

// polygon parts: part[0] the shell, then holes; rings closed
using Rings = std::vector<std::vector<XY>>;

// geometry.buffer(-r) (OffsetCurveSetBuilder.addPolygon, distance < 0)
inline void carved_field(const std::vector<Rings>& parts, double r, DepthField& f) {
  for (auto& part : parts) {
    if (part.empty()) continue;
    if (eroded_completely(part[0], -r)) continue;
    const auto shell = remove_repeated(part[0]);
    if (shell.size() < 3) continue;
    f.add_ring_side(shell, r, kRight, kExterior, kInterior);
    for (size_t h = 1; h < part.size(); h++) {
      const auto hole = remove_repeated(part[h]);
      f.add_ring_side(hole, r, kLeft, kInterior, kExterior);
    }
  }
}

// geometry.boundary.buffer(d) (addLineString -> addRingBothSides per ring), or
// geometry.buffer(d) (addPolygon, distance > 0) when `whole`
inline void band_field(const std::vector<Rings>& parts, double d, bool whole, DepthField& f) {
  for (auto& part : parts) {
    for (size_t k = 0; k < part.size(); k++) {
      const auto ring = remove_repeated(part[k]);
      if (ring.size() < 4 || !same(ring.front(), ring.back())) continue;
      if (!whole) {
        f.add_ring_side(ring, d, kLeft, kExterior, kInterior);
        f.add_ring_side(ring, d, kRight, kInterior, kExterior);
      } else if (k == 0) {
        f.add_ring_side(ring, d, kLeft, kExterior, kInterior);
      } else if (!eroded_completely(part[k], -d)) {
        f.add_ring_side(ring, d, kRight, kInterior, kExterior);
      }
    }
  }
}

}  // namespace jtsbuf
}  // namespace mgpu
