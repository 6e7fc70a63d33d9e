// Border-chip geometry as JTS 1.20 OverlayNG computes `polygon INTERSECTION cell` in its
// floating-precision mode (Geometry.intersection -> OverlayNGRobust: MCIndexNoder with an
// IntersectionAdder over RobustLineIntersector, validated noding), restated for one cell.
// JTS is a Maven dependency of the reference (pom.xml:98-102), absent here; its call sites:
// IndexSystem.getBorderChips (core/index/IndexSystem.scala:184-188) ->
// MosaicGeometryJTS.intersection (core/geometry/MosaicGeometryJTS.scala:139-152, multi-part
// results through compactCollection :277-315) -> coerceChipGeometry (IndexSystem.scala:293-303).
//
// What decides the chip's point set, and is restated exactly:
//  * every node where a polygon segment meets a cell segment is RobustLineIntersector's
//    point for the two ORIGINAL segments: an endpoint when one lies on the other segment
//    (Orientation.index == 0, CGAlgorithmsDD's filtered / double-double sign), else
//    Intersection.intersection (homogeneous coordinates about the midpoint of the two
//    envelopes' overlap, every product rounded on its own), replaced by the nearest
//    endpoint when it falls outside either segment's envelope; collinear overlaps node at
//    the overlap's endpoints (computeCollinearIntersection);
//  * the noded edges between those nodes, each kept when it lies in the other geometry's
//    interior -- a polygon edge in the cell, a cell edge in the polygon, a shared edge when
//    both interiors lie on one side -- located at its nodes by the angular sectors of the
//    other geometry's edges there (OverlayLabeller's propagation around a node; exact
//    orientation tests), and by point location when it touches none of them;
//  * the result rings as OverlayNG's PolygonBuilder forms them: minimal rings (at a node
//    with several result edges the ring turns into the face on its right), shells
//    clockwise, holes counter-clockwise, each hole in the smallest shell holding it -- so
//    a chip that falls apart is a MULTIPOLYGON of separate pieces, never one ring bridged
//    along the cell boundary;
//  * coerceChipGeometry's `difference(indexGeom.getBoundary)` when the chip's type differs
//    from the polygon's (a MULTIPOLYGON zone giving a one-piece chip, a POLYGON giving
//    several) or the overlay also produced lines / points (the polygon touching the cell
//    from outside: OverlayNG's non-strict mode keeps them, compactCollection makes a
//    GEOMETRYCOLLECTION): that second overlay re-nodes the chip's edges against the cell's
//    boundary segments, and a chip edge that crosses a cell segment within rounding -- a
//    crossing node a few ulps outside the cell -- gains that node.
// Not restated (documented in DESIGN.md): OverlayNGRobust's fallbacks when the validating
// noder rejects the floating noding (snapping / snap-rounding noders), the ring start
// vertex of OverlayNG's output (bytes, not the point set), and compactCollection's union of
// the pieces (disjoint pieces: no new node).
#pragma once
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <vector>

#include "jts_orient.h"

namespace mgpu {
namespace ovl {

struct P {
  double x, y;
};
inline bool eq(P a, P b) { return a.x == b.x && a.y == b.y; }
inline bool less(P a, P b) { return a.x < b.x || (a.x == b.x && a.y < b.y); }
inline int orient(P a, P b, P c) { return mgpu::pip::orientation(a.x, a.y, b.x, b.y, c.x, c.y); }

// Envelope.intersects(p1, p2, q)
inline bool env_has(P p1, P p2, P q) {
  return q.x >= (p1.x < p2.x ? p1.x : p2.x) && q.x <= (p1.x > p2.x ? p1.x : p2.x) &&
         q.y >= (p1.y < p2.y ? p1.y : p2.y) && q.y <= (p1.y > p2.y ? p1.y : p2.y);
}
// Envelope.intersects(p1, p2, q1, q2)
inline bool env_meet(P p1, P p2, P q1, P q2) {
  double minq = std::min(q1.x, q2.x), maxq = std::max(q1.x, q2.x), minp = std::min(p1.x, p2.x),
         maxp = std::max(p1.x, p2.x);
  if (minp > maxq || maxp < minq) return false;
  minq = std::min(q1.y, q2.y), maxq = std::max(q1.y, q2.y), minp = std::min(p1.y, p2.y), maxp = std::max(p1.y, p2.y);
  return !(minp > maxq || maxp < minq);
}

// Intersection.intersection (JTS 1.20 algorithm/Intersection.java); false = parallel (null)
inline bool hom_intersection(P p1, P p2, P q1, P q2, P* out) {
  const double minX0 = p1.x < p2.x ? p1.x : p2.x, minY0 = p1.y < p2.y ? p1.y : p2.y;
  const double maxX0 = p1.x > p2.x ? p1.x : p2.x, maxY0 = p1.y > p2.y ? p1.y : p2.y;
  const double minX1 = q1.x < q2.x ? q1.x : q2.x, minY1 = q1.y < q2.y ? q1.y : q2.y;
  const double maxX1 = q1.x > q2.x ? q1.x : q2.x, maxY1 = q1.y > q2.y ? q1.y : q2.y;
  const double intMinX = minX0 > minX1 ? minX0 : minX1, intMaxX = maxX0 < maxX1 ? maxX0 : maxX1;
  const double intMinY = minY0 > minY1 ? minY0 : minY1, intMaxY = maxY0 < maxY1 ? maxY0 : maxY1;
  const double midx = (intMinX + intMaxX) / 2.0, midy = (intMinY + intMaxY) / 2.0;
  const double p1x = p1.x - midx, p1y = p1.y - midy, p2x = p2.x - midx, p2y = p2.y - midy;
  const double q1x = q1.x - midx, q1y = q1.y - midy, q2x = q2.x - midx, q2y = q2.y - midy;
  const double px = p1y - p2y, py = p2x - p1x, pw = p1x * p2y - p2x * p1y;
  const double qx = q1y - q2y, qy = q2x - q1x, qw = q1x * q2y - q2x * q1y;
  const double x = py * qw - qy * pw, y = qx * pw - px * qw, w = px * qy - qx * py;
  const double xi = x / w, yi = y / w;
  if (std::isnan(xi) || std::isinf(xi) || std::isnan(yi) || std::isinf(yi)) return false;
  *out = {xi + midx, yi + midy};
  return true;
}

// Distance.pointToSegment (Coordinate.distance = Math.hypot)
inline double point_to_segment(P p, P a, P b) {
  if (a.x == b.x && a.y == b.y) return std::hypot(p.x - a.x, p.y - a.y);
  const double len2 = (b.x - a.x) * (b.x - a.x) + (b.y - a.y) * (b.y - a.y);
  const double r = ((p.x - a.x) * (b.x - a.x) + (p.y - a.y) * (b.y - a.y)) / len2;
  if (r <= 0.0) return std::hypot(p.x - a.x, p.y - a.y);
  if (r >= 1.0) return std::hypot(p.x - b.x, p.y - b.y);
  const double s = ((a.y - p.y) * (b.x - a.x) - (a.x - p.x) * (b.y - a.y)) / len2;
  return std::fabs(s) * std::sqrt(len2);
}

// RobustLineIntersector.nearestEndpoint
inline P nearest_endpoint(P p1, P p2, P q1, P q2) {
  P best = p1;
  double m = point_to_segment(p1, q1, q2), d;
  if ((d = point_to_segment(p2, q1, q2)) < m) m = d, best = p2;
  if ((d = point_to_segment(q1, p1, p2)) < m) m = d, best = q1;
  if ((d = point_to_segment(q2, p1, p2)) < m) m = d, best = q2;
  return best;
}

// RobustLineIntersector.computeIntersect: n points (0, 1 or 2 for a collinear overlap)
struct Hit {
  int n = 0;
  bool proper = false;
  P pt[2];
};
inline Hit line_intersect(P p1, P p2, P q1, P q2) {
  Hit h;
  if (!env_meet(p1, p2, q1, q2)) return h;
  const int Pq1 = orient(p1, p2, q1), Pq2 = orient(p1, p2, q2);
  if ((Pq1 > 0 && Pq2 > 0) || (Pq1 < 0 && Pq2 < 0)) return h;
  const int Qp1 = orient(q1, q2, p1), Qp2 = orient(q1, q2, p2);
  if ((Qp1 > 0 && Qp2 > 0) || (Qp1 < 0 && Qp2 < 0)) return h;
  if (Pq1 == 0 && Pq2 == 0 && Qp1 == 0 && Qp2 == 0) {  // computeCollinearIntersection
    const bool q1inP = env_has(p1, p2, q1), q2inP = env_has(p1, p2, q2);
    const bool p1inQ = env_has(q1, q2, p1), p2inQ = env_has(q1, q2, p2);
    auto two = [&](P a, P b, bool point) {
      h.pt[0] = a, h.pt[1] = b, h.n = point ? 1 : 2;
    };
    if (q1inP && q2inP) two(q1, q2, false);
    else if (p1inQ && p2inQ) two(p1, p2, false);
    else if (q1inP && p1inQ) two(q1, p1, eq(q1, p1) && !q2inP && !p2inQ);
    else if (q1inP && p2inQ) two(q1, p2, eq(q1, p2) && !q2inP && !p1inQ);
    else if (q2inP && p1inQ) two(q2, p1, eq(q2, p1) && !q1inP && !p2inQ);
    else if (q2inP && p2inQ) two(q2, p2, eq(q2, p2) && !q1inP && !p1inQ);
    return h;
  }
  h.n = 1;
  if (Pq1 == 0 || Pq2 == 0 || Qp1 == 0 || Qp2 == 0) {
    if (eq(p1, q1) || eq(p1, q2)) h.pt[0] = p1;
    else if (eq(p2, q1) || eq(p2, q2)) h.pt[0] = p2;
    else if (Pq1 == 0) h.pt[0] = q1;
    else if (Pq2 == 0) h.pt[0] = q2;
    else if (Qp1 == 0) h.pt[0] = p1;
    else h.pt[0] = p2;
    return h;
  }
  h.proper = true;
  P ip;
  if (!hom_intersection(p1, p2, q1, q2, &ip)) ip = nearest_endpoint(p1, p2, q1, q2);
  // isInSegmentEnvelopes, else the nearest endpoint
  if (!(env_has(p1, p2, ip) && env_has(q1, q2, ip))) ip = nearest_endpoint(p1, p2, q1, q2);
  h.pt[0] = ip;
  return h;
}

// Octant.octant and SegmentPointComparator.compare: the order of nodes along a segment
inline int octant(double dx, double dy) {
  const double adx = std::fabs(dx), ady = std::fabs(dy);
  if (dx >= 0) {
    if (dy >= 0) return adx >= ady ? 0 : 1;
    return adx >= ady ? 7 : 6;
  }
  if (dy >= 0) return adx >= ady ? 3 : 2;
  return adx >= ady ? 4 : 5;
}
inline int rel(double a, double b) { return a < b ? -1 : (a > b ? 1 : 0); }
inline int cmp_value(int a, int b) { return a < 0 ? -1 : a > 0 ? 1 : b < 0 ? -1 : b > 0 ? 1 : 0; }
inline int seg_compare(int oct, P p0, P p1) {
  if (eq(p0, p1)) return 0;
  const int xs = rel(p0.x, p1.x), ys = rel(p0.y, p1.y);
  switch (oct) {
    case 0: return cmp_value(xs, ys);
    case 1: return cmp_value(ys, xs);
    case 2: return cmp_value(ys, -xs);
    case 3: return cmp_value(-xs, ys);
    case 4: return cmp_value(-xs, -ys);
    case 5: return cmp_value(-ys, -xs);
    case 6: return cmp_value(-ys, xs);
    default: return cmp_value(xs, -ys);
  }
}

// Is direction d strictly inside the counter-clockwise sweep from direction a to
// direction b (all about the origin point o; a and b not parallel-same)?  Exact: the
// directions are the points A, B, D themselves.
inline int half(P o, P ref, P d) {  // 0: d in [ref, ref + 180), 1: otherwise
  const int s = orient(o, ref, d);
  if (s > 0) return 0;
  if (s < 0) return 1;
  // collinear with the ray o -> ref: same direction (0) or opposite (1)
  return ((d.x - o.x) * (ref.x - o.x) + (d.y - o.y) * (ref.y - o.y)) > 0 ? 0 : 1;
}
// ccw angle from ref to u is smaller than to v
inline bool ccw_before(P o, P ref, P u, P v) {
  const int hu = half(o, ref, u), hv = half(o, ref, v);
  if (hu != hv) return hu < hv;
  return orient(o, u, v) > 0;
}
// strictly between: a < d < b in ccw angle from a (d not on either ray)
inline bool in_sector(P o, P a, P b, P d) {
  if (orient(o, a, d) == 0 && half(o, a, d) == 0) return false;
  if (orient(o, b, d) == 0 && half(o, b, d) == 0) return false;
  if (eq(a, b) || (orient(o, a, b) == 0 && half(o, a, b) == 0)) return true;  // (a full turn)
  return ccw_before(o, a, d, b);
}

// One cell overlay.  Cell rings: closed, counter-clockwise (each a part of the cell).
// Subject: parts of rings (first = shell), closed; only segments meeting the cell's
// envelope take part.
struct Overlay {
  struct Seg {  // an input segment near the cell
    P a, b;
    int geom;     // 0 = subject, 1 = cell
    int ring;     // ring id within its geometry (subject: global ring index)
    bool int_left;  // the geometry's interior lies left of a -> b
    int k = 0;      // the segment's index in its ring
  };
  struct Edge {  // a noded sub-edge
    int u, v;      // node ids
    int geom, ring;
    bool int_left;
    int partner = -1;  // the coincident edge of the other geometry
    bool in_result = false, res_left = false;  // result interior left of u -> v
  };
  std::vector<Seg> segs;
  std::vector<std::pair<int, P>> seg_nodes;  // (seg, node found on it)
  std::vector<P> nodes;                   // node coordinates (sorted unique)
  std::vector<uint8_t> on_geom;           // per node: bit 0 subject, bit 1 cell boundary
  std::vector<Edge> edges;
  // subject part / hole bookkeeping of rings: ring -> part, is hole, is ccw
  std::vector<int> ring_part;
  std::vector<uint8_t> ring_hole;
  bool lower_dim = false;  // the overlay also produced lines / points (touching)

  void clear() {
    segs.clear();
    seg_nodes.clear();
    nodes.clear();
    on_geom.clear();
    edges.clear();
    lower_dim = false;
  }
  int node_id(P p) const {
    auto it = std::lower_bound(nodes.begin(), nodes.end(), p, [](P a, P b) { return less(a, b); });
    return (int)(it - nodes.begin());
  }
};

// shoelace about the first vertex (absolute coordinates would cancel a chip's area away)
inline double signed_area(const std::vector<P>& r) {
  if (r.size() < 4) return 0;
  const double x0 = r[0].x, y0 = r[0].y;
  double a = 0;
  for (size_t i = 1; i + 2 < r.size(); i++)
    a += (r[i].x - x0) * (r[i + 1].y - y0) - (r[i + 1].x - x0) * (r[i].y - y0);
  return 0.5 * a;
}

// Orientation.isCCW (JTS 1.20): the first highest point after a rising segment, the cap
// there by orientation index (or a flat cap's direction); a flat ring is not ccw
inline bool is_ccw(const std::vector<P>& ring) {
  const int n = (int)ring.size() - 1;
  if (n < 3) return false;
  P upHi = ring[0], upLow{};
  double prevY = upHi.y;
  int iUpHi = 0;
  for (int i = 1; i <= n; i++) {
    const double py = ring[i].y;
    if (py > prevY && py >= upHi.y) {
      upHi = ring[i];
      iUpHi = i;
      upLow = ring[i - 1];
    }
    prevY = py;
  }
  if (iUpHi == 0) return false;
  int iDownLow = iUpHi;
  do {
    iDownLow = (iDownLow + 1) % n;
  } while (iDownLow != iUpHi && ring[iDownLow].y == upHi.y);
  const P downLow = ring[iDownLow];
  const P downHi = ring[iDownLow > 0 ? iDownLow - 1 : n - 1];
  if (eq(upHi, downHi)) {
    if (eq(upLow, upHi) || eq(downLow, upHi) || eq(upLow, downLow)) return false;
    return orient(upLow, upHi, downLow) > 0;
  }
  return downHi.x - upHi.x < 0;
}

// JTS PointLocation.locateInRing (RayCrossingCounter): 1 interior, 0 boundary, -1 exterior
inline int locate_in_ring(P p, const std::vector<P>& ring) {
  int crossings = 0;
  for (size_t i = 1; i < ring.size(); i++) {
    const P p1 = ring[i - 1], p2 = ring[i];
    if (p1.x < p.x && p2.x < p.x) continue;
    if (eq(p, p2)) return 0;
    if (p1.y == p.y && p2.y == p.y) {
      double mn = p1.x, mx = p2.x;
      if (mn > mx) std::swap(mn, mx);
      if (p.x >= mn && p.x <= mx) return 0;
      continue;
    }
    if ((p1.y > p.y && p2.y <= p.y) || (p2.y > p.y && p1.y <= p.y)) {
      int o = orient(p1, p2, p);
      if (o == 0) return 0;
      if (p2.y < p1.y) o = -o;
      if (o > 0) crossings++;
    }
  }
  return (crossings & 1) ? 1 : -1;
}

// A polygon's segments bucketed on a uniform grid (one per polygon, built once): the
// segments whose envelope meets a box, each once, in (ring, index) order -- the overlay
// then visits the segments near a cell instead of all of them.
struct SegGrid {
  double x0 = 0, y0 = 0, inv = 1;
  long nx = 0, ny = 0;
  std::vector<uint32_t> start;
  std::vector<uint64_t> items;  // ring << 32 | index
  mutable std::vector<uint64_t> out;
  // the last query's box while `out` still holds its result (a cell's inside test and its
  // overlay ask for the same box in a row)
  mutable double qb[4] = {0, 0, 0, 0};
  mutable bool q_valid = false;

  void build(const std::vector<std::vector<std::vector<P>>>& parts, double cell) {
    double minx = INFINITY, miny = INFINITY, maxx = -INFINITY, maxy = -INFINITY;
    size_t nseg = 0;
    for (auto& part : parts)
      for (auto& r : part)
        for (auto& p : r) {
          minx = std::min(minx, p.x), maxx = std::max(maxx, p.x);
          miny = std::min(miny, p.y), maxy = std::max(maxy, p.y);
          nseg++;
        }
    if (!(minx <= maxx)) return;
    double s = std::max({cell, (maxx - minx) / 1024.0, (maxy - miny) / 1024.0, 1e-300});
    // (at most ~4 buckets per segment on average)
    s = std::max(s, std::sqrt((maxx - minx) * (maxy - miny) / (4.0 * (double)nseg + 1.0)));
    inv = 1.0 / s;
    x0 = minx, y0 = miny;
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
      uint32_t ring = 0;
      for (auto& part : parts)
        for (auto& r : part) {
          for (size_t k = 0; k + 1 < r.size(); k++) {
            const long i0 = col(std::min(r[k].x, r[k + 1].x)), i1 = col(std::max(r[k].x, r[k + 1].x));
            const long j0 = row(std::min(r[k].y, r[k + 1].y)), j1 = row(std::max(r[k].y, r[k + 1].y));
            for (long j = j0; j <= j1; j++)
              for (long i = i0; i <= i1; i++) {
                const size_t q = (size_t)(j * nx + i);
                if (pass) items[fill[q]++] = ((uint64_t)ring << 32) | (uint64_t)k;
                else start[q + 1]++;
              }
          }
          ring++;
        }
    }
  }
  long col(double x) const { return std::min(std::max((long)std::floor((x - x0) * inv), 0L), nx - 1); }
  long row(double y) const { return std::min(std::max((long)std::floor((y - y0) * inv), 0L), ny - 1); }
  // the segments in buckets meeting [bx0, bx1] x [by0, by1], sorted, each once
  const std::vector<uint64_t>& query(double bx0, double by0, double bx1, double by1) const {
    if (q_valid && qb[0] == bx0 && qb[1] == by0 && qb[2] == bx1 && qb[3] == by1) return out;
    out.clear();
    q_valid = false;
    if (start.empty()) return out;
    for (long j = row(by0); j <= row(by1); j++)
      for (long i = col(bx0); i <= col(bx1); i++) {
        const size_t c = (size_t)(j * nx + i);
        out.insert(out.end(), items.begin() + start[c], items.begin() + start[c + 1]);
      }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    qb[0] = bx0, qb[1] = by0, qb[2] = bx1, qb[3] = by1;
    q_valid = true;
    return out;
  }
  // the segments a rightward ray from (px, py) can meet or (px, py) can lie on: a segment
  // whose envelope spans py and reaches x >= px is in py's bucket row at or right of
  // px's bucket (clamping keeps both monotone) -- sorted, each once
  const std::vector<uint64_t>& ray_right(double px, double py) const {
    out.clear();
    q_valid = false;
    if (start.empty()) return out;
    const long j = row(py);
    for (long i = col(px); i < nx; i++) {
      const size_t c = (size_t)(j * nx + i);
      out.insert(out.end(), items.begin() + start[c], items.begin() + start[c + 1]);
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
  }
  // PointLocation.locateInRing (locate_in_ring below) of p in every ring at once, from the
  // ray_right segments only (the others are skipped by its first test or cross nothing):
  // loc[ring] = 1 interior, 0 boundary, -1 exterior
  void locate_rings(P p, const std::vector<const std::vector<P>*>& rings, std::vector<int8_t>& loc,
                    std::vector<int>& cross) const {
    loc.assign(rings.size(), -1);
    cross.assign(rings.size(), 0);
    for (uint64_t c : ray_right(p.x, p.y)) {
      const size_t r = (size_t)(c >> 32), k = (size_t)(c & 0xFFFFFFFFu);
      if (loc[r] == 0) continue;
      const P p1 = (*rings[r])[k], p2 = (*rings[r])[k + 1];
      if (p1.x < p.x && p2.x < p.x) continue;
      if (eq(p, p2)) {
        loc[r] = 0;
        continue;
      }
      if (p1.y == p.y && p2.y == p.y) {
        double mn = p1.x, mx = p2.x;
        if (mn > mx) std::swap(mn, mx);
        if (p.x >= mn && p.x <= mx) loc[r] = 0;
        continue;
      }
      if ((p1.y > p.y && p2.y <= p.y) || (p2.y > p.y && p1.y <= p.y)) {
        int o = orient(p1, p2, p);
        if (o == 0) {
          loc[r] = 0;
          continue;
        }
        if (p2.y < p1.y) o = -o;
        if (o > 0) cross[r]++;
      }
    }
    for (size_t r = 0; r < rings.size(); r++)
      if (loc[r] != 0) loc[r] = (cross[r] & 1) ? 1 : -1;
  }
};

// The result of one overlay: pieces (rings; ring 0 = shell, clockwise; holes ccw)
using Rings = std::vector<std::vector<P>>;

// test hook (mgpu_test_overlay_verify): when on, every cell the one-chain shortcut answers
// is also run through the general graph and the two results compared
struct OverlayVerify {
  std::atomic<bool> on{false};
  std::atomic<int64_t> shortcut{0}, differ{0};
};
inline OverlayVerify g_overlay_verify;

// polygon (parts of closed rings) INTERSECTION cell (closed ccw rings), as OverlayNG
// (header).  `whole_subject_rings[r]` must hold every subject ring (for point location);
// ring_ccw[r] its orientation.  Returns the pieces; *lower_dim when the overlay also
// produced lines or points.
struct Clipper {
  Overlay o;
  // scratch
  std::vector<int> out_start, out_list, cell_edge_begin, fill, prts, rs;
  std::vector<uint8_t> used;
  std::vector<P> pts;
  std::vector<std::pair<P, P>> sub;  // (from, to) coordinates
  std::vector<int> sub_seg;
  std::vector<int8_t> loc;
  std::vector<int> cand;  // candidate subject segments (ring << 32 | k) from the grid
  std::vector<uint64_t> cand64;
  std::vector<const std::vector<P>*> sub_rings;
  std::vector<int8_t> rloc;
  std::vector<int> rcross;
  // (the result-ring stage's scratch, reused across calls)
  std::vector<std::pair<int, int>> res;
  std::vector<P> tmp_chain, tmp_cycle, tmp_sorted;
  std::vector<uint8_t> touched;
  std::vector<int> rs_start, rs_list, rs_fill, shells, holes;
  std::vector<double> rarea;

  // the one-chain shortcut below (off: always the general noded graph)
  bool fast = true;

  // The commonest border cell: one ring of the subject crosses the cell's one ring twice,
  // both proper crossings (interiors of both segments, points off every endpoint), and the
  // subject's segments between them -- the same ring, in ring order -- are the only ones
  // inside.  The general graph below then labels exactly those subject edges and the cell
  // arc on the interior's side, and walks one ring: here it is written down directly, in
  // the order and from the node the graph's walk starts at (the first result edge in edge
  // order).  False (nothing written) when the configuration is anything else.
  bool one_crossing_chain(const std::vector<std::vector<std::vector<P>>>& parts, const std::vector<std::vector<P>>& cell,
                          std::vector<Rings>& pieces) {
    const int n_sub = (int)o.segs.size() - [&] {
      int c = 0;
      for (auto& sg : o.segs) c += sg.geom == 1;
      return c;
    }();
    // the two crossings: (subject seg, cell seg, point), in seg_nodes order
    const int s0 = o.seg_nodes[0].first, c0 = o.seg_nodes[1].first, s1 = o.seg_nodes[2].first, c1 = o.seg_nodes[3].first;
    const P h0 = o.seg_nodes[0].second, h1 = o.seg_nodes[2].second;
    if (eq(h0, h1)) return false;
    for (int q = 0; q < 2; q++) {
      const P h = q ? h1 : h0;
      const Overlay::Seg &ss = o.segs[q ? s1 : s0], &cs = o.segs[q ? c1 : c0];
      if (eq(h, ss.a) || eq(h, ss.b) || eq(h, cs.a) || eq(h, cs.b)) return false;
    }
    const std::vector<P>& cr = cell[0];
    const int ring = o.segs[s0].ring;
    if (o.segs[s1].ring != ring) return false;
    const std::vector<P>& R = *sub_rings[ring];
    const int nr = (int)R.size() - 1;  // segments of the ring
    // locations of the subject segs' start points (no crossing: the whole seg is there)
    int entry = -1, exit_ = -1;  // subject seg indices in o.segs
    P in_pt{}, out_pt{};
    int in_cell = -1, out_cell = -1;
    int n_inside = 0;
    for (int i = 0; i < n_sub; i++) {
      const int l = locate_in_ring(o.segs[i].a, cr);
      if (l == 0) return false;
      const bool a_in = l > 0;
      const bool hit0 = i == s0, hit1 = i == s1;
      if (hit0 && hit1) {  // both crossings on one seg: it enters and leaves
        if (a_in) return false;
        // the first along the seg enters
        const int oc = octant(o.segs[i].b.x - o.segs[i].a.x, o.segs[i].b.y - o.segs[i].a.y);
        const bool first0 = seg_compare(oc, h0, h1) < 0;
        entry = exit_ = i;
        in_pt = first0 ? h0 : h1, in_cell = first0 ? c0 : c1;
        out_pt = first0 ? h1 : h0, out_cell = first0 ? c1 : c0;
      } else if (hit0 || hit1) {
        const P h = hit0 ? h0 : h1;
        const int c = hit0 ? c0 : c1;
        if (!a_in) {
          if (entry >= 0) return false;
          entry = i, in_pt = h, in_cell = c;
        } else {
          if (exit_ >= 0) return false;
          exit_ = i, out_pt = h, out_cell = c;
        }
      } else if (a_in) {
        if (o.segs[i].ring != ring) return false;
        n_inside++;
      }
    }
    if (entry < 0 || exit_ < 0) return false;
    const int ke = o.segs[entry].k, kx = o.segs[exit_].k;
    // the chain: entry's end, the ring's vertices up to exit's start (degenerate segments
    // skipped, as the graph's segments are); every seg strictly between is inside
    std::vector<P>& chain = tmp_chain;
    chain.clear();
    chain.push_back(in_pt);
    int n_between = 0;
    if (entry != exit_) {
      for (int k = (ke + 1) % nr;; k = (k + 1) % nr) {
        if (!eq(R[k], chain.back())) chain.push_back(R[k]);
        if (k == kx) break;
        if (!eq(R[k], R[k + 1])) n_between++;
        if ((int)chain.size() > nr + 2) return false;
      }
    }
    if (n_between != n_inside) return false;
    chain.push_back(out_pt);
    // the cell side: cell segs are o.segs[n_sub ..], in ring order; the arc clockwise (the
    // result's interior on the right) from the chain's last point to its first
    const bool int_left = o.segs[entry].int_left;  // (one ring: one orientation)
    std::vector<P>& cyc = tmp_cycle;
    cyc.clear();
    P first = chain.front(), last = chain.back();
    int c_first = in_cell, c_last = out_cell;
    if (int_left) {  // result direction: the chain reversed
      std::reverse(chain.begin(), chain.end());
      std::swap(first, last);
      std::swap(c_first, c_last);
    }
    for (auto& q : chain) cyc.push_back(q);
    const int nc = (int)o.segs.size() - n_sub;
    const int jl = c_last - n_sub, jf = c_first - n_sub;
    bool direct = false;  // both on one cell seg with `first` before `last` clockwise
    if (jl == jf) {
      const Overlay::Seg& cs = o.segs[c_last];
      const int oc = octant(cs.b.x - cs.a.x, cs.b.y - cs.a.y);
      direct = seg_compare(oc, first, last) < 0;  // clockwise = against the seg's direction
    }
    if (!direct) {
      // clockwise from `last`: the start of its seg, then the previous segs' starts, down
      // to the end of first's seg
      int j = jl;
      for (int guard = 0; guard <= nc; guard++) {
        cyc.push_back(o.segs[n_sub + j].a);
        j = (j + nc - 1) % nc;
        if (j == jf) break;
        if (guard == nc) return false;
      }
    }
    if (cyc.size() < 3) return false;
    // distinct nodes (the graph would merge equal ones)
    tmp_sorted.assign(cyc.begin(), cyc.end());
    std::sort(tmp_sorted.begin(), tmp_sorted.end(), [](P a, P b) { return less(a, b); });
    for (size_t q = 1; q < tmp_sorted.size(); q++)
      if (eq(tmp_sorted[q], tmp_sorted[q - 1])) return false;
    // the walk starts at the first result edge in edge order: the subject edges come first,
    // by seg (o.segs order), each seg's sub-edges along it; a result edge runs (v, u) when
    // the interior is left of the subject direction, so it starts at the sub-edge's end
    int first_seg = entry;
    if (exit_ < first_seg) first_seg = exit_;
    for (int i = 0; i < n_sub; i++)
      if (i < first_seg && o.segs[i].ring == ring && locate_in_ring(o.segs[i].a, cr) > 0) {
        first_seg = i;
        break;
      }
    P u, v;  // the first inside sub-edge of first_seg, in subject direction
    if (first_seg == entry && entry == exit_) u = in_pt, v = out_pt;
    else if (first_seg == entry) u = in_pt, v = o.segs[entry].b;
    else if (first_seg == exit_) u = o.segs[exit_].a, v = out_pt;
    else u = o.segs[first_seg].a, v = o.segs[first_seg].b;
    const P start = int_left ? v : u;
    size_t s0i = cyc.size();
    for (size_t q = 0; q < cyc.size(); q++)
      if (eq(cyc[q], start)) {
        s0i = q;
        break;
      }
    if (s0i == cyc.size()) return false;
    std::vector<P> out;
    out.reserve(cyc.size() + 1);
    for (size_t q = 0; q < cyc.size(); q++) out.push_back(cyc[(s0i + q) % cyc.size()]);
    out.push_back(out[0]);
    if (is_ccw(out)) return false;  // (the graph would call it a hole)
    pieces.clear();
    pieces.push_back(Rings{std::move(out)});
    return true;
  }

  void build(const std::vector<std::vector<std::vector<P>>>& parts, const std::vector<uint8_t>& ring_ccw,
             const std::vector<std::vector<P>>& cell, std::vector<Rings>& pieces, bool* lower_dim,
             const SegGrid* grid = nullptr) {
    o.clear();
    pieces.clear();
    double cx0 = INFINITY, cy0 = INFINITY, cx1 = -INFINITY, cy1 = -INFINITY;
    for (auto& r : cell)
      for (auto& p : r) {
        cx0 = std::min(cx0, p.x), cx1 = std::max(cx1, p.x);
        cy0 = std::min(cy0, p.y), cy1 = std::max(cy1, p.y);
      }
    // 1. segments near the cell (repeated points dropped, as EdgeNodingBuilder does)
    o.ring_part.clear();
    o.ring_hole.clear();
    int ring_id = 0;
    sub_rings.clear();
    for (size_t pi = 0; pi < parts.size(); pi++)
      for (size_t ri = 0; ri < parts[pi].size(); ri++, ring_id++) {
        sub_rings.push_back(&parts[pi][ri]);
        o.ring_part.push_back((int)pi);
        o.ring_hole.push_back(ri > 0);
      }
    // interior of the polygon left of the ring's direction: shell ccw, hole cw
    auto add_seg = [&](int rid, size_t k) {
      const auto& r = *sub_rings[rid];
      const P a = r[k], b = r[k + 1];
      if (eq(a, b)) return;
      if (std::max(a.x, b.x) < cx0 || std::min(a.x, b.x) > cx1 || std::max(a.y, b.y) < cy0 || std::min(a.y, b.y) > cy1)
        return;
      o.segs.push_back({a, b, 0, rid, (o.ring_hole[rid] == 0) == (bool)ring_ccw[rid], (int)k});
    };
    if (grid) {
      for (uint64_t c : grid->query(cx0, cy0, cx1, cy1)) add_seg((int)(c >> 32), (size_t)(c & 0xFFFFFFFFu));
    } else {
      for (int rid = 0; rid < ring_id; rid++)
        for (size_t k = 0; k + 1 < sub_rings[rid]->size(); k++) add_seg(rid, k);
    }
    const size_t n_sub = o.segs.size();
    for (size_t ci = 0; ci < cell.size(); ci++)
      for (size_t k = 0; k + 1 < cell[ci].size(); k++)
        if (!eq(cell[ci][k], cell[ci][k + 1])) o.segs.push_back({cell[ci][k], cell[ci][k + 1], 1, (int)ci, true, (int)k});
    // 2. noding: every subject segment against every cell segment (IntersectionAdder)
    o.seg_nodes.clear();
    bool all_proper = true;
    for (size_t i = 0; i < n_sub; i++)
      for (size_t j = n_sub; j < o.segs.size(); j++) {
        const Hit h = line_intersect(o.segs[i].a, o.segs[i].b, o.segs[j].a, o.segs[j].b);
        if (h.n && (h.n != 1 || !h.proper)) all_proper = false;
        for (int q = 0; q < h.n; q++) {
          o.seg_nodes.push_back({(int)i, h.pt[q]});
          o.seg_nodes.push_back({(int)j, h.pt[q]});
        }
      }
    if (fast && all_proper && cell.size() == 1 && o.seg_nodes.size() == 4 && one_crossing_chain(parts, cell, pieces)) {
      *lower_dim = false;
      if (g_overlay_verify.on.load(std::memory_order_relaxed)) {
        g_overlay_verify.shortcut++;
        std::vector<Rings> gp;
        bool gl = false;
        fast = false;
        build(parts, ring_ccw, cell, gp, &gl, grid);
        fast = true;
        bool same = !gl && gp.size() == pieces.size();
        for (size_t a = 0; same && a < gp.size(); a++) {
          same = gp[a].size() == pieces[a].size();
          for (size_t r = 0; same && r < gp[a].size(); r++) {
            same = gp[a][r].size() == pieces[a][r].size();
            for (size_t q = 0; same && q < gp[a][r].size(); q++) same = eq(gp[a][r][q], pieces[a][r][q]);
          }
        }
        if (!same) g_overlay_verify.differ++;
      }
      return;
    }
    // 3. sub-edges between consecutive nodes along each segment (nodes by segment, then
    // in SegmentPointComparator order along it)
    std::sort(o.seg_nodes.begin(), o.seg_nodes.end(), [&](const std::pair<int, P>& u, const std::pair<int, P>& v) {
      if (u.first != v.first) return u.first < v.first;
      const Overlay::Seg& s = o.segs[u.first];
      return seg_compare(octant(s.b.x - s.a.x, s.b.y - s.a.y), u.second, v.second) < 0;
    });
    pts.clear();
    sub.clear();
    sub_seg.clear();
    size_t nq = 0;
    for (size_t i = 0; i < o.segs.size(); i++) {
      const Overlay::Seg& s = o.segs[i];
      pts.clear();
      pts.push_back(s.a);
      for (; nq < o.seg_nodes.size() && o.seg_nodes[nq].first == (int)i; nq++) {
        const P p = o.seg_nodes[nq].second;
        if (!eq(p, pts.back()) && !eq(p, s.b)) pts.push_back(p);
      }
      pts.push_back(s.b);
      for (size_t k = 0; k + 1 < pts.size(); k++) {
        sub.push_back({pts[k], pts[k + 1]});
        sub_seg.push_back((int)i);
      }
    }
    // node ids
    o.nodes.clear();
    for (auto& e : sub) {
      o.nodes.push_back(e.first);
      o.nodes.push_back(e.second);
    }
    // (lambdas: the comparisons inline)
    std::sort(o.nodes.begin(), o.nodes.end(), [](P a, P b) { return less(a, b); });
    o.nodes.erase(std::unique(o.nodes.begin(), o.nodes.end(), [](P a, P b) { return eq(a, b); }), o.nodes.end());
    o.on_geom.assign(o.nodes.size(), 0);
    o.edges.clear();
    cell_edge_begin.assign(cell.size() + 1, (int)sub.size());
    for (size_t k = sub.size(); k-- > 0;) {
      const Overlay::Seg& s = o.segs[sub_seg[k]];
      if (s.geom == 1) cell_edge_begin[s.ring] = (int)k;
    }
    for (size_t ci = cell.size(); ci-- > 0;)
      if (cell_edge_begin[ci] > cell_edge_begin[ci + 1]) cell_edge_begin[ci] = cell_edge_begin[ci + 1];
    for (size_t k = 0; k < sub.size(); k++) {
      const Overlay::Seg& s = o.segs[sub_seg[k]];
      Overlay::Edge e;
      e.u = o.node_id(sub[k].first);
      e.v = o.node_id(sub[k].second);
      e.geom = s.geom, e.ring = s.ring, e.int_left = s.int_left;
      o.on_geom[e.u] |= (uint8_t)(1 << s.geom);
      o.on_geom[e.v] |= (uint8_t)(1 << s.geom);
      o.edges.push_back(e);
    }
    // incidence (both directions) per node
    const int nn = (int)o.nodes.size(), ne = (int)o.edges.size();
    out_start.assign(nn + 1, 0);
    for (auto& e : o.edges) out_start[e.u + 1]++, out_start[e.v + 1]++;
    for (int q = 0; q < nn; q++) out_start[q + 1] += out_start[q];
    out_list.assign(out_start[nn], 0);
    fill.assign(out_start.begin(), out_start.end() - 1);
    for (int k = 0; k < ne; k++) {
      out_list[fill[o.edges[k].u]++] = k;
      out_list[fill[o.edges[k].v]++] = k;
    }
    // 4. coincident edges of the two geometries (EdgeMerger)
    for (int q = 0; q < nn; q++)
      for (int a = out_start[q]; a < out_start[q + 1]; a++)
        for (int b = a + 1; b < out_start[q + 1]; b++) {
          Overlay::Edge &e = o.edges[out_list[a]], &f = o.edges[out_list[b]];
          if (e.geom == f.geom) continue;
          if ((e.u == f.u && e.v == f.v) || (e.u == f.v && e.v == f.u)) {
            e.partner = out_list[b];
            f.partner = out_list[a];
          }
        }
    // 5. location of each edge in the other geometry
    // the ring neighbours of a node on one ring of geometry g: the other endpoints of that
    // ring's edges incident to the node (prev: the edge ending there, next: starting)
    auto ring_at = [&](int node, int geom, int ring, P* prev, P* next) {
      bool hp = false, hn = false;
      for (int a = out_start[node]; a < out_start[node + 1]; a++) {
        const Overlay::Edge& e = o.edges[out_list[a]];
        if (e.geom != geom || e.ring != ring) continue;
        if (e.v == node && !hp) *prev = o.nodes[e.u], hp = true;
        if (e.u == node && !hn) *next = o.nodes[e.v], hn = true;
      }
      return hp && hn;
    };
    // is direction node -> w inside the area enclosed by ring (g, ring) at node?
    auto in_ring_sector = [&](int node, int geom, int ring, bool ccw, P w) {
      P prev{}, next{};
      if (!ring_at(node, geom, ring, &prev, &next)) return false;
      const P X = o.nodes[node];
      // enclosed area left of travel (ccw): from next ccw to prev; else from prev to next
      return ccw ? in_sector(X, next, prev, w) : in_sector(X, prev, next, w);
    };
    // rings of geometry g through a node
    auto rings_at = [&](int node, int geom, std::vector<int>& rs) {
      rs.clear();
      for (int a = out_start[node]; a < out_start[node + 1]; a++) {
        const Overlay::Edge& e = o.edges[out_list[a]];
        if (e.geom == geom && std::find(rs.begin(), rs.end(), e.ring) == rs.end()) rs.push_back(e.ring);
      }
    };
    // subject interior at node (on the subject's boundary) in direction w: per part through
    // the node, inside its shell's sector (or inside the shell) and outside its holes' sectors
    auto subject_sector = [&](int node, P w) {
      rings_at(node, 0, rs);
      prts.clear();
      for (int r : rs)
        if (std::find(prts.begin(), prts.end(), o.ring_part[r]) == prts.end()) prts.push_back(o.ring_part[r]);
      for (int pt : prts) {
        bool in = true;
        bool shell_here = false;
        for (int r : rs) {
          if (o.ring_part[r] != pt) continue;
          const bool s = in_ring_sector(node, 0, r, ring_ccw[r], w);
          if (!o.ring_hole[r]) shell_here = true, in = in && s;
          else in = in && !s;
        }
        (void)shell_here;
        if (in) return true;
      }
      return false;
    };
    auto cell_sector = [&](int node, P w) {
      rings_at(node, 1, rs);
      for (int r : rs)
        if (in_ring_sector(node, 1, r, true, w)) return true;
      return false;
    };
    auto locate_cell = [&](P p) {  // not on the cell's boundary here
      for (auto& r : cell)
        if (locate_in_ring(p, r) >= 0) return true;
      return false;
    };
    auto locate_subject = [&](P p) {
      if (grid) grid->locate_rings(p, sub_rings, rloc, rcross);
      int ring = 0;
      for (size_t pi = 0; pi < parts.size(); pi++) {
        bool in = false;
        for (size_t ri = 0; ri < parts[pi].size(); ri++, ring++) {
          const int l = grid ? rloc[ring] : locate_in_ring(p, *sub_rings[ring]);
          if (ri == 0) in = l >= 0;
          else if (in && l > 0) in = false;
        }
        if (in) return true;
      }
      return false;
    };
    // located edges: at a node of the other geometry by its sectors; a subject edge touching
    // no cell node by point location in the cell (both ends, locateEdgeBothEnds)
    loc.assign(ne, -1);
    for (int k = 0; k < ne; k++) {
      const Overlay::Edge& e = o.edges[k];
      if (e.partner >= 0) continue;
      const int other = 1 - e.geom;
      const P U = o.nodes[e.u], V = o.nodes[e.v];
      if (o.on_geom[e.u] & (1 << other)) loc[k] = (other ? cell_sector(e.u, V) : subject_sector(e.u, V)) ? 1 : 0;
      else if (o.on_geom[e.v] & (1 << other)) loc[k] = (other ? cell_sector(e.v, U) : subject_sector(e.v, U)) ? 1 : 0;
      else if (other == 1) loc[k] = (locate_cell(U) && locate_cell(V)) ? 1 : 0;
    }
    // a cell edge touching no subject node lies where its ring's previous edge does (the
    // location changes only at subject nodes; a cell ring's edges are consecutive, in ring
    // order); a ring without any subject node: one point location in the subject
    for (size_t ci = 0; ci < cell.size(); ci++) {
      const int k0 = cell_edge_begin[ci], k1 = cell_edge_begin[ci + 1], m = k1 - k0;
      if (m <= 0) continue;
      int start = -1;
      for (int k = k0; k < k1 && start < 0; k++)
        if (loc[k] >= 0 || o.edges[k].partner >= 0) start = k;
      if (start < 0) {
        const int8_t l = locate_subject(o.nodes[o.edges[k0].u]) ? 1 : 0;
        for (int k = k0; k < k1; k++) loc[k] = l;
        continue;
      }
      int8_t cur = o.edges[start].partner >= 0 ? -1 : loc[start];
      for (int t = 1; t < m; t++) {
        const int k = k0 + (start - k0 + t) % m;
        if (o.edges[k].partner >= 0) {
          cur = -1;
          continue;
        }
        if (loc[k] >= 0) cur = loc[k];
        else if (cur >= 0) loc[k] = cur;
      }
      // (edges after a shared edge with no located edge before them: one more pass)
      for (int t = 0; t < m; t++) {
        const int k = k0 + (start - k0 + t) % m;
        if (loc[k] < 0 && o.edges[k].partner < 0) loc[k] = locate_subject(o.nodes[o.edges[k].u]) ? 1 : 0;
      }
    }
    for (int k = 0; k < ne; k++) {
      Overlay::Edge& e = o.edges[k];
      if (e.partner < 0 && loc[k] == 1) {
        e.in_result = true;
        e.res_left = e.int_left;
      }
    }
    // shared edges: in the result when both interiors lie on the same side
    for (int k = 0; k < ne; k++) {
      Overlay::Edge& e = o.edges[k];
      if (e.partner < 0 || e.geom != 0) continue;
      const Overlay::Edge& f = o.edges[e.partner];
      const bool f_left = (f.u == e.u) ? f.int_left : !f.int_left;  // f's interior side on e's direction
      if (f_left == e.int_left) {
        e.in_result = true;
        e.res_left = e.int_left;
      } else {
        o.lower_dim = true;  // a touching line (non-strict OverlayNG keeps it)
      }
    }
    // isolated touching points: a node on both boundaries with no result edge
    // 6. result edges directed with the result interior on their right (shells clockwise)
    res.clear();  // (from, to) node ids
    for (auto& e : o.edges)
      if (e.in_result) res.push_back(e.res_left ? std::make_pair(e.v, e.u) : std::make_pair(e.u, e.v));
    {
      touched.assign(nn, 0);
      for (auto& r : res) touched[r.first] = touched[r.second] = 1;
      for (int q = 0; q < nn; q++)
        if (o.on_geom[q] == 3 && !touched[q]) o.lower_dim = true;
    }
    *lower_dim = o.lower_dim;
    if (res.empty()) return;
    // 7. minimal rings: at each node leave by the first out-edge counter-clockwise from the
    // reversed incoming direction (the face on the right)
    const int nr = (int)res.size();
    rs_start.assign(nn + 1, 0);
    rs_list.assign(nr, 0);
    for (auto& r : res) rs_start[r.first + 1]++;
    for (int q = 0; q < nn; q++) rs_start[q + 1] += rs_start[q];
    {
      rs_fill.assign(rs_start.begin(), rs_start.end() - 1);
      for (int k = 0; k < nr; k++) rs_list[rs_fill[res[k].first]++] = k;
    }
    used.assign(nr, 0);
    std::vector<std::vector<P>> rings;
    for (int k0 = 0; k0 < nr; k0++) {
      if (used[k0]) continue;
      std::vector<P> ring;
      int k = k0;
      bool ok = true;
      while (true) {
        used[k] = 1;
        ring.push_back(o.nodes[res[k].first]);
        const int X = res[k].second;
        if (X == res[k0].first && (rs_start[X + 1] - rs_start[X] == 1)) break;
        // choose the next edge
        int best = -1;
        const P Xp = o.nodes[X], back = o.nodes[res[k].first];
        // (an edge straight back the way we came turns by a full circle: last)
        auto straight_back = [&](P d) {
          return orient(Xp, back, d) == 0 && half(Xp, back, d) == 0;
        };
        for (int a = rs_start[X]; a < rs_start[X + 1]; a++) {
          const int c = rs_list[a];
          const P d = o.nodes[res[c].second];
          if (best < 0) {
            best = c;
            continue;
          }
          const P bd = o.nodes[res[best].second];
          const bool sb = straight_back(d), sbb = straight_back(bd);
          if (sb != sbb) {
            if (!sb) best = c;
            continue;
          }
          if (ccw_before(Xp, back, d, bd)) best = c;
        }
        if (best == k0) break;
        if (best < 0 || used[best]) {
          ok = false;
          break;
        }
        k = best;
      }
      if (!ok || ring.size() < 3) continue;
      ring.push_back(ring[0]);
      rings.push_back(std::move(ring));
    }
    // 8. shells (clockwise) and holes (ccw); each hole to the smallest shell holding it
    shells.clear();
    holes.clear();
    std::vector<double>& area = rarea;
    area.assign(rings.size(), 0.0);
    // (OverlayEdgeRing: a ring is a hole iff Orientation.isCCW)
    for (size_t i = 0; i < rings.size(); i++) {
      area[i] = std::fabs(signed_area(rings[i]));
      if (!is_ccw(rings[i])) shells.push_back((int)i);
      else holes.push_back((int)i);
    }
    if (shells.empty()) return;
    std::vector<Rings> out(shells.size());
    for (size_t s = 0; s < shells.size(); s++) out[s].push_back(rings[shells[s]]);
    for (int h : holes) {
      int best = -1;
      for (size_t s = 0; s < shells.size(); s++) {
        const auto& sh = rings[shells[s]];
        // a hole vertex not on the shell
        int l = 0;
        for (auto& p : rings[h]) {
          l = locate_in_ring(p, sh);
          if (l != 0) break;
        }
        if (l > 0 && (best < 0 || area[shells[s]] < area[shells[best]])) best = (int)s;
      }
      if (best >= 0) out[best].push_back(rings[h]);
    }
    pieces = std::move(out);
  }
};

// coerceChipGeometry's difference with the cell boundary: each chip edge re-noded against
// the cell's segments (RobustLineIntersector; the chip edge first as IntersectionAdder's
// segment pair puts it); a node strictly inside an edge splits it
inline void renode_with_cell(std::vector<Rings>& pieces, const std::vector<std::vector<P>>& cell) {
  std::vector<P> nd, out;
  for (auto& piece : pieces)
    for (auto& ring : piece) {
      out.clear();
      for (size_t k = 0; k + 1 < ring.size(); k++) {
        const P a = ring[k], b = ring[k + 1];
        out.push_back(a);
        nd.clear();
        for (auto& cr : cell)
          for (size_t j = 0; j + 1 < cr.size(); j++) {
            const Hit h = line_intersect(a, b, cr[j], cr[j + 1]);
            for (int q = 0; q < h.n; q++)
              if (!eq(h.pt[q], a) && !eq(h.pt[q], b)) nd.push_back(h.pt[q]);
          }
        if (nd.empty()) continue;
        const int oc = octant(b.x - a.x, b.y - a.y);
        std::sort(nd.begin(), nd.end(), [&](P p, P q) { return seg_compare(oc, p, q) < 0; });
        for (size_t q = 0; q < nd.size(); q++)
          if (q == 0 || !eq(nd[q], nd[q - 1])) out.push_back(nd[q]);
      }
      out.push_back(out[0]);
      ring.swap(out);
    }
}

}  // namespace ovl
}  // namespace mgpu
