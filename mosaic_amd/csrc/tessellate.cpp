// grid_tessellateexplode: polygons -> chip rows (is_core, index_id, wkb).
//
// Replaces Mosaic.getChips / mosaicFill (core/Mosaic.scala:22-99) with
// IndexSystem.getCoreChips / getBorderChips (IndexSystem.scala:178-213) and
// coerceChipGeometry (:293-303), for H3 (H3IndexSystem.scala:79-154) and BNG
// (BNGIndexSystem.scala:151-209, 418-431).  Host code, run once per polygon set;
// its output is uploaded with mgpu_chips_upload.
//
// Every chip is `polygon INTERSECTION cell`, with the cell polygon in the
// polygon's coordinates exactly as indexToGeometry builds it (H3: the 6 boundary
// vertices joined by straight lon/lat edges; BNG: the square).  A cell is core
// when the intersection is the whole cell (IndexSystem.scala:185: isCore =
// coerced.equals(indexGeom)); cells with an empty intersection are dropped
// (MosaicChip.isEmpty).  The reference obtains the core set by polyfilling a
// negatively buffered polygon (Mosaic.scala:71-93); both constructions cover the
// polygon exactly once, so the join result is the same wherever the two agree on
// the cell geometry (the chip bytes themselves are "parity unpinned").
//
// Algorithm (O(V + cells) per polygon instead of O(V x cells)):
//  1. project the polygon into the grid's lattice space (H3: the hex2d plane of
//     the polygon's icosahedron face at `res`; BNG: metres / cell size),
//  2. border cells = lattice cells touched by any edge (dense edge walk + 1 ring),
//  3. interior cells = cells whose centre is inside the polygon (scanline in
//     lattice space) and that no edge touches -> core chips,
//  4. border cells: Sutherland-Hodgman clip of every ring against the convex cell
//     -> empty (dropped), whole cell (core) or a border chip.
// H3 polygons may span several icosahedron faces: steps 1-4 run once per face near
// the polygon (the faces of its vertices and, close to a face edge, the neighbour
// across it), each pass keeping the cells whose centre lies on that face (the face
// _h3ToFaceIjk gives the cell id), so every cell is considered exactly once.  The
// rings are densified along their lon/lat edges before projection, so the lattice
// walk follows the true edges (straight in lon/lat, curved in a face's gnomonic
// plane).  Cell geometry is H3's own h3ToGeoBoundary (h3_boundary.h), with the
// distortion vertices of Class III cells that cross an icosahedron edge.
// Cells as the reference shapes them (H3IndexSystem.indexToGeometry): the cell holding
// a pole is the cap from its boundary to the pole, a cell across the antimeridian its
// western and eastern parts (a MULTIPOLYGON; a chip clipped from it likewise).
// Limitations (MGPU_E_UNSUPPORTED): a polygon more than ~84 degrees from a face it
// touches; coordinates outside [-180, 180] x [-90, 90] (the reference's alignToGrid
// re-wraps such geometries first).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <set>
#include <string>
#include <mutex>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../../include/mosaic_gpu.h"
#include "error.h"
#include "bng_core.h"
#include "h3_core.h"
#include "h3_boundary.h"
#include "jts_buffer.h"
#include "jts_overlay.h"
#include "parallel.h"
#include "wkb.h"

namespace {

thread_local std::string t_err;

using Pt = mgpu::ovl::P;

double ring_area(const std::vector<Pt>& r) {
  double a = 0;
  for (size_t i = 0; i + 1 < r.size(); i++) a += r[i].x * r[i + 1].y - r[i + 1].x * r[i].y;
  return 0.5 * a;
}

// Sutherland-Hodgman clip of a closed ring against a convex ccw polygon `clip`
// (closed, first == last).  Returns a closed ring or empty.
std::vector<Pt> clip_ring(const std::vector<Pt>& ring, const std::vector<Pt>& clip) {
  std::vector<Pt> in(ring.begin(), ring.end() - 1), out;
  for (size_t e = 0; e + 1 < clip.size() && !in.empty(); e++) {
    Pt a = clip[e], b = clip[e + 1];
    auto side = [&](Pt p) { return (b.x - a.x) * (p.y - a.y) - (b.y - a.y) * (p.x - a.x); };
    out.clear();
    // (the previous vertex and its side carried over from the last step: the same values)
    Pt prev = in.back();
    double sp = side(prev);
    for (size_t i = 0; i < in.size(); i++) {
      const Pt cur = in[i];
      const double sc = side(cur);
      if (sc >= 0) {
        if (sp < 0) {
          double t = sp / (sp - sc);
          out.push_back({prev.x + t * (cur.x - prev.x), prev.y + t * (cur.y - prev.y)});
        }
        out.push_back(cur);
      } else if (sp >= 0) {
        double t = sp / (sp - sc);
        out.push_back({prev.x + t * (cur.x - prev.x), prev.y + t * (cur.y - prev.y)});
      }
      prev = cur, sp = sc;
    }
    in.swap(out);
  }
  if (in.size() < 3) return {};
  in.push_back(in[0]);
  return in;
}

bool point_in_ring(const std::vector<Pt>& r, Pt p) {
  bool c = false;
  for (size_t i = 0, j = r.size() - 1; i < r.size(); j = i++) {
    if (((r[i].y > p.y) != (r[j].y > p.y)) && (p.x < (r[j].x - r[i].x) * (p.y - r[i].y) / (r[j].y - r[i].y) + r[i].x))
      c = !c;
  }
  return c;
}

struct Polygon {
  std::vector<std::vector<std::vector<Pt>>> parts;  // part -> rings (first = shell)
  std::vector<uint8_t> ring_ccw;                    // per ring (parts' rings in order)
  bool multi = false;                               // a MULTIPOLYGON (else a POLYGON)
  std::vector<const std::vector<Pt>*> ring_ptr;     // per ring (parts' rings in order)
  mgpu::ovl::SegGrid grid;                          // the rings' segments, bucketed
};

// how border chips are cut (mgpu_tessellate_geom's chip_geometry)
enum ChipGeometry { kChipOverlay = 0, kChipSutherlandHodgman = 1 };

struct GeomStats {
  int64_t overlay_chips = 0;   // border chips cut by the overlay
  int64_t multi_piece = 0;     // ... that fell apart into several pieces
  int64_t coerced = 0;         // ... re-noded by coerceChipGeometry's difference
  int64_t coerce_nodes = 0;    // nodes that difference added
  int64_t lower_dim = 0;       // ... whose overlay also gave lines / points
};

thread_local mgpu::ovl::Clipper t_clip;

double cross3(Pt a, Pt b, Pt c) { return (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x); }

bool segments_touch(Pt a, Pt b, Pt c, Pt d) {
  double o1 = cross3(a, b, c), o2 = cross3(a, b, d), o3 = cross3(c, d, a), o4 = cross3(c, d, b);
  if (((o1 > 0 && o2 < 0) || (o1 < 0 && o2 > 0)) && ((o3 > 0 && o4 < 0) || (o3 < 0 && o4 > 0))) return true;
  auto on = [](Pt p, Pt q, Pt r) {  // r on segment pq given collinear
    return std::min(p.x, q.x) <= r.x && r.x <= std::max(p.x, q.x) && std::min(p.y, q.y) <= r.y &&
           r.y <= std::max(p.y, q.y);
  };
  return (o1 == 0 && on(a, b, c)) || (o2 == 0 && on(a, b, d)) || (o3 == 0 && on(c, d, a)) || (o4 == 0 && on(c, d, b));
}

// convex ccw closed polygon: p inside or on the boundary
bool in_convex(const std::vector<Pt>& cell, Pt p) {
  for (size_t i = 0; i + 1 < cell.size(); i++)
    if (cross3(cell[i], cell[i + 1], p) < 0) return false;
  return true;
}

bool is_convex(const std::vector<Pt>& c) {  // closed ccw ring
  const size_t n = c.size() - 1;
  for (size_t i = 0; i < n; i++)
    if (cross3(c[(i + n - 1) % n], c[i], c[(i + 1) % n]) < 0) return false;
  return true;
}

// A cell ring split into convex pieces (closed ccw rings).  H3 cells are convex in lon/lat
// except at the distortion vertices Class III cells gain where an edge crosses an
// icosahedron edge; those are split by ear clipping, then triangles sharing a diagonal
// are merged while the union stays convex (Hertel-Mehlhorn).
std::vector<std::vector<Pt>> convex_pieces(const std::vector<Pt>& cell) {
  if (is_convex(cell)) return {cell};
  const int n = (int)cell.size() - 1;
  std::vector<int> idx(n);
  for (int i = 0; i < n; i++) idx[i] = i;
  std::vector<std::vector<int>> pieces;
  while (idx.size() > 3) {
    const int m = (int)idx.size();
    bool cut = false;
    for (int k = 0; k < m && !cut; k++) {
      const int a = idx[(k + m - 1) % m], b = idx[k], c = idx[(k + 1) % m];
      if (cross3(cell[a], cell[b], cell[c]) <= 0) continue;
      bool empty = true;
      for (int q : idx)
        if (q != a && q != b && q != c && cross3(cell[a], cell[b], cell[q]) >= 0 &&
            cross3(cell[b], cell[c], cell[q]) >= 0 && cross3(cell[c], cell[a], cell[q]) >= 0)
          empty = false;
      if (!empty) continue;
      pieces.push_back({a, b, c});
      idx.erase(idx.begin() + k);
      cut = true;
    }
    if (!cut) break;  // degenerate: keep the remainder as one piece
  }
  pieces.push_back(idx);
  auto ring_of = [&](const std::vector<int>& v) {
    std::vector<Pt> r;
    for (int q : v) r.push_back(cell[q]);
    r.push_back(cell[v[0]]);
    return r;
  };
  for (bool merged = true; merged;) {
    merged = false;
    for (size_t i = 0; i < pieces.size() && !merged; i++)
      for (size_t j = i + 1; j < pieces.size() && !merged; j++) {
        const auto& P = pieces[i];
        const auto& Q = pieces[j];
        for (size_t e = 0; e < P.size() && !merged; e++) {
          const int a = P[e], b = P[(e + 1) % P.size()];
          for (size_t f = 0; f < Q.size(); f++) {
            if (Q[f] != b || Q[(f + 1) % Q.size()] != a) continue;
            // P with its edge a->b replaced by Q's path b -> ... -> a
            std::vector<int> W;
            for (size_t t = 0; t < P.size(); t++) W.push_back(P[(e + 1 + t) % P.size()]);  // b .. a
            for (size_t t = 2; t < Q.size(); t++) W.push_back(Q[(f + t) % Q.size()]);     // after a .. before b
            if (is_convex(ring_of(W))) {
              pieces[i] = W;
              pieces.erase(pieces.begin() + j);
              merged = true;
            }
            break;
          }
        }
      }
  }
  std::vector<std::vector<Pt>> out;
  for (auto& v : pieces) out.push_back(ring_of(v));
  return out;
}


// ---------------------------------------------------------------- grids

// the cell holding the north / south pole at `res` (H3IndexSystem.scala:240-246:
// geoToH3(+-90, 0, res))
uint64_t pole_cell(bool north, int res) {
  static uint64_t cache[2][16] = {};
  uint64_t& c = cache[north ? 1 : 0][res & 15];
  if (!c) {
    bool tie = false;
    c = mgpu::h3::point_to_cell(0.0, north ? 90.0 : -90.0, res, &tie);
  }
  return c;
}

// a cell's rings (Grid::boundary) as chip WKB: a Polygon, or a MultiPolygon of its parts
// (every ring its own polygon; each ring reversed when `rev`)
void write_cell_wkb(const std::vector<std::vector<Pt>>& rings, std::vector<uint8_t>& out, bool rev = false) {
  mgpu::wkb::write_polygons_pts<true>(out, rings, rev);
}

// JTS Intersection.intersection (JTS 1.20 algorithm/Intersection.java, what
// RobustLineIntersector computes for a proper crossing): homogeneous coordinates about the
// midpoint of the two segments' envelope overlap, every product rounded on its own
Pt jts_intersection(Pt p1, Pt p2, Pt q1, Pt q2) {
  const double minX0 = p1.x < p2.x ? p1.x : p2.x, minY0 = p1.y < p2.y ? p1.y : p2.y;
  const double maxX0 = p1.x > p2.x ? p1.x : p2.x, maxY0 = p1.y > p2.y ? p1.y : p2.y;
  const double minX1 = q1.x < q2.x ? q1.x : q2.x, minY1 = q1.y < q2.y ? q1.y : q2.y;
  const double maxX1 = q1.x > q2.x ? q1.x : q2.x, maxY1 = q1.y > q2.y ? q1.y : q2.y;
  const double midx = ((minX0 > minX1 ? minX0 : minX1) + (maxX0 < maxX1 ? maxX0 : maxX1)) / 2.0;
  const double midy = ((minY0 > minY1 ? minY0 : minY1) + (maxY0 < maxY1 ? maxY0 : maxY1)) / 2.0;
  const double p1x = p1.x - midx, p1y = p1.y - midy, p2x = p2.x - midx, p2y = p2.y - midy;
  const double q1x = q1.x - midx, q1y = q1.y - midy, q2x = q2.x - midx, q2y = q2.y - midy;
  const double px = p1y - p2y, py = p2x - p1x, pw = p1x * p2y - p2x * p1y;
  const double qx = q1y - q2y, qy = q2x - q1x, qw = q1x * q2y - q2x * q1y;
  const double x = py * qw - qy * pw, y = qx * pw - px * qw, w = px * qy - qx * py;
  return {x / w + midx, y / w + midy};
}

// The polar cap as makePoleGeometry builds it (H3IndexSystem.scala:361-380): the
// boundary's vertices shifted east (lng < 0: +360, shiftEast :277-280) and sorted by that
// longitude form a line; its part in [0, 180] (westernLine), the pole edge (180, pole) ->
// (-180, pole), its part in [180, 360] shifted back west (easternLine, lng - 360 in
// floating point, as shiftWest), closed at the first vertex.  Both parts end / start at the
// crossing JTS's overlay computes with the box edge x = 180.  That ring is ccw at the north
// pole and clockwise at the south pole; it is returned ccw (the tessellation's convex
// pieces and clipping need ccw) and write_cell_wkb writes the south cap reversed
// (Grid::cw_ring), which restores the reference's vertex order from the same start.
std::vector<Pt> pole_cap(const std::vector<Pt>& b, bool north) {
  std::vector<Pt> v;
  for (auto& q : b) v.push_back({q.x < 0 ? q.x + 360.0 : q.x, q.y});
  std::stable_sort(v.begin(), v.end(), [](const Pt& a, const Pt& c) { return a.x < c.x; });
  size_t k = 0;  // first vertex east of 180 (shifted)
  while (k < v.size() && v[k].x <= 180.0) k++;
  const double pl = north ? 90.0 : -90.0;
  std::vector<Pt> r(v.begin(), v.begin() + k);
  if (k > 0 && k < v.size()) {
    Pt cut = jts_intersection(v[k - 1], v[k], {180.0, -90.0}, {180.0, 90.0});
    if (r.back().x != cut.x || r.back().y != cut.y) r.push_back(cut);
    r.push_back({180.0, pl});
    r.push_back({-180.0, pl});
    if (cut.x >= 180.0) cut.x -= 360.0;
    r.push_back(cut);
  }
  for (size_t t = k; t < v.size(); t++) r.push_back({v[t].x >= 180.0 ? v[t].x - 360.0 : v[t].x, v[t].y});
  r.push_back(r[0]);
  if (!north) std::reverse(r.begin(), r.end());
  return r;
}

// A thread's memo of substrate vertex positions (cell_boundary's VertexGeo: a pure function
// of face, resolution and normalized ijk).  Neighbouring border cells share most of their
// vertices; the table is emptied when half full.
struct VertexCache {
  struct E {
    int32_t fr, i, j, k;
    mgpu::h3b::LatLon v;
  };
  std::vector<E> t;
  size_t n = 0;
  VertexCache() : t((size_t)1 << 12, E{-1, 0, 0, 0, {}}) {}
  mgpu::h3b::LatLon get(const mgpu::h3b::FaceIJK& f, int adj_res) {
    const int32_t fr = f.face * 32 + adj_res;
    uint64_t h = (uint64_t)(uint32_t)f.c.i * 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)f.c.j * 0xC2B2AE3D27D4EB4Full ^
                 (uint64_t)(uint32_t)f.c.k * 0x165667B19E3779F9ull ^ (uint64_t)(uint32_t)fr;
    h ^= h >> 31;
    const size_t mask = t.size() - 1;
    for (size_t q = h & mask;; q = (q + 1) & mask) {
      E& e = t[q];
      if (e.fr == fr && e.i == f.c.i && e.j == f.c.j && e.k == f.c.k) return e.v;
      if (e.fr >= 0) continue;
      const mgpu::h3b::LatLon v = mgpu::h3b::VertexGeo()(f, adj_res);
      if (2 * (n + 1) > t.size()) {
        for (auto& x : t) x.fr = -1;
        n = 0;
        return v;
      }
      e = E{fr, f.c.i, f.c.j, f.c.k, v};
      n++;
      return v;
    }
  }
};
thread_local VertexCache t_vcache;
struct CachedVertex {
  mgpu::h3b::LatLon operator()(const mgpu::h3b::FaceIJK& f, int adj_res) const { return t_vcache.get(f, adj_res); }
};

// H3IndexSystem.indexToGeometry (H3IndexSystem.scala:103-121): h3ToGeoBoundary in
// degrees, closed, ccw; the cell holding a pole as the cap between its boundary and
// the pole (makePoleGeometry, :361-384); a cell across the antimeridian cut into its
// western and eastern parts (makeSafeGeometry / crossesAntiMeridian, :386-410, :258-262)
std::vector<std::vector<Pt>> h3_cell_rings(uint64_t id, int res) {
  std::vector<Pt> b;
  for (auto& v : mgpu::h3b::cell_boundary(id, CachedVertex()))
    b.push_back({mgpu::h3b::to_degrees(v.lon), mgpu::h3b::to_degrees(v.lat)});
  const int pole = id == pole_cell(true, res) ? 1 : (id == pole_cell(false, res) ? -1 : 0);
  if (pole) return {pole_cap(b, pole > 0)};
  double lo = INFINITY, hi = -INFINITY;
  for (auto& q : b) {
    lo = std::min(lo, q.x);
    hi = std::max(hi, q.x);
  }
  b.push_back(b[0]);
  if (ring_area(b) < 0) std::reverse(b.begin(), b.end());
  // (crossesAntiMeridian's `|| !geometry.isValid` arm never fires here: no H3 cell of res
  // 0-3 -- every one enumerated, tests/test_tessellate_host.py -- with lo < 0 <= hi and a
  // span <= 180 is self-intersecting, and finer cells are smaller)
  if (!(lo < 0 && hi >= 0 && hi - lo > 180.0)) return {b};
  // across the antimeridian: shift the western longitudes east, cut at 180
  for (auto& q : b)
    if (q.x < 0) q.x += 360.0;
  if (ring_area(b) < 0) std::reverse(b.begin(), b.end());
  static const std::vector<Pt> west{{0, -90}, {180, -90}, {180, 90}, {0, 90}, {0, -90}};
  static const std::vector<Pt> east{{180, -90}, {360, -90}, {360, 90}, {180, 90}, {180, -90}};
  std::vector<std::vector<Pt>> out;
  auto w = clip_ring(b, west);
  if (!w.empty() && std::fabs(ring_area(w)) > 0) out.push_back(std::move(w));
  auto e = clip_ring(b, east);
  if (!e.empty() && std::fabs(ring_area(e)) > 0) {
    for (auto& q : e) q.x -= 360.0;
    out.push_back(std::move(e));
  }
  return out;
}

struct Grid {
  virtual ~Grid() {}
  // a cell whose centre is farther than this (lattice units) from every walked boundary
  // sample cannot meet the boundary (circumradius + sample spacing + H3's distortion)
  virtual double far_distance() const { return 1.0; }
  // whether this pass owns lattice cell (i, j) with id `id` (H3: the cell's centre lies on
  // this pass's face, and the id is the cell at that lattice position)
  virtual bool keep(int64_t, long, long) const { return true; }
  // lattice-space coordinate of an input point
  virtual Pt to_lattice(Pt p) const = 0;
  // lattice cell containing a lattice-space point
  virtual std::pair<long, long> cell_at(Pt q) const = 0;
  virtual Pt center(long i, long j) const = 0;  // lattice space
  virtual void neighbors(long i, long j, std::vector<std::pair<long, long>>& out) const = 0;
  // cell id (0 = not representable) and its geometry in input coords: one closed ccw
  // ring, or several (H3: a cell cut at the antimeridian); empty = no geometry
  virtual int64_t cell_id(long i, long j) const = 0;
  virtual std::vector<std::vector<Pt>> boundary(long i, long j) const = 0;
  // the same, for a cell whose id the caller has (cell_id(i, j))
  virtual std::vector<std::vector<Pt>> boundary_of(long i, long j, int64_t) const { return boundary(i, j); }
  // a cell whose reference geometry is a clockwise ring (H3's south polar cap)
  virtual bool cw_ring(int64_t) const { return false; }
  // the cell's centre in input coords (H3: h3ToGeo; BNG: the square's centre)
  virtual Pt center_input(long i, long j, int64_t id) const = 0;
  // lattice row/column iteration for the scanline: row index of a lattice y,
  // y of a row, and the column index of the cell centred at lattice x in a row
  virtual double row_y(long j) const = 0;
  virtual long row_of(double y, bool up) const = 0;
  virtual double col_x(long i, long j) const = 0;
  virtual long col_of(double x, long j, bool up) const = 0;
  // lattice cells (i0..i1, j0..j1) holding every cell_at of a point in the lattice-space
  // box and the neighbours of those cells
  virtual void cell_window(double xmin, double ymin, double xmax, double ymax, long* i0, long* j0, long* i1,
                           long* j1) const = 0;
};

struct H3Grid final : Grid {
  int face, res;
  // a lattice position inside the face triangle's inscribed circle (radius 1 in res-0
  // units; the vertices, where the pentagons sit, lie at 2), with a margin: no overage and
  // no pentagon near, so the id at that position is this face's cell centred there
  double inscribed2;
  explicit H3Grid(int f, int r) : face(f), res(r) {
    double q = 0.95;
    for (int i = 0; i < r; i++) q *= mgpu::h3::kSqrt7;
    inscribed2 = q * q;
  }
  Pt to_lattice(Pt p) const override {
    double lat = p.y * M_PI / 180.0, lon = p.x * M_PI / 180.0;
    // project onto THIS face (the polygon's), even slightly beyond its edge
    double slat = sin(lat), clat = cos(lat);
    double best = 0;
    {
      double x = cos(lon) * clat, y = sin(lon) * clat, z = slat;
      double dx = H3T_FACE_CENTER_POINT[face][0] - x, dy = H3T_FACE_CENTER_POINT[face][1] - y,
             dz = H3T_FACE_CENTER_POINT[face][2] - z;
      best = dx * dx + dy * dy + dz * dz;
    }
    double r = acos(1 - best / 2);
    if (r < 1e-16) return {0, 0};
    double flat = H3T_FACE_CENTER_GEO[face][0], flon = H3T_FACE_CENTER_GEO[face][1];
    double az = atan2(clat * sin(lon - flon), cos(flat) * slat - sin(flat) * clat * cos(lon - flon));
    double theta = mgpu::h3::pos_angle(H3T_FACE_AXES_AZ_CII[face][0] - mgpu::h3::pos_angle(az));
    if (res % 2) theta = mgpu::h3::pos_angle(theta - mgpu::h3::kAp7Rot);
    r = tan(r) / mgpu::h3::kRes0UGnomonic;
    for (int i = 0; i < res; i++) r *= mgpu::h3::kSqrt7;
    return {r * cos(theta), r * sin(theta)};
  }
  std::pair<long, long> cell_at(Pt q) const override {
    double m;
    mgpu::h3::IJK c = mgpu::h3::hex2d_to_ijk(q.x, q.y, &m);
    return {(long)c.i - c.k, (long)c.j - c.k};
  }
  Pt center(long i, long j) const override { return {i - 0.5 * j, j * mgpu::h3::kSin60}; }
  void neighbors(long i, long j, std::vector<std::pair<long, long>>& out) const override {
    static const int d[6][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, 1}, {-1, -1}};
    for (auto& v : d) out.push_back({i + v[0], j + v[1]});
  }
  int64_t cell_id(long i, long j) const override {
    mgpu::h3::IJK c{(int)i, (int)j, 0};
    mgpu::h3::ijk_normalize(c);
    return (int64_t)mgpu::h3::face_ijk_to_h3(face, c, res);
  }
  // exact H3 vertices are the lattice corners on this face; beyond a face edge the
  // neighbour's projection moves them by a second-order amount, a fraction of a
  // cell only at coarse resolutions
  double far_distance() const override { return res <= 4 ? 1.25 : 0.75; }
  // (keep and center_input both want the id's centre, mostly for the same cell in a row:
  // the last one is kept -- a grid belongs to one thread)
  mutable uint64_t cc_id = 0;
  mutable mgpu::h3b::LatLon cc_val{};
  const mgpu::h3b::LatLon& id_center(int64_t id) const {
    if ((uint64_t)id != cc_id || cc_id == 0) {
      cc_val = mgpu::h3b::cell_center((uint64_t)id);
      cc_id = (uint64_t)id;
    }
    return cc_val;
  }
  bool keep(int64_t id, long i, long j) const override {
    const Pt v = center(i, j);
    if (v.x * v.x + v.y * v.y < inscribed2) return true;
    if (mgpu::h3b::h3_to_face_ijk((uint64_t)id).face != face) return false;
    // near an icosahedron vertex the lattice positions beyond a pentagon's missing
    // sector map to ids of cells elsewhere: the id's centre must be this position
    const Pt g = to_geo(center(i, j));
    const auto c = id_center(id);
    const double dlat = g.y - mgpu::h3b::to_degrees(c.lat), dlon = g.x - mgpu::h3b::to_degrees(c.lon);
    double spacing = 20.0;  // ~ res-0 centre spacing in degrees
    for (int r = 0; r < res; r++) spacing /= 2.6457513110645906;
    return std::fabs(dlat) < 0.01 * spacing && std::fabs(std::remainder(dlon, 360.0)) < 0.01 * spacing / std::max(0.05, std::cos(g.y * M_PI / 180.0));
  }
  Pt to_geo(Pt v) const {
    // _hex2dToGeo (substrate = 0) then _geoAzDistanceRads
    double r = std::hypot(v.x, v.y);
    double lat0 = H3T_FACE_CENTER_GEO[face][0], lon0 = H3T_FACE_CENTER_GEO[face][1];
    double lat, lon;
    if (r < 1e-16) {
      lat = lat0;
      lon = lon0;
    } else {
      double theta = atan2(v.y, v.x);
      for (int i = 0; i < res; i++) r /= mgpu::h3::kSqrt7;
      r *= mgpu::h3::kRes0UGnomonic;
      r = atan(r);
      if (res % 2) theta = mgpu::h3::pos_angle(theta + mgpu::h3::kAp7Rot);
      double az = mgpu::h3::pos_angle(H3T_FACE_AXES_AZ_CII[face][0] - theta);
      double sinlat = sin(lat0) * cos(r) + cos(lat0) * sin(r) * cos(az);
      sinlat = std::max(-1.0, std::min(1.0, sinlat));
      lat = asin(sinlat);
      double sinlon = sin(az) * sin(r) / cos(lat);
      double coslon = (cos(r) - sin(lat0) * sin(lat)) / cos(lat0) / cos(lat);
      sinlon = std::max(-1.0, std::min(1.0, sinlon));
      coslon = std::max(-1.0, std::min(1.0, coslon));
      lon = lon0 + atan2(sinlon, coslon);
      while (lon > M_PI) lon -= 2 * M_PI;
      while (lon < -M_PI) lon += 2 * M_PI;
    }
    return {lon * 180.0 / M_PI, lat * 180.0 / M_PI};
  }
  std::vector<std::vector<Pt>> boundary(long i, long j) const override {
    const int64_t id = cell_id(i, j);
    if (!id) return {};
    return h3_cell_rings((uint64_t)id, res);
  }
  std::vector<std::vector<Pt>> boundary_of(long, long, int64_t id) const override {
    if (!id) return {};
    return h3_cell_rings((uint64_t)id, res);
  }
  bool cw_ring(int64_t id) const override { return (uint64_t)id == pole_cell(false, res); }
  Pt center_input(long, long, int64_t id) const override {
    const auto c = id_center(id);
    return {mgpu::h3b::to_degrees(c.lon), mgpu::h3b::to_degrees(c.lat)};
  }
  double row_y(long j) const override { return j * mgpu::h3::kSin60; }
  long row_of(double y, bool up) const override {
    double v = y / mgpu::h3::kSin60;
    return up ? (long)std::ceil(v) : (long)std::floor(v);
  }
  double col_x(long i, long j) const override { return i - 0.5 * j; }
  long col_of(double x, long j, bool up) const override {
    double v = x + 0.5 * j;
    return up ? (long)std::ceil(v) : (long)std::floor(v);
  }
  // (a point's cell centre lies within 0.58 of it: row within 1, column within 1 + half
  // a row; neighbours one more)
  void cell_window(double xmin, double ymin, double xmax, double ymax, long* i0, long* j0, long* i1,
                   long* j1) const override {
    *j0 = (long)std::floor(ymin / mgpu::h3::kSin60) - 3;
    *j1 = (long)std::ceil(ymax / mgpu::h3::kSin60) + 3;
    *i0 = (long)std::floor(xmin + 0.5 * (double)*j0) - 3;
    *i1 = (long)std::ceil(xmax + 0.5 * (double)*j1) + 3;
  }
};

struct BngGrid final : Grid {
  int res;
  double edge;
  // edge sizes of BNGIndexSystem.sizeMap: 10^(6-r) m, quadrant resolutions 10^(7-|r|) / 2 m
  explicit BngGrid(int r) : res(r) {
    int a = r < 0 ? -r : r;
    double ten = 1;
    for (int k = 0; k < (r < 0 ? 7 - a : 6 - a); k++) ten *= 10;
    edge = r < 0 ? ten / 2 : ten;
  }
  Pt to_lattice(Pt p) const override { return {p.x / edge, p.y / edge}; }
  double far_distance() const override { return 0.85; }  // circumradius sqrt(1/2) + 0.1 + slack
  std::pair<long, long> cell_at(Pt q) const override { return {(long)std::floor(q.x), (long)std::floor(q.y)}; }
  Pt center(long i, long j) const override { return {i + 0.5, j + 0.5}; }
  void neighbors(long i, long j, std::vector<std::pair<long, long>>& out) const override {
    for (int a = -1; a <= 1; a++)
      for (int b = -1; b <= 1; b++)
        if (a || b) out.push_back({i + a, j + b});
  }
  int64_t cell_id(long i, long j) const override {
    int64_t id = 0;
    mgpu::bng::point_to_cell((i + 0.5) * edge, (j + 0.5) * edge, res, &id);
    return id;
  }
  std::vector<std::vector<Pt>> boundary(long i, long j) const override {
    double x = i * edge, y = j * edge;
    return {{{x, y}, {x + edge, y}, {x + edge, y + edge}, {x, y + edge}, {x, y}}};
  }
  Pt center_input(long i, long j, int64_t) const override { return {(i + 0.5) * edge, (j + 0.5) * edge}; }
  double row_y(long j) const override { return j + 0.5; }
  long row_of(double y, bool up) const override { return up ? (long)std::ceil(y - 0.5) : (long)std::floor(y - 0.5); }
  double col_x(long i, long) const override { return i + 0.5; }
  long col_of(double x, long, bool up) const override {
    return up ? (long)std::ceil(x - 0.5) : (long)std::floor(x - 0.5);
  }
  void cell_window(double xmin, double ymin, double xmax, double ymax, long* i0, long* j0, long* i1,
                   long* j1) const override {
    *i0 = (long)std::floor(xmin) - 2, *j0 = (long)std::floor(ymin) - 2;
    *i1 = (long)std::floor(xmax) + 2, *j1 = (long)std::floor(ymax) + 2;
  }
};

// a row; its WKB is bytes [woff, woff + wlen) of its polygon's arena (one allocation per
// polygon, not per row: 9.4M rows on C3)
struct Chip {
  int64_t cell;
  int32_t poly;
  uint8_t core;
  uint32_t wlen;
  uint64_t woff;
};

// a row the core rule left undecided (mgpu_tess_result_undecided): kind 1 DP-sensitive,
// 2 unresolved; kept = whether the table holds it; its chip (the border chip the table
// holds, or the one a dropped row would have) for counting the pairs at stake
struct Undecided {
  int64_t cell;
  int32_t poly;
  uint8_t kind, kept, core;
  std::vector<uint8_t> wkb;
};

// ---------------------------------------------------------------- mosaicFill's core set
// The reference flags a chip core in two places (core/Mosaic.scala:61-99):
//  * getCoreChips (IndexSystem.scala:208-213): every cell of polyfill(buffer(-r)) -- a
//    cell whose centre lies in the polygon carved by r = getBufferRadius (H3IndexSystem.
//    scala:79-90: the largest planar distance from the polygon's centroid to a vertex of
//    the centroid's cell; BNGIndexSystem.scala:151-154: edge * sqrt(2) / 2), i.e. whose
//    centre is inside the polygon at distance >= r from its boundary;
//  * getBorderChips (IndexSystem.scala:178-195): isCore = coerced.equals(indexGeom), JTS
//    equalsExact (MosaicGeometryJTS.scala:209-212) of the OverlayNG intersection (or its
//    difference with the cell boundary, coerceChipGeometry :293-303) against the cell from
//    indexToGeometry.  JTS overlay builds result shells clockwise (OverlayEdgeRing: a ring
//    is a hole iff it is counter-clockwise) while indexToGeometry's cells are H3's
//    counter-clockwise boundary (BNG: the counter-clockwise square), so the two rings are
//    never exactly equal: a border-set cell is never core, even when the polygon holds all
//    of it -- its chip is then the whole cell (written clockwise here, as OverlayNG would).
// Cells neither in the core set nor in polyfill(boundary.buffer(1.01 r).simplify(0.01 r))
// are never visited by the reference (a blind spot: dropped).  CoreRule decides each row
// by its centre's signed distance d to the polygon boundary; rows within the bands where
// JTS's chord approximation of the buffers (8 segments per quadrant: <= 1.93% of r) and
// the 1% simplification could decide otherwise are counted as ambiguous.
struct SegIndex {
  double x0 = 0, y0 = 0, s = 1, inv = 1;
  long nx = 0, ny = 0;
  std::vector<uint32_t> start, items;
  std::vector<Pt> a, b;

  void build(const Polygon& poly, double cell) {
    double minx = INFINITY, miny = INFINITY, maxx = -INFINITY, maxy = -INFINITY;
    for (auto& part : poly.parts)
      for (auto& ring : part)
        for (size_t i = 0; i + 1 < ring.size(); i++) {
          a.push_back(ring[i]);
          b.push_back(ring[i + 1]);
          minx = std::min(minx, ring[i].x);
          maxx = std::max(maxx, ring[i].x);
          miny = std::min(miny, ring[i].y);
          maxy = std::max(maxy, ring[i].y);
        }
    if (a.empty()) return;
    s = std::max({cell, (maxx - minx) / 512.0, (maxy - miny) / 512.0, 1e-300});
    inv = 1.0 / s;
    x0 = minx;
    y0 = miny;
    nx = (long)((maxx - minx) * inv) + 1;
    ny = (long)((maxy - miny) * inv) + 1;
    start.assign((size_t)(nx * ny + 1), 0);
    auto range = [&](size_t k, long* i0, long* i1, long* j0, long* j1) {
      *i0 = col(std::min(a[k].x, b[k].x));
      *i1 = col(std::max(a[k].x, b[k].x));
      *j0 = row(std::min(a[k].y, b[k].y));
      *j1 = row(std::max(a[k].y, b[k].y));
    };
    for (int pass = 0; pass < 2; pass++) {
      std::vector<uint32_t> fill;
      if (pass) {
        for (size_t q = 1; q < start.size(); q++) start[q] += start[q - 1];
        items.assign(start.back(), 0);
        fill.assign(start.begin(), start.end() - 1);
      }
      for (size_t k = 0; k < a.size(); k++) {
        long i0, i1, j0, j1;
        range(k, &i0, &i1, &j0, &j1);
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
  static double seg_dist(Pt p, Pt u, Pt v) {
    const double dx = v.x - u.x, dy = v.y - u.y, l2 = dx * dx + dy * dy;
    double t = l2 > 0 ? ((p.x - u.x) * dx + (p.y - u.y) * dy) / l2 : 0.0;
    t = std::min(1.0, std::max(0.0, t));
    return std::hypot(u.x + t * dx - p.x, u.y + t * dy - p.y);
  }
  // distance from p to the nearest boundary segment, or INFINITY when none is within q.
  // (seg_dist's hypot only for a segment whose squared distance is within 1e-9 of the
  // smallest so far: the segment with the least hypot is always among them -- both round
  // within a few ulps of the exact distance -- so the minimum is seg_dist's, bit for bit)
  double min_dist(Pt p, double q) const {
    if (a.empty()) return INFINITY;
    double best = INFINITY, best2 = INFINITY;
    for (long j = row(p.y - q); j <= row(p.y + q); j++)
      for (long i = col(p.x - q); i <= col(p.x + q); i++) {
        const size_t c = (size_t)(j * nx + i);
        for (uint32_t k = start[c]; k < start[c + 1]; k++) {
          const Pt u = a[items[k]], v = b[items[k]];
          const double dx = v.x - u.x, dy = v.y - u.y, l2 = dx * dx + dy * dy;
          double t = l2 > 0 ? ((p.x - u.x) * dx + (p.y - u.y) * dy) / l2 : 0.0;
          t = std::min(1.0, std::max(0.0, t));
          const double ex = u.x + t * dx - p.x, ey = u.y + t * dy - p.y, d2 = ex * ex + ey * ey;
          if (d2 > best2 * (1.0 + 1e-9)) continue;
          best = std::min(best, std::hypot(ex, ey));
          best2 = std::min(best2, d2);
        }
      }
    return best <= q ? best : INFINITY;
  }
  // even-odd inside test of p (half-open crossing rule), from p's bucket row to the right;
  // a crossing is counted in the bucket holding its x, so a segment in several buckets
  // counts once
  bool inside(Pt p) const {
    if (a.empty() || p.y < y0 || p.y > y0 + ny * s) return false;
    const long j = row(p.y);
    bool in = false;
    for (long i = col(p.x); i < nx; i++) {
      const double bx0 = x0 + i * s, bx1 = i + 1 < nx ? x0 + (i + 1) * s : INFINITY;
      const size_t c = (size_t)(j * nx + i);
      for (uint32_t k = start[c]; k < start[c + 1]; k++) {
        const Pt u = a[items[k]], v = b[items[k]];
        if ((u.y > p.y) == (v.y > p.y)) continue;
        const double xi = (v.x - u.x) * (p.y - u.y) / (v.y - u.y) + u.x;
        if (p.x < xi && xi >= std::max(bx0, p.x) && xi < bx1) in = !in;
      }
    }
    return in;
  }
};

struct CoreStats {
  int64_t demoted = 0, promoted = 0, dropped = 0, ambiguous = 0;
  // the JTS restatement's verdicts near the thresholds (jts_buffer.h)
  int64_t carved_tests = 0, band_tests = 0;
  int64_t core_below_r = 0;   // core, centre < r deep: inside a fillet's chords
  int64_t border_above_r = 0; // not core, centre >= r deep: the input simplification
  int64_t band_dropped = 0;   // a chip cell outside the (unsimplified) band: never visited
  int64_t dp_sensitive = 0;   // band membership within the band simplification's 0.01 r
  int64_t unresolved = 0;     // a centre within 1e-9 r of a buffer curve
  int64_t carved_empty = 0;   // polygons whose buffer(-r) is empty
};

struct CoreRule {
  double r = 0;
  SegIndex seg;
  CoreStats st;
  // the exact-distance decision of round 4 (MGPU_CORE_DISTANCE) instead of the JTS
  // restatement
  bool distance_only = false;
  const Polygon* poly = nullptr;
  int carved_state = 0;  // 0 not built, 1 non-empty, 2 empty
  mgpu::jtsbuf::DepthField carved, band;
  bool band_built = false;
  // the last decide()'s undecided kind: 0 none, 1 DP-sensitive (band membership within the
  // band simplification's 0.01 r), 2 unresolved (a centre within 1e-9 r of a buffer curve)
  int last_flag = 0;
  enum Verdict { kCore, kBorder, kDrop };

  std::vector<mgpu::jtsbuf::Rings> parts() const {
    std::vector<mgpu::jtsbuf::Rings> o;
    for (auto& part : poly->parts) {
      mgpu::jtsbuf::Rings rs;
      for (auto& ring : part) {
        std::vector<mgpu::jtsbuf::XY> v;
        v.reserve(ring.size());
        for (auto& q : ring) v.push_back({q.x, q.y});
        rs.push_back(std::move(v));
      }
      o.push_back(std::move(rs));
    }
    return o;
  }
  // a centre decided core by its exact distance (>= 1.02 r deep): a point of buffer(-r)
  bool have_deep = false;
  mgpu::jtsbuf::XY deep{};
  void ensure_carved() {
    if (carved_state) return;
    mgpu::jtsbuf::carved_field(parts(), r, carved);
    carved.build_index(r);
    // non-empty when a known deep centre lies in it (the usual case: interior cells come
    // first), else the probe of every curve segment's sides
    carved_state = (have_deep && carved.depth(deep) >= 1) || carved.any_positive(1e-7 * r) ? 1 : 2;
    if (carved_state == 2) st.carved_empty++;
  }
  void ensure_band() {
    if (band_built) return;
    ensure_carved();
    mgpu::jtsbuf::band_field(parts(), 1.01 * r, carved_state == 2, band);
    band.build_index(r);
    band_built = true;
  }
  // the reference's flag of a chip cell with centre c; inside: the clip's knowledge (1 in,
  // 0 out, -1 unknown).  Every caller holds a cell with a non-empty chip.
  Verdict decide(Pt c, int inside) {
    last_flag = 0;
    const double q = 1.1 * r;
    double d = seg.min_dist(c, q);
    const bool in = inside >= 0 ? inside == 1 : seg.inside(c);
    if (!in) d = -d;
    if (distance_only) {
      if (std::fabs(d - r) <= 0.02 * r || std::fabs(-d - 1.01 * r) <= 0.03 * r) st.ambiguous++;
      if (d >= r) return kCore;
      if (-d > 1.04 * r) return kDrop;
      return kBorder;
    }
    // polyfill(carved): the centre in buffer(-r).  Its chords reach no deeper than
    // r cos(3 pi / 64) = 0.989 r and the input simplification removes < 0.0101 r: the
    // outline lies in [0.979 r, 1.0101 r], so outside [0.97 r, 1.02 r) the exact distance
    // decides (round 5 took 1.05 r: the same verdicts, more field builds)
    const mgpu::jtsbuf::XY p{c.x, c.y};
    bool core;
    if (d >= 1.02 * r) {
      core = true;
      if (!have_deep) have_deep = true, deep = p;
    } else if (d < 0.97 * r) {
      core = false;
    } else {
      ensure_carved();
      st.carved_tests++;
      core = carved_state == 1 && carved.depth(p) >= 1;
      if (carved_state == 1 && carved.outline_dist(p, 1e-9 * r, 1e-7 * r) < INFINITY)
        st.unresolved++, st.ambiguous++, last_flag = 2;
      if (core && d < r) st.core_below_r++;
      if (!core && d >= r) st.border_above_r++;
    }
    if (core) return kCore;
    // polyfill(band) diff core: the band's outline lies 1.01 r out, its chords and the
    // simplifications move it by < 0.03 r, and a centre within 0.01 r of it is flagged:
    // outside [0.97 r, 1.05 r] the exact distance decides (round 5: [0.95 r, 1.1 r])
    if (std::fabs(d) < 0.97 * r) return kBorder;
    if (-d > 1.05 * r) return kDrop;
    ensure_band();
    st.band_tests++;
    const bool in_band = band.depth(p) >= 1;
    const double near = band.outline_dist(p, 0.01 * r * (1 + 1e-6), 1e-7 * r);  // simplify(0.01 r)
    if (near < 1e-9 * r) st.unresolved++, st.ambiguous++, last_flag = 2;
    else if (near < INFINITY) st.dp_sensitive++, st.ambiguous++, last_flag = 1;
    if (!in_band) st.band_dropped++;
    return in_band ? kBorder : kDrop;
  }
};

// Grid::boundary's rings reversed (clockwise shells, as JTS overlay returns them)
std::vector<std::vector<Pt>> reversed(std::vector<std::vector<Pt>> rings) {
  for (auto& r : rings) std::reverse(r.begin(), r.end());
  return rings;
}

struct PairHash {
  size_t operator()(const std::pair<long, long>& p) const { return std::hash<long>()(p.first * 1000003L ^ p.second); }
};

// lattice cell -> smallest squared distance from its centre to a walked boundary sample
// (the walk looks a cell up ~7 times per sample): a dense window of the lattice around the
// polygon when that is small (-1: not walked), else open addressing
struct CellDist {
  struct Slot {
    long i, j;
    float d2;
    bool used;
  };
  std::vector<Slot> t;
  size_t n = 0, mask = 0;
  bool dense = false, overflow = false;
  long wi0 = 0, wj0 = 0, wni = 0, wnj = 0;
  std::vector<float> w;
  void clear_dense(long i0, long j0, long i1, long j1) {
    dense = true;
    overflow = false;
    wi0 = i0, wj0 = j0, wni = i1 - i0 + 1, wnj = j1 - j0 + 1;
    w.assign((size_t)(wni * wnj), -1.f);
  }
  float* cell(long i, long j) {
    const long a = i - wi0, b = j - wj0;
    return (a >= 0 && a < wni && b >= 0 && b < wnj) ? &w[(size_t)(a * wnj + b)] : nullptr;
  }
  // the smallest squared distance walked for (i, j), or -1
  float get(long i, long j) {
    if (dense) {
      const float* c = cell(i, j);
      return c ? *c : -1.f;
    }
    const Slot* q = find(i, j);
    return q ? q->d2 : -1.f;
  }
  void touch(long i, long j, float d2) {
    if (dense) {
      float* c = cell(i, j);
      if (!c) {  // (cell_window should hold every cell the walk reaches: then hash it)
        overflow = true;
        return;
      }
      if (*c < 0 || d2 < *c) *c = d2;
      return;
    }
    Slot* it = find(i, j);
    if (!it) put(i, j, d2);
    else if (d2 < it->d2) it->d2 = d2;
  }
  static size_t h(long i, long j) {
    uint64_t k = (uint64_t)i * 0x9E3779B97F4A7C15ull ^ ((uint64_t)j + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
    return (size_t)(k ^ (k >> 29));
  }
  void clear() {
    dense = overflow = false;
    t.assign(1024, Slot{0, 0, 0.f, false});
    mask = 1023;
    n = 0;
  }
  Slot* find(long i, long j) {
    for (size_t q = h(i, j) & mask;; q = (q + 1) & mask) {
      if (!t[q].used) return nullptr;
      if (t[q].i == i && t[q].j == j) return &t[q];
    }
  }
  void put(long i, long j, float d2) {
    if (2 * (n + 1) > t.size()) {
      std::vector<Slot> old;
      old.swap(t);
      t.assign(old.size() * 2, Slot{0, 0, 0.f, false});
      mask = t.size() - 1;
      n = 0;
      for (auto& s : old)
        if (s.used) put(s.i, s.j, s.d2);
    }
    size_t q = h(i, j) & mask;
    while (t[q].used) q = (q + 1) & mask;
    t[q] = Slot{i, j, d2, true};
    n++;
  }
};
thread_local CellDist t_border;

// Exact test that the cell lies in the interior of one part of the polygon: no ring
// vertex in/on the cell, no ring edge touching a cell edge, the cell centre inside
// the shell and outside every hole.  Such a cell's chip IS the cell geometry
// (isCore = coerced.equals(indexGeom), IndexSystem.scala:185).
bool cell_in_polygon(const std::vector<Pt>& cellb, const std::vector<std::vector<Pt>>& pieces, Pt cc,
                     const Polygon& poly) {
  double cminx = INFINITY, cminy = INFINITY, cmaxx = -INFINITY, cmaxy = -INFINITY;
  for (auto& p : cellb) {
    cminx = std::min(cminx, p.x);
    cmaxx = std::max(cmaxx, p.x);
    cminy = std::min(cminy, p.y);
    cmaxy = std::max(cmaxy, p.y);
  }
  for (uint64_t c : poly.grid.query(cminx, cminy, cmaxx, cmaxy)) {
    const auto& ring = *poly.ring_ptr[c >> 32];
    const size_t i = (size_t)(c & 0xFFFFFFFFu);
    Pt a = ring[i], b = ring[i + 1];
    if (std::max(a.x, b.x) < cminx || std::min(a.x, b.x) > cmaxx || std::max(a.y, b.y) < cminy ||
        std::min(a.y, b.y) > cmaxy)
      continue;
    for (auto& pc : pieces)
      if (in_convex(pc, a)) return false;
    for (size_t k = 0; k + 1 < cellb.size(); k++)
      if (segments_touch(a, b, cellb[k], cellb[k + 1])) return false;
  }
  // point_in_ring of the centre in every ring at once, over the segments a rightward ray
  // from it can cross (SegGrid::ray_right; the others add no crossing): the same terms
  thread_local std::vector<uint8_t> par;
  par.assign(poly.ring_ptr.size(), 0);
  for (uint64_t c : poly.grid.ray_right(cc.x, cc.y)) {
    const auto& ring = *poly.ring_ptr[c >> 32];
    const size_t k = (size_t)(c & 0xFFFFFFFFu);
    const Pt ri = ring[k + 1], rj = ring[k];
    if (((ri.y > cc.y) != (rj.y > cc.y)) && (cc.x < (rj.x - ri.x) * (cc.y - ri.y) / (rj.y - ri.y) + ri.x))
      par[c >> 32] ^= 1;
  }
  size_t r0 = 0;
  for (auto& part : poly.parts) {
    const size_t r1 = r0 + part.size();
    bool in = par[r0] != 0;
    for (size_t r = r0 + 1; in && r < r1; r++)
      if (par[r]) in = false;
    if (in) return true;
    r0 = r1;
  }
  return false;
}

// `lat_rings`: every ring in the grid's lattice space (densified for H3)
// (G: H3Grid or BngGrid -- final, so the per-sample calls bind statically)
template <class G>
void tessellate_polygon(const G& g, const Polygon& poly, const std::vector<std::vector<Pt>>& lat_rings, int32_t pid,
                        std::vector<uint8_t>& arena,
                        bool keep_core, CoreRule* rule, int chip_geometry, GeomStats& gs, std::vector<Chip>& out,
                        std::vector<Undecided>& und) {
  // a cell the polygon holds whole: core -- unless mosaicFill's rule (rule != null) puts
  // it in the border set (then its chip is the whole cell, not core)
  auto whole = [&](int64_t id, long i, long j, const std::vector<std::vector<Pt>>* rings) {
    const auto v = rule ? rule->decide(g.center_input(i, j, id), 1) : CoreRule::kCore;
    if (rule && rule->last_flag) {
      Undecided u{id, pid, (uint8_t)rule->last_flag, (uint8_t)(v != CoreRule::kDrop), (uint8_t)(v == CoreRule::kCore), {}};
      write_cell_wkb(rings ? *rings : g.boundary_of(i, j, id), u.wkb, true);
      und.push_back(std::move(u));
    }
    if (v == CoreRule::kDrop) {
      rule->st.dropped++;
      return;
    }
    if (v != CoreRule::kCore) {
      rule->st.demoted++;
      Chip ch{id, pid, 0, 0, arena.size()};
      write_cell_wkb(rings ? *rings : g.boundary_of(i, j, id), arena, true);
      ch.wlen = (uint32_t)(arena.size() - ch.woff);
      out.push_back(ch);
      return;
    }
    Chip ch{id, pid, 1, 0, arena.size()};
    if (keep_core) {
      const auto rs = rings ? *rings : g.boundary_of(i, j, id);
      write_cell_wkb(rs, arena, g.cw_ring(id));
      ch.wlen = (uint32_t)(arena.size() - ch.woff);
    }
    out.push_back(ch);
  };
  // 2. border cells: walk every edge in lattice space; per cell the smallest distance
  // from its centre to a walked sample (samples <= 0.2 apart)
  // (squared distances: the test against far_distance only chooses between two exact
  // constructions of the same chip -- a cell the boundary never reaches gives the same
  // row either way -- so its rounding at the threshold does not matter)
  CellDist& border = t_border;
  double xmin = INFINITY, ymin = INFINITY, xmax = -INFINITY, ymax = -INFINITY;
  double walk_len = 0;
  for (auto& r : lat_rings)
    for (size_t i = 0; i < r.size(); i++) {
      xmin = std::min(xmin, r[i].x), xmax = std::max(xmax, r[i].x);
      ymin = std::min(ymin, r[i].y), ymax = std::max(ymax, r[i].y);
      if (i + 1 < r.size()) walk_len += std::fabs(r[i + 1].x - r[i].x) + std::fabs(r[i + 1].y - r[i].y);
    }
  border.clear();
  if (xmin <= xmax) {
    // the dense window when it is not much larger than the cells the walk visits
    long i0, j0, i1, j1;
    g.cell_window(xmin, ymin, xmax, ymax, &i0, &j0, &i1, &j1);
    if ((double)(i1 - i0 + 1) * (double)(j1 - j0 + 1) <= 64.0 * walk_len + 65536.0) border.clear_dense(i0, j0, i1, j1);
  }
  std::vector<std::pair<long, long>> nb;
  auto touch = [&](const std::pair<long, long>& c, Pt s) {
    const Pt cc = g.center(c.first, c.second);
    const double dx = s.x - cc.x, dy = s.y - cc.y;
    border.touch(c.first, c.second, (float)(dx * dx + dy * dy));
  };
  auto walk = [&]() {
    for (auto& r : lat_rings)
      for (size_t i = 0; i + 1 < r.size(); i++) {
        Pt a = r[i], b = r[i + 1];
        double len = std::hypot(b.x - a.x, b.y - a.y);
        int steps = std::max(1, (int)std::ceil(len / 0.2));
        for (int s = 0; s <= steps; s++) {
          double t = (double)s / steps;
          const Pt q{a.x + t * (b.x - a.x), a.y + t * (b.y - a.y)};
          auto c = g.cell_at(q);
          touch(c, q);
          nb.clear();
          g.neighbors(c.first, c.second, nb);
          for (auto& n : nb) touch(n, q);
        }
      }
  };
  walk();
  if (border.overflow) {
    border.clear();
    walk();
  }
  // 3. interior cells: even-odd scanline over lattice rows (each row's sorted crossings
  // kept: they also place the far border cells below)
  std::vector<std::pair<long, long>> interior;
  const long row0 = ymin <= ymax ? g.row_of(ymin, true) : 0, row1 = ymin <= ymax ? g.row_of(ymax, false) : -1;
  std::vector<std::vector<double>> row_xs((size_t)std::max(0L, row1 - row0 + 1));
  for (long j = row0; j <= row1; j++) {
    double y = g.row_y(j);
    std::vector<double>& xs = row_xs[(size_t)(j - row0)];
    for (auto& r : lat_rings)
      for (size_t i = 0; i + 1 < r.size(); i++) {
        Pt a = r[i], b = r[i + 1];
        if ((a.y > y) != (b.y > y)) xs.push_back(a.x + (y - a.y) * (b.x - a.x) / (b.y - a.y));
      }
    std::sort(xs.begin(), xs.end());
    for (size_t k = 0; k + 1 < xs.size(); k += 2)
      for (long i = g.col_of(xs[k], j, true); i <= g.col_of(xs[k + 1], j, false); i++)
        if (border.get(i, j) < 0) interior.push_back({i, j});
  }
  for (auto& c : interior) {
    int64_t id = g.cell_id(c.first, c.second);
    if (!id || !g.keep(id, c.first, c.second)) continue;
    whole(id, c.first, c.second, nullptr);
  }
  // 4. border cells: clip -- unless the boundary never came near the cell (a ring
  // neighbour of a walked cell): then it lies wholly inside or outside, decided by its
  // centre, without its exact geometry
  std::vector<std::pair<long, long>> bl;
  if (border.dense) {
    for (long a = 0; a < border.wni; a++)  // (in (i, j) order already)
      for (long b = 0; b < border.wnj; b++)
        if (border.w[(size_t)(a * border.wnj + b)] >= 0) bl.push_back({border.wi0 + a, border.wj0 + b});
  } else {
    bl.reserve(border.n);
    for (auto& sl : border.t)
      if (sl.used) bl.push_back({sl.i, sl.j});
    std::sort(bl.begin(), bl.end());
  }
  for (auto& c : bl) {
    const int64_t cid = g.cell_id(c.first, c.second);
    if (!cid || !g.keep(cid, c.first, c.second)) continue;
    const double far = g.far_distance();
    if ((double)border.get(c.first, c.second) > far * far) {
      // no ring comes within 0.65 of the centre (samples <= 0.2 apart): the even-odd count
      // of its row's crossings right of it places it (the centre is on its row: col_x, row_y)
      const Pt cc = g.center(c.first, c.second);
      bool in = false;
      if (c.second >= row0 && c.second <= row1) {
        const auto& xs = row_xs[(size_t)(c.second - row0)];
        in = ((xs.end() - std::upper_bound(xs.begin(), xs.end(), cc.x)) & 1) != 0;
      }
      if (!in) continue;
      whole(cid, c.first, c.second, nullptr);
      continue;
    }
    const auto rings = g.boundary_of(c.first, c.second, cid);
    if (rings.empty()) continue;
    double cminx = INFINITY, cminy = INFINITY, cmaxx = -INFINITY, cmaxy = -INFINITY;
    for (auto& r : rings)
      for (auto& p : r) {
        cminx = std::min(cminx, p.x);
        cmaxx = std::max(cmaxx, p.x);
        cminy = std::min(cminy, p.y);
        cmaxy = std::max(cmaxy, p.y);
      }
    // every ring of the cell in convex pieces; the cell is core when each ring lies in
    // the polygon's interior (tested from a point inside the ring's first piece)
    std::vector<std::vector<Pt>> pieces;
    bool inside = true;
    for (auto& r : rings) {
      const auto pc = convex_pieces(r);
      Pt cc = {0, 0};
      for (size_t k = 0; k + 1 < pc[0].size(); k++) {
        cc.x += pc[0][k].x;
        cc.y += pc[0][k].y;
      }
      cc.x /= (pc[0].size() - 1);
      cc.y /= (pc[0].size() - 1);
      inside = inside && cell_in_polygon(r, pc, cc, poly);
      pieces.insert(pieces.end(), pc.begin(), pc.end());
    }
    if (inside) {
      whole(cid, c.first, c.second, &rings);
      continue;
    }
    // (a concave cell is clipped piece by piece: the chip is then a MULTIPOLYGON whose
    // parts meet along the pieces' diagonals -- the same point set, and PointLocator's
    // Mod-2 rule puts a point on such a seam in the interior, as for the whole cell)
    std::vector<mgpu::wkb::Polygon> parts;  // (Sutherland-Hodgman)
    std::vector<mgpu::ovl::Rings> pcs;      // (overlay)
    double area = 0;
    if (chip_geometry == kChipOverlay) {
      // polygon INTERSECTION cell as JTS OverlayNG computes it, then coerceChipGeometry
      // (jts_overlay.h)
      bool lower = false;
      t_clip.build(poly.parts, poly.ring_ccw, rings, pcs, &lower, &poly.grid);
      for (auto& pc : pcs)
        for (size_t k = 0; k < pc.size(); k++) area += (k == 0 ? 1.0 : -1.0) * std::fabs(mgpu::ovl::signed_area(pc[k]));
      if (pcs.empty() || area <= 0) continue;  // empty chip (lines / points only): dropped
      gs.overlay_chips++;
      if (pcs.size() > 1) gs.multi_piece++;
      if (lower) gs.lower_dim++;
      if (lower || poly.multi != (pcs.size() > 1)) {
        size_t before = 0, after = 0;
        for (auto& pc : pcs)
          for (auto& r : pc) before += r.size();
        mgpu::ovl::renode_with_cell(pcs, rings);
        for (auto& pc : pcs)
          for (auto& r : pc) after += r.size();
        gs.coerced++;
        gs.coerce_nodes += (int64_t)(after - before);
      }
    }
    if (chip_geometry == kChipSutherlandHodgman)
    for (auto& piece : pieces)
    for (auto& part : poly.parts) {
      mgpu::wkb::Polygon out_part;
      bool shell_ok = false;
      for (size_t ri = 0; ri < part.size(); ri++) {
        const auto& ring = part[ri];
        double rminx = INFINITY, rminy = INFINITY, rmaxx = -INFINITY, rmaxy = -INFINITY;
        for (auto& p : ring) {
          rminx = std::min(rminx, p.x);
          rmaxx = std::max(rmaxx, p.x);
          rminy = std::min(rminy, p.y);
          rmaxy = std::max(rmaxy, p.y);
        }
        std::vector<Pt> clipped;
        if (!(rmaxx < cminx || rminx > cmaxx || rmaxy < cminy || rminy > cmaxy)) clipped = clip_ring(ring, piece);
        double a = clipped.empty() ? 0 : std::fabs(ring_area(clipped));
        if (ri == 0) {
          if (a <= 0) break;
          shell_ok = true;
          area += a;
        } else {
          if (a <= 0) continue;
          area -= a;
        }
        std::vector<double> flat;
        for (auto& p : clipped) {
          flat.push_back(p.x);
          flat.push_back(p.y);
        }
        out_part.push_back(std::move(flat));
      }
      if (shell_ok) parts.push_back(std::move(out_part));
    }
    if ((chip_geometry == kChipOverlay ? pcs.empty() : parts.empty()) || area <= 0) continue;  // empty chip: dropped
    auto write_chip = [&](std::vector<uint8_t>& w) {
      if (chip_geometry == kChipOverlay) mgpu::wkb::write_polygons_pts<false>(w, pcs, false);
      else mgpu::wkb::write_polygons(w, parts);
    };
    if (rule) {
      // mosaicFill's sets: a cell whose centre is deep enough inside is in the core set
      // (its chip is the whole cell, core, even where the polygon does not cover it); one
      // whose centre is beyond the border band is never visited
      const auto v = rule->decide(g.center_input(c.first, c.second, cid), -1);
      if (rule->last_flag) {
        Undecided u{cid, pid, (uint8_t)rule->last_flag, (uint8_t)(v != CoreRule::kDrop), (uint8_t)(v == CoreRule::kCore),
                    {}};
        write_chip(u.wkb);
        und.push_back(std::move(u));
      }
      if (v == CoreRule::kDrop) {
        rule->st.dropped++;
        continue;
      }
      if (v == CoreRule::kCore) {
        rule->st.promoted++;
        Chip ch{cid, pid, 1, 0, arena.size()};
        if (keep_core) write_cell_wkb(rings, arena, g.cw_ring(cid));
        ch.wlen = (uint32_t)(arena.size() - ch.woff);
        out.push_back(ch);
        continue;
      }
    }
    Chip ch{cid, pid, 0, 0, arena.size()};
    write_chip(arena);
    ch.wlen = (uint32_t)(arena.size() - ch.woff);
    out.push_back(ch);
  }
}

// squared chord distances from a point (degrees) to the 20 face centres
void face_distances(double lon_deg, double lat_deg, double* d) {
  double lat = lat_deg * M_PI / 180.0, lon = lon_deg * M_PI / 180.0;
  double x = cos(lon) * cos(lat), y = sin(lon) * cos(lat), z = sin(lat);
  for (int f = 0; f < 20; f++) {
    double dx = H3T_FACE_CENTER_POINT[f][0] - x, dy = H3T_FACE_CENTER_POINT[f][1] - y,
           dz = H3T_FACE_CENTER_POINT[f][2] - z;
    d[f] = dx * dx + dy * dy + dz * dz;
  }
}

// a ring densified along its lon/lat edges: pieces of at most `step` degrees
std::vector<Pt> densify(const std::vector<Pt>& r, double step) {
  std::vector<Pt> o;
  for (size_t i = 0; i + 1 < r.size(); i++) {
    const Pt a = r[i], b = r[i + 1];
    const int n = std::max(1, (int)std::ceil(std::max(std::fabs(b.x - a.x), std::fabs(b.y - a.y)) / step));
    for (int k = 0; k < n; k++) o.push_back({a.x + (b.x - a.x) * k / n, a.y + (b.y - a.y) * k / n});
  }
  if (!r.empty()) o.push_back(r.back());
  return o;
}

// H3: every face whose cells can meet the polygon, with the polygon's rings densified
// (returns false when the polygon is too large for the per-face projection)
bool h3_faces(const Polygon& poly, int res, std::vector<std::vector<Pt>>& dense, std::vector<int>& faces) {
  // centre spacing of res-r cells ~ 0.3 / sqrt7^r rad; pieces of a tenth of it, or of half
  // of it from res 5 (a lon/lat edge bows off its lattice chord by ~L^2 k / 8 with k the
  // curvature in cells^-1, < 1e-3 there: far below the walk's 0.07 margin -- and the walk
  // samples every 0.2 along the chords anyway)
  double cell = 0.3;
  for (int i = 0; i < res; i++) cell /= 2.6457513110645906;
  const double step = std::min(1.0, (res >= 5 ? 0.5 : 0.1) * cell * 180.0 / M_PI);
  // a cell centred on face g can reach a point p only if g is nearest to some point
  // within a cell radius (<= 0.25 / sqrt7^r rad) of p; moving p by dt changes a
  // squared chord distance by <= 2 sin(t) dt, so d_g(p) - d_best(p) < 0.9 / sqrt7^r
  const double near_edge = 2.5 * cell;
  int used[20] = {0};  // 2: the nearest face of a vertex, 1: across a nearby face edge
  double d[20], dmax[20] = {0};
  for (auto& part : poly.parts)
    for (auto& ring : part) {
      dense.push_back(densify(ring, step));
      for (auto& p : dense.back()) {
        face_distances(p.x, p.y, d);
        int best = 0;
        for (int f = 1; f < 20; f++)
          if (d[f] < d[best]) best = f;
        used[best] = 2;
        for (int f = 0; f < 20; f++) {
          if (d[f] - d[best] < near_edge && !used[f]) used[f] = 1;
          dmax[f] = std::max(dmax[f], d[f]);
        }
      }
    }
  // the gnomonic projection onto a face must stay inside its hemisphere: a face across
  // an edge that some vertex is > ~84 degrees from is too far to matter; a face that is
  // some vertex's nearest must project the whole polygon
  for (int f = 0; f < 20; f++) {
    if (!used[f]) continue;
    if (dmax[f] > 1.8) {
      if (used[f] == 2) return false;
      continue;
    }
    faces.push_back(f);
  }
  return true;
}

}  // namespace

// the previous result's release (mgpu_tess_destroy)
struct TessRelease {
  std::mutex mu;
  std::thread th;
  void join() {
    std::lock_guard<std::mutex> g(mu);
    if (th.joinable()) th.join();
  }
  ~TessRelease() { join(); }
};
static TessRelease g_tess_release;

struct mgpu_tess {
  std::vector<Chip> chips;
  std::vector<uint32_t> chip_arena;          // chips[i]'s polygon (its arena)
  std::vector<std::vector<uint8_t>> arenas;  // per polygon
  CoreStats core_stats;
  GeomStats geom_stats;
  std::vector<Undecided> undecided;
};

namespace {

// getBufferRadius (H3IndexSystem.scala:79-90): the centroid's cell at `res`; its shell
// points' largest distance to the centroid (planar degrees) -- or, when indexToGeometry
// gives several parts (a cell across the antimeridian), the length of the longest part
// boundary, as the reference's second case computes it
double h3_buffer_radius(const Polygon& poly, int res) {
  double sx = 0, sy = 0, sa = 0;
  for (auto& part : poly.parts)
    for (size_t k = 0; k < part.size(); k++) {
      const auto& r = part[k];
      double a = 0, cx = 0, cy = 0;
      for (size_t i = 0; i + 1 < r.size(); i++) {
        const double cr = r[i].x * r[i + 1].y - r[i + 1].x * r[i].y;
        a += cr;
        cx += (r[i].x + r[i + 1].x) * cr;
        cy += (r[i].y + r[i + 1].y) * cr;
      }
      if (a == 0) continue;
      const double w = std::fabs(a / 2) * (k == 0 ? 1.0 : -1.0);
      sx += w * cx / (3 * a);
      sy += w * cy / (3 * a);
      sa += w;
    }
  if (!(sa > 0)) return 0;
  double gx = sx / sa, gy = sy / sa;
  if (gx > 180) gx = -180 + std::fmod(gx, 180.0);
  else if (gx < -180) gx = 180 - std::fmod(gx, 180.0);
  bool tie = false;
  const uint64_t id = mgpu::h3::point_to_cell(gx, gy, res, &tie);
  if (!id) return 0;
  const auto rings = h3_cell_rings(id, res);
  double r = 0;
  if (rings.size() == 1) {
    for (auto& q : rings[0]) r = std::max(r, std::hypot(q.x - gx, q.y - gy));
  } else {
    for (auto& ring : rings) {
      double len = 0;
      for (size_t i = 0; i + 1 < ring.size(); i++) len += std::hypot(ring[i + 1].x - ring[i].x, ring[i + 1].y - ring[i].y);
      r = std::max(r, len);
    }
  }
  return r;
}

}  // namespace

extern "C" {

int32_t mgpu_tessellate(int32_t index_system, int32_t res, int64_t n_polys, const int32_t* polygon_id,
                        const int64_t* poly_part_off, const int64_t* part_ring_off, const int64_t* ring_off,
                        const double* xy, int32_t keep_core_geometries, mgpu_tess** out) {
  return mgpu_tessellate_ex(index_system, res, n_polys, polygon_id, poly_part_off, part_ring_off, ring_off, xy,
                            keep_core_geometries, MGPU_CORE_MOSAICFILL, out);
}

int32_t mgpu_tessellate_ex(int32_t index_system, int32_t res, int64_t n_polys, const int32_t* polygon_id,
                           const int64_t* poly_part_off, const int64_t* part_ring_off, const int64_t* ring_off,
                           const double* xy, int32_t keep_core_geometries, int32_t core_rule, mgpu_tess** out) {
  return mgpu_tessellate_geom(index_system, res, n_polys, polygon_id, poly_part_off, part_ring_off, ring_off, xy,
                              nullptr, keep_core_geometries, core_rule, MGPU_CHIPS_OVERLAY, out);
}

int32_t mgpu_tessellate_geom(int32_t index_system, int32_t res, int64_t n_polys, const int32_t* polygon_id,
                             const int64_t* poly_part_off, const int64_t* part_ring_off, const int64_t* ring_off,
                             const double* xy, const uint8_t* poly_type, int32_t keep_core_geometries,
                             int32_t core_rule, int32_t chip_geometry, mgpu_tess** out) {
  if (!out || n_polys < 0) return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellate: bad arguments");
  g_tess_release.join();  // (the previous result's memory back before this one allocates)
  if (chip_geometry != MGPU_CHIPS_OVERLAY && chip_geometry != MGPU_CHIPS_SUTHERLAND_HODGMAN)
    return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellate: unknown chip geometry %d", chip_geometry);
  for (int64_t p = 0; poly_type && p < n_polys; p++)
    if (poly_type[p] != 3 && poly_type[p] != 6)
      return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellate: polygon type %d (3 = POLYGON, 6 = MULTIPOLYGON)",
                             (int)poly_type[p]);
  if (core_rule != MGPU_CORE_MOSAICFILL && core_rule != MGPU_CORE_CLIP && core_rule != MGPU_CORE_DISTANCE)
    return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellate: unknown core rule %d", core_rule);
  if (int32_t st = mgpu_check_resolution(index_system, res)) return st;
  if (index_system == MGPU_BNG && res == -1)
    // 500km ids depend on the easting letter only: no square cells to clip
    return mgpu::set_error(MGPU_E_RESOLUTION, "BNG resolution -1 (500km) cannot be tessellated");
  // polygons are independent: tessellate them in parallel into per-polygon chip lists,
  // then concatenate in input order (the output does not depend on the schedule)
  std::vector<std::vector<Chip>> per(n_polys);
  std::vector<std::vector<uint8_t>> arena(n_polys);
  std::vector<uint8_t> bad_poly(n_polys, 0);
  std::vector<CoreStats> pstats(n_polys);
  std::vector<GeomStats> gstats(n_polys);
  std::vector<std::vector<Undecided>> pund(n_polys);
  mgpu::parallel_for(n_polys, 64, [&](int64_t pb, int64_t pe, int) {
    for (int64_t p = pb; p < pe; p++) {
      Polygon poly;
      for (int64_t q = poly_part_off[p]; q < poly_part_off[p + 1]; q++) {
        std::vector<std::vector<Pt>> rings;
        for (int64_t r = part_ring_off[q]; r < part_ring_off[q + 1]; r++) {
          std::vector<Pt> ring;
          for (int64_t v = ring_off[r]; v < ring_off[r + 1]; v++) ring.push_back({xy[2 * v], xy[2 * v + 1]});
          if (ring.size() >= 2 && (ring.front().x != ring.back().x || ring.front().y != ring.back().y))
            ring.push_back(ring.front());
          if (ring.size() >= 4) rings.push_back(std::move(ring));
          else if (rings.empty()) break;  // degenerate shell: empty part
        }
        if (!rings.empty()) poly.parts.push_back(std::move(rings));
      }
      if (poly.parts.empty()) continue;
      // the geometry's type decides coerceChipGeometry (a MULTIPOLYGON unless told, when it
      // has several parts); each ring's orientation gives the interior's side of its edges
      poly.multi = poly_type ? poly_type[p] == 6 : poly.parts.size() > 1;
      for (auto& part : poly.parts)
        for (auto& ring : part) {
          poly.ring_ccw.push_back(mgpu::ovl::is_ccw(ring));
          poly.ring_ptr.push_back(&ring);
        }
      {
        // the segment grid's buckets about one cell (H3: the centre spacing at res)
        double cell = index_system == MGPU_H3 ? 20.0 : BngGrid(res).edge;
        for (int r = 0; index_system == MGPU_H3 && r < res; r++) cell /= 2.6457513110645906;
        poly.grid.build(poly.parts, cell);
      }
      // mosaicFill's core set (CoreRule) unless the clip rule was asked for
      CoreRule rule_storage;
      CoreRule* rule = nullptr;
      if (core_rule == MGPU_CORE_MOSAICFILL || core_rule == MGPU_CORE_DISTANCE) {
        rule_storage.r = index_system == MGPU_H3 ? h3_buffer_radius(poly, res)
                                                 : BngGrid(res).edge * std::sqrt(2.0) / 2.0;
        if (rule_storage.r > 0) {
          rule_storage.poly = &poly;
          rule_storage.distance_only = core_rule == MGPU_CORE_DISTANCE;
          rule_storage.seg.build(poly, rule_storage.r);
          rule = &rule_storage;
        }
      }
      if (index_system == MGPU_H3) {
        bool in_range = true;
        for (auto& part : poly.parts)
          for (auto& ring : part)
            for (auto& q : ring) in_range = in_range && std::fabs(q.x) <= 180.0 && std::fabs(q.y) <= 90.0;
        if (!in_range) {
          bad_poly[p] = 2;
          continue;
        }
        std::vector<std::vector<Pt>> dense;
        std::vector<int> faces;
        if (!h3_faces(poly, res, dense, faces)) {
          bad_poly[p] = 1;
          continue;
        }
        for (int face : faces) {
          H3Grid g(face, res);
          std::vector<std::vector<Pt>> lat_rings;
          for (auto& r : dense) {
            std::vector<Pt> lr;
            lr.reserve(r.size());
            for (auto& q : r) lr.push_back(g.to_lattice(q));
            lat_rings.push_back(std::move(lr));
          }
          tessellate_polygon(g, poly, lat_rings, polygon_id[p], arena[p], keep_core_geometries != 0, rule, chip_geometry,
                             gstats[p], per[p], pund[p]);
        }
        // a cell reached twice (two lattice positions around a pentagon map to one id):
        // its chip is computed from the id, so the copies are equal -- keep the first
        // (below, after the sort)
      } else {
        BngGrid g(res);
        std::vector<std::vector<Pt>> lat_rings;
        for (auto& part : poly.parts)
          for (auto& ring : part) {
            std::vector<Pt> lr;
            for (auto& q : ring) lr.push_back(g.to_lattice(q));
            lat_rings.push_back(std::move(lr));
          }
        tessellate_polygon(g, poly, lat_rings, polygon_id[p], arena[p], keep_core_geometries != 0, rule, chip_geometry,
                           gstats[p], per[p], pund[p]);
      }
      // the polygon's rows in cell order (stable: a repeated id keeps its first chip) -- the
      // output does not depend on which cells the walk classified as interior or border
      // (the chip-table blob keeps input rows, so the order is part of its bytes)
      std::stable_sort(per[p].begin(), per[p].end(), [](const Chip& a, const Chip& b) { return a.cell < b.cell; });
      per[p].erase(std::unique(per[p].begin(), per[p].end(), [](const Chip& a, const Chip& b) { return a.cell == b.cell; }),
                   per[p].end());
      if (rule) pstats[p] = rule->st;
    }
  });
  for (int64_t p = 0; p < n_polys; p++) {
    if (bad_poly[p] == 1)
      return mgpu::set_error(MGPU_E_UNSUPPORTED,
                             "tessellate: polygon %d is too large for this builder (more than ~84 degrees from an "
                             "icosahedron face it touches); split it first", polygon_id[p]);
    if (bad_poly[p] == 2)
      return mgpu::set_error(MGPU_E_UNSUPPORTED,
                             "tessellate: polygon %d has coordinates outside [-180, 180] x [-90, 90] (wrap them "
                             "first, as the reference's alignToGrid does)", polygon_id[p]);
  }
  mgpu_tess* t = new mgpu_tess();
  for (auto& v : pund)
    for (auto& u : v) t->undecided.push_back(std::move(u));
  for (auto& q : gstats) {
    t->geom_stats.overlay_chips += q.overlay_chips;
    t->geom_stats.multi_piece += q.multi_piece;
    t->geom_stats.coerced += q.coerced;
    t->geom_stats.coerce_nodes += q.coerce_nodes;
    t->geom_stats.lower_dim += q.lower_dim;
  }
  for (auto& q : pstats) {
    t->core_stats.demoted += q.demoted;
    t->core_stats.promoted += q.promoted;
    t->core_stats.dropped += q.dropped;
    t->core_stats.ambiguous += q.ambiguous;
    t->core_stats.carved_tests += q.carved_tests;
    t->core_stats.band_tests += q.band_tests;
    t->core_stats.core_below_r += q.core_below_r;
    t->core_stats.border_above_r += q.border_above_r;
    t->core_stats.band_dropped += q.band_dropped;
    t->core_stats.dp_sensitive += q.dp_sensitive;
    t->core_stats.unresolved += q.unresolved;
    t->core_stats.carved_empty += q.carved_empty;
  }
  size_t total = 0;
  for (auto& v : per) total += v.size();
  t->chips.reserve(total);
  t->chip_arena.reserve(total);
  for (int64_t p = 0; p < n_polys; p++) {
    t->chips.insert(t->chips.end(), per[p].begin(), per[p].end());
    t->chip_arena.insert(t->chip_arena.end(), per[p].size(), (uint32_t)p);
    std::vector<Chip>().swap(per[p]);
  }
  t->arenas.swap(arena);
  *out = t;
  return MGPU_OK;
}

int32_t mgpu_tess_result_sizes(const mgpu_tess* t, int64_t* n_chips, int64_t* wkb_bytes) {
  if (!t) return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellation result is NULL");
  int64_t b = 0;
  for (auto& c : t->chips) b += (int64_t)c.wlen;
  if (n_chips) *n_chips = (int64_t)t->chips.size();
  if (wkb_bytes) *wkb_bytes = b;
  return MGPU_OK;
}

int32_t mgpu_tess_result_copy(const mgpu_tess* t, int64_t* cell, int32_t* polygon_id, uint8_t* is_core,
                              int64_t* wkb_offsets, uint8_t* wkb) {
  if (!t) return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellation result is NULL");
  const int64_t n = (int64_t)t->chips.size();
  int64_t off = 0;
  for (int64_t i = 0; i < n; i++) {
    wkb_offsets[i] = off;
    off += (int64_t)t->chips[i].wlen;
  }
  wkb_offsets[n] = off;
  // (the columns and the bytes in parallel: first-touch of the caller's fresh pages too)
  mgpu::parallel_for(n, 1 << 15, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; i++) {
      const Chip& c = t->chips[i];
      cell[i] = c.cell;
      polygon_id[i] = c.poly;
      is_core[i] = c.core;
      if (c.wlen) memcpy(wkb + wkb_offsets[i], t->arenas[t->chip_arena[i]].data() + c.woff, c.wlen);
    }
  });
  return MGPU_OK;
}

int32_t mgpu_tess_result_stats(const mgpu_tess* t, int64_t* out6) {
  if (!t || !out6) return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellation result is NULL");
  int64_t core = 0;
  for (auto& c : t->chips) core += c.core;
  out6[0] = (int64_t)t->chips.size();
  out6[1] = core;
  out6[2] = t->core_stats.demoted;
  out6[3] = t->core_stats.promoted;
  out6[4] = t->core_stats.dropped;
  out6[5] = t->core_stats.ambiguous;
  return MGPU_OK;
}

int32_t mgpu_tess_result_core_stats(const mgpu_tess* t, int64_t* out, int32_t n) {
  if (!t || !out || n < 0) return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellation result is NULL");
  int64_t core = 0;
  for (auto& c : t->chips) core += c.core;
  const CoreStats& s = t->core_stats;
  const int64_t v[] = {(int64_t)t->chips.size(), core, s.demoted, s.promoted, s.dropped, s.ambiguous,
                       s.carved_tests, s.band_tests, s.core_below_r, s.border_above_r, s.band_dropped,
                       s.dp_sensitive, s.unresolved, s.carved_empty, t->geom_stats.overlay_chips,
                       t->geom_stats.multi_piece, t->geom_stats.coerced, t->geom_stats.coerce_nodes,
                       t->geom_stats.lower_dim};
  for (int32_t i = 0; i < n; i++) out[i] = i < (int32_t)(sizeof(v) / sizeof(v[0])) ? v[i] : 0;
  return MGPU_OK;
}

int32_t mgpu_tess_result_undecided(const mgpu_tess* t, int64_t* n, int64_t* wkb_bytes, int64_t* cell, int32_t* poly,
                                   uint8_t* kind_kept_core, int64_t* wkb_offsets, uint8_t* wkb) {
  if (!t || !n) return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellation result is NULL");
  *n = (int64_t)t->undecided.size();
  int64_t b = 0;
  for (auto& u : t->undecided) b += (int64_t)u.wkb.size();
  if (wkb_bytes) *wkb_bytes = b;
  if (!cell) return MGPU_OK;
  int64_t off = 0;
  for (size_t i = 0; i < t->undecided.size(); i++) {
    const Undecided& u = t->undecided[i];
    cell[i] = u.cell;
    poly[i] = u.poly;
    kind_kept_core[3 * i] = u.kind, kind_kept_core[3 * i + 1] = u.kept, kind_kept_core[3 * i + 2] = u.core;
    wkb_offsets[i] = off;
    if (!u.wkb.empty()) memcpy(wkb + off, u.wkb.data(), u.wkb.size());
    off += (int64_t)u.wkb.size();
  }
  wkb_offsets[t->undecided.size()] = off;
  return MGPU_OK;
}

int32_t mgpu_tess_destroy(mgpu_tess* t) {
  if (!t) return MGPU_OK;
  // (9.4M rows on C3: 0.2 s of page returns -- handed to a helper thread, joined by the
  // next tessellation and at exit, so at most one result is being freed at a time)
  std::lock_guard<std::mutex> g(g_tess_release.mu);
  if (g_tess_release.th.joinable()) g_tess_release.th.join();
  try {
    g_tess_release.th = std::thread([t] { delete t; });
  } catch (...) {
    delete t;
  }
  return MGPU_OK;
}

int32_t mgpu_test_overlay_verify(int32_t on, int64_t* out2) {
  auto& v = mgpu::ovl::g_overlay_verify;
  if (out2) out2[0] = v.shortcut.load(), out2[1] = v.differ.load();
  if (on) v.shortcut = 0, v.differ = 0;
  v.on = on != 0;
  return MGPU_OK;
}

int32_t mgpu_test_h3_boundary_host(const int64_t* cells, int64_t n, double* out_lonlat, int32_t* out_nverts,
                                   double* out_center) {
  for (int64_t i = 0; i < n; i++) {
    const uint64_t h = (uint64_t)cells[i];
    const int res = (int)((h >> 52) & 15), bc = (int)((h >> 45) & 127);
    if (((h >> 59) & 15) != 1 || bc >= H3T_NUM_BASE_CELLS || res > 15)
      return mgpu::set_error(MGPU_E_INVALID_ARG, "h3 boundary: not a cell id");
    const auto b = mgpu::h3b::cell_boundary(h);
    out_nverts[i] = (int32_t)b.size();
    for (size_t v = 0; v < b.size() && v < 10; v++) {
      out_lonlat[i * 20 + 2 * v] = mgpu::h3b::to_degrees(b[v].lon);
      out_lonlat[i * 20 + 2 * v + 1] = mgpu::h3b::to_degrees(b[v].lat);
    }
    const auto c = mgpu::h3b::cell_center(h);
    out_center[2 * i] = mgpu::h3b::to_degrees(c.lon);
    out_center[2 * i + 1] = mgpu::h3b::to_degrees(c.lat);
  }
  return MGPU_OK;
}

int32_t mgpu_test_h3_cell_wkb_host(int64_t cell, uint8_t* out, int64_t cap, int64_t* out_len) {
  const uint64_t h = (uint64_t)cell;
  const int res = (int)((h >> 52) & 15), bc = (int)((h >> 45) & 127);
  if (((h >> 59) & 15) != 1 || bc >= H3T_NUM_BASE_CELLS || !out_len)
    return mgpu::set_error(MGPU_E_INVALID_ARG, "h3 cell wkb: not a cell id");
  auto rings = h3_cell_rings(h, res);
  if (h == pole_cell(false, res)) rings = reversed(rings);  // as H3Grid::cw_ring
  std::vector<uint8_t> w;
  write_cell_wkb(rings, w);
  *out_len = (int64_t)w.size();
  if ((int64_t)w.size() > cap || !out) return mgpu::set_error(MGPU_E_CAPACITY, "h3 cell wkb: %zu bytes", w.size());
  std::memcpy(out, w.data(), w.size());
  return MGPU_OK;
}

}  // extern "C"
