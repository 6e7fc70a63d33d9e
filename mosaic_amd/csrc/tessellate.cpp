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
// Limitation: an H3 polygon must lie on a single icosahedron face.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <set>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/mosaic_gpu.h"
#include "error.h"
#include "bng_core.h"
#include "h3_core.h"
#include "parallel.h"
#include "wkb.h"

namespace {

thread_local std::string t_err;

struct Pt {
  double x, y;
};

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
    for (size_t i = 0; i < in.size(); i++) {
      Pt cur = in[i], prev = in[(i + in.size() - 1) % in.size()];
      double sc = side(cur), sp = side(prev);
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
};

double orient(Pt a, Pt b, Pt c) { return (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x); }

bool segments_touch(Pt a, Pt b, Pt c, Pt d) {
  double o1 = orient(a, b, c), o2 = orient(a, b, d), o3 = orient(c, d, a), o4 = orient(c, d, b);
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
    if (orient(cell[i], cell[i + 1], p) < 0) return false;
  return true;
}


// ---------------------------------------------------------------- grids

struct Grid {
  virtual ~Grid() {}
  // lattice-space coordinate of an input point
  virtual Pt to_lattice(Pt p) const = 0;
  // lattice cell containing a lattice-space point
  virtual std::pair<long, long> cell_at(Pt q) const = 0;
  virtual Pt center(long i, long j) const = 0;  // lattice space
  virtual void neighbors(long i, long j, std::vector<std::pair<long, long>>& out) const = 0;
  // cell id (0 = not representable) and its boundary in input coords (closed, ccw)
  virtual int64_t cell_id(long i, long j) const = 0;
  virtual std::vector<Pt> boundary(long i, long j) const = 0;
  // lattice row/column iteration for the scanline: row index of a lattice y,
  // y of a row, and the column index of the cell centred at lattice x in a row
  virtual double row_y(long j) const = 0;
  virtual long row_of(double y, bool up) const = 0;
  virtual double col_x(long i, long j) const = 0;
  virtual long col_of(double x, long j, bool up) const = 0;
};

struct H3Grid : Grid {
  int face, res;
  explicit H3Grid(int f, int r) : face(f), res(r) {}
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
  std::vector<Pt> boundary(long i, long j) const override {
    Pt c = center(i, j);
    std::vector<Pt> b;
    const double rad = 1.0 / std::sqrt(3.0);
    for (int k = 0; k < 6; k++) {
      double a = (30.0 + 60.0 * k) * M_PI / 180.0;
      b.push_back(to_geo({c.x + rad * cos(a), c.y + rad * sin(a)}));
    }
    b.push_back(b[0]);
    if (ring_area(b) < 0) std::reverse(b.begin(), b.end());
    return b;
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
};

struct BngGrid : Grid {
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
  std::vector<Pt> boundary(long i, long j) const override {
    double x = i * edge, y = j * edge;
    return {{x, y}, {x + edge, y}, {x + edge, y + edge}, {x, y + edge}, {x, y}};
  }
  double row_y(long j) const override { return j + 0.5; }
  long row_of(double y, bool up) const override { return up ? (long)std::ceil(y - 0.5) : (long)std::floor(y - 0.5); }
  double col_x(long i, long) const override { return i + 0.5; }
  long col_of(double x, long, bool up) const override {
    return up ? (long)std::ceil(x - 0.5) : (long)std::floor(x - 0.5);
  }
};

struct Chip {
  int64_t cell;
  int32_t poly;
  uint8_t core;
  std::vector<uint8_t> wkb;
};

struct PairHash {
  size_t operator()(const std::pair<long, long>& p) const { return std::hash<long>()(p.first * 1000003L ^ p.second); }
};

// Exact test that the cell lies in the interior of one part of the polygon: no ring
// vertex in/on the cell, no ring edge touching a cell edge, the cell centre inside
// the shell and outside every hole.  Such a cell's chip IS the cell geometry
// (isCore = coerced.equals(indexGeom), IndexSystem.scala:185).
bool cell_in_polygon(const std::vector<Pt>& cellb, Pt cc, const Polygon& poly) {
  double cminx = INFINITY, cminy = INFINITY, cmaxx = -INFINITY, cmaxy = -INFINITY;
  for (auto& p : cellb) {
    cminx = std::min(cminx, p.x);
    cmaxx = std::max(cmaxx, p.x);
    cminy = std::min(cminy, p.y);
    cmaxy = std::max(cmaxy, p.y);
  }
  for (auto& part : poly.parts)
    for (auto& ring : part)
      for (size_t i = 0; i + 1 < ring.size(); i++) {
        Pt a = ring[i], b = ring[i + 1];
        if (std::max(a.x, b.x) < cminx || std::min(a.x, b.x) > cmaxx || std::max(a.y, b.y) < cminy ||
            std::min(a.y, b.y) > cmaxy)
          continue;
        if (in_convex(cellb, a)) return false;
        for (size_t k = 0; k + 1 < cellb.size(); k++)
          if (segments_touch(a, b, cellb[k], cellb[k + 1])) return false;
      }
  for (auto& part : poly.parts) {
    if (!point_in_ring(part[0], cc)) continue;
    bool in_hole = false;
    for (size_t r = 1; r < part.size(); r++)
      if (point_in_ring(part[r], cc)) in_hole = true;
    if (!in_hole) return true;
  }
  return false;
}

void tessellate_polygon(const Grid& g, const Polygon& poly, int32_t pid, bool keep_core, std::vector<Chip>& out) {
  // lattice-space copy of every ring
  std::vector<std::vector<Pt>> lat_rings;
  std::vector<const std::vector<Pt>*> geo_rings;
  for (auto& part : poly.parts)
    for (auto& ring : part) {
      std::vector<Pt> lr;
      for (auto& p : ring) lr.push_back(g.to_lattice(p));
      lat_rings.push_back(std::move(lr));
      geo_rings.push_back(&ring);
    }
  // 2. border cells: walk every edge in lattice space
  std::unordered_set<std::pair<long, long>, PairHash> border;
  std::vector<std::pair<long, long>> nb;
  for (auto& r : lat_rings)
    for (size_t i = 0; i + 1 < r.size(); i++) {
      Pt a = r[i], b = r[i + 1];
      double len = std::hypot(b.x - a.x, b.y - a.y);
      int steps = std::max(1, (int)std::ceil(len / 0.2));
      for (int s = 0; s <= steps; s++) {
        double t = (double)s / steps;
        auto c = g.cell_at({a.x + t * (b.x - a.x), a.y + t * (b.y - a.y)});
        border.insert(c);
        nb.clear();
        g.neighbors(c.first, c.second, nb);
        for (auto& n : nb) border.insert(n);
      }
    }
  // 3. interior cells: even-odd scanline over lattice rows
  double ymin = INFINITY, ymax = -INFINITY;
  for (auto& r : lat_rings)
    for (auto& p : r) {
      ymin = std::min(ymin, p.y);
      ymax = std::max(ymax, p.y);
    }
  std::vector<std::pair<long, long>> interior;
  if (ymin <= ymax) {
    for (long j = g.row_of(ymin, true); j <= g.row_of(ymax, false); j++) {
      double y = g.row_y(j);
      std::vector<double> xs;
      for (auto& r : lat_rings)
        for (size_t i = 0; i + 1 < r.size(); i++) {
          Pt a = r[i], b = r[i + 1];
          if ((a.y > y) != (b.y > y)) xs.push_back(a.x + (y - a.y) * (b.x - a.x) / (b.y - a.y));
        }
      std::sort(xs.begin(), xs.end());
      for (size_t k = 0; k + 1 < xs.size(); k += 2)
        for (long i = g.col_of(xs[k], j, true); i <= g.col_of(xs[k + 1], j, false); i++)
          if (!border.count({i, j})) interior.push_back({i, j});
    }
  }
  for (auto& c : interior) {
    int64_t id = g.cell_id(c.first, c.second);
    if (!id) continue;
    Chip ch{id, pid, 1, {}};
    if (keep_core) {
      auto b = g.boundary(c.first, c.second);
      std::vector<mgpu::wkb::Polygon> parts(1);
      std::vector<double> flat;
      for (auto& p : b) {
        flat.push_back(p.x);
        flat.push_back(p.y);
      }
      parts[0].push_back(flat);
      mgpu::wkb::write_polygons(ch.wkb, parts);
    }
    out.push_back(std::move(ch));
  }
  // 4. border cells: clip
  std::vector<std::pair<long, long>> bl(border.begin(), border.end());
  std::sort(bl.begin(), bl.end());
  for (auto& c : bl) {
    auto cellb = g.boundary(c.first, c.second);
    double cminx = INFINITY, cminy = INFINITY, cmaxx = -INFINITY, cmaxy = -INFINITY;
    for (auto& p : cellb) {
      cminx = std::min(cminx, p.x);
      cmaxx = std::max(cmaxx, p.x);
      cminy = std::min(cminy, p.y);
      cmaxy = std::max(cmaxy, p.y);
    }
    double cell_area = std::fabs(ring_area(cellb));
    Pt cc = {0, 0};
    for (size_t k = 0; k + 1 < cellb.size(); k++) {
      cc.x += cellb[k].x;
      cc.y += cellb[k].y;
    }
    cc.x /= (cellb.size() - 1);
    cc.y /= (cellb.size() - 1);
    if (cell_in_polygon(cellb, cc, poly)) {
      int64_t id = g.cell_id(c.first, c.second);
      if (!id) continue;
      Chip ch{id, pid, 1, {}};
      if (keep_core) {
        std::vector<mgpu::wkb::Polygon> cp(1);
        std::vector<double> flat;
        for (auto& p : cellb) {
          flat.push_back(p.x);
          flat.push_back(p.y);
        }
        cp[0].push_back(flat);
        mgpu::wkb::write_polygons(ch.wkb, cp);
      }
      out.push_back(std::move(ch));
      continue;
    }
    std::vector<mgpu::wkb::Polygon> parts;
    double area = 0;
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
        if (!(rmaxx < cminx || rminx > cmaxx || rmaxy < cminy || rminy > cmaxy)) clipped = clip_ring(ring, cellb);
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
    if (parts.empty() || area <= 0) continue;  // empty chip: dropped
    int64_t id = g.cell_id(c.first, c.second);
    if (!id) continue;
    (void)cell_area;
    Chip ch{id, pid, 0, {}};
    mgpu::wkb::write_polygons(ch.wkb, parts);
    out.push_back(std::move(ch));
  }
}

int nearest_face(double lon_deg, double lat_deg) {
  double lat = lat_deg * M_PI / 180.0, lon = lon_deg * M_PI / 180.0;
  double x = cos(lon) * cos(lat), y = sin(lon) * cos(lat), z = sin(lat);
  int best = 0;
  double bd = 5;
  for (int f = 0; f < 20; f++) {
    double dx = H3T_FACE_CENTER_POINT[f][0] - x, dy = H3T_FACE_CENTER_POINT[f][1] - y,
           dz = H3T_FACE_CENTER_POINT[f][2] - z;
    double d = dx * dx + dy * dy + dz * dz;
    if (d < bd) {
      bd = d;
      best = f;
    }
  }
  return best;
}

}  // namespace

struct mgpu_tess {
  std::vector<Chip> chips;
};

extern "C" {

int32_t mgpu_tessellate(int32_t index_system, int32_t res, int64_t n_polys, const int32_t* polygon_id,
                        const int64_t* poly_part_off, const int64_t* part_ring_off, const int64_t* ring_off,
                        const double* xy, int32_t keep_core_geometries, mgpu_tess** out) {
  if (!out || n_polys < 0) return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellate: bad arguments");
  if (int32_t st = mgpu_check_resolution(index_system, res)) return st;
  if (index_system == MGPU_BNG && res == -1)
    // 500km ids depend on the easting letter only: no square cells to clip
    return mgpu::set_error(MGPU_E_RESOLUTION, "BNG resolution -1 (500km) cannot be tessellated");
  // polygons are independent: tessellate them in parallel into per-polygon chip lists,
  // then concatenate in input order (the output does not depend on the schedule)
  std::vector<std::vector<Chip>> per(n_polys);
  std::vector<uint8_t> multi_face(n_polys, 0);
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
      if (index_system == MGPU_H3) {
        int face = -1;
        bool one_face = true;
        for (auto& part : poly.parts)
          for (auto& ring : part)
            for (auto& pt : ring) {
              int f = nearest_face(pt.x, pt.y);
              if (face < 0) face = f;
              else if (f != face) one_face = false;
            }
        if (!one_face) {
          multi_face[p] = 1;
          continue;
        }
        H3Grid g(face, res);
        tessellate_polygon(g, poly, polygon_id[p], keep_core_geometries != 0, per[p]);
      } else {
        BngGrid g(res);
        tessellate_polygon(g, poly, polygon_id[p], keep_core_geometries != 0, per[p]);
      }
    }
  });
  for (int64_t p = 0; p < n_polys; p++)
    if (multi_face[p])
      return mgpu::set_error(MGPU_E_INVALID_ARG,
                             "tessellate: polygon %d spans several icosahedron faces (not supported by this "
                             "builder; split it first)", polygon_id[p]);
  mgpu_tess* t = new mgpu_tess();
  size_t total = 0;
  for (auto& v : per) total += v.size();
  t->chips.reserve(total);
  for (auto& v : per) {
    for (auto& c : v) t->chips.push_back(std::move(c));
    std::vector<Chip>().swap(v);
  }
  *out = t;
  return MGPU_OK;
}

int32_t mgpu_tess_result_sizes(const mgpu_tess* t, int64_t* n_chips, int64_t* wkb_bytes) {
  if (!t) return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellation result is NULL");
  int64_t b = 0;
  for (auto& c : t->chips) b += (int64_t)c.wkb.size();
  if (n_chips) *n_chips = (int64_t)t->chips.size();
  if (wkb_bytes) *wkb_bytes = b;
  return MGPU_OK;
}

int32_t mgpu_tess_result_copy(const mgpu_tess* t, int64_t* cell, int32_t* polygon_id, uint8_t* is_core,
                              int64_t* wkb_offsets, uint8_t* wkb) {
  if (!t) return mgpu::set_error(MGPU_E_INVALID_ARG, "tessellation result is NULL");
  int64_t off = 0;
  for (size_t i = 0; i < t->chips.size(); i++) {
    const Chip& c = t->chips[i];
    cell[i] = c.cell;
    polygon_id[i] = c.poly;
    is_core[i] = c.core;
    wkb_offsets[i] = off;
    if (!c.wkb.empty()) memcpy(wkb + off, c.wkb.data(), c.wkb.size());
    off += (int64_t)c.wkb.size();
  }
  wkb_offsets[t->chips.size()] = off;
  return MGPU_OK;
}

int32_t mgpu_tess_destroy(mgpu_tess* t) {
  delete t;
  return MGPU_OK;
}

}  // extern "C"
